set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06m
O=gpurun_out/r06m
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_neutron56_gpu.py > $O/n56.log 2>&1; rc=$?; grep -E "neutron56 E=8|passed|failed" $O/n56.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/cpu_table.py $O/cpu_table.md > $O/cpu_table.log 2>&1 || exit 1
tail -8 $O/cpu_table.md
