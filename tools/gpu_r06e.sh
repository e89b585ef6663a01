# wave-specialised WGRAD: bitwise test + A/B timing
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_f32_split_gpu.py -k wave_specialised > gpurun_out/r06e/t.log 2>&1; rc=$?; tail -3 gpurun_out/r06e/t.log; [ $rc -eq 0 ] || exit $rc
for l in c5 c0; do timeout -k 10 120 python -u tools/mb_ab.py $l wgrad es_conv_set_wgrad_ws 1024 4 10 || exit 1; done
