set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06i
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_f32_split_gpu.py -k wave_specialised > gpurun_out/r06i/t.log 2>&1; rc=$?; tail -2 gpurun_out/r06i/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/mb_ab.py c5 wgrad es_conv_set_wgrad_ws 1024 3 10 0,1 | tail -1 || exit 1
timeout -k 10 120 python -u tools/mb_ab.py c5 wgrad es_conv_set_wgrad_ws 1024 3 10 1,2 | tail -1 || exit 1
for v in 11 14; do timeout -k 10 120 python -u tools/mb_ab.py c5 wgrad es_conv_set_wgrad_ws 1024 2 10 1,$v | tail -1 || exit 1; done
timeout -k 10 120 python -u tools/mb_ab.py c0 wgrad es_conv_set_wgrad_ws 1024 3 10 0,1 | tail -1 || exit 1
