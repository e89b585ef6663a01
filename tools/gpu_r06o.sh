set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_f32_split_gpu.py -k "wave_specialised" > gpurun_out/r06o/t.log 2>&1; rc=$?; tail -2 gpurun_out/r06o/t.log; [ $rc -eq 0 ] || exit $rc
for lm in "c5 fwd" "c0 fwd" "c9 fwd" "c0 dgrad"; do timeout -k 10 120 python -u tools/mb_ab.py $lm es_conv_set_ring_ws 1024 3 10 0,1 | tail -1 || exit 1; done
for lm in "c5 wgrad" "c0 wgrad"; do timeout -k 10 120 python -u tools/mb_ab.py $lm es_conv_set_wgrad_ws 1024 3 10 0,1 | tail -1 || exit 1; done
