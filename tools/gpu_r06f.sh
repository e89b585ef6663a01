set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06f
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_f32_split_gpu.py -k wave_specialised > gpurun_out/r06f/t.log 2>&1; rc=$?; tail -2 gpurun_out/r06f/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/mb_ab.py c5 wgrad es_conv_set_wgrad_ws 1024 4 10 || exit 1
timeout -k 10 120 python -u tools/mb_ab.py c0 wgrad es_conv_set_wgrad_ws 1024 3 10 || exit 1
bash tools/gpu_pmc_ab.sh r06f c5 wgrad es_conv_set_wgrad_ws 1024 || exit 1
python3 tools/pmc_ab_summary.py gpurun_out/pmc_r06f wgrad_coop_kernel wgrad_ws_kernel wgrad_reduce
