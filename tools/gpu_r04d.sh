# planes (SPA) A/B + bitwise check, then the parity tests with their printed worst errors
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python tools/mb_spb4.py 1024 5 > gpurun_out/mb_spb4_r04d.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_train_step_gpu.py tests/test_grads_gpu.py tests/test_b512_gpu.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/t_parity_r04d.log 2>&1
