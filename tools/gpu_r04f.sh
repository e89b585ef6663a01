# resize materialisation: kernel tests (incl. the 35x19 -> 56x30 conv), f32 ring + proton parity tests, proton bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_f32_ring_gpu.py tests/test_spb4_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/t_r04f.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_train_step_gpu.py tests/test_grads_gpu.py -m gpu -q -x -k proton --timeout 200 --timeout-method thread >> $O/t_r04f.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --arch proton --batch 1024 --steps 20 --other-steps 0 --no-cpu-baseline > $O/proton1024_r04f.json 2> $O/proton1024_r04f.err
