# fp32 ring BN-reduce fold opt-in again: its kernel test, the golden / grads tests, a default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "bn_reduce" --timeout 200 --timeout-method thread > $O/t_r04n.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_train_step_gpu.py tests/test_grads_gpu.py tests/test_b512_gpu.py tests/test_determinism_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread >> $O/t_r04n.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline > $O/neutron_r04n.json 2> $O/neutron_r04n.err
