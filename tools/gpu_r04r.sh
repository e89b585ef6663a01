# thin-conv defaults (fwd / wgrad 2 chunks per lane): kernel + golden + determinism tests, then the knob A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_grads_gpu.py tests/test_b512_gpu.py tests/test_determinism_gpu.py tests/test_wgrad_reduce_gpu.py tests/test_f32_split_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/t_r04r.log 2>&1 || exit $?
bash tools/gpu_knobs.sh ES_SPB_NOSHORTK=1 ES_SPL_PRIO=0 ES_WGRAD_BN128=1 ES_SPB_NOSHORTK=1
