# fp32 thin dgrad + BatchNorm-backward reduction (k1_dgrad_bnred<float>): kernel tests, goldens, determinism,
# 20-step trajectory, then bench A/B (ES_THIN_BNRED=0 / 1) alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_grads_gpu.py tests/test_b512_gpu.py tests/test_determinism_gpu.py tests/test_bf16_stats_gpu.py -m gpu -q -x -s --timeout 350 --timeout-method thread -k "bn_reduce or train_step or grads or large_batch or determinism or training_statistics or step_gradients" > $O/t_r04aa.log 2>&1
echo "pytest rc=$?" >> $O/t_r04aa.log
bash tools/gpu_knobs.sh ES_THIN_BNRED=0 ES_THIN_BNRED=0
