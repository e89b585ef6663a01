# normalise-on-load of conv_layers.10 in conv_layers.13 (fp32): bitwise step test, kernel / golden /
# determinism / trajectory tests, then bench A/B (ES_NOL=0 / 1) alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_nol_gpu.py tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_grads_gpu.py tests/test_b512_gpu.py tests/test_determinism_gpu.py tests/test_bf16_stats_gpu.py tests/test_graph_gpu.py tests/test_eval_gpu.py -m gpu -q -s --timeout 350 --timeout-method thread -k "nol or conv_fwd_dgrad_wgrad or bn_reduce or train_step or large_batch or determinism or training_statistics or step_gradients or graph or eval" > $O/t_r04ab.log 2>&1
echo "pytest rc=$?" >> $O/t_r04ab.log
bash tools/gpu_knobs.sh ES_NOL=0 ES_NOL=0
