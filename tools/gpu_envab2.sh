# Kernel + step tests, then a bench A/B: bash tools/gpu_envab2.sh "<baseline env>" "<candidate env>"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t_env.log 2>&1 && \
bash tools/gpu_ab.sh "$1" "$2"
