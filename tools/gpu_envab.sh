# Env A/B with the step tests under the candidate env: bash tools/gpu_envab.sh "<candidate env>"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
env $1 timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_train_step_gpu.py tests/test_checkpoint_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t_env.log 2>&1 && \
bash tools/gpu_ab.sh "ES_NOTHING=0" "$1"
