# quick GPU loop: selected kernel tests + bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_train_step_gpu.py -x -v --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > $O/t_q.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_q.log 2>&1
