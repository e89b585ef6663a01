# round-2 baseline: full GPU test suite + bench lines at B=512 and B=1024
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_512.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --batch 1024 --no-cpu-baseline > $O/bench_1024.log 2>&1
