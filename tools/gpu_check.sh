# GPU round trip used during development: kernel + parity tests, smoke, bench, profile.
# usage (from the container): gpurun --timeout 1100 -- bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-dev}
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 && \
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 7 --warmup 2 --no-probe --graph off --no-cpu-baseline > $O/prof.log 2>&1
