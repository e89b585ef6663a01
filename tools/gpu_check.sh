# GPU round trip used during development: kernel + parity tests, micro-benchmarks, bench, profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 120 python tools/mb_norm.py > gpurun_out/mb.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 7 --warmup 2 --no-probe > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
