# kernel trace of a short eager bench run: <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --fp32-steps 0 --no-cpu-baseline --no-probe --graph off > $O/prof_$1.log 2>&1
