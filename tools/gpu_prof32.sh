# kernel trace of a short eager fp32 (parity mode) bench run at configs[2]: <tag> [batch]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
B=${2:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof32_$1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32 --batch $B --steps 5 --warmup 2 --fp32-steps 0 --no-cpu-baseline --no-probe --graph off > $O/prof32_$1.log 2>&1
