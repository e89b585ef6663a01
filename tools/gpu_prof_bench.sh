# rocprofv3 kernel trace of the bench command itself (graph replay of the fp32 headline, live probes),
# summarised on the box: <tag> [bench args...]   (default: 20 timed steps, no bf16 leg, no CPU leg)
# (tools/prof_summary.py: per-kernel totals over the whole run -- warm-up, capture and probe steps
# included -- and summed vs interval-union kernel time.)
set -o pipefail
tag=$1; shift
[ $# -eq 0 ] && set -- --steps 20 --warmup 3 --other-steps 0 --no-cpu-baseline
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/benchprof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 $R/bench.py "$@" > $O/bench.log 2>&1 || exit $?
db=$(find $O/raw -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $db 60 > $O/summary.md && rm -rf $O/raw
