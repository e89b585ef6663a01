# rocprofv3 kernel trace of the bench command itself (graph replay of the fp32 headline, live probes),
# summarised on the box: <tag> [bench args...]   (default: 20 timed steps, no bf16 leg, no CPU leg)
# Per-step columns divide by the number of step_metrics_kernel launches in the trace (one per step,
# warm-up / capture / probe steps included), not by the timed-step count.
set -o pipefail
tag=$1; shift
[ $# -eq 0 ] && set -- --steps 20 --warmup 3 --other-steps 0 --no-cpu-baseline
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/benchprof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $R/bench.py "$@" > $O/bench.log 2>&1 || exit $?
st=$(find $O/raw -name '*kernel_stats.csv' | head -1)
tr=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python3 $R/tools/prof_summary.py $st step_metrics_kernel $tr > $O/summary.md && rm -rf $O/raw
