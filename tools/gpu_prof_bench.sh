# rocprofv3 kernel trace of the bench command itself (graph replay, fp32 headline + bf16 secondary,
# live probes), summarised on the box: <tag> [bench args...]
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/benchprof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $R/bench.py "$@" > $O/bench.log 2>&1 || exit $?
st=$(find $O/raw -name '*kernel_stats.csv' | head -1)
tr=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python3 $R/tools/prof_summary.py $st 1 $tr > $O/summary.md && rm -rf $O/raw
