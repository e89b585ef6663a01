# kernel trace of graph-replayed train steps (tools/prof_step.py) summarised by tools/prof_summary.py
#   bash tools/gpu_trace_step.sh <tag> <prof_step args...>  -> gpurun_out/trace_<tag>.txt
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tr_$tag -o run -- python3 $R/tools/prof_step.py "$@" > $R/gpurun_out/tr_$tag.log 2>&1 || exit 1
db=$(find $R/gpurun_out/tr_$tag -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $db 70 > $R/gpurun_out/trace_$tag.txt && cp $db $R/gpurun_out/trace_$tag.db && rm -rf $R/gpurun_out/tr_$tag
head -3 $R/gpurun_out/trace_$tag.txt
