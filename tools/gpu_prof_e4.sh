# rocprofv3 kernel trace of E = 4, B = 512 fp32 graph replays (tools/prof_step.py), summarised on the box:
#   bash tools/gpu_prof_e4.sh <tag>   (summed vs interval-union kernel time shows the experts' overlap)
set -o pipefail
tag=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/e4prof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 $R/tools/prof_step.py --experts 4 --batch 512 --steps 20 > $O/run.log 2>&1 || exit $?
db=$(find $O/raw -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $db 60 > $O/summary.md && rm -rf $O/raw
