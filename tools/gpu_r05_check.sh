# round-5 check: parity tests touched by the change, then step timings and a kernel trace
#   bash tools/gpu_r05_check.sh <tag> <pytest files...>
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/t_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/t_$tag.log; [ $rc -eq 0 ] || exit $rc
for p in fp32 bf16; do timeout -k 10 200 python -u tools/prof_step.py --experts 1 --batch 1024 --precision $p --steps 30 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_$tag -o run -- python3 $R/tools/prof_step.py --experts 1 --batch 1024 --precision bf16 --steps 10 > $R/gpurun_out/kt_$tag.log 2>&1 || exit 1
db=$(find $R/gpurun_out/kt_$tag -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $db 60 > $R/gpurun_out/kt_${tag}_bf16.txt && rm -rf $R/gpurun_out/kt_$tag
grep -E "kernels|dmlp|dfront" $R/gpurun_out/kt_${tag}_bf16.txt
