# Kernel trace + PMC (HBM bytes, MFMA busy) of whole train steps: tools/prof_step.py replays of one
# configuration, one rocprofv3 pass per counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE
# cannot share a pass), each replay synchronised (one replay's packets in flight under the profiler).
#   bash tools/gpu_pmc_step.sh <tag> <prof_step args...>   e.g. r05_bf16 --experts 1 --batch 1024 --precision bf16
# -> gpurun_out/pmcstep_<tag>/summary.md (tools/pmc_step.py)
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcstep_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/prof_step.py $* --steps 2 --sync"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- $P > $O/mfma.log 2>&1 && \
python3 $R/tools/pmc_step.py $O 6 > $O/summary.md && rm -rf $O/kt $O/fetch $O/write $O/mfma && head -30 $O/summary.md
