# SPB loop: column tile at which waves 0-3 issue their step's DMA (ES_SPB_DMA_LO builds), waves 4-7 at 6: bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=2 bash tools/gpu_libab.sh b l1 l2 l3
