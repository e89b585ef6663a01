# SPB loop: column tile at which waves 4-7 split A(t+1) (ES_SPB_SPLIT_HI builds), with the DMA stagger: bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=2 bash tools/gpu_libab.sh b h1 h2 h6 h7
