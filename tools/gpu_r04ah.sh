# SPB loop: B-plane read-ahead depth (ES_SPB_PFD builds) with the DMA stagger: bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=2 bash tools/gpu_libab.sh b p1 p3
