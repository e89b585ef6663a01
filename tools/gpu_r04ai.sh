# bf16 ring_loop: waves 4-7 issue their step's DMA after their MFMAs (ES_RING_STAG build): bf16 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--precision bf16" REPS=3 bash tools/gpu_libab.sh b r1
