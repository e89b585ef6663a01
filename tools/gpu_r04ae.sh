# WGRAD coop kernel: two register stages of loads (ES_COOP2 build): bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=3 bash tools/gpu_libab.sh s0 p2
