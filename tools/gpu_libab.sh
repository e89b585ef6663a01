# A/B of two library builds on one box (graph-replayed train steps, tools/prof_step.py), alternating:
#   bash tools/gpu_libab.sh <libB path> [rounds 3] [prof_step args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
B=$1; shift
N=${1:-3}; shift
ARGS=${@:---experts 1 --batch 1024 --precision fp32 --steps 40}
for r in $(seq $N); do
  a=$(timeout -k 10 200 python -u tools/prof_step.py $ARGS 2>/dev/null | tail -1) || exit 1
  b=$(ES_LIB=$B timeout -k 10 200 python -u tools/prof_step.py $ARGS 2>/dev/null | tail -1) || exit 1
  echo "round $r  A(default): $a   B($B): $b"
done
