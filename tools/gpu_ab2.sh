# A/B of env settings on one box with the conv microbench + bench: bash tools/gpu_ab2.sh "ENV1" "ENV2"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
: > $O/ab.log
for cfg in "$@"; do
  echo "== [$cfg]" >> $O/ab.log
  env $cfg timeout -k 10 200 python -u tools/mb_conv.py 2>/dev/null | cut -c1-200 >> $O/ab.log || exit 1
done
for round in 1 2; do
  for cfg in "$@"; do
    v=$(env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "round $round [$cfg] $v" >> $O/ab.log
  done
done
