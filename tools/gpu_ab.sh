# A/B of env settings on one box: bash tools/gpu_ab.sh "ENV1" "ENV2" ...  (bench.py, 2 rounds each, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
: > $O/ab.log
for round in 1 2; do
  for cfg in "$@"; do
    v=$(env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "round $round [$cfg] $v" >> $O/ab.log
  done
done
