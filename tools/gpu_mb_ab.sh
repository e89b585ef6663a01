# per-op microbenchmark (tools/mb_one.py) under env configs: bash tools/gpu_mb_ab.sh "op1 mode1,op2 mode2" "CFG1" "CFG2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
OPS="$1"; shift
: > $O/mb_ab.log
for round in 1 2; do
  for cfg in "$@"; do
    IFS=',' read -ra L <<< "$OPS"
    for op in "${L[@]}"; do
      r=$(env $cfg timeout -k 10 120 python tools/mb_one.py $op 1 20 2>/dev/null | tail -1) || exit 1
      echo "[$cfg] $r" >> $O/mb_ab.log
    done
  done
done
