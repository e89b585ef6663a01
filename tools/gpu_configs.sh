# The BASELINE configs beyond the headline line, on one GPU: B=1024 (configs[2]), 4 experts at
# B=512 (configs[3]'s per-GPU shard, eager), fp32 parity mode, and the proton 56x30 secondary shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
: > $O/configs.log
for cfg in "--batch 1024" "--experts 4" "--precision fp32" "--arch proton" "--arch proton --batch 1024"; do
  v=$(timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe $cfg 2>/dev/null | tail -1) || exit 1
  echo "[$cfg] $v" >> $O/configs.log
done
