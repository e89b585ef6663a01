# Every BASELINE config on one GPU at its per-GPU shard (round 4): fp32 (the reference's precision) unless
# the config names bf16; multi-expert lines after 300 warm-up steps (per-expert graph keys cached)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
: > $O/configs_r04.log
run() {
  local lab=$1; shift
  v=$(timeout -k 10 400 python bench.py --other-steps 0 --no-cpu-baseline --no-probe "$@" 2>/dev/null | tail -1) || return 1
  echo "$lab | $* | $v" >> $O/configs_r04.log
}
run "configs[0] B=64 E=1 fp32" --batch 64 --steps 50 || exit 1
run "configs[1] B=512 E=1 bf16" --batch 512 --precision bf16 --steps 50 || exit 1
run "configs[1] B=512 E=1 fp32" --batch 512 --steps 50 || exit 1
run "configs[2] B=1024 E=1 fp32 (headline)" --batch 1024 --steps 50 || exit 1
run "configs[3] per-GPU shard B=512 E=4 fp32" --batch 512 --experts 4 --warmup 300 --steps 50 || exit 1
run "configs[4] per-GPU shard neutron56 B=512 E=8 fp32" --arch neutron56 --batch 512 --experts 8 --warmup 300 --steps 30 || exit 1
