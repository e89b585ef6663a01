# Every BASELINE config (and the per-GPU shards of the multi-GPU ones) on one GPU with bench.py's
# default warm-up, one JSON line each -> gpurun_out/configs_<tag>.jsonl:
#   bash tools/gpu_configs.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-configs}
O=$GRAFT_REPO_ROOT/gpurun_out/configs_$tag.jsonl
: > $O
run() {
  local v
  v=$(timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline --no-probe "$@" 2> /dev/null | tail -1) || return 1
  echo "{\"args\": \"$*\", \"line\": $v}" >> $O
  echo "[$*] ok"
}
run --batch 64 &&
run --batch 512 --precision bf16 &&
run --batch 512 &&
run --batch 1024 &&
run --batch 512 --experts 4 &&
run --batch 2048 --experts 4 &&
run --arch neutron56 --batch 512 --experts 8 &&
run --arch proton --batch 512 &&
run --arch proton --batch 1024
