# A/B of the WGRAD minimum K-steps per split (ES_WGRAD_MINK) at E=4 B=512 and E=1 B=1024
#   bash tools/gpu_mink.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-mink}
O=$GRAFT_REPO_ROOT/gpurun_out
for m in 8 32 64 8 32 64; do
  ES_WGRAD_MINK=$m timeout -k 10 300 python bench.py --batch 512 --experts 4 --steps 100 --warmup 120 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/${TAG}_e4_m$m.json 2> $O/${TAG}_e4_m$m.err || exit $?
  echo "e4 mink=$m $(python -c "import json;d=json.load(open('$O/${TAG}_e4_m$m.json'));print(d['ms_per_step'])")"
done
for m in 8 64; do
  ES_WGRAD_MINK=$m timeout -k 10 300 python bench.py --steps 100 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/${TAG}_e1_m$m.json 2> $O/${TAG}_e1_m$m.err || exit $?
  echo "e1 b1024 mink=$m $(python -c "import json;d=json.load(open('$O/${TAG}_e1_m$m.json'));print(d['ms_per_step'])")"
done
