# E=4 vs E=1 at B=512 (graph replay) in both precisions: bash tools/gpu_e4.sh <tag> [prof]
# (prof: also a kernel trace of the bf16 E=4 step)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-e4}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
for P in fp32 bf16; do
  timeout -k 10 300 python bench.py --precision $P --batch 512 --experts 1 --steps 60 --other-steps 0 --no-cpu-baseline --no-probe > $O/${P}_e1.json 2> $O/${P}_e1.err || exit $?
  timeout -k 10 400 python bench.py --precision $P --batch 512 --experts 4 --steps 60 --warmup 120 --other-steps 0 --no-cpu-baseline --no-probe > $O/${P}_e4.json 2> $O/${P}_e4.err || exit $?
done
[ "$2" = prof ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision bf16 --batch 512 --experts 4 --steps 20 --warmup 120 --other-steps 0 --no-cpu-baseline --no-probe > $O/prof.log 2>&1
