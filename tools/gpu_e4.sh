# E=4 vs E=1 at B=512 (graph replay) and a kernel trace of the E=4 graph step
#   bash tools/gpu_e4.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-e4}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python bench.py --batch 512 --experts 1 --steps 100 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/${TAG}_e1.json 2> $O/${TAG}_e1.err && \
timeout -k 10 400 python bench.py --batch 512 --experts 4 --steps 100 --warmup 120 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/${TAG}_e4.json 2> $O/${TAG}_e4.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 512 --experts 4 --steps 20 --warmup 120 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/prof_${TAG}.log 2>&1
