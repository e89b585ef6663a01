# fused dgrad + BatchNorm-backward reduction: its kernel tests, then the bench off / on and a
# kernel-trace profile (same box)
#   bash tools/gpu_bnred_quick.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-bnq}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "bn_reduce_fused" > $O/tk_$TAG.log 2>&1 || exit $?
ES_BNRED=0 timeout -k 10 300 python bench.py --fp32-steps 0 --no-cpu-baseline > $O/bench_${TAG}_off.json 2> $O/bench_${TAG}_off.err && \
timeout -k 10 300 python bench.py --fp32-steps 0 --no-cpu-baseline > $O/bench_${TAG}_on.json 2> $O/bench_${TAG}_on.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --fp32-steps 0 --no-cpu-baseline --graph off > $O/prof_$TAG.log 2>&1
