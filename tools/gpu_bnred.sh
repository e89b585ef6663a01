# fused dgrad + BatchNorm-backward reduction (es_conv2d_dgrad_bnred) and multi-tap WGRAD tiles:
# their kernel tests, the GPU suite, then the bench with the features off / on (same box)
#   bash tools/gpu_bnred.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-bnred}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "bn_reduce_fused or persist or wgrad_multitap or conv_fwd_dgrad_wgrad or subpixel" > $O/tk_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread > $O/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ES_BNRED=0 timeout -k 10 300 python bench.py --fp32-steps 0 --no-cpu-baseline > $O/bench_${TAG}_off.json 2> $O/bench_${TAG}_off.err && \
timeout -k 10 300 python bench.py --fp32-steps 0 --no-cpu-baseline > $O/bench_${TAG}_on.json 2> $O/bench_${TAG}_on.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --fp32-steps 0 --no-cpu-baseline --graph off > $O/prof_$TAG.log 2>&1
