set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ring or glds or conv_fwd or subpixel" -x -v --timeout 120 --timeout-method thread > $O/t_ring.log 2>&1 && \
timeout -k 10 200 python -u tools/mb_conv.py > $O/mb_conv.log 2>&1
