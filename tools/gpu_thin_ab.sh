set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
ES_K1_GRID=3 ES_THIN_WGRID=5 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_fwd_dgrad_wgrad" > $O/t_thin.log 2>&1 && \
bash tools/gpu_ab.sh "$@"
