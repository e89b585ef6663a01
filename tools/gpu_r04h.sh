# norm NT A/B (fp32 bench shapes); eager / data-parallel (RCCL world size 1) step cost against the
# graph replay; the captured data-parallel step against the eager one
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ddp_graph_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/ddpgraph_r04h.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --other-steps 0 --no-cpu-baseline --no-probe --graph off > $O/eager_r04h.json 2> $O/eager_r04h.err || exit $?
timeout -k 10 300 python bench.py --ddp --sync-bn --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/ddp1_r04h.json 2> $O/ddp1_r04h.err || exit $?
timeout -k 10 300 python bench.py --ddp --sync-bn --graph on --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/ddp1g_r04h.json 2> $O/ddp1g_r04h.err || exit $?
# wide linears as 16-row pixel blocks on the ring FWD (ConvOp._pixel_view): kernel test, goldens, bench
timeout -k 10 600 python -u -m pytest tests/test_f32_split_gpu.py tests/test_b512_gpu.py tests/test_train_step_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/linpix_r04h.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline > $O/neutron_r04h.json 2> $O/neutron_r04h.err || exit $?
