# The bf16/fp32 training-statistics test twice (run-to-run spread of its WS statistic), then the
# rest of the GPU suite.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for r in 1 2; do
  timeout -k 10 450 python -u -m pytest tests/test_bf16_stats_gpu.py -q -s --timeout 420 --timeout-method thread 2>&1 | grep -E "WS\(run|passed|failed" > $O/ws_$r.log
  rc=$?; [ $rc -gt 1 ] && exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread --deselect tests/test_bf16_stats_gpu.py::test_bf16_training_statistics_match_fp32_and_oracle > $O/t_rest.log 2>&1
echo "rc=$?" >> $O/t_rest.log
