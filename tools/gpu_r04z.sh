# 20-step trajectory against the oracle with the exact fp32 MFMA (ES_FP32_MFMA=exact): the spread of a
# different, unbiased fp32 rounding, for scale against the split builds (tools/gpu_r04y.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/traj_exact.log
ES_FP32_MFMA=exact timeout -k 10 400 python -u -m pytest tests/test_bf16_stats_gpu.py -m gpu -q -s --timeout 350 --timeout-method thread -k "training_statistics" > $O/traj_ex.log 2>&1
grep -E "trajectory|passed|failed" $O/traj_ex.log >> $O/traj_exact.log
ES_SPB_FRESH_DUMMY=1 ES_LIB=$PWD/_abl/cm_f2/libexpertsim_hip.so ES_SPL_PRIO=0 timeout -k 10 400 python -u -m pytest tests/test_bf16_stats_gpu.py -m gpu -q -s --timeout 350 --timeout-method thread -k "training_statistics" > $O/traj_f2p.log 2>&1
echo "== f2 with ES_SPL_PRIO=0 (another rounding-neutral schedule change)" >> $O/traj_exact.log
grep -E "trajectory|passed|failed" $O/traj_f2p.log >> $O/traj_exact.log
