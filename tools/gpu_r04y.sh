# 20-step training trajectory against the oracle (tests/test_bf16_stats_gpu.py) under ES_SPB_FRESH = 1 / 2
# builds, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/traj.log
for i in 1 2; do
  for v in cm_f1 cm_f2; do
    echo "== $v $i" >> $O/traj.log
    ES_LIB=$PWD/_abl/$v/libexpertsim_hip.so timeout -k 10 400 python -u -m pytest tests/test_bf16_stats_gpu.py -m gpu -q -s --timeout 350 --timeout-method thread -k "training_statistics" > $O/traj_$v.log 2>&1
    grep -E "trajectory|passed|failed" $O/traj_$v.log >> $O/traj.log
  done
done
