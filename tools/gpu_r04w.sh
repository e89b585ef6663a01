# K-steps per fresh accumulator in the split FWD / DGRAD (ES_SPB_FRESH = 1 / 2 / 4 builds): the B = 1024
# golden's gradient errors (noise-only biases printed) per build, then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/t_r04w.log
for v in cm_base cm_f2 cm_f4; do
  echo "== $v" >> $O/t_r04w.log
  ES_LIB=$PWD/_abl/$v/libexpertsim_hip.so timeout -k 10 600 python -u -m pytest tests/test_b512_gpu.py tests/test_f32_split_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread -k "b1024 or split_matches" > $O/t_$v.log 2>&1
  echo "rc=$?" >> $O/t_r04w.log
  grep -E "worst|passed|failed" $O/t_$v.log >> $O/t_r04w.log
done
bash tools/gpu_libab.sh cm_base cm_f2 cm_f4
