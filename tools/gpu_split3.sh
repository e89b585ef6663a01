# split-fp32: rounding bias, conv micro-benchmark, noise-only gradients
cd $GRAFT_REPO_ROOT
TAG=${1:-s}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/split_bias.py > $O/split_bias_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/mb_split.py 1024 5 > $O/mb_$TAG.log 2>&1 || exit $?
ES_FP32_MFMA=split timeout -k 10 200 python -u -m pytest tests/test_grads_gpu.py -m gpu -q -s -k "neutron_e1_b8" --timeout 120 --timeout-method thread > $O/noise_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> $O/noise_$TAG.log; exit $rc
