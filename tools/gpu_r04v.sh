# one fresh accumulator per two K-steps in the split FWD / DGRAD (ES_SPB_FRESH2 build): numerics under that
# build (split kernel tests, B = 512 / 1024 goldens, gradient goldens), then bench A/B against the base build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
ES_LIB=$PWD/_abl/cm_f2/libexpertsim_hip.so timeout -k 10 900 python -u -m pytest tests/test_f32_split_gpu.py tests/test_b512_gpu.py tests/test_grads_gpu.py tests/test_train_step_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/t_r04v.log 2>&1
echo "pytest rc=$?" >> $O/t_r04v.log
bash tools/gpu_libab.sh cm_base cm_f2
