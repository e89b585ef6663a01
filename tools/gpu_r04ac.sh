# SPB loop DMA stagger (ES_SPB_DMA_STAGGER build): bitwise kernel / golden tests under that build, then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
ES_LIB=$PWD/_abl/cm_stag/libexpertsim_hip.so timeout -k 10 600 python -u -m pytest tests/test_f32_split_gpu.py tests/test_b512_gpu.py tests/test_spb4_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/t_r04ac.log 2>&1
echo "pytest rc=$?" >> $O/t_r04ac.log
bash tools/gpu_libab.sh cm_base cm_stag
