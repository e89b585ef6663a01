# same-box A/B of library builds under _abl/<name>/ (ES_LIB) on the split-fp32 conv micro-benchmark,
# after the split tests on the default build
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_split_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > $O/t_abl.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t_abl.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/mb_split.py 1024 5 2>&1 | grep -v amdgpu > $O/abl_default.log || exit $?
for d in "$@"; do
  ES_LIB=$GRAFT_REPO_ROOT/_abl/$d/libexpertsim_hip.so timeout -k 10 200 python -u tools/mb_split.py 1024 5 2>&1 | grep -v amdgpu > $O/abl_$d.log || exit $?
done
