# fused discriminator front A/B: probe builds under _abl/ (tools/abl_build_tu.sh d_front2 ...), then the
# default build's kernel test
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/df2.log
for v in "$@"; do
  echo "== $v" >> $O/df2.log
  ES_LIB=$PWD/_abl/$v/libexpertsim_hip.so timeout -k 10 120 python tools/mb_dfront2.py >> $O/df2.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "dfront2" --timeout 200 --timeout-method thread >> $O/df2.log 2>&1
