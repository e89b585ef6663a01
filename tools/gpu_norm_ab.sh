# norm-kernel A/B: builds under _abl/ (tools/abl_build_tu.sh norm_fast ...), fp32 bench shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/norm_ab.log
for v in "$@"; do
  echo "== $v" >> $O/norm_ab.log
  MB_NORM_F32=1 ES_LIB=$PWD/_abl/$v/libexpertsim_hip.so timeout -k 10 180 python tools/mb_norm.py >> $O/norm_ab.log 2>&1 || exit $?
done
