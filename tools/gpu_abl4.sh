# same-box A/B of 4-wave kernel builds (_abl/<name>, tools/abl_build.sh) on tools/mb_spb4.py: <names...>
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 200 python -u tools/mb_spb4.py 1024 5 2>&1 | grep -v amdgpu > $O/abl4_default.log || exit $?
for d in "$@"; do
  ES_LIB=$GRAFT_REPO_ROOT/_abl/$d/libexpertsim_hip.so ES_MB_NOCHECK=1 timeout -k 10 200 python -u tools/mb_spb4.py 1024 5 2>&1 | grep -v amdgpu > $O/abl4_$d.log || exit $?
done
