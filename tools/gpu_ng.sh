set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for NGV in 8 16 32 64; do
  for L in c5 c0 c9; do for M in fwd dgrad; do
    ES_RING_NG=$NGV timeout -k 10 60 python tools/mb_one.py $L $M 1 10 2>&1 | grep -v amdgpu.ids | sed "s/^/ng=$NGV /" || exit 1
  done; done
done > $O/ng.log
