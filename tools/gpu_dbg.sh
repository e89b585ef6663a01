set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for L in ${LAYERS:-c5 c0}; do for M in ${MODES:-fwd dgrad wgrad}; do for D in 0 1 2; do
ES_RING_DBG=$D timeout -k 10 60 python tools/mb_one.py $L $M 1 10 2>&1 | grep -v amdgpu.ids || exit 1
done; done; done > $O/dbg.log
