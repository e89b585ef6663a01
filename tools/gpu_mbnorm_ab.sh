# norm microbenchmark under two library builds: bash tools/gpu_mbnorm_ab.sh <lib.so>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 200 python -u tools/mb_norm.py > $O/mbn_new.log 2>&1 && \
ES_LIB=$1 timeout -k 10 200 python -u tools/mb_norm.py > $O/mbn_base.log 2>&1
