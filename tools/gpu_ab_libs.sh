set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
ES_LIB=ab_libs/base.so timeout -k 10 200 python -u tools/mb_norm.py > $O/mbn_base.log 2>&1 && \
ES_LIB=ab_libs/${1:-nt}.so timeout -k 10 200 python -u tools/mb_norm.py > $O/mbn_nt.log 2>&1 && \
bash tools/gpu_ab.sh "ES_LIB=ab_libs/base.so" "ES_LIB=ab_libs/${1:-nt}.so"
