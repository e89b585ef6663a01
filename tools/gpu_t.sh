# one GPU test file / expression with output: bash tools/gpu_t.sh <tag> <pytest args...>
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest "$@" -m gpu -q -s -rf --timeout 200 --timeout-method thread > $O/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/t_$TAG.log; exit $rc
