# selected GPU tests with output:  PYK='expr' bash tools/gpu_tests.sh <tag> [test files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-q}; shift
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -q -s -rf --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > $O/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/t_$TAG.log
exit $rc
