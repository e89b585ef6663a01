# round-end check as the driver runs it: GPU suite, smoke(), default bench line
#   bash tools/gpu_verify.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-verify}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread > $O/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
