# GPU suite (stops on first failure) + a short bench line; args: <tag> [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-q}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread ${2:+-k "$2"} > $O/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 60 --fp32-steps 0 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err
