#!/bin/bash
# round-end state, as the driver runs it: the GPU suite, smoke(), the default bench line, and a
# kernel-trace profile of the bench command (tools/gpu_prof_bench.sh)
#   bash tools/gpu_r06_final.sh <tag> [tests|bench|all]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-final}; WHAT=${2:-all}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
if [ "$WHAT" != bench ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit $?
  timeout -k 10 200 python -u -m pytest tests/test_b512_gpu.py -q -s -k bf16 --timeout 240 --timeout-method thread > $O/bf16_step0.log 2>&1 || exit $?
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
if [ "$WHAT" != tests ]; then
  timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
  bash tools/gpu_prof_bench.sh $TAG || exit $?
fi
