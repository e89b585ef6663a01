# Parity tests of the changed kernels (+ the same tests under extra env), then an interleaved
# bench A/B of env configs: bash tools/gpu_exp.sh "<pytest -k expr>" "<extra test env>" "CFG1" "CFG2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
K="$1"; XENV="$2"; shift 2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_train_step_gpu.py -x -v --timeout 120 --timeout-method thread -k "$K" > $O/t_exp.log 2>&1 || exit 1
if [ -n "$XENV" ]; then
  env $XENV timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "subpixel or fused_bn" > $O/t_exp2.log 2>&1 || exit 1
fi
: > $O/ab.log
for round in 1 2; do
  for cfg in "$@"; do
    v=$(env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "round $round [$cfg] $v" >> $O/ab.log
  done
done
