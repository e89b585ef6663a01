# round 6: forked-graph / DP-expert tests, then DP E=4 timings
#   bash tools/gpu_r06a.sh <tag>
set -o pipefail
tag=${1:-r06a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_fork_graph_gpu.py tests/test_ddp_graph_gpu.py "tests/test_ddp_gpu.py::test_ddp_rank_without_expert_samples" \
  > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_grads_gpu.py tests/test_b512_gpu.py \
  > $O/grads.log 2>&1; rc=$?; tail -3 $O/grads.log; [ $rc -eq 0 ] || exit $rc
for args in "--experts 4 --batch 512" "--ddp --sync-bn --experts 4 --batch 512" "--ddp --sync-bn --experts 4 --batch 512 --graph on"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py $args --steps 60 --warmup 10 --other-steps 0 --no-cpu-baseline > $O/b_$n.json 2> $O/b_$n.err || exit 1
  python -c "import json;d=json.load(open('$O/b_$n.json'));print('$args', d['value'], d['ms_per_step'], d['step_launch'])"
done
