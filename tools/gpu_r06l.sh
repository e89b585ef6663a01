# DP E=4 (eager fork on per-expert communicators / captured serial) vs single-process E=4, plus the
# memory-lean serial capture of configs[4] (neutron56 E=8 B=4096) and the DP graph test
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06l
O=gpurun_out/r06l
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_ddp_graph_gpu.py tests/test_graph_gpu.py tests/test_fork_graph_gpu.py > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for args in "--ddp --sync-bn --experts 4 --batch 512 --graph on" "--experts 4 --batch 512" "--ddp --sync-bn --experts 4 --batch 512" "--ddp --sync-bn --batch 1024" "--ddp --sync-bn --batch 1024 --graph on"; do
  n=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py $args --steps 60 --warmup 10 --other-steps 0 --no-cpu-baseline > $O/b_$n.json 2> $O/b_$n.err || exit 1
  python -c "import json;d=json.load(open('$O/b_$n.json'));print('$args', d['value'], d['ms_per_step'], d['step_launch'])"
done
timeout -k 10 400 python -u bench.py --arch neutron56 --experts 8 --batch 4096 --steps 5 --warmup 2 --other-steps 0 --no-cpu-baseline --no-probe > $O/b_n56.json 2> $O/b_n56.err || exit 1
python -c "import json;d=json.load(open('$O/b_n56.json'));print('n56 E8 B4096', d['value'], d['ms_per_step'], d['step_launch'])"
