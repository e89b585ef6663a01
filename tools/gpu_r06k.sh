# broad GPU regression after the ring helper move + the wave-specialised WGRAD (default on)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06k
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_f32_split_gpu.py tests/test_f32_ring_gpu.py tests/test_dynamic_rows_gpu.py tests/test_train_step_gpu.py tests/test_b512_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_fork_graph_gpu.py tests/test_grads_gpu.py > gpurun_out/r06k/t.log 2>&1; rc=$?; tail -3 gpurun_out/r06k/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --other-steps 30 --no-cpu-baseline > gpurun_out/r06k/bench.json 2> gpurun_out/r06k/bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r06k/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel'][:40],d['perf_bf16']['value'])"
