#!/bin/bash
# bf16 B = 512 (configs[1]) and B = 1024 kernel traces of graph-replayed steps
set -o pipefail
mkdir -p gpurun_out/r06t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06t/b512 -o run -- python3 tools/prof_step.py --experts 1 --batch 512 --precision bf16 --steps 20 > gpurun_out/r06t/b512.log 2>&1 &&
timeout -k 10 300 python3 bench.py --batch 512 --precision bf16 --steps 100 --warmup 10 --other-steps 20 --no-cpu-baseline > gpurun_out/r06t/bench_b512_bf16.json 2> gpurun_out/r06t/bench_b512_bf16.err &&
timeout -k 10 400 python3 bench.py --arch neutron56 --experts 8 --batch 4096 --steps 3 --warmup 2 --other-steps 0 --no-cpu-baseline > gpurun_out/r06t/bench_n56.json 2> gpurun_out/r06t/bench_n56.err &&
bash tools/gpu_traffic32s.sh
