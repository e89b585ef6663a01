#!/bin/bash
# bf16 B = 512 (configs[1]) kernel trace of graph-replayed steps (csv stats)
set -o pipefail
mkdir -p gpurun_out/r06u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06u/b512 -o run -- python3 tools/prof_step.py --experts 1 --batch 512 --precision bf16 --steps 20 > gpurun_out/r06u/b512.log 2>&1
