#!/bin/bash
# E>1 roofline probe: bench lines for E=4 B=512 (headline-style) and the default headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --experts 4 --batch 512 --steps 10 --warmup 5 > gpurun_out/r06p_e4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --experts 4 --batch 2048 --steps 5 --warmup 3 > gpurun_out/r06p_e4b2048.log 2>&1
