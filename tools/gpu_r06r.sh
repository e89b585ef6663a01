#!/bin/bash
# E = 4 B = 2048 bench line (dropout_ahead off, the default), then the opt-in draw under per-expert graphs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler -u bench.py --experts 4 --batch 2048 --steps 5 --warmup 3 --other-steps 10 > gpurun_out/r06r_e4b2048.log 2>&1 &&
timeout -k 10 300 python -X faulthandler -u tools/cfg_ab.py --key train.dropout_ahead --vals false,true --experts 4 --batch 512 --rounds 2 --reps 20 > gpurun_out/r06r_ab_e4.log 2>&1
