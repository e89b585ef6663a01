#!/bin/bash
# dropout masks drawn ahead: parity tests, A/B fp32 / bf16 at the headline batch, E = 4 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dropout_ahead_gpu.py tests/test_train_step_gpu.py tests/test_b512_gpu.py > gpurun_out/r06q_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/cfg_ab.py --key train.dropout_ahead --vals false,true --batch 1024 --rounds 4 --reps 30 > gpurun_out/r06q_ab_fp32.log 2>&1 &&
timeout -k 10 300 python -u tools/cfg_ab.py --key train.dropout_ahead --vals false,true --batch 1024 --precision bf16 --rounds 4 --reps 40 > gpurun_out/r06q_ab_bf16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --experts 4 --batch 2048 --steps 5 --warmup 3 --other-steps 10 > gpurun_out/r06q_e4b2048.log 2>&1
