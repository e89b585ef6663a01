#!/bin/bash
# two-workgroup short-K DGRAD: bitwise / parity tests, whole-step A/B (fp32 B = 1024, E = 4 B = 512)
set -o pipefail
mkdir -p gpurun_out/r06ag
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_f32_split_gpu.py tests/test_f32_ring_gpu.py tests/test_train_step_gpu.py tests/test_b512_gpu.py tests/test_grads_gpu.py tests/test_dynamic_rows_gpu.py > gpurun_out/r06ag/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/cfg_ab.py --key es_conv_set_dgrad_occ2 --vals 0,1 --batch 1024 --rounds 4 --reps 30 > gpurun_out/r06ag/ab_b1024.log 2>&1 &&
timeout -k 10 300 python -u tools/cfg_ab.py --key es_conv_set_dgrad_occ2 --vals 0,1 --experts 4 --batch 512 --rounds 4 --reps 30 > gpurun_out/r06ag/ab_e4.log 2>&1
