#!/bin/bash
# bf16 image-chunked ring launches: kernel tests, bf16 / multi-expert parity, configs[3] bench line
set -o pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bf16_chunks_gpu.py tests/test_kernels_gpu.py tests/test_dropout_ahead_gpu.py tests/test_bf16_stats_gpu.py tests/test_dynamic_rows_gpu.py > gpurun_out/r06s/tests.log 2>&1 &&
timeout -k 10 300 python -X faulthandler -u bench.py --experts 4 --batch 2048 --steps 5 --warmup 3 --other-steps 10 > gpurun_out/r06s/b_e4b2048.json 2> gpurun_out/r06s/b_e4b2048.err &&
timeout -k 10 300 python -X faulthandler -u bench.py --steps 50 --warmup 10 > gpurun_out/r06s/b_b1024.json 2> gpurun_out/r06s/b_b1024.err
