set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_step_gpu.py tests/test_b512_gpu.py tests/test_grads_gpu.py tests/test_f32_ring_gpu.py tests/test_f32_split_gpu.py tests/test_kernels_gpu.py > gpurun_out/t_a.log 2>&1; rc=$?; tail -5 gpurun_out/t_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/op_times.py --batch 1024 > gpurun_out/ops_f32_b1024_c4.md || exit 1
grep "A0.c4\|labelled" gpurun_out/ops_f32_b1024_c4.md
timeout -k 10 200 python -u tools/prof_step.py --experts 1 --batch 1024 --steps 30 || exit 1
bash tools/gpu_pmc_step.sh r05_bf16_b1024 --experts 1 --batch 1024 --precision bf16
