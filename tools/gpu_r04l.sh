# multi-expert cost: E = 4 vs E = 1 at B = 512 fp32 (per-image), plus a kernel trace of E = 4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python bench.py --experts 4 --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/e4_r04l.json 2> $O/e4_r04l.err || exit $?
timeout -k 10 300 python bench.py --experts 1 --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/e1_r04l.json 2> $O/e1_r04l.err || exit $?
timeout -k 10 300 python bench.py --experts 4 --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/e4b_r04l.json 2> $O/e4b_r04l.err || exit $?
bash tools/gpu_prof_bench.sh r04l_e4 --experts 4 --batch 512 --steps 10 --warmup 3 --other-steps 0 --no-cpu-baseline --no-probe
