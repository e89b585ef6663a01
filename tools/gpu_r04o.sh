# multi-expert steady state: E = 4 B = 512 fp32 after 300 warm-up steps (per-expert graph keys cached),
# against the 10-warm-up transient and E = 1 B = 512
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python bench.py --experts 4 --batch 512 --warmup 300 --steps 50 --other-steps 0 --no-cpu-baseline --no-probe > $O/e4ss_r04o.json 2> $O/e4ss_r04o.err || exit $?
timeout -k 10 300 python bench.py --experts 1 --batch 512 --steps 50 --other-steps 0 --no-cpu-baseline --no-probe > $O/e1_r04o.json 2> $O/e1_r04o.err || exit $?
