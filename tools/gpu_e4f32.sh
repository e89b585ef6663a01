# fp32 (split) multi-expert cost: E=1 vs E=4 at B=512 on one GPU
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u bench.py --batch 512 --steps 30 --warmup 10 --other-steps 0 --no-cpu-baseline --no-probe > $O/e1_b512.json 2> $O/e1_b512.err || exit $?
timeout -k 10 500 python -u bench.py --batch 512 --experts 4 --steps 50 --warmup 120 --other-steps 0 --no-cpu-baseline --no-probe > $O/e4_b512.json 2> $O/e4_b512.err
