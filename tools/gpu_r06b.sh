cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06b
timeout -k 10 120 python -u tools/ddp_e4_probe.py 4 512 1 1 > gpurun_out/r06b/own_fork.log 2>&1; echo "own_fork rc=$?"
tail -5 gpurun_out/r06b/own_fork.log
