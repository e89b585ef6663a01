cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06d
TORCH_NCCL_CUDA_EVENT_CACHE=0 timeout -k 10 100 python -u tools/ddp_e4_probe.py 4 512 1 1 > gpurun_out/r06d/nocache.log 2>&1; echo "nocache rc=$?"
grep "^\[\|exception" gpurun_out/r06d/nocache.log | tail -4
timeout -k 10 100 python -u tools/ddp_e4_probe.py 4 512 0 1 > gpurun_out/r06d/main_fork.log 2>&1; echo "main_fork rc=$?"
grep "^\[\|exception" gpurun_out/r06d/main_fork.log | tail -4
