#!/bin/bash
# Data-parallel bench rehearsals on a 1-GPU box: 1-rank RCCL (the nccl code path) and 2 / 4 gloo
# ranks sharing the GPU (the N>1 control flow: collectives, max-over-ranks timing, rank-0 JSON).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-ddp}
run() {
    local name=$1; shift
    timeout -k 10 240 "$@" > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err
    local rc=$?
    echo "$name rc=$rc"
    return $rc
}
run nccl1 python -u bench.py --ddp --steps 20 --other-steps 5 --no-cpu-baseline &&
run nccl1_sync python -u bench.py --ddp --sync-bn --steps 20 --other-steps 0 --no-cpu-baseline --no-probe &&
run gloo2 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --backend gloo --batch 256 --steps 10 --warmup 3 &&
run gloo2_e4 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29612 bench.py --gpus 2 --backend gloo --batch 256 --experts 4 --steps 10 --warmup 3 --no-probe
