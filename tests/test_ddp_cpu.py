"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel plumbing.

The HIP train step itself needs a GPU; here the DataParallel bookkeeping that every rank runs is
exercised for real across two processes: global expert counts, the skip/participate decision,
flat-gradient SUM all-reduce and the 1/world scale handed to the fused Adam."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeModule:
    def __init__(self, rank):
        self.flat_grads = torch.full((1000,), float(rank + 1))


def _worker(rank, world, port, q):
    import sys
    from conftest import PKG_DIR
    sys.path.insert(0, PKG_DIR)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from expertsim.train.ddp import DataParallel
    ddp = DataParallel()
    # rank 0 routes 5 / 1 / 0 samples to experts 0..2, rank 1 routes 2 / 0 / 4
    local = {0: [5, 1, 0], 1: [2, 0, 4]}[rank]
    groups = [(e, None, c) for e, c in enumerate(local)]
    ddp.global_groups(groups, 6)
    counts = [ddp.global_count(e) for e in range(3)]
    active = [c > 1 for c in counts]
    m = _FakeModule(rank)
    ddp.allreduce_grads(m)
    q.put((rank, counts, active, ddp.global_batch, float(m.flat_grads[0]), m._grad_scale))
    dist.destroy_process_group()


def test_ddp_bookkeeping_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, active, gb, g0, scale in res:
        assert counts == [7, 1, 4]
        assert active == [True, False, True]
        assert gb == 12
        assert g0 == 3.0            # 1 + 2 summed; averaging happens inside Adam via grad_scale
        assert scale == 0.5
