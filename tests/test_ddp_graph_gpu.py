"""The data-parallel train step (expertsim/train/ddp.py, RCCL) captured as one HIP graph
(expertsim/graph.py) replays exactly the eager data-parallel steps.

One process, an RCCL ("nccl") process group of world size 1 on the test box's GPU (RCCL needs one
device per rank, and the box has one): the step then runs every data-parallel code path -- SyncBN
statistics and backward sums through collectives, the bucketed gradient all-reduces on the process
group's stream, the metric all-gather -- inside the capture.  Model A runs 3 eager DP steps; model B
(same seed) runs 1 eager warm-up step, is captured, and replayed twice.  fp32 parity mode: the
replayed steps must land on the same bits as the eager ones (metrics, every parameter).  The worker
runs in a spawned process so the process group does not outlive the test.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q, E, B):
    import sys
    from conftest import PKG_DIR, REPO
    for p in (PKG_DIR, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        import bench
        from expertsim.graph import StepGraph, graph_supported
        from expertsim.train.ddp import DataParallel
        from expertsim.utils.synthetic import make_batch
        b = make_batch(B, "neutron", seed=5)
        t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
        real = t["real_images"].unsqueeze(1).contiguous()
        runs = []
        for mode in ("eager", "graph"):
            moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, dev)
            moe.ddp = DataParallel(sync_bn=True)
            moe.rank = 0
            assert graph_supported(moe)
            args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, dev)
            if mode == "eager":
                for _ in range(3):
                    m = moe.train_step(*args)
            else:
                sg = StepGraph(moe, args, warmup=1)
                if E > 1:      # the experts forked onto their own streams and communicators
                    assert moe._side is not None and len(moe.ddp.expert_groups) == E
                for _ in range(2):
                    m = sg.replay()
                sg.sync_host_state([*og, *od, *oa, orr])
                assert moe.step_count == 3
            torch.cuda.synchronize()
            runs.append(({k: float(v) for k, v in m.items()},
                         # numpy: pickled by value (torch CPU tensors travel as shared-memory fds,
                         # which need the worker alive when the parent unpickles them)
                         {n: p.detach().cpu().numpy().copy() for n, p in moe.state_dict().items()}))
        q.put((runs, None))
    except Exception as e:         # report instead of hanging the parent
        q.put((None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("E,B", [(1, 64), (4, 512)])
def test_ddp_graph_replay_matches_eager_rccl_world1(E, B):
    """E = 4, B = 512 with SyncBN (BASELINE configs[3]'s per-GPU shard): the experts' programs run
    forked on their own streams, each with its own RCCL communicator, in the eager steps and inside
    the captured graph alike."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, E, B))
    p.start()
    try:
        # (the worker takes ~15 s; a stuck RCCL init is reported within 150 s, before a runner's
        # silence limit would take it for a hung GPU)
        runs, err = q.get(timeout=150)
        p.join(timeout=30)
    finally:
        if p.is_alive():           # a stuck worker must not outlive the test holding the GPU
            p.kill()
            p.join(timeout=30)
    assert err is None, err
    (ma, pa), (mb, pb) = runs
    assert ma == mb, (ma, mb)
    diff = [n for n in pa if not np.array_equal(pa[n], pb[n])]
    assert not diff, diff
