"""Data parallelism on the HIP path (expertsim/train/ddp.py) against the single-device step.

Two ranks share the one GPU of the test box (gloo process group: the collectives go through the
host; RCCL needs distinct devices).  Each rank trains on its half of a global batch of 96 with
``sync_bn=True`` — randomness at global sample indices, SyncBN, global SDI / router statistics,
averaged gradients, merged metrics — and the result is compared with ONE process running the
same seeds on the whole batch (fp32 parity mode, device RNG, no injection):

  * step 0: every metric <= 1e-4 relative (as the golden tests); parameters after the step
    |dp - p| <= 2 lr (Adam's first step turns rounding-level sign flips of tiny gradients into
    +-lr moves);
  * step 1: metrics <= 2e-2 relative (the reference's own step-1 sensitivity, see
    test_train_step_gpu.py); parameters <= 4 lr;
  * E = 1 and E = 3 (the router: global gate sums, summed router gradient, per-expert global
    sample offsets);
  * the per-rank-statistics mode (``sync_bn=False``, the default) runs and is reported.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
B_GLOBAL, STEPS, WORLD = 96, 2, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(E, B, rank=0, ddp=None, b_global=B_GLOBAL, steps=STEPS, expo=None):
    """expo: injected Exp(1) draws of the router's Gumbel noise for the GLOBAL batch (numpy
    [b_global, E]); this process reads its rows."""
    import bench
    from expertsim.utils.synthetic import make_batch
    dev = torch.device("cuda", 0)
    moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, dev)
    if ddp is not None:
        moe.ddp = ddp
        moe.rank = ddp.rank
    if expo is not None:
        mine = torch.from_numpy(expo[rank * B:(rank + 1) * B].copy())
        moe.gumbel_fn = lambda shape: mine
    out = []
    for s in range(steps):
        b = make_batch(b_global, "neutron", seed=70 + s)
        rows = slice(rank * B, (rank + 1) * B)
        t = {k: torch.from_numpy(v[rows].copy()).to(dev) for k, v in b.items()}
        m = moe.train_step(0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"],
                           t["intensity"], oa, og, od, orr, None, dev)
        torch.cuda.synchronize()
        if ddp is not None:
            # the overlapped / bucketed gradient all-reduces of the step cover every model's flat
            # gradient buffer exactly once (ddp.bucketer, ddp.allreduce_async)
            by_mod = {}
            for mod, lo, hi in ddp.issued:
                by_mod.setdefault(id(mod), (mod, []))[1].append((lo, hi))
            for mod, ranges in by_mod.values():
                ranges.sort()
                assert ranges[0][0] == 0 and ranges[-1][1] == mod.flat_grads.numel(), ranges
                assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:])), ranges
            assert len(by_mod) == 3 * E, len(by_mod)
            assert any(len(r) > 1 for _, r in by_mod.values())     # the generator's buckets
            ddp.issued.clear()
        params = {n: p.detach().double().cpu().numpy().copy() for n, p in moe.named_parameters()}
        out.append(({k: float(v) for k, v in m.items()}, params))
    lr = {"generators": cfg.model.generator.lr_g, "discriminators": cfg.model.discriminator.lr_d,
          "aux_regs": cfg.model.aux_reg.lr_a, "router": cfg.model.router.lr_r}
    return out, lr


def _worker(rank, world, port, q, E, sync, b_global=B_GLOBAL, steps=STEPS, expo=None):
    import sys
    from conftest import PKG_DIR, REPO
    for p in (PKG_DIR, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from expertsim.train.ddp import DataParallel
    try:
        res, _ = _run(E, b_global // world, rank, DataParallel(sync_bn=sync), b_global, steps, expo)
        q.put((rank, res, None))
    except Exception as e:         # report instead of hanging the parent
        q.put((rank, None, repr(e)))
    dist.destroy_process_group()


def _spawn(E, sync, world=WORLD, b_global=B_GLOBAL, steps=STEPS, expo=None):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, E, sync, b_global, steps, expo))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=400) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, r, err in res:
        assert err is None, (rank, err)
    return [r for _, r, _ in res]


def _deviation(single, dp, lr):
    out = []
    for s, ((ms, ps), (md, pd)) in enumerate(zip(single, dp)):
        mdev = max(abs(md[k] - v) / max(abs(v), 1e-3) for k, v in ms.items())
        pdev = max(float(np.max(np.abs(pd[n] - a))) / lr[n.split(".")[0]] for n, a in ps.items())
        out.append((mdev, pdev))
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("E", [1, 3])
def test_ddp_sync_bn_matches_single_device(E):
    single, lr = _run(E, B_GLOBAL)
    dp = _spawn(E, True)
    for (m0, p0), (m1, p1) in zip(dp[0], dp[1]):            # ranks agree on metrics and parameters
        assert m0 == m1
        assert all(np.array_equal(p0[n], p1[n]) for n in p0)
    dev = _deviation(single, dp[0], lr)
    local = _deviation(single, _spawn(E, False)[0], lr)
    print(f"E={E}: DP(sync-BN) vs single (metric rel, param / lr): {dev}; DP(per-rank BN): {local}")
    assert dev[0][0] <= 1e-4 and dev[0][1] <= 2.0 + 1e-3
    assert dev[1][0] <= 2e-2 and dev[1][1] <= 4.0 + 1e-3


@pytest.mark.timeout(900)
def test_ddp4_syncbn_e4_b2048_matches_single_device():
    """BASELINE configs[3] data parallel: 4 ranks x 512 (gloo on the one GPU, SyncBN, dynamic-rows
    multi-expert step) against ONE process on the global batch of 2048, step 0: every metric <= 1e-4
    relative, parameters <= 2 lr (Adam's first step), the ranks bitwise equal to each other."""
    single, lr = _run(4, 2048, b_global=2048, steps=1)
    dp = _spawn(4, True, world=4, b_global=2048, steps=1)
    for r in range(1, 4):
        assert dp[0][0][0] == dp[r][0][0]
        assert all(np.array_equal(dp[0][0][1][n], dp[r][0][1][n]) for n in dp[0][0][1])
    dev = _deviation(single, dp[0], lr)
    print("E=4 B=2048, 4-rank SyncBN vs single (metric rel, param / lr):", dev)
    assert dev[0][0] <= 1e-4 and dev[0][1] <= 2.0 + 1e-3


def _skewed_expo(sync, E=3, B=B_GLOBAL):
    """Gumbel Exp(1) draws that force the routing (an Exp draw of 1e-30 is a Gumbel of +69, far above
    any logit): rank 0's samples (the first half) go to experts 0 / 1 only -- or, for the per-rank
    BatchNorm mode, exactly one of them to expert 2 --, rank 1's samples to all three experts."""
    g = torch.Generator().manual_seed(9)
    expo = torch.empty(B, E).exponential_(generator=g)
    for j in range(B):
        if j < B // 2:
            k = 2 if (not sync and j == 0) else j % 2
        else:
            k = j % 3
        expo[j, k] = 1e-30
    return expo.numpy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sync", [True, False])
def test_ddp_rank_without_expert_samples(sync):
    """a rank that holds no sample (SyncBN) or a single sample (per-rank BatchNorm) of an
    expert that is active globally.  That rank runs the expert's program on zero live rows (BatchNorm
    partials of count 0, losses and metric weight 0, zero gradients) but joins every collective of
    the expert's communicator, so the ranks stay bitwise equal; with SyncBN the step equals the
    single-device step of the global batch (the same injected routing)."""
    E = 3
    expo = _skewed_expo(sync)
    dp = _spawn(E, sync, expo=expo)
    for (m0, p0), (m1, p1) in zip(dp[0], dp[1]):
        assert m0 == m1
        assert all(np.array_equal(p0[n], p1[n]) for n in p0)
        assert all(np.isfinite(v) for v in m0.values()), m0
    n2 = 16 + (0 if sync else 1)
    for m, _ in dp[0]:
        assert m["n_choosen_experts_mean_epoch_2"] == n2, m
    if sync:
        single, lr = _run(E, B_GLOBAL, expo=expo)
        dev = _deviation(single, dp[0], lr)
        print("rank 0 without expert-2 samples, SyncBN vs single (metric rel, param / lr):", dev)
        assert dev[0][0] <= 1e-4 and dev[0][1] <= 2.0 + 1e-3
        assert dev[1][0] <= 2e-2 and dev[1][1] <= 4.0 + 1e-3
    else:
        # expert 2 trained from rank 1's gradients (rank 0 contributed zeros through the same buckets)
        (_, p_first), (_, p_last) = dp[0][0], dp[0][-1]
        assert any(not np.array_equal(p_first[n], p_last[n]) for n in p_first if n.startswith("generators.2."))
