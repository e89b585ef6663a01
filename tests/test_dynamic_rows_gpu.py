"""Dynamic rows (multi-expert steps, hip.live_rows): kernels on a capacity-N batch with a device live
count n must give the static kernels' results on the first n samples, never read the padding.

The padding samples of every input are NaN: a kernel that lets one into a live result (a product, a
statistic, a weight-gradient sum) fails the comparison.  Each case runs the op twice -- on the
N-sample buffers inside ``hip.live_rows(N, n)`` and on n-sample copies without it -- and compares the
live rows / the reductions.  Tolerance: the reductions may split their K range differently (the
live-count split is recomputed on the device), so 1e-5 relative of max|ref| (fp32), 2e-2 (bf16);
elementwise results are expected bitwise equal up to that same bound.
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _env():
    from expertsim import hip, layers
    hip.lib()
    return hip, layers


def _live(hip, N, n):
    rows = torch.tensor([n], dtype=torch.int32, device=DEV)
    active = torch.tensor([1 if n > 1 else 0], dtype=torch.int32, device=DEV)
    return hip.live_rows(N, rows, active), rows


def _act_nan(layers, x_live, N, dtype):
    """NHWC Act of N samples: the first n from x_live (NCHW), the rest NaN."""
    n, Cc, H, W = x_live.shape
    a = layers.Act.nhwc(N, Cc, H, W, dtype, DEV)
    a.t.fill_(float("nan"))
    a.t[: n * H * W * Cc].copy_(x_live.permute(0, 2, 3, 1).reshape(-1).to(dtype))
    return a


def _act(layers, x, dtype):
    n, Cc, H, W = x.shape
    a = layers.Act.nhwc(n, Cc, H, W, dtype, DEV)
    a.t.copy_(x.permute(0, 2, 3, 1).reshape(-1).to(dtype))
    return a


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-12))


CONV = [
    # (N, n, Cin, H, W, Cout, k, stride, pad, upsample)
    (70, 37, 128, 13, 13, 256, 3, 1, 0, (2, 2)),    # neutron G conv_layers.0 (sub-pixel ring)
    # conv_layers.5 at an E = 4, B = 512 expert's scale: 256-row tiles over 16-image groups (the
    # dynamic-rows row order), 203 live = 12 whole groups + 11 images of a 13th
    (512, 203, 256, 24, 24, 128, 3, 1, 0, (2, 2)),
    (70, 37, 128, 46, 46, 64, 2, 1, 0, None),       # conv_layers.9 (ring / split-fp32 col WGRAD)
    (70, 70, 128, 46, 46, 64, 2, 1, 0, None),       # every row live
    (70, 0, 128, 46, 46, 64, 2, 1, 0, None),        # no row live
    (40, 9, 64, 45, 45, 1, 2, 1, 0, None),          # conv_layers.13 (thin kernels)
    (40, 9, 1, 44, 44, 32, 3, 1, 0, None),          # Cin = 1 (thin)
    (40, 17, 32, 21, 21, 16, 3, 1, 0, None),        # D conv_layers.4 (generic igemm)
    (40, 17, 256, 1, 1, 1024, 1, 1, 0, None),       # a linear (generic / split-K det)
    (512, 203, 256, 1, 1, 1024, 1, 1, 0, None),     # a wide linear: FWD over 16-sample pixel blocks
]


@pytest.mark.parametrize("case", CONV)
@pytest.mark.parametrize("mode", ["f32_split", "f32_exact", "bf16"])
def test_conv_dynamic_rows(case, mode):
    hip, layers = _env()
    N, n, Cin, H, W, Cout, k, stride, pad, up = case
    dtype = torch.bfloat16 if mode == "bf16" else torch.float32
    layers.set_deterministic(mode != "bf16")
    layers.set_f32_split(mode == "f32_split")
    g = torch.Generator().manual_seed(7)
    w = torch.nn.Parameter((torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).to(DEV))
    b = torch.nn.Parameter(torch.randn(Cout, generator=g).to(DEV) * 0.1)
    ups = layers.Upsample((H, W), scale=up) if up else None
    op = layers.ConvOp(w, b, stride=stride, pad=pad, upsample=ups)
    x = torch.randn(max(n, 1), Cin, H, W, generator=g)[:n]
    ref_x = _act(layers, x, dtype) if n else None
    ctx, _ = _live(hip, N, n)
    xin = _act_nan(layers, x, N, dtype)
    with ctx:
        y = op.fwd(xin, bn_stats=mode != "bf16")
    P, Q = y.dims[2], y.dims[3]
    dyl = torch.randn(max(n, 1), Cout, P, Q, generator=g)[:n]
    dy = _act_nan(layers, dyl, N, dtype)
    dw = torch.zeros_like(w)
    db = torch.zeros_like(b)
    with ctx:
        dx = op.dgrad(dy, xin)
        op.wgrad(dy, xin, dw, db, beta=0.0)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    if n == 0:
        assert float(dw.abs().max()) == 0.0 and float(db.abs().max()) == 0.0
        return
    yr = op.fwd(ref_x)
    dyr = _act(layers, dyl, dtype)
    dwr = torch.zeros_like(w)
    dbr = torch.zeros_like(b)
    dxr = op.dgrad(dyr, ref_x)
    op.wgrad(dyr, ref_x, dwr, dbr, beta=0.0)
    torch.cuda.synchronize()
    live = lambda a: a.torch_nchw()[:n].float()
    assert _rel(live(y), yr.torch_nchw().float()) <= tol
    if y.bn_part is not None:   # fused BatchNorm partials of the FWD epilogue: the live rows only
        part, chunks = y.bn_part
        st = torch.empty(3, Cout, device=DEV)
        hip.call("es_norm_stats_merge", hip.ptr(part), chunks, Cout, hip.ptr(st), hip.stream_ptr())
        yv = yr.torch_nchw().double().permute(1, 0, 2, 3).reshape(Cout, -1)
        mu = yv.mean(1)
        assert torch.equal(st[0].cpu(), torch.full((Cout,), float(yv.shape[1])))
        assert _rel(st[1].cpu(), mu.cpu()) <= 1e-5
        assert _rel(st[2].cpu(), ((yv - mu[:, None]) ** 2).sum(1).cpu()) <= 1e-4
    assert _rel(live(dx), dxr.torch_nchw().float()) <= tol
    assert _rel(dw, dwr) <= tol and _rel(db, dbr) <= tol
    assert torch.isfinite(dw).all() and torch.isfinite(db).all()


NORM = [
    # (kind, groups, N, n, C, H, W, dropout)
    ("bn", 1, 60, 23, 64, 13, 13, 0.2),     # fast NHWC BatchNorm + dropout + LeakyReLU
    ("bn", 1, 60, 23, 256, 1, 1, 0.2),      # BatchNorm1d of a linear
    ("bn", 1, 60, 0, 64, 5, 5, 0.0),        # no live row
    ("gn", 8, 60, 23, 32, 10, 10, 0.0),     # GroupNorm (fast: z = sample)
    ("ln", 1, 60, 23, 128, 1, 1, 0.0),      # LayerNorm (segred)
]


@pytest.mark.parametrize("case", NORM)
@pytest.mark.parametrize("sync", [False, True])
def test_norm_dynamic_rows(case, sync):
    hip, layers = _env()
    kind, groups, N, n, Cc, H, W, p = case
    if sync and kind != "bn":
        pytest.skip("SyncBN is BatchNorm only")
    layers.set_deterministic(True)
    K = {"bn": hip.NORM_BN, "gn": hip.NORM_GN, "ln": hip.NORM_LN}[kind]
    g = torch.Generator().manual_seed(11)
    gamma = (1 + 0.1 * torch.randn(Cc, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(Cc, generator=g)).to(DEV)

    def make():
        rm, rv = torch.zeros(Cc, device=DEV), torch.ones(Cc, device=DEV)
        nbt = torch.zeros((), dtype=torch.int64, device=DEV)
        return layers.NormOp(K, gamma, beta, groups=groups, running_mean=rm, running_var=rv,
                             num_batches=nbt if kind == "bn" else None)

    def chain():
        d = hip.dropout_struct(p, seed=5, stream=3, enabled=p > 0)
        return hip.chain_struct(hip.ACT_LRELU, 0.1, d)

    class Sync:       # one rank: the collectives are identities, the global count is n
        world = 1

        def __init__(self):
            self.cnt = torch.tensor([float(n)], device=DEV)

        def all_gather(self, t):
            return t.unsqueeze(0).contiguous()

        def all_reduce_(self, t):
            return t

        def global_count_ptr(self):
            return hip.ptr(self.cnt)

    x = 2 + torch.randn(max(n, 1), Cc, H, W, generator=g)[:n]
    dyl = torch.randn(max(n, 1), Cc, H, W, generator=g)[:n]
    ctx, _ = _live(hip, N, n)
    nm = make()
    dg, dbt, ds = torch.zeros(Cc, device=DEV), torch.zeros(Cc, device=DEV), torch.zeros(Cc, device=DEV)
    xin, dy = _act_nan(layers, x, N, torch.float32), _act_nan(layers, dyl, N, torch.float32)
    ch = chain()
    layers.set_norm_sync(Sync() if sync else None)
    try:
        with ctx:
            y, st = nm.fwd(xin, ch)
            dx = nm.bwd(xin, st, ch, dy, dgamma=dg, dbeta=dbt, dsum=ds)
    finally:
        layers.set_norm_sync(None)
    torch.cuda.synchronize()
    if n == 0:
        assert float(dg.abs().max()) == 0.0 and float(nm.rm.abs().max()) == 0.0   # running stats untouched
        if kind == "bn":
            assert int(nm.nbt) == 0                                               # (active = 0: no count)
        return
    nr = make()
    dgr, dbr, dsr = torch.zeros(Cc, device=DEV), torch.zeros(Cc, device=DEV), torch.zeros(Cc, device=DEV)
    xr, dyr = _act(layers, x, torch.float32), _act(layers, dyl, torch.float32)
    chr_ = chain()
    yr, str_ = nr.fwd(xr, chr_)
    dxr = nr.bwd(xr, str_, chr_, dyr, dgamma=dgr, dbeta=dbr, dsum=dsr)
    torch.cuda.synchronize()
    live = lambda a: a.torch_nchw()[:n]
    assert _rel(live(y), yr.torch_nchw()) <= 1e-5
    assert _rel(live(dx), dxr.torch_nchw()) <= 1e-5
    assert _rel(dg, dgr) <= 1e-5 and _rel(dbt, dbr) <= 1e-5
    # sum(dx) per channel: analytically 0 after a BatchNorm (rounding noise), compared absolutely
    assert float((ds - dsr).abs().max()) <= 1e-5 * float(dxr.torch_nchw().abs().sum()) / Cc
    if kind == "bn":
        assert _rel(nm.rm, nr.rm) <= 1e-6 and _rel(nm.rv, nr.rv) <= 1e-6


def test_batched_batchnorm_counts_multi_expert():
    """Dynamic rows: an expert program's BatchNorm num_batches_tracked increments are applied on the
    device in one launch at its end (layers.batch_live_counts -> es_counters_add_i64_if), gated on the
    expert's active flag.  After two E = 3 steps every generator BatchNorm of an expert that trained in
    both counts 4 (two generator forwards per step, moe.py:145,538), every aux BatchNorm 2, and the
    counts equal the per-forward launches' (the unbatched path)."""
    import bench
    from expertsim import layers
    from expertsim.utils.synthetic import make_batch
    b = make_batch(96, "neutron", seed=4)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()
    counts = []
    for batched in (True, False):
        moe, (og, od, oa, orr), cfg = bench.build("neutron", 3, "fp32", 11, torch.device(DEV))
        moe.expert_graphs = False
        orig = layers.batch_live_counts
        if not batched:
            class _Off:
                def __enter__(self):
                    return self

                def __exit__(self, *a):
                    return False
            import expertsim.models.moe as M
            M.batch_live_counts = _Off
        try:
            args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, DEV)
            for _ in range(2):
                m = moe.train_step(*args)
        finally:
            import expertsim.models.moe as M
            M.batch_live_counts = orig
        torch.cuda.synchronize()
        nbt = {n: int(v) for n, v in moe.state_dict().items() if n.endswith("num_batches_tracked")}
        counts.append(nbt)
        active = [float(m[f"n_choosen_experts_mean_epoch_{i}"]) > 1 for i in range(3)]
        for n, v in nbt.items():
            e = int(n.split(".")[1])
            if n.startswith("generators.") and active[e]:
                assert v in (2, 4), (n, v)      # 2 per step the expert trained
            if n.startswith("aux_regs.") and active[e]:
                assert v in (1, 2), (n, v)
    assert counts[0] == counts[1]
