"""fp32 (parity-mode) ring convolutions and the deterministic weight gradient.

The generator convs of the parity mode run on the 8-wave LDS-DMA ring kernels with
v_mfma_f32_16x16x4_f32 (conv_mfma.hip, ``T = float``), the x2-upsample convs through the sub-pixel
decomposition (combined weights summed in fp32), and the weight gradients through
``es_conv2d_wgrad_det`` (per-split partials + one ordered reduce, no float atomics).

Reference: torch CPU fp64 of upsample + conv2d (neutron/generator.py:23-35, proton/generator.py:26-38).
Tolerance: 2e-5 of max|ref| (an exact fp32 FMA chain over K <= 4608 plus the ~1e-7 rounding of the
summed sub-pixel weights), and bitwise equality of two runs (the deterministic reductions).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_kernels_gpu import DEV, _hip, from_act, rel, to_act

pytestmark = pytest.mark.gpu

CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, upsample factor or None)
    (8, 128, 13, 13, 256, 3, 1, 0, 2),    # neutron G conv_layers.0 (sub-pixel)
    (67, 256, 24, 24, 128, 3, 1, 0, 2),   # neutron G conv_layers.5 (sub-pixel), ragged image groups
    (70, 128, 46, 46, 64, 2, 1, 0, None),  # neutron G conv_layers.9
    (5, 512, 18, 10, 256, 4, 1, 1, 2),    # proton G conv_layers.1 (4x4, pad 1: unequal class geometry)
    (9, 128, 56, 30, 64, 3, 1, 1, None),  # proton G conv_layers.8 (3x3 pad 1)
    (12, 256, 16, 16, 128, 3, 1, 0, 2),   # neutron56 G conv_layers.5 shape family
    (9, 64, 7, 4, 64, 5, 1, 2, None),     # proton A res2.conv2 (64 x 64 WGRAD tiles)
    (6, 64, 14, 8, 128, 3, 1, 1, None),   # neutron A conv3 family (128 x 64 WGRAD tiles)
]


def _ref(case, seed=0):
    N, Cin, H, W, Cout, k, st, pad, up = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    xu = F.interpolate(xr, scale_factor=up, mode="nearest") if up else xr
    y = F.conv2d(xu, wr, br, st, pad)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    return x.float(), w.float(), b.float(), gy.float(), y.detach(), xr.grad, wr.grad, br.grad


def _run(case, x, w, b, gy):
    from expertsim.layers import ConvOp, Upsample
    N, Cin, H, W, Cout, k, st, pad, up = case
    upsample = Upsample((H, W), scale=(up, up)) if up else None
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=st, pad=pad, upsample=upsample)
    xa = to_act(x, torch.float32)
    ya = op.fwd(xa, out_dtype=torch.float32)
    gya = to_act(gy, torch.float32)
    dxa = op.dgrad(gya, xa, dx_dtype=torch.float32)
    dw = torch.zeros(Cout, Cin, k, k, device=DEV)
    db = torch.zeros(Cout, device=DEV)
    op.wgrad(gya, xa, dw, db, beta=1.0)
    torch.cuda.synchronize()
    return op, from_act(ya), from_act(dxa), dw.cpu(), db.cpu()


@pytest.fixture
def det():
    from expertsim import layers
    old = layers.deterministic()
    layers.set_deterministic(True)
    yield
    layers.set_deterministic(old)


@pytest.mark.parametrize("case", CASES)
def test_f32_ring_matches_fp64(case, det):
    _hip()
    x, w, b, gy, y, gx, gw, gb = _ref(case)
    op, ya, dxa, dw, db = _run(case, x, w, b, gy)
    if case[8]:
        from expertsim.layers import Act
        assert op.subpixel(op.desc(Act.nhwc(*x.shape, torch.float32, DEV)), torch.float32)
    assert rel(ya.double(), y) < 2e-5
    assert rel(dxa.double(), gx) < 2e-5
    assert rel(dw.double(), gw) < 2e-5
    assert rel(db.double(), gb) < 2e-5


@pytest.mark.parametrize("case", CASES[:3])
def test_f32_ring_bitwise_rerun(case, det):
    """Deterministic mode: two runs of fwd / dgrad / wgrad give identical bits."""
    _hip()
    x, w, b, gy, *_ = _ref(case, seed=3)
    r1 = _run(case, x, w, b, gy)[1:]
    r2 = _run(case, x, w, b, gy)[1:]
    for a, c in zip(r1, r2):
        assert torch.equal(a, c)


@pytest.mark.parametrize("case", [CASES[1], CASES[2]])
def test_f32_ring_image_chunks(case, det):
    """The 1 GiB operand limit makes large fp32 batches launch over image chunks: forced small
    chunks give bit-identical FWD / DGRAD (the per-element K order does not depend on the tiling)
    and the same WGRAD to summation-order rounding."""
    hip = _hip()
    x, w, b, gy, y, gx, gw, gb = _ref(case, seed=4)
    full = _run(case, x, w, b, gy)[1:]
    old = hip.lib().es_conv_set_f32_chunk(64)
    try:
        part = _run(case, x, w, b, gy)[1:]
    finally:
        hip.lib().es_conv_set_f32_chunk(old)
    assert torch.equal(full[0], part[0])
    assert torch.equal(full[1], part[1])
    assert rel(part[2].double(), gw) < 2e-5
    assert rel(part[2], full[2]) < 1e-5


def test_f32_ring_fused_bn_stats(det):
    """fp32 FWD with the fused BatchNorm partials (es_conv2d_fwd_stats on the ring) against the
    statistics of the stored output."""
    _hip()
    from expertsim import hip
    from expertsim.layers import ConvOp, NormOp, Upsample
    case = CASES[1]
    x, w, b, gy, *_ = _ref(case, seed=5)
    N, Cin, H, W, Cout, k, st, pad, up = case
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=st, pad=pad,
                upsample=Upsample((H, W), scale=(up, up)))
    xa = to_act(x, torch.float32)
    ya = op.fwd(xa, out_dtype=torch.float32, bn_stats=True)
    assert ya.bn_part is not None
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, invstd = NormOp(hip.NORM_BN, running_mean=rm, running_var=rv).stats(ya)
    yt = from_act(ya).double()
    m_ref = yt.mean(dim=(0, 2, 3))
    v_ref = yt.var(dim=(0, 2, 3), unbiased=False)
    assert rel(mean.cpu().double(), m_ref) < 1e-5
    assert rel(invstd.cpu().double(), 1.0 / torch.sqrt(v_ref + 1e-5)) < 1e-5


@pytest.mark.parametrize("shape", [(9, 256, 1, 1, 64, 1), (130, 32, 21, 21, 16, 3), (33, 1, 44, 44, 32, 3),
                                   (17, 64, 45, 45, 1, 2)])
def test_wgrad_det_generic_paths(shape, det):
    """es_conv2d_wgrad_det on the shapes the ring does not take (linear, narrow D conv, thin Cin = 1 /
    Cout = 1 convs): per-split partials + ordered reduce, against torch fp64 and bitwise on rerun."""
    _hip()
    from expertsim.layers import ConvOp
    N, Cin, H, W, Cout, k = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / np.sqrt(Cin * k * k)
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(x, wr)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy)
    op = ConvOp(torch.nn.Parameter(w.float().to(DEV)), None)
    xa, gya = to_act(x.float()), to_act(gy.float())
    outs = []
    for _ in range(2):
        dw = torch.full((Cout, Cin, k, k), 0.5, device=DEV)
        op.wgrad(gya, xa, dw, None, beta=1.0)
        outs.append(dw.cpu())
    assert torch.equal(outs[0], outs[1])
    assert rel(outs[0].double() - 0.5, wr.grad) < 2e-5


@pytest.mark.parametrize("shape", [(300, 21632, 256), (500, 1305, 128)])
def test_linear_det_splitk(shape, det):
    """Long-K fp32 linears (the generator's fc2 dgrad, K = 21632; the discriminator fc1 forward,
    K = 1305): deterministic split-K (es_conv2d_fwd_det / es_conv2d_dgrad_det), against torch fp64
    and bitwise on rerun."""
    _hip()
    from expertsim.layers import Act, ConvOp
    N, Fin, Fout = shape
    g = torch.Generator().manual_seed(12)
    x = torch.randn(N, Fin, generator=g, dtype=torch.float64)
    w = torch.randn(Fout, Fin, generator=g, dtype=torch.float64) / np.sqrt(Fin)
    b = torch.randn(Fout, generator=g, dtype=torch.float64)
    gy = torch.randn(N, Fout, generator=g, dtype=torch.float64)
    op = ConvOp(torch.nn.Parameter(w.float().to(DEV)), torch.nn.Parameter(b.float().to(DEV)))
    xa = Act.of(x.float().to(DEV).contiguous())
    gya = Act.of(gy.float().to(DEV).contiguous())
    outs = []
    for _ in range(2):
        y = op.fwd(xa, out_dtype=torch.float32)
        dx = op.dgrad(gya, xa, dx_dtype=torch.float32)
        torch.cuda.synchronize()
        outs.append((y.rows2d().cpu(), dx.rows2d().cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert rel(outs[0][0].double(), x @ w.T + b) < 2e-5
    assert rel(outs[0][1].double(), gy @ w) < 2e-5
