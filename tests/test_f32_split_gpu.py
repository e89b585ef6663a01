"""Split-fp32 MFMA arithmetic of the ring convolutions (train.fp32_mfma: split).

Every fp32 operand is the exact sum of three bf16 planes (x0 = rne(x), x1 = rne(x - x0),
x2 = x - x0 - x1) and a product is the sum of the six plane products with p + q <= 2 on
v_mfma_f32_16x16x32_bf16, accumulated in fp32 (conv_mfma.hip, split8 / mfma_split6).  The dropped
terms are below 2^-23 |a b| per product, so the result must be as close to the fp64 reference as
the exact fp32 MFMA result is.

Reference: torch CPU fp64 of upsample + conv2d (neutron/generator.py:23-35, proton/generator.py:26-38).
Tolerance: 2e-5 of max|ref| (the exact fp32 path's bound), and at most 2x the exact fp32 path's own
error + 1e-6; bitwise equality of two runs and of image-chunked launches (fixed order).
"""
import pytest
import torch

from test_f32_ring_gpu import CASES, _ref, _run
from test_kernels_gpu import _hip, rel

pytestmark = pytest.mark.gpu


@pytest.fixture
def det():
    from expertsim import layers
    old = layers.deterministic()
    layers.set_deterministic(True)
    yield
    layers.set_deterministic(old)
    layers.set_f32_split(False)


def _both(case, seed):
    from expertsim import layers
    x, w, b, gy, *ref = _ref(case, seed)
    layers.set_f32_split(False)
    exact = _run(case, x, w, b, gy)[1:]
    layers.set_f32_split(True)
    split = _run(case, x, w, b, gy)[1:]
    return ref, exact, split


# 64 output channels, taps x C a multiple of 512 without sub-pixel classes: the 64 x 512 split WGRAD
# tiles, whose B lanes carry taps of their own (pad 1: boundary taps masked per lane)
MT_CASES = [(9, 128, 20, 12, 64, 2, 1, 1, None), (7, 64, 11, 9, 64, 4, 2, 1, None)]


@pytest.mark.parametrize("case", CASES + MT_CASES)
def test_split_matches_fp64(case, det):
    _hip()
    ref, exact, split = _both(case, 0)
    for r, e, s in zip(ref, exact, split):
        es, ee = rel(s.double(), r), rel(e.double(), r)
        assert es < 2e-5, (es, ee)
        assert es <= 2 * ee + 1e-6, (es, ee)


@pytest.mark.parametrize("case", CASES[:3])
def test_split_bitwise_rerun(case, det):
    from expertsim import layers
    _hip()
    x, w, b, gy, *_ = _ref(case, seed=3)
    layers.set_f32_split(True)
    r1 = _run(case, x, w, b, gy)[1:]
    r2 = _run(case, x, w, b, gy)[1:]
    for a, c in zip(r1, r2):
        assert torch.equal(a, c)


@pytest.mark.parametrize("case", [CASES[1], CASES[2]])
def test_split_image_chunks(case, det):
    from expertsim import layers
    hip = _hip()
    x, w, b, gy, *_ = _ref(case, seed=4)
    layers.set_f32_split(True)
    full = _run(case, x, w, b, gy)[1:]
    old = hip.lib().es_conv_set_f32_chunk(64)
    try:
        part = _run(case, x, w, b, gy)[1:]
    finally:
        hip.lib().es_conv_set_f32_chunk(old)
    assert torch.equal(full[0], part[0])
    assert torch.equal(full[1], part[1])
    assert rel(part[2], full[2]) < 1e-5


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("case", [(8, 128, 13, 13, 256, 3, 1, 0, 2), CASES[1], (8, 256, 24, 24, 128, 3, 1, 0, 2)])
def test_fused_bn_stats_consistency(case, split, det):
    """The conv epilogue's BatchNorm partials against the stored output (bias x30: channel means far
    from zero): the mean must reproduce the stored values' mean to a rounding floor,
    |mean - mean(y)| <= 1e-6 max(|mean(y)|, std(y)) (the normalised map then sums to ~0 per channel,
    which the analytically-zero conv-bias gradients depend on)."""
    _hip()
    from expertsim import hip, layers
    from expertsim.layers import ConvOp, NormOp, Upsample
    from test_kernels_gpu import DEV, from_act, to_act
    layers.set_f32_split(split)
    x, w, b, gy, *_ = _ref(case, seed=5)
    N, Cin, H, W, Cout, k, st, pad, up = case
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter((b * 30).to(DEV)), stride=st, pad=pad,
                upsample=Upsample((H, W), scale=(up, up)))
    ya = op.fwd(to_act(x, torch.float32), out_dtype=torch.float32, bn_stats=True)
    assert ya.bn_part is not None
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, invstd = NormOp(hip.NORM_BN, running_mean=rm, running_var=rv).stats(ya)
    yt = from_act(ya).double()
    m_ref = yt.mean(dim=(0, 2, 3))
    scale = torch.maximum(m_ref.abs(), 1.0 / invstd.cpu().double())
    err = ((mean.cpu().double() - m_ref).abs() / scale).max().item()
    assert err <= 1e-6, err


@pytest.mark.parametrize("case", [(256, 256, 24, 24, 128, 3, 1, 0, 2), (320, 128, 13, 13, 256, 3, 1, 0, 2),
                                  (256, 128, 46, 46, 64, 2, 1, 0, None)])
def test_split_large_tiles_match_exact(case, det):
    """Batches that select the 256-row tiles (the bench's kernels; the fp64 cases above are too small
    for them): split-fp32 fwd / dgrad / wgrad against the exact fp32 MFMA path (itself pinned to
    fp64 above) within 1e-5 of max|exact|."""
    from expertsim import layers
    _hip()
    N, Cin, H, W, Cout, k, st, pad, up = case
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g)
    Ho = (H * (up or 1) + 2 * pad - k) // st + 1
    Wo = (W * (up or 1) + 2 * pad - k) // st + 1
    gy = torch.randn(N, Cout, Ho, Wo, generator=g)
    layers.set_f32_split(False)
    exact = _run(case, x, w, b, gy)[1:]
    layers.set_f32_split(True)
    split = _run(case, x, w, b, gy)[1:]
    for e, s_ in zip(exact, split):
        assert rel(s_, e) < 1e-5


@pytest.mark.parametrize("B,Cin,K,split", [(512, 256, 2048, True), (1024, 256, 21632, True), (256, 64, 1152, True),
                                           (512, 256, 2048, False)])
def test_wide_linear_pixel_view(B, Cin, K, split, det):
    """A wide linear (the generators' fc2, neutron/generator.py:17) runs as a 1x1 conv over 16-row
    pixel blocks of the same memory (ConvOp._pixel_view) on the ring FWD, with the BatchNorm1d
    statistics from its epilogue: output against torch fp64 F.linear at the fp32 bound (2e-5 of
    max|ref|), equal to the plain-linear path within the same bound, statistics against torch."""
    from expertsim import layers
    from expertsim.layers import Act, ConvOp, NormOp
    hip = _hip()
    layers.set_f32_split(split)
    torch.manual_seed(11)
    x = torch.randn(B, Cin, device="cuda")
    w = torch.nn.Parameter(torch.randn(K, Cin, device="cuda") / Cin ** 0.5)
    b = torch.nn.Parameter(0.1 * torch.randn(K, device="cuda"))
    op = ConvOp(w, b)
    xa = Act.of(x)
    assert (op._pixel_view(xa) is not None) == split      # (fp32 exact MFMA: the plain path)
    y = op.fwd(xa, bn_stats=True)
    ref = torch.nn.functional.linear(x.double().cpu(), w.detach().double().cpu(), b.detach().double().cpu())
    got = y.rows2d().double().cpu()
    assert rel(got, ref) < 2e-5, rel(got, ref)
    if split:
        assert y.bn_part is not None                       # statistics from the ring epilogue
        old = layers._LIN_PIX
        layers._LIN_PIX = False
        try:
            plain = op.fwd(xa).rows2d().double().cpu()
        finally:
            layers._LIN_PIX = old
        assert rel(got, plain) < 2e-5
        rm, rv = torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
        bn = NormOp(hip.NORM_BN, torch.ones(K, device="cuda"), torch.zeros(K, device="cuda"), running_mean=rm,
                    running_var=rv, momentum=0.1, eps=1e-5)
        mean, invstd = bn.stats(y)
        assert rel(mean.double().cpu(), ref.mean(0)) < 1e-5
        assert rel(invstd.double().cpu(), torch.rsqrt(ref.var(0, unbiased=False) + 1e-5)) < 1e-5


def test_wide_linear_pixel_view_bf16():
    """The bf16 performance mode takes the same pixel-block layout for the generators' fc2: against
    torch fp32 F.linear of the bf16-rounded operands (1e-2 of max|ref|), and the BatchNorm1d
    statistics from the epilogue against torch on the kernel's own output."""
    from expertsim.layers import Act, ConvOp, NormOp
    hip = _hip()
    torch.manual_seed(12)
    B, Cin, K = 1024, 256, 21632
    x = torch.randn(B, Cin, device="cuda").bfloat16()
    w = torch.nn.Parameter(torch.randn(K, Cin, device="cuda") / Cin ** 0.5)
    b = torch.nn.Parameter(0.1 * torch.randn(K, device="cuda"))
    op = ConvOp(w, b)
    xa = Act.of(x)
    assert op._pixel_view(xa) is not None
    y = op.fwd(xa, bn_stats=True)
    assert y.bn_part is not None
    ref = torch.nn.functional.linear(x.float(), w.detach().bfloat16().float(), b.detach())
    got = y.rows2d().float()
    assert rel(got.cpu(), ref.cpu()) < 1e-2, rel(got.cpu(), ref.cpu())
    bn = NormOp(hip.NORM_BN, torch.ones(K, device="cuda"), torch.zeros(K, device="cuda"),
                running_mean=torch.zeros(K, device="cuda"), running_var=torch.ones(K, device="cuda"),
                momentum=0.1, eps=1e-5)
    mean, invstd = bn.stats(y)
    assert rel(mean.cpu(), got.mean(0).cpu()) < 1e-3
    assert rel(invstd.cpu(), torch.rsqrt(got.var(0, unbiased=False) + 1e-5).cpu()) < 1e-3


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[3], CASES[5], CASES[7],
                                  (130, 256, 24, 24, 128, 3, 1, 0, 2), (33, 128, 13, 13, 256, 3, 1, 0, 2)])
def test_wave_specialised_wgrad_bitwise(case, det):
    """wgrad_ws_kernel (waves 0-3 MFMA, waves 4-7 load + split, es_conv_set_wgrad_ws(1), the default)
    against wgrad_coop_kernel (every wave loads, splits and multiplies): the same planes, K order and
    products, so bitwise the same weight / bias gradients, and within the fp64 bound."""
    from expertsim import layers
    hip = _hip()
    x, w, b, gy, y, gx, gw, gb = _ref(case, seed=5)
    layers.set_f32_split(True)
    old = hip.lib().es_conv_set_wgrad_ws(0)
    try:
        coop = _run(case, x, w, b, gy)[3:]
        hip.lib().es_conv_set_wgrad_ws(1)
        wsk = _run(case, x, w, b, gy)[3:]
    finally:
        hip.lib().es_conv_set_wgrad_ws(old)
    assert torch.equal(coop[0], wsk[0]) and torch.equal(coop[1], wsk[1])
    assert rel(wsk[0].double(), gw) < 2e-5
