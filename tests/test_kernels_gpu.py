"""HIP kernel unit tests: each kernel against a plain PyTorch fp32 CPU reference of the same op.

Tolerances (fp32 mode): MFMA f32 is an exact fp32 FMA chain, so conv/linear results agree with
torch's CPU fp32 to within summation-order rounding: rel <= 2e-5 of max|ref| (K up to 4608).
bf16 mode: rel <= 2e-2 of max|ref| (bf16 operands, fp32 accumulation).
Dropout masks are integer-exact against the host Philox restatement.
"""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _hip():
    from expertsim import hip
    hip.lib()
    return hip


def to_act(x_nchw, dtype=torch.float32):
    from expertsim.layers import Act
    N, Cc, H, W = x_nchw.shape
    a = Act.nhwc(N, Cc, H, W, dtype, DEV)
    a.t.copy_(x_nchw.permute(0, 2, 3, 1).reshape(-1).to(dtype))
    return a


def from_act(a):
    return a.torch_nchw().float().cpu()


def rel(a, b):
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-12))


CONV_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, upsample(scale or size) or None)
    (2, 128, 13, 13, 256, 3, 1, 0, (2, 2)),       # neutron G conv_layers.0 (after up x2)
    (2, 256, 24, 24, 128, 3, 1, 0, (2, 2)),       # neutron G conv_layers.5
    (3, 128, 46, 46, 64, 2, 1, 0, None),          # neutron G conv_layers.9
    (3, 64, 45, 45, 1, 2, 1, 0, None),            # neutron G conv_layers.13
    (2, 1, 44, 44, 32, 3, 1, 0, None),            # D / A first conv (Cin = 1, direct kernels)
    (24, 1, 44, 44, 32, 3, 1, 0, None),           # same, many wgrad blocks
    (2, 1, 20, 18, 16, 3, 2, 1, None),            # Cin = 1 direct path, stride 2, pad 1, K = 16
    (2, 64, 55, 29, 1, 2, 1, 1, None),            # proton G conv_layers.11 (Cout = 1, pad 1)
    (2, 32, 21, 21, 16, 3, 1, 0, None),           # D conv_layers.4
    (37, 32, 21, 21, 16, 3, 1, 0, None),          # same, many 128x32 / 32x128 tiles and K splits
    (5, 24, 11, 9, 8, 3, 1, 1, None),             # narrow tiles with ragged M / N / K
    (2, 1, 56, 30, 32, 5, 2, 1, None),            # proton A conv1 (stride 2, pad 1)
    (2, 32, 26, 13, 32, 5, 2, 2, None),           # proton A res conv1
    (2, 32, 26, 13, 64, 1, 2, 0, None),           # proton A downsample 1x1 s2
    (2, 256, 35, 19, 128, 4, 1, 1, "56x30"),      # proton G conv_layers.5 (resize 35x19 -> 56x30)
    (2, 512, 18, 10, 256, 4, 1, 1, (2, 2)),       # proton G conv_layers.1
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_fwd_dgrad_wgrad(case, dtype):
    _hip()
    from expertsim.layers import ConvOp, Upsample, Act
    N, Cin, H, W, Cout, k, st, pad, up = case
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W)
    w = (torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).requires_grad_(True)
    b = torch.randn(Cout).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    if up is None:
        xu, upsample = xr, None
    elif up == "56x30":
        xu, upsample = F.interpolate(xr, size=(56, 30), mode="nearest"), Upsample((H, W), out_hw=(56, 30))
    else:
        xu, upsample = F.interpolate(xr, scale_factor=up, mode="nearest"), Upsample((H, W), scale=up)
    y = F.conv2d(xu, w, b, st, pad)
    gy = torch.randn_like(y)
    y.backward(gy)
    wp = torch.nn.Parameter(w.detach().to(DEV))
    bp = torch.nn.Parameter(b.detach().to(DEV))
    op = ConvOp(wp, bp, stride=st, pad=pad, upsample=upsample)
    xa = to_act(x, dtype)
    ya = op.fwd(xa, out_dtype=torch.float32)
    tol = 3e-5 if dtype == torch.float32 else 3e-2
    assert ya.dims == tuple(y.shape)
    assert rel(from_act(ya), y.detach()) < tol
    gya = to_act(gy, dtype)
    dxa = op.dgrad(gya, xa, dx_dtype=torch.float32)
    assert rel(from_act(dxa), xr.grad) < tol
    dw = torch.zeros(Cout, Cin, k, k, device=DEV)
    db = torch.zeros(Cout, device=DEV)
    op.wgrad(gya, xa, dw, db, beta=1.0)
    assert rel(dw.cpu(), w.grad) < tol
    assert rel(db.cpu(), b.grad) < tol


GLDS_CASES = [
    # bf16 shapes that take the LDS-DMA main loop (one tap x 64 channels per K-step)
    (6, 128, 13, 13, 256, 3, 1, 0, (2, 2)),       # G conv_layers.0: fwd + folded dgrad
    (3, 256, 24, 24, 128, 3, 1, 0, (2, 2)),       # G conv_layers.5
    (4, 128, 46, 46, 64, 2, 1, 0, None),          # G conv_layers.9 (Ng = 64 tile)
    (3, 128, 17, 15, 64, 3, 2, 1, None),          # stride 2 + padding
    (3, 128, 17, 15, 128, 3, 2, 1, None),         # stride 2 + padding, WGRAD on the DMA path
    (2, 512, 18, 10, 256, 4, 1, 1, (2, 2)),       # proton G conv_layers.1 (pad 1, up x2)
]


@pytest.mark.parametrize("case", GLDS_CASES)
def test_conv_glds_matches_register_path(case):
    """The LDS-DMA kernel and the register-staged kernel accumulate in the same order: the bf16
    fwd and dgrad outputs must be bit-identical (and both close to torch fp32)."""
    hip = _hip()
    from expertsim.layers import ConvOp, Upsample
    N, Cin, H, W, Cout, k, st, pad, up = case
    torch.manual_seed(5)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout)
    upsample = Upsample((H, W), scale=up) if up else None
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=st, pad=pad, upsample=upsample)
    xa = to_act(x, torch.bfloat16)
    outs = []
    gy = None
    try:
        for on in (1, 0):
            hip.lib().es_conv_set_glds(on)
            ya = op.fwd(xa, out_dtype=torch.bfloat16)
            if gy is None:
                gy = torch.randn(ya.dims, generator=torch.Generator().manual_seed(9))
            gya = to_act(gy, torch.bfloat16)
            dxa = op.dgrad(gya, xa, dx_dtype=torch.bfloat16)
            dw = torch.zeros(Cout, Cin, k, k, device=DEV)
            op.wgrad(gya, xa, dw, None, beta=1.0)
            outs.append((ya.t.clone(), dxa.t.clone(), dw.cpu()))
    finally:
        hip.lib().es_conv_set_glds(1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    # WGRAD: same per-split sums; only the order of the fp32 atomics across K splits differs
    assert rel(outs[0][2], outs[1][2]) < 1e-5
    wr = w.clone().requires_grad_(True)
    xu_ = F.interpolate(x, scale_factor=up, mode="nearest") if up else x
    F.conv2d(xu_, wr, b, st, pad).backward(gy.to(torch.bfloat16).float())
    assert rel(outs[0][2], wr.grad) < 3e-2
    xu = F.interpolate(x, scale_factor=up, mode="nearest") if up else x
    y = F.conv2d(xu, w, b, st, pad)
    assert rel(outs[0][0].float().cpu().view(y.shape[0], y.shape[2], y.shape[3], -1).permute(0, 3, 1, 2), y) < 3e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_linear_as_conv(dtype):
    _hip()
    from expertsim.layers import Act, ConvOp
    torch.manual_seed(1)
    for (B, fin, fout) in [(8, 19, 256), (64, 256, 21632), (5, 1305, 128), (7, 64, 1), (3, 9, 128)]:
        x = torch.randn(B, fin)
        w = torch.randn(fout, fin).requires_grad_(True) / np.sqrt(fin)
        w = w.detach().requires_grad_(True)
        b = torch.randn(fout).requires_grad_(True)
        xr = x.clone().requires_grad_(True)
        y = F.linear(xr, w, b)
        gy = torch.randn_like(y)
        y.backward(gy)
        op = ConvOp(torch.nn.Parameter(w.detach().to(DEV)), torch.nn.Parameter(b.detach().to(DEV)))
        xa = Act.of(x.to(DEV, dtype).contiguous())
        ya = op.fwd(xa, out_dtype=torch.float32)
        tol = 3e-5 if dtype == torch.float32 else 3e-2
        assert rel(ya.rows2d().cpu(), y.detach()) < tol
        gya = Act.of(gy.to(DEV, dtype).contiguous())
        dxa = op.dgrad(gya, xa, dx_dtype=torch.float32)
        assert rel(dxa.rows2d().cpu(), xr.grad) < tol
        dw = torch.zeros(fout, fin, device=DEV)
        db = torch.zeros(fout, device=DEV)
        op.wgrad(gya, xa, dw, db, beta=1.0)
        assert rel(dw.cpu(), w.grad) < tol
        assert rel(db.cpu(), b.grad) < tol


def _chain_ref(y, p, mask, act, dropout_first):
    lre = (lambda t: F.leaky_relu(t, 0.1)) if act == "lrelu" else (F.relu if act == "relu" else (lambda t: t))
    if mask is None:
        return lre(y)
    scale = torch.tensor(1.0) / torch.tensor(1.0 - p)
    if dropout_first:
        return lre(y * (mask.float() * scale))
    return lre(y) * (mask.float() * scale)


@pytest.mark.parametrize("kind", ["bn2d", "bn1d", "gn", "ln", "bn2d_hw4", "bn1d_c8", "bn2d_bf16",
                                  "gn_hw4", "gn_c16_bf16", "gn_generic"])
@pytest.mark.parametrize("drop", [False, True])
def test_norm_chain(kind, drop):
    hip = _hip()
    from expertsim.layers import Act, NormOp
    from expertsim.utils import philox
    torch.manual_seed(2)
    dtype = torch.bfloat16 if kind.endswith("bf16") else torch.float32
    if kind in ("bn2d", "bn2d_bf16"):
        x = torch.randn(4, 32, 9, 7) * 3 + 1.5          # H*W % 4 != 0 (per-element Philox)
    elif kind == "bn2d_hw4":
        x = torch.randn(3, 64, 8, 6) * 2 + 0.5          # H*W % 4 == 0 (4 rows per Philox call)
    elif kind == "bn1d_c8":
        x = torch.randn(7, 304) * 2 + 0.5               # linear BN1d, C % 8 == 0 (fast path)
    elif kind == "gn":
        x = torch.randn(3, 32, 6, 5) * 2 - 1            # fast GN path, H*W % 4 != 0
    elif kind == "gn_hw4":
        x = torch.randn(5, 32, 12, 11) * 2 - 1          # fast GN path, H*W % 4 == 0, cg = 4
    elif kind == "gn_c16_bf16":
        x = torch.randn(4, 16, 7, 9) * 2 + 0.3          # fast GN path, bf16, cg = 2
    elif kind == "gn_generic":
        x = torch.randn(3, 12, 5, 5) * 2 - 1            # C % 8 != 0: generic segment reduction
    else:
        x = torch.randn(6, 300) * 2 + 0.5
    groups = 4 if kind == "gn_generic" else 8
    gamma = torch.rand(x.shape[1]) + 0.5
    beta = torch.randn(x.shape[1])
    p, seed, stream = 0.2, 1234, 77
    mask = torch.from_numpy(philox.dropout_mask(tuple(x.shape), p, seed, stream)) if drop else None
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).float()                 # reference sees the bf16-rounded input
    xr = x.clone().requires_grad_(True)
    g_, b_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rm, rv = torch.zeros(x.shape[1]), torch.ones(x.shape[1])
    if kind.startswith("bn"):
        z = F.batch_norm(xr, rm, rv, g_, b_, True, 0.1, 1e-5)
        nk = hip.NORM_BN
    elif kind.startswith("gn"):
        z = F.group_norm(xr, groups, g_, b_, 1e-5)
        nk = hip.NORM_GN
    else:
        z = F.layer_norm(xr, (x.shape[1],), g_, b_, 1e-5)
        nk = hip.NORM_LN
    y = _chain_ref(z, p, mask, "lrelu", True)
    gy = torch.randn_like(y)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).float()
    y.backward(gy)
    xa = to_act(x, dtype) if x.dim() == 4 else Act.of(x.to(DEV, dtype).contiguous())
    dg = torch.zeros_like(gamma, device=DEV)
    dbt = torch.zeros_like(beta, device=DEV)
    rmd, rvd = torch.zeros(x.shape[1], device=DEV), torch.ones(x.shape[1], device=DEV)
    op = NormOp(nk, gamma.to(DEV), beta.to(DEV), groups=groups, running_mean=rmd, running_var=rvd)
    d = hip.dropout_struct(p, seed, stream, enabled=drop)
    ch = hip.chain_struct(hip.ACT_LRELU, 0.1, d, dropout_first=True)
    ya, stats = op.fwd(xa, ch)
    out = from_act(ya) if x.dim() == 4 else ya.rows2d().float().cpu()
    ftol = 2e-5 if dtype == torch.float32 else 1e-2
    assert rel(out, y.detach()) < ftol
    if kind.startswith("bn"):
        assert rel(rmd.cpu(), rm) < 1e-5 and rel(rvd.cpu(), rv) < 1e-5
    gya = to_act(gy, dtype) if x.dim() == 4 else Act.of(gy.to(DEV, dtype).contiguous())
    dsum = torch.zeros(x.shape[1], device=DEV)
    dxa = op.bwd(xa, stats, ch, gya, dgamma=dg, dbeta=dbt, dsum=dsum)
    dx = from_act(dxa) if x.dim() == 4 else dxa.rows2d().float().cpu()
    btol = 1e-4 if dtype == torch.float32 else 2e-2
    assert rel(dx, xr.grad) < btol
    assert rel(dg.cpu(), g_.grad) < btol
    assert rel(dbt.cpu(), b_.grad) < btol
    red = (0, 2, 3) if x.dim() == 4 else (0,)
    assert float((dsum.cpu() - xr.grad.sum(red)).abs().max()) < 1e-3 * max(1.0, float(xr.grad.abs().max()))
    if drop and x.shape[1] % 8 == 0:
        # keep bits (es_chain_t.keep): the forward stores the mask it draws (bit-exact against the
        # host Philox), the backward reads it and reproduces the regenerating backward exactly
        ck = hip.chain_struct(hip.ACT_LRELU, 0.1, hip.dropout_struct(p, seed, stream, enabled=True),
                              dropout_first=True)
        C_ = x.shape[1]
        rows = x.numel() // C_
        kb = hip.attach_keep(ck, rows, C_, DEV)
        op2 = NormOp(nk, gamma.to(DEV), beta.to(DEV), groups=groups,
                     running_mean=torch.zeros(C_, device=DEV), running_var=torch.ones(C_, device=DEV))
        yk, sk = op2.fwd(xa, ck)
        assert torch.equal(yk.t, ya.t)
        bits = kb.cpu().numpy().reshape(rows, C_ // 8)
        keep = np.unpackbits(bits, axis=1, bitorder="little").astype(bool)     # [rows][C]
        m = mask.numpy()
        m_rows = m.transpose(0, 2, 3, 1).reshape(rows, C_) if x.dim() == 4 else m.reshape(rows, C_)
        assert np.array_equal(keep, m_rows.astype(bool))
        dg2, db2, ds2 = torch.zeros_like(dg), torch.zeros_like(dbt), torch.zeros_like(dsum)
        dxk = op2.bwd(xa, sk, ck, gya, dgamma=dg2, dbeta=db2, dsum=ds2)
        assert torch.equal(dxk.t, dxa.t)
        assert torch.equal(dg2, dg) and torch.equal(db2, dbt)


@pytest.mark.parametrize("shape", [(4, 64, 9, 7), (3, 64, 8, 6), (5, 16, 9, 9), (2, 32, 45, 45)])
@pytest.mark.parametrize("k", [1, 2, 3, 6])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_keep_bits_element_offset(shape, k, dtype):
    """Stored dropout keep bits with an element index_offset that is not a multiple of 4 (ADVICE
    r02): the fast forward's counter sharing (keep_bits_gen_shared, C <= 64, and the aligned path)
    depends on (i0 & 3) including the offset.  Bit-exact against the host Philox at that offset."""
    hip = _hip()
    from expertsim.layers import NormOp
    from expertsim.utils import philox
    torch.manual_seed(3)
    x = torch.randn(*shape) * 2 + 0.5
    N, C_, H, W = shape
    p, seed, stream = 0.2, 99, 41
    xa = to_act(x, dtype)
    ch = hip.chain_struct(hip.ACT_LRELU, 0.1, hip.dropout_struct(p, seed, stream, enabled=True, index_offset=k),
                          dropout_first=True)
    rows = N * H * W
    kb = hip.attach_keep(ch, rows, C_, DEV)
    op = NormOp(hip.NORM_BN, torch.ones(C_, device=DEV), torch.zeros(C_, device=DEV),
                running_mean=torch.zeros(C_, device=DEV), running_var=torch.ones(C_, device=DEV))
    op.fwd(xa, ch)
    torch.cuda.synchronize()
    bits = philox.random_bits(x.numel(), seed, stream, k)
    m = ((bits >> np.uint32(8)) < np.uint32(philox.keep_threshold(p))).reshape(shape)
    keep = np.unpackbits(kb.cpu().numpy().reshape(rows, C_ // 8), axis=1, bitorder="little").astype(bool)
    assert np.array_equal(keep, m.transpose(0, 2, 3, 1).reshape(rows, C_))


def test_dropout_mask_bit_exact():
    hip = _hip()
    from expertsim.utils import philox
    n = 100003
    for p, stream in ((0.2, 5), (0.3, 1 << 20)):
        d = hip.dropout_struct(p, 0x123456789, stream, enabled=True)
        out = torch.empty(n, dtype=torch.uint8, device=DEV)
        hip.call("es_dropout_mask", hip.ptr(out), n, C.byref(d), hip.stream_ptr())
        ref = philox.dropout_mask((n,), p, 0x123456789, stream)
        assert np.array_equal(out.cpu().numpy().astype(bool), ref)


@pytest.mark.parametrize("k,s", [((2, 2), (2, 2)), ((2, 1), (2, 1)), ((2, 2), (1, 1))])
def test_maxpool(k, s):
    _hip()
    from expertsim.layers import MaxPool
    torch.manual_seed(3)
    x = torch.randn(2, 8, 9, 7)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, k, s)
    gy = torch.randn_like(y)
    y.backward(gy)
    mp = MaxPool(k, s)
    xa = to_act(x)
    ya, idx = mp.fwd(xa)
    assert torch.equal(from_act(ya), y.detach())
    dxa = mp.bwd(to_act(gy), idx, xa.dims, torch.float32)
    assert rel(from_act(dxa), xr.grad) < 1e-6


def test_adam_matches_torch():
    hip = _hip()
    torch.manual_seed(4)
    p = torch.randn(10007)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-4)
    pd, m, v = p.to(DEV), torch.zeros(10007, device=DEV), torch.zeros(10007, device=DEV)
    for step in range(1, 4):
        g = torch.randn(10007)
        pt.grad = g.clone()
        opt.step()
        gd = g.to(DEV)
        hip.call("es_adam", hip.ptr(pd), hip.ptr(gd), hip.ptr(m), hip.ptr(v), pd.numel(), 1e-4, 0.9, 0.999, 1e-8,
                 step, 1.0, hip.stream_ptr())
    assert float((pd.cpu() - pt.detach()).abs().max()) < 1e-7


def test_randn_moments():
    hip = _hip()
    out = torch.empty(1 << 20, device=DEV)
    hip.call("es_randn", hip.ptr(out), out.numel(), 99, 3, hip.stream_ptr())
    assert abs(out.mean().item()) < 5e-3 and abs(out.std().item() - 1) < 5e-3
    hip.call("es_rand_exponential", hip.ptr(out), out.numel(), 99, 4, hip.stream_ptr())
    assert abs(out.mean().item() - 1) < 5e-3 and out.min().item() > 0


RING_CASES = [
    # bf16 shapes on the 8-wave ring kernels (conv_mfma.hip); rows not a multiple of the tile
    (3, 256, 24, 24, 128, 3, 1, 0, (2, 2)),       # G conv_layers.5: 256x128 FWD, folded DGRAD, WGRAD 128x256
    (7, 128, 13, 13, 256, 3, 1, 0, (2, 2)),       # G conv_layers.0: WGRAD 256x128
    (5, 128, 46, 46, 64, 2, 1, 0, None),          # G conv_layers.9: Ng = 64 tiles
    (3, 128, 17, 15, 128, 3, 2, 1, None),         # stride 2 + padding, WGRAD 128x128
    (2, 512, 18, 10, 256, 4, 1, 1, (2, 2)),       # proton G conv_layers.1 (pad 1, up x2)
]


@pytest.mark.parametrize("case", RING_CASES)
def test_conv_ring_matches_4wave(case):
    """The 8-wave ring kernels accumulate each output in the same K order as the 4-wave LDS-DMA
    kernels: bf16 fwd / dgrad outputs bit-identical, wgrad equal up to the order of the split-K
    fp32 atomics, and all close to torch fp32."""
    hip = _hip()
    from expertsim.layers import ConvOp, Upsample
    N, Cin, H, W, Cout, k, st, pad, up = case
    torch.manual_seed(11)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout)
    upsample = Upsample((H, W), scale=up) if up else None
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=st, pad=pad, upsample=upsample)
    xa = to_act(x, torch.bfloat16)
    outs = []
    gy = None
    sp_old = hip.lib().es_conv_set_subpixel(0)   # bit-exact comparison: same taps on both sides
    try:
        for on in (1, 0):
            hip.lib().es_conv_set_ring(on)
            ya = op.fwd(xa, out_dtype=torch.bfloat16)
            if gy is None:
                gy = torch.randn(ya.dims, generator=torch.Generator().manual_seed(3))
            gya = to_act(gy, torch.bfloat16)
            dxa = op.dgrad(gya, xa, dx_dtype=torch.bfloat16)
            dw = torch.zeros(Cout, Cin, k, k, device=DEV)
            op.wgrad(gya, xa, dw, None, beta=1.0)
            torch.cuda.synchronize()
            outs.append((ya.t.clone(), dxa.t.clone(), dw.cpu()))
    finally:
        hip.lib().es_conv_set_ring(1)
        hip.lib().es_conv_set_subpixel(sp_old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert rel(outs[0][2], outs[1][2]) < 1e-5
    xu = F.interpolate(x, scale_factor=up, mode="nearest") if up else x
    wr = w.clone().requires_grad_(True)
    xr = xu.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, b, st, pad)
    y.backward(gy.to(torch.bfloat16).float())
    assert rel(outs[0][0].float().cpu().view(y.shape[0], y.shape[2], y.shape[3], -1).permute(0, 3, 1, 2), y) < 3e-2
    assert rel(outs[0][2], wr.grad) < 3e-2


SUBPIXEL_CASES = [
    # x2-upsample convs on the sub-pixel path (4 parity-class convs on the source grid)
    (3, 256, 24, 24, 128, 3, 0),      # neutron G conv_layers.5 (3x3 -> 2x2 taps per class)
    (7, 128, 13, 13, 256, 3, 0),      # neutron G conv_layers.0
    (2, 512, 18, 10, 256, 4, 1),      # proton G conv_layers.1 (4x4, pad 1: 2/3 taps per class)
    (70, 64, 5, 7, 64, 3, 1),         # pad 1, N not a multiple of 64, odd grids
]


@pytest.mark.parametrize("case", SUBPIXEL_CASES)
def test_conv_subpixel(case):
    """Sub-pixel fwd / dgrad / wgrad (bf16) against torch fp32 of the upsample + conv, and the
    wgrad against the non-sub-pixel ring kernel."""
    hip = _hip()
    from expertsim.layers import ConvOp, Upsample
    N, Cin, H, W, Cout, k, pad = case
    torch.manual_seed(21)
    x = torch.randn(N, Cin, H, W).to(torch.bfloat16).float()
    w = torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout)
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=1, pad=pad,
                upsample=Upsample((H, W), scale=(2, 2)))
    xa = to_act(x, torch.bfloat16)
    assert op.subpixel(op.desc(xa), torch.bfloat16)
    ya = op.fwd(xa, out_dtype=torch.float32)
    xr = F.interpolate(x, scale_factor=(2, 2), mode="nearest").requires_grad_(True)
    xs = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(F.interpolate(xs, scale_factor=(2, 2), mode="nearest"), wr, b, 1, pad)
    assert ya.dims == tuple(y.shape)
    assert rel(from_act(ya), y.detach()) < 2e-2
    gy = torch.randn(y.shape).to(torch.bfloat16).float()
    y.backward(gy)
    gya = to_act(gy, torch.bfloat16)
    dxa = op.dgrad(gya, xa, dx_dtype=torch.float32)
    assert rel(from_act(dxa), xs.grad) < 2e-2
    dw = torch.zeros(Cout, Cin, k, k, device=DEV)
    op.wgrad(gya, xa, dw, None, beta=1.0)
    assert rel(dw.cpu(), wr.grad) < 2e-2
    old = hip.lib().es_conv_set_subpixel(0)
    try:
        dw0 = torch.zeros(Cout, Cin, k, k, device=DEV)
        op.wgrad(gya, xa, dw0, None, beta=1.0)
    finally:
        hip.lib().es_conv_set_subpixel(old)
    assert rel(dw.cpu(), dw0.cpu()) < 1e-4   # same products, fp32 sums in another order


@pytest.mark.parametrize("case", [(3, 256, 24, 24, 128, 3, (2, 2)), (70, 128, 13, 13, 256, 3, (2, 2)),
                                  (5, 128, 46, 46, 64, 2, None)])
def test_conv_fused_bn_stats(case):
    """es_conv2d_fwd_stats + es_norm_stats_finalize give the BatchNorm statistics of the stored
    bf16 output (count / mean / M2 partials from the ring epilogue) = es_norm_stats over it."""
    hip = _hip()
    from expertsim.layers import ConvOp, NormOp, Upsample
    N, Cin, H, W, Cout, k, up = case
    torch.manual_seed(4)
    x = torch.randn(N, Cin, H, W)
    w = torch.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout) + 2.0
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)),
                upsample=Upsample((H, W), scale=up) if up else None)
    xa = to_act(x, torch.bfloat16)
    y1 = op.fwd(xa, bn_stats=True)
    assert y1.bn_part is not None and y1.bn_part[1] > 0
    y0 = op.fwd(xa)
    assert torch.equal(y1.t, y0.t)
    mk = lambda: NormOp(hip.NORM_BN, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                        running_mean=torch.zeros(Cout, device=DEV), running_var=torch.ones(Cout, device=DEV))
    n1, n0 = mk(), mk()
    m1, i1 = n1.stats(y1)
    m0, i0 = n0.stats(y0)
    assert rel(m1.cpu(), m0.cpu()) < 1e-5
    assert rel(i1.cpu(), i0.cpu()) < 1e-5
    assert rel(n1.rv.cpu(), n0.rv.cpu()) < 1e-5 and rel(n1.rm.cpu(), n0.rm.cpu()) < 1e-5


@pytest.mark.parametrize("N,H,W", [(5, 44, 44), (3, 56, 30), (4, 10, 8)])
def test_dfront_fused(N, H, W):
    """es_dfront_fwd / es_dfront_bwd (fused SNconv 1->32 + GroupNorm(8) + LeakyReLU + maxpool 2x2,
    d_front.hip) against torch fp32 autograd of the same block: pooled output, GN statistics, pool
    argmax, image gradient and the gradients of W/sigma, bias, gamma, beta."""
    hip = _hip()
    from expertsim.layers import Act
    torch.manual_seed(17)
    x = torch.randn(N, 1, H, W)
    w = torch.randn(32, 1, 3, 3) / 3
    b, gm, bt = 0.1 * torch.randn(32), 1 + 0.1 * torch.randn(32), 0.1 * torch.randn(32)
    sigma = torch.tensor([1.7])
    xr = x.clone().requires_grad_(True)
    weff = (w * (1.0 / sigma)).requires_grad_(True)
    br, gmr, btr = (t.clone().requires_grad_(True) for t in (b, gm, bt))
    h = F.conv2d(xr, weff, br)
    y = F.leaky_relu(F.group_norm(h, 8, gmr, btr, 1e-5), 0.1)
    p, pidx = F.max_pool2d(y, 2, return_indices=True)
    gp = torch.randn_like(p)
    p.backward(gp)

    xd = x.to(DEV)
    dev_params = [w.to(DEV), sigma.to(DEV), b.to(DEV), gm.to(DEV), bt.to(DEV)]
    args = (hip.ptr(xd), hip.strides4(xd.stride()), N, H, W) + tuple(hip.ptr(t) for t in dev_params) + (1e-5, 0.1)
    Hp, Wp = (H - 2) // 2, (W - 2) // 2
    pooled = Act.nhwc(N, 32, Hp, Wp, torch.float32, DEV)
    idx = torch.empty(pooled.numel, dtype=torch.uint8, device=DEV)
    mean = torch.empty(N * 8, device=DEV)
    invstd = torch.empty(N * 8, device=DEV)
    hip.call("es_dfront_fwd", *args, hip.ptr(mean), hip.ptr(invstd), pooled.ptr, hip.ptr(idx), hip.stream_ptr())
    assert rel(from_act(pooled), p.detach()) < 1e-5
    hg = h.detach().view(N, 8, -1)
    assert rel(mean.cpu(), hg.mean(-1).reshape(-1)) < 1e-5
    assert rel(invstd.cpu(), torch.rsqrt(hg.var(-1, unbiased=False) + 1e-5).reshape(-1)) < 1e-4
    # argmax byte (window row-major) vs torch's flat index
    pi = torch.arange(Hp).view(1, 1, Hp, 1) * 2
    pj = torch.arange(Wp).view(1, 1, 1, Wp) * 2
    ref_bytes = (pidx // (W - 2) - pi) * 2 + (pidx % (W - 2) - pj)
    got = idx.cpu().view(N, Hp, Wp, 32).permute(0, 3, 1, 2).long()
    assert torch.equal(got, ref_bytes)

    dpooled = to_act(gp)
    dx = torch.empty(N, 1, H, W, device=DEV)
    part = torch.empty(hip.lib().es_dfront_part_floats(N), device=DEV)
    dw = torch.empty(32 * 9, device=DEV)
    db, dg, dbt = (torch.full((32,), 0.5, device=DEV) for _ in range(3))   # accumulated into
    hip.call("es_dfront_bwd", *args, hip.ptr(mean), hip.ptr(invstd), hip.ptr(idx), dpooled.ptr, hip.ptr(dx),
             hip.strides4(dx.stride()), hip.ptr(part), hip.ptr(dw), hip.ptr(db), hip.ptr(dg), hip.ptr(dbt),
             hip.stream_ptr())
    assert rel(dx.cpu(), xr.grad) < 1e-4
    assert rel(dw.cpu().view(32, 1, 3, 3), weff.grad) < 1e-4
    assert rel(db.cpu() - 0.5, br.grad) < 1e-4
    assert rel(dg.cpu() - 0.5, gmr.grad) < 1e-4
    assert rel(dbt.cpu() - 0.5, btr.grad) < 1e-4


@pytest.mark.parametrize("N,H,W,pool", [(5, 44, 44, (2, 2)), (3, 56, 30, (2, 1)), (4, 12, 14, (2, 2))])
def test_dfront2_fused(N, H, W, pool):
    """es_dfront2_fwd / es_dfront2_bwd (both discriminator conv blocks in one per-image kernel,
    d_front2.hip) against torch fp32 autograd of the reference block (neutron/discriminator.py:11-24,
    proton/discriminator.py:121-134): flattened features, GN statistics, image gradient and the
    gradients of both W/sigma, biases and GroupNorm affines -- for the D-step variant (weight
    gradients only), the G-step variant (image gradient only) and both at once."""
    hip = _hip()
    import ctypes as C
    torch.manual_seed(23)
    x = torch.randn(N, 1, H, W)
    w1 = torch.randn(32, 1, 3, 3) / 3
    w2 = torch.randn(16, 32, 3, 3) / 17
    b1, g1, be1 = 0.1 * torch.randn(32), 1 + 0.1 * torch.randn(32), 0.1 * torch.randn(32)
    b2, g2, be2 = 0.1 * torch.randn(16), 1 + 0.1 * torch.randn(16), 0.1 * torch.randn(16)
    s1, s2 = torch.tensor([1.7]), torch.tensor([1.3])
    xr = x.clone().requires_grad_(True)
    w1e = (w1 * (1.0 / s1)).requires_grad_(True)
    w2e = (w2 * (1.0 / s2)).requires_grad_(True)
    leaves = [t.clone().requires_grad_(True) for t in (b1, g1, be1, b2, g2, be2)]
    b1r, g1r, be1r, b2r, g2r, be2r = leaves
    h = F.conv2d(xr, w1e, b1r)
    p = F.max_pool2d(F.leaky_relu(F.group_norm(h, 8, g1r, be1r, 1e-5), 0.1), 2)
    h2 = F.conv2d(p, w2e, b2r)
    q = F.max_pool2d(F.leaky_relu(F.group_norm(h2, 8, g2r, be2r, 1e-5), 0.1), pool)
    feat = q.reshape(N, -1)
    gf = torch.randn_like(feat)
    feat.backward(gf)
    nf = feat.shape[1]
    Fs = nf + 9                                  # fc1 input rows: features | cond

    dv = {k: t.to(DEV) for k, t in dict(w1=w1, s1=s1, b1=b1, g1=g1, be1=be1, w2=w2, s2=s2, b2=b2, g2=g2,
                                        be2=be2).items()}
    prm = hip.DFront2Params()
    prm.w1, prm.sigma1, prm.b1, prm.g1, prm.be1 = (dv[k].data_ptr() for k in ("w1", "s1", "b1", "g1", "be1"))
    prm.w2, prm.sigma2, prm.b2, prm.g2, prm.be2 = (dv[k].data_ptr() for k in ("w2", "s2", "b2", "g2", "be2"))
    prm.eps1 = prm.eps2 = 1e-5
    prm.slope = 0.1
    prm.ph, prm.pw = pool
    assert hip.lib().es_dfront2_ok(H, W, *pool)
    xd = x.to(DEV)
    X = torch.full((N, Fs), 7.0, device=DEV)
    stats = torch.empty(N * 32, device=DEV)
    save = torch.empty(N * hip.lib().es_dfront2_save_floats(H, W, *pool), device=DEV)
    hip.call("es_dfront2_fwd", hip.ptr(xd), hip.strides4(xd.stride()), N, H, W, C.byref(prm), hip.ptr(stats),
             hip.ptr(X), Fs, hip.ptr(save), hip.stream_ptr())
    assert rel(X[:, :nf].cpu(), feat.detach()) < 1e-5
    X2 = torch.full((N, Fs), 7.0, device=DEV)      # inference form (no save): same features
    hip.call("es_dfront2_fwd", hip.ptr(xd), hip.strides4(xd.stride()), N, H, W, C.byref(prm), hip.ptr(stats),
             hip.ptr(X2), Fs, None, hip.stream_ptr())
    assert torch.equal(X, X2)
    # the save: pooled block-1 map, block-2 conv map
    sv = save.cpu().view(N, -1)
    np1 = p.shape[2] * p.shape[3]
    assert rel(sv[:, :np1 * 32].view(N, p.shape[2], p.shape[3], 32).permute(0, 3, 1, 2), p.detach()) < 1e-5
    assert rel(sv[:, 2 * np1 * 32:].view(N, h2.shape[2], h2.shape[3], 16).permute(0, 3, 1, 2), h2.detach()) < 1e-5
    assert torch.all(X[:, nf:] == 7.0)           # the cond columns are left alone
    st = stats.cpu().view(N, 4, 8)
    hg, h2g = h.detach().view(N, 8, -1), h2.detach().view(N, 8, -1)
    assert rel(st[:, 0], hg.mean(-1)) < 1e-5
    assert rel(st[:, 1], torch.rsqrt(hg.var(-1, unbiased=False) + 1e-5)) < 1e-4
    assert rel(st[:, 2], h2g.mean(-1)) < 1e-5
    assert rel(st[:, 3], torch.rsqrt(h2g.var(-1, unbiased=False) + 1e-5)) < 1e-4

    dX = torch.zeros(N, Fs, device=DEV)
    dX[:, :nf] = gf.to(DEV)
    refs = [w1e.grad, b1r.grad, g1r.grad, be1r.grad, w2e.grad, b2r.grad, g2r.grad, be2r.grad]
    for want_dx, want_w in ((False, True), (True, False), (True, True)):
        dx = torch.empty(N, 1, H, W, device=DEV) if want_dx else None
        part = torch.empty(hip.lib().es_dfront2_part_floats(N), device=DEV) if want_w else None
        outs = [torch.empty(32 * 9, device=DEV), torch.full((32,), 0.5, device=DEV),
                torch.full((32,), 0.5, device=DEV), torch.full((32,), 0.5, device=DEV),
                torch.empty(16 * 32 * 9, device=DEV), torch.full((16,), 0.5, device=DEV),
                torch.full((16,), 0.5, device=DEV), torch.full((16,), 0.5, device=DEV)]
        hip.call("es_dfront2_bwd", hip.ptr(xd), hip.strides4(xd.stride()), N, H, W, C.byref(prm), hip.ptr(stats),
                 hip.ptr(save), hip.ptr(dX), Fs, hip.ptr(dx), hip.strides4(dx.stride()) if dx is not None else None,
                 hip.ptr(part), *[hip.ptr(o) if want_w else None for o in outs], hip.stream_ptr())
        if want_dx:
            assert rel(dx.cpu(), xr.grad) < 1e-4, (want_dx, want_w)
        if want_w:
            for i, (o, r) in enumerate(zip(outs, refs)):
                got = o.cpu().view(r.shape) - (0.5 if i not in (0, 4) else 0.0)
                assert rel(got, r) < 1e-4, (i, rel(got, r))


@pytest.mark.parametrize("B,NF", [(70, 1305), (16, 2313), (5, 37)])
def test_dmlp_fused(B, NF):
    """es_dmlp_fwd / es_dmlp_bwd (the discriminator's fc tail in one kernel pair, d_mlp.hip) against
    torch fp32 autograd of the reference layers (neutron/discriminator.py:26-48): logit, latent,
    LayerNorm statistics, fc1-input gradient and every weight gradient (of W/sigma), for the
    D-step variant (weights only), the G-step variant (input gradient only) and both."""
    hip = _hip()
    import ctypes as C
    torch.manual_seed(31)
    X = torch.randn(B, NF)
    w1, w2, w3 = torch.randn(128, NF) / NF ** 0.5, torch.randn(64, 128) / 11, torch.randn(1, 64) / 8
    b1, b2, b3 = 0.1 * torch.randn(128), 0.1 * torch.randn(64), 0.1 * torch.randn(1)
    g1, be1, g2, be2 = 1 + 0.1 * torch.randn(128), 0.1 * torch.randn(128), 1 + 0.1 * torch.randn(64), 0.1 * torch.randn(64)
    s1, s2, s3 = torch.tensor([1.3]), torch.tensor([0.9]), torch.tensor([1.7])
    leaves = [t.clone().requires_grad_(True) for t in (b1, g1, be1, b2, g2, be2, b3)]
    b1r, g1r, be1r, b2r, g2r, be2r, b3r = leaves
    w1e, w2e, w3e = ((w * (1.0 / s)).requires_grad_(True) for w, s in ((w1, s1), (w2, s2), (w3, s3)))
    Xr = X.clone().requires_grad_(True)
    h3 = F.linear(Xr, w1e, b1r)
    y3 = F.leaky_relu(F.layer_norm(h3, (128,), g1r, be1r, 1e-5), 0.1)
    h4 = F.linear(y3, w2e, b2r)
    lat = F.leaky_relu(F.layer_norm(h4, (64,), g2r, be2r, 1e-5), 0.1)
    out = F.linear(lat, w3e, b3r)
    gout, glat = torch.randn(B, 1), torch.randn(B, 64)
    (out * gout).sum().backward(retain_graph=True)
    (lat * glat).sum().backward()

    d = {k: t.to(DEV) for k, t in dict(w1=w1, s1=s1, b1=b1, g1=g1, be1=be1, w2=w2, s2=s2, b2=b2, g2=g2, be2=be2,
                                        w3=w3, s3=s3, b3=b3).items()}
    prm = hip.DMlpParams()
    prm.w1, prm.sigma1, prm.b1, prm.g1, prm.be1 = (d[k].data_ptr() for k in ("w1", "s1", "b1", "g1", "be1"))
    prm.w2, prm.sigma2, prm.b2, prm.g2, prm.be2 = (d[k].data_ptr() for k in ("w2", "s2", "b2", "g2", "be2"))
    prm.w3, prm.sigma3, prm.b3 = (d[k].data_ptr() for k in ("w3", "s3", "b3"))
    prm.eps1 = prm.eps2 = 1e-5
    prm.slope = 0.1
    Xd = X.to(DEV)
    f32 = lambda *sh: torch.empty(*sh, device=DEV)
    H3, S3, H4, S4, LAT, OUT = f32(B, 128), f32(B, 2), f32(B, 64), f32(B, 2), f32(B, 64), f32(B)
    hip.call("es_dmlp_fwd", hip.ptr(Xd), NF, B, NF, C.byref(prm), hip.ptr(H3), hip.ptr(S3), hip.ptr(H4), hip.ptr(S4),
             hip.ptr(LAT), hip.ptr(OUT), hip.stream_ptr())
    assert rel(OUT.cpu(), out.detach().view(-1)) < 1e-4
    assert rel(LAT.cpu(), lat.detach()) < 1e-4
    assert rel(H3.cpu(), h3.detach()) < 1e-5 and rel(H4.cpu(), h4.detach()) < 1e-4
    assert rel(S3[:, 0].cpu(), h3.detach().mean(1)) < 1e-4
    refs = [w1e.grad, b1r.grad, g1r.grad, be1r.grad, w2e.grad, b2r.grad, g2r.grad, be2r.grad, w3e.grad, b3r.grad]
    gout_d, glat_d = gout.to(DEV).contiguous(), glat.to(DEV).contiguous()
    for want_dx, want_w in ((False, True), (True, False), (True, True)):
        dX = torch.full((B, NF), 3.0, device=DEV) if want_dx else None
        part = torch.empty(hip.lib().es_dmlp_part_floats(B, NF), device=DEV) if want_w else None
        outs = [f32(128, NF), torch.full((128,), 0.5, device=DEV), torch.full((128,), 0.5, device=DEV),
                torch.full((128,), 0.5, device=DEV), f32(64, 128), torch.full((64,), 0.5, device=DEV),
                torch.full((64,), 0.5, device=DEV), torch.full((64,), 0.5, device=DEV), f32(1, 64),
                torch.full((1,), 0.5, device=DEV)]
        hip.call("es_dmlp_bwd", hip.ptr(Xd), NF, B, NF, C.byref(prm), hip.ptr(H3), hip.ptr(S3), hip.ptr(H4),
                 hip.ptr(S4), hip.ptr(LAT), hip.ptr(gout_d), hip.ptr(glat_d), hip.ptr(dX), NF, hip.ptr(part),
                 *[hip.ptr(o) if want_w else None for o in outs], hip.stream_ptr())
        if want_dx:
            assert rel(dX.cpu(), Xr.grad) < 1e-4, (want_dx, want_w)
        if want_w:
            for i, (o, r) in enumerate(zip(outs, refs)):
                got = o.cpu().view(r.shape) - (0.0 if i in (0, 4, 8) else 0.5)
                assert rel(got, r) < 1e-4, (i, rel(got, r))


@pytest.mark.parametrize("case", [(200, 256, 24, 24, 128, 3), (200, 128, 13, 13, 256, 3)])
def test_conv_ring256_matches_ring128(case):
    """256 x 256 ring tiles with 32-deep K-steps (sub-pixel FWD with 256 output channels, DGRAD
    with 256 input channels) accumulate in the same K order as the 256 x 128 tiles: bf16 outputs
    bit-identical; fused BatchNorm statistics equal up to the merge order."""
    hip = _hip()
    from expertsim.layers import ConvOp, NormOp, Upsample
    N, Cin, H, W, Cout, k = case
    torch.manual_seed(5)
    w = torch.randn(Cout, Cin, k, k, device=DEV) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, device=DEV)
    op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(b), upsample=Upsample((H, W), scale=(2, 2)))
    from expertsim.layers import Act
    xa = Act.nhwc(N, Cin, H, W, torch.bfloat16, DEV)
    xa.t.normal_()
    outs = []
    old = hip.lib().es_conv_set_ring256(1)
    try:
        for on in (1, 0):
            hip.lib().es_conv_set_ring256(on)
            ya = op.fwd(xa, out_dtype=torch.bfloat16, bn_stats=True)
            gy = ya.like_nhwc(torch.bfloat16)
            gy.t.copy_(torch.randn(gy.t.shape, generator=torch.Generator().manual_seed(2)).to(DEV))
            dxa = op.dgrad(gy, xa, dx_dtype=torch.bfloat16)
            nm = NormOp(hip.NORM_BN, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                        running_mean=torch.zeros(Cout, device=DEV), running_var=torch.ones(Cout, device=DEV))
            m, istd = nm.stats(ya)
            torch.cuda.synchronize()
            outs.append((ya.t.clone(), dxa.t.clone(), m.cpu(), istd.cpu()))
    finally:
        hip.lib().es_conv_set_ring256(old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert rel(outs[0][2], outs[1][2]) < 1e-5 and rel(outs[0][3], outs[1][3]) < 1e-5


@pytest.mark.parametrize("case", [(200, 128, 46, 46, 64, 2), (70, 128, 23, 21, 64, 2), (33, 64, 9, 7, 128, 2)])
def test_conv_persist_matches_ring(case):
    """The persistent short-K kernel (generator conv_layers.9's DGRAD: <= 8 K-steps, one workgroup per
    CU over its tiles, weight panel resident in LDS) accumulates in the ring kernel's K order: bf16
    outputs bit-identical to the ring kernel; both close to torch fp32."""
    hip = _hip()
    from expertsim.layers import Act, ConvOp, NormOp
    N, Cin, H, W, Cout, k = case
    torch.manual_seed(9)
    w = torch.randn(Cout, Cin, k, k, device=DEV) / np.sqrt(Cin * k * k)
    b = torch.randn(Cout, device=DEV)
    op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(b))
    xa = Act.nhwc(N, Cin, H, W, torch.bfloat16, DEV)
    xa.t.normal_()
    outs = []
    old = hip.lib().es_conv_set_persist(1)
    try:
        for on in (1, 0):
            hip.lib().es_conv_set_persist(on)
            ya = op.fwd(xa, out_dtype=torch.bfloat16, bn_stats=True)
            assert ya.bn_part is not None
            gy = ya.like_nhwc(torch.bfloat16)
            gy.t.copy_(torch.randn(gy.t.shape, generator=torch.Generator().manual_seed(2)).to(DEV))
            dxa = op.dgrad(gy, xa, dx_dtype=torch.bfloat16)
            nm = NormOp(hip.NORM_BN, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                        running_mean=torch.zeros(Cout, device=DEV), running_var=torch.ones(Cout, device=DEV))
            m, istd = nm.stats(ya)
            torch.cuda.synchronize()
            outs.append((ya.t.clone(), dxa.t.clone(), m.cpu(), istd.cpu(), ya, gy))
    finally:
        hip.lib().es_conv_set_persist(old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert rel(outs[0][2], outs[1][2]) < 1e-5 and rel(outs[0][3], outs[1][3]) < 1e-5
    # against torch fp32 on the bf16 operands
    xr = xa.torch_nchw().float()
    wr = w.to(torch.bfloat16).float()
    yr = F.conv2d(xr, wr, b)
    assert rel(outs[0][4].torch_nchw().float().cpu(), yr.cpu()) < 1e-2
    dxr = torch.nn.grad.conv2d_input(xr.shape, wr, outs[0][5].torch_nchw().float())
    assert rel(from_act(Act(outs[0][1], dxa.dims, dxa.strides)).float(), dxr.cpu()) < 1e-2
    assert rel(outs[0][2], yr.mean((0, 2, 3)).cpu()) < 1e-2


@pytest.mark.parametrize("case", [(64, 128, 46, 46, 64, 2), (37, 128, 23, 21, 64, 2), (33, 64, 9, 7, 128, 2),
                                  (50, 64, 45, 45, 1, 2), (7, 64, 13, 11, 1, 2), (5, 32, 12, 10, 1, 3)])
@pytest.mark.parametrize("dfirst", [True, False])
def test_conv_dgrad_bn_reduce_fused(case, dfirst):
    """The dgrad fused with the reduction pass of the BatchNorm backward that consumes its output
    (es_conv2d_dgrad_bnred + es_norm_act_bwd_sums): the persistent DGRAD (generator conv_layers.9 ->
    conv_layers.6 BatchNorm + Dropout + LeakyReLU) and the thin Cout = 1 dgrad (conv_layers.13 ->
    conv_layers.10).  The dgrad output is bit-identical to the plain dgrad; the norm backward (dh, dgamma, dbeta, conv-bias sum) equals the unfused two-pass
    backward up to the summation order of the per-channel sums (fp32: <= 1e-4 relative for the
    parameter gradients; dh is bf16, within one bf16 rounding)."""
    hip = _hip()
    from expertsim.layers import Act, ConvOp, NormOp
    N, Cin, H, W, Cout, k = case
    torch.manual_seed(11)
    w = torch.randn(Cout, Cin, k, k, device=DEV) / np.sqrt(Cin * k * k)
    op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(torch.zeros(Cout, device=DEV)))
    h = Act.nhwc(N, Cin, H, W, torch.bfloat16, DEV)
    h.t.copy_((torch.randn(h.t.shape) * 2 + 0.3).to(DEV))
    gamma, beta = (torch.rand(Cin) + 0.5).to(DEV), torch.randn(Cin).to(DEV)
    bn = NormOp(hip.NORM_BN, gamma, beta, running_mean=torch.zeros(Cin, device=DEV),
                running_var=torch.ones(Cin, device=DEV))
    ch = hip.chain_struct(hip.ACT_LRELU, 0.1, hip.dropout_struct(0.2, 4321, 9, enabled=True), dropout_first=dfirst)
    kb = hip.attach_keep(ch, N * H * W, Cin, DEV)   # noqa: F841 (kept alive for the backward)
    y, stats = bn.fwd(h, ch)                     # writes the keep bits the backward reads
    P, Q = H - k + 1, W - k + 1
    gy = Act.nhwc(N, Cout, P, Q, torch.bfloat16, DEV)
    gy.t.copy_(torch.randn(gy.t.shape, generator=torch.Generator().manual_seed(3)).to(DEV))
    outs = []
    for fused in (False, True):
        dx = op.dgrad(gy, y, dx_dtype=torch.bfloat16, bn_reduce=(bn, h, stats, ch) if fused else None)
        if fused:
            assert getattr(dx, "bn_sums", None) is not None, "persistent dgrad did not fuse the reduction"
        dg, db, ds = (torch.zeros(Cin, device=DEV) for _ in range(3))
        dh = bn.bwd(h, stats, ch, dx, dgamma=dg, dbeta=db, dsum=ds)
        torch.cuda.synchronize()
        outs.append((dx.t.clone(), dh.t.float().cpu(), dg.cpu(), db.cpu(), ds.cpu()))
    (dx0, dh0, dg0, db0, ds0), (dx1, dh1, dg1, db1, ds1) = outs
    assert torch.equal(dx0, dx1)
    assert rel(dg1, dg0) < 1e-4 and rel(db1, db0) < 1e-4
    # sum(dh) per channel (the conv-bias gradient) vanishes analytically for a BatchNorm backward:
    # both are rounding residue, compared against the channel's sum of |dh|
    scale = float(dh0.abs().reshape(-1, Cin).sum(0).max())
    assert float((ds1 - ds0).abs().max()) < 1e-4 * scale
    assert rel(dh1, dh0) < 1e-2


@pytest.mark.parametrize("case", [(50, 64, 45, 45, 1, 2), (7, 64, 13, 11, 1, 2), (5, 32, 12, 10, 1, 3)])
@pytest.mark.parametrize("dfirst", [True, False])
def test_thin_dgrad_bn_reduce_fused_fp32(case, dfirst):
    """Round 4: the thin Cout = 1 dgrad fused with the BatchNorm-backward reduction in the fp32 parity
    mode (conv_layers.13 -> BatchNorm conv_layers.10 + Dropout + LeakyReLU, neutron/generator.py:33-37;
    k1_dgrad_bnred<float>): the dgrad output is bitwise the unfused one; dgamma / dbeta / the conv-bias
    sum / dh equal the two-pass backward up to the order of the per-channel sums."""
    hip = _hip()
    from expertsim import layers
    from expertsim.layers import Act, ConvOp, NormOp
    N, Cin, H, W, Cout, k = case
    old_det = layers.deterministic()
    layers.set_deterministic(True)
    try:
        torch.manual_seed(17)
        w = torch.randn(Cout, Cin, k, k, device=DEV) / np.sqrt(Cin * k * k)
        op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(torch.zeros(Cout, device=DEV)))
        h = Act.nhwc(N, Cin, H, W, torch.float32, DEV)
        h.t.copy_((torch.randn(h.t.shape) * 2 + 0.3).to(DEV))
        gamma, beta = (torch.rand(Cin) + 0.5).to(DEV), torch.randn(Cin).to(DEV)
        bn = NormOp(hip.NORM_BN, gamma, beta, running_mean=torch.zeros(Cin, device=DEV),
                    running_var=torch.ones(Cin, device=DEV))
        ch = hip.chain_struct(hip.ACT_LRELU, 0.1, hip.dropout_struct(0.2, 4321, 9, enabled=True), dropout_first=dfirst)
        kb = hip.attach_keep(ch, N * H * W, Cin, DEV)   # noqa: F841 (kept alive for the backward)
        y, stats = bn.fwd(h, ch)
        P, Q = H - k + 1, W - k + 1
        gy = Act.nhwc(N, Cout, P, Q, torch.float32, DEV)
        gy.t.copy_(torch.randn(gy.t.shape, generator=torch.Generator().manual_seed(3)).to(DEV))
        outs = []
        for fused in (False, True):
            dx = op.dgrad(gy, y, dx_dtype=torch.float32, bn_reduce=(bn, h, stats, ch) if fused else None)
            if fused:
                assert getattr(dx, "bn_sums", None) is not None, "fp32 thin dgrad did not fuse the reduction"
            dg, db, ds = (torch.zeros(Cin, device=DEV) for _ in range(3))
            dh = bn.bwd(h, stats, ch, dx, dgamma=dg, dbeta=db, dsum=ds)
            torch.cuda.synchronize()
            outs.append((dx.t.clone(), dh.t.float().cpu(), dg.cpu(), db.cpu(), ds.cpu()))
        (dx0, dh0, dg0, db0, ds0), (dx1, dh1, dg1, db1, ds1) = outs
        assert torch.equal(dx0, dx1)
        assert rel(dg1, dg0) < 1e-5 and rel(db1, db0) < 1e-5
        scale = float(dh0.abs().reshape(-1, Cin).sum(0).max())
        assert float((ds1 - ds0).abs().max()) < 1e-5 * scale
        assert rel(dh1, dh0) < 1e-5
    finally:
        layers.set_deterministic(old_det)


@pytest.mark.parametrize("case", [(70, 256, 24, 24, 128), (130, 128, 13, 13, 256), (600, 64, 20, 20, 64)])
def test_conv_p256_matches_ring(case):
    """The persistent 256 x 256 merged sub-pixel FWD (generator conv_layers.0 / .5: workgroups with
    a fixed column tile looping over row tiles, the ring continued across tiles) accumulates in the
    ring kernel's K order: bf16 output bit-identical (padding images past N and pixels past the
    class grid included); fused BatchNorm statistics (per (workgroup, class) partials, padding rows
    subtracted) equal up to the merge order, and close to torch fp32."""
    hip = _hip()
    from expertsim.layers import Act, ConvOp, NormOp, Upsample
    N, Cin, H, W, Cout = case
    torch.manual_seed(11)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV) / np.sqrt(Cin * 9)
    b = torch.randn(Cout, device=DEV) + 1.0
    op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(b), upsample=Upsample((H, W), scale=(2, 2)))
    xa = Act.nhwc(N, Cin, H, W, torch.bfloat16, DEV)
    xa.t.normal_()
    outs = []
    old = hip.lib().es_conv_set_p256(1)
    try:
        for on in (1, 0):
            hip.lib().es_conv_set_p256(on)
            ya = op.fwd(xa, out_dtype=torch.bfloat16, bn_stats=True)
            assert ya.bn_part is not None
            # the persistent kernel writes 4 partials per workgroup (256 workgroups)
            assert (ya.bn_part[1] == 1024) == (on == 1)
            nm = NormOp(hip.NORM_BN, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                        running_mean=torch.zeros(Cout, device=DEV), running_var=torch.ones(Cout, device=DEV))
            m, istd = nm.stats(ya)
            torch.cuda.synchronize()
            outs.append((ya.t.clone(), m.cpu(), istd.cpu(), ya))
    finally:
        hip.lib().es_conv_set_p256(old)
    assert torch.equal(outs[0][0], outs[1][0])
    assert rel(outs[0][1], outs[1][1]) < 1e-5 and rel(outs[0][2], outs[1][2]) < 1e-5
    yb = outs[0][3].torch_nchw().float()
    assert rel(outs[0][1], yb.mean((0, 2, 3)).cpu()) < 1e-5
    assert rel(outs[0][2], (1.0 / torch.sqrt(yb.var((0, 2, 3), unbiased=False) + 1e-5)).cpu()) < 1e-4


@pytest.mark.parametrize("shape", [(5, 128, 13, 13), (3, 70, 9, 7), (2, 3, 5, 4)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_copy_relayout(shape, dtype):
    """es_copy between dense NCHW and dense NHWC views (the LDS-tiled transpose path) is exact."""
    hip = _hip()
    from expertsim.layers import Act, copy_act
    N, Cc, H, W = shape
    x = torch.randn(shape).to(dtype).to(DEV)
    nchw = Act(x.reshape(-1), shape, (Cc * H * W, H * W, W, 1))
    nhwc = Act.nhwc(N, Cc, H, W, dtype, DEV)
    copy_act(nchw, nhwc)
    assert torch.equal(nhwc.torch_nchw().contiguous(), x)
    back = Act(torch.empty_like(x).reshape(-1), shape, (Cc * H * W, H * W, W, 1))
    copy_act(nhwc, back)
    assert torch.equal(back.t.view(shape), x)


@pytest.mark.parametrize("shape", [(4, 64, 55, 29), (8, 64, 55, 29), (16, 128, 55, 29), (16, 256, 35, 19),
                                   (3, 64, 55, 29), (5, 128, 55, 29)])
def test_gn_backward_proton_shapes(shape):
    """GroupNorm(32) + LeakyReLU backward at the proton generator's shapes (proton/generator.py:28-39)
    and the small per-expert batches of E > 1 steps, fp32, against torch autograd."""
    hip = _hip()
    from expertsim.layers import NormOp
    torch.manual_seed(sum(shape))
    x = torch.randn(*shape) * 2 - 0.5
    C = shape[1]
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    xr = x.clone().requires_grad_(True)
    g_, b_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    y = F.leaky_relu(F.group_norm(xr, 32, g_, b_, 1e-5), 0.1)
    gy = torch.randn_like(y)
    y.backward(gy)
    op = NormOp(hip.NORM_GN, gamma.to(DEV), beta.to(DEV), groups=32)
    ch = hip.chain_struct(hip.ACT_LRELU, 0.1)
    xa = to_act(x, torch.float32)
    ya, stats = op.fwd(xa, ch)
    assert rel(from_act(ya), y.detach()) < 2e-5
    dg, dbt, dsum = (torch.zeros(C, device=DEV) for _ in range(3))
    dxa = op.bwd(xa, stats, ch, to_act(gy, torch.float32), dgamma=dg, dbeta=dbt, dsum=dsum)
    assert rel(from_act(dxa), xr.grad) < 1e-4
    assert rel(dg.cpu(), g_.grad) < 1e-4 and rel(dbt.cpu(), b_.grad) < 1e-4


@pytest.mark.parametrize("B,E", [(12, 3), (1000, 5), (4096, 8), (3000, 1)])
def test_router_dispatch_is_stable_grouping(B, E):
    """es_router_dispatch == per expert (idx == e).nonzero() in batch order (moe.py:121-123)."""
    hip = _hip()
    g = torch.Generator().manual_seed(B + E)
    idx = torch.randint(0, E, (B,), generator=g, dtype=torch.int32)
    if E > 2:
        idx[idx == 1] = 0                            # an empty expert
    perm = torch.empty(B, dtype=torch.int32, device=DEV)
    offs = torch.empty(E + 1, dtype=torch.int32, device=DEV)
    hip.call("es_router_dispatch", hip.ptr(idx.to(DEV)), B, E, hip.ptr(perm), hip.ptr(offs), hip.stream_ptr())
    want = np.concatenate([np.nonzero(idx.numpy() == e)[0] for e in range(E)])
    counts = np.bincount(idx.numpy(), minlength=E)
    assert np.array_equal(perm.cpu().numpy(), want)
    assert np.array_equal(offs.cpu().numpy(), np.concatenate([[0], np.cumsum(counts)]))


def test_batched_weight_repack_matches_single_packs():
    """es_pack_conv_weights (the optimizer step's batched repack, layers.repack_ops) writes the same
    bytes as es_pack_conv_weight (+ es_pack_weight_planes) per job: every mode, both dtypes, the
    split-fp32 planes, and a wide mode-1 transpose (the LDS-tiled kernel inside the batch)."""
    import ctypes as C
    from expertsim import hip
    hip.lib()
    g = torch.Generator().manual_seed(3)
    shapes = [(128, 256, 3, 3, 2), (128, 256, 3, 3, 3), (64, 128, 2, 2, 0), (64, 128, 2, 2, 1),
              (32, 1, 3, 3, 0), (1, 64, 2, 2, 1), (4096, 256, 1, 1, 0), (4096, 256, 1, 1, 1), (48, 20, 3, 3, 1)]
    jobs, refs, outs = [], [], []
    for K, Cc, R, S, mode in shapes:
        w = torch.randn(K, Cc, R, S, generator=g).to(DEV)
        n = K * Cc * (hip.lib().es_subpixel_taps(R, S) if mode >= 2 else R * S)
        for dtype in (torch.float32, torch.bfloat16):
            planes = dtype == torch.float32
            total = (int(hip.lib().es_weight_planes_offset(n)) + 6 * n + 3) // 4 if planes else n
            ref = torch.zeros(total, dtype=dtype, device=DEV)
            hip.call("es_pack_conv_weight", hip.ptr(w), K, Cc, R, S, mode, None, None, hip.ptr(ref), hip.dt_of(ref),
                     hip.stream_ptr())
            if planes:
                hip.call("es_pack_weight_planes", hip.ptr(ref), n, hip.ptr(ref), hip.stream_ptr())
            out = torch.zeros_like(ref)
            j = hip.PackJob()
            j.w, j.K, j.C, j.R, j.S, j.mode = w.data_ptr(), K, Cc, R, S, mode
            j.dt, j.planes, j.out = hip.dt_of(out), int(planes), out.data_ptr()
            jobs.append(j)
            refs.append(ref)
            outs.append((out, w))
    arr = (hip.PackJob * len(jobs))(*jobs)
    hip.call("es_pack_conv_weights", arr, len(jobs), hip.stream_ptr())
    torch.cuda.synchronize()
    for (out, _), ref, (K, Cc, R, S, mode) in zip(outs, refs, [s for s in shapes for _ in (0, 1)]):
        assert torch.equal(out.view(torch.int16) if out.dtype == torch.bfloat16 else out.view(torch.int32),
                           ref.view(torch.int16) if ref.dtype == torch.bfloat16 else ref.view(torch.int32)), \
            (K, Cc, R, S, mode, out.dtype)
