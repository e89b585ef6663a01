"""The opt-in 4-wave split-fp32 kernels (conv_mfma.hip conv_ring_kernel SPL = 3, and SPL = 4 on a
pre-split planes operand, es_conv2d_fwd_planes / es_conv2d_dgrad_planes) against the default 8-wave
kernel: same products in the same order, so the outputs must be bitwise equal (sub-pixel
conv_layers.0 / .5 shapes of the neutron generator, generator.py:24,29; B = 64 / 128)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(128, 13, 13, 256), (256, 24, 24, 128)])
@pytest.mark.parametrize("N", [64, 128])
def test_spb4_and_planes_bitwise(shape, N):
    from expertsim import hip, layers
    from expertsim.layers import Act, ConvOp, Upsample, split_planes
    Cin, H, W, Cout = shape
    layers.set_deterministic(True)
    layers.set_f32_split(True)
    g = torch.Generator(device=DEV).manual_seed(N + Cin)
    w = torch.nn.Parameter(torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (Cin * 9) ** 0.5)
    b = torch.nn.Parameter(torch.randn(Cout, device=DEV, generator=g))
    op = ConvOp(w, b, upsample=Upsample((H, W), scale=(2, 2)))
    x = Act.nhwc(N, Cin, H, W, torch.float32, DEV)
    x.t.normal_(generator=g)
    y = op.fwd(x, out_dtype=torch.float32)
    dy = y.like_nhwc(torch.float32)
    dy.t.normal_(generator=g)
    old = hip.lib().es_conv_set_spb4(0)
    try:
        ref_f = op.fwd(x, out_dtype=torch.float32).t.clone()
        ref_d = op.dgrad(dy, x, dx_dtype=torch.float32).t.clone()
        hip.lib().es_conv_set_spb4(1)
        f4 = op.fwd(x, out_dtype=torch.float32).t.clone()
        d4 = op.dgrad(dy, x, dx_dtype=torch.float32).t.clone()
        fp = op.fwd(x, out_dtype=torch.float32, planes=split_planes(x)).t.clone()
        dp = op.dgrad(dy, x, dx_dtype=torch.float32, planes=split_planes(dy)).t.clone()
    finally:
        hip.lib().es_conv_set_spb4(old)
    torch.cuda.synchronize()
    for name, t, ref in (("fwd 4-wave", f4, ref_f), ("dgrad 4-wave", d4, ref_d), ("fwd planes", fp, ref_f),
                         ("dgrad planes", dp, ref_d)):
        assert torch.equal(t, ref), (name, float((t - ref).abs().max()))


def test_split_planes_exact():
    """es_split_planes: the three bf16 planes sum exactly to the fp32 value (k-permuted layout)."""
    from expertsim.layers import Act, split_planes
    x = Act.nhwc(3, 64, 5, 7, torch.float32, DEV)
    x.t.normal_()
    x.t.mul_(torch.logspace(-20, 20, x.t.numel(), device=DEV).reshape(x.t.shape))
    p = split_planes(x).float().reshape(3 * 5 * 7, 2, 3, 32)
    s = p[:, :, 0] + p[:, :, 1] + p[:, :, 2]                     # exact: the planes' bits do not overlap
    perm = [(4 * (q >> 3) + (q & 7)) if (q & 7) < 4 else (16 + 4 * (q >> 3) + (q & 7) - 4) for q in range(32)]
    ref = x.t.reshape(3 * 5 * 7, 2, 32)[:, :, perm]
    assert torch.equal(s, ref)
