"""Normalise-on-load (es_conv_norm_on_load, NormOp.fwd_deferred): the neutron generator's
conv_layers.10 BatchNorm + Dropout + LeakyReLU (neutron/generator.py:33-38) applied by conv_layers.13's
thin fp32 kernels as they load the pre-norm activation, instead of a stored y5.  Same expressions as
the apply pass, so the training step must be BITWISE the materialised one (fp32 parity mode, two
steps: metrics and every parameter), in train mode and for the eval-mode forward; and a conv path
that cannot honour the request must fail loudly instead of reading h as y."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _steps(nol, B=64, steps=2):
    import bench
    from expertsim.models.neutron import generator as gen
    from expertsim.utils.synthetic import make_batch
    old = gen._NOL
    gen._NOL = nol
    try:
        moe, (og, od, oa, orr), cfg = bench.build("neutron", 1, "fp32", 1234, torch.device(DEV))
        for s in range(steps):
            b = make_batch(B, "neutron", seed=40 + s)
            t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
            m = moe.train_step(0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"],
                               t["intensity"], oa, og, od, orr, None, DEV)
        torch.cuda.synchronize()
        g = moe.generators[0]
        g.eval()
        with torch.no_grad():
            img = g(torch.randn(B, 10, generator=torch.Generator().manual_seed(5)).to(DEV), t["cond"])
        g.train()
        torch.cuda.synchronize()
        return ({k: float(v) for k, v in m.items()}, {n: p.detach().clone() for n, p in moe.named_parameters()},
                img.detach().clone())
    finally:
        gen._NOL = old


def test_nol_step_bitwise_equals_materialised():
    ma, pa, ia = _steps(False)
    mb, pb, ib = _steps(True)
    assert ma == mb
    diff = [n for n in pa if not torch.equal(pa[n], pb[n])]
    assert not diff, diff
    assert torch.equal(ia, ib)


def test_nol_request_off_thin_path_fails_loudly():
    """A conv that is not a thin Cout = 1 fp32 conv refuses a pending normalise-on-load request."""
    from expertsim import hip
    from expertsim.layers import Act, ConvOp, NormOp
    hip.lib()
    op = ConvOp(torch.nn.Parameter(torch.randn(16, 64, 2, 2, device=DEV)), None)
    x = Act.nhwc(2, 64, 9, 9, torch.float32, DEV)
    x.t.normal_()
    bn = NormOp(hip.NORM_BN, torch.ones(64, device=DEV), torch.zeros(64, device=DEV),
                running_mean=torch.zeros(64, device=DEV), running_var=torch.ones(64, device=DEV))
    ch = hip.chain_struct(hip.ACT_LRELU, 0.1)
    y, _ = bn.fwd_deferred(x, ch, train=True)
    with pytest.raises(Exception):
        op.fwd(y, out_dtype=torch.float32)
    # the request is cleared after the failed call: a plain conv runs again
    op.fwd(x, out_dtype=torch.float32)
    torch.cuda.synchronize()
