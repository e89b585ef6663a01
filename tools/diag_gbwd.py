"""Diagnostic: generator backward of the HIP path vs the oracle's autograd for one fixed upstream
image gradient, per parameter tensor, over several batch sizes (fp32 mode).

usage: python tools/diag_gbwd.py <arch> <B> [<B> ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from expertsim.layers import Act  # noqa: E402
from oracle import expertsim_oracle as O  # noqa: E402

arch = sys.argv[1]
for B in [int(b) for b in sys.argv[2:]]:
    moe, opts, cfg = bench.build(arch, 1, "fp32", 1234, torch.device("cuda"))
    G = moe.generators[0]
    gen = torch.Generator().manual_seed(B)
    noise, cond = torch.randn(B, 10, generator=gen), torch.randn(B, 9, generator=gen)
    H, W = G.image_shape
    dimg = torch.randn(B, 1, H, W, generator=gen)
    G.zero_grads()
    img, ctx = G.fwd(noise.cuda(), cond.cuda(), seed=1234, stream_base=0, train=True)
    G.bwd(ctx, Act.of(dimg.cuda().contiguous()))
    torch.cuda.synchronize()
    mine = {n: p.grad.detach().double().cpu() for n, p in G.named_parameters()}
    st = O.build_all(arch, 1, 1234)
    P = st["G"][0]
    leaves = {k: P[k].requires_grad_(True) for k in O.trainable(P)}
    out = O.generator_forward(arch, P, noise, cond, drop=O.Dropper(1234, 0, 0, 0))
    (out * dimg).sum().backward()
    ie = float((img.torch_nchw().cpu() - out.detach()).abs().max() / out.detach().abs().max())
    print(f"== {arch} B={B}: image rel err {ie:.2e}")
    rows = []
    for k, t in leaves.items():
        a, b = mine[k], t.grad.double()
        rows.append((float((a - b).norm() / max(b.norm(), 1e-30)), k, float(b.norm())))
    for r in sorted(rows, reverse=True)[:8]:
        print(f"   {r[1]:28s} normrel {r[0]:.2e}  |g| {r[2]:.3e}")
