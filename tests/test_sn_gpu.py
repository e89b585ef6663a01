"""Spectral norm kernels (torch.nn.utils.spectral_norm, one power iteration per train-mode forward;
reference discriminators proton/discriminator.py:122-146, neutron/discriminator.py:12-39).

* the batched launches (es_sn_power_iter_batch / es_sn_bwd_batch: one block per layer) are
  bit-identical to the per-layer kernels (es_sn_power_iter / es_sn_bwd): each block runs the same
  per-layer body;
* sigma, the updated u / v and the weight_orig gradient agree with torch CPU fp32 (spectral_norm's
  own power iteration; autograd through W / sigma with u, v constant) to <= 1e-5 relative.
Shapes: the discriminator's layers (32x9, 16x288, 64x128, 1x64, neutron fc1 128x1305) plus odd ones.
"""
import copy

import pytest
import torch

from expertsim.layers import SpectralNorm

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(32, 9), (16, 288), (64, 128), (1, 64), (5, 7), (3, 1000), (128, 1305)]


def _modules():
    torch.manual_seed(0)
    return [torch.nn.utils.spectral_norm(torch.nn.Linear(wd, h)) for h, wd in SHAPES]


def _to_dev(mods):
    out = []
    for m in mods:
        m = copy.deepcopy(m).to(DEV)
        out.append(m)
    return out


def _torch_power_iter(m):
    """torch's spectral_norm training step on CPU: returns (sigma, u, v) and updates m in place."""
    w = m.weight_orig.detach()
    u, v = m.weight_u.clone(), m.weight_v.clone()
    with torch.no_grad():
        v = torch.nn.functional.normalize(torch.mv(w.t(), u), dim=0, eps=1e-12)
        u = torch.nn.functional.normalize(torch.mv(w, v), dim=0, eps=1e-12)
        sigma = torch.dot(u, torch.mv(w, v))
    return sigma, u, v


def test_sn_power_iteration_batched_matches_per_layer_and_torch():
    ref = _modules()
    a, b = _to_dev(ref), _to_dev(ref)
    per = [SpectralNorm(m).sigma(update=True) for m in a]
    bat = SpectralNorm.sigma_many([SpectralNorm(m) for m in b], update=True)
    torch.cuda.synchronize()
    for i, (h, wd) in enumerate(SHAPES):
        for x, y in zip(per[i], bat[i]):
            assert torch.equal(x, y), (h, wd)
        assert torch.equal(a[i].weight_u, b[i].weight_u) and torch.equal(a[i].weight_v, b[i].weight_v)
        sigma, u, v = _torch_power_iter(ref[i])
        assert abs(float(per[i][0]) - float(sigma)) <= 1e-5 * abs(float(sigma)), (h, wd)
        assert torch.allclose(a[i].weight_u.cpu(), u, rtol=0, atol=1e-5), (h, wd)
        assert torch.allclose(a[i].weight_v.cpu(), v, rtol=0, atol=1e-5), (h, wd)


def test_sn_backward_batched_matches_per_layer_and_torch():
    ref = _modules()
    a, b = _to_dev(ref), _to_dev(ref)
    gen = torch.Generator().manual_seed(1)
    grads = [torch.randn(h, wd, generator=gen) for h, wd in SHAPES]
    sa = [SpectralNorm(m) for m in a]
    sb = [SpectralNorm(m) for m in b]
    sig_a = [s.sigma(update=True) for s in sa]
    sig_b = [s.sigma(update=True) for s in sb]
    dwa = [torch.full((h, wd), 0.25, device=DEV) for h, wd in SHAPES]     # beta=1 accumulates
    dwb = [t.clone() for t in dwa]
    for s, g, sig, d in zip(sa, grads, sig_a, dwa):
        s.bwd(g.to(DEV), sig, d, beta=1.0)
    SpectralNorm.bwd_many([(s, g.to(DEV), sig, d) for s, g, sig, d in zip(sb, grads, sig_b, dwb)], beta=1.0)
    torch.cuda.synchronize()
    for i, (h, wd) in enumerate(SHAPES):
        assert torch.equal(dwa[i], dwb[i]), (h, wd)
        # torch: d/dW_orig of <W_orig / sigma(W_orig; u, v const), g>
        sigma, u, v = _torch_power_iter(ref[i])
        w = ref[i].weight_orig.detach().clone().requires_grad_(True)
        s = torch.dot(u, torch.mv(w, v))
        (w / s * grads[i]).sum().backward()
        want = w.grad + 0.25
        err = (dwa[i].cpu() - want).abs().max() / want.abs().max()
        assert err <= 1e-5, (h, wd, float(err))
