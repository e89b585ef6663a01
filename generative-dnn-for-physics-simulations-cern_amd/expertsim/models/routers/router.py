"""Router MLP + Gumbel-softmax — reference: expertsim/models/routers/router.py:6-26.

Linear 9->128 -> LReLU(0.1) -> 128->64 -> LReLU -> 64->32 -> LReLU -> 32->E, then
softmax((logits - log Exp(1)) / tau) (torch F.gumbel_softmax, hard=False), fused with the argmax /
bincount of moe.py:97-99 in es_router_gumbel.
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

from ... import hip
from ...layers import Act, ConvOp, act_bwd, act_fwd
from ..base import ExpertModule, build_tree, get_module

SLOPE = 0.1
LAYERS = ("fc_layers.0", "fc_layers.2", "fc_layers.4", "fc_layers.6")


class RouterNetwork(ExpertModule):
    def __init__(self, cond_dim, n_experts, **kwargs):
        super().__init__()
        self.name = "router-architecture-2"
        self.n_experts = int(n_experts)
        self.cond_dim = int(cond_dim)
        dims = (self.cond_dim, 128, 64, 32, self.n_experts)
        build_tree(self, [(LAYERS[i], lambda i=i: nn.Linear(dims[i], dims[i + 1])) for i in range(4)])

    def program(self):
        return {n: ConvOp(get_module(self, n).weight, get_module(self, n).bias) for n in LAYERS}

    def fwd(self, cond: torch.Tensor, expo: torch.Tensor, tau: float):
        """cond [B,9] fp32, expo [B,E] Exp(1) draws -> (gates, logits, idx int32, counts int32, ctx)."""
        o = self.ops()
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        x = Act.of(cond.contiguous())
        ctx = {"x": x, "h": [], "a": []}
        a = x
        for i, n in enumerate(LAYERS):
            h = o[n].fwd(a, out_dtype=torch.float32)
            ctx["h"].append(h)
            if i < 3:
                a = act_fwd(h, lr)
                ctx["a"].append(a)
        logits = ctx["h"][-1]
        B, E = cond.shape[0], self.n_experts
        gates = torch.empty(B, E, dtype=torch.float32, device=cond.device)
        idx = torch.empty(B, dtype=torch.int32, device=cond.device)
        counts = torch.zeros(E, dtype=torch.int32, device=cond.device)
        hip.call("es_router_gumbel", logits.ptr, hip.ptr(expo), B, E, float(tau), hip.ptr(gates), hip.ptr(idx),
                 hip.ptr(counts), hip.stream_ptr())
        return gates, logits.rows2d(), idx, counts, ctx

    def bwd(self, ctx, dlogits: torch.Tensor):
        o = self.ops()
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        g = lambda n, a="weight": getattr(get_module(self, n), a).grad
        d = Act.of(dlogits)
        for i in range(3, -1, -1):
            n = LAYERS[i]
            inp = ctx["x"] if i == 0 else ctx["a"][i - 1]
            o[n].wgrad(d, inp, g(n), g(n, "bias"))
            if i == 0:
                break
            da = o[n].dgrad(d, inp)
            d = act_bwd(ctx["h"][i - 1], lr, da)

    def forward(self, cond, tau=1.0, hard=False):
        """Reference signature (router.py:21): returns (gates, logits)."""
        if hard:
            raise NotImplementedError("hard gumbel routing is not used by the reference train step")
        expo = torch.empty(cond.shape[0], self.n_experts, dtype=torch.float32, device=cond.device)
        from ...rng import default_rng
        default_rng().exponential(expo)
        gates, logits, _, _, _ = self.fwd(cond, expo, tau)
        return gates, logits
