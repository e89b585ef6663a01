"""Proton-ZDC (56x30) generator — reference: expertsim/models/proton/generator.py:5-52.

Program (no dropout in this family):
  fc1 Linear 19->256 -> LN -> LReLU ; fc2 Linear 256->92160 -> LN(92160) -> LReLU
  view [B,512,18,10] -> NHWC ; up x2 (36x20) + conv4 p1 512->256 (35x19) -> GN(32) -> LReLU
  resize to 56x30 (nearest, folded into the gather) + conv4 p1 256->128 (55x29) -> GN(32) -> LReLU
  conv3 p1 128->64 (55x29) -> GN(32) -> LReLU ; conv2 p1 64->1 (56x30) -> ReLU
"""
from __future__ import annotations

import torch
from torch import nn

from ... import hip
from ...layers import Act, ConvOp, NormOp, Upsample, act_bwd, act_fwd, copy_act
from ..base import ExpertModule, build_tree, get_module

SLOPE = 0.1
FEAT = 512 * 18 * 10


class Generator(ExpertModule):
    # the parameters bwd() reports through ready(), in order (data-parallel gradient buckets)
    READY = ("conv_layers.11.weight", "conv_layers.8.weight", "conv_layers.5.weight", "conv_layers.1.weight",
             "fc2.0.weight", "fc1.0.weight")

    def __init__(self, noise_dim, cond_dim, di_strength, in_strength, **kwargs):
        super().__init__()
        self.name = "Generator-v5-bigkernel-res56x30"
        self.di_strength = di_strength
        self.in_strength = in_strength
        self.noise_dim, self.cond_dim = int(noise_dim), int(cond_dim)
        self.image_shape = (56, 30)
        build_tree(self, [
            ("fc1.0", lambda: nn.Linear(self.noise_dim + self.cond_dim, 256)),
            ("fc1.1", lambda: nn.LayerNorm(256)),
            ("fc2.0", lambda: nn.Linear(256, FEAT)),
            ("fc2.1", lambda: nn.LayerNorm(FEAT)),
            ("conv_layers.1", lambda: nn.Conv2d(512, 256, kernel_size=(4, 4), padding=(1, 1))),
            ("conv_layers.2", lambda: nn.GroupNorm(32, 256)),
            ("conv_layers.5", lambda: nn.Conv2d(256, 128, kernel_size=(4, 4), padding=(1, 1))),
            ("conv_layers.6", lambda: nn.GroupNorm(32, 128)),
            ("conv_layers.8", lambda: nn.Conv2d(128, 64, kernel_size=(3, 3), padding=(1, 1))),
            ("conv_layers.9", lambda: nn.GroupNorm(32, 64)),
            ("conv_layers.11", lambda: nn.Conv2d(64, 1, kernel_size=(2, 2), padding=(1, 1))),
        ])

    def program(self):
        m = lambda n: get_module(self, n)
        conv = lambda n, up=None: ConvOp(m(n).weight, m(n).bias, pad=1 if n.startswith("conv") else 0, upsample=up)
        ln = lambda n: NormOp(hip.NORM_LN, m(n).weight, m(n).bias, eps=m(n).eps)
        gn = lambda n: NormOp(hip.NORM_GN, m(n).weight, m(n).bias, groups=32, eps=m(n).eps)
        return {
            "fc1": conv("fc1.0"), "ln1": ln("fc1.1"), "fc2": conv("fc2.0"), "ln2": ln("fc2.1"),
            "c1": conv("conv_layers.1", Upsample((18, 10), scale=(2, 2))), "gn1": gn("conv_layers.2"),
            "c5": conv("conv_layers.5", Upsample((35, 19), out_hw=(56, 30))), "gn2": gn("conv_layers.6"),
            "c8": conv("conv_layers.8"), "gn3": gn("conv_layers.9"),
            "c11": conv("conv_layers.11"),
        }

    def fwd(self, noise, cond, seed=0, stream_base=0, train=True, n_offset=0):
        o = self.ops()
        cdt = self.compute_dtype
        dev = noise.device
        B = noise.shape[0]
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        x0 = Act.rows(B, self.noise_dim + self.cond_dim, cdt, dev)
        x0m = x0.t.view(B, -1)
        copy_act(Act.of(noise), Act.of(x0m[:, :self.noise_dim]))
        copy_act(Act.of(cond), Act.of(x0m[:, self.noise_dim:]))
        c = {"x0": x0}
        c["h1"] = o["fc1"].fwd(x0)
        c["y1"], c["s1"] = o["ln1"].fwd(c["h1"], lr)
        c["h2"] = o["fc2"].fwd(c["y1"])
        c["y2"], c["s2"] = o["ln2"].fwd(c["h2"], lr)
        c["y2n"] = Act.nhwc(B, 512, 18, 10, cdt, dev)
        copy_act(Act(c["y2"].t, (B, 512, 18, 10), (FEAT, 180, 10, 1)), c["y2n"])
        c["h3"] = o["c1"].fwd(c["y2n"])
        c["y3"], c["s3"] = o["gn1"].fwd(c["h3"], lr)
        c["h4"] = o["c5"].fwd(c["y3"])
        c["y4"], c["s4"] = o["gn2"].fwd(c["h4"], lr)
        c["h5"] = o["c8"].fwd(c["y4"])
        c["y5"], c["s5"] = o["gn3"].fwd(c["h5"], lr)
        c["h6"] = o["c11"].fwd(c["y5"], out_dtype=torch.float32)
        img = act_fwd(c["h6"], hip.chain_struct(hip.ACT_RELU))
        return img, c

    def bwd(self, c, dimg: Act, ready=None):
        """ready(name): gradients from parameter ``name`` to the end of the flat buffer are final."""
        ready = ready or (lambda name: None)
        o = self.ops()
        cdt = self.compute_dtype
        g = lambda n, a="weight": getattr(get_module(self, n), a).grad
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        dh6 = act_bwd(c["h6"], hip.chain_struct(hip.ACT_RELU), dimg, dx_dtype=cdt)
        o["c11"].wgrad(dh6, c["y5"], g("conv_layers.11"), g("conv_layers.11", "bias"))
        ready("conv_layers.11.weight")
        dy5 = o["c11"].dgrad(dh6, c["y5"])
        dh5 = o["gn3"].bwd(c["h5"], c["s5"], lr, dy5, dgamma=g("conv_layers.9"), dbeta=g("conv_layers.9", "bias"), dsum=g("conv_layers.8", "bias"))
        o["c8"].wgrad(dh5, c["y4"], g("conv_layers.8"), None)
        ready("conv_layers.8.weight")
        dy4 = o["c8"].dgrad(dh5, c["y4"])
        dh4 = o["gn2"].bwd(c["h4"], c["s4"], lr, dy4, dgamma=g("conv_layers.6"), dbeta=g("conv_layers.6", "bias"), dsum=g("conv_layers.5", "bias"))
        o["c5"].wgrad(dh4, c["y3"], g("conv_layers.5"), None)
        ready("conv_layers.5.weight")
        dy3 = o["c5"].dgrad(dh4, c["y3"])
        dh3 = o["gn1"].bwd(c["h3"], c["s3"], lr, dy3, dgamma=g("conv_layers.2"), dbeta=g("conv_layers.2", "bias"), dsum=g("conv_layers.1", "bias"))
        o["c1"].wgrad(dh3, c["y2n"], g("conv_layers.1"), None)
        ready("conv_layers.1.weight")
        dy2n = o["c1"].dgrad(dh3, c["y2n"])
        B = dy2n.dims[0]
        dy2 = Act.rows(B, FEAT, cdt, dy2n.t.device)
        copy_act(dy2n, Act(dy2.t, (B, 512, 18, 10), (FEAT, 180, 10, 1)))
        dh2 = o["ln2"].bwd(c["h2"], c["s2"], lr, dy2, dgamma=g("fc2.1"), dbeta=g("fc2.1", "bias"), dsum=g("fc2.0", "bias"))
        o["fc2"].wgrad(dh2, c["y1"], g("fc2.0"), None)
        ready("fc2.0.weight")
        dy1 = o["fc2"].dgrad(dh2, c["y1"], dx_dtype=torch.float32)   # fp32: split-K over K = 92160
        dh1 = o["ln1"].bwd(c["h1"], c["s1"], lr, dy1, dx_dtype=cdt, dgamma=g("fc1.1"), dbeta=g("fc1.1", "bias"), dsum=g("fc1.0", "bias"))
        o["fc1"].wgrad(dh1, c["x0"], g("fc1.0"), None)
        ready("fc1.0.weight")

    def forward(self, noise, cond):
        from ..autograd import generator_apply
        return generator_apply(self, noise, cond)
