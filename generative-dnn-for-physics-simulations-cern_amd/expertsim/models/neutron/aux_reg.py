"""Neutron-ZDC auxiliary max-pixel regressor — reference: expertsim/models/neutron/aux_reg.py:8-81.

Program (train): four [conv3 -> BN -> LReLU -> Dropout(0.2)] stages with max pools (2,2), (2,1),
(2,1) after the first three, a 1x1 conv 256->64 (no bias) -> BN -> LReLU, global average pool,
Linear 64->2.  44x44 -> 42x42 -> 21x21 -> 19x19 -> 9x19 -> 7x17 -> 3x17 -> 1x15.
Dropout follows the activation here (aux_reg.py:15-17), unlike the generator.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from ... import hip
from ...layers import Act, ConvOp, MaxPool, NormOp, avgpool_bwd, avgpool_fwd, copy_act
from ..base import ExpertModule, build_tree, get_module

SLOPE = 0.1
P_DROP = 0.2
FE = "feature_extractor."


class AuxRegNeutron(ExpertModule):
    def __init__(self, strength, **kwargs):
        super().__init__()
        self.name = "aux-architecture-1"
        self.strength = strength
        build_tree(self, [
            (FE + "conv1", lambda: nn.Conv2d(1, 32, kernel_size=3)),
            (FE + "conv1_bd.0", lambda: nn.BatchNorm2d(32)),
            (FE + "conv2", lambda: nn.Conv2d(32, 64, kernel_size=3)),
            (FE + "conv2_bd.0", lambda: nn.BatchNorm2d(64)),
            (FE + "conv3", lambda: nn.Conv2d(64, 128, kernel_size=3)),
            (FE + "conv3_bd.0", lambda: nn.BatchNorm2d(128)),
            (FE + "conv4", lambda: nn.Conv2d(128, 256, kernel_size=3)),
            (FE + "conv4_bd.0", lambda: nn.BatchNorm2d(256)),
            (FE + "reduce.0", lambda: nn.Conv2d(256, 64, kernel_size=1, bias=False)),
            (FE + "reduce.1", lambda: nn.BatchNorm2d(64)),
            ("dense", lambda: nn.Linear(64, 2)),
        ])
        get_module(self, "feature_extractor").name = "model_v1"

    @staticmethod
    def regressor_loss(real_coords, fake_coords):
        """aux_reg.py:70-74 (used on host tensors; the train step uses es_gen_losses)."""
        diff = fake_coords - real_coords
        return torch.mean(diff + F.softplus(-2.0 * diff) - math.log(2.0))

    def program(self):
        m = lambda n: get_module(self, n)

        def bn(n):
            b = m(n)
            return NormOp(hip.NORM_BN, b.weight, b.bias, running_mean=b.running_mean, running_var=b.running_var,
                          momentum=b.momentum, eps=b.eps, num_batches=b.num_batches_tracked)
        conv = lambda n: ConvOp(m(n).weight, m(n).bias)
        return {
            "c1": conv(FE + "conv1"), "b1": bn(FE + "conv1_bd.0"), "p1": MaxPool((2, 2)),
            "c2": conv(FE + "conv2"), "b2": bn(FE + "conv2_bd.0"), "p2": MaxPool((2, 1)),
            "c3": conv(FE + "conv3"), "b3": bn(FE + "conv3_bd.0"), "p3": MaxPool((2, 1)),
            "c4": conv(FE + "conv4"), "b4": bn(FE + "conv4_bd.0"),
            "r": conv(FE + "reduce.0"), "rb": bn(FE + "reduce.1"),
            "dense": conv("dense"),
        }

    def _chain(self, seed, stream_base, layer, train):
        if layer is None:
            return hip.chain_struct(hip.ACT_LRELU, SLOPE)
        d = hip.dropout_struct(P_DROP, seed, stream_base + layer, enabled=train)
        return hip.chain_struct(hip.ACT_LRELU, SLOPE, d, dropout_first=False)

    def fwd(self, img: Act, seed=0, stream_base=0, train=True, n_offset=0):
        """n_offset: first sample's index in the expert's global batch (dropout index offset)."""
        o = self.ops()
        cdt = self.compute_dtype
        x = img
        if img.t.dtype != cdt:
            x = img.like_nhwc(cdt)
            copy_act(img, x)
        ch = [self._chain(seed, stream_base, i, train) for i in range(4)] + [self._chain(0, 0, None, train)]
        c = {"x": x, "ch": ch}
        keep = c["keep"] = []   # dropout keep bits: drawn in the forward norm pass, re-read backward

        def bn(name, h, chain):
            hip.set_index_offset(chain.drop, n_offset, h.dims[1] * h.dims[2] * h.dims[3])
            keep.append(hip.attach_keep(chain, h.dims[0] * h.dims[2] * h.dims[3], h.dims[1], h.t.device))
            return o[name].fwd(h, chain, train=train)
        c["h1"] = o["c1"].fwd(x)
        c["y1"], c["s1"] = bn("b1", c["h1"], ch[0])
        c["q1"], c["i1"] = o["p1"].fwd(c["y1"])
        c["h2"] = o["c2"].fwd(c["q1"])
        c["y2"], c["s2"] = bn("b2", c["h2"], ch[1])
        c["q2"], c["i2"] = o["p2"].fwd(c["y2"])
        c["h3"] = o["c3"].fwd(c["q2"])
        c["y3"], c["s3"] = bn("b3", c["h3"], ch[2])
        c["q3"], c["i3"] = o["p3"].fwd(c["y3"])
        c["h4"] = o["c4"].fwd(c["q3"])
        c["y4"], c["s4"] = bn("b4", c["h4"], ch[3])
        c["h5"] = o["r"].fwd(c["y4"])
        c["y5"], c["s5"] = o["rb"].fwd(c["h5"], ch[4], train=train)
        c["f"] = avgpool_fwd(c["y5"])                                   # [B,64] fp32
        out = o["dense"].fwd(c["f"], out_dtype=torch.float32)          # [B,2] fp32 (fp32 GEMM)
        return out, c

    def bwd(self, c, dout: Act, input_grad=True):
        o = self.ops()
        cdt = self.compute_dtype
        g = lambda n, a="weight": getattr(get_module(self, n), a).grad
        ch = c["ch"]
        o["dense"].wgrad(dout, c["f"], g("dense"), g("dense", "bias"))
        df = o["dense"].dgrad(dout, c["f"])
        dy5 = avgpool_bwd(df, c["y5"].dims, cdt, df.t.device)
        dh5 = o["rb"].bwd(c["h5"], c["s5"], ch[4], dy5, dgamma=g(FE + "reduce.1"), dbeta=g(FE + "reduce.1", "bias"))
        o["r"].wgrad(dh5, c["y4"], g(FE + "reduce.0"), None)
        dy4 = o["r"].dgrad(dh5, c["y4"])
        dh4 = o["b4"].bwd(c["h4"], c["s4"], ch[3], dy4, dgamma=g(FE + "conv4_bd.0"), dbeta=g(FE + "conv4_bd.0", "bias"), dsum=g(FE + "conv4", "bias"))
        o["c4"].wgrad(dh4, c["q3"], g(FE + "conv4"), None)
        dq3 = o["c4"].dgrad(dh4, c["q3"])
        dy3 = o["p3"].bwd(dq3, c["i3"], c["y3"].dims, cdt)
        dh3 = o["b3"].bwd(c["h3"], c["s3"], ch[2], dy3, dgamma=g(FE + "conv3_bd.0"), dbeta=g(FE + "conv3_bd.0", "bias"), dsum=g(FE + "conv3", "bias"))
        o["c3"].wgrad(dh3, c["q2"], g(FE + "conv3"), None)
        dq2 = o["c3"].dgrad(dh3, c["q2"])
        dy2 = o["p2"].bwd(dq2, c["i2"], c["y2"].dims, cdt)
        dh2 = o["b2"].bwd(c["h2"], c["s2"], ch[1], dy2, dgamma=g(FE + "conv2_bd.0"), dbeta=g(FE + "conv2_bd.0", "bias"), dsum=g(FE + "conv2", "bias"))
        o["c2"].wgrad(dh2, c["q1"], g(FE + "conv2"), None)
        dq1 = o["c2"].dgrad(dh2, c["q1"])
        dy1 = o["p1"].bwd(dq1, c["i1"], c["y1"].dims, cdt)
        dh1 = o["b1"].bwd(c["h1"], c["s1"], ch[0], dy1, dgamma=g(FE + "conv1_bd.0"), dbeta=g(FE + "conv1_bd.0", "bias"), dsum=g(FE + "conv1", "bias"))
        o["c1"].wgrad(dh1, c["x"], g(FE + "conv1"), None)
        if not input_grad:
            return None
        return o["c1"].dgrad(dh1, c["x"], dx_dtype=torch.float32)

    def forward(self, x):
        from ..autograd import aux_apply
        if x.dim() == 3:
            x = x.unsqueeze(1)
        return aux_apply(self, x)
