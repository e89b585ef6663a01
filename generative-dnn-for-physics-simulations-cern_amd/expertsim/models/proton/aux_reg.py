"""Proton-ZDC auxiliary regressor — reference: expertsim/models/proton/aux_reg.py:11-131.

Program: conv5 s2 p1 1->32 -> GN(8) -> ReLU -> maxpool 2 s1 ; two residual blocks
[conv5 s2 p2 -> GN -> ReLU -> conv5 p2 -> GN] + [conv1x1 s2 -> GN], ReLU, maxpool 2 s1 (Norm2d
picks 32 groups for 32 and 64 channels, aux_reg.py:48-53) ; mean over (h,w) ; MLP head
64->128 LN LReLU Dropout(0.3) -> 64 LN LReLU Dropout(0.3) -> 2.
56x30 -> 27x14 -> 26x13 -> 13x7 -> 12x6 -> 6x3 -> 5x2.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from ... import hip
from ...layers import (Act, ConvOp, MaxPool, NormOp, avgpool_bwd, avgpool_fwd, copy_act)
from ..base import ExpertModule, build_tree, get_module

SLOPE = 0.1
P_DROP = 0.3
FE = "feature_extractor."


def _groups(c, groups=32):
    g = min(groups, c)
    while c % g != 0 and g > 1:
        g -= 1
    return g


class AuxReg(ExpertModule):
    def __init__(self, strength, output_dim=2, **kwargs):
        super().__init__()
        self.name = "regressor_v3_changed_loss_log_cosh"
        self.strength = strength
        self.output_dim = output_dim
        specs = [(FE + "conv1.0", lambda: nn.Conv2d(1, 32, kernel_size=5, stride=2, padding=1)),
                 (FE + "conv1.1", lambda: nn.GroupNorm(8, 32))]
        for blk, cin, cout in (("res1", 32, 32), ("res2", 32, 64)):
            q = FE + blk + "."
            specs += [
                (q + "conv1.0", lambda ci=cin, co=cout: nn.Conv2d(ci, co, kernel_size=5, stride=2, padding=2)),
                (q + "conv1.1", lambda co=cout: nn.GroupNorm(_groups(co), co)),
                (q + "conv2.0", lambda co=cout: nn.Conv2d(co, co, kernel_size=5, padding=2)),
                (q + "conv2.1", lambda co=cout: nn.GroupNorm(_groups(co), co)),
                (q + "downsample.0", lambda ci=cin, co=cout: nn.Conv2d(ci, co, kernel_size=1, stride=2)),
                (q + "downsample.1", lambda co=cout: nn.GroupNorm(_groups(co), co)),
            ]
        specs += [("regressor.0", lambda: nn.Linear(64, 128)), ("regressor.1", lambda: nn.LayerNorm(128)),
                  ("regressor.4", lambda: nn.Linear(128, 64)), ("regressor.5", lambda: nn.LayerNorm(64)),
                  ("regressor.8", lambda: nn.Linear(64, output_dim))]
        build_tree(self, specs)

    @staticmethod
    def regressor_loss(real_coords, fake_coords):
        diff = fake_coords - real_coords
        return torch.mean(diff + F.softplus(-2.0 * diff) - math.log(2.0))

    def program(self):
        m = lambda n: get_module(self, n)
        conv = lambda n: ConvOp(m(n).weight, m(n).bias, stride=getattr(m(n), "stride", (1,))[0],
                               pad=getattr(m(n), "padding", (0,))[0])
        gn = lambda n: NormOp(hip.NORM_GN, m(n).weight, m(n).bias, groups=m(n).num_groups, eps=m(n).eps)
        ops = {"c1": conv(FE + "conv1.0"), "g1": gn(FE + "conv1.1"), "pool": MaxPool(2, 1)}
        for blk in ("res1", "res2"):
            q = FE + blk + "."
            for part in ("conv1", "conv2", "downsample"):
                ops[blk + part] = conv(q + part + ".0")
                ops[blk + part + "n"] = gn(q + part + ".1")
        ops["l0"] = conv("regressor.0")
        ops["n1"] = NormOp(hip.NORM_LN, m("regressor.1").weight, m("regressor.1").bias)
        ops["l4"] = conv("regressor.4")
        ops["n5"] = NormOp(hip.NORM_LN, m("regressor.5").weight, m("regressor.5").bias)
        ops["l8"] = conv("regressor.8")
        return ops

    def fwd(self, img: Act, seed=0, stream_base=0, train=True, n_offset=0):
        o = self.ops()
        cdt = self.compute_dtype
        x = img
        if img.t.dtype != cdt:
            x = img.like_nhwc(cdt)
            copy_act(img, x)
        relu = hip.chain_struct(hip.ACT_RELU)
        none = hip.chain_struct(hip.ACT_NONE)
        c = {"x": x}
        c["h1"] = o["c1"].fwd(x)
        c["y1"], c["s1"] = o["g1"].fwd(c["h1"], relu)
        c["q1"], c["i1"] = o["pool"].fwd(c["y1"])
        inp = c["q1"]
        for blk in ("res1", "res2"):
            r = {"in": inp}
            r["a"] = o[blk + "conv1"].fwd(inp)
            r["ay"], r["as"] = o[blk + "conv1n"].fwd(r["a"], relu)
            r["b"] = o[blk + "conv2"].fwd(r["ay"])
            r["d"] = o[blk + "downsample"].fwd(inp)
            r["dy"], r["ds"] = o[blk + "downsamplen"].fwd(r["d"], none)
            r["bs"] = o[blk + "conv2n"].stats(r["b"])
            r["out"] = r["b"].like_nhwc()
            nm = o[blk + "conv2n"].norm_struct(*r["bs"])
            import ctypes as C
            hip.call("es_norm_act_fwd", C.byref(r["b"].view), r["b"].dt, C.byref(nm), C.byref(relu),
                     C.byref(r["dy"].view), r["dy"].dt, r["dy"].ptr, r["b"].ptr, C.byref(r["out"].view),
                     r["out"].dt, r["out"].ptr, hip.stream_ptr())
            r["q"], r["qi"] = o["pool"].fwd(r["out"])
            c[blk] = r
            inp = r["q"]
        c["f"] = avgpool_fwd(inp)
        fc = c["f"]
        if cdt != torch.float32:
            fc = c["f"].like_nhwc(cdt)
            copy_act(c["f"], fc)
        c["fc"] = fc
        d0 = hip.dropout_struct(P_DROP, seed, stream_base + 0, enabled=train)
        d1 = hip.dropout_struct(P_DROP, seed, stream_base + 1, enabled=train)
        hip.set_index_offset(d0, n_offset, 128)
        hip.set_index_offset(d1, n_offset, 64)
        c["ch0"] = hip.chain_struct(hip.ACT_LRELU, SLOPE, d0, dropout_first=False)
        c["ch1"] = hip.chain_struct(hip.ACT_LRELU, SLOPE, d1, dropout_first=False)
        c["r0"] = o["l0"].fwd(fc)
        c["r1"], c["rs1"] = o["n1"].fwd(c["r0"], c["ch0"])
        c["r4"] = o["l4"].fwd(c["r1"])
        c["r5"], c["rs5"] = o["n5"].fwd(c["r4"], c["ch1"])
        out = o["l8"].fwd(c["r5"], out_dtype=torch.float32)
        return out, c

    def bwd(self, c, dout: Act, input_grad=True):
        o = self.ops()
        cdt = self.compute_dtype
        g = lambda n, a="weight": getattr(get_module(self, n), a).grad
        relu = hip.chain_struct(hip.ACT_RELU)
        none = hip.chain_struct(hip.ACT_NONE)
        d = dout
        if cdt != torch.float32:
            d = dout.like_nhwc(cdt)
            copy_act(dout, d)
        o["l8"].wgrad(d, c["r5"], g("regressor.8"), g("regressor.8", "bias"))
        dr5 = o["l8"].dgrad(d, c["r5"])
        dr4 = o["n5"].bwd(c["r4"], c["rs5"], c["ch1"], dr5, dgamma=g("regressor.5"), dbeta=g("regressor.5", "bias"), dsum=g("regressor.4", "bias"))
        o["l4"].wgrad(dr4, c["r1"], g("regressor.4"), None)
        dr1 = o["l4"].dgrad(dr4, c["r1"])
        dr0 = o["n1"].bwd(c["r0"], c["rs1"], c["ch0"], dr1, dgamma=g("regressor.1"), dbeta=g("regressor.1", "bias"), dsum=g("regressor.0", "bias"))
        o["l0"].wgrad(dr0, c["fc"], g("regressor.0"), None)
        df = o["l0"].dgrad(dr0, c["fc"], dx_dtype=torch.float32)
        last = c["res2"]["q"]
        dcur = avgpool_bwd(df, last.dims, cdt, df.t.device)
        for blk in ("res2", "res1"):
            r = c[blk]
            q = FE + blk + "."
            dout_blk = o["pool"].bwd(dcur, r["qi"], r["out"].dims, cdt)
            # out = relu(gn2(b) + gn_ds(d)): both branches see dout * (out > 0)
            db = o[blk + "conv2n"].bwd(r["b"], r["bs"], relu, dout_blk, act_ref=r["out"],
                                       dgamma=g(q + "conv2.1"), dbeta=g(q + "conv2.1", "bias"), dsum=g(q + "conv2.0", "bias"))
            dd = o[blk + "downsamplen"].bwd(r["d"], r["ds"], relu, dout_blk, act_ref=r["out"],
                                            dgamma=g(q + "downsample.1"), dbeta=g(q + "downsample.1", "bias"), dsum=g(q + "downsample.0", "bias"))
            o[blk + "conv2"].wgrad(db, r["ay"], g(q + "conv2.0"), None)
            day = o[blk + "conv2"].dgrad(db, r["ay"])
            da = o[blk + "conv1n"].bwd(r["a"], r["as"], relu, day, dgamma=g(q + "conv1.1"), dbeta=g(q + "conv1.1", "bias"), dsum=g(q + "conv1.0", "bias"))
            o[blk + "conv1"].wgrad(da, r["in"], g(q + "conv1.0"), None)
            o[blk + "downsample"].wgrad(dd, r["in"], g(q + "downsample.0"), None)
            din = o[blk + "conv1"].dgrad(da, r["in"])
            o[blk + "downsample"].dgrad(dd, r["in"], dx=din, beta=1.0)
            dcur = din
        dy1 = o["pool"].bwd(dcur, c["i1"], c["y1"].dims, cdt)
        dh1 = o["g1"].bwd(c["h1"], c["s1"], relu, dy1, dgamma=g(FE + "conv1.1"), dbeta=g(FE + "conv1.1", "bias"), dsum=g(FE + "conv1.0", "bias"))
        o["c1"].wgrad(dh1, c["x"], g(FE + "conv1.0"), None)
        if not input_grad:
            return None
        return o["c1"].dgrad(dh1, c["x"], dx_dtype=torch.float32)

    def forward(self, x):
        from ..autograd import aux_apply
        if x.dim() == 3:
            x = x.unsqueeze(1)
        return aux_apply(self, x)
