"""Neutron-ZDC (44x44) generator — reference: expertsim/models/neutron/generator.py:5-49.

Program (train mode), every step a HIP kernel:
  x0 = [noise | cond]                                  es_copy into one [B,19] row buffer
  fc1 Linear 19->256 -> BN1d -> Dropout(0.2) -> LReLU  implicit GEMM + fused norm/drop/act
  fc2 Linear 256->21632 -> BN1d -> Dropout -> LReLU    (features in the reference's NCHW order)
  view [B,128,13,13] -> NHWC copy
  up x2 + conv3 128->256 -> BN2d -> Dropout -> LReLU   upsample folded into the conv gather
  up x2 + conv3 256->128 -> BN2d -> Dropout -> LReLU   (72 % of the step's FLOPs)
  conv2 128->64 -> BN2d -> Dropout -> LReLU
  conv2 64->1 -> ReLU                                  -> image [B,1,44,44] fp32
Dropout masks come from Philox streams (expertsim/utils/philox.py), layer index 0..4.

``GeneratorNeutron56`` is the declared 56x56 shape extension of BASELINE configs[4] (SURVEY.md
§8(d) C5; no reference model exists, parity unpinned): the same program with fc2 -> 128x16x16,
16 -> up 32 -> conv 30 -> up 60 -> conv 58 -> conv 57 -> conv 56.
"""
from __future__ import annotations


import ctypes as C

import torch
from torch import nn

from ... import hip
from ...layers import Act, ConvOp, NormOp, Upsample, act_bwd, act_fwd, copy_act
from ...utils import philox
from ..base import ExpertModule, build_tree, get_module


SLOPE = 0.1
P_DROP = 0.2


class GeneratorNeutron(ExpertModule):
    base = 13          # fc2 reshapes to 128 x base x base; the image is (4*base - 8)^2

    # the parameters bwd() reports through ready(), in order (data-parallel gradient buckets)
    READY = ("conv_layers.13.weight", "conv_layers.9.weight", "conv_layers.5.weight", "conv_layers.0.weight",
             "fc2.0.weight", "fc1.0.weight")

    def __init__(self, noise_dim, cond_dim, di_strength, in_strength, **kwargs):
        super().__init__()
        self.name = "Generator-neutron-1-original-architecture"
        self.di_strength = di_strength
        self.in_strength = in_strength
        self.noise_dim, self.cond_dim = int(noise_dim), int(cond_dim)
        k = self.base
        self.image_shape = (4 * k - 8, 4 * k - 8)
        self.fc2_features = 128 * k * k
        build_tree(self, [
            ("fc1.0", lambda: nn.Linear(self.noise_dim + self.cond_dim, 256)),
            ("fc1.1", lambda: nn.BatchNorm1d(256)),
            ("fc2.0", lambda: nn.Linear(256, self.fc2_features)),
            ("fc2.1", lambda: nn.BatchNorm1d(self.fc2_features)),
            ("conv_layers.0", lambda: nn.Conv2d(128, 256, kernel_size=(3, 3))),
            ("conv_layers.1", lambda: nn.BatchNorm2d(256)),
            ("conv_layers.5", lambda: nn.Conv2d(256, 128, kernel_size=(3, 3))),
            ("conv_layers.6", lambda: nn.BatchNorm2d(128)),
            ("conv_layers.9", lambda: nn.Conv2d(128, 64, kernel_size=(2, 2))),
            ("conv_layers.10", lambda: nn.BatchNorm2d(64)),
            ("conv_layers.13", lambda: nn.Conv2d(64, 1, kernel_size=(2, 2))),
        ])

    # --------------------------------------------------------------------------- program
    def program(self):
        m = lambda n: get_module(self, n)
        conv = lambda n, up=None: ConvOp(m(n).weight, m(n).bias, upsample=up)

        def bn(n):
            b = m(n)
            return NormOp(hip.NORM_BN, b.weight, b.bias, running_mean=b.running_mean,
                          running_var=b.running_var, momentum=b.momentum, eps=b.eps,
                          num_batches=b.num_batches_tracked)
        k = self.base
        return {
            "fc1": conv("fc1.0"), "bn1": bn("fc1.1"),
            "fc2": conv("fc2.0"), "bn2": bn("fc2.1"),
            "c0": conv("conv_layers.0", Upsample((k, k), scale=(2, 2))), "bn3": bn("conv_layers.1"),
            "c5": conv("conv_layers.5", Upsample((2 * k - 2, 2 * k - 2), scale=(2, 2))), "bn4": bn("conv_layers.6"),
            "c9": conv("conv_layers.9"), "bn5": bn("conv_layers.10"),
            "c13": conv("conv_layers.13"),
        }

    def _chain(self, seed, stream_base, layer, train):
        d = hip.dropout_struct(P_DROP, seed, stream_base + layer, enabled=train)
        return hip.chain_struct(hip.ACT_LRELU, SLOPE, d, dropout_first=True)

    # --------------------------------------------------------------------------- forward
    def _norm_shapes(self):
        """(channels, side) of the five normalised tensors, the order of the dropout layers 0..4."""
        k = self.base
        return ((256, 1), (self.fc2_features, 1), (256, 2 * k - 2), (128, 4 * k - 6), (64, 4 * k - 7))

    def keep_plan(self, B, dev, seed=0, stream_base=0, train=True, n_offset=0):
        """The five dropout chains of one forward and their keep-bit buffers [rows][C/8] (allocated on
        the current stream): the forward norm passes draw the masks into them, the backward re-reads
        them.  Returns (chains, buffers)."""
        ch = [self._chain(seed, stream_base, i, train) for i in range(5)]
        keep = [hip.attach_keep(ch[i], B * s * s, c, dev) for i, (c, s) in enumerate(self._norm_shapes())]
        for i, (c, s) in enumerate(self._norm_shapes()):
            hip.set_index_offset(ch[i].drop, n_offset, s * s * c)
        return ch, keep

    def draw_keep(self, plan, B):
        """Draw a keep_plan's masks now, on the current stream (es_dropout_keep_bits: the bits the
        norm passes would draw), and mark the chains so the forward reads them.  The caller runs this
        on a side stream beside work that leaves the chip's VALUs idle and joins it before fwd(pre=plan)
        (moe.MoEWrapper: the second forward's masks during the discriminator step)."""
        ch, keep = plan
        for i, (c, s) in enumerate(self._norm_shapes()):
            if keep[i] is None:
                continue
            v = hip.make_view((B, c, s, s), (s * s * c, 1, s * c, c))
            hip.call("es_dropout_keep_bits", C.byref(v), C.byref(ch[i]), hip.stream_ptr())
            ch[i].keep_ready = 1
        return plan

    def fwd(self, noise: torch.Tensor, cond: torch.Tensor, seed=0, stream_base=0, train=True, n_offset=0,
            pre=None):
        """noise [B,10] fp32, cond [B,9] fp32 (device) -> (image Act [B,1,44,44] fp32 NHWC, ctx).
        n_offset: index of the first sample in the expert's global batch (data parallel: dropout
        masks are drawn at the global sample index, expertsim/utils/philox.py).  pre: a keep_plan of
        the same arguments whose masks draw_keep has drawn (the norm passes read them)."""
        o = self.ops()
        k, F2 = self.base, self.fc2_features
        cdt = self.compute_dtype
        dev = noise.device
        B = noise.shape[0]
        x0 = Act.rows(B, self.noise_dim + self.cond_dim, cdt, dev)
        x0m = x0.t.view(B, -1)
        copy_act(Act.of(noise), Act.of(x0m[:, :self.noise_dim]))
        copy_act(Act.of(cond), Act.of(x0m[:, self.noise_dim:]))
        # dropout keep bits, drawn once (in the forward norm pass, or ahead by draw_keep) and re-read
        # by the backward
        ch, keep = pre if pre is not None else self.keep_plan(B, dev, seed, stream_base, train, n_offset)
        h1 = o["fc1"].fwd(x0)
        y1, s1 = o["bn1"].fwd(h1, ch[0], train=train)
        h2 = o["fc2"].fwd(y1, bn_stats=train)        # (ring FWD over 16-row pixel blocks: stats in its epilogue)
        y2, s2 = o["bn2"].fwd(h2, ch[1], train=train)
        # [B, 21632] rows are NCHW [B,128,13,13]; re-layout to NHWC for the vector gather
        y2n = Act.nhwc(B, 128, k, k, cdt, dev)
        copy_act(Act(y2.t, (B, 128, k, k), (F2, k * k, k, 1)), y2n)
        h3 = o["c0"].fwd(y2n, bn_stats=train)         # BatchNorm statistics from the conv epilogue
        y3, s3 = o["bn3"].fwd(h3, ch[2], train=train)
        h4 = o["c5"].fwd(y3, bn_stats=train)
        y4, s4 = o["bn4"].fwd(h4, ch[3], train=train)
        h5 = o["c9"].fwd(y4, bn_stats=train)
        y5, s5 = o["bn5"].fwd(h5, ch[4], train=train)
        h6 = o["c13"].fwd(y5, out_dtype=torch.float32)
        img = act_fwd(h6, hip.chain_struct(hip.ACT_RELU))
        ctx = dict(x0=x0, h1=h1, y1=y1, s1=s1, h2=h2, y2=y2, s2=s2, y2n=y2n, h3=h3, y3=y3, s3=s3,
                   h4=h4, y4=y4, s4=s4, h5=h5, y5=y5, s5=s5, h6=h6, ch=ch, keep=keep)
        return img, ctx

    # --------------------------------------------------------------------------- backward
    def bwd(self, ctx, dimg: Act, ready=None):
        """Accumulate parameter gradients (flat grad buffer) for d loss / d image.  ready(name): the
        gradients from parameter ``name`` to the end of the flat buffer are final (DP buckets)."""
        ready = ready or (lambda name: None)
        o = self.ops()
        cdt = self.compute_dtype
        g = lambda n, a: getattr(get_module(self, n), a).grad
        ch = ctx["ch"]
        dh6 = act_bwd(ctx["h6"], hip.chain_struct(hip.ACT_RELU), dimg, dx_dtype=cdt)
        o["c13"].wgrad(dh6, ctx["y5"], g("conv_layers.13", "weight"), g("conv_layers.13", "bias"))
        ready("conv_layers.13.weight")
        # (the thin dgrad also runs bn5's backward reduction over dy5, ConvOp.dgrad bn_reduce)
        dy5 = o["c13"].dgrad(dh6, ctx["y5"], bn_reduce=(o["bn5"], ctx["h5"], ctx["s5"], ch[4]))
        dh5 = o["bn5"].bwd(ctx["h5"], ctx["s5"], ch[4], dy5, dgamma=g("conv_layers.10", "weight"),
                           dbeta=g("conv_layers.10", "bias"), dsum=g("conv_layers.9", "bias"))
        o["c9"].wgrad(dh5, ctx["y4"], g("conv_layers.9", "weight"), None)
        ready("conv_layers.9.weight")
        # the dgrad epilogue also runs bn4's backward reduction over dy4 (ConvOp.dgrad bn_reduce)
        dy4 = o["c9"].dgrad(dh5, ctx["y4"], bn_reduce=(o["bn4"], ctx["h4"], ctx["s4"], ch[3]))
        dh4 = o["bn4"].bwd(ctx["h4"], ctx["s4"], ch[3], dy4, dgamma=g("conv_layers.6", "weight"),
                           dbeta=g("conv_layers.6", "bias"), dsum=g("conv_layers.5", "bias"))
        o["c5"].wgrad(dh4, ctx["y3"], g("conv_layers.5", "weight"), None)
        ready("conv_layers.5.weight")
        # no fused reduction here: the 256 x 256 sub-pixel DGRAD has no registers to spare for it in
        # bf16 (585 -> 871 us for a 146 us reduce pass), and a staged-epilogue fold in the split-fp32
        # ring DGRAD cost more than the reduce pass it removes (B = 1024 c5 DGRAD 3.16 -> 3.62 ms,
        # DESIGN.md §4; removed in round 5)
        dy3 = o["c5"].dgrad(dh4, ctx["y3"])
        dh3 = o["bn3"].bwd(ctx["h3"], ctx["s3"], ch[2], dy3, dgamma=g("conv_layers.1", "weight"),
                           dbeta=g("conv_layers.1", "bias"), dsum=g("conv_layers.0", "bias"))
        o["c0"].wgrad(dh3, ctx["y2n"], g("conv_layers.0", "weight"), None)
        ready("conv_layers.0.weight")
        dy2n = o["c0"].dgrad(dh3, ctx["y2n"])
        B, k, F2 = dy2n.dims[0], self.base, self.fc2_features
        dy2 = Act.rows(B, F2, cdt, dy2n.t.device)
        copy_act(dy2n, Act(dy2.t, (B, 128, k, k), (F2, k * k, k, 1)))
        dh2 = o["bn2"].bwd(ctx["h2"], ctx["s2"], ch[1], dy2, dgamma=g("fc2.1", "weight"),
                           dbeta=g("fc2.1", "bias"), dsum=g("fc2.0", "bias"))
        o["fc2"].wgrad(dh2, ctx["y1"], g("fc2.0", "weight"), None)
        ready("fc2.0.weight")
        # fp32 dense output: lets the K = 21632 GEMM split K across workgroups (8 output tiles)
        dy1 = o["fc2"].dgrad(dh2, ctx["y1"], dx_dtype=torch.float32)
        dh1 = o["bn1"].bwd(ctx["h1"], ctx["s1"], ch[0], dy1, dx_dtype=cdt, dgamma=g("fc1.1", "weight"),
                           dbeta=g("fc1.1", "bias"), dsum=g("fc1.0", "bias"))
        o["fc1"].wgrad(dh1, ctx["x0"], g("fc1.0", "weight"), None)
        ready("fc1.0.weight")

    # --------------------------------------------------------------------------- nn.Module API
    def forward(self, noise, cond):
        """Reference signature (generator.py:42): image [B,1,44,44]."""
        from ..autograd import generator_apply
        return generator_apply(self, noise, cond)


class GeneratorNeutron56(GeneratorNeutron):
    """Declared 56x56 extension (BASELINE configs[4]) -- parity unpinned."""
    base = 16

    def __init__(self, noise_dim, cond_dim, di_strength, in_strength, **kwargs):
        super().__init__(noise_dim, cond_dim, di_strength, in_strength, **kwargs)
        self.name = "Generator-neutron56-declared-extension"
