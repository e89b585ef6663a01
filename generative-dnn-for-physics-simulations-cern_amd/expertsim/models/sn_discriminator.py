"""Spectral-norm conv discriminator shared by both ZDC families.

References: expertsim/models/neutron/discriminator.py:6-48 (44x44 input, flatten 16*9*9 = 1296)
and expertsim/models/proton/discriminator.py:116-155 (56x30 input, second pool (2,1), flatten
16*12*12 = 2304).  Each forward in train mode runs one spectral-norm power iteration per layer
(torch.nn.utils.spectral_norm semantics) whose sigma divides the weight inside the GEMM weight
packing, so no host sync and no extra weight pass.

Program:
  SNconv3 1->32 -> GN(8) -> LReLU -> maxpool 2x2
  SNconv3 32->16 -> GN(8) -> LReLU -> maxpool pool2    -> written straight into the fc1 input
                                                         rows in NCHW-flatten order, cond after it
  SNlinear F+9->128 -> LN -> LReLU -> SNlinear 128->64 -> LN -> LReLU (= latent) -> SNlinear 64->1
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn
from torch.nn.utils import spectral_norm

from .. import hip
from ..layers import Act, ConvOp, MaxPool, NormOp, SpectralNorm, channel_sum, copy_act
from .base import ExpertModule, build_tree, get_module

SLOPE = 0.1
LAYERS = ("conv_layers.0", "conv_layers.4", "fc1.0", "fc2.0", "fc3")


class SNDiscriminator(ExpertModule):
    compute_dtype = torch.float32

    def __init__(self, cond_dim, image_shape, pool2, **kwargs):
        super().__init__()
        self.cond_dim = int(cond_dim)
        self.image_shape = tuple(image_shape)
        self.pool2 = tuple(pool2)
        H, W = self.image_shape
        h1, w1 = (H - 2) // 2, (W - 2) // 2
        self.feat_hw = ((h1 - 2 - pool2[0]) // pool2[0] + 1, (w1 - 2 - pool2[1]) // pool2[1] + 1)
        self.flat_dim = 16 * self.feat_hw[0] * self.feat_hw[1]
        build_tree(self, [
            ("conv_layers.0", lambda: spectral_norm(nn.Conv2d(1, 32, kernel_size=3))),
            ("conv_layers.1", lambda: nn.GroupNorm(8, 32)),
            ("conv_layers.4", lambda: spectral_norm(nn.Conv2d(32, 16, kernel_size=3))),
            ("conv_layers.5", lambda: nn.GroupNorm(8, 16)),
            ("fc1.0", lambda: spectral_norm(nn.Linear(self.flat_dim + self.cond_dim, 128))),
            ("fc1.1", lambda: nn.LayerNorm(128)),
            ("fc2.0", lambda: spectral_norm(nn.Linear(128, 64))),
            ("fc2.1", lambda: nn.LayerNorm(64)),
            ("fc3", lambda: spectral_norm(nn.Linear(64, 1))),
        ])

    def program(self):
        m = lambda n: get_module(self, n)
        ops = {}
        for n in LAYERS:
            mod = m(n)
            ops[n] = ConvOp(mod.weight_orig, mod.bias)
            ops["sn:" + n] = SpectralNorm(mod)
        ops["gn1"] = NormOp(hip.NORM_GN, m("conv_layers.1").weight, m("conv_layers.1").bias, groups=8)
        ops["gn2"] = NormOp(hip.NORM_GN, m("conv_layers.5").weight, m("conv_layers.5").bias, groups=8)
        ops["ln1"] = NormOp(hip.NORM_LN, m("fc1.1").weight, m("fc1.1").bias)
        ops["ln2"] = NormOp(hip.NORM_LN, m("fc2.1").weight, m("fc2.1").bias)
        ops["pool1"] = MaxPool(2)
        ops["pool2"] = MaxPool(self.pool2)
        return ops

    # ------------------------------------------------------------------ fused front (d_front.hip)
    # conv_layers.0..3 as the per-image fused kernels (tests switch it off to compare)
    fuse_front = True

    def front_fused(self, x: Act) -> bool:
        """SNconv 1->32 + GN + LReLU + pool as es_dfront_*: fp32, even 3x3-conv output grid (the 2x2
        pool then covers every conv output), image <= 2048 pixels (staged in LDS)."""
        N, Cc, H, W = x.dims
        return (self.fuse_front and x.t.dtype == torch.float32 and Cc == 1 and H >= 4 and W >= 4
                and (H - 2) % 2 == 0 and (W - 2) % 2 == 0 and H * W <= 2048 and (H - 2) * (W - 2) <= 1792)

    # both conv blocks as one per-image kernel pair (d_front2.hip); off: block 1 fused, block 2 on the
    # generic kernels (tests)
    fuse_front2 = True

    def front2_fused(self, x: Act) -> bool:
        N, Cc, H, W = x.dims
        return (self.fuse_front and self.fuse_front2 and x.t.dtype == torch.float32 and Cc == 1
                and self.compute_dtype == torch.float32
                and bool(hip.lib().es_dfront2_ok(H, W, self.pool2[0], self.pool2[1])))

    def _front2_params(self, sig):
        m = lambda n: get_module(self, n)
        c0, gn1, c4, gn2 = m("conv_layers.0"), m("conv_layers.1"), m("conv_layers.4"), m("conv_layers.5")
        p = hip.DFront2Params()
        p.w1, p.sigma1, p.b1 = c0.weight_orig.data_ptr(), sig["conv_layers.0"][0].data_ptr(), c0.bias.data_ptr()
        p.g1, p.be1 = gn1.weight.data_ptr(), gn1.bias.data_ptr()
        p.w2, p.sigma2, p.b2 = c4.weight_orig.data_ptr(), sig["conv_layers.4"][0].data_ptr(), c4.bias.data_ptr()
        p.g2, p.be2 = gn2.weight.data_ptr(), gn2.bias.data_ptr()
        p.eps1, p.eps2, p.slope = float(gn1.eps), float(gn2.eps), SLOPE
        p.ph, p.pw = int(self.pool2[0]), int(self.pool2[1])
        return p

    def front2_bwd(self, ctx, dX: Act, weight_grads, input_grad, sn_jobs):
        """Backward of both fused conv blocks from the fc1 input gradient rows; returns the image
        gradient (fp32 Act) or None.  Weight gradients: W/sigma grads into the spectral-norm jobs,
        biases and GroupNorm affines accumulated."""
        x = ctx["x"]
        assert ctx["fsave"] is not None, "discriminator forward ran with grad_ctx=False"
        B, _, H, W = x.dims
        dev = x.t.device
        m = lambda n: get_module(self, n)
        dx = Act.nhwc(B, 1, H, W, torch.float32, dev) if input_grad else None
        part = g0 = g4 = None
        grads = [None] * 8
        if weight_grads:
            part = torch.empty(hip.lib().es_dfront2_part_floats(B), dtype=torch.float32, device=dev)
            g0 = torch.empty_like(m("conv_layers.0").weight_orig)
            g4 = torch.empty_like(m("conv_layers.4").weight_orig)
            grads = [g0, m("conv_layers.0").bias.grad, m("conv_layers.1").weight.grad, m("conv_layers.1").bias.grad,
                     g4, m("conv_layers.4").bias.grad, m("conv_layers.5").weight.grad, m("conv_layers.5").bias.grad]
        F = self.flat_dim + self.cond_dim
        hip.call("es_dfront2_bwd", x.ptr, hip.strides4(x.strides), B, H, W, C.byref(ctx["front2"]),
                 hip.ptr(ctx["fstats"]), hip.ptr(ctx["fsave"]), dX.ptr, F, dx.ptr if dx is not None else None,
                 hip.strides4(dx.strides) if dx is not None else None, hip.ptr(part),
                 *[hip.ptr(t) for t in grads], hip.stream_ptr())
        if weight_grads:
            sig = ctx["sig"]
            o = self.ops()
            sn_jobs.append((o["sn:conv_layers.4"], g4, sig["conv_layers.4"], m("conv_layers.4").weight_orig.grad))
            sn_jobs.append((o["sn:conv_layers.0"], g0, sig["conv_layers.0"], m("conv_layers.0").weight_orig.grad))
        return dx

    def _front_params(self, sigma):
        c0, gn = get_module(self, "conv_layers.0"), get_module(self, "conv_layers.1")
        return (hip.ptr(c0.weight_orig), hip.ptr(sigma), hip.ptr(c0.bias), hip.ptr(gn.weight), hip.ptr(gn.bias),
                float(gn.eps), SLOPE)

    def front_fwd(self, x: Act, sigma):
        """-> pooled Act [B,32,Hp,Wp] fp32 NHWC, pool argmax bytes, GN (mean, invstd) [B*8]."""
        B, _, H, W = x.dims
        dev = x.t.device
        p1 = Act.nhwc(B, 32, (H - 2) // 2, (W - 2) // 2, torch.float32, dev)
        i1 = torch.empty(p1.numel, dtype=torch.uint8, device=dev)
        mean = torch.empty(B * 8, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        hip.call("es_dfront_fwd", x.ptr, hip.strides4(x.strides), B, H, W, *self._front_params(sigma),
                 hip.ptr(mean), hip.ptr(invstd), p1.ptr, hip.ptr(i1), hip.stream_ptr())
        return p1, i1, (mean, invstd)

    def front_bwd(self, ctx, dp1: Act, weight_grads, input_grad):
        """Backward of the fused front from d(pooled); returns the image gradient (fp32) or None."""
        x = ctx["x"]
        B, _, H, W = x.dims
        dev = x.t.device
        assert dp1.strides == ctx["p1"].strides, (dp1.strides, ctx["p1"].strides)
        c0, gn = get_module(self, "conv_layers.0"), get_module(self, "conv_layers.1")
        sig = ctx["sig"]["conv_layers.0"]
        mean, invstd = ctx["s1"]
        dx = Act.nhwc(B, 1, H, W, torch.float32, dev) if input_grad else None
        g_sn = torch.empty_like(c0.weight_orig) if weight_grads else None
        part = torch.empty(hip.lib().es_dfront_part_floats(B), dtype=torch.float32, device=dev)
        grad = (lambda t: hip.ptr(t.grad)) if weight_grads else (lambda t: None)
        hip.call("es_dfront_bwd", x.ptr, hip.strides4(x.strides), B, H, W, *self._front_params(sig[0]),
                 hip.ptr(mean), hip.ptr(invstd), hip.ptr(ctx["i1"]), dp1.ptr,
                 dx.ptr if dx is not None else None, hip.strides4(dx.strides) if dx is not None else None,
                 hip.ptr(part), hip.ptr(g_sn), grad(c0.bias), grad(gn.weight), grad(gn.bias), hip.stream_ptr())
        if weight_grads:
            self.ops()["sn:conv_layers.0"].bwd(g_sn, sig, c0.weight_orig.grad, beta=1.0)
        return dx

    # --------------------------------------------------------------------------- forward
    def fwd(self, img: Act, cond: torch.Tensor, train=True, grad_ctx=True):
        """img Act [B,1,H,W] (any dtype), cond [B,9] fp32 -> (out [B,1] fp32, latent [B,64] fp32, ctx).
        grad_ctx=False: no backward will follow (the fused front then saves no activations)."""
        o = self.ops()
        cdt = self.compute_dtype
        dev = cond.device
        B = img.dims[0]
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        x = img
        front = self.front_fused(img)               # the fused front reads the fp32 image directly
        if front and hip.live_on() and not self.front2_fused(img):
            front = False                           # (es_dfront_* has no live-row count: generic kernels)
        if img.t.dtype != cdt and not front:
            x = img.like_nhwc(cdt)
            copy_act(img, x)
        sig = dict(zip(LAYERS, SpectralNorm.sigma_many([o["sn:" + n] for n in LAYERS], update=train)))
        inv = lambda n: sig[n][0]
        F = self.flat_dim + self.cond_dim
        if front and self.front2_fused(x):
            # both conv blocks in one kernel: features straight into the fc1 input rows
            params = self._front2_params(sig)
            params.rows = hip.rows_ptr(B)
            fstats = torch.empty(B * 32, dtype=torch.float32, device=dev)
            # activations the backward reads (pooled block-1 map, argmax conv values, block-2 map)
            nsave = hip.lib().es_dfront2_save_floats(x.dims[2], x.dims[3], *self.pool2)
            fsave = torch.empty(B * nsave, dtype=torch.float32, device=dev) if grad_ctx else None
            X = Act.rows(B, F, cdt, dev)
            Xm = X.t.view(B, F)
            hip.call("es_dfront2_fwd", x.ptr, hip.strides4(x.strides), B, x.dims[2], x.dims[3], C.byref(params),
                     hip.ptr(fstats), X.ptr, F, hip.ptr(fsave), hip.stream_ptr())
            copy_act(Act.of(cond), Act.of(Xm[:, self.flat_dim:]))
            return self._fc_fwd(X, B, cdt, dev, sig, dict(x=x, sig=sig, front=True, front2=params, fstats=fstats,
                                                          fsave=fsave, X=X))
        if front:
            p1, i1, s1 = self.front_fwd(x, inv("conv_layers.0"))
            if p1.t.dtype != cdt:                   # bf16 mode: the GEMM layers after the front
                p1c = p1.like_nhwc(cdt)
                copy_act(p1, p1c)
                p1 = p1c
            h1 = y1 = None
        else:
            h1 = o["conv_layers.0"].fwd(x, inv_scale=inv("conv_layers.0"))
            y1, s1 = o["gn1"].fwd(h1, lr)
            p1, i1 = o["pool1"].fwd(y1)
        h2 = o["conv_layers.4"].fwd(p1, inv_scale=inv("conv_layers.4"))
        y2, s2 = o["gn2"].fwd(h2, lr)
        fh, fw = self.feat_hw
        X = Act.rows(B, F, cdt, dev)
        Xm = X.t.view(B, F)
        feat = Act(Xm, (B, 16, fh, fw), (F, fh * fw, fw, 1))       # NCHW flatten order (view(B,-1))
        _, i2 = o["pool2"].fwd(y2, out=feat)
        copy_act(Act.of(cond), Act.of(Xm[:, self.flat_dim:]))
        return self._fc_fwd(X, B, cdt, dev, sig, dict(x=x, sig=sig, front=front, front2=None, h1=h1, y1=y1, s1=s1,
                                                      p1=p1, i1=i1, h2=h2, y2=y2, s2=s2, i2=i2, X=X,
                                                      feat_dims=(B, 16, fh, fw)))

    # the fc tail as one per-16-samples kernel pair (d_mlp.hip); off: the layer-by-layer kernels (tests)
    fuse_mlp = True

    def _mlp_params(self, sig):
        m = lambda n: get_module(self, n)
        p = hip.DMlpParams()
        f1, n1, f2, n2, f3 = m("fc1.0"), m("fc1.1"), m("fc2.0"), m("fc2.1"), m("fc3")
        p.w1, p.sigma1, p.b1 = f1.weight_orig.data_ptr(), sig["fc1.0"][0].data_ptr(), f1.bias.data_ptr()
        p.g1, p.be1 = n1.weight.data_ptr(), n1.bias.data_ptr()
        p.w2, p.sigma2, p.b2 = f2.weight_orig.data_ptr(), sig["fc2.0"][0].data_ptr(), f2.bias.data_ptr()
        p.g2, p.be2 = n2.weight.data_ptr(), n2.bias.data_ptr()
        p.w3, p.sigma3, p.b3 = f3.weight_orig.data_ptr(), sig["fc3"][0].data_ptr(), f3.bias.data_ptr()
        p.eps1, p.eps2, p.slope = float(n1.eps), float(n2.eps), SLOPE
        return p

    def _fc_fwd(self, X: Act, B, cdt, dev, sig, ctx):
        """fc1 -> LN -> LReLU -> fc2 -> LN -> LReLU (latent) -> fc3 on the fc1 input rows X."""
        o = self.ops()
        if self.fuse_mlp and cdt == torch.float32:
            F = X.dims[1]
            params = self._mlp_params(sig)
            params.rows = hip.rows_ptr(B)
            f32 = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)
            h3, s3, h4, s4, lat, out = f32(B, 128), f32(B, 2), f32(B, 64), f32(B, 2), f32(B, 64), f32(B, 1)
            hip.call("es_dmlp_fwd", X.ptr, X.strides[0], B, F, C.byref(params), hip.ptr(h3), hip.ptr(s3),
                     hip.ptr(h4), hip.ptr(s4), hip.ptr(lat), hip.ptr(out), hip.stream_ptr())
            ctx.update(mlp=(params, h3, s3, h4, s4, lat))
            return Act.of(out), Act.of(lat), ctx
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        inv = lambda n: sig[n][0]
        h3 = o["fc1.0"].fwd(X, inv_scale=inv("fc1.0"))
        y3, s3 = o["ln1"].fwd(h3, lr)
        h4 = o["fc2.0"].fwd(y3, inv_scale=inv("fc2.0"))
        lat, s4 = o["ln2"].fwd(h4, lr, out_dtype=torch.float32)
        lat_c = lat
        if cdt != torch.float32:
            lat_c = lat.like_nhwc(cdt)
            copy_act(lat, lat_c)
        out = o["fc3"].fwd(lat_c, inv_scale=inv("fc3"), out_dtype=torch.float32)
        ctx.update(h3=h3, y3=y3, s3=s3, h4=h4, s4=s4, lat=lat_c)
        return out, lat, ctx

    # --------------------------------------------------------------------------- backward
    def bwd(self, ctx, dout: Act = None, dlat: Act = None, weight_grads=True, input_grad=True):
        """dout [B,1] fp32 (or None), dlat [B,64] fp32 (or None).  Returns d image (fp32 Act) or None.
        The spectral-norm weight_orig gradients of the layers are issued together at the end
        (SpectralNorm.bwd_many: the small layers share one launch)."""
        sn_jobs = []
        dimg = self._bwd(ctx, dout, dlat, weight_grads, input_grad, sn_jobs)
        # only on the normal return path: a failed _bwd leaves no half-issued gradient launch
        if sn_jobs:
            SpectralNorm.bwd_many(sn_jobs, beta=1.0)
        return dimg

    def _mlp_bwd(self, ctx, dout, dlat, weight_grads, sn_jobs):
        """Backward of the fused fc tail -> the fc1 input gradient rows dX (fp32 Act [B][F])."""
        params, h3, s3, h4, s4, lat = ctx["mlp"]
        X = ctx["X"]
        B, F = X.dims[0], X.dims[1]
        dev = X.t.device
        m = lambda n: get_module(self, n)
        dX = Act.rows(B, F, torch.float32, dev)
        part = None
        outs = [None] * 10
        if weight_grads:
            part = torch.empty(hip.lib().es_dmlp_part_floats(B, F), dtype=torch.float32, device=dev)
            g1 = torch.empty_like(m("fc1.0").weight_orig)
            g2 = torch.empty_like(m("fc2.0").weight_orig)
            g3 = torch.empty_like(m("fc3").weight_orig)
            outs = [g1, m("fc1.0").bias.grad, m("fc1.1").weight.grad, m("fc1.1").bias.grad,
                    g2, m("fc2.0").bias.grad, m("fc2.1").weight.grad, m("fc2.1").bias.grad,
                    g3, m("fc3").bias.grad]
        hip.call("es_dmlp_bwd", X.ptr, X.strides[0], B, F, C.byref(params), hip.ptr(h3), hip.ptr(s3), hip.ptr(h4),
                 hip.ptr(s4), hip.ptr(lat), dout.ptr if dout is not None else None,
                 dlat.ptr if dlat is not None else None, dX.ptr, F, hip.ptr(part),
                 *[hip.ptr(t) for t in outs], hip.stream_ptr())
        if weight_grads:
            o = self.ops()
            sig = ctx["sig"]
            for name, g in (("fc3", outs[8]), ("fc2.0", outs[4]), ("fc1.0", outs[0])):
                sn_jobs.append((o["sn:" + name], g, sig[name], m(name).weight_orig.grad))
        return dX

    def _bwd(self, ctx, dout, dlat, weight_grads, input_grad, sn_jobs):
        o = self.ops()
        if ctx.get("mlp") is not None:
            assert dout is None or (dout.t.dtype == torch.float32 and dout.strides[0] == 1), "dout: [B,1] fp32"
            assert dlat is None or (dlat.t.dtype == torch.float32 and dlat.strides[0] == 64), "dlat: [B,64] fp32"
            dX = self._mlp_bwd(ctx, dout, dlat, weight_grads, sn_jobs)
            if ctx["front2"] is not None:
                return self.front2_bwd(ctx, dX, weight_grads, input_grad, sn_jobs)
            return self._front_bwd_from_dX(ctx, dX, weight_grads, input_grad, sn_jobs)
        cdt = self.compute_dtype
        dev = ctx["X"].t.device
        B = ctx["X"].dims[0]
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        m = lambda n: get_module(self, n)
        sig = ctx["sig"]

        def wgrad(name, dy, x, bias_done=True):
            if not weight_grads:
                return
            mod = m(name)
            op = o[name]
            g_sn = torch.empty_like(mod.weight_orig)
            op.wgrad(dy, x, g_sn, None, beta=0.0)          # grad of W/sigma
            if not bias_done:                               # bias is not normalised
                channel_sum(dy, mod.bias.grad, beta=1.0)
            sn_jobs.append((o["sn:" + name], g_sn, sig[name], mod.weight_orig.grad))

        bias_g = (lambda n: m(n).bias.grad) if weight_grads else (lambda n: None)

        # latent gradient: dlat (SDI) + fc3^T dout
        dl = Act.rows(B, 64, cdt, dev, zero=True)
        if dlat is not None:
            copy_act(dlat, dl)
        if dout is not None:
            dout_c = dout
            if cdt != torch.float32:
                dout_c = dout.like_nhwc(cdt)
                copy_act(dout, dout_c)
            wgrad("fc3", dout_c, ctx["lat"], bias_done=False)
            o["fc3"].dgrad(dout_c, ctx["lat"], inv_scale=sig["fc3"][0], dx=dl, beta=1.0)
        dh4 = o["ln2"].bwd(ctx["h4"], ctx["s4"], lr, dl,
                           dgamma=m("fc2.1").weight.grad if weight_grads else None,
                           dbeta=m("fc2.1").bias.grad if weight_grads else None, dsum=bias_g("fc2.0"))
        wgrad("fc2.0", dh4, ctx["y3"])
        dy3 = o["fc2.0"].dgrad(dh4, ctx["y3"], inv_scale=sig["fc2.0"][0])
        dh3 = o["ln1"].bwd(ctx["h3"], ctx["s3"], lr, dy3,
                           dgamma=m("fc1.1").weight.grad if weight_grads else None,
                           dbeta=m("fc1.1").bias.grad if weight_grads else None, dsum=bias_g("fc1.0"))
        wgrad("fc1.0", dh3, ctx["X"])
        dX = o["fc1.0"].dgrad(dh3, ctx["X"], inv_scale=sig["fc1.0"][0])
        if ctx["front2"] is not None:
            return self.front2_bwd(ctx, dX, weight_grads, input_grad, sn_jobs)
        return self._front_bwd_from_dX(ctx, dX, weight_grads, input_grad, sn_jobs)

    def _front_bwd_from_dX(self, ctx, dX, weight_grads, input_grad, sn_jobs):
        """Backward of the conv blocks (unfused / block-1-fused forms) from the fc1 input gradient."""
        o = self.ops()
        cdt = self.compute_dtype
        B = ctx["X"].dims[0]
        lr = hip.chain_struct(hip.ACT_LRELU, SLOPE)
        m = lambda n: get_module(self, n)
        sig = ctx["sig"]

        def wgrad(name, dy, x):
            if not weight_grads:
                return
            mod = m(name)
            g_sn = torch.empty_like(mod.weight_orig)
            o[name].wgrad(dy, x, g_sn, None, beta=0.0)          # grad of W/sigma
            sn_jobs.append((o["sn:" + name], g_sn, sig[name], mod.weight_orig.grad))

        bias_g = (lambda n: m(n).bias.grad) if weight_grads else (lambda n: None)
        F = self.flat_dim + self.cond_dim
        B_, Cf, fh, fw = ctx["feat_dims"]
        dfeat = Act(dX.t.view(B, F), (B, 16, fh, fw), (F, fh * fw, fw, 1))
        dy2 = o["pool2"].bwd(dfeat, ctx["i2"], ctx["y2"].dims, cdt)
        dh2 = o["gn2"].bwd(ctx["h2"], ctx["s2"], lr, dy2,
                           dgamma=m("conv_layers.5").weight.grad if weight_grads else None,
                           dbeta=m("conv_layers.5").bias.grad if weight_grads else None,
                           dsum=bias_g("conv_layers.4"))
        wgrad("conv_layers.4", dh2, ctx["p1"])
        dp1 = o["conv_layers.4"].dgrad(dh2, ctx["p1"], inv_scale=sig["conv_layers.4"][0],
                                       dx_dtype=torch.float32 if ctx["front"] else None)
        if ctx["front"]:
            return self.front_bwd(ctx, dp1, weight_grads, input_grad)
        dy1 =o["pool1"].bwd(dp1, ctx["i1"], ctx["y1"].dims, cdt)
        dh1 = o["gn1"].bwd(ctx["h1"], ctx["s1"], lr, dy1,
                           dgamma=m("conv_layers.1").weight.grad if weight_grads else None,
                           dbeta=m("conv_layers.1").bias.grad if weight_grads else None,
                           dsum=bias_g("conv_layers.0"))
        wgrad("conv_layers.0", dh1, ctx["x"])
        if not input_grad:
            return None
        return o["conv_layers.0"].dgrad(dh1, ctx["x"], inv_scale=sig["conv_layers.0"][0],
                                        dx_dtype=torch.float32)

    def forward(self, img, cond):
        from .autograd import discriminator_apply
        return discriminator_apply(self, img, cond)
