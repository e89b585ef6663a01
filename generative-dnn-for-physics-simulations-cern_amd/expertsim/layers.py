"""Layer-level building blocks over the HIP kernels (explicit forward / backward, no autograd).

Each block keeps the reference's parameter tensors (fp32 masters, torch layouts, so state_dicts
match the reference's) and drives the C-ABI kernels of ``expertsim.hip``.  Activations are
``Act`` objects: a flat device buffer plus a logical (n, c, h, w) shape and element strides, so
conv activations live channels-last (NHWC) while linear activations are plain [rows][features].
"""
from __future__ import annotations

import ctypes as C
import os
import math

import numpy as np
import torch

from . import hip


class Act:
    """Logical (N, C, H, W) tensor over a flat device buffer with explicit element strides."""

    __slots__ = ("t", "dims", "strides", "bn_part", "bn_sums", "px", "sample")

    def __init__(self, t: torch.Tensor, dims, strides, sample: bool = True):
        self.px = 0               # > 0: each image's P*Q pixels are px consecutive samples (pixel view)
        # sample-major: dims[0] counts samples, so inside a dynamic-rows expert program a view of
        # capacity rows carries the live count (hip.make_view); False for any other leading dimension
        self.sample = bool(sample)
        self.bn_part = None       # (partials, chunks) of fused BatchNorm statistics (ConvOp.fwd)
        self.bn_sums = None       # (partials, chunks, norm) of a fused BatchNorm-backward reduction (ConvOp.dgrad)
        self.t = t
        self.dims = tuple(int(d) for d in dims)
        self.strides = tuple(int(s) for s in strides)

    # ---- constructors
    @staticmethod
    def nhwc(N, Cc, H, W, dtype, device, zero=False):
        f = torch.zeros if zero else torch.empty
        t = f(N * H * W * Cc, dtype=dtype, device=device)
        return Act(t, (N, Cc, H, W), (H * W * Cc, 1, W * Cc, Cc))

    @staticmethod
    def rows(N, F, dtype, device, zero=False):
        f = torch.zeros if zero else torch.empty
        return Act(f(N * F, dtype=dtype, device=device), (N, F, 1, 1), (F, 1, 1, 1))

    @staticmethod
    def of(t: torch.Tensor):
        """Wrap a torch tensor of rank 2 ([N,F]) or 4 ([N,C,H,W], any strides)."""
        if t.dim() == 2:
            return Act(t, (t.shape[0], t.shape[1], 1, 1), (t.stride(0), t.stride(1), 1, 1))
        assert t.dim() == 4, t.shape
        return Act(t, tuple(t.shape), tuple(t.stride()))

    def like_nhwc(self, dtype=None, zero=False):
        N, Cc, H, W = self.dims
        return Act.nhwc(N, Cc, H, W, dtype or self.t.dtype, self.t.device, zero)

    # ---- properties
    @property
    def view(self):
        return hip.make_view(self.dims, self.strides, self.sample)

    @property
    def dt(self):
        return hip.dt_of(self.t)

    @property
    def ptr(self):
        return C.c_void_p(self.t.data_ptr())

    @property
    def numel(self):
        n, c, h, w = self.dims
        return n * c * h * w

    def torch_nchw(self):
        """Strided torch view [N, C, H, W] of the same memory (no copy)."""
        base = self.t
        off = 0
        if base.dim() != 1:
            off = base.storage_offset()
            base = base.reshape(-1) if base.is_contiguous() else base
        return torch.as_strided(self.t, self.dims, self.strides, self.t.storage_offset())

    def head(self, n):
        """The first n samples (same memory)."""
        return Act(self.t, (int(n), *self.dims[1:]), self.strides, self.sample)

    def rows2d(self):
        n, c, h, w = self.dims
        assert h == 1 and w == 1
        return torch.as_strided(self.t, (n, c), (self.strides[0], self.strides[1]), self.t.storage_offset())


# ------------------------------------------------------------------------------ kernel probe
class KernelProbe:
    """HIP-event timing of selected kernel launches (labels like "G0.c5.fwd") on the launch
    stream, used by bench.py for the live roofline of the dominant kernel."""

    def __init__(self, targets):
        self.targets = set(targets)
        self.events = {t: [] for t in targets}
        self.launches = {t: [] for t in targets}   # MFMA conv kernels issued per probed op
        self.exec = {t: [] for t in targets}       # executed FLOPs per op [bf16 pipe, fp32 MFMA, VALU]

    def wants(self, label):
        return label in self.targets

    def record(self, label):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def add(self, label, start, end, launches=None, exec_flops=None):
        self.events[label].append((start, end))
        if launches is not None:
            self.launches[label].append(launches)
        if exec_flops is not None:
            self.exec[label].append(exec_flops)

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for k, pairs in self.events.items():
            if pairs:
                ms = [a.elapsed_time(b) for a, b in pairs]
                out[k] = {"count": len(ms), "total_ms": sum(ms), "avg_ms": sum(ms) / len(ms)}
                if self.launches[k]:
                    out[k]["kernel_launches_per_op"] = max(self.launches[k])
                if self.exec[k]:
                    out[k]["exec_flops_per_op"] = [max(e[i] for e in self.exec[k]) for i in range(3)]
        return out


_PROBE = None


def set_probe(p):
    global _PROBE
    _PROBE = p


class _probed:
    def __init__(self, label):
        self.label = label
        self.on = _PROBE is not None and label is not None and _PROBE.wants(label)

    def __enter__(self):
        if self.on:
            self.n0 = hip.lib().es_conv_launch_count()
            self.f0 = _exec_tally()
            self.t0 = _PROBE.record(self.label)

    def __exit__(self, *exc):
        if self.on:
            t1 = _PROBE.record(self.label)
            f1 = _exec_tally()
            _PROBE.add(self.label, self.t0, t1, hip.lib().es_conv_launch_count() - self.n0,
                       [b - a for a, b in zip(self.f0, f1)])


def _exec_tally():
    """The host tally of executed conv MFMA work so far (es_conv_exec_flops): [bf16 pipe, fp32 MFMA, VALU]."""
    out = (C.c_double * 3)()
    hip.call("es_conv_exec_flops", out, 0)
    return list(out)


def repack_ops(ops):
    """After a weight update: rebuild every cached weight packing of these ConvOps in place with one
    batched launch per 32 packings (es_pack_conv_weights) instead of one or two launches per layout
    at the next use; ops without a packing yet pack lazily as before.  Ops sharing a packing dict
    (a resized conv and its plain op) are packed once."""
    jobs, seen = [], set()
    for op in ops:
        pk = getattr(op, "_packed", None)
        if not pk or id(pk) in seen or not hasattr(op, "repack_jobs"):
            continue
        seen.add(id(pk))
        jobs += op.repack_jobs()
    if jobs:
        arr = (hip.PackJob * len(jobs))(*jobs)
        hip.call("es_pack_conv_weights", arr, len(jobs), hip.stream_ptr())


def copy_act(src: Act, dst: Act, alpha=1.0, beta=0.0):
    hip.call("es_copy", C.byref(src.view), src.dt, src.ptr, C.byref(dst.view), dst.dt, dst.ptr,
             float(alpha), float(beta), hip.stream_ptr())
    return dst


def ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# Deterministic reductions (the fp32 parity mode): weight gradients through es_conv2d_wgrad_det (split
# partials + one ordered reduce, no float atomics), no split-K atomics in the fp32 GEMMs, ordered
# conv-bias sums.  Two runs of the same step are then bitwise identical, as the reference's are.
_DET = False


def set_deterministic(on: bool):
    global _DET
    on = bool(on)
    if on != _DET:
        hip.lib().es_set_deterministic(1 if on else 0)
        _DET = on


def deterministic() -> bool:
    return _DET


# fp32 MFMA arithmetic of the ring convolutions: exact fp32 (v_mfma_f32_16x16x4_f32) or split-fp32
# (three bf16 planes per operand, six plane products on v_mfma_f32_16x16x32_bf16; es_conv_set_f32_split).
# Level 2 (the level used when on): the packed weights carry their planes (es_pack_weight_planes), so the
# FWD / DGRAD kernels split only the activations (level 1, both split in the kernel, stays a test hook).
# The level the C side uses is the single source of truth (es_conv_set_f32_split clamps to {0, 1, 2}),
# so the Python mirror is read back from C (packing the weight planes must follow the level the kernels run).
_F32_SPLIT = None
_SPLIT_LEVEL = 2
_LIN_PIX = True      # ConvOp._pixel_view (tests compare it against the plain linear path)


def set_f32_split(on: bool):
    global _F32_SPLIT
    lvl = _SPLIT_LEVEL if on else 0
    if lvl != f32_split_level():
        hip.lib().es_conv_set_f32_split(lvl)
        _F32_SPLIT = None
        f32_split_level()


def f32_split() -> bool:
    return f32_split_level() > 0


def f32_split_level() -> int:
    global _F32_SPLIT
    if _F32_SPLIT is None:   # read the C level back (set returns the previous value)
        lib = hip.lib()
        cur = int(lib.es_conv_set_f32_split(0))
        lib.es_conv_set_f32_split(cur)
        _F32_SPLIT = cur
    return _F32_SPLIT


# --------------------------------------------------------------------------------- upsample
class Upsample:
    """torch nearest upsample (``scale_factor`` or ``size``) as index maps for the conv gather.

    Source index = min(floor(dst * scale), in - 1) with scale = float32(1/scale_factor) when a
    scale factor is given, float32(in)/out otherwise (ATen upsample_nearest2d)."""

    def __init__(self, in_hw, out_hw=None, scale=None):
        self.in_hw = tuple(in_hw)
        # exact integer factors (x2 of the generators) are handled arithmetically in the kernels
        self.factor = None
        if scale is not None and all(float(f).is_integer() for f in scale):
            self.factor = (int(scale[0]), int(scale[1]))
        if out_hw is None:
            out_hw = (int(math.floor(in_hw[0] * scale[0])), int(math.floor(in_hw[1] * scale[1])))
        self.out_hw = tuple(out_hw)
        self.maps = []
        self.inv = []
        for ax in range(2):
            n_in, n_out = self.in_hw[ax], self.out_hw[ax]
            if scale is not None:
                sc = np.float32(1.0 / scale[ax])
            else:
                sc = np.float32(n_in) / np.float32(n_out)
            dst = np.arange(n_out, dtype=np.float32)
            src = np.minimum(np.floor(dst * sc).astype(np.int64), n_in - 1).astype(np.int32)
            self.maps.append(src)
            start = np.zeros(n_in, np.int32)
            count = np.zeros(n_in, np.int32)
            for i in range(n_in):
                where = np.nonzero(src == i)[0]
                assert where.size == 0 or (where[-1] - where[0] + 1 == where.size)
                start[i] = where[0] if where.size else 0
                count[i] = where.size
            self.inv.append((start, count))
        self._dev = {}

    def device_maps(self, device):
        key = str(device)
        if key not in self._dev:
            t = lambda a: torch.from_numpy(a).to(device)
            self._dev[key] = (t(self.maps[0]), t(self.maps[1]), t(self.inv[0][0]), t(self.inv[0][1]),
                              t(self.inv[1][0]), t(self.inv[1][1]))
        return self._dev[key]


# ------------------------------------------------------------------------------ conv / linear
class ConvOp:
    """nn.Conv2d / nn.Linear on the implicit-GEMM kernels.

    ``weight``: fp32 master [K, C, R, S] (or [K, C] for a linear); ``bias`` fp32 [K] or None.
    The packed GEMM copies (fwd [K][R][S][C], dgrad [C][R][S][K]) in the compute dtype are
    rebuilt when ``invalidate()`` is called (after every optimizer step) or per call when a
    spectral-norm sigma is given."""

    def __init__(self, weight: torch.nn.Parameter, bias, stride=1, pad=0, upsample: Upsample = None):
        self.weight = weight
        self.bias = bias
        self.stride = stride
        self.pad = pad
        self.up = upsample
        self.label = None
        # a non-integer nearest resize (the proton generator's 35x19 -> 56x30 before conv_layers.5):
        # the resized input is materialised (es_upsample_fwd) and the conv runs as a plain conv on it,
        # on the ring kernels (the gather-map conv only runs on the generic register-staged kernels)
        self._plain = None
        if upsample is not None and upsample.factor is None:
            self._plain = ConvOp(weight, bias, stride=stride, pad=pad, upsample=None)
        w = weight
        self.K = w.shape[0]
        self.C = w.shape[1]
        self.R = w.shape[2] if w.dim() == 4 else 1
        self.S = w.shape[3] if w.dim() == 4 else 1
        self._packed = {}
        if self._plain is not None:
            self._plain._packed = self._packed   # same weights, same packings (modes 0 / 1)

    def invalidate(self):
        self._packed.clear()

    def repack_jobs(self):
        """The es_pack_conv_weights jobs that rebuild this op's cached packings in place (the
        weights changed, the layouts and buffers did not)."""
        jobs = []
        for (dtype, mode, planes), out in self._packed.items():
            j = hip.PackJob()
            j.w, j.K, j.C, j.R, j.S, j.mode = self.weight.data_ptr(), self.K, self.C, self.R, self.S, mode
            j.dt, j.planes, j.out = hip.dt_of(out), int(planes), out.data_ptr()
            jobs.append(j)
        return jobs

    def _resized(self, x: Act) -> bool:
        """Materialise the resize for this call: dense NHWC input with 16-byte channel chunks."""
        if self._plain is None:
            return False
        N, Cc, H, W = x.dims
        vec = 4 if x.t.dtype == torch.float32 else 8
        return Cc % vec == 0 and tuple(x.strides) == (H * W * Cc, 1, W * Cc, Cc)

    def _resize(self, x: Act) -> Act:
        N, Cc, H, W = x.dims
        Hu, Wu = self.up.out_hw
        xu = Act.nhwc(N, Cc, Hu, Wu, x.t.dtype, x.t.device)
        maps = self.up.device_maps(x.t.device)
        hip.call("es_upsample_fwd", C.byref(x.view), x.dt, x.ptr, hip.ptr(maps[0]), hip.ptr(maps[1]),
                 C.byref(xu.view), xu.ptr, hip.stream_ptr())
        return xu

    def _plain_op(self):
        self._plain.label = self.label
        return self._plain

    def packed(self, dtype, mode, inv_scale=None):
        """Packed GEMM weights; fp32 with split level 2 also carries the bf16 planes behind the fp32
        packing (es_pack_weight_planes) that the split-fp32 ring kernels read."""
        planes = dtype == torch.float32 and f32_split_level() == 2
        key = (dtype, mode, planes)
        if inv_scale is None and key in self._packed:
            return self._packed[key]
        w = self.weight
        n = w.numel() if mode < 2 else self.K * self.C * hip.lib().es_subpixel_taps(self.R, self.S)
        total = n
        if planes:
            total = (int(hip.lib().es_weight_planes_offset(n)) + 6 * n + 3) // 4
        out = torch.empty(total, dtype=dtype, device=w.device)
        hip.call("es_pack_conv_weight", hip.ptr(w), self.K, self.C, self.R, self.S, mode,
                 hip.ptr(inv_scale), None, hip.ptr(out), hip.dt_of(out), hip.stream_ptr())
        if planes:
            hip.call("es_pack_weight_planes", hip.ptr(out), n, hip.ptr(out), hip.stream_ptr())
        if inv_scale is None:
            self._packed[key] = out
        return out

    def desc(self, x: Act):
        N, Cc, H, W = x.dims
        assert Cc == self.C, (Cc, self.C)
        d = hip.ConvDesc()
        d.N, d.C, d.H, d.W = N, Cc, H, W
        if self.up is not None:
            assert (H, W) == self.up.in_hw, ((H, W), self.up.in_hw)
            d.Hu, d.Wu = self.up.out_hw
            maps = self.up.device_maps(x.t.device)
            if self.up.factor is not None:
                d.hmap = d.wmap = None
                d.up_h, d.up_w = self.up.factor
            else:
                d.hmap, d.wmap = maps[0].data_ptr(), maps[1].data_ptr()
                d.up_h = d.up_w = 0
        else:
            d.Hu, d.Wu = H, W
            d.hmap = d.wmap = None
            d.up_h = d.up_w = 0
        d.K, d.R, d.S, d.stride, d.pad = self.K, self.R, self.S, self.stride, self.pad
        d.P = (d.Hu + 2 * self.pad - self.R) // self.stride + 1
        d.Q = (d.Wu + 2 * self.pad - self.S) // self.stride + 1
        d.rows = hip.rows_ptr(N)
        if x.px:   # a pixel view (ConvOp._pixel_view): the live count is in samples = pixels
            d.rows, d.rows_px = hip.rows_ptr(N * x.px), x.px
        return d

    def subpixel(self, d, dtype) -> bool:
        """Run this x2-upsample conv as 4 parity-class convs on the source grid (ring kernels,
        conv_mfma.hip; bf16, and fp32 with combined weights summed in fp32, whose rounding is ~1e-7
        relative): es_conv_subpixel_ok decides, the weights are packed in modes 2 / 3."""
        if self.up is None or self.up.factor != (2, 2) or dtype not in (torch.bfloat16, torch.float32):
            return False
        return bool(hip.lib().es_conv_subpixel_ok(C.byref(d), hip.dt_of_dtype(dtype)))

    def fwd(self, x: Act, out_dtype=None, inv_scale=None, out: Act = None, with_bias=True,
            bn_stats=False) -> Act:
        """bn_stats: also ask for the BatchNorm partials of the output (es_conv2d_fwd_stats); when
        the kernel provides them, out.bn_part = (part, chunks) and NormOp.stats merges those instead
        of re-reading the output."""
        if self._resized(x):
            return self._plain_op().fwd(self._resize(x), out_dtype, inv_scale, out, with_bias, bn_stats)
        xv = self._pixel_view(x) if out is None else None
        if xv is not None:
            o = self.fwd(xv, out_dtype, inv_scale, None, with_bias, bn_stats)
            res = Act(o.t, (x.dims[0], self.K, 1, 1), (self.K, 1, 1, 1))
            res.bn_part = o.bn_part
            return res
        d = self.desc(x)
        cdt = x.t.dtype
        if self.subpixel(d, cdt):
            d.subpixel = 1
            wk = self.packed(cdt, 2, inv_scale)
        else:
            wk = self.packed(cdt, 0, inv_scale)
        if out is None:
            out = Act.nhwc(d.N, d.K, d.P, d.Q, out_dtype or cdt, x.t.device)
        bias = self.bias if (with_bias and self.bias is not None) else None
        with _probed(self.label and self.label + ".fwd"):
            if bn_stats:
                # >= the ring's row tiles for every image-group size it may pick (8..64)
                tiles = ((d.N + 7) // 8) * (d.P * d.Q // 16 + 8) + ((d.N + 63) // 64) * (d.P * d.Q // 2 + 8)
                floats = tiles * 3 * d.K
                part = torch.empty(floats, dtype=torch.float32, device=x.t.device)
                chunks = C.c_int(0)
                hip.call("es_conv2d_fwd_stats", C.byref(d), x.dt, x.ptr, hip.strides4(x.strides), hip.ptr(wk),
                         hip.ptr(bias), out.ptr, out.dt, hip.strides4(out.strides), hip.ptr(part), floats,
                         C.byref(chunks), hip.stream_ptr())
                if chunks.value > 0:
                    out.bn_part = (part, chunks.value)
            elif _DET and self._linear_det(d, d.K, out):
                # deterministic split-K of a long-K linear (ordered partial sums, no atomics)
                nb = int(hip.lib().es_conv2d_splitk_ws_bytes(C.byref(d), 0))
                wsb = ws(nb, x.t.device)
                hip.call("es_conv2d_fwd_det", C.byref(d), x.dt, x.ptr, hip.strides4(x.strides), hip.ptr(wk),
                         hip.ptr(bias), out.ptr, out.dt, hip.strides4(out.strides), hip.ptr(wsb), nb,
                         hip.stream_ptr())
            else:
                hip.call("es_conv2d_fwd", C.byref(d), x.dt, x.ptr, hip.strides4(x.strides), hip.ptr(wk),
                         hip.ptr(bias), out.ptr, out.dt, hip.strides4(out.strides), hip.stream_ptr())
        return out

    def _pixel_view(self, x: Act):
        """A wide linear ([B, C] -> [B, K], K >= 1024) as a 1x1 conv over 16-pixel images of the same
        memory, NHWC (B/16, C, 16, 1): the ring FWD kernels (conv_mfma.hip) tile rows as (image group,
        pixel), so a linear's 1-pixel images would leave 3/4 of every 256-row tile empty (bf16) or miss
        the fp32 ring (>= 16 output pixels per image) and fall to the register-staged fp32-MFMA GEMM;
        the generators' fc2 (256 -> 21632 neutron, neutron/generator.py:17) is the case.  None when the
        layout does not apply."""
        if not _LIN_PIX or self.R != 1 or self.S != 1 or self.up is not None or self.stride != 1 or self.pad != 0:
            return None
        N, Cc, H, W = x.dims
        dt = x.t.dtype
        if H != 1 or W != 1 or N % 16 or N < 256 or self.K < 1024 or self.K % 64 or x.strides[:2] != (Cc, 1):
            return None
        if not ((dt == torch.float32 and f32_split_level() > 0 and Cc % 32 == 0) or (dt == torch.bfloat16 and Cc % 64 == 0)):
            return None
        v = Act(x.t, (N // 16, Cc, 16, 1), (16 * Cc, 1, Cc, Cc))
        v.px = 16       # (dynamic rows count samples: the view's pixels)
        return v

    def _linear_det(self, d, ng, out: Act) -> bool:
        """A linear (1x1 conv of 1x1 images) with a dense fp32 output of <= 4096 columns: the GEMMs
        whose split-K the deterministic mode runs through es_conv2d_*_det."""
        return (self.R == 1 and self.S == 1 and d.P == 1 and d.Q == 1 and d.Hu == 1 and d.Wu == 1
                and out.t.dtype == torch.float32 and ng <= 4096)

    def dgrad(self, dy: Act, x: Act, dx_dtype=None, inv_scale=None, dx: Act = None, beta=0.0,
              bn_reduce=None) -> Act:
        """Gradient w.r.t. the conv input x (folded through the upsample when present).

        bn_reduce = (norm, h, stats, chain): x = chain(norm(h)) is a BatchNorm + dropout + activation
        output; when the persistent dgrad kernel runs this conv, its epilogue also computes the
        reduction pass of that norm's backward (es_conv2d_dgrad_bnred) and dx.bn_sums = (part,
        chunks), which NormOp.bwd then finishes with the apply pass alone."""
        d = self.desc(x)
        cdt = dy.t.dtype
        if self.subpixel(d, cdt):
            d.subpixel = 1
            wd = self.packed(cdt, 3, inv_scale)
        else:
            wd = self.packed(cdt, 1, inv_scale)
        N, Cc, H, W = x.dims
        ddt = dx_dtype or cdt
        if self.up is None or self.up.factor is not None:   # no upsample, or folded in the GEMM
            if dx is None:
                dx = Act.nhwc(N, Cc, H, W, ddt, dy.t.device)
            fuse = (bn_reduce is not None and float(beta) == 0.0 and _NORM_SYNC is None
                    and bn_reduce[0].kind == hip.NORM_BN and bn_reduce[1].t.dtype == ddt == cdt
                    and bn_reduce[1].dims == dx.dims and tuple(bn_reduce[1].strides) == tuple(dx.strides))
            with _probed(self.label and self.label + ".dgrad"):
              if fuse:
                  norm, h, stats, chain = bn_reduce
                  nm = norm.norm_struct(*stats)
                  # >= the thin dgrad's blocks (<= 2048) / persistent workgroups / fp32 ring row tiles (one
                  # partial per 128- or 256-row tile of 64 images x >= 2 pixels, per image chunk)
                  floats = 3 * Cc * max(2048, ((N + 63) // 64 + 2) * ((H * W + 1) // 2 + 1))
                  part = torch.empty(floats, dtype=torch.float32, device=dy.t.device)
                  chunks = C.c_int(0)
                  hip.call("es_conv2d_dgrad_bnred", C.byref(d), dy.dt, dy.ptr, hip.strides4(dy.strides),
                           hip.ptr(wd), dx.ptr, dx.dt, hip.strides4(dx.strides), h.ptr, C.byref(nm),
                           C.byref(chain), hip.ptr(part), floats, C.byref(chunks), hip.stream_ptr())
                  if chunks.value > 0:
                      dx.bn_sums = (part, chunks.value, nm)
              elif _DET and float(beta) == 0.0 and self._linear_det(d, d.C, dx):
                  nb = int(hip.lib().es_conv2d_splitk_ws_bytes(C.byref(d), 1))
                  wsb = ws(nb, dy.t.device)
                  hip.call("es_conv2d_dgrad_det", C.byref(d), dy.dt, dy.ptr, hip.strides4(dy.strides), hip.ptr(wd),
                           dx.ptr, dx.dt, hip.strides4(dx.strides), hip.ptr(wsb), nb, hip.stream_ptr())
              else:
                  hip.call("es_conv2d_dgrad", C.byref(d), dy.dt, dy.ptr, hip.strides4(dy.strides), hip.ptr(wd),
                         dx.ptr, dx.dt, hip.strides4(dx.strides), float(beta), hip.stream_ptr())
            return dx
        dxu = Act.nhwc(N, Cc, d.Hu, d.Wu, torch.float32, dy.t.device)
        if self._resized(x):   # the plain conv's dgrad w.r.t. the materialised resized input
            # (x of the plain dgrad only gives the input geometry: dxu, exactly that shape and storage)
            self._plain_op().dgrad(dy, dxu, dx_dtype=torch.float32, inv_scale=inv_scale, dx=dxu)
        else:
          with _probed(self.label and self.label + ".dgrad"):
            hip.call("es_conv2d_dgrad", C.byref(d), dy.dt, dy.ptr, hip.strides4(dy.strides), hip.ptr(wd),
                     dxu.ptr, dxu.dt, hip.strides4(dxu.strides), 0.0, hip.stream_ptr())
        if dx is None:
            dx = Act.nhwc(N, Cc, H, W, ddt, dy.t.device)
        maps = self.up.device_maps(dy.t.device)
        hip.call("es_upsample_bwd", C.byref(dxu.view), dxu.dt, dxu.ptr, hip.ptr(maps[2]), hip.ptr(maps[3]),
                 hip.ptr(maps[4]), hip.ptr(maps[5]), C.byref(dx.view), dx.dt, dx.ptr, float(beta),
                 hip.stream_ptr())
        return dx

    def wgrad(self, dy: Act, x: Act, dw_out: torch.Tensor = None, db_out: torch.Tensor = None,
              beta=1.0):
        """dW (torch layout, fp32) accumulated into dw_out (beta=1) or written (beta=0)."""
        if self._resized(x):   # on the re-materialised resized input (not kept from the forward)
            return self._plain_op().wgrad(dy, self._resize(x), dw_out, db_out, beta)
        d = self.desc(x)
        dev = dy.t.device
        assert dy.t.dtype == x.t.dtype, (dy.t.dtype, x.t.dtype)
        if _DET and dw_out is not None and dw_out.dtype == torch.float32 and dw_out.is_contiguous():
            # ordered partial sums straight into the torch-layout gradient (es_conv2d_wgrad_det)
            ys, xs = hip.strides4(dy.strides), hip.strides4(x.strides)
            nb = int(hip.lib().es_conv2d_wgrad_det_ws_bytes(C.byref(d), dy.dt, ys, xs))
            wsb = ws(nb, dev)
            with _probed(self.label and self.label + ".wgrad"):
                hip.call("es_conv2d_wgrad_det", C.byref(d), dy.dt, dy.ptr, ys, x.ptr, xs, hip.ptr(dw_out),
                         float(beta), hip.ptr(wsb), nb, hip.stream_ptr())
            if db_out is not None:
                channel_sum(dy, db_out, beta)
            return dw_out
        # every wgrad kernel ACCUMULATES into its packed [K][R][S][C] output, so:
        #  * packed == torch layout (1x1 / linear, or Cin = 1) and beta = 1: accumulate straight
        #    into the parameter's gradient (no scratch, no unpack);
        #  * otherwise a persistent packed scratch that the unpack leaves zeroed (no zero fill).
        direct = (dw_out is not None and float(beta) == 1.0 and (self.R * self.S == 1 or self.C == 1)
                  and dw_out.is_contiguous() and dw_out.dtype == torch.float32)
        if direct:
            dwk = dw_out
        elif dw_out is not None:
            dwk = getattr(self, "_dwk", None)
            if dwk is None or dwk.device != dev:
                dwk = self._dwk = torch.zeros(self.weight.numel(), dtype=torch.float32, device=dev)
        else:
            dwk = torch.zeros(self.weight.numel(), dtype=torch.float32, device=dev)
        with _probed(self.label and self.label + ".wgrad"):
          hip.call("es_conv2d_wgrad", C.byref(d), dy.dt, dy.ptr, hip.strides4(dy.strides), x.ptr,
                 hip.strides4(x.strides), hip.ptr(dwk), hip.stream_ptr())
        if dw_out is not None and not direct:
            hip.call("es_unpack_conv_grad_clear", hip.ptr(dwk), self.K, self.C, self.R, self.S,
                     hip.ptr(dw_out), float(beta), hip.stream_ptr())
        if db_out is not None:
            channel_sum(dy, db_out, beta)
        return dwk


def channel_sum(x: Act, out: torch.Tensor, beta=1.0):
    wsb = ws(hip.lib().es_channel_sum_ws_bytes(C.byref(x.view)), x.t.device)
    hip.call("es_channel_sum", C.byref(x.view), x.dt, x.ptr, hip.ptr(out), float(beta), hip.ptr(wsb),
             hip.stream_ptr())


# ------------------------------------------------------------------------------ norm + act
# BatchNorm num_batches_tracked increments: one torch kernel per train-mode BN forward (15 per
# neutron step).  Inside MoEWrapper.train_step they are counted on the host and applied at the end
# as one multi-tensor add per distinct count (same final values).
_NBT_PENDING = None


class defer_num_batches:
    def __enter__(self):
        global _NBT_PENDING
        self.prev, _NBT_PENDING = _NBT_PENDING, {}
        return self

    def __exit__(self, exc_type, exc, tb):
        global _NBT_PENDING
        pending, _NBT_PENDING = _NBT_PENDING, self.prev
        if pending is None or exc_type is not None:
            return False     # a failed step applies none of its BatchNorm batch counts
        by_count = {}
        for t, k in pending.values():
            by_count.setdefault(k, []).append(t)
        for k, ts in by_count.items():
            torch._foreach_add_(ts, k)
        return False


def nbt_snapshot():
    """The pending BatchNorm batch counts of the running step (for graph captures to record)."""
    return {} if _NBT_PENDING is None else {k: (t, n) for k, (t, n) in _NBT_PENDING.items()}


def nbt_added(before):
    """[(counter tensor, increments)] added since ``before`` (nbt_snapshot)."""
    if _NBT_PENDING is None:
        return []
    return [(t, n - before.get(k, (t, 0))[1]) for k, (t, n) in _NBT_PENDING.items()
            if n != before.get(k, (t, 0))[1]]


def count_batches(nbt, k):
    """k increments of one counter (a replayed graph's BatchNorm batches)."""
    for _ in range(k):
        _count_batch(nbt)


# dynamic rows: the counts of one expert program, applied on the device in one launch at its end
_LIVE_NBT = None


class batch_live_counts:
    """Inside an expert program on dynamic rows: collect the BatchNorm batch counts and add them on
    the device in one launch when the program ends (es_counters_add_i64_if, gated on the expert's
    active flag) instead of one launch per train-mode BatchNorm forward."""

    def __enter__(self):
        global _LIVE_NBT
        self.prev, _LIVE_NBT = _LIVE_NBT, {}
        return self

    def __exit__(self, exc_type, exc, tb):
        global _LIVE_NBT
        pending, _LIVE_NBT = _LIVE_NBT, self.prev
        if exc_type is None and pending:
            items = list(pending.values())
            ptrs = (C.c_void_p * len(items))(*[t.data_ptr() for t, _ in items])
            vals = (C.c_int64 * len(items))(*[k for _, k in items])
            hip.call("es_counters_add_i64_if", ptrs, vals, len(items), hip.active_ptr(), hip.stream_ptr())
        return False


def _count_batch(nbt):
    if hip.live_on():
        # dynamic rows: +1 on the device when the running expert trains (a captured graph replays it)
        if _LIVE_NBT is not None:
            t, k = _LIVE_NBT.get(id(nbt), (nbt, 0))
            _LIVE_NBT[id(nbt)] = (t, k + 1)
        else:
            hip.call("es_counter_add_i64_if", hip.ptr(nbt), 1, hip.active_ptr(), hip.stream_ptr())
        return
    if _NBT_PENDING is None:
        nbt.add_(1)
    else:
        t, k = _NBT_PENDING.get(id(nbt), (nbt, 0))
        _NBT_PENDING[id(nbt)] = (t, k + 1)


# Data-parallel SyncBN (expertsim/train/ddp.py): while set, train-mode BatchNorm statistics are
# all-gathered and backward sums all-reduced across ranks (set around an expert's step by MoEWrapper)
_NORM_SYNC = None


def set_norm_sync(ddp):
    global _NORM_SYNC
    _NORM_SYNC = ddp


class NormOp:
    """BatchNorm (train: batch stats + running update), GroupNorm or LayerNorm, fused with the
    dropout / activation chain that follows it in the reference's nn.Sequential."""

    def __init__(self, kind, gamma=None, beta=None, groups=1, eps=1e-5, running_mean=None,
                 running_var=None, momentum=0.1, num_batches=None):
        self.kind, self.gamma, self.beta, self.groups, self.eps = kind, gamma, beta, groups, eps
        self.rm, self.rv, self.momentum, self.nbt = running_mean, running_var, momentum, num_batches

    def stats(self, x: Act, train=True):
        dev = x.t.device
        if self.kind == hip.NORM_BN and not train:
            mean = self.rm
            invstd = torch.empty_like(self.rv)
            # eval: invstd from running var (tiny host-side torch op on device buffers)
            invstd.copy_(torch.rsqrt(self.rv + self.eps))
            return mean, invstd
        n_groups = {hip.NORM_BN: x.dims[1], hip.NORM_GN: x.dims[0] * self.groups,
                    hip.NORM_LN: x.dims[0]}[self.kind]
        mean = torch.empty(n_groups, dtype=torch.float32, device=dev)
        invstd = torch.empty(n_groups, dtype=torch.float32, device=dev)
        bn_part = getattr(x, "bn_part", None)
        sync = _NORM_SYNC
        if self.kind == hip.NORM_BN and train and sync is not None:
            # SyncBN: the rank's (count, mean, M2) per channel, all-gathered, merged over the ranks
            Cc = x.dims[1]
            local = torch.empty(3, Cc, dtype=torch.float32, device=dev)
            if bn_part is not None:
                part, chunks = bn_part
                hip.call("es_norm_stats_merge", hip.ptr(part), chunks, Cc, hip.ptr(local), hip.stream_ptr())
            else:
                wsb = ws(hip.lib().es_norm_stats_ws_bytes(C.byref(x.view), self.kind, 1), dev)
                hip.call("es_norm_stats_local", C.byref(x.view), x.dt, x.ptr, hip.ptr(wsb), hip.ptr(local),
                         hip.stream_ptr())
            allp = sync.all_gather(local)
            hip.call("es_norm_stats_finalize", hip.ptr(allp), sync.world, Cc, float(self.eps), hip.ptr(mean),
                     hip.ptr(invstd), hip.ptr(self.rm), hip.ptr(self.rv), float(self.momentum), hip.stream_ptr())
            if self.nbt is not None:
                _count_batch(self.nbt)
            return mean, invstd
        if self.kind == hip.NORM_BN and train and bn_part is not None:
            # partials from the producing conv's epilogue (ConvOp.fwd(bn_stats=True))
            part, chunks = bn_part
            hip.call("es_norm_stats_finalize", hip.ptr(part), chunks, x.dims[1], float(self.eps), hip.ptr(mean),
                     hip.ptr(invstd), hip.ptr(self.rm), hip.ptr(self.rv), float(self.momentum), hip.stream_ptr())
            if self.nbt is not None:
                _count_batch(self.nbt)
            return mean, invstd
        wsb = ws(hip.lib().es_norm_stats_ws_bytes(C.byref(x.view), self.kind, self.groups), dev)
        upd = self.kind == hip.NORM_BN and train
        hip.call("es_norm_stats", C.byref(x.view), x.dt, x.ptr, self.kind, self.groups, float(self.eps),
                 hip.ptr(mean), hip.ptr(invstd), hip.ptr(self.rm) if upd else None,
                 hip.ptr(self.rv) if upd else None, float(self.momentum), hip.ptr(wsb), hip.stream_ptr())
        if upd and self.nbt is not None:
            _count_batch(self.nbt)
        return mean, invstd

    def norm_struct(self, mean, invstd):
        nm = hip.Norm()
        nm.kind, nm.groups = self.kind, self.groups
        nm.mean, nm.invstd = mean.data_ptr(), invstd.data_ptr()
        nm.gamma = self.gamma.data_ptr() if self.gamma is not None else None
        nm.beta = self.beta.data_ptr() if self.beta is not None else None
        return nm

    def fwd(self, x: Act, chain: hip.Chain, out_dtype=None, train=True, addend: Act = None, out: Act = None):
        mean, invstd = self.stats(x, train)
        nm = self.norm_struct(mean, invstd)
        y = out if out is not None else x.like_nhwc(out_dtype or x.t.dtype)
        hip.call("es_norm_act_fwd", C.byref(x.view), x.dt, C.byref(nm), C.byref(chain),
                 C.byref(addend.view) if addend is not None else None,
                 addend.dt if addend is not None else 0, addend.ptr if addend is not None else None,
                 x.ptr, C.byref(y.view), y.dt, y.ptr, hip.stream_ptr())
        return y, (mean, invstd)

    def bwd(self, x: Act, stats, chain: hip.Chain, dy: Act, dx_dtype=None, act_ref: Act = None,
            addend: Act = None, dgamma=None, dbeta=None, dx: Act = None, beta=0.0, dsum=None):
        """dsum: optional fp32 [C] accumulating sum(dx) per channel = grad of the conv bias feeding
        this norm (fused into the apply pass; falls back to a reduction for C > 1024)."""
        mean, invstd = stats
        nm = self.norm_struct(mean, invstd)
        if dx is None:
            dx = x.like_nhwc(dx_dtype or dy.t.dtype)
        wsb = ws(hip.lib().es_norm_bwd_ws_bytes(C.byref(x.view), self.kind, self.groups), x.t.device)
        assert addend is None, "residual addend handled through act_ref"
        sync = _NORM_SYNC
        sums = getattr(dy, "bn_sums", None)
        if (sums is not None and sync is None and self.kind == hip.NORM_BN and act_ref is None and beta == 0.0
                and x.dt == dy.dt == dx.dt and (dsum is None or x.dims[1] <= 1024)):
            # the reduction pass ran in the dgrad that produced dy (ConvOp.dgrad bn_reduce)
            part, chunks, _ = sums
            hip.call("es_norm_act_bwd_sums", C.byref(x.view), x.dt, x.ptr, C.byref(nm), C.byref(chain),
                     C.byref(dy.view), dy.dt, dy.ptr, C.byref(dx.view), dx.dt, dx.ptr, hip.ptr(part), chunks,
                     hip.ptr(dgamma), hip.ptr(dbeta), hip.ptr(dsum), hip.ptr(wsb), hip.stream_ptr())
            return dx
        if self.kind == hip.NORM_BN and sync is not None:
            # SyncBN backward: the rank's sums of dnorm and dnorm*xhat, all-reduced, applied with the
            # global row count (dgamma / dbeta stay local: parameter gradients are all-reduced later)
            assert act_ref is None and beta == 0.0, "SyncBN backward: no act_ref / accumulation"
            Cc = x.dims[1]
            sums = torch.empty(2, Cc, dtype=torch.float32, device=x.t.device)
            args = lambda ph, cnt, cmul, dsm: (ph, C.byref(x.view), x.dt, x.ptr, C.byref(nm), C.byref(chain),
                                         C.byref(dy.view), dy.dt, dy.ptr, C.byref(dx.view), dx.dt, dx.ptr,
                                         hip.ptr(sums), float(cnt), cmul, hip.ptr(dgamma) if ph == 0 else None,
                                         hip.ptr(dbeta) if ph == 0 else None, dsm, hip.ptr(wsb), hip.stream_ptr())
            hip.call("es_norm_bwd_sync", *args(0, 0.0, None, None))
            sync.all_reduce_(sums)
            rows = x.dims[0] * x.dims[2] * x.dims[3]
            if hip.live_on():   # dynamic rows: rows per sample x the expert's global count (device)
                cnt, cmul = x.dims[2] * x.dims[3], sync.global_count_ptr()
            else:
                cnt, cmul = sync.bn_rows(rows, x.dims[0]), None
            hip.call("es_norm_bwd_sync", *args(1, cnt, cmul,
                                                hip.ptr(dsum) if (dsum is not None and Cc <= 1024) else None))
            if dsum is not None and Cc > 1024:
                channel_sum(dx, dsum, 1.0)
            return dx
        hip.call("es_norm_act_bwd", C.byref(x.view), x.dt, x.ptr, C.byref(nm), C.byref(chain),
                 C.byref(dy.view), dy.dt, dy.ptr,
                 C.byref(act_ref.view) if act_ref is not None else None,
                 act_ref.dt if act_ref is not None else 0, act_ref.ptr if act_ref is not None else None,
                 C.byref(dx.view), dx.dt, dx.ptr, float(beta), hip.ptr(dgamma), hip.ptr(dbeta),
                 hip.ptr(dsum) if (dsum is not None and x.dims[1] <= 1024) else None,
                 hip.ptr(wsb), hip.stream_ptr())
        if dsum is not None and x.dims[1] > 1024:
            channel_sum(dx, dsum, 1.0)
        return dx


def act_fwd(x: Act, chain: hip.Chain, out: Act = None, out_dtype=None) -> Act:
    y = out if out is not None else x.like_nhwc(out_dtype or x.t.dtype)
    hip.call("es_act_fwd", C.byref(x.view), x.dt, x.ptr, C.byref(chain), C.byref(y.view), y.dt, y.ptr,
             hip.stream_ptr())
    return y


def act_bwd(x: Act, chain: hip.Chain, dy: Act, act_ref: Act = None, dx: Act = None, dx_dtype=None, beta=0.0):
    """Backward of a norm-free chain evaluated at x (or at act_ref)."""
    if dx is None:
        dx = x.like_nhwc(dx_dtype or dy.t.dtype)
    wsb = ws(hip.lib().es_norm_bwd_ws_bytes(C.byref(x.view), hip.NORM_NONE, 1), x.t.device)
    hip.call("es_norm_act_bwd", C.byref(x.view), x.dt, x.ptr, None, C.byref(chain), C.byref(dy.view), dy.dt,
             dy.ptr, C.byref(act_ref.view) if act_ref is not None else None,
             act_ref.dt if act_ref is not None else 0, act_ref.ptr if act_ref is not None else None,
             C.byref(dx.view), dx.dt, dx.ptr, float(beta), None, None, None, hip.ptr(wsb), hip.stream_ptr())
    return dx


# ------------------------------------------------------------------------------------ pools
class MaxPool:
    def __init__(self, k, s=None):
        self.kh, self.kw = (k, k) if isinstance(k, int) else k
        s = s if s is not None else (self.kh, self.kw)
        self.sh, self.sw = (s, s) if isinstance(s, int) else s

    def out_hw(self, h, w):
        return (h - self.kh) // self.sh + 1, (w - self.kw) // self.sw + 1

    def fwd(self, x: Act, out: Act = None):
        N, Cc, H, W = x.dims
        ho, wo = self.out_hw(H, W)
        y = out if out is not None else Act.nhwc(N, Cc, ho, wo, x.t.dtype, x.t.device)
        idx = torch.empty(y.numel, dtype=torch.uint8, device=x.t.device)
        hip.call("es_maxpool_fwd", C.byref(x.view), x.dt, x.ptr, self.kh, self.kw, self.sh, self.sw,
                 C.byref(y.view), y.ptr, hip.ptr(idx), hip.stream_ptr())
        return y, idx

    def bwd(self, dy: Act, idx, x_dims, dtype, dx: Act = None, beta=0.0):
        N, Cc, H, W = x_dims
        dx = dx if dx is not None else Act.nhwc(N, Cc, H, W, dtype, dy.t.device)
        assert dy.dt == dx.dt
        hip.call("es_maxpool_bwd", C.byref(dy.view), dy.dt, dy.ptr, hip.ptr(idx), self.kh, self.kw, self.sh,
                 self.sw, C.byref(dx.view), dx.ptr, float(beta), hip.stream_ptr())
        return dx


def avgpool_fwd(x: Act) -> Act:
    N, Cc, H, W = x.dims
    y = Act.rows(N, Cc, torch.float32, x.t.device)
    hip.call("es_avgpool_fwd", C.byref(x.view), x.dt, x.ptr, C.byref(y.view), y.ptr, hip.stream_ptr())
    return y


def avgpool_bwd(dy: Act, x_dims, dtype, device) -> Act:
    N, Cc, H, W = x_dims
    dx = Act.nhwc(N, Cc, H, W, dtype, device)
    hip.call("es_avgpool_bwd", C.byref(dy.view), dy.ptr, C.byref(dx.view), dx.dt, dx.ptr, 0.0, hip.stream_ptr())
    return dx


# ---------------------------------------------------------------------------- spectral norm
class SpectralNorm:
    """torch.nn.utils.spectral_norm state of one layer (weight_orig, weight_u, weight_v)."""

    def __init__(self, module):
        self.w = module.weight_orig
        self.u = module.weight_u
        self.v = module.weight_v
        self.h = self.w.shape[0]
        self.wd = self.w[0].numel()

    def sigma(self, update=True):
        """One power iteration (train mode) -> device tensor holding sigma (no host sync)."""
        h, wd = self.h, self.wd
        buf = torch.empty(1 + 2 * (h + wd), dtype=torch.float32, device=self.w.device)
        hip.call("es_sn_power_iter", hip.ptr(self.w), h, wd, hip.ptr(self.u), hip.ptr(self.v),
                 hip.ptr(buf), 1 if update else 0, hip.active_ptr(), hip.stream_ptr())
        # the kernel snapshots the u, v it used after the scratch (the next call updates them in place)
        o = 1 + h + wd
        return buf[:1], buf[o:o + h], buf[o + h:o + h + wd]

    @staticmethod
    def sigma_many(sns, update=True):
        """sigma() of several layers: the small ones (h*wd < 16384) share one launch (a block per
        layer); larger ones (discriminator fc1) run the multi-block mat-vecs."""
        out = [None] * len(sns)
        small = [i for i, sn in enumerate(sns) if sn.h * sn.wd < 16384]
        if len(small) < 2:
            small = []
        for i, sn in enumerate(sns):
            if i not in small:
                out[i] = sn.sigma(update)
        for c0 in range(0, len(small), 8):
            idx = small[c0:c0 + 8]
            n = len(idx)
            bufs = [torch.empty(1 + 2 * (sns[i].h + sns[i].wd), dtype=torch.float32, device=sns[i].w.device)
                    for i in idx]
            arr = lambda vals: (C.c_void_p * n)(*vals)
            hip.call("es_sn_power_iter_batch", n, arr([sns[i].w.data_ptr() for i in idx]),
                     (C.c_int * n)(*[sns[i].h for i in idx]), (C.c_int * n)(*[sns[i].wd for i in idx]),
                     arr([sns[i].u.data_ptr() for i in idx]), arr([sns[i].v.data_ptr() for i in idx]),
                     arr([b.data_ptr() for b in bufs]), 1 if update else 0, hip.active_ptr(), hip.stream_ptr())
            for i, b in zip(idx, bufs):
                h, wd = sns[i].h, sns[i].wd
                o = 1 + h + wd
                out[i] = (b[:1], b[o:o + h], b[o + h:o + h + wd])
        return out

    @staticmethod
    def bwd_many(jobs, beta=1.0):
        """bwd() of several layers, jobs = [(sn, g_sn, sig, dw_orig)]: the small ones share a launch."""
        small = [j for j in jobs if not (j[0].h * j[0].wd >= 16384 and j[0].h + j[0].wd >= 256)]
        if len(small) < 2:
            small = []
        for j in jobs:
            if not any(j is k for k in small):
                j[0].bwd(j[1], j[2], j[3], beta)
        for c0 in range(0, len(small), 8):
            part = small[c0:c0 + 8]
            n = len(part)
            arr = lambda vals: (C.c_void_p * n)(*vals)
            hip.call("es_sn_bwd_batch", n, arr([sn.w.data_ptr() for sn, _, _, _ in part]),
                     arr([g.data_ptr() for _, g, _, _ in part]),
                     (C.c_int * n)(*[sn.h for sn, _, _, _ in part]), (C.c_int * n)(*[sn.wd for sn, _, _, _ in part]),
                     arr([sig[1].data_ptr() for _, _, sig, _ in part]), arr([sig[2].data_ptr() for _, _, sig, _ in part]),
                     arr([sig[0].data_ptr() for _, _, sig, _ in part]), arr([d.data_ptr() for _, _, _, d in part]),
                     float(beta), hip.stream_ptr())

    def bwd(self, g_sn: torch.Tensor, sig, dw_orig: torch.Tensor, beta=1.0):
        sigma, u, v = sig
        hip.call("es_sn_bwd", hip.ptr(self.w), hip.ptr(g_sn), self.h, self.wd, hip.ptr(u), hip.ptr(v),
                 hip.ptr(sigma), hip.ptr(dw_orig), float(beta), hip.stream_ptr())
