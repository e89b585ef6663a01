"""ctypes binding of libexpertsim_hip.so (the C ABI in include/expertsim_hip.h).

The library is built in-tree (``csrc/Makefile`` -> ``expertsim/_lib/libexpertsim_hip.so``).  There
is no fallback: if the library or a HIP device is missing, every op raises.  Tensors are torch
tensors used purely as device memory; all arithmetic happens in the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

# ES_LIB: load another build of the library (same-box A/B of two builds, tools/gpu_ab.sh)
_LIB_PATH = os.environ.get("ES_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                     "libexpertsim_hip.so")
_lib = None

ES_F32, ES_BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2
NORM_NONE, NORM_BN, NORM_GN, NORM_LN = 0, 1, 2, 3


class View(C.Structure):
    _fields_ = [("n", C.c_int), ("c", C.c_int), ("h", C.c_int), ("w", C.c_int), ("s", C.c_int64 * 4),
                ("rows", C.c_void_p)]


class Dropout(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("stream", C.c_uint32), ("threshold", C.c_uint32),
                ("scale", C.c_float), ("enabled", C.c_int), ("step_ptr", C.c_void_p), ("step_mul", C.c_int32),
                ("index_offset", C.c_uint64), ("index_ptr", C.c_void_p), ("index_mul", C.c_int64)]


class ConvDesc(C.Structure):
    _fields_ = [("N", C.c_int), ("C", C.c_int), ("H", C.c_int), ("W", C.c_int), ("Hu", C.c_int),
                ("Wu", C.c_int), ("K", C.c_int), ("P", C.c_int), ("Q", C.c_int), ("R", C.c_int),
                ("S", C.c_int), ("stride", C.c_int), ("pad", C.c_int), ("hmap", C.c_void_p),
                ("wmap", C.c_void_p), ("up_h", C.c_int), ("up_w", C.c_int), ("subpixel", C.c_int),
                ("rows", C.c_void_p), ("rows_px", C.c_int)]


class Norm(C.Structure):
    _fields_ = [("kind", C.c_int), ("groups", C.c_int), ("mean", C.c_void_p),
                ("invstd", C.c_void_p), ("gamma", C.c_void_p), ("beta", C.c_void_p)]


class Chain(C.Structure):
    _fields_ = [("drop", Dropout), ("dropout_first", C.c_int), ("act", C.c_int), ("slope", C.c_float),
                ("keep", C.c_void_p), ("keep_ready", C.c_int)]


class GenLoss(C.Structure):
    _fields_ = [("n", C.c_int), ("latent", C.c_int), ("noise", C.c_int), ("di_strength", C.c_float),
                ("in_strength", C.c_float), ("aux_strength", C.c_float), ("std_mean", C.c_void_p),
                ("rows", C.c_void_p)]


class DFront2Params(C.Structure):
    _fields_ = [("w1", C.c_void_p), ("sigma1", C.c_void_p), ("b1", C.c_void_p), ("g1", C.c_void_p),
                ("be1", C.c_void_p), ("w2", C.c_void_p), ("sigma2", C.c_void_p), ("b2", C.c_void_p),
                ("g2", C.c_void_p), ("be2", C.c_void_p), ("eps1", C.c_float), ("eps2", C.c_float),
                ("slope", C.c_float), ("ph", C.c_int), ("pw", C.c_int), ("rows", C.c_void_p)]


class DMlpParams(C.Structure):
    _fields_ = [("w1", C.c_void_p), ("sigma1", C.c_void_p), ("b1", C.c_void_p), ("g1", C.c_void_p),
                ("be1", C.c_void_p), ("w2", C.c_void_p), ("sigma2", C.c_void_p), ("b2", C.c_void_p),
                ("g2", C.c_void_p), ("be2", C.c_void_p), ("w3", C.c_void_p), ("sigma3", C.c_void_p),
                ("b3", C.c_void_p), ("eps1", C.c_float), ("eps2", C.c_float), ("slope", C.c_float),
                ("rows", C.c_void_p)]


class PackJob(C.Structure):
    _fields_ = [("w", C.c_void_p), ("K", C.c_int), ("C", C.c_int), ("R", C.c_int), ("S", C.c_int),
                ("mode", C.c_int), ("dt", C.c_int), ("planes", C.c_int), ("out", C.c_void_p)]


P = C.c_void_p
I64 = C.c_int64
_SIGS = {
    "es_last_error": (C.c_char_p, []),
    "es_version": (C.c_int, []),
    "es_device_sync": (C.c_int, []),
    "es_conv_set_glds": (C.c_int, [C.c_int]),
    "es_conv_set_ring": (C.c_int, [C.c_int]),
    "es_conv_set_subpixel": (C.c_int, [C.c_int]),
    "es_conv_set_ring256": (C.c_int, [C.c_int]),
    "es_conv_set_persist": (C.c_int, [C.c_int]),
    "es_conv_set_p256": (C.c_int, [C.c_int]),
    "es_conv_subpixel_ok": (C.c_int, [P, C.c_int]),
    "es_subpixel_taps": (C.c_int, [C.c_int, C.c_int]),
    "es_conv2d_fwd": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_int, P, P]),
    "es_conv2d_fwd_stats": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_int, P, P, I64, P, P]),
    "es_conv2d_dgrad": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, P, C.c_float, P]),
    "es_conv2d_dgrad_bnred": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, P, P, P, P, P, I64, P, P]),
    "es_conv2d_wgrad": (C.c_int, [P, C.c_int, P, P, P, P, P, P]),
    "es_conv2d_wgrad_det_ws_bytes": (I64, [P, C.c_int, P, P]),
    "es_conv2d_wgrad_det": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_float, P, I64, P]),
    "es_set_deterministic": (C.c_int, [C.c_int]),
    "es_conv2d_splitk_ws_bytes": (I64, [P, C.c_int]),
    "es_conv2d_fwd_det": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_int, P, P, I64, P]),
    "es_conv2d_dgrad_det": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, P, P, I64, P]),
    "es_conv_set_f32_chunk": (C.c_int, [C.c_int]),
    "es_conv_set_f32_split": (C.c_int, [C.c_int]),
    "es_conv_set_wgrad_ws": (C.c_int, [C.c_int]),
    "es_weight_planes_offset": (C.c_int64, [C.c_int64]),
    "es_pack_weight_planes": (C.c_int, [P, C.c_int64, P, P]),
    "es_pack_conv_weights": (C.c_int, [P, C.c_int, P]),
    "es_conv_launch_count": (C.c_int64, []),
    "es_conv_exec_flops": (C.c_int, [C.POINTER(C.c_double), C.c_int]),
    "es_pack_conv_weight": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int, P]),
    "es_unpack_conv_grad": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, C.c_float, P]),
    "es_unpack_conv_grad_clear": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_float, P]),
    "es_norm_stats_ws_bytes": (I64, [P, C.c_int, C.c_int]),
    "es_norm_stats": (C.c_int, [P, C.c_int, P, C.c_int, C.c_int, C.c_float, P, P, P, P, C.c_float, P, P]),
    "es_norm_act_fwd": (C.c_int, [P, C.c_int, P, P, P, C.c_int, P, P, P, C.c_int, P, P]),
    "es_norm_stats_finalize": (C.c_int, [P, C.c_int, C.c_int, C.c_float, P, P, P, P, C.c_float, P]),
    "es_norm_bwd_ws_bytes": (I64, [P, C.c_int, C.c_int]),
    "es_norm_act_bwd": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, P, P, C.c_int, P, P, C.c_int, P,
                                  C.c_float, P, P, P, P, P]),
    "es_norm_act_bwd_sums": (C.c_int, [P, C.c_int, P, P, P, P, C.c_int, P, P, C.c_int, P, P, C.c_int, P, P, P,
                                       P, P]),
    "es_norm_stats_merge": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "es_norm_stats_local": (C.c_int, [P, C.c_int, P, P, P, P]),
    "es_norm_bwd_sync": (C.c_int, [C.c_int, P, C.c_int, P, P, P, P, C.c_int, P, P, C.c_int, P, P, C.c_float, P, P,
                                   P, P, P, P]),
    "es_act_fwd": (C.c_int, [P, C.c_int, P, P, P, C.c_int, P, P]),
    "es_dropout_keep_bits": (C.c_int, [P, P, P]),
    "es_channel_sum_ws_bytes": (I64, [P]),
    "es_channel_sum": (C.c_int, [P, C.c_int, P, P, C.c_float, P, P]),
    "es_maxpool_fwd": (C.c_int, [P, C.c_int, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P]),
    "es_maxpool_bwd": (C.c_int, [P, C.c_int, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, C.c_float, P]),
    "es_dfront_fwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, C.c_float, C.c_float, P, P, P, P,
                                P]),
    "es_dfront_part_floats": (I64, [C.c_int]),
    "es_dfront_bwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, C.c_float, C.c_float, P, P, P, P,
                                P, P, P, P, P, P, P, P]),
    "es_dfront2_ok": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "es_dfront2_part_floats": (I64, [C.c_int]),
    "es_dfront2_save_floats": (I64, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "es_dfront2_fwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, P, P, I64, P, P]),
    "es_dfront2_bwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, I64, P, P, P, P, P, P, P, P, P, P,
                                 P, P]),
    "es_dfront2_set_probe": (None, [P]),
    "es_dmlp_part_floats": (I64, [C.c_int, C.c_int]),
    "es_dmlp_fwd": (C.c_int, [P, I64, C.c_int, C.c_int, P, P, P, P, P, P, P, P]),
    "es_dmlp_bwd": (C.c_int, [P, I64, C.c_int, C.c_int, P, P, P, P, P, P, P, P, P, I64, P, P, P, P, P, P, P, P, P,
                              P, P, P]),
    "es_upsample_bwd": (C.c_int, [P, C.c_int, P, P, P, P, P, P, C.c_int, P, C.c_float, P]),
    "es_upsample_fwd": (C.c_int, [P, C.c_int, P, P, P, P, P, P]),
    "es_copy": (C.c_int, [P, C.c_int, P, P, C.c_int, P, C.c_float, C.c_float, P]),
    "es_avgpool_fwd": (C.c_int, [P, C.c_int, P, P, P, P]),
    "es_avgpool_bwd": (C.c_int, [P, P, P, C.c_int, P, C.c_float, P]),
    "es_gather_rows": (C.c_int, [P, I64, P, C.c_int, C.c_int, P, I64, P]),
    "es_gather_rows_at": (C.c_int, [P, I64, P, P, C.c_int, C.c_int, P, I64, P, P]),
    "es_scatter_rows_at": (C.c_int, [P, P, P, C.c_int, P, P, P]),
    "es_sn_power_iter": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int, P, P]),
    "es_sn_power_iter_batch": (C.c_int, [C.c_int, P, P, P, P, P, P, C.c_int, P, P]),
    "es_sn_bwd_batch": (C.c_int, [C.c_int, P, P, P, P, P, P, P, P, C.c_float, P]),
    "es_sn_bwd": (C.c_int, [P, P, C.c_int, C.c_int, P, P, P, P, C.c_float, P]),
    "es_hinge_d": (C.c_int, [P, P, C.c_int, P, P, P, P, P, P]),
    "es_image_expsum": (C.c_int, [P, C.c_int, P, P, P]),
    "es_channel_sums": (C.c_int, [P, C.c_int, P, C.c_int, P, P]),
    "es_gen_losses": (C.c_int, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "es_image_expsum_bwd": (C.c_int, [P, C.c_int, P, P, P, P, C.c_float, P]),
    "es_router_gumbel": (C.c_int, [P, P, C.c_int, C.c_int, C.c_float, P, P, P, P]),
    "es_router_alb": (C.c_int, [P, C.c_int, C.c_int, C.c_float, C.c_float, P, P, P]),
    "es_router_loss": (C.c_int, [P, P, P, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, P,
                                 C.c_int, P, P, C.c_int, P, P, P]),
    "es_router_colsum": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "es_router_dispatch": (C.c_int, [P, C.c_int, C.c_int, P, P, P]),
    "es_dp_metrics_merge": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "es_step_metrics": (C.c_int, [P, C.c_int, P, P, P, C.c_float, C.c_float, C.c_float, C.c_int, P, P]),
    "es_scatter_rows": (C.c_int, [P, P, C.c_int, P, P]),
    "es_adam": (C.c_int, [P, P, P, P, I64, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int,
                          C.c_float, P]),
    "es_adam_dev": (C.c_int, [P, P, P, P, I64, C.c_float, C.c_float, C.c_float, C.c_float, P, C.c_float, P, P]),
    "es_ema_update": (C.c_int, [P, P, I64, C.c_float, C.c_float, P]),
    "es_randn": (C.c_int, [P, I64, C.c_uint64, C.c_uint32, P]),
    "es_rand_exponential": (C.c_int, [P, I64, C.c_uint64, C.c_uint32, P]),
    "es_randn_dev": (C.c_int, [P, I64, C.c_uint64, C.c_uint32, P, C.c_int32, I64, P]),
    "es_rand_exponential_dev": (C.c_int, [P, I64, C.c_uint64, C.c_uint32, P, C.c_int32, I64, P]),
    "es_counter_add": (C.c_int, [P, C.c_int32, P]),
    "es_randn_dev_at": (C.c_int, [P, I64, C.c_uint64, C.c_uint32, P, C.c_int32, I64, P, I64, P]),
    "es_counter_add_if": (C.c_int, [P, C.c_int32, P, P]),
    "es_counter_add_i64_if": (C.c_int, [P, I64, P, P]),
    "es_counters_add_i64_if": (C.c_int, [P, P, C.c_int, P, P]),
    "es_expert_plan": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P]),
    "es_div_by": (C.c_int, [P, C.c_int, P, P]),
    "es_struct_size": (I64, [C.c_int]),
    "es_dropout_mask": (C.c_int, [P, I64, P, P]),
}


class HipError(RuntimeError):
    pass


def lib_path() -> str:
    return _LIB_PATH


_ABI_STRUCTS = (View, Dropout, ConvDesc, Norm, Chain, GenLoss, DFront2Params, DMlpParams, PackJob)


def lib():
    """Load the kernel library (raises if it was not built: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise HipError(f"{_LIB_PATH} missing: build it with `make -C csrc` "
                           f"(or __graft_entry__.build()); expertsim has no CPU fallback")
        L = C.CDLL(_LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        for i, st in enumerate(_ABI_STRUCTS):   # the mirrors must match the header's layouts
            if L.es_struct_size(i) != C.sizeof(st):
                raise HipError(f"{st.__name__}: ctypes size {C.sizeof(st)} != C size {L.es_struct_size(i)} "
                               f"(bindings out of date with include/expertsim_hip.h)")
        _lib = L
    return _lib


_FN = {}


def call(name, *args):
    fn = _FN.get(name)
    if fn is None:
        fn = _FN[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise HipError(f"{name} failed ({rc}): {lib().es_last_error().decode()}")
    return rc


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise HipError("expertsim kernels need tensors on a HIP device (no CPU fallback)")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def stream_ptr() -> int:
    """The current HIP stream of the current device (torch's stream context, graph capture
    included).  The raw accessors skip torch.cuda.current_stream()'s Python wrapping (~8 us a
    call; the eager step makes ~450 launches per expert)."""
    if _raw_stream is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def dt_of(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return ES_F32
    if t.dtype == torch.bfloat16:
        return ES_BF16
    raise HipError(f"unsupported dtype {t.dtype}")


def dt_of_dtype(dtype) -> int:
    if dtype == torch.float32:
        return ES_F32
    if dtype == torch.bfloat16:
        return ES_BF16
    raise HipError(f"unsupported dtype {dtype}")


def strides4(s):
    arr = (C.c_int64 * 4)()
    for i in range(4):
        arr[i] = int(s[i])
    return arr


# Dynamic rows (a multi-expert step without host synchronisation): while set, the running expert's
# buffers have a capacity of `cap` samples of which a device count (int32 [1]) is live; every view /
# conv descriptor whose leading (sample) dimension is `cap` carries that count (es_view_t.rows,
# es_conv_desc_t.rows) and the kernels skip the padding samples.  `active` (int32 [1], != 0 when the
# expert trains this step) gates its optimizer, spectral-norm and batch-counter updates.
_LIVE = None


class live_rows:
    """Context: the expert program that follows runs on `cap`-sample buffers with `rows` live."""

    def __init__(self, cap: int, rows: torch.Tensor, active: torch.Tensor):
        self.state = (int(cap), rows, active)

    def __enter__(self):
        global _LIVE
        self.prev, _LIVE = _LIVE, self.state
        return self

    def __exit__(self, *exc):
        global _LIVE
        _LIVE = self.prev
        return False


def live_on() -> bool:
    return _LIVE is not None


def rows_ptr(n: int):
    """The live-count pointer for a tensor of n samples (None outside a dynamic program or when n
    is not the capacity).  Callers pass sample counts only: a view whose leading dimension is not a
    sample dimension is built with sample=False (layers.Act), whatever its size."""
    if _LIVE is None or int(n) != _LIVE[0]:
        return None
    return _LIVE[1].data_ptr()


def active_ptr():
    """The running expert's active flag (device int32 [1]) as a pointer, or None (always active)."""
    return None if _LIVE is None else C.c_void_p(_LIVE[2].data_ptr())


def active_tensor():
    return None if _LIVE is None else _LIVE[2]


def live_count():
    """The running expert's live rows as a host int (synchronises; tests and debugging only), or None
    outside a dynamic-rows program."""
    return None if _LIVE is None else int(_LIVE[1].item())


def make_view(dims, strides, sample: bool = True) -> View:
    """sample: the leading dimension counts samples (layers.Act.sample); only such a view of the
    running expert's capacity carries its live count."""
    v = View()
    v.n, v.c, v.h, v.w = (int(d) for d in dims)
    for i in range(4):
        v.s[i] = int(strides[i])
    v.rows = rows_ptr(v.n) if sample else None
    return v


def set_index_offset(d: Dropout, n_offset, per: int):
    """A dropout's logical index offset: n_offset (the first sample's index in the expert's global
    batch) x elements per sample; n_offset may be a device int32 [1] (data-parallel dynamic rows:
    es_dropout_t.index_ptr, the offset added on the device)."""
    if isinstance(n_offset, torch.Tensor):
        d.index_offset = 0
        d.index_ptr = n_offset.data_ptr()
        d.index_mul = int(per)
    else:
        d.index_offset = int(n_offset) * int(per)
        d.index_ptr = None
        d.index_mul = 0


# Device step counter of the running train step (see set_step_counter): dropout structs built while
# it is set add step * STEP_STREAM_MUL to their stream ON THE DEVICE, so a captured graph of the
# step draws the masks of the step it is replayed for.
STEP_STREAM_MUL = 1024
_STEP_COUNTER = None


def set_step_counter(t):
    """t: device int32 tensor [1] holding the current step, or None (streams used as given)."""
    global _STEP_COUNTER
    _STEP_COUNTER = t


def dropout_struct(p: float = 0.0, seed: int = 0, stream: int = 0, enabled: bool = False,
                   index_offset: int = 0) -> Dropout:
    """index_offset: logical element index of the tensor's first element in the global batch
    (data-parallel ranks: first sample of the rank's rows x elements per sample)."""
    d = Dropout()
    d.enabled = 1 if (enabled and p > 0.0) else 0
    if d.enabled:
        d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        d.stream = int(stream) & 0xFFFFFFFF
        d.index_offset = int(index_offset)
        if _STEP_COUNTER is not None:
            d.step_ptr = _STEP_COUNTER.data_ptr()
            d.step_mul = STEP_STREAM_MUL
        d.threshold = int((1.0 - float(p)) * 16777216.0)   # floor, = philox.keep_threshold
        d.scale = float(np.float32(1.0) / np.float32(1.0 - p))   # torch: bernoulli_(1-p).div_(1-p) in fp32
    return d


def chain_struct(act=ACT_NONE, slope=0.1, drop: Dropout | None = None, dropout_first=True) -> Chain:
    ch = Chain()
    ch.act = act
    ch.slope = slope
    ch.dropout_first = 1 if dropout_first else 0
    if drop is not None:
        ch.drop = drop
    return ch


def attach_keep(chain: Chain, rows: int, channels: int, device):
    """Give a dropout chain a device keep-bit buffer [rows][channels/8] (es_chain_t.keep): the
    forward norm pass stores the mask it draws and the backward passes read it instead of re-running
    Philox.  Returns the buffer (the caller keeps it alive until the backward), or None when the
    chain has no dropout or channels % 8 != 0."""
    if not chain.drop.enabled or channels % 8:
        return None
    buf = torch.empty(rows * (channels // 8), dtype=torch.uint8, device=device)
    chain.keep = buf.data_ptr()
    return buf
