"""Phase timestamps of es_dfront2 kernels (workgroup 0; library built with -DES_DF2_PROBE into
tools/_probe/).  usage: ES_LIB=tools/_probe/libexpertsim_hip.so python tools/df2_probe.py [B]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "generative-dnn-for-physics-simulations-cern_amd"))
from expertsim import hip  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H = W = 44
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(B, 1, H, W, device=dev)
t = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc)
w1, w2 = t(32, 1, 3, 3, sc=0.3), t(16, 32, 3, 3, sc=0.06)
b1, g1, be1 = t(32, sc=0.1), 1 + t(32, sc=0.1), t(32, sc=0.1)
b2, g2, be2 = t(16, sc=0.1), 1 + t(16, sc=0.1), t(16, sc=0.1)
s1 = torch.tensor([1.7], device=dev)
s2 = torch.tensor([1.3], device=dev)
p = hip.DFront2Params()
p.w1, p.sigma1, p.b1, p.g1, p.be1 = (v.data_ptr() for v in (w1, s1, b1, g1, be1))
p.w2, p.sigma2, p.b2, p.g2, p.be2 = (v.data_ptr() for v in (w2, s2, b2, g2, be2))
p.eps1 = p.eps2 = 1e-5
p.slope = 0.1
p.ph = p.pw = 2
F = 1305
X = torch.zeros(B, F, device=dev)
stats = torch.empty(B * 32, device=dev)
probe = torch.zeros(32, dtype=torch.int64, device=dev)
hip.lib().es_dfront2_set_probe(C.c_void_p(probe.data_ptr()))
save = torch.empty(B * hip.lib().es_dfront2_save_floats(H, W, 2, 2), device=dev)
fwd = lambda: hip.call("es_dfront2_fwd", hip.ptr(x), hip.strides4(x.stride()), B, H, W, C.byref(p), hip.ptr(stats),
                       hip.ptr(X), F, hip.ptr(save), hip.stream_ptr())
dX = torch.randn(B, F, device=dev)
dx = torch.empty_like(x)
part = torch.empty(hip.lib().es_dfront2_part_floats(B), device=dev)
outs = [torch.zeros(n, device=dev) for n in (288, 32, 32, 32, 4608, 16, 16, 16)]


def bwd(want_dx, want_w):
    hip.call("es_dfront2_bwd", hip.ptr(x), hip.strides4(x.stride()), B, H, W, C.byref(p), hip.ptr(stats),
             hip.ptr(save), hip.ptr(dX), F, hip.ptr(dx) if want_dx else None, hip.strides4(dx.stride()) if want_dx else None,
             hip.ptr(part) if want_w else None, *[hip.ptr(o) if want_w else None for o in outs], hip.stream_ptr())


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def phases(lo, hi, names):
    v = probe.cpu().tolist()
    out = []
    for i in range(lo, hi):
        out.append(f"{names[i - lo]} {(v[i + 1] - v[i]) / 100:.1f}")   # wall_clock64: 100 MHz
    return ", ".join(out)


print(f"B={B} fwd {timeit(fwd):.1f} us |", phases(10, 14, ["b1stats", "b1out", "b2conv", "b2stats+pool"]))
fwd()
for wd, ww in ((False, True), (True, False)):
    us = timeit(lambda: bwd(wd, ww))
    print(f"bwd dx={wd} w={ww} {us:.1f} us |",
          phases(0, 8, ["b1out", "b2conv", "route+dense", "wgrad2", "dgrad2", "b1pass1", "b1pass2", "dx+wred"]))
