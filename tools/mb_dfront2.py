"""Micro-benchmark of the fused discriminator front (d_front2.hip) at the bench shape (GPU).

usage: python tools/mb_dfront2.py [N]     (ES_LIB=... selects an A/B build; builds with
-DES_DF2_PROBE also print workgroup 0's phase timestamps)"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))

from expertsim import hip  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    H = W = 44
    pool = (2, 2)
    dev = "cuda"
    L = hip.lib()
    torch.manual_seed(1)
    x = torch.randn(N, 1, H, W, device=dev)
    t = dict(w1=torch.randn(32, 1, 3, 3) / 3, s1=torch.tensor([1.7]), b1=0.1 * torch.randn(32),
             g1=1 + 0.1 * torch.randn(32), be1=0.1 * torch.randn(32), w2=torch.randn(16, 32, 3, 3) / 17,
             s2=torch.tensor([1.3]), b2=0.1 * torch.randn(16), g2=1 + 0.1 * torch.randn(16),
             be2=0.1 * torch.randn(16))
    dv = {k: v.to(dev) for k, v in t.items()}
    prm = hip.DFront2Params()
    for k in ("w1", "sigma1", "b1", "g1", "be1", "w2", "sigma2", "b2", "g2", "be2"):
        setattr(prm, k, dv[k.replace("sigma", "s")].data_ptr())
    prm.eps1 = prm.eps2 = 1e-5
    prm.slope = 0.1
    prm.ph, prm.pw = pool
    nf = 16 * 9 * 9
    Fs = nf + 9
    X = torch.zeros(N, Fs, device=dev)
    stats = torch.empty(N * 32, device=dev)
    save = torch.empty(N * L.es_dfront2_save_floats(H, W, *pool), device=dev)
    probe = torch.zeros(16, dtype=torch.int64, device=dev)
    L.es_dfront2_set_probe(C.c_void_p(probe.data_ptr()))
    fwd = lambda sv: hip.call("es_dfront2_fwd", hip.ptr(x), hip.strides4(x.stride()), N, H, W, C.byref(prm),
                              hip.ptr(stats), hip.ptr(X), Fs, hip.ptr(sv) if sv is not None else None,
                              hip.stream_ptr())
    dX = torch.randn(N, Fs, device=dev)
    dx = torch.empty(N, 1, H, W, device=dev)
    part = torch.empty(L.es_dfront2_part_floats(N), device=dev)
    outs = [torch.zeros(n, device=dev) for n in (288, 32, 32, 32, 4608, 16, 16, 16)]

    def bwd(want_dx, want_w):
        hip.call("es_dfront2_bwd", hip.ptr(x), hip.strides4(x.stride()), N, H, W, C.byref(prm), hip.ptr(stats),
                 hip.ptr(save), hip.ptr(dX), Fs, hip.ptr(dx) if want_dx else None,
                 hip.strides4(dx.stride()) if want_dx else None, hip.ptr(part) if want_w else None,
                 *[hip.ptr(o) if want_w else None for o in outs], hip.stream_ptr())

    res = {"fwd(save)": timed(lambda: fwd(save)), "fwd(no save)": timed(lambda: fwd(None))}
    fwd(save)
    torch.cuda.synchronize()
    pf = probe.cpu().tolist()
    res["bwd D-step (w)"] = timed(lambda: bwd(False, True))
    pw = probe.cpu().tolist()
    res["bwd G-step (dx)"] = timed(lambda: bwd(True, False))
    pd = probe.cpu().tolist()
    print(f"N={N} " + "  ".join(f"{k} {v:7.1f} us" for k, v in res.items()), flush=True)
    if any(pf):
        us = lambda p, i, j: (p[j] - p[i]) / 100.0   # wall_clock64: 100 MHz
        print("probe fwd (wg 0, us): stats %.2f out %.2f conv2 %.2f tail %.2f" % (
            us(pf, 10, 11), us(pf, 11, 12), us(pf, 12, 13), us(pf, 13, 14)))
        for name, p in (("bwd w", pw), ("bwd dx", pd)):
            print("probe %s (wg 0, us): load %.2f pool/gn2 %.2f wgrad2 %.2f dgrad2 %.2f b1sums %.2f b1 %.2f tail %.2f"
                  % (name, us(p, 0, 1), us(p, 2, 3), us(p, 3, 4), us(p, 4, 5), us(p, 5, 6), us(p, 6, 7),
                     us(p, 7, 8)))


if __name__ == "__main__":
    main()
