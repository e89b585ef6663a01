"""Time the generator's fp32 convs with exact fp32 MFMA vs split-fp32 (three bf16 planes, six
products) at B = 1024, and the split result's deviation from the exact one.

usage: python tools/mb_split.py [B] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))

from expertsim import hip, layers  # noqa: E402
from expertsim.layers import Act, ConvOp, Upsample  # noqa: E402

SHAPES = {"c0": (128, 13, 13, 256, 3, 1, 0, (2, 2)), "c5": (256, 24, 24, 128, 3, 1, 0, (2, 2)),
          "c9": (128, 46, 46, 64, 2, 1, 0, None)}


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = "cuda"
    layers.set_deterministic(True)
    torch.manual_seed(0)
    for name, (Cin, H, W, Cout, k, st, pad, up) in SHAPES.items():
        w = torch.nn.Parameter(torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5)
        b = torch.nn.Parameter(torch.randn(Cout, device=dev))
        op = ConvOp(w, b, stride=st, pad=pad, upsample=Upsample((H, W), scale=up) if up else None)
        x = Act.nhwc(N, Cin, H, W, torch.float32, dev)
        x.t.normal_()
        y = op.fwd(x, out_dtype=torch.float32)
        dy = y.like_nhwc(torch.float32)
        dy.t.normal_()
        flops = 2.0 * N * y.dims[2] * y.dims[3] * Cout * Cin * k * k
        res = {}
        for split in (0, 1):
            layers.set_f32_split(split)
            dw = torch.zeros_like(w)
            outs = {}
            t = {}
            t["fwd"] = timeit(lambda: op.fwd(x, out_dtype=torch.float32), reps)
            outs["fwd"] = op.fwd(x, out_dtype=torch.float32).t.clone()
            t["dgrad"] = timeit(lambda: op.dgrad(dy, x, dx_dtype=torch.float32), reps)
            outs["dgrad"] = op.dgrad(dy, x, dx_dtype=torch.float32).t.clone()
            t["wgrad"] = timeit(lambda: op.wgrad(dy, x, dw, None, beta=0.0), reps)
            op.wgrad(dy, x, dw, None, beta=0.0)
            outs["wgrad"] = dw.detach().clone()
            torch.cuda.synchronize()
            res[split] = (t, outs)
        for m in ("fwd", "dgrad", "wgrad"):
            te, ts = res[0][0][m], res[1][0][m]
            a, c = res[0][1][m], res[1][1][m]
            dev_rel = ((a - c).abs().max() / a.abs().max()).item()
            print(f"{name} {m} B={N}: exact {te:8.1f} us {flops / te / 1e6:6.1f} TF | split {ts:8.1f} us "
                  f"{flops / ts / 1e6:6.1f} TF | x{te / ts:.2f} | max|split-exact|/max|exact| {dev_rel:.2e}",
                  flush=True)
    layers.set_f32_split(False)


if __name__ == "__main__":
    main()
