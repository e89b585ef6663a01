"""Alternating A/B timing of one split-fp32 conv op of the neutron generator under a library switch.

usage: python tools/mb_ab.py <c0|c5|c9> <fwd|dgrad|wgrad> <switch, e.g. es_conv_set_wgrad_ws> [batch 1024]
[rounds 4] [reps 10] [switch values "0,1"]
Times `reps` ops per arm with HIP events on the launch stream, arms alternating each round (the first
timed arm rotates), prints per-round ms per op and the median per arm."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
from expertsim import hip, layers  # noqa: E402
from expertsim.layers import Act, ConvOp, Upsample  # noqa: E402

SHAPES = {"c0": (128, 13, 13, 256, 3, (2, 2)), "c5": (256, 24, 24, 128, 3, (2, 2)), "c9": (128, 46, 46, 64, 2, None)}


def main():
    layer, mode, switch = sys.argv[1], sys.argv[2], sys.argv[3]
    N = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 10
    vals = [int(v) for v in sys.argv[7].split(",")] if len(sys.argv) > 7 else [0, 1]
    Cin, H, W, Cout, k, up = SHAPES[layer]
    dev = "cuda"
    lib = hip.lib()
    layers.set_deterministic(True)
    layers.set_f32_split(True)
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.nn.Parameter(torch.randn(Cout, Cin, k, k, device=dev, generator=g) / (Cin * k * k) ** 0.5)
    b = torch.nn.Parameter(torch.randn(Cout, device=dev, generator=g))
    op = ConvOp(w, b, upsample=Upsample((H, W), scale=up) if up else None)
    x = Act.nhwc(N, Cin, H, W, torch.float32, dev)
    x.t.normal_(generator=g)
    y = op.fwd(x)
    dy = y.like_nhwc()
    dy.t.normal_(generator=g)
    dw, db = torch.zeros_like(w), torch.zeros_like(b)

    def one():
        if mode == "fwd":
            op.fwd(x, out=y)
        elif mode == "dgrad":
            op.dgrad(dy, x)
        else:
            op.wgrad(dy, x, dw, db, beta=0.0)

    fn = getattr(lib, switch)
    res = {0: [], 1: []}
    ref = {}
    for r in range(rounds + 1):
        for arm in ((0, 1) if r % 2 == 0 else (1, 0)):
            old = fn(vals[arm])
            one()
            torch.cuda.synchronize()
            if r == 0:
                ref[arm] = (dw.clone(), db.clone()) if mode == "wgrad" else None
                fn(old)
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                one()
            e1.record()
            torch.cuda.synchronize()
            fn(old)
            res[arm].append(e0.elapsed_time(e1) / reps)
        if r:
            print(f"round {r}: {vals[0]}: {res[0][-1]:.4f} ms  {vals[1]}: {res[1][-1]:.4f} ms", flush=True)
    same = None
    if mode == "wgrad":
        same = all(torch.equal(a, c) for a, c in zip(ref[0], ref[1]))
    print(f"{layer}.{mode} B={N} {switch}: {vals[0]} median {statistics.median(res[0]):.4f} ms, {vals[1]} median "
          f"{statistics.median(res[1]):.4f} ms; results bitwise equal: {same}")


if __name__ == "__main__":
    main()
