"""Time small linears on the conv path (ConvOp over [rows][features] activations).

usage: python tools/mb_linear.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))

from expertsim import hip  # noqa: E402
from expertsim.layers import Act, ConvOp  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    hip.lib()
    for (M, K, N, dt) in [(512, 19, 256, torch.bfloat16), (512, 9, 128, torch.float32), (512, 256, 21632, torch.bfloat16),
                          (512, 128, 128, torch.float32), (512, 1305, 128, torch.float32)]:
        w = torch.nn.Parameter(torch.randn(N, K, device="cuda") * 0.1)
        b = torch.nn.Parameter(torch.randn(N, device="cuda"))
        op = ConvOp(w, b)
        x = Act.rows(M, K, dt, "cuda")
        x.t.normal_()
        y = op.fwd(x)
        dy = y.like_nhwc()
        dy.t.normal_()
        tf = timed(lambda: op.fwd(x))
        td = timed(lambda: op.dgrad(dy, x))
        tw = timed(lambda: op.wgrad(dy, x, None, None))
        print(f"M={M} K={K} N={N} {dt}: fwd {tf:.1f} us  dgrad {td:.1f} us  wgrad {tw:.1f} us", flush=True)


if __name__ == "__main__":
    main()
