"""Run ONE conv op of the neutron generator a few times (for rocprofv3 --pmc passes).

usage: python tools/mb_one.py <c0|c5|c9|c13|p1|p5> <fwd|dgrad|wgrad> [ring 1|0] [reps]
(ES_MB_BATCH=<images> overrides the batch of 512; ES_MB_DTYPE=fp32 runs the parity mode's fp32 ring
kernels with the deterministic weight gradient, ES_MB_SPLIT=1 with split-fp32 arithmetic)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))

from expertsim import hip  # noqa: E402
from expertsim.layers import Act, ConvOp, Upsample  # noqa: E402

SHAPES = {"c0": (512, 128, 13, 13, 256, 3, 1, 0, (2, 2)), "c5": (512, 256, 24, 24, 128, 3, 1, 0, (2, 2)),
          "c9": (512, 128, 46, 46, 64, 2, 1, 0, None), "c13": (512, 64, 45, 45, 1, 2, 1, 0, None),
          # proton (proton/generator.py:26-38): conv_layers.1 on the x2 upsample, conv_layers.5 on the
          # 35x19 -> 56x30 resize
          "p1": (512, 512, 18, 10, 256, 4, 1, 1, (2, 2)), "p5": (512, 256, 35, 19, 128, 4, 1, 1, "56x30")}


def main():
    layer, mode = sys.argv[1], sys.argv[2]
    ring = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    N, Cin, H, W, Cout, k, st, pad, up = SHAPES[layer]
    N = int(os.environ.get("ES_MB_BATCH", N))
    dev = "cuda"
    hip.lib().es_conv_set_ring(ring)
    w = torch.nn.Parameter(torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5)
    b = torch.nn.Parameter(torch.randn(Cout, device=dev))
    if isinstance(up, str):
        ups = Upsample((H, W), out_hw=tuple(int(v) for v in up.split("x")))
    else:
        ups = Upsample((H, W), scale=up) if up else None
    op = ConvOp(w, b, stride=st, pad=pad, upsample=ups)
    f32 = os.environ.get("ES_MB_DTYPE", "bf16") == "fp32"
    dt = torch.float32 if f32 else torch.bfloat16
    if f32:
        from expertsim import layers
        layers.set_deterministic(True)
        layers.set_f32_split(os.environ.get("ES_MB_SPLIT", "0") == "1")
    x = Act.nhwc(N, Cin, H, W, dt, dev)
    x.t.normal_()
    y = op.fwd(x, out_dtype=dt)
    dy = y.like_nhwc(dt)
    dy.t.normal_()
    dw = torch.zeros_like(w)
    torch.cuda.synchronize()

    def run():
        if mode == "fwd":
            op.fwd(x, out_dtype=dt)
        elif mode == "dgrad":
            op.dgrad(dy, x, dx_dtype=dt)
        else:
            op.wgrad(dy, x, dw, None, beta=0.0)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    flops = 2.0 * N * y.dims[2] * y.dims[3] * Cout * Cin * k * k
    print(f"{layer} {mode} ring={ring} dbg={os.environ.get('ES_RING_DBG', '0')}: {us:.1f} us "
          f"{flops / us / 1e6:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
