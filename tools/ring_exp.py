"""Time the generator's big sub-pixel convs (conv_layers.0 / .5 fwd, .5 dgrad) at B = 1024 in
whatever library ES_LIB names (diagnostic ES_RING_EXP builds: tools/ring_exp_build.sh).
usage: ES_LIB=tools/_exp/expN/libexpertsim_hip.so python tools/ring_exp.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "generative-dnn-for-physics-simulations-cern_amd"))
from expertsim import hip  # noqa: E402
from expertsim.layers import Act, ConvOp, Upsample  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = "cuda"
torch.manual_seed(0)


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = []
for name, Cin, H, Cout in (("c0", 128, 13, 256), ("c5", 256, 24, 128)):
    w = torch.randn(Cout, Cin, 3, 3, device=dev) / np.sqrt(Cin * 9)
    b = torch.randn(Cout, device=dev)
    op = ConvOp(torch.nn.Parameter(w), torch.nn.Parameter(b), upsample=Upsample((H, H), scale=(2.0, 2.0)))
    x = Act.nhwc(B, Cin, H, H, torch.bfloat16, dev)
    x.t.normal_()
    y = op.fwd(x, out_dtype=torch.bfloat16, bn_stats=True)
    gy = y.like_nhwc(torch.bfloat16)
    gy.t.normal_()
    tf = timeit(lambda: op.fwd(x, out=y, bn_stats=True))
    flop = 2.0 * B * y.dims[2] * y.dims[3] * Cout * Cin * 9
    line = f"{name} fwd {tf:.1f} us ({flop / tf / 1e9:.0f} TFLOP/s alg)"
    if name == "c5":
        dx = x.like_nhwc(torch.bfloat16)
        td = timeit(lambda: op.dgrad(gy, x, dx=dx))
        line += f"  dgrad {td:.1f} us ({flop / td / 1e9:.0f} TFLOP/s alg)"
    res.append(line)
print(os.environ.get("ES_LIB", "default"), " | ".join(res), flush=True)
