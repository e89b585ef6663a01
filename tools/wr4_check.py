"""Deterministic weight gradients of the bench's conv / linear shapes (fp32 split-fp32 mode), saved for a
bitwise comparison between library builds or switches (e.g. ES_WGRAD_REDUCE4=0 / 1).

usage: python tools/wr4_check.py <out.npz>      |   python tools/wr4_check.py --compare a.npz b.npz"""
import os
import sys

import numpy as np

if len(sys.argv) == 4 and sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print("bitwise equal" if not bad else f"DIFFERENT: {bad}", f"({len(a.files)} gradients)")
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
from expertsim import layers  # noqa: E402
from expertsim.layers import Act, ConvOp, Upsample  # noqa: E402

CASES = {"c0": (256, 128, 13, 13, 256, 3, 0, (2, 2)), "c5": (256, 256, 24, 24, 128, 3, 0, (2, 2)),
         "c9": (256, 128, 46, 46, 64, 2, 0, None), "p1": (128, 512, 18, 10, 256, 4, 1, (2, 2)),
         "d2": (128, 32, 21, 21, 16, 3, 0, None), "a1": (128, 1, 44, 44, 32, 3, 0, None)}


def main():
    layers.set_deterministic(True)
    layers.set_f32_split(True)
    dev = "cuda"
    out = {}
    for name, (N, Cin, H, W, Cout, k, pad, up) in CASES.items():
        torch.manual_seed(3)
        w = torch.nn.Parameter(torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5)
        b = torch.nn.Parameter(torch.zeros(Cout, device=dev))
        op = ConvOp(w, b, pad=pad, upsample=Upsample((H, W), scale=up) if up else None)
        x = Act.nhwc(N, Cin, H, W, torch.float32, dev)
        x.t.normal_()
        y = op.fwd(x)
        dy = y.like_nhwc()
        dy.t.normal_()
        dw = torch.zeros_like(w)
        db = torch.zeros_like(b)
        op.wgrad(dy, x, dw, db, beta=0.0)
        torch.cuda.synchronize()
        out[name] = dw.cpu().numpy()
        out[name + ".bias"] = db.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1], flush=True)


if __name__ == "__main__":
    main()
