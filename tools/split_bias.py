"""Signed error of the fp32 ring convs (exact fp32 MFMA vs split-fp32) against fp64: a rounding
bias toward zero shows as a negative mean of (y - y64) * sign(y64) / mean|y64|.
usage: python tools/split_bias.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
from test_f32_ring_gpu import _ref, _run  # noqa: E402
from expertsim import layers  # noqa: E402

layers.set_deterministic(True)
for case in [(67, 256, 24, 24, 128, 3, 1, 0, 2), (8, 128, 13, 13, 256, 3, 1, 0, 2), (70, 128, 46, 46, 64, 2, 1, 0, None)]:
    x, w, b, gy, *ref = _ref(case, 0)
    for split in (False, True):
        layers.set_f32_split(split)
        out = _run(case, x, w, b, gy)[1:]
        s = []
        for name, o, r in zip(("fwd", "dgrad", "wgrad", "bias"), out, ref):
            o, r = o.double(), r.double()
            d = o - r
            s.append(f"{name}: bias {((d * r.sign()).mean() / r.abs().mean()).item():+.2e} "
                     f"rms {(d.pow(2).mean().sqrt() / r.abs().mean()).item():.2e} "
                     f"sum {((o.sum() - r.sum()) / r.abs().sum()).item():+.2e}")
        print(case[:5], "split" if split else "exact", " | ".join(s), flush=True)
