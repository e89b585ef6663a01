"""Sensitivity of the reference's parameter gradients to fp32-level perturbations.

Runs the oracle (bit-exact to the goldens) with every linear / conv output of the step multiplied by
(1 + eps * N(0, 1)) -- the size of the HIP path's own deviation from the reference (~1e-6 relative on
every module output) -- and reports, per optimizer and parameter, the gradient error against the
goldens in tests/test_grads_gpu.py's measure (norm-relative over the checksum samples / L2), worst over
the trials.  A HIP gradient error within this spread is the reference's own sensitivity, not a bug.
Step s > 0: the oracle runs steps 0..s with the perturbation in every step (the HIP path deviates in
every step) and the errors are those of step s.  The result is written to
tests/golden/sensitivity_<case>_s<step>.json (a fixture of the gradient tests).

usage: python tools/grad_sensitivity.py <case> [eps=1e-6] [trials=3] [step=0]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_utils import Golden, checksum  # noqa: E402
from test_grads_gpu import NOISE_ONLY  # noqa: E402
from oracle import expertsim_oracle as O  # noqa: E402


def grad_errors(case, eps, seed, step):
    g = Golden(case)
    m = O.OracleMoE(g.arch, g.E, g.oracle_cfg(O.DEFAULT_CFG), seed=g.seed)
    gen = torch.Generator().manual_seed(seed)
    lin, conv = O._lin, O._conv

    def noisy(t):
        return t * (1 + eps * torch.randn(t.shape, generator=gen, dtype=t.dtype)) if eps > 0 else t

    O._lin = lambda x, P, name: noisy(lin(x, P, name))
    O._conv = lambda x, P, name, stride=1, padding=0: noisy(conv(x, P, name, stride, padding))
    try:
        for s in range(step + 1):
            inp, nz = g.inputs(s), g.noise(s)
            _, tr = m.train_step(
                g.epoch, torch.from_numpy(inp["cond"]), torch.from_numpy(inp["real_images"]).unsqueeze(1),
                torch.from_numpy(inp["true_positions"]), torch.from_numpy(inp["std"]),
                torch.from_numpy(inp["intensity"]), lambda e, w, shape, nz=nz: torch.from_numpy(nz[(e, w)]),
                torch.from_numpy(g.gumbel(s)))
    finally:
        O._lin, O._conv = lin, conv
    out = {}
    for key in [k for k in tr if k.startswith("opt") and k.endswith("/grad")]:
        lab = key.split("/")[0]
        for n, t in tr[key].items():
            gk = f"s{step}/{lab}/grad/{n}"
            if not g.has(gk):
                continue
            ref = g[gk]
            if ref[2] == 0.0 or n in NOISE_ONLY.get(g.arch, {}).get(lab[3], set()):
                continue       # (analytically zero: compared absolutely by the tests)
            c = checksum(t.double().numpy())
            samp = float(np.linalg.norm(c[3:] - ref[3:]) / max(np.linalg.norm(ref[3:]), 1e-30))
            l2 = float(abs(c[2] - ref[2]) / ref[2])
            out[f"{lab}/{n}"] = max(samp, l2)
    return out


def main():
    case = sys.argv[1]
    eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
    trials = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    step = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    worst = {}
    for s in range(trials):
        e = grad_errors(case, eps, 100 + s, step)
        for k, v in e.items():
            worst[k] = max(worst.get(k, 0.0), v)
        top = sorted(e.items(), key=lambda kv: -kv[1])[:6]
        print(f"trial {s}:", [(k, f"{v:.2e}") for k, v in top], flush=True)
    print("worst over trials:", [(k, f"{v:.2e}") for k, v in sorted(worst.items(), key=lambda kv: -kv[1])[:12]])
    out = os.path.join(ROOT, "tests", "golden", f"sensitivity_{case}_s{step}.json")
    json.dump({"case": case, "step": step, "eps": eps, "trials": trials,
               "generator": "tools/grad_sensitivity.py", "worst": worst}, open(out, "w"), indent=1, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    main()
