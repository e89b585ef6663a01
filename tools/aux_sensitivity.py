"""Sensitivity of the reference's step-0 aux-regressor gradients to fp32-level input perturbations.

The aux regressor of the G step reads the generator's output (oracle moe restatement, reference
moe.py:529-571).  The HIP generator matches the reference's images to ~1e-6 relative, not bitwise,
so A sees a slightly different input; MaxPool argmax near-ties and LeakyReLU kinks can then route
gradients differently.  This runs the oracle (bit-exact to the goldens) with A's input multiplied
by (1 + eps * N(0, 1)) and reports the norm-relative gradient error of every A parameter against
the goldens (tests/test_grads_gpu.py's measure), over several perturbation seeds.

usage: python tools/aux_sensitivity.py <case> [eps=1e-6] [trials=8]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_utils import Golden, checksum  # noqa: E402
from oracle import expertsim_oracle as O  # noqa: E402


def a_grad_errors(case, eps, seed):
    torch.set_num_threads(1)
    g = Golden(case)
    m = O.OracleMoE(g.arch, g.E, g.oracle_cfg(O.DEFAULT_CFG), seed=g.seed)
    orig = O.aux_forward
    gen = torch.Generator().manual_seed(seed)

    def perturbed(arch, P, x, drop=None, training=True):
        if eps > 0:
            x = x * (1 + eps * torch.randn(x.shape, generator=gen, dtype=x.dtype))
        return orig(arch, P, x, drop, training)

    O.aux_forward = perturbed
    try:
        inp, nz = g.inputs(0), g.noise(0)
        _, tr = m.train_step(
            g.epoch, torch.from_numpy(inp["cond"]), torch.from_numpy(inp["real_images"]).unsqueeze(1),
            torch.from_numpy(inp["true_positions"]), torch.from_numpy(inp["std"]),
            torch.from_numpy(inp["intensity"]), lambda e, w, shape: torch.from_numpy(nz[(e, w)]),
            torch.from_numpy(g.gumbel(0)))
    finally:
        O.aux_forward = orig
    out = {}
    for key in [k for k in tr if k.startswith("optA") and k.endswith("/grad")]:
        lab = key.split("/")[0]
        for n, t in tr[key].items():
            ref = g[f"s0/{lab}/grad/{n}"]
            if ref[2] == 0.0 or n.endswith(".bias") and ("conv" in n or "downsample" in n):   # noise-only set
                continue
            c = checksum(t.double().numpy())
            samp = float(np.linalg.norm(c[3:] - ref[3:]) / max(np.linalg.norm(ref[3:]), 1e-30))
            l2 = float(abs(c[2] - ref[2]) / ref[2])
            out[f"{lab}/{n}"] = max(samp, l2)
    return out


if __name__ == "__main__":
    case = sys.argv[1]
    eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
    trials = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    worst = []
    for t in range(trials):
        errs = a_grad_errors(case, eps, 1000 + t)
        n, e = max(errs.items(), key=lambda kv: kv[1])
        worst.append(e)
        print(f"{case} eps={eps:g} trial {t}: worst {n} {e:.3e}", flush=True)
    print(f"{case} eps={eps:g}: worst-rel over {trials} trials: median {np.median(worst):.3e} "
          f"max {max(worst):.3e}")
