"""Debug: multi-expert dynamic-rows steps -- eager vs per-expert graphs vs whole-step graph (E = 3)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "generative-dnn-for-physics-simulations-cern_amd")
sys.path.insert(0, ".")
import bench
from expertsim.utils.synthetic import make_batch


def run(mode, E=3, B=96, steps=3):
    dev = torch.device("cuda", 0)
    moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, dev)
    moe.expert_graphs = mode == "egraph"
    out = []
    for s in range(steps):
        b = make_batch(B, "neutron", seed=70 + s)
        t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
        m = moe.train_step(0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"],
                           t["intensity"], oa, og, od, orr, None, dev)
        torch.cuda.synchronize()
        out.append({k: float(v) for k, v in m.items()})
    return out


a = run("eager")
b = run("egraph")
for s in range(len(a)):
    bad = {k: (a[s][k], b[s][k]) for k in a[s] if abs(a[s][k] - b[s][k]) > 1e-5 * max(1e-3, abs(a[s][k]))}
    print("step", s, "eager vs egraph diffs:", bad)
print("eager step1:", a[1])
