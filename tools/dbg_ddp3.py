"""Debug: step-0 Adam input gradients (flat_grads x grad_scale) single device vs SyncBN rank 0, per parameter."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, "generative-dnn-for-physics-simulations-cern_amd")
sys.path.insert(0, ".")
import test_ddp_gpu as T

G = {}


def patch():
    from expertsim.optim import FusedAdam
    from expertsim.models.moe import MoEWrapper
    MoEWrapper._expert_graphs_on = lambda self, E: False
    orig = FusedAdam.step

    def step(self, closure=None, grad_scale=None):
        gs = grad_scale if grad_scale is not None else getattr(self.module, "_grad_scale", 1.0)
        key = getattr(self.module, "_probe_prefix", None) or type(self.module).__name__
        k = (key, G.setdefault(("n", key), 0))
        G[("n", key)] += 1
        g = (self.module.flat_grads.detach().double() * gs).cpu().numpy()
        names = [(n, p.numel()) for n, p in self.module.named_parameters()]
        G[k] = (g, names)
        return orig(self, closure, grad_scale)
    FusedAdam.step = step


def worker(rank, world, port, q, E, sync):
    patch()
    T._worker(rank, world, port, q, E, sync)
    out = {f"{k[0]}|{k[1]}": v[0] for k, v in G.items() if k[0] != "n" and k[1] == 0}
    np.savez(f"gpurun_out/dbg_g{rank}.npz", **out)
    names = {f"{k[0]}|{k[1]}": v[1] for k, v in G.items() if k[0] != "n"}
    import json
    json.dump(names, open(f"gpurun_out/dbg_g{rank}.json", "w"))


if __name__ == "__main__":
    import json
    import torch.multiprocessing as mp
    patch()
    T._run(3, T.B_GLOBAL)
    S = {f"{k[0]}|{k[1]}": v for k, v in G.items() if k[0] != "n"}
    port = T._free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q, 3, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    R = np.load("gpurun_out/dbg_g0.npz")
    for key in sorted(S):
        if not key.endswith("|0"):
            continue           # step 0 only (first step() call of each optimizer)
        g, names = S[key]
        d = R[key]
        o = 0
        rows = []
        for n, cnt in names:
            a, b = g[o:o + cnt], d[o:o + cnt]
            rel = float(np.abs(a - b).max() / max(np.abs(a).max(), 1e-30))
            rows.append((rel, n))
            o += cnt
        rows.sort(reverse=True)
        nb = [r for r in rows if not r[1].endswith(".bias")]
        print(key, "worst grads rel (non-bias):", [(f"{r:.2e}", n) for r, n in nb[:4]])
    import os
    for r in range(2):
        os.remove(f"gpurun_out/dbg_g{r}.npz")
