"""Debug: step-1 generator outputs of expert 0, single device vs the two SyncBN ranks."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, "generative-dnn-for-physics-simulations-cern_amd")
sys.path.insert(0, ".")
import test_ddp_gpu as T
from expertsim import hip

SAVE = {}


def patch():
    from expertsim.models.neutron.generator import GeneratorNeutron as G
    orig = G.fwd

    def fwd(self, noise, cond, *a, **k):
        out = orig(self, noise, cond, *a, **k)
        n = hip.live_count()
        if getattr(self, "_probe_prefix", "") == "G0":
            SAVE.setdefault("calls", []).append((n, out[0].torch_nchw()[:n].detach().cpu().numpy().copy(),
                                                 noise[:n].detach().cpu().numpy().copy(),
                                                 cond[:n].detach().cpu().numpy().copy()))
        return out
    G.fwd = fwd
    from expertsim.models.moe import MoEWrapper
    MoEWrapper._expert_graphs_on = lambda self, E: False


def worker(rank, world, port, q, E, sync):
    patch()
    T._worker(rank, world, port, q, E, sync)
    np.save(f"gpurun_out/dbg_r{rank}.npy", np.array(SAVE["calls"], dtype=object), allow_pickle=True)


if __name__ == "__main__":
    import torch.multiprocessing as mp
    patch()
    single, lr = T._run(3, T.B_GLOBAL)
    S = SAVE["calls"]
    port = T._free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q, 3, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    R = [np.load(f"gpurun_out/dbg_r{r}.npy", allow_pickle=True) for r in range(2)]
    for c in range(len(S)):
        n, img, nz, cd = S[c]
        n0, img0, nz0, cd0 = R[0][c]
        n1, img1, nz1, cd1 = R[1][c]
        print(f"call {c}: single n={n} ranks n={n0},{n1}")
        if n0 + n1 != n:
            continue
        for nm, a, b in (("cond", cd, np.concatenate([cd0, cd1])), ("noise", nz, np.concatenate([nz0, nz1])),
                         ("img", img, np.concatenate([img0, img1]))):
            d0 = np.abs(a[:n0] - b[:n0]).max() if n0 else 0
            d1 = np.abs(a[n0:] - b[n0:]).max() if n1 else 0
            print(f"   {nm}: rank0 rows max diff {d0:.3e}, rank1 rows max diff {d1:.3e}")
