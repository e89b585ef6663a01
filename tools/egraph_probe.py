"""Per-step timing of a multi-expert step with per-expert graphs (captures vs replays).

usage: python tools/egraph_probe.py <experts> <batch> [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from expertsim.utils.synthetic import make_batch  # noqa: E402

E, B = int(sys.argv[1]), int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 30
dev = torch.device("cuda", 0)
moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "bf16", 1234, dev)
b = make_batch(B, "neutron", seed=1)
t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
args = (0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"], t["intensity"], oa, og, od, orr,
        None, dev)
for s in range(K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = moe.train_step(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    eg = moe._egraphs
    cnt = [int(m[f"n_choosen_experts_mean_epoch_{i}"]) for i in range(E)]
    print(f"step {s}: host {1e3 * (t1 - t0):7.2f} ms  wall {1e3 * (t2 - t0):7.2f} ms  counts {cnt}  "
          f"captures {eg.captures if eg else 0} replays {eg.replays if eg else 0}", flush=True)
