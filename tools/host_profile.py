"""Host-side cost of the eager train step: cProfile of K eager steps (GPU work overlaps; the
host issue time is what bounds small / multi-expert steps).

usage: python tools/host_profile.py <experts> <batch> [steps]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from expertsim.utils.synthetic import make_batch  # noqa: E402

E, B = int(sys.argv[1]), int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "bf16", 1234, dev)
b = make_batch(B, "neutron", seed=1)
t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
args = (0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"], t["intensity"], oa, og, od, orr,
        None, dev)
for _ in range(3):
    moe.train_step(*args)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    moe.train_step(*args)
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"E={E} B={B}: host issue {t_issue / K * 1e3:.2f} ms/step, wall {t_all / K * 1e3:.2f} ms/step "
      f"({B * K / t_all:.0f} img/s)")
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    moe.train_step(*args)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(20)
st.sort_stats("cumulative").print_stats(40)
