"""One-off CPU baseline table on this host (BASELINE.md "CPU-baseline plan"): the oracle (torch CPU fp32
restatement of MoEWrapper.train_step, pinned bit-exactly to the reference's goldens) at B = 64 / 512 /
1024 (E = 1) and E = 4, B = 2048, on every CPU the affinity / cgroup quota allows.  One untimed warm-up
step per configuration, then the median of the timed steps.  Prints one line per step (progress) and
the table as markdown at the end.

usage: python tools/cpu_table.py [out.md]
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from oracle import expertsim_oracle as O  # noqa: E402
from expertsim.utils.synthetic import make_batch  # noqa: E402

CONFIGS = [(1, 64, 20), (1, 512, 3), (1, 1024, 2), (4, 2048, 2)]    # (E, B, timed steps)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    threads, aff, quota = bench.cpu_threads()
    torch.set_num_threads(threads)
    rows = []
    for E, B, steps in CONFIGS:
        cfg = dict(O.DEFAULT_CFG)
        if E > 1:
            cfg["diff_strength"] = 1e-6      # default.yaml '1-6' 
        m = O.OracleMoE("neutron", E, cfg, seed=1234)
        g = torch.Generator().manual_seed(0)
        b = make_batch(B, "neutron", seed=0)
        t = {k: torch.from_numpy(v) for k, v in b.items()}
        times = []
        for i in range(steps + 1):
            t0 = time.perf_counter()
            m.train_step(0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"], t["intensity"],
                         lambda e, w, shape: torch.randn(shape, generator=g),
                         torch.empty(B, E).exponential_(generator=g))
            dt = time.perf_counter() - t0
            print(f"E={E} B={B} step {i}{' (warm-up)' if i == 0 else ''}: {dt:.2f} s = {B / dt:.2f} images/s",
                  flush=True)
            if i > 0:
                times.append(dt)
        med = statistics.median(times)
        rows.append((E, B, len(times), med, B / med))
    lines = [f"# CPU baseline table: the oracle on {bench.cpu_model()}, {threads} threads "
             f"(affinity {aff} CPUs, cgroup quota {quota if quota else 'none'})", "",
             "tools/cpu_table.py: neutron 44x44, synthetic batches, one untimed warm-up step per row, median of the "
             "timed steps.", "",
             "| E | B | timed steps | s / step (median) | images/s |", "|---|---|---|---|---|"]
    lines += [f"| {E} | {B} | {n} | {s:.2f} | {r:.2f} |" for E, B, n, s, r in rows]
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        open(out, "w").write(text)


if __name__ == "__main__":
    main()
