"""Time / profile graph replays of one train-step configuration (for rocprofv3 runs and A/B checks).

usage: python tools/prof_step.py --experts 4 --batch 512 [--serial] [--steps 10] [--precision fp32]
--serial: a multi-expert step's experts run one after another inside the graph (no stream fork),
so that kernel durations in a profile are not stretched by concurrent experts."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
sys.path.insert(0, ROOT)
import bench
from expertsim.graph import StepGraph
from expertsim.utils.synthetic import make_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--experts", type=int, default=4)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--arch", default="neutron")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--sync", action="store_true", help="synchronise after every replay (PMC passes: one "
                    "replay's packets in flight)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    moe, (og, od, oa, orr), cfg = bench.build(a.arch, a.experts, a.precision, 1234, dev)
    moe.expert_graphs_concurrent = not a.serial
    b = make_batch(a.batch, a.arch, seed=1000)
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    args = (0, t["cond"], t["real_images"].unsqueeze(1).contiguous(), t["true_positions"], t["std"], t["intensity"],
            oa, og, od, orr, None, dev)
    for _ in range(2):
        moe.train_step(*args)
    sg = StepGraph(moe, args, warmup=1)
    sg.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        sg.replay()
        if a.sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"E={a.experts} B={a.batch} {a.precision} serial={a.serial}: {dt * 1e3:.2f} ms/step")


if __name__ == "__main__":
    main()
