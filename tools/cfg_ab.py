"""Alternating A/B of a YAML config switch on captured whole-step graphs, one process, one box.

usage: python tools/cfg_ab.py --key train.dropout_ahead --vals false,true [--batch 1024]
       [--experts 1] [--precision fp32] [--rounds 3] [--reps 30]
One model per value (same seed), each captured as a StepGraph; the rounds alternate the values and
print ms/step per value per round, so box drift hits every value alike.  A key starting with "es_"
is a library switch (es_conv_set_*): set to the value while that model's steps are captured (the
dispatch is baked into the graph)."""
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


def parse(v):
    low = v.lower()
    if low in ("true", "false"):
        return low == "true"
    try:
        return int(v)
    except ValueError:
        return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True)
    ap.add_argument("--vals", required=True)
    ap.add_argument("--experts", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--arch", default="neutron")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    b = make_batch(a.batch, a.arch, seed=1000)
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()
    runs = []
    for v in [parse(x) for x in a.vals.split(",")]:
        moe, (og, od, oa, orr), cfg = bench.build(a.arch, a.experts, a.precision, 1234, dev)
        if a.key.startswith("es_"):
            from expertsim import hip
            getattr(hip.lib(), a.key)(int(v))
        else:
            node = cfg
            *path, leaf = a.key.split(".")
            for p in path:
                node = getattr(node, p)
            setattr(node, leaf, v)
        args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, dev)
        for _ in range(2):
            moe.train_step(*args)
        sg = StepGraph(moe, args, warmup=1)
        sg.replay()
        torch.cuda.synchronize()
        runs.append((v, sg, moe))
        print(f"captured {a.key}={v}", flush=True)
    for r in range(a.rounds):
        line = []
        for v, sg, _ in runs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                sg.replay()
            torch.cuda.synchronize()
            line.append(f"{v}: {(time.perf_counter() - t0) / a.reps * 1e3:.3f}")
        print(f"round {r} ({a.key}, E={a.experts} B={a.batch} {a.precision}) ms/step  " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
