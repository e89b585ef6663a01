"""Per-conv-op times of eager train steps (every labelled ConvOp fwd / dgrad / wgrad, HIP events on the
launch stream) with the pipe each op ran on (es_conv_exec_flops tally: bf16 pipe incl. split-fp32,
exact fp32 MFMA, VALU thin kernels).  Finds the layers still on a slow path.

usage: python tools/op_times.py [--experts 1] [--batch 1024] [--precision fp32] [--steps 3]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
sys.path.insert(0, ROOT)
import bench
from expertsim import layers
from expertsim.utils.synthetic import make_batch


class AllOps(layers.KernelProbe):
    def __init__(self):
        super().__init__([])

    def wants(self, label):
        if label not in self.events:
            self.events[label], self.launches[label], self.exec[label] = [], [], []
        return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--experts", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--arch", default="neutron")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    moe, (og, od, oa, orr), cfg = bench.build(a.arch, a.experts, a.precision, 1234, dev)
    moe.expert_graphs = False
    b = make_batch(a.batch, a.arch, seed=1000)
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    args = (0, t["cond"], t["real_images"].unsqueeze(1).contiguous(), t["true_positions"], t["std"], t["intensity"],
            oa, og, od, orr, None, dev)
    for _ in range(2):
        moe.train_step(*args)
    torch.cuda.synchronize()
    probe = AllOps()
    layers.set_probe(probe)
    for _ in range(a.steps):
        moe.train_step(*args)
    torch.cuda.synchronize()
    layers.set_probe(None)
    s = probe.summary()
    tot = sum(v["total_ms"] for v in s.values()) / a.steps
    print(f"E={a.experts} B={a.batch} {a.precision}: labelled conv ops {tot:.3f} ms per step")
    print("| ms/step | calls/step | avg ms | launches | pipe (exec GFLOP bf16 / fp32 / valu) | op |")
    print("|---|---|---|---|---|---|")
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["total_ms"]):
        ex = v.get("exec_flops_per_op", [0, 0, 0])
        pipe = ["bf16", "fp32", "valu"][max(range(3), key=lambda i: ex[i])] if any(ex) else "-"
        print(f"| {v['total_ms'] / a.steps:.3f} | {v['count'] / a.steps:.1f} | {v['avg_ms']:.3f} | "
              f"{v.get('kernel_launches_per_op', '-')} | {pipe} ({ex[0] / 1e9:.1f} / {ex[1] / 1e9:.1f} / "
              f"{ex[2] / 1e9:.1f}) | {k} |")


if __name__ == "__main__":
    main()
