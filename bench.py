#!/usr/bin/env python
"""Benchmark of the expertsim GAN training step on MI355X (BASELINE.json metric, configs[1]).

Workload: neutron 44x44 ZDC MoE-GAN, 1 expert, batch 512 per GPU, bf16 GEMM operands (fp32
accumulation / statistics / optimizer), synthetic data resident in HBM.  One "step" =
``MoEWrapper.train_step`` (router, G fwd x2, D fwd x4 + bwd x4, aux regressor fwd/bwd, losses,
four fused Adam updates; with N > 1 also the RCCL gradient all-reduces).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line (rank 0) with the metric, a live-measured roofline of the dominant kernel
(HIP events around its launches inside the timed region) and the CPU baseline (the oracle, a CPU
fp32 restatement of the same step, timed on this host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd")
sys.path.insert(0, PKG_DIR)
sys.path.insert(0, ROOT)

# algorithmic FLOPs per image per train_step (torch FlopCounterMode on the
# reference): neutron 10.573 GFLOP, proton 28.566 GFLOP
STEP_FLOP_PER_IMAGE = {"neutron": 10.573e9, "proton": 28.566e9}
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
# HBM traffic of the roofline kernel from committed PMC passes (tools/gpu_traffic.sh ->
# tools/traffic_json.py): FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch of G0.c5.fwd
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r01_s2h_c5_fwd_traffic.json")


def conv_flops_per_image(arch):
    """Forward FLOPs of the dominant generator conv per image (= the algorithmic count charged to
    each of its fwd / dgrad / wgrad launches, as torch's flop counter does)."""
    if arch == "neutron":   # conv_layers.5: 256x48x48 -> 128x46x46, k3
        return 2 * 46 * 46 * 128 * (256 * 9)
    return 2 * 55 * 29 * 128 * (256 * 16)   # proton conv_layers.5: 256x56x30 -> 128x55x29, k4 p1


def build(arch, E, precision, seed, device):
    import torch
    from expertsim.config import inject_shared, load_config
    from expertsim.models import build_model
    from expertsim.models.moe import MoEWrapper
    from expertsim.train.training_setup import setup_optimizers
    cfg = inject_shared(load_config(overrides=[f"model.architecture={arch}", f"model.n_experts={E}",
                                               f"train.precision={precision}", f"train.rng_seed={seed}"]))
    torch.manual_seed(seed)
    parts = [build_model(f"{arch}.{k}", getattr(cfg.model, k), device) for k in ("generator", "discriminator", "aux_reg")]
    router = build_model("router_v1", cfg.model.router, device)
    moe = MoEWrapper(*parts, router, E, cfg, image_shape=tuple(parts[0].image_shape)).to(device)
    return moe, setup_optimizers(moe, cfg), cfg


def cpu_baseline(arch, batch=64, steps=2):
    import torch
    from oracle import expertsim_oracle as O
    from expertsim.utils.synthetic import make_batch
    threads = torch.get_num_threads()
    m = O.OracleMoE(arch, 1, dict(O.DEFAULT_CFG), seed=1234)
    g = torch.Generator().manual_seed(0)
    b = make_batch(batch, arch, seed=0)
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    noise_fn = lambda e, w, shape: torch.randn(shape, generator=g)
    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        m.train_step(0, t["cond"], t["real_images"].unsqueeze(1), t["true_positions"], t["std"], t["intensity"],
                     noise_fn, torch.empty(batch, 1).exponential_(generator=g))
        times.append(time.perf_counter() - t0)
    dt = sum(times[1:]) / steps
    return {"value": round(batch / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{arch} E=1 B={batch}: {steps} timed train steps after 1 warm-up, "
                      f"oracle/expertsim_oracle.py (torch CPU fp32, {threads} threads)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="images per GPU")
    ap.add_argument("--arch", default="neutron")
    ap.add_argument("--experts", type=int, default=1)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-kernel HIP-event probe")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the step as a captured HIP graph (auto: single process, 1 expert)")
    ap.add_argument("--ddp", action="store_true",
                    help="run the data-parallel code path even on one process (1-rank RCCL group)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ddp = world > 1 or args.ddp
    if ddp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from expertsim import layers
    from expertsim.train.ddp import DataParallel
    from expertsim.utils.synthetic import make_batch
    moe, (og, od, oa, orr), cfg = build(args.arch, args.experts, args.precision, 1234, dev)
    if ddp:
        moe.ddp = DataParallel()
        moe.rank = rank
    b = make_batch(args.batch, args.arch, seed=1000 + rank)
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()

    step_args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, dev)

    def eager_step():
        moe.train_step(*step_args)

    # DDP stays eager: its eager step issues as fast as the graph replays (1-rank DDP 41.9k vs graph
    # 42.0k img/s on one MI355X), and capturing around the RCCL calls is not needed for that
    use_graph = args.graph == "on" or (args.graph == "auto" and not ddp and args.experts == 1)
    for _ in range(args.warmup):
        eager_step()
    step = eager_step
    if use_graph:
        from expertsim.graph import StepGraph
        sg = StepGraph(moe, step_args, warmup=1)
        step = sg.replay
    probe = None
    if not args.no_probe and not use_graph:
        probe = layers.KernelProbe(["G0.c5.fwd", "G0.c5.dgrad", "G0.c5.wgrad"])
        layers.set_probe(probe)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    layers.set_probe(None)
    if use_graph:
        sg.sync_host_state([og[0], od[0], oa[0], orr])
        if not args.no_probe:
            # a graph replay cannot be split per kernel: the per-launch HIP events are taken on
            # eager steps of the same model and batch right after the timed region
            probe = layers.KernelProbe(["G0.c5.fwd", "G0.c5.dgrad", "G0.c5.wgrad"])
            layers.set_probe(probe)
            for _ in range(min(args.steps, 5)):
                eager_step()
            torch.cuda.synchronize()
            layers.set_probe(None)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    images = args.batch * world * args.steps
    value = images / dt

    if rank == 0:
        roof = None
        if probe is not None:
            stats = probe.summary()
            flops = conv_flops_per_image(args.arch) * args.batch
            dom = max(stats, key=lambda k: stats[k]["total_ms"])
            avg_ms = stats[dom]["avg_ms"]
            achieved = flops / (avg_ms * 1e-3) / 1e12
            peak = PEAK_TFLOPS[args.precision]
            traffic, tnote = None, None
            if dom == "G0.c5.fwd" and args.arch == "neutron" and os.path.exists(TRAFFIC_JSON):
                tj = json.load(open(TRAFFIC_JSON))
                traffic = tj["traffic_bytes"]
                tnote = (f"bytes per launch: FETCH_SIZE x2 {tj['fetch_bytes']} + WRITE_SIZE {tj['write_bytes']} "
                         f"(algorithmic {tj['algorithmic_bytes']}), {os.path.relpath(TRAFFIC_JSON, ROOT)}")
            roof = {"bound": "mfma", "kernel": f"conv_ring {dom} (generator conv_layers.5)",
                    "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_note": tnote,
                    "avg_ms": round(avg_ms, 4), "launches": stats[dom]["count"],
                    "all_probed": {k: {"avg_ms": round(v["avg_ms"], 4),
                                       "tflops": round(flops / (v["avg_ms"] * 1e-3) / 1e12, 2)}
                                   for k, v in stats.items()}}
        step_flops = STEP_FLOP_PER_IMAGE[args.arch] * value
        out = {
            "metric": "GAN-step images/sec (44x44 ZDC) at 1/2/4/8 MI355X; conv MFMA util %",
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "step_launch": "hip_graph" if use_graph else "eager",
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"{args.arch} 44x44 MoE-GAN train_step, E={args.experts}, B={args.batch} per GPU "
                                   f"(BASELINE configs[1])", "arch": args.arch, "n_experts": args.experts,
                       "global_batch": args.batch * world, "image": "44x44" if args.arch == "neutron" else "56x30",
                       "parallelism": f"dp{world}"},
            "step_tflops": round(step_flops / 1e12, 2),
            "step_mfma_frac": round(step_flops / 1e12 / PEAK_TFLOPS[args.precision], 4),
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.arch)
        print(json.dumps(out), flush=True)
    if ddp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
