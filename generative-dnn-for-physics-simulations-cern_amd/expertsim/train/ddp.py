"""Data parallelism for the training step: one process per GPU, RCCL (backend "nccl") all-reduce.

The reference is single-device (expertsim/train/loop.py:39); north_star asks for the batch sharded
data-parallel over a node's GPUs.  Semantics chosen:
  * every rank routes and trains on its own shard of B_local samples;
  * per-expert loss weights use the LOCAL counts (B_e^r / B_r) and gradients are AVERAGED over
    ranks, which reproduces the single-device gradient exactly for every per-sample-mean term
    (hinge, generator hinge, intensity L1, log-cosh): (1/R) sum_r (1/B_r) sum_{b in r} g_b
    = (1/B) sum_b g_b;
  * batch-coupled statistics (BatchNorm batch stats, the SDI mean(std)^2 product) stay per rank,
    as torch DDP without SyncBatchNorm does;
  * an expert is trained iff its GLOBAL count is > 1 (the reference's skip rule, moe.py:126, on
    the global batch); a rank whose local count is <= 1 contributes zero gradients but still joins
    every collective, so the collective sequence is identical on all ranks;
  * one flat all-reduce per model per optimizer phase (D; G and A; router) — the flat parameter
    buffers make each model a single bucket.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


class DataParallel:
    def __init__(self, world_size=None, rank=None, group=None):
        self.group = group
        self.world = world_size if world_size is not None else dist.get_world_size(group)
        self.rank = rank if rank is not None else dist.get_rank(group)
        self._counts = None
        self.local_batch = None
        self._counts_dev = {}

    # ---------------------------------------------------------------- routing bookkeeping
    def global_groups(self, groups, B_local):
        """All-reduce the per-expert counts (one small collective) and keep local groups."""
        E = len(groups)
        self.local_batch = B_local
        if E == 1:
            # one expert holds every sample: its global count is the global batch (equal shards,
            # as DistributedSampler(drop_last=True) and bench.py give) -- no collective, no host sync
            self._counts = np.array([B_local * self.world], dtype=np.int64)
            return groups
        local = torch.tensor([g[2] for g in groups], dtype=torch.int64)
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"
        t = local.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        self._counts = t.cpu().numpy()
        self.local_batch = B_local
        return groups

    def global_count(self, e):
        return int(self._counts[e])

    @property
    def global_batch(self):
        return self.local_batch * self.world

    def global_counts_tensor(self, device):
        # cached per value: no host->device copy inside a captured step
        key = (str(device), tuple(int(c) for c in self._counts))
        if key not in self._counts_dev:
            self._counts_dev[key] = torch.from_numpy(self._counts.astype(np.float32)).to(device)
        return self._counts_dev[key]

    # ---------------------------------------------------------------- gradients
    def allreduce_grads(self, module):
        """SUM-all-reduce the flat gradient buffer; the 1/world average is folded into the fused
        Adam's grad_scale (module._grad_scale), so no extra pass over the gradients."""
        g = module.flat_grads
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
        module._grad_scale = 1.0 / self.world
