"""Data parallelism for the training step: one process per GPU, RCCL (backend "nccl") collectives.

The reference is single-device (expertsim/train/loop.py:39); north_star asks for the batch sharded
data-parallel over a node's GPUs.  Semantics:

  * the global batch is the ranks' equal shards in rank order; every rank routes its own shard;
  * randomness is drawn at GLOBAL sample indices: a rank holding samples [n0, n0 + n) of an
    expert's global batch draws exactly those rows of the single-device noise / Gumbel draws and
    dropout masks (expertsim/utils/philox.py), n0 = the lower ranks' counts for that expert
    (``sample_offset``);
  * per-expert loss weights use the LOCAL counts (B_e^r / B_r) and the gradients of the generator,
    discriminator and aux regressor are AVERAGED over ranks, which reproduces the single-device
    gradient exactly for every per-sample-mean term (hinge, generator hinge, intensity L1,
    log-cosh): (1/R) sum_r (1/B_r) sum_{b in r} g_b = (1/B) sum_b g_b;
  * batch-coupled statistics:
      - ``sync_bn=True``: BatchNorm batch statistics and backward sums of the neutron generator and
        aux regressor are all-gathered / all-reduced per layer (SyncBN), the SDI prefactor
        mean(std)^2 uses the expert's global mean, the router's ALB / entropy terms the global
        gate sums S_e and its ED term the all-gathered per-sample features -- with equal shards the
        data-parallel step then equals the single-device step of the global batch (tests:
        tests/test_ddp_gpu.py on the HIP path, tests/test_ddp_cpu.py on the oracle);
      - ``sync_bn=False`` (default, torch-DDP-without-SyncBatchNorm behaviour, no collective inside
        the forward / backward): those statistics stay per rank (tests/test_ddp_cpu.py measures the
        deviation from the global-batch step);
  * the router's gradient is SUMMED over ranks (its ALB / entropy / ED terms are functions of
    global sums, not per-sample means);
  * an expert is trained iff its GLOBAL count is > 1 (the reference's skip rule, moe.py:126, on
    the global batch); a rank with too few local samples contributes zero gradients but joins every
    collective, so the collective sequence is identical on all ranks;
  * metrics are merged across ranks on the device (one all-gather of the [E, 10] metric rows);
  * gradient all-reduces overlap the compute (``allreduce_async`` on the process group's stream):
    the discriminator's with the second generator forward, the aux regressor's with the generator
    backward, and the generator's in >= 1 MB buckets issued as its second backward finalises each
    layer group (``bucketer``; the flat buffer's tail first); the optimizer steps wait for them;
  * multi-expert steps run the experts CONCURRENTLY (each expert's program on its own HIP stream,
    reference per-expert loop moe.py:121-207): every expert gets a process group of its own over
    the same ranks (``expert_groups``, created once, in the same order on every rank), and its SyncBN
    gathers / backward sums, SDI mean and gradient buckets run on that communicator
    (``on_expert``), so no communicator is shared by two streams.  Each communicator still sees the
    same per-rank issue order (an expert's program is issued in full before the next); the routing
    counts, router and metric collectives stay on the main group, outside the fork.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch
import torch.distributed as dist

from .. import hip


class DataParallel:
    def __init__(self, world_size=None, rank=None, group=None, sync_bn=False):
        self.group = group         # the main group (routing counts, router, metrics)
        self.world = world_size if world_size is not None else dist.get_world_size(group)
        self.rank = rank if rank is not None else dist.get_rank(group)
        self.sync_bn = bool(sync_bn)
        self.gloo = dist.get_backend(group) != "nccl"
        self._counts = None        # global count per expert (single-expert steps)
        self._offsets = None       # this rank's first global sample index per expert
        self._local = None         # local count per expert
        self.local_batch = None
        self._counts_dev = {}
        self.expert = None         # expert whose step is running (global count for SyncBN)
        self.plan = None           # multi-expert steps: the device plan (MoEWrapper._plan)
        self.expert_groups = None  # one process group per expert (concurrent experts)
        self._cur = None           # the group of the running expert (None: the main group)
        self._pending = []         # async all-reduce works not yet waited for
        self.issued = []           # (module, lo, hi) of every gradient all-reduce (tests)

    # ---------------------------------------------------------------- per-expert communicators
    def ensure_expert_groups(self, E: int):
        """One process group per expert over the main group's ranks.  dist.new_group is collective
        over the world: every rank calls this at the same point of the same step (the first
        multi-expert step, before any capture)."""
        if self.expert_groups is not None and len(self.expert_groups) >= E:
            return self.expert_groups
        ranks = None if self.group is None else dist.get_process_group_ranks(self.group)
        have = list(self.expert_groups or [])
        while len(have) < E:
            have.append(dist.new_group(ranks=ranks))
        self.expert_groups = have
        return have

    @contextlib.contextmanager
    def on_expert(self, e: int, own_group: bool = True):
        """The collectives issued inside run on expert e's communicator (``own_group``) and
        SyncBN reads expert e's global count."""
        prev = (self.expert, self._cur)
        self.expert = e
        if own_group and self.expert_groups is not None:
            self._cur = self.expert_groups[e]
        try:
            yield self
        finally:
            self.expert, self._cur = prev

    @property
    def cur_group(self):
        return self.group if self._cur is None else self._cur

    # ---------------------------------------------------------------- collectives on device tensors
    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if self.gloo and t.is_cuda:        # gloo (CPU tests / single-GPU rehearsals): via the host
            h = t.cpu()
            dist.all_reduce(h, op=op, group=self.cur_group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=self.cur_group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] (rank order), contiguous."""
        t = t.contiguous()
        if self.gloo:
            src = t.cpu() if t.is_cuda else t
            parts = [torch.empty_like(src) for _ in range(self.world)]
            dist.all_gather(parts, src, group=self.cur_group)
            return torch.stack(parts).to(t.device)
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.cur_group)
        return out

    # ---------------------------------------------------------------- routing bookkeeping
    def global_groups(self, groups, B_local):
        """Single-expert step: the global count and this rank's sample offset (equal shards:
        DistributedSampler(drop_last=True) and bench.py give them) -- no collective, no host sync.
        Multi-expert steps keep their counts on the device (set_plan)."""
        assert len(groups) == 1, "multi-expert steps use the device plan (MoEWrapper._plan)"
        self.local_batch = B_local
        self._counts = np.array([B_local * self.world], dtype=np.int64)
        self._offsets = np.array([B_local * self.rank], dtype=np.int64)
        self._local = np.array([B_local], dtype=np.int64)
        return groups

    def set_plan(self, plan, B_local):
        """Multi-expert step: the per-expert counts live on the device (dynamic rows, no host copy)."""
        self.plan = plan
        self.local_batch = B_local

    def global_count_ptr(self):
        """Device float pointer to the running expert's global count (dynamic-rows SyncBN)."""
        return hip.ptr(self.plan["gcnt"][self.expert:self.expert + 1])

    def global_count(self, e):
        return int(self._counts[e])

    def sample_offset(self, e):
        """Index of this rank's first sample in expert e's global batch."""
        return int(self._offsets[e])

    @property
    def batch_offset(self):
        """Index of this rank's first sample in the global batch (equal shards)."""
        return self.local_batch * self.rank

    @property
    def global_batch(self):
        return self.local_batch * self.world

    def global_counts_tensor(self, device):
        # cached per value: no host->device copy inside a captured step
        key = (str(device), tuple(int(c) for c in self._counts))
        if key not in self._counts_dev:
            self._counts_dev[key] = torch.from_numpy(self._counts.astype(np.float32)).to(device)
        return self._counts_dev[key]

    # ---------------------------------------------------------------- SyncBN hooks (layers.NormOp)
    def bn_rows(self, local_rows, local_n):
        """Global row count of a BatchNorm input of the running expert: rows per sample x global n."""
        return (local_rows // max(local_n, 1)) * self.global_count(self.expert)

    # ---------------------------------------------------------------- gradients
    def allreduce_grads(self, module, average=True):
        """SUM-all-reduce the flat gradient buffer; the 1/world average is folded into the fused
        Adam's grad_scale (module._grad_scale), so no extra pass over the gradients."""
        g = module.flat_grads
        self.all_reduce_(g)
        module._grad_scale = 1.0 / self.world if average else 1.0

    # ---------------------------------------------------------------- overlapped gradient all-reduce
    def allreduce_async(self, module, average=True, lo=0, hi=None):
        """SUM-all-reduce flat_grads[lo:hi] on the process group's own stream, overlapping the compute
        issued after it; wait_all() makes the current stream wait before an optimizer reads the
        gradients.  Every rank issues the same ranges in the same order (the collectives of one
        process group run in issue order), so this never reorders collectives across ranks."""
        g = module.flat_grads
        hi = g.numel() if hi is None else hi
        if hi > lo:
            if self.gloo:
                self.all_reduce_(g[lo:hi])
            else:
                self._pending.append(dist.all_reduce(g[lo:hi], group=self.cur_group, async_op=True))
            self.issued.append((module, lo, hi))
        module._grad_scale = 1.0 / self.world if average else 1.0

    def wait_all(self):
        for w in self._pending:
            w.wait()
        self._pending = []

    def bucketer(self, module, min_floats=1 << 18):
        """``ready(name)`` hook for a module's backward: layers finish in reverse flat-buffer order,
        so once the backward reports parameter ``name`` done, every gradient from its offset to the
        end of the buffer is final; they are all-reduced in buckets of >= min_floats floats (1 MB)
        while the rest of the backward runs (the last call, at offset 0, flushes the remainder)."""
        offs = {n: o for (n, _), o in zip(module.named_parameters(), module._offsets())}
        state = {"hi": module.flat_grads.numel()}

        def ready(name):
            lo = offs[name]
            if state["hi"] - lo >= min_floats or lo == 0:
                self.allreduce_async(module, True, lo, state["hi"])
                state["hi"] = lo
        return ready

    # ---------------------------------------------------------------- metrics
    def merge_metrics(self, mbuf: torch.Tensor, lcnt: torch.Tensor = None):
        """mbuf [E, 9] (per expert: total, gen, div, int, aux, std_int, mean_int, w, disc) -> the
        global-batch values, in place (es_dp_metrics_merge over the all-gathered rows).  lcnt (device
        [E] float, multi-expert steps): the rows each expert ran on this rank (0: not run)."""
        E = mbuf.shape[0]
        rows = torch.empty(E, 10, dtype=torch.float32, device=mbuf.device)
        rows[:, :9].copy_(mbuf)
        if lcnt is not None:
            rows[:, 9].copy_(lcnt)
        else:
            ran = self._local >= (1 if self.sync_bn else 2)        # the ranks that ran the expert's step
            n = np.where(ran, self._local, 0).astype(np.float32)
            # one expert (E == 1): the shard size, a device constant cached per value (a pageable
            # host -> device copy_ would synchronise the stream at the end of every step)
            key = ("n", str(mbuf.device), tuple(float(v) for v in n))
            if key not in self._counts_dev:
                if len(self._counts_dev) > 64:
                    self._counts_dev.clear()
                self._counts_dev[key] = torch.from_numpy(n).to(mbuf.device)
            rows[:, 9].copy_(self._counts_dev[key])
        allr = self.all_gather(rows)
        hip.call("es_dp_metrics_merge", hip.ptr(allr), self.world, E, hip.ptr(mbuf), hip.stream_ptr())
        return mbuf
