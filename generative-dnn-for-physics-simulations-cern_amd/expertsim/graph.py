"""HIP-graph capture of one ``MoEWrapper.train_step``.

The step is ~600 kernel launches issued from Python; once the kernels are fast, the host issue
time shows up as idle gaps on the GPU.  A captured graph replays the whole step with one launch.
Everything that changes from step to step is read on the device, so a replay is exactly the
next training step:
  * dropout streams and noise / Gumbel streams add ``step * mul`` from MoEWrapper's device step
    counter (hip.set_step_counter, DeviceRNG.begin_step);
  * each FusedAdam reads its step (bias corrections) from a device counter;
  * both counters are advanced by kernels inside the step.
Inputs are the static tensors passed at capture time: copy new batches into them before replay.

Several experts: the step runs on dynamic rows (the expert sizes and the reference's ``B_e <= 1``
skip rule are read on the device, MoEWrapper._plan), so it captures like a single-expert step; one
process forks the experts' programs onto their own streams inside the graph.

Data parallel (RCCL process group): the step's collectives -- the expert counts' all-gather, the
SyncBN statistics / backward-sum reductions, the bucketed gradient all-reduces on the process
group's stream (joined back by ``wait``) and the metric all-gather -- are captured into the same
graph, so a replay issues no host work and no host synchronisation.  Every rank must capture and
replay in lockstep (same step count, equal shard sizes), as it issues the same collectives in the
same order: with more than one rank the capture is opt-in (``allow_dp``) and checks the shard sizes.

Not captured: gloo process groups (their collectives go through the host).
"""
from __future__ import annotations

import time

import torch


def graph_supported(moe, allow_dp: bool = False) -> bool:
    """True when ``moe.train_step`` issues no host synchronisation and can be captured: one process,
    or an RCCL group of one rank, or (``allow_dp``: the caller keeps the ranks in lockstep) several."""
    if moe.ddp is None:
        return True
    if moe.ddp.gloo:
        return False
    return moe.ddp.world == 1 or allow_dp


class StepGraph:
    def __init__(self, moe, step_args, warmup: int = 2, allow_dp: bool = False):
        if not graph_supported(moe, allow_dp):
            raise ValueError("StepGraph: gloo groups are not captured; more than one RCCL rank needs allow_dp=True")
        if moe.ddp is not None and moe.ddp.world > 1:
            # the ranks' captured collectives must match: equal local batches (one check at capture)
            import torch.distributed as dist
            b = torch.tensor([int(step_args[1].shape[0])], dtype=torch.int64, device=step_args[1].device)
            allb = [torch.zeros_like(b) for _ in range(moe.ddp.world)]
            dist.all_gather(allb, b, group=moe.ddp.group)
            sizes = [int(x.item()) for x in allb]
            if len(set(sizes)) != 1:
                raise ValueError(f"StepGraph: unequal local batch sizes across ranks {sizes}")
        self.moe = moe
        self.args = tuple(step_args)
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):            # warm-up on a side stream, as torch prescribes
            for _ in range(warmup):
                moe.train_step(*self.args)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if moe.ddp is not None and not moe.ddp.gloo:
            # let the process group's watchdog retire the eager steps' collectives (it polls every
            # ~100 ms) so that it queries no event while this thread captures: a watchdog query during
            # a capture aborted the process group once ("operation not permitted on an event last
            # recorded in a capturing stream", test_ddp_graph_gpu.py, 1 of 4 runs at E = 1)
            time.sleep(0.5)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: the capture does not forbid other threads' HIP calls -- the process group's
        # watchdog thread keeps querying the events of the eager steps' collectives while this thread
        # captures (in "global" mode that query failed the capture: hipErrorStreamCaptureUnsupported,
        # data-parallel E = 4 at world size 1, bench.py --graph on)
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.metrics = moe.train_step(*self.args)
        # capturing ran the Python side of one step without executing it on the device
        moe.step_count -= 1
        self.replays = 0

    def replay(self):
        """Run one train step; returns the (static) metrics dict of device scalars."""
        self.graph.replay()
        self.replays += 1
        self.moe.step_count += 1
        return self.metrics

    def sync_host_state(self, optimizers):
        """Bring host-side step counters in line with the device after replays."""
        for o in optimizers:
            o.sync_step()
        self.moe.step_count = int(self.moe._dstep.item())
