"""HIP-graph capture of one ``MoEWrapper.train_step`` (single process, n_experts == 1).

The step is ~600 kernel launches issued from Python; once the kernels are fast, the host issue
time shows up as idle gaps on the GPU.  A captured graph replays the whole step with one launch.
Everything that changes from step to step is read on the device, so a replay is exactly the
next training step:
  * dropout streams and noise / Gumbel streams add ``step * mul`` from MoEWrapper's device step
    counter (hip.set_step_counter, DeviceRNG.begin_step);
  * each FusedAdam reads its step (bias corrections) from a device counter;
  * both counters are advanced by kernels inside the step.
Inputs are the static tensors passed at capture time: copy new batches into them before replay.

Data parallel (RCCL process group, n_experts == 1): the step's collectives -- the SyncBN
statistics / backward-sum reductions, the bucketed gradient all-reduces on the process group's
stream (joined back by ``wait``) and the metric all-gather -- are captured into the same graph, so a
replay issues no host work and no host synchronisation (the global counts of E = 1 are known on the
host without a collective, ``DataParallel.global_groups``).  Every rank must capture and replay in
lockstep (same step count), as it issues the same collectives in the same order.

Not captured: n_experts > 1 (the expert sizes are read on the host for the reference's
``B_e <= 1`` skip rule) and gloo process groups (their collectives go through the host).
"""
from __future__ import annotations

import torch


def graph_supported(moe) -> bool:
    """True when ``moe.train_step`` issues no host synchronisation and can be captured."""
    return moe.n_experts == 1 and (moe.ddp is None or not moe.ddp.gloo)


class StepGraph:
    def __init__(self, moe, step_args, warmup: int = 2):
        if not graph_supported(moe):
            raise ValueError("StepGraph captures single-expert train steps (single process or RCCL data parallel)")
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
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
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
