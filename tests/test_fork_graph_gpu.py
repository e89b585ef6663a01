"""The whole multi-expert step captured as ONE HIP graph with the experts forked onto their own
streams (graph.StepGraph + MoEWrapper._fork_streams: the mode behind ``bench.py --experts 4`` and
BASELINE configs[3]'s single-GPU line) replays exactly the eager steps.

Reference: the per-expert loop of ``MoEWrapper.train_step`` (moe.py:121-207).  Model A (same seed)
runs eager steps with no graphs at all (``expert_graphs = False``: every expert's program issued
from the host, one after another).  Model B runs ONE eager step, is captured (warmup=0), and
replayed.  fp32 parity mode (deterministic reductions), so every metric and every parameter AND
buffer (BatchNorm running statistics / batch counts, spectral-norm u / v) must land on the same
bits.  The empty-expert case routes no sample to one expert through the captured step's first
replays (its Adam / spectral-norm / batch-counter updates gated off on the device), then lets it
train in the later replays: an expert's activity changes inside ONE captured graph.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _state(moe):
    """Every parameter and buffer, cloned (device)."""
    return {n: t.detach().clone() for n, t in moe.state_dict().items()}


def _diff(sa, sb):
    return sorted(n for n in sa if not torch.equal(sa[n], sb[n]))


def _run(E, B, steps, mode, seed, bias_at=None, experts_streams="concurrent"):
    """mode "eager": every step eager without graphs; "graph": 1 eager step, capture, replays.
    bias_at(step) -> the router's last bias for that step (None: untouched)."""
    import bench
    from expertsim.graph import StepGraph
    from expertsim.utils.synthetic import make_batch
    b = make_batch(B, "neutron", seed=seed)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()
    moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, torch.device(DEV))
    cfg.train.expert_streams = experts_streams
    bias = dict(moe.router.named_parameters())["fc_layers.6.bias"]
    if bias_at is not None:
        moe.cfg.model.router.stop_router_training_epoch = 0   # frozen router: the bias edits decide
    args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, DEV)
    counts, per_step = [], []

    def set_bias(i):
        if bias_at is not None:
            with torch.no_grad():
                bias.copy_(torch.tensor(bias_at(i), dtype=torch.float32))

    if mode == "eager":
        moe.expert_graphs = False
        for i in range(steps):
            set_bias(i)
            m = moe.train_step(*args)
            torch.cuda.synchronize()
            counts.append([float(m[f"n_choosen_experts_mean_epoch_{e}"]) for e in range(E)])
            per_step.append(({k: float(v) for k, v in m.items()}, _state(moe)))
    else:
        set_bias(0)
        m = moe.train_step(*args)
        torch.cuda.synchronize()
        counts.append([float(m[f"n_choosen_experts_mean_epoch_{e}"]) for e in range(E)])
        per_step.append(({k: float(v) for k, v in m.items()}, _state(moe)))
        sg = StepGraph(moe, args, warmup=0)
        assert getattr(moe, "_side", None) is not None or experts_streams == "serial"
        for i in range(1, steps):
            set_bias(i)
            m = sg.replay()
            torch.cuda.synchronize()
            counts.append([float(m[f"n_choosen_experts_mean_epoch_{e}"]) for e in range(E)])
            per_step.append(({k: float(v) for k, v in m.items()}, _state(moe)))
        sg.sync_host_state([*og, *od, *oa, orr])
        assert moe.step_count == steps and og[0]._step == steps
    return per_step, counts


def _compare(a, b):
    for i, ((ma, sa), (mb, sb)) in enumerate(zip(a, b)):
        dm = sorted(k for k in ma if ma[k] != mb[k])
        assert not dm, (i, dm, {k: (ma[k], mb[k]) for k in dm[:6]})
        ds = _diff(sa, sb)
        assert not ds, (i, ds[:10])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("streams", ["concurrent", "serial"])
def test_forked_step_graph_matches_eager_e4_b512(streams):
    """E = 4, B = 512 (the bench's --experts 4 workload): 4 eager steps vs 1 eager + capture + 3
    replays, bitwise in every metric, parameter and buffer after EVERY step.  ``serial`` is the
    memory-lean order (experts one after another inside the capture, train.expert_streams)."""
    eager, ce = _run(4, 512, 4, "eager", seed=21, experts_streams=streams)
    graph, cg = _run(4, 512, 4, "graph", seed=21, experts_streams=streams)
    assert ce == cg
    assert all(c > 1 for step in ce for c in step), ce       # every expert trained in every step
    _compare(eager, graph)


@pytest.mark.timeout(300)
def test_forked_step_graph_empty_expert():
    """E = 4, B = 256: expert 3 receives no sample in steps 0-2 (the eager step and the first two
    replays of the capture), then trains in steps 3-4 (replays of the same graph)."""
    bias = lambda i: [40.0, 40.0, 40.0, -40.0] if i < 3 else [0.0, 0.0, 0.0, 0.0]
    eager, ce = _run(4, 256, 5, "eager", seed=22, bias_at=bias)
    graph, cg = _run(4, 256, 5, "graph", seed=22, bias_at=bias)
    assert ce == cg
    assert all(step[3] == 0.0 for step in ce[:3]) and all(step[3] > 1 for step in ce[3:]), ce
    _compare(eager, graph)
    # the empty expert's parameters did not move while it had no sample, and did once it trained
    (_, s0), (_, s2), (_, s4) = eager[0], eager[2], eager[4]
    for n in s0:
        if n.startswith(("generators.3.", "discriminators.3.", "aux_regs.3.")) and s0[n].is_floating_point():
            assert torch.equal(s0[n], s2[n]), n
    assert any(not torch.equal(s2[n], s4[n]) for n in s2 if n.startswith("generators.3."))
