"""The second generator forward's dropout masks drawn ahead on a side stream (train.dropout_ahead:
es_dropout_keep_bits during the discriminator step, the norm passes then read the bits) give the
same training steps as masks drawn inside the norm passes.

Reference: the nn.Dropout layers of neutron/generator.py:13-36 (one mask per layer and forward).
The masks are data-independent Philox draws keyed on (seed, stream, step, logical index), so the
ahead-of-time draw must be bit-identical: fp32 parity mode (deterministic reductions), every metric,
parameter and buffer compared bitwise after every step, eager and in a captured whole-step graph.
The draw is single-expert only (MoEWrapper._bits_stream).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(E, B, steps, ahead, graph, seed):
    import bench
    from expertsim.graph import StepGraph
    from expertsim.utils.synthetic import make_batch
    b = make_batch(B, "neutron", seed=seed)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()
    moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, torch.device(DEV))
    cfg.train.dropout_ahead = ahead
    args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, DEV)
    out = []
    state = lambda: {n: v.detach().clone() for n, v in moe.state_dict().items()}
    if not graph:
        moe.expert_graphs = False
        for _ in range(steps):
            m = moe.train_step(*args)
            torch.cuda.synchronize()
            out.append(({k: float(v) for k, v in m.items()}, state()))
    else:
        m = moe.train_step(*args)
        torch.cuda.synchronize()
        out.append(({k: float(v) for k, v in m.items()}, state()))
        sg = StepGraph(moe, args, warmup=0)
        for _ in range(1, steps):
            m = sg.replay()
            torch.cuda.synchronize()
            out.append(({k: float(v) for k, v in m.items()}, state()))
        sg.sync_host_state([*og, *od, *oa, orr])
    assert (getattr(moe, "_bits_side", None) is not None) == ahead
    return out


def _compare(a, b):
    for i, ((ma, sa), (mb, sb)) in enumerate(zip(a, b)):
        dm = sorted(k for k in ma if ma[k] != mb[k])
        assert not dm, (i, dm[:6])
        ds = sorted(n for n in sa if not torch.equal(sa[n], sb[n]))
        assert not ds, (i, ds[:10])


@pytest.mark.timeout(240)
def test_dropout_ahead_graph_e1_matches_in_pass_draw():
    """E = 1, B = 256: eager steps drawing in the norm passes vs 1 eager step + a captured graph
    (the side-stream draw forked inside the capture) and 2 replays."""
    ref = _run(1, 256, 3, ahead=False, graph=False, seed=31)
    got = _run(1, 256, 3, ahead=True, graph=True, seed=31)
    _compare(ref, got)


@pytest.mark.timeout(240)
def test_dropout_ahead_eager_e1_b512():
    """E = 1, B = 512, eager steps both ways (the side-stream fork outside any capture)."""
    ref = _run(1, 512, 2, ahead=False, graph=False, seed=32)
    got = _run(1, 512, 2, ahead=True, graph=False, seed=32)
    _compare(ref, got)
