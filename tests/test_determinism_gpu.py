"""Bitwise-reproducible fp32 parity mode.

The reference's same-seed reruns are bit-identical.  The HIP fp32 mode sums every
float reduction in a fixed order (``train.deterministic``, default on: weight gradients as per-split
partials + one ordered reduce, es_conv2d_wgrad_det; no split-K float atomics; ordered conv-bias
sums), so two fresh runs of the same steps must agree BITWISE: every metric, every parameter and
every BatchNorm / spectral-norm buffer after the steps.
"""
import pytest
import torch

from golden_utils import Golden
from test_train_step_gpu import _build

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(g, steps):
    moe, (og, od, oa, orr), cfg = _build(g)
    mets = []
    for s in range(steps):
        inp = g.inputs(s)
        nz = g.noise(s)
        moe.noise_fn = lambda e, w, shape: torch.from_numpy(nz[(e, w)])
        gum = torch.from_numpy(g.gumbel(s))
        moe.gumbel_fn = lambda shape: gum
        t = lambda k: torch.from_numpy(inp[k]).to(DEV)
        m = moe.train_step(g.epoch, t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"),
                           t("intensity"), oa, og, od, orr, None, DEV)
        mets.append({k: float(v) for k, v in m.items()})
    torch.cuda.synchronize()
    state = {k: v.detach().clone().cpu() for k, v in moe.state_dict().items()}
    return mets, state


@pytest.mark.parametrize("case", ["neutron_e1_b8", "neutron_e3_b12", "proton_e1_b8", "neutron_e1_b512"])
def test_fp32_step_bitwise_rerun(case):
    g = Golden(case)
    steps = min(g.steps, 2)
    ma, sa = _run(g, steps)
    mb, sb = _run(g, steps)
    assert ma == mb
    assert sa.keys() == sb.keys()
    diff = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not diff, diff[:10]


def test_fp32_device_rng_bitwise_rerun():
    """Same, with the step's own device randomness (Philox noise / Gumbel / dropout streams), three
    steps at B = 256."""
    import bench
    from expertsim.utils.synthetic import make_batch
    outs = []
    for _ in range(2):
        moe, (og, od, oa, orr), cfg = bench.build("neutron", 1, "fp32", 21, torch.device(DEV))
        b = make_batch(256, "neutron", seed=2)
        t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
        args = (0, t["cond"], t["real_images"].unsqueeze(1).contiguous(), t["true_positions"], t["std"],
                t["intensity"], oa, og, od, orr, None, DEV)
        mets = [{k: float(v) for k, v in moe.train_step(*args).items()} for _ in range(3)]
        torch.cuda.synchronize()
        outs.append((mets, {k: v.detach().clone().cpu() for k, v in moe.state_dict().items()}))
    assert outs[0][0] == outs[1][0]
    assert all(torch.equal(outs[0][1][k], outs[1][1][k]) for k in outs[0][1])
