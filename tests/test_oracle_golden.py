"""The oracle (CPU restatement) against golden vectors captured from the reference itself.

Runs on CPU (``-m "not gpu"``).  Tolerance: the oracle uses the same torch CPU primitives as the
reference at 1 thread, so every recorded output, metric and gradient matches to <= 1e-6
relative (observed: bit-exact).  This pins the oracle before it is used to check HIP kernels.
"""
import numpy as np
import pytest
import torch

from golden_utils import CASES, Golden, checksum, rel_err
from oracle import expertsim_oracle as O

TOL = 1e-6


def _run(case):
    torch.set_num_threads(1)
    g = Golden(case)
    m = O.OracleMoE(g.arch, g.E, g.oracle_cfg(O.DEFAULT_CFG), seed=g.seed)
    return g, m


@pytest.mark.parametrize("case", CASES)
def test_init_checksums(case):
    g, m = _run(case)
    for comp, sd in (("G", m.state["G"][0]), ("D", m.state["D"][0]), ("A", m.state["A"][0]),
                     ("R", m.state["R"])):
        names = set(sd)
        assert names == {k.split("/", 2)[2] for k in g.keys(f"init/{comp}/")}
        for n, t in sd.items():
            np.testing.assert_array_equal(checksum(t.float().numpy()), g[f"init/{comp}/{n}"])


@pytest.mark.parametrize("case", CASES)
def test_train_steps_match_reference(case):
    g, m = _run(case)
    for s in range(g.steps):
        inp = g.inputs(s)
        nz = g.noise(s)
        met, tr = m.train_step(
            g.epoch, torch.from_numpy(inp["cond"]), torch.from_numpy(inp["real_images"]).unsqueeze(1),
            torch.from_numpy(inp["true_positions"]), torch.from_numpy(inp["std"]),
            torch.from_numpy(inp["intensity"]), lambda e, w, shape: torch.from_numpy(nz[(e, w)]),
            torch.from_numpy(g.gumbel(s)))
        gm = g.metrics(s)
        assert set(met) == set(gm)
        for k, v in gm.items():
            assert abs(met[k] - v) <= TOL * max(abs(v), 1e-6), (s, k, met[k], v)
        for e in range(g.E):
            for c in range(2):
                k = f"s{s}/G{e}/call{c}/out0"
                if g.has(k):
                    assert rel_err(tr[f"G{e}/{c}"].numpy(), g[k]) <= TOL
            for c in range(4):
                for j in range(2):
                    k = f"s{s}/D{e}/call{c}/out{j}"
                    if g.has(k):
                        assert rel_err(tr[f"D{e}/{c}"][j].numpy(), g[k]) <= TOL
            k = f"s{s}/A{e}/call0/out0"
            if g.has(k):
                assert rel_err(tr[f"A{e}/0"].numpy(), g[k]) <= TOL
        for key in [k for k in tr if k.endswith("/grad")]:
            lab = key.split("/")[0]
            for n, t in tr[key].items():
                ref = g[f"s{s}/{lab}/grad/{n}"]
                mine = checksum(t.numpy())
                assert abs(mine[2] - ref[2]) <= 1e-5 * max(ref[2], 1e-30), (s, lab, n)


def test_philox_known_answers():
    from expertsim.utils import philox
    assert [int(x) for x in philox.philox4x32(0, 0, 0, 0, 0, 0)] == \
        [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert [int(x) for x in philox.philox4x32(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344,
                                              0xa4093822, 0x299f31d0)] == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]
