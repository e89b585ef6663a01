"""Evaluation: the oracle and the host-side geometry against the goldens
captured from the reference (tests/golden/make_eval_goldens.py).  CPU only.

Tolerances: masks exact; channel sums <= 1e-5 relative (the reference sums the real images in
float32, the oracle in float64); eval-mode generator <= 1e-5 relative to max|x| (same torch CPU
primitives, 1 thread); Wasserstein means <= 1e-6 relative, their std over repetitions <= 1e-6 x the mean (absolute):
the generator is fp32 and the reference ran it in batches of 16.
"""
import json
import os

import numpy as np
import pytest
import torch

from golden_utils import GOLDEN_DIR
from oracle import expertsim_oracle as O

ARCHES = ["neutron", "proton"]


def _golden(arch):
    z = np.load(os.path.join(GOLDEN_DIR, f"eval_{arch}.npz"), allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def running_stats(n, expert):
    """Same closed form as make_eval_goldens.running_stats."""
    i = np.arange(n, dtype=np.float64)
    return ((0.1 * np.sin(0.37 * i + expert)).astype(np.float32),
            (0.75 + 0.25 * np.cos(0.11 * i + 2 * expert)).astype(np.float32))


def oracle_generator(arch, seed, expert):
    P = O.build_all(arch, 1, seed)["G"][0]
    for k in list(P):
        if k.endswith("running_mean"):
            m, v = running_stats(P[k].numel(), expert)
            P[k] = torch.from_numpy(m)
            P[k.replace("running_mean", "running_var")] = torch.from_numpy(v)
    return P


@pytest.mark.parametrize("arch", ARCHES)
def test_channel_masks(arch):
    from expertsim.train.utils import get_channel_masks
    z, meta = _golden(arch)
    for h, w in meta["mask_shapes"]:
        ref = z[f"masks/{h}x{w}"]
        np.testing.assert_array_equal(np.stack(O.channel_masks(h, w)).astype(np.uint8), ref)
        np.testing.assert_array_equal(np.stack(get_channel_masks(np.zeros((h, w), np.float32))).astype(np.uint8), ref)
        # the five masks partition the image
        np.testing.assert_array_equal(ref.sum(0), np.ones((h, w), np.uint8))


@pytest.mark.parametrize("arch", ARCHES)
def test_oracle_channel_sums(arch):
    z, _ = _golden(arch)
    got = O.channel_sums(np.expm1(z["real_images"]))
    np.testing.assert_allclose(got, z["ch_org"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(O.channel_sums(z["pred/res"]), z["pred/ch"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("arch", ARCHES)
def test_oracle_eval_generator(arch):
    torch.set_num_threads(1)
    z, meta = _golden(arch)
    P = oracle_generator(arch, meta["seed"], 1)
    n = meta["n_pred"]
    with torch.no_grad():
        out = O.generator_forward(arch, P, torch.from_numpy(z["pred/noise"]), torch.from_numpy(z["cond"][:n]),
                                  training=False)
    ref = z["pred/raw"]
    got = out.numpy().reshape(ref.shape)
    assert np.abs(got - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-6)


@pytest.mark.parametrize("arch", ARCHES)
def test_oracle_joint_ws(arch):
    """Replay the recorded noise through the oracle generators -> the reference's WS numbers."""
    torch.set_num_threads(1)
    z, meta = _golden(arch)
    assign, cond, ch_org = z["assign"], z["cond"], z["ch_org"]
    noise = z["ws/noise"]
    gens = [oracle_generator(arch, meta["seed"], e) for e in range(2)]
    idx = [np.where(assign == e)[0] for e in range(2)]
    runs, row = [], 0
    for _ in range(meta["n_calc"]):
        per = []
        for e in range(2):
            k = len(idx[e])
            with torch.no_grad():
                img = O.generator_forward(arch, gens[e], torch.from_numpy(noise[row:row + k]),
                                          torch.from_numpy(cond[idx[e]]), training=False)
            row += k
            per.append(O.channel_sums(np.expm1(img.numpy()[:, 0]).astype(np.float64)))
        runs.append(per)
    assert row == noise.shape[0]
    m, s, me, se = O.joint_ws(ch_org, [ch_org[ix] for ix in idx], runs)
    # the std over repetitions is a difference of near-equal numbers: compared on the mean's scale
    scale = float(z["ws/mean"])
    np.testing.assert_allclose(m, float(z["ws/mean"]), rtol=1e-6)
    np.testing.assert_allclose(me, z["ws/mean_exp"], rtol=1e-6)
    np.testing.assert_allclose(s, float(z["ws/std"]), rtol=0, atol=1e-6 * scale)
    np.testing.assert_allclose(se, z["ws/std_exp"], rtol=0, atol=1e-6 * scale)


def test_oracle_wasserstein_matches_scipy():
    from scipy.stats import wasserstein_distance
    rng = np.random.default_rng(0)
    for nu, nv in ((1, 1), (5, 9), (300, 170)):
        u, v = rng.lognormal(1, 1.2, nu), rng.lognormal(1.3, 1.0, nv)
        v[: nv // 3] = 0.0        # ties
        assert abs(O.wasserstein_1d(u, v) - wasserstein_distance(u, v)) <= 1e-12 * max(1.0, wasserstein_distance(u, v))
