"""Gradients of the HIP train step against the reference's recorded gradients.

The goldens (tests/golden/make_goldens.py:220-233) hold, for every optimizer step of the reference,
a checksum of each parameter's gradient as it enters ``Adam.step`` (sum, |.|-sum, L2 norm and 64
strided samples).  Here the HIP path's gradients are captured at the same point (the flat
gradient buffer each FusedAdam reads) and compared with SURVEY.md §8(c)'s contract:

  * norm-relative error <= 1e-2 (neutron, BatchNorm after every conv + dropout) / 1e-3 (proton),
    on the 64 sampled elements (||g_s - g_s,ref|| / ||g_s,ref||) and on the full L2 norm;
  * the noise-only set — biases that feed a normalisation with per-channel statistics, whose
    analytic gradient is exactly zero (neutron G fc1.0 / fc2.0 / conv_layers.{0,5,9} biases, the
    neutron aux regressor's BN-fed conv biases, the proton aux regressor's GroupNorm(C, C)-fed
    residual biases) — is checked absolutely: ||g|| <= 1e-5;
  * step 0 is the contract step.  At step 1 every parameter has moved by +-lr through Adam's
    first step whatever its gradient's size (SURVEY.md §8(c) hard part (c)), so rounding-level
    sign flips of tiny step-0 gradients change the step-1 gradients.  Their bound is the
    reference's OWN sensitivity, per parameter: tools/grad_sensitivity.py reruns the oracle
    (bit-exact to the goldens) with every linear / conv output of both steps perturbed by 1e-6
    relative (the HIP path's own deviation from the reference) and records the worst step-1 error
    against the goldens over 6 trials (tests/golden/sensitivity_<case>_s1.json); a parameter is held
    to max(step-0 bound, min(3 x that, 0.6)), and where that bound exceeds 0.1 its gradient must also
    have a cosine >= 0.75 with the reference's (sampled elements) and an L2 norm within 0.67-1.5x.  (proton_e1_b8's G conv_layers.11.bias: HIP 0.093 in round 4,
    the reference itself 0.076 under the perturbation -- the step-1 spread, not a defect.)

A second test drives the same step through the reference's nn.Module API — ``G(noise, cond)``,
``D(img, cond)``, ``A(img)``, losses in torch, ``loss.backward()``, ``opt.step()`` — i.e. the
drop-in path of INTEGRATION.md, and holds its outputs and gradients to the same goldens.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_utils import CASES, Golden, checksum
from test_train_step_gpu import _build

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {"neutron": 1e-2, "proton": 1e-3}
# proton_e3_b12: expert 1 trains on B_e = 4 samples.  One LeakyReLU input of its last GroupNorm
# lies within the fp32 forward's rounding of the kink (|z| < 1e-6), so the reference and any other
# fp32 evaluation order may take different branches there: measured (tools/diag_gbwd_layers.py)
# the HIP GroupNorm backward equals an fp64 evaluation on its own forward to 4.9e-8, while the
# torch-fp32 forward's branch choice moves that layer's input gradient by 2.7e-3 norm-relative and
# every gradient upstream by ~3e-3.  The case is held to the neutron bound instead.
CASE_TOL = {"proton_e3_b12": 1e-2}
# Step-0 aux-regressor gradients.  A reads the generator's images, which the HIP path reproduces to
# ~1e-6 relative, not bitwise, and the reference's own A gradients can jump on that scale: its
# step 0 rerun on the oracle with A's input multiplied by (1 + 1e-6 N(0, 1)) moves them by 4e-6 in
# 7 of 8 trials and by 4.49e-2 (one MaxPool near-tie taking the other branch) in the 8th
# (tools/aux_sensitivity.py; tests/test_aux_sensitivity_cpu.py).  Round 2 held A to 5e-2 because the
# fp32 mode's float-atomic reductions made the HIP branch box-dependent.  The fp32 mode is now
# deterministic (train.deterministic: ordered reductions, tests/test_determinism_gpu.py), so the
# branch is fixed and reproducible: measured on it (r03b) neutron_e1_b8 5.8e-6, neutron_e3_b12
# 4.8e-3, neutron_e1_b512 4.2e-3, all on the reference's branch, so A shares SURVEY §8(c)'s 1e-2.
# test_aux_grads_on_hip_images feeds the oracle the HIP path's own images: neutron 8.0e-3,
# proton 1.7e-5 (r03b).
A_STEP0_TOL = {"neutron": 1e-2}
A_ORACLE_TOL = {"neutron": 1e-2, "proton": 1e-3}
# noise-only set after Adam's +-lr first step: BatchNorm over B_e = 2 samples (neutron_e3 step 1
# experts 0 and 2) has invstd up to ~1e3, so the analytically-zero bias sums cancel at ~1e-4
# (measured 2.0e-5 and 1.06e-4 on fc1.0.bias)
STEP1_ABS = 1e-3
NOISE_ONLY = {
    "neutron": {"G": {"fc1.0.bias", "fc2.0.bias", "conv_layers.0.bias", "conv_layers.5.bias",
                      "conv_layers.9.bias"},
                "A": {"feature_extractor.conv1.bias", "feature_extractor.conv2.bias",
                      "feature_extractor.conv3.bias", "feature_extractor.conv4.bias"}},
    "proton": {"A": {"feature_extractor.res1.conv1.0.bias", "feature_extractor.res1.conv2.0.bias",
                     "feature_extractor.res1.downsample.0.bias"}},
}


def _capture(opts_by_label, store):
    """Wrap each FusedAdam.step: snapshot the module's parameter gradients before the update."""
    for label, (opt, module) in opts_by_label.items():
        orig = opt.step

        def step(*a, _orig=orig, _label=label, _module=module, **k):
            from expertsim import hip
            act = hip.active_tensor()   # dynamic rows: an expert the reference skips steps as a no-op
            if act is None or int(act.item()) != 0:
                store[_label] = {n: p.grad.detach().double().cpu().numpy().copy()
                                 for n, p in _module.named_parameters()}
            return _orig(*a, **k)
        opt.step = step


def grad_errors(g: Golden, s, label, grads, arch, comp):
    """[(name, kind, err)] for every parameter of one optimizer step."""
    out = []
    noise = NOISE_ONLY.get(arch, {}).get(comp, set())
    for n, gm in grads.items():
        key = f"s{s}/{label}/grad/{n}"
        assert g.has(key), key
        ref = g[key]
        c = checksum(gm)
        if n in noise or ref[2] == 0.0:
            out.append((n, "abs", float(c[2])))
            continue
        samp = float(np.linalg.norm(c[3:] - ref[3:]) / max(np.linalg.norm(ref[3:]), 1e-30))
        l2 = float(abs(c[2] - ref[2]) / ref[2])
        # direction and size of the gradient beside the error: the cosine of the 64 sampled elements
        # with the reference's and the L2-norm ratio (a zeroed or sign-flipped gradient fails these
        # whatever the error bound)
        cos = float(np.dot(c[3:], ref[3:]) / max(np.linalg.norm(c[3:]) * np.linalg.norm(ref[3:]), 1e-30))
        out.append((n, "rel", max(samp, l2), cos, float(c[2] / ref[2])))
    return out


def sensitivity(case, step):
    """The reference's own gradient sensitivity for a case and step (tests/golden/sensitivity_*.json,
    tools/grad_sensitivity.py: the oracle with every linear / conv output perturbed by 1e-6 relative,
    worst error against the goldens over its trials), {"optG0/name": err}; {} when not measured."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"sensitivity_{case}_s{step}.json")
    return json.load(open(p))["worst"] if os.path.exists(p) else {}


# step >= 1: a parameter's bound is 3 x the reference's own sensitivity, capped here (a bound
# near 1 would pass an all-zero gradient); where the bound exceeds SENS_DIRECTION the gradient must
# also point the reference's way (cosine of the sampled elements) at a comparable size (L2 ratio)
STEP1_CAP = 0.6
SENS_DIRECTION = 0.1
MIN_COS, L2_RATIO = 0.75, (0.67, 1.5)


def _check(errs, tol, what, abs_tol=1e-5, sens=None, label=None):
    """sens (per-parameter reference sensitivity): a parameter's bound is max(tol, min(3 x sens,
    STEP1_CAP)), plus the direction / size check where that bound exceeds SENS_DIRECTION."""
    worst = max((e for e in errs if e[1] == "rel"), key=lambda e: e[2], default=None)
    print(what, "worst rel:", worst, "worst abs:",
          max((e for e in errs if e[1] == "abs"), key=lambda e: e[2], default=None))
    print(what, "abs:", [(e[0], f"{e[2]:.2e}") for e in errs if e[1] == "abs"])
    for e in errs:
        n, kind, err = e[:3]
        if kind == "abs":
            assert err <= abs_tol, (what, n, err)
            continue
        s3 = 3.0 * (sens or {}).get(f"{label}/{n}", 0.0)
        bound = max(tol, min(s3, STEP1_CAP))
        if bound > SENS_DIRECTION:
            cos, ratio = e[3], e[4]
            print(what, n, f"err {err:.3g} bound {bound:.3g} cos {cos:.4f} L2 ratio {ratio:.4f}")
            assert cos >= MIN_COS and L2_RATIO[0] <= ratio <= L2_RATIO[1], (what, n, err, cos, ratio)
        assert err <= bound, (what, n, err, bound)


@pytest.mark.parametrize("case", CASES)
def test_step_gradients_match_reference(case):
    g = Golden(case)
    moe, (og, od, oa, orr), cfg = _build(g)
    store = {}
    labels = {}
    for e in range(g.E):
        labels[f"optG{e}"] = (og[e], moe.generators[e])
        labels[f"optD{e}"] = (od[e], moe.discriminators[e])
        labels[f"optA{e}"] = (oa[e], moe.aux_regs[e])
    labels["optR"] = (orr, moe.router)
    _capture(labels, store)
    for s in range(g.steps):
        store.clear()
        inp = g.inputs(s)
        nz = g.noise(s)
        moe.noise_fn = lambda e, w, shape: torch.from_numpy(nz[(e, w)])
        gum = torch.from_numpy(g.gumbel(s))
        moe.gumbel_fn = lambda shape: gum
        t = lambda k: torch.from_numpy(inp[k]).to(DEV)
        moe.train_step(g.epoch, t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"),
                       t("intensity"), oa, og, od, orr, None, DEV)
        torch.cuda.synchronize()
        want = {k.split("/")[1] for k in g.keys(f"s{s}/") if "/grad/" in k}
        assert set(store) == want, (s, sorted(store), sorted(want))
        tol = CASE_TOL.get(case, TOL[g.arch])
        sens = sensitivity(case, s) if s > 0 else None
        assert s == 0 or sens, f"{case}: no step-{s} sensitivity fixture (tools/grad_sensitivity.py)"
        for label, grads in store.items():
            comp = label[3]
            lt = max(tol, A_STEP0_TOL.get(g.arch, 0.0)) if comp == "A" and s == 0 else tol
            _check(grad_errors(g, s, label, grads, g.arch, comp), lt, (case, s, label),
                   abs_tol=1e-5 if s == 0 else STEP1_ABS, sens=sens, label=label)


@pytest.mark.parametrize("case", [c for c in CASES if "_e1_" in c])
def test_module_api_backward_matches_reference(case):
    """The reference's call pattern (moe.py:506-571) through the nn.Module API + loss.backward()."""
    from oracle import expertsim_oracle as O
    g = Golden(case)
    moe, (og, od, oa, orr), cfg = _build(g)
    G, D, A = moe.generators[0], moe.discriminators[0], moe.aux_regs[0]
    store = {}
    _capture({"optG0": (og[0], G), "optD0": (od[0], D), "optA0": (oa[0], A)}, store)
    inp = g.inputs(0)
    nz = g.noise(0)
    t = lambda k: torch.from_numpy(inp[k]).to(DEV)
    cond, real, pos, std, inten = t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"), \
        t("intensity")
    n1, n2 = (torch.from_numpy(nz[(0, w)]).to(DEV) for w in (0, 1))
    # the reference's step-0 dropout masks: (seed, dropout_stream(0, expert 0, pass, 0))
    G.dropout_keys = [(g.seed, 0), (g.seed, 8)]
    A.dropout_keys = [(g.seed, 16)]
    for o in (og[0], od[0], oa[0]):
        o.zero_grad(set_to_none=True)
    w = 1.0                                           # class_counts_adjusted with one expert

    fake = G(n1, cond)                                # moe.py:145
    ro, _ = D(real, cond)                             # discriminator_train_step, moe.py:513-527
    fo, _ = D(fake.detach(), cond)
    d_loss = (F.relu(1.0 - ro).mean() + F.relu(1.0 + fo).mean()) * w
    d_loss.backward()
    od[0].step()

    fake2 = G(n2, cond)                               # generator_train_step, moe.py:535-566
    fo1, fl1 = D(fake, cond)
    _, fl2 = D(fake2, cond)
    gen = -fo1.mean()
    div = O.sdi_gan_regularization(fl1, fl2, n1, n2, std, G.di_strength)
    il = O.intensity_regularization(fake, inten, G.in_strength)[0]
    coords = A(fake)
    aux = A.regressor_loss(pos, coords) * cfg.model.aux_reg.strength
    g_loss = (gen + div + il + aux) * w
    g_loss.backward()
    og[0].step()
    oa[0].step()
    torch.cuda.synchronize()

    rel = lambda a, b: float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-6))
    assert rel(fake.detach().cpu().numpy(), g["s0/G0/call0/out0"]) <= 1e-4
    assert rel(fake2.detach().cpu().numpy(), g["s0/G0/call1/out0"]) <= 1e-4
    assert rel(coords.detach().cpu().numpy(), g["s0/A0/call0/out0"]) <= 1e-4
    gm = g.metrics(0)
    assert abs(float(d_loss) - gm["disc_loss"]) <= 1e-4 * max(abs(gm["disc_loss"]), 1e-3)
    assert abs(float(g_loss) - gm["gen_loss"]) <= 1e-4 * max(abs(gm["gen_loss"]), 1e-3)
    for label, grads in store.items():
        tol = max(TOL[g.arch], A_STEP0_TOL.get(g.arch, 0.0)) if label[3] == "A" else TOL[g.arch]
        _check(grad_errors(g, 0, label, grads, g.arch, label[3]), tol, (case, "module-api", label))


@pytest.mark.parametrize("case", [c for c in CASES if "_e1_" in c])
def test_aux_grads_on_hip_images(case):
    """A's backward on the HIP path's own generated images: the oracle (torch CPU fp32, the same
    init parameters, the same step-0 Philox dropout masks) evaluates A's forward, the regressor loss
    (moe.py:558-561) and its parameter gradients on exactly the images the HIP generator produced,
    so the comparison does not inherit the generator's ~1e-6 differences (see A_STEP0_TOL)."""
    from expertsim.utils import philox
    from oracle import expertsim_oracle as O
    g = Golden(case)
    moe, (og, od, oa, orr), cfg = _build(g)
    G, A = moe.generators[0], moe.aux_regs[0]
    store = {}
    _capture({"optA0": (oa[0], A)}, store)
    inp = g.inputs(0)
    t = lambda k: torch.from_numpy(inp[k]).to(DEV)
    cond, pos = t("cond"), t("true_positions")
    n1 = torch.from_numpy(g.noise(0)[(0, 0)]).to(DEV)
    G.dropout_keys = [(g.seed, 0)]
    A.dropout_keys = [(g.seed, 16)]
    oa[0].zero_grad(set_to_none=True)
    with torch.no_grad():
        fake = G(n1, cond)
    coords = A(fake)
    aux = A.regressor_loss(pos, coords) * cfg.model.aux_reg.strength
    aux.backward()
    oa[0].step()
    torch.cuda.synchronize()

    torch.set_num_threads(1)
    om = O.OracleMoE(g.arch, g.E, g.oracle_cfg(O.DEFAULT_CFG), seed=g.seed)
    P = om.state["A"][0]
    leaves = om._grad_leaves(P)
    drop = O.Dropper(g.seed, 0, 0, philox.PASS_AUX)
    oc = O.aux_forward(g.arch, P, fake.detach().cpu(), drop)
    ol = O.regressor_loss(pos.cpu(), oc) * cfg.model.aux_reg.strength
    ref = dict(zip(leaves, torch.autograd.grad(ol, list(leaves.values()), allow_unused=True)))
    assert float(np.max(np.abs(coords.detach().cpu().numpy() - oc.detach().numpy()))) <= \
        1e-5 * max(float(oc.abs().max()), 1.0)
    noise = NOISE_ONLY.get(g.arch, {}).get("A", set())
    worst = (None, 0.0)
    for n, h in store["optA0"].items():
        r = ref[n]
        r = np.zeros_like(h) if r is None else r.double().numpy()
        if n in noise:
            assert float(np.linalg.norm(h)) <= 1e-5, (n, float(np.linalg.norm(h)))
            continue
        e = float(np.linalg.norm(h - r) / max(np.linalg.norm(r), 1e-30))
        worst = max(worst, (n, e), key=lambda x: x[1])
        assert e <= A_ORACLE_TOL[g.arch], (case, n, e)
    print(case, "A grads vs oracle on the HIP images: worst", worst)
