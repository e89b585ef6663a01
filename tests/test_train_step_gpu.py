"""Full training step on the HIP path (fp32 mode) against the reference's golden vectors.

The goldens were captured from the reference itself (tests/golden/make_goldens.py) with injected
noise / Gumbel draws and Philox dropout masks; the same randomness is injected here.
Tolerances (derived from the reference's own 1-vs-8-thread drift):
  step 0: generated images, D outputs/latents, aux coords and every loss metric <= 1e-4 relative
          (metrics: relative to max(|ref|, 1e-3) so near-zero terms are compared absolutely);
          post-Adam parameters |p - p_ref| <= 2*lr elementwise (64 strided samples per tensor);
  step 1: the same quantities <= STEP1_TOL[case] relative.  Adam's first step moves every
          parameter by ~+-lr whatever its gradient's size, so rounding-level differences that flip
          the sign of a tiny gradient (e.g. a ReLU-threshold pixel) become +-lr parameter moves.
          The reference's OWN step-1 sensitivity: the oracle (bit-exact to the reference) with 3e-6
          relative noise injected on every conv output moves step-1 metrics by up to 2.5e-3
          (neutron_e3), 1.3e-4 (..._e1 cases at 1e-6) and 4.6e-2 (proton_e3_b12).
          Round 4: the fp32 mode is bitwise deterministic, so each case's step-1 outcome is one fixed
          number; STEP1_TOL is ~3x that outcome (r04d, worst of metrics / images / D / A printed by this
          test: neutron_e1_b8 5.9e-5, neutron_e3_b12 1.5e-3, proton_e1_b8 2.1e-4, proton_e3_b12 1.7e-4)
          and never above 3x the reference's sensitivity (3.9e-4 for the E = 1 cases, 7.5e-3 neutron_e3).
"""
import numpy as np
import pytest
import torch

from golden_utils import CASES, Golden
from expertsim import hip
from expertsim.layers import Act

pytestmark = pytest.mark.gpu
DEV = "cuda"
STEP1_TOL = {"neutron_e1_b8": 2e-4, "neutron_e3_b12": 5e-3, "proton_e1_b8": 3.9e-4, "proton_e3_b12": 5e-4,
             "neutron_e3_b12_router": 5e-3}


def _build(g: Golden, precision="fp32"):
    from expertsim.config import inject_shared, load_config
    from expertsim.models import build_model
    from expertsim.models.moe import MoEWrapper
    from expertsim.train.training_setup import setup_optimizers
    ov = [f"model.architecture={g.arch}", f"model.n_experts={g.E}", f"train.precision={precision}",
          f"train.rng_seed={g.seed}", "model.router.diff_strength=1e-6", *g.overrides()]
    cfg = inject_shared(load_config(overrides=ov))
    torch.manual_seed(g.seed)
    gen = build_model(f"{g.arch}.generator", cfg.model.generator, DEV)
    disc = build_model(f"{g.arch}.discriminator", cfg.model.discriminator, DEV)
    aux = build_model(f"{g.arch}.aux_reg", cfg.model.aux_reg, DEV)
    router = build_model("router_v1", cfg.model.router, DEV)
    moe = MoEWrapper(gen, disc, aux, router, g.E, cfg, image_shape=tuple(gen.image_shape)).to(DEV)
    opts = setup_optimizers(moe, cfg)
    return moe, opts, cfg


def _record(moe):
    rec = {}

    def wrap(mod, label, kind):
        orig = mod.fwd

        def f(*a, **k):
            out = orig(*a, **k)
            # dynamic rows (multi-expert steps): buffers of the batch's capacity, the first n live
            n = hip.live_count()
            if n != 0:      # (an expert the reference skips runs on zero rows: nothing to compare)
                rec.setdefault(label, []).append(out if n is None else
                                                 tuple(o.head(n) if isinstance(o, Act) else o for o in out))
            return out
        mod.fwd = f
    for i in range(moe.n_experts):
        wrap(moe.generators[i], f"G{i}", "G")
        wrap(moe.discriminators[i], f"D{i}", "D")
        wrap(moe.aux_regs[i], f"A{i}", "A")
    return rec


def _rel(a, b, floor=1e-6):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), floor))


@pytest.mark.parametrize("case", CASES)
def test_train_step_matches_reference(case):
    g = Golden(case)
    moe, (og, od, oa, orr), cfg = _build(g)
    rec = _record(moe)
    lrs = {"G": cfg.model.generator.lr_g, "D": cfg.model.discriminator.lr_d, "A": cfg.model.aux_reg.lr_a,
           "R": cfg.model.router.lr_r}
    worst = {}   # per step: the largest relative error of each quantity (printed: the bounds' evidence)

    def note(s, what, e):
        k = (s, what)
        worst[k] = max(worst.get(k, 0.0), float(e))
        return e
    for s in range(g.steps):
        rec.clear()
        tol = 1e-4 if s == 0 else STEP1_TOL[case]
        inp = g.inputs(s)
        nz = g.noise(s)
        moe.noise_fn = lambda e, w, shape: torch.from_numpy(nz[(e, w)])
        gum = torch.from_numpy(g.gumbel(s))
        moe.gumbel_fn = lambda shape: gum
        t = lambda k: torch.from_numpy(inp[k]).to(DEV)
        met = moe.train_step(g.epoch, t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"),
                             t("intensity"), oa, og, od, orr, None, DEV)
        torch.cuda.synchronize()
        gm = g.metrics(s)
        assert set(met) == set(gm)
        for k, v in gm.items():
            mine = float(met[k])
            assert note(s, "metric", abs(mine - v) / max(abs(v), 1e-3)) <= tol, (s, k, mine, v)
        for e in range(g.E):
            for c, (img, _) in enumerate(rec.get(f"G{e}", [])):
                ref = g[f"s{s}/G{e}/call{c}/out0"]
                assert note(s, "G", _rel(img.torch_nchw().cpu().numpy(), ref)) <= tol, (s, e, c)
            for c, (out, lat, _) in enumerate(rec.get(f"D{e}", [])):
                assert note(s, "D", _rel(out.rows2d().cpu().numpy(), g[f"s{s}/D{e}/call{c}/out0"])) <= tol, (s, e, c)
                assert note(s, "D", _rel(lat.rows2d().cpu().numpy(), g[f"s{s}/D{e}/call{c}/out1"])) <= tol, (s, e, c)
            for c, (coords, _) in enumerate(rec.get(f"A{e}", [])):
                assert note(s, "A", _rel(coords.rows2d().cpu().numpy(), g[f"s{s}/A{e}/call{c}/out0"])) <= tol, (s, e, c)
        # post-Adam parameters
        mods = [("optG", moe.generators, "G"), ("optD", moe.discriminators, "D"), ("optA", moe.aux_regs, "A")]
        for lab, mlist, comp in mods:
            for e, m in enumerate(mlist):
                for n, p in m.named_parameters():
                    key = f"s{s}/{lab}{e}/param/{n}"
                    if not g.has(key):
                        continue
                    ref = g[key]
                    a = p.detach().double().reshape(-1).cpu().numpy()
                    idx = (np.arange(64) * a.size) // 64 if a.size >= 64 else np.arange(a.size)
                    bound = 2 * lrs[comp] * (s + 1) + 1e-6
                    dp = float(np.max(np.abs(a[idx] - ref[3:])))
                    note(s, f"param/{comp} (x lr)", dp / lrs[comp])
                    assert dp <= bound, (s, lab, e, n)
        print(case, f"step {s} worst relative errors:",
              {k[1]: f"{v:.2e}" for k, v in sorted(worst.items()) if k[0] == s})
