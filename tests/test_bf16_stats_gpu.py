"""Statistical parity of the bf16 performance mode (last row).

bf16 GEMM operands / activations are not elementwise-comparable with the reference's fp32, so the
bench's mode is validated on what the training run produces.  Three runs of the same neutron 44x44
E=1 train loop, B=64, 20 steps, identical seeds, data batches and injected noise:
  * ORC — the oracle (torch CPU fp32 restatement pinned bit-exactly to the reference's goldens);
  * F32 — the HIP path in fp32 parity mode;
  * B16 — the HIP path in bf16 mode (what bench.py measures).

Checked (tolerances from the measured spread):
  1. loss trajectories: for each of gen / disc / div / intensity / aux losses,
     max_step |run_s - ORC_s| / mean_step |ORC_s|  <=  TRAJ_TOL[run];
  2. generated photon-sum / 5-channel-sum distributions after training (eval-mode generators, 1024
     fixed conditions and noise, expm1 -> the reference's channel sums, train/utils.py:62-78):
     the per-channel Wasserstein distance between a run and ORC, relative to ORC's channel mean,
     <= WS_TOL[run]; for scale, the natural spread is the same distance between two ORC
     generations with independent noise (printed).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, STEPS, N_EVAL = 64, 20, 1024
KEYS = ("gen_loss", "disc_loss", "div_loss", "intensity_loss", "aux_reg_loss")
# measured on MI355X: trajectory max-dev fp32 0.008-0.014 / bf16 0.039-0.052 (gen_loss, the
# largest); WS/mean fp32 0.013-0.015 (one run of the same build 0.045) / bf16 0.011-0.069, natural
# spread of two oracle noise draws 0.0082.  The 20-step GAN trajectory is chaotic: builds that
# change only the rounding of a reduction (BN statistics merge order, spectral-norm mat-vec order)
# moved the bf16 WS between 0.011 and 0.069 with the same seeds, and float-atomic reductions make
# even two runs of one fp32 build differ (0.015, 0.015, 0.045 on one box), so the WS bounds sit
# above those measured spreads while the trajectory bounds stay tight
TRAJ_TOL = {"fp32": 0.02, "bf16": 0.08}
WS_TOL = {"fp32": 0.06, "bf16": 0.10}


def _inputs():
    from expertsim.utils.synthetic import make_batch
    gen = torch.Generator().manual_seed(11)
    steps = []
    for s in range(STEPS):
        b = {k: torch.from_numpy(v) for k, v in make_batch(B, "neutron", seed=500 + s).items()}
        noise = {(0, w): torch.randn(B, 10, generator=gen) for w in (0, 1)}
        gum = torch.empty(B, 1).exponential_(generator=gen)
        steps.append((b, noise, gum))
    ev = make_batch(N_EVAL, "neutron", seed=900)
    eval_cond = torch.from_numpy(ev["cond"])
    eval_noise = [torch.randn(N_EVAL, 10, generator=gen) for _ in range(2)]
    return steps, eval_cond, eval_noise


def _hip_run(precision, steps, eval_cond, eval_noise):
    import bench
    moe, (og, od, oa, orr), cfg = bench.build("neutron", 1, precision, 1234, torch.device(DEV))
    traj = []
    for b, noise, gum in steps:
        moe.noise_fn = lambda e, w, shape, _n=noise: _n[(e, w)]
        moe.gumbel_fn = lambda shape, _g=gum: _g
        t = lambda k: b[k].to(DEV)
        m = moe.train_step(0, t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"),
                           t("intensity"), oa, og, od, orr, None, DEV)
        traj.append({k: float(m[k]) for k in KEYS})
    with torch.no_grad():
        img, _ = moe.generators[0].fwd(eval_noise[0].to(DEV), eval_cond.to(DEV), train=False)
        x = img.torch_nchw().float().cpu().numpy()[:, 0]
    return traj, x


def _oracle_run(steps, eval_cond, eval_noise):
    from oracle import expertsim_oracle as O
    m = O.OracleMoE("neutron", 1, dict(O.DEFAULT_CFG), seed=1234)
    traj = []
    for b, noise, gum in steps:
        met, _ = m.train_step(0, b["cond"], b["real_images"].unsqueeze(1), b["true_positions"], b["std"],
                              b["intensity"], lambda e, w, shape, _n=noise: _n[(e, w)], gum)
        traj.append({k: met[k] for k in KEYS})
    with torch.no_grad():
        P = m.state["G"][0]
        xs = [O.generator_forward("neutron", P, n, eval_cond, training=False)[:, 0].numpy() for n in eval_noise]
    return traj, xs


def _ws_rel(x, ref):
    from oracle import expertsim_oracle as O
    a, r = O.channel_sums(np.expm1(x.astype(np.float64))), O.channel_sums(np.expm1(ref.astype(np.float64)))
    return max(O.wasserstein_1d(a[:, i], r[:, i]) / max(abs(r[:, i].mean()), 1e-9) for i in range(5))


@pytest.mark.timeout(400)
def test_bf16_training_statistics_match_fp32_and_oracle():
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    steps, eval_cond, eval_noise = _inputs()
    orc, orc_x = _oracle_run(steps, eval_cond, eval_noise)
    runs = {p: _hip_run(p, steps, eval_cond, eval_noise) for p in ("fp32", "bf16")}
    natural = _ws_rel(orc_x[1], orc_x[0])
    report = {}
    for p, (traj, x) in runs.items():
        dev = {}
        for k in KEYS:
            ref = np.array([s[k] for s in orc])
            mine = np.array([s[k] for s in traj])
            dev[k] = float(np.max(np.abs(mine - ref)) / max(np.mean(np.abs(ref)), 1e-12))
        ws = _ws_rel(x, orc_x[0])
        report[p] = (dev, ws)
        print(f"{p}: trajectory max-dev / mean|ref| {dev}; WS(run, ORC)/mean {ws:.4g}; "
              f"natural WS(ORC noise a, b)/mean {natural:.4g}")
    for p, (dev, ws) in report.items():
        for k, d in dev.items():
            assert d <= TRAJ_TOL[p], (p, k, d)
        assert ws <= WS_TOL[p], (p, ws, natural)


# ---------------------------------------------------------------------------------------------
# B = 512 (BASELINE configs[1]): the bf16 mode as one more sample of the same training process.
# Three HIP runs, 12 steps each, same init and data: F32a and B16a see the same injected noise /
# Gumbel draws, F32b another draw of them.  The natural spread of the training process is
# WS(F32b, F32a): the same fp32 training (pinned to the reference at this batch size by
# tests/test_b512_gpu.py) with only its random noise changed (F32b, F32c: two other draws, averaged).
# The bf16 run must stay within 3x of it: WS(B16a, F32a) <= 3 * mean(WS(F32b, F32a), WS(F32c, F32a))
# (per channel, relative to the channel mean; eval-mode
# generations of 4096 fixed conditions / noises), and likewise its loss trajectory.  Measured (r03j):
# WS 0.0428 vs natural 0.0182 (2.35x); trajectory 0.0107 vs natural 0.0572.
B512, STEPS512, EVAL512 = 512, 12, 4096


def _inputs512(noise_seed):
    from expertsim.utils.synthetic import make_batch
    gen = torch.Generator().manual_seed(noise_seed)
    steps = []
    for s in range(STEPS512):
        b = {k: torch.from_numpy(v) for k, v in make_batch(B512, "neutron", seed=700 + s).items()}
        noise = {(0, w): torch.randn(B512, 10, generator=gen) for w in (0, 1)}
        gum = torch.empty(B512, 1).exponential_(generator=gen)
        steps.append((b, noise, gum))
    return steps


@pytest.mark.timeout(400)
def test_bf16_training_statistics_b512():
    from expertsim.utils.synthetic import make_batch
    ev = make_batch(EVAL512, "neutron", seed=901)
    eval_cond = torch.from_numpy(ev["cond"])
    eval_noise = [torch.randn(EVAL512, 10, generator=torch.Generator().manual_seed(13))]
    sa, sb, sc = _inputs512(21), _inputs512(22), _inputs512(23)
    f32a = _hip_run("fp32", sa, eval_cond, eval_noise)
    f32b = _hip_run("fp32", sb, eval_cond, eval_noise)
    f32c = _hip_run("fp32", sc, eval_cond, eval_noise)
    b16a = _hip_run("bf16", sa, eval_cond, eval_noise)

    def traj_dev(run, ref):
        return max(float(np.max(np.abs(np.array([s[k] for s in run[0]]) - np.array([s[k] for s in ref[0]])))
                         / max(np.mean(np.abs([s[k] for s in ref[0]])), 1e-12)) for k in KEYS)
    # the natural spread as the mean over two other noise draws (one draw's WS is itself a noisy
    # estimate: r03 measured 0.0158 and 0.0182 for the same pair of seeds on two fp32 builds)
    natural_ws = 0.5 * (_ws_rel(f32b[1], f32a[1]) + _ws_rel(f32c[1], f32a[1]))
    natural_traj = 0.5 * (traj_dev(f32b, f32a) + traj_dev(f32c, f32a))
    ws = _ws_rel(b16a[1], f32a[1])
    tr = traj_dev(b16a, f32a)
    print(f"B=512: WS(bf16, fp32)/mean {ws:.4g} vs natural WS(fp32 noise b, a) {natural_ws:.4g}; "
          f"trajectory dev bf16 {tr:.4g} vs natural {natural_traj:.4g}")
    assert ws <= 3.0 * natural_ws, (ws, natural_ws)
    assert tr <= 3.0 * natural_traj, (tr, natural_traj)
