"""Capture evaluation golden vectors from the REFERENCE (run in the build container only).

Pins SURVEY.md §8(f) row 1 — the Wasserstein evaluation — against the reference's own functions:
  * get_channel_masks / sum_channels_parallel (train/utils.py:18-78) on several image shapes;
  * get_predictions_from_generator_results (train/utils.py:179-205): the generator in eval mode
    (BatchNorm running statistics, no dropout) with injected noise;
  * calculate_joint_ws_across_experts (train/utils.py:117-176) over two experts, with its
    ``torch.randn`` noise recorded so the build can replay it row by row (the rows are consumed in
    the same order whatever the generator batch size).
Generators are built as make_goldens.py builds them (torch.manual_seed(seed) before construction,
so the build reproduces the weights); BatchNorm running statistics are set from a closed-form
pattern (``running_stats`` below, restated in tests/test_eval_gpu.py) so nothing large is stored.

Output: tests/golden/eval_<arch>.npz.   Usage:  python tests/golden/make_eval_goldens.py
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_goldens as mg  # noqa: E402  (build-side helpers + reference loader, by path)

MASK_SHAPES = [(44, 44), (56, 30), (7, 5), (2, 3), (1, 1)]


def running_stats(n, expert):
    """Closed-form BatchNorm running statistics for an n-feature layer of expert `expert`."""
    i = np.arange(n, dtype=np.float64)
    mean = (0.1 * np.sin(0.37 * i + expert)).astype(np.float32)
    var = (0.75 + 0.25 * np.cos(0.11 * i + 2 * expert)).astype(np.float32)
    return mean, var


def set_running_stats(gen, expert):
    for name, m in gen.named_modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            mean, var = running_stats(m.num_features, expert)
            m.running_mean.copy_(torch.from_numpy(mean))
            m.running_var.copy_(torch.from_numpy(var))


def run(arch, ref, seed=1234, n=40, n_pred=8, n_calc=2):
    mods, _ = mg.load_reference(ref)
    for stub in ("seaborn", "wandb"):
        sys.modules.setdefault(stub, types.ModuleType(stub))
    U = mg._load_path("_ref_utils", os.path.join(ref, "expertsim", "train", "utils.py"))
    cfg = mg.load_cfg(ref, {"model.architecture": arch, "model.n_experts": 2})
    shape = tuple(mg.synthetic.image_shape(arch))
    out = {}
    for s in MASK_SHAPES:
        ms = U.get_channel_masks(np.zeros(s, dtype=np.float32))
        out[f"masks/{s[0]}x{s[1]}"] = np.stack(ms).astype(np.uint8)

    torch.manual_seed(seed)
    g0 = mods[f"{arch}.generator"](**cfg.model.generator)
    gens = [g0, copy.deepcopy(g0)]
    with torch.no_grad():
        for e, g in enumerate(gens):
            set_running_stats(g, e)

    b = mg.synthetic.make_batch(n, arch, seed=77)
    real = b["real_images"].astype(np.float32)          # [n,H,W] log1p domain, as the test loader
    cond = b["cond"].astype(np.float32)
    out["real_images"] = real
    out["cond"] = cond
    ch_org = np.array(list(U.sum_channels_parallel(np.expm1(real).reshape(-1, *shape))), dtype=np.float64)
    out["ch_org"] = ch_org
    rng = np.random.default_rng(5)
    assign = rng.permutation(n) % 2                     # 20 / 20 split over two experts
    assign[:3] = 0                                      # ... made uneven (23 / 17)
    out["assign"] = assign.astype(np.int64)

    # eval-mode predictions with injected noise
    noise = torch.from_numpy(np.random.default_rng(6).standard_normal((n_pred, 10)).astype(np.float32))
    res, raw = U.get_predictions_from_generator_results(3, n_pred, 10, torch.device("cpu"),
                                                        torch.from_numpy(cond[:n_pred]), gens[1],
                                                        shape_images=shape, input_noise=noise)
    out["pred/noise"] = noise.numpy()
    out["pred/raw"] = raw.astype(np.float32)
    out["pred/res"] = res
    out["pred/ch"] = np.array(list(U.sum_channels_parallel(res)), dtype=np.float64)

    # joint WS with recorded noise
    draws = []
    orig = torch.randn

    def rec_randn(*a, **k):
        t = orig(*a, **k)
        draws.append(t.detach().numpy().copy())
        return t
    idx = [np.where(assign == e)[0] for e in range(2)]
    torch.manual_seed(seed + 1)
    torch.randn = rec_randn
    try:
        ws = U.calculate_joint_ws_across_experts(
            n_calc, [real[ix] for ix in idx], [torch.from_numpy(cond[ix]) for ix in idx], gens, ch_org,
            [ch_org[ix] for ix in idx], 10, torch.device("cpu"), batch_size=16, n_experts=2, shape_images=shape)
    finally:
        torch.randn = orig
    out["ws/noise"] = np.concatenate(draws, 0).astype(np.float32)
    out["ws/mean"] = np.float64(ws[0])
    out["ws/std"] = np.float64(ws[1])
    out["ws/mean_exp"] = np.asarray(ws[2], dtype=np.float64)
    out["ws/std_exp"] = np.asarray(ws[3], dtype=np.float64)
    meta = dict(arch=arch, seed=seed, n=n, n_pred=n_pred, n_calc=n_calc, n_experts=2,
                mask_shapes=MASK_SHAPES, torch=torch.__version__)
    out["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"eval_{arch}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {os.path.getsize(path) / 1e3:.1f} kB; ws_mean {ws[0]:.6g} ws_std {ws[1]:.6g}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    torch.set_num_threads(1)
    for arch in ("neutron", "proton"):
        run(arch, args.ref)


if __name__ == "__main__":
    main()
