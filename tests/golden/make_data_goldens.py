"""Capture data-pipeline golden vectors from the REFERENCE (run in the build container only).

Pins SURVEY.md §8(f) row 2 — the on-disk data format and its preparation — against the
reference's own functions, get_dataset and transform_data_for_training
(expertsim/utils/data_transformations.py:23-257), loaded by path.  Each case builds small
synthetic DataFrames of the reference's column schema (6x5 images keep the fixture small; the
pipeline is shape-agnostic), writes them as pickles into a temporary directory (files this script
wrote itself), seeds numpy's global RNG and runs the reference.  Inputs and every output array go
into tests/golden/data_pipeline.npz; tests/test_data_pipeline_cpu.py replays the same inputs
through the build's pipeline under the same seed.

Usage:  python tests/golden/make_data_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_goldens as mg  # noqa: E402  (reference loader by path, AttrDict)

COND = ["Energy", "Vx", "Vy", "Vz", "Px", "Py", "Pz", "mass", "charge"]

# name: (zdc_type, n, seed, MIN, MAX, read_n_samples, limit_samples, shuffle)
CASES = {
    "neutron_basic": ("neutron", 240, 11, 1, 4000, None, None, True),
    "proton_uniform": ("proton", 240, 12, 1, None, 150, None, True),
    "neutron_noshuffle_limit": ("neutron", 240, 13, None, None, None, 200, False),
}


def make_inputs(zdc, n, seed):
    """Seeded frames in the reference schema; conditions drawn from a small set so that
    same-condition groups (the partner pairing) are non-trivial."""
    rng = np.random.default_rng(seed)
    levels = rng.normal(size=(12, len(COND))).round(3)
    cond = levels[rng.integers(0, 12, size=n)]
    cond[:, 7] = np.abs(cond[:, 7])
    photon_sum = np.floor(rng.lognormal(5.0, 1.5, size=n))
    photon_sum[rng.integers(0, n, size=10)] = 0.0            # fall below MIN_INTENSITY_THRESHOLD
    std = rng.uniform(0.1, 9.0, size=n)
    group = rng.integers(0, 4, size=n)
    images = np.log1p(rng.poisson(0.4, size=(n, 6, 5))).astype(np.float32)
    pos = rng.integers(0, 44, size=(n, 2)).astype(np.float64)
    out = {"cond": cond, "photon_sum": photon_sum, "std": std, "group": group, "images": images, "pos": pos}
    if zdc == "proton":
        out["expert_number"] = rng.integers(0, 3, size=n)
    return out


def frames(zdc, inp):
    import pandas as pd
    cols = {c: inp["cond"][:, i] for i, c in enumerate(COND)}
    if zdc == "proton":
        cols.update({"std_proton": inp["std"], "proton_photon_sum": inp["photon_sum"],
                     "group_number_proton": inp["group"], "expert_number": inp["expert_number"]})
    else:
        cols.update({"std": inp["std"], "neutron_photon_sum": inp["photon_sum"], "group_number": inp["group"]})
    return inp["images"], pd.DataFrame(cols), pd.DataFrame({"max_x": inp["pos"][:, 0], "max_y": inp["pos"][:, 1]})


def write_pickles(tmp, zdc, inp):
    import pandas as pd
    images, cond, pos = frames(zdc, inp)
    paths = [os.path.join(tmp, f) for f in ("images.pkl", "cond.pkl", "pos.pkl")]
    pd.to_pickle(images, paths[0])
    cond.to_pickle(paths[1])
    pos.to_pickle(paths[2])
    return paths


def case_cfg(zdc, paths, lo, hi, n_samples, limit, shuffle, tmp):
    A = mg.AttrDict
    return A(limit_samples=limit,
             config=A(run_name="golden", experiment_dir=os.path.join(tmp, "exp")),
             dataset=A(zdc_type=zdc, DATA_IMAGES_PATH=paths[0], DATA_COND_PATH=paths[1],
                       DATA_POSITIONS_PATH=paths[2], MIN_INTENSITY_THRESHOLD=lo,
                       MAX_INTENSITY_THRESHOLD=hi, read_n_samples=n_samples,
                       shuffle_train_test_split=shuffle, test_size=0.2),
             train=A(save_experiments_dir=tmp, checkpoint_experiment_dir=None, epoch_to_load=None,
                     save_experiment_data=False))


OUT_NAMES = ["x_train", "x_test", "x2_train", "x2_test", "cond_train", "cond_test", "std_train", "std_test",
             "intensity_train", "intensity_test", "pos_train", "pos_test", "expert_train", "expert_test"]


def main(ref="/root/reference"):
    mg.load_reference(ref)
    D = mg._load_path("_ref_data", os.path.join(ref, "expertsim", "utils", "data_transformations.py"))
    fixture, meta = {}, {}
    for name, (zdc, n, seed, lo, hi, ns, limit, shuffle) in CASES.items():
        inp = make_inputs(zdc, n, seed)
        for k, v in inp.items():
            fixture[f"{name}/in/{k}"] = v
        with tempfile.TemporaryDirectory() as tmp:
            paths = write_pickles(tmp, zdc, inp)
            cfg = case_cfg(zdc, paths, lo, hi, ns, limit, shuffle, tmp)
            np.random.seed(1000 + seed)
            data, data_cond, data_posi = D.get_dataset(cfg)
            out = D.transform_data_for_training(cfg, data, data_cond, data_posi)
        for k, v in zip(OUT_NAMES, out[:14]):
            fixture[f"{name}/out/{k}"] = np.asarray(v)
        meta[name] = {"zdc": zdc, "seed": 1000 + seed, "MIN": lo, "MAX": hi, "read_n_samples": ns,
                      "limit_samples": limit, "shuffle": shuffle, "names": list(out[15]),
                      "photon_sum_min": cfg.photon_sum_min, "photon_sum_max": cfg.photon_sum_max}
    fixture["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, "data_pipeline.npz")
    np.savez_compressed(path, **fixture)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
