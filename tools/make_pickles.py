"""Write a small dataset in the reference's on-disk format (three pandas pickles, neutron schema)
from the synthetic generator, for end-to-end runs of cli.py with dataset.source=pickle.

usage: python tools/make_pickles.py OUT_DIR [N]"""
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
from expertsim.utils.data_transformations import COND_COLUMNS  # noqa: E402
from expertsim.utils.synthetic import make_batch  # noqa: E402


def main(out, n=1200):
    os.makedirs(out, exist_ok=True)
    b = make_batch(n, "neutron", seed=5)
    rng = np.random.default_rng(5)
    cond = pd.DataFrame(rng.normal(size=(n, 9)).round(2), columns=COND_COLUMNS)
    cond["std"] = rng.uniform(0, 5, n)
    cond["neutron_photon_sum"] = b["intensity"][:, 0].astype(np.float64)
    cond["group_number"] = rng.integers(0, 3, n)
    pos = pd.DataFrame({"max_x": b["true_positions"][:, 0], "max_y": b["true_positions"][:, 1]})
    pd.to_pickle(b["real_images"], os.path.join(out, "images.pkl"))
    cond.to_pickle(os.path.join(out, "cond.pkl"))
    pos.to_pickle(os.path.join(out, "pos.pkl"))
    print("wrote", out, n)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1200)
