"""Synthetic ZDC batches (the reference ships no data).

The reference reads GEANT4 pickles (expertsim/utils/data_transformations.py:23-129) and yields
6-tuples ``(real_images, real_images_2, cond, std, intensity, true_positions)``
(data_transformations.py:260-309, consumed at expertsim/train/loop.py:170).  This module
produces batches of the same shapes and value ranges, seeded and host-side (numpy), so the
same bytes can be fed to the oracle, the HIP path and the golden-capture script:

* raw[b,h,w] = Bernoulli(rho) * ceil(LogNormal(1.0, 1.2)), clipped to the notebook maxima
  (591 for ZN 44x44, 765 for ZP 56x30); at least one non-zero pixel per image
  (MIN_INTENSITY_THRESHOLD = 1, default.yaml:43);
* real_images = log1p(raw)                       (data_filtering.ipynb, log transform)
* intensity   = sum(raw)                          [B,1]
* true_positions = (row, col) of argmax(raw)      [B,2] (train/utils.py:81-82)
* std ~ U(0,1) [B,1], cond ~ N(0,1) [B,9]         (MinMax / StandardScaler outputs)
"""
from __future__ import annotations

import numpy as np

# "neutron56": BASELINE configs[4]'s padded 56x56 extension: a 44x44 ZN
# response zero-padded to 56x56 keeps its photons, so the hit density scales by 44^2 / 56^2
_SHAPES = {"neutron": (44, 44), "proton": (56, 30), "neutron56": (56, 56)}
_RHO = {"neutron": 0.039, "proton": 0.011, "neutron56": 0.039 * 44 * 44 / (56 * 56)}
_CLIP = {"neutron": 591.0, "proton": 765.0, "neutron56": 765.0}


def image_shape(architecture: str) -> tuple:
    return _SHAPES[architecture]


def make_batch(batch_size: int, architecture: str = "neutron", seed: int = 0,
               cond_dim: int = 9, shape=None):
    """Return a dict of float32 numpy arrays for one batch.

    ``shape`` overrides the image shape (used by the 56x56 throughput-only extension).
    """
    rng = np.random.default_rng(seed)
    H, W = shape if shape is not None else _SHAPES[architecture]
    rho = _RHO.get(architecture, 0.039)
    clip = _CLIP.get(architecture, 765.0)
    hits = rng.random((batch_size, H, W)) < rho
    amp = np.ceil(rng.lognormal(mean=1.0, sigma=1.2, size=(batch_size, H, W)))
    raw = np.where(hits, np.minimum(amp, clip), 0.0)
    # enforce at least one photon per image
    empty = raw.reshape(batch_size, -1).sum(1) == 0
    if empty.any():
        idx = np.nonzero(empty)[0]
        flat = rng.integers(0, H * W, size=idx.size)
        raw.reshape(batch_size, -1)[idx, flat] = 1.0
    raw = raw.astype(np.float32)
    real = np.log1p(raw).astype(np.float32)
    intensity = raw.reshape(batch_size, -1).sum(1, keepdims=True).astype(np.float32)
    am = raw.reshape(batch_size, -1).argmax(1)
    pos = np.stack([am // W, am % W], axis=1).astype(np.float32)
    std = rng.random((batch_size, 1)).astype(np.float32)
    cond = rng.standard_normal((batch_size, cond_dim)).astype(np.float32)
    return {
        "real_images": real,          # [B,H,W] (loop.py unsqueezes to [B,1,H,W])
        "cond": cond,
        "std": std,
        "intensity": intensity,
        "true_positions": pos,
    }
