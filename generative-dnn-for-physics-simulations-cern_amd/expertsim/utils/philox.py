"""Counter-based dropout masks (host restatement of the device generator in csrc/rng.hip).

The reference draws dropout masks from torch's stateful CPU/CUDA generators
(``nn.Dropout`` in expertsim/models/neutron/generator.py:14,20,27,32,36, neutron/aux_reg.py:16,24,
32,40 and proton/aux_reg.py:24,28).  A stateful stream cannot be reproduced on the GPU, so the
build defines every mask as a pure function of (seed, stream, logical element index):

    x   = Philox4x32-10(key=(seed_lo, seed_hi), counter=(i >> 2, 0, stream, 0))[i & 3]
    keep = (x >> 8) < floor(keep_prob * 2**24)

``i`` is the element's row-major index in the reference's logical layout ([B, F] for linear
activations, [B, C, H, W] for conv activations), whatever the physical layout on the device.
The golden-capture script feeds exactly these masks to the reference, so masks are bit-exact
across reference, oracle and HIP kernels.

Stream ids (one per dropout call site, see ``dropout_stream``) are:
    stream = step * 1024 + expert * 32 + pass_id * 8 + layer        (expert < 32, layer < 8)
with pass_id 0 = generator forward #1 (moe.py:145), 1 = generator forward #2 (moe.py:538),
2 = auxiliary regressor forward (moe.py:557).  Counter word 3 is 0 for dropout; the device noise
and Gumbel draws (csrc/misc.hip randn / rand_exp) use 0x5EED0001 / 0x5EED0002 there, so the three
families never share a Philox block whatever their stream ids.

Data parallelism: the rank lives in neither the key nor the stream id but in the element index —
a rank holding samples [n0, n0 + n) of an expert's global batch (the global batch is the rank
shards in rank order, so n0 = the sum of the lower ranks' counts for that expert) draws elements
n0 * (elements per sample) onwards of the single-device draw, for dropout masks as for noise and
Gumbel draws (es_dropout_t.index_offset, es_randn_dev / es_rand_exponential_dev ``offset``).  Ranks
therefore draw independent masks and noise, and together exactly the single-device ones.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

PASS_G1, PASS_G2, PASS_AUX = 0, 1, 2


def dropout_stream(step: int, expert: int, pass_id: int, layer: int) -> int:
    if not (0 <= expert < 32 and 0 <= pass_id < 4 and 0 <= layer < 8):
        raise ValueError(f"dropout_stream: expert {expert} / pass {pass_id} / layer {layer} out of range")
    return int(step) * 1024 + int(expert) * 32 + int(pass_id) * 8 + int(layer)


def keep_threshold(p: float) -> int:
    """Integer threshold on the top 24 bits: keep iff (x >> 8) < threshold."""
    return int(np.floor((1.0 - float(p)) * 16777216.0))


def philox4x32(ctr0, ctr1, ctr2, ctr3, key0: int, key1: int):
    """Vectorised Philox4x32-10 over uint32 arrays; returns four uint32 arrays."""
    c0 = np.asarray(ctr0, dtype=np.uint64)
    c1 = np.asarray(ctr1, dtype=np.uint64) + np.zeros_like(c0)
    c2 = np.asarray(ctr2, dtype=np.uint64) + np.zeros_like(c0)
    c3 = np.asarray(ctr3, dtype=np.uint64) + np.zeros_like(c0)
    k0 = np.uint64(key0 & 0xFFFFFFFF)
    k1 = np.uint64(key1 & 0xFFFFFFFF)
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(W0)) & MASK32
            k1 = (k1 + np.uint64(W1)) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32),
            c3.astype(np.uint32))


def random_bits(n: int, seed: int, stream: int, offset: int = 0) -> np.ndarray:
    """uint32 word for each logical element index offset .. offset+n-1."""
    q = np.arange(offset // 4, (offset + n + 3) // 4, dtype=np.uint64)
    words = philox4x32(q & MASK32, q >> np.uint64(32), np.uint64(stream & 0xFFFFFFFF), 0,
                       seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    flat = np.stack(words, axis=1).reshape(-1)       # element i = word (i & 3) of counter i >> 2
    s = offset % 4
    return flat[s:s + n]


def dropout_mask(shape, p: float, seed: int, stream: int, n_offset: int = 0) -> np.ndarray:
    """Boolean keep-mask of ``shape`` (logical row-major element order); ``n_offset``: index of the
    tensor's first sample in the global batch (rows n_offset.. of the mask of the whole batch)."""
    n = int(np.prod(shape))
    per = n // shape[0] if shape[0] else 0
    x = random_bits(n, seed, stream, int(n_offset) * per)
    return ((x >> np.uint32(8)) < np.uint32(keep_threshold(p))).reshape(shape)
