"""EMA of the generators' weights — reference: EMAHelper (expertsim/train/loop.py:380-418).

Same API (``EMAHelper(moe, decay)``, ``update(moe, updated_indices)``, ``apply_shadow(moe)``,
``restore(moe)``, ``.shadow[i][name]``, ``.decay``).  The shadow of each generator is ONE flat fp32
buffer laid out like the generator's flat parameter storage (expertsim/models/base.py), so an
update is a single ``es_ema_update`` launch per generator (HBM-bound: 12 bytes per parameter) and
``shadow[i][name]`` are views into it.  The arithmetic is the reference's:
``decay*shadow + (1-decay)*param`` with both products rounded before the add.
Swapping weights copies into the flat parameter buffers in place (the HIP ops keep their
pointers) and invalidates the packed GEMM weights.
"""
from __future__ import annotations

import torch

from .. import hip


class EMAHelper:
    def __init__(self, moe, decay: float = 0.999):
        self.decay = decay
        self._flat = {}
        self.shadow = {}
        self.backup = {}
        for i, gen in enumerate(moe.generators):
            flat = gen.flat_params
            self._flat[i] = flat.detach().clone()
            self.shadow[i] = self._views(gen, self._flat[i])

    @staticmethod
    def _views(gen, flat):
        out, o = {}, 0
        for name, p in gen.named_parameters():
            n = p.numel()
            if p.requires_grad:
                out[name] = flat[o:o + n].view_as(p)
            o += n
        return out

    def update(self, moe, updated_indices):
        """Update EMA only for generators that got an optimizer step (loop.py:392-400)."""
        for i in updated_indices:
            flat = moe.generators[i].flat_params
            s = self._flat[i]
            hip.require_device(s)
            hip.call("es_ema_update", hip.ptr(s), hip.ptr(flat), flat.numel(), float(self.decay),
                     float(1.0 - self.decay), hip.stream_ptr())

    def apply_shadow(self, moe):
        """Swap all generators to the EMA weights (for evaluation)."""
        self.backup = {}
        for i, gen in enumerate(moe.generators):
            flat = gen.flat_params
            self.backup[i] = flat.detach().clone()
            flat.copy_(self._flat[i])
            gen.invalidate()

    def restore(self, moe):
        """Restore the training weights after evaluation."""
        for i, gen in enumerate(moe.generators):
            if i in self.backup:
                gen.flat_params.copy_(self.backup[i])
                gen.invalidate()
        self.backup = {}

    def state_dict(self):
        return {"decay": self.decay, "shadow": {i: f.detach().cpu().clone() for i, f in self._flat.items()}}

    def load_state_dict(self, sd):
        self.decay = sd["decay"]
        for i, f in sd["shadow"].items():
            self._flat[int(i)].copy_(f.to(self._flat[int(i)].device))
