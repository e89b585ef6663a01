"""Device random numbers (Philox4x32-10 counter streams) replacing torch.randn (moe.py:144,535)
and the Exp(1) draws inside F.gumbel_softmax (router.py:23).  Each call consumes a fresh stream id,
so no generator state lives on the device."""
from __future__ import annotations

import torch

from . import hip


class DeviceRNG:
    def __init__(self, seed: int = 1234, stream_base: int = 1 << 24):
        self.seed = int(seed)
        self.counter = int(stream_base)

    def _next(self):
        self.counter += 1
        return self.counter & 0xFFFFFFFF

    def normal(self, out: torch.Tensor):
        hip.require_device(out)
        hip.call("es_randn", hip.ptr(out), out.numel(), self.seed, self._next(), hip.stream_ptr())
        return out

    def exponential(self, out: torch.Tensor):
        hip.require_device(out)
        hip.call("es_rand_exponential", hip.ptr(out), out.numel(), self.seed, self._next(), hip.stream_ptr())
        return out


_default = None


def default_rng() -> DeviceRNG:
    global _default
    if _default is None:
        _default = DeviceRNG(torch.initial_seed())
    return _default
