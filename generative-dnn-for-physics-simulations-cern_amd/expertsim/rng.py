"""Device random numbers (Philox4x32-10 counter streams) replacing torch.randn (moe.py:144,535)
and the Exp(1) draws inside F.gumbel_softmax (router.py:23).  Each call consumes a fresh stream id,
so no generator state lives on the device.

Inside a train step (``begin_step(counter)``) the stream id of the i-th draw is
``stream_base + i + counter[0] * 256``, the step term added on the device: a captured HIP graph
of the step draws new numbers at every replay.  Every rank of a data-parallel run issues the same
sequence of draws (same stream ids) and takes its own rows of each through the element offset."""
from __future__ import annotations

import torch

from . import hip

STEP_MUL = 256   # draws per step stay below this


class DeviceRNG:
    def __init__(self, seed: int = 1234, stream_base: int = 1 << 24):
        self.seed = int(seed)
        self.stream_base = int(stream_base)
        self.counter = int(stream_base)
        self.step_counter = None
        self.calls = 0

    def begin_step(self, step_counter: torch.Tensor):
        """Key the following draws on a device step counter (int32 [1])."""
        self.step_counter = step_counter
        self.calls = 0

    def end_step(self):
        self.step_counter = None

    def _next(self):
        self.counter += 1
        return self.counter & 0xFFFFFFFF

    def _draw(self, name, out, offset=0):
        hip.require_device(out)
        if self.step_counter is not None:
            if self.calls >= STEP_MUL:
                raise RuntimeError("DeviceRNG: more than %d draws in one step" % STEP_MUL)
            sid = (self.stream_base + self.calls) & 0xFFFFFFFF
            self.calls += 1
            hip.call(name + "_dev", hip.ptr(out), out.numel(), self.seed, sid, hip.ptr(self.step_counter), STEP_MUL,
                     int(offset), hip.stream_ptr())
        else:
            hip.call(name + "_dev", hip.ptr(out), out.numel(), self.seed, self._next(), None, 0, int(offset),
                     hip.stream_ptr())
        return out

    def _draw_at(self, name, out, index, offset=0):
        """Draw on the step's stream ``stream_base + index`` (a fixed id per call site, so a captured
        per-expert graph draws the same stream whatever other experts ran)."""
        hip.require_device(out)
        if self.step_counter is None:
            return self._draw(name, out, offset)
        if not 0 <= index < STEP_MUL:
            raise RuntimeError("DeviceRNG: stream index %d outside [0, %d)" % (index, STEP_MUL))
        hip.call(name + "_dev", hip.ptr(out), out.numel(), self.seed, (self.stream_base + index) & 0xFFFFFFFF,
                 hip.ptr(self.step_counter), STEP_MUL, int(offset), hip.stream_ptr())
        return out

    def normal_at(self, out: torch.Tensor, index: int, offset: int = 0, off_ptr: torch.Tensor = None,
                  off_mul: int = 0):
        """off_ptr (device int32 [1]): the element offset is offset + off_ptr[0] * off_mul, read on the
        device (a data-parallel rank's first sample of an expert under dynamic rows)."""
        if off_ptr is None:
            return self._draw_at("es_randn", out, index, offset)
        hip.require_device(out)
        if self.step_counter is None:
            sid, sp, mul = self._next(), None, 0
        else:
            if not 0 <= index < STEP_MUL:
                raise RuntimeError("DeviceRNG: stream index %d outside [0, %d)" % (index, STEP_MUL))
            sid, sp, mul = (self.stream_base + index) & 0xFFFFFFFF, hip.ptr(self.step_counter), STEP_MUL
        hip.call("es_randn_dev_at", hip.ptr(out), out.numel(), self.seed, sid, sp, mul, int(offset),
                 hip.ptr(off_ptr), int(off_mul), hip.stream_ptr())
        return out

    def exponential_at(self, out: torch.Tensor, index: int, offset: int = 0):
        return self._draw_at("es_rand_exponential", out, index, offset)

    def normal(self, out: torch.Tensor, offset: int = 0):
        """out[i] = draw number offset + i of this call's stream (offset even): a data-parallel rank
        passes its first global row x row length and draws exactly its rows of the global draw."""
        return self._draw("es_randn", out, offset)

    def exponential(self, out: torch.Tensor, offset: int = 0):
        return self._draw("es_rand_exponential", out, offset)


_default = None


def default_rng() -> DeviceRNG:
    global _default
    if _default is None:
        _default = DeviceRNG(torch.initial_seed())
    return _default
