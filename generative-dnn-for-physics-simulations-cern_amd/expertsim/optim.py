"""Fused Adam over a model's flat parameter buffer (one HIP launch per model per step).

Drop-in for the ``torch.optim.Adam(module.parameters(), lr=...)`` objects the reference creates
in expertsim/train/training_setup.py:20-40 and steps in moe.py:439,526,565,566: same
hyper-parameters (betas 0.9/0.999, eps 1e-8, no weight decay), same update rule as torch's
single-tensor Adam, ``zero_grad`` / ``step`` / ``state_dict`` API.  Moments live in two flat
buffers whose per-parameter views are exposed as ``state[p]['exp_avg' / 'exp_avg_sq']``.

The step count lives on the device (a captured step replays it).  Inside a multi-expert step on
dynamic rows the update happens only when the expert trains, decided on the device, so the host
count is then stale: reading ``state`` or ``_step`` re-reads it from the device (one synchronisation,
never inside a graph capture); ``sync_step()`` does so explicitly.
"""
from __future__ import annotations

import torch

from . import hip


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, module, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay != 0.0:
            raise NotImplementedError("the reference uses weight_decay=0")
        self.module = module
        super().__init__(list(module.parameters()), dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0))
        self._m = self._v = None
        self._hstep = 0
        self._stale = False                # host step behind the device one (dynamic rows)
        self._step_t = torch.tensor(0.0)   # one host tensor shared by every parameter's state['step']
        self._dstep = None   # device copy of the step (read by the kernel: graph-capturable)

    # host views of the device step, re-read lazily after device-gated updates
    def _fresh(self):
        if self.__dict__.get("_stale") and not torch.cuda.is_current_stream_capturing():
            self.sync_step()

    @property
    def _step(self):
        self._fresh()
        return self._hstep

    @_step.setter
    def _step(self, v):
        self._hstep = int(v)

    @property
    def state(self):
        self._fresh()
        return self.__dict__["_opt_state"]

    @state.setter
    def state(self, v):
        self.__dict__["_opt_state"] = v

    def _buffers(self):
        flat = self.module.flat_params
        if self._m is None or self._m.numel() != flat.numel() or self._m.device != flat.device:
            self._m = torch.zeros_like(flat)
            self._v = torch.zeros_like(flat)
            o = 0
            for p in self.module.parameters():
                n = p.numel()
                self.__dict__["_opt_state"][p] = {"step": self._step_t,
                                 "exp_avg": self._m[o:o + n].view_as(p),
                                 "exp_avg_sq": self._v[o:o + n].view_as(p)}
                o += n
        return flat

    def prepare(self):
        """Create the lazily allocated state (moments, device step) now.  MoEWrapper calls this outside
        any graph capture before an expert's step may be captured: created inside a capture, the
        zero fills would be graph nodes and every replay would reset the moments and the step."""
        self._buffers()
        flat = self.module.flat_params
        if self._dstep is None or self._dstep.device != flat.device:
            self._dstep = torch.full((1,), self._hstep, dtype=torch.int32, device=flat.device)

    def zero_grad(self, set_to_none: bool = True):
        # the flat gradient buffer is kept (views stay valid); zeroing is one memset
        self.module.zero_grads()

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = None):
        flat = self._buffers()
        if grad_scale is None:
            grad_scale = getattr(self.module, "_grad_scale", 1.0)
        if self._dstep is None or self._dstep.device != flat.device:
            self._dstep = torch.full((1,), self._hstep, dtype=torch.int32, device=flat.device)
        # dynamic rows (multi-expert step): the update and the step count happen on the device only
        # when the running expert trains (hip.active_ptr); the host count is then re-read lazily
        active = hip.active_ptr()
        if active is None:
            self._hstep += 1
            self._step_t.fill_(float(self._hstep))
        else:
            self._stale = True
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        # step counter advanced and read on the device, so a captured step replays correctly
        hip.call("es_counter_add_if", hip.ptr(self._dstep), 1, active, hip.stream_ptr())
        hip.call("es_adam_dev", hip.ptr(flat), hip.ptr(self.module.flat_grads), hip.ptr(self._m), hip.ptr(self._v),
                 flat.numel(), float(g["lr"]), float(b1), float(b2), float(g["eps"]), hip.ptr(self._dstep),
                 float(grad_scale), active, hip.stream_ptr())
        self.module.invalidate()
        return None

    # ------------------------------------------------------------------ checkpointing
    def state_dict(self):
        """Flat form: {'step', 'exp_avg' [P], 'exp_avg_sq' [P], 'param_groups'} (host copies); loadable
        with torch.load(weights_only=True)."""
        self.sync_step()
        flat = self._buffers()
        return {"step": int(self._step), "numel": int(flat.numel()),
                "exp_avg": self._m.detach().cpu().clone(), "exp_avg_sq": self._v.detach().cpu().clone(),
                "param_groups": [{k: (list(v) if isinstance(v, tuple) else v) for k, v in g.items() if k != "params"}
                                 for g in self.param_groups]}

    def load_state_dict(self, sd):
        flat = self._buffers()
        if int(sd["numel"]) != flat.numel():
            raise ValueError(f"FusedAdam.load_state_dict: {sd['numel']} moments for {flat.numel()} parameters")
        self._m.copy_(sd["exp_avg"].to(flat.device))
        self._v.copy_(sd["exp_avg_sq"].to(flat.device))
        for g, src in zip(self.param_groups, sd["param_groups"]):
            g.update({k: (tuple(v) if k == "betas" else v) for k, v in src.items()})
        self._hstep, self._stale = int(sd["step"]), False
        if self._dstep is not None:          # keep the pointer a captured graph reads
            self._dstep.fill_(self._hstep)
        self._step_t.fill_(float(self._hstep))

    def sync_step(self):
        """Host step := device step (after replays of a captured train step)."""
        if self._dstep is not None:
            self._hstep = int(self._dstep.item())
            self._step_t.fill_(float(self._hstep))
        self._stale = False
        return self._hstep
