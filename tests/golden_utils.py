"""Helpers to read the reference golden vectors (tests/golden/*.npz, see make_goldens.py)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["neutron_e1_b8", "neutron_e3_b12", "proton_e1_b8", "proton_e3_b12", "neutron_e3_b12_router"]
# BASELINE batch sizes, compact (module outputs > 4096 values as checksums; inputs regenerated)
LARGE_CASES = ["neutron_e1_b512", "neutron_e1_b1024"]


class Golden:
    def __init__(self, case):
        self.case = case
        self.z = np.load(os.path.join(GOLDEN_DIR, f"{case}.npz"), allow_pickle=False)
        self.meta = json.loads(str(self.z["meta"]))
        self.arch = self.meta["arch"]
        self.E = self.meta["n_experts"]
        self.B = self.meta["batch"]
        self.steps = self.meta["steps"]
        self.seed = self.meta["seed"]
        self.epoch = self.meta["epoch"]

    def overrides(self):
        """The case's config overrides as load_config strings (``model.router.x=v``)."""
        return [f"{k}={v}" for k, v in self.meta.get("overrides", {}).items()
                if k not in ("model.architecture", "model.n_experts", "train.batch_size")]

    def oracle_cfg(self, base):
        """Flat oracle config (oracle.DEFAULT_CFG keys) with the case's router overrides applied."""
        cfg = dict(base)
        for k, v in self.meta.get("overrides", {}).items():
            leaf = k.split(".")[-1]
            if k.startswith("model.router.") and leaf in cfg:
                cfg[leaf] = float(v)
        return cfg

    def __getitem__(self, k):
        return self.z[k]

    def has(self, k):
        return k in self.z.files

    def keys(self, prefix):
        return [k for k in self.z.files if k.startswith(prefix)]

    def inputs(self, step):
        p = f"s{step}/in/"
        out = {k[len(p):]: self.z[k] for k in self.keys(p)}
        if out or not self.meta.get("compact"):
            return out
        # compact cases: the batch is regenerated from the same synthetic source and pinned by the
        # checksums the capture recorded (bit-exact: numpy's seeded generator)
        from expertsim.utils.synthetic import make_batch
        b = make_batch(self.B, self.arch, seed=self.meta["data_seed"] + step)
        for k, v in b.items():
            want = self.z[f"s{step}/in_ck/{k}"]
            assert np.array_equal(checksum(v), want), f"{self.case}: regenerated input {k} differs"
        return b

    def router_idx(self, step):
        gates = self.z[f"s{step}/R/call0/out0"]
        return gates.argmax(1)

    def noise(self, step):
        """(expert, which) -> recorded torch.randn draw, mapped by reference call order."""
        if not self.has(f"s{step}/R/call0/out0"):
            # compact cases (router output as a checksum): the capture's event order pairs each
            # draw with the generator call that follows it
            out, pending = {}, []
            for ev in self.meta["events"]:
                if ev[0] != step:
                    continue
                if ev[1] == "randn":
                    pending.append(ev[2])
                elif ev[1].startswith("G") and pending:
                    e = int(ev[1][1:])
                    out[(e, ev[2])] = self.z[f"s{step}/randn{pending.pop(0)}"]
            return out
        idx = self.router_idx(step)
        out, k = {}, 0
        for e in range(self.E):
            if (idx == e).sum() <= 1:
                continue
            for which in (0, 1):
                out[(e, which)] = self.z[f"s{step}/randn{k}"]
                k += 1
        return out

    def gumbel(self, step):
        return self.z[f"s{step}/gumbel_exp"]

    def metrics(self, step):
        p = f"s{step}/metric/"
        return {k[len(p):]: float(self.z[k]) for k in self.keys(p)}


def checksum(a):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    n = a.size
    idx = (np.arange(64) * n) // 64 if n >= 64 else np.arange(n)
    return np.concatenate([[a.sum(), np.abs(a).sum(), np.sqrt((a * a).sum())], a[idx]])


def rel_err(a, b, floor=1e-12):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), floor))
