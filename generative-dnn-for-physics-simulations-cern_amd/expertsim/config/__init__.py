"""Config loading with the reference's YAML schema (expertsim/config/default.yaml) and OmegaConf
semantics where they matter (cli.py:58-97): ``1e-4``-style strings become floats, ``a.b=c``
overrides are parsed as YAML scalars, and the loop.py:336-342 sub-config injection is applied by
``inject_shared``.  hydra/omegaconf are not installed here, so this is a small attribute-dict."""
from __future__ import annotations

import os

import yaml

DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "default.yaml")


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def get_path(self, path, default=None):
        node = self
        for p in path.split("."):
            if not isinstance(node, dict) or p not in node:
                return default
            node = node[p]
        return node


def _coerce(v):
    if isinstance(v, dict):
        return AttrDict({k: _coerce(x) for k, x in v.items()})
    if isinstance(v, list):
        return [_coerce(x) for x in v]
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return v
    return v


def load_config(path: str = DEFAULT_PATH, overrides=()):
    with open(path) as f:
        cfg = _coerce(yaml.safe_load(f))
    for ov in overrides or ():
        key, _, val = ov.partition("=")
        node = cfg
        parts = key.strip().split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, AttrDict())
        node[parts[-1]] = _coerce(yaml.safe_load(val))
    return cfg


def inject_shared(cfg):
    """expertsim/train/loop.py:336-342."""
    m = cfg.model
    m.generator.noise_dim = m.noise_dim
    m.generator.cond_dim = m.cond_dim
    m.generator.n_experts = m.n_experts
    m.discriminator.cond_dim = m.cond_dim
    m.discriminator.n_experts = m.n_experts
    m.router.cond_dim = m.cond_dim
    m.router.n_experts = m.n_experts
    return cfg


def cfg_get(cfg, path, default=None):
    node = cfg
    for p in path.split("."):
        try:
            node = node[p] if isinstance(node, dict) else getattr(node, p)
        except (KeyError, AttributeError):
            return default
    return node
