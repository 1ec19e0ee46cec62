"""Deterministic, portable, name-keyed parameter values.

``param_values(cfg, seed)`` gives every tensor of the model a value that depends only on
(seed, parameter name, element index) through numpy's PCG64 stream — the same on every host —
so the reference model (fixture generator), the CPU oracle and the HIP model can be loaded with
identical weights without shipping a 1.8 GB weight file.

``init_values(cfg, seed)`` is the reference's own initialisation scheme (BertPreTrainedModel.
init_weights, vilbert_k3m.py:1940-1951: N(0, initializer_range) for Linear/Embedding weights,
zero biases, LayerNorm 1/0), used for training from scratch.
"""
import zlib

import numpy as np

from .params import param_spec


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


def _is_ln(name):
    return "LayerNorm" in name


def param_values(cfg, seed=1234, std=0.02, bias_std=0.02, ln_std=0.05):
    """Test weights: non-trivial biases and LayerNorm affine params so every path is exercised."""
    out = {}
    for name, shape in param_spec(cfg):
        g = _rng(seed, name)
        if _is_ln(name) and name.endswith(".weight"):
            a = 1.0 + ln_std * g.standard_normal(shape, dtype=np.float32)
        elif name.endswith(".bias") or _is_ln(name):
            a = bias_std * g.standard_normal(shape, dtype=np.float32)
        else:
            a = std * g.standard_normal(shape, dtype=np.float32)
        out[name] = np.ascontiguousarray(a, dtype=np.float32)
    return out


def init_values(cfg, seed=0):
    out = {}
    std = getattr(cfg, "initializer_range", 0.02)
    for name, shape in param_spec(cfg):
        if _is_ln(name):
            a = np.ones(shape, np.float32) if name.endswith(".weight") else np.zeros(shape, np.float32)
        elif name.endswith(".bias"):
            a = np.zeros(shape, np.float32)
        else:
            a = std * _rng(seed, name).standard_normal(shape, dtype=np.float32)
        out[name] = a
    return out
