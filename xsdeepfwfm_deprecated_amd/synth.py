"""Deterministic synthetic weights and inputs.

Weights are derived from a counter-based integer hash (splitmix64), not from
numpy's Generator, so the same (name, shape, seed) gives bit-identical float32
values on every machine and numpy version: golden fixtures store only the
recipe plus inputs/outputs, and the GPU box regenerates the weights.

Scales follow the reference's init_weights (model/DeepFMs.py:472-495), as
uniform distributions with the same standard deviation:
  *1st_embeddings* N(0,1); *2nd_embeddings* 0.01*N(0,1);
  *linear* weight & bias sqrt(2/(fan_in+fan_out)) (bias shares its layer's);
  field_cov.weight sqrt(1/F); fm_1st / *fc.weight sqrt(2/last_layer_size);
  bias 0.01.
"""
from __future__ import annotations

import zlib

import numpy as np

# Criteo-39 field sizes (reference latency/criteo_latency.cpp:38-39)
CRITEO_FEATURE_SIZES = [1] * 13 + [1458, 556, 245197, 166166, 306, 20, 12055, 634, 4, 46330, 5229, 243454,
                                   3177, 27, 11745, 225322, 11, 4727, 2058, 5, 238640, 18, 16, 67856, 89, 50942]

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=False)
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _stream(key: str, seed: int, n: int) -> np.ndarray:
    base = np.uint64((zlib.crc32(key.encode()) << 32) ^ (seed & 0xFFFFFFFF))
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + splitmix64(np.array([base], dtype=np.uint64))[0] * _G
    return splitmix64(ctr)


def uniform(key: str, seed: int, shape, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """float32 in [lo, hi): 24 random bits -> exact float32 grid, then an affine map in float64."""
    n = int(np.prod(shape)) if len(shape) else 1
    bits = (_stream(key, seed, n) >> np.uint64(40)).astype(np.float64)  # 24 bits
    u = bits * (1.0 / (1 << 24))
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def randint(key: str, seed: int, shape, high) -> np.ndarray:
    """int64 in [0, high) per column (high: scalar or per-last-axis array)."""
    n = int(np.prod(shape))
    r = _stream(key, seed, n).reshape(shape)
    high = np.asarray(high, dtype=np.uint64)
    return (r % high).astype(np.int64)


def param_std(name: str, shape, field_size: int, embedding_size: int, last_layer_size: int,
              layer_glorot: dict) -> float:
    if "1st_embeddings" in name:
        return 1.0
    if "2nd_embeddings" in name:
        return 0.01
    if "linear" in name:
        layer = name.rsplit(".", 1)[0]
        if name.endswith("weight"):
            layer_glorot[layer] = float(np.sqrt(2.0 / np.sum(shape)))
        return layer_glorot[layer]
    if name == "field_cov.weight":
        return float(np.sqrt(2.0 / field_size / 2))
    if name in ("fm_1st.weight",) or "fc.weight" in name:
        return float(np.sqrt(2.0 / last_layer_size))
    return 0.0


def synth_state(shapes: dict, field_size: int, embedding_size: int, deep_nodes: int, use_second: bool,
                use_deep: bool, seed: int = 1234) -> dict:
    """name -> float32 array for every parameter name in `shapes` (an ordered name->shape dict,
    weights before biases as in named_parameters)."""
    last = (field_size + embedding_size if use_second else 0) + (deep_nodes + 1 if use_deep else 0)
    glorot = {}
    out = {}
    for name, shape in shapes.items():
        shape = tuple(int(s) for s in shape)
        if name == "bias":
            out[name] = np.full(shape, 0.01, dtype=np.float32)
            continue
        std = param_std(name, shape, field_size, embedding_size, last, glorot)
        a = std * np.sqrt(3.0)
        out[name] = uniform(name, seed, shape, -a, a)
    return out


def synth_inputs(feature_sizes, numerical: int, batch: int, seed: int = 0, xv_max: int = 64):
    """Xi int64 [batch, F-num] uniform over each field's table; Xv float32 integers in [0, xv_max)."""
    cat = np.asarray(feature_sizes[numerical:], dtype=np.int64)
    xi = randint("Xi", seed, (batch, len(cat)), cat)
    xv = randint("Xv", seed, (batch, numerical), xv_max).astype(np.float32)
    return xi, xv


def synth_labels(batch: int, seed: int = 0, rate: float = 0.25) -> np.ndarray:
    u = uniform("y", seed, (batch,), 0.0, 1.0)
    return (u < rate).astype(np.int64)


def zipf_inputs(feature_sizes, numerical: int, batch: int, seed: int = 0, s: float = 1.1):
    """Skewed categorical indices: rank ~ Zipf(s) mapped through a per-field hash permutation."""
    cat = np.asarray(feature_sizes[numerical:], dtype=np.int64)
    u = uniform("zipf", seed, (batch, len(cat)), 0.0, 1.0).astype(np.float64)
    # inverse-CDF of a bounded power law on [1, n]
    n = cat.astype(np.float64)[None, :]
    a = 1.0 - s
    rank = np.floor(((n ** a - 1.0) * u + 1.0) ** (1.0 / a)) - 1.0
    rank = np.clip(rank, 0, n - 1).astype(np.int64)
    perm = (splitmix64(rank.astype(np.uint64) + np.arange(len(cat), dtype=np.uint64)[None, :] * _G)
            % cat.astype(np.uint64)[None, :]).astype(np.int64)
    xv = randint("Xv", seed, (batch, numerical), 64).astype(np.float32)
    return perm, xv
