"""Portable counter-based PRNG (test infrastructure; see oracle/__init__.py).

splitmix64(seed, counter) -> 53-bit uniform in [0,1) -> Box-Muller normal.  Chosen so that
fixtures never need to carry weight tensors and never depend on torch's RNG across versions
(SURVEY.md §8c "Golden vectors to commit").  Pure numpy uint64 arithmetic, fully vectorised.
"""
import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(seed, n, offset=0):
    """n uniforms in [0,1) for stream `seed`, counters offset..offset+n-1 (float64)."""
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(seed) * np.uint64(0x2545F4914F6CDD1D) + np.uint64(1))
        ctr = np.arange(offset, offset + n, dtype=np.uint64)
        bits = _splitmix64(base ^ (ctr * _G))
    return (bits >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed, shape, std=1.0, mean=0.0):
    """Box-Muller normals, float32, deterministic in (seed, shape)."""
    n = int(np.prod(shape)) if len(shape) else 1
    m = (n + 1) // 2
    u1 = uniform(seed, m, 0)
    u2 = uniform(seed, m, m)
    r = np.sqrt(-2.0 * np.log1p(-u1))
    t = 2.0 * np.pi * u2
    z = np.concatenate([r * np.cos(t), r * np.sin(t)])[:n]
    return (z * std + mean).astype(np.float32).reshape(shape)


def uniform_f32(seed, shape, lo=0.0, hi=1.0):
    n = int(np.prod(shape)) if len(shape) else 1
    return (uniform(seed, n) * (hi - lo) + lo).astype(np.float32).reshape(shape)


def seed_for(name, base=0):
    """Stable per-tensor stream id from a parameter name (FNV-1a 64)."""
    h = 0xCBF29CE484222325
    for ch in name.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return (h ^ base) & 0xFFFFFFFFFFFFFFFF


def init_state_dict(shapes, base_seed=0, std=0.02, bias_std=0.01):
    """Weights for a state_dict given {name: shape}: conv weights N(0, std) like the reference's
    init_type='normal' (networks.py:67-98); biases small N(0, bias_std) instead of 0 so the bias
    path is exercised by parity tests."""
    out = {}
    for name, shape in shapes.items():
        s = std if name.endswith("weight") else bias_std
        out[name] = normal(seed_for(name, base_seed), tuple(shape), std=s)
    return out
