"""Minimal stand-in for ``gym.spaces.Box`` (gym is not installed offline). Carries what the
VecEnv / rl_games contract reads: low, high, shape, dtype, sample()."""
from __future__ import annotations

import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        low = np.asarray(low, dtype=dtype)
        high = np.asarray(high, dtype=dtype)
        if shape is not None:
            low = np.broadcast_to(low, shape).astype(dtype)
            high = np.broadcast_to(high, shape).astype(dtype)
        self.low, self.high, self.dtype = low, high, np.dtype(dtype)
        self.shape = tuple(low.shape)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi).astype(self.dtype)

    def __repr__(self):
        return f"Box({self.low.min() if self.low.size else ''}, {self.high.max() if self.high.size else ''}, {self.shape}, {self.dtype})"
