"""The build's counter-based random stream on the host (the CPU pipeline's reset draws).

Philox4x32-10 (Random123) keyed by the run seed, counter = {slot / 4, counter_hi, env id low
32 bits, env id high 32 bits ^ (stream << 28)}, one U[0, 1) float from the top 24 bits of output
word ``slot % 4``. This is the stream the HIP kernels draw from (``csrc/mi_device.hpp``), so the
CPU pipeline's reset noise is the GPU pipeline's, draw for draw, and both are independent of the
env count per process (DESIGN.md §5 "Reset noise": the reference draws torch.rand,
tasks/cartpole.py:119-125).

The rounds run on numpy uint64 arrays holding uint32 words: a product of two uint32 values is
exact in 64 bits, so its high and low halves are the 32x32 -> 64 multiply Philox needs. One
call yields all four words of a counter, i.e. slots 4k .. 4k+3 at once.
"""
from __future__ import annotations

import numpy as np
import torch

_M32 = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)
_MUL0, _MUL1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Ten Philox4x32 rounds on four uint64 arrays of uint32 values; returns the four words."""
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = c0 * _MUL0
        p1 = c2 * _MUL1
        c0, c1, c2, c3 = ((p1 >> _S32) ^ c1 ^ np.uint64(k0), p1 & _M32,
                          (p0 >> _S32) ^ c3 ^ np.uint64(k1), p0 & _M32)
    return c0, c1, c2, c3


def uniform4(seed: int, env_ids: torch.Tensor, counter_hi: torch.Tensor, block: int = 0,
             stream: int = 0) -> torch.Tensor:
    """[n, 4] U[0, 1) float32: slots 4*block .. 4*block+3 of (seed, global env id, counter)."""
    gid = env_ids.cpu().numpy().astype(np.uint64)
    n = gid.shape[0]
    c0 = np.full(n, block, dtype=np.uint64)
    c1 = counter_hi.cpu().numpy().astype(np.uint64) & _M32
    c2 = gid & _M32
    c3 = (gid >> _S32) ^ np.uint64((stream << 28) & 0xFFFFFFFF)
    words = np.stack(philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF), 1)
    u = (words >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return torch.from_numpy(u)


def uniform(seed: int, env_ids: torch.Tensor, counter_hi: torch.Tensor, slot: int,
            stream: int = 0) -> torch.Tensor:
    """U[0, 1) float32 per env: (seed, global env id, counter, slot, stream)."""
    return uniform4(seed, env_ids, counter_hi, slot >> 2, stream)[:, slot & 3].contiguous()
