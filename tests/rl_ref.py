"""Test-side restatements of the PPO learner's fused ops (checkers only, never imported by the
product): numpy GAE (rl_games discount_values) and the Philox4x32-10 + Box-Muller draw of
mi_rl_sample_gauss, built on the oracle's Random123-pinned Philox (oracle.oracle.philox)."""
import math

import numpy as np

from oracle.oracle import philox


def gae_np(rew, val, dones, last_val, last_dones, gamma, tau):
    """rl_games a2c_common.discount_values, float64, [H, N]."""
    H = rew.shape[0]
    adv = np.zeros_like(rew, dtype=np.float64)
    last = np.zeros(rew.shape[1], dtype=np.float64)
    for t in reversed(range(H)):
        if t == H - 1:
            nnt, nv = 1.0 - last_dones, last_val
        else:
            nnt, nv = 1.0 - dones[t + 1], val[t + 1]
        delta = rew[t] + gamma * nv * nnt - val[t]
        last = delta + gamma * tau * nnt * last
        adv[t] = last
    return adv, adv + val


def normals_np(seed: int, counter: int, rows: int, A: int) -> np.ndarray:
    """z[n, j] of mi_rl_sample_gauss (float32 Box-Muller on the Philox uniforms)."""
    z = np.zeros((rows, A), dtype=np.float32)
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]
    for n in range(rows):
        for b in range((A + 3) // 4):
            c = philox([b, n, counter & 0xFFFFFFFF, ((counter >> 32) ^ 0x5EEDA11C) & 0xFFFFFFFF], key)
            u = (((c >> np.uint32(8)) + np.uint32(1)).astype(np.float32) * np.float32(1.0 / 16777216.0))
            for p in range(2):
                r = np.sqrt(np.float32(-2.0) * np.log(u[2 * p]))
                th = np.float32(2.0 * math.pi) * u[2 * p + 1]
                for k, v in ((2 * p, r * np.cos(th)), (2 * p + 1, r * np.sin(th))):
                    j = 4 * b + k
                    if j < A:
                        z[n, j] = v
    return z
