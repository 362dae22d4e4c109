"""Env sharding across GPUs + the rollout gather.

One process per GPU. Rank r owns envs [r * n, (r + 1) * n) of a global grid of world * n envs;
env origins (GridCloner over global ids) and the Philox reset / action streams are keyed on
GLOBAL env ids, so every env behaves exactly as in a single-GPU run of the same global env.
Physics never communicates. The only collective is one all-gather per PPO horizon of the
rollout slab (obs, rew, done) — RCCL over xGMI on the GPU box, gloo in the CPU tests.

Zero-copy, overlapped: the fused env step writes obs / rew / done straight into the slab row of
the current horizon step (``slot(h)`` → ``VecEnvRLGames.step(actions, out=...)``), so no copy
kernels run per step. Slabs are double-buffered: the all-gather of a finished horizon is issued
asynchronously (RCCL runs on its own stream) while the next horizon steps into the other slab,
and ``wait()`` joins it before the slab is reused or its gathered copy is read.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_env_info() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, world: int, envs_per_rank: int) -> Tuple[int, int]:
    """(env_id_offset, global_num_envs) of this rank's shard."""
    return rank * envs_per_rank, world * envs_per_rank


class _Slab:
    """One horizon of rollout data in ONE flat byte buffer (one collective moves all of it):
    obs f32 [H, n, O] | rew f32 [H, n] | done i64 [H, n] — the dtypes VecEnvRLGames.step returns
    (vec_env_rlgames.py:41-46), so step can write here directly."""

    def __init__(self, H: int, n: int, O: int, device, lead: Tuple[int, ...] = ()):
        self.sizes = (H * n * O * 4, H * n * 4, H * n * 8)
        per = sum(self.sizes)
        self.buf = torch.empty(lead + (per,), dtype=torch.uint8, device=device)
        a, b = self.sizes[0], self.sizes[0] + self.sizes[1]
        self.obs = self.buf[..., :a].view(torch.float32).view(lead + (H, n, O))
        self.rew = self.buf[..., a:b].view(torch.float32).view(lead + (H, n))
        self.done = self.buf[..., b:].view(torch.int64).view(lead + (H, n))


class RolloutGather:
    """Per-horizon rollout slabs and their all-gather.

    ``slot(h)`` → (obs [n, O], rew [n], done [n]) views of the active slab's row h, for
    ``VecEnvRLGames.step(actions, out=slot(h))``; ``record`` copies tensors in instead (for a
    step path that returns its own tensors). ``gather(async_op=True)`` launches the collective
    for the active slab and flips to the other one.
    """

    def __init__(self, horizon: int, n: int, num_obs: int, device, world: int, buffers: int = 2):
        self.H, self.n, self.O, self.world = horizon, n, num_obs, world
        self.slabs = [_Slab(horizon, n, num_obs, device) for _ in range(buffers)]
        self.outs = [_Slab(horizon, n, num_obs, device, lead=(world,)) for _ in range(buffers)]
        self.active = 0
        self._work: List[Optional[object]] = [None] * buffers
        self._last = 0

    # compatibility views of the active slab
    @property
    def slab(self) -> _Slab:
        return self.slabs[self.active]

    @property
    def out(self) -> _Slab:
        return self.outs[self._last]

    def slot(self, h: int):
        s = self.slabs[self.active]
        return s.obs[h], s.rew[h], s.done[h]

    def record(self, h: int, obs: torch.Tensor, rew: torch.Tensor, done: torch.Tensor) -> None:
        o, r, d = self.slot(h)
        o.copy_(obs)
        r.copy_(rew)
        d.copy_(done)

    def _join(self, k: int) -> None:
        w = self._work[k]
        if w is not None:
            w.wait()
            self._work[k] = None

    def gather(self, group=None, async_op: bool = False) -> _Slab:
        """All-gather the active slab into outs[active] (rank r's rows at [r]); flips to the next
        slab, first joining any collective still in flight on it. Returns the output slab, valid
        after ``wait()`` when async."""
        k = self.active
        src, dst = self.slabs[k].buf, self.outs[k].buf
        if self.world == 1:
            dst[0].copy_(src)
        elif dist.get_backend(group) == "nccl":
            self._work[k] = dist.all_gather_into_tensor(dst.view(-1), src, group=group,
                                                        async_op=async_op)
        else:
            self._work[k] = dist.all_gather(list(dst.unbind(0)), src, group=group, async_op=async_op)
        if not async_op:
            self._work[k] = None
        self._last = k
        self.active = (k + 1) % len(self.slabs)
        self._join(self.active)   # the slab the next horizon writes must be free
        return self.outs[k]

    def wait(self) -> None:
        for k in range(len(self._work)):
            self._join(k)

    def global_view(self) -> torch.Tensor:
        """[H, world * n, O + 2] f32 (obs | rew | done) in global env order, of the last gather."""
        o = self.outs[self._last]
        self.wait()
        obs = o.obs.permute(1, 0, 2, 3).reshape(self.H, self.world * self.n, self.O)
        rew = o.rew.permute(1, 0, 2).reshape(self.H, self.world * self.n, 1)
        done = o.done.permute(1, 0, 2).reshape(self.H, self.world * self.n, 1).to(torch.float32)
        return torch.cat([obs, rew, done], dim=2)
