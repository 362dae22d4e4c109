"""Env sharding across GPUs + the rollout gather.

One process per GPU. Rank r owns envs [r * n, (r + 1) * n) of a global grid of world * n envs;
env origins (GridCloner over global ids) and the Philox reset / action streams are keyed on
GLOBAL env ids, so every env behaves exactly as in a single-GPU run of the same global env.
Physics never communicates. The only collective is one all-gather of the per-horizon rollout
slab (obs, rew, done) — RCCL over xGMI on the GPU box, gloo in the CPU tests.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_env_info() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, world: int, envs_per_rank: int) -> Tuple[int, int]:
    """(env_id_offset, global_num_envs) of this rank's shard."""
    return rank * envs_per_rank, world * envs_per_rank


class RolloutGather:
    """Per-horizon rollout slab [H, n, O + 2] (obs | rew | done) and its all-gather."""

    def __init__(self, horizon: int, n: int, num_obs: int, device, world: int):
        self.H, self.n, self.O, self.world = horizon, n, num_obs, world
        self.slab = torch.empty((horizon, n, num_obs + 2), device=device)
        self.out = torch.empty((world, horizon, n, num_obs + 2), device=device)

    def record(self, h: int, obs: torch.Tensor, rew: torch.Tensor, done: torch.Tensor) -> None:
        s = self.slab[h]
        s[:, : self.O].copy_(obs)
        s[:, self.O].copy_(rew)
        s[:, self.O + 1].copy_(done)

    def gather(self, group=None) -> torch.Tensor:
        """[world, H, n, O+2]: rank r's slab at out[r] (global env id = r * n + i)."""
        if self.world == 1:
            self.out[0].copy_(self.slab)
        elif dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(self.out.view(-1), self.slab.view(-1), group=group)
        else:
            dist.all_gather(list(self.out.unbind(0)), self.slab, group=group)
        return self.out

    def global_view(self) -> torch.Tensor:
        """[H, world * n, O+2] in global env order."""
        return self.out.permute(1, 0, 2, 3).reshape(self.H, self.world * self.n, self.O + 2)
