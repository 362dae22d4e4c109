"""Env sharding across GPUs + the rollout gather.

One process per GPU. Rank r owns envs [r * n, (r + 1) * n) of a global grid of world * n envs;
env origins (GridCloner over global ids) and the Philox reset / action streams are keyed on
GLOBAL env ids, so every env behaves exactly as in a single-GPU run of the same global env.
Physics never communicates. The only collective is one gather per PPO horizon of the rollout
slab (done, rew, obs [, learner fields]) to the learner rank — RCCL over xGMI on the GPU box,
gloo in the CPU tests.

Why a gather to the learner and not an all-gather: only the learner reads the global horizon
(`rlg.a2c_continuous` with `central_learner`). A gather moves each rank's slab once, over the
one xGMI link between that rank and the learner (8 GPUs: 7 links into the learner in parallel,
46.7 MB each for a Humanoid horizon, ≈0.3 ms at ≈153 GB/s per link). A ring all-gather would
push (world - 1) slabs through every link (≈2.2 ms at 8 GPUs) and leave 7 × 46.7 MB of copies on
ranks that never read them. ``mode="all_gather"`` stays for callers that want every rank to hold
the horizon.

Zero-copy, overlapped: the fused env step writes done / rew / obs straight into the slab row of
the current horizon step (``slot(h)`` → ``VecEnvRLGames.step(actions, out=...)``), so no copy
kernels run per step. A slab is step-major — row h holds every field of step h — so the first
``rows`` steps of a horizon are one contiguous prefix and a partial horizon can be gathered as
such. Slabs are double-buffered: the gather of a finished horizon is issued asynchronously
(RCCL runs on its own stream) while the next horizon steps into the other slab, and ``wait()``
joins it before the slab is reused or its gathered copy is read.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

_DTYPES = {torch.float32: 4, torch.int64: 8}


def shard_env_info() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, world: int, envs_per_rank: int) -> Tuple[int, int]:
    """(env_id_offset, global_num_envs) of this rank's shard."""
    return rank * envs_per_rank, world * envs_per_rank


def slab_fields(num_obs: int, extra: Sequence[Tuple[str, int, torch.dtype]] = (),
                with_done: bool = True):
    """Per-env fields of one slab row, 8-byte fields first: done i64, rew f32, obs f32 [O] — the
    dtypes VecEnvRLGames.step returns (vec_env_rlgames.py:41-46) — then any learner fields
    (name, width, dtype). ``with_done=False`` drops the i64 done field for a caller that keeps its
    own done field (the learner's f32 ``dones_f``), so no unread bytes cross xGMI."""
    f = [("done", 1, torch.int64)] if with_done else []
    f += [("rew", 1, torch.float32), ("obs", num_obs, torch.float32)]
    f += [(n, w, d) for n, w, d in extra]
    return f


class _Slab:
    """One horizon of rollout data in ONE flat byte buffer [lead..., H, step_bytes] (one collective
    moves all of it). Field k of step h is a contiguous [n, width] block of row h."""

    def __init__(self, H: int, n: int, fields, device, lead: Tuple[int, ...] = ()):
        offs, o = {}, 0
        for name, w, dt in fields:
            sz = _DTYPES[dt]
            o = (o + sz - 1) // sz * sz
            offs[name] = (o, w, dt)
            o += n * w * sz
        self.step_bytes = (o + 7) // 8 * 8
        self.H, self.n = H, n
        self.buf = torch.zeros(lead + (H, self.step_bytes), dtype=torch.uint8, device=device)
        self.views: Dict[str, torch.Tensor] = {}
        for name, (a, w, dt) in offs.items():
            b = a + n * w * _DTYPES[dt]
            v = self.buf[..., a:b].view(dt)
            self.views[name] = v.view(lead + (H, n, w)) if w > 1 or name == "obs" else v.view(lead + (H, n))

    @property
    def obs(self):
        return self.views["obs"]

    @property
    def rew(self):
        return self.views["rew"]

    @property
    def done(self):
        return self.views["done"]


class RolloutGather:
    """Per-horizon rollout slabs and their gather to the learner rank.

    ``slot(h)`` → (obs [n, O], rew [n], done [n]) views of the active slab's row h, for
    ``VecEnvRLGames.step(actions, out=slot(h))``; ``field(name, h)`` is the view of a learner
    field; ``record`` copies tensors in instead (for a step path that returns its own tensors).
    ``gather(async_op=True)`` launches the collective for the active slab (or its first ``rows``
    steps) and flips to the other one.
    """

    def __init__(self, horizon: int, n: int, num_obs: int, device, world: int, buffers: int = 2,
                 mode: str = "gather", dst: int = 0, rank: Optional[int] = None,
                 extra: Sequence[Tuple[str, int, torch.dtype]] = (), with_done: bool = True):
        if mode not in ("gather", "all_gather"):
            raise ValueError(f"mode must be 'gather' or 'all_gather' (got {mode!r})")
        self.H, self.n, self.O, self.world, self.mode, self.dst = horizon, n, num_obs, world, mode, dst
        self.rank = (dist.get_rank() if dist.is_initialized() else 0) if rank is None else rank
        fields = slab_fields(num_obs, extra, with_done)
        self.with_done = with_done
        self.slabs = [_Slab(horizon, n, fields, device) for _ in range(buffers)]
        # the learner (gather) or every rank (all_gather) holds [world, H, step_bytes]
        self.holds_output = mode == "all_gather" or self.rank == dst
        self.outs = [_Slab(horizon, n, fields, device, lead=(world,)) if self.holds_output else None
                     for _ in range(buffers)]
        self.step_bytes = self.slabs[0].step_bytes
        self.active = 0
        self._work: List[Optional[object]] = [None] * buffers
        self._last = 0
        self.last_rows = horizon
        self.gathers = 0           # collectives issued
        self.bytes_sent = 0        # slab bytes this rank contributed

    # compatibility views of the active slab
    @property
    def slab(self) -> _Slab:
        return self.slabs[self.active]

    @property
    def out(self) -> Optional[_Slab]:
        return self.outs[self._last]

    def slot(self, h: int):
        s = self.slabs[self.active]
        return s.obs[h], s.rew[h], (s.done[h] if self.with_done else None)

    def field(self, name: str, h: int) -> torch.Tensor:
        return self.slabs[self.active].views[name][h]

    def record(self, h: int, obs: torch.Tensor, rew: torch.Tensor,
               done: Optional[torch.Tensor] = None) -> None:
        """Copy one step into row h. A slab built with_done=False has no done field: `done`
        must then be None (its consumer keeps its own dones)."""
        o, r, d = self.slot(h)
        o.copy_(obs)
        r.copy_(rew)
        if d is not None:
            d.copy_(done)
        elif done is not None:
            raise ValueError("this slab has no done field (with_done=False): pass done=None")

    def _join(self, k: int) -> None:
        w = self._work[k]
        if w is not None:
            w.wait()
            self._work[k] = None

    def gather(self, group=None, async_op: bool = False, rows: Optional[int] = None) -> Optional[_Slab]:
        """Gather the active slab's first ``rows`` steps (default: the whole horizon) into
        outs[active] on the learner rank (rank r's rows at [r]); flips to the next slab, first
        joining any collective still in flight on it. Returns the output slab (None on a
        non-learner rank in gather mode), valid after ``wait()`` when async."""
        rows = self.H if rows is None else int(rows)
        if not 1 <= rows <= self.H:
            raise ValueError(f"rows must be in [1, {self.H}] (got {rows})")
        k = self.active
        src = self.slabs[k].buf[:rows]
        out = self.outs[k]
        if self.world == 1 and not dist.is_initialized():
            out.buf[0, :rows].copy_(src)
            self._work[k] = None
        elif self.mode == "all_gather":
            if rows == self.H and dist.get_backend(group) == "nccl":
                self._work[k] = dist.all_gather_into_tensor(out.buf.view(-1), src.reshape(-1),
                                                            group=group, async_op=async_op)
            else:
                self._work[k] = dist.all_gather([out.buf[r, :rows] for r in range(self.world)], src,
                                                group=group, async_op=async_op)
        else:
            lst = [out.buf[r, :rows] for r in range(self.world)] if out is not None else None
            self._work[k] = dist.gather(src, gather_list=lst, dst=self.dst, group=group,
                                        async_op=async_op)
        if not async_op:
            self._work[k] = None
        self.gathers += 1
        self.bytes_sent += rows * self.step_bytes
        self.last_rows = rows
        self._last = k
        self.active = (k + 1) % len(self.slabs)
        self._join(self.active)   # the slab the next horizon writes must be free
        return out

    def wait(self) -> None:
        for k in range(len(self._work)):
            self._join(k)

    def global_view(self) -> torch.Tensor:
        """[rows, world * n, O + 2] f32 (obs | rew | done) in global env order, of the last
        gather (learner rank, or any rank in all_gather mode)."""
        o = self.outs[self._last]
        if o is None:
            raise RuntimeError("global_view: this rank does not hold the gathered horizon")
        self.wait()
        R = self.last_rows
        obs = o.obs[:, :R].permute(1, 0, 2, 3).reshape(R, self.world * self.n, self.O)
        rew = o.rew[:, :R].permute(1, 0, 2).reshape(R, self.world * self.n, 1)
        done = o.done[:, :R].permute(1, 0, 2).reshape(R, self.world * self.n, 1).to(torch.float32)
        return torch.cat([obs, rew, done], dim=2)

    def global_field(self, name: str) -> torch.Tensor:
        """[rows, world * n, ...] of one field of the last gather, global env order."""
        o = self.outs[self._last]
        if o is None:
            raise RuntimeError("global_field: this rank does not hold the gathered horizon")
        self.wait()
        v = o.views[name][:, : self.last_rows]
        v = v.transpose(0, 1)
        # contiguous (at world 1 the reshape alone would be a strided view of the slab)
        return v.reshape((self.last_rows, self.world * self.n) + tuple(v.shape[3:])).contiguous()
