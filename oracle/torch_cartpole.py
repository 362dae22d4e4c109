"""TEST INFRASTRUCTURE ONLY — BASELINE config 1's "Cartpole 16 envs, analytic dynamics on CPU
torch": the reference's Cartpole task (tasks/cartpole.py:80-162) as torch ops on CPU tensors,
the way the reference runs it with pipeline=cpu, stepped by VecEnvRLGames.step's sequence
(envs/vec_env_rlgames.py:56-78): clamp actions, pre_physics_step (nonzero() -> reset_idx,
efforts), controlFrequencyInv x physics, post_physics_step (progress += 1, get_observations,
calculate_metrics, is_done), _process_data's obs clamp.

Physics: the closed PhysX CPU step is replaced by the build's analytic cart-pole (the same
equations as oracle/oracle.c cartpole_substep and the device's k_env_step, semi-implicit Euler
on the 2x2 mass matrix), written as torch ops.

Reset noise: ``noise="torch"`` draws torch.rand in the reference's order (cartpole.py:119-125:
cart pos, pole pos, cart vel, pole vel) — the timed CPU baseline; ``noise="philox"`` draws the
build's Philox4x32-10 stream (seed, global env id, reset count, slot) in torch int64
arithmetic, so the restatement can be checked against the C oracle step for step
(tests/test_cpu_torch_cartpole.py). Only tests/ and bench.py's cpu_baseline leg use this file.
"""
from __future__ import annotations

import math

import numpy as np
import torch

_M32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Philox4x32-10 on int64 tensors holding uint32 values (Random123; the build's stream,
    oracle.c orc_philox4x32_10). ctr: 4 tensors, key: 2 tensors (or ints)."""
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & _M32
            k1 = (k1 + 0xBB67AE85) & _M32
        p0 = c0 * 0xD2511F53            # < 2^64: wraps in int64, low 64 bits exact
        p1 = c2 * 0xCD9E8D57
        n0 = ((p1 >> 32) & _M32) ^ c1 ^ k0
        n2 = ((p0 >> 32) & _M32) ^ c3 ^ k1
        c1, c3 = p1 & _M32, p0 & _M32
        c0, c2 = n0, n2
    return c0, c1, c2, c3


def philox_uniform(seed: int, env_ids: torch.Tensor, counter_hi: torch.Tensor, slot: int, stream: int = 0):
    """orc_uniform (oracle.c) vectorised: U[0, 1) float32 from (seed, env id, counter, slot)."""
    gid = env_ids.to(torch.int64)
    z = torch.zeros_like(gid)
    ctr = (z + (slot >> 2), counter_hi.to(torch.int64) & _M32, gid & _M32,
           ((gid >> 32) & _M32) ^ ((stream << 28) & _M32))
    out = philox4x32_10(ctr, (seed & _M32, (seed >> 32) & _M32))[slot & 3]
    return (out >> 8).to(torch.float32) * (1.0 / 16777216.0)


class CpuTorchCartpole:
    """The reference's CartpoleTask + VecEnvRLGames.step on CPU torch tensors."""

    def __init__(self, model, sim_params, task_params, num_envs: int, seed: int = 42,
                 env_id_offset: int = 0, noise: str = "torch", control_frequency_inv: int = 2):
        if noise not in ("torch", "philox"):
            raise ValueError(noise)
        cp = model.cartpole
        self.mc, self.mp = float(cp["cart_mass"]), float(cp["pole_mass"])
        self.l, self.Ip = float(cp["pole_com"]), float(cp["pole_inertia"])
        self.cd, self.pd = float(cp["cart_damping"]), float(cp["pole_damping"])
        self.g = -float(sim_params.gravity[2])
        self.dt = float(sim_params.dt)
        self.n = int(num_envs)
        self.seed = int(seed)
        self.noise = noise
        self.cfi = int(control_frequency_inv)
        self.reset_dist = float(task_params.reset_dist)
        self.max_push_effort = float(task_params.max_push_effort)
        self.max_episode_length = float(task_params.max_episode_length)
        self.clip_actions = float(task_params.clip_actions)
        self.clip_obs = float(task_params.clip_obs)
        self.cart_idx, self.pole_idx = model.get_dof_index("cartJoint"), model.get_dof_index("poleJoint")
        self.env_ids = torch.arange(env_id_offset, env_id_offset + self.n, dtype=torch.int64)
        self.reset_count = torch.zeros(self.n, dtype=torch.int64)
        # RLTask.cleanup (rl_task.py:98-107)
        self.obs_buf = torch.zeros((self.n, 4), dtype=torch.float32)
        self.rew_buf = torch.zeros(self.n, dtype=torch.float32)
        self.reset_buf = torch.ones(self.n, dtype=torch.int64)
        self.progress_buf = torch.zeros(self.n, dtype=torch.int64)
        self.dof_pos = torch.zeros((self.n, 2), dtype=torch.float32)
        self.dof_vel = torch.zeros((self.n, 2), dtype=torch.float32)
        self.efforts = torch.zeros((self.n, 2), dtype=torch.float32)
        self.reset_idx(torch.arange(self.n))                     # post_reset (cartpole.py:136-141)

    # ---- cartpole.py:114-134
    def _rand(self, env_ids, slot):
        if self.noise == "torch":
            return torch.rand(len(env_ids))
        return philox_uniform(self.seed, self.env_ids[env_ids], self.reset_count[env_ids], slot)

    def reset_idx(self, env_ids):
        num_resets = len(env_ids)
        dof_pos = torch.zeros((num_resets, 2))
        dof_pos[:, self.cart_idx] = 1.0 * (1.0 - 2.0 * self._rand(env_ids, 0))
        dof_pos[:, self.pole_idx] = 0.125 * math.pi * (1.0 - 2.0 * self._rand(env_ids, 1))
        dof_vel = torch.zeros((num_resets, 2))
        dof_vel[:, self.cart_idx] = 0.5 * (1.0 - 2.0 * self._rand(env_ids, 2))
        dof_vel[:, self.pole_idx] = 0.25 * math.pi * (1.0 - 2.0 * self._rand(env_ids, 3))
        self.dof_pos[env_ids] = dof_pos
        self.dof_vel[env_ids] = dof_vel
        self.reset_count[env_ids] += 1
        self.reset_buf[env_ids] = 0
        self.progress_buf[env_ids] = 0

    # ---- cartpole.py:101-112
    def pre_physics_step(self, actions):
        reset_env_ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1)
        if len(reset_env_ids) > 0:
            self.reset_idx(reset_env_ids)
        forces = torch.zeros((self.n, 2), dtype=torch.float32)
        forces[:, self.cart_idx] = self.max_push_effort * actions[:, 0]
        self.efforts = forces

    # ---- World.step: the analytic cart-pole (oracle.c cartpole_substep, same operation order;
    # the scalar products are rounded to float32 one operation at a time, as in C)
    def physics_substep(self):
        f = np.float32
        x, th = self.dof_pos[:, 0], self.dof_pos[:, 1]
        xd, thd = self.dof_vel[:, 0], self.dof_vel[:, 1]
        s, c = torch.sin(th), torch.cos(th)
        mc, mp, l = f(self.mc), f(self.mp), f(self.l)
        mpl = float(mp * l)
        m11 = float(mc + mp)
        m12 = mpl * c
        m22 = float(f(self.Ip) + f(mp * l) * l)
        mgl = float(f(mp * f(self.g)) * l)
        r1 = self.efforts[:, 0] + mpl * s * thd * thd - float(f(self.cd)) * xd
        r2 = self.efforts[:, 1] + mgl * s - float(f(self.pd)) * thd
        det = m11 * m22 - m12 * m12
        xdd = (m22 * r1 - m12 * r2) / det
        thdd = (m11 * r2 - m12 * r1) / det
        xd = xd + self.dt * xdd
        thd = thd + self.dt * thdd
        self.dof_pos = torch.stack([x + self.dt * xd, th + self.dt * thd], dim=1)
        self.dof_vel = torch.stack([xd, thd], dim=1)

    # ---- cartpole.py:80-99, 143-162 via rl_task.py:231-251
    def post_physics_step(self):
        self.progress_buf[:] += 1
        self.obs_buf[:, 0] = self.dof_pos[:, self.cart_idx]
        self.obs_buf[:, 1] = self.dof_vel[:, self.cart_idx]
        self.obs_buf[:, 2] = self.dof_pos[:, self.pole_idx]
        self.obs_buf[:, 3] = self.dof_vel[:, self.pole_idx]
        cart_pos, cart_vel = self.obs_buf[:, 0], self.obs_buf[:, 1]
        pole_angle, pole_vel = self.obs_buf[:, 2], self.obs_buf[:, 3]
        reward = 1.0 - pole_angle * pole_angle - 0.01 * torch.abs(cart_vel) - 0.005 * torch.abs(pole_vel)
        reward = torch.where(torch.abs(cart_pos) > self.reset_dist, torch.ones_like(reward) * -2.0, reward)
        reward = torch.where(torch.abs(pole_angle) > np.pi / 2, torch.ones_like(reward) * -2.0, reward)
        self.rew_buf[:] = reward
        resets = torch.where(torch.abs(cart_pos) > self.reset_dist, 1, 0)
        resets = torch.where(torch.abs(pole_angle) > math.pi / 2, 1, resets)
        resets = torch.where(self.progress_buf >= self.max_episode_length, 1, resets)
        self.reset_buf[:] = resets
        return self.obs_buf, self.rew_buf, self.reset_buf, {}

    # ---- vec_env_rlgames.py:56-78 (+ _process_data :41-46)
    def step(self, actions):
        actions = torch.clamp(actions, -self.clip_actions, self.clip_actions).clone()
        self.pre_physics_step(actions)
        for _ in range(self.cfi):
            self.physics_substep()
        obs, rew, resets, extras = self.post_physics_step()
        obs = torch.clamp(obs, -self.clip_obs, self.clip_obs).clone()
        return {"obs": obs}, rew.clone(), resets.clone(), extras

    def reset(self):
        """vec_env_rlgames.py:80-89: flag every env (rl_task.py:218-221), one zero-action step."""
        self.reset_buf = torch.ones_like(self.reset_buf)
        return self.step(torch.zeros((self.n, 1)))[0]
