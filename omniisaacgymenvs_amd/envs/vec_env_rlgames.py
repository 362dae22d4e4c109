"""VecEnvRLGames — ROCm tensor-backed vectorized env (reference: envs/vec_env_rlgames.py:39-89
over omni.isaac.gym's closed VecEnvBase).

``step`` keeps the reference semantics exactly: clamp actions to ±clip_actions, task
pre_physics_step, controlFrequencyInv × World.step, task post_physics_step, get_states,
_process_data (obs/states clamp to ±clip_obs, move to rl_device, fresh tensors), return
({"obs", "states"}, rew, resets, extras). For the build's own tasks the whole sequence is one
HIP launch (task.fused_step → mi_env_step); a task that overrides any step method runs the
reference's method-by-method sequence, each built-in method still one HIP kernel.

Sharding: one process per GPU; a shard owns envs [env_id_offset, env_id_offset + num_envs)
of a global_num_envs grid, with env placement and RNG keyed on global ids.
"""
from __future__ import annotations

from datetime import datetime
from typing import Optional

import numpy as np
import torch

from ..utils.roctx import trace_range
from .world import Scene, World


class VecEnvRLGames:
    def __init__(self, headless: bool = True, sim_device: int = 0, enable_livestream: bool = False,
                 env_id_offset: int = 0, global_num_envs: Optional[int] = None) -> None:
        self._headless = headless
        self._render = not headless
        self._sim_device = sim_device
        self.env_id_offset = int(env_id_offset)
        self.global_num_envs = global_num_envs
        self.sim_frame_count = 0
        self._task = None
        self._world: Optional[World] = None
        self._fused = False
        self._ev_i = 0
        self._states = None
        self.kernel_events = None  # (start_events, end_events) bracketing each fused launch

    # ------------------------------------------------------------------ setup
    def set_task(self, task, backend: str = "torch", sim_params=None, init_sim: bool = True) -> None:
        """vec_env_rlgames.py:48-54 + VecEnvBase.set_task: build the world, set up the scene
        (creates the mi_sim handle), run post_reset."""
        self._task = task
        self._world = World(task=task, sim_params=sim_params or {}, device=task.device,
                            seed=getattr(self, "_seed", 42))
        task.set_up_scene(Scene(self._world))
        task.post_reset()
        self.num_envs = task.num_envs
        self.num_actions = task.num_actions
        self.num_observations = task.num_observations
        self.num_states = task.num_states
        self.action_space = task.action_space
        self.observation_space = task.observation_space
        self.state_space = task.state_space
        self._fused = task.supports_fused_step()

    def seed(self, seed: int = -1) -> int:
        if seed == -1:
            seed = np.random.randint(0, 2 ** 31 - 1)
        self._seed = int(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        return seed

    @property
    def task(self):
        return self._task

    @property
    def fused(self) -> bool:
        return self._fused

    def use_fused(self, on: bool) -> None:
        """Force the reference's method-by-method path (False) or the fused launch (True,
        only when the task supports it)."""
        self._fused = bool(on) and self._task.supports_fused_step()
        if not self._fused:
            # the fused launch may have bound task.obs_buf to a returned obs tensor (clip_obs =
            # inf, single write); the method-by-method path writes obs_buf in place
            self._task.obs_buf = self._task.obs_buf.clone()
            self._task._obs_aliased = False

    # ------------------------------------------------------------------ RL API
    def _process_data(self) -> None:
        t = self._task
        self._obs = torch.clamp(self._obs, -t.clip_obs, t.clip_obs).to(t.rl_device).clone()
        self._rew = self._rew.to(t.rl_device).clone()
        self._states = torch.clamp(self._states, -t.clip_obs, t.clip_obs).to(t.rl_device).clone()
        self._resets = self._resets.to(t.rl_device).clone()
        self._extras = self._extras.copy()

    def step(self, actions, out=None):
        """vec_env_rlgames.py:56-78. ``out`` (build extension, fused path only): (obs, rew, resets)
        buffers for the returned copies, e.g. a rollout slab row; by default fresh tensors."""
        t = self._task
        if out is not None and (not self._fused or str(t.rl_device) != str(t.device)):
            raise ValueError("step(out=...) needs the fused path with rl_device == sim device")
        if self._fused:
            # one launch = clamp + action DR + pre_physics_step + N substeps + post_physics_step +
            # observation DR + obs clamp
            ev = self.kernel_events
            if ev is not None:
                k = self._ev_i % len(ev[0])
                ev[0][k].record()
                obs, rew, resets = t.fused_step(actions, out)
                ev[1][k].record()
                self._ev_i += 1
            else:   # one launch: no per-phase ranges (the kernel trace names it)
                obs, rew, resets = t.fused_step(actions, out)
            self.sim_frame_count += t.control_frequency_inv
            # fresh tensors written by the launch itself (= _process_data's clones)
            rl = str(t.rl_device)
            self._obs = obs if rl == str(obs.device) else obs.to(t.rl_device)
            self._rew = rew if rl == str(rew.device) else rew.to(t.rl_device)
            self._resets = resets if rl == str(resets.device) else resets.to(t.rl_device)
            self._extras = t.extras.copy()
            st = t.get_states()
            if st.numel() == 0:       # no state space (Humanoid / Ant / Cartpole): nothing to clamp
                if self._states is None or self._states.shape != st.shape or str(self._states.device) != str(t.rl_device):
                    self._states = st.to(t.rl_device).clone()
            else:
                self._states = torch.clamp(st, -t.clip_obs, t.clip_obs).to(t.rl_device).clone()
            return {"obs": self._obs, "states": self._states}, self._rew, self._resets, self._extras
        actions = torch.clamp(actions, -t.clip_actions, t.clip_actions).to(t.device).clone()
        if t.randomize_actions:
            actions = t._dr_randomizer.apply_actions_randomization(actions=actions, reset_buf=t.reset_buf)
        with trace_range("pre_physics_step"):
            t.pre_physics_step(actions)
        with trace_range("physics (controlFrequencyInv x World.step)"):
            for _ in range(t.control_frequency_inv):
                self._world.step(render=self._render)
                self.sim_frame_count += 1
        with trace_range("post_physics_step"):
            self._obs, self._rew, self._resets, self._extras = t.post_physics_step()
        if t.randomize_observations:
            self._obs = t._dr_randomizer.apply_observations_randomization(observations=self._obs,
                                                                          reset_buf=t.reset_buf)
        self._states = t.get_states()
        self._process_data()
        return {"obs": self._obs, "states": self._states}, self._rew, self._resets, self._extras

    def reset(self):
        """vec_env_rlgames.py:80-89: flag every env and run one zero-action step."""
        now = datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        print(f"[{now}] Running RL reset")
        self._task.reset()
        actions = torch.zeros((self.num_envs, self._task.num_actions), device=self._task.device)
        obs_dict, _, _, _ = self.step(actions)
        return obs_dict

    def get_number_of_agents(self) -> int:
        return self._task.num_agents

    def render(self, mode: str = "human") -> None:
        return None

    def close(self) -> None:
        if self._task is not None:
            self._task.close()
