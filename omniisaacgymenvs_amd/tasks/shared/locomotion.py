"""LocomotionTask — shared Humanoid / Ant logic (reference: tasks/shared/locomotion.py:45-183).

Same configuration keys, buffers and method contract. Each method is ONE HIP kernel in
libmi_sim.so instead of a TorchScript chain + ArticulationView round trips:

  pre_physics_step   -> mi_task_pre_step    (mask-driven reset_idx: no nonzero() host sync)
  reset_idx(env_ids) -> mi_task_reset_idx
  get_observations   -> mi_task_observations
  calculate_metrics  -> mi_task_metrics     (incl. the task's get_dof_at_limit_cost)
  is_done            -> mi_task_is_done
and, when none of them is overridden, VecEnvRLGames.step runs the whole step as one
mi_env_step launch (fused_step).

RNG: reset noise comes from the build's counter-based Philox4x32-10 stream keyed on
(seed, global env id, reset count), identical on CPU oracle and GPU — a deliberate deviation
from the reference's torch.rand stream.
"""
from __future__ import annotations

import ctypes as C
import math
from abc import abstractmethod

import numpy as np
import torch

from ... import native as N
from ...tasks.base.rl_task import RLTask


class LocomotionTask(RLTask):
    TASK_KIND = None  # MI_TASK_ANT / MI_TASK_HUMANOID

    def __init__(self, name, env, offset=None) -> None:
        env_cfg = self._task_cfg["env"]
        self._num_envs = env_cfg["numEnvs"]
        self._env_spacing = env_cfg["envSpacing"]
        self._max_episode_length = env_cfg["episodeLength"]
        self.dof_vel_scale = env_cfg["dofVelocityScale"]
        self.angular_velocity_scale = env_cfg["angularVelocityScale"]
        self.contact_force_scale = env_cfg["contactForceScale"]
        self.power_scale = env_cfg["powerScale"]
        self.heading_weight = env_cfg["headingWeight"]
        self.up_weight = env_cfg["upWeight"]
        self.actions_cost_scale = env_cfg["actionsCost"]
        self.energy_cost_scale = env_cfg["energyCost"]
        self.joints_at_limit_cost_scale = env_cfg["jointsAtLimitCost"]
        self.death_cost = env_cfg["deathCost"]
        self.termination_height = env_cfg["terminationHeight"]
        self.alive_reward_scale = env_cfg["alive_reward_scale"]
        RLTask.__init__(self, name, env)

    @abstractmethod
    def set_up_scene(self, scene) -> None:
        pass

    @abstractmethod
    def get_robot(self):
        pass

    # ------------------------------------------------------------------ helpers
    def _h(self):
        return self._robots.handle

    def _stream(self):
        return self._robots.stream()

    def task_params(self) -> N.MiTaskParams:
        """mi_task_params for this task (host struct; arrays kept alive on self)."""
        tp = N.MiTaskParams()
        tp.task_kind = self.TASK_KIND
        tp.num_obs = self.num_observations
        tp.num_actions = self.num_actions
        tp.clip_actions = float(self.clip_actions)
        tp.clip_obs = float(self.clip_obs)
        tp.max_episode_length = float(self._max_episode_length)
        tp.power_scale = self.power_scale
        tp.heading_weight = self.heading_weight
        tp.up_weight = self.up_weight
        tp.actions_cost = self.actions_cost_scale
        tp.energy_cost = self.energy_cost_scale
        tp.dof_vel_scale = self.dof_vel_scale
        tp.angular_velocity_scale = self.angular_velocity_scale
        tp.contact_force_scale = self.contact_force_scale
        tp.joints_at_limit_cost = self.joints_at_limit_cost_scale
        tp.death_cost = self.death_cost
        tp.termination_height = self.termination_height
        tp.alive_reward_scale = self.alive_reward_scale
        tp.task_dt = self.dt
        tp.target[:] = [1000.0, 0.0, 0.0]
        tp.init_root_pos[:] = [float(v) for v in self._spawn_translation]
        tp.init_root_quat[:] = [1.0, 0.0, 0.0, 0.0]
        tp.dof_pos_noise = 0.2
        tp.dof_vel_noise = 0.1
        self._tp_arrays = (
            np.ascontiguousarray(self.joint_gears.cpu().numpy(), np.float32),
            np.ascontiguousarray(self.motor_effort_ratio.cpu().numpy(), np.float32),
            np.ascontiguousarray(self.initial_dof_pos[0].cpu().numpy(), np.float32),
        )
        tp.joint_gears = N.fptr(self._tp_arrays[0])
        tp.motor_effort_ratio = N.fptr(self._tp_arrays[1])
        tp.init_dof_pos = N.fptr(self._tp_arrays[2])
        return tp

    # ------------------------------------------------------------------ task API
    def get_observations(self) -> dict:
        N.check(N.lib().mi_task_observations(self._h(), self.actions.data_ptr(), self.obs_buf.data_ptr(),
                                             self.potentials.data_ptr(), self.prev_potentials.data_ptr(),
                                             self._stream()), "mi_task_observations")
        return {self._robots.name: {"obs_buf": self.obs_buf}}

    def pre_physics_step(self, actions) -> None:
        a = actions.to(self._device, dtype=torch.float32).contiguous()
        N.check(N.lib().mi_task_pre_step(self._h(), a.data_ptr(), self.reset_buf.data_ptr(),
                                         self.progress_buf.data_ptr(), self.potentials.data_ptr(),
                                         self.prev_potentials.data_ptr(), self.actions.data_ptr(),
                                         self._stream()), "mi_task_pre_step")

    def reset_idx(self, env_ids) -> None:
        ids = torch.as_tensor(env_ids, device=self._device).to(torch.int64).contiguous()
        N.check(N.lib().mi_task_reset_idx(self._h(), ids.data_ptr(), int(ids.numel()),
                                          self.reset_buf.data_ptr(), self.progress_buf.data_ptr(),
                                          self.potentials.data_ptr(), self.prev_potentials.data_ptr(),
                                          self._stream()), "mi_task_reset_idx")

    def post_reset(self) -> None:
        """locomotion.py:147-171."""
        self._robots = self.get_robot()
        self.initial_root_pos, self.initial_root_rot = self._robots.get_world_poses()
        self.initial_root_pos = self._env_pos + torch.tensor(self._spawn_translation, device=self._device)
        self.initial_root_rot = torch.tensor([1.0, 0.0, 0.0, 0.0], device=self._device).repeat(self.num_envs, 1)
        self.initial_dof_pos = torch.zeros((self.num_envs, self._robots.num_dof), device=self._device)

        self.start_rotation = torch.tensor([1, 0, 0, 0], device=self._device, dtype=torch.float32)
        self.up_vec = torch.tensor([0, 0, 1], dtype=torch.float32, device=self._device).repeat((self.num_envs, 1))
        self.heading_vec = torch.tensor([1, 0, 0], dtype=torch.float32, device=self._device).repeat((self.num_envs, 1))
        self.inv_start_rot = torch.tensor([1, -0.0, -0.0, -0.0], device=self._device).repeat((self.num_envs, 1))
        self.basis_vec0 = self.heading_vec.clone()
        self.basis_vec1 = self.up_vec.clone()
        self.targets = torch.tensor([1000, 0, 0], dtype=torch.float32, device=self._device).repeat((self.num_envs, 1))
        self.target_dirs = torch.tensor([1, 0, 0], dtype=torch.float32, device=self._device).repeat((self.num_envs, 1))
        self.dt = 1.0 / 60.0
        self.potentials = torch.tensor([-1000.0 / self.dt], dtype=torch.float32, device=self._device).repeat(self.num_envs)
        self.prev_potentials = self.potentials.clone()
        self.actions = torch.zeros((self.num_envs, self.num_actions), device=self._device)

        N.check(N.lib().mi_task_configure(self._h(), C.byref(self.task_params())), "mi_task_configure")
        self._set_up_dr()
        indices = torch.arange(self._robots.count, dtype=torch.int64, device=self._device)
        self.reset_idx(indices)

    def calculate_metrics(self) -> None:
        N.check(N.lib().mi_task_metrics(self._h(), self.actions.data_ptr(), self.obs_buf.data_ptr(),
                                        self.rew_buf.data_ptr(), self.potentials.data_ptr(),
                                        self.prev_potentials.data_ptr(), self._stream()),
                "mi_task_metrics")

    def is_done(self) -> None:
        N.check(N.lib().mi_task_is_done(self._h(), self.obs_buf.data_ptr(), self.reset_buf.data_ptr(),
                                        self.progress_buf.data_ptr(), self._stream()), "mi_task_is_done")

    # ------------------------------------------------------------------ fused path
    def fused_step(self, actions: torch.Tensor, out=None):
        """VecEnvRLGames.step in one launch; returns fresh (obs clamped, rew, resets) tensors,
        the copies _process_data hands back (vec_env_rlgames.py:41-46)."""
        a = actions.to(self._device, dtype=torch.float32).contiguous()
        obs_out, rew_out, reset_out = self._step_outputs(out)
        # clip_obs = inf (locomotion default, rl_task.py:69): the clamped copy equals obs_buf. With
        # fresh output tensors (out is None) the launch writes the row once and obs_buf becomes
        # that tensor: the env never writes it again (the next step returns another fresh
        # tensor), so it behaves as the reference's returned .clone() (vec_env_rlgames.py:43) as
        # long as the caller does not modify the returned obs in place and then read
        # task.obs_buf. With caller buffers (a rollout slab row, a graph-pool tensor) obs_buf
        # stays a persistent buffer of its own and the launch writes both
        # (tests/test_gpu_parity.py::test_returned_obs_contract).
        single = math.isinf(self.clip_obs) and out is None
        if not single and getattr(self, "_obs_aliased", False):
            self.obs_buf = torch.empty_like(self.obs_buf)   # never write a tensor handed out
            self._obs_aliased = False
        N.check(N.lib().mi_env_step(self._h(), a.data_ptr(), int(self.control_frequency_inv),
                                    obs_out.data_ptr(), 0 if single else self.obs_buf.data_ptr(),
                                    self.rew_buf.data_ptr(),
                                    self.reset_buf.data_ptr(), self.progress_buf.data_ptr(),
                                    self.potentials.data_ptr(), self.prev_potentials.data_ptr(),
                                    self.actions.data_ptr(), rew_out.data_ptr(), reset_out.data_ptr(),
                                    self._stream()), "mi_env_step")
        if single:
            self.obs_buf = obs_out
            self._obs_aliased = True
        return obs_out, rew_out, reset_out

