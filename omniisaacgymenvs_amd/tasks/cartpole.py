"""CartpoleTask (reference: tasks/cartpole.py:41-162): 4 observations, 1 action
(cart force = maxEffort * a), timeout at progress >= 500.

Two pipelines, as in the reference (cfg/config.yaml:20-23):
* GPU (``sim_device=cuda:N``, the default): the analytic cart-pole of libmi_sim.so; obs /
  reward / done / reset are the fused device kernels, and VecEnvRLGames.step is one launch.
* CPU (``pipeline=cpu`` / ``sim_device=cpu``, BASELINE config 1): the task's methods are the
  reference's torch ops on CPU tensors over :class:`CpuCartpoleView` (robots/cpu_cartpole.py),
  stepped method by method. Reset noise is the build's Philox stream on both pipelines
  (utils/philox.py), so the two agree draw for draw."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from .. import native as N
from ..robots.articulations import ArticulationView, Cartpole
from ..robots.cpu_cartpole import CpuCartpoleView
from ..tasks.base.rl_task import RLTask
from ..utils import philox


class CartpoleTask(RLTask):
    def __init__(self, name, sim_config, env, offset=None) -> None:
        self._sim_config = sim_config
        self._cfg = sim_config.config
        self._task_cfg = sim_config.task_config
        self._num_envs = self._task_cfg["env"]["numEnvs"]
        self._env_spacing = self._task_cfg["env"]["envSpacing"]
        self._cartpole_positions = torch.tensor([0.0, 0.0, 2.0])
        self._reset_dist = self._task_cfg["env"]["resetDist"]
        self._max_push_effort = self._task_cfg["env"]["maxEffort"]
        self._max_episode_length = 500
        self._num_observations = 4
        self._num_actions = 1
        RLTask.__init__(self, name, env)
        self._cpu = torch.device(self._device).type == "cpu"

    def set_up_scene(self, scene) -> None:
        self.model = self.get_cartpole()
        super().set_up_scene(scene)
        view = CpuCartpoleView if self._cpu else ArticulationView
        self._cartpoles = view(self.model, name="cartpole_view", prim_paths_expr="/World/envs/.*/Cartpole")
        self._cartpoles.actor_name = "Cartpole"
        scene.add(self._cartpoles)

    def get_cartpole(self):
        return Cartpole()

    def get_robot(self):
        return self._cartpoles

    def _h(self):
        return self._cartpoles.handle

    def _stream(self):
        return self._cartpoles.stream()

    def task_params(self) -> N.MiTaskParams:
        tp = N.MiTaskParams()
        tp.task_kind = N.MI_TASK_CARTPOLE
        tp.num_obs = 4
        tp.num_actions = 1
        tp.clip_actions = float(self.clip_actions)
        tp.clip_obs = float(self.clip_obs)
        tp.max_episode_length = float(self._max_episode_length)
        tp.reset_dist = float(self._reset_dist)
        tp.max_push_effort = float(self._max_push_effort)
        return tp

    def supports_fused_step(self) -> bool:
        return not self._cpu and super().supports_fused_step()

    def get_observations(self) -> dict:
        if self._cpu:                                      # cartpole.py:80-99
            dof_pos = self._cartpoles.get_joint_positions(clone=False)
            dof_vel = self._cartpoles.get_joint_velocities(clone=False)
            self.obs_buf[:, 0] = dof_pos[:, self._cart_dof_idx]
            self.obs_buf[:, 1] = dof_vel[:, self._cart_dof_idx]
            self.obs_buf[:, 2] = dof_pos[:, self._pole_dof_idx]
            self.obs_buf[:, 3] = dof_vel[:, self._pole_dof_idx]
            return {self._cartpoles.name: {"obs_buf": self.obs_buf}}
        N.check(N.lib().mi_task_observations(self._h(), None, self.obs_buf.data_ptr(), None, None,
                                             self._stream()), "mi_task_observations")
        return {self._cartpoles.name: {"obs_buf": self.obs_buf}}

    def pre_physics_step(self, actions) -> None:
        if self._cpu:                                      # cartpole.py:101-112
            reset_env_ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1)
            if len(reset_env_ids) > 0:
                self.reset_idx(reset_env_ids)
            actions = actions.to(self._device)
            forces = torch.zeros((self._cartpoles.count, self._cartpoles.num_dof), dtype=torch.float32)
            forces[:, self._cart_dof_idx] = self._max_push_effort * actions[:, 0]
            indices = torch.arange(self._cartpoles.count, dtype=torch.int32)
            self._cartpoles.set_joint_efforts(forces, indices=indices)
            return
        a = actions.to(self._device, dtype=torch.float32).contiguous()
        N.check(N.lib().mi_task_pre_step(self._h(), a.data_ptr(), self.reset_buf.data_ptr(),
                                         self.progress_buf.data_ptr(), None, None, None,
                                         self._stream()), "mi_task_pre_step")

    def reset_idx(self, env_ids) -> None:
        if self._cpu:                                      # cartpole.py:114-134
            v = self._cartpoles
            env_ids = torch.as_tensor(env_ids).to(torch.int64)
            num_resets = len(env_ids)
            # the reference's four torch.rand(num_resets) draws, in its order: slots 0..3 of
            # the env's Philox counter (global env id, reset count)
            u = philox.uniform4(v.seed, v.env_ids[env_ids], v.reset_count[env_ids])
            dof_pos = torch.zeros((num_resets, v.num_dof))
            dof_pos[:, self._cart_dof_idx] = 1.0 * (1.0 - 2.0 * u[:, 0])
            dof_pos[:, self._pole_dof_idx] = 0.125 * math.pi * (1.0 - 2.0 * u[:, 1])
            dof_vel = torch.zeros((num_resets, v.num_dof))
            dof_vel[:, self._cart_dof_idx] = 0.5 * (1.0 - 2.0 * u[:, 2])
            dof_vel[:, self._pole_dof_idx] = 0.25 * math.pi * (1.0 - 2.0 * u[:, 3])
            indices = env_ids.to(dtype=torch.int32)
            v.set_joint_positions(dof_pos, indices=indices)
            v.set_joint_velocities(dof_vel, indices=indices)
            v.reset_count[env_ids] += 1
            self.reset_buf[env_ids] = 0
            self.progress_buf[env_ids] = 0
            return
        ids = torch.as_tensor(env_ids, device=self._device).to(torch.int64).contiguous()
        N.check(N.lib().mi_task_reset_idx(self._h(), ids.data_ptr(), int(ids.numel()),
                                          self.reset_buf.data_ptr(), self.progress_buf.data_ptr(),
                                          None, None, self._stream()), "mi_task_reset_idx")

    def post_reset(self):
        self._cart_dof_idx = self._cartpoles.get_dof_index("cartJoint")
        self._pole_dof_idx = self._cartpoles.get_dof_index("poleJoint")
        if self._cpu:
            if self._dr_randomizer.randomize:
                raise NotImplementedError("observation / action noise DR runs in the HIP kernels: "
                                          "not available on the CPU pipeline")
            self.reset_idx(torch.arange(self._cartpoles.count, dtype=torch.int64))
            return
        N.check(N.lib().mi_task_configure(self._h(), C.byref(self.task_params())), "mi_task_configure")
        self._set_up_dr()
        indices = torch.arange(self._cartpoles.count, dtype=torch.int64, device=self._device)
        self.reset_idx(indices)

    def calculate_metrics(self) -> None:
        if self._cpu:                                      # cartpole.py:143-153
            cart_pos, cart_vel = self.obs_buf[:, 0], self.obs_buf[:, 1]
            pole_angle, pole_vel = self.obs_buf[:, 2], self.obs_buf[:, 3]
            reward = 1.0 - pole_angle * pole_angle - 0.01 * torch.abs(cart_vel) - 0.005 * torch.abs(pole_vel)
            reward = torch.where(torch.abs(cart_pos) > self._reset_dist, torch.ones_like(reward) * -2.0, reward)
            reward = torch.where(torch.abs(pole_angle) > np.pi / 2, torch.ones_like(reward) * -2.0, reward)
            self.rew_buf[:] = reward
            return
        N.check(N.lib().mi_task_metrics(self._h(), None, self.obs_buf.data_ptr(), self.rew_buf.data_ptr(),
                                        None, None, self._stream()), "mi_task_metrics")

    def is_done(self) -> None:
        if self._cpu:                                      # cartpole.py:155-162
            cart_pos, pole_pos = self.obs_buf[:, 0], self.obs_buf[:, 2]
            resets = torch.where(torch.abs(cart_pos) > self._reset_dist, 1, 0)
            resets = torch.where(torch.abs(pole_pos) > math.pi / 2, 1, resets)
            resets = torch.where(self.progress_buf >= self._max_episode_length, 1, resets)
            # the build's NaN guard (as the device's): a non-finite state resets its env
            resets = torch.where(self._cartpoles.take_nan_flags(), 1, resets)
            self.reset_buf[:] = resets
            return
        N.check(N.lib().mi_task_is_done(self._h(), self.obs_buf.data_ptr(), self.reset_buf.data_ptr(),
                                        self.progress_buf.data_ptr(), self._stream()), "mi_task_is_done")

    def fused_step(self, actions: torch.Tensor, out=None):
        a = actions.to(self._device, dtype=torch.float32).contiguous()
        obs_out, rew_out, reset_out = self._step_outputs(out)
        N.check(N.lib().mi_env_step(self._h(), a.data_ptr(), int(self.control_frequency_inv),
                                    obs_out.data_ptr(), self.obs_buf.data_ptr(), self.rew_buf.data_ptr(),
                                    self.reset_buf.data_ptr(), self.progress_buf.data_ptr(), None, None,
                                    None, rew_out.data_ptr(), reset_out.data_ptr(), self._stream()),
                "mi_env_step")
        return obs_out, rew_out, reset_out


CartpoleTask._native_task_class = CartpoleTask
