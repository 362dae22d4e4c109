"""CartpoleTask (reference: tasks/cartpole.py:41-162): 4 observations, 1 action
(cart force = maxEffort * a), timeout at progress >= 500. Dynamics: the analytic cart-pole
of libmi_sim.so; obs/reward/done/reset are the fused device kernels."""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from .. import native as N
from ..robots.articulations import ArticulationView, Cartpole
from ..tasks.base.rl_task import RLTask


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

    def set_up_scene(self, scene) -> None:
        self.model = self.get_cartpole()
        super().set_up_scene(scene)
        self._cartpoles = ArticulationView(self.model, name="cartpole_view", prim_paths_expr="/World/envs/.*/Cartpole")
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

    def get_observations(self) -> dict:
        N.check(N.lib().mi_task_observations(self._h(), None, self.obs_buf.data_ptr(), None, None,
                                             self._stream()), "mi_task_observations")
        return {self._cartpoles.name: {"obs_buf": self.obs_buf}}

    def pre_physics_step(self, actions) -> None:
        a = actions.to(self._device, dtype=torch.float32).contiguous()
        N.check(N.lib().mi_task_pre_step(self._h(), a.data_ptr(), self.reset_buf.data_ptr(),
                                         self.progress_buf.data_ptr(), None, None, None,
                                         self._stream()), "mi_task_pre_step")

    def reset_idx(self, env_ids) -> None:
        ids = torch.as_tensor(env_ids, device=self._device).to(torch.int64).contiguous()
        N.check(N.lib().mi_task_reset_idx(self._h(), ids.data_ptr(), int(ids.numel()),
                                          self.reset_buf.data_ptr(), self.progress_buf.data_ptr(),
                                          None, None, self._stream()), "mi_task_reset_idx")

    def post_reset(self):
        self._cart_dof_idx = self._cartpoles.get_dof_index("cartJoint")
        self._pole_dof_idx = self._cartpoles.get_dof_index("poleJoint")
        N.check(N.lib().mi_task_configure(self._h(), C.byref(self.task_params())), "mi_task_configure")
        self._set_up_dr()
        indices = torch.arange(self._cartpoles.count, dtype=torch.int64, device=self._device)
        self.reset_idx(indices)

    def calculate_metrics(self) -> None:
        N.check(N.lib().mi_task_metrics(self._h(), None, self.obs_buf.data_ptr(), self.rew_buf.data_ptr(),
                                        None, None, self._stream()), "mi_task_metrics")

    def is_done(self) -> None:
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
