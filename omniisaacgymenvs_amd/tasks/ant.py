"""AntLocomotionTask (reference: tasks/ant.py:46-95): 60 observations, 8 actions, gears 15,
limit cost = count of scaled DOF positions > 0.99 (no abs, no scale — as the reference)."""
from __future__ import annotations

import torch

from .. import native as N
from ..robots.articulations import Ant, ArticulationView
from ..tasks.base.rl_task import RLTask
from ..tasks.shared.locomotion import LocomotionTask


class AntLocomotionTask(LocomotionTask):
    TASK_KIND = N.MI_TASK_ANT

    def __init__(self, name, sim_config, env, offset=None) -> None:
        self._sim_config = sim_config
        self._cfg = sim_config.config
        self._task_cfg = sim_config.task_config
        self._num_observations = 60
        self._num_actions = 8
        self._ant_positions = torch.tensor([0, 0, 0.5])
        self._spawn_translation = (0.0, 0.0, 0.5)
        LocomotionTask.__init__(self, name=name, env=env)

    def set_up_scene(self, scene) -> None:
        self.model = self.get_ant()
        RLTask.set_up_scene(self, scene)
        self._ants = ArticulationView(self.model, name="ant_view", prim_paths_expr="/World/envs/.*/Ant/torso")
        self._ants.actor_name = "Ant"
        scene.add(self._ants)

    def get_ant(self):
        return Ant()

    def get_robot(self):
        return self._ants

    def post_reset(self):
        self.joint_gears = torch.tensor([15, 15, 15, 15, 15, 15, 15, 15], dtype=torch.float32, device=self._device)
        dof_limits = self._ants.get_dof_limits()
        self.dof_limits_lower = dof_limits[0, :, 0].to(self._device)
        self.dof_limits_upper = dof_limits[0, :, 1].to(self._device)
        self.motor_effort_ratio = torch.ones_like(self.joint_gears, device=self._device)
        LocomotionTask.post_reset(self)

    def get_dof_at_limit_cost(self):
        """ant.py:92-95 (informational: the device reward kernel fuses it)."""
        return torch.sum(self.obs_buf[:, 12:12 + self._ants.num_dof] > 0.99, dim=-1)


AntLocomotionTask._native_task_class = AntLocomotionTask
