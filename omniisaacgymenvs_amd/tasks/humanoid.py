"""HumanoidLocomotionTask (reference: tasks/humanoid.py:47-127): 87 observations, 21 actions,
per-joint gears in BFS DOF order, limit cost weighted by the motor effort ratio."""
from __future__ import annotations

import torch

from .. import native as N
from ..robots.articulations import ArticulationView, Humanoid
from ..tasks.base.rl_task import RLTask
from ..tasks.shared.locomotion import LocomotionTask


class HumanoidLocomotionTask(LocomotionTask):
    TASK_KIND = N.MI_TASK_HUMANOID

    def __init__(self, name, sim_config, env, offset=None) -> None:
        self._sim_config = sim_config
        self._cfg = sim_config.config
        self._task_cfg = sim_config.task_config
        self._num_observations = 87
        self._num_actions = 21
        self._humanoid_positions = torch.tensor([0, 0, 1.34])
        self._spawn_translation = (0.0, 0.0, 1.34)
        LocomotionTask.__init__(self, name=name, env=env)

    def set_up_scene(self, scene) -> None:
        self.model = self.get_humanoid()
        RLTask.set_up_scene(self, scene)
        self._humanoids = ArticulationView(self.model, name="humanoid_view",
                                           prim_paths_expr="/World/envs/.*/Humanoid/torso")
        self._humanoids.actor_name = "Humanoid"
        scene.add(self._humanoids)

    def get_humanoid(self):
        return Humanoid()

    def get_robot(self):
        return self._humanoids

    def post_reset(self):
        # gears in BFS DOF order (humanoid.py:82-107)
        self.joint_gears = torch.tensor(
            [67.5, 67.5,            # lower_waist
             67.5, 67.5,            # right_upper_arm
             67.5, 67.5,            # left_upper_arm
             67.5,                  # pelvis
             45.0, 45.0,            # right / left lower arm
             45.0, 135.0, 45.0,     # right_thigh x y z
             45.0, 135.0, 45.0,     # left_thigh x y z
             90.0, 90.0,            # knees
             22.5, 22.5, 22.5, 22.5],  # feet
            device=self._device)
        self.max_motor_effort = torch.max(self.joint_gears)
        self.motor_effort_ratio = self.joint_gears / self.max_motor_effort
        dof_limits = self._humanoids.get_dof_limits()
        self.dof_limits_lower = dof_limits[0, :, 0].to(self._device)
        self.dof_limits_upper = dof_limits[0, :, 1].to(self._device)
        LocomotionTask.post_reset(self)

    def get_dof_at_limit_cost(self):
        """humanoid.py:120-127 (informational: the device reward kernel fuses it)."""
        obs = self.obs_buf[:, 12:33]
        scaled = self.joints_at_limit_cost_scale * (torch.abs(obs) - 0.98) / 0.02
        return torch.sum((torch.abs(obs) > 0.98) * scaled * self.motor_effort_ratio.unsqueeze(0), dim=-1)


HumanoidLocomotionTask._native_task_class = HumanoidLocomotionTask
