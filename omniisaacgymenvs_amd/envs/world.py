"""World / Scene — the slice of omni.isaac.core's World/SimulationContext the tasks touch
(World.step at envs/vec_env_rlgames.py:65, is_playing at tasks/base/rl_task.py:244,
scene.add at tasks/humanoid.py:70). A world step is one physics substep of every registered
articulation (mi_sim_step), stream-ordered on torch's current stream."""
from __future__ import annotations

from typing import List


class World:
    def __init__(self, task, sim_params: dict, device: str, seed: int = 42):
        self._task = task
        self._sim_params = sim_params
        self.device = device
        self.seed = int(seed)
        self._views: List = []
        self.current_time_step_index = 0

    def add_view(self, view) -> None:
        t = self._task
        env = t._env
        view.initialize(sim_params=t._sim_config.mi_sim_params(view.actor_name),
                        num_envs=t.num_envs, env_origins=t.env_pos_cpu, device=t.device,
                        seed=self.seed, env_id_offset=getattr(env, "env_id_offset", 0))
        self._views.append(view)

    def step(self, render: bool = False) -> None:
        for v in self._views:
            v.sim_step(1)
        self.current_time_step_index += 1

    def is_playing(self) -> bool:
        return True

    def get_physics_dt(self) -> float:
        return float(self._task._sim_config.sim_params["dt"])


class Scene:
    def __init__(self, world: World):
        self._world = world

    def add(self, view):
        self._world.add_view(view)
        return view

    def add_default_ground_plane(self, *args, **kwargs) -> None:
        """The ground plane z = 0 is built into the contact model."""
        return None
