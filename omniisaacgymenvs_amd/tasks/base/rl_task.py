"""RLTask — task base class (reference: tasks/base/rl_task.py:42-251).

Same constructor contract, buffers (dtypes and init values), properties and
``post_physics_step`` orchestration as the reference; the scene is an mi_sim handle instead
of a USD stage, and env origins come from :class:`GridCloner` over the GLOBAL env ids so a
sharded run places env k exactly where a single-GPU run would.
"""
from __future__ import annotations

from abc import abstractmethod

import numpy as np
import torch

from ...robots.articulations import GridCloner
from ...utils.domain_randomization.randomize import Randomizer
from ...utils.spaces import Box


class RLTask:
    def __init__(self, name, env, offset=None) -> None:
        self._name = name
        self.test = self._cfg.get("test", False)
        self._device = self._cfg["sim_device"]
        self._dr_randomizer = Randomizer(self._sim_config)
        print("Task Device:", self._device)

        self.randomize_actions = False
        self.randomize_observations = False

        self.clip_obs = self._cfg["task"]["env"].get("clipObservations", np.inf)
        self.clip_actions = self._cfg["task"]["env"].get("clipActions", np.inf)
        self.rl_device = self._cfg.get("rl_device", "cuda:0")
        self.control_frequency_inv = self._cfg["task"]["env"].get("controlFrequencyInv", 1)
        print("RL device: ", self.rl_device)

        self._env = env
        if not hasattr(self, "_num_agents"):
            self._num_agents = 1
        if not hasattr(self, "_num_states"):
            self._num_states = 0
        if not hasattr(self, "action_space"):
            self.action_space = Box(np.ones(self.num_actions) * -1.0, np.ones(self.num_actions) * 1.0)
        if not hasattr(self, "observation_space"):
            self.observation_space = Box(np.ones(self.num_observations) * -np.inf,
                                         np.ones(self.num_observations) * np.inf)
        if not hasattr(self, "state_space"):
            self.state_space = Box(np.ones(self.num_states) * -np.inf, np.ones(self.num_states) * np.inf)

        self._cloner = GridCloner(spacing=self._env_spacing)
        self.cleanup()

    def cleanup(self) -> None:
        """Torch buffers for RL data collection (rl_task.py:98-107).

        ``obs_buf`` on the fused locomotion step (clip_obs = inf) is rebound to the fresh obs
        tensor that step returns (one HBM write instead of two; LocomotionTask.fused_step): the
        env never writes that tensor again, but an in-place change of the returned obs is visible
        through ``obs_buf`` until the next step. With caller-provided output buffers it stays a
        buffer of its own."""
        self.obs_buf = torch.zeros((self._num_envs, self.num_observations), device=self._device, dtype=torch.float)
        self.states_buf = torch.zeros((self._num_envs, self.num_states), device=self._device, dtype=torch.float)
        self.rew_buf = torch.zeros(self._num_envs, device=self._device, dtype=torch.float)
        self.reset_buf = torch.ones(self._num_envs, device=self._device, dtype=torch.long)
        self.progress_buf = torch.zeros(self._num_envs, device=self._device, dtype=torch.long)
        self.extras = {}

    def set_up_scene(self, scene) -> None:
        """Env grid + ground plane (rl_task.py:109-131). Envs never collide with each other:
        each env is its own articulation instance in the solver."""
        self._scene = scene
        env = self._env
        first = getattr(env, "env_id_offset", 0)
        total = getattr(env, "global_num_envs", None) or self._num_envs
        self.env_pos_cpu = self._cloner.get_clone_positions(total, first, self._num_envs)
        self._env_pos = torch.tensor(self.env_pos_cpu, device=self._device, dtype=torch.float)

    @property
    def default_base_env_path(self):
        return "/World/envs"

    @property
    def default_zero_env_path(self):
        return f"{self.default_base_env_path}/env_0"

    @property
    def name(self):
        return self._name

    @property
    def device(self):
        return self._device

    @property
    def num_envs(self):
        return self._num_envs

    @property
    def num_actions(self):
        return self._num_actions

    @property
    def num_observations(self):
        return self._num_observations

    @property
    def num_states(self):
        return self._num_states

    @property
    def num_agents(self):
        return self._num_agents

    def get_states(self):
        return self.states_buf

    def get_extras(self):
        return self.extras

    def reset(self):
        """Flags all environments for reset (rl_task.py:218-221)."""
        self.reset_buf = torch.ones_like(self.reset_buf)

    def pre_physics_step(self, actions):
        pass

    @abstractmethod
    def post_reset(self):
        pass

    def get_observations(self):
        return {}

    def calculate_metrics(self) -> None:
        pass

    def is_done(self) -> None:
        pass

    def post_physics_step(self):
        """rl_task.py:231-251."""
        self.progress_buf[:] += 1
        if self._env._world.is_playing():
            self.get_observations()
            self.get_states()
            self.calculate_metrics()
            self.is_done()
            self.get_extras()
        return self.obs_buf, self.rew_buf, self.reset_buf, self.extras

    # ---- fused fast path -------------------------------------------------------------
    _FUSABLE = ("pre_physics_step", "post_physics_step", "get_observations", "calculate_metrics",
                "is_done", "get_states", "get_extras", "reset_idx", "get_dof_at_limit_cost")

    def supports_fused_step(self) -> bool:
        """True when this task runs the build's own task methods unmodified, so
        VecEnvRLGames.step may replace pre -> N x World.step -> post by ONE mi_env_step
        (observation / action noise DR included: the launch applies it)."""
        native = getattr(self, "_native_task_class", None)
        if native is None:
            return False
        return all(getattr(type(self), m, None) is getattr(native, m, None) for m in self._FUSABLE)

    def _set_up_dr(self) -> None:
        """Observation / action noise DR from the task YAML (randomize.py:126-174). The
        reference's locomotion and cartpole tasks never call it; here a `domain_randomization`
        block with randomize: True in their YAML turns it on (after mi_task_configure)."""
        if self._dr_randomizer.randomize:
            self._dr_randomizer.set_up_domain_randomization(self)

    def _step_outputs(self, out=None):
        """(obs, rew, reset) buffers a fused launch writes its returned copies into: fresh
        tensors (_process_data's clones), or caller-provided views such as a rollout slab row
        (utils/distributed.py RolloutGather.slot) — checked here, since the kernel trusts them."""
        if out is None:
            return (torch.empty_like(self.obs_buf), torch.empty_like(self.rew_buf),
                    torch.empty_like(self.reset_buf))
        obs, rew, reset = out
        for t, ref in ((obs, self.obs_buf), (rew, self.rew_buf), (reset, self.reset_buf)):
            if t.shape != ref.shape or t.dtype != ref.dtype or t.device != ref.device or not t.is_contiguous():
                raise ValueError(f"step output buffer {tuple(t.shape)} {t.dtype} {t.device} does not "
                                 f"match {tuple(ref.shape)} {ref.dtype} {ref.device} (contiguous)")
        return obs, rew, reset

    def close(self) -> None:
        view = getattr(self, "_robots", None)
        if view is not None:
            view.close()
