"""rl_games adapter (reference: utils/rlgames/rlgames_utils.py:94-118). rl_games is not
installable offline, so :class:`RLGPUEnv` implements the ``IVecEnv`` contract directly; when
rl_games is importable it also subclasses its IVecEnv and can be registered exactly as
scripts/rlgames_train.py:58-63 does (``vecenv.register('RLGPU', ...)``)."""
from __future__ import annotations

try:  # pragma: no cover - rl_games absent in this image
    from rl_games.common import env_configurations, vecenv

    _Base = vecenv.IVecEnv
except Exception:  # noqa: BLE001
    env_configurations = None
    vecenv = None
    _Base = object

_CONFIGS = {}


def register_env(name: str, creator) -> None:
    """env_configurations.register(name, {'vecenv_type': 'RLGPU', 'env_creator': creator})."""
    _CONFIGS[name] = {"vecenv_type": "RLGPU", "env_creator": creator}
    if env_configurations is not None:  # pragma: no cover
        env_configurations.register(name, _CONFIGS[name])


class RLGPUEnv(_Base):
    def __init__(self, config_name, num_actors, **kwargs):
        cfgs = env_configurations.configurations if env_configurations is not None else _CONFIGS
        self.env = cfgs[config_name]["env_creator"](**kwargs)

    def step(self, action):
        return self.env.step(action)

    def reset(self):
        return self.env.reset()

    def get_number_of_agents(self):
        return self.env.get_number_of_agents()

    def get_env_info(self):
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space}
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info
