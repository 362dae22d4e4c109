"""rl_games-compatible PPO learner: the caller of the hot path.
See a2c_continuous.py for what is restated from rl-games 1.5.2 and how it maps to MI355X."""
from .a2c_continuous import A2CAgent, A2CPlayer  # noqa: F401
from .runner import Runner  # noqa: F401
