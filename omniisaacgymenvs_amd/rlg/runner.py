"""rl_games torch_runner.Runner subset used by scripts/rlgames_train.py:67-84:
``Runner(observer).load(train_cfg_dict)`` then ``run({'train', 'play', 'checkpoint', 'sigma'})``
over the env registered as 'rlgpu' (utils/rlgames/rlgames_utils.py)."""
from __future__ import annotations

from typing import Dict, Optional

from ..utils.rlgames.rlgames_utils import RLGPUEnv
from .a2c_continuous import A2CAgent, A2CPlayer


class Runner:
    def __init__(self, algo_observer=None) -> None:
        self.algo_observer = algo_observer
        self.params: Optional[Dict] = None

    def load(self, config: Dict) -> None:
        params = config["params"]
        algo = params["algo"]["name"]
        if algo != "a2c_continuous":
            raise ValueError(f"algo {algo!r} not supported (a2c_continuous only)")
        if params["model"]["name"] != "continuous_a2c_logstd":
            raise ValueError(f"model {params['model']['name']!r} not supported")
        self.params = params

    def reset(self) -> None:
        pass

    def _env(self):
        cfg = self.params["config"]
        return RLGPUEnv(cfg.get("env_name", "rlgpu"), int(cfg["num_actors"]))

    def run(self, args: Dict):
        checkpoint = args.get("checkpoint") or None
        if args.get("train", False):
            agent = A2CAgent(self._env(), self.params)
            if checkpoint:
                agent.restore(checkpoint)
            return agent.train()
        if args.get("play", False):
            player = A2CPlayer(self._env(), self.params)
            if checkpoint:
                player.restore(checkpoint)
            return player.run()
        raise ValueError("run(): set 'train' or 'play'")
