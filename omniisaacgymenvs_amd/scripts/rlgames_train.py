"""Training / play entry point, mirroring scripts/rlgames_train.py:31-137 of the reference:

    python -m omniisaacgymenvs_amd.scripts.rlgames_train task=Humanoid headless=True
    python -m omniisaacgymenvs_amd.scripts.rlgames_train task=Ant test=True checkpoint=runs/Ant/nn/Ant.pth

Hydra-style overrides are composed by utils/hydra_cfg (hydra-core is not installable here);
the env is VecEnvRLGames over the HIP hot path; the 'rlgpu' registration and the Runner call
follow RLGTrainer.launch_rlg_hydra / run (:41-84); the run's config is dumped to
runs/<name>/config.yaml (:70-75).
"""
from __future__ import annotations

import os
import sys

import torch
import yaml


def main(argv=None) -> int:
    from ..envs.vec_env_rlgames import VecEnvRLGames
    from ..rlg.runner import Runner
    from ..utils.hydra_cfg.hydra_utils import compose
    from ..utils.rlgames.rlgames_utils import register_env
    from ..utils.task_util import initialize_task

    overrides = list(sys.argv[1:] if argv is None else argv)
    cfg = compose(overrides)
    if cfg.get("checkpoint"):
        if not os.path.exists(cfg["checkpoint"]):
            print(f"checkpoint {cfg['checkpoint']} not found")
            return 1
    env = VecEnvRLGames(headless=bool(cfg.get("headless", True)), sim_device=int(cfg.get("device_id", 0)))
    seed = int(cfg.get("seed", 42))
    if seed == -1:
        seed = env.seed(-1)
    else:
        env.seed(seed)
    cfg["seed"] = seed
    cfg["train"]["params"]["seed"] = seed
    env.task_cfg = cfg
    initialize_task(cfg, env)
    cfg["task"]["test"] = cfg.get("test", False)
    register_env("rlgpu", lambda **kwargs: env)
    runner = Runner()
    runner.load(cfg["train"])
    runner.reset()
    exp_dir = os.path.join("runs", str(cfg["train"]["params"]["config"]["name"]))
    os.makedirs(exp_dir, exist_ok=True)
    with open(os.path.join(exp_dir, "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    runner.run({"train": not cfg.get("test", False), "play": bool(cfg.get("test", False)),
                "checkpoint": cfg.get("checkpoint") or None, "sigma": None})
    env.close()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
