"""Training / play entry point, mirroring scripts/rlgames_train.py:31-137 of the reference:

    python -m omniisaacgymenvs_amd.scripts.rlgames_train task=Humanoid headless=True
    python -m omniisaacgymenvs_amd.scripts.rlgames_train task=Ant test=True checkpoint=runs/Ant/nn/Ant.pth

Hydra-style overrides are composed by utils/hydra_cfg (hydra-core is not installable here);
the env is VecEnvRLGames over the HIP hot path; the 'rlgpu' registration and the Runner call
follow RLGTrainer.launch_rlg_hydra / run (:41-84); the run's config is dumped to
runs/<name>/config.yaml (:70-75).

Multi-GPU (one process per GPU):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m omniisaacgymenvs_amd.scripts.rlgames_train task=Humanoid train.params.config.multi_gpu=True

Rank r drives device LOCAL_RANK and owns envs [r n, (r + 1) n) of the global grid (num_envs per
rank). train.params.config.multi_gpu_mode picks the learner (rlg.a2c_continuous):
data_parallel (default, rl_games' multi_gpu: a learner per rank, gradients + KL all-reduced per
minibatch) or central (rank 0 learns on one rollout gather per horizon, weights broadcast back).
Only rank 0 writes run files.
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
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:   # torch.distributed.run: this rank's device
        local = int(os.environ.get("LOCAL_RANK", "0"))
        overrides += [f"device_id={local}", f"rl_device=cuda:{local}"]
    cfg = compose(overrides)
    if cfg.get("checkpoint"):
        if not os.path.exists(cfg["checkpoint"]):
            print(f"checkpoint {cfg['checkpoint']} not found")
            return 1
    multi = bool(cfg["train"]["params"]["config"].get("multi_gpu", False)) and int(os.environ.get("WORLD_SIZE", "1")) > 1
    rank, world, offset, total = 0, 1, 0, None
    if multi:
        import torch.distributed as dist
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        n = int(cfg["task"]["env"]["numEnvs"])
        offset, total = rank * n, world * n
    env = VecEnvRLGames(headless=bool(cfg.get("headless", True)), sim_device=int(cfg.get("device_id", 0)),
                        env_id_offset=offset, global_num_envs=total)
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
    if rank == 0:
        exp_dir = os.path.join("runs", str(cfg["train"]["params"]["config"]["name"]))
        os.makedirs(exp_dir, exist_ok=True)
        with open(os.path.join(exp_dir, "config.yaml"), "w") as f:
            yaml.safe_dump(cfg, f, sort_keys=False)
    runner.run({"train": not cfg.get("test", False), "play": bool(cfg.get("test", False)),
                "checkpoint": cfg.get("checkpoint") or None, "sigma": None})
    env.close()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if multi:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
