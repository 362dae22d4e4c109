"""Task registry + construction (reference: utils/task_util.py:30-72), restricted to the three
tasks of this build's hot path."""
from __future__ import annotations

from typing import Optional, Sequence


def _task_map():
    from ..tasks.ant import AntLocomotionTask
    from ..tasks.cartpole import CartpoleTask
    from ..tasks.humanoid import HumanoidLocomotionTask

    return {"Ant": AntLocomotionTask, "Cartpole": CartpoleTask, "Humanoid": HumanoidLocomotionTask}


def initialize_task(config, env, init_sim: bool = True):
    from .config_utils.sim_config import SimConfig

    sim_config = SimConfig(config)
    cfg = sim_config.config
    task = _task_map()[cfg["task_name"]](name=cfg["task_name"], sim_config=sim_config, env=env)
    env.set_task(task=task, sim_params=sim_config.get_physics_params(), backend="torch", init_sim=init_sim)
    return task


def make_env(task_name: str, num_envs: Optional[int] = None, device: str = "cuda:0", seed: int = 42,
             overrides: Optional[Sequence[str]] = None, env_id_offset: int = 0,
             global_num_envs: Optional[int] = None):
    """Compose the config the way scripts/rlgames_train.py does and build env + task."""
    from ..envs.vec_env_rlgames import VecEnvRLGames
    from .hydra_cfg.hydra_utils import compose

    ov = [f"task={task_name}", f"seed={seed}"] + list(overrides or [])
    if num_envs is not None:
        ov.append(f"num_envs={int(num_envs)}")
    dev_id = 0
    if device.startswith("cuda"):
        dev_id = int(device.split(":")[1]) if ":" in device else 0
        ov += [f"device_id={dev_id}", f"rl_device={device}"]
    else:
        ov += ["pipeline=cpu", "sim_device=cpu", f"rl_device={device}"]
    cfg = compose(ov)
    env = VecEnvRLGames(headless=True, sim_device=dev_id, env_id_offset=env_id_offset,
                        global_num_envs=global_num_envs)
    env.seed(seed)
    env.task_cfg = cfg
    initialize_task(cfg, env)
    return env
