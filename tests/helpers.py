"""Test helpers: build a device env and an oracle twin in the same state."""
from __future__ import annotations

import numpy as np
import torch

from omniisaacgymenvs_amd import native as N
from oracle.oracle import OracleSim, make_buffers


def sim_params(**kw) -> N.MiSimParams:
    p = N.MiSimParams()
    p.dt = 0.0083
    p.gravity[:] = [0.0, 0.0, -9.81]
    p.solver_iterations = 4
    p.contact_offset = 0.02
    p.rest_offset = 0.001
    p.friction = 1.0
    p.max_depenetration_velocity = 10.0
    p.erp = 0.2
    p.enable_self_collisions = 0
    p.max_angular_velocity = 100.0
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def reset_counts(view) -> np.ndarray:
    out = np.zeros(view.count, np.uint32)
    N.check(N.lib().mi_get_reset_count(view.handle, out.ctypes.data), "mi_get_reset_count")
    return out


def oracle_twin(env, seed: int):
    """OracleSim with the device env's model, params, origins, seed and current state."""
    task = env.task
    view = task.get_robot()
    orc = OracleSim(task.model, view.sim_params, task.num_envs, task.env_pos_cpu, seed=seed,
                    env_id_offset=env.env_id_offset)
    orc.configure(task.task_params(), keep=task)
    sync_oracle(env, orc)
    return orc


def sync_oracle(env, orc):
    task = env.task
    view = task.get_robot()
    torch.cuda.synchronize()
    p, q = view.get_world_poses()
    v = view.get_velocities()
    orc.set_root_state(p.cpu().numpy(), q.cpu().numpy(), v.cpu().numpy())
    orc.set_dof_state(view.get_joint_positions().cpu().numpy(), view.get_joint_velocities().cpu().numpy())
    orc.set_reset_count(reset_counts(view))
    torch.cuda.synchronize()


def task_buffers(env):
    task = env.task
    b = make_buffers(task.num_envs, task.num_observations, task.num_actions)
    b["reset"][:] = task.reset_buf.cpu().numpy()
    b["progress"][:] = task.progress_buf.cpu().numpy()
    if hasattr(task, "potentials"):
        b["pot"][:] = task.potentials.cpu().numpy()
        b["prev"][:] = task.prev_potentials.cpu().numpy()
    return b


def rand_actions(n, a, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand((n, a), generator=g) * 2.4 - 1.2)  # exercises the ±1 clamp
