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


def task_params_from_cfg(task_name: str):
    """MiTaskParams straight from the composed task config (no GPU / no task object)."""
    from omniisaacgymenvs_amd.robots.model import load_robot
    from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import compose

    cfg = compose([f"task={task_name}"])["task"]["env"]
    tp = N.MiTaskParams()
    m = load_robot(task_name)
    if task_name == "Cartpole":
        tp.task_kind, tp.num_obs, tp.num_actions = N.MI_TASK_CARTPOLE, 4, 1
        tp.clip_actions, tp.clip_obs = cfg["clipActions"], cfg["clipObservations"]
        tp.max_episode_length = 500.0
        tp.reset_dist, tp.max_push_effort = cfg["resetDist"], cfg["maxEffort"]
        return tp, m, None
    D, S = m.num_dof, m.num_sensors
    tp.task_kind = N.MI_TASK_HUMANOID if task_name == "Humanoid" else N.MI_TASK_ANT
    tp.num_obs, tp.num_actions = 12 + 3 * D + 6 * S, D
    tp.clip_actions, tp.clip_obs = cfg["clipActions"], float("inf")
    tp.max_episode_length = float(cfg["episodeLength"])
    for k_c, k_t in [("powerScale", "power_scale"), ("headingWeight", "heading_weight"),
                     ("upWeight", "up_weight"), ("actionsCost", "actions_cost"),
                     ("energyCost", "energy_cost"), ("dofVelocityScale", "dof_vel_scale"),
                     ("angularVelocityScale", "angular_velocity_scale"),
                     ("contactForceScale", "contact_force_scale"),
                     ("jointsAtLimitCost", "joints_at_limit_cost"), ("deathCost", "death_cost"),
                     ("terminationHeight", "termination_height"),
                     ("alive_reward_scale", "alive_reward_scale")]:
        setattr(tp, k_t, float(cfg[k_c]))
    tp.task_dt = 1.0 / 60.0
    tp.target[:] = [1000.0, 0.0, 0.0]
    tp.init_root_pos[:] = [0.0, 0.0, 1.34 if task_name == "Humanoid" else 0.5]
    tp.init_root_quat[:] = [1.0, 0.0, 0.0, 0.0]
    tp.dof_pos_noise, tp.dof_vel_noise = 0.2, 0.1
    if task_name == "Humanoid":
        gears = np.array([67.5] * 7 + [45.0, 45.0, 45.0, 135.0, 45.0, 45.0, 135.0, 45.0, 90.0, 90.0]
                         + [22.5] * 4, np.float32)
    else:
        gears = np.full(D, 15.0, np.float32)
    ratio = (gears / gears.max()).astype(np.float32) if task_name == "Humanoid" else np.ones(D, np.float32)
    init = np.zeros(D, np.float32)
    tp._keep = (gears, ratio, init)
    tp.joint_gears, tp.motor_effort_ratio, tp.init_dof_pos = N.fptr(gears), N.fptr(ratio), N.fptr(init)
    return tp, m, (gears, ratio, init)


def oracle_sensitivity(env, seed, actions, substeps, bufs_before, groups, rel=2.0 ** -22, rng_seed=0,
                       probes=None, per_probe=None):
    """Oracle-side estimate of how much this step amplifies rounding-level differences, per env
    and observation group: oracle twins of the device's CURRENT state (call before the device
    steps) with root pose (quaternion included) / velocity, q and qd each scaled by
    (1 + rel * u), u ~ U(-1, 1) (2 ulp of float32), stepped with the same actions; the response
    is the largest over `probes` independent perturbations (default tests/parity_bounds.py
    SENS_PROBES: one random direction under-reads an ill-conditioned step's worst direction).
    Returns ({group: [N] max |obs_pert - obs_ref|}, [N] |rew_pert - rew_ref|, the unperturbed
    twin's buffers); per_probe (a list) receives each probe's ({group: ...}, rew) too. Contact /
    PGS conditioning (stacked contacts, near-singular Delassus blocks) shows up here as a large
    value, so a device-vs-oracle difference can be judged against the step's own conditioning
    rather than against the device's measured error."""
    import copy

    from tests.parity_bounds import SENS_PROBES

    probes = SENS_PROBES if probes is None else int(probes)
    rng = np.random.default_rng(rng_seed)
    ref = oracle_twin(env, seed)
    b_ref = copy.deepcopy(bufs_before)
    ref.env_step(actions, substeps, b_ref)
    ref.close()
    out = {g: np.zeros(len(b_ref["rew"])) for g in groups}
    rew = np.zeros(len(b_ref["rew"]))
    for _ in range(probes):
        pert = oracle_twin(env, seed)
        p, q, v = pert.root_state()
        jq, jqd = pert.dof_state()
        f = lambda a: (a * (1.0 + rel * rng.uniform(-1, 1, a.shape))).astype(np.float32)
        if env.task.model.root_free:
            pert.set_root_state(f(p), f(q), f(v))
        pert.set_dof_state(f(jq), f(jqd))
        b_pert = copy.deepcopy(bufs_before)
        pert.env_step(actions, substeps, b_pert)
        pert.close()
        d = np.abs(b_pert["obs"] - b_ref["obs"])
        og = {g: d[:, sl].max(axis=1) for g, sl in groups.items()}
        rg = np.abs(b_pert["rew"] - b_ref["rew"])
        if per_probe is not None:
            per_probe.append((og, rg))
        for g in groups:
            out[g] = np.maximum(out[g], og[g])
        rew = np.maximum(rew, rg)
    return out, rew, b_ref
