"""Pins the oracle: Random123 Philox known-answer vectors, and the hand-derived known-answer
tests of SURVEY §8(c) for the task math (the reference has no tests or fixtures; these KATs
are derived from its source text: tasks/shared/locomotion.py, tasks/humanoid.py, tasks/ant.py,
tasks/cartpole.py, envs/vec_env_rlgames.py)."""
import math

import numpy as np
import pytest

from oracle.oracle import OracleSim, cartpole_post_math, loco_post_math, make_buffers, philox
from tests.helpers import sim_params, task_params_from_cfg


def test_philox_random123_kat():
    # Random123 kat_vectors, philox4x32_10
    assert [hex(x) for x in philox([0, 0, 0, 0], [0, 0])] == [
        "0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    assert [hex(x) for x in philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)] == [
        "0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]
    assert [hex(x) for x in philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                                   [0xA4093822, 0x299F31D0])] == [
        "0xd16cfe09", "0x94fdcceb", "0x5001e420", "0x24126ea1"]


def _upright(tp, m, xyz, n=1, q=None, progress=0, reset=0, actions=None, vel=None):
    D, S = m.num_dof, m.num_sensors
    lim = m.dof_limits()
    pos = np.tile(np.asarray(xyz, np.float32), (n, 1))
    quat = np.tile(np.array([1, 0, 0, 0], np.float32), (n, 1))
    vel = np.zeros((n, 6), np.float32) if vel is None else vel
    q = np.zeros((n, D), np.float32) if q is None else q
    qd = np.zeros((n, D), np.float32)
    sens = np.zeros((n, S, 6), np.float32)
    act = np.zeros((n, D), np.float32) if actions is None else actions
    tx, ty = 1000.0 - pos[:, 0], -pos[:, 1]
    pot0 = (-np.sqrt(tx * tx + ty * ty) / (1 / 60)).astype(np.float32)
    return loco_post_math(tp, pos, quat, vel, q, qd, sens, act, lim[:, 0], lim[:, 1],
                          np.full(n, reset), np.full(n, progress), pot0, pot0)


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat1_upright_at_rest(task):
    tp, m, _ = task_params_from_cfg(task)
    x, y, z = 3.0, -2.0, 1.2
    o = _upright(tp, m, (x, y, z))["obs"][0]
    assert o[0] == np.float32(z)
    assert np.all(o[1:7] == 0.0)
    assert o[7] == 0.0 and o[8] == 0.0                       # yaw, roll
    assert o[10] == 1.0                                       # up_proj
    np.testing.assert_allclose(o[11], (1000 - x) / math.hypot(1000 - x, -y), rtol=1e-6)
    np.testing.assert_allclose(o[9], math.atan2(-z, 1000 - x), rtol=1e-6)   # atan2(z, x) quirk


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat2_reward_zero_actions_upright(task):
    tp, m, (gears, ratio, _) = task_params_from_cfg(task)
    r = _upright(tp, m, (0.0, 0.0, 1.3))
    # pot - prev = 0 (same position), heading_proj = 1 > 0.8 -> full heading weight
    lim = m.dof_limits()
    q0 = (2 * 0 - lim[:, 1] - lim[:, 0]) / (lim[:, 1] - lim[:, 0])
    if task == "Humanoid":
        a = np.abs(q0)
        limit = np.sum((a > 0.98) * (0.25 * (a - 0.98) / 0.02) * ratio)
    else:
        limit = np.sum(q0 > 0.99)
    expect = 0.0 + tp.alive_reward_scale + tp.up_weight + tp.heading_weight - limit
    np.testing.assert_allclose(r["rew"][0], expect, rtol=1e-5)
    assert r["reset"][0] == 0 and r["progress"][0] == 1


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat3_death(task):
    tp, m, _ = task_params_from_cfg(task)
    r = _upright(tp, m, (0.0, 0.0, tp.termination_height - 0.01))
    assert r["rew"][0] == np.float32(tp.death_cost)
    assert r["reset"][0] == 1


def test_kat4_timeouts():
    tp, m, _ = task_params_from_cfg("Humanoid")
    # progress is incremented first (rl_task.py:242): 998 -> 999 >= 1000 - 1 -> reset
    assert _upright(tp, m, (0, 0, 1.3), progress=998)["reset"][0] == 1
    assert _upright(tp, m, (0, 0, 1.3), progress=997)["reset"][0] == 0
    # an already-set reset_buf stays set (torch.where(..., reset_buf))
    assert _upright(tp, m, (0, 0, 1.3), reset=1)["reset"][0] == 1
    tpc, _, _ = task_params_from_cfg("Cartpole")
    z = np.zeros((1, 2), np.float32)
    assert cartpole_post_math(tpc, z, z, [0], [498])["reset"][0] == 0   # -> 499: no reset
    assert cartpole_post_math(tpc, z, z, [0], [499])["reset"][0] == 1   # -> 500: reset (no -1)
    # cartpole's is_done does NOT keep a previous reset flag (cartpole.py:155-162)
    assert cartpole_post_math(tpc, z, z, [1], [0])["reset"][0] == 0


def test_kat5_limits():
    tp, m, (gears, ratio, _) = task_params_from_cfg("Humanoid")
    lim = m.dof_limits()
    lo, hi = lim[:, 0], lim[:, 1]
    o = _upright(tp, m, (0, 0, 1.3), q=lo[None, :].copy())["obs"][0]
    np.testing.assert_allclose(o[12:33], -1.0, atol=1e-6)
    o = _upright(tp, m, (0, 0, 1.3), q=hi[None, :].copy())["obs"][0]
    np.testing.assert_allclose(o[12:33], 1.0, atol=1e-6)
    # |unscaled| = 0.99 on joint 0 only -> limit cost 0.125 * ratio_0
    j0 = 0.5 * (0.99 * (hi[0] - lo[0]) + hi[0] + lo[0])
    q = 0.5 * (lo + hi)[None, :].copy()
    q[0, 0] = j0
    r0 = _upright(tp, m, (0, 0, 1.3), q=0.5 * (lo + hi)[None, :].copy())
    r1 = _upright(tp, m, (0, 0, 1.3), q=q)
    np.testing.assert_allclose(r0["rew"][0] - r1["rew"][0], 0.125 * ratio[0], rtol=2e-3)
    # Ant counts scaled > 0.99 only, no abs: -1 costs nothing, +1 costs 1 each
    tpa, ma, _ = task_params_from_cfg("Ant")
    la = ma.dof_limits()
    base = _upright(tpa, ma, (0, 0, 0.6), q=(0.5 * (la[:, 0] + la[:, 1]))[None, :].copy())["rew"][0]
    at_lo = _upright(tpa, ma, (0, 0, 0.6), q=la[None, :, 0].copy())["rew"][0]
    at_hi = _upright(tpa, ma, (0, 0, 0.6), q=la[None, :, 1].copy())["rew"][0]
    np.testing.assert_allclose(base - at_lo, 0.0, atol=1e-4)
    np.testing.assert_allclose(base - at_hi, 8.0, atol=1e-4)


def test_kat6_cartpole_reward():
    tp, _, _ = task_params_from_cfg("Cartpole")
    r = cartpole_post_math(tp, np.array([[0.0, 0.1]], np.float32), np.array([[1.0, 2.0]], np.float32), [0], [0])
    np.testing.assert_allclose(r["rew"][0], 0.97, rtol=1e-6)
    assert r["reset"][0] == 0
    np.testing.assert_array_equal(r["obs"][0], np.array([0.0, 1.0, 0.1, 2.0], np.float32))
    r = cartpole_post_math(tp, np.array([[3.01, 0.0]], np.float32), np.zeros((1, 2), np.float32), [0], [0])
    assert r["rew"][0] == -2.0 and r["reset"][0] == 1
    r = cartpole_post_math(tp, np.array([[0.0, 1.6]], np.float32), np.zeros((1, 2), np.float32), [0], [0])
    assert r["rew"][0] == -2.0 and r["reset"][0] == 1


def test_kat7_vecenv_clamping():
    """Cartpole obs clamped to ±5 in the returned obs, task obs_buf unclamped; actions ±1."""
    tp, m, _ = task_params_from_cfg("Cartpole")
    n = 4
    orc = OracleSim(m, sim_params(), n, np.zeros((n, 3), np.float32), seed=1)
    orc.configure(tp)
    b = make_buffers(n, 4, 1)
    orc.env_step(np.zeros((n, 1), np.float32), 2, b)        # initial resets
    orc.set_dof_state(np.zeros((n, 2), np.float32), np.array([[9.0, 0.0]] * n, np.float32))
    acts = np.array([[3.0], [-3.0], [0.5], [1.0]], np.float32)
    orc.env_step(acts, 2, b)
    assert np.all(np.abs(b["obs"]) <= 5.0)
    assert np.any(np.abs(b["obs_task"]) > 5.0)
    np.testing.assert_array_equal(b["actions"][:, 0], [1.0, -1.0, 0.5, 1.0])


def test_kat8_reset_timing():
    """Done at t => terminal obs at t; re-init in pre_physics_step of t+1; progress = 1 after."""
    tp, m, _ = task_params_from_cfg("Humanoid")
    n = 2
    orc = OracleSim(m, sim_params(), n, np.zeros((n, 3), np.float32), seed=3)
    orc.configure(tp)
    b = make_buffers(n, tp.num_obs, tp.num_actions)
    orc.env_step(np.zeros((n, 21), np.float32), 2, b)
    assert np.all(b["progress"] == 1) and np.all(b["reset"] == 0)
    # drop env 0 below the termination height
    p, q, v = orc.root_state()
    p[0, 2] = 0.3
    orc.set_root_state(p, q, v)
    orc.env_step(np.zeros((n, 21), np.float32), 2, b)
    assert b["reset"][0] == 1 and b["obs"][0, 0] < tp.termination_height   # terminal obs at t
    assert b["rew"][0] == np.float32(tp.death_cost)
    assert b["progress"][0] == 2
    orc.env_step(np.zeros((n, 21), np.float32), 2, b)                     # t+1 re-inits env 0
    assert b["progress"][0] == 1 and b["reset"][0] == 0
    assert b["obs"][0, 0] > 1.0


# --------------------------------------------------------------------------------------------
# Multi-formula KATs, each derived by hand from the reference text:
#   get_observations  tasks/shared/locomotion.py:219-252 (to_target z zeroed, potentials =
#                     -|to_target|/dt, compute_heading_and_up / compute_rot, unscale, the obs cat)
#   calculate_metrics tasks/shared/locomotion.py:290-320; Humanoid limit cost tasks/humanoid.py:120-127
# with dt = 1/60 (locomotion.py:163) and the wxyz quaternion convention. Expected values are
# computed here in float64 from closed forms (rotations by hand), not by calling the oracle.

def _pose(task, pos, quat, vel=None, q=None, qd=None, sens=None, act=None, prev=None):
    tp, m, (gears, ratio, _) = task_params_from_cfg(task)
    D, S = m.num_dof, m.num_sensors
    lim = m.dof_limits()
    mid = (0.5 * (lim[:, 0] + lim[:, 1]))[None, :]
    pos = np.asarray(pos, np.float32)[None, :]
    # the potential at this position as the reference's float32 tensors compute it:
    # -norm(to_target) / dt with dt = 1/60 a float32 (locomotion.py:163, :223)
    tx, ty = np.float32(1000.0) - pos[0, 0], np.float32(0.0) - pos[0, 1]
    pot_here = -np.sqrt(tx * tx + ty * ty) / np.float32(1 / 60)
    out = loco_post_math(tp, pos, np.asarray(quat, np.float32)[None, :],
                         np.zeros((1, 6), np.float32) if vel is None else np.asarray(vel, np.float32)[None, :],
                         mid.astype(np.float32) if q is None else q,
                         np.zeros((1, D), np.float32) if qd is None else qd,
                         np.zeros((1, S, 6), np.float32) if sens is None else sens,
                         np.zeros((1, D), np.float32) if act is None else act,
                         lim[:, 0], lim[:, 1], np.zeros(1), np.zeros(1),
                         np.full(1, pot_here if prev is None else prev, np.float32),
                         np.full(1, pot_here if prev is None else prev, np.float32))
    return tp, m, ratio, out


def _yaw_quat(deg):
    h = math.radians(deg) / 2
    return [math.cos(h), 0.0, 0.0, math.sin(h)]


def _wrap(a):
    return math.atan2(math.sin(a), math.cos(a))   # normalize_angle, locomotion.py:190-192


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
@pytest.mark.parametrize("yaw_deg", [90.0, 45.0, 200.0])
def test_kat9_yawed_torso(task, yaw_deg):
    """Torso yawed about z by psi at (x, y, z): heading_vec = (cos psi, sin psi, 0), up_vec = e_z
    (compute_heading_and_up), so obs7 = wrap(psi) (get_euler_xyz yaw mod 2 pi, then
    normalize_angle), obs8 = 0, obs10 = 1, obs11 = heading_vec . (1000 - x, -y)/|.|, and obs9 =
    wrap(atan2(0 - z, 1000 - x) - psi) (compute_rot's atan2(z, x) target angle)."""
    x, y, z = 4.0, -3.0, 1.1
    psi = math.radians(yaw_deg)
    tp, m, ratio, r = _pose(task, (x, y, z), _yaw_quat(yaw_deg))
    o = r["obs"][0]
    tx, ty = 1000.0 - x, -y
    L = math.hypot(tx, ty)
    np.testing.assert_allclose(o[7], _wrap(psi), atol=2e-6)
    np.testing.assert_allclose(o[8], 0.0, atol=1e-6)
    np.testing.assert_allclose(o[9], _wrap(math.atan2(-z, tx) - psi), atol=2e-6)
    np.testing.assert_allclose(o[10], 1.0, atol=1e-6)
    np.testing.assert_allclose(o[11], (math.cos(psi) * tx + math.sin(psi) * ty) / L, atol=2e-6)
    # reward: heading term switches to hw * obs11 / 0.8 below 0.8 (locomotion.py:290-293)
    h = (math.cos(psi) * tx + math.sin(psi) * ty) / L
    heading = tp.heading_weight if h > 0.8 else tp.heading_weight * h / 0.8
    expect = tp.alive_reward_scale + tp.up_weight + heading     # progress 0, mid-range joints
    np.testing.assert_allclose(r["rew"][0], expect, atol=2e-6)


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat10_moving_tilted_torso_local_frame(task):
    """Torso yawed +90 deg: quat_rotate_inverse maps world (vx, vy, vz) to (vy, -vx, vz) (a
    rotation by -90 deg about z); obs1-3 = that, obs4-6 = the same map of the angular velocity
    times angularVelocityScale (locomotion.py:239-240). A +30 deg roll about x instead: up_vec =
    (0, -sin 30, cos 30) -> obs10 = cos 30 < 0.93 -> no up reward (locomotion.py:296-297), obs8 =
    pi/6, and obs1-3 = (vx, vy cos30 + vz sin30, -vy sin30 + vz cos30)."""
    v, w = (1.0, 2.0, 3.0), (0.1, -0.2, 0.3)
    tp, m, ratio, r = _pose(task, (0.0, 0.0, 1.3), _yaw_quat(90.0), vel=[*v, *w])
    o = r["obs"][0]
    s = tp.angular_velocity_scale
    np.testing.assert_allclose(o[1:4], [v[1], -v[0], v[2]], atol=1e-5)
    np.testing.assert_allclose(o[4:7], [s * w[1], -s * w[0], s * w[2]], atol=1e-6)
    np.testing.assert_allclose(o[0], 1.3, atol=0)
    c, sn = math.cos(math.radians(30)), math.sin(math.radians(30))
    roll_q = [math.cos(math.radians(15)), math.sin(math.radians(15)), 0.0, 0.0]
    tp, m, ratio, r = _pose(task, (0.0, 0.0, 1.3), roll_q, vel=[*v, *w])
    o = r["obs"][0]
    np.testing.assert_allclose(o[1:4], [v[0], v[1] * c + v[2] * sn, -v[1] * sn + v[2] * c], atol=1e-5)
    np.testing.assert_allclose(o[4:7], [s * w[0], s * (w[1] * c + w[2] * sn), s * (-w[1] * sn + w[2] * c)],
                               atol=1e-6)
    np.testing.assert_allclose(o[8], math.pi / 6, atol=2e-6)
    np.testing.assert_allclose(o[7], 0.0, atol=1e-6)
    np.testing.assert_allclose(o[10], c, atol=1e-6)
    np.testing.assert_allclose(o[11], 1.0, atol=1e-6)        # heading_vec stays e_x
    expect = tp.alive_reward_scale + 0.0 + tp.heading_weight   # up_proj 0.866 < 0.93
    np.testing.assert_allclose(r["rew"][0], expect, atol=2e-6)


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat11_dof_and_sensor_scaling(task):
    """obs[12+D:12+2D] = qd * dofVelocityScale, obs[12+2D:12+2D+6S] = sensors (row-major [S, 6])
    * contactForceScale, obs[12+2D+6S:] = actions (locomotion.py:246-249)."""
    tp0, m, _, _ = _pose(task, (0.0, 0.0, 1.3), [1, 0, 0, 0])
    D, S = m.num_dof, m.num_sensors
    qd = np.linspace(-3.0, 4.0, D, dtype=np.float32)[None, :]
    sens = np.arange(S * 6, dtype=np.float32).reshape(1, S, 6) * 7.5 - 40.0
    act = np.linspace(-1.0, 1.0, D, dtype=np.float32)[None, :]
    tp, m, ratio, r = _pose(task, (0.0, 0.0, 1.3), [1, 0, 0, 0], qd=qd, sens=sens, act=act)
    o = r["obs"][0]
    np.testing.assert_allclose(o[12 + D:12 + 2 * D], qd[0].astype(np.float64) * tp.dof_vel_scale, rtol=1e-6)
    np.testing.assert_allclose(o[12 + 2 * D:12 + 2 * D + 6 * S],
                               sens.reshape(-1).astype(np.float64) * tp.contact_force_scale, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(o[12 + 2 * D + 6 * S:], act[0])
    assert o.shape[0] == 12 + 3 * D + 6 * S == tp.num_obs


@pytest.mark.parametrize("task", ["Humanoid", "Ant"])
def test_kat12_full_reward_moving_actions_velocities(task):
    """Every reward term at once (locomotion.py:290-320): torso yawed 45 deg (heading below 0.8:
    hw * cos45 / 0.8), moved 0.1 m toward the target since the previous potential (progress =
    (|to_target_prev| - |to_target|) / dt = 6), non-zero actions and DOF velocities (action cost
    ac * sum a^2, electricity ec * sum |a * qd * dofVelocityScale| * ratio), one joint at 0.995 of
    its range (Humanoid: 0.25 * (0.995 - 0.98) / 0.02 * ratio_j, humanoid.py:120-127; Ant: counts
    unscaled > 0.99, ant.py:92-95)."""
    tp0, m, ratio, _ = _pose(task, (0.0, 0.0, 1.3), [1, 0, 0, 0])
    D = m.num_dof
    lim = m.dof_limits().astype(np.float64)
    lo, hi = lim[:, 0], lim[:, 1]
    q = 0.5 * (lo + hi)
    j = 2
    q[j] = 0.5 * (0.995 * (hi[j] - lo[j]) + hi[j] + lo[j])  # unscale -> 0.995
    act = np.array([(-1) ** k * (0.1 + 0.8 * k / D) for k in range(D)], np.float32)[None, :]
    qd = np.array([0.5 + 0.3 * k for k in range(D)], np.float32)[None, :] * np.where(np.arange(D) % 3 == 0, -1, 1)
    prev = -np.float32(1000.0) / np.float32(1 / 60)            # potential at x = 0, y = 0
    tp, m, ratio, r = _pose(task, (0.1, 0.0, 1.3), _yaw_quat(45.0), q=q[None, :].astype(np.float32),
                            qd=qd.astype(np.float32), act=act, prev=prev)
    a64, qd64 = act[0].astype(np.float64), qd[0].astype(np.float64)
    progress = (1000.0 - 999.9) * 60.0
    heading = tp.heading_weight * math.cos(math.radians(45.0)) / 0.8
    act_cost = float(np.sum(a64 ** 2))
    elec = float(np.sum(np.abs(a64 * qd64 * tp.dof_vel_scale) * np.asarray(ratio, np.float64)))
    if task == "Humanoid":
        limit = tp.joints_at_limit_cost * (0.995 - 0.98) / 0.02 * float(ratio[j])
    else:
        limit = 1.0
    expect = (progress + tp.alive_reward_scale + tp.up_weight + heading
              - tp.actions_cost * act_cost - tp.energy_cost * elec - limit)
    # float32 potentials are ~6e4 in magnitude (ulp 3.9e-3): the progress term carries that error
    np.testing.assert_allclose(r["rew"][0], expect, atol=1.2e-2)
    # the same step without the progress term pins every other term to float32 rounding
    tp, m, ratio, r0 = _pose(task, (0.1, 0.0, 1.3), _yaw_quat(45.0), q=q[None, :].astype(np.float32),
                             qd=qd.astype(np.float32), act=act)
    np.testing.assert_allclose(r0["rew"][0], expect - progress, atol=2e-5)
    np.testing.assert_allclose(r["pot"][0] - prev, progress, atol=1.2e-2)
    assert r["prev"][0] == prev
