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
