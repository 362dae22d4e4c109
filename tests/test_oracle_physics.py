"""Physics self-consistency of the CPU oracle. PhysX is closed, so the build's
integrator is pinned by invariants rather than by reference outputs:
  * ABA (Featherstone) == dense J^T I J mass matrix + Cholesky solve
  * mass matrix symmetric positive definite
  * free flight without gravity: linear + angular momentum conserved
  * no damping / no contact: energy drift bounded (semi-implicit Euler)
  * joint limits respected after a hard push
  * the articulation engine reproduces the analytic cart-pole
"""
import numpy as np
import pytest

from omniisaacgymenvs_amd.robots.model import load_robot, compile_mjcf, asset_path
from oracle.oracle import OracleSim
from tests.helpers import sim_params


def _random_state(sim, m, z, seed, vel_scale=0.5):
    rng = np.random.default_rng(seed)
    n = sim.N
    pos = np.tile([0.0, 0.0, z], (n, 1)).astype(np.float32)
    q4 = rng.normal(size=(n, 4)).astype(np.float32)
    q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
    vel = (rng.normal(size=(n, 6)) * vel_scale).astype(np.float32)
    lo, hi = m.lower[1:], m.upper[1:]
    q = np.clip(rng.uniform(-0.5, 0.5, (n, m.num_dof)), lo, hi).astype(np.float32)
    qd = rng.uniform(-1, 1, (n, m.num_dof)).astype(np.float32)
    sim.set_root_state(pos, q4, vel)
    sim.set_dof_state(q, qd)
    return q, qd


@pytest.mark.parametrize("damp", [0.0, 0.05])
@pytest.mark.parametrize("name", ["Humanoid", "Ant"])
def test_aba_matches_dense_solve(name, damp):
    m = load_robot(name)
    sim = OracleSim(m, sim_params(angular_damping=damp), 4, np.zeros((4, 3), np.float32))
    q, qd = _random_state(sim, m, 3.0, 0)
    rng = np.random.default_rng(1)
    for env in range(4):
        M, Cb = sim.dynamics_terms(env)
        assert np.abs(M - M.T).max() < 1e-5 * np.abs(M).max()
        assert np.linalg.eigvalsh(M.astype(np.float64)).min() > 0
        tau = np.zeros(M.shape[0], np.float32)
        tau[6:] = rng.uniform(-20, 20, m.num_dof)
        rhs = (tau - Cb).astype(np.float64)
        rhs[6:] -= m.damping[1:] * qd[env]
        ref = np.linalg.solve(M.astype(np.float64), rhs)
        got = sim.aba(env, tau)
        np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-3 * np.abs(ref).max())


@pytest.mark.parametrize("name", ["Humanoid", "Ant"])
def test_free_flight_conserves_momentum(name):
    m = load_robot(name)
    m.damping[:] = 0.0
    m.lower[:], m.upper[:] = 1.0, 0.0           # no limits
    sim = OracleSim(m, sim_params(gravity=(0.0, 0.0, 0.0), dt=0.002), 2, np.zeros((2, 3), np.float32))
    _random_state(sim, m, 50.0, 2)
    h0 = [sim.momentum(e) for e in range(2)]
    sim.set_efforts(np.zeros((2, m.num_dof), np.float32))
    for _ in range(100):
        sim.step(1)
    for e in range(2):
        h1 = sim.momentum(e)
        np.testing.assert_allclose(h1[3:], h0[e][3:], rtol=0, atol=2e-3 * max(1.0, np.abs(h0[e][3:]).max()))
        np.testing.assert_allclose(h1[:3], h0[e][:3], rtol=0, atol=2e-2 * max(1.0, np.abs(h0[e][:3]).max()))


def test_energy_drift_bounded():
    m = load_robot("Ant")
    m.damping[:] = 0.0
    m.lower[:], m.upper[:] = 1.0, 0.0
    sim = OracleSim(m, sim_params(dt=0.001), 2, np.zeros((2, 3), np.float32))
    _random_state(sim, m, 100.0, 3, vel_scale=0.3)
    e0 = [sim.energy(e) for e in range(2)]
    sim.set_efforts(np.zeros((2, m.num_dof), np.float32))
    for _ in range(200):
        sim.step(1)
    for e in range(2):
        assert abs(sim.energy(e) - e0[e]) < 0.02 * max(1.0, abs(e0[e]))


@pytest.mark.parametrize("solver", [0, 1])
def test_joint_limits_hold(solver):
    m = load_robot("Humanoid")
    n = 8
    sim = OracleSim(m, sim_params(solver_type=solver), n, np.zeros((n, 3), np.float32))
    sim.set_root_state(np.tile([0, 0, 1.34], (n, 1)).astype(np.float32),
                       np.tile([1, 0, 0, 0], (n, 1)).astype(np.float32), np.zeros((n, 6), np.float32))
    sim.set_dof_state(np.zeros((n, 21), np.float32), np.zeros((n, 21), np.float32))
    gears = np.array([67.5] * 7 + [45.0, 45.0, 45.0, 135.0, 45.0, 45.0, 135.0, 45.0, 90.0, 90.0] + [22.5] * 4)
    sim.set_efforts((np.sign(np.arange(n) % 2 - 0.5)[:, None] * gears[None, :]).astype(np.float32))
    for _ in range(60):
        sim.step(2)
    q, _ = sim.dof_state()
    lo, hi = m.lower[1:], m.upper[1:]
    slack = 0.05  # rad: velocity-level limits with erp=0.2 allow a small transient overshoot
    assert np.all(q >= lo - slack) and np.all(q <= hi + slack)
    assert sim.nan_count() == 0


def test_articulation_matches_analytic_cartpole():
    m_an = load_robot("Cartpole")
    m_ar = compile_mjcf(asset_path("cartpole.xml"))      # same file, generic articulation engine
    n = 16
    rng = np.random.default_rng(5)
    q = rng.uniform(-0.5, 0.5, (n, 2)).astype(np.float32)
    qd = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    eff = np.stack([rng.uniform(-100, 100, n), np.zeros(n)], 1).astype(np.float32)
    outs = []
    for m in (m_an, m_ar):
        sim = OracleSim(m, sim_params(solver_iterations=0), n, np.zeros((n, 3), np.float32))
        sim.set_dof_state(q, qd)
        sim.set_efforts(eff)
        for _ in range(20):
            sim.step(2)
        outs.append(sim.dof_state())
    np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(outs[0][1], outs[1][1], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("solver", [0, 1])
def test_humanoid_settles_without_nan(solver):
    m = load_robot("Humanoid")
    n = 4
    sim = OracleSim(m, sim_params(solver_type=solver), n, np.zeros((n, 3), np.float32))
    sim.set_root_state(np.tile([0, 0, 1.34], (n, 1)).astype(np.float32),
                       np.tile([1, 0, 0, 0], (n, 1)).astype(np.float32), np.zeros((n, 6), np.float32))
    sim.set_dof_state(np.zeros((n, 21), np.float32), np.zeros((n, 21), np.float32))
    sim.set_efforts(np.zeros((n, 21), np.float32))
    for _ in range(200):
        sim.step(2)
    p, _, v = sim.root_state()
    assert sim.nan_count() == 0
    assert np.all(p[:, 2] > 0.0) and np.all(p[:, 2] < 0.5)     # fell and lies on the ground
    assert np.abs(v).max() < 1.0
    s = sim.sensors()
    assert np.isfinite(s).all()


@pytest.mark.parametrize("solver", [0, 1])
def test_self_collision_limits_penetration(solver):
    """Humanoid self-collision (Humanoid.yaml:80): with the pair contacts on, limbs stay
    (nearly) apart under random actions; with them off they pass through each other."""
    from oracle.oracle import OracleSim, make_buffers
    from omniisaacgymenvs_amd.robots.model import load_robot
    from tests.helpers import sim_params, task_params_from_cfg

    m = load_robot("Humanoid")
    assert m.pairs.shape[0] > 100
    worst = {}
    for esc in (1, 0):
        n = 32
        orc = OracleSim(m, sim_params(enable_self_collisions=esc, solver_type=solver), n,
                        np.zeros((n, 3), np.float32), seed=3)
        tp, _, keep = task_params_from_cfg("Humanoid")
        orc.configure(tp, keep=keep)
        b = make_buffers(n, tp.num_obs, tp.num_actions)
        b["reset"][:] = 1
        rng = np.random.default_rng(0)
        w = np.inf
        for step in range(120):
            orc.env_step(rng.uniform(-1, 1, (n, tp.num_actions)).astype(np.float32), 2, b)
            if step % 10 == 9:
                w = min(w, min(orc.self_min_gap(e) for e in range(n)))
        assert orc.nan_count() == 0
        worst[esc] = w
    assert worst[1] > -0.06, worst
    assert worst[0] < worst[1] - 0.03, worst


SPHERE_XML = """<mujoco model="ball"><compiler angle="degree"/><worldbody>
<body name="ball" pos="0 0 5"><freejoint name="root"/><geom type="sphere" size="0.3" density="800"/>
</body></worldbody></mujoco>"""


@pytest.mark.parametrize("damp", [0.05, 2.0])
def test_link_angular_damping_decays_spin(tmp_path, damp):
    """KAT for the per-link angular damping (PhysX link default 0.05,
    docs/transfering_policies_from_isaac_gym.md:74): a free sphere (isotropic inertia, so no
    gyroscopic coupling) spinning without gravity loses angular velocity as
    omega_{n+1} = (1 - c dt) omega_n (semi-implicit step, damping torque -c I omega), and its
    linear velocity is untouched."""
    f = tmp_path / "ball.xml"
    f.write_text(SPHERE_XML)
    m = compile_mjcf(str(f))
    dt, n = 0.0083, 50
    sim = OracleSim(m, sim_params(gravity=(0.0, 0.0, 0.0), dt=dt, angular_damping=damp), 1,
                    np.zeros((1, 3), np.float32))
    w0 = np.array([1.5, -2.0, 0.7], np.float32)
    v0 = np.array([0.3, 0.1, -0.2], np.float32)
    sim.set_root_state(np.array([[0.0, 0.0, 5.0]], np.float32), np.array([[1.0, 0, 0, 0]], np.float32),
                       np.concatenate([v0, w0])[None])
    for _ in range(n):
        sim.step(1)
    _, _, vel = sim.root_state()
    np.testing.assert_allclose(vel[0, 3:], w0 * (1.0 - damp * dt) ** n, rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(vel[0, :3], v0, rtol=1e-5, atol=1e-6)


def test_tgs_without_constraints_equals_pgs():
    """No constraint rows (free flight): every TGS sub-step sees the same velocity u*, so the
    sub-steps' mean is u* and TGS integrates exactly as PGS (include/mi_sim.h MI_SOLVER_TGS)."""
    m = load_robot("Humanoid")
    n = 4
    rng = np.random.default_rng(2)
    states = []
    for solver in (0, 1):
        sim = OracleSim(m, sim_params(gravity=(0.0, 0.0, -9.81), solver_type=solver), n,
                        np.zeros((n, 3), np.float32))
        sim.set_root_state(np.tile([0, 0, 50.0], (n, 1)).astype(np.float32),
                           np.tile([1, 0, 0, 0], (n, 1)).astype(np.float32),
                           rng.uniform(-1, 1, (n, 6)).astype(np.float32) * 0 + 0.3)
        sim.set_dof_state(np.zeros((n, 21), np.float32), np.full((n, 21), 0.05, np.float32))
        sim.set_efforts(np.full((n, 21), 1.0, np.float32))
        for _ in range(3):        # short: no joint reaches a limit (no limit rows either)
            sim.step(2)
        assert sim.contact_count(0) == 0
        states.append((sim.root_state(), sim.dof_state()))
    for a, b in zip(states[0][0] + states[0][1], states[1][0] + states[1][1]):
        assert np.array_equal(a, b)


def test_tgs_resolves_penetration_within_the_substep():
    """A sphere placed 2 cm into the ground: TGS's sub-steps re-evaluate the separation, so one
    substep pushes it out by more than PGS's single Baumgarte correction (erp 0.2) does, and
    neither overshoots above the rest offset by more than the max depenetration allows."""
    import os
    import tempfile
    xml = SPHERE_XML
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ball.xml")
        open(path, "w").write(xml)
        m = compile_mjcf(path)
    heights = {}
    for solver in (0, 1):
        sim = OracleSim(m, sim_params(gravity=(0.0, 0.0, 0.0), solver_type=solver), 1, np.zeros((1, 3), np.float32))
        sim.set_root_state(np.array([[0, 0, 0.3 + 0.001 - 0.02]], np.float32), np.array([[1, 0, 0, 0]], np.float32),
                           np.zeros((1, 6), np.float32))
        sim.step(1)
        heights[solver] = float(sim.root_state()[0][0, 2])
    pen0 = 0.02
    moved = {k: v - (0.3 + 0.001 - pen0) for k, v in heights.items()}
    assert moved[0] > 0 and moved[1] > moved[0], moved
    assert heights[1] <= 0.3 + 0.001 + 1e-4, heights
