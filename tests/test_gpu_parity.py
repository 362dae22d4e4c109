"""GPU parity: libmi_sim.so (HIP, gfx950) vs the CPU oracle on identical seeded inputs.

Tolerances (fp32): task math from identical state rtol=atol=1e-4
(transcendentals: device ocml vs glibc differ by a few ulp); one fused env step incl.
physics: tests/parity_bounds.py (per task / field group bounds for envs away from a contact /
limit threshold, a capped oracle-side conditioning allowance needed by < 1 % of the envs, the
float32 quantisation of the potentials; median / 99th-percentile regression bounds per field
group); reset / done masks and progress are compared BIT-EXACT.
"""
import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.utils.task_util import make_env
from oracle import oracle as oracle_mod
from oracle.oracle import lib as orc_lib
from tests.helpers import oracle_sensitivity, oracle_twin, rand_actions, sync_oracle, task_buffers

pytestmark = pytest.mark.gpu
TASKS = ["Cartpole", "Ant", "Humanoid"]


@pytest.fixture(scope="module", params=TASKS)
def env_pair(request, gpu):
    env = make_env(request.param, num_envs=256, device="cuda:0", seed=11)
    orc = oracle_twin(env, seed=11)
    yield request.param, env, orc
    orc.close()
    env.close()


def test_philox_device_matches_oracle(gpu):
    env = make_env("Cartpole", num_envs=128, device="cuda:0", seed=5)
    view = env.task.get_robot()
    out = torch.empty((128, 7), device="cuda:0")
    N.check(N.lib().mi_fill_uniform(view.handle, out.data_ptr(), 7, 1234, 9, -1.0, 1.0, view.stream()))
    got = out.cpu().numpy()
    ref = np.array([[2.0 * orc_lib().orc_uniform(1234, i, 9, c, 1) + -1.0 for c in range(7)]
                    for i in range(128)], np.float32)
    assert np.array_equal(got, ref)
    env.close()


def test_initial_reset_matches_oracle(env_pair):
    """post_reset -> reset_idx(all): Philox noise, clamp to limits, spawn pose."""
    name, env, orc = env_pair
    task = env.task
    view = task.get_robot()
    # re-run the reset on both sides from the same counters
    ids = np.arange(task.num_envs, dtype=np.int64)
    sync_oracle(env, orc)
    b = task_buffers(env)
    task.reset_idx(torch.arange(task.num_envs, device="cuda:0"))
    orc.reset_idx(ids, b)
    torch.cuda.synchronize()
    q_dev = view.get_joint_positions().cpu().numpy()
    qd_dev = view.get_joint_velocities().cpu().numpy()
    q_orc, qd_orc = orc.dof_state()
    assert np.array_equal(q_dev, q_orc)
    assert np.array_equal(qd_dev, qd_orc)
    if name != "Cartpole":
        p_dev, r_dev = view.get_world_poses()
        p_orc, r_orc, _ = orc.root_state()
        assert np.array_equal(p_dev.cpu().numpy(), p_orc)
        assert np.array_equal(r_dev.cpu().numpy(), r_orc)
        np.testing.assert_allclose(task.potentials.cpu().numpy(), b["pot"], rtol=1e-6)


def test_task_math_from_identical_state(env_pair):
    """post_physics_step kernels vs oracle task math on the SAME state (no physics)."""
    name, env, orc = env_pair
    task = env.task
    view = task.get_robot()
    sync_oracle(env, orc)
    n, A, O = task.num_envs, task.num_actions, task.num_observations
    acts = rand_actions(n, A, 3).clamp(-1, 1)
    # randomise the state a bit more so thresholds / limits / falls are exercised
    g = torch.Generator().manual_seed(4)
    q = view.get_joint_positions().cpu()
    q = q + (torch.rand(q.shape, generator=g) - 0.5) * 3.0
    view.set_joint_positions(q.to("cuda:0"))
    if name != "Cartpole":
        p, r = view.get_world_poses()
        p = p.cpu()
        p[:, 2] = torch.rand(n, generator=g) * 1.5
        rq = torch.nn.functional.normalize(torch.randn((n, 4), generator=g), dim=-1)
        view.set_world_poses(p.to("cuda:0"), rq.to("cuda:0"))
        view.set_velocities((torch.randn((n, 6), generator=g)).to("cuda:0"))
    task.progress_buf[:] = torch.randint(0, 1000, (n,), generator=g).to("cuda:0")
    task.reset_buf.zero_()
    torch.cuda.synchronize()
    sync_oracle(env, orc)
    b = task_buffers(env)
    task.actions = acts.to("cuda:0") if name != "Cartpole" else None
    # device: the modular post_physics_step (progress += 1, obs, reward, done)
    task.post_physics_step()
    torch.cuda.synchronize()
    p_orc, r_orc, v_orc = orc.root_state()
    q_orc, qd_orc = orc.dof_state()
    if name == "Cartpole":
        ref = oracle_mod.cartpole_post_math(task.task_params(), q_orc, qd_orc, b["reset"], b["progress"])
    else:
        lim = task.model.dof_limits()
        sens = np.zeros((n, task.model.num_sensors, 6), np.float32)
        ref = oracle_mod.loco_post_math(task.task_params(), p_orc, r_orc, v_orc, q_orc, qd_orc, sens,
                                        acts.numpy(), lim[:, 0], lim[:, 1], b["reset"], b["progress"],
                                        b["pot"], b["prev"])
    b.update(ref)
    obs = task.obs_buf.cpu().numpy()
    if name != "Cartpole":
        obs[:, 12 + 2 * task.model.num_dof: 12 + 2 * task.model.num_dof + 6 * task.model.num_sensors] = 0
        b["obs"][:, 12 + 2 * task.model.num_dof: 12 + 2 * task.model.num_dof + 6 * task.model.num_sensors] = 0
    np.testing.assert_allclose(obs, b["obs"], rtol=1e-4, atol=1e-4)
    assert np.array_equal(task.reset_buf.cpu().numpy(), b["reset"])
    assert np.array_equal(task.progress_buf.cpu().numpy(), b["progress"])
    if name == "Cartpole":
        np.testing.assert_allclose(task.rew_buf.cpu().numpy(), b["rew"], rtol=1e-5, atol=1e-5)


def _sensor_cols(task):
    D, S = task.model.num_dof, task.model.num_sensors
    return slice(12 + 2 * D, 12 + 2 * D + 6 * S)


# One-step bounds (per task / field group, conditioning allowance capped and counted, threshold
# allowance): tests/parity_bounds.py
from tests.parity_bounds import DECISION_EPS, GROUP_TOL, group_slices  # noqa: E402
from tests import parity_bounds  # noqa: E402


def obs_groups(task):
    return group_slices(task.model.num_dof, task.model.num_sensors)


def oracle_sens(env, seed, actions, bufs):
    """Per-env oracle-side rounding sensitivity of the coming step (call BEFORE the device steps;
    None for Cartpole, whose analytic step has no ill-conditioned solve)."""
    if env.task.model.dyn_kind != 0:
        return None
    sg, sr, _ = oracle_sensitivity(env, seed, np.asarray(actions, np.float32),
                                   env.task.control_frequency_inv, bufs, obs_groups(env.task))
    return np.maximum(np.max(np.stack(list(sg.values())), axis=0), sr)


def pot_mag(b):
    return np.maximum(np.abs(b["pot"]), np.abs(b["prev"]))


def check_pair(name, task, obs, rew, obs_ref, rew_ref, tol, margin, sens=None, pot=None,
               quantiles=True):
    """Per-env parity after one fused step from identical state.

    Cartpole: every env within `tol` (1e-4). Locomotion: tests/parity_bounds.check — per task
    and field group base bounds away from decision thresholds, the oracle-side conditioning
    allowance capped at SENS_CAP and needed by fewer than 1 % of the envs (count and widest
    bound printed), the reward's potential quantisation, < 2 % of envs at a threshold differing;
    with `quantiles`, the median / 99th percentile of each group's per-env error within GROUP_TOL."""
    if name == "Cartpole":
        bad = ~np.all(np.isclose(obs, obs_ref, rtol=tol, atol=tol), axis=1)
        bad |= ~np.isclose(rew, rew_ref, rtol=tol, atol=tol)
        assert not bad.any(), f"{name}: envs {np.nonzero(bad)[0]}"
        return None
    key = parity_bounds.bounds_key(name, task.get_robot().sim_params.solver_type)
    return parity_bounds.check(key, obs_groups(task), obs, rew, obs_ref, rew_ref, margin, sens=sens,
                               pot=pot, quantiles=quantiles)


def check_device_pair(name, obs_a, rew_a, obs_b, rew_b, tol, margin):
    """Two DEVICE kernels (e.g. wave vs thread path) run several steps without re-sync: per-env
    within `tol` except envs at a decision threshold (< 2 %)."""
    bad = ~np.all(np.isclose(obs_a, obs_b, rtol=tol, atol=tol), axis=1)
    bad |= ~np.isclose(rew_a, rew_b, rtol=tol, atol=tol)
    near = margin < DECISION_EPS
    unexplained = bad & ~near
    assert not unexplained.any(), (
        f"{name}: envs {np.nonzero(unexplained)[0]} differ with decision margins "
        f"{margin[unexplained]}")
    assert bad.mean() < 0.02, f"{name}: {bad.sum()} envs at a threshold differ"


def test_fused_env_step_matches_oracle(env_pair):
    name, env, orc = env_pair
    task = env.task
    n, A = task.num_envs, task.num_actions
    env.reset()
    torch.cuda.synchronize()
    sync_oracle(env, orc)
    for step in range(3):
        b = task_buffers(env)
        acts = rand_actions(n, A, 100 + step)
        sens = oracle_sens(env, 11, acts.numpy(), b)
        obs_dict, rew, resets, _ = env.step(acts.to("cuda:0"))
        torch.cuda.synchronize()
        orc.env_step(acts.numpy(), task.control_frequency_inv, b)
        tol = 1e-4 if name == "Cartpole" else 2e-3
        check_pair(name, task, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"], b["rew"],
                   tol, orc.decision_margin(), sens=sens, pot=pot_mag(b))
        assert np.array_equal(resets.cpu().numpy(), b["reset"])
        assert np.array_equal(task.progress_buf.cpu().numpy(), b["progress"])
        sync_oracle(env, orc)   # re-align (chaotic contact dynamics)


def test_fused_equals_modular(gpu):
    """One mi_env_step launch == pre + 2 x World.step + post method sequence."""
    for name in TASKS:
        ea = make_env(name, num_envs=128, device="cuda:0", seed=21)
        eb = make_env(name, num_envs=128, device="cuda:0", seed=21)
        eb.use_fused(False)
        assert ea.fused and not eb.fused
        for step in range(5):
            acts = rand_actions(128, ea.num_actions, step).to("cuda:0")
            oa, ra, da, _ = ea.step(acts)
            ob, rb, db, _ = eb.step(acts)
            torch.cuda.synchronize()
            np.testing.assert_allclose(oa["obs"].cpu().numpy(), ob["obs"].cpu().numpy(), rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(ra.cpu().numpy(), rb.cpu().numpy(), rtol=1e-5, atol=1e-5)
            assert torch.equal(da, db)
        ea.close()
        eb.close()


def test_wave_path_matches_thread_path(gpu, monkeypatch):
    """Wavefront-per-env kernel (default) vs the one-lane-per-env reference kernel. The
    one-lane kernel has no self-collision (it refuses it), so Humanoid runs without it here."""
    for name in ("Ant", "Humanoid"):
        ov = [f"task.sim.{name}.enable_self_collisions=False"]
        ea = make_env(name, num_envs=128, device="cuda:0", seed=31, overrides=ov)
        monkeypatch.setenv("MI_SIM_PATH", "thread")
        eb = make_env(name, num_envs=128, device="cuda:0", seed=31, overrides=ov)
        monkeypatch.delenv("MI_SIM_PATH")
        orc = oracle_twin(ea, 31)   # only to measure decision margins of the same state
        for step in range(3):
            acts = rand_actions(128, ea.num_actions, 50 + step)
            sync_oracle(ea, orc)
            orc.env_step(acts.numpy(), ea.task.control_frequency_inv, task_buffers(ea))
            oa, ra, da, _ = ea.step(acts.to("cuda:0"))
            ob, rb, db, _ = eb.step(acts.to("cuda:0"))
            torch.cuda.synchronize()
            check_device_pair(name, oa["obs"].cpu().numpy(), ra.cpu().numpy(), ob["obs"].cpu().numpy(),
                              rb.cpu().numpy(), 2e-3, orc.decision_margin())
            assert torch.equal(da, db)
        ea.close()
        eb.close()


def test_compiled_topology_matches_runtime_tables(gpu, monkeypatch):
    """Model-specialised (compile-time topology) wave kernel vs the runtime-table wave kernel:
    same algorithm and operation order; FMA contraction may differ between the unrolled and the
    looped code, and the two envs run 3 steps without re-sync, hence the 2e-3 bound."""
    for name in ("Ant", "Humanoid"):
        ea = make_env(name, num_envs=128, device="cuda:0", seed=41)
        monkeypatch.setenv("MI_SIM_TOPO", "runtime")
        eb = make_env(name, num_envs=128, device="cuda:0", seed=41)
        monkeypatch.delenv("MI_SIM_TOPO")
        assert ea.task.get_robot().sim_topology() != 0 and eb.task.get_robot().sim_topology() == 0
        orc = oracle_twin(ea, 41)
        for step in range(3):
            acts = rand_actions(128, ea.num_actions, 70 + step)
            sync_oracle(ea, orc)
            orc.env_step(acts.numpy(), ea.task.control_frequency_inv, task_buffers(ea))
            oa, ra, da, _ = ea.step(acts.to("cuda:0"))
            ob, rb, db, _ = eb.step(acts.to("cuda:0"))
            torch.cuda.synchronize()
            check_device_pair(name, oa["obs"].cpu().numpy(), ra.cpu().numpy(), ob["obs"].cpu().numpy(),
                              rb.cpu().numpy(), 2e-3, orc.decision_margin())
            assert torch.equal(da, db)
        ea.close()
        eb.close()


def test_self_collision_on_uncompiled_model_uses_runtime_tables(gpu, monkeypatch):
    """The compiled Ant topology carries no self-collision code (the shipped Ant has no pairs).
    An Ant given self-collision pairs runs on the runtime-table kernel, which has it, and still
    matches the oracle."""
    import omniisaacgymenvs_amd.tasks.ant as ant_mod
    from omniisaacgymenvs_amd.robots.model import asset_path, compile_mjcf

    monkeypatch.setattr(ant_mod, "Ant", lambda: compile_mjcf(asset_path("ant.xml"), sensor_bodies=[
        "front_left_foot", "front_right_foot", "left_back_foot", "right_back_foot"],
        self_collision=True))
    env = make_env("Ant", num_envs=64, device="cuda:0", seed=9,
                   overrides=["task.sim.Ant.enable_self_collisions=True"])
    rob = env.task.get_robot()
    assert rob.model.pairs.shape[0] > 0 and rob.sim_params.enable_self_collisions == 1
    assert rob.sim_topology() == 0
    orc = oracle_twin(env, 9)
    env.reset()
    torch.cuda.synchronize()
    for step in range(3):
        sync_oracle(env, orc)
        b = task_buffers(env)
        acts = rand_actions(64, env.num_actions, 90 + step)
        sens = oracle_sens(env, 9, acts.numpy(), b)
        o, r, d, _ = env.step(acts.to("cuda:0"))
        torch.cuda.synchronize()
        orc.env_step(acts.numpy(), env.task.control_frequency_inv, b)
        check_pair("AntSelf", env.task, o["obs"].cpu().numpy(), r.cpu().numpy(), b["obs"], b["rew"],
                   2e-3, orc.decision_margin(), sens=sens, pot=pot_mag(b))
    env.close()


def test_self_collision_thread_path_refused(gpu, monkeypatch):
    """The one-lane-per-env kernel has no self-collision: asking for it fails loudly."""
    monkeypatch.setenv("MI_SIM_PATH", "thread")
    with pytest.raises(RuntimeError, match="self-collision"):
        make_env("Humanoid", num_envs=8, device="cuda:0", seed=1)


def test_self_collision_active_on_device(gpu):
    """Humanoid (self-collision on) vs the oracle over a longer random rollout, re-synced each
    step; the oracle confirms self-contacts occur in the sampled states."""
    env = make_env("Humanoid", num_envs=256, device="cuda:0", seed=5)
    task = env.task
    assert task.get_robot().sim_params.enable_self_collisions == 1
    orc = oracle_twin(env, 5)
    env.reset()
    torch.cuda.synchronize()
    sync_oracle(env, orc)
    touching = 0
    for step in range(12):
        b = task_buffers(env)
        acts = rand_actions(256, task.num_actions, 300 + step)
        sens = oracle_sens(env, 5, acts.numpy(), b)
        obs_dict, rew, resets, _ = env.step(acts.to("cuda:0"))
        torch.cuda.synchronize()
        orc.env_step(acts.numpy(), task.control_frequency_inv, b)
        check_pair("Humanoid", task, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"],
                   b["rew"], 2e-3, orc.decision_margin(), sens=sens, pot=pot_mag(b))
        assert np.array_equal(resets.cpu().numpy(), b["reset"])
        sync_oracle(env, orc)
        touching += sum(orc.self_min_gap(e) < 0.02 for e in range(0, 256, 8))
    assert touching > 0
    env.close()


@pytest.mark.parametrize("name", ["Humanoid", "Ant"])
def test_pipelined_post_step_equals_one_tile(gpu, monkeypatch, name):
    """k_loco_post_pipe (MI_POST_TILE=32p: each workgroup walks several 32-env tiles and holds
    the next tile's loads in registers; 16p: the same with 16-env tiles) is bit-identical to the
    one-tile kernel (32s). A grid of 7 workgroups over 4113 envs forces many tiles per workgroup
    and a ragged last tile."""
    env = make_env(name, num_envs=4113, device="cuda:0", seed=5)
    t = env.task
    env.reset()
    for k in range(3):
        env.step(rand_actions(t.num_envs, t.num_actions, 40 + k).to("cuda:0"))
    t.actions = rand_actions(t.num_envs, t.num_actions, 50).to("cuda:0")
    t.progress_buf[:] = torch.randint(0, 1000, (t.num_envs,), device="cuda:0")
    t.reset_buf[::3] = 1
    torch.cuda.synchronize()
    bufs = ("obs_buf", "rew_buf", "reset_buf", "progress_buf", "potentials", "prev_potentials")
    start = {b: getattr(t, b).clone() for b in bufs}
    h, s = t.get_robot().handle, t.get_robot().stream()
    out = {}
    for var, grid in (("32s", None), ("32p", "7"), ("32p", None), ("16p", "7")):
        for b in bufs:
            getattr(t, b).copy_(start[b])
        monkeypatch.setenv("MI_POST_TILE", var)
        if grid:
            monkeypatch.setenv("MI_POST_GRID", grid)
        else:
            monkeypatch.delenv("MI_POST_GRID", raising=False)
        N.check(N.lib().mi_task_post_step(h, t.actions.data_ptr(), t.obs_buf.data_ptr(),
                                          t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
                                          t.progress_buf.data_ptr(), t.potentials.data_ptr(),
                                          t.prev_potentials.data_ptr(), s), "mi_task_post_step")
        torch.cuda.synchronize()
        out[(var, grid)] = {b: getattr(t, b).clone() for b in bufs}
        kname, kgrid = t.get_robot().post_kernel()
        # 129 tiles without MI_POST_GRID: under two tiles per resident workgroup, the one-tile kernel
        want = {"32p": "k_loco_post_pipe", "16p": "k_loco_post_pipe<16>"}.get(var) if grid else "k_loco_post_tiled<32s>"
        assert kname == want, (var, grid, kname)
        if grid:
            assert kgrid == int(grid)
    ref = out[("32s", None)]
    assert not torch.equal(ref["obs_buf"], start["obs_buf"])
    for key in (("32p", "7"), ("32p", None), ("16p", "7")):
        for b in bufs:
            assert torch.equal(out[key][b], ref[b]), (key, b)
    env.close()


@pytest.mark.parametrize("var", ["32p", "32s"])
def test_post_step_nan_guard(gpu, monkeypatch, var):
    """The NaN guard inlined in the obs/reward fuse kernels (nan_guard: a non-finite physics state
    forces a reset and counts it): poison the DOF state of a few envs, one physics
    substep sets their nan_flag, one mi_task_post_step must reset exactly those envs (plus the
    ones is_done resets anyway) and count each once; the flags are cleared."""
    env = make_env("Humanoid", num_envs=4113, device="cuda:0", seed=5)
    t, view = env.task, env.task.get_robot()
    env.reset()
    env.step(rand_actions(t.num_envs, t.num_actions, 60).to("cuda:0"))
    monkeypatch.setenv("MI_POST_TILE", var)
    if var == "32p":
        monkeypatch.setenv("MI_POST_GRID", "7")
    bad = torch.tensor([0, 31, 32, 1000, 4112], device="cuda:0", dtype=torch.int64)
    q = view.get_joint_positions()[bad].clone()
    q[:, 3] = float("nan")
    view.set_joint_positions(q, indices=bad)
    env._world.step()
    torch.cuda.synchronize()
    t.progress_buf.zero_()
    t.reset_buf.zero_()
    n0 = view.nan_count()
    N.check(N.lib().mi_task_post_step(view.handle, t.actions.data_ptr(), t.obs_buf.data_ptr(),
                                      t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
                                      t.progress_buf.data_ptr(), t.potentials.data_ptr(),
                                      t.prev_potentials.data_ptr(), view.stream()), "mi_task_post_step")
    torch.cuda.synchronize()
    assert view.post_kernel()[0] == ("k_loco_post_pipe" if var == "32p" else "k_loco_post_tiled<32s>")
    assert view.nan_count() - n0 == len(bad)
    assert (t.reset_buf[bad] == 1).all()
    ok = torch.ones(t.num_envs, dtype=torch.bool, device="cuda:0")
    ok[bad] = False
    # the others reset only where is_done says so (obs[:, 0] = height below the threshold)
    height_reset = t.obs_buf[:, 0] < t.termination_height
    assert torch.equal(t.reset_buf[ok].bool(), height_reset[ok])
    # flags were cleared: a second launch counts nothing new for the poisoned envs' flags
    N.check(N.lib().mi_task_post_step(view.handle, t.actions.data_ptr(), t.obs_buf.data_ptr(),
                                      t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
                                      t.progress_buf.data_ptr(), t.potentials.data_ptr(),
                                      t.prev_potentials.data_ptr(), view.stream()), "mi_task_post_step")
    torch.cuda.synchronize()
    assert view.nan_count() - n0 == len(bad)
    env.close()


def test_modular_step_roctx_ranges(gpu, monkeypatch):
    """the method-by-method step brackets pre_physics_step / the physics substeps /
    post_physics_step in roctx ranges (utils/roctx.py), in the reference's order."""
    from omniisaacgymenvs_amd.utils import roctx

    calls = []

    class Rec:
        def roctxRangePushA(self, name):
            calls.append(("push", name.decode()))
            return 0

        def roctxRangePop(self):
            calls.append(("pop",))
            return 0

    monkeypatch.setattr(roctx, "_LIB", Rec())
    monkeypatch.setattr(roctx, "_TRIED", True)
    env = make_env("Ant", num_envs=64, device="cuda:0", seed=2)
    env.use_fused(False)
    env.step(torch.zeros((64, env.num_actions), device="cuda:0"))
    names = [c[1] for c in calls if c[0] == "push"]
    assert names == ["pre_physics_step", "physics (controlFrequencyInv x World.step)", "post_physics_step"]
    assert sum(c[0] == "pop" for c in calls) == 3
    env.close()


@pytest.mark.parametrize("name", ["Humanoid", "Cartpole"])
def test_returned_obs_contract(gpu, name):
    """The returned obs vs the reference's `_process_data` (vec_env_rlgames.py:43:
    `clamp(obs_buf).clone()`, a tensor independent of the task's obs_buf). Documented deviation
    (LocomotionTask.fused_step, RLTask.cleanup): with clip_obs = inf and fresh outputs, the fused
    launch writes the obs row once and task.obs_buf IS the returned tensor; the env never writes
    a tensor it has handed out (every step returns a new one), so a caller that keeps step k's
    obs sees it unchanged after step k + 1. With a finite clip (Cartpole) or caller buffers
    (out=...), obs_buf is a buffer of its own, as in the reference."""
    env = make_env(name, num_envs=64, device="cuda:0", seed=3)
    t = env.task
    env.reset()
    o1, _, _, _ = env.step(rand_actions(64, t.num_actions, 1).to("cuda:0"))
    obs1 = o1["obs"]
    kept = obs1.clone()
    assert torch.equal(obs1, torch.clamp(t.obs_buf, -t.clip_obs, t.clip_obs))   # the reference's values
    if name == "Humanoid":
        assert obs1.data_ptr() == t.obs_buf.data_ptr()          # the deviation: aliased, not cloned
    else:
        assert obs1.data_ptr() != t.obs_buf.data_ptr()          # finite clip: an independent copy
    o2, _, _, _ = env.step(rand_actions(64, t.num_actions, 2).to("cuda:0"))
    torch.cuda.synchronize()
    assert o2["obs"].data_ptr() != obs1.data_ptr()              # a new tensor every step
    assert torch.equal(obs1, kept)                              # step k's obs untouched by step k + 1
    # caller buffers: obs_buf stays separate (the launch writes both)
    out = (torch.empty_like(kept), torch.empty(64, device="cuda:0"), torch.empty(64, dtype=torch.int64, device="cuda:0"))
    if env.fused:
        o3, _, _, _ = env.step(rand_actions(64, t.num_actions, 3).to("cuda:0"), out=out)
        torch.cuda.synchronize()
        assert o3["obs"].data_ptr() == out[0].data_ptr() != t.obs_buf.data_ptr()
        assert torch.equal(o3["obs"], torch.clamp(t.obs_buf, -t.clip_obs, t.clip_obs))
    env.close()


@pytest.mark.parametrize("z,min_contacts", [(0.08, 11), (0.05, 18)])   # 33+ rows: wide; 54+ rows
@pytest.mark.parametrize("solver", [0, 1])
def test_wide_pgs_pair_with_empty_partner(gpu, solver, z, min_contacts):
    """The paired kernel's wide PGS (a half with 33..64 rows) next to a partner env with no rows
    at all: even envs lie flat on the ground (many contacts), odd envs float (no contact, no
    limit). Both solvers; TGS must still integrate the empty partner with u-bar = u* (the wide
    path skips an empty half). One fused step against the oracle from identical state."""
    n = 64
    env = make_env("Humanoid", num_envs=n, device="cuda:0", seed=9, overrides=[f"solver_type={solver}"])
    task = env.task
    view = task.get_robot()
    assert view.sim_params.solver_type == solver
    env.reset()
    torch.cuda.synchronize()
    pos0, _ = view.get_world_poses()
    pos = pos0.clone()
    s = float(np.sqrt(0.5))
    rot = torch.tensor([[s, 0.0, s, 0.0]] * n, device="cuda:0")      # 90 deg about y: lying
    pos[0::2, 2] = z
    pos[1::2, 2] = 5.0
    rot[1::2] = torch.tensor([1.0, 0.0, 0.0, 0.0], device="cuda:0")
    view.set_world_poses(pos, rot)
    view.set_velocities(torch.zeros((n, 6), device="cuda:0"))
    view.set_joint_positions(torch.zeros((n, task.num_actions), device="cuda:0"))
    view.set_joint_velocities(torch.zeros((n, task.num_actions), device="cuda:0"))
    task.reset_buf.zero_()
    torch.cuda.synchronize()
    orc = oracle_twin(env, 9)
    b = task_buffers(env)
    acts = torch.zeros((n, task.num_actions))
    orc.env_step(acts.numpy(), task.control_frequency_inv, b)
    heavy = [orc.contact_count(e) for e in range(0, n, 2)]
    assert min(heavy) >= min_contacts, heavy        # >= 33 rows: past the narrow path
    assert max(orc.contact_count(e) for e in range(1, n, 2)) == 0
    sync_oracle(env, orc)
    b = task_buffers(env)
    sens = oracle_sens(env, 9, acts.numpy(), b)
    obs_dict, rew, resets, _ = env.step(acts.to("cuda:0"))
    torch.cuda.synchronize()
    orc.env_step(acts.numpy(), task.control_frequency_inv, b)
    check_pair("Humanoid", task, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"], b["rew"],
               2e-3, orc.decision_margin(), sens=sens, pot=pot_mag(b), quantiles=False)
    assert np.array_equal(resets.cpu().numpy(), b["reset"])
    p_dev, _ = view.get_world_poses()
    p_orc = orc.root_state()[0]
    np.testing.assert_allclose(p_dev.cpu().numpy()[1::2], p_orc[1::2], rtol=1e-5, atol=1e-5)
    orc.close()
    env.close()


@pytest.mark.parametrize("solver", [1, 0])
@pytest.mark.parametrize("name", ["Ant", "Humanoid"])
def test_velocity_iterations_match_oracle(gpu, name, solver):
    """solver_velocity_iteration_count = 2 (the reference configs ship 0, but the knob is part of
    the physx block every task reads): under TGS, after the 4 position iterations two more sweeps
    with speculative bias only and no further sub-step motion; under PGS, 6 sweeps
    (include/mi_sim.h).
    One fused step from identical state against the oracle, the solver's parity bounds, reset /
    progress bit-exact; the sweeps must change the result (the knob is not ignored)."""
    ov = [f"solver_type={solver}", f"task.sim.{name}.solver_velocity_iteration_count=2"]
    env = make_env(name, num_envs=512, device="cuda:0", seed=17, overrides=ov)
    ref = make_env(name, num_envs=512, device="cuda:0", seed=17, overrides=[f"solver_type={solver}"])
    sp, sr = env.task.get_robot().sim_params, ref.task.get_robot().sim_params
    assert sp.solver_type == sr.solver_type == solver
    if solver == 1:     # TGS: separate velocity sweeps
        assert (sp.solver_iterations, sp.velocity_iterations, sr.velocity_iterations) == (4, 2, 0)
    else:               # PGS: the sum as sweeps (utils/config_utils/sim_config.py)
        assert (sp.solver_iterations, sp.velocity_iterations, sr.solver_iterations) == (6, 0, 4)
    orc = oracle_twin(env, 17)
    task = env.task
    env.reset()
    ref.reset()
    differs = False
    for step in range(3):
        sync_oracle(env, orc)
        b = task_buffers(env)
        acts = rand_actions(512, task.num_actions, 300 + step)
        sens = oracle_sens(env, 17, acts.numpy(), b)
        obs_dict, rew, resets, _ = env.step(acts.to("cuda:0"))
        ro, _, _, _ = ref.step(acts.to("cuda:0"))
        torch.cuda.synchronize()
        orc.env_step(acts.numpy(), task.control_frequency_inv, b)
        check_pair(name, task, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"], b["rew"], 2e-3,
                   orc.decision_margin(), sens=sens, pot=pot_mag(b))
        assert np.array_equal(resets.cpu().numpy(), b["reset"])
        assert np.array_equal(task.progress_buf.cpu().numpy(), b["progress"])
        differs |= not torch.equal(obs_dict["obs"], ro["obs"])
    assert differs
    orc.close()
    env.close()
    ref.close()
