"""GPU: the ArticulationView tensor API with the reference's exact call shapes.

The reference drives PhysX through indexed setters:
  * reset_idx (tasks/shared/locomotion.py:130-134): set_joint_positions / set_joint_velocities
    (x [n, D], indices = int64 env_ids), set_world_poses(pos [n, 3], quat [n, 4], indices),
    set_velocities(v [n, 6], indices);
  * pre_physics_step (locomotion.py:111-114): set_joint_efforts(forces [N, D],
    indices = arange(N, int32)); Cartpole passes int32 indices to its setters too
    (tasks/cartpole.py:112,129-130).
Each setter is one scatter kernel into the device state; the getters read it back. The expected
state is the numpy scatter of the same rows (row r of the values goes to env indices[r]);
bit-exact. Efforts have no getter: they are checked through one physics substep against the CPU
oracle stepped from the same state with the numpy-scattered efforts. Edge cases: ragged env
count, duplicate ids (each column from one of the env's rows), out-of-range ids (ignored), empty
index lists.
"""
import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd.utils.task_util import make_env
from tests.helpers import oracle_twin

pytestmark = pytest.mark.gpu
NENV = 257


def _state(view):
    torch.cuda.synchronize()
    p, r = view.get_world_poses(clone=False)
    return {"pos": p.cpu().numpy(), "rot": r.cpu().numpy(), "vel": view.get_velocities().cpu().numpy(),
            "q": view.get_joint_positions().cpu().numpy(), "qd": view.get_joint_velocities().cpu().numpy()}


@pytest.mark.parametrize("idx_dtype", [torch.int64, torch.int32])
@pytest.mark.parametrize("name", ["Humanoid", "Ant", "Cartpole"])
def test_indexed_setters_reference_shapes(gpu, name, idx_dtype):
    env = make_env(name, num_envs=NENV, device="cuda:0", seed=5)
    env.reset()
    view = env.task.get_robot()
    ref = _state(view)
    D = view.num_dof
    rng = np.random.default_rng(7)
    ids = rng.choice(NENV, 61, replace=False)
    n = ids.size
    vals = {"q": rng.uniform(-1, 1, (n, D)), "qd": rng.uniform(-3, 3, (n, D)),
            "pos": rng.uniform(-5, 5, (n, 3)), "rot": rng.normal(size=(n, 4)),
            "vel": rng.uniform(-2, 2, (n, 6))}
    vals["rot"] /= np.linalg.norm(vals["rot"], axis=1, keepdims=True)
    vals = {k: v.astype(np.float32) for k, v in vals.items()}
    t = {k: torch.from_numpy(v).to("cuda:0") for k, v in vals.items()}
    env_ids = torch.from_numpy(ids).to("cuda:0", dtype=idx_dtype)
    # locomotion.py:130-134 (reset_idx), in the reference's order
    view.set_joint_positions(t["q"], indices=env_ids)
    view.set_joint_velocities(t["qd"], indices=env_ids)
    if name != "Cartpole":
        view.set_world_poses(t["pos"], t["rot"], indices=env_ids)
        view.set_velocities(t["vel"], indices=env_ids)
    got = _state(view)
    exp = {k: v.copy() for k, v in ref.items()}
    for k in (("q", "qd") if name == "Cartpole" else ("q", "qd", "pos", "rot", "vel")):
        exp[k][ids] = vals[k]
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
    env.close()


def test_setter_edge_cases(gpu):
    env = make_env("Ant", num_envs=NENV, device="cuda:0", seed=6)
    env.reset()
    view = env.task.get_robot()
    ref = _state(view)
    D = view.num_dof
    # out-of-range ids are ignored, the rest applied
    ids = torch.tensor([3, -1, NENV, NENV + 40, 200], dtype=torch.int64, device="cuda:0")
    q = torch.arange(5 * D, dtype=torch.float32, device="cuda:0").view(5, D)
    view.set_joint_positions(q, indices=ids)
    got = _state(view)
    exp = ref["q"].copy()
    exp[3], exp[200] = q[0].cpu().numpy(), q[4].cpu().numpy()
    assert np.array_equal(got["q"], exp)
    # the same through the int32 setters (mi_set_dof_state_i32 / mi_set_root_state_i32)
    ids32 = torch.tensor([4, -1, NENV, 201], dtype=torch.int32, device="cuda:0")
    view.set_joint_positions(q[:4] + 0.5, indices=ids32)
    view.set_velocities(torch.ones((4, 6), device="cuda:0"), indices=ids32)
    got = _state(view)
    exp[4], exp[201] = (q[0] + 0.5).cpu().numpy(), (q[3] + 0.5).cpu().numpy()
    assert np.array_equal(got["q"], exp)
    expv = ref["vel"].copy()
    expv[[4, 201]] = 1.0
    assert np.array_equal(got["vel"], expv)
    # duplicate ids: element-wise scatter (one lane per (row, column), mi_sim.hip k_rows_to_soa),
    # so each column of the env takes its value from one of the duplicate rows, unspecified
    # which — torch's own index_put_ leaves duplicates undefined, and so does PhysX's indexed
    # setter; a caller that needs whole rows passes unique ids (as reset_idx does)
    ids = torch.tensor([10, 11, 10], dtype=torch.int64, device="cuda:0")
    q2 = torch.stack([torch.full((D,), 1.0), torch.full((D,), 2.0), torch.full((D,), 3.0)]).cuda()
    view.set_joint_positions(q2, indices=ids)
    got = _state(view)
    assert np.array_equal(got["q"][11], np.full(D, 2.0, np.float32))
    assert np.all(np.isin(got["q"][10], [1.0, 3.0]))
    # empty index list: no-op
    before = _state(view)
    view.set_velocities(torch.empty((0, 6), device="cuda:0"), indices=torch.empty(0, dtype=torch.int64,
                                                                                   device="cuda:0"))
    after = _state(view)
    for k in before:
        assert np.array_equal(before[k], after[k])
    env.close()


@pytest.mark.parametrize("name", ["Humanoid", "Ant", "Cartpole"])
def test_indexed_efforts_through_a_substep(gpu, name):
    """set_joint_efforts(forces, indices=arange(N) int32) (locomotion.py:111-114), then a subset
    overwritten (int32 ids); one physics substep against the oracle with the numpy-scattered
    efforts from the identical state."""
    env = make_env(name, num_envs=NENV, device="cuda:0", seed=9)
    env.reset()
    task = env.task
    view = task.get_robot()
    D = view.num_dof
    rng = np.random.default_rng(3)
    F = rng.uniform(-50, 50, (NENV, D)).astype(np.float32)
    ids = rng.choice(NENV, 40, replace=False)
    G = rng.uniform(-50, 50, (ids.size, D)).astype(np.float32)
    orc = oracle_twin(env, seed=9)
    view.set_joint_efforts(torch.from_numpy(F).cuda(), indices=torch.arange(NENV, dtype=torch.int32, device="cuda:0"))
    view.set_joint_efforts(torch.from_numpy(G).cuda(), indices=torch.from_numpy(ids).to("cuda:0", torch.int32))
    view.sim_step(1)
    got = _state(view)
    eff = F.copy()
    eff[ids] = G
    orc.set_efforts(eff)
    orc.step(1)
    p, r, v = orc.root_state()
    q, qd = orc.dof_state()
    tol = 1e-4 if name == "Cartpole" else 2e-3
    np.testing.assert_allclose(got["q"], q, rtol=tol, atol=tol)
    np.testing.assert_allclose(got["qd"], qd, rtol=tol, atol=tol * 10)
    if name != "Cartpole":
        np.testing.assert_allclose(got["pos"], p, rtol=tol, atol=tol)
    orc.close()
    env.close()


# kernel variants the deferred / mirror tests run on: (envs, MI_WAVE_PAIR, expected physics path
# of the locomotion tasks): the default paired kernel (even N), the one-env-per-wave kernel by
# choice (MI_WAVE_PAIR=0) and by an odd N (the paired kernel needs both halves of a wave)
KERNELS = [(256, None, 2), (256, "0", 1), (NENV, None, 1)]


def _make(name, n, pair, monkeypatch, **kw):
    if pair is not None:
        monkeypatch.setenv("MI_WAVE_PAIR", pair)
    env = make_env(name, num_envs=n, device="cuda:0", **kw)
    monkeypatch.delenv("MI_WAVE_PAIR", raising=False)
    return env


def _check_path(env, name, path):
    got = env.task.get_robot().sim_kernel_path()[0]
    assert got == (0 if name == "Cartpole" else path), (name, got)


@pytest.mark.parametrize("n,pair,path", KERNELS)
@pytest.mark.parametrize("name", ["Humanoid", "Ant", "Cartpole"])
def test_deferred_substeps_equal_immediate_launches(gpu, name, n, pair, path, monkeypatch):
    """World.step() twice (vec_env_rlgames.py:64-66) is one launch of two substeps, issued by the
    next call that touches the state (include/mi_sim.h mi_sim_step): bit-identical to one launch
    per World.step (MI_SIM_DEFER=0) through the method-by-method step and the getters — on every
    physics kernel (first / last-substep flags of coalesced launches), and past the 64-substep
    cap of one launch."""
    NENV = n
    ea = _make(name, n, pair, monkeypatch, seed=4)
    monkeypatch.setenv("MI_SIM_DEFER", "0")
    eb = _make(name, n, pair, monkeypatch, seed=4)
    monkeypatch.delenv("MI_SIM_DEFER")
    _check_path(ea, name, path)
    for e in (ea, eb):
        e.use_fused(False)
        e.reset()
    g = torch.Generator().manual_seed(8)
    for k in range(4):
        acts = (torch.rand((NENV, ea.num_actions), generator=g) * 2 - 1).cuda()
        oa, ra, da, _ = ea.step(acts)
        ob, rb, db, _ = eb.step(acts)
        assert torch.equal(oa["obs"], ob["obs"]) and torch.equal(ra, rb) and torch.equal(da, db), k
    # the reference's path (A) order: efforts, two World.step, then the getters
    for e in (ea, eb):
        v = e.task.get_robot()
        v.set_joint_efforts(torch.ones((NENV, v.num_dof), device="cuda:0"))
        e._world.step()
        e._world.step()
    sa, sb = _state(ea.task.get_robot()), _state(eb.task.get_robot())
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    # 70 World.step()s in a row: two launches (64 + 6) when deferred, 70 when not
    for e in (ea, eb):
        for _ in range(70):
            e._world.step()
    sa, sb = _state(ea.task.get_robot()), _state(eb.task.get_robot())
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    ea.close()
    eb.close()


def _direct(view):
    """The state through the per-call gathers (mi_get_root_state / mi_get_dof_state /
    mi_get_sensor_wrench), bypassing the view's mirrors."""
    from omniisaacgymenvs_amd import native as N
    lib, n, D, S = N.lib(), view.count, view.num_dof, view.num_sensors
    t = {k: torch.empty(s, device="cuda:0") for k, s in
         (("pos", (n, 3)), ("rot", (n, 4)), ("vel", (n, 6)), ("q", (n, D)), ("qd", (n, D)), ("sens", (n, S, 6)))}
    st = view.stream()
    assert lib.mi_get_root_state(view.handle, t["pos"].data_ptr(), t["rot"].data_ptr(), t["vel"].data_ptr(), st) == 0
    assert lib.mi_get_dof_state(view.handle, t["q"].data_ptr(), t["qd"].data_ptr(), st) == 0
    if S:
        assert lib.mi_get_sensor_wrench(view.handle, t["sens"].data_ptr(), st) == 0
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in t.items()}


def _mirrored(view):
    p, r = view.get_world_poses(clone=False)
    out = {"pos": p, "rot": r, "vel": view.get_velocities(clone=False), "q": view.get_joint_positions(clone=False),
           "qd": view.get_joint_velocities(clone=False), "sens": view._physics_view.get_force_sensor_forces()}
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("n,pair,path", KERNELS)
@pytest.mark.parametrize("name", ["Humanoid", "Ant", "Cartpole"])
def test_state_mirrors_track_every_state_write(gpu, name, n, pair, path, monkeypatch):
    """The getters' state mirrors (include/mi_sim.h mi_sim_set_mirror / mi_get_state_mirror) equal
    the per-call gathers bit for bit after every kind of state write: deferred World.step()s,
    indexed setters (reset_idx's shapes), the fused env step (its mask-driven resets included) and
    the method-by-method step; clone=False hands out the mirror itself (a view the next step
    overwrites, as Isaac's clone=False), clone=True a copy; a read on another stream is ordered
    after the refresh."""
    NENV = n
    env = _make(name, n, pair, monkeypatch, seed=12)
    _check_path(env, name, path)
    env.reset()
    view = env.task.get_robot()
    D = view.num_dof

    def same():
        a, b = _mirrored(view), _direct(view)
        for k in a:
            assert np.array_equal(a[k], b[k]), k

    same()
    q0 = view.get_joint_positions(clone=False)
    qc = view.get_joint_positions()
    assert view.get_joint_positions(clone=False) is q0 and qc is not q0 and torch.equal(qc, q0)
    before = qc.clone()
    view.set_joint_efforts(torch.full((NENV, D), 3.0, device="cuda:0"))
    env._world.step()
    env._world.step()
    same()                                                   # the deferred substeps, then one refresh
    assert torch.equal(qc, before) and not torch.equal(q0, before)   # the clone kept, the view moved
    ids = torch.tensor([1, 5, 77], dtype=torch.int64, device="cuda:0")
    view.set_joint_velocities(torch.full((3, D), 0.25, device="cuda:0"), indices=ids)
    same()
    if name != "Cartpole":
        view.set_velocities(torch.full((3, 6), 0.5, device="cuda:0"), indices=ids)
        same()
    # int32 ids (Cartpole's, cartpole.py:129-130) take the library's _i32 setters: they mark the
    # mirrors stale as well
    view.set_joint_positions(torch.full((3, D), 0.125, device="cuda:0"), indices=ids.to(torch.int32))
    same()
    if name != "Cartpole":
        view.set_velocities(torch.full((3, 6), -0.5, device="cuda:0"), indices=ids.to(torch.int32))
        same()
    g = torch.Generator().manual_seed(2)
    for fused in (True, False):
        env.use_fused(fused)
        for _ in range(3):
            env.step((torch.rand((NENV, env.num_actions), generator=g) * 2 - 1).cuda())
            same()
    # refresh on the default stream, read on a side stream: the library orders the side stream
    # after the refresh (event wait), so the side copy sees the refreshed mirror
    env._world.step()
    q = view.get_joint_positions(clone=False)            # refresh (default stream)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        q2 = view.get_joint_positions(clone=False)       # valid mirror: event wait only
        copy = q2.clone()
    side.synchronize()
    assert q2 is q and np.array_equal(copy.cpu().numpy(), _direct(view)["q"])
    # read on a side stream, then a step on the default stream that rewrites the mirrors: the
    # write waits for the side stream's queued copy (delayed here so an unordered write would
    # land first), so the copy holds the pre-step state
    before = _direct(view)["q"]
    with torch.cuda.stream(side):
        q3 = view.get_joint_positions(clone=False)
        torch.cuda._sleep(20_000_000)
        late = q3.clone()
    env._world.step()
    env._world.step()
    view.get_joint_positions(clone=False)                # issues the physics (+ mirror) launch
    torch.cuda.synchronize()
    assert np.array_equal(late.cpu().numpy(), before)
    same()
    env.close()


@pytest.mark.parametrize("name", ["Humanoid", "Ant"])
def test_state_mirrors_after_captured_steps(gpu, name):
    """Steps captured in a HIP graph (the physics launch and a getter's refresh inside the
    capture): after each replay the getters' mirrors equal the per-call gathers — events are not
    recorded during capture, so a getter outside it refreshes on its own stream."""
    env = make_env(name, num_envs=256, device="cuda:0", seed=21)
    env.reset()
    view = env.task.get_robot()
    env.use_fused(False)
    acts = (torch.rand((256, env.num_actions), generator=torch.Generator().manual_seed(3)) * 2 - 1).cuda()
    env.step(acts)                                      # warm the method-by-method path
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            view.set_joint_efforts(acts * 2.0)
            env._world.step()
            env._world.step()
            inside = view.get_joint_positions(clone=True)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        a, b = _mirrored(view), _direct(view)
        for k in a:
            assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(inside.cpu().numpy(), b["q"])
    env.close()
