"""Pairing by load in the two-envs-per-wavefront kernel (mi_sim.hip pair_env_by_load) and the
envs' independence from their wave partner (VERDICT r5 "next" #3; the reference steps every env
on its own: rl_task.py:127-128, vec_env_rlgames.py:56-78).

Round 5's pairing-by-load build faulted (hipErrorIllegalAddress at the sync after a graph replay)
until the wide PGS addressed its partner's W slab by the partner's env id and its scratch by the
wave index (commit 8741b69; DESIGN §6 "Pairing by load: the round-5 fault"). This test crafts the
layout that fault needed — heavy (wide-path, > 32 constraint rows) envs paired with NON-adjacent
partners, and waves whose BOTH halves are wide — through mi_sim_pair_load, which sets the load
keys the next launch ranks by. It steps the same state under the index pairing and under the
crafted pairing and checks, env by env:
  * every output (obs, reward, reset, progress, potentials) and the next physics state are
    bit-identical under both pairings: an env's result does not depend on its partner, nor on
    whether its partner sends the wave down the narrow or the wide PGS path;
  * copies of one heavy env's state in four slots of a workgroup (partnered with light envs in
    one run, with each other in the other) give bit-identical rows;
  * every env matches the oracle within the one-step parity bounds (tests/parity_bounds.py)."""
import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.utils.task_util import make_env
from tests import parity_bounds as PB
from tests.helpers import oracle_sensitivity, oracle_twin, reset_counts, task_buffers

pytestmark = pytest.mark.gpu

N_ENVS = 2048
WIDE = 32          # mi_pair.hpp kLamRows: a half above this sends its wave to the wide PGS


def _loads(view, keys=None, pairing=-1):
    out = np.zeros(view.count, np.int32)
    kin = None if keys is None else np.ascontiguousarray(keys, np.int32)
    N.check(N.lib().mi_sim_pair_load(view.handle, out.ctypes.data,
                                     None if kin is None else kin.ctypes.data, int(pairing)),
            "mi_sim_pair_load")
    return out


def _snap(env):
    t, v = env.task, env.task.get_robot()
    torch.cuda.synchronize()
    p, q = v.get_world_poses()
    return {"pos": p.clone(), "quat": q.clone(), "vel": v.get_velocities().clone(),
            "q": v.get_joint_positions().clone(), "qd": v.get_joint_velocities().clone(),
            "reset": t.reset_buf.clone(), "prog": t.progress_buf.clone(),
            "pot": t.potentials.clone(), "prev": t.prev_potentials.clone(), "rc": reset_counts(v)}


def _restore(env, s):
    t, v = env.task, env.task.get_robot()
    v.set_world_poses(s["pos"], s["quat"])
    v.set_velocities(s["vel"])
    v.set_joint_positions(s["q"])
    v.set_joint_velocities(s["qd"])
    t.reset_buf.copy_(s["reset"])
    t.progress_buf.copy_(s["prog"])
    t.potentials.copy_(s["pot"])
    t.prev_potentials.copy_(s["prev"])
    N.check(N.lib().mi_set_reset_count(v.handle, np.ascontiguousarray(s["rc"]).ctypes.data),
            "mi_set_reset_count")
    torch.cuda.synchronize()


def _step(env, acts):
    t, v = env.task, env.task.get_robot()
    o, r, d, _ = env.step(acts)
    torch.cuda.synchronize()
    p, q = v.get_world_poses()
    return {"obs": o["obs"].cpu().numpy().copy(), "rew": r.cpu().numpy().copy(),
            "reset": d.cpu().numpy().copy(), "prog": t.progress_buf.cpu().numpy().copy(),
            "pot": t.potentials.cpu().numpy().copy(), "pos": p.cpu().numpy(), "quat": q.cpu().numpy(),
            "vel": v.get_velocities().cpu().numpy(), "q": v.get_joint_positions().cpu().numpy(),
            "qd": v.get_joint_velocities().cpu().numpy()}


def _acts(n, a, k):
    g = torch.Generator().manual_seed(1000 + k)
    return torch.rand((n, a), generator=g) * 2.0 - 1.0


def test_pairing_by_load_is_partner_independent_and_matches_oracle(gpu):
    env = make_env("Humanoid", num_envs=N_ENVS, device="cuda:0", seed=5)
    t, v = env.task, env.task.get_robot()
    assert v.sim_kernel_path()[0] == 2, "the paired kernel is the default for Humanoid"
    A = env.num_actions
    env.reset()
    # free-run until a step from a snapshot has a heavy env that does not reset in that step
    heavy, snap, acts = None, None, None
    for k in range(120):
        s = _snap(env)
        a = _acts(N_ENVS, A, k)
        _loads(v, pairing=0)
        _step(env, a.cuda())
        L = _loads(v)
        cand = [i for i in np.nonzero(L > WIDE)[0] if int(s["reset"][i]) == 0 and int(s["prog"][i]) > 0]
        if cand:
            heavy, snap, acts = int(cand[0]), s, a
            break
    assert heavy is not None, "no env above 32 constraint rows in 120 steps"
    rows = int(L[heavy])
    # the crafted layout: four copies of the heavy env's state (and actions) in one workgroup at
    # slots 0, 3, 9, 14 (not adjacent to each other); index pairing partners each copy with a
    # light neighbour (slots 1, 2, 8, 15); the crafted keys pair 0 with 9 and 3 with 14 (two wide
    # halves per wave), and the light neighbours with each other (narrow path)
    base = (heavy // 16) * 16
    slots = [base + j for j in (0, 3, 9, 14)]
    crafted = {kk: (vv.clone() if torch.is_tensor(vv) else vv.copy()) for kk, vv in snap.items()}
    for sl in slots:
        for kk in ("pos", "quat", "vel", "q", "qd", "reset", "prog", "pot", "prev"):
            crafted[kk][sl] = snap[kk][heavy]
        crafted["rc"][sl] = snap["rc"][heavy]
    acts = acts.clone()
    acts[slots] = acts[heavy].clone()
    keys = np.array(L, np.int32)
    mid = [j for j in range(16) if j not in (0, 3, 9, 14)]
    keys[base + 0], keys[base + 9], keys[base + 3], keys[base + 14] = 100, 0, 99, 1
    for r_, j in enumerate(mid):
        keys[base + j] = 50 + r_
    # run 1: index pairing
    _restore(env, crafted)
    _loads(v, pairing=0)
    out_idx = _step(env, acts.cuda())
    L_idx = _loads(v)
    # run 2: the crafted pairing by load
    _restore(env, crafted)
    _loads(v, keys=keys, pairing=1)
    out_lod = _step(env, acts.cuda())
    _loads(v, pairing=1)
    assert all(L_idx[sl] == rows for sl in slots), (rows, L_idx[slots])   # copies are heavy too
    assert L_idx[slots].min() > WIDE
    # 1) partner independence, env by env, bit for bit
    diff = {}
    for kk in out_idx:
        a_, b_ = out_idx[kk].reshape(N_ENVS, -1), out_lod[kk].reshape(N_ENVS, -1)
        bad = ~np.all((a_ == b_) | (np.isnan(a_) & np.isnan(b_)), axis=1)
        if bad.any():
            diff[kk] = (int(bad.sum()), np.nonzero(bad)[0][:8].tolist(),
                        float(np.nanmax(np.abs(a_[bad].astype(np.float64) - b_[bad]))))
    print(f"[pairing] heavy env {heavy} ({rows} rows), workgroup {base}..{base + 15}, differences {diff}")
    assert not diff, f"per-env results depend on the wave partner: {diff}"
    # 2) the four copies agree with each other in both runs (heavy-light vs heavy-heavy waves)
    for out in (out_idx, out_lod):
        for kk in ("obs", "rew", "pot", "q", "qd", "pos", "quat", "vel"):
            ref = out[kk][slots[0]]
            for sl in slots[1:]:
                assert np.array_equal(out[kk][sl], ref), (kk, sl)
    # 3) the crafted state against the oracle (one-step bounds of tests/parity_bounds.py)
    _restore(env, crafted)
    orc = oracle_twin(env, seed=5)
    b = task_buffers(env)
    groups = PB.group_slices(t.model.num_dof, t.model.num_sensors)
    sg, sr, _ = oracle_sensitivity(env, 5, acts.numpy(), t.control_frequency_inv, b, groups)
    sens = np.maximum(np.max(np.stack(list(sg.values())), axis=0), sr)
    orc.env_step(acts.numpy(), t.control_frequency_inv, b)
    PB.check(PB.bounds_key("Humanoid", v.sim_params.solver_type), groups, out_lod["obs"], out_lod["rew"],
             b["obs"], b["rew"], orc.decision_margin(), sens=sens,
             pot=np.maximum(np.abs(b["pot"]), np.abs(b["prev"])), quantiles=False)
    assert np.array_equal(out_lod["reset"], b["reset"]) and np.array_equal(out_lod["prog"], b["progress"])
    orc.close()
    env.close()
