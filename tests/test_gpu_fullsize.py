"""GPU tests at BASELINE.json's full sizes (configs 1-4: 4096 envs per GPU).

- oracle parity at 4096 envs: one fused env step from the device state, checked env by env
  against the CPU oracle (multi-threaded) with the locomotion tolerance and the decision-margin
  allowance; reset / progress masks bit-exact;
- idempotence: two sims with the same seed produce bit-identical rollouts (the launch is
  deterministic: no atomics on the data path, fixed summation orders);
- shard invariance (config 5's partitioning, on one GPU): the global grid of 4096 envs run as
  two shards [0, 2048) and [2048, 4096) (env_id_offset, global_num_envs) equals the single
  4096-env sim bit for bit — what every rank of a multi-GPU run computes for its envs;
- rollout properties over 64 steps: finite obs / rewards, most humanoids toppled and reset
  under random actions, NaN guard silent.
"""
import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.utils.task_util import make_env
from oracle.oracle import lib as orc_lib
from tests.helpers import oracle_twin, sync_oracle, task_buffers
from tests.test_gpu_parity import check_pair, oracle_sens, pot_mag

pytestmark = pytest.mark.gpu

TASKS = ["Cartpole", "Ant", "Humanoid"]
NFULL = 4096


def _actions(env, k, seed=42):
    view = env.task.get_robot()
    a = torch.empty((env.num_envs, env.num_actions), device="cuda:0")
    N.check(N.lib().mi_fill_uniform(view.handle, a.data_ptr(), env.num_actions, seed, k, -1.0, 1.0,
                                    view.stream()), "mi_fill_uniform")
    return a


@pytest.mark.parametrize("name", TASKS)
def test_full_size_step_matches_oracle(gpu, name):
    env = make_env(name, num_envs=NFULL, device="cuda:0", seed=3)
    task = env.task
    env.reset()
    for k in range(3):                 # leave the reset-only regime
        env.step(_actions(env, k))
    torch.cuda.synchronize()
    orc_lib().orc_set_threads(8)
    orc = oracle_twin(env, seed=3)
    for k in range(3, 5):
        b = task_buffers(env)
        acts = _actions(env, k)
        sens = oracle_sens(env, 3, acts.cpu().numpy(), b)
        obs_dict, rew, resets, _ = env.step(acts)
        torch.cuda.synchronize()
        orc.env_step(acts.cpu().numpy(), task.control_frequency_inv, b)
        tol = 1e-4 if name == "Cartpole" else 2e-3
        check_pair(name, task, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"], b["rew"],
                   tol, orc.decision_margin(), sens=sens, pot=pot_mag(b))
        assert np.array_equal(resets.cpu().numpy(), b["reset"])
        assert np.array_equal(task.progress_buf.cpu().numpy(), b["progress"])
        sync_oracle(env, orc)
    orc.close()
    orc_lib().orc_set_threads(1)
    env.close()


@pytest.mark.parametrize("name", TASKS)
def test_full_size_deterministic_and_shard_invariant(gpu, name):
    full = make_env(name, num_envs=NFULL, device="cuda:0", seed=8)
    again = make_env(name, num_envs=NFULL, device="cuda:0", seed=8)
    half = NFULL // 2
    shards = [make_env(name, num_envs=half, device="cuda:0", seed=8, env_id_offset=r * half,
                       global_num_envs=NFULL) for r in range(2)]
    for e in [full, again] + shards:
        e.reset()
    for k in range(12):
        a = _actions(full, k)
        of, rf, df, _ = full.step(a)
        oa, ra, da, _ = again.step(a)
        parts = [s.step(a[r * half:(r + 1) * half].contiguous()) for r, s in enumerate(shards)]
        torch.cuda.synchronize()
        assert torch.equal(of["obs"], oa["obs"]) and torch.equal(rf, ra) and torch.equal(df, da)
        assert torch.equal(of["obs"], torch.cat([p[0]["obs"] for p in parts]))
        assert torch.equal(rf, torch.cat([p[1] for p in parts]))
        assert torch.equal(df, torch.cat([p[2] for p in parts]))
    for e in [full, again] + shards:
        e.close()


@pytest.mark.parametrize("name", TASKS)
def test_full_size_rollout_properties(gpu, name):
    env = make_env(name, num_envs=NFULL, device="cuda:0", seed=12)
    env.reset()
    ever_reset = torch.zeros(NFULL, dtype=torch.bool, device="cuda:0")
    total = torch.zeros((), dtype=torch.float64, device="cuda:0")
    for k in range(64):
        obs, rew, done, _ = env.step(_actions(env, k, seed=12))
        assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
        ever_reset |= done.bool()
        total += rew.double().sum()
    torch.cuda.synchronize()
    assert torch.isfinite(total)
    if name == "Humanoid":
        # random actions topple most humanoids within 64 steps (terminationHeight 0.8)
        assert ever_reset.float().mean().item() > 0.5
    assert env.task.get_robot().nan_count() == 0
    env.close()


@pytest.mark.parametrize("name", ["Humanoid", "Ant"])
@pytest.mark.parametrize("n", [4113, 524288])
def test_obs_reward_fuse_matches_oracle(gpu, name, n):
    """RLTask.post_physics_step as ONE launch (mi_task_post_step, the obs/reward fuse bench.py
    reports) against the oracle's post_physics_step math on the same device state. 4113 envs run
    the one-tile kernel (ragged last tile); 524 288 envs the pipelined kernel (8 tiles per
    resident workgroup). Checked on 2048 sampled envs: obs rtol = atol = 1e-4 (device ocml vs
    glibc transcendentals), reward likewise except where the heading / up bonus decision sits
    within 1e-4 of its threshold, reset / progress / potentials' bookkeeping bit-exact."""
    env = make_env(name, num_envs=n, device="cuda:0", seed=9)
    t, view = env.task, env.task.get_robot()
    env.reset()
    for k in range(3):
        env.step(_actions(env, k))
    t.actions = _actions(env, 7)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    t.progress_buf[:] = torch.randint(0, 1000, (n,), device="cuda:0", generator=g)
    t.progress_buf[::7] = 999                     # episode-length resets among the samples
    torch.cuda.synchronize()
    idx = np.sort(np.random.default_rng(0).choice(n, min(n, 2048), replace=False))
    ii = torch.as_tensor(idx, device="cuda:0")
    pos, rot = view.get_world_poses()
    vel = view.get_velocities()
    state = [x[ii].cpu().numpy() for x in (pos, rot, vel, view.get_joint_positions(),
                                           view.get_joint_velocities(),
                                           view._physics_view.get_force_sensor_forces())]
    before = {k: getattr(t, k)[ii].cpu().numpy()
              for k in ("reset_buf", "progress_buf", "potentials", "prev_potentials")}
    acts = t.actions[ii].cpu().numpy()
    N.check(N.lib().mi_task_post_step(view.handle, t.actions.data_ptr(), t.obs_buf.data_ptr(),
                                      t.rew_buf.data_ptr(), t.reset_buf.data_ptr(),
                                      t.progress_buf.data_ptr(), t.potentials.data_ptr(),
                                      t.prev_potentials.data_ptr(), view.stream()), "mi_task_post_step")
    torch.cuda.synchronize()
    assert view.post_kernel()[0] == ("k_loco_post_pipe" if n >= 256 * 1024 else "k_loco_post_tiled<32s>")
    lim = t.model.dof_limits()
    from oracle import oracle as oracle_mod
    ref = oracle_mod.loco_post_math(t.task_params(), *state, acts, lim[:, 0], lim[:, 1],
                                    before["reset_buf"], before["progress_buf"],
                                    before["potentials"], before["prev_potentials"])
    obs = t.obs_buf[ii].cpu().numpy()
    np.testing.assert_allclose(obs, ref["obs"], rtol=1e-4, atol=1e-4)
    assert np.array_equal(t.reset_buf[ii].cpu().numpy(), ref["reset"])
    assert np.array_equal(t.progress_buf[ii].cpu().numpy(), ref["progress"])
    np.testing.assert_allclose(t.potentials[ii].cpu().numpy(), ref["pot"], rtol=1e-6, atol=1e-6)
    assert np.array_equal(t.prev_potentials[ii].cpu().numpy(), ref["prev"])
    rew = t.rew_buf[ii].cpu().numpy()
    bad = ~np.isclose(rew, ref["rew"], rtol=1e-4, atol=1e-4)
    near = (np.abs(ref["obs"][:, 10] - 0.93) < 1e-4) | (np.abs(ref["obs"][:, 11] - 0.8) < 1e-4)
    assert not (bad & ~near).any(), np.nonzero(bad & ~near)[0]
    assert (ref["reset"] == 1).any() and (ref["reset"] == 0).any()
    env.close()
