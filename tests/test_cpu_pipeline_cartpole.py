"""BASELINE config 1 — Cartpole, 16 envs, the reference's CPU pipeline (pipeline=cpu /
sim_device=cpu, cfg/config.yaml:20-23) — served by the PRODUCT: make_env(..., device="cpu")
builds CartpoleTask over robots/cpu_cartpole.py and VecEnvRLGames steps it method by method
(vec_env_rlgames.py:56-78, cartpole.py:80-162). Checked against the C oracle (checker only):
Philox reset draws and initial state bit-exact, 300 steps re-synced (obs / reward within 1e-5:
torch's vectorised sin / cos vs glibc; reset / progress masks and reset counters bit-exact),
SURVEY §8c KATs 6-8 through the product env, and the product/GPU boundary rules."""
import math

import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd import native as N
from omniisaacgymenvs_amd.robots.cpu_cartpole import CpuCartpoleView
from omniisaacgymenvs_amd.utils import philox
from omniisaacgymenvs_amd.utils.task_util import make_env
from oracle.oracle import OracleSim, lib as orc_lib, make_buffers

N_ENVS = 16


@pytest.fixture(autouse=True, params=[pytest.param("cpu-suite", id="cpu"),
                                      pytest.param("gpu-record", id="gpu-record", marks=pytest.mark.gpu)])
def _suite(request):
    """Every test here needs no GPU, but runs twice: once in the CPU suite and once under the
    `gpu` mark, so the round-end `pytest -m gpu` on the MI355X box records config 1's parity
    too."""
    return request.param


def _env(seed=42, n=N_ENVS, env_id_offset=0, global_num_envs=None):
    return make_env("Cartpole", num_envs=n, device="cpu", seed=seed, env_id_offset=env_id_offset,
                    global_num_envs=global_num_envs)


def _twin(env, seed=42):
    """Oracle with the product env's model, params, origins, seed and current state."""
    t, v = env.task, env.task.get_robot()
    orc = OracleSim(t.model, v.sim_params, t.num_envs, t.env_pos_cpu, seed=seed,
                    env_id_offset=env.env_id_offset)
    orc.configure(t.task_params())
    _resync(env, orc)
    b = make_buffers(t.num_envs, 4, 1)
    b["reset"][:] = t.reset_buf.numpy()
    b["progress"][:] = t.progress_buf.numpy()
    return orc, b


def _resync(env, orc):
    v = env.task.get_robot()
    orc.set_dof_state(v.get_joint_positions().numpy(), v.get_joint_velocities().numpy())
    orc.set_reset_count(v.reset_count.numpy().astype(np.uint32))


def test_product_cpu_pipeline_shape():
    env = _env()
    t = env.task
    assert t.device == "cpu" and t.rl_device == "cpu"
    assert isinstance(t.get_robot(), CpuCartpoleView)
    assert not env.fused                               # method by method, as the reference
    assert t.reset_buf.dtype == torch.int64 and t.progress_buf.dtype == torch.int64
    assert t.obs_buf.shape == (N_ENVS, 4) and t.clip_obs == 5.0 and t.clip_actions == 1.0


def test_philox_matches_oracle_stream():
    ids = torch.arange(0, 37, dtype=torch.int64) * 1000003 + (1 << 33)
    cnt = torch.arange(37, dtype=torch.int64) % 5
    for stream in (0, 3):
        for slot in range(9):
            got = philox.uniform(0xDEADBEEF12345678, ids, cnt, slot, stream).numpy()
            ref = np.array([orc_lib().orc_uniform(0xDEADBEEF12345678, int(i), int(c), slot, stream)
                            for i, c in zip(ids, cnt)], np.float32)
            assert np.array_equal(got, ref), (slot, stream)


def test_initial_reset_matches_oracle():
    """post_reset's reset_idx of every env: the oracle's reset draws, bit for bit."""
    for off in (0, 4096):
        env = _env(seed=11, env_id_offset=off, global_num_envs=off + N_ENVS)
        v = env.task.get_robot()
        orc = OracleSim(env.task.model, v.sim_params, N_ENVS, env.task.env_pos_cpu, seed=11,
                        env_id_offset=off)
        orc.configure(env.task.task_params())
        orc.reset_idx(np.arange(N_ENVS), make_buffers(N_ENVS, 4, 1))
        q, qd = orc.dof_state()
        assert np.array_equal(v.get_joint_positions().numpy(), q)
        assert np.array_equal(v.get_joint_velocities().numpy(), qd)
        assert np.array_equal(v.reset_count.numpy().astype(np.uint32), orc.reset_count())
        orc.close()


def test_product_cpu_pipeline_matches_oracle_resynced():
    env = _env()
    orc, b = _twin(env)
    env.task.reset()                                    # VecEnvRLGames.reset flags every env
    b["reset"][:] = 1
    rng = np.random.default_rng(3)
    resets = 0
    for k in range(300):
        a = rng.uniform(-1.5, 1.5, (N_ENVS, 1)).astype(np.float32)
        obs, rew, done, extras = env.step(torch.from_numpy(a))
        orc.env_step(a, 2, b)
        assert obs["obs"].dtype == torch.float32 and obs["states"].shape == (N_ENVS, 0)
        np.testing.assert_allclose(obs["obs"].numpy(), b["obs"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(rew.numpy(), b["rew"], rtol=1e-5, atol=1e-5)
        assert np.array_equal(done.numpy(), b["reset"]), k
        assert np.array_equal(env.task.progress_buf.numpy(), b["progress"]), k
        assert np.array_equal(env.task.get_robot().reset_count.numpy().astype(np.uint32),
                              orc.reset_count()), k
        assert extras == {}
        resets += int(done.sum())
        q, qd = orc.dof_state()                         # re-sync (rounding of sin / cos)
        v = env.task.get_robot()
        v.set_joint_positions(torch.from_numpy(q.copy()))
        v.set_joint_velocities(torch.from_numpy(qd.copy()))
    assert resets > 10
    orc.close()


def test_product_cpu_pipeline_free_run_masks():
    """60 free-running steps (no re-sync) against the oracle from the same start: the same
    episodes end at the same steps while the trajectories agree to rounding."""
    env = _env(seed=5)
    orc, b = _twin(env, seed=5)
    rng = np.random.default_rng(1)
    agree = 0
    for k in range(60):
        a = rng.uniform(-1, 1, (N_ENVS, 1)).astype(np.float32)
        _, _, done, _ = env.step(torch.from_numpy(a))
        orc.env_step(a, 2, b)
        agree += int(np.array_equal(done.numpy(), b["reset"]))
    assert agree == 60


def test_kat6_cartpole_reward_and_reset_via_product():
    """SURVEY §8c KAT 6 through the product's task methods: (x, xd, th, thd) = (0, 1, 0.1, 2)
    -> 0.97; |x| = 3.01 -> -2 and reset."""
    env = _env()
    t = env.task
    t.obs_buf[:] = torch.tensor([0.0, 1.0, 0.1, 2.0])
    t.obs_buf[1] = torch.tensor([3.01, 0.0, 0.0, 0.0])
    t.progress_buf[:] = 3
    t.calculate_metrics()
    t.is_done()
    assert abs(float(t.rew_buf[0]) - 0.97) < 1e-6
    assert float(t.rew_buf[1]) == -2.0 and int(t.reset_buf[1]) == 1 and int(t.reset_buf[0]) == 0
    t.obs_buf[2] = torch.tensor([0.0, 0.0, math.pi / 2 + 1e-3, 0.0])
    t.calculate_metrics()
    t.is_done()
    assert float(t.rew_buf[2]) == -2.0 and int(t.reset_buf[2]) == 1


def test_kat4_kat7_kat8_timeout_clamps_and_reset_timing():
    env = _env()
    t, v = env.task, env.task.get_robot()
    env.reset()
    assert int(t.progress_buf.max()) == 1 and int(t.reset_buf.sum()) == 0
    # KAT 7: actions clamped to +-1 (efforts = 400 * 1), obs clamped to +-5
    env.step(torch.full((N_ENVS, 1), 7.0))
    assert torch.all(v.get_joint_efforts()[:, 0] == 400.0)
    v.set_joint_velocities(torch.tensor([[9.0, 0.0]] * N_ENVS))
    obs, _, _, _ = env.step(torch.zeros((N_ENVS, 1)))
    assert torch.all(obs["obs"][:, 1] == 5.0) and torch.all(t.obs_buf[:, 1] > 5.0)
    # KAT 4 (Cartpole): progress 499 -> no timeout, 500 -> timeout; KAT 8: terminal obs returned,
    # state re-initialised at the next step's pre_physics_step, progress 1 after that step
    v.set_joint_positions(torch.zeros((N_ENVS, 2)))
    v.set_joint_velocities(torch.zeros((N_ENVS, 2)))
    t.progress_buf[:] = 498
    _, _, done, _ = env.step(torch.zeros((N_ENVS, 1)))
    assert int(done.sum()) == 0 and int(t.progress_buf[0]) == 499
    obs_t, _, done, _ = env.step(torch.zeros((N_ENVS, 1)))
    assert int(done.sum()) == N_ENVS and int(t.progress_buf[0]) == 500
    q_terminal = v.get_joint_positions()
    assert torch.equal(obs_t["obs"][:, 0], q_terminal[:, 0])
    cnt = v.reset_count.clone()
    env.step(torch.zeros((N_ENVS, 1)))
    assert torch.all(v.reset_count == cnt + 1) and torch.all(t.progress_buf == 1)


def test_cpu_pipeline_serves_cartpole_only_and_gpu_stays_native():
    """The CPU pipeline is the reference's pipeline=cpu for Cartpole, not a fallback: the
    articulated tasks refuse it, and a cuda device without a GPU / libmi_sim.so still fails."""
    with pytest.raises(N.NativeUnavailable):
        make_env("Humanoid", num_envs=8, device="cpu")
    with pytest.raises(N.NativeUnavailable):
        make_env("Ant", num_envs=8, device="cpu")
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            make_env("Cartpole", num_envs=8, device="cuda:0")
