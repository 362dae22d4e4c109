"""BASELINE config 1 on CPU torch (oracle/torch_cartpole.py, the reference's Cartpole task as
torch ops on CPU tensors, timed by bench.py's cpu_baseline as config1_cpu_torch) checked against
the C oracle: Philox reset draws bit-exact, then 300 VecEnvRLGames steps from the oracle's state
each step (re-synced): obs / reward within 1e-5 (torch's vectorised sin / cos vs glibc),
reset / progress masks bit-exact; and free-running episode statistics equal."""
import numpy as np
import torch

from omniisaacgymenvs_amd.robots.articulations import GridCloner
from oracle.oracle import OracleSim, lib as orc_lib, make_buffers
from oracle.torch_cartpole import CpuTorchCartpole, philox_uniform
from tests.helpers import sim_params, task_params_from_cfg

N = 16


def _pair(seed=42):
    tp, m, _ = task_params_from_cfg("Cartpole")
    sp = sim_params(rest_offset=0.001)
    orc = OracleSim(m, sp, N, GridCloner(4.0).get_clone_positions(N), seed=seed)
    orc.configure(tp)
    b = make_buffers(N, 4, 1)
    orc.reset_idx(np.arange(N), b)              # post_reset, as CpuTorchCartpole.__init__
    b["reset"][:] = 1                            # RLTask.cleanup: reset_buf = ones
    t = CpuTorchCartpole(m, sp, tp, N, seed=seed, noise="philox")
    return tp, orc, b, t


def test_philox_uniform_matches_oracle():
    ids = torch.arange(0, 37, dtype=torch.int64) * 1000003 + (1 << 33)
    cnt = torch.arange(37, dtype=torch.int64) % 5
    for slot in range(6):
        got = philox_uniform(0xDEADBEEF12345678, ids, cnt, slot).numpy()
        ref = np.array([orc_lib().orc_uniform(0xDEADBEEF12345678, int(i), int(c), slot, 0)
                        for i, c in zip(ids, cnt)], np.float32)
        assert np.array_equal(got, ref)


def test_cpu_torch_cartpole_matches_oracle_resynced():
    tp, orc, b, t = _pair()
    q, qd = orc.dof_state()
    assert np.array_equal(t.dof_pos.numpy(), q) and np.array_equal(t.dof_vel.numpy(), qd)
    t.reset_buf[:] = 1                           # VecEnvRLGames.reset flags every env
    rng = np.random.default_rng(3)
    resets = 0
    for k in range(300):
        a = rng.uniform(-1.5, 1.5, (N, 1)).astype(np.float32)
        obs, rew, done, _ = t.step(torch.from_numpy(a))
        orc.env_step(a, 2, b)
        np.testing.assert_allclose(obs["obs"].numpy(), b["obs"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(rew.numpy(), b["rew"], rtol=1e-5, atol=1e-5)
        assert np.array_equal(done.numpy(), b["reset"]), k
        assert np.array_equal(t.progress_buf.numpy(), b["progress"]), k
        assert np.array_equal(t.reset_count.numpy().astype(np.uint32), orc.reset_count()), k
        resets += int(done.sum())
        q, qd = orc.dof_state()                  # re-sync (rounding of sin / cos)
        t.dof_pos = torch.from_numpy(q.copy())
        t.dof_vel = torch.from_numpy(qd.copy())
    assert resets > 10
    orc.close()


def test_cpu_torch_cartpole_reference_noise_runs():
    """noise="torch" (the reference's torch.rand draws): the timed baseline's configuration."""
    tp, m, _ = task_params_from_cfg("Cartpole")
    torch.manual_seed(0)
    t = CpuTorchCartpole(m, sim_params(rest_offset=0.001), tp, N, noise="torch")
    for _ in range(600):
        obs, rew, done, _ = t.step(torch.rand((N, 1)) * 2 - 1)
    assert torch.isfinite(obs["obs"]).all() and obs["obs"].abs().max() <= 5.0
    assert t.reset_count.min() >= 2
