"""GPU: observation / action noise DR (randomize.py:212-306) through the C ABI.

- the fused env step with DR on (noise applied inside the one launch) against the CPU oracle
  started from the identical state: obs / reward within the locomotion tolerance, reset masks
  and the per-env DR schedule state bit-exact;
- fused == method-by-method path (mi_dr_apply_actions / mi_dr_apply_observations kernels
  around the task kernels, as VecEnvRLGames.step orders them);
- the standalone apply kernels against the oracle on random buffers and reset masks.
"""
import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd.utils.task_util import make_env
from tests.helpers import oracle_twin, rand_actions, sync_oracle, task_buffers
from tests.test_gpu_parity import check_device_pair

pytestmark = pytest.mark.gpu

TASKS = ["Cartpole", "Ant", "Humanoid"]
DRK = "task.domain_randomization"
DR_OVERRIDES = [
    f"+{DRK}.randomize=True",
    f"{DRK}.randomization_params.observations.on_reset.operation=additive",
    f"{DRK}.randomization_params.observations.on_reset.distribution=gaussian",
    f"{DRK}.randomization_params.observations.on_reset.distribution_parameters=[0.0,0.01]",
    f"{DRK}.randomization_params.observations.on_interval.frequency_interval=2",
    f"{DRK}.randomization_params.observations.on_interval.operation=scaling",
    f"{DRK}.randomization_params.observations.on_interval.distribution=uniform",
    f"{DRK}.randomization_params.observations.on_interval.distribution_parameters=[0.95,1.05]",
    f"{DRK}.randomization_params.actions.on_reset.operation=additive",
    f"{DRK}.randomization_params.actions.on_reset.distribution=uniform",
    f"{DRK}.randomization_params.actions.on_reset.distribution_parameters=[-0.05,0.05]",
    f"{DRK}.randomization_params.actions.on_interval.frequency_interval=1",
    f"{DRK}.randomization_params.actions.on_interval.operation=additive",
    f"{DRK}.randomization_params.actions.on_interval.distribution=gaussian",
    f"{DRK}.randomization_params.actions.on_interval.distribution_parameters=[0.0,0.02]",
]


def _dr_state(env):
    from omniisaacgymenvs_amd import native as N
    view = env.task.get_robot()
    out = np.zeros((view.count, 6), np.uint32)
    N.check(N.lib().mi_get_dr_state(view.handle, out.ctypes.data), "mi_get_dr_state")
    return out


@pytest.mark.parametrize("name", TASKS)
def test_fused_env_step_with_dr_matches_oracle(gpu, name):
    env = make_env(name, num_envs=64, device="cuda:0", seed=9, overrides=DR_OVERRIDES)
    task = env.task
    assert task.randomize_actions and task.randomize_observations and env.fused
    orc = oracle_twin(env, seed=9)
    orc.set_dr(task._dr_randomizer.params())
    n, A = task.num_envs, task.num_actions
    task.reset()                                    # VecEnvRLGames.reset: flag all, zero actions
    for step in range(5):
        b = task_buffers(env)
        acts = torch.zeros((n, A)) if step == 0 else rand_actions(n, A, 40 + step)
        obs_dict, rew, resets, _ = env.step(acts.to("cuda:0"))
        torch.cuda.synchronize()
        orc.env_step(acts.numpy(), task.control_frequency_inv, b)
        tol = 1e-4 if name == "Cartpole" else 2e-3
        # 5 steps without re-sync: per-env tolerance (device and oracle rollouts drift apart)
        check_device_pair(name, obs_dict["obs"].cpu().numpy(), rew.cpu().numpy(), b["obs"], b["rew"],
                          tol, orc.decision_margin())
        assert np.array_equal(resets.cpu().numpy(), b["reset"]), f"step {step}"
        np.testing.assert_array_equal(_dr_state(env), orc.dr_state(), err_msg=f"step {step}")
        if name != "Cartpole":   # task.actions carries the noisy actions
            np.testing.assert_allclose(task.actions.cpu().numpy(), b["actions"], rtol=1e-6, atol=1e-6)
        sync_oracle(env, orc)
    orc.close()
    env.close()


def test_fused_equals_modular_with_dr(gpu):
    for name in TASKS:
        ea = make_env(name, num_envs=96, device="cuda:0", seed=13, overrides=DR_OVERRIDES)
        eb = make_env(name, num_envs=96, device="cuda:0", seed=13, overrides=DR_OVERRIDES)
        eb.use_fused(False)
        assert ea.fused and not eb.fused
        for step in range(5):
            acts = rand_actions(96, ea.num_actions, step).to("cuda:0")
            oa, ra, da, _ = ea.step(acts)
            ob, rb, db, _ = eb.step(acts)
            torch.cuda.synchronize()
            np.testing.assert_allclose(oa["obs"].cpu().numpy(), ob["obs"].cpu().numpy(), rtol=1e-5,
                                       atol=1e-5, err_msg=f"{name} step {step}")
            np.testing.assert_allclose(ra.cpu().numpy(), rb.cpu().numpy(), rtol=1e-5, atol=1e-5)
            assert torch.equal(da, db)
            np.testing.assert_array_equal(_dr_state(ea), _dr_state(eb))
        ea.close()
        eb.close()


def test_apply_kernels_match_oracle(gpu):
    env = make_env("Humanoid", num_envs=128, device="cuda:0", seed=17, overrides=DR_OVERRIDES)
    task = env.task
    orc = oracle_twin(env, seed=17)
    orc.set_dr(task._dr_randomizer.params())
    rnd = task._dr_randomizer
    g = np.random.default_rng(0)
    for step in range(6):
        reset = (g.random(128) < 0.3).astype(np.int64)
        if step == 0:
            reset[:] = 1
        obs = g.normal(size=(128, task.num_observations)).astype(np.float32)
        act = g.uniform(-1, 1, size=(128, task.num_actions)).astype(np.float32)
        rb = torch.from_numpy(reset).to("cuda:0")
        od, ad = torch.from_numpy(obs).to("cuda:0"), torch.from_numpy(act).to("cuda:0")
        rnd.apply_observations_randomization(od, rb)
        rnd.apply_actions_randomization(ad, rb)
        orc.dr_apply_observations(obs, reset)
        orc.dr_apply_actions(act, reset)
        torch.cuda.synchronize()
        np.testing.assert_allclose(od.cpu().numpy(), obs, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(ad.cpu().numpy(), act, rtol=1e-5, atol=1e-6)
        np.testing.assert_array_equal(_dr_state(env), orc.dr_state())
    orc.close()
    env.close()
