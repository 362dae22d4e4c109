"""PPO learner on CPU: the torch statements of its ops against numpy
restatements of rl-games 1.5.2, and BASELINE config 0 — Cartpole, 16 envs, CPU torch, the
learner's full train loop over the IVecEnv contract (env = the product's CPU pipeline,
make_env("Cartpole", device="cpu"), tests/test_cartpole_cpu_rollout.py)."""
import math
import os

import numpy as np
import torch

from omniisaacgymenvs_amd.rlg import ops
from omniisaacgymenvs_amd.rlg.a2c_continuous import (A2CAgent, AdaptiveScheduler, AverageMeter,
                                                      policy_kl, swap_and_flatten01)
from omniisaacgymenvs_amd.rlg.models import ModelA2CContinuousLogStd, RunningMeanStd
from omniisaacgymenvs_amd.utils.hydra_cfg.hydra_utils import compose
from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
from tests.rl_ref import gae_np
from tests.test_cartpole_cpu_rollout import N_ENVS, cartpole_cpu_env


def test_gae_torch_matches_numpy():
    rng = np.random.default_rng(0)
    H, N = 16, 37
    rew = rng.normal(size=(H, N)).astype(np.float32)
    val = rng.normal(size=(H, N)).astype(np.float32)
    dones = (rng.random((H, N)) < 0.1).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    ld = (rng.random(N) < 0.1).astype(np.float32)
    adv, ret = ops.gae(*(torch.from_numpy(x) for x in (rew, val, dones, lv, ld)), 0.99, 0.95)
    a_np, r_np = gae_np(rew, val, dones, lv, ld, 0.99, 0.95)
    np.testing.assert_allclose(adv.numpy(), a_np, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.numpy(), r_np, rtol=1e-5, atol=1e-5)


def test_gae_done_cuts_bootstrap():
    """A done flag before step t+1 stops the value and advantage flowing back into t."""
    H, N = 4, 1
    rew = torch.ones((H, N))
    val = torch.zeros((H, N))
    dones = torch.zeros((H, N))
    dones[2, 0] = 1.0
    adv, _ = ops.gae(rew, val, dones, torch.full((N,), 100.0), torch.zeros(N), 0.5, 1.0)
    assert adv[1, 0].item() == 1.0                       # cut: only its own reward
    assert adv[3, 0].item() == 1.0 + 0.5 * 100.0          # bootstraps from last_values


def test_running_mean_std_matches_batch_moments():
    torch.manual_seed(0)
    rms = RunningMeanStd(3)
    rms.train()
    chunks = [torch.randn(50, 3) * 2 + 1, torch.randn(70, 3) * 0.5 - 2, torch.randn(30, 3)]
    for c in chunks:
        rms(c)
    allx = torch.cat(chunks).double()
    # the merge starts from (mean 0, var 1, count 1): fold that prior sample in
    n = allx.shape[0]
    mean = (allx.sum(0)) / (n + 1)
    np.testing.assert_allclose(rms.running_mean.numpy(), mean.numpy(), rtol=1e-6, atol=1e-6)
    assert float(rms.count) == n + 1
    rms.eval()
    x = torch.randn(4, 3)
    y = rms(x)
    ref = ((x - rms.running_mean.float()) / torch.sqrt(rms.running_var.float() + 1e-5)).clamp(-5, 5)
    assert torch.allclose(y, ref)
    assert float(rms.count) == n + 1                      # eval: no update
    u = rms(y, unnorm=True)
    assert torch.allclose(u, x, atol=1e-5)


def test_policy_kl_zero_and_closed_form():
    mu = torch.randn(8, 3)
    sg = torch.rand(8, 3) + 0.5
    assert abs(policy_kl(mu, sg, mu, sg).item()) < 1e-4
    mu1, sg1 = mu + 0.3, sg * 1.2
    kl = policy_kl(mu, sg, mu1, sg1).item()
    ref = (torch.log(sg1 / sg) + (sg ** 2 + 0.09) / (2 * sg1 ** 2) - 0.5).sum(-1).mean().item()
    assert abs(kl - ref) < 1e-3


def test_meter_and_scheduler():
    m = AverageMeter(100)
    m.update_moments(10, 2.0)
    m.update_moments(30, 4.0)
    assert abs(m.get_mean() - 3.5) < 1e-12 and m.current_size == 40
    m.update_moments(200, 1.0)                           # more than max_size: window resets
    assert m.current_size == 100 and abs(m.get_mean() - 1.0) < 1e-12
    s = AdaptiveScheduler(0.008)
    assert s.update(1e-3, 0.02) == 1e-3 / 1.5
    assert s.update(1e-3, 0.001) == 1e-3 * 1.5
    assert s.update(1e-3, 0.008) == 1e-3
    assert s.update(1e-2, 0.0) == 1e-2 and s.update(1e-6, 1.0) == 1e-6


def test_model_init_and_train_forward():
    net_cfg = compose(["task=Humanoid"])["train"]["params"]["network"]
    m = ModelA2CContinuousLogStd(87, 21, net_cfg, True, True)
    assert [l.out_features for l in m.a2c_network.actor_mlp if isinstance(l, torch.nn.Linear)] == [400, 200, 100]
    for mod in m.modules():
        if isinstance(mod, torch.nn.Linear):
            assert torch.count_nonzero(mod.bias) == 0
    assert torch.count_nonzero(m.a2c_network.sigma) == 0
    obs, act = torch.randn(5, 87), torch.randn(5, 21)
    res = m.forward_train(obs, act)
    mu, logstd = res["mus"], torch.log(res["sigmas"])
    ref = ops.neglogp_torch(act, mu, res["sigmas"], logstd)
    assert torch.allclose(res["prev_neglogp"], ref)
    dist = torch.distributions.Normal(mu, res["sigmas"])
    assert torch.allclose(-dist.log_prob(act).sum(-1), ref, atol=1e-4)
    assert torch.allclose(dist.entropy().sum(-1), res["entropy"], atol=1e-5)


def test_swap_and_flatten01_is_actor_major():
    x = torch.arange(2 * 3).reshape(2, 3)            # [H=2, N=3]
    assert swap_and_flatten01(x).tolist() == [0, 3, 1, 4, 2, 5]


def _cartpole_cpu_params(minibatch=64):
    cfg = compose(["task=Cartpole", "rl_device=cpu", "sim_device=cpu", "pipeline=cpu",
                   f"num_envs={N_ENVS}", f"train.params.config.minibatch_size={minibatch}"])
    params = cfg["train"]["params"]
    assert params["config"]["num_actors"] == N_ENVS and params["config"]["device"] == "cpu"
    return params


def test_config0_ppo_train_loop_cpu(tmp_path):
    """Config 0: the learner's full epoch (rollout, GAE, value/advantage normalisation, PPO
    minibatches with the adaptive LR, meters, checkpoints) on CPU torch over RLGPUEnv."""
    register_env("rlgpu_cfg0", lambda **kw: cartpole_cpu_env())
    env = RLGPUEnv("rlgpu_cfg0", N_ENVS)
    params = _cartpole_cpu_params()
    params["config"]["save_frequency"] = 2
    agent = A2CAgent(env, params, run_dir=str(tmp_path))
    assert agent.batch_size == 16 * N_ENVS and agent.num_minibatches == 4
    lr0 = agent.last_lr
    st = agent.train(max_epochs=4, log=None)
    assert st["epoch"] == 4 and st["frames"] == 4 * agent.batch_size
    for k in ("a_loss", "c_loss", "kl", "entropy"):
        assert math.isfinite(st[k]), k
    assert st["games"] > 0                     # cartpole episodes end under a random policy
    assert agent.last_lr != lr0                # the adaptive schedule moved the LR
    assert float(agent.model.running_mean_std.count) > 1
    assert float(agent.model.value_mean_std.count) > 1
    ck = os.path.join(str(tmp_path), "nn", "last_Cartpole_ep_4.pth")
    assert os.path.exists(ck)
    agent2 = A2CAgent(RLGPUEnv("rlgpu_cfg0", N_ENVS), params, run_dir=str(tmp_path))
    agent2.restore(ck)
    for (k, a), b in zip(agent.model.state_dict().items(), agent2.model.state_dict().values()):
        assert torch.equal(a, b), k
    assert agent2.epoch_num == 4 and agent2.last_lr == agent.last_lr


def test_minibatch_must_divide_batch():
    register_env("rlgpu_cfg0b", lambda **kw: cartpole_cpu_env())
    params = _cartpole_cpu_params(minibatch=8192)        # CartpolePPO default: 256 % 8192 != 0
    try:
        A2CAgent(RLGPUEnv("rlgpu_cfg0b", N_ENVS), params)
    except ValueError as e:
        assert "troubleshoot" in str(e)
    else:
        raise AssertionError("expected ValueError")
