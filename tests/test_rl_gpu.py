"""PPO learner on the GPU: the HIP kernels of libmi_rl.so (include/mi_rl.h) against their
numpy / torch fp32 statements, and the learner driving the real hot path (graph-captured
rollout == eager rollout, bit for bit)."""
import math

import numpy as np
import pytest
import torch

from omniisaacgymenvs_amd.rlg import ops
from tests.rl_ref import gae_np, normals_np

pytestmark = pytest.mark.gpu


def test_gae_kernel_matches_numpy(gpu):
    rng = np.random.default_rng(1)
    H, N = 32, 4096
    rew = rng.normal(size=(H, N)).astype(np.float32)
    val = rng.normal(size=(H, N)).astype(np.float32)
    dones = (rng.random((H, N)) < 0.05).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    ld = (rng.random(N) < 0.05).astype(np.float32)
    t = [torch.from_numpy(x).to(gpu) for x in (rew, val, dones, lv, ld)]
    adv, ret = ops.gae(*t, 0.99, 0.95)
    torch.cuda.synchronize()
    a_np, r_np = gae_np(rew, val, dones, lv, ld, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), a_np, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.cpu().numpy(), r_np, rtol=1e-5, atol=1e-5)
    a_t, r_t = ops.gae_torch(*t, 0.99, 0.95)
    torch.testing.assert_close(adv, a_t, rtol=1e-5, atol=1e-5)


def test_sample_kernel_matches_philox_box_muller(gpu):
    R, A = 64, 21
    g = torch.Generator().manual_seed(3)
    mu = (torch.rand((R, A), generator=g) * 2 - 1).to(gpu)
    ls = (torch.rand((A,), generator=g) - 0.5).to(gpu)
    seed, counter = 0x1234_5678_9ABC_DEF0, 7
    base = torch.tensor([5], dtype=torch.int64, device=gpu)
    act, nlp = ops.sample_gauss(mu, ls, seed, base, counter - 5)
    torch.cuda.synchronize()
    z = normals_np(seed, counter, R, A)
    ref = mu.cpu().numpy() + np.exp(ls.cpu().numpy())[None, :] * z
    np.testing.assert_allclose(act.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    sig = torch.exp(ls).expand_as(mu)
    nlp_ref = ops.neglogp_torch(act, mu, sig, ls.expand_as(mu))
    torch.testing.assert_close(nlp, nlp_ref, rtol=1e-5, atol=1e-4)
    # per-row log-std (logstd_stride = A) draws the same normals
    act2, _ = ops.sample_gauss(mu, ls.expand_as(mu).contiguous(), seed, None, counter)
    torch.testing.assert_close(act2, act, rtol=0, atol=0)


def test_sample_kernel_moments(gpu):
    R, A = 8192, 21
    mu = torch.zeros((R, A), device=gpu)
    ls = torch.zeros((A,), device=gpu)
    a, _ = ops.sample_gauss(mu, ls, 99, None, 0)
    a2, _ = ops.sample_gauss(mu, ls, 99, None, 1)
    assert abs(a.mean().item()) < 0.01 and abs(a.std().item() - 1.0) < 0.01
    assert abs((a ** 4).mean().item() - 3.0) < 0.1                   # Gaussian kurtosis
    assert abs(torch.corrcoef(torch.stack([a.flatten(), a2.flatten()]))[0, 1].item()) < 0.01


def _agent(task, n, graph, seed=11):
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env(task, num_envs=n, device="cuda:0", seed=seed,
                   overrides=[f"train.params.config.minibatch_size={n * 4}"])
    name = f"rlgpu_{task}_{int(graph)}"
    register_env(name, lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    params["config"]["graph_rollout"] = graph
    params["config"]["save_frequency"] = 0
    params["config"]["save_best_after"] = 10 ** 9
    params["seed"] = seed
    return env, A2CAgent(RLGPUEnv(name, n), params)


def test_graph_rollout_equals_eager(gpu):
    """Epochs 2+ replay one captured HIP graph of the whole rollout; it must reproduce the
    eager launches exactly (same kernels, same buffers)."""
    n = 1024
    env_g, ag_g = _agent("Ant", n, True)
    env_e, ag_e = _agent("Ant", n, False)
    ag_g.graph_update = ag_e.graph_update = False     # isolate the rollout graph
    ag_g.env_reset(); ag_e.env_reset()
    for _ in range(4):
        sg = ag_g.train_epoch()
        se = ag_e.train_epoch()
    assert ag_g.graph is not None and ag_e.graph is None
    for k in ("a_loss", "c_loss", "kl", "mean_rewards"):
        assert sg[k] == se[k], (k, sg[k], se[k])
    for (k, a), b in zip(ag_g.model.state_dict().items(), ag_e.model.state_dict().values()):
        assert torch.equal(a, b), k
    assert torch.equal(ag_g.buf["obses"], ag_e.buf["obses"])
    env_g.close(); env_e.close()


def test_graph_update_matches_eager(gpu):
    """Epochs 2+ replay captured HIP graphs of each minibatch update (loss, backward,
    GradScaler + fused Adam, device-side adaptive LR). One graphed epoch from the same state as
    the eager sync-free update must give the same losses, LR and parameters (to GEMM rounding:
    the BLAS may pick other kernels under stream capture)."""
    n = 1024
    env_g, ag_g = _agent("Ant", n, True)
    env_e, ag_e = _agent("Ant", n, True)
    ag_e.graph_update = False
    ag_g.env_reset(); ag_e.env_reset()
    for _ in range(2):                       # epoch 1 eager in both, epoch 2 graphed in ag_g
        sg = ag_g.train_epoch()
        se = ag_e.train_epoch()
    assert len(ag_g.upd_graphs) > 0 and len(ag_e.upd_graphs) == 0
    for k in ("a_loss", "c_loss", "kl", "entropy"):
        assert math.isclose(sg[k], se[k], rel_tol=1e-3, abs_tol=1e-6), (k, sg[k], se[k])
    assert sg["lr"] == se["lr"]
    for (k, a), b in zip(ag_g.model.state_dict().items(), ag_e.model.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=k)
    for pa, pb in zip(ag_g.model.parameters(), ag_e.model.parameters()):
        sa, sb = ag_g.optimizer.state[pa], ag_e.optimizer.state[pb]
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-3, atol=1e-7)
        assert torch.equal(sa["step"], sb["step"])
    env_g.close(); env_e.close()


@pytest.mark.parametrize("mixed", [False, True])
def test_fused_loss_matches_torch_loss(gpu, mixed):
    """mi_rl_ppo_loss (one launch: loss terms, KL, head gradients) against the torch statement
    of rl_games calc_gradients on the same minibatch and weights: losses / KL, the mu / sigma
    write-back and every parameter gradient after autograd through the MLP."""
    env, ag = _agent("Humanoid", 256, False)
    ag.mixed_precision = mixed
    if not mixed:
        ag.scaler = torch.amp.GradScaler("cuda", enabled=False)
    ag.env_reset()
    ag.play_steps()
    ag.model.train()
    ag.model.running_mean_std.eval()     # freeze the obs statistics: both paths see the same
    data = ag.prepare_dataset()
    mb = {k: v[:2048] for k, v in data.items()}
    mb_f = {k: v.clone() for k, v in mb.items()}
    mb_t = {k: v.clone() for k, v in mb.items()}
    mb_f["mu"] += 0.01                   # a non-trivial KL reference
    mb_t["mu"] += 0.01
    ag._optimizer_step = lambda: None    # keep the gradients, skip the update
    a_f, c_f, e_f, kl_f, b_f = (x.item() for x in ag._calc_gradients_fused(mb_f))
    g_f = [p.grad.detach().float().clone() for p in ag.model.parameters()]
    a_t, c_t, e_t, kl_t, cmu, csig, b_t = ag.calc_gradients(mb_t)
    g_t = [p.grad.detach().float().clone() for p in ag.model.parameters()]
    tol = 2e-2 if mixed else 1e-4
    for x, y in ((a_f, a_t.item()), (c_f, c_t.item()), (e_f, e_t.item()), (kl_f, kl_t.item()), (b_f, b_t.item())):
        assert math.isclose(x, y, rel_tol=tol, abs_tol=1e-6), (x, y)
    # mixed: the fused trunk (mi_rl_mlp_train_fwd) and the per-layer autocast path sum in a
    # different order, so mu agrees to a few f16 ulps of the head's magnitude, not to 1e-5
    mu_atol = 4.0 * 2.0 ** -10 * cmu.abs().max().item() if mixed else 1e-5
    torch.testing.assert_close(mb_f["mu"], cmu, rtol=tol, atol=mu_atol)
    torch.testing.assert_close(mb_f["sigma"], csig, rtol=1e-6, atol=1e-7)
    for (name, _), gf, gt in zip(ag.model.named_parameters(), g_f, g_t):
        # the fused path sums weight / bias gradients in fp32 (models._LinearSplitKShadow); the
        # fp16 statement's scaled sum can overflow (value.bias: -1.15e5 > 65504 -> -inf, which
        # GradScaler would answer by skipping the step): there the fused one must be finite
        fin = torch.isfinite(gt)
        assert bool(torch.isfinite(gf).all()), name
        if fin.any():
            torch.testing.assert_close(gf[fin], gt[fin], rtol=tol,
                                       atol=tol * gt[fin].abs().max().item() + 1e-8, msg=name)
        if mixed and not fin.all():
            assert bool((torch.sign(gf[~fin]) == torch.sign(gt[~fin])).all()), name
    env.close()


def test_train_checkpoint_resume_play(gpu, tmp_path, monkeypatch):
    """scripts/rlgames_train end to end (rlgames_train.py:67-84 flow): train a few epochs with
    best-checkpoint saving, resume training from the checkpoint (optimizer state with the device
    LR, fresh graphs), then play it (test=True)."""
    import os

    from omniisaacgymenvs_amd.scripts.rlgames_train import main

    monkeypatch.chdir(tmp_path)
    base = ["task=Cartpole", "num_envs=512", "train.params.config.minibatch_size=2048",
            "train.params.config.save_best_after=1"]
    assert main(base + ["train.params.config.max_epochs=4"]) == 0
    ck = os.path.join("runs", "Cartpole", "nn", "Cartpole.pth")
    assert os.path.exists(ck)
    sd = torch.load(ck, map_location="cuda:0", weights_only=True)
    assert sd["epoch"] >= 1 and "optimizer" in sd and "scaler" in sd
    assert main(base + ["train.params.config.max_epochs=6", f"checkpoint={ck}"]) == 0
    assert main(["task=Cartpole", "num_envs=64", "test=True", f"checkpoint={ck}"]) == 0


def test_ppo_learns_cartpole(gpu):
    env, ag = _agent("Cartpole", 4096, True, seed=5)
    ag.env_reset()
    first = None
    for ep in range(25):
        st = ag.train_epoch()
        assert math.isfinite(st["a_loss"]) and math.isfinite(st["c_loss"])
        if ep == 1:
            first = st["mean_rewards"]
    assert ag.graph is not None
    assert st["mean_rewards"] > first + 20.0, (first, st["mean_rewards"])
    env.close()


def test_ppo_learns_ant_on_reference_schedule(gpu):
    """AntPPO.yaml as shipped (4096 envs, horizon 16, minibatch 32768, 4 mini-epochs, adaptive
    LR) through the learner and the fused Ant step: after 100 epochs the mean episode reward
    must be >= 1000 and >= 20x the first finished episodes'. Under PGS the first episodes read
    8.1 and epoch 101 2199 (profiles/r04/train_curve_ant.jsonl); under TGS (the default since
    round 5) 48.7-50.6 and 1870-2059 (two runs); the bound leaves room for GEMM / box drift."""
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env("Ant", device="cuda:0", seed=42)
    register_env("rlgpu_ant_learn", lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    params["config"]["save_frequency"] = 0
    params["config"]["save_best_after"] = 10 ** 9
    ag = A2CAgent(RLGPUEnv("rlgpu_ant_learn", env.num_envs), params, run_dir="/tmp/ant_learn")
    assert ag.num_actors == 4096 and ag.minibatch_size == 32768 and ag.horizon == 16
    ag.env_reset()
    first = None
    for ep in range(100):
        st = ag.train_epoch()
        assert math.isfinite(st["a_loss"]) and math.isfinite(st["c_loss"])
        if first is None and st["games"] > 0:
            first = st["mean_rewards"]
    assert ag.graph is not None and ag.upd_graphs
    assert st["mean_rewards"] >= 1000.0 and st["mean_rewards"] > 20.0 * max(first, 1.0), (first, st["mean_rewards"])
    env.close()


def test_ppo_learns_humanoid_on_reference_schedule(gpu):
    """HumanoidPPO.yaml as shipped (cfg/train/HumanoidPPO.yaml:59 max_epochs; 4096 envs, horizon
    32, minibatch 32768, 5 mini-epochs, adaptive LR, fp16 update) through the learner — fused
    rollout policy included — and the fused Humanoid step: after 150 epochs the mean episode
    reward must be >= 600 and >= 8x the first finished episodes' (~55-62). The committed curve
    (profiles/r04/train_curve_humanoid.jsonl, same seed) reads 62 at epoch 1, 401 at epoch 100,
    818 at 125 and 2097 at 150; the bound leaves room for ~25 epochs of GEMM / box drift."""
    from omniisaacgymenvs_amd.rlg.a2c_continuous import A2CAgent
    from omniisaacgymenvs_amd.utils.rlgames.rlgames_utils import RLGPUEnv, register_env
    from omniisaacgymenvs_amd.utils.task_util import make_env

    env = make_env("Humanoid", device="cuda:0", seed=42)
    register_env("rlgpu_humanoid_learn", lambda **kw: env)
    params = env.task_cfg["train"]["params"]
    params["config"]["save_frequency"] = 0
    params["config"]["save_best_after"] = 10 ** 9
    ag = A2CAgent(RLGPUEnv("rlgpu_humanoid_learn", env.num_envs), params, run_dir="/tmp/humanoid_learn")
    assert ag.num_actors == 4096 and ag.minibatch_size == 32768 and ag.horizon == 32
    assert ag.fused_policy is not None and ag.recorder is not None
    ag.env_reset()
    first = None
    for ep in range(150):
        st = ag.train_epoch()
        assert math.isfinite(st["a_loss"]) and math.isfinite(st["c_loss"])
        if first is None and st["games"] > 0:
            first = st["mean_rewards"]
    assert ag.graph is not None and ag.upd_graphs
    print(f"humanoid: first {first:.1f}, epoch 150 {st['mean_rewards']:.1f}")
    assert st["mean_rewards"] >= 600.0 and st["mean_rewards"] > 8.0 * max(first, 1.0), (first, st["mean_rewards"])
    env.close()
