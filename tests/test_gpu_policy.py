"""The fused rollout policy (mi_rl_policy_step, rlg/ops.py FusedPolicy) against the torch fp32
statement of the same network (rlg/models.py ModelA2CContinuousLogStd in eval mode: rl_games'
get_action_values during play_steps; cfg/train/*PPO.yaml network blocks).

Tolerance: mu and values within 1e-5 relative (|err| <= 1e-5 * max(1, |ref|)): the f32 MFMA
forms exact f32 products with f32 accumulation, so the kernel differs from torch's fp32 GEMMs
only in summation order. Actions / neglogp: bit-identical to mi_rl_sample_gauss applied to the
kernel's own mu (same Philox draws, same arithmetic)."""
import pytest
import torch

from omniisaacgymenvs_amd.rlg import ops
from omniisaacgymenvs_amd.rlg.models import ModelA2CContinuousLogStd

pytestmark = pytest.mark.gpu

NETS = {"Humanoid": (87, 21, [400, 200, 100]), "Ant": (60, 8, [256, 128, 64]), "Cartpole": (4, 1, [32, 32])}


def _model(O, A, units, seed, norm=True):
    torch.manual_seed(seed)
    cfg = {"mlp": {"units": units, "activation": "elu"},
           "space": {"continuous": {"fixed_sigma": True, "sigma_init": {"val": 0.0}}}}
    m = ModelA2CContinuousLogStd(O, A, cfg, norm, norm).cuda()
    with torch.no_grad():                          # non-trivial biases, sigma and statistics
        for p in m.a2c_network.parameters():
            p.add_(0.05 * torch.randn_like(p))
        if norm:
            rms = m.running_mean_std
            rms.running_mean.copy_(torch.randn(O, dtype=torch.float64, device="cuda") * 0.5)
            rms.running_var.copy_(torch.rand(O, dtype=torch.float64, device="cuda") * 3 + 0.05)
            m.value_mean_std.running_mean.fill_(1.7)
            m.value_mean_std.running_var.fill_(4.2)
    m.eval()
    return m


def _ref(m, obs):
    with torch.no_grad():
        mu, logstd, v = m.policy(obs)
        return mu, logstd, m.unnorm_value(v).squeeze(-1)


def _close(got, ref, what):
    err = (got - ref).abs()
    bound = 1e-5 * ref.abs().clamp(min=1.0)
    assert bool((err <= bound).all()), f"{what}: max err {err.max().item():.3e} (worst ratio {(err / bound).max().item():.2f})"


@pytest.mark.parametrize("task", list(NETS))
@pytest.mark.parametrize("rows", [4096, 4113, 7])
def test_fused_policy_matches_torch_fp32(gpu, task, rows):
    O, A, units = NETS[task]
    m = _model(O, A, units, seed=rows)
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((rows, O), device="cuda") * 2.0
    obs[:, :3] *= 20.0                               # past the +-5 normalisation clamp
    cnt = torch.tensor([11], dtype=torch.int64, device="cuda")
    out = {k: torch.full((rows, w), float("nan"), device="cuda") for k, w in
           (("obs", O), ("act", A), ("nlp", 1), ("val", 1), ("mu", A), ("sg", A))}
    fp.step(obs, seed=1234, counter_base=cnt, counter_offset=3, obs_out=out["obs"], actions=out["act"],
            neglogp=out["nlp"], values=out["val"], mu=out["mu"], sigma=out["sg"])
    torch.cuda.synchronize()
    mu, logstd, val = _ref(m, obs)
    assert torch.equal(out["obs"], obs)
    _close(out["mu"], mu, "mu")
    _close(out["val"].squeeze(-1), val, "value")
    assert torch.equal(out["sg"], torch.exp(logstd))
    act, nlp = ops.sample_gauss(out["mu"], m.a2c_network.sigma.detach(), 1234, cnt, 3)
    assert torch.equal(out["act"], act) and torch.equal(out["nlp"].squeeze(-1), nlp)


def test_fused_policy_without_normalisation_and_partial_outputs(gpu):
    O, A, units = NETS["Humanoid"]
    m = _model(O, A, units, seed=5, norm=False)
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((512, O), device="cuda")
    val = torch.empty((512,), device="cuda")
    fp.step(obs, values=val)                          # value only (the rollout's bootstrap)
    torch.cuda.synchronize()
    _, _, ref = _ref(m, obs)
    _close(val, ref, "value")


def test_fused_policy_tracks_weight_updates_after_repack(gpu):
    O, A, units = NETS["Ant"]
    m = _model(O, A, units, seed=9)
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((256, O), device="cuda")
    mu0 = torch.empty((256, A), device="cuda")
    fp.step(obs, mu=mu0)
    with torch.no_grad():
        m.a2c_network.mu.weight.mul_(-1.5)           # an optimizer step, in place
    fp.pack()
    mu1 = torch.empty((256, A), device="cuda")
    fp.step(obs, mu=mu1)
    torch.cuda.synchronize()
    mu_ref, _, _ = _ref(m, obs)
    _close(mu1, mu_ref, "mu after repack")
    assert not torch.allclose(mu0, mu1)


def test_fused_policy_replays_in_a_graph(gpu):
    """Pack + step captured once; replays see new weights, new obs and advance the noise."""
    O, A, units = NETS["Humanoid"]
    m = _model(O, A, units, seed=2)
    fp = ops.FusedPolicy(m)
    obs = torch.randn((1024, O), device="cuda")
    cnt = torch.zeros((1,), dtype=torch.int64, device="cuda")
    act = torch.empty((1024, A), device="cuda")
    mu = torch.empty((1024, A), device="cuda")
    fp.pack()
    fp.step(obs, seed=7, counter_base=cnt, actions=act, mu=mu)     # warm up outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fp.pack()
        fp.step(obs, seed=7, counter_base=cnt, actions=act, mu=mu)
    firsts = []
    for k in range(3):
        obs.copy_(torch.randn_like(obs))
        with torch.no_grad():
            m.a2c_network.value.bias.add_(0.1)
        g.replay()
        torch.cuda.synchronize()
        mu_ref, _, _ = _ref(m, obs)
        _close(mu, mu_ref, f"replay {k}")
        firsts.append((act - mu).clone())
        cnt.add_(1)
    assert not torch.equal(firsts[0], firsts[1])     # fresh noise per counter


def test_fused_policy_speed(gpu):
    """Informational: one Humanoid rollout policy step (4096 rows) vs the torch statement."""
    O, A, units = NETS["Humanoid"]
    m = _model(O, A, units, seed=1)
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((4096, O), device="cuda")
    cnt = torch.zeros((1,), dtype=torch.int64, device="cuda")
    bufs = [torch.empty((4096, w), device="cuda") for w in (O, A, 1, 1, A, A)]

    def fused():
        fp.step(obs, 3, cnt, 0, *bufs)

    def torch_path():
        with torch.no_grad():
            mu, logstd, v = m.policy(obs)
            ops.sample_gauss(mu, m.a2c_network.sigma.detach(), 3, cnt, 0)
            m.unnorm_value(v)
            torch.exp(logstd)

    res = {}
    for name, fn in (("fused", fused), ("torch", torch_path)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()                   # 8 steps per graph: device time, no host
        with torch.cuda.graph(g):
            for _ in range(8):
                fn()
        g.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / 80 * 1000.0
    print(f"policy step 4096 rows (graph replay): fused {res['fused']:.1f} us, torch {res['torch']:.1f} us")
    assert res["fused"] < res["torch"]


def test_fused_env_actions_equal_preprocess_actions(gpu):
    """env_actions = rl_games preprocess_actions(actions) (clamp +-1, rescale), bit for bit."""
    O, A, units = NETS["Ant"]
    m = _model(O, A, units, seed=4)
    with torch.no_grad():
        m.a2c_network.sigma.fill_(0.7)               # wide noise: many actions past +-1
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((999, O), device="cuda")
    lo = torch.linspace(-2.0, -0.5, A, device="cuda")
    hi = torch.linspace(0.25, 3.0, A, device="cuda")
    act = torch.empty((999, A), device="cuda")
    env_act = torch.empty((999, A), device="cuda")
    fp.step(obs, seed=5, actions=act, env_actions=env_act, action_low=lo, action_high=hi)
    torch.cuda.synchronize()
    a = torch.clamp(act, -1.0, 1.0)
    assert bool((act.abs() > 1.0).any())
    assert torch.equal(env_act, lo + (a + 1.0) * 0.5 * (hi - lo))


def test_record_step_matches_torch_statements(gpu):
    """mi_rl_record_step against the rollout's torch statements (a2c_continuous._rollout_body),
    replayed twice so the ticket reset is exercised; episode sums to f64 rounding."""
    N, O = 4113, 87
    g = torch.Generator(device="cuda").manual_seed(0)
    rec = ops.RolloutRecorder(N, "cuda")
    cur_r = torch.randn((N,), device="cuda", generator=g)
    cur_l = torch.randint(0, 900, (N,), device="cuda", generator=g).float()
    ref_r, ref_l = cur_r.clone(), cur_l.clone()
    for k in range(3):
        obs_in = torch.randn((N, O), device="cuda", generator=g)
        rew = torch.randn((N,), device="cuda", generator=g)
        done = (torch.rand((N,), device="cuda", generator=g) < 0.1).long()
        obs_state, rew_out, done_state = torch.empty_like(obs_in), torch.empty_like(rew), torch.empty_like(rew)
        sums = torch.full((3,), -1.0, device="cuda", dtype=torch.float64)
        rec.step(obs_in, rew, done, 0.01, obs_state, rew_out, done_state, cur_r, cur_l, sums)
        torch.cuda.synchronize()
        d = done.float()
        ref_r.add_(rew)
        ref_l.add_(1.0)
        want = torch.stack([d.double().sum(), (ref_r.double() * d.double()).sum(),
                            (ref_l.double() * d.double()).sum()])
        ref_r.mul_(1.0 - d)
        ref_l.mul_(1.0 - d)
        assert torch.equal(obs_state, obs_in) and torch.equal(done_state, d)
        assert torch.equal(rew_out, rew * 0.01)
        assert torch.equal(cur_r, ref_r) and torch.equal(cur_l, ref_l)
        assert torch.allclose(sums, want, rtol=1e-12, atol=1e-9), (sums, want)
        assert int(rec.ticket.item()) == 0
