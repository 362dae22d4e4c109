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


def test_fused_policy_lds_limit(gpu):
    """k_policy_step's dynamic LDS grows with the widest padded layer. A layout past
    the 64 KB launch limit ([512, 256, 128]: 70 144 B) is refused at construction (ValueError,
    the agent then keeps the torch policy); the widest layout that fits (464: 64 000 B) runs and
    matches the torch statement."""
    with pytest.raises(ValueError, match="LDS"):
        ops.FusedPolicy(_model(87, 21, [512, 256, 128], seed=1))
    m = _model(87, 21, [464, 256, 128], seed=2)
    fp = ops.FusedPolicy(m)
    fp.pack()
    obs = torch.randn((300, 87), device="cuda")
    mu_o = torch.empty((300, 21), device="cuda")
    val_o = torch.empty((300, 1), device="cuda")
    fp.step(obs, mu=mu_o, values=val_o)
    torch.cuda.synchronize()
    mu, _, val = _ref(m, obs)
    _close(mu_o, mu, "mu (464 wide)")
    _close(val_o.squeeze(-1), val, "value (464 wide)")


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


@pytest.mark.parametrize("clip", [1.0, 0.0])
def test_fused_adam_step_matches_torch(gpu, clip):
    """ops.FusedAdamStep (mi_rl_adam_step) against rl-games' torch sequence on a twin model:
    GradScaler.unscale_, clip_grad_norm_ (when clipping), GradScaler.step(fused capturable
    Adam), GradScaler.update, then the legacy adaptive LR on a KL. Ten steps with random
    scaled gradients, one of them non-finite (skipped step, scale backed off), scale growth
    every 3 clean steps: parameters and moments within 1e-5 relative, step / scale / growth
    tracker / LR exactly."""
    from omniisaacgymenvs_amd.rlg.a2c_continuous import AdaptiveScheduler
    from omniisaacgymenvs_amd.rlg.models import ActorCriticMLP

    torch.manual_seed(3)
    net_f, net_t = ActorCriticMLP(87, 21).cuda(), ActorCriticMLP(87, 21).cuda()
    net_t.load_state_dict(net_f.state_dict())
    flat = ops.flatten_parameters(net_f.parameters())
    sched = AdaptiveScheduler(0.008)
    mk = lambda net, lr: (torch.optim.Adam(net.parameters(), lr=lr, eps=1e-8, fused=True, capturable=True),
                          torch.amp.GradScaler("cuda", init_scale=2.0 ** 10, growth_interval=3))
    lr_f = torch.tensor(3e-4, device="cuda")
    lr_t = torch.tensor(3e-4, device="cuda")
    opt_f, sc_f = mk(net_f, lr_f)
    opt_t, sc_t = mk(net_t, lr_t)
    for sc in (sc_f, sc_t):
        sc.scale(torch.zeros((), device="cuda"))
    fo = ops.FusedAdamStep(net_f.parameters(), flat, opt_f, sc_f, lr_f, clip, sched)
    ps_f, ps_t = list(net_f.parameters()), list(net_t.parameters())
    for k in range(10):
        grads = [torch.randn_like(p) * (0.05 if k % 2 else 3.0) * sc_t._scale for p in ps_t]
        if k == 4:
            grads[2].view(-1)[5] = float("inf")
        kl = torch.tensor([0.001, 0.02, 0.008][k % 3], device="cuda")
        for p, g in zip(ps_t, grads):
            p.grad = g.clone()
        sc_t.unscale_(opt_t)
        if clip:
            torch.nn.utils.clip_grad_norm_(net_t.parameters(), clip)
        sc_t.step(opt_t)
        sc_t.update()
        down = torch.clamp(lr_t / 1.5, min=sched.min_lr)
        lr1 = torch.where(kl > 2.0 * sched.kl_threshold, down, lr_t)
        up = torch.clamp(lr1 * 1.5, max=sched.max_lr)
        lr_t.copy_(torch.where(kl < 0.5 * sched.kl_threshold, up, lr1))
        fo.step(torch.cat([g.reshape(-1) for g in grads]), kl=kl)
        torch.cuda.synchronize()
        assert float(sc_f._scale) == float(sc_t._scale), k
        assert int(sc_f._growth_tracker) == int(sc_t._growth_tracker), k
        assert float(lr_f) == float(lr_t), k
        st_t = opt_t.state[ps_t[0]]
        assert float(fo.step_t) == float(st_t["step"]), k
        for pf, pt in zip(ps_f, ps_t):
            torch.testing.assert_close(pf, pt, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(opt_f.state[pf]["exp_avg"], opt_t.state[pt]["exp_avg"], rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(opt_f.state[pf]["exp_avg_sq"], opt_t.state[pt]["exp_avg_sq"], rtol=5e-5, atol=1e-9)
    assert float(fo.step_t) == 9.0                     # the non-finite step was skipped
    t = fo.tickets.tolist()
    assert t[0] == 0 and t[4] == 0 and t[1] == 1 and t[3] == -1   # tickets left 0, one skip
    assert t[2] == sum(p.numel() for p in ps_f[:2]) + 5           # grads[2].view(-1)[5]


def test_fused_adam_step_state_dict_round_trip(gpu):
    """The torch optimizer's state is bound to the flat moments: its state_dict saves them,
    and load_state_dict + bind() restores them into the flat buffers."""
    from omniisaacgymenvs_amd.rlg.models import ActorCriticMLP

    net = ActorCriticMLP(87, 21).cuda()
    flat = ops.flatten_parameters(net.parameters())
    lr = torch.tensor(1e-3, device="cuda")
    opt = torch.optim.Adam(net.parameters(), lr=lr, eps=1e-8, fused=True, capturable=True)
    sc = torch.amp.GradScaler("cuda")
    sc.scale(torch.zeros((), device="cuda"))
    fo = ops.FusedAdamStep(net.parameters(), flat, opt, sc, lr, 1.0, None)
    for _ in range(3):
        fo.step(torch.randn_like(flat) * sc._scale)
    import copy

    sd = copy.deepcopy(opt.state_dict())   # (the live state dict holds views of the flat buffers)
    saved = (fo.exp_avg.clone(), fo.exp_avg_sq.clone(), float(fo.step_t))
    fo.exp_avg.zero_(); fo.exp_avg_sq.zero_(); fo.step_t.zero_()
    opt.load_state_dict(sd)
    fo.bind()
    torch.testing.assert_close(fo.exp_avg, saved[0], rtol=0, atol=0)
    torch.testing.assert_close(fo.exp_avg_sq, saved[1], rtol=0, atol=0)
    assert float(fo.step_t) == saved[2] == 3.0


def test_fused_adam_step_reproduces_f16_gradient_overflow(gpu):
    """Gradients the reference forms in f16 under autocast (the Linear ones, from f16_begin on)
    are f32 sums here; a scaled value at or beyond 65520 (f16 inf) must skip the step and back
    the scale off as GradScaler does for the reference's inf gradient — below f16_begin (the
    log-std, f32 in the reference too) it must not."""
    from omniisaacgymenvs_amd.rlg.models import ActorCriticMLP

    net = ActorCriticMLP(87, 21).cuda()
    flat = ops.flatten_parameters(net.parameters())
    lr = torch.tensor(1e-3, device="cuda")
    opt = torch.optim.Adam(net.parameters(), lr=lr, eps=1e-8, fused=True, capturable=True)
    sc = torch.amp.GradScaler("cuda", init_scale=2.0 ** 16)
    sc.scale(torch.zeros((), device="cuda"))
    fo = ops.FusedAdamStep(net.parameters(), flat, opt, sc, lr, 1.0, None, f16_begin=21)
    g = torch.zeros_like(flat)
    g[5] = 70000.0                     # the log-std's: f32 in the reference too
    before = flat.clone()
    fo.step(g)
    torch.cuda.synchronize()
    assert float(fo.step_t) == 1.0 and float(sc._scale) == 2.0 ** 16 and not torch.equal(flat, before)
    g.zero_()
    g[100] = 65520.0                   # a Linear weight's: inf in f16
    before = flat.clone()
    fo.step(g)
    torch.cuda.synchronize()
    assert float(fo.step_t) == 1.0 and float(sc._scale) == 2.0 ** 15 and torch.equal(flat, before)
    g[100] = 65519.0                   # still finite in f16 (rounds to 65504)
    fo.step(g)
    torch.cuda.synchronize()
    assert float(fo.step_t) == 2.0 and float(sc._scale) == 2.0 ** 15
