"""The PPO update's minibatch network on fp16 MFMA (mi_rl_mlp_train_*, rlg/ops.py FusedTrainMLP,
rlg/models.py _FusedMLPTrain) against the per-layer path it replaces (_LinearSplitKShadow under
torch autocast fp16: rl_games calc_gradients with mixed_precision, cfg/train/HumanoidPPO.yaml).

Both compute in f16 with f32 accumulation and differ in summation order and in the ELU
derivative's form (exp(z) from the stored pre-activation in torch, h + 1 from the stored
activation here), so they are compared through an fp32 statement of the same network on the
same f16-rounded weights: the fused path's error against it must stay within 1.5x the autocast
path's own error (+ a small floor), for the heads and for every parameter gradient, and the two
paths must agree to fp16 tolerance directly."""
import pytest
import torch

from omniisaacgymenvs_amd.rlg import ops
from omniisaacgymenvs_amd.rlg.models import ModelA2CContinuousLogStd

pytestmark = pytest.mark.gpu

NETS = {"Humanoid": (87, 21, [400, 200, 100]), "Ant": (60, 8, [256, 128, 64])}


def _net(O, A, units, seed):
    torch.manual_seed(seed)
    cfg = {"mlp": {"units": units, "activation": "elu"},
           "space": {"continuous": {"fixed_sigma": True, "sigma_init": {"val": 0.0}}}}
    m = ModelA2CContinuousLogStd(O, A, cfg, True, True).cuda()
    with torch.no_grad():
        for p in m.a2c_network.parameters():
            p.add_(0.05 * torch.randn_like(p))
    net = m.a2c_network
    flat = ops.flatten_parameters(net.parameters())
    net.shadow_weights(torch.float16, flat)
    return net


def _run(net, x, gmu, gv, fused: bool):
    saved = net._train_mlp
    if not fused:
        net._train_mlp = None
    try:
        for p in net.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.float16):
            mu, v = net.heads_train(x, 32)
        torch.autograd.backward((mu, v), (gmu, gv))
        torch.cuda.synchronize()
        grads = [p.grad.detach().clone() for m in net._linears() for p in (m.weight, m.bias)]
        return mu.detach().float(), v.detach().float(), grads
    finally:
        net._train_mlp = saved


def _ref32(net, x, gmu, gv):
    """fp32 statement on the f16-rounded weights and input (what both f16 paths approximate)."""
    lin = net._linears()
    ws = [m.weight.detach().half().float().requires_grad_(True) for m in lin]
    bs = [m.bias.detach().half().float().requires_grad_(True) for m in lin]
    h = x.half().float()
    for i in range(3):
        h = torch.nn.functional.elu(h @ ws[i].t() + bs[i])
    mu = h @ ws[3].t() + bs[3]
    v = h @ ws[4].t() + bs[4]
    torch.autograd.backward((mu, v), (gmu.float(), gv.float()))
    grads = [t.grad for pair in zip(ws, bs) for t in pair]
    return mu.detach(), v.detach(), grads


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-30))


@pytest.mark.parametrize("task", list(NETS))
@pytest.mark.parametrize("rows", [32768, 4100])
def test_fused_train_mlp_matches_autocast_path(gpu, task, rows):
    O, A, units = NETS[task]
    net = _net(O, A, units, seed=rows)
    assert net._train_mlp is not None, "the fused trunk is compiled for this layout"
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn((rows, O), device="cuda", generator=g).clamp(-5, 5)      # normalised obs range
    gmu = (torch.randn((rows, A), device="cuda", generator=g) * 1e-2).half()
    gv = (torch.randn((rows, 1), device="cuda", generator=g) * 1e-2).half()
    mu_f, v_f, g_f = _run(net, x, gmu, gv, fused=True)
    mu_t, v_t, g_t = _run(net, x, gmu, gv, fused=False)
    mu_r, v_r, g_r = _ref32(net, x, gmu, gv)
    names = [f"{n}.{k}" for n in ("l1", "l2", "l3", "mu", "value") for k in ("weight", "bias")]
    # heads
    for what, f, t, r in (("mu", mu_f, mu_t, mu_r), ("value", v_f, v_t, v_r)):
        ef, et = _rel(f, r), _rel(t, r)
        assert ef <= 1.5 * et + 2e-4, f"{task} {what}: fused err {ef:.3e} vs autocast err {et:.3e}"
        assert _rel(f, t) <= 5e-3, f"{task} {what}: fused vs autocast {_rel(f, t):.3e}"
    # every parameter gradient
    for n, f, t, r in zip(names, g_f, g_t, g_r):
        assert f.dtype == torch.float32 and f.shape == t.shape
        ef, et = _rel(f, r), _rel(t, r)
        assert ef <= 1.5 * et + 1e-3, f"{task} {n}: fused err {ef:.3e} vs autocast err {et:.3e}"
        assert _rel(f, t) <= 2e-2, f"{task} {n}: fused vs autocast {_rel(f, t):.3e}"


def test_fused_train_mlp_refuses_other_layouts(gpu):
    net = _net(87, 21, [256, 256, 128], seed=1)       # not compiled: the per-layer path stays
    assert net._train_mlp is None
    with pytest.raises(ValueError, match="not compiled"):
        ops.FusedTrainMLP(net)
