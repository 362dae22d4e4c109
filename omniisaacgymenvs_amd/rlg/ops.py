"""Fused per-sample ops of the PPO learner: ctypes binding of libmi_rl.so (include/mi_rl.h)
plus the plain-torch statements of the same ops.

On a GPU device the learner calls the HIP kernels and nothing else: :func:`kernels` raises
when libmi_rl.so is missing (no silent fallback). The torch statements are the fp32
references the GPU numerics tests compare against, and the implementation of BASELINE
config 0 (Cartpole, 16 envs, CPU torch), where no GPU exists.

Semantics follow rl-games 1.5.2 (setup.py:17; not vendored, absent from this image):
``common/a2c_common.py`` ``discount_values`` and ``algos_torch/models.py``
``ModelA2CContinuousLogStd`` (sample + ``neglogp``).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import Optional, Tuple

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MI_RL_LIB", os.path.join(_HERE, "libmi_rl.so"))
_LIB: Optional[C.CDLL] = None
LOG_SQRT_2PI = 0.5 * math.log(2.0 * math.pi)


class RLKernelsUnavailable(RuntimeError):
    pass


MI_RL_MAX_HIDDEN = 4


class MiRlMlp(C.Structure):
    """include/mi_rl.h mi_rl_mlp."""
    _fields_ = [("num_obs", C.c_int32), ("num_actions", C.c_int32), ("num_hidden", C.c_int32),
                ("units", C.c_int32 * MI_RL_MAX_HIDDEN),
                ("w", C.c_void_p * (MI_RL_MAX_HIDDEN + 2)), ("b", C.c_void_p * (MI_RL_MAX_HIDDEN + 2))]


class MiRlAdamCfg(C.Structure):
    """include/mi_rl.h mi_rl_adam_cfg."""
    _fields_ = [("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("weight_decay", C.c_float),
                ("max_grad_norm", C.c_float), ("growth_factor", C.c_float), ("backoff_factor", C.c_float),
                ("growth_interval", C.c_int32), ("adaptive_lr", C.c_int32), ("kl_threshold", C.c_float),
                ("min_lr", C.c_float), ("max_lr", C.c_float), ("f16_overflow", C.c_float),
                ("f16_begin", C.c_int64)]


def load_library() -> C.CDLL:
    """Load libmi_rl.so and declare every prototype of include/mi_rl.h (no GPU needed)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RLKernelsUnavailable(f"{LIB_PATH} not built (python -c 'import __graft_entry__ as g; g.build()')")
        lib = C.CDLL(LIB_PATH)
        vp, f, i32, u64 = C.c_void_p, C.c_float, C.c_int32, C.c_uint64
        lib.mi_rl_abi_version.restype = i32
        lib.mi_rl_abi_version.argtypes = []
        lib.mi_rl_last_error.restype = C.c_char_p
        lib.mi_rl_last_error.argtypes = []
        lib.mi_rl_build_id.restype = C.c_char_p
        lib.mi_rl_build_id.argtypes = []
        lib.mi_rl_gae.restype = i32
        lib.mi_rl_gae.argtypes = [vp, vp, vp, vp, vp, i32, i32, f, f, vp, vp, vp]
        lib.mi_rl_sample_gauss.restype = i32
        lib.mi_rl_sample_gauss.argtypes = [vp, vp, i32, i32, i32, u64, vp, u64, vp, vp, vp]
        lib.mi_rl_ppo_loss.restype = i32
        lib.mi_rl_ppo_loss.argtypes = [vp, i32, vp, vp, i32] + [vp] * 7 + [i32, i32, f, i32, f, f, f] + [vp] * 8
        lib.mi_rl_mlp_packed_size.restype = C.c_int64
        lib.mi_rl_mlp_packed_size.argtypes = [C.POINTER(MiRlMlp)]
        lib.mi_rl_mlp_pack.restype = i32
        lib.mi_rl_mlp_pack.argtypes = [C.POINTER(MiRlMlp), vp, vp]
        lib.mi_rl_policy_step.restype = i32
        lib.mi_rl_policy_step.argtypes = ([C.POINTER(MiRlMlp), vp, vp, i32, vp, vp, vp, vp, f, vp, u64, vp, u64]
                                          + [vp] * 10)
        lib.mi_rl_record_step.restype = i32
        lib.mi_rl_record_step.argtypes = [vp, i32, vp, vp, i32, f] + [vp] * 9
        lib.mi_rl_adam_step.restype = i32
        lib.mi_rl_mlp_train_packed_size.restype = C.c_int64
        lib.mi_rl_mlp_train_packed_size.argtypes = [C.POINTER(MiRlMlp)]
        lib.mi_rl_mlp_train_pack.restype = i32
        lib.mi_rl_mlp_train_pack.argtypes = [C.POINTER(MiRlMlp), vp, vp]
        lib.mi_rl_mlp_train_fwd.restype = i32
        lib.mi_rl_mlp_train_fwd.argtypes = [C.POINTER(MiRlMlp), vp, vp, i32, C.POINTER(vp), vp, vp, vp]
        lib.mi_rl_mlp_train_bwd.restype = i32
        lib.mi_rl_mlp_train_bwd.argtypes = [C.POINTER(MiRlMlp), vp, C.POINTER(vp), vp, vp, i32, C.POINTER(vp), vp]
        lib.mi_rl_adam_step.argtypes = [C.POINTER(MiRlAdamCfg), vp, vp, vp, vp, C.c_int64, vp, vp, vp, vp, vp,
                                        vp, C.c_int64, vp, vp]
        _LIB = lib
    return _LIB


def kernels() -> C.CDLL:
    lib = load_library()
    if not torch.cuda.is_available():
        raise RLKernelsUnavailable("libmi_rl.so needs a GPU")
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {load_library().mi_rl_last_error().decode()}")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


# ------------------------------------------------------------------------------ GAE
def gae_torch(rewards, values, dones, last_values, last_dones, gamma: float, tau: float):
    """rl_games discount_values on [H, N] tensors (dones[t] = done flag before step t).
    Returns (advantages, returns)."""
    H = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    lastgaelam = torch.zeros_like(rewards[0])
    for t in reversed(range(H)):
        if t == H - 1:
            nnt = 1.0 - last_dones
            nv = last_values
        else:
            nnt = 1.0 - dones[t + 1]
            nv = values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        lastgaelam = delta + gamma * tau * nnt * lastgaelam
        adv[t] = lastgaelam
    return adv, adv + values


def gae(rewards, values, dones, last_values, last_dones, gamma: float, tau: float,
        advantages: Optional[torch.Tensor] = None, returns: Optional[torch.Tensor] = None
        ) -> Tuple[torch.Tensor, torch.Tensor]:
    """GAE over a time-major [H, N] rollout (f32, contiguous). GPU: mi_rl_gae (one launch);
    CPU: gae_torch."""
    if rewards.device.type != "cuda":
        return gae_torch(rewards, values, dones, last_values, last_dones, gamma, tau)
    H, N = rewards.shape
    for name, t in (("rewards", rewards), ("values", values), ("dones", dones)):
        if t.shape != (H, N) or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"gae: {name} must be contiguous f32 [{H}, {N}], got {tuple(t.shape)} {t.dtype}")
    for name, t in (("last_values", last_values), ("last_dones", last_dones)):
        if t.numel() != N or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"gae: {name} must be contiguous f32 [{N}]")
    adv = torch.empty_like(rewards) if advantages is None else advantages
    ret = torch.empty_like(rewards) if returns is None else returns
    _check(kernels().mi_rl_gae(rewards.data_ptr(), values.data_ptr(), dones.data_ptr(),
                               last_values.data_ptr(), last_dones.data_ptr(), H, N, float(gamma),
                               float(tau), adv.data_ptr(), ret.data_ptr(), _stream(rewards)),
           "mi_rl_gae")
    return adv, ret


# ------------------------------------------------------------------------------ sampling
def neglogp_torch(x, mean, std, logstd):
    """rl_games ModelA2CContinuousLogStd.neglogp."""
    return (0.5 * (((x - mean) / std) ** 2).sum(dim=-1) + LOG_SQRT_2PI * x.size()[-1]
            + logstd.sum(dim=-1))


def sample_gauss(mu: torch.Tensor, logstd: torch.Tensor, seed: int,
                 counter_base: Optional[torch.Tensor] = None, counter_offset: int = 0,
                 generator: Optional[torch.Generator] = None):
    """action ~ Normal(mu, exp(logstd)) and its neg-log-prob. GPU: mi_rl_sample_gauss (Philox
    keyed on (seed, counter, row, j); counter = counter_base[0] + counter_offset); CPU:
    torch.normal with ``generator``. logstd is [A] (fixed sigma) or [R, A]."""
    R, A = mu.shape
    if mu.device.type != "cuda":
        sigma = torch.exp(logstd)
        a = torch.normal(mu, sigma.expand_as(mu), generator=generator)
        return a, neglogp_torch(a, mu, sigma.expand_as(mu), logstd.expand_as(mu))
    if mu.dtype != torch.float32 or logstd.dtype != torch.float32:
        raise ValueError("sample_gauss: f32 mu / logstd expected")
    mu = mu.contiguous()
    ls = logstd.contiguous()
    stride = 0 if ls.dim() == 1 else A
    if ls.numel() != (A if stride == 0 else R * A):
        raise ValueError(f"sample_gauss: logstd shape {tuple(ls.shape)} vs mu {tuple(mu.shape)}")
    if counter_base is not None and (counter_base.dtype != torch.int64 or counter_base.device != mu.device):
        raise ValueError("sample_gauss: counter_base must be an int64 tensor on the mu device")
    act = torch.empty_like(mu)
    nlp = torch.empty((R,), device=mu.device, dtype=torch.float32)
    _check(kernels().mi_rl_sample_gauss(mu.data_ptr(), ls.data_ptr(), stride, R, A,
                                        int(seed) & ((1 << 64) - 1), _ptr(counter_base),
                                        int(counter_offset), act.data_ptr(), nlp.data_ptr(),
                                        _stream(mu)), "mi_rl_sample_gauss")
    return act, nlp


# ------------------------------------------------------------------------------ PPO loss
def ppo_loss(mu: torch.Tensor, logstd: torch.Tensor, value: torch.Tensor, mb: dict,
             e_clip: float, clip_value: bool, critic_coef: float, entropy_coef: float,
             bounds_coef: float, grad_scale: Optional[torch.Tensor]):
    """rl_games calc_gradients' loss, fused (mi_rl_ppo_loss): returns (grad_mu, grad_value,
    grad_logstd [A], sums [5] = mean a_loss, c_loss, entropy, b_loss, kl) and writes mu /
    exp(logstd) into mb["mu"] / mb["sigma"] (the next mini-epoch's KL reference). The gradients
    are those of grad_scale x loss w.r.t. the heads; mu / value may be f16 (autocast)."""
    B, A = mu.shape
    for t, dt in ((mu, None), (value, None)):
        if t.dtype not in (torch.float16, torch.float32) or not t.is_contiguous():
            raise ValueError("ppo_loss: mu / value must be contiguous f16 or f32")
    if value.numel() != B or logstd.numel() != A or logstd.dtype != torch.float32:
        raise ValueError(f"ppo_loss: value {tuple(value.shape)} / logstd {tuple(logstd.shape)} vs mu {tuple(mu.shape)}")
    keys = ("actions", "old_logp_actions", "advantages", "old_values", "returns", "mu", "sigma")
    for k in keys:
        t = mb[k]
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() not in (B, B * A):
            raise ValueError(f"ppo_loss: mb[{k!r}] must be contiguous f32 with B or B*A elements")
    if grad_scale is not None and (grad_scale.dtype != torch.float32 or grad_scale.numel() != 1):
        raise ValueError("ppo_loss: grad_scale must be a 1-element f32 tensor")
    nblk = (B + 255) // 256
    g_mu = torch.empty_like(mu)
    g_val = torch.empty_like(value)
    part_ls = torch.empty((nblk, A), device=mu.device, dtype=torch.float32)
    part_sums = torch.empty((nblk, 5), device=mu.device, dtype=torch.float32)
    ls = logstd.contiguous()
    _check(kernels().mi_rl_ppo_loss(
        mu.data_ptr(), int(mu.dtype == torch.float16), ls.data_ptr(), value.data_ptr(),
        int(value.dtype == torch.float16), mb["actions"].data_ptr(), mb["old_logp_actions"].data_ptr(),
        mb["advantages"].data_ptr(), mb["old_values"].data_ptr(), mb["returns"].data_ptr(),
        mb["mu"].data_ptr(), mb["sigma"].data_ptr(), B, A, float(e_clip), int(bool(clip_value)),
        float(critic_coef), float(entropy_coef), float(bounds_coef), _ptr(grad_scale),
        g_mu.data_ptr(), g_val.data_ptr(), part_ls.data_ptr(), part_sums.data_ptr(),
        mb["mu"].data_ptr(), mb["sigma"].data_ptr(), _stream(mu)), "mi_rl_ppo_loss")
    return g_mu, g_val, part_ls.sum(0), part_sums.sum(0) * (1.0 / B)


# ------------------------------------------------------------------------------ rollout policy
class FusedPolicy:
    """The rollout's policy evaluation as ONE launch (mi_rl_policy_step): running-mean-std obs
    normalisation, the ELU MLP trunk, mu / value heads on the f32 MFMA, value un-normalisation
    and the Gaussian sample (mi_rl_sample_gauss's draws). ``model`` is a
    ModelA2CContinuousLogStd with fixed sigma and ELU; its weights are repacked into a padded
    copy by :meth:`pack` (call after every weight update; capturable)."""

    def __init__(self, model):
        net = model.a2c_network
        lin = [m for m in net.actor_mlp if isinstance(m, torch.nn.Linear)]
        acts = [m for m in net.actor_mlp if not isinstance(m, torch.nn.Linear)]
        if not net.fixed_sigma or not all(isinstance(a, torch.nn.ELU) for a in acts):
            raise ValueError("FusedPolicy: fixed-sigma ELU networks only")
        if not 1 <= len(lin) <= MI_RL_MAX_HIDDEN:
            raise ValueError(f"FusedPolicy: {len(lin)} hidden layers (1..{MI_RL_MAX_HIDDEN})")
        self.model = model
        d = MiRlMlp()
        d.num_obs, d.num_actions, d.num_hidden = lin[0].in_features, net.mu.out_features, len(lin)
        layers = lin + [net.mu, net.value]
        for i, m in enumerate(lin):
            d.units[i] = m.out_features
        for i, m in enumerate(layers):
            if m.weight.dtype != torch.float32 or not m.weight.is_contiguous() or not m.bias.is_contiguous():
                raise ValueError("FusedPolicy: contiguous f32 weights expected")
            d.w[i], d.b[i] = m.weight.data_ptr(), m.bias.data_ptr()
        self.desc = d
        self._params = layers                  # keep the weights the descriptor points at alive
        n = kernels().mi_rl_mlp_packed_size(C.byref(d))
        if n < 0:
            raise ValueError(f"FusedPolicy: {load_library().mi_rl_last_error().decode()}")
        dev = lin[0].weight.device
        self.packed = torch.zeros((int(n),), device=dev, dtype=torch.float32)

    def pack(self) -> None:
        _check(kernels().mi_rl_mlp_pack(C.byref(self.desc), self.packed.data_ptr(), _stream(self.packed)),
               "mi_rl_mlp_pack")

    def step(self, obs: torch.Tensor, seed: int = 0, counter_base: Optional[torch.Tensor] = None,
             counter_offset: int = 0, obs_out=None, actions=None, neglogp=None, values=None,
             mu=None, sigma=None, env_actions=None, action_low=None, action_high=None) -> None:
        """Writes the given outputs ([R, O] / [R, A] / [R] f32, contiguous). env_actions: the
        actions clamped to +-1 and rescaled to [action_low, action_high] (rl_games
        preprocess_actions)."""
        m = self.model
        R = obs.shape[0]
        if obs.dtype != torch.float32 or not obs.is_contiguous() or obs.shape[1] != self.desc.num_obs:
            raise ValueError(f"FusedPolicy.step: obs {tuple(obs.shape)} {obs.dtype}")
        A = self.desc.num_actions
        if env_actions is not None:
            for t in (action_low, action_high):
                if t is None or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != A:
                    raise ValueError("FusedPolicy.step: env_actions need [A] f32 action bounds")
        for t, w in ((obs_out, self.desc.num_obs), (actions, A), (neglogp, 1), (values, 1), (mu, A),
                     (sigma, A), (env_actions, A)):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != R * w
                                  or t.device != obs.device):
                raise ValueError("FusedPolicy.step: outputs must be contiguous f32 of the obs rows")
        om = ov = vm = vv = None
        if m.normalize_input:
            om, ov = m.running_mean_std.running_mean, m.running_mean_std.running_var
        if m.normalize_value:
            vm, vv = m.value_mean_std.running_mean, m.value_mean_std.running_var
        eps = m.running_mean_std.epsilon if m.normalize_input else 1e-5
        if counter_base is not None and (counter_base.dtype != torch.int64 or counter_base.device != obs.device):
            raise ValueError("FusedPolicy.step: counter_base must be an int64 tensor on the obs device")
        ls = m.a2c_network.sigma
        _check(kernels().mi_rl_policy_step(
            C.byref(self.desc), self.packed.data_ptr(), obs.data_ptr(), R, _ptr(om), _ptr(ov), _ptr(vm),
            _ptr(vv), float(eps), ls.data_ptr(), int(seed) & ((1 << 64) - 1), _ptr(counter_base),
            int(counter_offset), _ptr(obs_out), _ptr(actions), _ptr(neglogp), _ptr(values), _ptr(mu),
            _ptr(sigma), _ptr(action_low), _ptr(action_high), _ptr(env_actions), _stream(obs)),
            "mi_rl_policy_step")


class RolloutRecorder:
    """The rollout's bookkeeping after env.step in one launch (mi_rl_record_step): shaped rewards
    into the experience buffer, next obs / dones, episode meters, the step's finished-episode
    sums. Owns the reduction scratch and the ticket counter."""

    def __init__(self, num_envs: int, device):
        self.n = int(num_envs)
        self.scratch = torch.zeros(((self.n + 255) // 256, 3), device=device, dtype=torch.float64)
        self.ticket = torch.zeros((1,), device=device, dtype=torch.int32)

    def step(self, obs_in, rewards, dones, reward_scale: float, obs_state, rewards_out, dones_state,
             cur_rewards, cur_lengths, episode_sums) -> None:
        N, O = obs_in.shape
        if N != self.n or obs_state.shape != obs_in.shape:
            raise ValueError("RolloutRecorder.step: obs shape")
        for t, dt, k in ((obs_in, torch.float32, N * O), (rewards, torch.float32, N), (dones, torch.int64, N),
                         (obs_state, torch.float32, N * O), (rewards_out, torch.float32, N),
                         (dones_state, torch.float32, N), (cur_rewards, torch.float32, N),
                         (cur_lengths, torch.float32, N), (episode_sums, torch.float64, 3)):
            if t.dtype != dt or not t.is_contiguous() or t.numel() != k or t.device != obs_in.device:
                raise ValueError(f"RolloutRecorder.step: {tuple(t.shape)} {t.dtype}, want {k} x {dt}")
        _check(kernels().mi_rl_record_step(
            obs_in.data_ptr(), O, rewards.data_ptr(), dones.data_ptr(), N, float(reward_scale),
            obs_state.data_ptr(), rewards_out.data_ptr(), dones_state.data_ptr(), cur_rewards.data_ptr(),
            cur_lengths.data_ptr(), episode_sums.data_ptr(), self.scratch.data_ptr(), self.ticket.data_ptr(),
            _stream(obs_in)), "mi_rl_record_step")


# ------------------------------------------------------------------------------ optimizer step
def flatten_parameters(params) -> torch.Tensor:
    """Re-home the given parameters into ONE flat f32 buffer in the given order (each becomes a
    view of it) and return the buffer; call before an optimizer or a FusedPolicy takes their
    storage."""
    ps = list(params)
    if not ps or any(p.dtype != torch.float32 for p in ps):
        raise ValueError("flatten_parameters: f32 parameters expected")
    flat = torch.empty((sum(p.numel() for p in ps),), device=ps[0].device, dtype=torch.float32)
    o = 0
    for p in ps:
        k = p.numel()
        flat[o:o + k].copy_(p.data.reshape(-1))
        p.data = flat[o:o + k].view_as(p)
        o += k
    return flat


class FusedAdamStep:
    """rl-games' trancate_gradients_and_step (GradScaler.unscale_, clip_grad_norm_, Adam,
    GradScaler.update) plus the legacy adaptive LR, over a flat f32 parameter buffer, as two
    launches (mi_rl_adam_step). Adam's moments live in flat buffers too; the torch optimizer's
    per-parameter state is bound to views of them (and a shared device step), so its
    state_dict saves and restores them (call :meth:`bind` again after load_state_dict)."""

    def __init__(self, params, flat: torch.Tensor, optimizer: torch.optim.Adam, scaler, lr_t: torch.Tensor,
                 max_grad_norm: float = 0.0, scheduler=None, f16_begin: Optional[int] = None) -> None:
        """f16_begin: the flat index from which the gradients are the f32 sums that the reference
        forms in f16 under autocast (models._LinearSplitKShadow): a scaled one beyond f16 range
        counts as an overflow (GradScaler skips the step), as the reference's f16 gradient would
        be inf. None: no such gradients."""
        self.params = list(params)
        n = sum(p.numel() for p in self.params)
        if flat.numel() != n or flat.dtype != torch.float32 or not flat.is_contiguous():
            raise ValueError("FusedAdamStep: flat buffer does not hold the parameters")
        if self.params[0].data_ptr() != flat.data_ptr():
            raise ValueError("FusedAdamStep: parameters are not views of the flat buffer (flatten_parameters)")
        g = optimizer.param_groups[0]
        if len(optimizer.param_groups) != 1 or g.get("amsgrad") or g.get("maximize"):
            raise ValueError("FusedAdamStep: one plain Adam param group expected")
        b1, b2 = g["betas"]
        self.cfg = MiRlAdamCfg(beta1=b1, beta2=b2, eps=g["eps"], weight_decay=g["weight_decay"],
                               max_grad_norm=float(max_grad_norm) if max_grad_norm else 0.0,
                               growth_factor=scaler.get_growth_factor() if scaler.is_enabled() else 2.0,
                               backoff_factor=scaler.get_backoff_factor() if scaler.is_enabled() else 0.5,
                               growth_interval=scaler.get_growth_interval() if scaler.is_enabled() else 2000,
                               adaptive_lr=int(scheduler is not None),
                               kl_threshold=float(getattr(scheduler, "kl_threshold", 0.0)),
                               min_lr=float(getattr(scheduler, "min_lr", 0.0)),
                               max_lr=float(getattr(scheduler, "max_lr", 0.0)),
                               f16_overflow=65520.0 if f16_begin is not None else 0.0,
                               f16_begin=int(f16_begin or 0))
        dev = flat.device
        self.flat, self.n, self.optimizer, self.scaler, self.lr_t = flat, n, optimizer, scaler, lr_t
        self.grads = torch.zeros((n,), device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros((n,), device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros((n,), device=dev, dtype=torch.float32)
        self.step_t = torch.zeros((), device=dev, dtype=torch.float32)
        self.scratch = torch.zeros((1028,), device=dev, dtype=torch.float64)
        # [0] / [4] launch tickets, [1] skipped steps, [2] first offending index of the latest
        self.tickets = torch.tensor([0, 0, -1, -1, 0], device=dev, dtype=torch.int32)
        self.bind()

    def bind(self) -> None:
        """Point the torch optimizer's state at the flat moments (after construction or after
        optimizer.load_state_dict, whose restored values are copied in first)."""
        st = self.optimizer.state
        o = 0
        for p in self.params:
            k = p.numel()
            s = st.get(p, {})
            m, v = self.exp_avg[o:o + k].view_as(p), self.exp_avg_sq[o:o + k].view_as(p)
            if "exp_avg" in s and s["exp_avg"].data_ptr() != m.data_ptr():
                m.copy_(s["exp_avg"])
                v.copy_(s["exp_avg_sq"])
                self.step_t.copy_(torch.as_tensor(s["step"], dtype=torch.float32).reshape(()))
            st[p] = {"step": self.step_t, "exp_avg": m, "exp_avg_sq": v}
            o += k

    def step(self, grads: Optional[torch.Tensor] = None, kl: Optional[torch.Tensor] = None) -> None:
        """One optimizer step. grads: a flat f32 gradient buffer in parameter order (at least n
        entries; default: the parameters' .grad gathered into self.grads); kl: device f32 scalar
        for the adaptive LR (None: LR unchanged)."""
        if grads is None:
            torch.cat([p.grad.reshape(-1) for p in self.params], out=self.grads)
            grads = self.grads
        if grads.dtype != torch.float32 or not grads.is_contiguous() or grads.numel() < self.n:
            raise ValueError("FusedAdamStep.step: flat f32 gradients expected")
        sc = self.scaler
        scale = tracker = None
        if sc.is_enabled():
            if sc._scale is None:
                sc._lazy_init_scale_growth_tracker(self.flat.device)
            scale, tracker = sc._scale, sc._growth_tracker
        if kl is not None and (kl.dtype != torch.float32 or kl.numel() != 1):
            raise ValueError("FusedAdamStep.step: kl must be a device f32 scalar")
        _check(kernels().mi_rl_adam_step(
            C.byref(self.cfg), self.flat.data_ptr(), grads.data_ptr(), self.exp_avg.data_ptr(),
            self.exp_avg_sq.data_ptr(), self.n, self.step_t.data_ptr(), self.lr_t.data_ptr(), _ptr(scale),
            _ptr(tracker), _ptr(kl) if self.cfg.adaptive_lr else None, self.scratch.data_ptr(),
            self.scratch.numel(), self.tickets.data_ptr(), _stream(self.flat)), "mi_rl_adam_step")


class FusedTrainMLP:
    """The PPO update's minibatch network on fp16 MFMA (mi_rl_mlp_train_*): the forward (3 ELU
    layers + the mu / value heads) and the dgrad chain are one launch each; the weight and bias
    gradients stay split-K batched GEMMs over the layer inputs the forward stores with a ones
    column (models._LinearSplitKShadow's scheme). ``net`` is an ActorCriticMLP whose Linear
    parameters are views of one flat f32 buffer; :meth:`pack` refreshes the f16 operand images
    from those masters (one launch per minibatch: it replaces the shadow-copy cast)."""

    def __init__(self, net):
        lin = [m for m in net.actor_mlp if isinstance(m, torch.nn.Linear)]
        acts = [m for m in net.actor_mlp if not isinstance(m, torch.nn.Linear)]
        if not net.fixed_sigma or not all(isinstance(a, torch.nn.ELU) for a in acts) or len(lin) != 3:
            raise ValueError("FusedTrainMLP: fixed-sigma networks of 3 ELU layers only")
        d = MiRlMlp()
        d.num_obs, d.num_actions, d.num_hidden = lin[0].in_features, net.mu.out_features, 3
        self.layers = lin + [net.mu, net.value]
        for i, m in enumerate(lin):
            d.units[i] = m.out_features
        for i, m in enumerate(self.layers):
            if m.weight.dtype != torch.float32 or not m.weight.is_cuda:
                raise ValueError("FusedTrainMLP: f32 CUDA weights expected")
            d.w[i], d.b[i] = m.weight.data_ptr(), m.bias.data_ptr()
        n = kernels().mi_rl_mlp_train_packed_size(C.byref(d))
        if n < 0:
            raise ValueError(f"FusedTrainMLP: layout {d.num_obs}-{list(d.units)[:3]}-{d.num_actions} not compiled")
        self.desc = d
        self.dims = (d.num_obs, lin[0].out_features, lin[1].out_features, lin[2].out_features, d.num_actions)
        self.packed = torch.zeros((int(n),), device=lin[0].weight.device, dtype=torch.float16)
        self._ptrs = tuple(p.data_ptr() for m in self.layers for p in (m.weight, m.bias))

    def check_views(self) -> None:
        """The descriptor points at the parameters' storage: fail loudly if it moved."""
        if tuple(p.data_ptr() for m in self.layers for p in (m.weight, m.bias)) != self._ptrs:
            raise RuntimeError("FusedTrainMLP: parameter storage moved since construction")

    def pack(self) -> None:
        _check(kernels().mi_rl_mlp_train_pack(C.byref(self.desc), self.packed.data_ptr(), _stream(self.packed)),
               "mi_rl_mlp_train_pack")

    def forward(self, x: torch.Tensor):
        """x [K, O] f32 contiguous -> (mu f16 [K, A], value f16 [K, 1], the 4 layer inputs f16
        [K, width + 1] with a ones column: views of row-padded buffers)."""
        O, H1, H2, H3, A = self.dims
        K = x.shape[0]
        if x.dtype != torch.float32 or not x.is_contiguous() or x.shape[1] != O:
            raise ValueError(f"FusedTrainMLP.forward: x {tuple(x.shape)} {x.dtype}")
        f16 = torch.float16
        # row stride padded to 8 halfs (mi_rl.h): the kernel's 8-byte accesses stay aligned; the
        # [K, width + 1] views are what the split-K weight gradients read
        acts = [torch.empty((K, (w + 1 + 7) & ~7), device=x.device, dtype=f16)[:, :w + 1] for w in (O, H1, H2, H3)]
        mu = torch.empty((K, A), device=x.device, dtype=f16)
        val = torch.empty((K, 1), device=x.device, dtype=f16)
        ptrs = (C.c_void_p * 4)(*[a.data_ptr() for a in acts])
        _check(kernels().mi_rl_mlp_train_fwd(C.byref(self.desc), self.packed.data_ptr(), x.data_ptr(), K, ptrs,
                                             mu.data_ptr(), val.data_ptr(), _stream(x)), "mi_rl_mlp_train_fwd")
        return mu, val, acts

    def backward(self, acts, gmu: torch.Tensor, gval: torch.Tensor):
        """(gradients w.r.t. the 3 hidden pre-activations, f16 [K, width])."""
        O, H1, H2, H3, A = self.dims
        K = gmu.shape[0]
        gmu = gmu.to(torch.float16).contiguous()
        gval = gval.to(torch.float16).contiguous()
        gs = [torch.empty((K, w), device=gmu.device, dtype=torch.float16) for w in (H1, H2, H3)]
        aptr = (C.c_void_p * 4)(*[a.data_ptr() for a in acts])
        gptr = (C.c_void_p * 3)(*[g.data_ptr() for g in gs])
        _check(kernels().mi_rl_mlp_train_bwd(C.byref(self.desc), self.packed.data_ptr(), aptr, gmu.data_ptr(),
                                             gval.data_ptr(), K, gptr, _stream(gmu)), "mi_rl_mlp_train_bwd")
        return gs, gmu, gval
