"""Actor-critic network of the reference's PPO configs (cfg/train/*PPO.yaml ``network``:
``actor_critic``, ``separate: False``, ``mlp.units``, ``activation: elu``, ``space.continuous``
with ``fixed_sigma: True``; ``model: continuous_a2c_logstd``), restating rl-games 1.5.2
``algos_torch/network_builder.py`` (A2CBuilder) and ``algos_torch/models.py``
(ModelA2CContinuousLogStd) and ``algos_torch/running_mean_std.py``.

Statistics buffers are updated IN PLACE so a captured HIP graph of the rollout (which reads
them by address) always sees the current values.
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch
import torch.nn as nn

from .ops import neglogp_torch

# 0.5 + 0.5 log(2 pi), evaluated in float32 like rl_games' tensor expression
_HALF_LOG_2PI_E = float((0.5 + 0.5 * torch.log(torch.tensor(2.0 * torch.pi, dtype=torch.float32))).item())

# bias gradients of layers at least this wide as a split-K batched GEMM against ones (MI355X,
# K = 32768 fp16, tools/reduce_bench.py: out 400 14 us vs gy.sum(0) 26 us, out 200 13 vs 16;
# narrower layers lose: out 100 24 vs 13, out 22 12 vs 9)
_BIAS_BMM_MIN_OUT = 200
_ONES = {}


def _ones(S: int, k: int, like: torch.Tensor) -> torch.Tensor:
    key = (S, k, like.dtype, like.device)
    t = _ONES.get(key)
    if t is None:
        t = torch.ones((S, 1, k), dtype=like.dtype, device=like.device)
        # cached only when filled now: under stream capture the fill is a graph node that has
        # not run yet, so that tensor stays private to the graph
        if not (like.is_cuda and torch.cuda.is_current_stream_capturing()):
            _ONES[key] = t
    return t

_ACT = {"elu": nn.ELU, "relu": nn.ReLU, "tanh": nn.Tanh, "selu": nn.SELU, "None": nn.Identity,
        None: nn.Identity}


class _LinearSplitK(torch.autograd.Function):
    """y = x Wᵀ + b whose weight gradient dW = dYᵀ X (a K = minibatch-rows reduction into a
    small [out, in] tile) runs as split-K: a batched GEMM over `splits` row blocks and a sum.
    A single GEMM leaves most of the chip idle on these shapes (MI355X, K = 32768:
    90-140 µs untuned, 48-88 µs tuned per GEMM; split-32: ~27 µs, tools/wgrad_bench.py)."""

    @staticmethod
    def forward(ctx, x, w, b, splits: int):
        ctx.save_for_backward(x, w)
        ctx.splits = splits
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        S = ctx.splits
        gx = gy @ w if ctx.needs_input_grad[0] else None
        K, O = x.shape[0], gy.shape[1]
        split = S > 1 and K % S == 0
        if split:
            gys = gy.reshape(S, K // S, O)
            gw = torch.bmm(gys.transpose(1, 2), x.reshape(S, K // S, -1)).sum(0)
        else:
            gw = gy.t() @ x
        gb = None
        if ctx.needs_input_grad[2]:
            if split and gy.is_cuda and O >= _BIAS_BMM_MIN_OUT:
                gb = torch.bmm(_ones(S, K // S, gy), gys).sum(0).reshape(O)
            else:
                gb = gy.sum(0)
        return gx, gw, gb, None


class _LinearSplitKShadow(torch.autograd.Function):
    """_LinearSplitK on a pre-cast low-precision copy (w16, b16) of the fp32 master weights
    (w, b): the GEMMs run in the copy's dtype, the weight / bias gradients are summed in fp32
    straight into the masters' dtype. Under autocast this replaces a cast launch per weight and
    bias in the forward and another per gradient in the backward (one copy of the whole flat
    weight buffer per minibatch instead: ActorCriticMLP.shadow_weights)."""

    @staticmethod
    def forward(ctx, x, w, b, w16, b16, splits: int):
        K, I = x.shape
        ctx.splits = splits
        ctx.fused = splits > 1 and K % splits == 0 and x.is_cuda
        if ctx.fused:
            # the input with a ones column appended: the backward forms the weight AND the bias
            # gradient in ONE split-K GEMM (tools/reduce_bench.py, profiles/r05: 12-29 us vs
            # 30-41 us for the weight GEMM plus the bias GEMM against ones, per layer)
            xa = torch.empty((K, I + 1), dtype=x.dtype, device=x.device)
            xa[:, :I].copy_(x)
            xa[:, I].fill_(1.0)
            ctx.save_for_backward(xa, w16)
        else:
            ctx.save_for_backward(x, w16)
        return torch.nn.functional.linear(x, w16, b16)

    @staticmethod
    def backward(ctx, gy):
        x, w16 = ctx.saved_tensors
        S = ctx.splits
        gx = gy @ w16 if ctx.needs_input_grad[0] else None
        K, O = x.shape[0], gy.shape[1]
        f32 = torch.float32
        if ctx.fused:
            # [gW | gb] = gy^T [x | 1], split-K in S row blocks (fp16 block partials, as the
            # autocast GEMM's output, summed in f32). Every bias gradient is a GEMM: torch's
            # column reductions over the 32768 rows take multi-block (global staging) paths that,
            # replayed from the update graph, now and then returned overflowing sums for the
            # 100-wide layer (GradScaler skips seen by mi_rl_adam_step's counters)
            I = x.shape[1] - 1
            gys = gy.reshape(S, K // S, O)
            gwb = torch.bmm(gys.transpose(1, 2), x.reshape(S, K // S, I + 1)).sum(0, dtype=f32)
            return gx, gwb[:, :I], gwb[:, I], None, None, None
        split = S > 1 and K % S == 0
        if split:
            gys = gy.reshape(S, K // S, O)
            gw = torch.bmm(gys.transpose(1, 2), x.reshape(S, K // S, -1)).sum(0, dtype=f32)
        else:
            gw = (gy.t() @ x).to(f32)
        gb = gy.sum(0, dtype=f32)
        return gx, gw, gb, None, None, None


def _split_k_wgrad(gy: torch.Tensor, xa: torch.Tensor, S: int) -> torch.Tensor:
    """[gW | gb] = gyᵀ [x | 1] as _LinearSplitKShadow forms it: S row blocks (fp16 partials of
    the batched GEMM), summed in f32."""
    K, O = gy.shape
    if S > 1 and K % S == 0:
        return torch.bmm(gy.reshape(S, K // S, O).transpose(1, 2),
                         xa.reshape(S, K // S, xa.shape[1])).sum(0, dtype=torch.float32)
    return (gy.t() @ xa).to(torch.float32)


class _FusedMLPTrain(torch.autograd.Function):
    """The minibatch trunk + heads of the PPO update on fp16 MFMA (ops.FusedTrainMLP, one launch
    forward, one launch for the dgrad chain), returning (mu, value) in f16 as the autocast Linears
    do; the weight / bias gradients of the f32 masters are the split-K GEMMs of
    _LinearSplitKShadow over the layer inputs the forward stored with a ones column."""

    @staticmethod
    def forward(ctx, x, fused, splits, *params):
        mu, val, acts = fused.forward(x.contiguous())
        ctx.fused, ctx.splits = fused, splits
        ctx.save_for_backward(*acts)
        return mu, val

    @staticmethod
    def backward(ctx, gmu, gval):
        acts = ctx.saved_tensors
        fused, S = ctx.fused, ctx.splits
        if gmu is None:
            gmu = torch.zeros((acts[0].shape[0], fused.dims[4]), device=acts[0].device, dtype=torch.float16)
        if gval is None:
            gval = torch.zeros((acts[0].shape[0], 1), device=acts[0].device, dtype=torch.float16)
        (g1, g2, g3), gmu, gval = fused.backward(acts, gmu, gval)
        out = []
        for gy, xa in ((g1, acts[0]), (g2, acts[1]), (g3, acts[2]), (gmu, acts[3]), (gval, acts[3])):
            gwb = _split_k_wgrad(gy, xa, S)
            I = xa.shape[1] - 1
            out += [gwb[:, :I], gwb[:, I]]
        return (None, None, None, *out)


def linear_train(x: torch.Tensor, layer: nn.Linear, splits: int = 32, shadow=None) -> torch.Tensor:
    """nn.Linear for the learner's minibatch forward (autocast-aware: runs in the autocast dtype
    when autocast is on, as nn.Linear would), with the split-K weight gradient. shadow: the
    layer's (w16, b16) views of ActorCriticMLP's refreshed low-precision weight copy."""
    w, b = layer.weight, layer.bias
    if shadow is not None:
        w16, b16 = shadow
        with torch.autocast(device_type=x.device.type, enabled=False):
            return _LinearSplitKShadow.apply(x.to(w16.dtype), w, b, w16, b16, splits)
    if torch.is_autocast_enabled(x.device.type):
        dt = torch.get_autocast_dtype(x.device.type)
        x, w = x.to(dt), w.to(dt)
        b = b.to(dt) if b is not None else None
        with torch.autocast(device_type=x.device.type, enabled=False):
            return _LinearSplitK.apply(x, w, b, splits)
    return _LinearSplitK.apply(x, w, b, splits)


def _merge_moments(mean: torch.Tensor, var: torch.Tensor, n: float):
    """(mean, unbiased var, count) of the union of every rank's batch of n rows (equal n), from
    each rank's own: two all-reduces (parallel-variance merge)."""
    import torch.distributed as dist

    w = dist.get_world_size()
    if w == 1:
        return mean, var, n
    gmean = mean.clone()
    dist.all_reduce(gmean)
    gmean /= w
    m2 = var * (n - 1.0) + n * (mean - gmean) ** 2
    dist.all_reduce(m2)
    tot = n * w
    return gmean, m2 / (tot - 1.0), tot


class RunningMeanStd(nn.Module):
    """Running mean / variance of a batch stream (parallel-variance merge), f64 buffers;
    forward normalises (clamped to ±5) or un-normalises. Statistics update only in
    training mode."""

    def __init__(self, insize, epsilon: float = 1e-05, norm_only: bool = False) -> None:
        super().__init__()
        self.epsilon = epsilon
        self.norm_only = norm_only
        shape = (insize,) if isinstance(insize, int) else tuple(insize)
        self.register_buffer("running_mean", torch.zeros(shape, dtype=torch.float64))
        self.register_buffer("running_var", torch.ones(shape, dtype=torch.float64))
        self.register_buffer("count", torch.ones((), dtype=torch.float64))
        # data-parallel learner: the batch moments are those of the union of the ranks' batches
        # (equal batch sizes), merged by all-reduce, so every replica keeps the same statistics
        self.all_reduce = False

    @torch.no_grad()
    def _update(self, x: torch.Tensor) -> None:
        # per-feature moments as row reductions of the transposed batch ([C, B]: one contiguous
        # row per feature) instead of strided column reductions over B
        bv, bm = torch.var_mean(x.detach().transpose(0, 1).contiguous(), dim=1)  # unbiased
        batch_mean = bm.double()
        batch_var = bv.double()
        batch_count = float(x.shape[0])
        if self.all_reduce:
            batch_mean, batch_var, batch_count = _merge_moments(batch_mean, batch_var, batch_count)
        delta = batch_mean - self.running_mean
        tot = self.count + batch_count
        new_mean = self.running_mean + delta * batch_count / tot
        m2 = (self.running_var * self.count + batch_var * batch_count
              + delta ** 2 * self.count * batch_count / tot)
        self.running_mean.copy_(new_mean)
        self.running_var.copy_(m2 / tot)
        self.count.copy_(tot)

    def forward(self, x: torch.Tensor, unnorm: bool = False) -> torch.Tensor:
        if self.training and not unnorm:
            self._update(x)
        mean = self.running_mean.float()
        var = self.running_var.float()
        if unnorm:
            y = torch.clamp(x, min=-5.0, max=5.0)
            return torch.sqrt(var + self.epsilon) * y + mean
        if self.norm_only:
            return x / torch.sqrt(var + self.epsilon)
        y = (x - mean) / torch.sqrt(var + self.epsilon)
        return torch.clamp(y, min=-5.0, max=5.0)


class ActorCriticMLP(nn.Module):
    """A2CBuilder.Network with separate=False, continuous space, fixed sigma: a shared MLP
    trunk, linear mu and value heads, sigma a free [A] parameter (log-std). Linear weights keep
    torch's default init, every Linear bias starts at 0, sigma at ``sigma_init`` (the
    builder's initialisation)."""

    def __init__(self, num_obs: int, num_actions: int, units: Sequence[int] = (400, 200, 100),
                 activation: str = "elu", sigma_init: float = 0.0, fixed_sigma: bool = True) -> None:
        super().__init__()
        layers = []
        d = num_obs
        for u in units:
            layers += [nn.Linear(d, u), _ACT[activation]()]
            d = u
        self.actor_mlp = nn.Sequential(*layers)
        self.value = nn.Linear(d, 1)
        self.mu = nn.Linear(d, num_actions)
        self.fixed_sigma = fixed_sigma
        if fixed_sigma:
            self.sigma = nn.Parameter(torch.zeros(num_actions, dtype=torch.float32), requires_grad=True)
        else:
            self.sigma = nn.Linear(d, num_actions)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.zeros_(m.bias)
        with torch.no_grad():
            if fixed_sigma:
                self.sigma.fill_(sigma_init)
            else:
                self.sigma.weight.fill_(sigma_init)

    def _linears(self):
        return [m for m in self.actor_mlp if isinstance(m, nn.Linear)] + [self.mu, self.value]

    def shadow_weights(self, dtype: torch.dtype, flat: torch.Tensor) -> None:
        """Keep a flat low-precision copy of ``flat``, the f32 buffer every Linear weight and
        bias is a view of (rlg.ops.flatten_parameters): heads_train under autocast refreshes the
        copy with one cast launch per minibatch and runs the layers on its views
        (_LinearSplitKShadow)."""
        low = torch.empty_like(flat, dtype=dtype)
        views = {}
        base, n = flat.data_ptr(), flat.numel()
        for m in self._linears():
            for p in (m.weight, m.bias):
                o = (p.data_ptr() - base) // flat.element_size()
                if p.data_ptr() < base or o + p.numel() > n:
                    raise ValueError("shadow_weights: a Linear parameter is not a view of the flat buffer")
                views[id(p)] = low[o:o + p.numel()].view_as(p)
        self._flat32, self._flat_low, self._low_views = flat, low, views
        # the fused fp16-MFMA trunk (mi_rl_mlp_train_*) when the layout is compiled; MI_RL_FUSED_MLP=0
        # or cfg fused_train_mlp: False keeps the per-layer path (A/B)
        self._train_mlp = None
        if dtype == torch.float16 and flat.is_cuda and getattr(self, "fused_train_mlp", True):
            import os

            if os.environ.get("MI_RL_FUSED_MLP", "1") != "0":
                from .ops import FusedTrainMLP
                try:
                    self._train_mlp = FusedTrainMLP(self)
                except ValueError:
                    self._train_mlp = None

    def heads_train(self, obs: torch.Tensor, splits: int = 32):
        """(mu, value) of the minibatch forward through linear_train (split-K weight grads)."""
        low = getattr(self, "_flat_low", None)
        sh = None
        fused = getattr(self, "_train_mlp", None)
        if (fused is not None and low is not None and torch.is_autocast_enabled(obs.device.type)
                and torch.get_autocast_dtype(obs.device.type) == low.dtype and obs.dtype == torch.float32):
            fused.pack()                     # f16 operand images of the current masters: one launch
            params = [p for m in self._linears() for p in (m.weight, m.bias)]
            with torch.autocast(device_type=obs.device.type, enabled=False):
                return _FusedMLPTrain.apply(obs, fused, splits, *params)
        if (low is not None and torch.is_autocast_enabled(obs.device.type)
                and torch.get_autocast_dtype(obs.device.type) == low.dtype):
            low.copy_(self._flat32)          # every layer's low-precision weights: one launch
            v = self._low_views
            sh = {id(m): (v[id(m.weight)], v[id(m.bias)]) for m in self._linears()}
        out = obs
        for m in self.actor_mlp:
            if isinstance(m, nn.Linear):
                out = linear_train(out, m, splits, sh[id(m)] if sh else None)
            else:
                out = m(out)
        return (linear_train(out, self.mu, splits, sh[id(self.mu)] if sh else None),
                linear_train(out, self.value, splits, sh[id(self.value)] if sh else None))

    def forward(self, obs: torch.Tensor):
        out = self.actor_mlp(obs)
        value = self.value(out)
        mu = self.mu(out)
        logstd = mu * 0.0 + self.sigma if self.fixed_sigma else self.sigma(out)
        return mu, logstd, value


class ModelA2CContinuousLogStd(nn.Module):
    """Observation / value normalisation around the network; the train-mode forward returns
    what the PPO loss needs (rl_games ModelA2CContinuousLogStd.Network.forward, is_train)."""

    def __init__(self, num_obs: int, num_actions: int, network_cfg: Dict, normalize_input: bool,
                 normalize_value: bool) -> None:
        super().__init__()
        mlp = network_cfg.get("mlp", {})
        space = network_cfg.get("space", {}).get("continuous", {})
        sigma_init = float(space.get("sigma_init", {}).get("val", 0.0))
        self.a2c_network = ActorCriticMLP(num_obs, num_actions, tuple(mlp.get("units", (400, 200, 100))),
                                          mlp.get("activation", "elu"), sigma_init,
                                          bool(space.get("fixed_sigma", True)))
        self.normalize_input = normalize_input
        self.normalize_value = normalize_value
        if normalize_input:
            self.running_mean_std = RunningMeanStd(num_obs)
        if normalize_value:
            self.value_mean_std = RunningMeanStd(1)

    def norm_obs(self, obs: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            return self.running_mean_std(obs) if self.normalize_input else obs

    def unnorm_value(self, value: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            return self.value_mean_std(value, unnorm=True) if self.normalize_value else value

    def policy(self, obs: torch.Tensor):
        """(mu, logstd, normalised value) of raw observations."""
        return self.a2c_network(self.norm_obs(obs))

    def forward_train(self, obs: torch.Tensor, prev_actions: torch.Tensor):
        mu, logstd, value = self.policy(obs)
        sigma = torch.exp(logstd)
        # host constant, no tensor creation inside the step (graph-capturable)
        entropy = (_HALF_LOG_2PI_E + logstd).sum(dim=-1)
        prev_neglogp = neglogp_torch(prev_actions, mu, sigma, logstd)
        return {"prev_neglogp": prev_neglogp, "values": value, "entropy": entropy, "mus": mu,
                "sigmas": sigma}
