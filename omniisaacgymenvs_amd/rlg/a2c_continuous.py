"""PPO agent with the semantics of rl-games 1.5.2 ``a2c_continuous`` (setup.py:17; the library
is neither vendored nor installable here), driving the hot path through the IVecEnv contract
(``RLGPUEnv``, utils/rlgames/rlgames_utils.py:94-118) the way scripts/rlgames_train.py:67-84
does. Hyper-parameters come from cfg/train/<Task>PPO.yaml ``params.config``.

What is restated from rl-games (per epoch):
  play_steps    horizon_length env steps under the eval-mode policy; the experience buffer
                holds obs, dones-before-step, actions, neglogp, values (un-normalised), mus,
                sigmas and shaped rewards (reward_shaper.scale_value); per-env episode return /
                length meters (games_to_track = 100).
  GAE           discount_values(gamma, tau); returns = advantages + values.
  prepare       swap_and_flatten01 (actor-major batch), value normalisation of values and
                returns (value RunningMeanStd in train mode, values first), advantage
                normalisation over the batch.
  train         mini_epochs x (batch / minibatch_size) contiguous minibatches (no shuffling),
                clipped surrogate + clipped value loss (x 0.5 critic_coef) + bound loss
                (soft bound 1.1) - entropy_coef x entropy; Adam(eps 1e-8), fp16 autocast +
                GradScaler when mixed_precision, grad-norm clip; the mu/sigma of each minibatch
                written back for the next mini-epoch's KL; the legacy adaptive LR schedule
                after every minibatch (KL > 2 thr: lr / 1.5; KL < thr / 2: lr x 1.5; clamped to
                [1e-6, 1e-2]); obs statistics updated during the first mini-epoch only.

MI355X-first execution:
  * GAE and action sampling are single HIP launches (libmi_rl.so, include/mi_rl.h);
  * the whole rollout — horizon x (policy GEMMs, sampling, mi_env_step, buffer writes, meter
    sums) — is captured once into a HIP graph and replayed every epoch, so a rollout costs one
    graph launch instead of ~30 launches per env step; episode meters are accumulated on
    device as per-step (count, sum) pairs and folded into the host meters with one copy per
    epoch (no nonzero() host syncs in the loop);
  * the minibatch update is sync-free — the learning rate is a device tensor the legacy
    adaptive schedule updates in place (no kl.item() per minibatch), fused capturable Adam takes
    it and GradScaler's found_inf / scale on the device, the dataset lives in persistent
    buffers — and is captured once per (obs-statistics mode, minibatch index) into a HIP graph
    replayed from epoch 2 on; the update's only host sync is the per-epoch stats read;
  * on CPU (BASELINE config 0) the same code runs eagerly with the torch statements of
    those ops.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import ops
from .models import ModelA2CContinuousLogStd, RunningMeanStd


def _f(x) -> float:
    return float(x)


_TUNINGS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_mi355x.csv")


def _use_shipped_gemm_tunings() -> bool:
    """Route the learner's GEMMs through TunableOp with the solutions measured on MI355X for
    these shapes (rollout fp32 + update fp16 GEMMs of the 400-200-100 MLP at 4096 / 32768 rows:
    rocBLAS / hipBLASLt solution per shape; tuning itself stays off). The file's validator lines
    pin the torch / HIP / BLAS versions; on a mismatch TunableOp rejects it and the default
    solutions run. Skipped when the user drives TunableOp through its environment variables."""
    if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") is not None or not os.path.exists(_TUNINGS):
        return False
    import shutil
    import tempfile

    from torch.cuda import tunable

    # TunableOp may write its database back to the file it was given: hand it a private copy
    path = os.path.join(tempfile.gettempdir(), f"mi_tunableop_{os.getpid()}.csv")
    shutil.copyfile(_TUNINGS, path)
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.set_filename(path, insert_device_ordinal=False)
    return bool(tunable.read_file(path))


class AverageMeter:
    """rl_games torch_ext.AverageMeter: mean over the last max_size values, updated with
    batches (size, mean)."""

    def __init__(self, max_size: int = 100) -> None:
        self.max_size = max_size
        self.current_size = 0
        self.mean = 0.0

    def update_moments(self, size: int, mean: float) -> None:
        if size <= 0:
            return
        size = int(np.clip(size, 0, self.max_size))
        old_size = min(self.max_size - size, self.current_size)
        size_sum = old_size + size
        self.current_size = size_sum
        self.mean = float((self.mean * old_size + mean * size) / size_sum)

    def clear(self) -> None:
        self.current_size = 0
        self.mean = 0.0

    def get_mean(self) -> float:
        return self.mean


class AdaptiveScheduler:
    def __init__(self, kl_threshold: float = 0.008, min_lr: float = 1e-6, max_lr: float = 1e-2) -> None:
        self.kl_threshold, self.min_lr, self.max_lr = kl_threshold, min_lr, max_lr

    def update(self, lr: float, kl: float) -> float:
        if kl > 2.0 * self.kl_threshold:
            lr = max(lr / 1.5, self.min_lr)
        if kl < 0.5 * self.kl_threshold:
            lr = min(lr * 1.5, self.max_lr)
        return lr


def policy_kl(p0_mu, p0_sigma, p1_mu, p1_sigma):
    """rl_games torch_ext.policy_kl, reduced (mean over rows of the per-row sum)."""
    c1 = torch.log(p1_sigma / p0_sigma + 1e-5)
    c2 = (p0_sigma ** 2 + (p1_mu - p0_mu) ** 2) / (2.0 * (p1_sigma ** 2 + 1e-5))
    return (c1 + c2 - 0.5).sum(dim=-1).mean()


def swap_and_flatten01(x: torch.Tensor) -> torch.Tensor:
    """[H, N, ...] -> [N * H, ...] (actor-major), rl_games a2c_common.swap_and_flatten01."""
    s = x.shape
    return x.transpose(0, 1).reshape(s[0] * s[1], *s[2:])


class A2CAgent:
    """rl_games a2c_continuous.A2CAgent over an IVecEnv."""

    def __init__(self, env, params: Dict, run_dir: Optional[str] = None) -> None:
        cfg = params["config"]
        self.env = env
        self.cfg = cfg
        self.params = params
        self.device = torch.device(cfg.get("device", "cuda:0"))
        info = env.get_env_info()
        self.num_obs = int(np.prod(info["observation_space"].shape))
        self.num_actions = int(np.prod(info["action_space"].shape))
        self.actions_low = torch.as_tensor(np.asarray(info["action_space"].low, np.float32), device=self.device)
        self.actions_high = torch.as_tensor(np.asarray(info["action_space"].high, np.float32), device=self.device)
        self.num_actors = int(cfg["num_actors"])
        self.horizon = int(cfg["horizon_length"])
        # multi-GPU (multi_gpu: True under torch.distributed.run), one process per
        # GPU stepping its env shard; two learner modes (`multi_gpu_mode`):
        #  * "data_parallel" (default; rl_games' multi_gpu): every rank runs GAE and the PPO
        #    epochs on its own shard (num_actors and minibatch_size per rank); per minibatch the
        #    gradients and the policy KL are averaged over the ranks in ONE all-reduce (RCCL)
        #    before the optimizer step, so every replica takes the same step with the same
        #    adaptive LR; the obs / value normalisation statistics merge the ranks' batch moments
        #    (all-reduce), so replicas stay identical; weights broadcast once at start;
        #  * "central": every horizon is gathered to the learner (rank 0) in ONE collective
        #    (utils.distributed.RolloutGather), the learner trains on all ranks' actors (world x
        #    the batch, world x the minibatches) and broadcasts the weights back.
        # `distributed` also holds at world size 1 under an initialised process group (the
        # single-GPU rehearsal of config 5's collectives, tests/test_gpu_nccl.py)
        self.distributed = (bool(cfg.get("multi_gpu", False)) and dist.is_available()
                            and dist.is_initialized())
        self.world = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        mode = str(cfg.get("multi_gpu_mode", "data_parallel"))
        if mode not in ("data_parallel", "central"):
            raise ValueError(f"multi_gpu_mode must be 'data_parallel' or 'central', got {mode!r}")
        self.dp = self.distributed and mode == "data_parallel"
        self.central = self.distributed and mode == "central"
        self.is_learner = self.rank == 0 or not self.central
        self.batch_size = self.horizon * self.num_actors * (self.world if self.central else 1)
        self.minibatch_size = int(cfg["minibatch_size"])
        if self.batch_size % self.minibatch_size != 0:
            raise ValueError(f"minibatch_size {self.minibatch_size} must divide horizon x actors = "
                             f"{self.batch_size} (docs/troubleshoot.md:44)")
        self.num_minibatches = self.batch_size // self.minibatch_size
        # frames one epoch adds over the whole job (rl_games multi_gpu: curr_frames * world):
        # data-parallel ranks each step their own shard; central's batch is already global
        self.frames_per_epoch = self.batch_size * (self.world if self.dp else 1)
        self.mini_epochs = int(cfg["mini_epochs"])
        self.gamma, self.tau = _f(cfg["gamma"]), _f(cfg["tau"])
        self.e_clip = _f(cfg["e_clip"])
        self.clip_value = bool(cfg.get("clip_value", False))
        self.critic_coef = _f(cfg["critic_coef"])
        self.entropy_coef = _f(cfg.get("entropy_coef", 0.0))
        self.bounds_loss_coef = cfg.get("bounds_loss_coef", None)
        self.grad_norm = _f(cfg.get("grad_norm", 1.0))
        self.truncate_grads = bool(cfg.get("truncate_grads", False))
        self.normalize_advantage = bool(cfg.get("normalize_advantage", True))
        self.normalize_value = bool(cfg.get("normalize_value", False))
        self.normalize_input = bool(cfg.get("normalize_input", False))
        self.value_bootstrap = bool(cfg.get("value_bootstrap", False))
        self.reward_scale = _f(cfg.get("reward_shaper", {}).get("scale_value", 1.0))
        self.last_lr = _f(cfg["learning_rate"])
        self.lr_schedule = cfg.get("lr_schedule", None)
        self.scheduler = AdaptiveScheduler(_f(cfg.get("kl_threshold", 0.008))) if self.lr_schedule == "adaptive" else None
        self.max_epochs = int(cfg.get("max_epochs", 1000))
        self.save_best_after = int(cfg.get("save_best_after", 100))
        self.save_frequency = int(cfg.get("save_frequency", 0))
        self.score_to_win = _f(cfg.get("score_to_win", math.inf))
        self.mixed_precision = bool(cfg.get("mixed_precision", False)) and self.device.type == "cuda"
        self.name = cfg.get("name", "run")
        self.run_dir = run_dir or os.path.join("runs", str(self.name))
        self.seed = int(params.get("seed", 42))

        torch.manual_seed(self.seed)
        if self.device.type == "cuda" and bool(cfg.get("tunableop", True)):
            _use_shipped_gemm_tunings()
        self.model = ModelA2CContinuousLogStd(self.num_obs, self.num_actions, params["network"],
                                              self.normalize_input, self.normalize_value).to(self.device)
        if self.dp:   # merged batch moments over the ranks (replicas keep identical statistics)
            for m in self.model.modules():
                if isinstance(m, RunningMeanStd):
                    m.all_reduce = True
        wd = float(cfg.get("weight_decay", 0.0))
        self._flat_params = None
        if self.device.type == "cuda":
            # every parameter in one flat f32 buffer (before the optimizer and the fused policy
            # take their storage): the fused optimizer step runs over it, and under mixed
            # precision its fp16 copy (one cast launch per minibatch) feeds the minibatch GEMMs
            self._flat_params = ops.flatten_parameters(self.model.parameters())
        fused_opt = (self._flat_params is not None
                     and bool(cfg.get("fused_optimizer", os.environ.get("MI_RL_FUSED_OPT", "1") != "0")))
        # the shadow weights' gradients are f32 sums; only the fused optimizer step reproduces
        # the f16 overflow of the reference's autocast gradients (GradScaler's skipped steps)
        self._shadow = (fused_opt and self.mixed_precision
                        and bool(cfg.get("shadow_weights", os.environ.get("MI_RL_SHADOW", "1") != "0")))
        if self._shadow:
            self.model.a2c_network.shadow_weights(torch.float16, self._flat_params)
        if self.device.type == "cuda":
            # LR lives on the device and the legacy adaptive schedule updates it there (no
            # kl.item() per minibatch); fused Adam takes the tensor LR and GradScaler's
            # found_inf / scale without host syncs, so a minibatch update is graph-capturable
            self.lr_t = torch.tensor(self.last_lr, device=self.device, dtype=torch.float32)
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lr_t, eps=1e-08,
                                              weight_decay=wd, fused=True, capturable=True)
        else:
            self.lr_t = None
            self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.last_lr, eps=1e-08,
                                              weight_decay=wd)
        self.scaler = torch.amp.GradScaler("cuda", enabled=self.mixed_precision)
        if self.mixed_precision:     # materialise the device scale now (the fused loss reads it)
            self.scaler.scale(torch.zeros((), device=self.device))
        # GradScaler unscale + grad-norm clip + Adam + scaler update + adaptive LR as two
        # launches over the flat buffer (mi_rl_adam_step) instead of ~20 torch kernels
        self.fused_opt = None
        self._f16_begin = None
        if fused_opt:
            f16_begin = None
            if self._shadow:   # the Linear parameters follow the log-std in parameters() order
                net = self.model.a2c_network
                f16_begin = min((p.data_ptr() - self._flat_params.data_ptr()) // 4
                                for m in net._linears() for p in (m.weight, m.bias))
            self.fused_opt = ops.FusedAdamStep(self.model.parameters(), self._flat_params, self.optimizer,
                                               self.scaler, self.lr_t, self.grad_norm if self.truncate_grads else 0.0,
                                               self.scheduler, f16_begin)
            self._f16_begin = f16_begin
        # loss + head gradients as one HIP launch (mi_rl_ppo_loss); needs the fixed log-std head
        self.fused_loss = (self.device.type == "cuda" and bool(cfg.get("fused_loss", True))
                           and self.model.a2c_network.fixed_sigma)
        # the rollout's policy evaluation (normalisation, MLP, heads, sampling) as ONE launch
        # (mi_rl_policy_step, f32 MFMA) instead of the torch modules + sampling kernel
        self.fused_policy = None
        self._env_act = None
        if self.device.type == "cuda" and bool(cfg.get("fused_policy", True)):
            try:
                self.fused_policy = ops.FusedPolicy(self.model)
            except ValueError as e:        # a network the kernel does not cover: torch modules
                print(f"[rlg] fused rollout policy off ({e})")
        # the rollout's per-step bookkeeping after env.step as one launch (mi_rl_record_step)
        self.recorder = (ops.RolloutRecorder(self.num_actors, self.device)
                         if self.fused_policy is not None else None)
        # split-K weight gradients of the minibatch GEMMs (models.linear_train); 1 = one GEMM
        self.wgrad_splits = int(cfg.get("wgrad_splits", 32))
        # action-noise streams: one per rank (replicas must not share exploration noise)
        self.sample_gen = torch.Generator(device="cpu").manual_seed(self.seed + 7919 * self.rank)
        self.sample_seed = ((self.seed * 0x9E3779B97F4A7C15 + 1) ^ (self.rank * 0xD1B54A32D192ED03)) & ((1 << 64) - 1)

        H, N, O, A = self.horizon, self.num_actors, self.num_obs, self.num_actions
        dev, f32 = self.device, torch.float32
        self.rollout = None
        if self.central:
            # the rollout buffers ARE the gather slab's fields (zero copy; one slab, so the
            # captured rollout graph keeps writing the same addresses)
            from ..utils.distributed import RolloutGather
            self.rollout = RolloutGather(H, N, O, dev, self.world, buffers=1, mode="gather", dst=0,
                                         extra=self._SLAB_EXTRA(A), with_done=False)
            v = self.rollout.slabs[0].views
            self.buf = {"obses": v["obs"], "rewards": v["rew"], "dones": v["dones_f"],
                        "actions": v["actions"].view(H, N, A), "neglogpacs": v["neglogpacs"],
                        "values": v["values"], "mus": v["mus"].view(H, N, A),
                        "sigmas": v["sigmas"].view(H, N, A)}
        else:
            self.buf = {
                "obses": torch.zeros((H, N, O), device=dev, dtype=f32),
                "dones": torch.zeros((H, N), device=dev, dtype=f32),
                "actions": torch.zeros((H, N, A), device=dev, dtype=f32),
                "neglogpacs": torch.zeros((H, N), device=dev, dtype=f32),
                "values": torch.zeros((H, N), device=dev, dtype=f32),
                "mus": torch.zeros((H, N, A), device=dev, dtype=f32),
                "sigmas": torch.zeros((H, N, A), device=dev, dtype=f32),
                "rewards": torch.zeros((H, N), device=dev, dtype=f32),
            }
        self.obs = torch.zeros((N, O), device=dev, dtype=f32)      # static rollout input
        self.dones = torch.zeros((N,), device=dev, dtype=f32)
        self.last_values = torch.zeros((N,), device=dev, dtype=f32)
        self.current_rewards = torch.zeros((N,), device=dev, dtype=f32)
        self.current_lengths = torch.zeros((N,), device=dev, dtype=f32)
        self.episode_sums = torch.zeros((H, 3), device=dev, dtype=torch.float64)  # count, rew, len
        self.rng_counter = torch.zeros((1,), device=dev, dtype=torch.int64)
        self.game_rewards = AverageMeter(int(cfg.get("games_to_track", 100)))
        self.game_lengths = AverageMeter(int(cfg.get("games_to_track", 100)))
        self.use_graph = self.device.type == "cuda" and bool(cfg.get("graph_rollout", True))
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # minibatch updates: one captured graph per (obs-statistics mode, minibatch index)
        self.graph_update = self.device.type == "cuda" and bool(cfg.get("graph_update", True))
        self.upd_graphs: Dict = {}
        # data-parallel: gradients (+ the policy KL) of a minibatch in one flat buffer, averaged
        # over the ranks by one all-reduce between the two captured halves of the update
        self._params = [p for p in self.model.parameters()]
        self._flat = (torch.zeros(sum(p.numel() for p in self._params) + 1, device=dev, dtype=f32)
                      if self.dp else None)
        self._data: Optional[Dict[str, torch.Tensor]] = None
        self._mb_out = torch.zeros((self.num_minibatches, 5), device=dev, dtype=f32)
        self._mb_stats = torch.zeros((self.mini_epochs, self.num_minibatches, 5), device=dev, dtype=f32)
        self.epoch_num = 0
        self.frame = 0
        if self.distributed:
            self._broadcast_weights()   # every replica starts from the learner's initial weights
        self.last_mean_rewards = -100500.0
        self.stats: Dict[str, float] = {}

    @staticmethod
    def _SLAB_EXTRA(A: int):
        f32 = torch.float32
        return [("dones_f", 1, f32), ("actions", A, f32), ("neglogpacs", 1, f32), ("values", 1, f32),
                ("mus", A, f32), ("sigmas", A, f32)]

    # ------------------------------------------------------------------ multi-GPU
    def _gather_horizon(self):
        """The horizon's rollout slab to the learner in one gather, plus the bootstrap values /
        final dones [2, N] per rank; episode statistics summed over ranks. Returns the learner's
        global (buffers, last_values, dones) in global actor order (rank-major), else None."""
        g = self.rollout
        g.gather(async_op=False)
        tail = torch.stack([self.last_values, self.dones])
        lst = [torch.empty_like(tail) for _ in range(self.world)] if self.is_learner else None
        dist.gather(tail, gather_list=lst, dst=0)
        dist.all_reduce(self.episode_sums)
        if not self.is_learner:
            return None
        H, A = self.horizon, self.num_actions
        names = {"obses": "obs", "rewards": "rew", "dones": "dones_f", "actions": "actions",
                 "neglogpacs": "neglogpacs", "values": "values", "mus": "mus", "sigmas": "sigmas"}
        b = {k: g.global_field(f) for k, f in names.items()}
        for k in ("actions", "mus", "sigmas"):
            b[k] = b[k].reshape(H, -1, A)
        tails = torch.stack(lst)                     # [world, 2, N]
        return b, tails[:, 0].reshape(-1), tails[:, 1].reshape(-1)

    def _broadcast_weights(self) -> None:
        """The learner's parameters and statistics buffers to every policy replica, in place (the
        captured rollout graphs read them by address)."""
        for t in self.model.state_dict().values():
            dist.broadcast(t, src=0)

    # ------------------------------------------------------------------ env plumbing
    def _obs_tensor(self, obs) -> torch.Tensor:
        o = obs["obs"] if isinstance(obs, dict) else obs
        return o.to(self.device, dtype=torch.float32)

    def env_reset(self) -> None:
        self.obs.copy_(self._obs_tensor(self.env.reset()))

    def preprocess_actions(self, actions: torch.Tensor) -> torch.Tensor:
        """clip_actions: clamp to [-1, 1] then rescale to the action space."""
        a = torch.clamp(actions, -1.0, 1.0)
        return self.actions_low + (a + 1.0) * 0.5 * (self.actions_high - self.actions_low)

    # ------------------------------------------------------------------ rollout
    def _policy_step(self, obs: torch.Tensor, n: int):
        """Eval-mode policy on raw obs: actions, neglogp, un-normalised values, mu, sigma."""
        mu, logstd, value = self.model.policy(obs)
        mu = mu.float()
        logstd = logstd.float()
        if self.device.type == "cuda":
            act, nlp = ops.sample_gauss(mu, self.model.a2c_network.sigma.detach().float()
                                        if self.model.a2c_network.fixed_sigma else logstd,
                                        self.sample_seed, self.rng_counter, n)
        else:
            act, nlp = ops.sample_gauss(mu, logstd, 0, generator=self.sample_gen)
        values = self.model.unnorm_value(value.float()).squeeze(-1)
        return act, nlp, values, mu, torch.exp(logstd)

    def _record_fused(self, obs, rewards, dones, infos) -> bool:
        """The fused bookkeeping applies when the env hands back device f32 obs / rewards and
        i64 dones and no time-out bootstrap is requested (the reference's tasks set none)."""
        if self.recorder is None:
            return False
        if self.value_bootstrap and isinstance(infos, dict) and "time_outs" in infos:
            return False
        o = obs["obs"] if isinstance(obs, dict) else obs
        return (o.device == self.device and o.dtype == torch.float32 and o.is_contiguous()
                and rewards.device == self.device and rewards.dtype == torch.float32
                and rewards.is_contiguous() and dones.device == self.device
                and dones.dtype == torch.int64 and dones.is_contiguous())

    def _rollout_body(self) -> None:
        """horizon env steps; everything stays on the device (graph-capturable)."""
        b = self.buf
        fp = self.fused_policy
        if fp is not None:
            fp.pack()                  # this epoch's weights (the graph replays the repack)
        for n in range(self.horizon):
            b["dones"][n].copy_(self.dones)
            if fp is not None:         # the policy writes its outputs straight into slot n
                if self._env_act is None:
                    self._env_act = torch.empty_like(b["actions"][n])
                fp.step(self.obs, self.sample_seed, self.rng_counter, n, obs_out=b["obses"][n],
                        actions=b["actions"][n], neglogp=b["neglogpacs"][n], values=b["values"][n],
                        mu=b["mus"][n], sigma=b["sigmas"][n], env_actions=self._env_act,
                        action_low=self.actions_low, action_high=self.actions_high)
                values = b["values"][n]
                obs, rewards, dones, infos = self.env.step(self._env_act)
            else:
                act, nlp, values, mu, sigma = self._policy_step(self.obs, n)
                b["obses"][n].copy_(self.obs)
                b["actions"][n].copy_(act)
                b["neglogpacs"][n].copy_(nlp)
                b["values"][n].copy_(values)
                b["mus"][n].copy_(mu)
                b["sigmas"][n].copy_(sigma)
                obs, rewards, dones, infos = self.env.step(self.preprocess_actions(act))
            if self._record_fused(obs, rewards, dones, infos):
                self.recorder.step(self._obs_tensor(obs), rewards, dones, self.reward_scale, self.obs,
                                   b["rewards"][n], self.dones, self.current_rewards,
                                   self.current_lengths, self.episode_sums[n])
                continue
            rewards = rewards.to(self.device, dtype=torch.float32).view(-1)
            shaped = rewards * self.reward_scale
            if self.value_bootstrap and isinstance(infos, dict) and "time_outs" in infos:
                shaped = shaped + self.gamma * values * infos["time_outs"].to(self.device).float()
            b["rewards"][n].copy_(shaped)
            self.obs.copy_(self._obs_tensor(obs))
            self.dones.copy_(dones.to(self.device).view(-1).float())
            self.current_rewards.add_(rewards)
            self.current_lengths.add_(1.0)
            d = self.dones
            self.episode_sums[n, 0] = d.double().sum()
            self.episode_sums[n, 1] = (self.current_rewards.double() * d.double()).sum()
            self.episode_sums[n, 2] = (self.current_lengths.double() * d.double()).sum()
            self.current_rewards.mul_(1.0 - d)
            self.current_lengths.mul_(1.0 - d)
        # bootstrap value of the state after the last step
        if fp is not None:
            fp.step(self.obs, values=self.last_values)
        else:
            _, _, value = self.model.policy(self.obs)
            self.last_values.copy_(self.model.unnorm_value(value.float()).squeeze(-1))
        self.rng_counter.add_(self.horizon)

    def play_steps(self) -> float:
        """Run the rollout (graph replay on GPU after the first epoch); returns seconds."""
        self.model.eval()
        t0 = time.perf_counter()
        with torch.no_grad():
            if self.use_graph and self.graph is None and self.epoch_num >= 2:
                self._capture()
            if self.graph is not None:
                self.graph.replay()
            else:
                self._rollout_body()
        self._global = self._gather_horizon() if self.central else None
        if self.dp:                                     # global episode statistics in the logs
            dist.all_reduce(self.episode_sums)
        ep = self.episode_sums.cpu().numpy()           # the rollout's one host sync
        for cnt, rsum, lsum in ep:
            if cnt > 0:
                self.game_rewards.update_moments(int(cnt), rsum / cnt)
                self.game_lengths.update_moments(int(cnt), lsum / cnt)
        return time.perf_counter() - t0

    def _capture(self) -> None:
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                self._rollout_body()
        except Exception as e:  # noqa: BLE001 - fall back to eager launches, loudly
            print(f"[rlg] rollout graph capture failed ({e}); running the rollout eagerly")
            self.use_graph = False
            torch.cuda.synchronize(self.device)
            return
        self.graph = g   # capture records the launches without running them

    # ------------------------------------------------------------------ training
    def prepare_dataset(self) -> Dict[str, torch.Tensor]:
        b, last_values, dones = self.buf, self.last_values, self.dones
        if self.central:                 # the learner: every rank's actors, gathered
            b, last_values, dones = self._global
        adv, ret = ops.gae(b["rewards"], b["values"], b["dones"], last_values, dones,
                           self.gamma, self.tau)
        values = swap_and_flatten01(b["values"]).unsqueeze(1)
        returns = swap_and_flatten01(ret).unsqueeze(1)
        advantages = (returns - values).squeeze(1)
        if self.normalize_value:
            vms = self.model.value_mean_std
            vms.train()
            values = vms(values)
            returns = vms(returns)
            vms.eval()
        if self.normalize_advantage:
            advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        fresh = {
            "old_values": values, "old_logp_actions": swap_and_flatten01(b["neglogpacs"]),
            "advantages": advantages, "returns": returns,
            "actions": swap_and_flatten01(b["actions"]), "obs": swap_and_flatten01(b["obses"]),
            "mu": swap_and_flatten01(b["mus"]), "sigma": swap_and_flatten01(b["sigmas"]),
        }
        # persistent dataset buffers: the captured minibatch updates read them by address
        if self._data is None:
            self._data = {k: torch.empty_like(v).contiguous() for k, v in fresh.items()}
        for k, v in fresh.items():
            self._data[k].copy_(v)
        return self._data

    def _lr_update_device(self, kl: torch.Tensor) -> None:
        """AdaptiveScheduler.update on the device LR (legacy schedule, every minibatch)."""
        s, lr = self.scheduler, self.lr_t
        down = torch.clamp(lr / 1.5, min=s.min_lr)
        lr1 = torch.where(kl > 2.0 * s.kl_threshold, down, lr)
        up = torch.clamp(lr1 * 1.5, max=s.max_lr)
        lr.copy_(torch.where(kl < 0.5 * s.kl_threshold, up, lr1))

    def _minibatch_device(self, i: int) -> None:
        """One minibatch update on the device, without host syncs (graph-capturable): PPO loss,
        backward, GradScaler + fused Adam, mu / sigma write-back, adaptive LR, stats row i."""
        self._mb_grad(i)
        self._mb_apply(i)

    def _mb_grad(self, i: int) -> None:
        """First half of a minibatch update: PPO loss and gradients (p.grad), mu / sigma
        write-back; data-parallel: gradients and KL packed into the flat all-reduce buffer."""
        s, e = i * self.minibatch_size, (i + 1) * self.minibatch_size
        data = self._data
        mb = {k: v[s:e] for k, v in data.items()}
        if self.fused_loss:        # mu / sigma written back by the loss kernel itself
            a_loss, c_loss, ent, kl, b_loss = self._calc_gradients_fused(mb, step=False)
        else:
            a_loss, c_loss, ent, kl, cmu, csigma, b_loss = self.calc_gradients(mb, step=False)
            data["mu"][s:e].copy_(cmu)
            data["sigma"][s:e].copy_(csigma)
        self._mb_out[i].copy_(torch.stack([a_loss.float(), c_loss.float(), ent.float(), kl.float(),
                                           b_loss.float()]))
        if self.dp:
            torch.cat([p.grad.reshape(-1) for p in self._params] + [self._mb_out[i, 3:4]], out=self._flat)
            self._f16_overflow_to_inf()

    def _f16_overflow_to_inf(self) -> None:
        """Data-parallel + fp16 shadow weights: the reference's autocast Linear gradients are f16
        on every rank, so one rank's overflow is inf BEFORE the all-reduce and the sum carries it
        to every replica (GradScaler skips the step and backs off the scale everywhere). Here the
        gradients are f32 sums: apply the f16 range rule (|scaled grad| >= 65520 is f16 inf,
        mi_rl_adam_step's f16_overflow) per rank before the all-reduce, else an overflow on one
        rank could be averaged back under the threshold. Capturable (no host sync)."""
        if self._f16_begin is None:
            return
        seg = self._flat[self._f16_begin:self.fused_opt.n]
        seg.masked_fill_(seg.abs() >= 65520.0, float("inf"))

    def _mb_apply(self, i: int) -> None:
        """Second half: (data-parallel: the all-reduced flat buffer / world back into p.grad and
        the KL) GradScaler + Adam step, adaptive LR on the (averaged) KL."""
        if self.fused_opt is not None:     # one flat gradient buffer in, two launches
            if self.dp:
                self._flat.mul_(1.0 / self.world)
                self._mb_out[i, 3].copy_(self._flat[self.fused_opt.n])
                self.fused_opt.step(self._flat, kl=self._mb_out[i, 3])
            else:
                self.fused_opt.step(None, kl=self._mb_out[i, 3])
            return
        if self.dp:
            self._flat.mul_(1.0 / self.world)
            o = 0
            views = []
            for p in self._params:
                views.append(self._flat[o:o + p.numel()].view_as(p))
                o += p.numel()
            torch._foreach_copy_([p.grad for p in self._params], views)
            self._mb_out[i, 3].copy_(self._flat[o])
        self._optimizer_step()
        if self.scheduler is not None:
            self._lr_update_device(self._mb_out[i, 3])

    def _allreduce_flat(self) -> None:
        dist.all_reduce(self._flat)

    def _minibatch_graphed(self, mode: int, i: int) -> None:
        """Replay the captured update of (obs-statistics mode, minibatch i), capturing it on first
        use. Data-parallel: two graphs with the gradient all-reduce between them."""
        key = (mode, i)
        g = self.upd_graphs.get(key)
        if g is None:
            torch.cuda.synchronize(self.device)
            if self.dp:
                ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga):   # records the launches without running them
                    self._mb_grad(i)
                with torch.cuda.graph(gb, pool=ga.pool()):
                    self._mb_apply(i)
                g = (ga, gb)
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._minibatch_device(i)
            self.upd_graphs[key] = g
        if self.dp:
            g[0].replay()
            self._allreduce_flat()
            g[1].replay()
        else:
            g.replay()

    def _minibatch_eager_dp(self, i: int) -> None:
        self._mb_grad(i)
        self._allreduce_flat()
        self._mb_apply(i)

    def _optimizer_step(self) -> None:
        if self.fused_opt is not None:
            self.fused_opt.step()          # no KL here: the LR stays (as below)
            return
        if self.truncate_grads:
            self.scaler.unscale_(self.optimizer)
            nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_norm)
        self.scaler.step(self.optimizer)
        self.scaler.update()

    def _calc_gradients_fused(self, mb: Dict[str, torch.Tensor], step: bool = True):
        """calc_gradients with the loss and its head gradients in one HIP launch
        (mi_rl_ppo_loss): the MLP forward under autocast, the fused loss, autograd from the
        heads down, then the same GradScaler / clip / Adam step. Writes mu / sigma into mb."""
        net = self.model.a2c_network
        with torch.autocast(device_type=self.device.type, dtype=torch.float16, enabled=self.mixed_precision,
                            cache_enabled=False):
            mu, value = net.heads_train(self.model.norm_obs(mb["obs"]), self.wgrad_splits)
            value = value.view(-1)
        gscale = self.scaler._scale if self.mixed_precision else None   # device scale, no sync
        g_mu, g_val, g_ls, sums = ops.ppo_loss(
            mu, net.sigma.detach(), value, mb, self.e_clip, self.clip_value, self.critic_coef,
            self.entropy_coef, float(self.bounds_loss_coef or 0.0), gscale)
        for p in self.model.parameters():
            p.grad = None
        torch.autograd.backward([mu, value], [g_mu, g_val])
        net.sigma.grad = g_ls        # logstd = mu * 0 + sigma: the rows' log-std grads sum here
        if step:
            self._optimizer_step()
        b_loss = sums[3] if self.bounds_loss_coef is not None else sums[3] * 0.0
        return sums[0], sums[1], sums[2], sums[4], b_loss

    def calc_gradients(self, mb: Dict[str, torch.Tensor], step: bool = True):
        # autocast's weight cast cache off: every cast is a recorded launch (graph replay)
        with torch.autocast(device_type=self.device.type, dtype=torch.float16, enabled=self.mixed_precision,
                            cache_enabled=False):
            res = self.model.forward_train(mb["obs"], mb["actions"])
            nlp, values, entropy, mu, sigma = (res["prev_neglogp"], res["values"], res["entropy"],
                                               res["mus"], res["sigmas"])
            ratio = torch.exp(mb["old_logp_actions"] - nlp)
            surr1 = mb["advantages"] * ratio
            surr2 = mb["advantages"] * torch.clamp(ratio, 1.0 - self.e_clip, 1.0 + self.e_clip)
            a_loss = torch.max(-surr1, -surr2)
            if self.clip_value:
                vpc = mb["old_values"] + (values - mb["old_values"]).clamp(-self.e_clip, self.e_clip)
                c_loss = torch.max((values - mb["returns"]) ** 2, (vpc - mb["returns"]) ** 2)
            else:
                c_loss = (mb["returns"] - values) ** 2
            if self.bounds_loss_coef is not None:
                soft_bound = 1.1
                hi = torch.clamp_min(mu - soft_bound, 0.0) ** 2
                lo = torch.clamp_max(mu + soft_bound, 0.0) ** 2
                b_loss = (lo + hi).sum(dim=-1)
            else:
                b_loss = torch.zeros_like(a_loss)
            a_loss, c_loss, entropy, b_loss = a_loss.mean(), c_loss.mean(), entropy.mean(), b_loss.mean()
            loss = (a_loss + 0.5 * c_loss * self.critic_coef - entropy * self.entropy_coef
                    + b_loss * float(self.bounds_loss_coef or 0.0))
        for p in self.model.parameters():
            p.grad = None
        self.scaler.scale(loss).backward()
        with torch.no_grad():
            kl = policy_kl(mu.detach().float(), sigma.detach().float(), mb["mu"], mb["sigma"])
        if step:
            if self.dp:        # eager (CPU / gloo) data-parallel step: average grads and KL first
                kl = self._allreduce_grads_kl(kl)
            self._optimizer_step()
        return a_loss.detach(), c_loss.detach(), entropy.detach(), kl, mu.detach().float(), sigma.detach().float(), b_loss.detach()

    def _allreduce_grads_kl(self, kl: torch.Tensor) -> torch.Tensor:
        """Data-parallel, eager: p.grad and the KL averaged over the ranks in one all-reduce."""
        flat = torch.cat([p.grad.reshape(-1) for p in self._params] + [kl.reshape(1).float()])
        dist.all_reduce(flat)
        flat.mul_(1.0 / self.world)
        o = 0
        for p in self._params:
            p.grad.copy_(flat[o:o + p.numel()].view_as(p))
            o += p.numel()
        return flat[o].to(kl.dtype)

    def update_lr(self, lr: float) -> None:
        if self.lr_t is not None:      # device LR: one tensor shared by every param group
            self.lr_t.fill_(lr)
            lr = self.lr_t
        for g in self.optimizer.param_groups:
            g["lr"] = lr

    def train_epoch(self) -> Dict[str, float]:
        self.epoch_num += 1
        play_time = self.play_steps()
        t0 = time.perf_counter()
        if not self.is_learner:        # a policy replica: wait for the learner's weights
            self._broadcast_weights()
            self.frame += self.frames_per_epoch
            st = {"epoch": self.epoch_num, "frames": self.frame, "play_time": play_time,
                  "update_time": time.perf_counter() - t0,
                  "fps_step_inference": self.frames_per_epoch / play_time,
                  "fps_total": self.frames_per_epoch / (play_time + time.perf_counter() - t0),
                  "mean_rewards": self.game_rewards.get_mean(),
                  "mean_lengths": self.game_lengths.get_mean(), "games": self.game_rewards.current_size}
            self.stats = st
            return st
        self.model.train()
        data = self.prepare_dataset()
        if self.device.type == "cuda":
            # device path: per-minibatch work is sync-free; epochs >= 2 replay captured graphs
            # (epoch 1 runs eagerly: Adam state, BLAS handles and autocast are initialised)
            graphed = self.graph_update and self.epoch_num >= 2
            for mini_ep in range(self.mini_epochs):
                mode = int(self.normalize_input and mini_ep == 0)   # obs statistics update on
                if self.dp and self.normalize_input:
                    # data-parallel: the obs statistics update (merged over the ranks: a
                    # collective) runs eagerly before each minibatch's captured halves, which
                    # then see the statistics frozen — the order of the in-forward update
                    self.model.running_mean_std.eval()
                for i in range(self.num_minibatches):
                    if self.dp:
                        if mode:
                            s, e = i * self.minibatch_size, (i + 1) * self.minibatch_size
                            self.model.running_mean_std._update(self._data["obs"][s:e])
                        if graphed:
                            self._minibatch_graphed(0, i)
                        else:
                            self._minibatch_eager_dp(i)
                    elif graphed:
                        self._minibatch_graphed(mode, i)
                    else:
                        self._minibatch_device(i)
                    self._mb_stats[mini_ep, i].copy_(self._mb_out[i])
                if self.normalize_input:
                    self.model.running_mean_std.eval()   # statistics from the first mini-epoch only
            ms = self._mb_stats.mean(dim=(0, 1)).tolist()           # the update's one host sync
            self.last_lr = float(self.lr_t.item())
            a_loss_m, c_loss_m, ent_m, kl_m, b_loss_m = ms
        else:
            kls, a_l, c_l, b_l, ents = [], [], [], [], []
            for mini_ep in range(self.mini_epochs):
                ep_kls = []
                for i in range(self.num_minibatches):
                    s, e = i * self.minibatch_size, (i + 1) * self.minibatch_size
                    mb = {k: v[s:e] for k, v in data.items()}
                    a_loss, c_loss, ent, kl, cmu, csigma, b_loss = self.calc_gradients(mb)
                    data["mu"][s:e] = cmu
                    data["sigma"][s:e] = csigma
                    ep_kls.append(kl); a_l.append(a_loss); c_l.append(c_loss); ents.append(ent); b_l.append(b_loss)
                    if self.scheduler is not None:
                        self.last_lr = self.scheduler.update(self.last_lr, kl.item())
                        self.update_lr(self.last_lr)
                kls.append(torch.stack(ep_kls).mean())
                if self.normalize_input:
                    self.model.running_mean_std.eval()   # statistics from the first mini-epoch only
            a_loss_m, c_loss_m = torch.stack(a_l).mean().item(), torch.stack(c_l).mean().item()
            b_loss_m, ent_m = torch.stack(b_l).mean().item(), torch.stack(ents).mean().item()
            kl_m = torch.stack(kls).mean().item()
        if self.central:
            self._broadcast_weights()
        update_time = time.perf_counter() - t0
        self.frame += self.frames_per_epoch
        st = {
            "epoch": self.epoch_num, "frames": self.frame, "play_time": play_time,
            "update_time": update_time,
            "fps_step_inference": self.frames_per_epoch / play_time,
            "fps_total": self.frames_per_epoch / (play_time + update_time),
            "a_loss": a_loss_m, "c_loss": c_loss_m, "b_loss": b_loss_m, "entropy": ent_m,
            "kl": kl_m, "lr": self.last_lr,
            "mean_rewards": self.game_rewards.get_mean(), "mean_lengths": self.game_lengths.get_mean(),
            "games": self.game_rewards.current_size,
        }
        self.stats = st
        return st

    def train(self, max_epochs: Optional[int] = None, log=print) -> Dict[str, float]:
        max_epochs = self.max_epochs if max_epochs is None else int(max_epochs)
        self.env_reset()
        st: Dict[str, float] = {}
        while self.epoch_num < max_epochs:
            st = self.train_epoch()
            if log is not None:
                log(f"fps step and policy inference: {st['fps_step_inference']:.0f} fps total: "
                    f"{st['fps_total']:.0f} epoch: {st['epoch']}/{max_epochs} "
                    f"mean reward: {st['mean_rewards']:.3f} mean length: {st['mean_lengths']:.1f}")
            mean_rewards = st["mean_rewards"]
            if self.rank == 0 and self.save_frequency > 0 and self.epoch_num % self.save_frequency == 0:
                self.save(os.path.join(self.run_dir, "nn", f"last_{self.name}_ep_{self.epoch_num}"))
            if (self.game_rewards.current_size > 0 and mean_rewards > self.last_mean_rewards
                    and self.epoch_num >= self.save_best_after):
                self.last_mean_rewards = mean_rewards
                if self.rank == 0:
                    self.save(os.path.join(self.run_dir, "nn", str(self.name)))
                if mean_rewards > self.score_to_win:
                    break
        return st

    # ------------------------------------------------------------------ checkpoints
    def get_full_state_weights(self) -> Dict:
        # plain Python scalars only: the file must load with torch.load(weights_only=True)
        return {"model": self.model.state_dict(), "epoch": int(self.epoch_num), "frame": int(self.frame),
                "optimizer": self.optimizer.state_dict(),
                "last_mean_rewards": float(self.last_mean_rewards),
                "scaler": self.scaler.state_dict(), "last_lr": float(self.last_lr)}

    def save(self, fn: str) -> str:
        os.makedirs(os.path.dirname(fn) or ".", exist_ok=True)
        path = fn if fn.endswith(".pth") else fn + ".pth"
        torch.save(self.get_full_state_weights(), path)
        return path

    def restore(self, fn: str) -> None:
        ck = torch.load(fn, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["model"])
        self.epoch_num = int(ck.get("epoch", 0))
        self.frame = int(ck.get("frame", 0))
        self.last_mean_rewards = float(ck.get("last_mean_rewards", -100500.0))
        self.last_lr = float(ck.get("last_lr", self.last_lr))
        if "optimizer" in ck:
            self.optimizer.load_state_dict(ck["optimizer"])
            if self.fused_opt is not None:
                self.fused_opt.bind()      # the restored moments into the flat buffers
        if "scaler" in ck:
            self.scaler.load_state_dict(ck["scaler"])
        self.update_lr(self.last_lr)   # re-binds the device LR tensor to the param groups
        self.graph = None
        self.upd_graphs = {}           # captured updates referenced the old optimizer state


class A2CPlayer:
    """rl_games PpoPlayerContinuous: deterministic policy (mu) rollouts of a checkpoint."""

    def __init__(self, env, params: Dict) -> None:
        # a player never trains: the training batch geometry (minibatch | horizon x actors) of
        # the config does not constrain it (play runs typically use few envs)
        cfg = dict(params["config"])
        cfg["minibatch_size"] = int(cfg["horizon_length"]) * int(cfg["num_actors"])
        self.agent = A2CAgent(env, {**params, "config": cfg})
        self.env = env

    def restore(self, fn: str) -> None:
        self.agent.restore(fn)

    @torch.no_grad()
    def run(self, games: int = 10, max_steps: int = 108000, log=print) -> Dict[str, float]:
        ag = self.agent
        ag.model.eval()
        ag.env_reset()
        cr = torch.zeros_like(ag.current_rewards)
        cl = torch.zeros_like(ag.current_lengths)
        done_games, rew_sum, len_sum = 0, 0.0, 0.0
        for _ in range(max_steps):
            mu, _, _ = ag.model.policy(ag.obs)
            obs, r, d, _ = self.env.step(ag.preprocess_actions(mu.float()))
            ag.obs.copy_(ag._obs_tensor(obs))
            d = d.to(ag.device).view(-1).float()
            cr += r.to(ag.device).view(-1)
            cl += 1.0
            n = int(d.sum().item())
            if n:
                rew_sum += float((cr * d).sum().item())
                len_sum += float((cl * d).sum().item())
                done_games += n
                cr *= 1.0 - d
                cl *= 1.0 - d
            if done_games >= games:
                break
        res = {"games": done_games, "mean_reward": rew_sum / max(1, done_games),
               "mean_length": len_sum / max(1, done_games)}
        if log is not None:
            log(f"av reward: {res['mean_reward']:.3f} av steps: {res['mean_length']:.1f}")
        return res
