/*
 * mi_rl.h — C ABI of libmi_rl.so: the fused elementwise ops of the PPO learner that drives
 * the hot path (the caller of VecEnvRLGames.step).
 *
 * The reference trains with rl-games 1.5.2 (setup.py:17; not vendored under /root/reference,
 * absent from this image). Its call sites are scripts/rlgames_train.py:67-84 (Runner over the
 * 'rlgpu' env) and the hyper-parameters in cfg/train/{Humanoid,Ant,Cartpole}PPO.yaml. The
 * per-sample work of its a2c_continuous agent that is not GEMMs is fused here:
 *   mi_rl_gae          — rl_games common/a2c_common.py discount_values (GAE(gamma, tau)
 *                        over the horizon, returns = advantages + values)
 *   mi_rl_sample_gauss — rl_games algos_torch/models.py ModelA2CContinuousLogStd forward in
 *                        eval mode: action ~ Normal(mu, exp(logstd)) and its neg-log-prob
 *   mi_rl_ppo_loss     — rl_games algos_torch/a2c_continuous.py calc_gradients: the PPO loss
 *                        terms, the policy KL and the loss gradient w.r.t. the network heads
 *   mi_rl_policy_step  — the rollout's whole policy evaluation (normalisation, MLP, heads,
 *                        sampling, action rescale) as one f32-MFMA launch
 *   mi_rl_record_step  — the rollout's per-step bookkeeping after env.step
 *   mi_rl_adam_step    — rl_games a2c_common trancate_gradients_and_step (GradScaler unscale,
 *                        grad-norm clip, Adam, scaler update) + the adaptive LR, two launches
 * The training minibatch GEMMs stay in hipBLASLt (torch.nn.Linear, autograd).
 *
 * Conventions: as mi_sim.h — 0 on success or a negative MI_E_* code (mi_rl_last_error());
 * device pointers; `stream` is a hipStream_t passed as void*; stream-ordered, non-blocking.
 */
#ifndef MI_RL_H
#define MI_RL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_RL_ABI_VERSION 2

int32_t mi_rl_abi_version(void);
/* SHA-256 (hex) of the sources this library was compiled from (csrc/mi_rl.hip, the csrc .hpp headers,
 * the include headers; __graft_entry__.source_hash), as mi_build_id of libmi_sim.so. */
const char* mi_rl_build_id(void);
const char* mi_rl_last_error(void);

/* GAE over a rollout stored time-major [H][N] (rl_games experience buffer layout).
 * dones[t][n] = episode-end flag BEFORE step t (rl_games stores self.dones before env.step);
 * last_values / last_dones: bootstrap value and done flags after the last step.
 *   delta_t = r_t + gamma * v_{t+1} * (1 - d_{t+1}) - v_t
 *   A_t     = delta_t + gamma * tau * (1 - d_{t+1}) * A_{t+1}
 * Writes advantages [H][N] and returns = advantages + values [H][N] (either may be NULL). */
int32_t mi_rl_gae(const float* rewards, const float* values, const float* dones,
                  const float* last_values, const float* last_dones, int32_t horizon,
                  int32_t num_envs, float gamma, float tau, float* advantages, float* returns,
                  void* stream);

/* actions[n][j] = mu[n][j] + exp(logstd[n * logstd_stride + j]) * z, z ~ N(0, 1) from the
 * counter-based Philox4x32-10 stream keyed (seed, counter, row n, j) — Box-Muller on pairs of
 * uniforms; neglogp[n] = 0.5 sum_j ((a - mu) / sigma)^2 + 0.5 log(2 pi) A + sum_j logstd,
 * exactly rl_games' ModelA2CContinuousLogStd.neglogp on the sampled action.
 * logstd_stride = 0 broadcasts one [A] row (fixed_sigma), = A for per-row sigmas.
 * counter = *counter_base + counter_offset when counter_base (a device int64) is given, so a
 * captured HIP graph draws fresh noise on every replay once the base is advanced on device. */
int32_t mi_rl_sample_gauss(const float* mu, const float* logstd, int32_t logstd_stride,
                           int32_t num_rows, int32_t num_actions, uint64_t seed,
                           const int64_t* counter_base, uint64_t counter_offset, float* actions,
                           float* neglogp, void* stream);

/* The PPO loss of rl_games a2c_continuous.calc_gradients (algos_torch/a2c_continuous.py: clipped
 * surrogate, value loss — clipped when clip_value —, entropy, bound loss with soft bound 1.1,
 * policy KL against the stored mu / sigma) fused for one minibatch of num_rows rows, together
 * with the gradient of  grad_scale x loss  w.r.t. the network heads, for autograd to carry
 * through the MLP:
 *   mu [B,A], value [B]        network heads, f16 (mu_half / value_half = 1) or f32
 *   logstd [A]                 the fixed-sigma log-std parameter (f32)
 *   actions [B,A], old_logp, advantages, old_values, returns [B], old_mu, old_sigma [B,A]  f32
 *   grad_scale                 device f32 scalar (GradScaler scale) or NULL (1)
 * Outputs: grad_mu (dtype of mu), grad_value (dtype of value); grad_logstd_part [nblk][A] and
 * sums_part [nblk][5] (a_loss, c_loss, entropy, b_loss, kl row sums) per 256-row block,
 * nblk = ceil(B / 256), summed by the caller; mu_out / sigma_out [B,A] f32 = mu, exp(logstd)
 * (may alias old_mu / old_sigma: each element is read before it is written).
 * loss = mean(a) + 0.5 critic_coef mean(c) - entropy_coef mean(entropy) + bounds_coef mean(b). */
int32_t mi_rl_ppo_loss(const void* mu, int32_t mu_half, const float* logstd, const void* value,
                       int32_t value_half, const float* actions, const float* old_logp,
                       const float* advantages, const float* old_values, const float* returns,
                       const float* old_mu, const float* old_sigma, int32_t num_rows,
                       int32_t num_actions, float e_clip, int32_t clip_value, float critic_coef,
                       float entropy_coef, float bounds_coef, const float* grad_scale,
                       void* grad_mu, void* grad_value, float* grad_logstd_part,
                       float* sums_part, float* mu_out, float* sigma_out, void* stream);

/* The rollout policy of rl_games a2c_continuous (play_steps: ModelA2CContinuousLogStd in eval mode
 * -> get_action_values), fused: RunningMeanStd input normalisation, the MLP trunk (ELU), the mu
 * and value heads, value un-normalisation and the Gaussian sample of mi_rl_sample_gauss, for
 * every row, in ONE launch (f32 MFMA GEMMs, activations in LDS). Network: HumanoidPPO.yaml:24-25
 * (units [400, 200, 100], elu, fixed sigma); torch nn.Linear weights [out][in]. */
#define MI_RL_MAX_HIDDEN 4
typedef struct {
    int32_t num_obs;                          /* O */
    int32_t num_actions;                      /* A (<= 64) */
    int32_t num_hidden;                       /* hidden layers, 1 .. MI_RL_MAX_HIDDEN */
    int32_t units[MI_RL_MAX_HIDDEN];          /* hidden widths (<= 512) */
    const float* w[MI_RL_MAX_HIDDEN + 2];     /* device: hidden layers, then mu [A][u], value [1][u] */
    const float* b[MI_RL_MAX_HIDDEN + 2];
} mi_rl_mlp;
/* floats of the packed weight buffer (zero-padded [N16][K16] per layer + bias; the heads as one
 * [A + 1] layer), or -1 on a bad description */
int64_t mi_rl_mlp_packed_size(const mi_rl_mlp* mlp);
/* Repack the network's current weights (stream-ordered; call after every weight update). */
int32_t mi_rl_mlp_pack(const mi_rl_mlp* mlp, float* packed, void* stream);
/* The minibatch network of the PPO update (rl_games calc_gradients under autocast fp16,
 * HumanoidPPO.yaml mixed_precision: True) on fp16 MFMA, one launch each for the forward and for
 * the dgrad chain; the weight / bias gradients stay split-K GEMMs over the stored layer inputs.
 * Supported layouts (else packed size -1 and the learner keeps its torch path): 3 hidden ELU
 * layers 87-400-200-100 with 21 actions (HumanoidPPO.yaml:24-25) or 60-256-128-64 with 8
 * (AntPPO.yaml). mi_rl_mlp_train_pack: f16 A-operand images of every layer's W (forward) and
 * W^T (backward) plus the biases, from the f32 masters the descriptor points at (call after every
 * optimizer step; stream-ordered). */
int64_t mi_rl_mlp_train_packed_size(const mi_rl_mlp* mlp);   /* halfs, or -1 */
int32_t mi_rl_mlp_train_pack(const mi_rl_mlp* mlp, void* packed /*f16*/, void* stream);
/* x [rows][O] f32 (the normalised observations); acts: 4 device buffers, f16 [rows][O + 1],
 * [rows][H1 + 1], [rows][H2 + 1], [rows][H3 + 1]: each layer's input with a ones column (the
 * bias column of the weight gradient), each row padded to a multiple of 8 halfs (row stride
 * (width + 1 + 7) & ~7); mu f16 [rows][A], value f16 [rows] (the heads, as autocast's f16
 * linears return them). */
int32_t mi_rl_mlp_train_fwd(const mi_rl_mlp* mlp, const void* packed, const float* x, int32_t rows,
                            void* const* acts, void* mu, void* value, void* stream);
/* grad_mu f16 [rows][A], grad_value f16 [rows] (the loss gradient w.r.t. the heads);
 * grads: 3 device buffers f16 [rows][H1], [rows][H2], [rows][H3], the gradient w.r.t. each hidden
 * layer's pre-activation (after the ELU derivative, from acts[1..3]). */
int32_t mi_rl_mlp_train_bwd(const mi_rl_mlp* mlp, const void* packed, void* const* acts,
                            const void* grad_mu, const void* grad_value, int32_t rows,
                            void* const* grads, void* stream);
/* For rows n < num_rows of obs [R][O]: obs_out[n] = obs[n] (the rollout slot; may be NULL);
 * x = clamp((obs - mean) / sqrt(var + eps), +-5) when obs_mean / obs_var (f64 running
 * statistics) are given; mu, v = heads(MLP(x)); values[n] = sqrt(var_v + eps) clamp(v, +-5) +
 * mean_v when value_mean / value_var are given, else v; sigma = exp(logstd) ([A], fixed sigma);
 * actions / neglogp exactly as mi_rl_sample_gauss(mu, logstd, 0, ..., seed, counter_base,
 * counter_offset); mu_out / sigma_out [R][A]; env_actions [R][A] = rl_games preprocess_actions
 * (clamp to +-1, rescale to [action_low, action_high], [A] each). Any output may be NULL
 * (neglogp and env_actions need actions). */
int32_t mi_rl_policy_step(const mi_rl_mlp* mlp, const float* packed, const float* obs,
                          int32_t num_rows, const double* obs_mean, const double* obs_var,
                          const double* value_mean, const double* value_var, float eps,
                          const float* logstd, uint64_t seed, const int64_t* counter_base,
                          uint64_t counter_offset, float* obs_out, float* actions, float* neglogp,
                          float* values, float* mu_out, float* sigma_out, const float* action_low,
                          const float* action_high, float* env_actions, void* stream);

/* The rollout's bookkeeping after env.step (rl_games a2c_common play_steps), one launch:
 *   rewards_out[n] = rewards[n] * reward_scale      (the experience buffer row; reward_shaper)
 *   obs_state[n]   = obs_in[n]  ([N][O]),  dones_state[n] = (float) dones[n]
 *   cur_rewards[n] += rewards[n]; cur_lengths[n] += 1
 *   episode_sums[0..2] = sum_n d, sum_n d * cur_rewards, sum_n d * cur_lengths  (f64; the
 *                        finished episodes' count, reward and length sums of this step)
 *   cur_rewards[n] *= 1 - d; cur_lengths[n] *= 1 - d
 * scratch: f64 [ceil(N / 256)][3]; ticket: a device uint32 that is 0 before the first call
 * (the launch leaves it 0 again, so the call can be captured in a graph and replayed). */
int32_t mi_rl_record_step(const float* obs_in, int32_t num_obs, const float* rewards,
                          const int64_t* dones, int32_t num_envs, float reward_scale,
                          float* obs_state, float* rewards_out, float* dones_state,
                          float* cur_rewards, float* cur_lengths, double* episode_sums,
                          double* scratch, uint32_t* ticket, void* stream);

/* The learner's optimizer step over its flat fp32 parameter buffer, as rl-games a2c_common
 * (rl_games 1.5.2 calc_gradients -> trancate_gradients_and_step with truncate_grads: True and
 * mixed precision) runs it through torch: GradScaler.unscale_, clip_grad_norm_(grad_norm),
 * GradScaler.step(Adam), GradScaler.update, then the legacy adaptive LR on the minibatch KL
 * (AdaptiveScheduler.update). Two launches, no host synchronisation (graph-capturable):
 *   pass 1: g = grads * (1 / scale); found_inf = any g non-finite, or any f16-formed scaled
 *           gradient beyond f16 range (only with a scaler, as GradScaler's); norm = ||g||_2 (f64 sums of
 *           f32 squares, per-block partials added in block order by the last block);
 *           coef = max_grad_norm > 0 ? min(max_grad_norm / (norm + 1e-6), 1) : 1
 *   pass 2: unless found_inf, with t = *step + 1 (torch Adam, weight_decay as L2):
 *             g' = (g * coef) + weight_decay * p
 *             m = beta1 m + (1 - beta1) g';  v = beta2 v + (1 - beta2) g'^2
 *             p -= (lr / (1 - beta1^t)) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
 *           then (the last block, after every block has read them): *step = t unless found_inf;
 *           GradScaler.update on *scale / *growth_tracker (scale == NULL: no scaler); and with
 *           adaptive_lr, lr <- lr / 1.5 (>= min_lr) if *kl > 2 kl_threshold, lr * 1.5
 *           (<= max_lr) if *kl < kl_threshold / 2.
 * params / grads / exp_avg / exp_avg_sq: n f32 (grads are read, not modified); step, lr, scale:
 * device f32 scalars; growth_tracker: device int32; kl: device f32 (NULL: no LR update).
 * scratch: f64, at least 1028 entries; tickets: 5 device uint32 — [0] and [4] launch tickets, 0
 * before the first call and left 0 (graph-capturable); [1] counts the skipped (found_inf) steps,
 * [2] holds the lowest offending flat index of the latest one, [3] is 0xFFFFFFFF between calls. */
typedef struct {
    float beta1, beta2, eps, weight_decay;
    float max_grad_norm;               /* <= 0: no clipping */
    float growth_factor, backoff_factor;
    int32_t growth_interval;
    int32_t adaptive_lr;
    float kl_threshold, min_lr, max_lr;
    /* > 0: grads[i] for i >= f16_begin were formed in f16 under autocast by the reference (its
     * Linear weight / bias gradients); a scaled value with |g| >= f16_overflow (65520: rounds to
     * f16 inf) makes found_inf, as the reference's f16 gradient would be inf */
    float f16_overflow;
    int64_t f16_begin;
} mi_rl_adam_cfg;

int32_t mi_rl_adam_step(const mi_rl_adam_cfg* cfg, float* params, const float* grads, float* exp_avg,
                        float* exp_avg_sq, int64_t n, float* step, float* lr, float* scale,
                        int32_t* growth_tracker, const float* kl, double* scratch, int64_t scratch_len,
                        uint32_t* tickets, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MI_RL_H */
