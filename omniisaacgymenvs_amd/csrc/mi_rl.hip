// mi_rl.hip — fused per-sample kernels of the PPO learner (include/mi_rl.h).
//
// The ops are HBM/latency-trivial elementwise work next to the learner's GEMMs; they exist
// so a rollout step (policy GEMMs + sampling + env step), the GAE pass and a minibatch's loss
// are a handful of stream-ordered launches that a HIP graph can capture, instead of tens of
// small torch kernels each. One lane per row: rows are independent, and every access of a lane
// walks its own row (GAE: time-major columns, coalesced across lanes).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>

#include "../../include/mi_rl.h"
#include "mi_device.hpp"

namespace {
thread_local char g_err[512] = "";
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}
constexpr int kOk = 0, kNull = -1, kShape = -2, kHip = -3;
constexpr int kBlock = 256;

int launch_check(const char* what) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? kOk : fail(kHip, "%s: %s", what, hipGetErrorString(e));
}
}  // namespace

// rl_games a2c_common.py discount_values, one lane per env, t = H-1 .. 0
__global__ void k_gae(const float* __restrict__ rew, const float* __restrict__ val,
                      const float* __restrict__ dones, const float* __restrict__ last_val,
                      const float* __restrict__ last_dones, int H, int N, float gamma, float tau,
                      float* __restrict__ adv, float* __restrict__ ret) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float lastgaelam = 0.0f;
    float next_nt = 1.0f - last_dones[n];
    float next_v = last_val[n];
    for (int t = H - 1; t >= 0; --t) {
        const size_t o = (size_t)t * N + n;
        const float v = val[o];
        const float delta = rew[o] + gamma * next_v * next_nt - v;
        lastgaelam = delta + gamma * tau * next_nt * lastgaelam;
        if (adv) adv[o] = lastgaelam;
        if (ret) ret[o] = lastgaelam + v;
        next_nt = 1.0f - dones[o];
        next_v = v;
    }
}

// Philox4x32-10 keyed (seed); counter (block j/4, row, step lo, step hi ^ tag): 4 uniforms in
// (0, 1] -> 2 Box-Muller pairs -> normals 4b .. 4b+3 of the row
__device__ __forceinline__ void normal4(uint64_t seed, uint64_t counter, uint32_t row, uint32_t blk,
                                        float z[4]) {
    uint32_t c[4] = {blk, row, (uint32_t)counter, (uint32_t)(counter >> 32) ^ 0x5EEDA11Cu};
    mi::philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = (float)((c[k] >> 8) + 1u) * (1.0f / 16777216.0f);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const float r = sqrtf(-2.0f * logf(u[2 * p]));
        const float th = 6.2831853071795865f * u[2 * p + 1];
        z[2 * p] = r * cosf(th);
        z[2 * p + 1] = r * sinf(th);
    }
}

__global__ void k_sample_gauss(const float* __restrict__ mu, const float* __restrict__ logstd,
                               int ls_stride, int R, int A, uint64_t seed,
                               const int64_t* __restrict__ cbase, uint64_t coff,
                               float* __restrict__ act, float* __restrict__ nlp) {
#pragma clang fp contract(off)
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= R) return;
    const uint64_t counter = (cbase ? (uint64_t)cbase[0] : 0ull) + coff;
    float sq = 0.0f, lsum = 0.0f;
    float z[4];
    for (int j = 0; j < A; ++j) {
        if ((j & 3) == 0) normal4(seed, counter, (uint32_t)n, (uint32_t)(j >> 2), z);
        const float m = mu[(size_t)n * A + j];
        const float ls = logstd[(size_t)n * ls_stride + j];
        const float sg = expf(ls);
        const float a = m + sg * z[j & 3];
        act[(size_t)n * A + j] = a;
        const float d = (a - m) / sg;
        sq += d * d;
        lsum += ls;
    }
    if (nlp) nlp[n] = 0.5f * sq + 0.918938533204672742f * (float)A + lsum;
}

// rl_games a2c_continuous.calc_gradients, fused: one lane per minibatch row. Forward terms of
// the PPO loss (clipped surrogate, (clipped) value loss, entropy, bound loss) and the policy KL
// against the stored mu / sigma; the gradient of loss x grad_scale w.r.t. the heads (mu rows,
// value rows, the fixed log-std vector); mu / sigma written back in f32 for the next
// mini-epoch's KL. Per-block partial sums (deterministic two-stage reduction, no atomics).
// Derivatives follow torch autograd of the reference expression: torch.max / maximum split
// the gradient evenly on ties, torch.clamp passes it on [lo, hi] inclusive.
template <typename T>
__device__ __forceinline__ float ldf(const void* p, size_t i) {
    return (float)((const T*)p)[i];
}
template <typename T>
__device__ __forceinline__ void stf(void* p, size_t i, float v) {
    ((T*)p)[i] = (T)v;
}

template <typename MT, typename VT>
__global__ __launch_bounds__(256) void k_ppo_loss(
    const void* __restrict__ mu, const float* __restrict__ logstd, const void* __restrict__ value,
    const float* __restrict__ act, const float* __restrict__ old_lp, const float* __restrict__ adv,
    const float* __restrict__ old_v, const float* __restrict__ ret,
    const float* old_mu, const float* old_sg,   // may alias mu_out / sg_out (read-then-write)
    int B, int A, float e_clip, int clip_value, float cc,
    float ec, float bc, const float* __restrict__ gscale, void* __restrict__ g_mu,
    void* __restrict__ g_val, float* __restrict__ part_ls, float* __restrict__ part_sums,
    float* mu_out, float* sg_out) {
#pragma clang fp contract(off)
    extern __shared__ float sred[];                 // [256][A + 1] log-std grads, then [256][5]
    const int tid = threadIdx.x, r = blockIdx.x * blockDim.x + tid;
    const bool on = r < B;
    const float LOG_SQRT_2PI = 0.918938533204672742f;
    const float gs = (gscale ? gscale[0] : 1.0f) / (float)B;
    float a_r = 0.0f, c_r = 0.0f, ent_r = 0.0f, b_r = 0.0f, kl_r = 0.0f;
    float da_dnlp = 0.0f;
    if (on) {
        float sq = 0.0f, lsum = 0.0f;
        for (int j = 0; j < A; ++j) {
            const float m = ldf<MT>(mu, (size_t)r * A + j);
            const float ls = logstd[j];
            const float sg = expf(ls);
            const float d = (act[(size_t)r * A + j] - m) / sg;
            sq += d * d;
            lsum += ls;
            ent_r += 0.5f + LOG_SQRT_2PI + ls;
            const float hi = fmaxf(m - 1.1f, 0.0f), lo = fminf(m + 1.1f, 0.0f);
            b_r += lo * lo + hi * hi;
            const float osg = old_sg[(size_t)r * A + j], omu = old_mu[(size_t)r * A + j];
            const float c1 = logf(osg / sg + 1e-5f);
            const float c2 = (sg * sg + (omu - m) * (omu - m)) / (2.0f * (osg * osg + 1e-5f));
            kl_r += c1 + c2 - 0.5f;
            mu_out[(size_t)r * A + j] = m;
            sg_out[(size_t)r * A + j] = sg;
        }
        const float nlp = 0.5f * sq + LOG_SQRT_2PI * (float)A + lsum;
        const float ratio = expf(old_lp[r] - nlp);
        const float av = adv[r];
        const float rc = fminf(fmaxf(ratio, 1.0f - e_clip), 1.0f + e_clip);
        const float n1 = -(av * ratio), n2 = -(av * rc);
        a_r = fmaxf(n1, n2);
        const float dclip = (ratio >= 1.0f - e_clip && ratio <= 1.0f + e_clip) ? 1.0f : 0.0f;
        const float w1 = n1 > n2 ? 1.0f : (n1 < n2 ? 0.0f : 0.5f);
        const float da_dratio = w1 * (-av) + (1.0f - w1) * (-av * dclip);
        da_dnlp = da_dratio * (-ratio);
        // value loss
        const float v = ldf<VT>(value, r), R = ret[r];
        float dc_dv;
        if (clip_value) {
            const float ov = old_v[r], dv = v - ov;
            const float vpc = ov + fminf(fmaxf(dv, -e_clip), e_clip);
            const float l1 = (v - R) * (v - R), l2 = (vpc - R) * (vpc - R);
            c_r = fmaxf(l1, l2);
            const float wv = l1 > l2 ? 1.0f : (l1 < l2 ? 0.0f : 0.5f);
            const float dvpc = (dv >= -e_clip && dv <= e_clip) ? 1.0f : 0.0f;
            dc_dv = wv * 2.0f * (v - R) + (1.0f - wv) * 2.0f * (vpc - R) * dvpc;
        } else {
            c_r = (R - v) * (R - v);
            dc_dv = 2.0f * (v - R);
        }
        stf<VT>(g_val, r, gs * 0.5f * cc * dc_dv);
        // mu gradients (surrogate through nlp + bound loss)
        for (int j = 0; j < A; ++j) {
            const float m = ldf<MT>(mu, (size_t)r * A + j);
            const float sg = expf(logstd[j]);
            const float dm = act[(size_t)r * A + j] - m;
            const float dnlp_dm = -dm / (sg * sg);
            const float db = 2.0f * fmaxf(m - 1.1f, 0.0f) + 2.0f * fminf(m + 1.1f, 0.0f);
            stf<MT>(g_mu, (size_t)r * A + j, gs * (da_dnlp * dnlp_dm + bc * db));
        }
    }
    // log-std gradient rows -> per-block column sums
    const int AP = A + 1;
    for (int j = 0; j < A; ++j) {
        float g = 0.0f;
        if (on) {
            const float sg = expf(logstd[j]);
            const float d = (act[(size_t)r * A + j] - ldf<MT>(mu, (size_t)r * A + j)) / sg;
            g = gs * (da_dnlp * (1.0f - d * d) - ec);
        }
        sred[tid * AP + j] = g;
    }
    __syncthreads();
    if (tid < A) {
        float s = 0.0f;
        for (int q = 0; q < (int)blockDim.x; ++q) s += sred[q * AP + tid];
        part_ls[(size_t)blockIdx.x * A + tid] = s;
    }
    __syncthreads();
    sred[tid * 5 + 0] = a_r; sred[tid * 5 + 1] = c_r; sred[tid * 5 + 2] = ent_r;
    sred[tid * 5 + 3] = b_r; sred[tid * 5 + 4] = kl_r;
    __syncthreads();
    if (tid < 5) {
        float s = 0.0f;
        for (int q = 0; q < (int)blockDim.x; ++q) s += sred[q * 5 + tid];
        part_sums[(size_t)blockIdx.x * 5 + tid] = s;
    }
}

extern "C" {

int32_t mi_rl_abi_version(void) { return MI_RL_ABI_VERSION; }
#ifndef MI_BUILD_ID
#define MI_BUILD_ID "unknown"
#endif
// the string carries a marker prefix so the build id can be found in the binary file
const char* mi_rl_build_id(void) {
    static const char id[] = MI_BUILD_ID;
    return (sizeof(id) > 12 && id[0] == 'M' && id[11] == ':') ? id + 12 : id;
}

int32_t mi_rl_ppo_loss(const void* mu, int32_t mu_half, const float* logstd, const void* value,
                       int32_t value_half, const float* actions, const float* old_logp,
                       const float* advantages, const float* old_values, const float* returns,
                       const float* old_mu, const float* old_sigma, int32_t num_rows,
                       int32_t num_actions, float e_clip, int32_t clip_value, float critic_coef,
                       float entropy_coef, float bounds_coef, const float* grad_scale,
                       void* grad_mu, void* grad_value, float* grad_logstd_part,
                       float* sums_part, float* mu_out, float* sigma_out, void* stream) {
    if (!mu || !logstd || !value || !actions || !old_logp || !advantages || !old_values ||
        !returns || !old_mu || !old_sigma || !grad_mu || !grad_value || !grad_logstd_part ||
        !sums_part || !mu_out || !sigma_out)
        return fail(kNull, "mi_rl_ppo_loss: null buffer");
    if (num_rows <= 0 || num_actions <= 0 || num_actions > 64)
        return fail(kShape, "mi_rl_ppo_loss: B=%d A=%d", num_rows, num_actions);
    const dim3 g((num_rows + kBlock - 1) / kBlock);
    const size_t lds = sizeof(float) * kBlock * (size_t)(num_actions + 1 > 5 ? num_actions + 1 : 5);
#define PPO_LAUNCH(MT, VT)                                                                       \
    hipLaunchKernelGGL((k_ppo_loss<MT, VT>), g, dim3(kBlock), lds, (hipStream_t)stream, mu,      \
                       logstd, value, actions, old_logp, advantages, old_values, returns, old_mu, \
                       old_sigma, num_rows, num_actions, e_clip, clip_value, critic_coef,         \
                       entropy_coef, bounds_coef, grad_scale, grad_mu, grad_value,                \
                       grad_logstd_part, sums_part, mu_out, sigma_out)
    if (mu_half && value_half) PPO_LAUNCH(_Float16, _Float16);
    else if (mu_half) PPO_LAUNCH(_Float16, float);
    else if (value_half) PPO_LAUNCH(float, _Float16);
    else PPO_LAUNCH(float, float);
#undef PPO_LAUNCH
    return launch_check("mi_rl_ppo_loss");
}
const char* mi_rl_last_error(void) { return g_err; }

int32_t mi_rl_gae(const float* rewards, const float* values, const float* dones,
                  const float* last_values, const float* last_dones, int32_t horizon,
                  int32_t num_envs, float gamma, float tau, float* advantages, float* returns,
                  void* stream) {
    if (!rewards || !values || !dones || !last_values || !last_dones)
        return fail(kNull, "mi_rl_gae: null input");
    if (!advantages && !returns) return fail(kNull, "mi_rl_gae: no output");
    if (horizon <= 0 || num_envs <= 0) return fail(kShape, "mi_rl_gae: H=%d N=%d", horizon, num_envs);
    hipLaunchKernelGGL(k_gae, dim3((num_envs + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       (hipStream_t)stream, rewards, values, dones, last_values, last_dones, horizon,
                       num_envs, gamma, tau, advantages, returns);
    return launch_check("mi_rl_gae");
}

int32_t mi_rl_sample_gauss(const float* mu, const float* logstd, int32_t logstd_stride,
                           int32_t num_rows, int32_t num_actions, uint64_t seed,
                           const int64_t* counter_base, uint64_t counter_offset, float* actions,
                           float* neglogp, void* stream) {
    if (!mu || !logstd || !actions) return fail(kNull, "mi_rl_sample_gauss: null buffer");
    if (num_rows <= 0 || num_actions <= 0 || (logstd_stride != 0 && logstd_stride != num_actions))
        return fail(kShape, "mi_rl_sample_gauss: R=%d A=%d stride=%d", num_rows, num_actions,
                    logstd_stride);
    hipLaunchKernelGGL(k_sample_gauss, dim3((num_rows + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       (hipStream_t)stream, mu, logstd, logstd_stride, num_rows, num_actions, seed,
                       counter_base, counter_offset, actions, neglogp);
    return launch_check("mi_rl_sample_gauss");
}

}  // extern "C"
