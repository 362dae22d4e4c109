// mi_rl.hip — fused per-sample kernels of the PPO learner (include/mi_rl.h).
//
// Both ops are HBM/latency-trivial elementwise work next to the learner's GEMMs; they exist
// so a rollout step (policy GEMMs + sampling + env step) and the GAE pass are a handful of
// stream-ordered launches that a HIP graph can capture, instead of ~15 small torch kernels
// each. One lane per env row: rows are independent, and every access of a lane walks its own
// row (GAE: time-major columns, coalesced across lanes).
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

extern "C" {

int32_t mi_rl_abi_version(void) { return MI_RL_ABI_VERSION; }
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
