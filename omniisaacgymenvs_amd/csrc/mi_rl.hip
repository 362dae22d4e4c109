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

// ---------------------------------------------------------------------------------------
// Rollout policy step: rl_games ModelA2CContinuousLogStd in eval mode (running-mean-std input
// normalisation, the MLP trunk with ELU, the mu / value heads, value un-normalisation) plus the
// Gaussian sample, for a tile of 16 rows per workgroup, in ONE launch. The GEMMs run on the f32
// MFMA (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation — torch's fp32 matmul up to
// summation order); activations stay in LDS between layers, weights stream from L2 (the packed
// copy is ~0.55 MB for the Humanoid network, shared by every workgroup).
//
// MFMA operand maps (16x16x4 f32): lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15];
// D register i of lane l is row 4 (l >> 4) + i, column l & 15. A K-chunk of 16 is consumed as 4
// MFMAs whose k index is permuted (step s, lane group j = l >> 4 -> k = 4 j + s), so each lane
// fetches ONE float4 of the activation row (LDS) and ONE float4 of the weight row (global) per
// chunk and feeds component s to step s; the sum over the chunk is unchanged.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int kPolRows = 16;      // rows per workgroup (one MFMA row tile)
#ifndef MI_POL_WAVES
#define MI_POL_WAVES 8
#endif
constexpr int kPolWaves = MI_POL_WAVES;   // waves per workgroup (column tiles dealt round-robin)
constexpr int kPolTiles = 8;      // max 16-column tiles per wave per layer (N_pad <= 512)
constexpr int kPolMaxLayers = MI_RL_MAX_HIDDEN + 1;
constexpr int kPolMaxWidth = 16 * kPolWaves * kPolTiles < 512 ? 16 * kPolWaves * kPolTiles : 512;

struct PolLayer {
    int K, N, Kp, Np;             // true and padded (multiple of 16) input / output widths
    long long w, b;               // float offsets of the packed [Np][Kp] weights and [Np] bias
};
struct PolDesc {
    int O, A, L;                  // obs, actions, layers incl. the head (hidden + 1)
    int xs;                       // LDS activation row stride (floats)
    PolLayer ly[kPolMaxLayers];
    long long total;              // floats in the packed buffer
};

int pad16(int x) { return (x + 15) & ~15; }

constexpr size_t kPolMaxLds = 65536;   // default dynamic-LDS limit of a launch
size_t pol_lds_bytes(const PolDesc& d) {
    return sizeof(float) * ((size_t)2 * kPolRows * d.xs + (size_t)kPolRows * 64);
}

int pol_desc(const mi_rl_mlp* m, PolDesc* d) {
    if (!m) return fail(kNull, "mi_rl: null mlp");
    if (m->num_obs <= 0 || m->num_actions <= 0 || m->num_actions > 64 || m->num_hidden < 1 ||
        m->num_hidden > MI_RL_MAX_HIDDEN)
        return fail(kShape, "mi_rl: mlp O=%d A=%d hidden=%d", m->num_obs, m->num_actions, m->num_hidden);
    d->O = m->num_obs;
    d->A = m->num_actions;
    d->L = m->num_hidden + 1;
    long long off = 0;
    int in = m->num_obs, mx = pad16(m->num_obs);
    for (int l = 0; l < d->L; ++l) {
        const int out = l < m->num_hidden ? m->units[l] : m->num_actions + 1;   // head: mu | value
        if (out <= 0 || pad16(out) > kPolMaxWidth)
            return fail(kShape, "mi_rl: layer %d width %d (max %d)", l, out, kPolMaxWidth);
        PolLayer& y = d->ly[l];
        y.K = in; y.N = out; y.Kp = pad16(in); y.Np = pad16(out);
        y.w = off; off += (long long)y.Np * y.Kp;
        y.b = off; off += y.Np;
        if (y.Np > mx) mx = y.Np;
        in = out;
    }
    d->xs = mx + 4;               // +4 floats: rows start on different LDS banks
    d->total = off;
    // k_policy_step's dynamic LDS (two activation tiles + the head scratch) must fit the default
    // 64 KB per-launch limit: refuse the layout here, so mi_rl_mlp_packed_size fails and the
    // caller (FusedPolicy) falls back to the torch policy instead of a failed launch later
    const size_t lds = pol_lds_bytes(*d);
    if (lds > kPolMaxLds)
        return fail(kShape, "mi_rl: mlp needs %zu B of LDS (widest padded layer / obs %d; max %zu B)", lds,
                    mx, kPolMaxLds);
    return kOk;
}

__global__ void k_pol_pack(PolDesc d, mi_rl_mlp m, float* __restrict__ packed) {
    // one thread per packed element (zeros in the padding)
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.total) return;
    for (int l = 0; l < d.L; ++l) {
        const PolLayer& y = d.ly[l];
        const bool head = l == d.L - 1;
        if (i >= y.w && i < y.w + (long long)y.Np * y.Kp) {
            const int n = (int)((i - y.w) / y.Kp), k = (int)((i - y.w) % y.Kp);
            float v = 0.0f;
            if (k < y.K && n < y.N) {
                if (!head) v = m.w[l][(size_t)n * y.K + k];
                else v = n < d.A ? m.w[l][(size_t)n * y.K + k] : m.w[l + 1][k];   // mu rows, value row
            }
            packed[i] = v;
            return;
        }
        if (i >= y.b && i < y.b + y.Np) {
            const int n = (int)(i - y.b);
            float v = 0.0f;
            if (n < y.N) v = !head ? m.b[l][n] : (n < d.A ? m.b[l][n] : m.b[l + 1][0]);
            packed[i] = v;
            return;
        }
    }
}

typedef float pf4 __attribute__((ext_vector_type(4)));

constexpr int kPolDepth = 3;      // weight chunks in flight per tile (L2 latency vs MFMA time)

// T column tiles of one layer for this wave (tiles wave, wave + 4, ...), K-chunk loop with the
// weight float4s of the next kPolDepth chunks in flight; T is a template constant so every
// accumulator and ring slot is a fixed register (a runtime tile count with per-tile predicates
// made the compiler shuffle the whole accumulator array around each MFMA)
template <int T>
__device__ __forceinline__ void pol_tiles(const PolLayer& y, const float* __restrict__ packed,
                                          const float* X, float* Y, int xs, bool elu, int wave,
                                          int lane) {
    const int r = lane & 15, j = lane >> 4;
    const int Kp = y.Kp, nc = Kp >> 4;
    const float* W = packed + y.w + (size_t)(16 * wave + r) * Kp + 4 * j;
    const size_t tstride = (size_t)16 * kPolWaves * Kp;          // next tile of this wave
    const float* xp = X + r * xs + 4 * j;
    pf4 acc[T];
    pf4 ring[kPolDepth][T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = pf4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int p = 0; p < kPolDepth; ++p) {
        const int c = p < nc ? p : nc - 1;
#pragma unroll
        for (int t = 0; t < T; ++t) ring[p][t] = *(const pf4*)(W + t * tstride + 16 * c);
    }
    // whole groups of kPolDepth chunks: no branch inside, so the waits before each chunk's
    // MFMAs count only that chunk's loads (the later chunks' stay in flight)
    pf4 a = *(const pf4*)xp;
    int c0 = 0;
    for (; c0 + kPolDepth <= nc; c0 += kPolDepth) {
#pragma unroll
        for (int p = 0; p < kPolDepth; ++p) {
            const int c = c0 + p;
            const pf4 an = *(const pf4*)(xp + 16 * (c + 1 < nc ? c + 1 : c));   // next chunk's A
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int t = 0; t < T; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], ring[p][t][s], acc[t], 0, 0, 0);
            }
            const int cn = c + kPolDepth < nc ? c + kPolDepth : nc - 1;
#pragma unroll
            for (int t = 0; t < T; ++t) ring[p][t] = *(const pf4*)(W + t * tstride + 16 * cn);
            a = an;
        }
    }
    // the last nc % kPolDepth chunks: ring slot p holds chunk c0 + p
#pragma unroll
    for (int p = 0; p < kPolDepth - 1; ++p) {
        if (c0 + p < nc) {
            const pf4 ap = *(const pf4*)(xp + 16 * (c0 + p));
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int t = 0; t < T; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[s], ring[p][t][s], acc[t], 0, 0, 0);
            }
        }
    }
    const float* B = packed + y.b;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int col = 16 * (wave + kPolWaves * t) + r;
        const float bias = B[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float v = acc[t][i] + bias;
            if (elu) v = v > 0.0f ? v : expm1f(v);
            Y[(4 * j + i) * xs + col] = v;
        }
    }
}

// one layer for the workgroup's 16 rows: Y[16][Np] = act(X[16][Kp] W^T + b), X / Y in LDS
__device__ __forceinline__ void pol_layer(const PolLayer& y, const float* __restrict__ packed,
                                          const float* X, float* Y, int xs, bool elu, int wave,
                                          int lane) {
    const int nt = y.Np >> 4;
    const int mine = __builtin_amdgcn_readfirstlane((nt - wave + kPolWaves - 1) / kPolWaves);
    switch (mine) {
        case 1: pol_tiles<1>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 2: pol_tiles<2>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 3: pol_tiles<3>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 4: pol_tiles<4>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 5: pol_tiles<5>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 6: pol_tiles<6>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 7: pol_tiles<7>(y, packed, X, Y, xs, elu, wave, lane); break;
        case 8: pol_tiles<8>(y, packed, X, Y, xs, elu, wave, lane); break;
        default: break;                           // 0: this wave has no tile in this layer
    }
}

__global__ __launch_bounds__(64 * kPolWaves) void k_policy_step(
    PolDesc d, const float* __restrict__ packed, const float* __restrict__ obs, int R,
    const double* __restrict__ om, const double* __restrict__ ov, const double* __restrict__ vm,
    const double* __restrict__ vv, float eps, const float* __restrict__ logstd, uint64_t seed,
    const int64_t* __restrict__ cbase, uint64_t coff, float* __restrict__ obs_out,
    float* __restrict__ act, float* __restrict__ nlp, float* __restrict__ val,
    float* __restrict__ mu_out, float* __restrict__ sg_out, const float* __restrict__ alo,
    const float* __restrict__ ahi, float* __restrict__ env_act) {
#pragma clang fp contract(off)
    extern __shared__ float pl[];                 // two [16][xs] activation tiles + noise [16][64]
    float* X0 = pl;
    float* X1 = pl + kPolRows * d.xs;
    float* Z = pl + 2 * kPolRows * d.xs;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row0 = blockIdx.x * kPolRows;
    const int O = d.O, A = d.A;
    // input tile: raw obs -> obs_out (the rollout slot), normalised (running mean / std,
    // clamped to +-5, rl_games RunningMeanStd.forward in eval mode) -> X0, zero padding
    const int Kp0 = d.ly[0].Kp;
    for (int e = tid; e < kPolRows * Kp0; e += blockDim.x) {
        const int rr = e / Kp0, k = e - rr * Kp0, n = row0 + rr;
        float x = 0.0f;
        if (k < O && n < R) {
            const float raw = obs[(size_t)n * O + k];
            if (obs_out) obs_out[(size_t)n * O + k] = raw;
            x = raw;
            if (om) {
                const float mean = (float)om[k], var = (float)ov[k];
                x = (raw - mean) / sqrtf(var + eps);
                x = fminf(fmaxf(x, -5.0f), 5.0f);
            }
        }
        X0[rr * d.xs + k] = x;
    }
    __syncthreads();
    float* X = X0;
    float* Y = X1;
    for (int l = 0; l < d.L; ++l) {
        const bool head = l == d.L - 1;
        pol_layer(d.ly[l], packed, X, Y, d.xs, !head, wave, lane);
        __syncthreads();
        float* tmp = X; X = Y; Y = tmp;
    }
    // X: head outputs [16][Np]: mu in columns 0..A-1, the normalised value in column A
    const int nb = (A + 3) >> 2;
    if (act) {   // Gaussian noise of k_sample_gauss: Philox block q of row n -> normals 4q .. 4q+3
        const uint64_t counter = (cbase ? (uint64_t)cbase[0] : 0ull) + coff;
        for (int e = tid; e < kPolRows * nb; e += blockDim.x) {
            const int rr = e / nb, q = e - rr * nb, n = row0 + rr;
            if (n >= R) continue;
            float z[4];
            normal4(seed, counter, (uint32_t)n, (uint32_t)q, z);
#pragma unroll
            for (int k = 0; k < 4; ++k) Z[rr * 64 + 4 * q + k] = z[k];
        }
    }
    __syncthreads();
    // element-wise outputs: mu, sigma = exp(logstd), action = mu + sigma z
    for (int e = tid; e < kPolRows * A; e += blockDim.x) {
        const int rr = e / A, jj = e - rr * A, n = row0 + rr;
        if (n >= R) continue;
        const float m = X[rr * d.xs + jj];
        const float sg = expf(logstd[jj]);
        if (mu_out) mu_out[(size_t)n * A + jj] = m;
        if (sg_out) sg_out[(size_t)n * A + jj] = sg;
        if (act) {
            const float a = m + sg * Z[rr * 64 + jj];
            act[(size_t)n * A + jj] = a;
            if (env_act) {   // rl_games preprocess_actions: clamp to +-1, rescale to [low, high]
                const float ac = fminf(fmaxf(a, -1.0f), 1.0f);
                env_act[(size_t)n * A + jj] = alo[jj] + (ac + 1.0f) * 0.5f * (ahi[jj] - alo[jj]);
            }
        }
    }
    // per row: value (un-normalised: sqrt(var + eps) * clamp(v, +-5) + mean) and neglogp in
    // k_sample_gauss's order
    if (tid < kPolRows) {
        const int n = row0 + tid;
        if (n < R) {
            float v = X[tid * d.xs + A];
            if (vm) {
                const float mean = (float)vm[0], var = (float)vv[0];
                v = sqrtf(var + eps) * fminf(fmaxf(v, -5.0f), 5.0f) + mean;
            }
            if (val) val[n] = v;
            if (act && nlp) {
                float sq = 0.0f, lsum = 0.0f;
                for (int jj = 0; jj < A; ++jj) {
                    const float m = X[tid * d.xs + jj];
                    const float ls = logstd[jj];
                    const float sg = expf(ls);
                    const float a = m + sg * Z[tid * 64 + jj];
                    const float dd = (a - m) / sg;
                    sq += dd * dd;
                    lsum += ls;
                }
                nlp[n] = 0.5f * sq + 0.918938533204672742f * (float)A + lsum;
            }
        }
    }
}
}  // namespace

// ---------------------------------------------------------------------------------------
// Rollout bookkeeping after env.step (rl_games a2c_common play_steps): shaped rewards into the
// experience buffer, the next obs / dones, the running episode reward / length meters and the
// per-step sums of finished episodes — ~20 small torch kernels per step, here one launch.
// The episode sums reduce deterministically: per-block partials in fixed order, the last block
// to finish (ticket counter, reset by that block for the next launch / graph replay) adds them
// in block order.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int kRecBlock = 256;

// blocks [0, nb_env) own 256 envs each (per-env updates + the episode-sum partials); every
// block also copies a grid-stride share of the obs rows as float4s (the copy is the bulk: 1.4 MB
// for Humanoid; on 16 blocks alone it took ~27 us)
__global__ __launch_bounds__(kRecBlock) void k_record_step(
    const float* __restrict__ obs_in, int O, const float* __restrict__ rew_in,
    const int64_t* __restrict__ done_in, int N, float scale, float* __restrict__ obs_state,
    float* __restrict__ rew_out, float* __restrict__ done_state, float* __restrict__ cur_rew,
    float* __restrict__ cur_len, double* __restrict__ sums, double* __restrict__ partial,
    unsigned* __restrict__ ticket, int nb_env, int vec4) {
#pragma clang fp contract(off)
    __shared__ double red[3][kRecBlock];
    __shared__ bool last;
    const int tid = threadIdx.x;
    const size_t total = (size_t)N * O;
    if (vec4) {
        const size_t n4 = total >> 2;
        const float4* src = (const float4*)obs_in;
        float4* dst = (float4*)obs_state;
        for (size_t e = (size_t)blockIdx.x * kRecBlock + tid; e < n4; e += (size_t)gridDim.x * kRecBlock)
            dst[e] = src[e];
    } else {
        for (size_t e = (size_t)blockIdx.x * kRecBlock + tid; e < total; e += (size_t)gridDim.x * kRecBlock)
            obs_state[e] = obs_in[e];
    }
    if ((int)blockIdx.x >= nb_env) return;           // copy-only block
    const int n = blockIdx.x * kRecBlock + tid;
    double c = 0.0, rs = 0.0, ls = 0.0;
    if (n < N) {
        const float r = rew_in[n];
        rew_out[n] = r * scale;
        const float d = (float)done_in[n];
        done_state[n] = d;
        const float cr = cur_rew[n] + r, cl = cur_len[n] + 1.0f;
        c = (double)d;
        rs = (double)cr * (double)d;
        ls = (double)cl * (double)d;
        cur_rew[n] = cr * (1.0f - d);
        cur_len[n] = cl * (1.0f - d);
    }
    red[0][tid] = c; red[1][tid] = rs; red[2][tid] = ls;
    __syncthreads();
    for (int w = kRecBlock / 2; w > 0; w >>= 1) {
        if (tid < w)
            for (int k = 0; k < 3; ++k) red[k][tid] += red[k][tid + w];
        __syncthreads();
    }
    if (tid == 0) {
        for (int k = 0; k < 3; ++k) partial[(size_t)blockIdx.x * 3 + k] = red[k][0];
        __threadfence();
        last = atomicAdd(ticket, 1u) == (unsigned)nb_env - 1;
    }
    __syncthreads();
    if (last && tid < 3) {
        __threadfence();
        double t = 0.0;
        for (int b = 0; b < nb_env; ++b) t += ((volatile double*)partial)[(size_t)b * 3 + tid];
        sums[tid] = t;
        if (tid == 0) *ticket = 0u;
    }
}
}  // namespace

// ---------------------------------------------------------------------------------------
// The learner's optimizer step (include/mi_rl.h mi_rl_adam_step): GradScaler.unscale_ +
// clip_grad_norm_ + Adam + GradScaler.update + the adaptive LR over the flat parameter buffer.
// Pass 1 reduces the squared unscaled gradient (f64 per block, blocks added in order by the
// last one, which leaves coef / found_inf / inv_scale in the scratch tail); pass 2 applies Adam
// and its last block updates step, scale, growth tracker and LR after every block has read them.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int kAdamBlock = 256, kAdamMaxBlocks = 1024;

__device__ double block_sum_f64(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k];
    return t;   // valid on thread 0
}

__global__ __launch_bounds__(kAdamBlock) void k_adam_norm(const float* __restrict__ g, int64_t n,
                                                          const float* __restrict__ scale,
                                                          float max_norm, float f16_overflow, int64_t f16_begin,
                                                          double* __restrict__ scratch,
                                                          uint32_t* __restrict__ ticket) {
    __shared__ double red[kAdamBlock / 64];
    __shared__ bool last;
    // torch's unscale_: inv_scale = 1 / scale in f64, rounded to f32
    const float inv = scale ? (float)(1.0 / (double)*scale) : 1.0f;
    double acc = 0.0;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i], x = gi * inv;
        const bool b = !isfinite(x) || (f16_overflow > 0.0f && i >= f16_begin && fabsf(gi) >= f16_overflow);
        if (b && scale) atomicMin(ticket + 3, (uint32_t)(i < 0xFFFFFFFFll ? i : 0xFFFFFFFEll));
        bad |= b;
        acc += (double)x * (double)x;
    }
    const int anybad = __syncthreads_or(bad);
    const double t = block_sum_f64(acc, red);
    if (threadIdx.x == 0) {
        scratch[blockIdx.x] = anybad ? __builtin_nan("") : t;
        __threadfence();
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the last block adds the partials: each thread a fixed strided share, then the block tree
    // (a fixed order: deterministic; one thread walking them serially took ~20 us)
    __threadfence();
    double part = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) part += ((volatile double*)scratch)[b];
    __syncthreads();   // red[] is reused
    const double tot_all = block_sum_f64(part, red);
    if (threadIdx.x == 0) {
        const double tot = tot_all;
        // found_inf is GradScaler's: without a scaler torch steps whatever the gradients hold
        const bool found = scale && !isfinite(tot);
        // clip_grad_norm_: total norm in f32, coef = max_norm / (norm + 1e-6) clamped to 1
        const float norm = (float)sqrt(tot);
        const float coef = max_norm > 0.0f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
        scratch[kAdamMaxBlocks + 0] = coef;
        scratch[kAdamMaxBlocks + 1] = found ? 1.0 : 0.0;
        scratch[kAdamMaxBlocks + 2] = inv;
        scratch[kAdamMaxBlocks + 3] = norm;
        if (found) {   // skipped-step statistics: count, first offending index of the latest
            ticket[1] += 1u;
            ticket[2] = ticket[3];
        }
        ticket[3] = 0xFFFFFFFFu;
        *ticket = 0u;
    }
}

__global__ __launch_bounds__(kAdamBlock) void k_adam_apply(mi_rl_adam_cfg c, float* __restrict__ p,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           int64_t n, float* __restrict__ step,
                                                           float* __restrict__ lr, float* __restrict__ scale,
                                                           int32_t* __restrict__ tracker,
                                                           const float* __restrict__ kl,
                                                           const double* __restrict__ scratch,
                                                           uint32_t* __restrict__ ticket) {
    __shared__ bool last;
    const bool found = scratch[kAdamMaxBlocks + 1] != 0.0;
    const float s_old = *step;
    if (!found) {
        const float coef = (float)scratch[kAdamMaxBlocks + 0], inv = (float)scratch[kAdamMaxBlocks + 2];
        const float t = s_old + 1.0f;
        const float bc1 = 1.0f - powf(c.beta1, t), bc2 = 1.0f - powf(c.beta2, t);
        const float step_size = *lr / bc1, bc2s = sqrtf(bc2);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            float gi = (g[i] * inv) * coef;          // unscale_, then the clip's multiply
            float pi = p[i];
            if (c.weight_decay != 0.0f) gi = gi + c.weight_decay * pi;
            const float mi = c.beta1 * m[i] + (1.0f - c.beta1) * gi;
            const float vi = c.beta2 * v[i] + (1.0f - c.beta2) * gi * gi;
            const float denom = sqrtf(vi) / bc2s + c.eps;
            pi = pi - step_size * mi / denom;
            m[i] = mi;
            v[i] = vi;
            p[i] = pi;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        if (!found) *step = s_old + 1.0f;
        if (scale) {   // GradScaler.update (torch._amp_update_scale_)
            if (found) {
                *scale = *scale * c.backoff_factor;
                *tracker = 0;
            } else {
                const int32_t tr = *tracker + 1;
                if (tr == c.growth_interval) {
                    const float grown = *scale * c.growth_factor;
                    if (isfinite(grown)) *scale = grown;
                    *tracker = 0;
                } else {
                    *tracker = tr;
                }
            }
        }
        if (c.adaptive_lr && kl) {   // a2c_continuous _lr_update_device (legacy AdaptiveScheduler)
            const float k = *kl, l0 = *lr;
            const float down = fmaxf(l0 / 1.5f, c.min_lr);
            const float l1 = k > 2.0f * c.kl_threshold ? down : l0;
            const float up = fminf(l1 * 1.5f, c.max_lr);
            *lr = k < 0.5f * c.kl_threshold ? up : l1;
        }
        *ticket = 0u;
    }
}
}  // namespace

// ---------------------------------------------------------------------------------------
// Training minibatch MLP on fp16 MFMA (v_mfma_f32_16x16x32_f16): the forward and the dgrad chain
// of the PPO update's network (rl_games calc_gradients under autocast fp16; HumanoidPPO.yaml
// mixed_precision: True, units [400, 200, 100], elu), each ONE launch for the whole minibatch.
//
// Transposed products, activations in registers. A wave owns 16 minibatch rows and computes
// D = W . X^T (out features x its 16 rows): the A operand is the weight (packed per minibatch
// from the f32 masters by mi_rl_mlp_train_pack), the B operand the previous layer's output.
// D register i of lane l is feature 16 t + 4 (l >> 4) + i of row l & 15, i.e. the layer's output
// already sits in the lanes the next product's B operand needs, so the layers chain with no LDS
// round trip: one 32-k step of the next product takes tiles 2 s and 2 s + 1, element j of lane
// group h being feature 16 (j >> 2) + 4 h + (j & 3) of the step (mlp_perm); the weights are
// packed in the SAME permuted k order, so every product pairs equal k. Each k-step's weight
// chunk (T tiles x 1 KB) is staged through LDS by the workgroup's 4 waves (64 rows), double
// buffered, the next chunk's global loads in flight during the current chunk's MFMAs.
//
// Numerics follow torch autocast: f16 operands, f32 accumulation; a linear's bias is added to the
// f32 accumulator and the sum rounded once to f16; ELU is evaluated in f32 on the f16 value and
// rounded to f16. Backward: dA = f16(G . W) (f32 accumulation), times the ELU derivative from the
// stored activation h (1 for h > 0, else h + 1 = exp(z)), rounded once to f16.
// ---------------------------------------------------------------------------------------
namespace {
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float mf4 __attribute__((ext_vector_type(4)));

// row stride (halfs) of a stored layer input [rows][N + 1 (ones column)]: padded to 8 halfs, so
// a lane's 4 consecutive features (D registers 0..3) are one aligned 8-byte access
__host__ __device__ constexpr int mlp_act_ld(int N) { return (N + 1 + 7) & ~7; }

constexpr int kMlpRows = 64;             // rows per workgroup: 4 waves x 16
constexpr int kMlpChunk = 512;           // halfs per 16-row tile and 32-k step (64 lanes x 8)

__host__ __device__ constexpr int mlp_perm(int h, int j) { return 16 * (j >> 2) + 4 * h + (j & 3); }

template <int O_, int H1_, int H2_, int H3_, int A_>
struct MlpShape {
    static constexpr int O = O_, H1 = H1_, H2 = H2_, H3 = H3_, A = A_, NH = A_ + 1;
    static constexpr int KS0 = (O + 31) / 32;                  // k-steps of the input
    static constexpr int T1 = 2 * ((H1 + 31) / 32), T2 = 2 * ((H2 + 31) / 32), T3 = 2 * ((H3 + 31) / 32);
    static constexpr int TH = (NH + 15) / 16;                  // head tiles (mu rows, value row)
    static_assert(NH <= 32, "heads: one 32-k step in the backward");
    // packed sections (halfs), in this order
    static constexpr long long F1 = 0;
    static constexpr long long F2 = F1 + (long long)KS0 * T1 * kMlpChunk;
    static constexpr long long F3 = F2 + (long long)(T1 / 2) * T2 * kMlpChunk;
    static constexpr long long FH = F3 + (long long)(T2 / 2) * T3 * kMlpChunk;
    static constexpr long long BH = FH + (long long)(T3 / 2) * TH * kMlpChunk;   // heads^T, 1 k-step
    static constexpr long long B3 = BH + (long long)T3 * kMlpChunk;
    static constexpr long long B2 = B3 + (long long)(T3 / 2) * T2 * kMlpChunk;
    static constexpr long long BIAS = B2 + (long long)(T2 / 2) * T1 * kMlpChunk;
    static constexpr long long TOTAL = BIAS + 16LL * (T1 + T2 + T3 + TH);
    static constexpr int LDS = 2 * T1 * kMlpChunk * 2;         // bytes: two chunks of the widest layer
};
using MlpHumanoid = MlpShape<87, 400, 200, 100, 21>;   // cfg/train/HumanoidPPO.yaml:24-25
using MlpAnt = MlpShape<60, 256, 128, 64, 8>;          // cfg/train/AntPPO.yaml

int mlp_shape_id(const mi_rl_mlp* m) {
    if (!m || m->num_hidden != 3) return 0;
    auto is = [&](int o, int a, int b, int c, int na) {
        return m->num_obs == o && m->units[0] == a && m->units[1] == b && m->units[2] == c && m->num_actions == na;
    };
    if (is(87, 400, 200, 100, 21)) return 1;
    if (is(60, 256, 128, 64, 8)) return 2;
    return 0;
}

// One packed element: section, k-step s, tile t, lane l, element j. Forward sections pack W
// [out][in] as the A operand (row 16 t + (l & 15), k 32 s + perm); backward ones W^T (row = in
// feature 16 t + (l & 15), k = out feature 32 s + perm); the head is the mu rows then the value
// row. Zero padding everywhere else.
template <class S>
__global__ void k_mlp_train_pack(mi_rl_mlp m, _Float16* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S::TOTAL) return;
    const int in_dim[4] = {S::O, S::H1, S::H2, S::H3};
    const int out_dim[4] = {S::H1, S::H2, S::H3, S::NH};
    auto W = [&](int layer, int n, int k) -> float {
        if (n >= out_dim[layer] || k >= in_dim[layer]) return 0.0f;
        if (layer < 3) return m.w[layer][(size_t)n * in_dim[layer] + k];
        return n < S::A ? m.w[3][(size_t)n * in_dim[3] + k] : m.w[4][k];
    };
    float v = 0.0f;
    if (i < S::BIAS) {
        long long o;
        int layer, T;
        bool fwd = true;
        if (i < S::F2) { o = i - S::F1; layer = 0; T = S::T1; }
        else if (i < S::F3) { o = i - S::F2; layer = 1; T = S::T2; }
        else if (i < S::FH) { o = i - S::F3; layer = 2; T = S::T3; }
        else if (i < S::BH) { o = i - S::FH; layer = 3; T = S::TH; }
        else if (i < S::B3) { o = i - S::BH; layer = 3; T = S::T3; fwd = false; }
        else if (i < S::B2) { o = i - S::B3; layer = 2; T = S::T2; fwd = false; }
        else { o = i - S::B2; layer = 1; T = S::T1; fwd = false; }
        const int j = (int)(o & 7), l = (int)((o >> 3) & 63);
        const long long st = o >> 9;                 // k-step major, then tile
        const int t = (int)(st % T), s = (int)(st / T);
        const int r = 16 * t + (l & 15), k = 32 * s + mlp_perm(l >> 4, j);
        v = fwd ? W(layer, r, k) : W(layer, k, r);
    } else {
        long long o = i - S::BIAS;
        const int lens[4] = {16 * S::T1, 16 * S::T2, 16 * S::T3, 16 * S::TH};
        int layer = 0;
        while (layer < 3 && o >= lens[layer]) { o -= lens[layer]; ++layer; }
        const int n = (int)o;
        if (n < out_dim[layer]) v = layer < 3 ? m.b[layer][n] : (n < S::A ? m.b[3][n] : m.b[4][0]);
    }
    out[i] = (_Float16)v;
}

// this wave's accumulators of one product: acc[t] = sum_s A(s, t) . B[s]; the workgroup stages
// each k-step's weight chunk (T tiles) into LDS (double buffer, 2 x T x 1 KB)
template <int T, int KS, int TT = T>
__device__ __forceinline__ void mlp_mm(const _Float16* __restrict__ Ap, const h8 (&B)[KS], mf4 (&acc)[T],
                                       _Float16* lds, int tid, int lane) {
    // tiles [T0, T0 + T) of a product with TT tiles per k-step chunk: Ap points at tile T0 of
    // chunk 0, the k-steps are TT x 1 KB apart
    constexpr int CH = T * kMlpChunk;                 // halfs per (partial) chunk staged
    constexpr int PER = (CH / 8 + 255) / 256;         // 16-B pieces per thread
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = mf4{0.0f, 0.0f, 0.0f, 0.0f};
    h8 stg[PER];
    __syncthreads();                                  // the previous product's readers are done
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int o = (tid + 256 * q) * 8;
        if (o < CH) stg[q] = *(const h8*)(Ap + o);
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int o = (tid + 256 * q) * 8;
        if (o < CH) *(h8*)(lds + o) = stg[q];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const _Float16* cur = lds + (s & 1) * CH;
        _Float16* nxt = lds + ((s + 1) & 1) * CH;
        if (s + 1 < KS) {   // the next chunk's global loads in flight during this chunk's MFMAs
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int o = (tid + 256 * q) * 8;
                if (o < CH) stg[q] = *(const h8*)(Ap + (size_t)(s + 1) * TT * kMlpChunk + o);
            }
        }
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const h8 a = *(const h8*)(cur + t * kMlpChunk + lane * 8);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, B[s], acc[t], 0, 0, 0);
        }
        if (s + 1 < KS) {
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int o = (tid + 256 * q) * 8;
                if (o < CH) *(h8*)(nxt + o) = stg[q];
            }
            __syncthreads();
        }
    }
}

// ELU without branches (rounded to f16 by the caller): v > 0: v; otherwise expm1(v), as a degree-6
// Taylor polynomial for |v| < 1/4 (truncation < 2e-6 relative) and exp(v) - 1 by v_exp_f32 below
// (no cancellation there: exp(v) <= 0.78). Both are far inside the f16 rounding of the result;
// libm's expm1f branched per element (the epilogue's 180 divergent sections per wave).
__device__ __forceinline__ float mlp_elu(float v) {
    const float p = v * (1.0f + v * (0.5f + v * (1.0f / 6.0f + v * (1.0f / 24.0f + v * (1.0f / 120.0f + v * (1.0f / 720.0f))))));
    const float e = __builtin_amdgcn_exp2f(v * 1.44269504088896341f) - 1.0f;
    const float m = v > -0.25f ? p : e;
    return v > 0.0f ? v : m;
}

// hidden-layer epilogue (forward): y = f16(elu(f16(acc + b))) stored to act [rows][N + 1] (the ones
// column at N: the bias column of the split-K weight gradient), and the next product's B
// fragments (features >= N are 0)
template <int T, int N, int T0 = 0, int BN = T / 2>
__device__ __forceinline__ void mlp_fwd_epi(const mf4 (&acc)[T], const _Float16* __restrict__ bias,
                                            _Float16* __restrict__ act, int row, bool live, int lane,
                                            h8 (&Bn)[BN]) {
    // acc holds tiles T0 .. T0 + T - 1 of the layer (T0 > 0: the second half of a split layer)
    static_assert(N % 4 == 0, "whole groups of 4 features");
    constexpr int LD = mlp_act_ld(N);
    const int h = lane >> 4;
#pragma unroll
    for (int tl = 0; tl < T; ++tl) {
        const int t = T0 + tl;
        const int f0 = 16 * t + 4 * h;
        const bool in = 16 * (t + 1) <= N || f0 < N;   // compile-time true below the last tile
        const h4 b4 = *(const h4*)(bias + f0);          // (the padded bias is 0 past N)
        h4 y4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const _Float16 z = (_Float16)(acc[tl][i] + (float)b4[i]);
            const _Float16 y = (_Float16)mlp_elu((float)z);
            y4[i] = in ? y : (_Float16)0.0f;
            Bn[t >> 1][4 * (t & 1) + i] = y4[i];
        }
        if (live && in) *(h4*)(act + (size_t)row * LD + f0) = y4;
    }
    if (T0 == 0 && live && h == 0) act[(size_t)row * LD + N] = (_Float16)1.0f;   // the ones column
}

template <class S>
__global__ __launch_bounds__(256) void k_mlp_train_fwd(const _Float16* __restrict__ pk, const float* __restrict__ x,
                                                       int rows, _Float16* __restrict__ xa, _Float16* __restrict__ h1a,
                                                       _Float16* __restrict__ h2a, _Float16* __restrict__ h3a,
                                                       _Float16* __restrict__ mu, _Float16* __restrict__ val) {
    extern __shared__ __attribute__((aligned(16))) _Float16 mlp_lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 4;
    const int row = blockIdx.x * kMlpRows + wave * 16 + (lane & 15);
    const bool live = row < rows;
    // the input: f32 -> f16 (autocast's cast) B fragments, and [x | 1] f16 for layer 1's weight
    // gradient (each (row, k) lies in exactly one lane's fragment)
    h8 B0[S::KS0];
#pragma unroll
    for (int s = 0; s < S::KS0; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 32 * s + mlp_perm(h, j);
            const float v = (live && k < S::O) ? x[(size_t)row * S::O + k] : 0.0f;
            const _Float16 hv = (_Float16)v;
            B0[s][j] = hv;
            if (live && k < S::O) xa[(size_t)row * mlp_act_ld(S::O) + k] = hv;
        }
    }
    if (live && h == 0) xa[(size_t)row * mlp_act_ld(S::O) + S::O] = (_Float16)1.0f;   // the ones column
    const _Float16* bias = pk + S::BIAS;
    h8 B1[S::T1 / 2];
    {   // the widest layer in two halves of its output tiles (half the accumulators live at once)
        constexpr int HA = S::T1 / 2, HB = S::T1 - HA;
        {
            mf4 acc[HA];
            mlp_mm<HA, S::KS0, S::T1>(pk + S::F1, B0, acc, mlp_lds, tid, lane);
            mlp_fwd_epi<HA, S::H1, 0, S::T1 / 2>(acc, bias, h1a, row, live, lane, B1);
        }
        mf4 acc[HB];
        mlp_mm<HB, S::KS0, S::T1>(pk + S::F1 + HA * kMlpChunk, B0, acc, mlp_lds, tid, lane);
        mlp_fwd_epi<HB, S::H1, HA, S::T1 / 2>(acc, bias, h1a, row, live, lane, B1);
    }
    h8 B2[S::T2 / 2];
    {
        mf4 acc[S::T2];
        mlp_mm<S::T2, S::T1 / 2>(pk + S::F2, B1, acc, mlp_lds, tid, lane);
        mlp_fwd_epi<S::T2, S::H2>(acc, bias + 16 * S::T1, h2a, row, live, lane, B2);
    }
    h8 B3[S::T3 / 2];
    {
        mf4 acc[S::T3];
        mlp_mm<S::T3, S::T2 / 2>(pk + S::F3, B2, acc, mlp_lds, tid, lane);
        mlp_fwd_epi<S::T3, S::H3>(acc, bias + 16 * (S::T1 + S::T2), h3a, row, live, lane, B3);
    }
    mf4 acc[S::TH];
    mlp_mm<S::TH, S::T3 / 2>(pk + S::FH, B3, acc, mlp_lds, tid, lane);
    const _Float16* bh = bias + 16 * (S::T1 + S::T2 + S::T3);
#pragma unroll
    for (int t = 0; t < S::TH; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = 16 * t + 4 * h + i;
            const _Float16 z = (_Float16)(acc[t][i] + (float)bh[f]);
            if (live) {
                if (f < S::A) mu[(size_t)row * S::A + f] = z;
                else if (f == S::A) val[row] = z;
            }
        }
    }
}

// backward epilogue: g = f16(f16(acc) * elu'(h)), h the stored activation of this layer
// (act [rows][N + 1]); stored to g [rows][N] and, when chaining on, the next product's B
template <int T, int N, bool NEXT, int T0 = 0, int BN = T / 2 + 1>
__device__ __forceinline__ void mlp_bwd_epi(const mf4 (&acc)[T], const _Float16* __restrict__ act,
                                            _Float16* __restrict__ g, int row, bool live, int lane,
                                            h8 (&Bn)[BN]) {
    static_assert(N % 4 == 0, "whole groups of 4 features");
    constexpr int LD = mlp_act_ld(N);
    const int h = lane >> 4;
#pragma unroll
    for (int tl = 0; tl < T; ++tl) {
        const int t = T0 + tl;
        const int f0 = 16 * t + 4 * h;
        h4 g4 = {(_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f};
        if (live && (16 * (t + 1) <= N || f0 < N)) {   // the second test only in the last tile
            const h4 a4 = *(const h4*)(act + (size_t)row * LD + f0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float hv = (float)a4[i];
                const float d = (float)(_Float16)acc[tl][i];
                g4[i] = (_Float16)(d * (hv > 0.0f ? 1.0f : hv + 1.0f));
            }
            *(h4*)(g + (size_t)row * N + f0) = g4;
        }
        if constexpr (NEXT) {
#pragma unroll
            for (int i = 0; i < 4; ++i) Bn[t >> 1][4 * (t & 1) + i] = g4[i];
        }
    }
}

template <class S>
__global__ __launch_bounds__(256) void k_mlp_train_bwd(const _Float16* __restrict__ pk, int rows,
                                                       const _Float16* __restrict__ h1a,
                                                       const _Float16* __restrict__ h2a,
                                                       const _Float16* __restrict__ h3a,
                                                       const _Float16* __restrict__ gmu,
                                                       const _Float16* __restrict__ gval,
                                                       _Float16* __restrict__ g1, _Float16* __restrict__ g2,
                                                       _Float16* __restrict__ g3) {
    extern __shared__ __attribute__((aligned(16))) _Float16 mlp_lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 4;
    const int row = blockIdx.x * kMlpRows + wave * 16 + (lane & 15);
    const bool live = row < rows;
    // the heads' gradient [gmu | gval] as the B fragment of one 32-k step
    h8 BH[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = mlp_perm(h, j);
        _Float16 v = (_Float16)0.0f;
        if (live) {
            if (k < S::A) v = gmu[(size_t)row * S::A + k];
            else if (k == S::A) v = gval[row];
        }
        BH[0][j] = v;
    }
    h8 B3[S::T3 / 2];
    {
        mf4 acc[S::T3];
        mlp_mm<S::T3, 1>(pk + S::BH, BH, acc, mlp_lds, tid, lane);
        mlp_bwd_epi<S::T3, S::H3, true, 0, S::T3 / 2>(acc, h3a, g3, row, live, lane, B3);
    }
    h8 B2[S::T2 / 2];
    {
        mf4 acc[S::T2];
        mlp_mm<S::T2, S::T3 / 2>(pk + S::B3, B3, acc, mlp_lds, tid, lane);
        mlp_bwd_epi<S::T2, S::H2, true, 0, S::T2 / 2>(acc, h2a, g2, row, live, lane, B2);
    }
    // the widest product in two halves of its output tiles
    constexpr int HA = S::T1 / 2, HB = S::T1 - HA;
    h8 none[1];
    {
        mf4 acc[HA];
        mlp_mm<HA, S::T2 / 2, S::T1>(pk + S::B2, B2, acc, mlp_lds, tid, lane);
        mlp_bwd_epi<HA, S::H1, false, 0, 1>(acc, h1a, g1, row, live, lane, none);
    }
    mf4 acc[HB];
    mlp_mm<HB, S::T2 / 2, S::T1>(pk + S::B2 + HA * kMlpChunk, B2, acc, mlp_lds, tid, lane);
    mlp_bwd_epi<HB, S::H1, false, HA, 1>(acc, h1a, g1, row, live, lane, none);
}

template <class S>
int mlp_train_fwd_launch(const _Float16* pk, const float* x, int rows, void* const* acts, void* mu, void* val,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_mlp_train_fwd<S>, dim3((rows + kMlpRows - 1) / kMlpRows), dim3(256), S::LDS, st, pk, x,
                       rows, (_Float16*)acts[0], (_Float16*)acts[1], (_Float16*)acts[2], (_Float16*)acts[3],
                       (_Float16*)mu, (_Float16*)val);
    return launch_check("mi_rl_mlp_train_fwd");
}

template <class S>
int mlp_train_bwd_launch(const _Float16* pk, int rows, void* const* acts, const void* gmu, const void* gval,
                         void* const* grads, hipStream_t st) {
    hipLaunchKernelGGL(k_mlp_train_bwd<S>, dim3((rows + kMlpRows - 1) / kMlpRows), dim3(256), S::LDS, st, pk, rows,
                       (const _Float16*)acts[1], (const _Float16*)acts[2], (const _Float16*)acts[3],
                       (const _Float16*)gmu, (const _Float16*)gval, (_Float16*)grads[0], (_Float16*)grads[1],
                       (_Float16*)grads[2]);
    return launch_check("mi_rl_mlp_train_bwd");
}
}  // namespace

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

int64_t mi_rl_mlp_packed_size(const mi_rl_mlp* mlp) {
    PolDesc d;
    if (pol_desc(mlp, &d)) return -1;
    return d.total;
}

int32_t mi_rl_mlp_pack(const mi_rl_mlp* mlp, float* packed, void* stream) {
    PolDesc d;
    if (int rc = pol_desc(mlp, &d)) return rc;
    if (!packed) return fail(kNull, "mi_rl_mlp_pack: null packed buffer");
    for (int l = 0; l < mlp->num_hidden + 2; ++l)
        if (!mlp->w[l] || !mlp->b[l]) return fail(kNull, "mi_rl_mlp_pack: null weight / bias of layer %d", l);
    hipLaunchKernelGGL(k_pol_pack, dim3((unsigned)((d.total + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, d, *mlp, packed);
    return launch_check("mi_rl_mlp_pack");
}

int32_t mi_rl_policy_step(const mi_rl_mlp* mlp, const float* packed, const float* obs,
                          int32_t num_rows, const double* obs_mean, const double* obs_var,
                          const double* value_mean, const double* value_var, float eps,
                          const float* logstd, uint64_t seed, const int64_t* counter_base,
                          uint64_t counter_offset, float* obs_out, float* actions, float* neglogp,
                          float* values, float* mu_out, float* sigma_out, const float* action_low,
                          const float* action_high, float* env_actions, void* stream) {
    PolDesc d;
    if (int rc = pol_desc(mlp, &d)) return rc;
    if (!packed || !obs || !logstd) return fail(kNull, "mi_rl_policy_step: null packed / obs / logstd");
    if ((obs_mean == nullptr) != (obs_var == nullptr) || (value_mean == nullptr) != (value_var == nullptr))
        return fail(kNull, "mi_rl_policy_step: mean and var come in pairs");
    if (num_rows <= 0) return fail(kShape, "mi_rl_policy_step: R=%d", num_rows);
    if ((neglogp || env_actions) && !actions) return fail(kNull, "mi_rl_policy_step: neglogp / env_actions need actions");
    if (env_actions && (!action_low || !action_high)) return fail(kNull, "mi_rl_policy_step: env_actions need the action bounds");
    const size_t lds = pol_lds_bytes(d);   // <= kPolMaxLds (pol_desc)
    hipLaunchKernelGGL(k_policy_step, dim3((num_rows + kPolRows - 1) / kPolRows), dim3(64 * kPolWaves),
                       lds, (hipStream_t)stream, d, packed, obs, num_rows, obs_mean, obs_var,
                       value_mean, value_var, eps, logstd, seed, counter_base, counter_offset,
                       obs_out, actions, neglogp, values, mu_out, sigma_out, action_low, action_high,
                       env_actions);
    return launch_check("mi_rl_policy_step");
}

int32_t mi_rl_record_step(const float* obs_in, int32_t num_obs, const float* rewards,
                          const int64_t* dones, int32_t num_envs, float reward_scale,
                          float* obs_state, float* rewards_out, float* dones_state,
                          float* cur_rewards, float* cur_lengths, double* episode_sums,
                          double* scratch, uint32_t* ticket, void* stream) {
    if (!obs_in || !rewards || !dones || !obs_state || !rewards_out || !dones_state || !cur_rewards ||
        !cur_lengths || !episode_sums || !scratch || !ticket)
        return fail(kNull, "mi_rl_record_step: null buffer");
    if (num_envs <= 0 || num_obs <= 0) return fail(kShape, "mi_rl_record_step: N=%d O=%d", num_envs, num_obs);
    const int nb_env = (num_envs + kRecBlock - 1) / kRecBlock;
    const size_t total = (size_t)num_envs * num_obs;
    const int vec4 = (total % 4 == 0) && ((uintptr_t)obs_in % 16 == 0) && ((uintptr_t)obs_state % 16 == 0);
    // enough blocks that the obs copy has ~8 float4s per thread
    const size_t per = (size_t)kRecBlock * (vec4 ? 32 : 8);
    int nb = (int)((total + per - 1) / per);
    nb = nb < nb_env ? nb_env : (nb > 1024 ? 1024 : nb);
    hipLaunchKernelGGL(k_record_step, dim3(nb), dim3(kRecBlock), 0, (hipStream_t)stream, obs_in, num_obs,
                       rewards, dones, num_envs, reward_scale, obs_state, rewards_out, dones_state,
                       cur_rewards, cur_lengths, episode_sums, scratch, ticket, nb_env, vec4);
    return launch_check("mi_rl_record_step");
}

int32_t mi_rl_adam_step(const mi_rl_adam_cfg* cfg, float* params, const float* grads, float* exp_avg,
                        float* exp_avg_sq, int64_t n, float* step, float* lr, float* scale,
                        int32_t* growth_tracker, const float* kl, double* scratch, int64_t scratch_len,
                        uint32_t* tickets, void* stream) {
    if (!cfg || !params || !grads || !exp_avg || !exp_avg_sq || !step || !lr || !scratch || !tickets)
        return fail(kNull, "mi_rl_adam_step: null buffer");
    if (scale && !growth_tracker) return fail(kNull, "mi_rl_adam_step: scale without growth tracker");
    if (n <= 0) return fail(kShape, "mi_rl_adam_step: n=%lld", (long long)n);
    if (scratch_len < kAdamMaxBlocks + 4)
        return fail(kShape, "mi_rl_adam_step: scratch %lld < %d doubles", (long long)scratch_len, kAdamMaxBlocks + 4);
    int nb = (int)((n + kAdamBlock * 4 - 1) / (kAdamBlock * 4));
    nb = nb < 1 ? 1 : (nb > kAdamMaxBlocks ? kAdamMaxBlocks : nb);
    hipLaunchKernelGGL(k_adam_norm, dim3(nb), dim3(kAdamBlock), 0, (hipStream_t)stream, grads, n, scale,
                       cfg->max_grad_norm, scale ? cfg->f16_overflow : 0.0f, cfg->f16_begin, scratch, tickets);
    int32_t rc = launch_check("mi_rl_adam_step (norm)");
    if (rc) return rc;
    hipLaunchKernelGGL(k_adam_apply, dim3(nb), dim3(kAdamBlock), 0, (hipStream_t)stream, *cfg, params, grads,
                       exp_avg, exp_avg_sq, n, step, lr, scale, growth_tracker, kl, scratch, tickets + 4);
    return launch_check("mi_rl_adam_step (apply)");
}

int64_t mi_rl_mlp_train_packed_size(const mi_rl_mlp* mlp) {
    switch (mlp_shape_id(mlp)) {
        case 1: return MlpHumanoid::TOTAL;
        case 2: return MlpAnt::TOTAL;
        default: return -1;
    }
}

int32_t mi_rl_mlp_train_pack(const mi_rl_mlp* mlp, void* packed, void* stream) {
    const int id = mlp_shape_id(mlp);
    if (!id) return fail(kShape, "mi_rl_mlp_train_pack: unsupported network layout");
    if (!packed) return fail(kNull, "mi_rl_mlp_train_pack: null packed buffer");
    for (int l = 0; l < 5; ++l)
        if (!mlp->w[l] || !mlp->b[l]) return fail(kNull, "mi_rl_mlp_train_pack: null weight / bias of layer %d", l);
    const long long n = id == 1 ? MlpHumanoid::TOTAL : MlpAnt::TOTAL;
    const dim3 g((unsigned)((n + kBlock - 1) / kBlock));
    if (id == 1) hipLaunchKernelGGL(k_mlp_train_pack<MlpHumanoid>, g, dim3(kBlock), 0, (hipStream_t)stream, *mlp, (_Float16*)packed);
    else hipLaunchKernelGGL(k_mlp_train_pack<MlpAnt>, g, dim3(kBlock), 0, (hipStream_t)stream, *mlp, (_Float16*)packed);
    return launch_check("mi_rl_mlp_train_pack");
}

int32_t mi_rl_mlp_train_fwd(const mi_rl_mlp* mlp, const void* packed, const float* x, int32_t rows,
                            void* const* acts, void* mu, void* value, void* stream) {
    const int id = mlp_shape_id(mlp);
    if (!id) return fail(kShape, "mi_rl_mlp_train_fwd: unsupported network layout");
    if (!packed || !x || !acts || !mu || !value) return fail(kNull, "mi_rl_mlp_train_fwd: null buffer");
    for (int l = 0; l < 4; ++l)
        if (!acts[l]) return fail(kNull, "mi_rl_mlp_train_fwd: null activation buffer %d", l);
    if (rows <= 0) return fail(kShape, "mi_rl_mlp_train_fwd: rows=%d", rows);
    return id == 1 ? mlp_train_fwd_launch<MlpHumanoid>((const _Float16*)packed, x, rows, acts, mu, value, (hipStream_t)stream)
                   : mlp_train_fwd_launch<MlpAnt>((const _Float16*)packed, x, rows, acts, mu, value, (hipStream_t)stream);
}

int32_t mi_rl_mlp_train_bwd(const mi_rl_mlp* mlp, const void* packed, void* const* acts, const void* grad_mu,
                            const void* grad_value, int32_t rows, void* const* grads, void* stream) {
    const int id = mlp_shape_id(mlp);
    if (!id) return fail(kShape, "mi_rl_mlp_train_bwd: unsupported network layout");
    if (!packed || !acts || !grad_mu || !grad_value || !grads) return fail(kNull, "mi_rl_mlp_train_bwd: null buffer");
    for (int l = 1; l < 4; ++l)
        if (!acts[l] || !grads[l - 1]) return fail(kNull, "mi_rl_mlp_train_bwd: null buffer of layer %d", l);
    if (rows <= 0) return fail(kShape, "mi_rl_mlp_train_bwd: rows=%d", rows);
    return id == 1 ? mlp_train_bwd_launch<MlpHumanoid>((const _Float16*)packed, rows, acts, grad_mu, grad_value, grads, (hipStream_t)stream)
                   : mlp_train_bwd_launch<MlpAnt>((const _Float16*)packed, rows, acts, grad_mu, grad_value, grads, (hipStream_t)stream);
}

}  // extern "C"
