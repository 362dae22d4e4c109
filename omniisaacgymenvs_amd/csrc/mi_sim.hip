// mi_sim.hip — kernels + C ABI of libmi_sim.so (include/mi_sim.h), gfx950.
//
// Round-1 mapping: one lane per env, `block` lanes per workgroup (default 64 = one wave).
// The fused env step (mi_env_step) is ONE launch per VecEnvRLGames.step: mask-driven reset,
// action clamp + efforts, controlFrequencyInv physics substeps, obs / reward / done and the
// VecEnv obs clamp, with the per-env solver workspace resident in L2 / MALL between phases.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "mi_artic.hpp"
#include "mi_device.hpp"
#include "mi_task.hpp"
#include "mi_wave.hpp"
#include "mi_pair.hpp"

using namespace mi;

// ---------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(MI_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                       \
    } while (0)

#define LAUNCH_CHECK()                                                                   \
    do {                                                                                 \
        hipError_t e_ = hipGetLastError();                                               \
        if (e_ != hipSuccess) return fail(MI_E_HIP, "launch: %s", hipGetErrorString(e_)); \
    } while (0)

// ---------------------------------------------------------------------------------------
// handle
// ---------------------------------------------------------------------------------------
struct mi_sim {
    int device = 0;
    int N = 0;
    int block = 64;
    DevModel dm{};
    DevState ds{};
    SimP sp{};
    DevTask tp{};
    bool task_ok = false;
    bool wave = false;      // wavefront-per-env articulation path (mi_wave.hpp)
    bool pair = false;      // two envs per wavefront (mi_pair.hpp), 16 envs per workgroup
    int topo = 0;           // generated compile-time topology id (0: runtime tables)
    WaveTabs wt{};
    float* rows = nullptr;  // per-env global constraint-row slab of the wave path
    size_t lds_bytes = 0;
    void* kp_dev = nullptr;  // device copy of KParams (wave path)
    int num_cu = 0;          // compute units of the device (queried on first use)
    int post_kernel = -1, post_grid = 0;   // last mi_task_post_step launch (mi_task_post_kernel)
    // deferred physics substeps (mi_sim_step): World.step() twice in a row (the reference's
    // controlFrequencyInv loop, vec_env_rlgames.py:64-66) becomes ONE launch of two substeps,
    // issued by the next entry point that touches the state (flush_pending)
    bool defer = true;
    int pending = 0;
    hipStream_t pending_stream = nullptr;
    hipEvent_t pending_ev = nullptr;
    // state mirrors (mi_sim_set_mirror): row-major pos, quat, vel, q, qd, sens; valid = every
    // mirror equals the state (set by mi_get_state_mirror, cleared by every state write)
    float* mir[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool mir_valid = false;
    hipStream_t mir_stream = nullptr;   // stream of the last refresh; a reader on another stream
    hipEvent_t mir_ev = nullptr;        // waits on mir_ev (recorded after that refresh)
    hipStream_t mir_reader = nullptr;   // a stream other than the writer's that was handed the
    hipEvent_t rd_ev = nullptr;         // mirrors: the next mirror write waits for its queued reads
    std::vector<float> lower, upper;  // host copy for mi_sim_info
    std::vector<void*> allocs;
    // launch timing (mi_sim_time_launches): every tev_every-th mi_env_step launch carries a
    // start / stop event pair on its own dispatch (hipExtLaunchKernelGGL), no marker packets
    std::vector<hipEvent_t> tev;      // [2 * capacity]: start, stop of recorded launch k
    int tev_every = 0;
    long long tev_seen = 0;
    int tev_rec = 0;
};
static hipError_t timed_launch(mi_sim* s, void* stream, hipEvent_t* ev0, hipEvent_t* ev1);
static int flush_pending(mi_sim* s, void* stream);

static int dev_alloc(mi_sim* s, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    HIP_TRY(hipMalloc(p, bytes));
    s->allocs.push_back(*p);
    HIP_TRY(hipMemset(*p, 0, bytes));
    return MI_OK;
}

template <typename T>
static int upload(mi_sim* s, const T* host, size_t count, const T** out) {
    void* p = nullptr;
    int rc = dev_alloc(s, &p, count * sizeof(T));
    if (rc) return rc;
    if (count && host) HIP_TRY(hipMemcpy(p, host, count * sizeof(T), hipMemcpyHostToDevice));
    *out = (const T*)p;
    return MI_OK;
}

static inline dim3 grid_for(const mi_sim* s, int n) { return dim3((n + s->block - 1) / s->block); }

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void physics_env(const DevModel& m, const DevState& st, const SimP& p,
                                            int i, int substeps) {
    if (m.dyn == MI_DYN_CARTPOLE) {
        const int N = st.N;
        float x = st.q[sx(st, 0, i)], th = st.q[sx(st, 1, i)], xd = st.qd[sx(st, 0, i)], thd = st.qd[sx(st, 1, i)];
        const float F0 = st.eff[sx(st, 0, i)], F1 = st.eff[sx(st, 1, i)];
        for (int s = 0; s < substeps; ++s) cartpole_substep(m, p, x, th, xd, thd, F0, F1);
        st.q[sx(st, 0, i)] = x; st.q[sx(st, 1, i)] = th; st.qd[sx(st, 0, i)] = xd; st.qd[sx(st, 1, i)] = thd;
        if (!(isfinite(x) && isfinite(th) && isfinite(xd) && isfinite(thd))) st.nan_flag[i] = 1;
    } else {
        for (int s = 0; s < substeps; ++s) artic_substep(m, st, p, i);
    }
}

__global__ void k_sim_step(DevModel m, DevState st, SimP p, int substeps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    physics_env(m, st, p, i, substeps);
}

__global__ void k_pre_step(DevModel m, DevState st, DevTask tp, const float* actions,
                           int64_t* reset_buf, int64_t* progress_buf, float* pot, float* prev,
                           float* actions_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    task_pre_env(m, st, tp, i, actions, reset_buf, progress_buf, pot, prev, actions_out, false);
}

// locomotion post for one env from a row buffer R (unclamped obs row). act = actions row.
__device__ __forceinline__ void loco_post(const DevModel& m, const DevState& st, const DevTask& tp,
                                          int i, const float* act, float act_clip, float* R,
                                          float* rew, int64_t* reset_buf, int64_t* progress_buf,
                                          float* pot, float* prev) {
    const int64_t progress = progress_buf[i] + 1;                 // rl_task.py:242
    loco_obs_env(m, st, tp, i, act, act_clip, R, pot, prev);      // get_observations
    const float* ca = R + 12 + 2 * m.D + 6 * m.S;                 // task.actions (clamped)
    rew[i] = loco_reward(tp, m.D, R, ca, pot[i], prev[i]);        // calculate_metrics
    reset_buf[i] = nan_guard(st, i, loco_done(tp, R[0], reset_buf[i], progress));  // is_done
    progress_buf[i] = progress;
}

__device__ __forceinline__ void cartpole_post(const DevState& st, const DevTask& tp, int i, float* R,
                                              float* rew, int64_t* reset_buf,
                                              int64_t* progress_buf) {
    const int64_t progress = progress_buf[i] + 1;
    cartpole_obs_env(st, i, R);
    rew[i] = cartpole_reward(tp, R);
    reset_buf[i] = nan_guard(st, i, cartpole_done(tp, R, progress));
    progress_buf[i] = progress;
}

// RLTask.post_physics_step (rl_task.py:231-251) for the built-in tasks, one launch
__global__ void k_post_step(DevModel m, DevState st, DevTask tp, const float* actions, float* obs,
                            float* rew, int64_t* reset_buf, int64_t* progress_buf, float* pot,
                            float* prev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    float* R = obs + (size_t)tp.O * i;
    if (tp.kind == MI_TASK_CARTPOLE)
        cartpole_post(st, tp, i, R, rew, reset_buf, progress_buf);
    else
        loco_post(m, st, tp, i, actions + (size_t)tp.A * i, INFINITY, R, rew, reset_buf,
                  progress_buf, pot, prev);
}

// RLTask.post_physics_step for the locomotion tasks on the per-env record layout (fs = 1,
// es = record floats): TE envs per 64-lane workgroup, HBM-streaming. The block's records and
// action rows are contiguous in HBM: loaded with coalesced float4 reads into padded LDS rows;
// lanes < TE then run the same per-env task math as k_post_step (loco_obs_env / loco_reward /
// loco_done) on an LDS view of their env. STAGE: the obs rows go through an LDS tile and leave
// as coalesced float4 stores (the [N, O] rows of TE consecutive envs are one contiguous span);
// otherwise each lane stores its own row.
MI_D void tile_load(const float* __restrict__ src, int count, float* dst, int row, int pad) {
    // count floats (a multiple of row) from src into dst rows of `pad` floats
    const int lane = threadIdx.x;
    if ((((uintptr_t)src) & 15) == 0 && (row & 3) == 0) {
        const float4* s4 = (const float4*)src;
        for (int k = lane; k < count / 4; k += 64) {
            const float4 v = s4[k];
            const int f = 4 * k, e = f / row, c = f - e * row;
            float* d = dst + e * pad + c;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
    } else {
        for (int k = lane; k < count; k += 64) {
            const int e = k / row;
            dst[e * pad + (k - e * row)] = src[k];
        }
    }
}

template <int TE, bool STAGE>
__global__ __launch_bounds__(64) void k_loco_post_tiled(DevModel m, DevState st, DevTask tp,
                                                        const float* __restrict__ actions,
                                                        float* obs, float* rew, int64_t* reset_buf,
                                                        int64_t* progress_buf, float* pot,
                                                        float* prev) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x, e0 = blockIdx.x * TE;
    const int n = min(TE, st.N - e0);
    const int O = tp.O, A = tp.A;
    if (TE == 32 && STAGE) {
        // compact tile: each record's used fields only (root 13, q, qd: the float4s up to the end
        // of qd, so the efforts line is never fetched) and the env's sensor wrenches from their
        // own array; actions read in place
        const int D = m.D, S = m.S;
        const int k0 = 13 + 2 * D, ne4 = (k0 + 3) >> 2, ns = 6 * S, PC = (k0 + ns) | 1;   // odd row stride: no LDS bank aliasing across envs
        float* srec = sm;
        float* sobs = sm + TE * PC;
        float* sterm = sobs + TE * O;                          // [TE][3] sums
        {
            const float4* s4 = (const float4*)(st.root_pos + (size_t)e0 * st.es);
            for (int k = lane; k < n * ne4; k += 64) {         // es % 4 == 0 (whole lines)
                const int e = k / ne4, c4 = k - e * ne4;
                const float4 v4 = s4[e * (st.es >> 2) + c4];
                const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = 4 * c4 + q;
                    if (c < k0) srec[e * PC + c] = vv[q];
                }
            }
            for (int k = lane; k < n * ns; k += 64) {
                const int e = k / ns, c = k - e * ns;
                srec[e * PC + k0 + c] = st.sens[ssx(st, c, e0 + e)];
            }
        }
        __syncthreads();
        DevState v = st;                    // the block's envs, viewed in LDS
        v.fs = 1; v.es = PC;
        v.root_pos = srec; v.root_quat = srec + 3; v.root_vel = srec + 7;
        v.q = srec + 13; v.qd = srec + 13 + D; v.sens = srec + k0;
        v.sfs = 1; v.ses = PC;
        // split by lane halves: lanes 0..31 the root-frame block of env `lane`, lanes 32..63 the
        // per-DOF / sensor block and the reward's DOF-order sums of env `lane - 32`
        const int e = lane & 31;
        float* R = sobs + (size_t)e * O;
        if (e < n) {
            if (lane < 32) {
                loco_obs_root(v, tp, e, R, pot + e0, prev + e0);
            } else {
                loco_obs_dof(m, v, tp, e, actions + (size_t)(e0 + e) * A, INFINITY, R);
                const LocoTerms lt = loco_reward_terms(tp, m.D, R, R + 12 + 2 * m.D + 6 * m.S);
                sterm[3 * e] = lt.limit_cost; sterm[3 * e + 1] = lt.act_cost; sterm[3 * e + 2] = lt.elec;
            }
        }
        __syncthreads();
        if (lane < n) {
            const int i = e0 + lane;
            const LocoTerms lt{sterm[3 * lane], sterm[3 * lane + 1], sterm[3 * lane + 2]};
            const int64_t progress = progress_buf[i] + 1;               // rl_task.py:242
            rew[i] = loco_reward_total(tp, R[0], R[10], R[11], pot[i], prev[i], lt);
            reset_buf[i] = nan_guard(st, i, loco_done(tp, R[0], reset_buf[i], progress));
            progress_buf[i] = progress;
        }
        __syncthreads();
        float* dst = obs + (size_t)e0 * O;
        const int cnt = n * O;
        if ((((uintptr_t)dst) & 15) == 0 && (cnt & 3) == 0) {
            for (int k = lane; k < cnt / 4; k += 64)
                ((float4*)dst)[k] = ((const float4*)sobs)[k];   // sobs 16-B aligned: ds_read_b128
        } else {
            for (int k = lane; k < cnt; k += 64) dst[k] = sobs[k];
        }
        return;
    }
    const int P = st.es + 1, AP = A + 1;
    float* srec = sm;
    float* sact = sm + TE * P;
    float* sobs = sact + TE * AP;
    tile_load(st.root_pos + (size_t)e0 * st.es, n * st.es, srec, st.es, P);
    tile_load(actions + (size_t)e0 * A, n * A, sact, A, AP);
    __syncthreads();
    DevState v = st;                        // the block's envs, viewed in LDS
    v.fs = 1; v.es = P;
    v.root_pos = srec; v.root_quat = srec + (st.root_quat - st.root_pos);
    v.root_vel = srec + (st.root_vel - st.root_pos);
    v.q = srec + (st.q - st.root_pos); v.qd = srec + (st.qd - st.root_pos);
    v.sens = st.sens + ssx(st, 0, e0);      // sensor wrenches read in place (their own array)
    if (lane < n) {
        const int i = e0 + lane;
        float* R = STAGE ? sobs + (size_t)lane * O : obs + (size_t)i * O;
        const int64_t progress = progress_buf[i] + 1;                   // rl_task.py:242
        loco_obs_env(m, v, tp, lane, sact + lane * AP, INFINITY, R, pot + e0, prev + e0);
        const float* ca = R + 12 + 2 * m.D + 6 * m.S;
        rew[i] = loco_reward(tp, m.D, R, ca, pot[i], prev[i]);        // calculate_metrics
        reset_buf[i] = nan_guard(st, i, loco_done(tp, R[0], reset_buf[i], progress));  // is_done
        progress_buf[i] = progress;
    }
    if (!STAGE) return;
    __syncthreads();
    float* dst = obs + (size_t)e0 * O;
    const int cnt = n * O;
    if ((((uintptr_t)dst) & 15) == 0 && (cnt & 3) == 0) {
        for (int k = lane; k < cnt / 4; k += 64)
            ((float4*)dst)[k] = ((const float4*)sobs)[k];   // sobs 16-B aligned: ds_read_b128
    } else {
        for (int k = lane; k < cnt; k += 64) dst[k] = sobs[k];
    }
}

static size_t post_tile_lds(int te, bool stage, int es, int A, int O, int D, int S) {
    if (te == 32 && stage)   // compact record tile + obs tile + reward sums
        return sizeof(float) * (size_t)(te * (13 + 2 * D + 6 * S + 1) + te * O + 3 * te);
    return sizeof(float) * (size_t)(te * (es + 1) + te * (A + 1) + (stage ? te * O : 0));
}

// variant of the tiled post-step (MI_POST_TILE=32p|16p|64s|64d|32s|32d, read per launch so a
// test can compare variants in one process; default 32p = k_loco_post_pipe with 32-env tiles,
// 16p the same kernel with 16-env tiles)
static int post_tile_variant() {
    const char* e = getenv("MI_POST_TILE");
    if (e && !strcmp(e, "64s")) return 0;
    if (e && !strcmp(e, "64d")) return 1;
    if (e && !strcmp(e, "32s")) return 2;
    if (e && !strcmp(e, "32d")) return 3;
    if (e && !strcmp(e, "16p")) return 6;
    return 4;   // 32p
}

// the three task methods as separate kernels, for tasks that override some of them
__global__ void k_observations(DevModel m, DevState st, DevTask tp, const float* actions,
                               float* obs, float* pot, float* prev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    float* R = obs + (size_t)tp.O * i;
    if (tp.kind == MI_TASK_CARTPOLE)
        cartpole_obs_env(st, i, R);
    else
        loco_obs_env(m, st, tp, i, actions + (size_t)tp.A * i, INFINITY, R, pot, prev);
}
__global__ void k_metrics(DevModel m, DevState st, DevTask tp, const float* actions,
                          const float* obs, float* rew, const float* pot, const float* prev) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    const float* R = obs + (size_t)tp.O * i;
    rew[i] = tp.kind == MI_TASK_CARTPOLE
                 ? cartpole_reward(tp, R)
                 : loco_reward(tp, m.D, R, actions + (size_t)tp.A * i, pot[i], prev[i]);
}
__global__ void k_is_done(DevState st, DevTask tp, const float* obs, int64_t* reset_buf,
                          const int64_t* progress_buf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    const float* R = obs + (size_t)tp.O * i;
    const int64_t d = tp.kind == MI_TASK_CARTPOLE
                          ? cartpole_done(tp, R, progress_buf[i])
                          : loco_done(tp, R[0], reset_buf[i], progress_buf[i]);
    reset_buf[i] = nan_guard(st, i, d);
}

__global__ void k_env_step(DevModel m, DevState st, SimP p, DevTask tp, const float* actions,
                           int substeps, float* obs_out, float* obs_task, float* rew,
                           int64_t* reset_buf, int64_t* progress_buf, float* pot, float* prev,
                           float* actions_out, float* rew_out, int64_t* reset_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    // 1. VecEnvRLGames.step:57 action clamp + pre_physics_step (reset_idx, efforts)
    task_pre_env(m, st, tp, i, actions, reset_buf, progress_buf, pot, prev, actions_out, true);
    // 2. controlFrequencyInv x World.step
    physics_env(m, st, p, i, substeps);
    // 3. post_physics_step into the unclamped row, then _process_data's obs clamp
    const int O = tp.O;
    float* R = (obs_task ? obs_task : obs_out) + (size_t)O * i;
    if (tp.kind == MI_TASK_CARTPOLE)
        cartpole_post(st, tp, i, R, rew, reset_buf, progress_buf);
    else if (tp.dr_act)   // task.actions = the noisy actions pre_physics_step received
        loco_post(m, st, tp, i, actions_out + (size_t)tp.A * i, INFINITY, R, rew, reset_buf,
                  progress_buf, pot, prev);
    else
        loco_post(m, st, tp, i, actions + (size_t)tp.A * i, tp.clip_actions, R, rew, reset_buf,
                  progress_buf, pot, prev);
    // 4. observation noise DR on task.obs_buf with the new reset_buf (vec_env_rlgames.py:70-71)
    if (tp.dr_obs) dr_row(st, tp, 0, i, R, O, reset_buf[i] != 0);
    const float co = tp.clip_obs;
    float* OUT = obs_out + (size_t)O * i;
    if (obs_task) {
        for (int k = 0; k < O; ++k) OUT[k] = clampf(R[k], -co, co);
    } else if (co < INFINITY) {
        for (int k = 0; k < O; ++k) OUT[k] = clampf(OUT[k], -co, co);
    }
    if (rew_out) rew_out[i] = rew[i];
    if (reset_out) reset_out[i] = reset_buf[i];
}

// ---- wavefront-per-env articulation path (one 64-lane workgroup = one env) -------------
// All model / table / state / task parameters sit in ONE device-resident block read through
// a __restrict__ const pointer: fields are scalar-loaded on use instead of pinning ~1.2 KB
// of by-value kernel arguments in SGPRs (which spilled).
struct KParams {
    DevModel m;
    WaveTabs t;
    DevState st;
    SimP p;
    DevTask tp;
    float* rows;
};

// launch with the model's compile-time topology (mi_topo_gen.hpp) or the runtime tables
// (per solver: TGS instantiations are Tgs<topology>)
template <class F>
static void with_topo(int id, bool tgs, F&& f) {
    auto go = [&](auto T) {
        if (tgs) f(Tgs<decltype(T)>{});
        else f(T);
    };
    switch (id) {
        case RobotHumanoid::id: go(TopoCT<RobotHumanoid>{}); break;
#ifndef MI_DEV_ONLY_HUMANOID   // register / spill inspection builds (tools/regs.sh): one topology
        case RobotAnt::id: go(TopoCT<RobotAnt>{}); break;
        default: go(TopoRuntime{}); break;
#else
        default: break;
#endif
    }
}

static inline dim3 wave_block(const mi_sim* s) { return dim3((s->pair ? 32 : 64) * s->wt.envs_per_wg); }
static inline dim3 wave_grid(const mi_sim* s) {
    return dim3((s->N + s->wt.envs_per_wg - 1) / s->wt.envs_per_wg);
}

// id of the generated topology whose link tree equals the model's (0: none)
static int match_topology(const mi_model_desc* md, bool self_on) {
    const int nr = md->root_free ? 6 : 0;
    for (const GenTopo& g : kGenTopos) {
        if (g.L != md->num_links || g.nr != nr) continue;
        if (self_on && !g.self) continue;   // compiled without self-collision: runtime tables
        bool same = true;
        for (int l = 1; l < g.L && same; ++l) same = g.link_parent[l] == md->parent[l];
        if (same) return g.id;
    }
    return 0;
}

static int sync_kparams(mi_sim* s) {
    if (!s->wave) return MI_OK;
    KParams h{};
    h.m = s->dm; h.t = s->wt; h.st = s->ds; h.p = s->sp; h.tp = s->tp; h.rows = s->rows;
    if (!s->kp_dev) {
        void* p = nullptr;
        int rc = dev_alloc(s, &p, sizeof(KParams));
        if (rc) return rc;
        s->kp_dev = p;
    }
    HIP_TRY(hipMemcpy(s->kp_dev, &h, sizeof(KParams), hipMemcpyHostToDevice));
    return MI_OK;
}

// The parameter block is loop-invariant across substeps; laundering its pointer per substep
// keeps the compiler from hoisting every field it reads into SGPRs for the whole loop
// (hundreds of values, spilled to VGPR lanes). Fields are re-read (scalar cache hits).
// The laundering goes through the constant address space: KParams is read-only while kernels
// run, so the compiler may read its fields with scalar loads (through a generic pointer it
// would emit flat vector loads, each a full memory round trip, for every parameter read).
using CKParams = const __attribute__((address_space(4))) KParams;
__device__ __forceinline__ const KParams* opaque_kp(const KParams* kp) {
    CKParams* c = (CKParams*)kp;
    asm volatile("" : "+s"(c));
    return (const KParams*)c;
}

// copy the per-model constant block into this workgroup's LDS (once per launch; shared by the
// workgroup's envs). The one workgroup barrier of the wave kernels.
__device__ __forceinline__ void stage_model_constants(const WaveTabs& t, float* smem) {
    for (int q = threadIdx.x; q < t.mc_len; q += blockDim.x) smem[t.s_mc + q] = t.g_mc[q];
    __syncthreads();
}

// XCD-aware env order (cdna_hip_programming.md T1): workgroups are dealt round-robin over the
// 8 XCDs (blocks b and b + 8 share one, each XCD has its own L2), so workgroup b takes slot
// (b % 8) * (G / 8) + b / 8 and each XCD owns one contiguous env range. The per-env scalars
// one lane writes (rew, reset, progress, potentials and their returned copies) and the obs rows
// that share a 128-B line are then written through ONE L2 and leave it as whole lines instead of
// eight partial ones. Speed only: any placement gives the same results. G % 8 != 0: identity.
__device__ __forceinline__ int xcd_block() {
    const unsigned G = gridDim.x, b = blockIdx.x;
    return (G & 7u) ? (int)b : (int)((b & 7u) * (G >> 3) + (b >> 3));
}
// env of this wave (workgroup = envs_per_wg consecutive envs, one wave each)
__device__ __forceinline__ int wave_env() {
    return (int)(xcd_block() * (blockDim.x >> 6) + (threadIdx.x >> 6));
}
__device__ __forceinline__ float* wave_env_lds(const WaveTabs& t, float* smem) {
    return smem + (threadIdx.x >> 6) * t.env_stride;
}

// k_loco_post_tiled<32, true> with the HBM latency hidden behind the math: each workgroup walks
// the tiles t = blockIdx.x, + gridDim.x, ... (grid = resident workgroups) and, while it computes
// tile t from LDS, holds the global loads of tile t + gridDim.x in registers (records, action
// rows, per-env scalars). Same arithmetic and write order per env as k_loco_post_tiled<32, true>
// (bit-identical outputs).
// Data movement is whole float4s with wave-uniform trip counts and no per-element guards:
//  - record tile in LDS: per env the record's first ne4 float4s (root, q, qd: the whole lines the
//    task reads; the efforts line is never fetched) and the env's ns4 float4s of sensor wrenches
//    from their own [N][6S] array, at an odd float4 stride P4 so one field of 32 envs spreads
//    over the banks; loads past the tile land in a spare float4 after the tile;
//  - loads clamp their index to the tile (a ragged last tile re-reads its last element into
//    slots nobody reads) instead of branching;
//  - the parameter block is read through the laundered KParams pointer once per tile (scalar
//    loads), so no loop-invariant parameter occupies an SGPR across the tile loop;
//  - the record / sensor tile loads and the obs tile stores are nontemporal (each byte is read or
//    written once; Humanoid 1 M envs 4.45-4.55 -> 4.63-4.65 TB/s with the stores, 4.75-4.86 with
//    the loads too).
// NR4 = record float4s per lane per tile (>= 32 ne4 / 64) and NS4 = sensor float4s per lane per
// tile (>= 32 ns4 / 64), template constants: the loads of a tile are one straight-line block,
// every register defined on every path (a guarded block made the compiler stage the tile through
// scratch). Action rows: always MI_PIPE_A loads per lane, the index clamped to the tile, the
// overhang written to a spare float. Host-checked: records (fs = 1), sensors (sfs = 1,
// ses = 6S, 6S % 4 == 0); 1 <= A <= 32; D, 6S <= 64.
constexpr int mi_pipe_a(int te) { return te / 2; }   // te envs x <= 32 actions / 64 lanes
// floor(x / d) for 0 <= x < 4096, 1 <= d <= 128: (x * ceil(2^20 / d)) >> 20 (exact there)
MI_D int div_small(int x, unsigned magic) { return (int)(((unsigned)x * magic) >> 20); }

typedef float v4f __attribute__((ext_vector_type(4)));   // native 16-B vector (no struct copies)

struct PipeGeo {   // record-tile geometry of k_loco_post_pipe (floats unless noted)
    int es4, ne4, ns4, P4, P, s0;
};
__host__ __device__ inline PipeGeo pipe_geo(int es, int D, int S) {
    PipeGeo g;
    g.es4 = es >> 2;
    g.ne4 = (13 + 2 * D + 3) >> 2;                        // record float4s up to the end of qd
    g.ns4 = (6 * S) >> 2;                                 // sensor float4s (6S % 4 == 0)
    g.P4 = (g.ne4 + g.ns4) | 1;                           // odd float4 stride
    g.P = 4 * g.P4;
    g.s0 = 4 * g.ne4;                                     // sensors in the LDS record
    return g;
}
constexpr int pipe_nr4(int ne4, int te = 32) { return (te * ne4 + 63) / 64; }
constexpr int pipe_ns4(int ns4, int te = 32) { return (te * ns4 + 63) / 64; }
static size_t post_pipe_lds(int es, int A, int O, int D, int S, int te = 32) {
    const PipeGeo g = pipe_geo(es, D, S);
    // records [te][P] + a spare float4, obs tile [te][O], potentials in / out, spare float (the
    // reward sums stay in registers: lane pairs). Humanoid, 32-env tiles: 20 128 B, 8 workgroups
    // per CU; 16-env tiles: 10 112 B
    return sizeof(float) * (size_t)(te * g.P + 4 + te * O + 2 * te + 4);
}

#ifndef MI_PIPE_ROT
#define MI_PIPE_ROT 1   // rotated pipeline with fixed-count stores (0: loads consumed at the loop head)
#endif
// NO4: obs float4s per lane per tile (>= TE O / 256, host-checked).
// TE envs per tile (32, or 16: half the LDS and prefetch registers per workgroup, so more
// workgroups stay resident; lanes e + 16 then repeat env e's root / reward chains, writing nothing)
template <int TE, int NR4, int NS4, int NO4>
__global__ __launch_bounds__(64) void k_loco_post_pipe(const KParams* __restrict__ kp_arg,
                                                      const float* __restrict__ actions,
                                                      float* obs, float* rew, int64_t* reset_buf,
                                                      int64_t* progress_buf, float* pot,
                                                      float* prev) {
    static_assert(TE == 32 || TE == 16, "tile of 32 or 16 envs");
    constexpr int MI_PIPE_A = mi_pipe_a(TE);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x;
    const KParams* kp = opaque_kp(kp_arg);
    const int O = kp->tp.O, A = kp->tp.A, D = kp->m.D, S = kp->m.S, es = kp->st.es, N = kp->st.N;
    const int ntiles = (N + TE - 1) / TE;
    const PipeGeo g = pipe_geo(es, D, S);
    const int ns = 6 * S, ka = 12 + 2 * D + ns;            // obs column of actions[0]
    const unsigned mag_ne = ((1u << 20) + g.ne4 - 1) / g.ne4, mag_a = ((1u << 20) + A - 1) / A;
    const unsigned mag_ns = ((1u << 20) + g.ns4 - 1) / g.ns4;
    v4f* srec4 = reinterpret_cast<v4f*>(sm);
    float* srec = sm;
    const int spare4 = TE * g.P4;                          // float4 slot past the record tile
    float* sobs = sm + TE * g.P + 4;
    float* spot = sobs + TE * O;                           // [TE] potentials (in / out)
    float* sprev = spot + TE;                              // [TE] prev_potentials (out)
    const int trash_o = TE * O + 2 * TE;                   // spare float past sprev (action overhang), from sobs
    v4f rr[NR4], rsn[NS4];
    float ra[MI_PIPE_A];
    int64_t pg = 0, rs = 0;
    int nf = 0;
    float pt = 0.0f;
    // global loads of tile T into registers (no wait here). A macro, not a lambda: through a
    // lambda's by-reference captures the compiler kept rr in scratch.
#define MI_PIPE_ISSUE(K, T)                                                                     \
    do {                                                                                        \
        const int e0_ = (T) * TE, n_ = min(TE, N - e0_);                                        \
        const int c4_ = n_ * g.ne4, cs_ = n_ * g.ns4, ca_ = n_ * A;                              \
        const v4f* s4_ = reinterpret_cast<const v4f*>((K)->st.root_pos + (size_t)e0_ * es);       \
        const v4f* ss_ = reinterpret_cast<const v4f*>((K)->st.sens + (size_t)e0_ * ns);           \
        const float* ga_ = actions + (size_t)e0_ * A;                                           \
        _Pragma("unroll") for (int r = 0; r < NR4; ++r) {                                       \
            const int k_ = min(lane + 64 * r, c4_ - 1), e_ = div_small(k_, mag_ne);              \
            rr[r] = __builtin_nontemporal_load(s4_ + e_ * g.es4 + (k_ - e_ * g.ne4));             \
        }                                                                                       \
        _Pragma("unroll") for (int r = 0; r < NS4; ++r) rsn[r] = __builtin_nontemporal_load(ss_ + min(lane + 64 * r, cs_ - 1)); \
        _Pragma("unroll") for (int r = 0; r < MI_PIPE_A; ++r) ra[r] = ga_[min(lane + 64 * r, ca_ - 1)]; \
        const int i_ = e0_ + min(lane, n_ - 1);                                                 \
        pg = progress_buf[i_];                                                                  \
        rs = reset_buf[i_];                                                                     \
        nf = (K)->st.nan_flag[i_];                                                              \
        pt = pot[i_];                                                                           \
    } while (0)
    // lane constants of the element-wise obs phase
    const int dof_pe = 64 / D, dof_le = lane / D, dof_j = lane - dof_le * D;
    const bool dof_lane = dof_le < dof_pe;
    const float dof_lo = dof_lane ? kp->m.lower[dof_j + 1] : 0.0f;
    const float dof_hi = dof_lane ? kp->m.upper[dof_j + 1] : 1.0f;
    const int sen_pe = ns > 0 ? 64 / ns : 0, sen_le = ns > 0 ? lane / ns : 0, sen_c = lane - sen_le * ns;
    const bool sen_lane = ns > 0 && sen_le < sen_pe;
#if MI_PIPE_ROT
    // Rotated pipeline: tile t + G's loads are issued after tile t's first barrier and moved
    // into LDS at the END of iteration t, after tile t's stores. Every memory op between the two
    // is an unconditional store of a fixed count (per-env outputs from all 64 lanes, NO4 obs
    // float4s + one tail dword per lane, indices clamped: lanes past the tile re-store the
    // tile's last element with the same data), so the wait for the loads is vmcnt(<that count>)
    // and tile t's stores stay in flight. (With the loads consumed at the loop head, the
    // variable-count store loops made the compiler wait for all but two of the tile's stores
    // before each next tile: store acknowledgements on the chain of every tile.)
    int64_t c_progress = 0, c_rb = 0;
    int c_nflag = 0;
#define MI_PIPE_STAGE(T)                                                                         \
    do {                                                                                        \
        _Pragma("unroll") for (int r = 0; r < NR4; ++r) {                                        \
            const int kk = lane + 64 * r, e = div_small(kk, mag_ne);                            \
            srec4[kk < TE * g.ne4 ? e * g.P4 + (kk - e * g.ne4) : spare4] = rr[r];               \
        }                                                                                       \
        _Pragma("unroll") for (int r = 0; r < NS4; ++r) {                                        \
            const int kk = lane + 64 * r, e = div_small(kk, mag_ns);                            \
            srec4[kk < TE * g.ns4 ? e * g.P4 + g.ne4 + (kk - e * g.ns4) : spare4] = rsn[r];      \
        }                                                                                       \
        _Pragma("unroll") for (int r = 0; r < MI_PIPE_A; ++r) {                                  \
            const int kk = lane + 64 * r, e = div_small(kk, mag_a);                             \
            sobs[kk < TE * A ? e * O + ka + (kk - e * A) : trash_o] = ra[r];                    \
        }                                                                                       \
        c_progress = pg + 1;                  /* rl_task.py:242 */                              \
        c_rb = rs;                                                                              \
        c_nflag = nf;                                                                           \
        if (lane < TE) spot[lane] = pt;                                                         \
    } while (0)
    int t = blockIdx.x;
    if (t < ntiles) {
        MI_PIPE_ISSUE(kp, t);
        MI_PIPE_STAGE(t);
    }
    for (; t < ntiles; t += gridDim.x) {
        const KParams* k = opaque_kp(kp_arg);
        const int e0 = t * TE, n = min(TE, N - e0);
        const int64_t progress = c_progress, rb = c_rb;
        const int nflag = c_nflag;
        __syncthreads();
        if (nflag && lane < n) {              // nan_guard bookkeeping, ahead of the next loads
            k->st.nan_flag[e0 + lane] = 0;
            atomicAdd(k->st.nan_total, 1ull);
        }
        const bool more = t + (int)gridDim.x < ntiles;
        if (more) MI_PIPE_ISSUE(k, t + (int)gridDim.x);   // in flight during the math and stores
        if (dof_lane) {
            const float vs = k->tp.dof_vel_scale;
            for (int e = dof_le; e < n; e += dof_pe) {
                const float* r = srec + e * g.P;
                float* o = sobs + e * O;
                o[12 + dof_j] = ref_unscale(r[13 + dof_j], dof_lo, dof_hi);
                o[12 + D + dof_j] = r[13 + D + dof_j] * vs;
            }
        }
        if (sen_lane) {
            const float cs = k->tp.contact_force_scale;
            for (int e = sen_le; e < n; e += sen_pe)
                sobs[e * O + 12 + 2 * D + sen_c] = srec[e * g.P + g.s0 + sen_c] * cs;
        }
        __syncthreads();
        const int pl = TE == 32 ? lane : ((lane & 15) | (lane & 32));
        const bool pw = TE == 32 || (lane & 16) == 0;
        {
            const DevTask& tp = k->tp;
            const int e = pl & 31;
            float* R = sobs + (size_t)e * O;
            loco_obs_root_pair(srec + e * g.P, tp, pl, R, spot, sprev, e < n && pw);
        }
        const LocoTerms lt = loco_reward_terms_pair(k->tp, D, sobs + (size_t)(pl & 31) * O,
                                                    sobs + (size_t)(pl & 31) * O + ka, pl);
        {
            // per-env outputs: computed on each lane for slot lane & (TE - 1) (valid where the
            // lower half holds that env), then every lane stores env el's values from lane el
            const DevTask& tp = k->tp;
            const int sl = lane & (TE - 1);
            const float* R = sobs + (size_t)sl * O;
            const float rv = loco_reward_total(tp, R[0], R[10], R[11], spot[sl], sprev[sl], lt);
            const int64_t d = nflag ? 1 : loco_done(tp, R[0], rb, progress);
            const int el = min(sl, n - 1), i = e0 + el;
            const float rew_v = __shfl(rv, el);
            const int d_v = __shfl((int)d, el);
            const uint32_t pr_lo = (uint32_t)__shfl((int)(uint32_t)progress, el);
            const uint32_t pr_hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)progress >> 32), el);
            rew[i] = rew_v;
            pot[i] = spot[el];
            prev[i] = sprev[el];
            reset_buf[i] = (int64_t)d_v;
            progress_buf[i] = (int64_t)(((uint64_t)pr_hi << 32) | pr_lo);
        }
        __syncthreads();
        {
            float* dst = obs + (size_t)e0 * O;   // 16-B aligned (host-checked), e0 * O * 4 B = 128 B multiples
            const int cnt = n * O, n4 = cnt >> 2;
#pragma unroll
            for (int r = 0; r < NO4; ++r) {
                const int kk = min(lane + 64 * r, n4 - 1);
                __builtin_nontemporal_store(reinterpret_cast<const v4f*>(sobs)[kk], reinterpret_cast<v4f*>(dst) + kk);
            }
            const int kt = min(4 * n4 + lane, cnt - 1);   // ragged tail (< 4 floats), else a re-store
            dst[kt] = sobs[kt];
        }
        __syncthreads();                    // the next tile overwrites the LDS tiles
        if (more) MI_PIPE_STAGE(t + (int)gridDim.x);
    }
#undef MI_PIPE_STAGE
#undef MI_PIPE_ISSUE
}
#else
    int t = blockIdx.x;
    if (t < ntiles) MI_PIPE_ISSUE(kp, t);
    for (; t < ntiles; t += gridDim.x) {
        const KParams* k = opaque_kp(kp_arg);
        const int e0 = t * TE, n = min(TE, N - e0);
        // registers -> LDS: records (float4 slots), actions into the obs rows' action columns
#pragma unroll
        for (int r = 0; r < NR4; ++r) {
            const int kk = lane + 64 * r, e = div_small(kk, mag_ne);
            srec4[kk < TE * g.ne4 ? e * g.P4 + (kk - e * g.ne4) : spare4] = rr[r];
        }
#pragma unroll
        for (int r = 0; r < NS4; ++r) {
            const int kk = lane + 64 * r, e = div_small(kk, mag_ns);
            srec4[kk < TE * g.ns4 ? e * g.P4 + g.ne4 + (kk - e * g.ns4) : spare4] = rsn[r];
        }
#pragma unroll
        for (int r = 0; r < MI_PIPE_A; ++r) {
            const int kk = lane + 64 * r, e = div_small(kk, mag_a);
            sobs[kk < TE * A ? e * O + ka + (kk - e * A) : trash_o] = ra[r];
        }
        const int64_t progress = pg + 1, rb = rs;          // rl_task.py:242
        const int nflag = nf;
        if (lane < TE) spot[lane] = pt;
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) MI_PIPE_ISSUE(k, t + (int)gridDim.x);   // in flight during the math
        // get_observations per-DOF and sensor entries (locomotion.py:226-228), the arithmetic of
        // loco_obs_dof, on all 64 lanes: lane = (env slot, column), the column a lane constant
        if (dof_lane) {
            const float vs = k->tp.dof_vel_scale;
            for (int e = dof_le; e < n; e += dof_pe) {
                const float* r = srec + e * g.P;
                float* o = sobs + e * O;
                o[12 + dof_j] = ref_unscale(r[13 + dof_j], dof_lo, dof_hi);
                o[12 + D + dof_j] = r[13 + D + dof_j] * vs;
            }
        }
        if (sen_lane) {
            const float cs = k->tp.contact_force_scale;
            for (int e = sen_le; e < n; e += sen_pe)
                sobs[e * O + 12 + 2 * D + sen_c] = srec[e * g.P + g.s0 + sen_c] * cs;
        }
        __syncthreads();
        // root-frame block and the reward's DOF-order sums: env lane & (TE - 1) on both lane
        // halves (the pair helpers see lane `pl`: with 16-env tiles lanes 16..31 / 48..63 act as
        // 0..15 / 32..47 and write nothing)
        const int pl = TE == 32 ? lane : ((lane & 15) | (lane & 32));
        const bool pw = TE == 32 || (lane & 16) == 0;
        {
            const DevTask& tp = k->tp;
            const int e = pl & 31;
            float* R = sobs + (size_t)e * O;
            loco_obs_root_pair(srec + e * g.P, tp, pl, R, spot, sprev, e < n && pw);
        }
        const LocoTerms lt = loco_reward_terms_pair(k->tp, D, sobs + (size_t)(pl & 31) * O,
                                                    sobs + (size_t)(pl & 31) * O + ka, pl);
        if (lane < n) {
            const int i = e0 + lane;
            const DevTask& tp = k->tp;
            float* R = sobs + (size_t)lane * O;
            const float p_new = spot[lane], p_old = sprev[lane];
            rew[i] = loco_reward_total(tp, R[0], R[10], R[11], p_new, p_old, lt);
            pot[i] = p_new;
            prev[i] = p_old;
            int64_t d = loco_done(tp, R[0], rb, progress);
            if (nflag) {                                                // nan_guard
                k->st.nan_flag[i] = 0;
                atomicAdd(k->st.nan_total, 1ull);
                d = 1;
            }
            reset_buf[i] = d;
            progress_buf[i] = progress;
        }
        __syncthreads();
        float* dst = obs + (size_t)e0 * O;
        const int cnt = n * O;
        if ((((uintptr_t)obs) & 15) == 0) {   // e0 * O * 4 B is a multiple of 128 B
            const int n4 = cnt >> 2;
            for (int kk = lane; kk < n4; kk += 64)
                __builtin_nontemporal_store(reinterpret_cast<const v4f*>(sobs)[kk], reinterpret_cast<v4f*>(dst) + kk);
            for (int kk = 4 * n4 + lane; kk < cnt; kk += 64) dst[kk] = sobs[kk];
        } else {
            for (int kk = lane; kk < cnt; kk += 64) dst[kk] = sobs[kk];
        }
        __syncthreads();                    // the next tile overwrites the LDS tiles
    }
#undef MI_PIPE_ISSUE
}
#endif

// register budget of the wave kernels: TopoCT::kWaves waves per SIMD
#define MI_WAVE_OCC __attribute__((amdgpu_waves_per_eu(T::kWaves, T::kWaves)))
template <class T>
__global__ __launch_bounds__(256) MI_WAVE_OCC void k_sim_step_wave(const KParams* __restrict__ kp, int substeps) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WaveTabs& t = kp->t;
    const int i = wave_env();
    stage_model_constants(t, smem);
    if (i >= kp->st.N) return;
    float* gW = kp->rows + (size_t)i * t.g_row_stride;
    float* sm = wave_env_lds(t, smem);
    for (int s = 0; s < substeps; ++s) {
        const KParams* k = opaque_kp(kp);
        wave_artic_substep<T>(k->m, k->t, k->st, k->p, i, smem, sm, gW, s == 0, s == substeps - 1);
    }
}

template <class T>
__global__ __launch_bounds__(256) MI_WAVE_OCC void k_env_step_wave(const KParams* __restrict__ kp,
                                                      const float* actions, int substeps,
                                                      float* obs_out, float* obs_task, float* rew,
                                                      int64_t* reset_buf, int64_t* progress_buf,
                                                      float* pot, float* prev, float* actions_out,
                                                      float* rew_out, int64_t* reset_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const DevModel& m = kp->m;
    const WaveTabs& t = kp->t;
    const DevState& st = kp->st;
    const SimP& p = kp->p;
    const DevTask& tp = kp->tp;
    float* rows = kp->rows;
    const int i = wave_env();
    const bool live = i < st.N;
    // 1. clamp + pre_physics_step (wave-cooperative); model constants into LDS
    STAMP_BEGIN();
    float a_lane = 0.0f;
    if (live)
        a_lane = wave_task_pre(m, t, st, tp, i, actions, reset_buf, progress_buf, pot, prev, actions_out);
    stage_model_constants(t, smem);
    if (!live) return;
    STAMP(13);
    // 2. controlFrequencyInv x World.step, wave-cooperative
    float* gW = rows + (size_t)i * t.g_row_stride;
    float* sm = wave_env_lds(t, smem);
    for (int s = 0; s < substeps; ++s) {
        const KParams* k = opaque_kp(kp);
        wave_artic_substep<T>(k->m, k->t, k->st, k->p, i, smem, sm, gW, s == 0, s == substeps - 1);
    }
    // 3. post_physics_step + obs clamp, wave-cooperative from the LDS-resident state
    STAMP_RESET();
    wave_loco_post(m, t, st, tp, i, sm, a_lane, obs_out, obs_task, rew, reset_buf, progress_buf,
                   pot, prev, rew_out, reset_out);
    STAMP(14);
}

// ---- paired kernels (mi_pair.hpp): 8 waves x 2 envs = 16 envs per workgroup, 2 waves / SIMD
// env of this lane's half: workgroup slot (threadIdx.x >> 5) = 2 wave + half
__device__ __forceinline__ int pair_env() { return (int)(xcd_block() * (blockDim.x >> 5) + (threadIdx.x >> 5)); }
__device__ __forceinline__ float* pair_env_lds(const WaveTabs& t, float* smem) {
    return smem + (threadIdx.x >> 5) * t.env_stride;
}
// the first env of this lane's wave (N is even: both halves of a wave are live together)
__device__ __forceinline__ bool pair_live(int N) {
    return (int)(xcd_block() * (blockDim.x >> 5) + ((threadIdx.x >> 6) << 1)) < N;
}
// this wave's index over the launch (its wide-PGS scratch slot)
__device__ __forceinline__ int pair_wave() { return (int)(xcd_block() * (blockDim.x >> 6) + (threadIdx.x >> 6)); }
// Pairing by load (DevState::pair_by_load): a wave's PGS is as long as its heavier env's and, on
// the wide path (33..64 rows), as long as BOTH envs' one after the other, so two heavy envs in
// one wave set the launch's tail. Each wave ranks its workgroup's 16 envs by their constraint rows
// in the last fused env-step (`load`, heavier first, ties by index) and takes ranks w and 15 - w
// (w = wave in the workgroup): heaviest with lightest. A permutation inside the workgroup, the
// same for every wave of it (every wave computes it); full workgroups only, and only those
// holding an env above MI_PAIR_LOAD_MIN constraint rows.
__device__ __forceinline__ int pair_env_by_load(const DevState& st) {
    const int e0 = (int)(xcd_block() * (blockDim.x >> 5));
    const int slot = (int)(threadIdx.x >> 5);
    if (!st.pair_by_load || blockDim.x != 512 || e0 + 16 > st.N) return e0 + slot;
    const int l = (int)(threadIdx.x & 63u);
    const int key = l < 16 ? st.load[e0 + l] : -1;
    int rank = 0, kmax = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int kj = __builtin_amdgcn_readlane(key, j);
        rank += (kj > key || (kj == key && j < l)) ? 1 : 0;
        kmax = max(kmax, kj);
    }
    // only workgroups with an env above MI_PAIR_LOAD_MIN rows are re-paired (st.pair_by_load =
    // 1 + MI_PAIR_LOAD_MIN; default 0: all but an all-zero workgroup). Re-pairing costs write
    // traffic (adjacent envs' obs / reward rows share cache lines and are no longer written by
    // one wave: 7.29 -> 8.38 MB per launch) but not time
    if (kmax < st.pair_by_load) return e0 + slot;
    // (A/B round 5: giving waves 4..7 the middle ranks, so that the heaviest env's SIMD partner
    // is lighter, measured neutral: 0.1177 vs 0.1178 ms)
    const int w = slot >> 1;
    const unsigned long long heavy = __ballot(l < 16 && rank == w);
    const unsigned long long light = __ballot(l < 16 && rank == 15 - w);
    return e0 + (int)__builtin_ctzll((slot & 1) ? light : heavy);
}
#define MI_PAIR_OCC __attribute__((amdgpu_waves_per_eu(2, 2)))

// row-major state mirrors (mi_sim_set_mirror) a physics launch refreshes itself: pos, quat, vel,
// q, qd, sensor wrenches; p[0] == nullptr: none
struct Mirrors { float* p[6]; };

template <class T>
__global__ __launch_bounds__(512) MI_PAIR_OCC void k_sim_step_pair(const KParams* __restrict__ kp, int substeps,
                                                    Mirrors mir) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WaveTabs& t = kp->t;
    const bool live = pair_live(kp->st.N);
    const int i = live ? pair_env_by_load(kp->st) : pair_env();
    stage_model_constants(t, smem);
    if (!live) return;
    float* gW = kp->rows + (size_t)i * t.g_row_stride;
    float* sm = pair_env_lds(t, smem);
    int prio = 0;                          // issue priority so far (mi_pair.hpp MI_PRIO_C*)
    int load = 0;                          // this env's most constraint rows in a substep (unused here)
    for (int s = 0; s < substeps; ++s) {
        const KParams* k = opaque_kp(kp);
        pair_artic_substep<T>(k->m, k->t, k->st, k->p, i, pair_wave(), smem, sm, gW, s == 0, s == substeps - 1,
                              prio, load);
    }
    // World.step() then the getters (locomotion.py:81-89): the final state is still in LDS, so the
    // launch writes the getters' row-major mirrors itself (the same values it stored to the
    // state) and the mirror refresh launch is not needed
    if (mir.p[0]) {
        const KParams* k = opaque_kp(kp);
        const int lane = (int)(threadIdx.x & 31u), D = k->m.D, nr = k->m.nr, S6 = 6 * k->m.S;
        const WaveTabs& tk = k->t;
        if (lane < 3) mir.p[0][3 * i + lane] = sm[tk.s_rp + lane];
        if (lane < 4) mir.p[1][4 * i + lane] = sm[tk.s_rp + 4 + lane];
        if (lane < 6) mir.p[2][6 * i + lane] = sm[tk.s_us + lane];
        if (lane < D) {
            mir.p[3][(size_t)D * i + lane] = sm[tk.s_q + lane];
            mir.p[4][(size_t)D * i + lane] = sm[tk.s_us + nr + lane];
        }
        for (int c = lane; c < S6; c += 32) mir.p[5][(size_t)S6 * i + c] = sm[tk.s_rb + c];
    }
}

template <class T>
__global__ __launch_bounds__(512) MI_PAIR_OCC void k_env_step_pair(const KParams* __restrict__ kp,
                                                    const float* actions, int substeps,
                                                    float* obs_out, float* obs_task, float* rew,
                                                    int64_t* reset_buf, int64_t* progress_buf,
                                                    float* pot, float* prev, float* actions_out,
                                                    float* rew_out, int64_t* reset_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const DevModel& m = kp->m;
    const WaveTabs& t = kp->t;
    const DevState& st = kp->st;
    const DevTask& tp = kp->tp;
    const bool live = pair_live(st.N);
    const int i = live ? pair_env_by_load(st) : pair_env();
    STAMP_BEGIN();
    float a_lane = 0.0f;
    if (live)
        a_lane = pair_task_pre(m, st, tp, i, actions, reset_buf, progress_buf, pot, prev, actions_out);
    stage_model_constants(t, smem);
    if (!live) return;
    STAMP(13);
    float* gW = kp->rows + (size_t)i * t.g_row_stride;
    float* sm = pair_env_lds(t, smem);
    int prio = 0;                          // issue priority so far (mi_pair.hpp MI_PRIO_C*)
    int load = 0;                          // this env's most constraint rows in a substep
    for (int s = 0; s < substeps; ++s) {
        const KParams* k = opaque_kp(kp);
        pair_artic_substep<T>(k->m, k->t, k->st, k->p, i, pair_wave(), smem, sm, gW, s == 0, s == substeps - 1,
                              prio, load);
    }
    STAMP_RESET();
    pair_loco_post(m, t, st, tp, i, sm, a_lane, obs_out, obs_task, rew, reset_buf, progress_buf,
                   pot, prev, rew_out, reset_out);
    // the next fused step pairs by it (only the fused step writes it: World.step launches of one
    // env-step, deferred or not, all see the same pairing)
    if ((threadIdx.x & 31u) == 0) st.load[i] = load;
    STAMP(14);
}

// launch a paired kernel for the topologies that have one (compiled, nv <= 32)
template <class T>
constexpr bool has_pair() {
    if constexpr (T::kCT) return T::nv <= 32;
    else return false;
}

// Randomizer.apply_{observations,actions}_randomization (randomize.py:212-260), modular path
__global__ void k_dr_apply(DevState st, DevTask tp, int which, float* buf, int C,
                           const int64_t* reset_buf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    dr_row(st, tp, which, i, buf + (size_t)C * i, C, reset_buf[i] != 0);
}

__global__ void k_reset_idx(DevModel m, DevState st, DevTask tp, const int64_t* ids, int n,
                            int64_t* reset_buf, int64_t* progress_buf, float* pot, float* prev) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int64_t i = ids ? ids[t] : t;
    if (i < 0 || i >= st.N) return;
    task_reset_env(m, st, tp, (int)i, pot, prev);
    if (reset_buf) reset_buf[i] = 0;
    if (progress_buf) progress_buf[i] = 0;
}

// state fields (field stride fs, env stride es: DevState) <-> row-major [N,C] torch tensors
// (ArticulationView getters / setters, gather / scatter with optional indices). One element per
// lane with the column fastest, so the row-major side is one contiguous stream; on the
// per-env-record layout (fs = 1) the state side is too (the C fields of a record are adjacent).
// The field-major layout of the one-lane-per-env path (es = 1) gathers through an LDS tile:
// field-major reads in, row-major writes out, both coalesced.
constexpr int MI_GATHER_TILE = 256, MI_GATHER_MAXC = 32;
// Several fields of one ArticulationView call (get_world_poses: pos + quat; set_world_poses;
// get / set_velocities, ...), or all six state mirrors, in ONE launch: blockIdx.y picks the field.
// fs / es: the state side's field / env strides of this field (gathers: per field, since the
// sensor wrenches have strides of their own; scatters take the record strides as arguments)
struct GField { const float* src; float* dst; int C; int fs = 0, es = 0; };
struct GFields { GField f[6]; };
__global__ __launch_bounds__(256) void k_soa_to_rows_multi(GFields fs3, int N) {
    const GField g = fs3.f[blockIdx.y];
    const int fs = g.fs, es = g.es;
    const int64_t e0 = (int64_t)blockIdx.x * MI_GATHER_TILE;
    const int ne = (int)min((int64_t)MI_GATHER_TILE, (int64_t)N - e0);
    const int C = g.C, tot = ne * C;
    float* out = g.dst + e0 * C;
    if (es != 1 || C > MI_GATHER_MAXC) {           // records (or too wide for the tile)
        for (int t = threadIdx.x; t < tot; t += blockDim.x) {
            const int e = t / C, c = t - e * C;
            out[t] = g.src[(size_t)c * fs + (size_t)(e0 + e) * es];
        }
        return;
    }
    __shared__ float tile[MI_GATHER_MAXC * (MI_GATHER_TILE + 1)];   // [c][e], odd stride
    for (int c = 0; c < C; ++c)
        if ((int)threadIdx.x < ne) tile[c * (MI_GATHER_TILE + 1) + threadIdx.x] = g.src[(size_t)c * fs + e0 + threadIdx.x];
    __syncthreads();
    for (int t = threadIdx.x; t < tot; t += blockDim.x) {
        const int e = t / C, c = t - e * C;
        out[t] = tile[c * (MI_GATHER_TILE + 1) + e];
    }
}
// Scatter: one lane per (row, column). With duplicate ids each column of the env takes its
// value from one of the duplicate rows, unspecified which (torch index_put_ and PhysX's indexed
// setters leave duplicates undefined as well; tests/test_gpu_view.py).
template <typename IDX>
__global__ __launch_bounds__(256) void k_rows_to_soa_multi(GFields fs3, int n, const IDX* __restrict__ idx,
                                                          int N, int fs, int es) {
    const GField g = fs3.f[blockIdx.y];
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)n * g.C) return;
    const int r = (int)(t / g.C), c = (int)(t - (int64_t)r * g.C);
    const int64_t i = idx ? (int64_t)idx[r] : r;
    if (i < 0 || i >= N) return;                   // out-of-range ids are ignored
    const_cast<float*>(g.dst)[(size_t)c * fs + (size_t)i * es] = g.src[t];
}
static inline dim3 gather_grid(int N) { return dim3((N + MI_GATHER_TILE - 1) / MI_GATHER_TILE); }
static inline dim3 scatter_grid(int n, int C) { return dim3((unsigned)(((int64_t)n * C + 255) / 256)); }

__global__ void k_init_state(DevState st, int D) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.N) return;
    const int N = st.N;
    for (int k = 0; k < 3; ++k) st.root_pos[sx(st, k, i)] = st.origins[(size_t)k * N + i];
    st.root_quat[sx(st, 0, i)] = 1.0f;
}

__global__ void k_fill_uniform(int N, int64_t off, float* out, int cols, uint64_t seed,
                               uint64_t step, float lo, float hi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint64_t gid = (uint64_t)(off + i);
    const float w = hi - lo;
    float u[4];
    for (int c = 0; c < cols; ++c) {
        if ((c & 3) == 0) uniform4(seed, gid, (uint32_t)step, (uint32_t)(c >> 2), 1, u);
        out[(size_t)i * cols + c] = w * u[c & 3] + lo;
    }
}

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int mi_abi_version(void) { return MI_ABI_VERSION; }
#ifndef MI_BUILD_ID
#define MI_BUILD_ID "unknown"
#endif
// the string carries a marker prefix so the build id can be found in the binary file
const char* mi_build_id(void) {
    static const char id[] = MI_BUILD_ID;
    return (sizeof(id) > 12 && id[0] == 'M' && id[11] == ':') ? id + 12 : id;
}

#ifdef MI_STAMPS
// diagnostic build only: phase stamps of workgroup MI_STAMP_BLOCK's last substep
int mi_debug_stamps(unsigned long long* out, int n) {
    if (!out || n <= 0 || n > 32) return MI_E_ARG;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<unsigned long long> all((size_t)MI_STAMP_SLOTS * 32);
    HIP_TRY(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(g_phase), all.size() * sizeof(unsigned long long)));
    for (int k = 0; k < n; ++k) {
        unsigned long long acc = 0;
        for (size_t b = 0; b < (size_t)MI_STAMP_SLOTS; ++b) acc += all[b * 32 + k];
        out[k] = acc;
    }
    std::fill(all.begin(), all.end(), 0ull);   // read-and-reset
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), all.data(), all.size() * sizeof(unsigned long long)));
    return MI_OK;
}
#endif
#ifdef MI_STAMPS
// diagnostic build only: the raw per-wave phase accumulators [slots][32] (slot = wave index of
// the launch modulo MI_STAMP_SLOTS), read-and-reset (tools/pair_tail.py)
int mi_debug_stamps_raw(unsigned long long* out, int slots) {
    if (!out || slots <= 0 || slots > MI_STAMP_SLOTS) return MI_E_ARG;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<unsigned long long> all((size_t)MI_STAMP_SLOTS * 32);
    HIP_TRY(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(g_phase), all.size() * sizeof(unsigned long long)));
    std::copy(all.begin(), all.begin() + (size_t)slots * 32, out);
    std::fill(all.begin(), all.end(), 0ull);
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_phase), all.data(), all.size() * sizeof(unsigned long long)));
    return MI_OK;
}
#endif
const char* mi_last_error(void) { return g_err.c_str(); }

int mi_sim_create(const mi_model_desc* md, const mi_sim_params* prm, int32_t N, int64_t off,
                  int32_t device_id, const float* env_origins, uint64_t seed, mi_sim** out) {
    if (!md || !prm || !out || !env_origins) return fail(MI_E_NULL, "mi_sim_create: null argument");
    *out = nullptr;
    if (N <= 0) return fail(MI_E_SHAPE, "num_envs must be > 0 (got %d)", N);
    const int L = md->num_links;
    if (L < 1 || L - 1 > MI_MAXA) return fail(MI_E_MODEL, "num_links %d out of range [1,%d]", L, MI_MAXA + 1);
    if (md->dyn_kind != MI_DYN_ARTICULATION && md->dyn_kind != MI_DYN_CARTPOLE)
        return fail(MI_E_ARG, "bad dyn_kind %d", md->dyn_kind);
    if (md->dyn_kind == MI_DYN_CARTPOLE && L != 3)
        return fail(MI_E_MODEL, "cart-pole dynamics needs exactly 2 joints");
    if (!md->parent || !md->jtype || !md->axis || !md->pos || !md->quat || !md->mass || !md->com ||
        !md->inertia || !md->lower || !md->upper || !md->damping || !md->armature)
        return fail(MI_E_NULL, "model arrays must not be null");
    if (md->num_geoms < 0 || md->num_sensors < 0 || md->num_pairs < 0)
        return fail(MI_E_MODEL, "negative counts");
    if (md->num_geoms && (!md->geom_link || !md->geom_type || !md->geom_p0 || !md->geom_p1 || !md->geom_radius))
        return fail(MI_E_NULL, "geom arrays must not be null");
    if (md->num_sensors && (!md->sensor_link || !md->sensor_pos))
        return fail(MI_E_NULL, "sensor arrays must not be null");
    for (int l = 1; l < L; ++l)
        if (md->parent[l] < 0 || md->parent[l] >= l)
            return fail(MI_E_MODEL, "parent[%d]=%d must be in [0,%d)", l, md->parent[l], l);
    for (int g = 0; g < md->num_geoms; ++g)
        if (md->geom_link[g] < 0 || md->geom_link[g] >= L) return fail(MI_E_MODEL, "geom_link[%d] out of range", g);
    for (int s = 0; s < md->num_sensors; ++s)
        if (md->sensor_link[s] < 0 || md->sensor_link[s] >= L) return fail(MI_E_MODEL, "sensor_link[%d] out of range", s);
    if (md->num_pairs && !md->pairs) return fail(MI_E_NULL, "pairs must not be null");
    for (int q = 0; q < 2 * md->num_pairs; ++q)
        if (md->pairs[q] < 0 || md->pairs[q] >= md->num_geoms)
            return fail(MI_E_MODEL, "pairs[%d]=%d is not a geom index", q, md->pairs[q]);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MI_E_NODEV, "no HIP device visible");
    if (device_id < 0 || device_id >= ndev) return fail(MI_E_NODEV, "device_id %d out of range (%d devices)", device_id, ndev);
    HIP_TRY(hipSetDevice(device_id));

    mi_sim* s = new mi_sim();
    s->device = device_id;
    s->N = N;
    if (const char* d = getenv("MI_SIM_DEFER")) s->defer = atoi(d) != 0;
    if (const char* b = getenv("MI_SIM_BLOCK")) {
        int v = atoi(b);
        if (v >= 1 && v <= 1024) s->block = v;
    }
    auto cleanup = [&](int rc) { mi_sim_destroy(s); return rc; };
    DevModel& m = s->dm;
    m.dyn = md->dyn_kind;
    m.root_free = md->root_free ? 1 : 0;
    m.L = L;
    m.D = L - 1;
    m.nr = m.root_free ? 6 : 0;
    m.nv = m.nr + m.D;
    m.G = md->num_geoms;
    m.S = md->num_sensors;
    if (m.nv > MI_MAXNV) return cleanup(fail(MI_E_MODEL, "too many dofs"));
    // derived tables
    std::vector<int> dof_parent(m.nv > 0 ? m.nv : 1), dof_link(m.nv > 0 ? m.nv : 1), pt_geom, pt_end;
    for (int k = 0; k < m.nr; ++k) { dof_parent[k] = k - 1; dof_link[k] = 0; }
    for (int l = 1; l < L; ++l) {
        const int k = m.nr + l - 1, P = md->parent[l];
        dof_parent[k] = P == 0 ? m.nr - 1 : m.nr + P - 1;
        dof_link[k] = l;
    }
    for (int g = 0; g < m.G; ++g) {
        pt_geom.push_back(g); pt_end.push_back(0);
        if (md->geom_type[g] == MI_GEOM_CAPSULE) { pt_geom.push_back(g); pt_end.push_back(1); }
    }
    m.npts = (int)pt_geom.size();
    // self-collision rows share the MI_MAX_ROWS budget (mi_sim.h); ground + limit rows must fit
    const bool self_on = prm->enable_self_collisions && md->num_pairs > 0 &&
                         md->dyn_kind == MI_DYN_ARTICULATION;
    m.max_rows = 3 * m.npts + m.D;
    if (m.max_rows > MI_MAX_ROWS)
        return cleanup(fail(MI_E_MODEL, "%d contact points + %d joints exceed the %d-row budget",
                            m.npts, m.D, MI_MAX_ROWS));
    if (self_on) m.max_rows = std::min(MI_MAX_ROWS, 3 * (m.npts + md->num_pairs) + m.D);
    int rc = 0;
#define UP(field, src, cnt) if ((rc = upload(s, src, (size_t)(cnt), &m.field))) return cleanup(rc)
    UP(parent, md->parent, L); UP(jtype, md->jtype, L); UP(axis, md->axis, 3 * L);
    UP(pos, md->pos, 3 * L); UP(quat, md->quat, 4 * L); UP(mass, md->mass, L);
    UP(com, md->com, 3 * L); UP(inertia, md->inertia, 6 * L); UP(lower, md->lower, L);
    UP(upper, md->upper, L); UP(damping, md->damping, L); UP(armature, md->armature, L);
    UP(dof_parent, dof_parent.data(), dof_parent.size()); UP(dof_link, dof_link.data(), dof_link.size());
    UP(geom_link, md->geom_link, m.G); UP(geom_p0, md->geom_p0, 3 * m.G);
    UP(geom_p1, md->geom_p1, 3 * m.G); UP(geom_radius, md->geom_radius, m.G);
    UP(pt_geom, pt_geom.data(), pt_geom.size()); UP(pt_end, pt_end.data(), pt_end.size());
    UP(sensor_link, md->sensor_link, m.S); UP(sensor_pos, md->sensor_pos, 3 * m.S);
#undef UP
    m.cart_mass = md->cart_mass; m.pole_mass = md->pole_mass; m.pole_com = md->pole_com;
    m.pole_inertia = md->pole_inertia; m.cart_damping = md->cart_damping;
    m.pole_damping = md->pole_damping;
    // workspace slots (articulation only)
    int o = 0;
    if (m.dyn == MI_DYN_ARTICULATION) {
        const int nv = m.nv, R = m.max_rows;
        m.o_R = o; o += 9 * L;
        m.o_o = o; o += 3 * L;
        m.o_aw = o;
        m.o_Ic = o; o += 10 * L;
        m.o_S = o; o += 6 * nv;
        m.o_V = o; o += 6 * L;
        m.o_A = o; o += 6 * L;
        m.o_F = o; o += 6 * L;
        m.o_M = o; o += nv * nv;
        m.o_u = o; o += nv;
        m.o_r = o; o += nv;
        m.o_Jr = o; o += R * nv;
        m.o_W = o; o += R * nv;
        m.o_b = o; o += R;
        m.o_lam = o; o += R;
        m.o_Ad = o; o += R;
        m.o_rk = o; o += R;
        m.o_ds = o; o += R;     // TGS: a row's separation change over the sub-steps so far
        m.o_cp = o; o += 3 * m.npts;
        m.o_cl = o; o += m.npts;
    }
    m.slots = o;
    // wavefront-per-env path: eligibility + host-built tree tables + LDS layout
    {
        const char* path = getenv("MI_SIM_PATH");
        const bool want_thread = path && std::string(path) == "thread";
        // (the post-step keeps sensor wrenches + reward terms in the row-bias region)
        s->wave = m.dyn == MI_DYN_ARTICULATION && !want_thread && m.nv <= WNV && m.npts <= 64 &&
                  m.max_rows <= 128 && L <= 64 && m.max_rows >= 6 * m.S + 3 * m.D;
        if (self_on && !s->wave)
            return cleanup(fail(MI_E_MODEL, "self-collision needs the wavefront-per-env path "
                                            "(one-lane-per-env path %s)", want_thread ? "forced by MI_SIM_PATH" : "selected"));
    }
    if (s->wave) {
        const char* tsel = getenv("MI_SIM_TOPO");
        s->topo = (tsel && std::string(tsel) == "runtime") ? 0 : match_topology(md, self_on);
        WaveTabs& t = s->wt;
        std::vector<int> depth(L, 0);
        int maxd = 0;
        for (int l = 1; l < L; ++l) { depth[l] = depth[md->parent[l]] + 1; maxd = std::max(maxd, depth[l]); }
        t.nlev = maxd + 1;
        std::vector<int> lev_start(t.nlev + 1, 0), lev_links;
        for (int d = 0; d < t.nlev; ++d) {
            lev_start[d] = (int)lev_links.size();
            for (int l = 0; l < L; ++l) if (depth[l] == d) lev_links.push_back(l);
        }
        lev_start[t.nlev] = (int)lev_links.size();
        std::vector<int> child_start(L + 1, 0), child_list;
        for (int l = 0; l < L; ++l) {
            child_start[l] = (int)child_list.size();
            for (int c = l + 1; c < L; ++c) if (md->parent[c] == l) child_list.push_back(c);
        }
        child_start[L] = (int)child_list.size();
        std::vector<int> desc_start(L + 1, 0), desc_list;
        for (int l = 0; l < L; ++l) {
            desc_start[l] = (int)desc_list.size();
            for (int c = l + 1; c < L; ++c) {
                int x = md->parent[c];
                while (x > l) x = md->parent[x];
                if (x == l) desc_list.push_back(c);
            }
        }
        desc_start[L] = (int)desc_list.size();
        if (desc_list.empty()) desc_list.push_back(0);
        std::vector<int> anc_start(m.nv + 1, 0), anc_list;
        int na_max = 0;
        for (int k = 0; k < m.nv; ++k) {
            anc_start[k] = (int)anc_list.size();
            for (int j = dof_parent[k]; j >= 0; j = dof_parent[j]) anc_list.push_back(j);
            na_max = std::max(na_max, (int)anc_list.size() - anc_start[k]);
        }
        anc_start[m.nv] = (int)anc_list.size();
        std::vector<unsigned long long> link_mask(L, 0ull);
        for (int l = 0; l < L; ++l) {
            unsigned long long msk = 0ull;
            for (int k = 0; k < m.nr; ++k) msk |= 1ull << k;
            for (int x = l; x > 0; x = md->parent[x]) msk |= 1ull << (m.nr + x - 1);
            link_mask[l] = msk;
        }
        std::vector<unsigned char> tri_p, tri_q;
        for (int q = 0; q < na_max; ++q)
            for (int p2 = 0; p2 <= q; ++p2) { tri_p.push_back((unsigned char)p2); tri_q.push_back((unsigned char)q); }
        if (tri_p.empty()) { tri_p.push_back(0); tri_q.push_back(0); }
        if (child_list.empty()) child_list.push_back(0);
        if (anc_list.empty()) anc_list.push_back(0);
#define UPW(field, vec) if ((rc = upload(s, vec.data(), vec.size(), &t.field))) return cleanup(rc)
        UPW(lev_start, lev_start); UPW(lev_links, lev_links); UPW(child_start, child_start);
        UPW(child_list, child_list); UPW(anc_start, anc_start); UPW(anc_list, anc_list);
        UPW(desc_start, desc_start); UPW(desc_list, desc_list);
        std::vector<int> chain_start(L + 1, 0), chain_list;
        for (int l = 0; l < L; ++l) {
            chain_start[l] = (int)chain_list.size();
            std::vector<int> up;
            for (int x = l; x > 0; x = md->parent[x]) up.push_back(x);
            chain_list.insert(chain_list.end(), up.rbegin(), up.rend());
        }
        chain_start[L] = (int)chain_list.size();
        if (chain_list.empty()) chain_list.push_back(0);
        UPW(chain_start, chain_start); UPW(chain_list, chain_list);
        UPW(link_mask, link_mask); UPW(tri_p, tri_p); UPW(tri_q, tri_q);
        // per-model constant block (SoA), staged into LDS by every workgroup (McField & co.)
        {
            const int np = (int)pt_geom.size(), ns = md->num_sensors;
            std::vector<float> mcb((size_t)MC_NLINKF * L, 0.0f);
            for (int l = 0; l < L; ++l) {
                auto put = [&](int f, float v) { mcb[(size_t)f * L + l] = v; };
                for (int c = 0; c < 3; ++c) {
                    put(MC_POS + c, md->pos[3 * l + c]); put(MC_AXIS + c, md->axis[3 * l + c]);
                    put(MC_COM + c, md->com[3 * l + c]);
                }
                for (int c = 0; c < 4; ++c) put(MC_QUAT + c, md->quat[4 * l + c]);
                for (int c = 0; c < 6; ++c) put(MC_INER + c, md->inertia[6 * l + c]);
                put(MC_JTYPE, (float)md->jtype[l]); put(MC_MASS, md->mass[l]);
                put(MC_ARM, md->armature[l]); put(MC_DAMP, md->damping[l]);
                put(MC_LO, md->lower[l]); put(MC_HI, md->upper[l]);
                const unsigned lo32 = (unsigned)(link_mask[l] & 0xffffffffull);
                float mf; std::memcpy(&mf, &lo32, 4); put(MC_MASK, mf);
            }
            auto pad4 = [&]() { while (mcb.size() % 4) mcb.push_back(0.0f); };
            pad4();
            t.mc_pts = (int)mcb.size();
            mcb.resize(mcb.size() + (size_t)MP_NF * np, 0.0f);
            for (int c = 0; c < np; ++c) {
                const int g = pt_geom[c];
                const float* pg = pt_end[c] ? md->geom_p1 + 3 * g : md->geom_p0 + 3 * g;
                mcb[t.mc_pts + (size_t)MP_LINK * np + c] = (float)md->geom_link[g];
                for (int q = 0; q < 3; ++q) mcb[t.mc_pts + (size_t)(MP_X + q) * np + c] = pg[q];
                mcb[t.mc_pts + (size_t)MP_RAD * np + c] = md->geom_radius[g];
            }
            pad4();
            t.mc_sens = (int)mcb.size();
            mcb.resize(mcb.size() + (size_t)MS_NF * ns, 0.0f);
            for (int c = 0; c < ns; ++c) {
                mcb[t.mc_sens + (size_t)MS_LINK * ns + c] = (float)md->sensor_link[c];
                for (int q = 0; q < 3; ++q)
                    mcb[t.mc_sens + (size_t)(MS_X + q) * ns + c] = md->sensor_pos[3 * c + q];
            }
            auto put_ints = [&](const std::vector<int>& v) {
                pad4();
                const int at = (int)mcb.size();
                for (int x : v) { float f; std::memcpy(&f, &x, 4); mcb.push_back(f); }
                return at;
            };
            t.mc_chs = put_ints(chain_start); t.mc_chl = put_ints(chain_list);
            t.mc_dss = put_ints(desc_start); t.mc_dsl = put_ints(desc_list);
            std::vector<int> lim;
            for (int l = 1; l < L; ++l)
                if (md->lower[l] < md->upper[l]) lim.push_back(l - 1);
            t.nlimc = (int)lim.size();
            if (lim.empty()) lim.push_back(0);
            t.mc_lim = put_ints(lim);
            // self-collision geometry: per geom (link, p0, p1, radius) and the geom pairs;
            // global copies, and inside the LDS block when self-collision is on
            std::vector<float> geo((size_t)8 * std::max(1, md->num_geoms), 0.0f);
            for (int g = 0; g < md->num_geoms; ++g) {
                geo[8 * g] = (float)md->geom_link[g];
                for (int q = 0; q < 3; ++q) {
                    geo[8 * g + 1 + q] = md->geom_p0[3 * g + q];
                    geo[8 * g + 4 + q] = md->geom_p1[3 * g + q];
                }
                geo[8 * g + 7] = md->geom_radius[g];
            }
            std::vector<int> prs(md->pairs ? md->pairs : nullptr,
                                 md->pairs ? md->pairs + 2 * md->num_pairs : nullptr);
            if (prs.empty()) prs.assign(2, 0);
            t.mc_geo = t.mc_pairs = -1;
            if (self_on) {
                pad4();
                t.mc_geo = (int)mcb.size();
                mcb.insert(mcb.end(), geo.begin(), geo.begin() + 8 * md->num_geoms);
                // the pair table stays global (cache-resident, read once per substep by the
                // broad phase): its LDS room goes to W rows
            }
            pad4();
            t.mc_len = (int)mcb.size();
            t.npts = np; t.nsens = ns;
            UPW(g_mc, mcb);
            UPW(g_geo, geo); UPW(g_pairs, prs);
        }
#undef UPW
        auto al4 = [](int x) { return (x + 3) & ~3; };
        const bool ct = s->topo != 0;
        int so = 0;
        auto take = [&](int n) { const int at = so; so += al4(n); return at; };
        // Residency: the kernels' register budget allows TopoCT::kWaves waves per SIMD, i.e.
        // envs_cu = 4 kWaves resident envs per CU (Humanoid 8, Ant 16: all 4096 envs of a launch
        // in one round); the paired kernels hold 16 envs per CU (two per wave, 2 waves per SIMD).
        // E envs per workgroup share one copy of the constant block; each env's region
        // [s_R, s_total) gets the floats that leave envs_cu envs inside the CU's 160 KB.
        int waves = 2, lam_rows = 0;
        bool pair_ok = false;
        with_topo(s->topo, s->sp.tgs != 0, [&](auto T) {
            waves = decltype(T)::kWaves; lam_rows = decltype(T)::kLamRows;
            pair_ok = has_pair<decltype(T)>();
        });
        // paired kernels (mi_pair.hpp, two envs per wavefront, 16 per workgroup, 2 waves per
        // SIMD): the default for the compiled topologies (Humanoid 0.219 -> 0.205 ms, Ant 0.0765
        // -> 0.0589 ms against their one-env-per-wave kernels at 2 and 4 waves per SIMD; 4096
        // envs in one resident round either way); MI_WAVE_PAIR=0 selects one env per wave
        const char* pe = getenv("MI_WAVE_PAIR");
        const bool pair_want = pe ? atoi(pe) != 0 : true;
        s->pair = ct && pair_ok && N % 2 == 0 && pair_want;
        const int envs_cu = s->pair ? 16 : 4 * std::max(1, waves);
        t.envs_per_wg = s->pair ? 16 : (ct && waves >= 4 ? 4 : 1);
        if (const char* e = getenv("MI_WAVE_ENVS"); e && !s->pair) t.envs_per_wg = std::max(1, std::min(4, atoi(e)));
        const int E = t.envs_per_wg;
        const int env_budget = ((163840 / (int)sizeof(float)) / std::max(1, envs_cu / E) - al4(t.mc_len)) / E;
        const int R = m.max_rows;
        t.self_on = self_on ? 1 : 0;
        t.npairs = self_on ? md->num_pairs : 0;
        t.ncmax = std::min(m.npts + t.npairs, MI_MAX_ROWS / 3);
        const int C = t.ncmax;
        int lr = 0;   // CT path: published factor rows (each padded to 4) + 1/D (DofTree::lrow)
        for (int k = 0; k < m.nv; ++k) lr += (anc_start[k + 1] - anc_start[k] + 3) & ~3;
        bool overlay = false;
        int span0 = 0, span1 = 0, ro = 0;
        if (s->pair) {
            // paired layout: the persistent regions first, then the P1-P4 span whose dead space
            // takes the contact / row data and the W rows, which continue past the span up to
            // the env's share (one W segment); no J rows (rebuilt), no second W segment
            t.s_mc = take(t.mc_len);
            t.s_R = take(9 * L); t.s_o = take(3 * L); t.s_S = take(6 * m.nv);
            t.s_D = take(4); t.s_r = take(WNV); t.s_us = take(WNV); t.s_q = take(WNV); t.s_rp = take(8);
            t.s_xs = take(4);
            t.s_L = take(lr + m.nv);
            t.j_rows_lds = 0;
            t.s_J = take(4);
            t.s_lam = take(4);
            span0 = so;
            t.s_F = take(16 * L); t.s_Ic = take(4); t.s_M = take(m.nv * m.nv); t.s_X = take(16 * L);
            span1 = so;
            overlay = true;
            ro = span0;
            auto take_r = [&](int n) { const int at = ro; ro += al4(n); return at; };
            t.s_cp = take_r(3 * C); t.s_cl = take_r(C); t.s_cl2 = take_r(C); t.s_cn = take_r(3 * C);
            // no row-kind array: the paired kernels derive a row's kind from its index (contact
            // rows are (normal, friction, friction) triples, then the limit rows); its R floats
            // buy W rows (Humanoid: 28 -> 32 LDS rows, so the narrow PGS never reads the slab)
            t.s_rl = take_r(R); t.s_rb = take_r(R); t.s_rk = -1; t.s_ad = take_r(R);
            t.s_lsg = take_r(WNV);
            t.s_W = ro;
            int w = std::min(64, (t.s_R + env_budget - ro) / m.nv);
            while (w > 0 && ro + al4(w * m.nv) > t.s_R + env_budget) --w;
            w &= ~3;   // whole 4-row groups (mi_pair.hpp pw_idx: DOF-major inside a group)
            t.w_rows_lds = t.w_rows_a = std::max(0, w);
            const char* spe = getenv("MI_SENS_PAR");
            t.sens_par = (!spe || atoi(spe) != 0) && 6 * m.S * (C + 1) <= t.w_rows_lds * m.nv ? 1 : 0;
            t.s_W2 = 0;
            so = std::max(span1, ro + al4(t.w_rows_lds * m.nv));
        } else {
        t.s_mc = take(t.mc_len);
        t.s_R = take(9 * L); t.s_o = take(3 * L); t.s_S = take(6 * m.nv);
        // P1..P4 working span: link inertias / forces, M, aux (local transforms, composites).
        // On the compiled-topology path it is dead once P4 has moved M into registers, and
        // P8/P9 reuse it for the contact and row data and the first W rows.
        span0 = so;
        t.s_F = take(16 * L);   // per-link records: inertia (10) + Newton-Euler force (6)
        t.s_Ic = take(4);       // (kept for the layout order; records live at s_F)
        t.s_M = take(m.nv * m.nv);
        t.s_X = take(16 * L);
        span1 = so;
        t.s_D = take(ct ? 4 : WNV); t.s_r = take(WNV); t.s_us = take(WNV);
        t.s_q = take(WNV); t.s_rp = take(8);
        // contacts: ground points + self pairs, at most MI_MAX_ROWS / 3 in total
        const int rows_len = 8 * al4(C) + 4 * al4(R) + WNV;
        overlay = ct && rows_len <= span1 - span0;
        ro = overlay ? span0 : so;
        auto take_r = [&](int n) { const int at = ro; ro += al4(n); return at; };
        t.s_cp = take_r(3 * C); t.s_cl = take_r(C); t.s_cl2 = take_r(C); t.s_cn = take_r(3 * C);
        t.s_rl = take_r(R);
        t.s_rb = take_r(R); t.s_rk = take_r(R); t.s_ad = take_r(R); t.s_lsg = take_r(WNV);
        if (!overlay) so = ro;
        // lane-private solve vectors of the runtime-table solves (CT solves run in registers)
        t.s_xs = take(ct ? 4 : WNV * 64);
        t.s_L = take(ct ? lr + m.nv : 4);
        // Residency: the kernels' register budget allows TopoCT::kWaves waves per SIMD, i.e.
        // envs_cu = 4 kWaves resident envs per CU (Humanoid 8, Ant 16: all 4096 envs of a launch
        // in one round). E envs per workgroup share one copy of the constant block; each env's
        // region [s_R, s_total) gets the floats that leave envs_cu envs inside the CU's 160 KB.
        // CT path: J rows of the first constraint rows for the PGS; a 16-envs/CU budget keeps
        // the rows the Delassus-space sweeps use (kLamRows), the 8-envs/CU one up to 48; the
        // paired kernels rebuild J rows instead
        t.j_rows_lds = ct && !s->pair ? std::min(waves >= 4 ? lam_rows : 48, m.max_rows) : 0;
        t.s_J = take(t.j_rows_lds > 0 ? t.j_rows_lds * m.nv : 4);
        t.s_lam = take(4);
        // CT path: W rows for the P9 -> P10 hand-over. First choice: the rest of the dead
        // span; when that holds fewer rows than a one-bank PGS can use and the LDS budget of
        // the wave path (8 envs / CU, 20 KB each) has room, a dedicated region instead, so
        // the global slab is only the fallback of rare row-heavy substeps.
        // Otherwise, a second segment at the end takes whatever rows the budget still holds
        // (rows [w_rows_a, w_rows_lds) at s_W2).
        t.s_W = ro;
        t.w_rows_lds = overlay ? std::min(64, (span1 - ro) / m.nv) : 0;
        t.w_rows_a = t.w_rows_lds;
        t.s_W2 = 0;
        {
            const int want = std::min(64, m.max_rows);
            const int lds_budget_floats = t.s_R + env_budget;   // end of this env's share
            int fit = want;   // the most W rows a dedicated region can hold within the share
            while (fit > 0 && so + al4(fit * m.nv) > lds_budget_floats) --fit;
            if (ct && t.w_rows_lds < fit && (fit == want || !self_on || s->pair)) {
                t.s_W = take(fit * m.nv);
                t.w_rows_lds = t.w_rows_a = fit;
            } else if (ct && self_on && t.w_rows_lds < want && !s->pair) {   // (w_row<kSelf> on device)
                const int extra = std::min(want - t.w_rows_lds, (lds_budget_floats - so - 3) / m.nv);
                if (extra > 0) {
                    t.s_W2 = take(extra * m.nv);
                    t.w_rows_lds += extra;
                }
            }
        }
        }
        t.s_total = so;
        // E envs per workgroup share the constant block [0, s_env); env w's region is shifted
        // by w * env_stride
        t.s_env = t.s_R;
        t.env_stride = so - t.s_env;
        if (!s->pair) {   // the sequential regions strictly increase; the row data sits inside the dead
            // span (overlay) or between s_rp and s_xs
            const int offs[] = {t.s_mc, t.s_R, t.s_o, t.s_S, t.s_F, t.s_Ic, t.s_M, t.s_X,
                                t.s_D, t.s_r, t.s_us, t.s_q, t.s_rp, t.s_xs, t.s_L, t.s_J,
                                t.s_lam, t.s_total};
            for (size_t c = 1; c < sizeof(offs) / sizeof(offs[0]); ++c)
                if (offs[c] <= offs[c - 1]) return cleanup(fail(MI_E_STATE, "wave LDS layout: region %zu overlaps", c));
            const bool rows_ok = overlay ? (t.s_cp == span0 && ro <= span1)
                                         : (t.s_cp > t.s_rp && ro <= t.s_xs);
            if (!rows_ok) return cleanup(fail(MI_E_STATE, "wave LDS layout: row data misplaced"));
        }
        t.max_rows = m.max_rows;
        t.g_row_stride = (size_t)m.max_rows * WNV;
        // P8 self-collision scratch (segments + broad-phase survivors) in the same free span
        t.ngeoms = md->num_geoms;
        t.s_seg = -1; t.s_surv = -1;
        if (overlay && self_on && al4(12 * md->num_geoms) + al4(md->num_pairs) <= span1 - ro) {
            t.s_seg = ro;
            t.s_surv = ro + al4(12 * md->num_geoms);
        }
        s->lds_bytes = (size_t)(so + (t.envs_per_wg - 1) * t.env_stride) * sizeof(float);
        if (getenv("MI_SIM_DEBUG"))
            fprintf(stderr, "[mi_sim] wave layout: pair=%d envs/wg=%d lds/wg=%zu B env_stride=%d floats "
                            "mc=%d w_rows_lds=%d (a %d) j_rows_lds=%d s_seg=%d max_rows=%d ncmax=%d\n",
                    (int)s->pair, t.envs_per_wg, s->lds_bytes, t.env_stride, t.mc_len, t.w_rows_lds,
                    t.w_rows_a, t.j_rows_lds, t.s_seg, m.max_rows, t.ncmax);
        if (s->pair && ((self_on && t.s_seg < 0) || s->lds_bytes > 163840))
            return cleanup(fail(MI_E_STATE, "paired wave layout does not fit (%zu B of LDS per workgroup)",
                                s->lds_bytes));
        // the paired kernels' narrow PGS reads its W rows from LDS only (mi_pair.hpp WSrc)
        if (s->pair && t.w_rows_lds < lam_rows)
            return cleanup(fail(MI_E_STATE, "paired wave layout: %d LDS W rows < %d Delassus rows",
                                t.w_rows_lds, lam_rows));
    }
    s->lower.assign(md->lower, md->lower + L);
    s->upper.assign(md->upper, md->upper + L);
    // params
    s->sp.dt = prm->dt;
    for (int k = 0; k < 3; ++k) s->sp.g[k] = prm->gravity[k];
    if (prm->solver_type != MI_SOLVER_PGS && prm->solver_type != MI_SOLVER_TGS)
        return cleanup(fail(MI_E_ARG, "solver_type %d: this build implements 0 (PGS) and 1 (TGS)",
                            prm->solver_type));
    if (prm->solver_iterations < 1 || prm->solver_iterations > 64 || prm->velocity_iterations < 0 ||
        prm->velocity_iterations > 64)
        return cleanup(fail(MI_E_ARG, "solver iterations %d / velocity iterations %d out of range",
                            prm->solver_iterations, prm->velocity_iterations));
    s->sp.iters = prm->solver_iterations;
    s->sp.tgs = prm->solver_type == MI_SOLVER_TGS ? 1 : 0;
    s->sp.viters = s->sp.tgs ? prm->velocity_iterations : 0;
    s->sp.h = s->sp.tgs ? prm->dt / (float)prm->solver_iterations : prm->dt;
    s->sp.contact_offset = prm->contact_offset;
    s->sp.rest_offset = prm->rest_offset;
    s->sp.friction = prm->friction;
    s->sp.max_depen = prm->max_depenetration_velocity;
    s->sp.erp = prm->erp;
    s->sp.max_angvel = prm->max_angular_velocity;
    s->sp.ang_damp = prm->angular_damping;
    if (!(prm->angular_damping >= 0.0f)) return cleanup(fail(MI_E_ARG, "angular_damping must be >= 0"));
    // state
    DevState& st = s->ds;
    st.N = N;
    st.off = off;
    st.seed = seed;
    const int D = m.D > 0 ? m.D : 1, S = m.S > 0 ? m.S : 1;
    void* p = nullptr;
#define AL(field, T, cnt) if ((rc = dev_alloc(s, &p, sizeof(T) * (size_t)(cnt)))) return cleanup(rc); st.field = (T*)p
    if (s->wave) {
        // one record per env: pos 3, quat 4, vel 6, q D, qd D, eff D, padded to whole 128-B
        // lines (the wave touches only its own lines, each access coalesced); the sensor
        // wrenches in a [N][6S] array of their own (DevState::sfs / ses)
        const int rec = (13 + 3 * D + 31) & ~31;
        float* r = nullptr;
        if ((rc = dev_alloc(s, &p, sizeof(float) * (size_t)rec * N))) return cleanup(rc);
        r = (float*)p;
        st.fs = 1; st.es = rec;
        st.root_pos = r; st.root_quat = r + 3; st.root_vel = r + 7; st.q = r + 13;
        st.qd = r + 13 + D; st.eff = r + 13 + 2 * D;
        AL(sens, float, (size_t)6 * S * N);
        st.sfs = 1; st.ses = 6 * S;
    } else {
        st.fs = N; st.es = 1;
        AL(root_pos, float, 3 * N); AL(root_quat, float, 4 * N); AL(root_vel, float, 6 * N);
        AL(q, float, (size_t)D * N); AL(qd, float, (size_t)D * N); AL(eff, float, (size_t)D * N);
        AL(sens, float, (size_t)6 * S * N);
        st.sfs = N; st.ses = 1;
    }
    AL(reset_count, uint32_t, N); AL(nan_flag, int32_t, N); AL(dr_state, uint32_t, (size_t)6 * N);
    AL(load, int32_t, N);
    {   // MI_PAIR_LOAD=0: the paired kernels keep the index pairing (A/B); MI_PAIR_LOAD_MIN: a
        // workgroup is re-paired only when one of its envs had more constraint rows than this
        const char* e = getenv("MI_PAIR_LOAD");
        const char* mn = getenv("MI_PAIR_LOAD_MIN");
        // (A/B, round 5: 0 -> 0.1174 ms, 18 -> 0.1177, 24 -> 0.1187, 30 -> 0.1219, off 0.1245)
        const int minrows = mn ? atoi(mn) : 0;
        st.pair_by_load = (e && atoi(e) == 0) ? 0 : 1 + (minrows > 0 ? minrows : 0);

    }
    AL(nan_total, unsigned long long, 1);
    if (s->wave) {
        if ((rc = dev_alloc(s, &p, sizeof(float) * (size_t)N * s->wt.g_row_stride))) return cleanup(rc);
        s->rows = (float*)p;
        s->wt.g_wa = nullptr;
        if (s->pair) {   // wide-PGS scratch: kWideScratchRows x 64 lanes per wave (mi_pair.hpp)
            const size_t nb = sizeof(float) * (size_t)(N / 2) * 64 * (size_t)(kWideScratchRows > 0 ? kWideScratchRows : 1);
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && nb > fr)
                return cleanup(fail(MI_E_ARG, "%d envs: the wide-PGS scratch needs %.1f MB (%d B per env), "
                                              "%.1f MB of device memory free", N, nb / 1e6,
                                    (int)(nb / (size_t)N), fr / 1e6));
            if ((rc = dev_alloc(s, &p, nb))) return cleanup(rc);
            s->wt.g_wa = (float*)p;
        }
        AL(ws, float, 64);
    } else {
        AL(ws, float, (size_t)((N + 63) / 64) * 64 * (m.slots > 0 ? m.slots : 1));
    }
#undef AL
    std::vector<float> org((size_t)3 * N);
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) org[(size_t)k * N + i] = env_origins[(size_t)3 * i + k];
    const float* od = nullptr;
    if ((rc = upload(s, org.data(), org.size(), &od))) return cleanup(rc);
    st.origins = od;
    hipLaunchKernelGGL(k_init_state, grid_for(s, N), dim3(s->block), 0, 0, st, m.D);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return cleanup(fail(MI_E_HIP, "init: %s", hipGetErrorString(e)));
    if ((rc = sync_kparams(s))) return cleanup(rc);
    if (s->wave && s->lds_bytes > 64 * 1024) {   // above the default dynamic-LDS limit
        hipError_t e1 = hipSuccess, e2 = hipSuccess;
        with_topo(s->topo, s->sp.tgs != 0, [&](auto T) {
            if constexpr (has_pair<decltype(T)>()) {
                if (s->pair) {
                    e1 = hipFuncSetAttribute((const void*)k_env_step_pair<decltype(T)>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->lds_bytes);
                    e2 = hipFuncSetAttribute((const void*)k_sim_step_pair<decltype(T)>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->lds_bytes);
                    return;
                }
            }
            e1 = hipFuncSetAttribute((const void*)k_env_step_wave<decltype(T)>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->lds_bytes);
            e2 = hipFuncSetAttribute((const void*)k_sim_step_wave<decltype(T)>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->lds_bytes);
        });
        if (e1 != hipSuccess || e2 != hipSuccess)
            return cleanup(fail(MI_E_HIP, "wave kernels: %zu B of LDS per workgroup refused", s->lds_bytes));
    }
    *out = s;
    return MI_OK;
}

int mi_sim_destroy(mi_sim* s) {
    if (!s) return MI_OK;
    (void)hipSetDevice(s->device);
    // deferred substeps are issued, not dropped (their state is about to be freed, but a
    // mirror or a caller's event may still order after them), then everything drains
    if (s->pending) (void)flush_pending(s, s->pending_stream);
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : s->tev) (void)hipEventDestroy(e);
    if (s->pending_ev) (void)hipEventDestroy(s->pending_ev);
    if (s->mir_ev) (void)hipEventDestroy(s->mir_ev);
    if (s->rd_ev) (void)hipEventDestroy(s->rd_ev);
    for (void* p : s->allocs) (void)hipFree(p);
    delete s;
    return MI_OK;
}

int mi_sim_info(const mi_sim* s, int32_t* num_envs, int32_t* num_dof, int32_t* num_links,
                int32_t* num_sensors, float* dof_limits) {
    if (!s) return fail(MI_E_NULL, "null sim");
    if (num_envs) *num_envs = s->N;
    if (num_dof) *num_dof = s->dm.D;
    if (num_links) *num_links = s->dm.L;
    if (num_sensors) *num_sensors = s->dm.S;
    if (dof_limits)
        for (int j = 0; j < s->dm.D; ++j) {
            dof_limits[2 * j] = s->lower[j + 1];
            dof_limits[2 * j + 1] = s->upper[j + 1];
        }
    return MI_OK;
}

#define STREAM(x) ((hipStream_t)(x))
#define NEED(p) if (!(p)) return fail(MI_E_NULL, "%s: null %s", __func__, #p)

static bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Before a launch on `w` overwrites the state mirrors: reads of them queued on another stream
// (a getter called there, then torch's copies of the handed-out tensor) must finish first. The
// host enqueued those reads before this call, so an event recorded on the reader's stream now
// covers them.
static int order_mirror_write(mi_sim* s, hipStream_t w) {
    hipStream_t r = s->mir_reader;
    s->mir_reader = nullptr;
    if (!r || r == w || capturing(r) || capturing(w)) return MI_OK;
    if (!s->rd_ev) HIP_TRY(hipEventCreateWithFlags(&s->rd_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s->rd_ev, r));
    HIP_TRY(hipStreamWaitEvent(w, s->rd_ev, 0));
    return MI_OK;
}

// After a launch on `w` wrote the mirrors: valid in stream order, with an event for readers on
// other streams. Under stream capture nothing has run yet (and an event recorded at capture
// time is not re-recorded by a replay), so the mirrors are left invalid: the next getter
// refreshes them on its own stream.
static int publish_mirrors(mi_sim* s, hipStream_t w) {
    if (capturing(w)) {
        s->mir_valid = false;
        s->mir_stream = nullptr;
        return MI_OK;
    }
    if (!s->mir_ev) HIP_TRY(hipEventCreateWithFlags(&s->mir_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s->mir_ev, w));
    s->mir_stream = w;
    s->mir_valid = true;
    return MI_OK;
}

static int launch_sim(mi_sim* s, int substeps, hipStream_t stream) {
    s->mir_valid = false;
    // the paired kernel refreshes the mirrors itself (free-root models: the state it writes is
    // the mirrors' whole content)
    const bool mirrored = s->wave && s->pair && s->mir[0] && s->dm.nr == 6 && (s->dm.S == 0 || s->mir[5]);
    if (mirrored)
        if (int rc = order_mirror_write(s, stream)) return rc;
    if (s->wave)
        with_topo(s->topo, s->sp.tgs != 0, [&](auto T) {
            if constexpr (has_pair<decltype(T)>()) {
                if (s->pair) {
                    Mirrors mir{};
                    if (mirrored)
                        for (int k = 0; k < 6; ++k) mir.p[k] = s->mir[k];
                    hipLaunchKernelGGL(k_sim_step_pair<decltype(T)>, wave_grid(s), wave_block(s), s->lds_bytes,
                                       stream, (const KParams*)s->kp_dev, substeps, mir);
                    return;
                }
            }
            hipLaunchKernelGGL(k_sim_step_wave<decltype(T)>, wave_grid(s), wave_block(s), s->lds_bytes,
                               stream, (const KParams*)s->kp_dev, substeps);
        });
    else
        hipLaunchKernelGGL(k_sim_step, grid_for(s, s->N), dim3(s->block), 0, stream, s->dm, s->ds,
                           s->sp, substeps);
    LAUNCH_CHECK();
    if (mirrored) return publish_mirrors(s, stream);   // valid after this launch (mi_get_state_mirror)
    return MI_OK;
}


// Issue the substeps mi_sim_step deferred, on the stream they were requested on; a caller on
// another stream waits for them. Substeps requested before a stream capture began cannot be
// issued into it: that is refused loudly (call the step inside the capture, or synchronise).
static int flush_pending(mi_sim* s, void* stream) {
    if (s->pending == 0) return MI_OK;
    const int k = s->pending;
    hipStream_t ps = s->pending_stream;
    if (capturing(ps) || (stream && capturing(STREAM(stream))))
        return fail(MI_E_STATE, "%d physics substep(s) requested before a stream capture began are "
                                "still pending: synchronise before capturing", k);
    s->pending = 0;
    HIP_TRY(hipSetDevice(s->device));
    int rc = launch_sim(s, k, ps);
    if (rc) return rc;
    if (STREAM(stream) != ps) {
        if (!s->pending_ev) HIP_TRY(hipEventCreateWithFlags(&s->pending_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->pending_ev, ps));
        HIP_TRY(hipStreamWaitEvent(STREAM(stream), s->pending_ev, 0));
    }
    return MI_OK;
}
#define FLUSH(s, stream) do { int rc_ = flush_pending((s), (stream)); if (rc_) return rc_; } while (0)

static int gather_fields(mi_sim* s, GFields f, int nf, void* stream) {
    if (nf == 0) return MI_OK;
    dim3 g = gather_grid(s->N);
    g.y = (unsigned)nf;
    hipLaunchKernelGGL(k_soa_to_rows_multi, g, dim3(256), 0, STREAM(stream), f, s->N);
    LAUNCH_CHECK();
    return MI_OK;
}

extern "C++" template <typename IDX>
static int scatter_fields(mi_sim* s, GFields f, int nf, int n, const IDX* idx, void* stream) {
    if (nf == 0 || n == 0) return MI_OK;
    int cmax = 0;
    for (int k = 0; k < nf; ++k) cmax = std::max(cmax, f.f[k].C);
    dim3 g = scatter_grid(n, cmax);
    g.y = (unsigned)nf;
    hipLaunchKernelGGL(k_rows_to_soa_multi<IDX>, g, dim3(256), 0, STREAM(stream), f, n, idx, s->N,
                       s->ds.fs, s->ds.es);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_get_root_state(mi_sim* s, float* pos, float* quat, float* vel, void* stream) {
    NEED(s);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    GFields f{};
    int nf = 0;
    const int fs = s->ds.fs, es = s->ds.es;
    if (pos) f.f[nf++] = {s->ds.root_pos, pos, 3, fs, es};
    if (quat) f.f[nf++] = {s->ds.root_quat, quat, 4, fs, es};
    if (vel) f.f[nf++] = {s->ds.root_vel, vel, 6, fs, es};
    return gather_fields(s, f, nf, stream);
}

int mi_get_dof_state(mi_sim* s, float* q, float* qd, void* stream) {
    NEED(s);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    GFields f{};
    int nf = 0;
    const int fs = s->ds.fs, es = s->ds.es;
    if (q) f.f[nf++] = {s->ds.q, q, s->dm.D, fs, es};
    if (qd) f.f[nf++] = {s->ds.qd, qd, s->dm.D, fs, es};
    return gather_fields(s, f, nf, stream);
}

int mi_get_sensor_wrench(mi_sim* s, float* out, void* stream) {
    NEED(s); NEED(out);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    if (s->dm.S == 0) return MI_OK;
    GFields f{};
    f.f[0] = {s->ds.sens, out, 6 * s->dm.S, s->ds.sfs, s->ds.ses};
    return gather_fields(s, f, 1, stream);
}

int mi_set_dof_efforts(mi_sim* s, const float* eff, const int32_t* idx, int32_t n, void* stream) {
    NEED(s); NEED(eff);
    if (n < 0 || n > s->N || (!idx && n != s->N)) return fail(MI_E_SHAPE, "mi_set_dof_efforts: bad n=%d", n);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    GFields f{};
    f.f[0] = {eff, s->ds.eff, s->dm.D};
    return scatter_fields<int32_t>(s, f, 1, n, idx, stream);
}

extern "C++" template <typename IDX>
static int set_dof_state(mi_sim* s, const float* q, const float* qd, const IDX* idx, int32_t n, void* stream) {
    NEED(s);
    if (n < 0 || n > s->N || (!idx && n != s->N)) return fail(MI_E_SHAPE, "mi_set_dof_state: bad n=%d", n);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    GFields f{};
    int nf = 0;
    if (q) f.f[nf++] = {q, s->ds.q, s->dm.D};
    if (qd) f.f[nf++] = {qd, s->ds.qd, s->dm.D};
    if (nf && n) s->mir_valid = false;
    return scatter_fields<IDX>(s, f, nf, n, idx, stream);
}

extern "C++" template <typename IDX>
static int set_root_state(mi_sim* s, const float* pos, const float* quat, const float* vel, const IDX* idx,
                          int32_t n, void* stream) {
    NEED(s);
    if (n < 0 || n > s->N || (!idx && n != s->N)) return fail(MI_E_SHAPE, "mi_set_root_state: bad n=%d", n);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    GFields f{};
    int nf = 0;
    if (pos) f.f[nf++] = {pos, s->ds.root_pos, 3};
    if (quat) f.f[nf++] = {quat, s->ds.root_quat, 4};
    if (vel) f.f[nf++] = {vel, s->ds.root_vel, 6};
    if (nf && n) s->mir_valid = false;
    return scatter_fields<IDX>(s, f, nf, n, idx, stream);
}

int mi_set_dof_state(mi_sim* s, const float* q, const float* qd, const int64_t* idx, int32_t n,
                     void* stream) {
    return set_dof_state<int64_t>(s, q, qd, idx, n, stream);
}
int mi_set_dof_state_i32(mi_sim* s, const float* q, const float* qd, const int32_t* idx, int32_t n,
                         void* stream) {
    return set_dof_state<int32_t>(s, q, qd, idx, n, stream);
}
int mi_set_root_state(mi_sim* s, const float* pos, const float* quat, const float* vel,
                      const int64_t* idx, int32_t n, void* stream) {
    return set_root_state<int64_t>(s, pos, quat, vel, idx, n, stream);
}
int mi_set_root_state_i32(mi_sim* s, const float* pos, const float* quat, const float* vel,
                          const int32_t* idx, int32_t n, void* stream) {
    return set_root_state<int32_t>(s, pos, quat, vel, idx, n, stream);
}

int mi_sim_set_mirror(mi_sim* s, float* pos, float* quat, float* vel, float* q, float* qd, float* sens) {
    NEED(s);
    float* m[6] = {pos, quat, vel, q, qd, sens};
    int set = 0;
    for (int k = 0; k < 6; ++k) set += m[k] != nullptr;
    if (s->dm.S == 0 && !sens && set == 5) ++set;          // no sensors: no sensor mirror needed
    if (set != 0 && set != 6) return fail(MI_E_NULL, "mi_sim_set_mirror: register all six mirrors or none");
    for (int k = 0; k < 6; ++k) s->mir[k] = m[k];
    s->mir_valid = false;
    return MI_OK;
}

int mi_get_state_mirror(mi_sim* s, void* stream) {
    NEED(s);
    if (!s->mir[0]) return fail(MI_E_STATE, "mi_get_state_mirror: no mirrors registered (mi_sim_set_mirror)");
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    if (s->mir_valid) {
        if (STREAM(stream) != s->mir_stream) {  // the refresh ran on another stream: order after it
            HIP_TRY(hipStreamWaitEvent(STREAM(stream), s->mir_ev, 0));
            s->mir_reader = STREAM(stream);     // and the next mirror write after this reader
        }
        return MI_OK;
    }
    if (int rc = order_mirror_write(s, STREAM(stream))) return rc;
    GFields f{};
    int nf = 0;
    const int fs = s->ds.fs, es = s->ds.es;
    f.f[nf++] = {s->ds.root_pos, s->mir[0], 3, fs, es};
    f.f[nf++] = {s->ds.root_quat, s->mir[1], 4, fs, es};
    f.f[nf++] = {s->ds.root_vel, s->mir[2], 6, fs, es};
    f.f[nf++] = {s->ds.q, s->mir[3], s->dm.D, fs, es};
    f.f[nf++] = {s->ds.qd, s->mir[4], s->dm.D, fs, es};
    if (s->dm.S > 0) f.f[nf++] = {s->ds.sens, s->mir[5], 6 * s->dm.S, s->ds.sfs, s->ds.ses};
    const int rc = gather_fields(s, f, nf, stream);
    if (rc) return rc;
    return publish_mirrors(s, STREAM(stream));
}

int mi_sim_step(mi_sim* s, int32_t substeps, void* stream) {
    NEED(s);
    if (substeps < 0 || substeps > 64) return fail(MI_E_ARG, "substeps %d out of range", substeps);
    if (substeps == 0) return MI_OK;
    HIP_TRY(hipSetDevice(s->device));
    // deferred: consecutive steps on one stream with nothing reading or writing the state in
    // between are issued as one launch (identical results: later substeps of a launch continue
    // from the LDS copy of exactly the state a separate launch would reload); inside a stream
    // capture, and with MI_SIM_DEFER=0, every call launches at once
    if (!s->defer || capturing(STREAM(stream))) {
        FLUSH(s, stream);
        return launch_sim(s, substeps, STREAM(stream));
    }
    if (s->pending && (s->pending_stream != STREAM(stream) || s->pending + substeps > 64))
        FLUSH(s, stream);                  // one launch never carries more than 64 substeps
    s->pending += substeps;
    s->pending_stream = STREAM(stream);
    if (s->pending == 64) FLUSH(s, stream);
    return MI_OK;
}

int mi_sim_flush(mi_sim* s, void* stream) {
    NEED(s);
    FLUSH(s, stream);
    return MI_OK;
}

int mi_task_configure(mi_sim* s, const mi_task_params* t) {
    NEED(s); NEED(t);
    if (t->task_kind < MI_TASK_CARTPOLE || t->task_kind > MI_TASK_HUMANOID)
        return fail(MI_E_ARG, "bad task_kind %d", t->task_kind);
    const int D = s->dm.D;
    if (t->task_kind == MI_TASK_CARTPOLE) {
        if (s->dm.dyn != MI_DYN_CARTPOLE) return fail(MI_E_ARG, "cartpole task needs cart-pole dynamics");
        if (t->num_actions != 1 || t->num_obs != 4) return fail(MI_E_SHAPE, "cartpole: A=1, O=4");
    } else {
        if (s->dm.dyn != MI_DYN_ARTICULATION || !s->dm.root_free)
            return fail(MI_E_ARG, "locomotion needs a floating-base articulation");
        if (t->num_actions != D) return fail(MI_E_SHAPE, "locomotion: num_actions %d != num_dof %d", t->num_actions, D);
        if (t->num_obs != 12 + 3 * D + 6 * s->dm.S)
            return fail(MI_E_SHAPE, "locomotion: num_obs %d != 12+3D+6S = %d", t->num_obs, 12 + 3 * D + 6 * s->dm.S);
        if (!t->joint_gears || !t->motor_effort_ratio) return fail(MI_E_NULL, "gears / effort ratio required");
    }
    DevTask& d = s->tp;
    d = DevTask{};
    d.kind = t->task_kind; d.O = t->num_obs; d.A = t->num_actions;
    d.clip_actions = t->clip_actions; d.clip_obs = t->clip_obs;
    d.max_episode_length = t->max_episode_length;
    d.power_scale = t->power_scale; d.heading_weight = t->heading_weight; d.up_weight = t->up_weight;
    d.actions_cost = t->actions_cost; d.energy_cost = t->energy_cost;
    d.dof_vel_scale = t->dof_vel_scale; d.angular_velocity_scale = t->angular_velocity_scale;
    d.contact_force_scale = t->contact_force_scale; d.joints_at_limit_cost = t->joints_at_limit_cost;
    d.death_cost = t->death_cost; d.termination_height = t->termination_height;
    d.alive_reward_scale = t->alive_reward_scale; d.task_dt = t->task_dt;
    for (int k = 0; k < 3; ++k) { d.target[k] = t->target[k]; d.init_root_pos[k] = t->init_root_pos[k]; }
    for (int k = 0; k < 4; ++k) d.init_root_quat[k] = t->init_root_quat[k];
    d.dof_pos_noise = t->dof_pos_noise; d.dof_vel_noise = t->dof_vel_noise;
    d.reset_dist = t->reset_dist; d.max_push_effort = t->max_push_effort;
    for (int j = 0; j < t->num_actions && j < MI_MAXA; ++j) {
        d.gears[j] = t->joint_gears ? t->joint_gears[j] : 1.0f;
        d.ratio[j] = t->motor_effort_ratio ? t->motor_effort_ratio[j] : 1.0f;
    }
    for (int j = 0; j < D && j < MI_MAXA; ++j) d.init_dof[j] = t->init_dof_pos ? t->init_dof_pos[j] : 0.0f;
    s->task_ok = true;
    if (int rc = sync_kparams(s)) return rc;
    return MI_OK;
}

#define NEED_TASK(s) if (!(s)->task_ok) return fail(MI_E_STATE, "%s: mi_task_configure not called", __func__)

int mi_task_pre_step(mi_sim* s, const float* actions, int64_t* reset_buf, int64_t* progress_buf,
                     float* potentials, float* prev_potentials, float* actions_out, void* stream) {
    NEED(s); NEED_TASK(s); NEED(actions); NEED(reset_buf); NEED(progress_buf);
    if (s->tp.kind != MI_TASK_CARTPOLE) { NEED(potentials); NEED(prev_potentials); }
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    s->mir_valid = false;   // the mask-driven resets write the state
    hipLaunchKernelGGL(k_pre_step, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->dm,
                       s->ds, s->tp, actions, reset_buf, progress_buf, potentials, prev_potentials,
                       actions_out);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_task_reset_idx(mi_sim* s, const int64_t* env_ids, int32_t n, int64_t* reset_buf,
                      int64_t* progress_buf, float* potentials, float* prev_potentials, void* stream) {
    NEED(s); NEED_TASK(s);
    if (n < 0 || n > s->N || (!env_ids && n != s->N)) return fail(MI_E_SHAPE, "mi_task_reset_idx: bad n=%d", n);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    if (n == 0) return MI_OK;
    s->mir_valid = false;
    hipLaunchKernelGGL(k_reset_idx, grid_for(s, n), dim3(s->block), 0, STREAM(stream), s->dm, s->ds,
                       s->tp, env_ids, n, reset_buf, progress_buf, potentials, prev_potentials);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_task_post_step(mi_sim* s, const float* actions, float* obs, float* rew, int64_t* reset_buf,
                      int64_t* progress_buf, float* potentials, float* prev_potentials, void* stream) {
    NEED(s); NEED_TASK(s); NEED(obs); NEED(rew); NEED(reset_buf); NEED(progress_buf);
    if (s->tp.kind != MI_TASK_CARTPOLE) { NEED(actions); NEED(potentials); NEED(prev_potentials); }
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    int var = post_tile_variant();
    if (var == 4 || var == 6) {   // 32p / 16p: several tiles per resident workgroup, next tile's loads in flight
        const int es = s->ds.es, ns = 6 * s->dm.S;
        const int pte = var == 6 ? 16 : 32;
        const size_t tile = post_pipe_lds(es, s->tp.A, s->tp.O, s->dm.D, s->dm.S, pte);
        const PipeGeo pg = pipe_geo(es, s->dm.D, s->dm.S);
        // shipped (TE, NR4, NS4) instantiations: Humanoid (32, 7, 2) / (16, 4, 1), Ant (32, 4, 3) /
        // (16, 2, 2); other models take the one-tile kernel
        const int nr4 = pipe_nr4(pg.ne4, pte), ns4 = pipe_ns4(pg.ns4, pte);
        const int combo = pte == 32 ? ((nr4 == 7 && ns4 == 2) ? 1 : (nr4 == 4 && ns4 == 3) ? 2 : 0)
                                    : ((nr4 == 4 && ns4 == 1) ? 3 : (nr4 == 2 && ns4 == 2) ? 4 : 0);
        if (s->tp.kind != MI_TASK_CARTPOLE && s->wave && s->kp_dev && s->ds.fs == 1 && es % 32 == 0 &&
            s->ds.sfs == 1 && s->ds.ses == ns && ns % 4 == 0 && combo &&
            s->tp.A >= 1 && s->tp.A <= 32 && s->dm.D >= 1 && s->dm.D <= 64 &&
            ns <= 64 && tile <= 64 * 1024 && s->tp.O >= 4 && (((uintptr_t)obs) & 15) == 0 &&
            (pte * s->tp.O + 255) / 256 <= (combo == 1 ? 11 : combo == 2 ? 8 : combo == 3 ? 6 : 4)) {
            if (s->num_cu <= 0)
                HIP_TRY(hipDeviceGetAttribute(&s->num_cu, hipDeviceAttributeMultiprocessorCount, s->device));
            const int ntiles = (s->N + pte - 1) / pte;
            const void* fn = combo == 1 ? (const void*)k_loco_post_pipe<32, 7, 2, 11>
                           : combo == 2 ? (const void*)k_loco_post_pipe<32, 4, 3, 8>
                           : combo == 3 ? (const void*)k_loco_post_pipe<16, 4, 1, 6>
                                        : (const void*)k_loco_post_pipe<16, 2, 2, 4>;
            // one resident round: workgroups per CU as registers and LDS allow together
            int per_cu = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, tile));
            int grid = std::min(ntiles, s->num_cu * std::max(1, per_cu));
            const char* g = getenv("MI_POST_GRID");
            if (g) grid = std::max(1, std::min(grid, atoi(g)));
            // with one tile per resident workgroup there is nothing to overlap: the one-tile
            // kernel. Crossover: MI_POST_PIPE_MIN tiles per workgroup (default 2).
            const char* pm = getenv("MI_POST_PIPE_MIN");   // tiles per workgroup (tuning)
            if (!g && ntiles < (pm ? atoi(pm) : 2) * grid) goto one_tile;
            const KParams* kp = (const KParams*)s->kp_dev;
            hipEvent_t ev0 = nullptr, ev1 = nullptr;
            HIP_TRY(timed_launch(s, stream, &ev0, &ev1));
#define POST_PIPE(T, R, Q, W) do { if (ev0) hipExtLaunchKernelGGL((k_loco_post_pipe<T, R, Q, W>), dim3(grid), dim3(64), (uint32_t)tile, \
            STREAM(stream), ev0, ev1, 0, kp, actions, obs, rew, reset_buf, progress_buf, potentials, prev_potentials); \
            else hipLaunchKernelGGL((k_loco_post_pipe<T, R, Q, W>), dim3(grid), dim3(64), tile, STREAM(stream), kp, \
            actions, obs, rew, reset_buf, progress_buf, potentials, prev_potentials); } while (0)
            switch (combo) {
                case 1: POST_PIPE(32, 7, 2, 11); break;
                case 2: POST_PIPE(32, 4, 3, 8); break;
                case 3: POST_PIPE(16, 4, 1, 6); break;
                default: POST_PIPE(16, 2, 2, 4); break;
            }
#undef POST_PIPE
            LAUNCH_CHECK();
            s->post_kernel = var; s->post_grid = grid;
            return MI_OK;
        }
    one_tile:
        var = 2;      // shapes / sizes the pipelined kernel does not take: the one-tile kernel
    }
    const int te = var < 2 ? 64 : 32;
    const bool stage = (var & 1) == 0;
    const size_t tile = post_tile_lds(te, stage, s->ds.es, s->tp.A, s->tp.O, s->dm.D, s->dm.S);
    if (s->tp.kind != MI_TASK_CARTPOLE && s->ds.fs == 1 && tile <= 64 * 1024) {
        const dim3 g((s->N + te - 1) / te);
        hipEvent_t ev0 = nullptr, ev1 = nullptr;
        HIP_TRY(timed_launch(s, stream, &ev0, &ev1));
#define POST_TILED(TE, ST) do { if (ev0) hipExtLaunchKernelGGL((k_loco_post_tiled<TE, ST>), g, dim3(64), (uint32_t)tile, \
            STREAM(stream), ev0, ev1, 0, s->dm, s->ds, s->tp, actions, obs, rew, reset_buf, progress_buf, potentials, \
            prev_potentials); \
            else hipLaunchKernelGGL((k_loco_post_tiled<TE, ST>), g, dim3(64), tile, STREAM(stream), \
            s->dm, s->ds, s->tp, actions, obs, rew, reset_buf, progress_buf, potentials, prev_potentials); } while (0)
        switch (var) {
            case 0: POST_TILED(64, true); break;
            case 1: POST_TILED(64, false); break;
            case 2: POST_TILED(32, true); break;
            default: POST_TILED(32, false); break;
        }
#undef POST_TILED
        s->post_kernel = var; s->post_grid = (int)g.x;
    } else {
        hipLaunchKernelGGL(k_post_step, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->dm,
                           s->ds, s->tp, actions, obs, rew, reset_buf, progress_buf, potentials,
                           prev_potentials);
        s->post_kernel = 5; s->post_grid = (int)grid_for(s, s->N).x;
    }
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_task_post_kernel(const mi_sim* s, int32_t* kernel, int32_t* grid) {
    NEED(s);
    if (kernel) *kernel = s->post_kernel;
    if (grid) *grid = s->post_grid;
    return MI_OK;
}

int mi_task_observations(mi_sim* s, const float* actions, float* obs, float* potentials,
                         float* prev_potentials, void* stream) {
    NEED(s); NEED_TASK(s); NEED(obs);
    if (s->tp.kind != MI_TASK_CARTPOLE) { NEED(actions); NEED(potentials); NEED(prev_potentials); }
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    hipLaunchKernelGGL(k_observations, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->dm,
                       s->ds, s->tp, actions, obs, potentials, prev_potentials);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_task_metrics(mi_sim* s, const float* actions, const float* obs, float* rew,
                    const float* potentials, const float* prev_potentials, void* stream) {
    NEED(s); NEED_TASK(s); NEED(obs); NEED(rew);
    if (s->tp.kind != MI_TASK_CARTPOLE) { NEED(actions); NEED(potentials); NEED(prev_potentials); }
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    hipLaunchKernelGGL(k_metrics, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->dm,
                       s->ds, s->tp, actions, obs, rew, potentials, prev_potentials);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_task_is_done(mi_sim* s, const float* obs, int64_t* reset_buf, const int64_t* progress_buf,
                    void* stream) {
    NEED(s); NEED_TASK(s); NEED(obs); NEED(reset_buf); NEED(progress_buf);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    hipLaunchKernelGGL(k_is_done, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->ds,
                       s->tp, obs, reset_buf, progress_buf);
    LAUNCH_CHECK();
    return MI_OK;
}

// Timed launch (mi_sim_time_launches): the event pair of this launch, or nulls. The events ride on
// the kernel's own dispatch (hipExtLaunchKernelGGL); launches into a capturing stream are not timed.
static hipError_t timed_launch(mi_sim* s, void* stream, hipEvent_t* ev0, hipEvent_t* ev1) {
    *ev0 = *ev1 = nullptr;
    if (s->tev_every > 0 && s->tev_rec < (int)s->tev.size() / 2 && (s->tev_seen++ % s->tev_every) == 0) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const hipError_t e = hipStreamIsCapturing(STREAM(stream), &cs);
        if (e != hipSuccess) return e;
        if (cs == hipStreamCaptureStatusNone) {
            *ev0 = s->tev[2 * s->tev_rec];
            *ev1 = s->tev[2 * s->tev_rec + 1];
            ++s->tev_rec;
        }
    }
    return hipSuccess;
}

int mi_env_step(mi_sim* s, const float* actions, int32_t substeps, float* obs_out, float* obs_task,
                float* rew, int64_t* reset_buf, int64_t* progress_buf, float* potentials,
                float* prev_potentials, float* actions_out, float* rew_out, int64_t* reset_out,
                void* stream) {
    NEED(s); NEED_TASK(s); NEED(actions); NEED(obs_out); NEED(rew); NEED(reset_buf); NEED(progress_buf);
    if (s->tp.kind != MI_TASK_CARTPOLE) { NEED(potentials); NEED(prev_potentials); }
    if (s->tp.dr_act && s->tp.kind != MI_TASK_CARTPOLE && !actions_out)
        return fail(MI_E_NULL, "mi_env_step: action DR needs actions_out (task.actions)");
    if (substeps < 0 || substeps > 64) return fail(MI_E_ARG, "substeps %d out of range", substeps);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, stream);
    s->mir_valid = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    HIP_TRY(timed_launch(s, stream, &ev0, &ev1));
    if (s->wave && s->tp.kind != MI_TASK_CARTPOLE)
        with_topo(s->topo, s->sp.tgs != 0, [&](auto T) {
            if constexpr (has_pair<decltype(T)>()) {
                if (s->pair) {
                    if (ev0)
                        hipExtLaunchKernelGGL(k_env_step_pair<decltype(T)>, wave_grid(s), wave_block(s),
                                              (uint32_t)s->lds_bytes, STREAM(stream), ev0, ev1, 0,
                                              (const KParams*)s->kp_dev, actions, substeps, obs_out, obs_task,
                                              rew, reset_buf, progress_buf, potentials, prev_potentials,
                                              actions_out, rew_out, reset_out);
                    else
                        hipLaunchKernelGGL(k_env_step_pair<decltype(T)>, wave_grid(s), wave_block(s), s->lds_bytes,
                                           STREAM(stream), (const KParams*)s->kp_dev, actions, substeps,
                                           obs_out, obs_task, rew, reset_buf, progress_buf, potentials,
                                           prev_potentials, actions_out, rew_out, reset_out);
                    return;
                }
            }
            if (ev0)
                hipExtLaunchKernelGGL(k_env_step_wave<decltype(T)>, wave_grid(s), wave_block(s),
                                      (uint32_t)s->lds_bytes, STREAM(stream), ev0, ev1, 0,
                                      (const KParams*)s->kp_dev, actions, substeps, obs_out, obs_task,
                                      rew, reset_buf, progress_buf, potentials, prev_potentials,
                                      actions_out, rew_out, reset_out);
            else
                hipLaunchKernelGGL(k_env_step_wave<decltype(T)>, wave_grid(s), wave_block(s), s->lds_bytes,
                                   STREAM(stream), (const KParams*)s->kp_dev, actions, substeps,
                                   obs_out, obs_task, rew, reset_buf, progress_buf, potentials,
                                   prev_potentials, actions_out, rew_out, reset_out);
        });
    else if (ev0)
        hipExtLaunchKernelGGL(k_env_step, grid_for(s, s->N), dim3(s->block), 0u, STREAM(stream), ev0, ev1, 0,
                              s->dm, s->ds, s->sp, s->tp, actions, substeps, obs_out, obs_task, rew,
                              reset_buf, progress_buf, potentials, prev_potentials, actions_out, rew_out,
                              reset_out);
    else
        hipLaunchKernelGGL(k_env_step, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->dm,
                           s->ds, s->sp, s->tp, actions, substeps, obs_out, obs_task, rew, reset_buf,
                           progress_buf, potentials, prev_potentials, actions_out, rew_out, reset_out);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_sim_time_launches(mi_sim* s, int32_t every, int32_t capacity) {
    NEED(s);
    if (every > 0 && (capacity < 1 || capacity > (1 << 20)))
        return fail(MI_E_ARG, "mi_sim_time_launches: capacity %d out of range", capacity);
    HIP_TRY(hipSetDevice(s->device));
    s->tev_every = every > 0 ? every : 0;
    s->tev_seen = 0;
    s->tev_rec = 0;
    const size_t want = every > 0 ? 2 * (size_t)capacity : 0;
    while (s->tev.size() < want) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreate(&e));
        s->tev.push_back(e);
    }
    while (s->tev.size() > want) {
        (void)hipEventDestroy(s->tev.back());
        s->tev.pop_back();
    }
    return MI_OK;
}

int mi_sim_launch_times(mi_sim* s, float* ms_out, int32_t max_out, int32_t* n_out) {
    NEED(s); NEED(n_out);
    if (max_out > 0) NEED(ms_out);
    HIP_TRY(hipSetDevice(s->device));
    const int n = std::min(s->tev_rec, std::max(0, (int)max_out));
    for (int k = 0; k < n; ++k) {
        HIP_TRY(hipEventSynchronize(s->tev[2 * k + 1]));
        HIP_TRY(hipEventElapsedTime(&ms_out[k], s->tev[2 * k], s->tev[2 * k + 1]));
    }
    *n_out = s->tev_rec;
    return MI_OK;
}

int mi_task_set_dr(mi_sim* s, const mi_dr_params* dr) {
    NEED(s); NEED_TASK(s);
    mi_dr_params z{};
    const mi_dr_params& d = dr ? *dr : z;
    const mi_dr_noise* all[4] = {&d.obs_on_reset, &d.obs_on_interval, &d.act_on_reset, &d.act_on_interval};
    for (int k = 0; k < 4; ++k) {
        const mi_dr_noise& n = *all[k];
        if (!n.enabled) continue;
        if (n.operation < MI_DR_OP_ADDITIVE || n.operation > MI_DR_OP_SCALING)
            return fail(MI_E_ARG, "DR: bad operation %d", n.operation);
        if (n.distribution < MI_DR_DIST_GAUSSIAN || n.distribution > MI_DR_DIST_LOGUNIFORM)
            return fail(MI_E_ARG, "DR: bad distribution %d", n.distribution);
        if (n.distribution == MI_DR_DIST_LOGUNIFORM && !(n.params[0] > 0.0f && n.params[1] > 0.0f))
            return fail(MI_E_ARG, "DR: loguniform needs positive bounds");
        if ((k & 1) && n.frequency_interval < 1)
            return fail(MI_E_ARG, "DR: on_interval frequency_interval %d < 1", n.frequency_interval);
    }
    DevTask& t = s->tp;
    t.obs_r = d.obs_on_reset; t.obs_i = d.obs_on_interval;
    t.act_r = d.act_on_reset; t.act_i = d.act_on_interval;
    t.dr_obs = d.obs_on_reset.enabled || d.obs_on_interval.enabled;
    t.dr_act = d.act_on_reset.enabled || d.act_on_interval.enabled;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemset(s->ds.dr_state, 0, sizeof(uint32_t) * 6 * (size_t)s->N));
    return sync_kparams(s);
}

int mi_dr_apply_actions(mi_sim* s, float* actions, const int64_t* reset_buf, void* stream) {
    NEED(s); NEED_TASK(s); NEED(actions); NEED(reset_buf);
    if (!s->tp.dr_act) return MI_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipLaunchKernelGGL(k_dr_apply, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->ds, s->tp,
                       1, actions, s->tp.A, reset_buf);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_dr_apply_observations(mi_sim* s, float* obs, const int64_t* reset_buf, void* stream) {
    NEED(s); NEED_TASK(s); NEED(obs); NEED(reset_buf);
    if (!s->tp.dr_obs) return MI_OK;
    HIP_TRY(hipSetDevice(s->device));
    hipLaunchKernelGGL(k_dr_apply, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->ds, s->tp,
                       0, obs, s->tp.O, reset_buf);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_get_dr_state(mi_sim* s, uint32_t* out) {
    NEED(s); NEED(out);
    HIP_TRY(hipSetDevice(s->device));
    std::vector<uint32_t> f((size_t)6 * s->N);
    HIP_TRY(hipMemcpy(f.data(), s->ds.dr_state, f.size() * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < s->N; ++i)
        for (int k = 0; k < 6; ++k) out[(size_t)6 * i + k] = f[(size_t)k * s->N + i];
    return MI_OK;
}

int mi_fill_uniform(mi_sim* s, float* out, int32_t cols, uint64_t seed, uint64_t step, float lo,
                    float hi, void* stream) {
    NEED(s); NEED(out);
    if (cols <= 0) return fail(MI_E_SHAPE, "cols must be > 0");
    HIP_TRY(hipSetDevice(s->device));
    hipLaunchKernelGGL(k_fill_uniform, grid_for(s, s->N), dim3(s->block), 0, STREAM(stream), s->N,
                       s->ds.off, out, cols, seed, step, lo, hi);
    LAUNCH_CHECK();
    return MI_OK;
}

int mi_get_reset_count(mi_sim* s, uint32_t* out) {
    NEED(s); NEED(out);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, s->pending_stream);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, s->ds.reset_count, sizeof(uint32_t) * s->N, hipMemcpyDeviceToHost));
    return MI_OK;
}

int mi_set_reset_count(mi_sim* s, const uint32_t* in) {
    NEED(s); NEED(in);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, s->pending_stream);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(s->ds.reset_count, in, sizeof(uint32_t) * s->N, hipMemcpyHostToDevice));
    return MI_OK;
}

int mi_sim_pair_load(mi_sim* s, int32_t* out, const int32_t* in, int32_t pairing) {
    NEED(s);
    if (pairing < -1 || pairing > 1) return fail(MI_E_ARG, "pairing %d (expected -1, 0 or 1)", pairing);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, s->pending_stream);
    HIP_TRY(hipDeviceSynchronize());
    if (out) HIP_TRY(hipMemcpy(out, s->ds.load, sizeof(int32_t) * s->N, hipMemcpyDeviceToHost));
    if (in) HIP_TRY(hipMemcpy(s->ds.load, in, sizeof(int32_t) * s->N, hipMemcpyHostToDevice));
    if (pairing >= 0 && (pairing ? 1 : 0) != (s->ds.pair_by_load ? 1 : 0)) {
        s->ds.pair_by_load = pairing;   // 1: re-pair every workgroup with a loaded env (MIN 0)
        return sync_kparams(s);
    }
    return MI_OK;
}

int mi_sim_nan_count(mi_sim* s, int64_t* count) {
    NEED(s); NEED(count);
    HIP_TRY(hipSetDevice(s->device));
    FLUSH(s, s->pending_stream);           // deferred substeps count too
    HIP_TRY(hipStreamSynchronize(s->pending_stream));
    unsigned long long v = 0;
    HIP_TRY(hipMemcpy(&v, s->ds.nan_total, sizeof v, hipMemcpyDeviceToHost));
    *count = (int64_t)v;
    return MI_OK;
}

int mi_sim_kernel_path(const mi_sim* s, int32_t* path, int32_t* topology, int32_t* lds_bytes) {
    NEED(s);
    if (path) *path = s->wave ? 1 : 0;
    if (topology) *topology = s->wave ? s->topo : 0;
    // per env: the workgroup's LDS (shared constants + envs_per_wg env regions) / envs_per_wg
    if (lds_bytes) *lds_bytes = s->wave ? (int32_t)(s->lds_bytes / s->wt.envs_per_wg) : 0;
    if (path && s->pair) *path = 2;
    return MI_OK;
}

}  // extern "C"
