// mi_wave.hpp — wavefront-per-env articulated substep (gfx950).
//
// Same algorithm and constraint-row order as mi_artic.hpp (and the CPU oracle); the mapping
// is what changes. One 64-lane wavefront owns one env and keeps that env's working set in
// LDS; every phase is parallel over the tree's links, DOFs, candidate contact points or
// constraint rows:
//   P1  forward kinematics / velocities / Newton-Euler, level-synchronous over link depth
//   P2  composite inertia + force sums, deepest level first (each parent sums its children
//       in a fixed order: deterministic, no atomics)
//   P3  bias C_k and CRBA row k (lane k walks its ancestor chain)
//   P4  tree LTDL factorisation, k = nv-1..0, lanes over the (i,j) ancestor pairs of k
//   P5  X = L^-1, lanes over columns (uniform row loop, lane-private column in LDS)
//   P6  M~^-1 = X D^-1 X^T, lanes over entries, stored dense + zero-padded to 32x32
//   P7  u* = u + dt M~^-1 rhs
//   P8  contact / limit detection, lanes over candidates, ballot-prefix row compaction
//       (rows in candidate order, as the oracle)
//   P9  lanes over rows: J_r and W_r = M~^-1 J_r^T in registers (32x32 FMAs, Minv rows
//       read as LDS broadcasts), A_rr = J_r . W_r; rows spilled to the env's global slab
//   P10 projected Gauss-Seidel, lanes over DOFs (u_k in a register), one wave reduction
//       per row update; lambda and row metadata live in lane registers (readlane)
//   P11 force sensors, semi-implicit integration, write-back.
// Requirements checked on the host: nv <= 32, npts <= 64, rows <= 128, L <= 64.
#pragma once
#include "mi_artic.hpp"
#include "mi_device.hpp"
#include "mi_topo_gen.hpp"
#include "../../include/mi_geom.h"

namespace mi {

constexpr int WNV = 32;  // padded DOF count of the wave path

// One wavefront = one env; a workgroup holds E envs (E waves) that share the LDS copy of the
// model constants and otherwise never interact. Lane id inside the env's wave:
__device__ __forceinline__ int wave_lane() { return (int)(threadIdx.x & 63u); }
// Sync point between two phases of ONE env (its wave): every lane's earlier LDS and global
// accesses are visible to the wave's later accesses. No s_barrier (the other waves of the
// workgroup are other envs), and wavefront scope: a wave's memory operations are performed in
// order (LDS and the vector memory path), so the fences only stop the compiler from moving
// accesses across the sync.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Diagnostic phase timers (built only with -DMI_STAMPS into a separate library; the product
// build compiles them out). Every workgroup adds the s_memtime delta of each phase to its own
// slot g_phase[block % MI_STAMP_SLOTS][id] (lane 0, plain adds: no contention); [31] counts
// substeps. The host sums the slots. IDs: see tools/phase_stamps.py.
#ifdef MI_STAMPS
#define MI_STAMP_SLOTS 16384
#define MI_STAMP_ENV (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6))
__device__ unsigned long long g_phase[MI_STAMP_SLOTS][32];
#define STAMP_BEGIN()                                                                     \
    unsigned long long stamp_t_;                                                          \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_t_)::"memory");  \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)
#define STAMP(id)                                                                         \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        unsigned long long t_;                                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        if ((threadIdx.x & 63) == 0) g_phase[MI_STAMP_ENV % MI_STAMP_SLOTS][id] += t_ - stamp_t_;  \
        stamp_t_ = t_;                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)
#define STAMP_END()                                                                       \
    do {                                                                                  \
        if ((threadIdx.x & 63) == 0) g_phase[MI_STAMP_ENV % MI_STAMP_SLOTS][31] += 1ull;           \
    } while (0)
#define STAT(id, v)                                                                       \
    do {                                                                                  \
        if ((threadIdx.x & 63) == 0) g_phase[MI_STAMP_ENV % MI_STAMP_SLOTS][id] += (unsigned long long)(v); \
    } while (0)
#define STAMP_RESET()                                                                     \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_t_)::"memory");  \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)
#else
#define STAT(id, v) do { } while (0)
#define STAMP_RESET() do { } while (0)
#define STAMP_BEGIN() do { } while (0)
#define STAMP(id) do { } while (0)
#define STAMP_END() do { } while (0)
#endif

struct WaveTabs {
    int nlev;
    const int* lev_start;     // [nlev+1]
    const int* lev_links;     // [L]
    const int* child_start;   // [L+1]
    const int* child_list;    // [L]
    const int* chain_start;   // [L+1] links on the path root -> l, excl. the root, root first
    const int* chain_list;
    const int* desc_start;    // [L+1] descendants of link l (excl. l), increasing index
    const int* desc_list;
    const int* anc_start;     // [nv+1] ancestors of dof k (excl. k), nearest first
    const int* anc_list;
    const unsigned long long* link_mask;  // [L] dofs on the root..l path
    const unsigned char* tri_p;           // pair index -> (p, q), p <= q
    const unsigned char* tri_q;
    // LDS float offsets
    int s_mc, s_R, s_o, s_S, s_F, s_Ic, s_M, s_X, s_D, s_r, s_us, s_q, s_rp, s_cp, s_cl,
        s_rl, s_lsg, s_rb, s_rk, s_ad, s_xs, s_L, s_total;
    int max_rows;
    size_t g_row_stride;  // floats per env in the global W-row slab (max_rows * WNV)
    // W rows [0, w_rows_lds) are handed from P9 to P10 through LDS at s_W (stride nv, in the
    // span that is dead by then); rows beyond go through the global slab
    int s_W, w_rows_lds;
    int s_W2, w_rows_a;   // rows [w_rows_a, w_rows_lds) in a second segment at s_W2
    // E envs per workgroup: env w of the workgroup uses [s_env, s_total) shifted by
    // w * env_stride floats (env_stride = s_total - s_env); [0, s_env) is the shared constant block
    int envs_per_wg, s_env, env_stride;
    // J rows [0, j_rows_lds) kept in LDS at s_J (stride nv) for the PGS sweeps
    int s_J, j_rows_lds;
    // per-model constant block (see McLayout): global copy, staged into LDS at s_mc once per
    // launch by every workgroup
    const float* g_mc;
    int mc_len, mc_pts, mc_sens, mc_chs, mc_chl, mc_dss, mc_dsl, mc_lim;   // block offsets
    int mc_geo, mc_pairs;   // self-collision geom table [G][8] and pairs [P][2] (or -1)
    int npts, nsens;
    int nlimc;   // joints with a limit (lower < upper): limit-row candidates, joint ids at mc_lim
    // self-collision (mi_geom.h): geom table [G][8] = link, p0 (3), p1 (3), radius and the
    // geom pairs [P][2], global (lane-indexed, cache-resident); contact capacity ncmax
    int self_on, npairs, ncmax;
    const float* g_geo;
    const int* g_pairs;
    int s_cl2, s_cn;   // per contact: second link (-1: ground), normal (3)
    int s_seg, s_surv; // P8 scratch (in the W span, free until P9): world segments [G][8],
                       // bounding spheres [G][4] at s_seg + 8G, broad-phase survivors [P];
                       // s_seg < 0: not enough room, direct path
    int ngeoms;
    // paired-env kernels (mi_pair.hpp): lambda per constraint row of the u-space fallback sweeps
    int s_lam;
    // paired-env kernels: contact-parallel force sensors (buffer [ncmax][S][6] + sums in the
    // dead W rows; 0: the serial per-sensor loop)
    int sens_par;
    // paired-env kernels: per-wave Delassus scratch of the wide PGS ([N / 2][64][64] floats)
    float* g_wa;
};

// Per-model constants in the LDS block, structure-of-arrays so lane-indexed reads (lane = link,
// point or sensor) hit consecutive banks. Link field f of link l at [f * L + l].
enum McField {
    MC_POS = 0, MC_QUAT = 3, MC_AXIS = 7, MC_JTYPE = 10, MC_MASS = 11, MC_COM = 12,
    MC_INER = 15, MC_ARM = 21, MC_DAMP = 22, MC_LO = 23, MC_HI = 24, MC_MASK = 25,
    MC_NLINKF = 26
};
// point fields (at mc_pts + f * npts + c): link, x, y, z (link frame), radius
enum McPoint { MP_LINK = 0, MP_X = 1, MP_RAD = 4, MP_NF = 5 };
// sensor fields (at mc_sens + f * nsens + s): link, x, y, z
enum McSensor { MS_LINK = 0, MS_X = 1, MS_NF = 4 };

struct MC {
    const float* b;
    const int* bi;
    int L, np, ns;
    const WaveTabs* t;
    MI_D float lf(int f, int l) const { return b[f * L + l]; }
    MI_D void lf3(int f, int l, float* o) const { o[0] = lf(f, l); o[1] = lf(f + 1, l); o[2] = lf(f + 2, l); }
    MI_D int jtype(int l) const { return (int)lf(MC_JTYPE, l); }
    MI_D unsigned mask(int l) const { return (unsigned)bi[MC_MASK * L + l]; }
    MI_D float pf(int f, int c) const { return b[t->mc_pts + f * np + c]; }
    MI_D float sf(int f, int s) const { return b[t->mc_sens + f * ns + s]; }
    MI_D int chain_start(int l) const { return bi[t->mc_chs + l]; }
    MI_D int chain(int j) const { return bi[t->mc_chl + j]; }
    MI_D int desc_start(int l) const { return bi[t->mc_dss + l]; }
    MI_D int desc(int j) const { return bi[t->mc_dsl + j]; }
    MI_D int lim(int j) const { return bi[t->mc_lim + j]; }
};

// Spatial force direction of contact row r = 3 ci + tt at contact point pc: normal (tt 0,
// +z) or friction (tt 1: +x, tt 2: +y), f = (pc x dir, dir). Rebuilt where needed from the
// contact point instead of stored per row (saves 6 floats x rows of LDS); same arithmetic.
// Contact ci's directions (normal, t1, t2): ground +z / +x / +y, self-contact the stored
// normal and mi_contact_basis (same as the oracle).
// SELF = false (a model compiled without self-collision pairs): every contact is a ground contact.
template <bool SELF>
MI_D void contact_dirs(const float* sm, const WaveTabs& t, int ci, float (&d)[9]) {
    if (!SELF || sm[t.s_cl2 + ci] < 0.0f) {
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = (k == 2 || k == 3 || k == 7) ? 1.0f : 0.0f;
    } else {
        d[0] = sm[t.s_cn + 3 * ci]; d[1] = sm[t.s_cn + 3 * ci + 1]; d[2] = sm[t.s_cn + 3 * ci + 2];
        mi_contact_basis(d, d + 3, d + 6);
    }
}

template <bool SELF>
MI_D void contact_row_f(const float* sm, const WaveTabs& t, int r, float (&f)[6]) {
    const int ci = r / 3, tt = r - 3 * ci;
    const float pc[3] = {sm[t.s_cp + 3 * ci], sm[t.s_cp + 3 * ci + 1], sm[t.s_cp + 3 * ci + 2]};
    float d[9];
    contact_dirs<SELF>(sm, t, ci, d);
    const float dir[3] = {d[3 * tt], d[3 * tt + 1], d[3 * tt + 2]};
    cross3(pc, dir, f);
    f[3] = dir[0]; f[4] = dir[1]; f[5] = dir[2];
}

MI_D MC make_mc(const WaveTabs& t, const float* mcb, int L) {
    MC c;
    c.b = mcb;
    c.bi = (const int*)mcb;
    c.L = L; c.np = t.npts; c.ns = t.nsens;
    c.t = &t;
    return c;
}

MI_D float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// LDS W row r. Two segments (WaveTabs::s_W2) only on self-collision topologies (the host
// creates the second segment only for them); otherwise one.
template <bool SEG2>
MI_D float* w_row(const WaveTabs& t, float* sm, int r, int nv) {
    if constexpr (!SEG2) return sm + t.s_W + r * nv;
    return sm + (r < t.w_rows_a ? t.s_W + r * nv : t.s_W2 + (r - t.w_rows_a) * nv);
}

MI_D float readlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
template <int CTRL, int ROW_MASK = 0xF, bool BOUND_CTRL = true>
MI_D float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, BOUND_CTRL));
}
// Sum over each 32-lane half of the wave with DPP only (no LDS crossbar): quad swaps,
// half-row / row mirrors, then row_bcast:15 folds row 0 into row 1 (and 2 into 3).
// Lane 31 holds sum(lanes 0..31), lane 63 holds sum(lanes 32..63).
MI_D float half_sums(float v) {
    v += dpp<0xB1>(v);          // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);          // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);         // row_half_mirror
    v += dpp<0x140>(v);         // row_mirror
    v += dpp<0x142, 0xA, false>(v);  // row_bcast:15 into rows 1 and 3
    return v;
}

// x <- M~^-1 x (tree LTDL factor of M~ in Mx, 1/D in Dinv) on a lane-private vector kept in LDS: element c of lane's vector at
// xs[c * 64 + lane] (uniform offsets, consecutive banks: conflict-free). LDS operations of
// one wave complete in order, so a read after a write to the same slot sees the write.
MI_D void tree_solve_lds(const WaveTabs& t, const float* Mx, const float* Dinv, int nv,
                         float* xs) {
    for (int i = nv - 1; i >= 0; --i) {
        const float xi = xs[i * 64];
        for (int a = t.anc_start[i]; a < t.anc_start[i + 1]; ++a) {
            const int j = t.anc_list[a];
            xs[j * 64] -= Mx[i * nv + j] * xi;
        }
    }
    for (int i = 0; i < nv; ++i) xs[i * 64] *= Dinv[i];
    for (int i = 0; i < nv; ++i) {
        float xi = xs[i * 64];
        for (int a = t.anc_start[i]; a < t.anc_start[i + 1]; ++a) {
            const int j = t.anc_list[a];
            xi -= Mx[i * nv + j] * xs[j * 64];
        }
        xs[i * 64] = xi;
    }
}

// ---- compile-time-topology (CT) tree kernels --------------------------------------------
// Layout: lane c holds column c of M~ in Mc[0..nv-1] (Mc[r] = M~[r][c], lower triangle and
// tree pattern only; every other entry exactly 0). Factor entries are broadcast with
// v_readlane at compile-time (register, lane) pairs, so no LDS or barrier is involved.
// Arithmetic is operation-for-operation that of the runtime-table path above.

// Mc[r] <- Mx[r][lane] for lane == r or lane an ancestor of r, else 0
// An opaque copy of the lane id: lane-compare masks built from it cannot be hoisted out of
// the unrolled step that uses them (dozens of hoisted 64-bit masks would spill SGPRs).
MI_D int lane_here(int lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}

template <class T>
MI_D void ct_load_columns(const float* Mx, int lane, float (&Mc)[T::nvc]) {
    const int c = lane < T::nv ? lane : 0;
    sfor<0, T::nv>([&](auto R) {
        constexpr int r = R;
        constexpr unsigned long long keep = (unsigned long long)T::dof.anc_mask[r] | (1ull << r);
        const float v = Mx[r * T::nv + c];   // loaded by every lane, then selected: no branch
        Mc[r] = ((keep >> lane_here(lane)) & 1ull) ? v : 0.0f;
    });
}

// in-register tree LTDL: M~ = L^T D L, L strictly below the diagonal, D on it
template <class T>
MI_D void ct_ltdl(int lane, float (&Mc)[T::nvc]) {
    sfor_down<0, T::nv>([&](auto K) {
        constexpr int k = K;
        __builtin_amdgcn_sched_barrier(0);
        const int ln = lane_here(lane);
        // hardware reciprocal (1 ulp) instead of the ~10-instruction IEEE division on the
        // factorisation's dependent chain
        const float inv = __builtin_amdgcn_rcpf(readlane(Mc[k], k));
        sfor<T::dof.anc_start[k], T::dof.anc_start[k + 1]>([&](auto A) {
            constexpr int ii = T::dof.anc[A];
            const float s = readlane(Mc[k], ii) * inv;
            if (ln <= ii) Mc[ii] -= s * Mc[k];
        });
        if (ln < k) Mc[k] = Mc[k] * inv;
    });
}

// lane c: 1 / D_c (lanes >= nv: unused)
template <class T>
MI_D float ct_dinv(int lane, const float (&Mc)[T::nvc]) {
    float dg = 1.0f;
    sfor<0, T::nv>([&](auto I) { dg = lane_here(lane) == I ? Mc[I] : dg; });
    return __builtin_amdgcn_rcpf(dg);
}

template <class T>
MI_D void ct_opaque(float (&Mc)[T::nvc]) {
#pragma unroll
    for (int i = 0; i < T::nv; ++i) asm volatile("" : "+v"(Mc[i]));
}

// x <- M~^-1 x on a lane-private register vector. Mc is made opaque before each pass so the
// compiler re-issues the factor readlanes where they are used instead of keeping hundreds
// of them live in SGPRs (which spill).
// Step fence for the unrolled solves: every element of x and the factor column used next
// pass through empty volatile asm (ordered among themselves), so the next step's readlanes
// cannot be issued before this step's FMAs have consumed theirs. Without it the scheduler
// front-loads ~200 readlanes into SGPRs and spills them. No instructions are emitted.
template <class T>
MI_D void ct_step_fence(float (&x)[T::nvc], float& mcol) {
#pragma unroll
    for (int c = 0; c < T::nv; ++c) asm volatile("" : "+v"(x[c]));
    asm volatile("" : "+v"(mcol));
}

// x <- M~^-1 x on a lane-private register vector (same operation order as tree_solve_lds)
template <class T>
MI_D void ct_solve(float (&Mc)[T::nvc], float dvec, float (&x)[T::nvc]) {
    sfor_down<0, T::nv>([&](auto I) {                 // x <- L^-T x (leaves -> root)
        constexpr int i = I;
        ct_step_fence<T>(x, Mc[i]);
        const float xi = x[i];
        sfor<T::dof.anc_start[i], T::dof.anc_start[i + 1]>([&](auto A) {
            constexpr int j = T::dof.anc[A];
            x[j] -= readlane(Mc[i], j) * xi;
        });
    });
    sfor<0, T::nv>([&](auto I) { x[I] *= readlane(dvec, I); });   // x <- D^-1 x
    sfor<0, T::nv>([&](auto I) {                      // x <- L^-1 x (root -> leaves)
        constexpr int i = I;
        ct_step_fence<T>(x, Mc[i]);
        float xi = x[i];
        sfor<T::dof.anc_start[i], T::dof.anc_start[i + 1]>([&](auto A) {
            constexpr int j = T::dof.anc[A];
            xi -= readlane(Mc[i], j) * x[j];
        });
        x[i] = xi;
    });
}

// Publish the factor for the batched solves: lane j (column j) writes each entry L[i][j]
// (j an ancestor of i) into row i's compact ancestor list, position = depth(i) - depth(j) - 1
// (lists run nearest ancestor first); then 1/D. dj = depth of DOF j (its ancestor count).
template <class T>
MI_D void ct_publish_factor(int lane, int dj, const float (&Mc)[T::nvc], float dvec, float* Lr) {
    if (lane < T::nv) {
        sfor<0, T::nv>([&](auto I) {
            constexpr int i = I;
            constexpr int na = T::dof.anc_start[i + 1] - T::dof.anc_start[i];
            if ((T::dof.anc_mask[i] >> lane_here(lane)) & 1u) Lr[T::dof.lrow[i] + na - 1 - dj] = Mc[i];
        });
        Lr[T::dof.lrow[T::nv] + lane] = dvec;
    }
}

// x <- M~^-1 x on a lane-private register vector (a: see below), factor entries read from the published
// LDS rows: every read is a wave-uniform broadcast (no VALU readlanes; adjacent entries
// merge into wide LDS reads). Same operation order as ct_solve / tree_solve_lds.
// most ancestors of any DOF (size of the one-step prefetch buffers of ct_solve_l)
template <class T>
constexpr int ct_max_anc() {
    int m = 1;
    for (int i = 0; i < T::nv; ++i) {
        const int n = T::dof.anc_start[i + 1] - T::dof.anc_start[i];
        if (n > m) m = n;
    }
    return m;
}

// The step fences keep each step's FMAs in order (and the factor loads from being front-loaded
// into hundreds of live registers), which also kept every step's LDS broadcast reads behind
// the previous step: one LDS round trip exposed per step, 2 nv per solve. The factor entries
// of step s + PD are therefore read before step s's fence (PD steps of prefetch, (PD + 1)
// ct_max_anc registers): their latency overlaps the FMAs of the steps in between (the paired
// kernel runs PD = 3: Humanoid fused step 0.1672 -> 0.1652 ms against PD = 1). Same values, same
// operation order.
template <class T, int PD = 1>
MI_D void ct_solve_l(const float* Lr, float (&x)[T::nvc], float& a) {
    // PD steps of prefetch: the factor entries of step s + PD are read before step s's fence,
    // into a ring of PD + 1 buffers indexed at compile time (no copies between steps)
    constexpr int MA = ct_max_anc<T>();
    constexpr int NB = PD + 1;
    float buf[NB][MA];
    auto load = [&](auto I, auto B) {
        constexpr int i = I, bb = B;
        constexpr int na = T::dof.anc_start[i + 1] - T::dof.anc_start[i];
        constexpr int off = T::dof.lrow[i];
        sfor<0, na>([&](auto A) { buf[bb][A] = Lr[off + A]; });
    };
    sfor<0, PD>([&](auto S) {                         // steps 0 .. PD-1 of the first pass
        constexpr int i = T::nv - 1 - (int)S;
        if constexpr (i >= 0) load(std::integral_constant<int, i>{}, std::integral_constant<int, (int)S % NB>{});
    });
    sfor_down<0, T::nv>([&](auto I) {                 // x <- L^-T x (leaves -> root)
        constexpr int i = I;
        constexpr int st = T::nv - 1 - i;
        constexpr int a0 = T::dof.anc_start[i], na = T::dof.anc_start[i + 1] - a0;
        if constexpr (i - PD >= 0)
            load(std::integral_constant<int, i - PD>{}, std::integral_constant<int, (st + PD) % NB>{});
#pragma unroll
        for (int c = 0; c < T::nv; ++c) asm volatile("" : "+v"(x[c]));   // step fence
        const float xi = x[i];
        sfor<0, na>([&](auto A) {
            constexpr int j = T::dof.anc[a0 + A];
            x[j] -= buf[st % NB][A] * xi;
        });
    });
    // x <- D^-1 x; a = y^T D^-1 y with y = L^-T x_in, i.e. x_in^T M~^-1 x_in (for x_in = J_r^T
    // this is A_rr = J_r W_r, computed before the second pass needs no copy of J_r)
    a = 0.0f;
    sfor<0, PD>([&](auto S) {                         // steps 0 .. PD-1 of the second pass
        constexpr int i = (int)S;
        if constexpr (i < T::nv) load(std::integral_constant<int, i>{}, std::integral_constant<int, i % NB>{});
    });
    sfor<0, T::nv>([&](auto I) {
        const float y = x[I];
        x[I] = y * Lr[T::dof.lrow[T::nv] + I];
        a += y * x[I];
    });
    sfor<0, T::nv>([&](auto I) {                      // x <- L^-1 x (root -> leaves)
        constexpr int i = I;
        constexpr int a0 = T::dof.anc_start[i], na = T::dof.anc_start[i + 1] - a0;
        if constexpr (i + PD < T::nv)
            load(std::integral_constant<int, i + PD>{}, std::integral_constant<int, (i + PD) % NB>{});
#pragma unroll
        for (int c = 0; c < T::nv; ++c) asm volatile("" : "+v"(x[c]));
        float xi = x[i];
        sfor<0, na>([&](auto A) {
            constexpr int j = T::dof.anc[a0 + A];
            xi -= buf[i % NB][A] * x[j];
        });
        x[i] = xi;
    });
}

// P1a: local joint transform of link l >= 1 (independent of every other link):
// aux[15 l ..] = {Rloc = Rq Rot(axis, q) (9), tloc (3), aloc = Rq axis (3)}
MI_D void wave_link_local(const MC& mc, const WaveTabs& t, float* sm, int l) {
    float* aux = sm + t.s_X + 15 * l;
    float Rq[9], a[3], qt[4], ax[3], tl[3];
    qt[0] = mc.lf(MC_QUAT, l); qt[1] = mc.lf(MC_QUAT + 1, l);
    qt[2] = mc.lf(MC_QUAT + 2, l); qt[3] = mc.lf(MC_QUAT + 3, l);
    mc.lf3(MC_AXIS, l, ax);
    mc.lf3(MC_POS, l, tl);
    m3_from_quat(qt, Rq);
    m3_vec(Rq, ax, a);
    const float qj = sm[t.s_q + l - 1];
    float R[9];
    if (mc.jtype(l) == MI_JOINT_HINGE) {
        float Ra[9];
        m3_axis_angle(ax, qj, Ra);
        m3_mul(Rq, Ra, R);
    } else {
#pragma unroll
        for (int c = 0; c < 9; ++c) R[c] = Rq[c];
#pragma unroll
        for (int c = 0; c < 3; ++c) tl[c] += a[c] * qj;
    }
#pragma unroll
    for (int c = 0; c < 9; ++c) aux[c] = R[c];
#pragma unroll
    for (int c = 0; c < 3; ++c) { aux[9 + c] = tl[c]; aux[12 + c] = a[c]; }
}

// P1b helpers. Root frame: orientation from the root quaternion, origin p0 (the spatial
// origin), fictitious base acceleration -g (- w x v for a free root).
MI_D void link_root(const WaveTabs& t, const float* sm, const SimP& p, int nr, float (&R)[9],
                    float (&o)[3], float (&V)[6], float (&A)[6]) {
    m3_from_quat(sm + t.s_rp + 4, R);
    o[0] = o[1] = o[2] = 0.0f;
    A[0] = A[1] = A[2] = 0.0f;
    A[3] = -p.g[0]; A[4] = -p.g[1]; A[5] = -p.g[2];
    if (nr) {
        const float* u = sm + t.s_us;
        const float v[3] = {u[0], u[1], u[2]};
        const float om[3] = {u[3], u[4], u[5]};
        float wv[3];
        cross3(om, v, wv);
        A[3] -= wv[0]; A[4] -= wv[1]; A[5] -= wv[2];
        V[0] = om[0]; V[1] = om[1]; V[2] = om[2];
        V[3] = v[0]; V[4] = v[1]; V[5] = v[2];
    } else {
#pragma unroll
        for (int c = 0; c < 6; ++c) V[c] = 0.0f;
    }
}

// One tree step: link c's frame, DOF subspace s, velocity and velocity-product acceleration
// from its parent's (R, o, V, A), updated in place.
MI_D void link_step(const MC& mc, int nr, const WaveTabs& t, const float* sm, int c, float (&R)[9],
                    float (&o)[3], float (&V)[6], float (&A)[6], float (&s)[6]) {
    const int k = nr + c - 1;
    const float* aux = sm + t.s_X + 15 * c;
    float RP[9], a[3], op[3];
#pragma unroll
    for (int q = 0; q < 9; ++q) RP[q] = R[q];
    m3_mul(RP, aux, R);
    m3_vec(RP, aux + 9, op);
    m3_vec(RP, aux + 12, a);
#pragma unroll
    for (int q = 0; q < 3; ++q) o[q] = o[q] + op[q];
    if (mc.jtype(c) == MI_JOINT_HINGE) {
        s[0] = a[0]; s[1] = a[1]; s[2] = a[2];
        cross3(o, a, s + 3);
    } else {
        s[0] = s[1] = s[2] = 0.0f;
        s[3] = a[0]; s[4] = a[1]; s[5] = a[2];
    }
    const float uk = sm[t.s_us + k];
    float sd[6];
    crm(V, s, sd);
#pragma unroll
    for (int q = 0; q < 6; ++q) { V[q] = V[q] + s[q] * uk; A[q] = A[q] + sd[q] * uk; }
}

// P1b+c: link l's world frame, subspace, velocity and velocity-product acceleration, composed
// along its own root-to-l chain (no barriers between tree levels: every lane walks its chain;
// each step is the same arithmetic a level-by-level sweep would do, so results are identical),
// then the link's spatial inertia about p0 and Newton-Euler force from the register values.
MI_D void wave_link_forward(const MC& mc, int nr, const WaveTabs& t, float* sm, int l,
                            const SimP& p) {
    float R[9], o[3], V[6], A[6], s[6];
    link_root(t, sm, p, nr, R, o, V, A);
    for (int j = mc.chain_start(l); j < mc.chain_start(l + 1); ++j)
        link_step(mc, nr, t, sm, mc.chain(j), R, o, V, A, s);
    if (l > 0) {
#pragma unroll
        for (int c = 0; c < 6; ++c) sm[t.s_S + 6 * (nr + l - 1) + c] = s[c];
    }
#pragma unroll
    for (int c = 0; c < 9; ++c) sm[t.s_R + 9 * l + c] = R[c];
#pragma unroll
    for (int c = 0; c < 3; ++c) sm[t.s_o + 3 * l + c] = o[c];

    float I[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float F[6] = {0, 0, 0, 0, 0, 0};
    const float mass = mc.lf(MC_MASS, l);
    if (mass > 0.0f) {
        float c3[3], T[9], Iw[9], com[3];
        mc.lf3(MC_COM, l, com);
        m3_vec(R, com, c3);
        c3[0] += o[0]; c3[1] += o[1]; c3[2] += o[2];
        float in[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) in[c] = mc.lf(MC_INER + c, l);
        const float Ib[9] = {in[0], in[3], in[4], in[3], in[1], in[5], in[4], in[5], in[2]};
        m3_mul(R, Ib, T);
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b)
                Iw[3 * a + b] = T[3 * a] * R[3 * b] + T[3 * a + 1] * R[3 * b + 1] + T[3 * a + 2] * R[3 * b + 2];
        const float cc = dot3(c3, c3);
        I[0] = mass;
        I[1] = mass * c3[0]; I[2] = mass * c3[1]; I[3] = mass * c3[2];
        I[4] = Iw[0] + mass * (cc - c3[0] * c3[0]);
        I[5] = Iw[4] + mass * (cc - c3[1] * c3[1]);
        I[6] = Iw[8] + mass * (cc - c3[2] * c3[2]);
        I[7] = Iw[1] - mass * c3[0] * c3[1];
        I[8] = Iw[2] - mass * c3[0] * c3[2];
        I[9] = Iw[5] - mass * c3[1] * c3[2];
        float IA[6], IV[6], tt[6];
        inertia_mul(I, A, IA);
        inertia_mul(I, V, IV);
        crf(V, IV, tt);
#pragma unroll
        for (int c = 0; c < 6; ++c) F[c] = IA[c] + tt[c];
        // link angular damping (PhysX default 0.05): the torque -c I_com omega on the link,
        // in the bias as +c I_com omega (same arithmetic as the thread path and the oracle)
        float Iwv[3];
        m3_vec(Iw, V, Iwv);
#pragma unroll
        for (int c = 0; c < 3; ++c) F[c] = F[c] + p.ang_damp * Iwv[c];
    }
    // one 16-float record per link (inertia 10, force 6): 4 aligned 16-B LDS accesses
    float4* rec = reinterpret_cast<float4*>(sm + t.s_F) + 4 * l;
    rec[0] = make_float4(I[0], I[1], I[2], I[3]);
    rec[1] = make_float4(I[4], I[5], I[6], I[7]);
    rec[2] = make_float4(I[8], I[9], F[0], F[1]);
    rec[3] = make_float4(F[2], F[3], F[4], F[5]);
}

// One articulated substep of env i, executed by the whole 64-lane workgroup.
// sm: this env's LDS region; gW: this env's global slab of W rows [max_rows][WNV].
// load_state: read the env's state record from HBM (first substep of a launch; later ones
// continue from LDS); store_state: write the state and sensor wrenches back (last substep).
template <class TP>
MI_D void wave_artic_substep(const DevModel& m, const WaveTabs& t, const DevState& st,
                             const SimP& p, int i, const float* mcb, float* sm, float* gW,
                             bool load_state, bool store_state) {
    const int lane = wave_lane();
    const int N = st.N, L = m.L, D = m.D, nv = m.nv, nr = m.nr;
    const float dt = p.dt;
    float* us = sm + t.s_us;   // u, then u*
    float* rhs = sm + t.s_r;
    float* Mx = sm + t.s_M;    // M (lower), then dense padded M~^-1 [WNV][WNV]
    float* Dv = sm + t.s_D;
    float* Ss = sm + t.s_S;
    const MC mc = make_mc(t, mcb, L);

    STAMP_BEGIN();
    // ---- load state into LDS (later substeps of a launch start from the state the previous
    // substep's P11 left in LDS)
    if (load_state) {
        if (lane < 3) sm[t.s_rp + lane] = st.root_pos[sx(st, lane, i)];
        if (lane < 4) sm[t.s_rp + 4 + lane] = st.root_quat[sx(st, lane, i)];
        if (lane < nr) us[lane] = st.root_vel[sx(st, lane, i)];
        else if (lane < nv) us[lane] = st.qd[sx(st, lane - nr, i)];
        if (lane < D) sm[t.s_q + lane] = st.q[sx(st, lane, i)];
    }
    if (nr && lane < 6) {
        float s[6] = {0, 0, 0, 0, 0, 0};
        if (lane < 3) s[3 + lane] = 1.0f; else s[lane - 3] = 1.0f;
#pragma unroll
        for (int c = 0; c < 6; ++c) Ss[6 * lane + c] = s[c];
    }
    wave_sync();

    STAMP(0);   // load
    // ---- P1a: local joint transforms, every link at once
    for (int l = 1 + lane; l < L; l += 64) wave_link_local(mc, t, sm, l);
    wave_sync();
    // ---- P1b+c: world frames / subspaces / velocities along each link's chain, then the
    // link's inertia and Newton-Euler force (same lane: no barrier in between)
    for (int l = lane; l < L; l += 64) wave_link_forward(mc, nr, t, sm, l, p);
    wave_sync();
    STAMP(1);   // P1
    // ---- P2: composite inertia / force = own + sum over the subtree (fixed descendant order,
    // every link at once; results into the aux region: Ic at 16 l, F at 16 l + 10)
    float* aux = sm + t.s_X;
    {
        const float4* recs = reinterpret_cast<const float4*>(sm + t.s_F);
        for (int l = lane; l < L; l += 64) {
            float4 a0 = recs[4 * l], a1 = recs[4 * l + 1], a2 = recs[4 * l + 2], a3 = recs[4 * l + 3];
            for (int di = mc.desc_start(l); di < mc.desc_start(l + 1); ++di) {
                const int d = mc.desc(di);
                const float4 b0 = recs[4 * d], b1 = recs[4 * d + 1], b2 = recs[4 * d + 2], b3 = recs[4 * d + 3];
                a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
                a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
                a2.x += b2.x; a2.y += b2.y; a2.z += b2.z; a2.w += b2.w;
                a3.x += b3.x; a3.y += b3.y; a3.z += b3.z; a3.w += b3.w;
            }
            float4* o = reinterpret_cast<float4*>(aux) + 4 * l;   // Ic at 16 l, F at 16 l + 10
            o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3;
        }
    }
    wave_sync();
    STAMP(2);   // P2
    // ---- P3: bias + CRBA (lane k = dof k)
    if (lane < nv) {
        const int k = lane, l = k < nr ? 0 : k - nr + 1;
        float s[6], I[10], f[6], F[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) s[c] = Ss[6 * k + c];
        {
            const float4* rec = reinterpret_cast<const float4*>(aux) + 4 * l;
            const float4 a0 = rec[0], a1 = rec[1], a2 = rec[2], a3 = rec[3];
            I[0] = a0.x; I[1] = a0.y; I[2] = a0.z; I[3] = a0.w;
            I[4] = a1.x; I[5] = a1.y; I[6] = a1.z; I[7] = a1.w;
            I[8] = a2.x; I[9] = a2.y; F[0] = a2.z; F[1] = a2.w;
            F[2] = a3.x; F[3] = a3.y; F[4] = a3.z; F[5] = a3.w;
        }
        inertia_mul(I, s, f);
        float diag = dot6(s, f);
        float r = -dot6(s, F);
        if (k >= nr) {
            const float damp = mc.lf(MC_DAMP, l);
            diag += mc.lf(MC_ARM, l) + dt * damp;
            r += st.eff[sx(st, k - nr, i)] - damp * us[k];
        }
        rhs[k] = r;
        if constexpr (TP::kCT) {
            // row k of M~: S_j . f for every j, branch-free (uniform j: the S_j reads are LDS
            // broadcasts). Only the ancestors of k are ever read (ct_load_columns masks the
            // rest), so the other entries are written but dead; a lane-varying ancestor branch
            // per j cost more than the 6 FMAs it skipped. The diagonal goes last.
            sfor<0, TP::nv>([&](auto J) {
                constexpr int j = J;
                float sj[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) sj[c] = Ss[6 * j + c];
                Mx[k * nv + j] = dot6(sj, f);
            });
            Mx[k * nv + k] = diag;
        } else {
            Mx[k * nv + k] = diag;
            for (int a = t.anc_start[k]; a < t.anc_start[k + 1]; ++a) {
                const int j = t.anc_list[a];
                float sj[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) sj[c] = Ss[6 * j + c];
                Mx[k * nv + j] = dot6(sj, f);
            }
        }
    }
    wave_sync();
    STAMP(3);   // P3
    // ---- P4: LTDL in place (M = L^T D L, L strictly below the diagonal)
    float Mc[TP::nvc];     // CT path: column `lane` of M~, then of its factor (rows 0..nv-1)
    float dvec = 1.0f;    // CT path: lane c holds 1 / D_c
    if constexpr (TP::kCT) {
        ct_load_columns<TP>(Mx, lane, Mc);
        ct_ltdl<TP>(lane, Mc);
        dvec = ct_dinv<TP>(lane, Mc);
        const int dj = lane < nr ? lane : __builtin_popcount(mc.mask(lane < nv ? lane - nr + 1 : 0)) - 1;
        ct_publish_factor<TP>(lane, dj, Mc, dvec, sm + t.s_L);
    } else {
        for (int k = nv - 1; k >= 0; --k) {
            const int a0 = t.anc_start[k], na = t.anc_start[k + 1] - a0;
            const float inv = 1.0f / Mx[k * nv + k];
            const int npair = na * (na + 1) / 2;
            for (int pi = lane; pi < npair; pi += 64) {
                const int ii = t.anc_list[a0 + t.tri_p[pi]], jj = t.anc_list[a0 + t.tri_q[pi]];
                Mx[ii * nv + jj] -= (Mx[k * nv + ii] * inv) * Mx[k * nv + jj];
            }
            wave_sync();
            if (lane < na) {
                const int ii = t.anc_list[a0 + lane];
                Mx[k * nv + ii] = Mx[k * nv + ii] * inv;
            }
            wave_sync();
        }
    }
    STAMP(4);   // P4 (+ factor publish)
    // ---- P5: 1/D of the factor
    if constexpr (!TP::kCT) {
        if (lane < nv) Dv[lane] = 1.0f / Mx[lane * nv + lane];
        wave_sync();
    }
    STAMP(5);   // P5


    // ---- P8: candidate contact points (lane c), ballot compaction in candidate order
    int ncon = 0;
    {
        const float rpz = sm[t.s_rp + 2];
        bool act = false;
        float pc[3] = {0, 0, 0}, bn = 0.0f;
        int l = 0;
        if (lane < t.npts) {
            l = (int)mc.pf(MP_LINK, lane);
            const float pl[3] = {mc.pf(MP_X, lane), mc.pf(MP_X + 1, lane), mc.pf(MP_X + 2, lane)};
            float R[9], x[3];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
            m3_vec(R, pl, x);
#pragma unroll
            for (int q = 0; q < 3; ++q) x[q] += sm[t.s_o + 3 * l + q];
            const float r = mc.pf(MP_RAD, lane);
            const float gap = rpz + x[2] - r;
            act = gap < p.contact_offset;
            pc[0] = x[0]; pc[1] = x[1]; pc[2] = x[2] - r;
            const float d = gap - p.rest_offset;
            bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
        }
        const unsigned long long mask = __ballot(act);
        ncon = __popcll(mask);
        if (act) {
            const int ci = __popcll(mask & ((1ull << lane) - 1ull));
#pragma unroll
            for (int q = 0; q < 3; ++q) sm[t.s_cp + 3 * ci + q] = pc[q];
            sm[t.s_cl + ci] = (float)l;
            sm[t.s_cl2 + ci] = -1.0f;
#pragma unroll
            for (int tt = 0; tt < 3; ++tt) {
                const int r = 3 * ci + tt;
                sm[t.s_rl + r] = (float)l;
                sm[t.s_rb + r] = tt == 0 ? bn : 0.0f;
                sm[t.s_rk + r] = (float)tt;
            }
        }
    }
    // self-contacts (Humanoid.yaml:80): lanes over geom pairs, compacted in pair order within
    // the MI_MAX_ROWS budget, after the ground contacts (as the oracle)
    if (TP::kSelf && t.self_on && t.s_seg >= 0) {
        // world segments of every geom, once (lanes over geoms)
        float* seg = sm + t.s_seg;
        float* bnd = seg + 8 * t.ngeoms;   // bounding sphere: centre (3), half-length + radius
        const float* geo = mcb + t.mc_geo;                                // LDS copy
        // geom pairs from the global table (cache-resident), the first 256 prefetched ahead of
        // the segment pass
        const int2* gpr = reinterpret_cast<const int2*>(t.g_pairs);
        int2 gpf[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int pi = 64 * q + lane;
            gpf[q] = pi < t.npairs ? gpr[pi] : make_int2(0, 0);
        }
        for (int g = lane; g < t.ngeoms; g += 64) {
            const float* A = geo + 8 * g;
            const int l = (int)A[0];
            float R[9], a0[3], a1[3];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
            m3_vec(R, A + 1, a0); m3_vec(R, A + 4, a1);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                seg[8 * g + q] = a0[q] + sm[t.s_o + 3 * l + q];
                seg[8 * g + 3 + q] = a1[q] + sm[t.s_o + 3 * l + q];
            }
            seg[8 * g + 6] = A[7];
            seg[8 * g + 7] = (float)l;
            float e2 = 0.0f;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                bnd[4 * g + q] = sm[t.s_o + 3 * l + q] + 0.5f * (a0[q] + a1[q]);
                e2 += (a1[q] - a0[q]) * (a1[q] - a0[q]);
            }
            bnd[4 * g + 3] = 0.5f * sqrtf(e2) + A[7];
        }
        wave_sync();
        // broad phase (conservative bounding spheres: the segments' distance is at least the
        // centre distance minus both half-lengths), survivors compacted in pair order
        int* surv = reinterpret_cast<int*>(sm + t.s_surv);
        int nsv = 0;
        const float slack = p.contact_offset + 1e-3f;
        auto broad = [&](int pb, int2 gpq, bool pref) {
            const int pi = pb + lane;
            bool keep = false;
            int2 gp = make_int2(0, 0);
            if (pi < t.npairs) {
                gp = pref ? gpq : gpr[pi];
                const float4 A = *reinterpret_cast<const float4*>(bnd + 4 * gp.x);
                const float4 B = *reinterpret_cast<const float4*>(bnd + 4 * gp.y);
                const float cx = A.x - B.x, cy = A.y - B.y, cz = A.z - B.z;
                const float reach = A.w + B.w + slack;
                keep = cx * cx + cy * cy + cz * cz < reach * reach;
            }
            const unsigned long long mask = __ballot(keep);
            if (keep) surv[nsv + __popcll(mask & ((1ull << lane) - 1ull))] = gp.x | (gp.y << 16);
            nsv += __popcll(mask);
        };
        // the prefetched blocks by compile-time index (a runtime pick among them went to scratch)
        sfor<0, 4>([&](auto Q) { if (64 * (int)Q < t.npairs) broad(64 * (int)Q, gpf[Q], true); });
        for (int pb = 256; pb < t.npairs; pb += 64) broad(pb, make_int2(0, 0), false);
        nsv = __builtin_amdgcn_readfirstlane(nsv);
        wave_sync();
        // narrow phase on the survivors (mi_geom.h, as the oracle)
        int budget = (MI_MAX_ROWS - 3 * ncon - t.nlimc) / 3;
        for (int sb = 0; sb < nsv && budget > 0; sb += 64) {
            const int sidx = sb + lane;
            bool act = false;
            float pc[3], n[3], bn = 0.0f;
            int la = 0, lb = 0;
            if (sidx < nsv) {
                const int pk = surv[sidx];                 // geom pair, packed (a | b << 16)
                const float* A = seg + 8 * (pk & 0xffff);
                const float* B = seg + 8 * (pk >> 16);
                la = (int)A[7]; lb = (int)B[7];
                const float gap = mi_pair_contact(A, A + 3, A[6], B, B + 3, B[6], pc, n);
                act = gap < p.contact_offset;
                const float d = gap - p.rest_offset;
                bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
            }
            const unsigned long long mask = __ballot(act);
            const int rank = __popcll(mask & ((1ull << lane) - 1ull));
            if (act && rank < budget) {
                const int ci = ncon + rank;
#pragma unroll
                for (int q = 0; q < 3; ++q) { sm[t.s_cp + 3 * ci + q] = pc[q]; sm[t.s_cn + 3 * ci + q] = n[q]; }
                sm[t.s_cl + ci] = (float)la;
                sm[t.s_cl2 + ci] = (float)lb;
#pragma unroll
                for (int tt = 0; tt < 3; ++tt) {
                    const int r = 3 * ci + tt;
                    sm[t.s_rl + r] = (float)la;
                    sm[t.s_rb + r] = tt == 0 ? bn : 0.0f;
                    sm[t.s_rk + r] = (float)tt;
                }
            }
            const int took = min(__popcll(mask), budget);
            ncon += took;
            budget -= took;
        }
        ncon = __builtin_amdgcn_readfirstlane(ncon);
    } else if (TP::kSelf && t.self_on) {
        int budget = (MI_MAX_ROWS - 3 * ncon - t.nlimc) / 3;
        for (int pb = 0; pb < t.npairs && budget > 0; pb += 64) {
            const int pi = pb + lane;
            bool act = false;
            float pc[3], n[3], bn = 0.0f;
            int la = 0, lb = 0;
            if (pi < t.npairs) {
                const int ga = t.g_pairs[2 * pi], gb = t.g_pairs[2 * pi + 1];
                const float* A = t.g_geo + 8 * ga;
                const float* B = t.g_geo + 8 * gb;
                la = (int)A[0]; lb = (int)B[0];
                float Ra[9], Rb[9], a0[3], a1[3], b0[3], b1[3];
#pragma unroll
                for (int q = 0; q < 9; ++q) { Ra[q] = sm[t.s_R + 9 * la + q]; Rb[q] = sm[t.s_R + 9 * lb + q]; }
                m3_vec(Ra, A + 1, a0); m3_vec(Ra, A + 4, a1);
                m3_vec(Rb, B + 1, b0); m3_vec(Rb, B + 4, b1);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    a0[q] += sm[t.s_o + 3 * la + q]; a1[q] += sm[t.s_o + 3 * la + q];
                    b0[q] += sm[t.s_o + 3 * lb + q]; b1[q] += sm[t.s_o + 3 * lb + q];
                }
                const float gap = mi_pair_contact(a0, a1, A[7], b0, b1, B[7], pc, n);
                act = gap < p.contact_offset;
                const float d = gap - p.rest_offset;
                bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
            }
            const unsigned long long mask = __ballot(act);
            const int rank = __popcll(mask & ((1ull << lane) - 1ull));
            if (act && rank < budget) {
                const int ci = ncon + rank;
#pragma unroll
                for (int q = 0; q < 3; ++q) { sm[t.s_cp + 3 * ci + q] = pc[q]; sm[t.s_cn + 3 * ci + q] = n[q]; }
                sm[t.s_cl + ci] = (float)la;
                sm[t.s_cl2 + ci] = (float)lb;
#pragma unroll
                for (int tt = 0; tt < 3; ++tt) {
                    const int r = 3 * ci + tt;
                    sm[t.s_rl + r] = (float)la;
                    sm[t.s_rb + r] = tt == 0 ? bn : 0.0f;
                    sm[t.s_rk + r] = (float)tt;
                }
            }
            const int took = min(__popcll(mask), budget);
            ncon += took;
            budget -= took;
        }
        ncon = __builtin_amdgcn_readfirstlane(ncon);
    }
    const int nc = 3 * ncon;
    wave_sync();

    STAMP(6);   // P8 contacts
    // ---- P7+P9: one batch, lanes over solve vectors b (64 per pass):
    //   b = 0                 rhs          -> u* = u + dt M~^-1 rhs
    //   b = 1 .. nlim         e_k of each limited DOF k (limit-row candidates; the row's
    //                         sign +-1 is applied once the limit test has run: exact)
    //   b = 1 + nlim + r      contact row r: J_r, W_r = M~^-1 J_r^T, A_rr = J_r . W_r
    // The limit test needs u*, so it runs inside the first pass (uniform barrier); limit rows
    // follow the contact rows in DOF order, as in the oracle.
    const int nlim = t.nlimc;
    const int total = 1 + nlim + nc;
    int nrows = nc;
    unsigned long long limact = 0ull;   // bit d: joint d has an active limit row
    float* xs = sm + t.s_xs + lane;     // generic path: this lane's private solve vector
    // u* (lane 0's solution) and the limit rows: first pass only, uniform barriers
    auto limit_rows = [&](const auto& res) {
        constexpr int NR = sizeof(res) / sizeof(res[0]);
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NR; ++c)
                if (c < nv) us[c] = us[c] + dt * res[c];
        }
        wave_sync();
        // limit rows from u* (lane = joint), compacted after the contact rows
        bool act = false;
        float bl = 0.0f, sg = 0.0f;
        if (lane < D) {
            const int l = lane + 1, k = nr + lane;
            const float lo = mc.lf(MC_LO, l), hi = mc.lf(MC_HI, l);
            if (lo < hi) {
                const float qj = sm[t.s_q + lane];
                const float qp = qj + dt * us[k];
                float d = 0.0f;
                if (qj < lo || qp < lo) { d = qj - lo; sg = 1.0f; act = true; }
                else if (qj > hi || qp > hi) { d = hi - qj; sg = -1.0f; act = true; }
                bl = p.tgs ? d : row_bias(p, d, dt, true);
            }
        }
        limact = __ballot(act);
        if (act) {
            const int rl = nc + __popcll(limact & ((1ull << lane) - 1ull));
            sm[t.s_rl + rl] = -(float)(nr + lane) - 1.0f;  // negative: limit row on dof
            sm[t.s_lsg + lane] = sg;   // sign of joint lane's limit row
            sm[t.s_rb + rl] = bl;
            sm[t.s_rk + rl] = 3.0f;
        }
        nrows = __builtin_amdgcn_readfirstlane(nc + __popcll(limact));   // wave-uniform
        wave_sync();
    };
    // file this lane's W row: contact row r (A_rr given), or an active limit row with its sign
    auto file_row = [&](const auto& res, bool on, int r, int kd, float a_contact) {
        constexpr int NR = sizeof(res) / sizeof(res[0]);
        int slot = -1;
        float sc = 1.0f, a = 0.0f;
        if (on && r >= 0) {
            slot = r;
            a = a_contact;
        } else if (kd >= 0) {
            const int d = kd - nr;
            if ((limact >> d) & 1ull) {
                slot = nc + __popcll(limact & ((1ull << d) - 1ull));
                sc = sm[t.s_lsg + d];
                float wk = 0.0f;
#pragma unroll
                for (int c = 0; c < NR; ++c) wk = c == kd ? res[c] : wk;
                a = wk;                          // J.W = sg^2 (M~^-1)_kk
            }
        }
        if (slot >= 0) {
            sm[t.s_ad + slot] = a > 1e-12f ? a : 1e-12f;
            if (kd >= 0 && slot < t.j_rows_lds) {    // limit row: J = sg e_kd
                float* jl = sm + t.s_J + slot * nv;
#pragma unroll
                for (int c = 0; c < WNV; ++c)
                    if (c < nv) jl[c] = c == kd ? sc : 0.0f;
            }
            if (nrows <= t.w_rows_lds) {   // uniform: every row of this substep fits in LDS
                float* wl = w_row<TP::kSelf>(t, sm, slot, nv);
#pragma unroll
                for (int c = 0; c < NR; ++c)
                    if (c < nv) wl[c] = res[c] * sc;
            } else {
#pragma unroll
                for (int c = 0; c < WNV; ++c) gW[(size_t)slot * WNV + c] = c < NR ? res[c] * sc : 0.0f;
            }
        }
    };
    for (int base = 0; base < total; base += 64) {
        const int bv = base + lane;
        const bool on = bv < total;
        const int r = bv - 1 - nlim;    // contact row (valid when r >= 0)
        const int kd = (on && bv > 0 && r < 0) ? nr + mc.lim(bv - 1) : -1;   // limit candidate
        if constexpr (TP::kCT) {
            // solve vector built in place: J_r, e_kd or the rhs
            float x[TP::nvc];
            // J_r = J_a^T f - J_b^T f (b: the second body of a self-contact, else none). Built
            // branch-free over the DOFs for every lane at once: S_c comes from wave-uniform LDS
            // broadcasts, each lane selects its own entry (contact row, rhs or e_kd), so the
            // contact lanes and the others no longer run as two serialised exec-masked halves
            // with a divergent branch per DOF. Same operations per entry (last-bit rounding of
            // the generated code differs; results agree to rounding, see the parity tests).
            const bool crow = on && r >= 0;
            float f[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
            unsigned msk = 0u, msk2 = 0u;
            if (crow) {
                const int l = (int)sm[t.s_rl + r];
                const float l2 = TP::kSelf ? sm[t.s_cl2 + r / 3] : -1.0f;
                msk = mc.mask(l);
                msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
                contact_row_f<TP::kSelf>(sm, t, r, f);
            }
            sfor<0, TP::nv>([&](auto C) {
                constexpr int c = C;
                float sv[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) sv[q] = Ss[6 * c + q];
                const float v = dot6(sv, f);
                const bool ia = (msk >> c) & 1u, ib = (msk2 >> c) & 1u;
                float xc = (ia ? v : 0.0f) - (ib ? v : 0.0f);
                float rc = rhs[c];   // uniform LDS broadcast
                // materialised on every lane: otherwise the compiler sinks the dot product and
                // the load into a divergent branch per DOF again
                asm volatile("" : "+v"(xc), "+v"(rc));
                x[c] = crow ? xc : (bv == 0 ? rc : (kd == c ? 1.0f : 0.0f));
            });
            if (on && r >= 0 && r < t.j_rows_lds) {   // keep J_r for the PGS sweeps
                float* jl = sm + t.s_J + r * TP::nv;
                sfor<0, TP::nv>([&](auto C) { jl[C] = x[C]; });
            }
            STAMP(7);   // P9 J build
            float a;                              // J M~^-1 J^T from the half solve
            ct_solve_l<TP>(sm + t.s_L, x, a);     // factor rows from LDS broadcasts
            STAMP(8);   // P9 solves
            if (base == 0) {
                limit_rows(x);
                STAMP(9);   // P9 u* + limit rows
            }
            file_row(x, on, r, kd, a);
        } else {
            float jr[WNV];
#pragma unroll
            for (int c = 0; c < WNV; ++c) jr[c] = 0.0f;
            if (on && r >= 0) {
                const int l = (int)sm[t.s_rl + r];
                const float l2 = TP::kSelf ? sm[t.s_cl2 + r / 3] : -1.0f;
                const unsigned msk = mc.mask(l), msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
                float f[6];
                contact_row_f<TP::kSelf>(sm, t, r, f);
#pragma unroll
                for (int c = 0; c < WNV; ++c) {
                    const bool ia = (msk >> c) & 1u, ib = (msk2 >> c) & 1u;
                    float v = 0.0f;
                    if (ia || ib) {
                        float sv[6];
#pragma unroll
                        for (int q = 0; q < 6; ++q) sv[q] = Ss[6 * c + q];
                        v = dot6(sv, f);
                    }
                    jr[c] = (ia ? v : 0.0f) - (ib ? v : 0.0f);
                }
            }
            STAMP(7);
            float wr[WNV];
#pragma unroll
            for (int c = 0; c < WNV; ++c)
                if (c < nv) xs[c * 64] = bv == 0 ? rhs[c] : (r >= 0 ? jr[c] : (kd == c ? 1.0f : 0.0f));
            tree_solve_lds(t, Mx, Dv, nv, xs);
#pragma unroll
            for (int c = 0; c < WNV; ++c) wr[c] = c < nv ? xs[c * 64] : 0.0f;
            STAMP(8);
            if (base == 0) {
                limit_rows(wr);
                STAMP(9);
            }
            float a = 0.0f;
#pragma unroll
            for (int c = 0; c < WNV; ++c) a += jr[c] * wr[c];
            file_row(wr, on, r, kd, a);
        }
        STAMP(10);
    }
    nrows = __builtin_amdgcn_readfirstlane(nrows);
    wave_sync();

    STAMP(10);  // P9 row filing + trailing barrier
    STAT(15, nrows);
    STAT(16, nrows > t.w_rows_lds);
    STAT(17, nrows > 64);
    STAT(18, total > 64);
    STAT(19, nrows > t.j_rows_lds);
    STAT(20, ncon);
    STAT(21, nrows > 16);
    STAT(22, nrows > 24);
    STAT(23, nrows > 32);
    STAT(24, nrows > 40);
    STAT(25, nrows > 48);
    STAT(26, t.w_rows_lds);
    STAT(27, t.j_rows_lds);
    // ---- P10: projected Gauss-Seidel. Lane k (mod 32) owns dof k; the wave's lower half
    // holds J / W of rows 0..63 in registers, the upper half rows 64..127. Rows are swept in
    // order; only the half owning the current row is active and u is copied across halves
    // between the two sub-sweeps. Row metadata and lambdas live in lane registers (row r in
    // lane r % 64, bank r / 64) and are read with readlane.
#ifndef MI_DIAG_NO_PGS
    // Delassus-space (lambda-space) sweeps on the compiled-topology path when every row's J and
    // W sit in LDS (the common case): lane r holds row r's v_r = J_r . u and its Delassus row
    // A[r][s] = J_r . W_s, so a row update is readlanes + the projection + one FMA per lane,
    // with no cross-lane reduction on the dependent chain; u = u* + sum_r W_r lambda_r after the
    // sweeps. Same row order, projection and lambda carry as the u-space sweeps below (equal in
    // exact arithmetic; float rounding differs).
    bool lam_done = false;
    if constexpr (TP::kCT) {
        if (nrows <= TP::kLamRows && nrows <= t.j_rows_lds && nrows <= t.w_rows_lds) {   // wave-uniform
            constexpr int NV = TP::nv;
            constexpr int RMAX = TP::kLamRows;                      // rows of this path
            const float* sJ = sm + t.s_J;
            float b = 0.0f, ia = 1.0f, lam = 0.0f;   // row kinds follow from the row index
            if (lane < nrows) {
                b = sm[t.s_rb + lane];
                ia = 1.0f / sm[t.s_ad + lane];
            }
            const int rl = lane < nrows ? lane : 0;
            float Jr[NV];
            sfor<0, NV>([&](auto C) { Jr[C] = sJ[rl * NV + C]; });
            float v = 0.0f;
            sfor<0, NV>([&](auto C) { v += Jr[C] * us[C]; });
            // Delassus row of lane r: A[r][s] = J_r . W_s. Four rows s per uniform branch, their
            // dot products interleaved (four independent FMA chains instead of one per basic
            // block); each chain keeps its sequential order (the generated code rounds a few
            // entries differently in the last bit: results agree to rounding, see the parity
            // tests). Rows past nrows in the last group re-read row nrows - 1 and are never used.
            float Ar[RMAX];
            static_assert(RMAX % 4 == 0, "Delassus rows are built four at a time");
#pragma unroll
            for (int g0 = 0; g0 < RMAX; g0 += 4) {
                float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
                if (g0 < nrows) {
                    const float* w0 = w_row<TP::kSelf>(t, sm, g0, NV);
                    const float* w1 = w_row<TP::kSelf>(t, sm, min(g0 + 1, nrows - 1), NV);
                    const float* w2 = w_row<TP::kSelf>(t, sm, min(g0 + 2, nrows - 1), NV);
                    const float* w3 = w_row<TP::kSelf>(t, sm, min(g0 + 3, nrows - 1), NV);
                    sfor<0, NV>([&](auto C) {
                        a0 += Jr[C] * w0[C];
                        a1 += Jr[C] * w1[C];
                        a2 += Jr[C] * w2[C];
                        a3 += Jr[C] * w3[C];
                    });
                }
                Ar[g0] = a0; Ar[g0 + 1] = a1; Ar[g0 + 2] = a2; Ar[g0 + 3] = a3;
            }
            const float mu = p.friction;
            // TGS: b holds the row's separation, ds the row's motion over the earlier sub-steps,
            // lsum its lambda summed over the sub-steps (u-bar = u* + W lsum / iters)
            [[maybe_unused]] const float sep = b;
            [[maybe_unused]] float ds = 0.0f, lsum = 0.0f;
            [[maybe_unused]] const int kdl = lane < nc ? lane % 3 : 3;
            for (int it = 0; it < p.iters + p.viters; ++it) {
                if constexpr (TP::kTgs)
                    b = (kdl == 1 || kdl == 2) ? 0.0f : row_bias(p, sep + ds, p.h, it < p.iters);
                // opaque per sweep: keeps the loop-invariant readlanes inside the sweep
                asm volatile("" : "+v"(b), "+v"(ia));
                int nrow_it = nrows;
                asm volatile("" : "+s"(nrow_it));
                float lamn = 0.0f;
                // fully unrolled by template (a rolled loop indexes Ar through s_set_gpr_idx and
                // branches per row); rows past nrows skipped by a uniform branch. Row kinds follow
                // from the row index: contact rows are (normal, friction, friction) triples, then
                // the limit rows.
                sfor<0, RMAX>([&](auto RR) {
                    constexpr int rr = RR;
                    if (rr < nrow_it) {
                        __builtin_amdgcn_sched_barrier(0);
                        const float vr = readlane(v, rr);
                        const float br = readlane(b, rr), iar = readlane(ia, rr);
                        const float l0 = readlane(lam, rr);
                        const int kind = rr < nc ? rr % 3 : 3;
                        const bool fric = kind == 1 || kind == 2;
                        const float lim = mu * lamn;
                        // normal / limit: lambda >= 0; friction: |lambda| <= mu lambda_n (one med3;
                        // lamn >= 0)
                        const float ln = __builtin_amdgcn_fmed3f(l0 + (br - vr) * iar, fric ? -lim : 0.0f,
                                                                 fric ? lim : __builtin_huge_valf());
                        if constexpr (rr % 3 == 0) lamn = kind == 0 ? ln : lamn;
                        v += Ar[rr] * (ln - l0);
                        lam = lane_here(lane) == rr ? ln : lam;
                    }
                });
                if constexpr (TP::kTgs) {
                    if (it < p.iters) { ds += p.h * v; lsum += lam; }
                }
            }
            float u = lane < NV ? us[lane] : 0.0f;
            [[maybe_unused]] float ub = u;
            [[maybe_unused]] const float lbar = lsum / (float)p.iters;
            const int kc = lane < NV ? lane : 0;
            // u = u* + sum_r W_r lambda_r in row order; four rows' W loads per uniform branch
            // (one LDS round trip per group instead of per row); rows past nrows add W 0
#pragma unroll
            for (int g0 = 0; g0 < RMAX; g0 += 4) {
                if (g0 >= nrows) break;
                float wq[4], lq[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    wq[q] = w_row<TP::kSelf>(t, sm, min(g0 + q, nrows - 1), NV)[kc];
                    lq[q] = g0 + q < nrows ? readlane(lam, g0 + q) : 0.0f;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) u += wq[q] * lq[q];
                if constexpr (TP::kTgs) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) ub += wq[q] * (g0 + q < nrows ? readlane(lbar, g0 + q) : 0.0f);
                }
            }
            if (lane < NV) us[lane] = u;
            if constexpr (TP::kTgs)   // the positions' velocity, in the dead rhs
                if (lane < NV) sm[t.s_r + lane] = ub;
            if (lane < nrows) sm[t.s_ad + lane] = lam;           // reuse: lambda of row lane
            lam_done = true;
        }
    }
    if (!lam_done)
    {
        const int half = lane >> 5, kl = lane & 31;
        // J_r[kl] is rebuilt per row from this lane's DOF subspace and the row's force
        // direction (the same dot6 as P9), so only W_r occupies registers
        float S6[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) S6[q] = kl < nv ? Ss[6 * kl + q] : 0.0f;
        // W rows: from LDS when this substep's rows all fit there (uniform branch), else by
        // bounded buffer loads from the slab (the descriptor covers rows [0, nrows), so slots
        // past the last row read as 0 without touching memory).
        // one bank (nrows <= 64): both half-waves hold rows 0..63, so every lane applies every
        // row's update and no half-to-half hand-over is needed; two banks: half h holds rows
        // 64h .. 64h+63.
        const bool one_bank = nrows <= 64;
        float Wr[64];
        if (nrows <= t.w_rows_lds) {                  // implies one_bank (w_rows_lds <= 64)
            const float km = kl < nv ? 1.0f : 0.0f;
            const int kc = kl < nv ? kl : 0;
            if constexpr (TP::kCT) {
#pragma unroll
                for (int rr = 0; rr < 64; ++rr)
                    Wr[rr] = w_row<TP::kSelf>(t, sm, min(rr, t.w_rows_lds - 1), TP::nv)[kc] * km;
            } else {
#pragma unroll
                for (int rr = 0; rr < 64; ++rr)
                    Wr[rr] = w_row<TP::kSelf>(t, sm, min(rr, t.w_rows_lds - 1), nv)[kc] * km;
            }
        } else {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)gW, (short)0, nrows * WNV * (int)sizeof(float), 0x00020000);
            const int vo = ((one_bank ? 0 : 64 * half) * WNV + kl) * (int)sizeof(float);
#pragma unroll
            for (int rr = 0; rr < 64; ++rr)
                Wr[rr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                       rs, vo + rr * WNV * (int)sizeof(float), 0, 0));
        }
        // row r's data in lane r % 64, bank r / 64: b, 1/A_rr, kind, DOF mask, f (6)
        float b0 = 0, b1 = 0, ia0 = 1, ia1 = 1, k0 = 0, k1 = 0, lam0 = 0.0f, lam1 = 0.0f;
        float fa[6] = {0, 0, 0, 0, 0, 0}, fb[6] = {0, 0, 0, 0, 0, 0};
        unsigned ma = 0u, mb = 0u, ma2 = 0u, mb2 = 0u;   // DOF masks of body a / body b
        {
            auto load_row = [&](int r, float& b, float& ia, float& k, float (&f)[6], unsigned& msk,
                                unsigned& msk2) {
                b = sm[t.s_rb + r];
                ia = 1.0f / sm[t.s_ad + r];
                k = sm[t.s_rk + r];
                const float lk = sm[t.s_rl + r];
                if (lk >= 0.0f) {
                    contact_row_f<TP::kSelf>(sm, t, r, f);
                    msk = mc.mask((int)lk);
                    const float l2 = TP::kSelf ? sm[t.s_cl2 + r / 3] : -1.0f;
                    msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
                } else {
                    const int kdof = (int)(-lk - 1.0f);
                    f[0] = sm[t.s_lsg + kdof - nr];      // limit row: J = sg e_k
                    msk = 1u << kdof;
                }
            };
            if (lane < nrows) load_row(lane, b0, ia0, k0, fa, ma, ma2);
            if (lane + 64 < nrows) load_row(lane + 64, b1, ia1, k1, fb, mb, mb2);
        }
        const float mu = p.friction;
        float u = kl < nv ? us[kl] : 0.0f;
        // One Gauss-Seidel sweep schedule. Per row: J_r . u by a DPP half-wave sum, the
        // projected lambda update, u += W_r dlambda. The next row's J (readlanes + dot6, no
        // dependence on u) is built inside the current row's schedule region so it overlaps the
        // reduction chain. The friction rows of a contact follow its normal row in the same
        // sweep, so the normal's current lambda is carried in a wave-uniform value.
        const float* sJl = sm + t.s_J + (kl < nv ? kl : 0);
        const float kin = kl < nv ? 1.0f : 0.0f;
        // TGS in u space: b0 / b1 hold the rows' separations; usum sums the sub-steps'
        // velocities (lane = DOF; each half keeps its copy), so row r has moved by h J_r usum
        [[maybe_unused]] float usum = 0.0f;
        auto sweeps = [&](auto ONE_, auto JL_) {
            constexpr bool ONE = decltype(ONE_)::value;
            constexpr bool JL = decltype(JL_)::value;   // J rows from LDS (one bank only)
            for (int it = 0; it < p.iters + p.viters; ++it) {
                // opaque per sweep: stops the compiler hoisting the loop-invariant readlanes of
                // every row out of the iteration loop (they would pin hundreds of SGPRs)
                asm volatile("" : "+v"(b0), "+v"(b1), "+v"(ia0), "+v"(ia1), "+v"(k0), "+v"(k1),
                             "+v"(ma), "+v"(mb), "+v"(ma2), "+v"(mb2));
                asm volatile("" : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]),
                             "+v"(fa[5]), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]),
                             "+v"(fb[4]), "+v"(fb[5]));
                int nrow_it = nrows;   // opaque: 128 hoisted "r < nrows" masks would spill
                asm volatile("" : "+s"(nrow_it));
                float lamn = 0.0f;
#pragma unroll
                for (int h = 0; h < (ONE ? 1 : 2); ++h) {
                    if (64 * h >= nrow_it) continue;
                    const float bb = h ? b1 : b0, ii = h ? ia1 : ia0, kk = h ? k1 : k0;
                    const unsigned mm = h ? mb : ma, mm2 = h ? mb2 : ma2;
                    auto jrow = [&](int rr, int& kind) -> float {
                        if constexpr (JL) {
                            kind = (int)readlane(kk, rr);
                            return sJl[rr * nv] * kin;
                        }
                        float fr[6];
#pragma unroll
                        for (int q = 0; q < 6; ++q) fr[q] = readlane(h ? fb[q] : fa[q], rr);
                        const unsigned msk = (unsigned)__builtin_amdgcn_readlane((int)mm, rr);
                        const unsigned msk2 = (unsigned)__builtin_amdgcn_readlane((int)mm2, rr);
                        kind = (int)readlane(kk, rr);
                        const float jc = kind == 3 ? fr[0] : dot6(S6, fr);
                        return (((msk >> kl) & 1u) ? jc : 0.0f) - (((msk2 >> kl) & 1u) ? jc : 0.0f);
                    };
                    int kind_c;
                    float jc_c = jrow(0, kind_c);
                    // fully unrolled (no early exit) so Wr stays register-indexed
#pragma unroll
                    for (int rr = 0; rr < 64; ++rr) {
                        const int r = rr + 64 * h;
                        if (r >= nrow_it) continue;
                        __builtin_amdgcn_sched_barrier(0);
                        int kind_n = 0;
                        float jc_n = 0.0f;
                        if (rr + 1 < 64) jc_n = jrow(rr + 1, kind_n);
                        const float s = half_sums(jc_c * u);
                        const float jv = readlane(s, h ? 63 : 31);
                        float br = readlane(bb, rr);
                        const float iar = readlane(ii, rr);
                        if constexpr (TP::kTgs) {
                            const float su = readlane(half_sums(jc_c * usum), h ? 63 : 31);
                            br = (kind_c == 1 || kind_c == 2) ? 0.0f : row_bias(p, br + p.h * su, p.h, it < p.iters);
                        }
                        const float l0 = readlane(h ? lam1 : lam0, rr);
                        float ln = l0 + (br - jv) * iar;
                        const bool fric = kind_c == 1 || kind_c == 2;
                        const float lim = mu * lamn;
                        ln = fmaxf(ln, fric ? -lim : 0.0f);     // normal / limit: lambda >= 0
                        ln = fric ? fminf(ln, lim) : ln;         // friction: |lambda| <= mu lambda_n
                        lamn = kind_c == 0 ? ln : lamn;
                        const float dl = ln - l0;
                        const int ln_id = lane_here(lane);
                        if constexpr (ONE) {
                            u += Wr[rr] * dl;
                        } else {
                            if ((ln_id >> 5) == h) u += Wr[rr] * dl;
                        }
                        if (ln_id == rr) { if (h) lam1 = ln; else lam0 = ln; }
                        jc_c = jc_n;
                        kind_c = kind_n;
                    }
                    // hand u to the other half for its sub-sweep
                    if constexpr (!ONE) u = __shfl(u, kl + 32 * h, 64);
                }
                if constexpr (TP::kTgs)
                    if (it < p.iters) usum += u;
            }
        };
        if (one_bank && nrows <= t.j_rows_lds) sweeps(std::true_type{}, std::true_type{});
        else if (one_bank) sweeps(std::true_type{}, std::false_type{});
        else sweeps(std::false_type{}, std::false_type{});
        if (lane < nv) us[lane] = u;
        if constexpr (TP::kTgs)   // the positions' velocity: the sub-steps' mean
            if (lane < nv) sm[t.s_r + lane] = usum / (float)p.iters;
        if (lane < nrows) sm[t.s_ad + lane] = lam0;          // reuse: lambda of row lane
        if (lane + 64 < nrows) sm[t.s_ad + lane + 64] = lam1;
    }
#endif
    wave_sync();

    STAMP(11);  // P10 PGS
    // ---- P11a: force sensors (lane s)
    if (lane < m.S) {
        const int si = lane, l = (int)mc.sf(MS_LINK, si);
        float R[9], xs[3], F[3] = {0, 0, 0}, T[3] = {0, 0, 0};
#pragma unroll
        for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
        const float sp[3] = {mc.sf(MS_X, si), mc.sf(MS_X + 1, si), mc.sf(MS_X + 2, si)};
        m3_vec(R, sp, xs);
#pragma unroll
        for (int q = 0; q < 3; ++q) xs[q] += sm[t.s_o + 3 * l + q];
        for (int c = 0; c < ncon; ++c) {
#pragma clang fp contract(off)
            // contact wrench on link l: +f on body a, -f on body b of a self-contact
            const float sgn = (int)sm[t.s_cl + c] == l ? 1.0f :
                              ((TP::kSelf && (int)sm[t.s_cl2 + c] == l) ? -1.0f : 0.0f);
            if (sgn == 0.0f) continue;
            const float* lam = sm + t.s_ad;
            const float fn = lam[3 * c] / dt, f1 = lam[3 * c + 1] / dt, f2 = lam[3 * c + 2] / dt;
            float d[9];
            contact_dirs<TP::kSelf>(sm, t, c, d);
            float fc[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) fc[q] = sgn * (fn * d[q] + f1 * d[3 + q] + f2 * d[6 + q]);
            float rr[3], tc[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) rr[q] = sm[t.s_cp + 3 * c + q] - xs[q];
            cross3(rr, fc, tc);
#pragma unroll
            for (int q = 0; q < 3; ++q) { F[q] += fc[q]; T[q] += tc[q]; }
        }
        float Fl[3], Tl[3];
        m3_tvec(R, F, Fl);
        m3_tvec(R, T, Tl);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            sm[t.s_rb + 6 * si + q] = Fl[q];         // LDS copy for the post-step and the
            sm[t.s_rb + 6 * si + 3 + q] = Tl[q];     // write-back (rb is dead after the PGS)
        }
    }
    // ---- P11b: integrate; non-finite -> nan flag
    bool finite = true;
    // TGS: positions advance with the sub-steps' mean velocity (in the dead rhs), the velocity
    // state is the last sweep's
    const float* up = TP::kTgs ? sm + t.s_r : us;
    if (lane < D) {
        const float v = us[nr + lane];
        const float qn = sm[t.s_q + lane] + dt * up[nr + lane];
        if (store_state) {
            st.qd[sx(st, lane, i)] = v;
            st.q[sx(st, lane, i)] = qn;
        }
        sm[t.s_q + lane] = qn;                       // final state stays in LDS (post-step)
        finite = isfinite(v) && isfinite(qn);
    }
    if (store_state && lane < 6 * m.S) st.sens[ssx(st, lane, i)] = sm[t.s_rb + lane];
    if (nr && lane == 0) {
        float u6[6], p6[6], rp[3], rq[4];
#pragma unroll
        for (int k = 0; k < 6; ++k) { u6[k] = us[k]; p6[k] = up[k]; }
#pragma unroll
        for (int k = 0; k < 3; ++k) rp[k] = sm[t.s_rp + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) rq[k] = sm[t.s_rp + 4 + k];
        if constexpr (TP::kTgs) {   // the velocity state's angular velocity cap
            const float wv = sqrtf(dot3(u6 + 3, u6 + 3));
            if (wv > p.max_angvel) {
                const float sc = p.max_angvel / wv;
                u6[3] *= sc; u6[4] *= sc; u6[5] *= sc;
            }
        }
        float* om = p6 + 3;
        float wn = sqrtf(dot3(om, om));
        if (wn > p.max_angvel) {
            const float sc = p.max_angvel / wn;
            om[0] *= sc; om[1] *= sc; om[2] *= sc;
            wn = p.max_angvel;
        }
        if constexpr (!TP::kTgs)
#pragma unroll
            for (int k = 0; k < 6; ++k) u6[k] = p6[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) rp[k] += dt * p6[k];
        const float th = wn * dt;
        if (th > 0.0f) {
            float sh, ch;
            sincosf(0.5f * th, &sh, &ch);
            sh = sh / wn;
            const float w0 = ch, x0 = om[0] * sh, y0 = om[1] * sh, z0 = om[2] * sh;
            const float w1 = rq[0], x1 = rq[1], y1 = rq[2], z1 = rq[3];
            float nq[4] = {w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1,
                           w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                           w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1,
                           w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1};
            const float nn = 1.0f / sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) rq[k] = nq[k] * nn;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) sm[t.s_rp + k] = rp[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) sm[t.s_rp + 4 + k] = rq[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) us[k] = u6[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) finite &= isfinite(rp[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) finite &= isfinite(rq[k]);
#pragma unroll
        for (int k = 0; k < 6; ++k) finite &= isfinite(u6[k]);
    }
    // root write-back from LDS, one field per lane (LDS operations of the wave complete in
    // order: lane 0's writes above are visible)
    if (nr && store_state) {
        if (lane < 3) st.root_pos[sx(st, lane, i)] = sm[t.s_rp + lane];
        else if (lane < 7) st.root_quat[sx(st, lane - 3, i)] = sm[t.s_rp + 4 + lane - 3];
        else if (lane < 13) st.root_vel[sx(st, lane - 7, i)] = us[lane - 7];
    }
    if (__any(!finite) && lane == 0) st.nan_flag[i] = 1;
    wave_sync();
    STAMP(12);  // P11
    STAMP_END();
}

// ---------------------------------------------------------------------------------------
// Wave-cooperative task layer of the fused env step (locomotion tasks). Same formulas, same
// evaluation order and the same Philox streams as the one-lane versions in mi_task.hpp; the
// work is spread over lanes (lane j = DOF j) and reads the LDS-resident physics state.
// ---------------------------------------------------------------------------------------

// VecEnvRLGames.step's clamp + action noise DR (vec_env_rlgames.py:57-60), then
// pre_physics_step (locomotion.py:103-145): mask-driven reset_idx, efforts. Returns lane j's
// action as pre_physics_step received it (task.actions[i, j]; 0 on lanes >= A).
MI_D float wave_task_pre(const DevModel& m, const WaveTabs& t, const DevState& st,
                         const DevTask& tp, int i, const float* actions, int64_t* reset_buf,
                         int64_t* progress_buf, float* potentials, float* prev_potentials,
                         float* actions_out) {
#pragma clang fp contract(off)
    const int lane = wave_lane(), N = st.N, D = m.D, A = tp.A;
    const bool flagged = reset_buf[i] != 0;      // wave-uniform
    mi_dr_env dre{};
    if (tp.dr_act) dre = dr_begin(st, tp, 1, i, flagged);
    if (flagged) {
        const uint64_t gid = (uint64_t)(st.off + i);
        const uint32_t cnt = st.reset_count[i];
        const float pn = tp.dof_pos_noise, vn = tp.dof_vel_noise;
        const float pw = (float)((double)pn - (double)(-pn));
        const float vw = (float)((double)vn - (double)(-vn));
        if (lane < D) {
            const int j = lane;
            float u[4];
            uniform4(st.seed, gid, cnt, (uint32_t)(j >> 2), 0, u);
            float v = tp.init_dof[j] + (pw * u[j & 3] + (-pn));
            const float lo = m.lower[j + 1], hi = m.upper[j + 1];
            if (lo < hi) { v = v < hi ? v : hi; v = v > lo ? v : lo; }
            st.q[sx(st, j, i)] = v;
            const int s = D + j;
            uniform4(st.seed, gid, cnt, (uint32_t)(s >> 2), 0, u);
            st.qd[sx(st, j, i)] = vw * u[s & 3] + (-vn);
        }
        if (lane < 3) {
            const float rp = st.origins[(size_t)lane * N + i] + tp.init_root_pos[lane];
            st.root_pos[sx(st, lane, i)] = rp;
        }
        if (lane < 4) st.root_quat[sx(st, lane, i)] = tp.init_root_quat[lane];
        if (lane < 6) st.root_vel[sx(st, lane, i)] = 0.0f;
        if (lane == 0) {
            float rp[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) rp[k] = st.origins[(size_t)k * N + i] + tp.init_root_pos[k];
            float tx = tp.target[0] - rp[0], ty = tp.target[1] - rp[1];
            float pot = -sqrtf(tx * tx + ty * ty + 0.0f * 0.0f) / tp.task_dt;
            prev_potentials[i] = pot;
            potentials[i] = pot;
            st.reset_count[i] = cnt + 1;
            reset_buf[i] = 0;
            progress_buf[i] = 0;
        }
    }
    float a = 0.0f;
    if (lane < A) {
        const int j = lane;
        a = clampf(actions[(size_t)A * i + j], -tp.clip_actions, tp.clip_actions);
        if (tp.dr_act) a = dr_col(st, tp, 1, dre, i, j, a);
        if (actions_out) actions_out[(size_t)A * i + j] = a;
        st.eff[sx(st, j, i)] = a * tp.gears[j] * tp.power_scale;
    }
    if (tp.dr_act && lane == 0) dr_store(st, 1, i, dre);
    return a;
}

// post_physics_step (rl_task.py:231-251 -> locomotion.py:80-101,173-183), observation noise
// DR (vec_env_rlgames.py:70-71) and _process_data's obs clamp, from the final physics state the
// last substep left in LDS. Writes the unclamped (noisy) row to obs_task (when given) and the
// clamped row to obs_out. a_lane: lane j's task.actions entry (wave_task_pre).
MI_D void wave_loco_post(const DevModel& m, const WaveTabs& t, const DevState& st,
                         const DevTask& tp, int i, float* sm, float a_lane,
                         float* obs_out, float* obs_task, float* rew, int64_t* reset_buf,
                         int64_t* progress_buf, float* potentials, float* prev_potentials,
                         float* rew_out, int64_t* reset_out) {
#pragma clang fp contract(off)
    const int lane = wave_lane(), D = m.D, S = m.S, O = tp.O;
    const float co = tp.clip_obs;
    const float* us = sm + t.s_us;
    float* out = obs_out + (size_t)O * i;
    float* raw = obs_task ? obs_task + (size_t)O * i : nullptr;
    // is_done's decision first (wave-uniform: obs0 = root z, progress, reset_buf, NaN flag) —
    // the observation noise schedule keys on the reset_buf it produces
    // (read by lane 0, which wrote them earlier in this launch, and broadcast)
    int64_t progress = 0, flagged = 0;
    int nan_env = 0;
    if (lane == 0) {
        progress = progress_buf[i] + 1;                      // rl_task.py:242
        flagged = reset_buf[i];
        nan_env = st.nan_flag[i];
    }
    progress = __shfl(progress, 0);
    flagged = __shfl(flagged, 0);
    nan_env = __shfl(nan_env, 0);
    const int64_t done = nan_env ? 1 : loco_done(tp, sm[t.s_rp + 2], flagged, progress);
    mi_dr_env dre{};
    if (tp.dr_obs) dre = dr_begin(st, tp, 0, i, done != 0);
    auto put = [&](int k, float v) {
        if (tp.dr_obs) v = dr_col(st, tp, 0, dre, i, k, v);
        if (raw) raw[k] = v;
        out[k] = clampf(v, -co, co);
    };
    float* terms = sm + t.s_rb + 6 * S;          // [3][D]: act^2, |a v| ratio, limit term
    // per-DOF entries (lane j)
    if (lane < D) {
        const int j = lane;
        const float pos = ref_unscale(sm[t.s_q + j], m.lower[j + 1], m.upper[j + 1]);
        const float vel = us[m.nr + j] * tp.dof_vel_scale;
        const float a = a_lane;
        put(12 + j, pos);
        put(12 + D + j, vel);
        put(12 + 2 * D + 6 * S + j, a);
        terms[j] = a * a;
        terms[D + j] = fabsf(a * vel) * tp.ratio[j];
        if (tp.kind == MI_TASK_HUMANOID) {
            const float aa = fabsf(pos);
            const float sc = tp.joints_at_limit_cost * (aa - 0.98f) / 0.02f;
            terms[2 * D + j] = (aa > 0.98f ? 1.0f : 0.0f) * sc * tp.ratio[j];
        } else {
            terms[2 * D + j] = pos > 0.99f ? 1.0f : 0.0f;
        }
    }
    if (lane < 6 * S) put(12 + 2 * D + lane, sm[t.s_rb + lane] * tp.contact_force_scale);
    wave_sync();
    if (lane == 0) {
        float rp[3], rq[4], rv[6];
#pragma unroll
        for (int k = 0; k < 3; ++k) rp[k] = sm[t.s_rp + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) rq[k] = sm[t.s_rp + 4 + k];
#pragma unroll
        for (int k = 0; k < 6; ++k) rv[k] = us[k];
        float tt[3] = {tp.target[0] - rp[0], tp.target[1] - rp[1], tp.target[2] - rp[2]};
        tt[2] = 0.0f;
        const float prev_p = potentials[i];
        const float nrm = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
        const float new_p = -nrm / tp.task_dt;
        const float inv_start[4] = {1.0f, -0.0f, -0.0f, -0.0f};
        float tq[4];
        ref_quat_mul(rq, inv_start, tq);
        const float b0[3] = {1.0f, 0.0f, 0.0f}, b1[3] = {0.0f, 0.0f, 1.0f};
        float up[3], hd[3];
        ref_quat_rotate<false>(tq, b1, up);
        ref_quat_rotate<false>(tq, b0, hd);
        float tn = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
        tn = tn > 1e-9f ? tn : 1e-9f;
        const float td[3] = {tt[0] / tn, tt[1] / tn, tt[2] / tn};
        const float heading_proj = hd[0] * td[0] + hd[1] * td[1] + hd[2] * td[2];
        float vl[3], al[3];
        ref_quat_rotate<true>(tq, rv, vl);
        ref_quat_rotate<true>(tq, rv + 3, al);
        float roll, pitch, yaw;
        ref_get_euler_xyz(tq, roll, pitch, yaw);
        const float walk = atan2f(tp.target[2] - rp[2], tp.target[0] - rp[0]);
        const float angle_to_target = walk - yaw;
        const float o10 = up[2], o11 = heading_proj;
        put(0, rp[2]);
        put(1, vl[0]); put(2, vl[1]); put(3, vl[2]);
        put(4, al[0] * tp.angular_velocity_scale);
        put(5, al[1] * tp.angular_velocity_scale);
        put(6, al[2] * tp.angular_velocity_scale);
        put(7, ref_normalize_angle(yaw));
        put(8, ref_normalize_angle(roll));
        put(9, ref_normalize_angle(angle_to_target));
        put(10, o10);
        put(11, o11);
        potentials[i] = new_p;
        prev_potentials[i] = prev_p;
        // calculate_metrics: sums in DOF order, as loco_reward
        float limit_cost = 0.0f, act_cost = 0.0f, elec = 0.0f;
        if (tp.kind == MI_TASK_HUMANOID) {
            for (int j = 0; j < D; ++j) limit_cost += terms[2 * D + j];
        } else {
            int64_t cnt = 0;
            for (int j = 0; j < D; ++j) cnt += terms[2 * D + j] != 0.0f;
            limit_cost = (float)cnt;
        }
        const float heading = o11 > 0.8f ? tp.heading_weight : tp.heading_weight * o11 / 0.8f;
        const float upr = o10 > 0.93f ? 0.0f + tp.up_weight : 0.0f;
        for (int j = 0; j < D; ++j) act_cost += terms[j];
        for (int j = 0; j < D; ++j) elec += terms[D + j];
        float total = (new_p - prev_p) + tp.alive_reward_scale + upr + heading -
                      tp.actions_cost * act_cost - tp.energy_cost * elec - limit_cost;
        if (rp[2] < tp.termination_height) total = tp.death_cost;
        rew[i] = total;
        // is_done + NaN guard (decided above); progress_buf += 1
        if (nan_env) {
            st.nan_flag[i] = 0;
            atomicAdd(st.nan_total, 1ull);
        }
        if (tp.dr_obs) dr_store(st, 0, i, dre);
        reset_buf[i] = done;
        progress_buf[i] = progress;
        if (rew_out) rew_out[i] = total;          // _process_data's returned copies
        if (reset_out) reset_out[i] = done;
    }
}

}  // namespace mi
