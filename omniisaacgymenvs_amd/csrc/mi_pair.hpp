// mi_pair.hpp — two envs per wavefront (gfx950), for compiled topologies with nv <= 32.
//
// The wavefront-per-env kernel (mi_wave.hpp) runs most phases on one lane per DOF, link or
// constraint row: 22-27 of the 64 lanes for the Humanoid. Here each 32-lane half of a wave owns
// one env, so every instruction advances two envs, and a workgroup of 8 waves holds 16 envs —
// the whole per-CU share of a 4096-env launch resident in ONE round (the wave kernel runs two
// rounds of 8 envs per CU: its registers allow 2 waves per SIMD). Same algorithm, same constraint
// rows in the same order, same task math as mi_wave.hpp and the oracle; what changes is the
// mapping:
//   * lane = lane & 31 inside the env's half; cross-lane broadcasts read the half's own lane
//     (pbc: two v_readlane + a select), ballots are taken per half (hballot);
//   * per-env counts (contacts, constraint rows, survivors) are per-half values; loops run to
//     the larger of the two halves with per-half guards;
//   * LDS per env is cut to what 16 envs per CU allow: no stored J rows (the Delassus set-up
//     rebuilds J_r in lane r from the contact data), W rows up to the budget (the rest of a
//     row-heavy substep goes through the env's global slab).
// Requirements checked on the host: compiled topology, nv <= 32, npts <= 64, even env count.
#pragma once
#include "mi_wave.hpp"

// Issue priority by contact load: the launch lasts as long as its slowest waves, and those are
// the contact-heavy envs (constraint rows grow every later phase: P9 solves and filing, the PGS
// width, the sensor sums). Once a half of the wave has more than MI_PRIO_C1 / C2 / C3 contact rows
// in a substep, the wave takes its SIMD's issue slots ahead of a lighter partner at priority
// 1 / 2 / 3 for the rest of its life (never lowered: `prio` carries across substeps). The light
// partner has slack: it finishes early anyway. Priority moves the schedule, never a result.
#ifndef MI_PAIR_SOLVE_PD
#define MI_PAIR_SOLVE_PD 3   // factor-entry prefetch depth of the P9 solves (ct_solve_l)
#endif
#ifndef MI_PRIO_C1
#define MI_PRIO_C1 12
#endif
#ifndef MI_PRIO_C2
#define MI_PRIO_C2 18
#endif
#ifndef MI_PRIO_C3
#define MI_PRIO_C3 27
#endif

namespace mi {

MI_D int pair_l64() { return (int)(threadIdx.x & 63u); }
// v of lane k of this lane's half (k wave-uniform)
MI_D float pbc(float v, int k) {
    const float a = readlane(v, k), b = readlane(v, k + 32);
    return (pair_l64() & 32) ? b : a;
}
// the same for a compile-time k, without SGPRs: row_newbcast:(k % 16) (DPP, gfx90a+) gives every
// 16-lane row the value of its own lane k % 16; v_permlane16_swap (gfx950) of that register with
// itself then spreads the even rows (k < 16: rows 0 and 2 hold lanes k and 32 + k) or the odd
// rows (k >= 16) over their 32-lane half. Two VALU ops instead of two v_readlane, two v_mov and
// a v_cndmask; exact (a broadcast)
template <int K>
MI_D float pbcc(float v) {
    static_assert(K >= 0 && K < 32, "lane of the half");
    const int t = __builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + (K & 15), 0xF, 0xF, false);
    const auto r = __builtin_amdgcn_permlane16_swap(t, t, false, false);
    return __int_as_float((int)(K < 16 ? r[0] : r[1]));
}
MI_D int pbci(int v, int k) {
    const int a = __builtin_amdgcn_readlane(v, k), b = __builtin_amdgcn_readlane(v, k + 32);
    return (pair_l64() & 32) ? b : a;
}
// ballot of this lane's half, bit j = half lane j
MI_D unsigned hballot(bool p) {
    const unsigned long long m = __ballot(p);
    return (unsigned)(m >> (pair_l64() & 32));
}
MI_D unsigned lanemask_lt(int lane) { return (1u << lane) - 1u; }
// index of the j-th (0-based) set bit of m, j < popc(m): binary search on popcounts
MI_D int nth_bit(unsigned m, int j) {
    int b = 0;
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const int c = __popc((m >> b) & ((1u << w) - 1u));
        if (j >= c) { j -= c; b += w; }
    }
    return b;
}
// the k lowest set bits of m
MI_D unsigned low_bits(unsigned m, int k) {
    return k >= __popc(m) ? m : (m & ((1u << nth_bit(m, k)) - 1u));
}
// larger of the two halves' (half-uniform) values: wave-uniform
MI_D int pmax(int v) { return max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 32)); }
// sum over each 32-lane half, returned to every lane of the half
MI_D float psum(float v) { return pbc(half_sums(v), 31); }

// in-register tree LTDL (ct_ltdl) with per-half broadcasts
template <class T>
MI_D void ct_ltdl_pair(int lane, float (&Mc)[T::nvc]) {
    sfor_down<0, T::nv>([&](auto K) {
        constexpr int k = K;
        // no scheduling barrier per pivot: pivots of different limbs overlap (0.1262 -> 0.1254
        // ms A/B; a barrier every 2 or 4 pivots the same; no spills either way)
        const int ln = lane_here(lane);
        const float inv = __builtin_amdgcn_rcpf(pbcc<k>(Mc[k]));
        sfor<T::dof.anc_start[k], T::dof.anc_start[k + 1]>([&](auto A) {
            constexpr int ii = T::dof.anc[A];
            const float s = pbcc<ii>(Mc[k]) * inv;
            if (ln <= ii) Mc[ii] -= s * Mc[k];
        });
        if (ln < k) Mc[k] = Mc[k] * inv;
    });
}

// Per-DOF loop over the motion subspaces S_c (6 floats per DOF in LDS, uniform per half) and,
// with R, the rhs entries R[c]: fn(c, S_c, R[c]) with the loads of DOF c + SP issued before DOF c's
// arithmetic, into a ring of SP + 1 buffers indexed at compile time. Each DOF's arithmetic is a
// handful of VALU ops, so with the loads in line every DOF exposed a full LDS round trip.
// S0: the first DOF whose S_c is read (the callers that know S_c of the free root's six DOFs
// at compile time pass TP::nr; fn then gets an unread sv for c < S0).
template <class TP, int SP, bool WITH_R, int S0 = 0, class F>
MI_D void sdof_loop(const float* Ss, const float* R, F&& fn) {
    constexpr int NB = SP + 1;
    float sb[NB][6], rb[NB];
    auto load = [&](auto C) {
        constexpr int c = C;
        if constexpr (c >= S0) {
#pragma unroll
            for (int q = 0; q < 6; ++q) sb[c % NB][q] = Ss[6 * c + q];
        }
        if constexpr (WITH_R) rb[c % NB] = R[c];
    };
    sfor<0, (SP < TP::nv ? SP : TP::nv)>([&](auto C) { load(C); });
    sfor<0, TP::nv>([&](auto C) {
        constexpr int c = C;
        if constexpr (c + SP < TP::nv) load(std::integral_constant<int, c + SP>{});
        fn(C, sb[c % NB], WITH_R ? rb[c % NB] : 0.0f);
    });
}
#ifndef MI_PAIR_WIDE_PD
#define MI_PAIR_WIDE_PD 16   // W-row prefetch depth of the wide Delassus set-up (A/B round 4: 4 0.1360, 8 0.1335, 12 0.1331 ms; later 12 0.1240, 16 0.1226)
#endif
#ifndef MI_PAIR_WIDE_AREG
// wide-PGS Delassus rows in registers (a multiple of 4, <= 64); the rest streamed from the wave's
// scratch. 28 since round 6: at 32 the TGS kernel spilled 16 B of VGPRs per lane (stored once
// per wave: 512 B/env of scratch writes, 1 241 B/env of WRITE_SIZE); at 28 it is spill-free
// (863 B/env) for +0.3 % kernel time (alternating A/B, profiles/r06/ab_areg/)
#define MI_PAIR_WIDE_AREG 28
#endif
#ifndef MI_PAIR_WIDE_MFMA_HOIST
#define MI_PAIR_WIDE_MFMA_HOIST 1   // MFMA set-up: all row blocks' J operands loaded before the tiles
#endif
#ifndef MI_PAIR_WIDE_MFMA
#define MI_PAIR_WIDE_MFMA 0   // wide Delassus set-up as f32 MFMA tiles through the wave's scratch (0: per-lane FMA rows;
                                // A/B round 5: MFMA 0.1371 ms, operands hoisted 0.1272, FMA 0.1245)
#endif
// the wave's global scratch of the wide sweeps, rows of 64 lanes of f32 per wave (N / 2 waves):
// with the MFMA set-up the whole 64 x 64 Delassus block plus J^T (up to 32 DOF columns); else
// the rows AREG..63 the sweeps stream (the rest stay in registers)
constexpr int kWideScratchRows = MI_PAIR_WIDE_MFMA ? 64 + 32 : 64 - MI_PAIR_WIDE_AREG;
#ifndef MI_PAIR_WIDE_AP
#define MI_PAIR_WIDE_AP 8   // Delassus rows streamed ahead of the wide sweeps' chain
#endif
#ifndef MI_PAIR_SWEEP_FMA
#define MI_PAIR_SWEEP_FMA 1   // PGS row step as two FMAs around the projection (0: l0 + (b - v) / A_rr, v + A (ln - l0))
#endif
#ifndef MI_PAIR_WIDE_UPF
#define MI_PAIR_WIDE_UPF 1   // wide u update: next group's W column loaded ahead (0: in order)
#endif
#ifndef MI_PAIR_LIM_NEAR
#define MI_PAIR_LIM_NEAR 0.05f   // rad / m: a joint this close to a limit is speculated on first
#endif
#ifndef MI_PAIR_LIM_SPEC_MIN_D
#define MI_PAIR_LIM_SPEC_MIN_D 16   // speculative limit-candidate lanes for models with >= this many DOFs
#endif
#ifndef MI_PAIR_JREUSE_MAXNV
#define MI_PAIR_JREUSE_MAXNV 16   // narrow PGS reuses P9's J rows for models with nv <= this
#endif
#ifndef MI_PAIR_SDOF_PD
#define MI_PAIR_SDOF_PD 6   // DOF-loop prefetch depth (sdof_loop): 2 -> 0.1609 ms, 4 -> 0.1592 (A/B, round 3); 6: 0.1356 -> 0.1349 (round 4)
#endif

// S_c . f for DOF c: the free root's six DOFs have unit subspaces (linear x, y, z then angular
// x, y, z: the P1 set-up below), so their dot product is one component of f (what dot6 with a
// unit vector returns, up to the sign of a zero); the joint DOFs' from S_c in LDS
typedef float pv2 __attribute__((ext_vector_type(2)));
// dot6 as two packed-FP32 chains (even / odd terms, v_pk_mul + 2 v_pk_fma + one add: 4 VALU
// ops instead of 6); the summation order is (a0 b0 + a2 b2 + a4 b4) + (a1 b1 + a3 b3 + a5 b5)
MI_D float dot6p(const float (&a)[6], const float (&b)[6]) {
    pv2 p = pv2{a[0], a[1]} * pv2{b[0], b[1]};
    p = __builtin_elementwise_fma(pv2{a[2], a[3]}, pv2{b[2], b[3]}, p);
    p = __builtin_elementwise_fma(pv2{a[4], a[5]}, pv2{b[4], b[5]}, p);
    return p.x + p.y;
}
// J_r . u over the NV DOFs (u in LDS, uniform per half) as two packed-FP32 chains (even / odd
// DOFs), then their sum: the narrow and the wide PGS form v_r the same way
template <int NV, int NVC>
MI_D float pk_jdot(const float (&J)[NVC], const float* u) {
#if MI_PK_DOT
    pv2 p = {0.0f, 0.0f};
    sfor<0, NV / 2>([&](auto H) {
        constexpr int c = 2 * H;
        p = __builtin_elementwise_fma(pv2{J[c], J[c + 1]}, pv2{u[c], u[c + 1]}, p);
    });
    float v = p.x + p.y;
    if constexpr (NV % 2) v += J[NV - 1] * u[NV - 1];
    return v;
#else
    float v = 0.0f;
    sfor<0, NV>([&](auto C) { v += J[C] * u[C]; });
    return v;
#endif
}
template <class TP, int c>
MI_D float sdot(const float (&sv)[6], const float (&f)[6]) {
    if constexpr (TP::nr == 6 && c < 6) return f[c < 3 ? 3 + c : c - 3];
#if MI_PK_DOT
    else return dot6p(sv, f);
#else
    else return dot6(sv, f);
#endif
}
constexpr int sdof_first_loaded(int nr) { return nr == 6 ? 6 : 0; }

// J_r[c] of this lane's constraint row r (contact or limit), for every DOF c (lane = row)
template <class TP>
MI_D void pair_jrow(const MC& mc, const WaveTabs& t, const float* sm, int r, int nr,
                    float (&J)[TP::nvc]) {
    const float lk = sm[t.s_rl + r];
    float f[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    unsigned msk = 0u, msk2 = 0u;
    float sg = 0.0f;
    int kdof = -1;
    if (lk >= 0.0f) {
        msk = mc.mask((int)lk);
        const float l2 = TP::kSelf ? sm[t.s_cl2 + r / 3] : -1.0f;
        msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
        contact_row_f<TP::kSelf>(sm, t, r, f);
    } else {
        kdof = (int)(-lk - 1.0f);
        sg = sm[t.s_lsg + kdof - nr];
    }
    const float* Ss = sm + t.s_S;
    sdof_loop<TP, MI_PAIR_SDOF_PD, false, sdof_first_loaded(TP::nr)>(Ss, nullptr, [&](auto C, const float (&sv)[6], float) {
        constexpr int c = C;
        const float v = sdot<TP, c>(sv, f);
        const bool ia = (msk >> c) & 1u, ib = (msk2 >> c) & 1u;
        float xc = (ia ? v : 0.0f) - (ib ? v : 0.0f);
        asm volatile("" : "+v"(xc));
        J[c] = kdof >= 0 ? (kdof == c ? sg : 0.0f) : xc;
    });
}

// W row r of this lane's env: LDS rows [0, w_rows_lds) (one segment: the pair layout has no
// second), the env's global slab beyond
// LDS-typed pointer: loads through it are ds_reads even where the compiler would merge them
// with the slab path of the same expression into flat loads
typedef const float __attribute__((address_space(3)))* lds_cf;
MI_D lds_cf lds_ptr(const float* p) { return (lds_cf)p; }
// The LDS W rows of the paired kernels sit in groups of four rows, DOF-major inside a group:
// entry (r, c) at s_W + (r & ~3) nv + 4 c + (r & 3). One ds_read_b128 then returns rows
// 4g..4g+3 of one DOF — the Delassus set-up's four row chains (one uniform address for the
// wave) and the u update's four rows of the lane's DOF — instead of four ds_read_b32.
// w_rows_lds is a multiple of 4 (host), so a group is wholly in LDS or wholly in the slab.
typedef float pv4 __attribute__((ext_vector_type(4)));
#ifndef MI_PK_FMA
#define MI_PK_FMA 1   // Delassus set-up on packed FP32 FMAs (v_pk_fma_f32)
#endif
#ifndef MI_PK_DOT
#define MI_PK_DOT 1   // S_c . f (J rows, CRBA columns) as two packed-FP32 chains
#endif
typedef const pv4 __attribute__((address_space(3)))* lds_cf4;
MI_D int pw_idx(int r, int c, int nv) { return (r & ~3) * nv + 4 * c + (r & 3); }
// The env's global W slab (rows >= w_rows_lds, up to MI_MAX_ROWS) uses the same 4-row groups,
// WNV (32) columns: entry (r, c) at (r & ~3) WNV + 4 c + (r & 3), so a slab group is one
// global_load_dwordx4 per DOF as well (column WNV - 1 is the fallback sweeps' lambda slot)
MI_D size_t pair_sidx(int r, int c) { return (size_t)(r & ~3) * WNV + 4 * c + (r & 3); }
typedef const pv4* glb_cf4;

// The W-row sources of one env for a PGS phase, read from the parameter block ONCE: through
// WaveTabs every 4-row group re-read w_rows_lds / s_W with a scalar load and waited for it
// before its first W load (a serial round trip per group in the set-up and the u update).
// kLds: the narrow path, whose rows are all LDS rows (host-checked: w_rows_lds >= kLamRows).
struct WSrc {
    lds_cf W;          // the env's LDS W rows
    const float* gW;   // the env's slab (rows >= nl)
    int nl;            // LDS rows
};
MI_D WSrc make_wsrc(const WaveTabs& t, const float* sm, const float* gW) {
    WSrc w;
    w.W = lds_ptr(sm + t.s_W);
    int nl = t.w_rows_lds;
    asm volatile("" : "+s"(nl));   // kept (or spilled to a lane), not re-read from memory
    w.nl = nl;
    w.gW = gW;
    return w;
}

// Delassus entries A[r][g0 + q] = J_r . W_{g0+q}, q < 4, of this lane's row r (the PGS set-up of
// both widths), the loads of DOF c + PD issued before DOF c's FMAs (a ring indexed at compile
// time, see sdof_loop). The env has n rows; group rows past them are 0 (they hold stale data,
// finite or not, and the sweeps only ever scale them by a zero lambda change).
// (W rows from a WSrc: LDS rows [0, nl), the slab beyond; kLds: LDS rows only)
template <class TP, int PD, bool kLds>
MI_D void pair_dgroup_w(const WSrc& ws, int g0, int n, const float (&Jr)[TP::nvc], float (&a)[4]) {
    constexpr int NV = TP::nv, NB = PD + 1;
#if MI_PK_FMA
    // two rows' chains per v_pk_fma_f32 (the same fused multiply-add per element, half the
    // VALU instructions)
    pv2 a01 = {0.0f, 0.0f}, a23 = {0.0f, 0.0f};
    auto acc = [&](auto C, const pv4& w) {
        const pv2 j = {Jr[C], Jr[C]};
        a01 = __builtin_elementwise_fma(j, w.xy, a01);
        a23 = __builtin_elementwise_fma(j, w.zw, a23);
    };
#else
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    auto acc = [&](auto C, const pv4& w) {
        a0 += Jr[C] * w.x;
        a1 += Jr[C] * w.y;
        a2 += Jr[C] * w.z;
        a3 += Jr[C] * w.w;
    };
#endif
    if (kLds || g0 + 3 < ws.nl) {
        const lds_cf4 W = (lds_cf4)(ws.W + g0 * NV);
        pv4 wb[NB];
        sfor<0, (PD < NV ? PD : NV)>([&](auto C) { wb[C % NB] = W[C]; });
        sfor<0, NV>([&](auto C) {
            constexpr int c = C;
            if constexpr (c + PD < NV) wb[(c + PD) % NB] = W[c + PD];
            acc(C, wb[c % NB]);
        });
    } else {
        const glb_cf4 W = (glb_cf4)(ws.gW + (size_t)g0 * WNV);
        pv4 wb[NB];
        sfor<0, (PD < NV ? PD : NV)>([&](auto C) { wb[C % NB] = W[C]; });
        sfor<0, NV>([&](auto C) {
            constexpr int c = C;
            if constexpr (c + PD < NV) wb[(c + PD) % NB] = W[c + PD];
            acc(C, wb[c % NB]);
        });
    }
#if MI_PK_FMA
    const float a0 = a01.x, a1 = a01.y, a2 = a23.x, a3 = a23.y;
#endif
    a[0] = g0 < n ? a0 : 0.0f;
    a[1] = g0 + 1 < n ? a1 : 0.0f;
    a[2] = g0 + 2 < n ? a2 : 0.0f;
    a[3] = g0 + 3 < n ? a3 : 0.0f;
}
// W entries of rows g0..g0+3 at this lane's DOF kc (the u update of both PGS widths; rows past
// the env's count are read but never used: the caller selects them away)
template <bool kLds>
MI_D void pair_wcol_w(const WSrc& ws, int g0, int kc, int nv, float (&wq)[4]) {
    const pv4 w = (kLds || g0 + 3 < ws.nl) ? ((lds_cf4)(ws.W + g0 * nv))[kc]
                                           : ((glb_cf4)(ws.gW + (size_t)g0 * WNV))[kc];
    wq[0] = w.x; wq[1] = w.y; wq[2] = w.z; wq[3] = w.w;
}


// One articulated substep of the env of this lane's half (env i, LDS region sm, W slab gW).
template <class TP>
MI_D void pair_artic_substep(const DevModel& m, const WaveTabs& t, const DevState& st,
                             const SimP& p, int i, int wv_, const float* mcb, float* sm, float* gW,
                             bool load_state, bool store_state, int& prio, int& load) {
    static_assert(TP::kCT && TP::nv <= 32, "paired kernel: compiled topology, nv <= 32");
    const int lane = pair_l64() & 31;
    const int N = st.N, L = m.L, D = m.D, nv = m.nv, nr = m.nr;
    (void)N;
    const float dt = p.dt;
    float* us = sm + t.s_us;
    float* rhs = sm + t.s_r;
    float* Mx = sm + t.s_M;
    float* Ss = sm + t.s_S;
    const MC mc = make_mc(t, mcb, L);

    STAMP_BEGIN();
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
    STAMP(0);
    // ---- P1: local transforms, then chain walks + link inertia / Newton-Euler (lane = link)
    for (int l = 1 + lane; l < L; l += 32) wave_link_local(mc, t, sm, l);
    wave_sync();
    for (int l = lane; l < L; l += 32) wave_link_forward(mc, nr, t, sm, l, p);
    wave_sync();
    STAMP(1);
    // ---- P2: composite inertia / force
    float* aux = sm + t.s_X;
    {
        // native 4-vectors: each record sum is two v_pk_add_f32 per float4 (the same adds)
        const pv4* recs = reinterpret_cast<const pv4*>(sm + t.s_F);
        for (int l = lane; l < L; l += 32) {
            pv4 a0 = recs[4 * l], a1 = recs[4 * l + 1], a2 = recs[4 * l + 2], a3 = recs[4 * l + 3];
            for (int di = mc.desc_start(l); di < mc.desc_start(l + 1); ++di) {
                const int d = mc.desc(di);
                a0 += recs[4 * d];
                a1 += recs[4 * d + 1];
                a2 += recs[4 * d + 2];
                a3 += recs[4 * d + 3];
            }
            pv4* o = reinterpret_cast<pv4*>(aux) + 4 * l;
            o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3;
        }
    }
    wave_sync();
    STAMP(2);
    // ---- P3: bias + CRBA rows (lane = DOF)
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
        sdof_loop<TP, MI_PAIR_SDOF_PD, false, sdof_first_loaded(TP::nr)>(Ss, nullptr, [&](auto J, const float (&sj)[6], float) {
            constexpr int j = J;
            Mx[k * nv + j] = sdot<TP, j>(sj, f);
        });
        Mx[k * nv + k] = diag;
    }
    wave_sync();
    STAMP(3);
    // ---- P4: register LTDL (lane = column), factor published to LDS
    float Mc[TP::nvc];
    ct_load_columns<TP>(Mx, lane, Mc);
    ct_ltdl_pair<TP>(lane, Mc);
    STAMP(5);
    const float dvec = ct_dinv<TP>(lane, Mc);
    {
        const int dj = lane < nr ? lane : __builtin_popcount(mc.mask(lane < nv ? lane - nr + 1 : 0)) - 1;
        ct_publish_factor<TP>(lane, dj, Mc, dvec, sm + t.s_L);
    }
    STAMP(4);
    // ---- P8: ground contacts (lanes over candidate points, two passes past 32), ballot
    // compaction per half in candidate order
    int ncon = 0;
    {
        const float rpz = sm[t.s_rp + 2];
        for (int c0 = 0; c0 < t.npts; c0 += 32) {
            const int c = c0 + lane;
            bool act = false;
            float pc[3] = {0, 0, 0}, bn = 0.0f;
            int l = 0;
            if (c < t.npts) {
                l = (int)mc.pf(MP_LINK, c);
                const float pl[3] = {mc.pf(MP_X, c), mc.pf(MP_X + 1, c), mc.pf(MP_X + 2, c)};
                float R[9], x[3];
#pragma unroll
                for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
                m3_vec(R, pl, x);
#pragma unroll
                for (int q = 0; q < 3; ++q) x[q] += sm[t.s_o + 3 * l + q];
                const float rr = mc.pf(MP_RAD, c);
                const float gap = rpz + x[2] - rr;
                act = gap < p.contact_offset;
                pc[0] = x[0]; pc[1] = x[1]; pc[2] = x[2] - rr;
                const float d = gap - p.rest_offset;
                bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
            }
            const unsigned mask = hballot(act);
            if (act) {
                const int ci = ncon + __popc(mask & lanemask_lt(lane));
#pragma unroll
                for (int q = 0; q < 3; ++q) sm[t.s_cp + 3 * ci + q] = pc[q];
                sm[t.s_cl + ci] = (float)l;
                sm[t.s_cl2 + ci] = -1.0f;
#pragma unroll
                for (int tt = 0; tt < 3; ++tt) {
                    const int r = 3 * ci + tt;
                    sm[t.s_rl + r] = (float)l;
                    sm[t.s_rb + r] = tt == 0 ? bn : 0.0f;
                }
            }
            ncon += __popc(mask);
        }
    }
    // self-contacts (Humanoid.yaml:80): lanes over geom pairs, compacted in pair order within the
    // MI_MAX_ROWS budget, after the ground contacts (as the oracle)
    if constexpr (TP::kSelf) {
        if (t.self_on) {
            float* seg = sm + t.s_seg;
            float* bnd = seg + 8 * t.ngeoms;
            const float* geo = mcb + t.mc_geo;
            const int2* gpr = reinterpret_cast<const int2*>(t.g_pairs);
            int2 gpf[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const int pi = 32 * q + lane;
                gpf[q] = pi < t.npairs ? gpr[pi] : make_int2(0, 0);
            }
            for (int g = lane; g < t.ngeoms; g += 32) {
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
                const unsigned mask = hballot(keep);
                if (keep) surv[nsv + __popc(mask & lanemask_lt(lane))] = gp.x | (gp.y << 16);
                nsv += __popc(mask);
            };
            // the prefetched blocks by compile-time index (a runtime pick among them went to scratch)
            sfor<0, 5>([&](auto Q) { if (32 * (int)Q < t.npairs) broad(32 * (int)Q, gpf[Q], true); });
            for (int pb = 160; pb < t.npairs; pb += 32) broad(pb, make_int2(0, 0), false);
            wave_sync();
            int budget = (MI_MAX_ROWS - 3 * ncon - t.nlimc) / 3;
            const int nsv_max = pmax(nsv);
            for (int sb = 0; sb < nsv_max; sb += 32) {
                const int sidx = sb + lane;
                bool act = false;
                float pc[3], n[3], bn = 0.0f;
                int la = 0, lb = 0;
                if (sidx < nsv && budget > 0) {
                    const int pk = surv[sidx];
                    const float* A = seg + 8 * (pk & 0xffff);
                    const float* B = seg + 8 * (pk >> 16);
                    la = (int)A[7]; lb = (int)B[7];
                    const float gap = mi_pair_contact(A, A + 3, A[6], B, B + 3, B[6], pc, n);
                    act = gap < p.contact_offset;
                    const float d = gap - p.rest_offset;
                    bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
                }
                const unsigned mask = hballot(act);
                const int rank = __popc(mask & lanemask_lt(lane));
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
                    }
                }
                const int took = budget > 0 ? min(__popc(mask), budget) : 0;
                ncon += took;
                budget -= took;
            }
        }
    }
    const int nc = 3 * ncon;
    {
        const int cr = pmax(nc);                              // uniform
        if (cr > MI_PRIO_C3 && prio < 3) { __builtin_amdgcn_s_setprio(3); prio = 3; }
        else if (cr > MI_PRIO_C2 && prio < 2) { __builtin_amdgcn_s_setprio(2); prio = 2; }
        else if (cr > MI_PRIO_C1 && prio < 1) { __builtin_amdgcn_s_setprio(1); prio = 1; }
    }
    wave_sync();
    STAMP(6);
    // ---- P7+P9: one batch per half, lanes over solve vectors: the contact rows first (lane =
    // row in the first pass, as in the P10 Delassus set-up, which may then take their J rows
    // from this pass's registers), then the rhs, then limit candidates; passes of 32 to the
    // larger half's count.
    // Limit candidates: only the rhs's solve tells which limits are active, so the pass holding
    // the rhs fills its spare lanes with candidates speculatively — joints near a limit first
    // (q or q + dt u within MI_PAIR_LIM_NEAR of it), then the others in joint order — and later
    // passes take only the active candidates that were not among them. Which lane solves a
    // candidate changes neither its solve nor its filing (slot by joint index): the results of
    // solving every candidate, with a pass fewer whenever the spare lanes hold the active ones
    // (Humanoid: 1 + 21 + 14 solve vectors were two passes; 14 contact rows, the rhs and 17
    // candidates are one).
    // (models with few limited joints, e.g. Ant's 8, never need the second pass for them: there
    // every candidate follows the rhs, no speculation bookkeeping)
    constexpr bool kSpec = TP::D >= MI_PAIR_LIM_SPEC_MIN_D;
    unsigned cmask = 0u, nmask = 0u;
    if constexpr (kSpec) {
        bool cand = false, near = false;
        if (lane < D) {
            const float lo = mc.lf(MC_LO, lane + 1), hi = mc.lf(MC_HI, lane + 1);
            const float qj = sm[t.s_q + lane], qp = qj + dt * us[nr + lane];
            const float mg = MI_PAIR_LIM_NEAR;
            cand = lo < hi;
            near = cand && (qj < lo + mg || qp < lo + mg || qj > hi - mg || qp > hi - mg);
        }
        cmask = hballot(cand);
        nmask = hballot(near);
    }
    const unsigned fmask = cmask & ~nmask;
    const int nN = __popc(nmask);
    const int nspec = kSpec ? min(__popc(cmask), 31 - (nc & 31)) : t.nlimc;   // spare lanes of the rhs's pass
    int total = nc + 1 + nspec;
    int total_max = pmax(total);
    unsigned rem = 0u;                   // active candidates the spare lanes did not solve
    int nrows = nc;
    unsigned limact = 0u;
    // res: the rhs lane's solve (unconstrained acceleration); here: the rhs sits in this pass for
    // this half (half-uniform; the halves' rhs may sit in different passes)
    auto limit_rows = [&](const auto& res, bool here, bool rhs_lane) {
        constexpr int NR = sizeof(res) / sizeof(res[0]);
        if (rhs_lane) {
#pragma unroll
            for (int c = 0; c < NR; ++c)
                if (c < TP::nv) us[c] = us[c] + dt * res[c];
        }
        wave_sync();
        bool act = false;
        float bl = 0.0f, sg = 0.0f;
        if (here && lane < D) {
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
        const unsigned lb = hballot(act);
        if (here) limact = lb;
        if (act) {
            const int rl = nc + __popc(limact & lanemask_lt(lane));
            sm[t.s_rl + rl] = -(float)(nr + lane) - 1.0f;
            sm[t.s_lsg + lane] = sg;
            sm[t.s_rb + rl] = bl;
        }
        nrows = nc + __popc(limact);
        wave_sync();
    };
    auto file_row = [&](const auto& res, bool on, int r, int kd, float a_contact) {
        constexpr int NR = sizeof(res) / sizeof(res[0]);
        int slot = -1;
        float sc = 1.0f, a = 0.0f;
        if (on && r >= 0) {
            slot = r;
            a = a_contact;
        } else if (kd >= 0) {
            const int d = kd - nr;
            if ((limact >> d) & 1u) {
                slot = nc + __popc(limact & lanemask_lt(d));
                sc = sm[t.s_lsg + d];
                float wk = 0.0f;
#pragma unroll
                for (int c = 0; c < NR; ++c) wk = c == kd ? res[c] : wk;
                a = wk;
            }
        }
        if (slot >= 0) {
            sm[t.s_ad + slot] = a > 1e-12f ? a : 1e-12f;
            if (slot < t.w_rows_lds) {
                float* wl = sm + t.s_W + (slot & ~3) * nv + (slot & 3);
#pragma unroll
                for (int c = 0; c < NR; ++c)
                    if (c < TP::nv) wl[4 * c] = res[c] * sc;
            } else {
#pragma unroll
                for (int c = 0; c < WNV; ++c) gW[pair_sidx(slot, c)] = c < NR ? res[c] * sc : 0.0f;
            }
        }
    };
    // J rows of contact rows 0..31 (first pass), kept for the narrow PGS set-up when the model's
    // J row is short enough to stay live through the second pass without spilling (Ant: 0.0512
    // -> 0.0498 ms; Humanoid, nv 27: rebuilt in P10 instead, keeping the kernel spill-free)
    constexpr bool kReuseJ = TP::nv <= MI_PAIR_JREUSE_MAXNV;
    float Jc[TP::nvc];
    for (int base = 0; base < total_max; base += 32) {
        const int bv = base + lane;
        const bool on = bv < total;
        const bool crow = on && bv < nc;
        const int r = crow ? bv : -1;
        int kd = -1;
        if (on && bv > nc) {
            const int sl = bv - nc - 1;
            if constexpr (kSpec)
                kd = nr + (sl < nspec ? (sl < nN ? nth_bit(nmask, sl) : nth_bit(fmask, sl - nN))
                                      : nth_bit(rem, sl - nspec));
            else
                kd = nr + mc.lim(sl);
        }
        float x[TP::nvc];
        float f[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        unsigned msk = 0u, msk2 = 0u;
        if (crow) {
            const int l = (int)sm[t.s_rl + r];
            const float l2 = TP::kSelf ? sm[t.s_cl2 + r / 3] : -1.0f;
            msk = mc.mask(l);
            msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
            contact_row_f<TP::kSelf>(sm, t, r, f);
        }
        sdof_loop<TP, MI_PAIR_SDOF_PD, true, sdof_first_loaded(TP::nr)>(Ss, rhs, [&](auto C, const float (&sv)[6], float rcl) {
            constexpr int c = C;
            const float v = sdot<TP, c>(sv, f);
            const bool ia = (msk >> c) & 1u, ib = (msk2 >> c) & 1u;
            float xc = (ia ? v : 0.0f) - (ib ? v : 0.0f);
            float rc = rcl;
            asm volatile("" : "+v"(xc), "+v"(rc));
            x[c] = crow ? xc : (bv == nc ? rc : (kd == c ? 1.0f : 0.0f));
        });
        if constexpr (kReuseJ) {
            if (base == 0) sfor<0, TP::nv>([&](auto C) { Jc[C] = x[C]; });
        }
        STAMP(7);
        float a;
        ct_solve_l<TP, MI_PAIR_SOLVE_PD>(sm + t.s_L, x, a);
        STAMP(8);
        const bool rhs_here = base <= nc && nc < base + 32;
        if (pmax(rhs_here ? 1 : 0)) {
            limit_rows(x, rhs_here, bv == nc);
            if (kSpec && rhs_here) {
                const unsigned spec = nspec <= nN ? low_bits(nmask, nspec) : (nmask | low_bits(fmask, nspec - nN));
                rem = limact & ~spec;
                total += __popc(rem);
            }
            total_max = pmax(total);
        }
        STAMP(9);
        file_row(x, on, r, kd, a);
        STAMP(10);
    }
    wave_sync();
    STAT(15, pmax(nrows));
    STAT(16, total_max > 32);
    STAT(17, pmax(nrows) > 64);
    STAT(18, total_max > 64);
    STAT(19, pmax(nrows) > TP::kLamRows);
    STAT(20, pmax(ncon));
    STAT(21, pmax(nrows) > 16);
    STAT(22, pmax(nrows) > 24);
    STAT(23, pmax(nrows) > 20);
    STAT(26, t.w_rows_lds);
    // ---- P10: projected Gauss-Seidel, 4 sweeps
    load = max(load, nrows);   // half-uniform: this env's constraint rows (contact + limit; A/B
                               // round 5: 0.1166 ms vs 0.1178 ranking by contact rows alone)
    const int nrows_max = pmax(nrows);
    const float mu = p.friction;
    if (nrows_max <= TP::kLamRows) {
        // Delassus space: lane r holds row r's v_r = J_r . u and A[r][s] = J_r . W_s (J_r rebuilt
        // here from the contact data: no J rows in LDS; W rows past the LDS ones from the slab).
        // Every lane keeps every row's lambda in registers (it computes each row's update anyway),
        // and reads the row's bias / A_rr / kind from LDS ahead of the chain, so a row costs one
        // cross-lane broadcast (v_r) instead of five.
        constexpr int NV = TP::nv;
        constexpr int RMAX = TP::kLamRows;
        // J_r: with kReuseJ a contact row's from P9's first pass (same lane), a limit row's
        // sg e_k, a dead lane's 0 (v 0: its projection keeps lambda 0); else rebuilt
        float Jr[TP::nvc];
        if constexpr (kReuseJ) {
            int kdof = -1;
            float sg = 0.0f;
            if (lane >= nc && lane < nrows) {
                kdof = (int)(-sm[t.s_rl + lane] - 1.0f);
                sg = sm[t.s_lsg + kdof - nr];
            }
            const bool own = lane < nc;
            sfor<0, NV>([&](auto C) { Jr[C] = own ? Jc[C] : (kdof == C ? sg : 0.0f); });
        } else {
            if (nrows > 0) pair_jrow<TP>(mc, t, sm, lane < nrows ? lane : 0, nr, Jr);
            else sfor<0, NV>([&](auto C) { Jr[C] = 0.0f; });
        }
        float v = pk_jdot<NV>(Jr, us);
        STAMP(24);
        const WSrc wsn = make_wsrc(t, sm, gW);
        float Ar[RMAX];
        static_assert(RMAX % 4 == 0, "Delassus rows are built four at a time");
        sfor<0, RMAX / 4>([&](auto G) {
            constexpr int g0 = 4 * G;
            float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            if (g0 < nrows_max) pair_dgroup_w<TP, MI_PAIR_SDOF_PD, true>(wsn, g0, nrows, Jr, a);
            Ar[g0] = a[0]; Ar[g0 + 1] = a[1]; Ar[g0 + 2] = a[2]; Ar[g0 + 3] = a[3];
        });
        STAMP(25);
        // lane r's own row: bias, 1 / A_rr, kind (contact rows are (normal, friction, friction)
        // triples 3c..3c+2, then the limit rows)
        float b = 0.0f, ia = 0.0f;   // ia 0: a dead row's projection keeps its lambda 0
        int kd = 0;
        if (lane < nrows) {
            b = sm[t.s_rb + lane];
            ia = 1.0f / sm[t.s_ad + lane];
            kd = lane < nc ? lane % 3 : 3;   // row kind from the row index (no LDS array)
        }
        const int nnorm = 3 * ncon;   // rows below this with r % 3 == 0 are normal rows
        STAMP(27);
        float lamv[RMAX];
#pragma unroll
        for (int rr = 0; rr < RMAX; ++rr) lamv[rr] = 0.0f;
        // TGS: b holds the row's separation; each sub-step's bias comes from the separation plus
        // h x the row velocities J_r u of the earlier sub-steps (ds), and the owner lane sums its
        // row's lambda over the sub-steps (lsum: u-bar = u* + W lsum / iters)
        [[maybe_unused]] const float sep = b;
        [[maybe_unused]] float ds = 0.0f, lsum = 0.0f;
        for (int it = 0; it < p.iters + p.viters; ++it) {
            if constexpr (TP::kTgs)
                b = (kd == 1 || kd == 2) ? 0.0f : row_bias(p, sep + ds, p.h, it < p.iters);
            asm volatile("" : "+v"(b), "+v"(ia), "+v"(kd));
            int nrow_it = nrows_max;
            asm volatile("" : "+s"(nrow_it));
            float lamn = 0.0f;
            sfor<0, RMAX>([&](auto RR) {   // fully unrolled: Ar / lamv stay register-indexed
                constexpr int rr = RR;
                // uniform, per group of four rows: rows past the count in the last group run as
                // dead rows (owner ia 0, A entries 0: lambda and v unchanged), one branch per group
                if ((rr & ~3) < nrow_it) {
                    __builtin_amdgcn_sched_barrier(0);
                    // the row's owner (lane rr of each half) holds v_rr, b, 1 / A_rr and its kind:
                    // it alone projects, and one broadcast hands the new lambda to its half
                    // (a row past its half's count projects to its lambda 0 unchanged: the
                    // owner lane holds ia = 0, kind 0)
                    const float l0 = lamv[rr];
                    const bool fric = kd == 1 || kd == 2;
                    const float lim = mu * lamn;
#if MI_PAIR_SWEEP_FMA
                    // x = (l0 + b / A_rr) - v / A_rr and v + A (ln - l0) = (v - A l0) + A ln: the
                    // l0 terms come off the chain, which is then fma -> med3 -> broadcast -> fma
                    const float x = __builtin_fmaf(-v, ia, __builtin_fmaf(b, ia, l0));
#else
                    const float x = l0 + (b - v) * ia;
#endif
                    // one med3: max(., lo) then, for friction, min(., lim) (lo <= hi: lamn >= 0)
                    const float mine = __builtin_amdgcn_fmed3f(x, fric ? -lim : 0.0f,
                                                               fric ? lim : __builtin_huge_valf());
                    const float ln = pbcc<rr>(mine);
                    if constexpr (rr % 3 == 0) lamn = rr < nnorm ? ln : lamn;
#if MI_PAIR_SWEEP_FMA
                    v = __builtin_fmaf(Ar[rr], ln, __builtin_fmaf(-Ar[rr], l0, v));
#else
                    v += Ar[rr] * (ln - l0);
#endif
                    lamv[rr] = ln;
                }
            });
            if constexpr (TP::kTgs) {
                if (it < p.iters) {   // the sub-step moves row r by h v_r; its lambda joins the sum
                    ds += p.h * v;
                    float lo = 0.0f;
#pragma unroll
                    for (int rr = 0; rr < RMAX; ++rr) lo = lane_here(lane) == rr ? lamv[rr] : lo;
                    lsum += lo;
                }
            }
        }
        STAMP(28);
        float u = lane < NV ? us[lane] : 0.0f;
        [[maybe_unused]] float ub = u;
        [[maybe_unused]] const float lbar = lsum / (float)p.iters;
        const int kc = lane < NV ? lane : 0;
        sfor<0, RMAX / 4>([&](auto G) {
            constexpr int g0 = 4 * G;
            if (g0 < nrows_max) {
                float wq[4];
                pair_wcol_w<true>(wsn, g0, kc, NV, wq);
#pragma unroll
                for (int q = 0; q < 4; ++q) u = g0 + q < nrows ? u + wq[q] * lamv[g0 + q] : u;
                if constexpr (TP::kTgs) {
                    sfor<0, 4>([&](auto Q) {
                        constexpr int q = Q;
                        const float lq = pbcc<g0 + q>(lbar);
                        ub = g0 + q < nrows ? ub + wq[q] * lq : ub;
                    });
                }
            }
        });
        if (lane < NV) us[lane] = u;
        if constexpr (TP::kTgs)   // the positions' velocity (sub-steps' mean), in the dead rhs
            if (lane < NV) sm[t.s_r + lane] = ub;
        wave_sync();
        {   // reuse: lambda of row rr, written by lane rr (one select chain, one store)
            float lo = 0.0f;
#pragma unroll
            for (int rr = 0; rr < RMAX; ++rr) lo = lane_here(lane) == rr ? lamv[rr] : lo;
            if (lane < nrows) sm[t.s_ad + lane] = lo;
        }
    } else if (nrows_max <= 64) {
#ifndef MI_EXP_NO_WIDE
        // Wide Delassus (a half with 33..64 rows: 0.4 % of Humanoid substeps, but they set the
        // launch's slowest waves): the two envs one after the other, each on all 64 lanes, lane
        // r = row r of that env. Per row: the owner lane projects, one v_readlane hands the new
        // lambda to the wave (its old one is read off the chain), one FMA per lane updates v.
        // The Delassus block does not stay in registers (64 per lane would set the kernel's
        // register peak and spill it): the set-up stores it to the wave's global scratch t.g_wa
        // as A[s][r] (lane-contiguous rows, coalesced; A is symmetric, so row s holds every
        // lane's A[r][s]), and the sweeps stream it back MI_PAIR_WIDE_AP rows ahead of the chain
        // (L2-resident, off the dependency chain).
        constexpr int NV = TP::nv;
        constexpr int PA = MI_PAIR_WIDE_AP;
        constexpr int AR = MI_PAIR_WIDE_AREG;   // Delassus rows kept in registers; the rest streamed
        const int l64 = pair_l64(), me = l64 >> 5;
        const int kc = l64 < NV ? l64 : 0;
        // this wave's scratch (its slot over the launch: the same for both halves), addressed through a buffer
        // resource: one lane offset register for every row (Delassus row s at soffset 256 (s -
        // A0), A0 = 0 with the MFMA set-up (all 64 rows there), else AR); loads past the record
        // range (prefetch beyond the last row) return 0
        const int wv = __builtin_amdgcn_readfirstlane(wv_);   // the wave's slot (pairs may be permuted)
        constexpr int WR = kWideScratchRows > 0 ? kWideScratchRows : 1;
        constexpr int A0 = MI_PAIR_WIDE_MFMA ? 0 : AR;
        const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(t.g_wa + (size_t)wv * (WR * 64)), (short)0, WR * 64 * (int)sizeof(float), 0x00020000);
        const int avo = l64 * (int)sizeof(float);
        STAMP(29);
        for (int h = 0; h < 2; ++h) {
            const int nrh = __builtin_amdgcn_readlane(nrows, 32 * h);
            const int nnh = 3 * __builtin_amdgcn_readlane(ncon, 32 * h);
            float* smh = sm + (h - me) * t.env_stride;                 // env of half h
            if (nrh == 0) {
                // no rows: u = u*; TGS integrates positions with u-bar = u* as well
                if constexpr (TP::kTgs) {
                    if (l64 < NV) smh[t.s_r + l64] = smh[t.s_us + l64];
                    wave_sync();
                }
                continue;
            }
            // the env of half h: its slab (the pair need not be adjacent envs: pairing by load)
            const int ih = __builtin_amdgcn_readlane(i, 32 * h);
            const float* gWh = gW + (ptrdiff_t)(ih - i) * (ptrdiff_t)t.g_row_stride;
            const WSrc wsh = make_wsrc(t, smh, gWh);
            const int rl = l64 < nrh ? l64 : 0;
            float Jr[TP::nvc];
            pair_jrow<TP>(mc, t, smh, rl, nr, Jr);
            const float* ush = smh + t.s_us;
            float v = pk_jdot<NV>(Jr, ush);
            STAMP(30);
            float Ar[AR > 0 ? AR : 1];
#if MI_PAIR_WIDE_MFMA
            {
                // A = J W^T as v_mfma_f32_16x16x4f32 tiles (A[m][k] at lane m + 16 k, B[k][n] at
                // lane n + 16 k, D[4 (l >> 4) + i][l & 15] in register i): J^T goes to the scratch
                // (column c at row 64 + c, lane = constraint row; rows past the env's count and the
                // padding columns 0), each 16-row block of J comes back in the A-operand layout, W
                // in the B-operand layout straight from LDS / the slab. A tile's D is stored as
                // scratch rows 16 R + 4 (l >> 4) + i, lanes 16 S + (l & 15): row s then holds
                // A[s][r] at lane r (A symmetric), the layout the sweeps read. Every 16-lane
                // column block is written (rows past the count come out 0), row blocks up to the
                // count only (the sweeps read no further). Sums in the MFMA's order, not DOF order.
                constexpr int KP = (NV + 3) & ~3, KC = KP / 4;
                static_assert(KP <= 32, "wide scratch holds 32 J^T columns");
                sfor<0, KP>([&](auto C) {
                    constexpr int c = C;
                    float jv = 0.0f;
                    if constexpr (c < NV) jv = l64 < nrh ? Jr[c] : 0.0f;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, jv), ars, avo, (64 + c) * 256, 0);
                });
                wave_sync();   // J^T stored before the A-operand loads read it back
                const int lr = l64 & 15, lk = l64 >> 4;
                const int jvo = ((64 + lk) * 64 + lr) * (int)sizeof(float);
                const int dvo = (4 * lk * 64 + lr) * (int)sizeof(float);
#if MI_PAIR_WIDE_MFMA_HOIST
                // every row block's A operands in flight at once (one L2 round trip, not one per tile)
                float jall[4][KC];
                sfor<0, 4>([&](auto R) {
                    sfor<0, KC>([&](auto K) {
                        jall[R][K] = 16 * R < nrh ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                                  ars, jvo, (K * 256 + 16 * R) * 4, 0))
                                                  : 0.0f;
                    });
                });
#endif
                sfor<0, 4>([&](auto S) {   // column block: lanes 16 S .. 16 S + 15
                    const int s = 16 * S + lr;
                    float wb[KC];
                    sfor<0, KC>([&](auto K) {
                        const int c = 4 * K + lk;
                        float w = 0.0f;
                        if (16 * S < nrh && s < nrh && c < NV) {
                            if (s < t.w_rows_lds) w = lds_ptr(smh)[t.s_W + pw_idx(s, c, NV)];
                            else w = gWh[pair_sidx(s, c)];
                        }
                        wb[K] = w;
                    });
                    sfor<0, 4>([&](auto R) {   // row block: scratch rows 16 R .. 16 R + 15
                        if (16 * R < nrh) {
                            pv4 d = {0.0f, 0.0f, 0.0f, 0.0f};
                            sfor<0, KC>([&](auto K) {
#if MI_PAIR_WIDE_MFMA_HOIST
                                const float ja = jall[R][K];
#else
                                const float ja = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                               ars, jvo, (K * 256 + 16 * R) * 4, 0));
#endif
                                d = __builtin_amdgcn_mfma_f32_16x16x4f32(ja, wb[K], d, 0, 0, 0);
                            });
                            // D moved to VGPRs first: stored straight from the accumulator tuple, this
                            // compiler (ROCm 7.2) emits four stores of its first register
                            // (tools/mfma_wide_check.hip)
                            float o4[4] = {d.x, d.y, d.z, d.w};
                            asm volatile("" : "+v"(o4[0]), "+v"(o4[1]), "+v"(o4[2]), "+v"(o4[3]));
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o4[q]), ars, dvo,
                                                                      ((16 * R + q) * 64 + 16 * S) * 4, 0);
                        }
                    });
                });
                wave_sync();   // the tiles stored before the rows are read back lane = row
                if constexpr (AR > 0) {
                    sfor<0, AR / 4>([&](auto G) {
                        constexpr int g0 = 4 * G;
                        if (g0 < nrh) {
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                Ar[g0 + q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                           ars, avo, (g0 + q) * 256, 0));
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) Ar[g0 + q] = 0.0f;
                        }
                    });
                }
            }
#else
            sfor<0, 16>([&](auto G) {
                constexpr int g0 = 4 * G;
                float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                if (g0 < nrh) {
                    pair_dgroup_w<TP, MI_PAIR_WIDE_PD, false>(wsh, g0, nrh, Jr, a);
                    if constexpr (g0 >= AR) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, a[q]), ars, avo,
                                                                  (g0 + q - AR) * 256, 0);
                    }
                }
                if constexpr (g0 < AR) { Ar[g0] = a[0]; Ar[g0 + 1] = a[1]; Ar[g0 + 2] = a[2]; Ar[g0 + 3] = a[3]; }
            });
            if constexpr (AR < 64) wave_sync();
#endif
            STAMP(27);
            float b = 0.0f, ia = 0.0f, lam = 0.0f;    // ia 0: a dead row keeps its lambda 0
            int kd = 0;
            if (l64 < nrh) {
                b = smh[t.s_rb + l64];
                ia = 1.0f / smh[t.s_ad + l64];
                kd = l64 < nnh ? l64 % 3 : 3;
            }
            // TGS as in the narrow sweeps: b holds the separation, ds the sub-steps' motion of
            // the row, lsum the row's lambda summed over the sub-steps (lane = row here)
            [[maybe_unused]] const float sep = b;
            [[maybe_unused]] float ds = 0.0f, lsum = 0.0f;
            for (int it = 0; it < p.iters + p.viters; ++it) {
                if constexpr (TP::kTgs)
                    b = (kd == 1 || kd == 2) ? 0.0f : row_bias(p, sep + ds, p.h, it < p.iters);
                asm volatile("" : "+v"(b), "+v"(ia), "+v"(kd));
                int nrow_it = nrh;
                asm volatile("" : "+s"(nrow_it));
                float lamn = 0.0f;
#if MI_PAIR_SWEEP_FMA
                const float tl = __builtin_fmaf(b, ia, lam);   // lane = row: lam changes at its own row only
                float muv = mu, lov = 0.0f, hiv = 0.0f;        // mu in a VGPR: mu lambda_n in one v_mul
                asm volatile("" : "+v"(muv));
#endif
                // rows rr .. rr + PA - 1 of A in flight. The scratch is NOT zeroed (no memset at
                // creation): correctness rests on the invariant that the set-up writes every row
                // of every group of four it processes ((rr & ~3) < nrh, the sweeps' condition),
                // so a row the sweeps use is always written before it is read; rows loaded past
                // the last processed group are never used (a stale value there never reaches v)
                // a fresh pointer each sweep: the loads must not be hoisted out of the sweep loop
                // (they would all stay live: the register peak this scratch is here to remove)
                int vo = avo, lw = l64;
                // per-sweep copies: the loads and the 64 `lane == row` masks must not be hoisted
                // out of the sweep loop (64 SGPR-pair masks would spill and reload per row)
                asm volatile("" : "+v"(vo), "+v"(lw));
                auto ald = [&](int r) {
                    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ars, vo, (r - A0) * 256, 0));
                };
                // rows AR.. streamed: their first PA loads are issued before the sweep, so the
                // register rows' steps hide their latency
                float ab[PA];
                if constexpr (AR < 64) sfor<0, PA>([&](auto Q) { ab[Q] = ald(AR + Q); });
                sfor<0, 64>([&](auto RR) {
                    constexpr int rr = RR;
                    if ((rr & ~3) < nrow_it) {   // per group of four rows, as in the narrow sweeps
                        __builtin_amdgcn_sched_barrier(0);
                        float arr;
                        if constexpr (rr < AR) {
                            arr = Ar[rr];
                        } else {
                            arr = ab[(rr - AR) % PA];
                            if constexpr (rr + PA < 64) ab[(rr - AR) % PA] = ald(rr + PA);
                        }
#if MI_PAIR_SWEEP_FMA
                        // the narrow sweeps' arithmetic (bit for bit: an env's result does not
                        // depend on the path its partner sends the wave down): the new lambda
                        // and the row's old one leave the owner by v_readlane (the old one off
                        // the chain), v_writelane stores the new one in the owner lane. Row
                        // kinds are wave-uniform here (lane = row of one env): rows 3c are
                        // normal or limit rows, [0, inf); rows 3c + 1, 3c + 2 friction rows
                        // (+-mu lambda_3c, one v_mul per contact) below nnh, limit rows past it
                        const float xr = __builtin_fmaf(-v, ia, tl);
                        const float mine = rr % 3 == 0 ? __builtin_amdgcn_fmed3f(xr, 0.0f, __builtin_huge_valf())
                                                       : __builtin_amdgcn_fmed3f(xr, lov, hiv);
                        const float ln = readlane(mine, rr), l0 = readlane(lam, rr);
                        if constexpr (rr % 3 == 0) {   // the next two rows' bounds (uniform select)
                            const float lm = muv * ln;
                            const bool fr = rr + 1 < nnh;
                            hiv = fr ? lm : __builtin_huge_valf();
                            lov = fr ? -lm : 0.0f;
                        }
                        v = __builtin_fmaf(arr, ln, __builtin_fmaf(-arr, l0, v));
                        asm("v_writelane_b32 %0, %1, %2" : "+v"(lam) : "s"(ln), "i"(rr));
                        (void)lw;
#else
                        const bool fric = kd == 1 || kd == 2;
                        const float lim = mu * lamn;
                        const float mine = __builtin_amdgcn_fmed3f(lam + (b - v) * ia, fric ? -lim : 0.0f,
                                                                   fric ? lim : __builtin_huge_valf());
                        // the owner forms the lambda change itself (mine - lam there is exactly
                        // ln - l0) and keeps mine as its lambda: one v_readlane per row (two for
                        // the normal rows, whose lambda bounds the next two), no SGPR pair to
                        // move back for the subtraction
                        const float dl = readlane(mine - lam, rr);
                        if constexpr (rr % 3 == 0) lamn = rr < nnh ? readlane(mine, rr) : lamn;
                        v += arr * dl;
                        lam = lw == rr ? mine : lam;
#endif
                    }
                });
                if constexpr (TP::kTgs) {
                    if (it < p.iters) { ds += p.h * v; lsum += lam; }
                }
            }
            STAMP(28);
            // u = u* + sum_r W_r lambda_r, lane = DOF (TGS: and u-bar = u* + W lsum / iters)
            float u = ush[kc];
            [[maybe_unused]] float ub = u;
            [[maybe_unused]] const float lbar = lsum / (float)p.iters;
#if MI_PAIR_WIDE_UPF
            // the next group's W column is loaded before this group's FMAs (rows past the LDS
            // ones come from the slab: one L2 round trip per group on the chain otherwise)
            float wn[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            pair_wcol_w<false>(wsh, 0, kc, NV, wn);
#endif
            sfor<0, 16>([&](auto G) {
                constexpr int g0 = 4 * G;
                if (g0 < nrh) {
                    float wq[4];
#if MI_PAIR_WIDE_UPF
#pragma unroll
                    for (int q = 0; q < 4; ++q) wq[q] = wn[q];
                    if constexpr (g0 + 4 < 64)
                        if (g0 + 4 < nrh) pair_wcol_w<false>(wsh, g0 + 4, kc, NV, wn);
#else
                    pair_wcol_w<false>(wsh, g0, kc, NV, wq);
#endif
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float lq = readlane(lam, g0 + q);
                        u = g0 + q < nrh ? u + wq[q] * lq : u;
                        if constexpr (TP::kTgs) {
                            const float lb = readlane(lbar, g0 + q);
                            ub = g0 + q < nrh ? ub + wq[q] * lb : ub;
                        }
                    }
                }
            });
            wave_sync();
            if (l64 < NV) smh[t.s_us + l64] = u;
            if constexpr (TP::kTgs)
                if (l64 < NV) smh[t.s_r + l64] = ub;
            if (l64 < nrh) smh[t.s_ad + l64] = lam;            // reuse: lambda of row l64
            wave_sync();
            STAMP(11);
        }
#endif
    } else {
#ifndef MI_EXP_NO_FALLBACK
        // fallback (a half with more rows than the Delassus registers hold, 0.4 % of Humanoid
        // substeps): u-space sweeps, lane = DOF. Rows 0..63 as the wave kernel's one-bank
        // sweeps with 32-lane banks: row r's data in lane r & 31 of bank r >> 5 (J rebuilt per row
        // from the contact force direction and the lane's DOF subspace), W rows prefetched into
        // registers; rows 64.. (a handful of substeps in a million) row by row from LDS and the
        // slab, their lambdas in the slab's spare column.
        float S6[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) S6[q] = lane < nv ? Ss[6 * lane + q] : 0.0f;
        float u = lane < nv ? us[lane] : 0.0f;
        const int kc = lane < nv ? lane : 0;
        const float kin = lane < nv ? 1.0f : 0.0f;
        float b0 = 0.0f, b1 = 0.0f, ia0 = 1.0f, ia1 = 1.0f, k0 = 0.0f, k1 = 0.0f, lam0 = 0.0f, lam1 = 0.0f;
        float fa[6] = {0, 0, 0, 0, 0, 0}, fb[6] = {0, 0, 0, 0, 0, 0};
        unsigned ma = 0u, mb = 0u, ma2 = 0u, mb2 = 0u;
        auto load_row = [&](int r, float& b, float& ia, float& k, float (&f)[6], unsigned& msk,
                            unsigned& msk2) {
            b = sm[t.s_rb + r];
            ia = 1.0f / sm[t.s_ad + r];
            k = (float)(r < nc ? r % 3 : 3);
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
        if (lane + 32 < nrows) load_row(lane + 32, b1, ia1, k1, fb, mb, mb2);
        const int nnorm = 3 * ncon;
        // W entry of row rr at the lane's DOF (uniform branch: LDS rows, then the slab); read
        // per row (a handful of substeps in a million: registers matter more than latency here)
        const float* wsm = sm;
        const float* wgW = gW;
        auto wrow = [&](int rr) {
            return (rr < t.w_rows_lds ? wsm[t.s_W + pw_idx(rr, kc, nv)] : wgW[pair_sidx(rr, kc)]) * kin;
        };
        for (int r = 64 + lane; r < nrows; r += 32) gW[pair_sidx(r, WNV - 1)] = 0.0f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        STAMP(27);
        // TGS in u space: b0 / b1 / s_rb hold the rows' separations; usum sums the sub-steps'
        // velocities (lane = DOF), so row r has moved by h J_r usum before the current sub-step
        [[maybe_unused]] float usum = 0.0f;
        for (int it = 0; it < p.iters + p.viters; ++it) {
            asm volatile("" : "+v"(b0), "+v"(b1), "+v"(ia0), "+v"(ia1),
                         "+v"(ma), "+v"(mb), "+v"(ma2), "+v"(mb2));
            int lfb = lane, nrl = nrows;
            // per-row W reads and lane / row-count masks stay inside the sweep (hoisted, 64 masks
            // of each would spill SGPRs)
            asm volatile("" : "+v"(wsm), "+v"(wgW), "+v"(lfb), "+v"(nrl));
            int nrow_it = nrows_max;
            asm volatile("" : "+s"(nrow_it));
            float lamn = 0.0f;
#pragma unroll
            for (int rr = 0; rr < 64; ++rr) {
                if (rr >= nrow_it) continue;
                __builtin_amdgcn_sched_barrier(0);
                const int bank = rr >> 5, w = rr & 31;
                float fr[6];
#pragma unroll
                for (int q = 0; q < 6; ++q) fr[q] = pbc(bank ? fb[q] : fa[q], w);
                const unsigned msk = (unsigned)pbci((int)(bank ? mb : ma), w);
                const unsigned msk2 = (unsigned)pbci((int)(bank ? mb2 : ma2), w);
                const int kind = rr < nnorm ? rr % 3 : 3;   // (normal, friction, friction) triples, limits
                float d6 = dot6(S6, fr);
                asm volatile("" : "+v"(d6));                 // computed on every lane: no branch
                const float j0 = kind == 3 ? fr[0] : d6;
                const float jc = ((((msk >> lane) & 1u) ? j0 : 0.0f) - (((msk2 >> lane) & 1u) ? j0 : 0.0f)) * kin;
                const float jv = psum(jc * u);
                float br = pbc(bank ? b1 : b0, w);
                const float iar = pbc(bank ? ia1 : ia0, w);
                if constexpr (TP::kTgs)
                    br = (kind == 1 || kind == 2) ? 0.0f : row_bias(p, br + p.h * psum(jc * usum), p.h, it < p.iters);
                const float l0 = pbc(bank ? lam1 : lam0, w);
                float ln = l0 + (br - jv) * iar;
                const bool fric = kind == 1 || kind == 2;
                const float lim = mu * lamn;
                ln = fmaxf(ln, fric ? -lim : 0.0f);
                ln = fric ? fminf(ln, lim) : ln;
                const bool live_row = rr < nrl;
                lamn = (live_row && kind == 0) ? ln : lamn;
                u = live_row ? u + wrow(rr) * (ln - l0) : u;
                const bool own = live_row && lfb == w;
                if (bank) lam1 = own ? ln : lam1;
                else lam0 = own ? ln : lam0;
            }
            for (int r = 64; r < nrow_it; ++r) {
                const bool live_row = r < nrows;
                const int rs = live_row ? r : 0;
                const float br = sm[t.s_rb + rs], ar = sm[t.s_ad + rs];
                const int kind = rs < nc ? rs % 3 : 3;
                const float lk = sm[t.s_rl + rs];
                float jc;
                if (lk >= 0.0f) {
                    float fr[6];
                    contact_row_f<TP::kSelf>(sm, t, rs, fr);
                    const unsigned msk = mc.mask((int)lk);
                    const float l2 = TP::kSelf ? sm[t.s_cl2 + rs / 3] : -1.0f;
                    const unsigned msk2 = l2 >= 0.0f ? mc.mask((int)l2) : 0u;
                    const float v6 = dot6(S6, fr);
                    jc = (((msk >> lane) & 1u) ? v6 : 0.0f) - (((msk2 >> lane) & 1u) ? v6 : 0.0f);
                } else {
                    const int kdof = (int)(-lk - 1.0f);
                    jc = lane == kdof ? sm[t.s_lsg + kdof - nr] : 0.0f;
                }
                jc *= kin;
                const float jv = psum(jc * u);
                float* lp = gW + pair_sidx(rs, WNV - 1);
                const float l0 = live_row ? *lp : 0.0f;
                float brt = br;
                if constexpr (TP::kTgs)
                    brt = (kind == 1 || kind == 2) ? 0.0f : row_bias(p, br + p.h * psum(jc * usum), p.h, it < p.iters);
                float ln = l0 + (brt - jv) * (1.0f / ar);
                const bool fric = kind == 1 || kind == 2;
                const float lim = mu * lamn;
                ln = fmaxf(ln, fric ? -lim : 0.0f);
                ln = fric ? fminf(ln, lim) : ln;
                if (live_row) {
                    lamn = kind == 0 ? ln : lamn;
                    u += gW[pair_sidx(rs, kc)] * kin * (ln - l0);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                if (live_row && lane == 0) *lp = ln;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if constexpr (TP::kTgs)
                if (it < p.iters) usum += u;
        }
        STAMP(28);
        if (lane < nv) us[lane] = u;
        if constexpr (TP::kTgs)   // the positions' velocity: the sub-steps' mean
            if (lane < nv) sm[t.s_r + lane] = usum / (float)p.iters;
        if (lane < nrows) sm[t.s_ad + lane] = lam0;          // reuse: lambda of row lane
        if (lane + 32 < nrows) sm[t.s_ad + lane + 32] = lam1;
        for (int r = 64 + lane; r < nrows; r += 32) sm[t.s_ad + r] = gW[pair_sidx(r, WNV - 1)];
#endif
    }
    wave_sync();
    STAMP(11);
    // ---- P11a: force sensors. Contact-parallel when the buffer fits the dead W rows
    // (t.sens_par): lane = contact computes its force and, for every sensor whose link it
    // touches, its torque about the sensor, into [contact][sensor][6] at s_W; then lane =
    // (sensor, component) sums its component over the contacts in contact order — the serial
    // loop's terms and summation order (a non-touching contact adds a signed zero, which leaves
    // a sum started at +0 unchanged), without its per-contact latency chain.
    if (t.sens_par) {
        const int S = m.S;
        float* sb = sm + t.s_W;
        float* sums = sb + 6 * S * t.ncmax;
        const int nc_max = pmax(ncon);
        for (int c0 = 0; c0 < nc_max; c0 += 32) {
            const int c = c0 + lane;
            if (c < ncon) {
#pragma clang fp contract(off)
                const int la = (int)sm[t.s_cl + c];
                const int lb = TP::kSelf ? (int)sm[t.s_cl2 + c] : -1;
                const float* lamp = sm + t.s_ad;
                const float fn = lamp[3 * c] / dt, f1 = lamp[3 * c + 1] / dt, f2 = lamp[3 * c + 2] / dt;
                float d[9];
                contact_dirs<TP::kSelf>(sm, t, c, d);
                const float cp[3] = {sm[t.s_cp + 3 * c], sm[t.s_cp + 3 * c + 1], sm[t.s_cp + 3 * c + 2]};
                for (int si = 0; si < S; ++si) {
                    const int l = (int)mc.sf(MS_LINK, si);
                    const float sgn = la == l ? 1.0f : ((TP::kSelf && lb == l) ? -1.0f : 0.0f);
                    float R[9], xs[3];
#pragma unroll
                    for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
                    const float sp[3] = {mc.sf(MS_X, si), mc.sf(MS_X + 1, si), mc.sf(MS_X + 2, si)};
                    m3_vec(R, sp, xs);
#pragma unroll
                    for (int q = 0; q < 3; ++q) xs[q] += sm[t.s_o + 3 * l + q];
                    float fc[3], rr[3], tc[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q) fc[q] = sgn * (fn * d[q] + f1 * d[3 + q] + f2 * d[6 + q]);
#pragma unroll
                    for (int q = 0; q < 3; ++q) rr[q] = cp[q] - xs[q];
                    cross3(rr, fc, tc);
                    float* o = sb + 6 * (S * c + si);
#pragma unroll
                    for (int q = 0; q < 3; ++q) { o[q] = sgn == 0.0f ? 0.0f : fc[q]; o[3 + q] = sgn == 0.0f ? 0.0f : tc[q]; }
                }
            }
        }
        wave_sync();
        if (lane < 6 * S) {
            const int si = lane / 6, q = lane - 6 * si;
            float acc = 0.0f;
            for (int c = 0; c < ncon; ++c) acc += sb[6 * (S * c + si) + q];
            sums[lane] = acc;
        }
        wave_sync();
        if (lane < S) {
            const int si = lane, l = (int)mc.sf(MS_LINK, si);
            float R[9], F[3], T[3], Fl[3], Tl[3];
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = sm[t.s_R + 9 * l + q];
#pragma unroll
            for (int q = 0; q < 3; ++q) { F[q] = sums[6 * si + q]; T[q] = sums[6 * si + 3 + q]; }
            m3_tvec(R, F, Fl);
            m3_tvec(R, T, Tl);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                sm[t.s_rb + 6 * si + q] = Fl[q];
                sm[t.s_rb + 6 * si + 3 + q] = Tl[q];
            }
        }
    } else if (lane < m.S) {
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
            const float sgn = (int)sm[t.s_cl + c] == l ? 1.0f :
                              ((TP::kSelf && (int)sm[t.s_cl2 + c] == l) ? -1.0f : 0.0f);
            if (sgn == 0.0f) continue;
            const float* lamp = sm + t.s_ad;
            const float fn = lamp[3 * c] / dt, f1 = lamp[3 * c + 1] / dt, f2 = lamp[3 * c + 2] / dt;
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
            sm[t.s_rb + 6 * si + q] = Fl[q];
            sm[t.s_rb + 6 * si + 3 + q] = Tl[q];
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
        sm[t.s_q + lane] = qn;
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
    if (nr && store_state) {
        if (lane < 3) st.root_pos[sx(st, lane, i)] = sm[t.s_rp + lane];
        else if (lane < 7) st.root_quat[sx(st, lane - 3, i)] = sm[t.s_rp + 4 + lane - 3];
        else if (lane < 13) st.root_vel[sx(st, lane - 7, i)] = us[lane - 7];
    }
    if (hballot(!finite) != 0u && lane == 0) st.nan_flag[i] = 1;
    wave_sync();
    STAMP(12);
    STAMP_END();
}

// Task layer of the paired kernel: wave_task_pre / wave_loco_post of mi_wave.hpp with the env
// of this lane's half (lane = lane & 31; the half's lane 0 does the sequential parts).
MI_D float pair_task_pre(const DevModel& m, const DevState& st, const DevTask& tp, int i,
                         const float* actions, int64_t* reset_buf, int64_t* progress_buf,
                         float* potentials, float* prev_potentials, float* actions_out) {
#pragma clang fp contract(off)
    const int lane = pair_l64() & 31, N = st.N, D = m.D, A = tp.A;
    const bool flagged = reset_buf[i] != 0;      // half-uniform
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
        if (lane < 3) st.root_pos[sx(st, lane, i)] = st.origins[(size_t)lane * N + i] + tp.init_root_pos[lane];
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

MI_D void pair_loco_post(const DevModel& m, const WaveTabs& t, const DevState& st,
                         const DevTask& tp, int i, float* sm, float a_lane,
                         float* obs_out, float* obs_task, float* rew, int64_t* reset_buf,
                         int64_t* progress_buf, float* potentials, float* prev_potentials,
                         float* rew_out, int64_t* reset_out) {
#pragma clang fp contract(off)
    const int lane = pair_l64() & 31, D = m.D, S = m.S, O = tp.O;
    const int h0 = pair_l64() & 32;
    const float co = tp.clip_obs;
    const float* us = sm + t.s_us;
    float* out = obs_out + (size_t)O * i;
    float* raw = obs_task ? obs_task + (size_t)O * i : nullptr;
    int64_t progress = 0, flagged = 0;
    int nan_env = 0;
    if (lane == 0) {
        progress = progress_buf[i] + 1;
        flagged = reset_buf[i];
        nan_env = st.nan_flag[i];
    }
    progress = __shfl(progress, h0);
    flagged = __shfl(flagged, h0);
    nan_env = __shfl(nan_env, h0);
    const int64_t done = nan_env ? 1 : loco_done(tp, sm[t.s_rp + 2], flagged, progress);
    mi_dr_env dre{};
    if (tp.dr_obs) dre = dr_begin(st, tp, 0, i, done != 0);
    auto put = [&](int k, float v) {
        if (tp.dr_obs) v = dr_col(st, tp, 0, dre, i, k, v);
        if (raw) raw[k] = v;
        out[k] = clampf(v, -co, co);
    };
    float* terms = sm + t.s_rb + 6 * S;
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
    for (int k = lane; k < 6 * S; k += 32) put(12 + 2 * D + k, sm[t.s_rb + k] * tp.contact_force_scale);
    wave_sync();
    // The three DOF-order reward sums (limit, action, electricity; ref humanoid.py / ant.py
    // calculate_metrics) run side by side on lanes 0..2 of each half: one instruction stream with
    // a per-lane base, each sum still accumulated in DOF order. Ant's limit count sums 0/1 floats,
    // exact far below 2^24, so it equals the reference's integer count.
    float part = 0.0f;
    if (lane < 3) {
        const float* tb = terms + (lane == 0 ? 2 * D : (lane == 1 ? 0 : D));
        for (int j = 0; j < D; ++j) part += tb[j];
    }
    const float limit_cost = __shfl(part, h0), act_cost = __shfl(part, h0 + 1),
                elec = __shfl(part, h0 + 2);
    if (lane < 3) {
        // lanes 0..2 share the root-frame prelude (same LDS words, same arithmetic), then run the
        // three angle chains of observations 7..9 side by side: yaw, roll and the walk-target
        // angle each go through one atan2 (+ fmod for the Euler angles) and normalize_angle,
        // instead of lane 0 running six atan2 and three sin/cos in sequence.
        float rp[3], rq[4], rv[6];
#pragma unroll
        for (int k = 0; k < 3; ++k) rp[k] = sm[t.s_rp + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) rq[k] = sm[t.s_rp + 4 + k];
        const float inv_start[4] = {1.0f, -0.0f, -0.0f, -0.0f};
        float tq[4];
        ref_quat_mul(rq, inv_start, tq);
        float ay, ax;
        if (lane < 2) {
            ref_euler_atan2_args(tq, lane, ay, ax);
        } else {
            ay = tp.target[2] - rp[2];
            ax = tp.target[0] - rp[0];
        }
        float ang = atan2f(ay, ax);
        if (lane < 2) ang = ref_fmod_pos(ang, 6.283185307179586f);
        const float yaw = __shfl(ang, h0);
        if (lane == 2) ang = ang - yaw;                          // angle_to_target = walk - yaw
        put(7 + lane, ref_normalize_angle(ang));
        if (lane != 0) return;
#pragma unroll
        for (int k = 0; k < 6; ++k) rv[k] = us[k];
        float tt[3] = {tp.target[0] - rp[0], tp.target[1] - rp[1], tp.target[2] - rp[2]};
        tt[2] = 0.0f;
        const float prev_p = potentials[i];
        const float nrm = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
        const float new_p = -nrm / tp.task_dt;
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
        const float o10 = up[2], o11 = heading_proj;
        put(0, rp[2]);
        put(1, vl[0]); put(2, vl[1]); put(3, vl[2]);
        put(4, al[0] * tp.angular_velocity_scale);
        put(5, al[1] * tp.angular_velocity_scale);
        put(6, al[2] * tp.angular_velocity_scale);
        put(10, o10);
        put(11, o11);
        potentials[i] = new_p;
        prev_potentials[i] = prev_p;
        const float heading = o11 > 0.8f ? tp.heading_weight : tp.heading_weight * o11 / 0.8f;
        const float upr = o10 > 0.93f ? 0.0f + tp.up_weight : 0.0f;
        float total = (new_p - prev_p) + tp.alive_reward_scale + upr + heading -
                      tp.actions_cost * act_cost - tp.energy_cost * elec - limit_cost;
        if (rp[2] < tp.termination_height) total = tp.death_cost;
        if (nan_env) {
            st.nan_flag[i] = 0;
            atomicAdd(st.nan_total, 1ull);
        }
        if (tp.dr_obs) dr_store(st, 0, i, dre);
        rew[i] = total;
        reset_buf[i] = done;
        progress_buf[i] = progress;
        if (rew_out) rew_out[i] = total;
        if (reset_out) reset_out[i] = done;
    }
}

}  // namespace mi
