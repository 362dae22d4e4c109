// mi_device.hpp — device-side building blocks of libmi_sim.so (gfx950).
//
// Layout:
//   * physics state (DevState): per-env records for the wavefront-per-env kernels (a wave
//     reads / writes its env's fields in whole 128-B lines), field-major SoA [field][N] for
//     the one-lane-per-env kernels (lane i touches element i of every field: coalesced);
//   * the per-env solver workspace is [env/64][slot][64] — a wave's workspace is one
//     contiguous slab and every slot access is one coalesced 256-B line;
//   * the model (link tree, inertias, geoms) is shared by all envs and read through
//     wave-uniform addresses (scalar loads, SGPR-resident).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mi_sim.h"
#include "../../include/mi_dr.h"

#define MI_D __device__ __forceinline__
#define MI_MAXA 32     // max actions / joint DOFs handled by the task kernels
#define MI_MAXNV 64    // max generalized velocities (6 + D)

namespace mi {

constexpr float kPi = 3.14159265358979323846f;

// ---------------------------------------------------------------------------------------
// device views
// ---------------------------------------------------------------------------------------
struct DevModel {
    int dyn, root_free, L, D, nv, nr, G, S, npts, max_rows, slots;
    const int* parent;      // [L]
    const int* jtype;       // [L]
    const float* axis;      // [L*3]
    const float* pos;       // [L*3]
    const float* quat;      // [L*4]
    const float* mass;      // [L]
    const float* com;       // [L*3]
    const float* inertia;   // [L*6]
    const float* lower;     // [L]
    const float* upper;     // [L]
    const float* damping;   // [L]
    const float* armature;  // [L]
    const int* dof_parent;  // [nv]
    const int* dof_link;    // [nv]
    const int* geom_link;   // [G]
    const float* geom_p0;   // [G*3]
    const float* geom_p1;   // [G*3]
    const float* geom_radius;
    const int* pt_geom;     // [npts]
    const int* pt_end;      // [npts]
    const int* sensor_link; // [S]
    const float* sensor_pos;// [S*3]
    float cart_mass, pole_mass, pole_com, pole_inertia, cart_damping, pole_damping;
    // workspace slot offsets
    int o_R, o_o, o_aw, o_Ic, o_S, o_V, o_A, o_F, o_M, o_u, o_r, o_Jr, o_W, o_b, o_lam, o_Ad,
        o_rk, o_cp, o_cl, o_ds;
};

// Physics state element (field k, env i) lives at k * fs + i * es floats from the field's
// base pointer. Two layouts (chosen at mi_sim_create):
//   per-env records (wavefront-per-env kernels): fs = 1, es = record length (a multiple of
//     32 floats = whole 128-B lines); the wave reads / writes its env's state with one
//     coalesced access per field group;
//   field-major SoA (one-lane-per-env kernels): fs = N, es = 1; lane-consecutive envs.
// The sensor wrenches have strides of their own (sfs, ses): with records they are NOT in the
// record but in a [N][6S] array next to it (sfs = 1, ses = 6S), so the state the obs/reward fuse
// reads fits whole lines (Humanoid: pos, quat, vel, q, qd = 55 floats, 2 of the record's 3 lines,
// + 48 contiguous sensor bytes, instead of all 3 lines); field-major: sfs = N, ses = 1.
struct DevState {
    int N;
    int fs, es;           // field stride, env stride (floats)
    int sfs, ses;         // sensor field / env stride (floats)
    int64_t off;          // global id of env 0 (multi-GPU shard offset)
    uint64_t seed;
    const float* origins; // [3][N]
    float* root_pos;      // 3 fields, world
    float* root_quat;     // 4 fields, wxyz
    float* root_vel;      // 6 fields: lin, ang (world)
    float* q;             // D fields
    float* qd;            // D fields
    float* eff;           // D fields
    float* sens;          // 6 S fields
    uint32_t* reset_count;// [N]
    int32_t* nan_flag;    // [N]
    unsigned long long* nan_total;
    uint32_t* dr_state;   // [6][N] obs counter, epoch, draws; act counter, epoch, draws (or null)
    float* ws;            // workspace [N/64][slots][64]
    int32_t* load;        // [N] constraint rows of each env's last fused env-step (paired kernels' pairing)
    int pair_by_load;     // paired kernels: pair each workgroup's envs heaviest with lightest by `load`
};

MI_D size_t sx(const DevState& st, int k, int i) {
    return (size_t)k * (size_t)st.fs + (size_t)i * (size_t)st.es;
}
// sensor element k of env i (st.sens)
MI_D size_t ssx(const DevState& st, int k, int i) {
    return (size_t)k * (size_t)st.sfs + (size_t)i * (size_t)st.ses;
}

struct DevTask {
    int kind, O, A;
    float clip_actions, clip_obs, max_episode_length;
    float power_scale, heading_weight, up_weight, actions_cost, energy_cost;
    float dof_vel_scale, angular_velocity_scale, contact_force_scale;
    float joints_at_limit_cost, death_cost, termination_height, alive_reward_scale;
    float task_dt, target[3], init_root_pos[3], init_root_quat[4];
    float dof_pos_noise, dof_vel_noise, reset_dist, max_push_effort;
    float gears[MI_MAXA], ratio[MI_MAXA], init_dof[MI_MAXA];
    int dr_obs, dr_act;                       // observation / action noise DR on
    mi_dr_noise obs_r, obs_i, act_r, act_i;   // schedules (include/mi_sim.h, mi_dr.h)
};

// ---------------------------------------------------------------------------------------
// Philox4x32-10 — identical stream to oracle/oracle.c:orc_uniform
// ---------------------------------------------------------------------------------------
MI_D void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    }
}
// 4 consecutive uniforms of slots [4*blk, 4*blk+4)
MI_D void uniform4(uint64_t seed, uint64_t gid, uint32_t cnt, uint32_t blk, uint32_t stream,
                   float o[4]) {
    uint32_t c[4] = {blk, cnt, (uint32_t)gid, (uint32_t)(gid >> 32) ^ (stream << 28)};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (float)(c[k] >> 8) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------------------
// 3-vectors / rotations
// ---------------------------------------------------------------------------------------
MI_D void cross3(const float* a, const float* b, float* o) {
    float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2],
          t2 = a[0] * b[1] - a[1] * b[0];
    o[0] = t0; o[1] = t1; o[2] = t2;
}
MI_D float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
MI_D float dot6(const float* a, const float* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
MI_D void m3_from_quat(const float* q, float* R) {
    float w = q[0], x = q[1], y = q[2], z = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
    R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
    R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
MI_D void m3_mul(const float* A, const float* B, float* C) {
    float T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int k = 0; k < 9; ++k) C[k] = T[k];
}
MI_D void m3_vec(const float* A, const float* v, float* o) {
    float t0 = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
    float t1 = A[3] * v[0] + A[4] * v[1] + A[5] * v[2];
    float t2 = A[6] * v[0] + A[7] * v[1] + A[8] * v[2];
    o[0] = t0; o[1] = t1; o[2] = t2;
}
MI_D void m3_tvec(const float* A, const float* v, float* o) {
    float t0 = A[0] * v[0] + A[3] * v[1] + A[6] * v[2];
    float t1 = A[1] * v[0] + A[4] * v[1] + A[7] * v[2];
    float t2 = A[2] * v[0] + A[5] * v[1] + A[8] * v[2];
    o[0] = t0; o[1] = t1; o[2] = t2;
}
MI_D void m3_axis_angle(const float* a, float t, float* R) {
    float s, c;
    sincosf(t, &s, &c);
    float C = 1.0f - c, x = a[0], y = a[1], z = a[2];
    R[0] = c + x * x * C;     R[1] = x * y * C - z * s; R[2] = x * z * C + y * s;
    R[3] = y * x * C + z * s; R[4] = c + y * y * C;     R[5] = y * z * C - x * s;
    R[6] = z * x * C - y * s; R[7] = z * y * C + x * s; R[8] = c + z * z * C;
}
// spatial motion cross [w;v] x [a;b] = [w x a; w x b + v x a]
MI_D void crm(const float* V, const float* s, float* o) {
    float t[6], u[3];
    cross3(V, s, t);
    cross3(V, s + 3, t + 3);
    cross3(V + 3, s, u);
    o[0] = t[0]; o[1] = t[1]; o[2] = t[2];
    o[3] = t[3] + u[0]; o[4] = t[4] + u[1]; o[5] = t[5] + u[2];
}
// spatial force cross [w;v] x* [n;f] = [w x n + v x f; w x f]
MI_D void crf(const float* V, const float* f, float* o) {
    float t[3], u[3], w[3];
    cross3(V, f, t);
    cross3(V + 3, f + 3, u);
    cross3(V, f + 3, w);
    o[0] = t[0] + u[0]; o[1] = t[1] + u[1]; o[2] = t[2] + u[2];
    o[3] = w[0]; o[4] = w[1]; o[5] = w[2];
}
// compact spatial inertia about p0: I10 = {m, h(3) = m c, Ibar(6) = xx yy zz xy xz yz}
// I * [w; v] = [Ibar w + h x v ; m v - h x w]
MI_D void inertia_mul(const float* I, const float* v, float* o) {
    const float* w = v;
    const float* l = v + 3;
    float hxv[3], hxw[3];
    cross3(I + 1, l, hxv);
    cross3(I + 1, w, hxw);
    o[0] = I[4] * w[0] + I[7] * w[1] + I[8] * w[2] + hxv[0];
    o[1] = I[7] * w[0] + I[5] * w[1] + I[9] * w[2] + hxv[1];
    o[2] = I[8] * w[0] + I[9] * w[1] + I[6] * w[2] + hxv[2];
    o[3] = I[0] * l[0] - hxw[0];
    o[4] = I[0] * l[1] - hxw[1];
    o[5] = I[0] * l[2] - hxw[2];
}

// ---------------------------------------------------------------------------------------
// per-env workspace accessor: ws[(env/64)*slots*64 + slot*64 + env%64]
// ---------------------------------------------------------------------------------------
struct WS {
    float* p;
    MI_D WS(float* ws, int slots, int env) : p(ws + (size_t)(env >> 6) * slots * 64 + (env & 63)) {}
    MI_D float& operator[](int slot) const { return p[(size_t)slot * 64]; }
};

}  // namespace mi
