// mi_task.hpp — fused task-layer math, one env per lane.
//
// Restates, op for op, the reference's TorchScript task kernels so the fp32 results track
// the reference's evaluation order (no FMA contraction inside these functions):
//   get_observations   tasks/shared/locomotion.py:194-254 (+ normalize_angle :190-192)
//   calculate_metrics  tasks/shared/locomotion.py:271-321
//   is_done            tasks/shared/locomotion.py:257-268
//   limit costs        tasks/humanoid.py:120-127, tasks/ant.py:92-95
//   reset_idx          tasks/shared/locomotion.py:116-145, tasks/cartpole.py:114-134
//   cartpole obs/rew/done tasks/cartpole.py:80-99,143-162
// and the closed omni.isaac.core.utils.torch helpers (compute_heading_and_up, compute_rot,
// quat_mul, quat_rotate(_inverse), get_euler_xyz, normalize, unscale) in wxyz convention.
#pragma once
#include "mi_device.hpp"

namespace mi {

MI_D void ref_quat_mul(const float* a, const float* b, float* o) {
#pragma clang fp contract(off)
    float w1 = a[0], x1 = a[1], y1 = a[2], z1 = a[3];
    float w2 = b[0], x2 = b[1], y2 = b[2], z2 = b[3];
    float ww = (z1 + x1) * (x2 + y2);
    float yy = (w1 - y1) * (w2 + z2);
    float zz = (w1 + y1) * (w2 - z2);
    float xx = ww + yy + zz;
    float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
    o[0] = qq - ww + (z1 - y1) * (y2 - z2);
    o[1] = qq - xx + (x1 + w1) * (x2 + w2);
    o[2] = qq - yy + (w1 - x1) * (y2 + z2);
    o[3] = qq - zz + (z1 + y1) * (w2 - x2);
}

template <bool INVERSE>
MI_D void ref_quat_rotate(const float* q, const float* v, float* o) {
#pragma clang fp contract(off)
    float w = q[0], x = q[1], y = q[2], z = q[3];
    float s = 2.0f * (w * w) - 1.0f;
    float cx = y * v[2] - z * v[1], cy = z * v[0] - x * v[2], cz = x * v[1] - y * v[0];
    float d = x * v[0] + y * v[1] + z * v[2];
    float bx = cx * w * 2.0f, by = cy * w * 2.0f, bz = cz * w * 2.0f;
    float ccx = x * d * 2.0f, ccy = y * d * 2.0f, ccz = z * d * 2.0f;
    if (INVERSE) {
        o[0] = v[0] * s - bx + ccx; o[1] = v[1] * s - by + ccy; o[2] = v[2] * s - bz + ccz;
    } else {
        o[0] = v[0] * s + bx + ccx; o[1] = v[1] * s + by + ccy; o[2] = v[2] * s + bz + ccz;
    }
}

MI_D float ref_fmod_pos(float a, float b) {
    float r = fmodf(a, b);
    if (r != 0.0f && ((r < 0.0f) != (b < 0.0f))) r += b;
    return r;
}

MI_D void ref_get_euler_xyz(const float* q, float& roll, float& pitch, float& yaw) {
#pragma clang fp contract(off)
    const float two_pi = 6.283185307179586f;
    float w = q[0], x = q[1], y = q[2], z = q[3];
    float sinr = 2.0f * (w * x + y * z);
    float cosr = w * w - x * x - y * y + z * z;
    float r = atan2f(sinr, cosr);
    float sinp = 2.0f * (w * y - z * x);
    float p = fabsf(sinp) >= 1.0f ? copysignf(1.5707963267948966f, sinp) : asinf(sinp);
    float siny = 2.0f * (w * z + x * y);
    float cosy = w * w + x * x - y * y - z * z;
    float yw = atan2f(siny, cosy);
    roll = ref_fmod_pos(r, two_pi);
    pitch = ref_fmod_pos(p, two_pi);
    yaw = ref_fmod_pos(yw, two_pi);
}

/* The atan2 arguments of get_euler_xyz's yaw (k = 0) and roll (k = 1), evaluated exactly as in
 * ref_get_euler_xyz, so lanes can run the angle chains side by side (mi_pair.hpp). */
MI_D void ref_euler_atan2_args(const float* q, int k, float& sy, float& sx) {
#pragma clang fp contract(off)
    float w = q[0], x = q[1], y = q[2], z = q[3];
    if (k == 0) {
        sy = 2.0f * (w * z + x * y);
        sx = w * w + x * x - y * y - z * z;
    } else {
        sy = 2.0f * (w * x + y * z);
        sx = w * w - x * x - y * y + z * z;
    }
}

MI_D float ref_normalize_angle(float x) { return atan2f(sinf(x), cosf(x)); }

MI_D float ref_unscale(float x, float l, float u) {
#pragma clang fp contract(off)
    return (2.0f * x - u - l) / (u - l);
}

MI_D float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// ---------------------------------------------------------------------------------------
// observation / action noise DR (randomize.py:212-306); noise math in include/mi_dr.h.
// which: 0 observations, 1 actions. State [6][N] field-major: coalesced across lanes = envs.
// ---------------------------------------------------------------------------------------
MI_D mi_dr_env dr_begin(const DevState& st, const DevTask& tp, int which, int i, bool reset) {
    const mi_dr_noise& r = which ? tp.act_r : tp.obs_r;
    const mi_dr_noise& v = which ? tp.act_i : tp.obs_i;
    const uint32_t* s = st.dr_state + (size_t)(3 * which) * st.N;
    return mi_dr_begin(s[i], s[st.N + i], s[2 * (size_t)st.N + i], reset ? 1 : 0, r.enabled,
                       v.enabled, v.frequency_interval);
}
MI_D void dr_store(const DevState& st, int which, int i, const mi_dr_env& e) {
    uint32_t* s = st.dr_state + (size_t)(3 * which) * st.N;
    s[i] = e.counter;
    s[st.N + i] = e.epoch;
    s[2 * (size_t)st.N + i] = e.draws;
}
// column k of env i's row after both schedules (correlated noise recomputed from the epoch)
MI_D float dr_col(const DevState& st, const DevTask& tp, int which, const mi_dr_env& e, int i,
                  int k, float x) {
    const mi_dr_noise& r = which ? tp.act_r : tp.obs_r;
    const mi_dr_noise& v = which ? tp.act_i : tp.obs_i;
    const uint64_t gid = (uint64_t)(st.off + i);
    float u[4];
    if (r.enabled) {
        float c = 0.0f;                      // epoch 0: the reference's zero-initialised buffer
        if (e.epoch) {
            uniform4(st.seed, gid, e.epoch, (uint32_t)(k >> 1),
                     which ? MI_DR_STREAM_ACT_RESET : MI_DR_STREAM_OBS_RESET, u);
            c = mi_dr_value(r.distribution, r.params[0], r.params[1], u, k);
        }
        x = mi_dr_op(r.operation, x, c);
    }
    if (v.enabled && e.fire) {
        uniform4(st.seed, gid, e.draws, (uint32_t)(k >> 1),
                 which ? MI_DR_STREAM_ACT_INTERVAL : MI_DR_STREAM_OBS_INTERVAL, u);
        x = mi_dr_op(v.operation, x, mi_dr_value(v.distribution, v.params[0], v.params[1], u, k));
    }
    return x;
}
// one env's whole row (one-lane-per-env kernels)
MI_D void dr_row(const DevState& st, const DevTask& tp, int which, int i, float* x, int C,
                 bool reset) {
    const mi_dr_env e = dr_begin(st, tp, which, i, reset);
    for (int k = 0; k < C; ++k) x[k] = dr_col(st, tp, which, e, i, k, x[k]);
    dr_store(st, which, i, e);
}

// ---------------------------------------------------------------------------------------
// reset_idx for one env (mask-driven on the device: no nonzero()/host sync)
// ---------------------------------------------------------------------------------------
MI_D void task_reset_env(const DevModel& m, const DevState& st, const DevTask& tp, int i,
                         float* potentials, float* prev_potentials) {
#pragma clang fp contract(off)
    const int N = st.N, D = m.D;
    const uint64_t gid = (uint64_t)(st.off + i);
    const uint32_t cnt = st.reset_count[i];
    if (tp.kind == MI_TASK_CARTPOLE) {
        float u[4];
        uniform4(st.seed, gid, cnt, 0, 0, u);
        st.q[sx(st, 0, i)] = 1.0f * (1.0f - 2.0f * u[0]);
        st.q[sx(st, 1, i)] = 0.39269908169872414f * (1.0f - 2.0f * u[1]);
        st.qd[sx(st, 0, i)] = 0.5f * (1.0f - 2.0f * u[2]);
        st.qd[sx(st, 1, i)] = 0.7853981633974483f * (1.0f - 2.0f * u[3]);
    } else {
        const float pn = tp.dof_pos_noise, vn = tp.dof_vel_noise;
        const float pw = (float)((double)pn - (double)(-pn));
        const float vw = (float)((double)vn - (double)(-vn));
        float u[4];
        for (int j = 0; j < D; ++j) {
            if ((j & 3) == 0) uniform4(st.seed, gid, cnt, (uint32_t)(j >> 2), 0, u);
            float v = tp.init_dof[j] + (pw * u[j & 3] + (-pn));
            const float lo = m.lower[j + 1], hi = m.upper[j + 1];
            if (lo < hi) { v = v < hi ? v : hi; v = v > lo ? v : lo; }
            st.q[sx(st, j, i)] = v;
        }
        for (int j = 0; j < D; ++j) {
            const int s = D + j;
            if (j == 0 || (s & 3) == 0) uniform4(st.seed, gid, cnt, (uint32_t)(s >> 2), 0, u);
            st.qd[sx(st, j, i)] = vw * u[s & 3] + (-vn);
        }
        float rp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            rp[k] = st.origins[(size_t)k * N + i] + tp.init_root_pos[k];
            st.root_pos[sx(st, k, i)] = rp[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) st.root_quat[sx(st, k, i)] = tp.init_root_quat[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) st.root_vel[sx(st, k, i)] = 0.0f;
        float tx = tp.target[0] - rp[0], ty = tp.target[1] - rp[1];
        float pot = -sqrtf(tx * tx + ty * ty + 0.0f * 0.0f) / tp.task_dt;
        if (prev_potentials) prev_potentials[i] = pot;
        if (potentials) potentials[i] = pot;
    }
    st.reset_count[i] = cnt + 1;
}

// pre_physics_step for one env: reset if flagged, clamp actions, efforts = a*gear*power
// fused: VecEnvRLGames.step's clamp + action noise DR (vec_env_rlgames.py:57-60) first
MI_D void task_pre_env(const DevModel& m, const DevState& st, const DevTask& tp, int i,
                       const float* actions, int64_t* reset_buf, int64_t* progress_buf,
                       float* potentials, float* prev_potentials, float* actions_out,
                       bool fused) {
#pragma clang fp contract(off)
    const int N = st.N, A = tp.A;
    const bool clamp_actions = fused, dr = fused && tp.dr_act;
    mi_dr_env e{};
    if (dr) e = dr_begin(st, tp, 1, i, reset_buf[i] != 0);
    if (reset_buf[i] != 0) {
        task_reset_env(m, st, tp, i, potentials, prev_potentials);
        reset_buf[i] = 0;
        progress_buf[i] = 0;
    }
    if (tp.kind == MI_TASK_CARTPOLE) {
        float a = actions[(size_t)A * i];
        if (clamp_actions) a = clampf(a, -tp.clip_actions, tp.clip_actions);
        if (dr) a = dr_col(st, tp, 1, e, i, 0, a);
        if (actions_out) actions_out[(size_t)A * i] = a;
        st.eff[sx(st, 0, i)] = tp.max_push_effort * a;
        st.eff[sx(st, 1, i)] = 0.0f;
    } else {
        for (int j = 0; j < A; ++j) {
            float a = actions[(size_t)A * i + j];
            if (clamp_actions) a = clampf(a, -tp.clip_actions, tp.clip_actions);
            if (dr) a = dr_col(st, tp, 1, e, i, j, a);
            if (actions_out) actions_out[(size_t)A * i + j] = a;
            st.eff[sx(st, j, i)] = a * tp.gears[j] * tp.power_scale;
        }
    }
    if (dr) dr_store(st, 1, i, e);
}

// ---------------------------------------------------------------------------------------
// get_observations (locomotion.py:80-101,194-254) for one env: writes the UNCLAMPED obs row
// and updates potentials / prev_potentials.
// ---------------------------------------------------------------------------------------
// get_observations, root-frame block: obs[0..11] + potentials / prev_potentials
MI_D void loco_obs_root(const DevState& st, const DevTask& tp, int i, float* orow,
                        float* potentials, float* prev_potentials) {
#pragma clang fp contract(off)
    float rp[3], rq[4], rv[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) rp[k] = st.root_pos[sx(st, k, i)];
#pragma unroll
    for (int k = 0; k < 4; ++k) rq[k] = st.root_quat[sx(st, k, i)];
#pragma unroll
    for (int k = 0; k < 6; ++k) rv[k] = st.root_vel[sx(st, k, i)];
    float tt[3] = {tp.target[0] - rp[0], tp.target[1] - rp[1], tp.target[2] - rp[2]};
    tt[2] = 0.0f;
    const float prev_p = potentials[i];
    const float nrm = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
    const float new_p = -nrm / tp.task_dt;
    // compute_heading_and_up
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
    // compute_rot
    float vl[3], al[3];
    ref_quat_rotate<true>(tq, rv, vl);
    ref_quat_rotate<true>(tq, rv + 3, al);
    float roll, pitch, yaw;
    ref_get_euler_xyz(tq, roll, pitch, yaw);
    const float walk = atan2f(tp.target[2] - rp[2], tp.target[0] - rp[0]);
    const float angle_to_target = walk - yaw;
    orow[0] = rp[2];
    orow[1] = vl[0]; orow[2] = vl[1]; orow[3] = vl[2];
    orow[4] = al[0] * tp.angular_velocity_scale;
    orow[5] = al[1] * tp.angular_velocity_scale;
    orow[6] = al[2] * tp.angular_velocity_scale;
    orow[7] = ref_normalize_angle(yaw);
    orow[8] = ref_normalize_angle(roll);
    orow[9] = ref_normalize_angle(angle_to_target);
    orow[10] = up[2];
    orow[11] = heading_proj;
    potentials[i] = new_p;
    prev_potentials[i] = prev_p;
}

// get_observations, per-DOF / sensor block: obs[12 ..]
MI_D void loco_obs_dof(const DevModel& m, const DevState& st, const DevTask& tp, int i,
                       const float* act /* row */, float act_clip, float* orow) {
#pragma clang fp contract(off)
    const int D = m.D, S = m.S;
    for (int j = 0; j < D; ++j) {
        orow[12 + j] = ref_unscale(st.q[sx(st, j, i)], m.lower[j + 1], m.upper[j + 1]);
        orow[12 + D + j] = st.qd[sx(st, j, i)] * tp.dof_vel_scale;
        orow[12 + 2 * D + 6 * S + j] = clampf(act[j], -act_clip, act_clip);
    }
    for (int k = 0; k < 6 * S; ++k)
        orow[12 + 2 * D + k] = st.sens[ssx(st, k, i)] * tp.contact_force_scale;
}

// ---------------------------------------------------------------------------------------
// get_observations (locomotion.py:80-101,194-254) for one env: writes the UNCLAMPED obs row
// and updates potentials / prev_potentials.
// ---------------------------------------------------------------------------------------
MI_D void loco_obs_env(const DevModel& m, const DevState& st, const DevTask& tp, int i,
                       const float* act /* row */, float act_clip, float* orow,
                       float* potentials, float* prev_potentials) {
    loco_obs_root(st, tp, i, orow, potentials, prev_potentials);
    loco_obs_dof(m, st, tp, i, act, act_clip, orow);
}

// calculate_metrics (locomotion.py:271-321 + humanoid.py:120-127 / ant.py:92-95), split into
// the per-DOF sums (DOF order) and the total
struct LocoTerms { float limit_cost, act_cost, elec; };
MI_D LocoTerms loco_reward_terms(const DevTask& tp, int D, const float* orow, const float* act) {
#pragma clang fp contract(off)
    LocoTerms r{0.0f, 0.0f, 0.0f};
    if (tp.kind == MI_TASK_HUMANOID) {
        for (int j = 0; j < D; ++j) {
            const float a = fabsf(orow[12 + j]);
            const float sc = tp.joints_at_limit_cost * (a - 0.98f) / 0.02f;
            r.limit_cost += (a > 0.98f ? 1.0f : 0.0f) * sc * tp.ratio[j];
        }
    } else {
        int64_t cnt = 0;
        for (int j = 0; j < D; ++j) cnt += orow[12 + j] > 0.99f;
        r.limit_cost = (float)cnt;
    }
    for (int j = 0; j < D; ++j) r.act_cost += act[j] * act[j];
    for (int j = 0; j < D; ++j) r.elec += fabsf(act[j] * orow[12 + D + j]) * tp.ratio[j];
    return r;
}
MI_D float loco_reward_total(const DevTask& tp, float o0, float o10, float o11, float pot,
                             float prev, const LocoTerms& t) {
#pragma clang fp contract(off)
    const float heading = o11 > 0.8f ? tp.heading_weight : tp.heading_weight * o11 / 0.8f;
    const float upr = o10 > 0.93f ? 0.0f + tp.up_weight : 0.0f;
    float total = (pot - prev) + tp.alive_reward_scale + upr + heading -
                  tp.actions_cost * t.act_cost - tp.energy_cost * t.elec - t.limit_cost;
    if (o0 < tp.termination_height) total = tp.death_cost;
    return total;
}
MI_D float loco_reward(const DevTask& tp, int D, const float* orow, const float* act, float pot,
                       float prev) {
    return loco_reward_total(tp, orow[0], orow[10], orow[11], pot, prev,
                             loco_reward_terms(tp, D, orow, act));
}

// is_done (locomotion.py:257-268)
MI_D int64_t loco_done(const DevTask& tp, float obs0, int64_t reset, int64_t progress) {
    int64_t r = obs0 < tp.termination_height ? 1 : reset;
    if ((float)progress >= tp.max_episode_length - 1.0f) r = 1;
    return r;
}

// The root-frame block and the reward sums of a 32-env tile on all 64 lanes of a wave (the
// obs/reward fuse k_loco_post_pipe): lanes e and e + 32 both hold env e. Every value is the
// same operation sequence as loco_obs_root / loco_reward_terms (bit-identical results); only
// the assignment of the costly chains to lanes differs:
//  - get_euler_xyz's roll (lower half) and yaw (upper half) run as ONE instruction stream
//    (atan2 -> fmod -> normalize_angle on a per-lane selection of the inputs), then the target
//    angle on every lane with env e's yaw from the upper half (ds_bpermute);
//  - the energy sum (lower half) and the action cost (upper half) run as one loop of
//    |x_j y_j| w_j: with x = y = a, w = 1 it is a_j a_j exactly (a square is >= 0; * 1 exact).
// rec: env e's record in LDS (pos 3, quat 4, vel 6); writes obs[0..11] of orow (obs[7] from the
// upper half) and potentials / prev_potentials of env e when `write`.
MI_D void loco_obs_root_pair(const float* rec, const DevTask& tp, int lane, float* orow,
                             float* potentials, float* prev_potentials, bool write) {
#pragma clang fp contract(off)
    const int e = lane & 31;
    const bool hi = lane >= 32;
    float rp[3], rq[4], rv[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) rp[k] = rec[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) rq[k] = rec[3 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) rv[k] = rec[7 + k];
    float tt[3] = {tp.target[0] - rp[0], tp.target[1] - rp[1], tp.target[2] - rp[2]};
    tt[2] = 0.0f;
    const float prev_p = potentials[e];
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
    // ref_get_euler_xyz: roll on the lower half, yaw on the upper half
    const float two_pi = 6.283185307179586f;
    const float w = tq[0], x = tq[1], y = tq[2], z = tq[3];
    const float sinr = 2.0f * (w * x + y * z);
    const float cosr = w * w - x * x - y * y + z * z;
    const float siny = 2.0f * (w * z + x * y);
    const float cosy = w * w + x * x - y * y - z * z;
    const float ang = ref_fmod_pos(atan2f(hi ? siny : sinr, hi ? cosy : cosr), two_pi);
    const float nang = ref_normalize_angle(ang);                  // obs[8] roll / obs[7] yaw
    const float yaw = __shfl(ang, e + 32);
    const float walk = atan2f(tp.target[2] - rp[2], tp.target[0] - rp[0]);
    const float n_target = ref_normalize_angle(walk - yaw);
    if (!write) return;
    if (hi) {
        orow[7] = nang;
        return;
    }
    orow[0] = rp[2];
    orow[1] = vl[0]; orow[2] = vl[1]; orow[3] = vl[2];
    orow[4] = al[0] * tp.angular_velocity_scale;
    orow[5] = al[1] * tp.angular_velocity_scale;
    orow[6] = al[2] * tp.angular_velocity_scale;
    orow[8] = nang;
    orow[9] = n_target;
    orow[10] = up[2];
    orow[11] = heading_proj;
    potentials[e] = new_p;
    prev_potentials[e] = prev_p;
}
// loco_reward_terms on lane pairs (see above): valid on the lower half
MI_D LocoTerms loco_reward_terms_pair(const DevTask& tp, int D, const float* orow, const float* act,
                                      int lane) {
#pragma clang fp contract(off)
    const bool hi = lane >= 32;
    LocoTerms r{0.0f, 0.0f, 0.0f};
    if (tp.kind == MI_TASK_HUMANOID) {
        for (int j = 0; j < D; ++j) {
            const float a = fabsf(orow[12 + j]);
            const float sc = tp.joints_at_limit_cost * (a - 0.98f) / 0.02f;
            r.limit_cost += (a > 0.98f ? 1.0f : 0.0f) * sc * tp.ratio[j];
        }
    } else {
        int64_t cnt = 0;
        for (int j = 0; j < D; ++j) cnt += orow[12 + j] > 0.99f;
        r.limit_cost = (float)cnt;
    }
    const float* yv = hi ? act : orow + 12 + D;
    float sum = 0.0f;
    for (int j = 0; j < D; ++j) sum += fabsf(act[j] * yv[j]) * (hi ? 1.0f : tp.ratio[j]);
    r.elec = sum;
    r.act_cost = __shfl(sum, (lane & 31) + 32);
    return r;
}

// NaN guard: a non-finite physics state forces a reset of that env
MI_D int64_t nan_guard(const DevState& st, int i, int64_t done) {
    if (st.nan_flag[i]) {
        st.nan_flag[i] = 0;
        atomicAdd(st.nan_total, 1ull);
        return 1;
    }
    return done;
}

// cartpole.py:80-99
MI_D void cartpole_obs_env(const DevState& st, int i, float* orow) {
    const int N = st.N;
    orow[0] = st.q[sx(st, 0, i)];
    orow[1] = st.qd[sx(st, 0, i)];
    orow[2] = st.q[sx(st, 1, i)];
    orow[3] = st.qd[sx(st, 1, i)];
}
// cartpole.py:143-153
MI_D float cartpole_reward(const DevTask& tp, const float* o) {
#pragma clang fp contract(off)
    const float x = o[0], xd = o[1], th = o[2], thd = o[3];
    const float half_pi = 1.5707963267948966f;
    float r = 1.0f - th * th - 0.01f * fabsf(xd) - 0.005f * fabsf(thd);
    if (fabsf(x) > tp.reset_dist) r = -2.0f;
    if (fabsf(th) > half_pi) r = -2.0f;
    return r;
}
// cartpole.py:155-162 (note: no "-1" and no OR with the previous reset_buf)
MI_D int64_t cartpole_done(const DevTask& tp, const float* o, int64_t progress) {
    const float half_pi = 1.5707963267948966f;
    int64_t d = fabsf(o[0]) > tp.reset_dist ? 1 : 0;
    if (fabsf(o[2]) > half_pi) d = 1;
    if ((float)progress >= tp.max_episode_length) d = 1;
    return d;
}

}  // namespace mi
