// mi_artic.hpp — articulated-body physics substep, one env per lane (round-1 mapping).
//
// Replaces the closed PhysX GPU articulation step behind World.step
// (envs/vec_env_rlgames.py:64-66; solver settings cfg/task/Humanoid.yaml:34-63). Algorithm
// (DESIGN.md §Physics), every spatial quantity about p0 = the root origin with world axes,
// so composite inertias and forces accumulate without coordinate transforms:
//   1. root->leaf: forward kinematics, motion subspaces s_k, link velocities V, velocity-
//      product accelerations (gravity as a fictitious base acceleration), Newton-Euler forces
//   2. leaf->root: composite inertias Ic and force sums (RNE bias C = s_k . F)
//   3. CRBA on the DOF tree (M_jk = s_j . Ic_k s_k over ancestors only)
//   4. tree-sparse LTDL factorisation (Featherstone RBDA §6.5: no fill-in in BFS order) of
//      M~ = M + diag(armature + dt*damping) (implicit joint damping)
//   5. free velocity u* = u + dt M~^-1 (tau - C - B u)
//   6. ground contacts (sphere / capsule end points vs z = 0, speculative within
//      contact_offset) and joint limits as velocity rows; W_r = M~^-1 J_r^T by two sparse
//      triangular solves; projected Gauss-Seidel (solver_position_iteration_count sweeps),
//      box friction |l_t| <= mu l_n
//   7. foot force sensors = contact wrench on the sensor link, link frame
//   8. semi-implicit Euler; root quaternion by the exponential map.
// The CPU oracle restates the same model with a dense J^T I J mass matrix and Cholesky.
#pragma once
#include "mi_device.hpp"

namespace mi {

struct SimP {
    float dt, g[3];
    int iters;        // PGS: sweeps; TGS: position iterations (sub-steps)
    float contact_offset, rest_offset, friction, max_depen, erp, max_angvel;
    float ang_damp;   // per-link angular damping (1/s): torque -ang_damp * I_com * omega
    int tgs;          // solver_type 1 (include/mi_sim.h MI_SOLVER_TGS)
    int viters;       // TGS velocity iterations
    float h;          // TGS sub-step dt / iters (PGS: dt)
};

// Constraint-row bias of a normal / limit row with separation e. PGS: over the substep (the
// row stores its bias). TGS: over the sub-step h from the row's current separation; position
// iterations correct a penetration (erp), velocity iterations only keep the speculative part.
MI_D float row_bias(const SimP& p, float e, float step, bool correct) {
    // e >= 0 ? -e / step : (correct ? -erp e / step : 0), with ONE division: the numerator is
    // selected first (same roundings; a lane-divergent select ran both divisions' ~10-op
    // sequences under exec masks, once per sweep in the TGS sweeps)
    const float num = e >= 0.0f ? -e : (correct ? -p.erp * e : 0.0f);
    const float b = num / step;
    return b > p.max_depen ? p.max_depen : b;
}

MI_D void cartpole_substep(const DevModel& m, const SimP& p, float& x, float& th, float& xd,
                           float& thd, float F0, float F1) {
    const float mc = m.cart_mass, mp = m.pole_mass, l = m.pole_com, Ip = m.pole_inertia;
    const float g = -p.g[2], dt = p.dt;
    float s, c;
    sincosf(th, &s, &c);
    const float m11 = mc + mp, m12 = mp * l * c, m22 = Ip + mp * l * l;
    const float r1 = F0 + mp * l * s * thd * thd - m.cart_damping * xd;
    const float r2 = F1 + mp * g * l * s - m.pole_damping * thd;
    const float det = m11 * m22 - m12 * m12;
    const float xdd = (m22 * r1 - m12 * r2) / det;
    const float thdd = (m11 * r2 - m12 * r1) / det;
    xd = xd + dt * xdd;
    thd = thd + dt * thdd;
    x = x + dt * xd;
    th = th + dt * thd;
}

// x <- M~^-1 x with the in-place LTDL factor stored in the M slots (lower triangle)
MI_D void ltdl_solve(const DevModel& m, const WS& w, int xo) {
    const int nv = m.nv;
    for (int i = nv - 1; i >= 0; --i) {
        const float xi = w[xo + i];
        int j = m.dof_parent[i];
        while (j >= 0) {
            w[xo + j] -= w[m.o_M + i * nv + j] * xi;
            j = m.dof_parent[j];
        }
    }
    for (int i = 0; i < nv; ++i) w[xo + i] = w[xo + i] / w[m.o_M + i * nv + i];
    for (int i = 0; i < nv; ++i) {
        float xi = w[xo + i];
        int j = m.dof_parent[i];
        while (j >= 0) {
            xi -= w[m.o_M + i * nv + j] * w[xo + j];
            j = m.dof_parent[j];
        }
        w[xo + i] = xi;
    }
}

// dense constraint row r <- J for a unit spatial force f applied to link l
MI_D void make_row(const DevModel& m, const WS& w, int r, int l, const float* f) {
    const int nv = m.nv, nr = m.nr;
    const int ro = m.o_Jr + r * nv;
    for (int k = 0; k < nv; ++k) w[ro + k] = 0.0f;
    int x = l;
    while (x > 0) {
        const int k = nr + x - 1;
        float s[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) s[c] = w[m.o_S + 6 * k + c];
        w[ro + k] = dot6(s, f);
        x = m.parent[x];
    }
    if (nr) {
        // root dofs: linear k -> f.lin[k], angular k -> f.ang[k]
#pragma unroll
        for (int k = 0; k < 3; ++k) { w[ro + k] = f[3 + k]; w[ro + 3 + k] = f[k]; }
    }
}

MI_D void artic_substep(const DevModel& m, const DevState& st, const SimP& p, int i) {
    const int N = st.N, L = m.L, D = m.D, nv = m.nv, nr = m.nr;
    const float dt = p.dt;
    WS w(st.ws, m.slots, i);
    float rp[3], rq[4];
#pragma unroll
    for (int k = 0; k < 3; ++k) rp[k] = st.root_pos[sx(st, k, i)];
#pragma unroll
    for (int k = 0; k < 4; ++k) rq[k] = st.root_quat[sx(st, k, i)];
    for (int k = 0; k < nr; ++k) w[m.o_u + k] = st.root_vel[sx(st, k, i)];
    for (int j = 0; j < D; ++j) w[m.o_u + nr + j] = st.qd[sx(st, j, i)];

    // ---------------- pass 1: root -> leaves ----------------
    for (int l = 0; l < L; ++l) {
        float R[9], o[3], V[6], A[6];
        if (l == 0) {
            m3_from_quat(rq, R);
            o[0] = o[1] = o[2] = 0.0f;
            A[0] = A[1] = A[2] = 0.0f;
            A[3] = -p.g[0]; A[4] = -p.g[1]; A[5] = -p.g[2];
            if (nr) {
                const float v[3] = {w[m.o_u + 0], w[m.o_u + 1], w[m.o_u + 2]};
                const float om[3] = {w[m.o_u + 3], w[m.o_u + 4], w[m.o_u + 5]};
                float wv[3];
                cross3(om, v, wv);
                A[3] -= wv[0]; A[4] -= wv[1]; A[5] -= wv[2];
                V[0] = om[0]; V[1] = om[1]; V[2] = om[2];
                V[3] = v[0]; V[4] = v[1]; V[5] = v[2];
            } else {
#pragma unroll
                for (int c = 0; c < 6; ++c) V[c] = 0.0f;
            }
        } else {
            const int P = m.parent[l], k = nr + l - 1;
            float RP[9], oP[3], VP[6], AP[6], Rq[9], Rj[9], a[3], op[3];
#pragma unroll
            for (int c = 0; c < 9; ++c) RP[c] = w[m.o_R + 9 * P + c];
#pragma unroll
            for (int c = 0; c < 3; ++c) oP[c] = w[m.o_o + 3 * P + c];
#pragma unroll
            for (int c = 0; c < 6; ++c) { VP[c] = w[m.o_V + 6 * P + c]; AP[c] = w[m.o_A + 6 * P + c]; }
            m3_from_quat(m.quat + 4 * l, Rq);
            m3_mul(RP, Rq, Rj);
            m3_vec(Rj, m.axis + 3 * l, a);
            m3_vec(RP, m.pos + 3 * l, op);
            const float qj = st.q[sx(st, l - 1, i)];
            float s[6];
            if (m.jtype[l] == MI_JOINT_HINGE) {
                float Ra[9];
                m3_axis_angle(m.axis + 3 * l, qj, Ra);
                m3_mul(Rj, Ra, R);
#pragma unroll
                for (int c = 0; c < 3; ++c) o[c] = oP[c] + op[c];
                s[0] = a[0]; s[1] = a[1]; s[2] = a[2];
                cross3(o, a, s + 3);
            } else {
#pragma unroll
                for (int c = 0; c < 9; ++c) R[c] = Rj[c];
#pragma unroll
                for (int c = 0; c < 3; ++c) o[c] = oP[c] + op[c] + a[c] * qj;
                s[0] = s[1] = s[2] = 0.0f;
                s[3] = a[0]; s[4] = a[1]; s[5] = a[2];
            }
#pragma unroll
            for (int c = 0; c < 6; ++c) w[m.o_S + 6 * k + c] = s[c];
            const float uk = w[m.o_u + k];
            float sd[6];
            crm(VP, s, sd);
#pragma unroll
            for (int c = 0; c < 6; ++c) { V[c] = VP[c] + s[c] * uk; A[c] = AP[c] + sd[c] * uk; }
        }
#pragma unroll
        for (int c = 0; c < 9; ++c) w[m.o_R + 9 * l + c] = R[c];
#pragma unroll
        for (int c = 0; c < 3; ++c) w[m.o_o + 3 * l + c] = o[c];
#pragma unroll
        for (int c = 0; c < 6; ++c) { w[m.o_V + 6 * l + c] = V[c]; w[m.o_A + 6 * l + c] = A[c]; }
        // link spatial inertia about p0 (compact) and Newton-Euler force
        float I[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        float F[6] = {0, 0, 0, 0, 0, 0};
        const float mass = m.mass[l];
        if (mass > 0.0f) {
            float c[3], T[9], Iw[9];
            m3_vec(R, m.com + 3 * l, c);
            c[0] += o[0]; c[1] += o[1]; c[2] += o[2];
            const float* in = m.inertia + 6 * l;
            const float Ib[9] = {in[0], in[3], in[4], in[3], in[1], in[5], in[4], in[5], in[2]};
            m3_mul(R, Ib, T);
            // Iw = T R^T
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    Iw[3 * a + b] = T[3 * a] * R[3 * b] + T[3 * a + 1] * R[3 * b + 1] + T[3 * a + 2] * R[3 * b + 2];
            const float cc = dot3(c, c);
            I[0] = mass;
            I[1] = mass * c[0]; I[2] = mass * c[1]; I[3] = mass * c[2];
            I[4] = Iw[0] + mass * (cc - c[0] * c[0]);
            I[5] = Iw[4] + mass * (cc - c[1] * c[1]);
            I[6] = Iw[8] + mass * (cc - c[2] * c[2]);
            I[7] = Iw[1] - mass * c[0] * c[1];
            I[8] = Iw[2] - mass * c[0] * c[2];
            I[9] = Iw[5] - mass * c[1] * c[2];
            float IA[6], IV[6], t[6];
            inertia_mul(I, A, IA);
            inertia_mul(I, V, IV);
            crf(V, IV, t);
#pragma unroll
            for (int c2 = 0; c2 < 6; ++c2) F[c2] = IA[c2] + t[c2];
            // link angular damping: the torque -c I_com omega enters the bias as +c I_com omega
            float Iwv[3];
            m3_vec(Iw, V, Iwv);
#pragma unroll
            for (int c2 = 0; c2 < 3; ++c2) F[c2] = F[c2] + p.ang_damp * Iwv[c2];
        }
#pragma unroll
        for (int c = 0; c < 10; ++c) w[m.o_Ic + 10 * l + c] = I[c];
#pragma unroll
        for (int c = 0; c < 6; ++c) w[m.o_F + 6 * l + c] = F[c];
    }
    // ---------------- pass 2: leaves -> root ----------------
    for (int l = L - 1; l >= 1; --l) {
        const int P = m.parent[l];
#pragma unroll
        for (int c = 0; c < 10; ++c) w[m.o_Ic + 10 * P + c] += w[m.o_Ic + 10 * l + c];
#pragma unroll
        for (int c = 0; c < 6; ++c) w[m.o_F + 6 * P + c] += w[m.o_F + 6 * l + c];
    }
    if (nr) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            float s[6] = {0, 0, 0, 0, 0, 0};
            if (k < 3) s[3 + k] = 1.0f; else s[k - 3] = 1.0f;
#pragma unroll
            for (int c = 0; c < 6; ++c) w[m.o_S + 6 * k + c] = s[c];
        }
    }
    // ---------------- CRBA + RHS ----------------
    for (int k = 0; k < nv; ++k) {
        const int l = m.dof_link[k];
        float s[6], I[10], f[6], F[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) { s[c] = w[m.o_S + 6 * k + c]; F[c] = w[m.o_F + 6 * l + c]; }
#pragma unroll
        for (int c = 0; c < 10; ++c) I[c] = w[m.o_Ic + 10 * l + c];
        inertia_mul(I, s, f);
        float diag = dot6(s, f);
        const float Ck = dot6(s, F);
        float rhs = -Ck;
        if (k >= nr) {
            diag += m.armature[l] + dt * m.damping[l];
            rhs += st.eff[sx(st, k - nr, i)] - m.damping[l] * w[m.o_u + k];
        }
        w[m.o_M + k * nv + k] = diag;
        w[m.o_r + k] = rhs;
        int j = m.dof_parent[k];
        while (j >= 0) {
            float sj[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) sj[c] = w[m.o_S + 6 * j + c];
            w[m.o_M + k * nv + j] = dot6(sj, f);
            j = m.dof_parent[j];
        }
    }
    // ---------------- LTDL factorisation (in place) ----------------
    for (int k = nv - 1; k >= 0; --k) {
        const float dkk = w[m.o_M + k * nv + k];
        int a_ = m.dof_parent[k];
        while (a_ >= 0) {
            const float a = w[m.o_M + k * nv + a_] / dkk;
            int j = a_;
            while (j >= 0) {
                w[m.o_M + a_ * nv + j] -= a * w[m.o_M + k * nv + j];
                j = m.dof_parent[j];
            }
            w[m.o_M + k * nv + a_] = a;
            a_ = m.dof_parent[a_];
        }
    }
    ltdl_solve(m, w, m.o_r);
    for (int k = 0; k < nv; ++k) w[m.o_u + k] = w[m.o_u + k] + dt * w[m.o_r + k];

    // ---------------- constraint rows ----------------
    int nrows = 0, ncon = 0;
    for (int c = 0; c < m.npts; ++c) {
        const int g = m.pt_geom[c], l = m.geom_link[g];
        const float* pl = m.pt_end[c] ? m.geom_p1 + 3 * g : m.geom_p0 + 3 * g;
        float R[9], x[3];
#pragma unroll
        for (int q = 0; q < 9; ++q) R[q] = w[m.o_R + 9 * l + q];
        m3_vec(R, pl, x);
#pragma unroll
        for (int q = 0; q < 3; ++q) x[q] += w[m.o_o + 3 * l + q];
        const float r = m.geom_radius[g];
        const float gap = rp[2] + x[2] - r;
        if (!(gap < p.contact_offset)) continue;
        const float pc[3] = {x[0], x[1], x[2] - r};
        const float d = gap - p.rest_offset;
        const float bn = p.tgs ? d : row_bias(p, d, dt, true);   // TGS: the row keeps its separation
#pragma unroll
        for (int q = 0; q < 3; ++q) w[m.o_cp + 3 * ncon + q] = pc[q];
        w[m.o_cl + ncon] = (float)l;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const float dir[3] = {t == 1 ? 1.0f : 0.0f, t == 2 ? 1.0f : 0.0f, t == 0 ? 1.0f : 0.0f};
            float f[6];
            cross3(pc, dir, f);
            f[3] = dir[0]; f[4] = dir[1]; f[5] = dir[2];
            make_row(m, w, nrows, l, f);
            w[m.o_rk + nrows] = (float)t;
            w[m.o_b + nrows] = t == 0 ? bn : 0.0f;
            ++nrows;
        }
        ++ncon;
    }
    for (int j = 0; j < D; ++j) {
        const int l = j + 1, k = nr + j;
        const float lo = m.lower[l], hi = m.upper[l];
        if (!(lo < hi)) continue;
        const float qj = st.q[sx(st, j, i)];
        const float qp = qj + dt * w[m.o_u + k];
        float d, sg;
        if (qj < lo || qp < lo) { d = qj - lo; sg = 1.0f; }
        else if (qj > hi || qp > hi) { d = hi - qj; sg = -1.0f; }
        else continue;
        const int ro = m.o_Jr + nrows * nv;
        for (int q = 0; q < nv; ++q) w[ro + q] = 0.0f;
        w[ro + k] = sg;
        w[m.o_b + nrows] = p.tgs ? d : row_bias(p, d, dt, true);
        w[m.o_rk + nrows] = 3.0f;
        ++nrows;
    }
    for (int r = 0; r < nrows; ++r) {
        const int ro = m.o_Jr + r * nv, wo = m.o_W + r * nv;
        for (int q = 0; q < nv; ++q) w[wo + q] = w[ro + q];
        ltdl_solve(m, w, wo);
        float a = 0.0f;
        for (int q = 0; q < nv; ++q) a += w[ro + q] * w[wo + q];
        w[m.o_Ad + r] = a > 1e-12f ? a : 1e-12f;
        w[m.o_lam + r] = 0.0f;
    }
    // ---------------- projected Gauss-Seidel ----------------
    const float mu = p.friction;
    // TGS (include/mi_sim.h): o_b holds the row's separation, o_ds its change over the sub-steps
    // so far, o_r (the solved rhs, dead here) the running sum of the sub-steps' velocities
    for (int r = 0; r < nrows; ++r) w[m.o_ds + r] = 0.0f;
    for (int q = 0; q < nv; ++q) w[m.o_r + q] = 0.0f;
    for (int it = 0; it < p.iters + p.viters; ++it) {
        for (int r = 0; r < nrows; ++r) {
            const int ro = m.o_Jr + r * nv, wo = m.o_W + r * nv;
            float jv = 0.0f;
            for (int q = 0; q < nv; ++q) jv += w[ro + q] * w[m.o_u + q];
            const float l0 = w[m.o_lam + r];
            const int kd = (int)w[m.o_rk + r];
            const float br = !p.tgs ? w[m.o_b + r]
                             : (kd == 1 || kd == 2) ? 0.0f
                             : row_bias(p, w[m.o_b + r] + w[m.o_ds + r], p.h, it < p.iters);
            float ln = l0 + (br - jv) / w[m.o_Ad + r];
            const int kind = (int)w[m.o_rk + r];
            if (kind == 1 || kind == 2) {
                const float lim = mu * w[m.o_lam + r - kind];
                ln = ln > lim ? lim : (ln < -lim ? -lim : ln);
            } else {
                ln = ln > 0.0f ? ln : 0.0f;
            }
            const float dl = ln - l0;
            for (int q = 0; q < nv; ++q) w[m.o_u + q] += w[wo + q] * dl;
            w[m.o_lam + r] = ln;
        }
        if (p.tgs && it < p.iters) {   // the sub-step moves the rows by h J u, the positions by h u
            for (int r = 0; r < nrows; ++r) {
                const int ro = m.o_Jr + r * nv;
                float jv = 0.0f;
                for (int q = 0; q < nv; ++q) jv += w[ro + q] * w[m.o_u + q];
                w[m.o_ds + r] += p.h * jv;
            }
            for (int q = 0; q < nv; ++q) w[m.o_r + q] += w[m.o_u + q];
        }
    }
    if (p.tgs)   // the positions' velocity: the sub-steps' mean
        for (int q = 0; q < nv; ++q) w[m.o_r + q] = w[m.o_r + q] / (float)p.iters;
    const int o_up = p.tgs ? m.o_r : m.o_u;
    // ---------------- force sensors ----------------
    for (int si = 0; si < m.S; ++si) {
        const int l = m.sensor_link[si];
        float R[9], xs[3], F[3] = {0, 0, 0}, T[3] = {0, 0, 0};
#pragma unroll
        for (int q = 0; q < 9; ++q) R[q] = w[m.o_R + 9 * l + q];
        m3_vec(R, m.sensor_pos + 3 * si, xs);
#pragma unroll
        for (int q = 0; q < 3; ++q) xs[q] += w[m.o_o + 3 * l + q];
        for (int c = 0; c < ncon; ++c) {
            if ((int)w[m.o_cl + c] != l) continue;
            const float fn = w[m.o_lam + 3 * c] / dt, f1 = w[m.o_lam + 3 * c + 1] / dt,
                        f2 = w[m.o_lam + 3 * c + 2] / dt;
            const float fc[3] = {f1, f2, fn};
            float rr[3], tc[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) rr[q] = w[m.o_cp + 3 * c + q] - xs[q];
            cross3(rr, fc, tc);
#pragma unroll
            for (int q = 0; q < 3; ++q) { F[q] += fc[q]; T[q] += tc[q]; }
        }
        float Fl[3], Tl[3];
        m3_tvec(R, F, Fl);
        m3_tvec(R, T, Tl);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            st.sens[ssx(st, 6 * si + q, i)] = Fl[q];
            st.sens[ssx(st, 6 * si + 3 + q, i)] = Tl[q];
        }
    }
    // ---------------- integrate ----------------
    bool finite = true;
    if (nr) {
        float u[6], up[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) { u[k] = w[m.o_u + k]; up[k] = w[o_up + k]; }
        if (p.tgs) {   // the velocity state's angular velocity cap
            const float wv = sqrtf(dot3(u + 3, u + 3));
            if (wv > p.max_angvel) {
                const float sc = p.max_angvel / wv;
                u[3] *= sc; u[4] *= sc; u[5] *= sc;
            }
        }
        float* om = up + 3;
        float wn = sqrtf(dot3(om, om));
        if (wn > p.max_angvel) {
            const float sc = p.max_angvel / wn;
            om[0] *= sc; om[1] *= sc; om[2] *= sc;
            wn = p.max_angvel;
        }
        if (!p.tgs)
#pragma unroll
            for (int k = 0; k < 6; ++k) u[k] = up[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) rp[k] += dt * up[k];
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
        for (int k = 0; k < 3; ++k) { st.root_pos[sx(st, k, i)] = rp[k]; finite &= isfinite(rp[k]); }
#pragma unroll
        for (int k = 0; k < 4; ++k) { st.root_quat[sx(st, k, i)] = rq[k]; finite &= isfinite(rq[k]); }
#pragma unroll
        for (int k = 0; k < 6; ++k) { st.root_vel[sx(st, k, i)] = u[k]; finite &= isfinite(u[k]); }
    }
    for (int j = 0; j < D; ++j) {
        const float v = w[m.o_u + nr + j];
        const float qn = st.q[sx(st, j, i)] + dt * w[o_up + nr + j];
        st.qd[sx(st, j, i)] = v;
        st.q[sx(st, j, i)] = qn;
        finite &= isfinite(v) && isfinite(qn);
    }
    if (!finite) st.nan_flag[i] = 1;
}

}  // namespace mi
