/* mi_geom.h — contact geometry shared, as source, by the HIP kernels and the CPU oracle.
 *
 * Header-only and plain C: hipcc compiles it into the device path, gcc into oracle/ (test
 * infrastructure). Both see the same operation order with FP contraction off, so the contact
 * decisions of device and oracle agree to rounding of their (separately computed) inputs.
 *
 * Self-collision (Humanoid.yaml:80 enable_self_collisions): capsule / sphere pairs as segments
 * with radii (a sphere is a segment of length 0). The contact normal points from geom B to
 * geom A, the contact point is midway between the two surfaces, and the friction directions
 * come from mi_contact_basis (ground contacts keep +x / +y).
 */
#ifndef MI_GEOM_H
#define MI_GEOM_H

#include <math.h>

#if defined(__HIPCC__)
#define MI_GEOM_FN static inline __host__ __device__
#else
#define MI_GEOM_FN static inline
#endif

#if defined(__clang__)
#define MI_GEOM_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define MI_GEOM_NO_CONTRACT
#endif

MI_GEOM_FN float mi_g_clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

/* closest points ca on [a0, a1] and cb on [b0, b1] (segments may be points) */
MI_GEOM_FN void mi_segment_closest(const float* a0, const float* a1, const float* b0,
                                   const float* b1, float* ca, float* cb) {
    MI_GEOM_NO_CONTRACT
    float d1[3], d2[3], r[3];
    for (int k = 0; k < 3; ++k) { d1[k] = a1[k] - a0[k]; d2[k] = b1[k] - b0[k]; r[k] = a0[k] - b0[k]; }
    const float a = d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2];
    const float e = d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2];
    const float f = d2[0] * r[0] + d2[1] * r[1] + d2[2] * r[2];
    float s = 0.0f, t = 0.0f;
    if (a <= 1e-12f && e <= 1e-12f) {
        s = 0.0f; t = 0.0f;
    } else if (a <= 1e-12f) {
        s = 0.0f; t = mi_g_clamp01(f / e);
    } else {
        const float c = d1[0] * r[0] + d1[1] * r[1] + d1[2] * r[2];
        if (e <= 1e-12f) {
            t = 0.0f; s = mi_g_clamp01(-c / a);
        } else {
            const float b = d1[0] * d2[0] + d1[1] * d2[1] + d1[2] * d2[2];
            const float den = a * e - b * b;
            s = den > 1e-12f ? mi_g_clamp01((b * f - c * e) / den) : 0.0f;
            t = (b * s + f) / e;
            if (t < 0.0f) { t = 0.0f; s = mi_g_clamp01(-c / a); }
            else if (t > 1.0f) { t = 1.0f; s = mi_g_clamp01((b - c) / a); }
        }
    }
    for (int k = 0; k < 3; ++k) { ca[k] = a0[k] + d1[k] * s; cb[k] = b0[k] + d2[k] * t; }
}

/* orthonormal friction directions t1, t2 for a unit normal n */
MI_GEOM_FN void mi_contact_basis(const float* n, float* t1, float* t2) {
    MI_GEOM_NO_CONTRACT
    const float ax[3] = {n[0] < 0.57735f && n[0] > -0.57735f ? 1.0f : 0.0f,
                         n[0] < 0.57735f && n[0] > -0.57735f ? 0.0f : 1.0f, 0.0f};
    float c[3] = {n[1] * ax[2] - n[2] * ax[1], n[2] * ax[0] - n[0] * ax[2], n[0] * ax[1] - n[1] * ax[0]};
    const float cl = sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    for (int k = 0; k < 3; ++k) t1[k] = c[k] / cl;
    t2[0] = n[1] * t1[2] - n[2] * t1[1];
    t2[1] = n[2] * t1[0] - n[0] * t1[2];
    t2[2] = n[0] * t1[1] - n[1] * t1[0];
}

/* Pair test. Returns the surface gap (negative = penetration); writes the contact point pc
 * (midway between the surfaces) and the unit normal n from B to A. */
MI_GEOM_FN float mi_pair_contact(const float* a0, const float* a1, float ra, const float* b0,
                                 const float* b1, float rb, float* pc, float* n) {
    MI_GEOM_NO_CONTRACT
    float ca[3], cb[3];
    mi_segment_closest(a0, a1, b0, b1, ca, cb);
    float d[3] = {ca[0] - cb[0], ca[1] - cb[1], ca[2] - cb[2]};
    const float dist = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (dist > 1e-9f) {
        for (int k = 0; k < 3; ++k) n[k] = d[k] / dist;
    } else {
        n[0] = 0.0f; n[1] = 0.0f; n[2] = 1.0f;
    }
    const float gap = dist - ra - rb;
    for (int k = 0; k < 3; ++k) pc[k] = cb[k] + n[k] * (rb + 0.5f * gap);
    return gap;
}

#endif /* MI_GEOM_H */
