/* mi_dr.h — observation / action noise domain randomization, shared as source by the HIP
 * kernels and the CPU oracle (like mi_geom.h: plain C, FP contraction off).
 *
 * Restates the noise half of the reference's Randomizer
 * (utils/domain_randomization/randomize.py:212-306, applied from envs/vec_env_rlgames.py:59-60,70-71):
 *
 *   apply_X_randomization(buf, reset_buf):
 *     counter[reset] = 0; counter += 1                                       (:215-216, :240-241)
 *     on_reset:    corr[reset] = draw();  buf = buf (+|*) corr               (:218-226, :286-306)
 *     on_interval: ids = counter >= frequency_interval; counter[ids] = 0;
 *                  buf[ids] = buf[ids] (+|*) draw()                          (:228-236, :269-284)
 *
 * MI355X-first storage: the correlated-noise buffer [N, C] of the reference is NOT stored. A
 * draw is a pure function of (seed, stream, global env id, key, column) through the build's
 * Philox4x32-10, so the correlated noise of an env is recomputed from its per-env "epoch" (the
 * number of on_reset redraws so far; epoch 0 = the reference's zero-initialised buffer,
 * randomize.py:192,209) and an uncorrelated draw is keyed on the per-env interval-draw count.
 * Per env and buffer the state is 3 uint32 (counter, epoch, draws) instead of C floats.
 *
 * Distributions (randomize.py:270-275 / 290-296): gaussian|normal N(p0, p1) by Box-Muller on
 * two uniforms; uniform (p1 - p0) * u + p0; loguniform exp((ln p1 - ln p0) * u + ln p0).
 * RNG streams differ from torch's (statistically equivalent), like the reset noise.
 */
#ifndef MI_DR_H
#define MI_DR_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MI_DR_FN static inline __host__ __device__
#else
#define MI_DR_FN static inline
#endif

#if defined(__clang__)
#define MI_DR_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define MI_DR_NO_CONTRACT
#endif

/* Philox stream ids of the four schedules (0: reset noise, 1: random-policy actions) */
#define MI_DR_STREAM_OBS_RESET 2u
#define MI_DR_STREAM_OBS_INTERVAL 3u
#define MI_DR_STREAM_ACT_RESET 4u
#define MI_DR_STREAM_ACT_INTERVAL 5u

/* One noise value from the four uniforms of Philox block (column >> 1); column parity picks
 * the pair. Uniforms are the 24-bit grid k / 2^24 in [0, 1). */
MI_DR_FN float mi_dr_value(int32_t distribution, float p0, float p1, const float u[4], int column) {
    MI_DR_NO_CONTRACT
    const float ua = u[2 * (column & 1)], ub = u[2 * (column & 1) + 1];
    if (distribution == 0) {                       /* gaussian / normal */
        const float r = sqrtf(-2.0f * logf(1.0f - ua));
        return p0 + p1 * (r * cosf(6.283185307179586f * ub));
    }
    if (distribution == 1) return (p1 - p0) * ua + p0;   /* uniform */
    {                                                  /* loguniform */
        const float l0 = logf(p0), l1 = logf(p1);
        return expf((l1 - l0) * ua + l0);
    }
}

MI_DR_FN float mi_dr_op(int32_t operation, float x, float noise) {
    MI_DR_NO_CONTRACT
    return operation == 0 ? x + noise : x * noise;
}

/* Per-env schedule decision for one apply call (wave-uniform on the device). */
typedef struct mi_dr_env {
    uint32_t counter, epoch, draws;
    int fire;        /* on_interval noise applies this call */
} mi_dr_env;

MI_DR_FN mi_dr_env mi_dr_begin(uint32_t counter, uint32_t epoch, uint32_t draws, int reset,
                               int on_reset, int on_interval, int frequency_interval) {
    mi_dr_env e;
    e.counter = (reset ? 0u : counter) + 1u;
    e.epoch = epoch + ((on_reset && reset) ? 1u : 0u);
    e.draws = draws;
    e.fire = 0;
    if (on_interval && (int64_t)e.counter >= (int64_t)frequency_interval) {
        e.counter = 0u;
        e.draws = draws + 1u;
        e.fire = 1;
    }
    return e;
}

#endif /* MI_DR_H */
