/* Exhaustive check of div_by_0p02 (omniisaacgymenvs_amd/csrc/mi_task.hpp) against the IEEE
 * quotient x / 0.02f over all 2^32 float bit patterns (NaN payloads compared as "both NaN").
 * Same operation sequence as the device helper: q = x * 50, q = fma(fma(-q, 0.02, x), 50, q),
 * the division itself outside 2^-90 <= |x| <= 2^100. Prints the mismatch count. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float div_by_0p02(float x) {
    const float ax = fabsf(x);
    float q = x * 50.0f;
    q = fmaf(fmaf(-q, 0.02f, x), 50.0f, q);
    if (!(ax >= 0x1p-90f && ax <= 0x1p100f)) q = x / 0.02f;
    return q;
}

int main(void) {
    volatile float d = 0.02f;
    uint64_t bad = 0, fast = 0;
    for (uint64_t u = 0; u < (1ull << 32); ++u) {
        const uint32_t b = (uint32_t)u;
        float x;
        memcpy(&x, &b, 4);
        const float a = x / d, f = div_by_0p02(x);
        uint32_t ba, bf;
        memcpy(&ba, &a, 4);
        memcpy(&bf, &f, 4);
        const float ax = fabsf(x);
        fast += ax >= 0x1p-90f && ax <= 0x1p100f;
        if (ba != bf && !(isnan(a) && isnan(f))) ++bad;
    }
    printf("mismatches %llu fast-path inputs %llu\n", (unsigned long long)bad,
           (unsigned long long)fast);
    return bad != 0;
}
