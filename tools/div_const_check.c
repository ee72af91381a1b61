/* Exhaustive CPU check of env_device.h div_const<Y>: for every positive finite fp32 x,
 * q0 = x*RN(1/Y); r = fma(-q0, Y, x); q1 = fma(r, RN(1/Y), q0) against IEEE x/Y (SSE, no FTZ).
 * All operations are sign-symmetric under round-to-nearest, so negative x behave the same.
 * Prints the number of mismatches and the largest mismatching x per divisor (observed: all
 * below 2^-122, i.e. subnormal quotients; the kernels take the IEEE division below 2^-100).
 * Build/run: gcc -O2 -ffp-contract=off -o /tmp/dcc tools/div_const_check.c -lm && /tmp/dcc
 * (about a minute per divisor). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t to_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(void) {
    const float divisors[2] = {400.0f, 600.0f};
    int fail = 0;
    for (int k = 0; k < 2; ++k) {
        volatile float yv = divisors[k];
        const float y = yv, c = 1.0f / y;
        uint64_t bad = 0, bad_above = 0;
        float max_bad = 0.0f;
        for (uint32_t u = 0; u < 0x7F800000u; ++u) {
            const float x = from_bits(u);
            const float q0 = x * c, r = fmaf(-q0, y, x), q1 = fmaf(r, c, q0);
            if (to_bits(q1) != to_bits(x / y)) {
                ++bad;
                if (x > max_bad) max_bad = x;
                if (x >= 0x1p-100f) ++bad_above;
            }
        }
        printf("Y=%g RN(1/Y)=%a mismatches=%llu (largest x %a) mismatches with x>=2^-100: %llu\n",
               y, c, (unsigned long long)bad, max_bad, (unsigned long long)bad_above);
        fail |= bad_above != 0;
    }
    return fail;
}
