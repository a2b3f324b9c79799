/* CPU check of the slab kernels' quotient (engine.hip div_rc): with y = RN(1/b),
 * q0 = RN(a*y), r = fma(-b, q0, a), q = fma(r, y, q0) must equal the IEEE
 * quotient RN(a/b) for operands in {0} U [2^-59, 2^60) and divisors in
 * [2^-60, 2^60] (the ranges the kernels keep to; others take IEEE division).
 * Usage: div_rc_check N [seed]  -> prints mismatches, exit 1 if any.
 *        div_rc_check exhaustive    -> every numerator for the default config's divisors.
 *
 * Exhaustive mode.  The sequence is exactly scale invariant in the normal range
 * (scaling a or b by 2^k scales y, q0, r and q by powers of two exactly, and the
 * kernels keep every intermediate normal), so its result for a numerator depends
 * only on the numerator's 23-bit mantissa and sign (symmetric).  Checking all
 * 2^23 mantissas against each divisor mantissa therefore covers every f32
 * numerator in range.  The divisors the slab kernels pass to div_rc are, per
 * level h (engine.hip run_level, LevelGeo): r_h, r_h * S3, -r_h * S3 (hex.rs:69-70),
 * the grandchild cell size 1000 / 2^(h+2), the grandchild radius r_{h+2}
 * (metadata.rs:91-97, cell.rs:276-278) and 3 (hex.rs:76-78).  All levels'
 * divisors are power-of-two scalings of those of level 0 (cell_size halves
 * exactly), so five mantissas cover every level of the default config. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 88172645463325252ull;
static uint64_t rnd(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
}
static float u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static float div_rc(float a, float b, float y) {
    volatile float q0 = a * y; /* rounded product, never contracted */
    const float r = fmaf(-b, q0, a);
    return fmaf(r, y, q0);
}

static int exhaustive(void) {
    const float S3 = 1.73205080757f;                               /* hex.rs:3 */
    const float cr = (1000.0f / 96.0f) / 2.0f;                     /* metadata.rs:96, cell.rs:277 */
    const float div[5] = {cr, cr * S3, (-cr) * S3, 1000.0f, 3.0f};
    long bad = 0;
    for (int d = 0; d < 5; d++) {
        const float b = div[d], y = 1.0f / b;
        for (uint32_t m = 0; m < (1u << 23); m++) {
            const float a = u2f((127u << 23) | m);               /* [1, 2) */
            const float q = div_rc(a, b, y), e = a / b;
            if (memcmp(&q, &e, 4) != 0) {
                if (bad < 5) printf("mismatch a=%a b=%a q=%a ieee=%a\n", a, b, q, e);
                bad++;
            }
        }
        printf("divisor %a: %u numerator mantissas checked\n", b, 1u << 23);
    }
    printf("div_rc_check exhaustive mismatches=%ld\n", bad);
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "exhaustive") == 0) return exhaustive();
    const long n = argc > 1 ? atol(argv[1]) : 10000000;
    if (argc > 2) st ^= (uint64_t)atoll(argv[2]) * 0x9E3779B97F4A7C15ull;
    long bad = 0;
    for (long t = 0; t < n; t++) {
        const uint32_t eb = (uint32_t)(127 - 60 + (rnd() % 121)); /* divisor exponent in [-60, 60] */
        float b = u2f((eb << 23) | (uint32_t)(rnd() & 0x7FFFFF));
        if (rnd() & 1) b = -b;
        float a;
        switch (t % 4) {
            case 0: { /* operand exponent in [-59, 59] */
                const uint32_t ea = (uint32_t)(127 - 59 + (rnd() % 119));
                a = u2f((ea << 23) | (uint32_t)(rnd() & 0x7FFFFF));
                break;
            }
            case 1: /* coordinates on a millimetre grid */
                a = ((float)(int32_t)(rnd() % 4000001) - 2000000.0f) * 0.001f;
                break;
            case 2: /* a near an integer multiple of b: quotients near integers */
                a = (float)((int32_t)(rnd() % 20001) - 10000) * b;
                break;
            default: /* the hex sums divided by 3 */
                b = 3.0f;
                a = (float)((int32_t)(rnd() % 2001) - 1000) + u2f((uint32_t)(127 - 24 + (rnd() % 24)) << 23);
                break;
        }
        if (rnd() & 1) a = -a;
        const float y = 1.0f / b;
        const float q = div_rc(a, b, y), e = a / b;
        if (memcmp(&q, &e, 4) != 0 && !(q == 0.0f && e == 0.0f)) {
            if (bad < 5) printf("mismatch a=%a b=%a q=%a ieee=%a\n", a, b, q, e);
            bad++;
        }
    }
    printf("div_rc_check n=%ld mismatches=%ld\n", n, bad);
    return bad ? 1 : 0;
}
