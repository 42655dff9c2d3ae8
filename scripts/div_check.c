/* div_check.c — host check of a reciprocal division tried in round 5 for
 * the step kernels (measured slower on gfx950, not shipped):
 * q = RN(a y) with y = RN(1/b), then
 * RN(q + (a - b q) y), taken only for a, b, q in the safe exponent range
 * (a zero dividend: q itself), must equal a / b bit for bit.  Random pairs
 * over narrow and wide exponent ranges, divisors of all-ones / all-zeros
 * significands, signed zeros; fp64 and fp32.
 *
 *   gcc -O2 -mfma -ffp-contract=off -o /tmp/div_check scripts/div_check.c -lm
 *   /tmp/div_check [pairs per precision = 4e8]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static inline uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

static inline double rd(int emin, int emax) {
    uint64_t bits = ((uint64_t)(emin + (int)(rnd() % (uint64_t)(emax - emin + 1)) + 1023) << 52) |
                    (rnd() & ((1ull << 52) - 1));
    if (rnd() & 1) bits |= 1ull << 63;
    double d; memcpy(&d, &bits, 8); return d;
}
static inline float rf(int emin, int emax) {
    uint32_t bits = ((uint32_t)(emin + (int)(rnd() % (uint64_t)(emax - emin + 1)) + 127) << 23) |
                    (uint32_t)(rnd() & ((1u << 23) - 1));
    if (rnd() & 1) bits |= 1u << 31;
    float d; memcpy(&d, &bits, 4); return d;
}
static inline int safe_d(double a) { double x = fabs(a); return x >= 0x1p-900 && x <= 0x1p900; }
static inline int safe_f(float a) { float x = fabsf(a); return x >= 0x1p-100f && x <= 0x1p100f; }

static inline double div_d(double a, double b, double y, int *fast) {
    const double q = a * y;
    const int ok = safe_d(b) && (a == 0 || (safe_d(a) && safe_d(q)));
    *fast = ok;
    return ok ? (a == 0 ? q : fma(fma(-b, q, a), y, q)) : a / b;
}
static inline float div_f(float a, float b, float y, int *fast) {
    const float q = a * y;
    const int ok = safe_f(b) && (a == 0 || (safe_f(a) && safe_f(q)));
    *fast = ok;
    return ok ? (a == 0 ? q : fmaf(fmaf(-b, q, a), y, q)) : a / b;
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 400000000;
    long bad = 0, fast = 0;
    for (long i = 0; i < n; ++i) {
        double a, b;
        switch (i % 4) {
        case 0: a = rd(-60, 60); b = rd(-60, 60); if ((i & 255) == 0) a = (rnd() & 1) ? 0.0 : -0.0; break;
        case 1: a = rd(-1000, 1000); b = rd(-1000, 1000); break;
        case 2: a = rd(-20, 20); b = fabs(rd(-2, 2)); break;
        default: {
            a = rd(-30, 30); b = rd(-10, 10);
            uint64_t bb; memcpy(&bb, &b, 8);
            const uint64_t k = rnd() % 3, ones = (1ull << 52) - 1;
            bb = k == 0 ? (bb | ones) : k == 1 ? (bb & ~ones) : (bb | (ones - rnd() % 64));
            memcpy(&b, &bb, 8);
        }
        }
        volatile double y = 1.0 / b;
        int f;
        const double q1 = div_d(a, b, y, &f), q0 = a / b;
        fast += f;
        if (memcmp(&q0, &q1, 8)) { if (bad < 10) printf("fp64 mismatch a=%a b=%a: %a vs %a\n", a, b, q0, q1); ++bad; }
    }
    printf("fp64: %ld pairs, %ld on the fast path, %ld mismatches\n", n, fast, bad);
    long badf = 0; fast = 0;
    for (long i = 0; i < n; ++i) {
        float a, b;
        switch (i % 4) {
        case 0: a = rf(-30, 30); b = rf(-30, 30); if ((i & 255) == 0) a = (rnd() & 1) ? 0.0f : -0.0f; break;
        case 1: a = rf(-126, 127); b = rf(-126, 127); break;
        case 2: a = rf(-20, 20); b = fabsf(rf(-2, 2)); break;
        default: {
            a = rf(-30, 30); b = rf(-10, 10);
            uint32_t bb; memcpy(&bb, &b, 4);
            const uint32_t k = rnd() % 3, ones = (1u << 23) - 1;
            bb = k == 0 ? (bb | ones) : k == 1 ? (bb & ~ones) : (bb | (ones - (uint32_t)(rnd() % 64)));
            memcpy(&b, &bb, 4);
        }
        }
        volatile float y = 1.0f / b;
        int f;
        const float q1 = div_f(a, b, y, &f), q0 = a / b;
        fast += f;
        if (memcmp(&q0, &q1, 4)) { if (badf < 10) printf("fp32 mismatch a=%a b=%a: %a vs %a\n", a, b, q0, q1); ++badf; }
    }
    printf("fp32: %ld pairs, %ld on the fast path, %ld mismatches\n", n, fast, badf);
    return bad || badf;
}
