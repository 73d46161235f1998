/* Exhaustive-ish check of the division the traversal kernel uses in the sphere test (render.hip div_rn):
 *     q0 = x*y;  q1 = fma(fma(-a, q0, x), y, q0);  q = fma(fma(-a, q1, x), y, q1)     with y = RN(1/a)
 * against the IEEE quotient x/a.  Markstein's theorem makes the last step correctly rounded once q1 is
 * within one ulp; this program checks it bit for bit wherever the quotient is a normal float and
 * |x| >= 2^-100 (the residual cannot underflow), and checks that the sphere test's acceptance
 * kTmin < t < t_best is unchanged for every input (smaller x give quotients < 2^-60: rejected either way).
 *   gcc -O2 -ffp-contract=off -fopenmp tools/check_fastdiv.c -o /tmp/check_fastdiv -lm && /tmp/check_fastdiv 1e9
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static inline float div_rn(float x, float a, float y) {
    const float q0 = x * y;
    const float q1 = fmaf(fmaf(-a, q0, x), y, q0);
    return fmaf(fmaf(-a, q1, x), y, q1);
}

static inline uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* a: positive, exponent within [-40, 40] (the kernel's per-ray guard); x: any sign, exponent in [-140, 127] */
static inline float rand_a(uint64_t r) { return u2f((uint32_t)((127 - 40 + (int)((r >> 23) % 81)) << 23) | (uint32_t)(r & 0x7fffff)); }
static inline float rand_x(uint64_t r) {
    const uint32_t e = (uint32_t)((r >> 24) % 255);  /* 0 = zero/subnormal, 254 = up to FLT_MAX */
    return u2f(((uint32_t)(r >> 40) & 1u) << 31 | e << 23 | (uint32_t)(r & 0x7fffff));
}

int main(int argc, char** argv) {
    const double n = argc > 1 ? atof(argv[1]) : 1e8;
    const long long N = (long long)n;
    long long bad = 0, normal = 0;
    const float kTmin = 0.001f;
#pragma omp parallel for reduction(+ : bad, normal) schedule(static)
    for (long long i = 0; i < N; i++) {
        uint64_t s = (uint64_t)i * 0x2545f4914f6cdd1dull + 12345u;
        const uint64_t r1 = splitmix(&s), r2 = splitmix(&s), r3 = splitmix(&s);
        const float a = rand_a(r1);
        /* mix fully random x with quotients that land near round-to-nearest ties */
        float x = rand_x(r2);
        if ((r3 & 3u) == 0) x = a * u2f((uint32_t)(r3 >> 8) & 0x7fffffffu);
        const float y = 1.0f / a;
        const float e = x / a, f = div_rn(x, a, y);
        /* bit-exact wherever the residual fma(-a, q, x) cannot underflow (|x| >= 2^-100) */
        if (isnormal(e) && fabsf(x) >= 0x1p-100f) {
            normal++;
            if (f2u(e) != f2u(f)) bad++;
        }
        /* below that every quotient is < 2^-60, so both are rejected by t > kTmin; check acceptance for all */
        const float tb = u2f((uint32_t)(r3 >> 32) & 0x7f7fffffu);  /* finite positive t_best */
        const int acc_e = e > kTmin && e < tb, acc_f = f > kTmin && f < tb;
        if (acc_e != acc_f || (acc_e && f2u(e) != f2u(f))) bad++;
    }
    printf("cases %lld, bit-compared quotients %lld, mismatches %lld\n", N, normal, bad);
    return bad != 0;
}
