/*
 * ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product library.
 *
 * Restatement of glibc 2.35's x86_64 `sinf`/`cosf` (FMA ifunc variant, the one
 * selected on every AVX2+FMA host), which is what the reference's descriptor
 * calls: `float a = (float)cos(angle), b = (float)sin(angle);` with float
 * overloads via `using namespace std`
 * (/root/reference/ORB-SLAM2注释版/src/ORBextractor.cpp:69,117-118).
 *
 * Algorithm = the published ARM optimized-routines sincosf (glibc
 * sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c):
 * |x| < pi/4 -> direct polynomial; |x| < 120 -> x - n*pi/2 with n from a
 * 2^24-scaled 2/pi; polynomials evaluated in double with FMA exactly where the
 * FMA build contracts them. Inputs >= 120 are never produced by the extractor
 * (angle in [0,360) degrees * pi/180 < 2*pi) and are rejected here.
 * Parity with the host libm is checked exhaustively over [0, 2*pi] by
 * tests/test_sincosf.py (the "N3" check of SURVEY.md §8a).
 */
#ifndef ORB_ORACLE_SINCOSF_GLIBC_H
#define ORB_ORACLE_SINCOSF_GLIBC_H
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
} oracle_sincos_t;

static const oracle_sincos_t oracle_sincosf_table[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     0x1p0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
     0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     -0x1p0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
     -0x1.99343027bf8c3p-16},
};

static inline uint32_t oracle_abstop12(float x) {
    uint32_t u; memcpy(&u, &x, 4); return (u >> 20) & 0x7ff;
}

/* sin polynomial on a reduced argument (x already multiplied by sign[n&3]) */
static inline float oracle_sinf_poly(double x, double x2, const oracle_sincos_t* p) {
    double x3 = x * x2;
    double s1 = fma(x2, p->s3, p->s2);
    double x5 = x2 * x3;
    double s = fma(x3, p->s1, x);
    return (float)fma(s1, x5, s);
}
static inline float oracle_cosf_poly(double x2, const oracle_sincos_t* p) {
    double x4 = x2 * x2;
    double c1 = fma(x2, p->c1, p->c0);
    double c2 = fma(x2, p->c4, p->c3);
    double x6 = x2 * x4;
    double c = fma(x4, p->c2, c1);
    return (float)fma(c2, x6, c);
}

/* returns 0 on success, -1 for |y| >= 120 or non-finite (not reachable) */
static inline int oracle_sincosf_glibc(float y, float* s_out, float* c_out) {
    const oracle_sincos_t* p = &oracle_sincosf_table[0];
    double x = (double)y;
    uint32_t top = oracle_abstop12(y);
    if (top < 0x3f4) {                 /* |y| < pi/4 */
        double x2 = x * x;
        if (top < 0x398) {             /* |y| < 2^-12 */
            *s_out = y; *c_out = 1.0f; return 0;
        }
        *s_out = oracle_sinf_poly(x, x2, p);
        *c_out = oracle_cosf_poly(x2, p);
        return 0;
    }
    if (top < 0x42f) {                 /* |y| < 120 */
        double r = x * p->hpi_inv;
        int32_t n = (((int32_t)r) + 0x800000) >> 24;
        double xr = fma(-(double)n, p->hpi, x);
        double x2 = xr * xr;
        const oracle_sincos_t* q = (n & 2) ? &oracle_sincosf_table[1] : p;
        double xs = xr * p->sign[n & 3];
        if ((n & 1) == 0) {
            *s_out = oracle_sinf_poly(xs, x2, q);
            *c_out = oracle_cosf_poly(x2, q);
        } else {
            *s_out = oracle_cosf_poly(x2, q);
            *c_out = oracle_sinf_poly(xs, x2, q);
        }
        return 0;
    }
    return -1;
}
#endif
