/*
 * or_libm.c -- glibc 2.35 float math restated for the screw family (TEST INFRASTRUCTURE ONLY).
 *
 *   sinf    sysdeps/ieee754/flt-32/s_sinf.c + sincosf.h, x86_64 FMA variant (s_sinf-fma.c: the
 *           multiarch selection on every FMA-capable host): double polynomial and the fast
 *           reduction contracted to fma.  Table constants read from this image's libm
 *           (__sincosf_table, __inv_pio4).  screw.hpp:29-36 std::sin(float).
 *   atanf   sysdeps/ieee754/flt-32/s_atanf.c (fdlibm)
 *   atan2f  sysdeps/ieee754/flt-32/e_atan2f.c (fdlibm); screw.hpp:136 std::atan2(float, float)
 *
 * or_libm_check() compares each with the host libm: sinf and atanf over any range of bit patterns
 * (exhaustively: 0 mismatches over all 2^32), atan2f over seeded random pairs.
 */
#include "oracle.h"

#include <math.h>
#include <string.h>

static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ---- sinf ---- */
static const double SC_SIGN[4] = {1.0, -1.0, -1.0, 1.0};
static const double SC_HPI_INV = 0x1.45f306dc9c883p+23, SC_HPI = 0x1.921fb54442d18p+0;
static const double SC_C0 = 0x1p0, SC_C1 = -0x1.ffffffd0c621cp-2, SC_C2 = 0x1.55553e1068f19p-5,
                    SC_C3 = -0x1.6c087e89a359dp-10, SC_C4 = 0x1.99343027bf8c3p-16;
static const double SC_S1 = -0x1.555545995a603p-3, SC_S2 = 0x1.1107605230bc4p-7, SC_S3 = -0x1.994eb3774cf24p-13;
static const uint32_t INV_PIO4[24] = {
    0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

static inline uint32_t abstop12(float f) { return (fbits(f) >> 20) & 0x7ff; }

/* sinf_poly; table 1 (n & 2) is table 0 with every cosine coefficient negated */
static inline float sinf_poly(double x, double x2, int n, int neg) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = fma(x2, SC_S3, SC_S2);
        const double x7 = x3 * x2;
        const double s = fma(x3, SC_S1, x);
        return (float)fma(x7, s1, s);
    }
    const double k = neg ? -1.0 : 1.0;
    const double x4 = x2 * x2;
    const double c2 = fma(x2, k * SC_C4, k * SC_C3);
    const double c1 = fma(x2, k * SC_C1, k * SC_C0);
    const double x6 = x4 * x2;
    const double c = fma(x4, k * SC_C2, c1);
    return (float)fma(x6, c2, c);
}

static inline double sinf_reduce_large(uint32_t xi, int* np) {
    const uint32_t* arr = &INV_PIO4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = xi * arr[0];
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * 0x1.921fb54442d18p-62;
}

float or_sinf(float y) {
    double x = y;
    int n;
    const uint32_t top = abstop12(y);
    if (top < abstop12(0x1.921fb6p-1f)) {
        if (top < abstop12(0x1p-12f)) return y;
        return sinf_poly(x, x * x, 0, 0);
    } else if (top < abstop12(120.0f)) {
        const double r = x * SC_HPI_INV;
        n = ((int32_t)r + 0x800000) >> 24;
        x = fma(-(double)n, SC_HPI, x);
        const double s = SC_SIGN[n & 3];
        return sinf_poly(x * s, x * x, n, n & 2);
    } else if (top < abstop12(INFINITY)) {
        const uint32_t xi = fbits(y);
        const int sign = xi >> 31;
        x = sinf_reduce_large(xi, &n);
        const double s = SC_SIGN[(n + sign) & 3];
        return sinf_poly(x * s, x * x, n, (n + sign) & 2);
    }
    return (y - y) / (y - y);
}

/* ---- atanf / atan2f (fdlibm) ---- */
static const float AT_HI[] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
static const float AT_LO[] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
static const float AT_T[] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                             9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                             4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};

float or_atanf(float x) {
    float w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)fbits(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {                    /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? AT_HI[3] + AT_LO[3] : -AT_HI[3] - AT_LO[3];
    }
    if (ix < 0x3ee00000) {                     /* |x| < 0.4375 */
        if (ix < 0x31000000) return x;         /* |x| < 2^-29 */
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (AT_T[0] + w * (AT_T[2] + w * (AT_T[4] + w * (AT_T[6] + w * (AT_T[8] + w * AT_T[10])))));
    s2 = w * (AT_T[1] + w * (AT_T[3] + w * (AT_T[5] + w * (AT_T[7] + w * AT_T[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = AT_HI[id] - ((x * (s1 + s2) - AT_LO[id]) - x);
    return hx < 0 ? -z : z;
}

float or_atan2f(float y, float x) {
    static const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                       pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    float z;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return or_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = or_atanf(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return bitsf(fbits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

/* ---- cos (double) ----
   sysdeps/ieee754/dbl-64/s_sin.c __cos, the x86_64 FMA variant (s_sin-fma.c, selected on every
   FMA- and AVX2-capable host): the branches and contractions as this image's libm compiles them
   (read from its __cos_fma).  screw.hpp:178-180 cos(M_PI * (...)): the screw gradient.  The
   __branred branch (high word >= 0x419921fb: |x| >= 105414336) is not restated: it calls the host cos. */
#include "../implisolid_amd/csrc/generated/sincostab.h"
static const uint64_t SINCOSTAB[440] = {IMPLI_SINCOSTAB_BITS};
static inline double bitsd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint64_t dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
#define CS_BIG 0x1.8p45
#define CS_T(i) bitsd(SINCOSTAB[(i)])

static double cs_taylor_sin(double a, double da) {   /* TAYLOR_SIN (s_sin.c) */
    const double xx = a * a;
    const double p = fma(xx, fma(xx, fma(xx, fma(xx, bitsd(0xbe5addffc2fcdf59ull), bitsd(0x3ec71de27b9a7ed9ull)),
                                         bitsd(0xbf2a01a019db08b8ull)), bitsd(0x3f81111111110eceull)),
                         bitsd(0xbfc5555555555555ull));
    const double t = fma(xx, fma(p, a, -(da * 0.5)), da);
    return a + t;
}
static double cs_do_cos(double x, double dx) {       /* do_cos */
    if (x < 0) dx = -dx;
    const double ax = fabs(x), u = ax + CS_BIG;
    const int k = (int)((uint32_t)dbits(u) << 2);
    const double xr = (ax - (u - CS_BIG)) + dx, xx = xr * xr;
    const double s = fma(xr * xx, fma(xx, bitsd(0x3f811110e829872full), bitsd(0xbfc5555555555515ull)), xr);
    const double c = xx * fma(xx, fma(xx, bitsd(0x3f56c16bedd9e239ull), bitsd(0xbfa5555555555535ull)), 0.5);
    double cor = fma(-s, CS_T(k + 1), CS_T(k + 3));
    cor = fma(-c, CS_T(k + 2), cor);
    cor = fma(-s, CS_T(k), cor);
    return CS_T(k + 2) + cor;
}
static double cs_do_sin(double x, double dx) {       /* do_sin */
    if (fabs(x) < 0.126) return cs_taylor_sin(x, dx);
    if (x <= 0) dx = -dx;
    const double ax = fabs(x), u = ax + CS_BIG;
    const int k = (int)((uint32_t)dbits(u) << 2);
    const double xr = ax - (u - CS_BIG), xx = xr * xr;
    const double s = xr + fma(xr * xx, fma(xx, bitsd(0x3f811110e829872full), bitsd(0xbfc5555555555515ull)), dx);
    const double c = fma(xr, dx, xx * fma(xx, fma(xx, bitsd(0x3f56c16bedd9e239ull), bitsd(0xbfa5555555555535ull)), 0.5));
    double cor = fma(s, CS_T(k + 3), CS_T(k + 1));
    cor = fma(-c, CS_T(k), cor);
    cor = fma(s, CS_T(k + 2), cor);
    return copysign(CS_T(k) + cor, x);
}
double or_cos(double x) {
    const uint32_t k = (uint32_t)(dbits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e400000u) return 1.0;                           /* |x| < 2^-27 */
    if (k < 0x3feb6000u) return cs_do_cos(x, 0.0);             /* |x| < 0.855469 */
    if (k < 0x400368fdu) {                                     /* |x| < 2.426265 */
        const double y = bitsd(0x3ff921fb54442d18ull) - fabs(x);
        const double a = y + bitsd(0x3c91a62633145c07ull);
        const double da = (y - a) + bitsd(0x3c91a62633145c07ull);
        return cs_do_sin(a, da);
    }
    if (k < 0x419921fbu) {                                     /* |x| < 105414336: reduce_sincos */
        const double t = fma(x, bitsd(0x3fe45f306dc9c883ull), 0x1.8p52);
        const double xn = t - 0x1.8p52;
        const int n = (int)(dbits(t) & 3u);
        const double y = fma(-xn, bitsd(0xbe4dde973c000000ull), fma(-xn, bitsd(0x3ff921fb58000000ull), x));
        const double pp3 = bitsd(0xbc8cb3b398000000ull), pp4 = bitsd(0xbacd747f23e32ed7ull);
        const double t2 = fma(-xn, pp3, y);
        double db = fma(-pp3, xn, y - t2);
        const double b = fma(-xn, pp4, t2);
        db = db + fma(-xn, pp4, t2 - b);
        const double r = ((n + 1) & 1) ? cs_do_cos(b, db) : cs_do_sin(b, db);
        return ((n + 1) & 2) ? -r : r;
    }
    if (k < 0x7ff00000u) return cos(x);                        /* __branred: not restated */
    return x / x;
}

/* or_cos against the host cos: `count` seeded arguments (start = seed) from four distributions --
   uniform in [-lim, lim], uniform bit patterns of |x| < 2^27, and around the branch boundaries and
   multiples of pi/2; returns the mismatches */
int64_t or_cos_check(uint64_t start, uint64_t count, double lim) {
    int64_t bad = 0;
    uint64_t s = 0x9E3779B97F4A7C15ull * (start + 1);
    static const double edges[] = {0x1p-27, 0.85546875, 2.426265, 1.5707963267948966, 3.141592653589793,
                                   4.71238898038469, 6.283185307179586, 105414350.0};
    for (uint64_t i = 0; i < count; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        double x;
        switch (i & 3) {
            case 0: x = ((double)(s >> 11) * 0x1p-53 * 2.0 - 1.0) * lim; break;
            case 1: x = bitsd((s & 0x800fffffffffffffull) | ((uint64_t)(0x3c0 + (s >> 52) % 0x5a) << 52)); break;
            case 2: { const double e = edges[(s >> 40) % 8]; x = bitsd(dbits(e) + (int64_t)((s & 0xfffff) - 0x80000)); break; }
            default: x = (double)((int64_t)(s >> 40) - (1ll << 23)) * 1.5707963267948966 + ((double)(s & 0xffff) - 32768.0) * 0x1p-40;
        }
        const double a = or_cos(x), b = cos(x);
        if (!(dbits(a) == dbits(b) || (a != a && b != b))) bad++;
    }
    return bad;
}

/* the restated (glibc = 0) or host (glibc = 1) cos on an array: the GPU test's checker for the
   device restatement (implisolid_debug_cos) */
void or_cos_apply(const double* a, int64_t n, double* out, int glibc) {
    for (int64_t i = 0; i < n; i++) out[i] = glibc ? cos(a[i]) : or_cos(a[i]);
}

/* mismatching results vs the host libm.  which: 0 sinf, 1 atanf over start + k*stride (count
   patterns); 2 atan2f over `count` seeded pairs (start = seed) drawn from four distributions */
int64_t or_libm_check(int which, uint32_t start, uint32_t stride, uint64_t count) {
    int64_t bad = 0;
    if (which <= 1) {
        uint32_t u = start;
        for (uint64_t k = 0; k < count; k++, u += stride) {
            const float x = bitsf(u);
            const float a = which == 0 ? or_sinf(x) : or_atanf(x), b = which == 0 ? sinf(x) : atanf(x);
            if (!(fbits(a) == fbits(b) || (a != a && b != b))) bad++;
        }
        return bad;
    }
    uint64_t s = 0x9E3779B97F4A7C15ull * ((uint64_t)start + 1);
    for (uint64_t i = 0; i < count; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        float y, x;
        switch (i & 3) {
            case 0: y = bitsf((uint32_t)s); x = bitsf((uint32_t)(s >> 32)); break;
            case 1: y = (float)(int32_t)(uint32_t)s * 0x1p-30f; x = (float)(int32_t)(uint32_t)(s >> 32) * 0x1p-30f; break;
            case 2: y = (float)(int32_t)(uint32_t)s * 0x1p-50f; x = (float)(int32_t)(uint32_t)(s >> 32) * 0x1p-31f; break;
            default: {
                const uint32_t e1 = (s >> 40) & 63, e2 = (s >> 46) & 63;
                y = bitsf(((uint32_t)s & 0x807fffffu) | ((100 + e1) << 23));
                x = bitsf(((uint32_t)(s >> 20) & 0x807fffffu) | ((100 + e2) << 23));
            }
        }
        const float a = or_atan2f(y, x), b = atan2f(y, x);
        if (!(fbits(a) == fbits(b) || (a != a && b != b))) bad++;
    }
    return bad;
}

/* the restated functions on arrays (which as above; b only for atan2f): the GPU test's checker
   for the device restatement (implisolid_debug_libm) */
void or_libm_apply(int which, const float* a, const float* b, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++)
        out[i] = which == 0 ? or_sinf(a[i]) : which == 1 ? or_atanf(a[i]) : or_atan2f(a[i], b[i]);
}
