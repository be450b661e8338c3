// ifunc_device.hpp -- implicit-function primitives and the node-program interpreter (device).
//
// Every primitive reproduces the reference's float/double expression order operation for
// operation (the whole library is compiled with -ffp-contract=off, so no FMA fusion; HIP's default
// f32 division and sqrt are correctly rounded, like the CPU's).  Library calls are restated:
//   std::pow(float, int 2)   -> exact double square                  (torus, double mushroom)
//   std::pow(double, 0.5)    -> correctly rounded sqrt               (torus)
//   std::pow(double, 2)      -> correctly rounded product            (torus, heart gradient)
//   std::pow(double, 3)      -> correctly rounded cube (double-double) (heart)
// glibc's pow is correctly rounded outside hard cases, so these agree with the reference
// except on inputs whose result lies within ~2^-60 ulp of a rounding boundary.
#pragma once
#ifndef __HIPCC_RTC__   // hipRTC (jit.cpp) provides these through its prelude
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "generated/tables.h"
#include "generated/sincostab.h"
#include "program.hpp"

namespace impli {
namespace dev {

struct V3 { float x, y, z; };

__device__ __forceinline__ float bits2f(uint32_t u) { return __uint_as_float(u); }

// std::min(a, b) == (b < a) ? b : a
__device__ __forceinline__ float stdmin(float a, float b) { return (b < a) ? b : a; }

__device__ __forceinline__ double sq_exact(float v) { const double d = (double)v; return d * d; }

// correctly rounded d^3 (two-product + error compensation; exact to ~2^-104 relative)
__device__ __forceinline__ double cube_cr(double d) {
    const double p = d * d;
    const double pe = __fma_rn(d, d, -p);
    const double c = p * d;
    const double ce = __fma_rn(p, d, -c);
    return c + (ce + pe * d);
}

// matrix_vector_product (basic_functions.hpp:140-177), left to right
__device__ __forceinline__ V3 xform(const float* __restrict__ m, float x, float y, float z) {
    V3 r;
    r.x = m[0] * x + m[1] * y + m[2] * z + m[3];
    r.y = m[4] * x + m[5] * y + m[6] * z + m[7];
    r.z = m[8] * x + m[9] * y + m[10] * z + m[11];
    return r;
}
// an XF_DIAG matrix's rows at a finite point (program.hpp XformPattern): m_dd v + m_d3
__device__ __forceinline__ V3 xform_diag(const float* __restrict__ m, float x, float y, float z) {
    V3 r;
    r.x = m[0] * x + m[3];
    r.y = m[5] * y + m[7];
    r.z = m[10] * z + m[11];
    return r;
}
// gradient post-transform inv^T * g (e.g. transformed_union.hpp:76-83)
__device__ __forceinline__ V3 grad_xform(const float* __restrict__ m, V3 g) {
    V3 r;
    r.x = m[0] * g.x + m[4] * g.y + m[8] * g.z;
    r.y = m[1] * g.x + m[5] * g.y + m[9] * g.z;
    r.z = m[2] * g.x + m[6] * g.y + m[10] * g.z;
    return r;
}

// ---- egg (iellipsoid), egg.hpp:93-128, a=b=c=0.5 ------------------------------------------
__device__ __forceinline__ float egg_f(float x, float y, float z) {
    const float u = (x - 0.f) / 0.5f, v = (y - 0.f) / 0.5f, w = (z - 0.f) / 0.5f;
    return 1.f - (u * u + v * v + w * w);
}
__device__ __forceinline__ V3 egg_g(float x, float y, float z) {
    const double a2 = (double)(0.5f * 0.5f);
    return V3{(float)(-2. * (double)(x - 0.f) / a2), (float)(-2. * (double)(y - 0.f) / a2),
              (float)(-2. * (double)(z - 0.f) / a2)};
}

// ---- cube = rabbit SDF table, cube.hpp:176-272 ----------------------------------------------
// The table (+ the object's trailing members and zero padding for out-of-table reads, F8d)
// is passed as a device pointer; RABBIT_PAD entries are readable.
constexpr int kRabbitN = IMPLI_RABBIT_NX * IMPLI_RABBIT_NY * IMPLI_RABBIT_NZ;
// readable entries: the point function reads up to 23 + 19*22 + 23*396 = 9549; the interval
// bound's 2x2x2 blocks (ifunc_interval.hpp cube_iv) start at <= 9549 and read 419 further
constexpr int kRabbitPadded = 10240;
// after the table: float2 {min, max} over the eight reads b + {0,1} + {0,sx} + {0,sx*sy} of every
// flat index b (cube_iv's O(1) range lookups)
constexpr int kRabbitBlockMinMax = kRabbitPadded;

__device__ __forceinline__ float cube_f(const float* __restrict__ tab, float X, float Y, float Z) {
    const int sx = IMPLI_RABBIT_NX, sy = IMPLI_RABBIT_NY, sz = IMPLI_RABBIT_NZ;
    const float gs = bits2f(IMPLI_RABBIT_GRID_SIZE_BITS);
    const float ox = bits2f(IMPLI_RABBIT_ORIGIN_X_BITS), oy = bits2f(IMPLI_RABBIT_ORIGIN_Y_BITS),
                oz = bits2f(IMPLI_RABBIT_ORIGIN_Z_BITS);
    float res = 10000.f;
    const bool out = (ox + gs * (float)sx < X || X < ox) || (oy + gs * (float)sy < Y || Y < oy) ||
                     (oz + gs * (float)sz < Z || Z < oz);
    if (!out) {
        const int xg = (int)((X - ox) / gs), yg = (int)((Y - oy) / gs), zg = (int)((Z - oz) / gs);
        const float xl = ox + (float)xg * gs, yl = oy + (float)yg * gs, zl = oz + (float)zg * gs;
        const float xd = (X - xl) / gs, yd = (Y - yl) / gs, zd = (Z - zl) / gs;
        const int b = xg + yg * sx + zg * sx * sy;
        const float r000 = tab[b], r100 = tab[b + 1], r010 = tab[b + sx], r110 = tab[b + 1 + sx];
        const float r001 = tab[b + sx * sy], r101 = tab[b + 1 + sx * sy], r011 = tab[b + sx + sx * sy],
                    r111 = tab[b + 1 + sx + sx * sy];
        const float c00 = r000 * (1.f - xd) + r100 * xd;
        const float c01 = r001 * (1.f - xd) + r101 * xd;
        const float c10 = r010 * (1.f - xd) + r110 * xd;
        const float c11 = r011 * (1.f - xd) + r111 * xd;
        const float c0 = c00 * (1.f - yd) + c10 * yd;
        const float c1 = c01 * (1.f - yd) + c11 * yd;
        res = c0 * (1.f - zd) + c1 * zd;
    }
    return -res;
}
// cube.hpp:273-315 -- the old six-plane gradient (does not match the rabbit field, F3)
// The chosen face's normal is carried through the unrolled loop (constant indices only): indexing
// the table with the winning face made it a private array, which the compiler kept in registers in
// some processes and in LDS or scratch in others for the same source (18 KB of LDS per workgroup:
// the f + gradient passes 3-5x slower).
__device__ __forceinline__ V3 cube_g(float i1, float i2, float i3) {
    const float P[18] = {0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f};
    float mn = 0.f, gx = -P[0], gy = -P[1], gz = -P[2];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double v = (double)((i1 - 0.f - P[3 * k]) * P[3 * k]) * (-2.) +
                         (double)((i2 - 0.f - P[3 * k + 1]) * P[3 * k + 1]) * (-2.) +
                         (double)((i3 - 0.f - P[3 * k + 2]) * P[3 * k + 2]) * (-2.);
        if (k == 0) mn = (float)v;
        if (v < (double)mn) {
            mn = (float)v;
            gx = -P[3 * k];
            gy = -P[3 * k + 1];
            gz = -P[3 * k + 2];
        }
    }
    return V3{gx, gy, gz};
}

// ---- scylinder, scylinder.hpp:97-166 (radius .5, length 1, centre (0,0,-.5), axis z) ---------
__device__ __forceinline__ void cyl_parts(float i0, float i1, float i2, float& t0, float& t1, float& r_) {
    const float w0 = 0.f, w1 = 0.f, w2 = 1.f, X = 0.f, Y = 0.f, Zc = -0.5f;
    t0 = (i0 - X) * w0 + (i1 - Y) * w1 + (i2 - Zc) * w2;
    t1 = 1.f - t0;
    const float a = i0 - w0 * t0 - X, b = i1 - w1 * t0 - Y, c = i2 - w2 * t0 - Zc;
    r_ = 0.5f - sqrtf(a * a + b * b + c * c);
}
__device__ __forceinline__ float cyl_f(float x, float y, float z) {
    float t0, t1, r_;
    cyl_parts(x, y, z, t0, t1, r_);
    return stdmin(t0, stdmin(t1, r_));
}
__device__ __forceinline__ V3 cyl_g(float i0, float i1, float i2) {
    const float w0 = 0.f, w1 = 0.f, w2 = 1.f, X = 0.f, Y = 0.f, Zc = -0.5f;
    float t0, t1, r_;
    cyl_parts(i0, i1, i2, t0, t1, r_);
    const float c0 = (t0 <= t1 && t0 <= r_) ? 1.f : 0.f;
    const float c1 = (t1 <= t0 && t1 <= r_) ? 1.f : 0.f;
    const float cr = (r_ <= t0 && r_ <= t1) ? 1.f : 0.f;
    return V3{c0 * w0 + c1 * (-w0) + cr * (w0 * t0 + X - i0), c0 * w1 + c1 * (-w1) + cr * (w1 * t0 + Y - i1),
              c0 * w2 + c1 * (-w2) + cr * (w2 * t0 + Zc - i2)};
}

// ---- scone, scone.hpp:81-151 (h 1, r1 0, r2 .5, centre (0,0,.5)) ----------------------------
__device__ __forceinline__ float cone_f(float x, float y, float z) {
    const float q = 0.5f / 1.f, a2 = q * q, z0 = 0.5f;
    const float f = -sqrtf((x - 0.f) * (x - 0.f) + (y - 0.f) * (y - 0.f)) + sqrtf((z - z0) * (z - z0) * a2);
    const float up = -(z - z0) - 0.f, lo = (z - z0) + 1.f;
    return stdmin(f, stdmin(up, lo));
}
__device__ __forceinline__ V3 cone_g(float x, float y, float z) {
    const float q = 0.5f / 1.f, a2 = q * q, z0 = 0.5f;
    const float f = -(x - 0.f) * (x - 0.f) / a2 - (y - 0.f) * (y - 0.f) / a2 + (z - z0) * (z - z0);
    const float up = -(z - z0) - 0.f, lo = (z - z0) + 1.f;
    if (up < f && up < lo) return V3{0.f, 0.f, -1.f};
    if (lo < f && lo < up) return V3{0.f, 0.f, 1.f};
    return V3{-2.f * (x - 0.f) / a2, -2.f * (y - 0.f) / a2, 2.f * (z - z0)};
}

// ---- heart, heart.hpp:82-132 ------------------------------------------------------------------
__device__ __forceinline__ double heart_T(float i1, float i2, float i3) {
    return (double)(i1 * i1) + (9. / 4.) * (double)i2 * (double)i2 + (double)(i3 * i3) - 1.;
}
__device__ __forceinline__ float heart_f(float i1, float i2, float i3) {
    const double t3 = cube_cr(heart_T(i1, i2, i3));
    const float a = i1 * i1 * i3 * i3 * i3;
    const double b = (9. / 200.) * (double)i2 * (double)i2 * (double)i3 * (double)i3 * (double)i3;
    return (float)(-(t3 - (double)a - b));
}
__device__ __forceinline__ V3 heart_g(float i1, float i2, float i3) {
    const double T = heart_T(i1, i2, i3);
    const float a = (float)(T * T);
    const double d1 = i1, d2 = i2, d3 = i3, da = a;
    return V3{(float)(-6. * d1 * da + 2. * d1 * d3 * d3 * d3),
              (float)(-(27. / 2) * d2 * da + (9. / 100.) * d2 * d3 * d3 * d3),
              (float)(-6. * d3 * da + 3. * d1 * d1 * d3 * d3 + (27. / 200.) * d2 * d2 * d3 * d3)};
}

// ---- torus, torus.hpp:68-124 (r 4, rx=ry=rz=.2) ---------------------------------------------
__device__ __forceinline__ float torus_f(float x, float y, float z) {
    const float r = 4.f, rx = 0.2f, ry = 0.2f, rz = 0.2f;
    const double s = sq_exact(x / rx) + sq_exact(y / ry);
    const double q = (double)r - sqrt(s);
    return (float)(1. - q * q - sq_exact(z / rz));
}
__device__ __forceinline__ V3 torus_g(float x, float y, float z) {
    const float r = 4.f, rx = 0.2f, ry = 0.2f, rz = 0.2f;
    const float s = x * x / (rx * rx) + y * y / (ry * ry);
    const float a = (float)sqrt((double)s);
    return V3{(2.f * x / (rx * rx * a)) * (r - a), (2.f * y / (ry * ry * a)) * (r - a), -2.f * z / (rz * rz)};
}

// ---- double mushroom via linearly_transformed, object_factory.hpp:86-100,
//      double_mushroom.hpp:90-160 with (0.9, 0.4/2, 0.4/2, 1/0.2) -------------------------------
// a / D for the double square a of a float and a constant D, by one correction step from
// R = RN(1/D): q0 = a R, q = q0 + (a - q0 D) R with both steps fused (q0 when not finite).  Equal to
// the IEEE quotient for all 2^32 floats at the constant dm_f uses (tools/divconst_check.c, run by
// test_divconst_identity_exhaustive); three f64 ops instead of the division's scale / reciprocal /
// refinement / fixup sequence.
__device__ __forceinline__ double div_sq_const(double a, double D, double R) {
    const double q0 = a * R;
    return __builtin_isfinite(q0) ? __fma_rn(__fma_rn(-q0, D, a), R, q0) : q0;
}
__device__ __forceinline__ float dm_f(float x, float y, float z) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = a * a, c2 = c * c;
    // a2 == b2 == c2 (object_factory.hpp:86-100): one constant, one reciprocal
    const double D = (double)a2, R = 1.0 / (double)a2;
    static_assert(0.2f * 0.2f == (float)(0.4 / 2) * (float)(0.4 / 2), "the checked constant");
    // the body is computed for every sample and the caps selected after (no branch): the x and y
    // terms of a brick's two layers are then one computation (JIT pair code)
    const double v = div_sq_const(sq_exact(x - 0.f), D, R) + div_sq_const(sq_exact(y - 0.f), (double)b2, R) -
                     div_sq_const(sq_exact(z - 0.f), (double)c2, R) - 1;
    return z > r ? r - z : z < -r ? r + z : (float)(-v);
}
__device__ __forceinline__ V3 dm_g(float x, float y, float z) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = a * a, c2 = c * c;   // a = b (object_factory.hpp:89)
    if (z < -r) return V3{0.f, 0.f, 1.f};
    if (z > r) return V3{0.f, 0.f, -1.f};
    return V3{-2.f * (x - 0.f) / a2, -2.f * (y - 0.f) / b2, 2.f * (z - 0.f) / c2};
}

// ---- glibc 2.35 float math used by the screw family -----------------------------------------
// sinf: sysdeps/ieee754/flt-32/s_sinf.c + sincosf.h, the x86_64 FMA variant (s_sinf-fma.c, chosen
// on every FMA-capable host): the double polynomial and the fast reduction are fma-contracted.
// atanf / atan2f: fdlibm (s_atanf.c, e_atan2f.c).  All three are checked bit-exact against the
// host libm by the oracle's restatement (or_libm.c; sinf and atanf over all 2^32 patterns).
__device__ __forceinline__ uint32_t abstop12(float f) { return (__float_as_uint(f) >> 20) & 0x7ffu; }

// __inv_pio4: 32-bit windows of 2/pi, in constant memory (a function-local table indexed at run
// time is a private array whose placement -- registers, LDS, scratch -- the compiler chose
// differently from process to process)
static __constant__ uint32_t kInvPio4[24] = {
    0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd,
    0xf534ddc0, 0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43,
    0x993c4390, 0x3c439041};
__device__ __forceinline__ uint32_t inv_pio4(int i) { return kInvPio4[i]; }

// sinf_poly; __sincosf_table[1] (n & 2) is table 0 with the cosine coefficients negated.  The sine
// (n even) and cosine (n odd) polynomials as one chain of the same operations on selected operands:
//   sine   x3 = x x2, x7 = x3 x2:  fma(x7, fma(x2, S3, S2), fma(x3, S1, x))
//   cosine x4 = x2 x2, x6 = x4 x2: fma(x6, fma(x2, C3, C2), fma(x4, C1, fma(x2, C0, 1)))
// (k = -1 negates every cosine coefficient, an exact sign flip) -- lanes of one wave whose n differ
// in parity no longer run both polynomials one after the other
__device__ __forceinline__ float sinf_poly(double x, double x2, int n, bool neg) {
    const bool sn = (n & 1) == 0;
    const double k = neg ? -1.0 : 1.0;
    const double u = sn ? x : x2;
    const double v = u * x2, w = v * x2;                  // x3, x7 | x4, x6
    const double c1 = __fma_rn(x2, k * -0x1.ffffffd0c621cp-2, k * 0x1p0);
    const double base = sn ? x : c1;
    const double mid = __fma_rn(v, sn ? -0x1.555545995a603p-3 : k * 0x1.55553e1068f19p-5, base);
    const double t = __fma_rn(x2, sn ? -0x1.994eb3774cf24p-13 : k * 0x1.99343027bf8c3p-16,
                              sn ? 0x1.1107605230bc4p-7 : k * -0x1.6c087e89a359dp-10);
    return (float)__fma_rn(w, t, mid);
}

__device__ __forceinline__ float glibc_sinf(float y) {
    const uint32_t top = abstop12(y);
    if (top < 0x42fu) {                                   // |y| < 120: reduce_fast
        // (|y| < pi/4 is glibc's unreduced branch: here n = 0, the fma returns x and the sign 1,
        // the same polynomial call; |y| < 2^-12 returns y)
        double x = y;
        const double r = x * 0x1.45f306dc9c883p+23;
        const int n = ((int32_t)r + 0x800000) >> 24;
        x = __fma_rn(-(double)n, 0x1.921fb54442d18p+0, x);
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
        const float p = sinf_poly(x * s, x * x, n, (n & 2) != 0);
        return top < 0x398u ? y : p;
    }
    if (top < 0x7f8u) {                                   // reduce_large
        uint32_t xi = __float_as_uint(y);
        const int sign = (int)(xi >> 31);
        const int idx = (int)((xi >> 26) & 15);
        const int shift = (int)((xi >> 23) & 7);
        xi = (xi & 0xffffffu) | 0x800000u;
        xi <<= shift;
        uint64_t res0 = (uint64_t)(xi * inv_pio4(idx));
        const uint64_t res1 = (uint64_t)xi * inv_pio4(idx + 4);
        const uint64_t res2 = (uint64_t)xi * inv_pio4(idx + 8);
        res0 = (res2 >> 32) | (res0 << 32);
        res0 += res1;
        const uint64_t nn = (res0 + (1ull << 61)) >> 62;
        res0 -= nn << 62;
        const int n = (int)nn;
        const double x = (double)(int64_t)res0 * 0x1.921fb54442d18p-62;
        const int q = (n + sign) & 3;
        const double s = (q == 1 || q == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, n, (q & 2) != 0);
    }
    return (y - y) / (y - y);
}

// fdlibm's four argument reductions select their operands into one division: each lane divides
// exactly the numerator and denominator of its own branch (a wave whose lanes span several ranges
// ran up to four IEEE division sequences)
__device__ __forceinline__ float glibc_atanf(float x) {
    const float hi0 = 4.6364760399e-01f, hi1 = 7.8539812565e-01f, hi2 = 9.8279368877e-01f, hi3 = 1.5707962513e+00f;
    const float lo0 = 5.0121582440e-09f, lo1 = 3.7748947079e-08f, lo2 = 3.4473217170e-08f, lo3 = 7.5497894159e-08f;
    const int32_t hx = (int32_t)__float_as_uint(x), ix = hx & 0x7fffffff;
    const float a = fabsf(x);
    const bool small = ix < 0x3ee00000;                   // id = -1: no reduction
    const int id = ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float num = id == 0 ? 2.0f * a - 1.0f : id == 1 ? a - 1.0f : id == 2 ? a - 1.5f : -1.0f;
    const float den = id == 0 ? 2.0f + a : id == 1 ? a + 1.0f : id == 2 ? 1.0f + 1.5f * a : a;
    const float q = num / den;
    const float t = small ? x : q;
    const float z = t * t, w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    const float h = id == 0 ? hi0 : id == 1 ? hi1 : id == 2 ? hi2 : hi3;
    const float l = id == 0 ? lo0 : id == 1 ? lo1 : id == 2 ? lo2 : lo3;
    const float r = h - ((t * (s1 + s2) - l) - t);
    float res = small ? t - t * (s1 + s2) : (hx < 0 ? -r : r);
    if (ix < 0x31000000) res = x;
    if (ix >= 0x4c000000) res = ix > 0x7f800000 ? x + x : (hx > 0 ? hi3 + lo3 : -hi3 - lo3);
    return res;
}

// e_atan2f.c; x == 1 (atanf(y)) shares the one atanf with the general path (atanf(|y / x|))
__device__ __forceinline__ float glibc_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)__float_as_uint(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)__float_as_uint(y), iy = hy & 0x7fffffff;
    const bool one = hx == 0x3f800000;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const int32_t k = (iy - ix) >> 23;
    const float za = glibc_atanf(one ? y : fabsf(y / x));
    float z = k > 60 ? pi_o_2 + 0.5f * pi_lo : (hx < 0 && k < -60) ? 0.0f : za;
    float res = m == 0 ? z : m == 1 ? __uint_as_float(__float_as_uint(z) ^ 0x80000000u)
                       : m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
    // the special operands, in e_atan2f.c's order
    if (iy == 0x7f800000) res = hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000)
            res = m == 0 ? pi_o_4 + tiny : m == 1 ? -pi_o_4 - tiny : m == 2 ? 3.0f * pi_o_4 + tiny : -3.0f * pi_o_4 - tiny;
        else
            res = m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) res = hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (iy == 0) res = m <= 1 ? y : (m == 2 ? pi + tiny : -pi - tiny);
    if (one) res = za;
    if (ix > 0x7f800000 || iy > 0x7f800000) res = x + y;
    return res;
}

// ---- glibc 2.35 double cos (sysdeps/ieee754/dbl-64/s_sin.c __cos), the x86_64 FMA variant
// (s_sin-fma.c, selected on every FMA- and AVX2-capable host), with the contractions that libm's
// __cos_fma holds: the screw gradient's cos(M_PI * (...)) (screw.hpp:178-180).  oracle/or_libm.c
// or_cos is the same restatement, checked against the host cos (0 mismatches over 2 G seeded
// arguments); the GPU test compares this one with it.  __sincostab (i/128: sin hi, lo, cos hi, lo)
// from the host libm (tools/extract_sincostab.py), in constant memory.  |x| >= 105414336 (glibc's
// __branred: high word >= 0x419921fb) is not restated: the device libm's cos.
static __constant__ uint64_t kSinCosTab[440] = {IMPLI_SINCOSTAB_BITS};
__device__ __forceinline__ double sct(int i) { return __longlong_as_double((long long)kSinCosTab[i]); }
__device__ __forceinline__ double bits2d(uint64_t u) { return __longlong_as_double((long long)u); }
// do_cos / do_sin of (x, dx) (TAYLOR_SIN for do_sin of |x| < 0.126)
__device__ __forceinline__ double glibc_sincos_red(bool is_cos, double x, double dx) {
    const double xx0 = x * x;
    if (!is_cos && fabs(x) < 0.126) {
        const double p = __fma_rn(xx0, __fma_rn(xx0, __fma_rn(xx0, __fma_rn(xx0, bits2d(0xbe5addffc2fcdf59ull),
                                  bits2d(0x3ec71de27b9a7ed9ull)), bits2d(0xbf2a01a019db08b8ull)),
                                  bits2d(0x3f81111111110eceull)), bits2d(0xbfc5555555555555ull));
        return x + __fma_rn(xx0, __fma_rn(p, x, -(dx * 0.5)), dx);
    }
    if (is_cos ? x < 0 : x <= 0) dx = -dx;
    const double big = 0x1.8p45, ax = fabs(x), u = ax + big;
    const int k = (int)((uint32_t)__double_as_longlong(u) << 2);
    const double xr = is_cos ? (ax - (u - big)) + dx : ax - (u - big), xx = xr * xr;
    const double ps = __fma_rn(xx, bits2d(0x3f811110e829872full), bits2d(0xbfc5555555555515ull));
    const double pc = xx * __fma_rn(xx, __fma_rn(xx, bits2d(0x3f56c16bedd9e239ull), bits2d(0xbfa5555555555535ull)), 0.5);
    const double sn = sct(k), ssn = sct(k + 1), cs = sct(k + 2), ccs = sct(k + 3);
    if (is_cos) {
        const double s = __fma_rn(xr * xx, ps, xr);
        double cor = __fma_rn(-s, ssn, ccs);
        cor = __fma_rn(-pc, cs, cor);
        cor = __fma_rn(-s, sn, cor);
        return cs + cor;
    }
    const double s = xr + __fma_rn(xr * xx, ps, dx);
    const double c = __fma_rn(xr, dx, pc);
    double cor = __fma_rn(s, ccs, ssn);
    cor = __fma_rn(-c, sn, cor);
    cor = __fma_rn(s, cs, cor);
    return copysign(sn + cor, x);
}
__device__ __forceinline__ double glibc_cos(double x) {
    const uint32_t k = (uint32_t)((uint64_t)__double_as_longlong(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e400000u) return 1.0;                                   // |x| < 2^-27
    if (k < 0x3feb6000u) return glibc_sincos_red(true, x, 0.0);        // |x| < 0.855469
    if (k < 0x400368fdu) {                                             // |x| < 2.426265
        const double y = bits2d(0x3ff921fb54442d18ull) - fabs(x);
        const double a = y + bits2d(0x3c91a62633145c07ull);
        return glibc_sincos_red(false, a, (y - a) + bits2d(0x3c91a62633145c07ull));
    }
    if (k < 0x419921fbu) {                                             // reduce_sincos
        const double t = __fma_rn(x, bits2d(0x3fe45f306dc9c883ull), 0x1.8p52);
        const double xn = t - 0x1.8p52;
        const int n = (int)((uint64_t)__double_as_longlong(t) & 3u) + 1;
        const double y = __fma_rn(-xn, bits2d(0xbe4dde973c000000ull), __fma_rn(-xn, bits2d(0x3ff921fb58000000ull), x));
        const double pp3 = bits2d(0xbc8cb3b398000000ull), pp4 = bits2d(0xbacd747f23e32ed7ull);
        const double t2 = __fma_rn(-xn, pp3, y);
        const double b = __fma_rn(-xn, pp4, t2);
        const double db = __fma_rn(-pp3, xn, y - t2) + __fma_rn(-xn, pp4, t2 - b);
        const double r = glibc_sincos_red((n & 1) != 0, b, db);
        return (n & 2) ? -r : r;
    }
    if (k < 0x7ff00000u) return cos(x);                                // __branred: not restated
    return x / x;
}

// ---- screw, screw.hpp:98-150 at its constructor's constants (u, v, w = the axes, A = (0,0,-0.5),
//      UVW = I; the factory forces the identity transformation_matrix, object_factory.hpp:304-351).
//      prm = {twist_rate, r0, delta}.  Eigen orders: GEMV t = (x - A) w into a zeroed result; outer
//      product p = w t + A; GEMM ab = UVW^-1 (x - p) accumulated from zero; norm a0 + (a1 + a2).
__device__ __forceinline__ float screw_f(const float* __restrict__ prm, float x, float y, float z) {
    const float tw = prm[0], r0 = prm[1], delta = prm[2];
    const float a0 = x - 0.f, a1 = y - 0.f, a2 = z - (-0.5f);
    const float t = ((0.f + a0 * 0.f) + a1 * 0.f) + a2 * 1.f;
    const float p0 = 0.f * t + 0.f, p1 = 0.f * t + 0.f, p2 = 1.f * t + (-0.5f);
    const float d0 = x - p0, d1 = y - p1, d2 = z - p2;
    const float ab0 = 0.f + (((0.f + 1.f * d0) + 0.f * d1) + 0.f * d2);
    const float ab1 = 0.f + (((0.f + 0.f * d0) + 1.f * d1) + 0.f * d2);
    const float theta = glibc_atan2f(ab1, ab0);
    const float r = sqrtf(d0 * d0 + (d1 * d1 + d2 * d2));
    const float pi = (float)3.1415926535897, pi2 = pi * 2;   // screw.hpp:20, :140
    const float ph = t / tw - theta / pi2;
    return (-r + r0) + delta * glibc_sinf(ph * 2 * pi);       // phi (screw.hpp:29-36)
}
// screw_f at two points (a brick's two layers): the same operations per point, one atan2f when
// both points' (ab1, ab0) agree bit for bit (the screw axis is z: they do whenever the transforms
// above keep x and y independent of z)
__device__ __forceinline__ void screw_f2(const float* __restrict__ prm, float xa, float ya, float za, float xb, float yb,
                                         float zb, float& fa, float& fb) {
    const float tw = prm[0], r0 = prm[1], delta = prm[2];
    const float pi = (float)3.1415926535897, pi2 = pi * 2;
    float t[2], ab0[2], ab1[2], r[2];
    const float X[2] = {xa, xb}, Y[2] = {ya, yb}, Z[2] = {za, zb};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float a0 = X[k] - 0.f, a1 = Y[k] - 0.f, a2 = Z[k] - (-0.5f);
        t[k] = ((0.f + a0 * 0.f) + a1 * 0.f) + a2 * 1.f;
        const float p0 = 0.f * t[k] + 0.f, p1 = 0.f * t[k] + 0.f, p2 = 1.f * t[k] + (-0.5f);
        const float d0 = X[k] - p0, d1 = Y[k] - p1, d2 = Z[k] - p2;
        ab0[k] = 0.f + (((0.f + 1.f * d0) + 0.f * d1) + 0.f * d2);
        ab1[k] = 0.f + (((0.f + 0.f * d0) + 1.f * d1) + 0.f * d2);
        r[k] = sqrtf(d0 * d0 + (d1 * d1 + d2 * d2));
    }
    const float th0 = glibc_atan2f(ab1[0], ab0[0]);
    float th1 = th0;
    if (__float_as_uint(ab0[1]) != __float_as_uint(ab0[0]) || __float_as_uint(ab1[1]) != __float_as_uint(ab1[0]))
        th1 = glibc_atan2f(ab1[1], ab0[1]);
    const float ph0 = t[0] / tw - th0 / pi2, ph1 = t[1] / tw - th1 / pi2;
    fa = (-r[0] + r0) + delta * glibc_sinf(ph0 * 2 * pi);
    fb = (-r[1] + r0) + delta * glibc_sinf(ph1 * 2 * pi);
}
// screw.hpp:152-160 (sympy gradient) at the same constants, with the C++ type of every
// sub-expression: std::pow(float, 2) -> exact double square, atan2(float, float) -> atanf path,
// cos(double) -> glibc's double cos (glibc_cos above), M_PI double.
__device__ __forceinline__ V3 screw_g(const float* __restrict__ prm, float x, float y, float z) {
    const double kPi = 3.14159265358979323846;
    const float tw = prm[0], delta = prm[2];
    const float ax = 0.f, ay = 0.f, az = -0.5f, wx = 0.f, wy = 0.f, wz = 1.f, phi0 = 0.f;
    const float u00 = 1.f, u01 = 0.f, u02 = 0.f, u10 = 0.f, u11 = 1.f, u12 = 0.f;
    const float s = (wx * (-ax + x) + wy * (-ay + y)) + wz * (-az + z);
    const float X1 = (-ax - wx * s) + x, Y1 = (-ay - wy * s) + y, Z1 = (-az - wz * s) + z;
    const float U0 = (u00 * X1 + u01 * Y1) + u02 * Z1;
    const float U1 = (u10 * X1 + u11 * Y1) + u12 * Z1;
    const float nU1 = ((-u10 * X1) - u11 * Y1) - u12 * Z1;
    const double G = sq_exact(U0) + sq_exact(U1);
    const double sq = sqrt((sq_exact(X1) + sq_exact(Y1)) + sq_exact(Z1));
    const float th = glibc_atan2f(U1, U0);
    const double cv = glibc_cos(kPi * (((double)(2 * phi0) - (double)th / kPi) + (double)((2 * s) / tw)));
    const double wx2 = sq_exact(wx), wy2 = sq_exact(wy), wz2 = sq_exact(wz);
    const double pd = kPi * (double)delta;
    const double cAx = ((double)u00 * (-wx2 + 1) - (double)(u01 * wx * wy)) - (double)(u02 * wx * wz);
    const double cBx = ((double)u10 * (-wx2 + 1) - (double)(u11 * wx * wy)) - (double)(u12 * wx * wz);
    const double Ax = -(cAx * (double)nU1 / G + (double)U0 * cBx / G) / kPi + (double)(2 * wx / tw);
    const double Cx = (double)(-wx * wy * Y1 - wx * wz * Z1) + (1.0 / 2.0) * (-2 * wx2 + 2) * (double)X1;
    const double cAy = ((double)(-u10 * wx * wy) + (double)u11 * (-wy2 + 1)) - (double)(u12 * wy * wz);
    const double cBy = ((double)(-u00 * wx * wy) + (double)u01 * (-wy2 + 1)) - (double)(u02 * wy * wz);
    const double Ay = -((double)U0 * cAy / G + (double)nU1 * cBy / G) / kPi + (double)(2 * wy / tw);
    const double Cy = (double)(-wx * wy * X1 - wy * wz * Z1) + (1.0 / 2.0) * (-2 * wy2 + 2) * (double)Y1;
    const double cAz = (double)(-u10 * wx * wz - u11 * wy * wz) + (double)u12 * (-wz2 + 1);
    const double cBz = (double)(-u00 * wx * wz - u01 * wy * wz) + (double)u02 * (-wz2 + 1);
    const double Az = -((double)U0 * cAz / G + (double)nU1 * cBz / G) / kPi + (double)(2 * wz / tw);
    const double Cz = (double)(-wx * wz * X1 - wy * wz * Y1) + (1.0 / 2.0) * (-2 * wz2 + 2) * (double)Z1;
    return V3{(float)(pd * Ax * cv - Cx / sq), (float)(pd * Ay * cv - Cy / sq), (float)(pd * Az * cv - Cz / sq)};
}

// ---- top_bottom_lid.hpp:117-161: std::max(z - 0.5, (z + 0.5) * -1); gradient always (0,0,1)
__device__ __forceinline__ float lid_f(float z) {
    const float a = z - 0.5f, b = (z + 0.5f) * -1.f;
    return (a < b) ? b : a;
}

// ---- inf_top_bot_bound (inf_top_bot_bound.hpp:65-96) over the screw of the same matrix
//      ("screw_gradient_wrong", object_factory.hpp:435-479), at x' = M^-1 x: Eigen's
//      imp.min(tbb * -1) = std::min(screw, -lid); prm = {twist, r0, delta} | (next row) M^-1
__device__ __forceinline__ float tbb_f(const float* __restrict__ prm, float x, float y, float z) {
    return stdmin(screw_f(prm, x, y, z), lid_f(z) * -1.f);
}
__device__ __forceinline__ void tbb_f2(const float* __restrict__ prm, float xa, float ya, float za, float xb, float yb,
                                       float zb, float& fa, float& fb) {
    float sa, sb;
    screw_f2(prm, xa, ya, za, xb, yb, zb, sa, sb);
    fa = stdmin(sa, lid_f(za) * -1.f);
    fb = stdmin(sb, lid_f(zb) * -1.f);
}
// :142-166: the screw's gradient with its own M^-T (screw.hpp:476-486), replaced by (0, 0, -1)
// where z' >= 0.5 and (0, 0, 1) where z' <= -0.5, whichever operand the min chose; the node's
// M^-T is applied after this (the leaf's grad_xform), as the reference applies it again
__device__ __forceinline__ V3 tbb_g(const float* __restrict__ prm, float x, float y, float z) {
    if (z >= 0.5f) return V3{0.f, 0.f, -1.f};
    if (z <= -0.5f) return V3{0.f, 0.f, 1.f};
    return grad_xform(prm + 12, screw_g(prm, x, y, z));
}

// ---- half_plane.hpp:150-190: GEMV (x - plane_point) . plane_vector; prm = {unit pv, pp}
__device__ __forceinline__ float hp_f(const float* __restrict__ prm, float x, float y, float z) {
    const float d0 = x - prm[3], d1 = y - prm[4], d2 = z - prm[5];
    return ((0.f + d0 * prm[0]) + d1 * prm[1]) + d2 * prm[2];
}
__device__ __forceinline__ V3 hp_g(const float* __restrict__ prm, float x, float y, float z) {
    const float k = hp_f(prm, x, y, z) >= 0 ? -1.f : 1.f;
    return V3{k * prm[0], k * prm[1], k * prm[2]};
}

// ---- tetrahedron.hpp:129-178: min of four oriented planes (std::min); gradient of the first
//      minimal plane.  The planes (getPlanes :20-120, corners moved by the node matrix) are host data.
__device__ __forceinline__ float tet_plane(const float* __restrict__ P, int k, float x, float y, float z) {
    return ((P[4 * k] * x + P[4 * k + 1] * y) + P[4 * k + 2] * z) + P[4 * k + 3];
}
__device__ __forceinline__ float tet_f(const float* __restrict__ P, float x, float y, float z) {
    return stdmin(tet_plane(P, 0, x, y, z), stdmin(tet_plane(P, 1, x, y, z), stdmin(tet_plane(P, 2, x, y, z), tet_plane(P, 3, x, y, z))));
}
__device__ __forceinline__ V3 tet_g(const float* __restrict__ P, float x, float y, float z) {
    int index = 0;
    float mn = tet_plane(P, 0, x, y, z);
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        const float v = tet_plane(P, i, x, y, z);
        if (v < mn) { index = i; mn = v; }
    }
    return V3{P[4 * index], P[4 * index + 1], P[4 * index + 2]};
}

// ---- meta_balls_Rydgard.hpp:80-124 (4 balls): sum of (strength / h - subtract) / 100, 1/h a
//      double division stored to float; the gradient's h is summed in double (its 1e-6 literal)
__device__ __forceinline__ float meta_f(const float* __restrict__ P, float x, float y, float z) {
    float out = 0.0f;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float* B = P + 5 * b;
        const float fx = x - B[0], fx2 = fx * fx;
        const float fy = y - B[1], fy2 = fy * fy;
        const float fz = z - B[2], fz2 = fz * fz;
        const float h = (((float)0.000001 + fx2) + fy2) + fz2;
        const float hinv = (float)(1.0 / (double)h);
        const float val = B[3] * hinv - B[4];
        out += val / 100;
    }
    return out;
}
__device__ __forceinline__ V3 meta_g(const float* __restrict__ P, float x, float y, float z) {
    float gx = 0, gy = 0, gz = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float* B = P + 5 * b;
        const float fz = z - B[2], fz2 = fz * fz;
        const float fy = y - B[1], fy2 = fy * fy;
        const float fx = x - B[0], fx2 = fx * fx;
        const float h = (float)(((0.000001 + (double)fx2) + (double)fy2) + (double)fz2);
        const float hinv = (float)(1.0 / (double)h);
        gx += B[3] * (-2 * fx * hinv * hinv) / 100;
        gy += B[3] * (-2 * fy * hinv * hinv) / 100;
        gz += B[3] * (-2 * fz * hinv * hinv) / 100;
    }
    return V3{gx, gy, gz};
}

// ---- extrusion.hpp:103-118 over convex_polygon (2d/GDT/convex_polygon.hpp:97-140): min over edges
//      of -(x nx + y ny - n0), first minimal edge on ties; gradient (-nx, -ny, 0)
__device__ __forceinline__ float extr_eval(const float* __restrict__ P, float x, float y, int& which) {
    const int n = (int)P[0];
    float minv = 0.f;
    int w = -1;
    for (int j = 0; j < n; ++j) {
        const float v = -((x * P[1 + 3 * j] + y * P[2 + 3 * j]) - P[3 + 3 * j]);
        if (v < minv || w < 0) { minv = v; w = j; }
    }
    which = w;
    return minv;
}
__device__ __forceinline__ float extr_f(const float* __restrict__ P, float x, float y) {
    int w;
    return extr_eval(P, x, y, w);
}
__device__ __forceinline__ V3 extr_g(const float* __restrict__ P, float x, float y) {
    int w;
    extr_eval(P, x, y, w);
    return V3{-P[1 + 3 * w], -P[2 + 3 * w], 0.f};
}

__device__ __forceinline__ float prim_f(int t, const float* __restrict__ tab, const float* __restrict__ prm, float x,
                                        float y, float z) {
    switch (t) {
        case NT_ELLIPSOID: return egg_f(x, y, z);
        case NT_CUBE: return cube_f(tab, x, y, z);
        case NT_CYLINDER: return cyl_f(x, y, z);
        case NT_CONE: return cone_f(x, y, z);
        case NT_HEART: return heart_f(x, y, z);
        case NT_TORUS: return torus_f(x, y, z);
        case NT_SCREW: return screw_f(prm, x, y, z);
        case NT_LID: return lid_f(z);
        case NT_HALF_PLANE: return hp_f(prm, x, y, z);
        case NT_TETRA: return tet_f(prm, x, y, z);
        case NT_METABALLS: return meta_f(prm, x, y, z);
        case NT_EXTRUSION: return extr_f(prm, x, y);
        case NT_SCREW_TBB: return tbb_f(prm, x, y, z);
        default: return dm_f(x, y, z);
    }
}
__device__ __forceinline__ V3 prim_g(int t, const float* __restrict__ prm, float x, float y, float z) {
    switch (t) {
        case NT_ELLIPSOID: return egg_g(x, y, z);
        case NT_CUBE: return cube_g(x, y, z);
        case NT_CYLINDER: return cyl_g(x, y, z);
        case NT_CONE: return cone_g(x, y, z);
        case NT_HEART: return heart_g(x, y, z);
        case NT_TORUS: return torus_g(x, y, z);
        case NT_SCREW: return screw_g(prm, x, y, z);
        case NT_LID: return V3{0.f, 0.f, 1.f};
        case NT_HALF_PLANE: return hp_g(prm, x, y, z);
        case NT_TETRA: return tet_g(prm, x, y, z);
        case NT_METABALLS: return meta_g(prm, x, y, z);
        case NT_EXTRUSION: return extr_g(prm, x, y);
        case NT_SCREW_TBB: return tbb_g(prm, x, y, z);
        default: return dm_g(x, y, z);
    }
}

// CSG select, transformed_union.hpp:48 / transformed_intersection.hpp:50 / transformed_subtract.hpp:52
__device__ __forceinline__ bool csg_first(int t, float f1, float f2) {
    return (t == NT_UNION) ? (f1 > f2) : (t == NT_INTERSECTION) ? !(f1 > f2) : (f1 < -f2);
}

// ---- the interpreter -------------------------------------------------------------------------
// prog/mats are wave-uniform (scalar loads).  D = stack capacity chosen at launch from the
// program's depth, so the stacks are small VGPR arrays indexed by uniform counters.
template <int D>
__device__ __forceinline__ float eval_f(const Program* __restrict__ prog, const float* __restrict__ tab, float x,
                                        float y, float z) {
    float px[D], py[D], pz[D], vf[D];
    int sp = 0, vp = 0;
    px[0] = x; py[0] = y; pz[0] = z;
    const int n = prog->n_instr;
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = prog->instr[pc];
        if (I.op == OP_XFORM) {
            const V3 q = xform(prog->mats[I.mat], px[sp], py[sp], pz[sp]);
            ++sp;
            px[sp] = q.x; py[sp] = q.y; pz[sp] = q.z;
        } else if (I.op == OP_PRIM) {
            vf[vp++] = prim_f(I.type, tab, prog->mats[I.prm], px[sp], py[sp], pz[sp]);
            --sp;
        } else {
            --sp;
            const float f2 = vf[--vp];
            const float f1 = vf[vp - 1];
            const float f = (I.type == NT_UNION) ? ((f1 > f2) ? f1 : f2)
                          : (I.type == NT_INTERSECTION) ? ((f1 > f2) ? f2 : f1)
                                                       : ((f1 < -f2) ? f1 : -f2);
            vf[vp - 1] = f;
        }
    }
    return vf[0];
}

// joint (f, grad): every node's gradient is M^-T * (selected child gradient)
template <int D>
__device__ __forceinline__ float eval_fg(const Program* __restrict__ prog, const float* __restrict__ tab, float x,
                                         float y, float z, V3& g_out) {
    float px[D], py[D], pz[D], vf[D], gx[D], gy[D], gz[D];
    int sp = 0, vp = 0;
    px[0] = x; py[0] = y; pz[0] = z;
    const int n = prog->n_instr;
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = prog->instr[pc];
        if (I.op == OP_XFORM) {
            const V3 q = xform(prog->mats[I.mat], px[sp], py[sp], pz[sp]);
            ++sp;
            px[sp] = q.x; py[sp] = q.y; pz[sp] = q.z;
        } else if (I.op == OP_PRIM) {
            const float f = prim_f(I.type, tab, prog->mats[I.prm], px[sp], py[sp], pz[sp]);
            V3 g = prim_g(I.type, prog->mats[I.prm], px[sp], py[sp], pz[sp]);
            g = grad_xform(prog->mats[I.mat], g);
            vf[vp] = f; gx[vp] = g.x; gy[vp] = g.y; gz[vp] = g.z;
            ++vp;
            --sp;
        } else {
            --vp;
            const float f2 = vf[vp], f1 = vf[vp - 1];
            V3 g2{gx[vp], gy[vp], gz[vp]}, g1{gx[vp - 1], gy[vp - 1], gz[vp - 1]};
            if (I.type == NT_DIFFERENCE) { g2.x = -g2.x; g2.y = -g2.y; g2.z = -g2.z; }
            const bool first = csg_first(I.type, f1, f2);
            const float f = (I.type == NT_UNION) ? ((f1 > f2) ? f1 : f2)
                          : (I.type == NT_INTERSECTION) ? ((f1 > f2) ? f2 : f1)
                                                       : ((f1 < -f2) ? f1 : -f2);
            const V3 g = grad_xform(prog->mats[I.mat], first ? g1 : g2);
            vf[vp - 1] = f; gx[vp - 1] = g.x; gy[vp - 1] = g.y; gz[vp - 1] = g.z;
            --sp;
        }
    }
    g_out = V3{gx[0], gy[0], gz[0]};
    return vf[0];
}

}  // namespace dev
}  // namespace impli
