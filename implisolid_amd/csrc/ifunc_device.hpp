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
__device__ __forceinline__ V3 cube_g(float i1, float i2, float i3) {
    const float P[18] = {0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f};
    int index = 0;
    float mn = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double v = (double)((i1 - 0.f - P[3 * k]) * P[3 * k]) * (-2.) +
                         (double)((i2 - 0.f - P[3 * k + 1]) * P[3 * k + 1]) * (-2.) +
                         (double)((i3 - 0.f - P[3 * k + 2]) * P[3 * k + 2]) * (-2.);
        if (k == 0) mn = (float)v;
        if (v < (double)mn) { index = k; mn = (float)v; }
    }
    return V3{-P[index * 3], -P[index * 3 + 1], -P[index * 3 + 2]};
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
__device__ __forceinline__ float dm_f(float x, float y, float z) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = a * a, c2 = c * c;
    if (z > r) return r - z;
    if (z < -r) return r + z;
    const double v = sq_exact(x - 0.f) / (double)a2 + sq_exact(y - 0.f) / (double)b2 - sq_exact(z - 0.f) / (double)c2 - 1;
    return (float)(-v);
}
__device__ __forceinline__ V3 dm_g(float x, float y, float z) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = a * a, c2 = c * c;   // a = b (object_factory.hpp:89)
    if (z < -r) return V3{0.f, 0.f, 1.f};
    if (z > r) return V3{0.f, 0.f, -1.f};
    return V3{-2.f * (x - 0.f) / a2, -2.f * (y - 0.f) / b2, 2.f * (z - 0.f) / c2};
}

__device__ __forceinline__ float prim_f(int t, const float* __restrict__ tab, float x, float y, float z) {
    switch (t) {
        case NT_ELLIPSOID: return egg_f(x, y, z);
        case NT_CUBE: return cube_f(tab, x, y, z);
        case NT_CYLINDER: return cyl_f(x, y, z);
        case NT_CONE: return cone_f(x, y, z);
        case NT_HEART: return heart_f(x, y, z);
        case NT_TORUS: return torus_f(x, y, z);
        default: return dm_f(x, y, z);
    }
}
__device__ __forceinline__ V3 prim_g(int t, float x, float y, float z) {
    switch (t) {
        case NT_ELLIPSOID: return egg_g(x, y, z);
        case NT_CUBE: return cube_g(x, y, z);
        case NT_CYLINDER: return cyl_g(x, y, z);
        case NT_CONE: return cone_g(x, y, z);
        case NT_HEART: return heart_g(x, y, z);
        case NT_TORUS: return torus_g(x, y, z);
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
            vf[vp++] = prim_f(I.type, tab, px[sp], py[sp], pz[sp]);
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
            const float f = prim_f(I.type, tab, px[sp], py[sp], pz[sp]);
            V3 g = prim_g(I.type, px[sp], py[sp], pz[sp]);
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
