// ifunc_interval.hpp -- interval bounds of the node program over a box of sample points (device).
//
// Used to prune CSG operands per brick of samples: if over the whole brick a union/intersection/
// difference provably returns one operand, the per-sample interpreter (eval_f_pruned) skips the
// other operand's subtree.  The per-sample result is then bit-identical to the unpruned one,
// because the skipped select would have returned exactly the kept operand's value.
//
// Soundness: every interval operation below computes its endpoints with the same IEEE operation
// (same precision, round to nearest) that the point evaluator applies, in the same expression
// order.  Rounding to nearest is monotone, and + - x / sqrt are monotone in each argument on the
// box, so the rounded point result lies between the rounded endpoint results.  Primitive outputs
// are additionally widened by a relative 2^-16 margin; non-finite bounds become [-inf, inf]; a
// decision is only taken on strict separation, and NaN never satisfies a comparison.
#pragma once
#include "ifunc_device.hpp"

namespace impli {
namespace dev {

struct Iv { float lo, hi; };
struct IvD { double lo, hi; };

__device__ __forceinline__ Iv ivc(float c) { return Iv{c, c}; }
__device__ __forceinline__ float fmin2(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float fmax2(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ double dmin2(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double dmax2(double a, double b) { return a > b ? a : b; }

__device__ __forceinline__ Iv add(Iv a, Iv b) { return Iv{a.lo + b.lo, a.hi + b.hi}; }
__device__ __forceinline__ Iv sub(Iv a, Iv b) { return Iv{a.lo - b.hi, a.hi - b.lo}; }
__device__ __forceinline__ Iv neg(Iv a) { return Iv{-a.hi, -a.lo}; }
__device__ __forceinline__ Iv mul(Iv a, Iv b) {
    const float p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    return Iv{fmin2(fmin2(p0, p1), fmin2(p2, p3)), fmax2(fmax2(p0, p1), fmax2(p2, p3))};
}
__device__ __forceinline__ Iv mulc(Iv a, float c) {   // a * c
    const float p0 = a.lo * c, p1 = a.hi * c;
    return Iv{fmin2(p0, p1), fmax2(p0, p1)};
}
__device__ __forceinline__ Iv divc(Iv a, float c) {   // a / c, c > 0
    return Iv{a.lo / c, a.hi / c};
}
__device__ __forceinline__ Iv sqr(Iv a) {   // a * a with the same operand
    const float l = a.lo * a.lo, h = a.hi * a.hi;
    if (a.lo >= 0.f) return Iv{l, h};
    if (a.hi <= 0.f) return Iv{h, l};
    return Iv{0.f, fmax2(l, h)};
}
__device__ __forceinline__ Iv sqrt_iv(Iv a) { return Iv{sqrtf(fmax2(a.lo, 0.f)), sqrtf(fmax2(a.hi, 0.f))}; }
__device__ __forceinline__ Iv min_iv(Iv a, Iv b) { return Iv{fmin2(a.lo, b.lo), fmin2(a.hi, b.hi)}; }
__device__ __forceinline__ Iv hull(Iv a, Iv b) { return Iv{fmin2(a.lo, b.lo), fmax2(a.hi, b.hi)}; }
// std::min(a, b) = (b < a) ? b : a  -- as an interval simply the endpoint-wise minimum
__device__ __forceinline__ Iv stdmin_iv(Iv a, Iv b) { return min_iv(a, b); }

__device__ __forceinline__ IvD addd(IvD a, IvD b) { return IvD{a.lo + b.lo, a.hi + b.hi}; }
__device__ __forceinline__ IvD subd(IvD a, IvD b) { return IvD{a.lo - b.hi, a.hi - b.lo}; }
__device__ __forceinline__ IvD muld(IvD a, IvD b) {
    const double p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    return IvD{dmin2(dmin2(p0, p1), dmin2(p2, p3)), dmax2(dmax2(p0, p1), dmax2(p2, p3))};
}
__device__ __forceinline__ IvD mulcd(IvD a, double c) {
    const double p0 = a.lo * c, p1 = a.hi * c;
    return IvD{dmin2(p0, p1), dmax2(p0, p1)};
}
__device__ __forceinline__ IvD divcd(IvD a, double c) { return IvD{a.lo / c, a.hi / c}; }   // c > 0
__device__ __forceinline__ IvD sqrd(IvD a) {
    const double l = a.lo * a.lo, h = a.hi * a.hi;
    if (a.lo >= 0.) return IvD{l, h};
    if (a.hi <= 0.) return IvD{h, l};
    return IvD{0., dmax2(l, h)};
}
__device__ __forceinline__ IvD tod(Iv a) { return IvD{(double)a.lo, (double)a.hi}; }
__device__ __forceinline__ Iv tof(IvD a) { return Iv{(float)a.lo, (float)a.hi}; }
// sq_exact(v) = (double)v * (double)v
__device__ __forceinline__ IvD sq_exact_iv(Iv a) { return sqrd(tod(a)); }

// widen by a relative margin; anything non-finite (or NaN) becomes the whole line
__device__ __forceinline__ Iv settle(Iv a) {
    const float m = fmax2(fabsf(a.lo), fabsf(a.hi));
    const float s = m * (1.f / 65536.f) + 1e-30f;
    Iv r{a.lo - s, a.hi + s};
    if (!(r.lo <= r.hi) || !(fabsf(r.lo) <= 3.0e38f) || !(fabsf(r.hi) <= 3.0e38f)) r = Iv{-INFINITY, INFINITY};
    return r;
}
__device__ __forceinline__ Iv settle_point(Iv a) {   // transformed coordinates: only sanitise
    if (!(a.lo <= a.hi)) return Iv{-INFINITY, INFINITY};
    return a;
}

struct Box { Iv x, y, z; };

__device__ __forceinline__ Box xform_iv(const float* __restrict__ m, Box p) {
    Box r;
    r.x = settle_point(add(add(add(mulc(p.x, m[0]), mulc(p.y, m[1])), mulc(p.z, m[2])), ivc(m[3])));
    r.y = settle_point(add(add(add(mulc(p.x, m[4]), mulc(p.y, m[5])), mulc(p.z, m[6])), ivc(m[7])));
    r.z = settle_point(add(add(add(mulc(p.x, m[8]), mulc(p.y, m[9])), mulc(p.z, m[10])), ivc(m[11])));
    return r;
}

// an XF_DIAG matrix (program.hpp XformPattern) over a box of finite points: each row's term of its
// own coordinate plus the translation -- the dropped +-0 terms change at most the sign of a zero
// endpoint, which no decision or class reads (jit.cpp xform_iv_row emits the same rows)
__device__ __forceinline__ Box xform_iv_diag(const float* __restrict__ m, Box p) {
    Box r;
    r.x = settle_point(add(mulc(p.x, m[0]), ivc(m[3])));
    r.y = settle_point(add(mulc(p.y, m[5]), ivc(m[7])));
    r.z = settle_point(add(mulc(p.z, m[10]), ivc(m[11])));
    return r;
}

// ---- primitives (mirroring ifunc_device.hpp operation for operation) ------------------------
__device__ __forceinline__ Iv egg_iv(Box p) {
    const Iv u = divc(sub(p.x, ivc(0.f)), 0.5f), v = divc(sub(p.y, ivc(0.f)), 0.5f), w = divc(sub(p.z, ivc(0.f)), 0.5f);
    return sub(ivc(1.f), add(add(sqr(u), sqr(v)), sqr(w)));
}

// range of the rabbit table values any point of the box can read (cube_f)
__device__ __forceinline__ Iv cube_iv(const float* __restrict__ tab, float2 tab_range, Box p) {
    const int sx = IMPLI_RABBIT_NX, sy = IMPLI_RABBIT_NY, sz = IMPLI_RABBIT_NZ;
    const float gs = bits2f(IMPLI_RABBIT_GRID_SIZE_BITS);
    const float ox = bits2f(IMPLI_RABBIT_ORIGIN_X_BITS), oy = bits2f(IMPLI_RABBIT_ORIGIN_Y_BITS),
                oz = bits2f(IMPLI_RABBIT_ORIGIN_Z_BITS);
    const float xm = ox + gs * (float)sx, ym = oy + gs * (float)sy, zm = oz + gs * (float)sz;
    // point is "out" iff xm < X || X < ox || ... (per axis)
    const bool all_in = p.x.lo >= ox && p.x.hi <= xm && p.y.lo >= oy && p.y.hi <= ym && p.z.lo >= oz && p.z.hi <= zm;
    const bool none_in = p.x.lo > xm || p.x.hi < ox || p.y.lo > ym || p.y.hi < oy || p.z.lo > zm || p.z.hi < oz;
    const Iv outside{-10000.f, -10000.f};
    if (none_in) return outside;
    // in-table points: xg = (int)((X - ox) / gs) is monotone in X
    const int x0 = (int)((fmax2(p.x.lo, ox) - ox) / gs), x1 = (int)((fmin2(p.x.hi, xm) - ox) / gs);
    const int y0 = (int)((fmax2(p.y.lo, oy) - oy) / gs), y1 = (int)((fmin2(p.y.hi, ym) - oy) / gs);
    const int z0 = (int)((fmax2(p.z.lo, oz) - oz) / gs), z1 = (int)((fmin2(p.z.hi, zm) - oz) / gs);
    float vmin, vmax;
    const int cnt = (x1 - x0 + 2) * (y1 - y0 + 2) * (z1 - z0 + 2);
    if (x1 - x0 <= 1 && y1 - y0 <= 1 && z1 - z0 <= 1 && p.x.lo <= p.x.hi) {
        // the read range per axis ([x0, x1 + 1], 2 or 3 entries) is covered by the 2-blocks at
        // x0 and x1: at most eight independent loads of the block min / max table
        const float2* mm = reinterpret_cast<const float2*>(tab + kRabbitBlockMinMax);
        vmin = INFINITY; vmax = -INFINITY;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int x = (k & 1) ? x1 : x0, y = (k & 2) ? y1 : y0, z = (k & 4) ? z1 : z0;
            const float2 m = mm[x + y * sx + z * sx * sy];
            vmin = fmin2(vmin, m.x);
            vmax = fmax2(vmax, m.y);
        }
    } else if (cnt > 512 || !(p.x.lo <= p.x.hi)) {
        vmin = tab_range.x; vmax = tab_range.y;
    } else {
        vmin = INFINITY; vmax = -INFINITY;
        // the reads are b + {0, 1} + {0, sx} + {0, sx*sy} with b = xg + yg*sx + zg*sx*sy
        for (int z = z0; z <= z1 + 1; ++z)
            for (int y = y0; y <= y1 + 1; ++y)
                for (int x = x0; x <= x1 + 1; ++x) {
                    const float v = tab[x + y * sx + z * sx * sy];
                    vmin = fmin2(vmin, v);
                    vmax = fmax2(vmax, v);
                }
    }
    // trilinear weights are in [0, 1] up to a few ulps; cover the extrapolation generously
    const float s = (fabsf(vmin) + fabsf(vmax)) * 1e-4f + 1e-6f;
    Iv r{-(vmax + s), -(vmin - s)};
    if (!all_in) r = hull(r, outside);
    return r;
}

__device__ __forceinline__ Iv cyl_iv(Box p) {
    const float w0 = 0.f, w1 = 0.f, w2 = 1.f, X = 0.f, Y = 0.f, Zc = -0.5f;
    const Iv t0 = add(add(mulc(sub(p.x, ivc(X)), w0), mulc(sub(p.y, ivc(Y)), w1)), mulc(sub(p.z, ivc(Zc)), w2));
    const Iv t1 = sub(ivc(1.f), t0);
    const Iv a = sub(sub(p.x, mulc(t0, w0)), ivc(X)), b = sub(sub(p.y, mulc(t0, w1)), ivc(Y)),
             c = sub(sub(p.z, mulc(t0, w2)), ivc(Zc));
    const Iv r_ = sub(ivc(0.5f), sqrt_iv(add(add(sqr(a), sqr(b)), sqr(c))));
    return stdmin_iv(t0, stdmin_iv(t1, r_));
}

__device__ __forceinline__ Iv cone_iv(Box p) {
    const float q = 0.5f / 1.f, a2 = q * q, z0 = 0.5f;
    const Iv dx = sub(p.x, ivc(0.f)), dy = sub(p.y, ivc(0.f)), dz = sub(p.z, ivc(z0));
    const Iv f = add(neg(sqrt_iv(add(sqr(dx), sqr(dy)))), sqrt_iv(mulc(sqr(dz), a2)));
    const Iv up = sub(neg(dz), ivc(0.f)), lo = add(dz, ivc(1.f));
    return stdmin_iv(f, stdmin_iv(up, lo));
}

__device__ __forceinline__ IvD cube_cr_iv(IvD t) {   // x^3 is monotone
    return IvD{cube_cr(t.lo), cube_cr(t.hi)};
}
__device__ __forceinline__ Iv heart_iv(Box p) {
    const IvD d2 = tod(p.y), d3 = tod(p.z);
    const IvD T = subd(addd(addd(tod(sqr(p.x)), muld(mulcd(d2, 9. / 4.), d2)), tod(sqr(p.z))), IvD{1., 1.});
    const IvD t3 = cube_cr_iv(T);
    const Iv a = mul(mul(mul(sqr(p.x), p.z), p.z), p.z);
    const IvD b = muld(muld(muld(muld(mulcd(d2, 9. / 200.), d2), d3), d3), d3);
    const IvD v = subd(subd(t3, tod(a)), b);
    return tof(IvD{-v.hi, -v.lo});
}

__device__ __forceinline__ Iv torus_iv(Box p) {
    const float r = 4.f, rx = 0.2f, ry = 0.2f, rz = 0.2f;
    const IvD s = addd(sq_exact_iv(divc(p.x, rx)), sq_exact_iv(divc(p.y, ry)));
    const IvD q{(double)r - sqrt(dmax2(s.hi, 0.)), (double)r - sqrt(dmax2(s.lo, 0.))};
    const IvD v = subd(subd(IvD{1., 1.}, sqrd(q)), sq_exact_iv(divc(p.z, rz)));
    return tof(v);
}

__device__ __forceinline__ Iv dm_iv(Box p) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = a * a, c2 = c * c;
    bool any = false;
    Iv res{INFINITY, -INFINITY};
    if (p.z.hi > r) { res = hull(res, sub(ivc(r), p.z)); any = true; }
    if (p.z.lo < -r) { res = hull(res, add(ivc(r), p.z)); any = true; }
    if (p.z.lo <= r && p.z.hi >= -r) {
        // the endpoints are exact squares of floats (or 0): dm_f's one-correction-step quotient is
        // the IEEE quotient for every one of them (tools/divconst_check.c), three f64 operations
        // instead of a division sequence -- the bounds are bit for bit those of divcd
        const double D = (double)a2, R = 1.0 / (double)a2;
        static_assert(0.2f * 0.2f == (float)(0.4 / 2) * (float)(0.4 / 2), "the checked constant");
        auto q = [&](IvD t) { return IvD{div_sq_const(t.lo, D, R), div_sq_const(t.hi, D, R)}; };
        (void)b2;
        (void)c2;
        const IvD v = subd(subd(addd(q(sq_exact_iv(sub(p.x, ivc(0.f)))), q(sq_exact_iv(sub(p.y, ivc(0.f))))),
                                q(sq_exact_iv(sub(p.z, ivc(0.f))))),
                          IvD{1., 1.});
        res = hull(res, tof(IvD{-v.hi, -v.lo}));
        any = true;
    }
    if (!any) res = Iv{-INFINITY, INFINITY};
    return res;
}

// screw: f = (-r + r0) + delta * sinf(arg) with r = |(x, y, d2)|, where d2 = z - p2 is the rounding
// residual of p2 = (z + 0.5) - 0.5: |d2| <= 2^-23 (|z| + 1) (bounded by twice that), and
// arg = 2 pi (t / tw - theta / 2 pi), t = z + 0.5, theta = atan2(y, x) (screw_f).
__device__ __forceinline__ float absmin_iv(Iv a) { return a.lo > 0.f ? a.lo : (a.hi < 0.f ? -a.hi : 0.f); }
__device__ __forceinline__ float absmax_iv(Iv a) { return fmax2(fabsf(a.lo), fabsf(a.hi)); }
// Range of sinf(arg) over the box, from the box's centre: the xy rectangle lies in the disc of
// radius R (half diagonal) around (xc, yc), at distance d from the axis, so theta is within
// asin(R / d) <= 1.0472 R / d (R / d <= 1/2) of atan2(yc, xc) -- modulo 2 pi, which the sine does
// not see (theta's jump at atan2's cut and y = -0 reading as +0 change arg by 2 pi).  With
// arg = 2 pi u - theta, u = t / tw, |arg - ac| <= h and sin is 1-Lipschitz.  A margin of
// 2^-12 (1 + |ac| + h) on arg and 2^-16 on the sine covers the device atan2f / sinf errors (a
// few ulps) and the rounding of the reference's float expression (t / tw - theta / pi2) * 2 * pi
// (|ac| < 2^12 is required, else [-1, 1]).  One atan2f and one sinf per box.
__device__ __forceinline__ Iv screw_sin_iv(float tw, Box p) {
    const Iv full{-1.f, 1.f};
    const float xc = 0.5f * (p.x.lo + p.x.hi), yc = 0.5f * (p.y.lo + p.y.hi);
    const float hx = 0.5f * (p.x.hi - p.x.lo), hy = 0.5f * (p.y.hi - p.y.lo);
    const float R = sqrtf(hx * hx + hy * hy), d = sqrtf(xc * xc + yc * yc);
    const float u0 = (p.z.lo + 0.5f) / tw, u1 = (p.z.hi + 0.5f) / tw;
    const float kPi = 3.14159265358979323846f;
    const float ac = kPi * (u0 + u1) - atan2f(yc, xc);
    const float h0 = kPi * fabsf(u1 - u0) + 1.0472f * (R / d);
    const float h = h0 + (1.f + fabsf(ac) + h0) * 0x1p-12f;
    // NaN / infinite inputs fail the comparisons
    if (!(R < 0.5f * d) || !(fabsf(ac) < 4096.f) || !(h < 2.f)) return full;
    const float s = sinf(ac);
    return Iv{fmax2(s - h - 0x1p-16f, -1.f), fmin2(s + h + 0x1p-16f, 1.f)};
}
__device__ __forceinline__ Iv screw_iv(const float* __restrict__ prm, Box p) {
    const float r0 = prm[1];
    const float ax = absmax_iv(p.x), ay = absmax_iv(p.y), bx = absmin_iv(p.x), by = absmin_iv(p.y);
    const float dz = (absmax_iv(p.z) + 1.f) * 0x1p-22f;
    const float rhi = sqrtf(ax * ax + (ay * ay + dz * dz)), rlo = sqrtf(bx * bx + (by * by + 0.f));
    const Iv ds = mulc(screw_sin_iv(prm[0], p), prm[2]);
    return Iv{(-rhi + r0) + ds.lo, (-rlo + r0) + ds.hi};
}
__device__ __forceinline__ Iv lid_iv(Box p) {
    const Iv a = sub(p.z, ivc(0.5f)), b = mulc(add(p.z, ivc(0.5f)), -1.f);
    return Iv{fmax2(a.lo, b.lo), fmax2(a.hi, b.hi)};
}
__device__ __forceinline__ Iv tbb_iv(const float* __restrict__ prm, Box p) {   // tbb_f
    return stdmin_iv(screw_iv(prm, p), mulc(lid_iv(p), -1.f));
}
__device__ __forceinline__ Iv hp_iv(const float* __restrict__ prm, Box p) {
    return add(add(add(ivc(0.f), mulc(sub(p.x, ivc(prm[3])), prm[0])), mulc(sub(p.y, ivc(prm[4])), prm[1])),
               mulc(sub(p.z, ivc(prm[5])), prm[2]));
}

__device__ __forceinline__ Iv tet_iv(const float* __restrict__ P, Box p) {
    Iv r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        r[k] = add(add(add(mulc(p.x, P[4 * k]), mulc(p.y, P[4 * k + 1])), mulc(p.z, P[4 * k + 2])), ivc(P[4 * k + 3]));
    return stdmin_iv(r[0], stdmin_iv(r[1], stdmin_iv(r[2], r[3])));
}
// each ball's term is monotone decreasing in h, h monotone in each square; 1/h rounds monotonely
__device__ __forceinline__ Iv meta_iv(const float* __restrict__ P, Box p) {
    Iv out = ivc(0.0f);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float* B = P + 5 * b;
        const Iv h = add(add(add(ivc((float)0.000001), sqr(sub(p.x, ivc(B[0])))), sqr(sub(p.y, ivc(B[1])))),
                         sqr(sub(p.z, ivc(B[2]))));
        const Iv hinv{(float)(1.0 / (double)h.hi), (float)(1.0 / (double)h.lo)};
        out = add(out, divc(sub(mulc(hinv, B[3]), ivc(B[4])), 100.f));
    }
    return out;
}
__device__ __forceinline__ Iv extr_iv(const float* __restrict__ P, Box p) {
    const int n = (int)P[0];
    Iv r{INFINITY, INFINITY};
    for (int j = 0; j < n; ++j) {
        const Iv v = neg(sub(add(mulc(p.x, P[1 + 3 * j]), mulc(p.y, P[2 + 3 * j])), ivc(P[3 + 3 * j])));
        r = min_iv(r, v);
    }
    return r;
}

__device__ __forceinline__ Iv prim_iv(int t, const float* __restrict__ tab, float2 tab_range,
                                      const float* __restrict__ prm, Box p) {
    Iv r;
    switch (t) {
        case NT_ELLIPSOID: r = egg_iv(p); break;
        case NT_CUBE: r = cube_iv(tab, tab_range, p); break;
        case NT_CYLINDER: r = cyl_iv(p); break;
        case NT_CONE: r = cone_iv(p); break;
        case NT_HEART: r = heart_iv(p); break;
        case NT_TORUS: r = torus_iv(p); break;
        case NT_SCREW: r = screw_iv(prm, p); break;
        case NT_LID: r = lid_iv(p); break;
        case NT_HALF_PLANE: r = hp_iv(prm, p); break;
        case NT_TETRA: r = tet_iv(prm, p); break;
        case NT_METABALLS: r = meta_iv(prm, p); break;
        case NT_EXTRUSION: r = extr_iv(prm, p); break;
        case NT_SCREW_TBB: r = tbb_iv(prm, p); break;
        default: r = dm_iv(p); break;
    }
    return settle(r);
}

// decision for one CSG node (transformed_union.hpp:48 etc.):
//   union        f = (f1 > f2) ? f1 : f2
//   intersection f = (f1 > f2) ? f2 : f1
//   difference   f = (f1 < -f2) ? f1 : -f2
__device__ __forceinline__ uint32_t csg_decide(int t, Iv a, Iv b, Iv& out) {
    if (t == NT_UNION) {
        if (a.lo > b.hi) { out = a; return PM_LEFT; }
        if (a.hi <= b.lo) { out = b; return PM_RIGHT; }
        out = Iv{fmax2(a.lo, b.lo), fmax2(a.hi, b.hi)};
        return PM_BOTH;
    }
    if (t == NT_INTERSECTION) {
        if (a.lo > b.hi) { out = b; return PM_RIGHT; }
        if (a.hi <= b.lo) { out = a; return PM_LEFT; }
        out = min_iv(a, b);
        return PM_BOTH;
    }
    const Iv nb = neg(b);
    if (a.hi < nb.lo) { out = a; return PM_LEFT; }
    if (a.lo >= nb.hi) { out = nb; return PM_RIGHT; }
    out = min_iv(a, nb);
    return PM_BOTH;
}

__device__ __forceinline__ uint32_t mode_of(uint64_t modes, int csg);

// interval interpreter over a box; returns the root interval and the per-node modes.  Operands
// already pruned by `modes_in` (the modes of an enclosing box, valid for this sub-box) are
// skipped and their decision kept.  The stacks are kept as separate scalar arrays (structure of
// arrays) so that the uniform-index accesses stay in VGPRs (arrays of Iv structs were demoted to
// scratch).
// one instruction through any program pointer (field by field: an Instr in another address space
// does not bind to the copy constructor's reference)
template <class ProgP>
__device__ __forceinline__ Instr instr_at(ProgP prog, int pc) {
    const auto& s = prog->instr[pc];
    Instr I;
    I.op = s.op; I.type = s.type; I.mat = s.mat; I.csg = s.csg;
    I.skip_csg = s.skip_csg; I.skip_child = s.skip_child; I.skip_to = s.skip_to; I.prm = s.prm;
    return I;
}

// a matrix / parameter row as a generic pointer (after inlining, the address space is inferred
// back from the cast, so constant-space rows are still read with scalar loads)
template <class ProgP>
__device__ __forceinline__ const float* mat_row(ProgP prog, int i) { return (const float*)prog->mats[i]; }

// ProgP: the program pointer -- const Program*, or a constant-address-space pointer when it was
// loaded from memory (merged object streams: scalar loads of the instructions, eval.hip ProgC)
template <int D, class ProgP>
__device__ __forceinline__ Iv eval_iv(ProgP __restrict__ prog, const float* __restrict__ tab,
                                      float2 tab_range, Box p0, uint64_t modes_in, uint64_t& modes) {
    float xl[D], xh[D], yl[D], yh[D], zl[D], zh[D], vl[D], vh[D];
    int sp = 0, vp = 0;
    xl[0] = p0.x.lo; xh[0] = p0.x.hi; yl[0] = p0.y.lo; yh[0] = p0.y.hi; zl[0] = p0.z.lo; zh[0] = p0.z.hi;
    modes = modes_in;
    const int n = prog->n_instr;
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = instr_at(prog, pc);
        if (I.skip_csg >= 0) {
            const uint32_t m = mode_of(modes_in, I.skip_csg);
            if (m == (I.skip_child ? (uint32_t)PM_LEFT : (uint32_t)PM_RIGHT)) {
                pc = I.skip_to - 1;
                continue;
            }
        }
        const Box cur{Iv{xl[sp], xh[sp]}, Iv{yl[sp], yh[sp]}, Iv{zl[sp], zh[sp]}};
        if (I.op == OP_XFORM) {
            const Box q = I.type == XF_DIAG ? xform_iv_diag(mat_row(prog, I.mat), cur) : xform_iv(mat_row(prog, I.mat), cur);
            ++sp;
            xl[sp] = q.x.lo; xh[sp] = q.x.hi; yl[sp] = q.y.lo; yh[sp] = q.y.hi; zl[sp] = q.z.lo; zh[sp] = q.z.hi;
        } else if (I.op == OP_PRIM) {
            const Iv r = prim_iv(I.type, tab, tab_range, mat_row(prog, I.prm), cur);
            vl[vp] = r.lo; vh[vp] = r.hi;
            ++vp;
            --sp;
        } else {
            --sp;
            const uint32_t pm = mode_of(modes_in, I.csg);
            if (pm == PM_BOTH) {
                --vp;
                const Iv b{vl[vp], vh[vp]};
                const Iv a{vl[vp - 1], vh[vp - 1]};
                Iv o;
                const uint32_t m = csg_decide(I.type, a, b, o);
                if (I.csg < kMaxPruned) modes |= (uint64_t)m << (2 * I.csg);
                vl[vp - 1] = o.lo; vh[vp - 1] = o.hi;
            } else if (pm == PM_RIGHT && I.type == NT_DIFFERENCE) {   // the kept operand is -f2
                const float lo = vl[vp - 1];
                vl[vp - 1] = -vh[vp - 1];
                vh[vp - 1] = -lo;
            }
        }
    }
    return Iv{vl[0], vh[0]};
}

__device__ __forceinline__ uint32_t mode_of(uint64_t modes, int csg) {
    return (csg >= 0 && csg < kMaxPruned) ? (uint32_t)(modes >> (2 * csg)) & 3u : (uint32_t)PM_BOTH;
}

// point interpreter that skips pruned operands; bit-identical to eval_f for points in the brick
template <int D, class ProgP>
__device__ __forceinline__ float eval_f_pruned(ProgP __restrict__ prog, const float* __restrict__ tab,
                                               uint64_t modes, float x, float y, float z) {
    float px[D], py[D], pz[D], vf[D];
    int sp = 0, vp = 0;
    px[0] = x; py[0] = y; pz[0] = z;
    const int n = prog->n_instr;
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = instr_at(prog, pc);
        if (I.skip_csg >= 0) {
            const uint32_t m = mode_of(modes, I.skip_csg);
            if (m == (I.skip_child ? (uint32_t)PM_LEFT : (uint32_t)PM_RIGHT)) {
                pc = I.skip_to - 1;
                continue;
            }
        }
        if (I.op == OP_XFORM) {
            const float* M = mat_row(prog, I.mat);
            const V3 q = I.type == XF_DIAG ? xform_diag(M, px[sp], py[sp], pz[sp]) : xform(M, px[sp], py[sp], pz[sp]);
            ++sp;
            px[sp] = q.x; py[sp] = q.y; pz[sp] = q.z;
        } else if (I.op == OP_PRIM) {
            vf[vp++] = prim_f(I.type, tab, mat_row(prog, I.prm), px[sp], py[sp], pz[sp]);
            --sp;
        } else {
            --sp;
            const uint32_t m = mode_of(modes, I.csg);
            if (m == PM_BOTH) {
                const float f2 = vf[--vp];
                const float f1 = vf[vp - 1];
                vf[vp - 1] = (I.type == NT_UNION) ? ((f1 > f2) ? f1 : f2)
                           : (I.type == NT_INTERSECTION) ? ((f1 > f2) ? f2 : f1)
                                                        : ((f1 < -f2) ? f1 : -f2);
            } else if (m == PM_RIGHT && I.type == NT_DIFFERENCE) {
                vf[vp - 1] = -vf[vp - 1];
            }
        }
    }
    return vf[0];
}

}  // namespace dev
}  // namespace impli
