/*
 * or_ifunc.c -- oracle restatement of the implicit-function library (TEST INFRASTRUCTURE ONLY).
 *
 * Per-point recursion with exactly the reference's float/double arithmetic.  The reference
 * evaluates node by node over whole batches (prepare_inner_vectors copies, basic_functions.hpp:
 * 361-379); evaluation order per point is identical, so the values are identical.
 *
 * Library calls: std::pow(float,int) is restated as the exact double square; std::pow(double,0.5)
 * as sqrt (glibc pow is correctly rounded outside hard cases); std::pow(double,3) uses libm pow.
 * See DESIGN.md "fp discipline".
 */
#include "oracle.h"

#include <math.h>
#include <string.h>
#include "../implisolid_amd/csrc/generated/tables.h"

static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ---------------------------------------------------------------------------------------- */
/* basic_functions.hpp:77-128 invert_matrix: ublas lu_factorize + lu_substitute on a 4x4 float
   matrix whose last row is (0,0,0,1).  ublas (Boost ~1.57) lu.hpp: partial pivoting by the
   first max |.| in the column (index_norm_inf), column scaled by value_type(1)/pivot, rank-1
   update m -= l*u; lu_substitute = swap_rows(pm), unit-lower forward solve, upper back solve
   (triangular.hpp inplace_solve, "t = e2(n,l) /= e1(n,n); if (t != 0) e2(m,l) -= e1(m,n)*t"). */
int or_invert_matrix(const float in12[12], float out12[12]) {
    float A[4][4], E[4][4];
    int pm[4], i, j, r, c;
    for (i = 0; i < 3; i++)
        for (j = 0; j < 4; j++) A[i][j] = in12[i * 4 + j];
    A[3][0] = 0.f; A[3][1] = 0.f; A[3][2] = 0.f; A[3][3] = 1.f;
    for (i = 0; i < 4; i++) pm[i] = i;
    int singular = 0;
    for (i = 0; i < 4; i++) {
        int inorm = 0; float t = 0.f;
        for (r = i; r < 4; r++) { float u = fabsf(A[r][i]); if (u > t) { inorm = r - i; t = u; } }
        inorm += i;
        if (A[inorm][i] != 0.f) {
            if (inorm != i) {
                pm[i] = inorm;
                for (c = 0; c < 4; c++) { float tmp = A[inorm][c]; A[inorm][c] = A[i][c]; A[i][c] = tmp; }
            }
            float rcp = 1.f / A[i][i];
            for (r = i + 1; r < 4; r++) A[r][i] *= rcp;
        } else if (singular == 0) {
            singular = i + 1;
        }
        for (r = i + 1; r < 4; r++)
            for (c = i + 1; c < 4; c++) {
                float prod = A[r][i] * A[i][c];
                A[r][c] -= prod;
            }
    }
    if (singular) return 0;
    for (i = 0; i < 4; i++) for (j = 0; j < 4; j++) E[i][j] = (i == j) ? 1.f : 0.f;
    for (i = 0; i < 4; i++)
        if (i != pm[i]) for (c = 0; c < 4; c++) { float tmp = E[i][c]; E[i][c] = E[pm[i]][c]; E[pm[i]][c] = tmp; }
    /* unit lower: diagonal is 1 (division by 1 is exact and omitted) */
    for (int n = 0; n < 4; n++)
        for (int l = 0; l < 4; l++) {
            float t = E[n][l];
            if (t != 0.f)
                for (int m = n + 1; m < 4; m++) { float prod = A[m][n] * t; E[m][l] -= prod; }
        }
    for (int n = 3; n >= 0; n--)
        for (int l = 3; l >= 0; l--) {
            float t = (E[n][l] /= A[n][n]);
            if (t != 0.f)
                for (int m = n - 1; m >= 0; m--) { float prod = A[m][n] * t; E[m][l] -= prod; }
        }
    for (i = 0; i < 3; i++)
        for (j = 0; j < 4; j++) out12[i * 4 + j] = E[i][j];
    return 1;
}

void or_tree_prepare(or_node* nodes, int n) {
    for (int i = 0; i < n; i++) or_invert_matrix(nodes[i].m, nodes[i].minv);
}

/* basic_functions.hpp:140-177 matrix_vector_product: m00*x + m01*y + m02*z + m03 (left to right) */
static inline void xform(const float* m, const float p[3], float q[3]) {
    float x = p[0], y = p[1], z = p[2];
    q[0] = m[0] * x + m[1] * y + m[2] * z + m[3];
    q[1] = m[4] * x + m[5] * y + m[6] * z + m[7];
    q[2] = m[8] * x + m[9] * y + m[10] * z + m[11];
}

/* gradient post-transform, e.g. transformed_union.hpp:76-83: inv^T * g */
static inline void grad_xform(const float* m, const float g[3], float o[3]) {
    float gx = g[0], gy = g[1], gz = g[2];
    o[0] = m[0] * gx + m[4] * gy + m[8] * gz;
    o[1] = m[1] * gx + m[5] * gy + m[9] * gz;
    o[2] = m[2] * gx + m[6] * gy + m[10] * gz;
}

/* std::min(a,b) = (b < a) ? b : a */
static inline float stdmin(float a, float b) { return (b < a) ? b : a; }

static inline double sq_exact(float v) { double d = (double)v; return d * d; }

/* ---------------- primitives (local coordinates = after the node's own inverse matrix) ------ */

/* egg.hpp:93-106 (a=b=c=0.5, x0=y0=z0=0, ctor egg.hpp:42-58) */
static float egg_f(const float p[3]) {
    const float a = 0.5f, b = 0.5f, c = 0.5f;
    float u = (p[0] - 0.f) / a, v = (p[1] - 0.f) / b, w = (p[2] - 0.f) / c;
    float ns = u * u + v * v + w * w;          /* norm_squared basic_functions.hpp:18-20 */
    return 1.f - ns;
}
/* egg.hpp:108-128 */
static void egg_g(const float p[3], float g[3]) {
    const float a2 = 0.5f * 0.5f, b2 = a2, c2 = a2;
    g[0] = (float)(-2. * (double)(p[0] - 0.f) / (double)a2);
    g[1] = (float)(-2. * (double)(p[1] - 0.f) / (double)b2);
    g[2] = (float)(-2. * (double)(p[2] - 0.f) / (double)c2);
}

/* cube.hpp:176-272: trilinear lookup in the rabbit table, returns -res (res = 10000 outside).
   Out-of-table reads (F8d) see the object's trailing members then zeros. */
static float rabbit_at(int idx) {
    if (idx >= 0 && idx < IMPLI_RABBIT_NX * IMPLI_RABBIT_NY * IMPLI_RABBIT_NZ) return bitsf(IMPLI_RABBIT_BITS[idx]);
    switch (idx - IMPLI_RABBIT_NX * IMPLI_RABBIT_NY * IMPLI_RABBIT_NZ) {
        case 0: return bitsf(IMPLI_RABBIT_GRID_SIZE_BITS);
        case 1: return bitsf(IMPLI_RABBIT_ORIGIN_X_BITS);
        case 2: return bitsf(IMPLI_RABBIT_ORIGIN_Y_BITS);
        case 3: return bitsf(IMPLI_RABBIT_ORIGIN_Z_BITS);
        default: return 0.f;
    }
}
static int trunc_index(float v) { return v == v ? (int)v : 0; }
static float cube_f(const float p[3]) {
    const int sx = IMPLI_RABBIT_NX, sy = IMPLI_RABBIT_NY, sz = IMPLI_RABBIT_NZ;
    const float gs = bitsf(IMPLI_RABBIT_GRID_SIZE_BITS);
    const float ox = bitsf(IMPLI_RABBIT_ORIGIN_X_BITS), oy = bitsf(IMPLI_RABBIT_ORIGIN_Y_BITS),
                oz = bitsf(IMPLI_RABBIT_ORIGIN_Z_BITS);
    const float X = p[0], Y = p[1], Z = p[2];
    float res = 10000.f;
    if (ox + gs * (float)sx < X || X < ox) {
    } else if (oy + gs * (float)sy < Y || Y < oy) {
    } else if (oz + gs * (float)sz < Z || Z < oz) {
    } else {
        /* a NaN coordinate passes the bounds test and reaches the conversion, which is undefined
           behaviour in the reference (cube.hpp:222-224); the value is NaN whatever the index
           (xd is NaN), so the index is taken as 0, the device conversion's result (found by the
           sanitizer run, tests/test_sanitize.py) */
        int xg = trunc_index((X - ox) / gs);
        int yg = trunc_index((Y - oy) / gs);
        int zg = trunc_index((Z - oz) / gs);
        float xl = ox + (float)xg * gs;
        float yl = oy + (float)yg * gs;
        float zl = oz + (float)zg * gs;
        float xd = (X - xl) / gs, yd = (Y - yl) / gs, zd = (Z - zl) / gs;
        float r000 = rabbit_at(xg + yg * sx + zg * sx * sy);
        float r100 = rabbit_at((xg + 1) + yg * sx + zg * sx * sy);
        float r010 = rabbit_at(xg + (yg + 1) * sx + zg * sx * sy);
        float r110 = rabbit_at((xg + 1) + (yg + 1) * sx + zg * sx * sy);
        float r001 = rabbit_at(xg + yg * sx + (zg + 1) * sx * sy);
        float r101 = rabbit_at((xg + 1) + yg * sx + (zg + 1) * sx * sy);
        float r011 = rabbit_at(xg + (yg + 1) * sx + (zg + 1) * sx * sy);
        float r111 = rabbit_at((xg + 1) + (yg + 1) * sx + (zg + 1) * sx * sy);
        float c00 = r000 * (1.f - xd) + r100 * xd;
        float c01 = r001 * (1.f - xd) + r101 * xd;
        float c10 = r010 * (1.f - xd) + r110 * xd;
        float c11 = r011 * (1.f - xd) + r111 * xd;
        float c0 = c00 * (1.f - yd) + c10 * yd;
        float c1 = c01 * (1.f - yd) + c11 * yd;
        res = c0 * (1.f - zd) + c1 * zd;
    }
    return -res;
}
/* cube.hpp:273-315: gradient of the OLD 6-plane cube (mismatched with the rabbit field, F3) */
static void cube_g(const float p[3], float g[3]) {
    static const float P[18] = {0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f, 0, 0, 0, 0.5f, 0, 0, -0.5f};
    const float cx = 0.f, cy = 0.f, cz = 0.f;
    float i1 = p[0], i2 = p[1], i3 = p[2];
    int index = 0;
#define PLANE(k) ((double)((i1 - cx - P[0 + (k) * 3]) * P[0 + (k) * 3]) * (-2.) + \
                  (double)((i2 - cy - P[1 + (k) * 3]) * P[1 + (k) * 3]) * (-2.) + \
                  (double)((i3 - cz - P[2 + (k) * 3]) * P[2 + (k) * 3]) * (-2.))
    float mn = (float)PLANE(0);
    for (int k = 0; k < 6; k++) {
        if (PLANE(k) < (double)mn) { index = k; mn = (float)PLANE(k); }
    }
#undef PLANE
    g[0] = -P[index * 3 + 0];
    g[1] = -P[index * 3 + 1];
    g[2] = -P[index * 3 + 2];
}

/* scylinder.hpp:97-124 (ctor :21-41: radius 0.5, c_len 1, centre (0,0,-0.5), w=(0,0,1)) */
static void cyl_parts(const float p[3], float* t0o, float* t1o, float* ro) {
    const float X = 0.f, Y = 0.f, Zc = -0.5f, w0 = 0.f, w1 = 0.f, w2 = 1.f, clen = 1.f, ru = 0.5f;
    float i0 = p[0], i1 = p[1], i2 = p[2];
    float t0 = (i0 - X) * w0 + (i1 - Y) * w1 + (i2 - Zc) * w2;
    float t1 = clen - t0;
    float a = i0 - w0 * t0 - X, b = i1 - w1 * t0 - Y, c = i2 - w2 * t0 - Zc;
    float r_ = ru - sqrtf(a * a + b * b + c * c);
    *t0o = t0; *t1o = t1; *ro = r_;
}
static float cyl_f(const float p[3]) {
    float t0, t1, r_;
    cyl_parts(p, &t0, &t1, &r_);
    return stdmin(t0, stdmin(t1, r_));
}
/* scylinder.hpp:125-166 */
static void cyl_g(const float p[3], float g[3]) {
    const float X = 0.f, Y = 0.f, Zc = -0.5f, w0 = 0.f, w1 = 0.f, w2 = 1.f;
    float t0, t1, r_;
    cyl_parts(p, &t0, &t1, &r_);
    float i0 = p[0], i1 = p[1], i2 = p[2];
    float c_t0 = (t0 <= t1 && t0 <= r_) ? 1.f : 0.f;
    float c_t1 = (t1 <= t0 && t1 <= r_) ? 1.f : 0.f;
    float c_r = (r_ <= t0 && r_ <= t1) ? 1.f : 0.f;
    g[0] = c_t0 * w0 + c_t1 * (-w0) + c_r * (w0 * t0 + X - i0);
    g[1] = c_t0 * w1 + c_t1 * (-w1) + c_r * (w1 * t0 + Y - i1);
    g[2] = c_t0 * w2 + c_t1 * (-w2) + c_r * (w2 * t0 + Zc - i2);
}

/* scone.hpp:81-109 (ctor :18-33: h=1, r1=0, r2=0.5, centre (0,0,0.5)) */
static float cone_f(const float p[3]) {
    const float h = 1.f, r1 = 0.f, r2 = 0.5f, x0 = 0.f, y0 = 0.f, z0 = 0.5f;
    const float q = r2 / h;
    const float a2 = q * q;
    float x = p[0], y = p[1], z = p[2];
    float f = -sqrtf((x - x0) * (x - x0) + (y - y0) * (y - y0)) + sqrtf((z - z0) * (z - z0) * a2);
    float up = -(z - z0) - r1;
    float lo = (z - z0) + h;
    return stdmin(f, stdmin(up, lo));
}
/* scone.hpp:110-151 */
static void cone_g(const float p[3], float g[3]) {
    const float h = 1.f, r1 = 0.f, r2 = 0.5f, x0 = 0.f, y0 = 0.f, z0 = 0.5f;
    const float q = r2 / h;
    const float a2 = q * q;
    float x = p[0], y = p[1], z = p[2];
    float f = -(x - x0) * (x - x0) / a2 - (y - y0) * (y - y0) / a2 + (z - z0) * (z - z0);
    float up = -(z - z0) - r1;
    float lo = (z - z0) + h;
    if (up < f && up < lo) { g[0] = 0.f; g[1] = 0.f; g[2] = -1.f; }
    else if (lo < f && lo < up) { g[0] = 0.f; g[1] = 0.f; g[2] = 1.f; }
    else { g[0] = -2.f * (x - x0) / a2; g[1] = -2.f * (y - y0) / a2; g[2] = 2.f * (z - z0); }
}

/* heart.hpp:82-103 */
static float heart_f(const float p[3]) {
    float i1 = p[0], i2 = p[1], i3 = p[2];
    double T = (double)(i1 * i1) + (9. / 4.) * (double)i2 * (double)i2 + (double)(i3 * i3) - 1.;
    double t3 = pow(T, 3);
    float a = i1 * i1 * i3 * i3 * i3;
    double b = (9. / 200.) * (double)i2 * (double)i2 * (double)i3 * (double)i3 * (double)i3;
    return (float)(-(t3 - (double)a - b));
}
/* heart.hpp:104-132 */
static void heart_g(const float p[3], float g[3]) {
    float i1 = p[0], i2 = p[1], i3 = p[2];
    double T = (double)(i1 * i1) + (9. / 4.) * (double)i2 * (double)i2 + (double)(i3 * i3) - 1.;
    float a = (float)(T * T);  /* pow(T, 2) */
    double d1 = (double)i1, d2 = (double)i2, d3 = (double)i3, da = (double)a;
    g[0] = (float)(-6. * d1 * da + 2. * d1 * d3 * d3 * d3);
    g[1] = (float)(-(27. / 2) * d2 * da + (9. / 100.) * d2 * d3 * d3 * d3);
    g[2] = (float)(-6. * d3 * da + 3. * d1 * d1 * d3 * d3 + (27. / 200.) * d2 * d2 * d3 * d3);
}

/* torus.hpp:68-94 (ctor :46-60: r = 4, rx = ry = rz = 0.2) */
static float torus_f(const float p[3]) {
    const float r = 4.f, rx = 0.2f, ry = 0.2f, rz = 0.2f;
    float x = p[0], y = p[1], z = p[2];
    double s = sq_exact(x / rx) + sq_exact(y / ry);
    double q = (double)r - sqrt(s);          /* std::pow(s, 0.5) */
    double f = 1. - q * q - sq_exact(z / rz); /* std::pow(q, 2) */
    return (float)f;
}
/* torus.hpp:96-124 */
static void torus_g(const float p[3], float g[3]) {
    const float r = 4.f, rx = 0.2f, ry = 0.2f, rz = 0.2f;
    float x = p[0], y = p[1], z = p[2];
    float s = x * x / (rx * rx) + y * y / (ry * ry);
    float a = (float)sqrt((double)s);   /* std::pow(float, 0.5) -> double */
    g[0] = (2.f * x / (rx * rx * a)) * (r - a);
    g[1] = (2.f * y / (ry * ry * a)) * (r - a);
    g[2] = -2.f * z / (rz * rz);
}

/* double_mushroom.hpp:90-121 with the factory's parameters object_factory.hpp:89
   double_mushroom(0.9, 0.4/2, 0.4/2, 1/0.2): r = 0.9f/2, a = b = 0.2f, c = 1/5.0f.
   The inner identity transform (ctor :29-40) changes nothing but signs of zero (omitted). */
static float dm_f(const float p[3]) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), b = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = b * b, c2 = c * c;
    float x = p[0], y = p[1], z = p[2];
    if (z > r) return r - z;
    if (z < -r) return r + z;
    double v = sq_exact(x - 0.f) / (double)a2 + sq_exact(y - 0.f) / (double)b2 - sq_exact(z - 0.f) / (double)c2 - 1;
    return (float)(-v);
}
/* double_mushroom.hpp:122-160 */
static void dm_g(const float p[3], float g[3]) {
    const float r = 0.9f / 2, a = (float)(0.4 / 2), b = (float)(0.4 / 2), c = 1.f / (float)(1 / 0.2);
    const float a2 = a * a, b2 = b * b, c2 = c * c;
    float x = p[0], y = p[1], z = p[2];
    if (z < -r) { g[0] = 0.f; g[1] = 0.f; g[2] = 1.f; }
    else if (z > r) { g[0] = 0.f; g[1] = 0.f; g[2] = -1.f; }
    else { g[0] = -2.f * (x - 0.f) / a2; g[1] = -2.f * (y - 0.f) / b2; g[2] = 2.f * (z - 0.f) / c2; }
}

/* ---------------- screw.hpp:98-150 (implicitFunction) at the constants its constructor sets:
   u = (1,0,0), v = (0,1,0), w = (0,0,1), A = (0,0,-slen/2) = (0,0,-0.5), UVW = I (screw.hpp:
   222-330); the factory forces the identity transformation_matrix (object_factory.hpp:304-351).
   prm = {twist_rate = pitch, r0 = inner/2, delta = outer/2 - inner/2} (outer = |v| = 1, inner =
   outer/delta_ratio).  Eigen evaluation orders: t = (x - A) w is a GEMV (columns accumulated into
   a zeroed result), p = w t^T + A an outer product, ab = UVW^-1 (x - p) a GEMM (depth accumulated
   from zero, then added to the zeroed destination), |x - p| the 3-term redux a0 + (a1 + a2). */
static const double OR_M_PI = 3.14159265358979323846;   /* <cmath> M_PI */
static const float SCREW_PI = (float)3.1415926535897;   /* screw.hpp:20 const REAL pi */

static float screw_f(const float p[3], const float* prm) {
    const float x = p[0], y = p[1], z = p[2];
    const float tw = prm[0], r0 = prm[1], delta = prm[2];
    const float a0 = x - 0.f, a1 = y - 0.f, a2 = z - (-0.5f);
    const float t = ((0.f + a0 * 0.f) + a1 * 0.f) + a2 * 1.f;
    const float p0 = 0.f * t + 0.f, p1 = 0.f * t + 0.f, p2 = 1.f * t + (-0.5f);
    const float d0 = x - p0, d1 = y - p1, d2 = z - p2;
    const float ab0 = 0.f + (((0.f + 1.f * d0) + 0.f * d1) + 0.f * d2);
    const float ab1 = 0.f + (((0.f + 0.f * d0) + 1.f * d1) + 0.f * d2);
    const float theta = or_atan2f(ab1, ab0);
    const float r = sqrtf(d0 * d0 + (d1 * d1 + d2 * d2));
    const float pi2 = SCREW_PI * 2;
    const float ph = t / tw - theta / pi2;
    return (-r + r0) + delta * or_sinf(ph * 2 * SCREW_PI);   /* phi, screw.hpp:29-36 */
}

/* screw.hpp:152-160 gradient (sympy expression) at the same constants; the C++ types of each
   sub-expression are kept: std::pow(float, 2) promotes to an exact double square, atan2 of two
   floats is atan2f (basic_data_structures.hpp's `using namespace std`), cos of a double is the
   double cos, M_PI is double. */
static void screw_g(const float p[3], const float* prm, float g[3]) {
    const float x = p[0], y = p[1], z = p[2];
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
    const float th = or_atan2f(U1, U0);
    const double cv = cos(OR_M_PI * (((double)(2 * phi0) - (double)th / OR_M_PI) + (double)((2 * s) / tw)));
    const double wx2 = sq_exact(wx), wy2 = sq_exact(wy), wz2 = sq_exact(wz);
    const double pd = OR_M_PI * (double)delta;
    const double cAx = ((double)u00 * (-wx2 + 1) - (double)(u01 * wx * wy)) - (double)(u02 * wx * wz);
    const double cBx = ((double)u10 * (-wx2 + 1) - (double)(u11 * wx * wy)) - (double)(u12 * wx * wz);
    const double Ax = -(cAx * (double)nU1 / G + (double)U0 * cBx / G) / OR_M_PI + (double)(2 * wx / tw);
    const double Cx = (double)(-wx * wy * Y1 - wx * wz * Z1) + (1.0 / 2.0) * (-2 * wx2 + 2) * (double)X1;
    const double cAy = ((double)(-u10 * wx * wy) + (double)u11 * (-wy2 + 1)) - (double)(u12 * wy * wz);
    const double cBy = ((double)(-u00 * wx * wy) + (double)u01 * (-wy2 + 1)) - (double)(u02 * wy * wz);
    const double Ay = -((double)U0 * cAy / G + (double)nU1 * cBy / G) / OR_M_PI + (double)(2 * wy / tw);
    const double Cy = (double)(-wx * wy * X1 - wy * wz * Z1) + (1.0 / 2.0) * (-2 * wy2 + 2) * (double)Y1;
    const double cAz = (double)(-u10 * wx * wz - u11 * wy * wz) + (double)u12 * (-wz2 + 1);
    const double cBz = (double)(-u00 * wx * wz - u01 * wy * wz) + (double)u02 * (-wz2 + 1);
    const double Az = -((double)U0 * cAz / G + (double)nU1 * cBz / G) / OR_M_PI + (double)(2 * wz / tw);
    const double Cz = (double)(-wx * wz * X1 - wy * wz * Y1) + (1.0 / 2.0) * (-2 * wz2 + 2) * (double)Z1;
    g[0] = (float)(pd * Ax * cv - Cx / sq);
    g[1] = (float)(pd * Ay * cv - Cy / sq);
    g[2] = (float)(pd * Az * cv - Cz / sq);
}

/* top_bottom_lid.hpp:117-161: max(z - 0.5, (z + 0.5) * -1) (Eigen max = std::max); the gradient's
   condition `z >= 0.5 && (0.0 > z && z >= -0.5)` never holds, so it is always (0, 0, 1) */
static float lid_f(const float p[3]) {
    const float a = p[2] - 0.5f, b = (p[2] + 0.5f) * -1.f;
    return (a < b) ? b : a;
}

/* half_plane.hpp:150-190: (x - plane_point) . plane_vector as an Eigen GEMV (zeroed result,
   columns accumulated in order); gradient -plane_vector where f >= 0, else plane_vector */
static float hp_f(const float p[3], const float* prm) {
    const float d0 = p[0] - prm[3], d1 = p[1] - prm[4], d2 = p[2] - prm[5];
    return ((0.f + d0 * prm[0]) + d1 * prm[1]) + d2 * prm[2];
}
static void hp_g(const float p[3], const float* prm, float g[3]) {
    const float k = hp_f(p, prm) >= 0 ? -1.f : 1.f;   /* exact sign flips of plane_vector */
    g[0] = k * prm[0]; g[1] = k * prm[1]; g[2] = k * prm[2];
}

/* ---------------- tetrahedron.hpp:129-150: min of the four oriented planes (std::min); the
   gradient is the first minimal plane's normal (:152-178).  Planes: getPlanes (:20-120) on the
   corners transformed by the node matrix, computed on the host (oracle/__init__.py). */
static inline float tet_plane(const float* P, int k, const float p[3]) {
    return ((P[4 * k] * p[0] + P[4 * k + 1] * p[1]) + P[4 * k + 2] * p[2]) + P[4 * k + 3];
}
static float tet_f(const float p[3], const float* P) {
    return stdmin(tet_plane(P, 0, p), stdmin(tet_plane(P, 1, p), stdmin(tet_plane(P, 2, p), tet_plane(P, 3, p))));
}
static void tet_g(const float p[3], const float* P, float g[3]) {
    int index = 0;
    float mn = tet_plane(P, 0, p);
    for (int i = 1; i < 4; i++) {
        const float v = tet_plane(P, i, p);
        if (v < mn) { index = i; mn = v; }
    }
    g[0] = P[4 * index]; g[1] = P[4 * index + 1]; g[2] = P[4 * index + 2];
}

/* ---------------- meta_balls_Rydgard.hpp: 4 balls, f = sum (strength/h - subtract)/100 with
   h = 1e-6f + fx^2 + fy^2 + fz^2 (implicit_ball :80-98); the gradient's h sums in double from the
   double literal (gradient_ball :99-124).  1/h is a double division stored to float. */
static float meta_f(const float p[3], const float* P) {
    float out = 0.0f;
    for (int b = 0; b < 4; b++) {
        const float* B = P + 5 * b;
        const float fx = p[0] - B[0], fx2 = fx * fx;
        const float fy = p[1] - B[1], fy2 = fy * fy;
        const float fz = p[2] - B[2], fz2 = fz * fz;
        const float h = (((float)0.000001 + fx2) + fy2) + fz2;
        const float hinv = (float)(1.0 / (double)h);
        const float val = B[3] * hinv - B[4];
        out += val / 100;
    }
    return out;
}
static void meta_g(const float p[3], const float* P, float g[3]) {
    float gx = 0, gy = 0, gz = 0;
    for (int b = 0; b < 4; b++) {
        const float* B = P + 5 * b;
        const float fz = p[2] - B[2], fz2 = fz * fz;
        const float fy = p[1] - B[1], fy2 = fy * fy;
        const float fx = p[0] - B[0], fx2 = fx * fx;
        const float h = (float)(((0.000001 + (double)fx2) + (double)fy2) + (double)fz2);
        const float hinv = (float)(1.0 / (double)h);
        gx += B[3] * (-2 * fx * hinv * hinv) / 100;
        gy += B[3] * (-2 * fy * hinv * hinv) / 100;
        gz += B[3] * (-2 * fz * hinv * hinv) / 100;
    }
    g[0] = gx; g[1] = gy; g[2] = gz;
}

/* ---------------- extrusion.hpp:103-118 -> convex_polygon (2d/GDT/convex_polygon.hpp:97-140):
   f = min_j -(x nx_j + y ny_j - n0_j), first minimal edge on ties; gradient (-nx_w, -ny_w, 0) (the
   2-D gradient leaves the zero-initialised z component) */
static float extr_eval(const float p[3], const float* P, int* which) {
    const int n = (int)P[0];
    float minv = 0.f;
    int w = -1;
    for (int j = 0; j < n; j++) {
        const float v = -((p[0] * P[1 + 3 * j] + p[1] * P[2 + 3 * j]) - P[3 + 3 * j]);
        if (v < minv || w < 0) { minv = v; w = j; }
    }
    *which = w;
    return minv;
}
static float extr_f(const float p[3], const float* P) { int w; return extr_eval(p, P, &w); }
static void extr_g(const float p[3], const float* P, float g[3]) {
    int w;
    extr_eval(p, P, &w);
    g[0] = -P[1 + 3 * w]; g[1] = -P[2 + 3 * w]; g[2] = 0.f;
}

/* ---------------- tree recursion ---------------- */
static float eval1(const or_node* N, int i, const float p[3]) {
    const or_node* n = &N[i];
    float l[3];
    xform(n->minv, p, l);            /* prepare_inner_vectors / x_copy + matrix_vector_product */
    switch (n->type) {
        case OR_UNION: {            /* transformed_union.hpp:33-50 */
            float f1 = eval1(N, n->child[0], l), f2 = eval1(N, n->child[1], l);
            return (f1 > f2) ? f1 : f2;
        }
        case OR_INTERSECTION: {     /* transformed_intersection.hpp:35-51 */
            float f1 = eval1(N, n->child[0], l), f2 = eval1(N, n->child[1], l);
            return (f1 > f2) ? f2 : f1;
        }
        case OR_DIFFERENCE: {       /* transformed_subtract.hpp:36-53 */
            float f1 = eval1(N, n->child[0], l), f2 = eval1(N, n->child[1], l);
            return (f1 < -f2) ? f1 : -f2;
        }
        case OR_ELLIPSOID: return egg_f(l);
        case OR_CUBE: return cube_f(l);
        case OR_CYLINDER: return cyl_f(l);
        case OR_CONE: return cone_f(l);
        case OR_HEART: return heart_f(l);
        case OR_TORUS: return torus_f(l);
        case OR_DMUSHROOM: return dm_f(l);   /* linearly_transformed.hpp:24-33 */
        case OR_SCREW: return screw_f(l, n->prm);
        case OR_LID: return lid_f(l);
        case OR_HALF_PLANE: return hp_f(l, n->prm);
        case OR_TETRA: return tet_f(l, n->prm);
        case OR_METABALLS: return meta_f(l, n->prm);
        case OR_EXTRUSION: return extr_f(l, n->prm);
        case OR_SCREW_TBB: {        /* inf_top_bot_bound.hpp:65-96: imp.min(tbb * -1), std::min */
            const float s = screw_f(l, n->prm), t = lid_f(l) * -1.f;
            return (t < s) ? t : s;
        }
    }
    return NAN;
}

static void grad1(const or_node* N, int i, const float p[3], float o[3]) {
    const or_node* n = &N[i];
    float l[3], g[3];
    xform(n->minv, p, l);
    switch (n->type) {
        case OR_UNION: case OR_INTERSECTION: case OR_DIFFERENCE: {
            float f1 = eval1(N, n->child[0], l), f2 = eval1(N, n->child[1], l);
            float g1[3], g2[3];
            grad1(N, n->child[0], l, g1);
            grad1(N, n->child[1], l, g2);
            int first;
            if (n->type == OR_UNION) first = f1 > f2;                 /* transformed_union.hpp:73 */
            else if (n->type == OR_INTERSECTION) first = !(f1 > f2);  /* transformed_intersection.hpp:79 */
            else { g2[0] = -g2[0]; g2[1] = -g2[1]; g2[2] = -g2[2]; first = f1 < -f2; }  /* subtract :79-93 */
            memcpy(g, first ? g1 : g2, sizeof g);
            break;
        }
        case OR_ELLIPSOID: egg_g(l, g); break;
        case OR_CUBE: cube_g(l, g); break;
        case OR_CYLINDER: cyl_g(l, g); break;
        case OR_CONE: cone_g(l, g); break;
        case OR_HEART: heart_g(l, g); break;
        case OR_TORUS: torus_g(l, g); break;
        case OR_DMUSHROOM: dm_g(l, g); break;
        case OR_SCREW: screw_g(l, n->prm, g); break;
        case OR_LID: g[0] = 0.f; g[1] = 0.f; g[2] = 1.f; break;
        case OR_HALF_PLANE: hp_g(l, n->prm, g); break;
        case OR_TETRA: tet_g(l, n->prm, g); break;
        case OR_METABALLS: meta_g(l, n->prm, g); break;
        case OR_EXTRUSION: extr_g(l, n->prm, g); break;
        case OR_SCREW_TBB:          /* inf_top_bot_bound.hpp:142-166 over screw.hpp:450-486 */
            if (l[2] >= 0.5) { g[0] = 0.f; g[1] = 0.f; g[2] = -1.f; }
            else if (l[2] <= -0.5) { g[0] = 0.f; g[1] = 0.f; g[2] = 1.f; }
            else {
                float gs[3];
                screw_g(l, n->prm, gs);
                grad_xform(n->minv, gs, g);   /* the screw's own M^-T; the node's follows below */
            }
            break;
        default: g[0] = g[1] = g[2] = NAN;
    }
    grad_xform(n->minv, g, o);
}

void or_eval(const or_node* nodes, int root, const float* xyz, int64_t n, float* f_out) {
    for (int64_t k = 0; k < n; k++) f_out[k] = eval1(nodes, root, xyz + 3 * k);
}

void or_grad(const or_node* nodes, int root, const float* xyz, int64_t n, float* g_out) {
    for (int64_t k = 0; k < n; k++) grad1(nodes, root, xyz + 3 * k, g_out + 3 * k);
}

/* ---------------- glibc 2.35 sysdeps/ieee754/flt-32/e_acosf.c (fdlibm) ---------------- */
float or_acosf(float x) {
    static const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f,
                       pio2_lo = 7.5497894159e-08f, pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f,
                       pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f,
                       pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
                       qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
    float z, p, q, r, w, s, c, df;
    int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return (hx > 0) ? 0.0f : pi + 2.0f * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        z = x * x;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {
        z = (one + x) * 0.5f;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        s = sqrtf(z);
        r = p / q;
        w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    } else {
        z = (one - x) * 0.5f;
        s = sqrtf(z);
        df = bitsf(fbits(s) & 0xfffff000u);
        c = (z - df * df) / (s + df);
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        w = r * s + c;
        return 2.0f * (df + w);
    }
}

/* self-check of the restatement against the host libm's acosf (glibc 2.35 in this image):
 * number of mismatching bit patterns among start, start+stride, ... (count values) */
int64_t or_acosf_check(uint32_t start, uint32_t stride, uint64_t count) {
    int64_t bad = 0;
    uint32_t u = start;
    for (uint64_t k = 0; k < count; k++, u += stride) {
        const float x = bitsf(u);
        const float a = or_acosf(x), b = acosf(x);
        if (!(fbits(a) == fbits(b) || (a != a && b != b))) bad++;
    }
    return bad;
}
