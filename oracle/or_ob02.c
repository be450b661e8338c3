/*
 * or_ob02.c -- oracle restatement of the Ohtake-Belyaev loop, steps 1-3 (TEST INFRA ONLY).
 *
 *   step 1  apply_vertex_resampling_to_MC_buffers__VMS   apply_v_s_to_mc_buffers.hpp:280-326
 *           -> process2_vertex_resampling_relaxation_v1  vertex_resampling.hpp:152-225
 *   step 2  centroids_projection                         centroids_projection.cpp:1219-1311
 *           -> set_centers_on_surface                    centroids_projection.cpp:421-1214
 *           -> bisection                                 polygoniser/bisection.hpp:117-459
 *           -> vertex_apply_qem                          qem.hpp:321-599 (Eigen JacobiSVD restated)
 *   step 3  my_subdiv_                                   centroids_projection.cpp:1314-1367
 *           -> subdivide_multiple_facets_1to4            subdivision/subdiv_1to4.hpp:44-488
 *           -> randomize_verts                           basic_functions.hpp:551-557 (glibc rand())
 *
 * Intended-semantics decisions (documented in DESIGN.md "reference UB"):
 *  - make_edge_lookup (mesh_algorithms.hpp:50-110) inserts its long key through pair<int,int>, so
 *    keys >= 2^31 (meshes with more than ~53k faces) are truncated and never found again, which
 *    leads to out-of-bounds writes.  We implement the intended lookup (first/last face per edge).
 *  - the same function stores the int edge id in edges_of_faces, a multi_array of short_edge_type
 *    = short int (basic_data_structures.hpp:196-197; mesh_algorithms.hpp:92,100).  Edge ids >= 2^15
 *    wrap: ids 32768..65535 become negative, 65536..98303 alias edges 0..32767, and so on.
 *    build_faces_of_faces (mesh_algorithms.hpp:111-131) then indexes faces_of_edges with the wrapped
 *    id -- an out-of-bounds read (negative) or another edge's faces (aliased).  Any mesh with more
 *    than 32767 edges, i.e. F > 21845 faces, is affected (config 2 at R = 128: F = 113 360; config 3
 *    at R = 256: F = 179 656).  We keep the full int edge id.  OB02 parity for such meshes is parity
 *    against the reference's intended semantics, not against what its binary would compute.
 *  - compute_average_edge_length starts from an uninitialised float (centroids_projection.cpp:72);
 *    we start from 0.
 *  - create_directions_bundle slices alpha_list_full.begin()+10 even when the list is shorter
 *    (centroids_projection.cpp:211); we clamp to the list length.
 *  - bisection has no iteration cap (bisection.hpp:190-378); we stop after OR_BISECT_CAP rounds.
 */
#include "oracle.h"

#include <limits.h>

#define MAX_ALPHA_HALVINGS 200   /* ob02_device.hpp kMaxHalvings */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ROOT_TOL ((float)(0.001 / 10.0))   /* configs.hpp:33 ROOT_TOLERANCE */
#define OR_BISECT_CAP 200

static inline float norm2f(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

/* implicit_vectorised_algorithms.hpp:161-171 */
static void centroids_of(const float* v, const int32_t* f, int64_t nf, float* c) {
    for (int64_t j = 0; j < nf; j++) {
        const int32_t a = f[3 * j], b = f[3 * j + 1], d = f[3 * j + 2];
        for (int k = 0; k < 3; k++) c[3 * j + k] = (v[3 * a + k] + v[3 * b + k] + v[3 * d + k]) / (float)(3.0);
    }
}

/* normalise_inplace.hpp:60-70 normalize_1111 */
static void normalize_1111(float* a, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        float nm = norm2f(a[3 * i], a[3 * i + 1], a[3 * i + 2]);
        for (int k = 0; k < 3; k++) a[3 * i + k] = a[3 * i + k] / nm;
    }
}

/* normalise_inplace.hpp:26-54 normalise_inplace */
static void normalise_inplace1(float* a, float min_norm) {
    float nm = norm2f(a[0], a[1], a[2]);
    nm = (nm < min_norm) ? (float)1.0 : nm;
    float factor = (float)(1.0 / (double)nm);
    a[0] = a[0] * factor; a[1] = a[1] * factor; a[2] = a[2] * factor;
}

/* mesh_algorithms.hpp:178-209 make_neighbour_faces_of_vertex, as CSR (ascending face order) */
static int umbrellas(const int32_t* f, int64_t nf, int64_t nv, int64_t** off_o, int32_t** lst_o) {
    int64_t* off = (int64_t*)calloc((size_t)nv + 1, sizeof(int64_t));
    int32_t* lst = (int32_t*)malloc(sizeof(int32_t) * (size_t)(3 * nf + 1));
    int64_t* fill = (int64_t*)calloc((size_t)nv + 1, sizeof(int64_t));
    if (!off || !lst || !fill) { free(off); free(lst); free(fill); return -1; }
    for (int64_t j = 0; j < 3 * nf; j++) off[f[j] + 1]++;
    for (int64_t i = 0; i < nv; i++) off[i + 1] += off[i];
    for (int64_t j = 0; j < nf; j++)
        for (int s = 0; s < 3; s++) { int32_t v = f[3 * j + s]; lst[off[v] + fill[v]++] = (int32_t)j; }
    free(fill);
    *off_o = off; *lst_o = lst;
    return 0;
}

/* mesh_algorithms.hpp:50-131: faces_of_faces with the reference's first/last rule.
   faces_of_edges[e] = [first face, last face seen]; [1] is value-initialised 0 (boost multi_array). */
typedef struct { int64_t key; int32_t first, last; } edge_rec;
static int faces_of_faces(const int32_t* f, int64_t nf, int64_t nv, int32_t* fof) {
    int64_t cap = 1; while (cap < 4 * nf + 16) cap <<= 1;
    edge_rec* tab = (edge_rec*)malloc(sizeof(edge_rec) * (size_t)cap);
    int64_t* eof = (int64_t*)malloc(sizeof(int64_t) * (size_t)(3 * nf + 1));
    if (!tab || !eof) { free(tab); free(eof); return -1; }
    for (int64_t i = 0; i < cap; i++) tab[i].key = -1;
    for (int64_t fi = 0; fi < nf; fi++)
        for (int vj = 0; vj < 3; vj++) {
            int64_t e1 = f[3 * fi + vj], e2 = f[3 * fi + (vj + 1) % 3];
            int64_t key = (e2 > e1) ? e1 + e2 * nv : e2 + e1 * nv;
            uint64_t h = (uint64_t)key * 0x9E3779B97F4A7C15ull;
            int64_t s = (int64_t)(h >> 17) & (cap - 1);
            while (tab[s].key != -1 && tab[s].key != key) s = (s + 1) & (cap - 1);
            if (tab[s].key == -1) { tab[s].key = key; tab[s].first = (int32_t)fi; tab[s].last = 0; }
            else tab[s].last = (int32_t)fi;
            eof[3 * fi + vj] = s;
        }
    for (int64_t fi = 0; fi < nf; fi++)
        for (int e = 0; e < 3; e++) {
            const edge_rec* r = &tab[eof[3 * fi + e]];
            fof[3 * fi + e] = (r->first != fi) ? r->first : r->last;
        }
    free(tab); free(eof);
    return 0;
}

/* vertex_resampling.hpp:47-77 kij */
static float kij(int64_t i, int64_t j, const float* C, const float* N) {
    float mimj = N[3 * i] * N[3 * j] + N[3 * i + 1] * N[3 * j + 1] + N[3 * i + 2] * N[3 * j + 2];
    if (mimj > 1.0) mimj = 1.0f;
    if (mimj < -1.0) mimj = -1.0f;
    float pipj = norm2f(C[3 * i] - C[3 * j], C[3 * i + 1] - C[3 * j + 1], C[3 * i + 2] - C[3 * j + 2]);
    if (pipj == 0) return 0;
    return or_acosf(mimj) / pipj;
}

int or_vertex_resampling(const or_node* nodes, int root, float c, float* verts, int64_t nv,
                         const int32_t* faces, int64_t nf, float* centroids_out) {
    float* C = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    float* N = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    float* W = (float*)malloc(sizeof(float) * (size_t)nf + 4);
    int32_t* fof = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)nf + 4);
    float* nvv = (float*)malloc(sizeof(float) * 3 * (size_t)nv + 4);
    int64_t* off = NULL; int32_t* lst = NULL;
    int rc = -1;
    if (!C || !N || !W || !fof || !nvv) goto done;
    centroids_of(verts, faces, nf, C);
    or_grad(nodes, root, C, nf, N);                 /* vertex_resampling.hpp:187-189 */
    normalize_1111(N, nf);
    if (umbrellas(faces, nf, nv, &off, &lst)) goto done;
    if (faces_of_faces(faces, nf, nv, fof)) goto done;
    for (int64_t i = 0; i < nf; i++) {              /* wi, vertex_resampling.hpp:79-91 */
        float ki = 0;
        for (int j = 0; j < 3; j++) ki += kij(i, fof[3 * i + j], C, N);
        W[i] = (float)(1.0 + (double)(c * ki));
    }
    for (int64_t v = 0; v < nv; v++) {              /* vertex_resampling_VV1 :108-140 */
        float sum_w = 0;
        for (int64_t k = off[v]; k < off[v + 1]; k++) sum_w += W[lst[k]];
        float x = 0, y = 0, z = 0;
        for (int64_t k = off[v]; k < off[v + 1]; k++) {
            int32_t fj = lst[k];
            float w = W[fj] / sum_w;
            x += w * C[3 * fj]; y += w * C[3 * fj + 1]; z += w * C[3 * fj + 2];
        }
        nvv[3 * v] = x; nvv[3 * v + 1] = y; nvv[3 * v + 2] = z;
    }
    memcpy(verts, nvv, sizeof(float) * 3 * (size_t)nv);
    if (centroids_out) memcpy(centroids_out, C, sizeof(float) * 3 * (size_t)nf);
    rc = 0;
done:
    free(C); free(N); free(W); free(fof); free(nvv); free(off); free(lst);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* boost::random::mt11213b seeded 12 + uniform_01<float> (vectorised_algorithms/make_random_pm1.hpp) */
typedef struct { uint32_t x[351]; int i; } mt11213b;
static void mt_seed(mt11213b* m, uint32_t s) {
    m->x[0] = s;
    for (int i = 1; i < 351; i++) m->x[i] = 1812433253u * (m->x[i - 1] ^ (m->x[i - 1] >> 30)) + (uint32_t)i;
    m->i = 351;
}
static uint32_t mt_next(mt11213b* m) {
    const int n = 351, mm = 175;
    const uint32_t upper = 0xffffffffu << 19, lower = ~upper, a = 0xccab8ee7u;
    if (m->i >= n) {
        for (int k = 0; k < n; k++) {
            uint32_t y = (m->x[k] & upper) | (m->x[(k + 1) % n] & lower);
            m->x[k] = m->x[(k + mm) % n] ^ (y >> 1) ^ ((y & 1u) ? a : 0u);
        }
        m->i = 0;
    }
    uint32_t z = m->x[m->i++];
    z ^= (z >> 11) & 0xffffffffu;
    z ^= (z << 7) & 0x31b6ab00u;
    z ^= (z << 15) & 0xffe50000u;
    z ^= (z >> 17);
    return z;
}
static float uniform01f(mt11213b* m) {
    const float factor = 1.0f / ((float)4294967295u + 1.0f);
    for (;;) {
        float r = (float)mt_next(m) * factor;
        if (r < 1.0f) return r;
    }
}

/* make_alpha_list centroids_projection.cpp:144-194 */
static int make_alpha_list(float initial_step, float min_step, float max_dist, int max_iter, float** out) {
    int cap = 64, n = 0;
    float* a = (float*)malloc(sizeof(float) * cap);
    float unit = max_dist, step = initial_step;
    int halvings = 0;
    /* the reference loops forever on an infinite average; the library stops after
       MAX_ALPHA_HALVINGS halvings (any finite average ends within 140) */
    while (step > min_step && halvings++ < MAX_ALPHA_HALVINGS) {
        step = (float)(step * 0.5);
        const double q = floor((double)(max_dist / fabsf(step)) + 0.001);
        /* (int) of a double as x86's cvttsd2si, the reference build's conversion: out of range or
           NaN gives INT_MIN (undefined behaviour in C, so spelled out; found by the sanitizer run) */
        int total = (q >= -2147483648.0 && q < 2147483648.0) ? (int)q : INT_MIN;
        int ms = (max_iter < total) ? max_iter : total;
        for (int i = 1; i < ms + 1; i += 2) {
            float alpha = (float)i * step;
            if (n + 2 > cap) { cap *= 2; a = (float*)realloc(a, sizeof(float) * cap); }
            a[n++] = alpha / unit;
            a[n++] = -alpha / unit;
        }
    }
    *out = a;
    return n;
}

static inline float get_sign(float v) { return (v > ROOT_TOL) ? 1.f : (v < -ROOT_TOL) ? -1.f : 0.f; }

static inline void cross3(const float* a, const float* b, float* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* produce_facet_normals implicit_vectorised_algorithms.hpp:52-133 (force_normalisation=true) */
static void facet_normals(const float* v, const int32_t* f, int64_t nf, float* out) {
    /* configs.hpp:57-65: MICROMETER = 1.0f/1000.0, NANOMETER = MICROMETER/1000.0 (double ops,
       stored as float), MIN_AREA = (30*NANOMETER)^2 in float */
    const float micrometer = (float)(1.0 / 1000.0);
    const float nanometer = (float)((double)micrometer / 1000.0);
    const float min_area = (30 * nanometer) * (30 * nanometer);
    const float min_norm_sq = min_area * min_area;
    const float osqrt3 = (float)(1.0 / (double)sqrtf((float)3.0));
    for (int64_t fi = 0; fi < nf; fi++) {
        const float* p0 = v + 3 * f[3 * fi]; const float* p1 = v + 3 * f[3 * fi + 1]; const float* p2 = v + 3 * f[3 * fi + 2];
        float x1 = p1[0] - p0[0], y1 = p1[1] - p0[1], z1 = p1[2] - p0[2];
        float x2 = p2[0] - p0[0], y2 = p2[1] - p0[1], z2 = p2[2] - p0[2];
        float x = y1 * z2 - z1 * y2, y = z1 * x2 - x1 * z2, z = x1 * y2 - y1 * x2;
        float n2 = x * x + y * y + z * z;
        if (n2 < min_norm_sq) { x = osqrt3; y = osqrt3; z = osqrt3; }
        else { float n = sqrtf(n2); x = x / n; y = y / n; z = z / n; }
        out[3 * fi] = x; out[3 * fi + 1] = y; out[3 * fi + 2] = z;
    }
}

/* set_centers_on_surface, per centroid (the reference's vectorised passes are independent per
   centroid: a centroid stays active until its first (type, alpha) trial whose sign product is
   <= 0, centroids_projection.cpp:604-892). */
static void set_centers_on_surface(const or_node* nodes, int root, const float* X, int64_t n,
                                   float max_dist, const float* fnorm, float* out) {
    const float min_grad = 0.000001f;
    float* alphas = NULL;
    int nal = make_alpha_list((float)(max_dist * 1.0), (float)(0.001 * 1.0), max_dist, 20, &alphas);
    int n10 = nal < 10 ? nal : 10;
    float* fc = (float*)malloc(sizeof(float) * n + 4);
    float* g = (float*)malloc(sizeof(float) * 3 * n + 4);
    float* pert = (float*)malloc(sizeof(float) * 3 * n + 4);
    or_eval(nodes, root, X, n, fc);
    or_grad(nodes, root, X, n, g);
    /* perturbation for direction type 2 (make_random_pm1(count,3,1e-6), seed 12), drawn in order */
    {
        mt11213b m; mt_seed(&m, 12);
        const float R = 0.000001f;
        for (int64_t i = 0; i < 3 * n; i++) pert[i] = (float)(((double)uniform01f(&m) * 2.0 - 1.0) * (double)R);
    }
    for (int64_t j = 0; j < n; j++) {
        const float* x = X + 3 * j;
        float gd[3] = {g[3 * j], g[3 * j + 1], g[3 * j + 2]};
        normalise_inplace1(gd, min_grad);
        float sc = get_sign(fc[j]);
        if (sc < 0.0) { gd[0] = -gd[0]; gd[1] = -gd[1]; gd[2] = -gd[2]; }
        float d0[3] = {-gd[0] * sc, -gd[1] * sc, -gd[2] * sc};
        /* directions per type */
        float d2[3], d3[3];
        {
            float z[3]; cross3(fnorm + 3 * j, pert + 3 * j, z);
            float nm = norm2f(z[0], z[1], z[2]);
            d2[0] = z[0] / nm; d2[1] = z[1] / nm; d2[2] = z[2] / nm;   /* normalize_1111 */
            /* replace_zero_normals_with_gaussian_random never fires on normalised facet normals */
            cross3(fnorm + 3 * j, d2, d3);
            normalise_inplace1(d3, min_grad);
        }
        int found = 0;
        float best[3] = {x[0], x[1], x[2]};
        for (int t = 0; t < 7 && !found; t++) {
            const float* d;
            float ax[3];
            int na = (t == 0) ? nal : n10;
            if (t == 0) d = d0;
            else if (t == 1) d = fnorm + 3 * j;
            else if (t == 2) d = d2;
            else if (t == 3) d = d3;
            else { ax[0] = (t == 4) ? 1.f : 0.f; ax[1] = (t == 5) ? 1.f : 0.f; ax[2] = (t == 6) ? 1.f : 0.f; d = ax; }
            for (int ai = 0; ai < na; ai++) {
                float cc = (float)(((double)(max_dist * alphas[ai]) * 4.0) / 4.0);
                float p[3] = {x[0] + cc * d[0], x[1] + cc * d[1], x[2] + cc * d[2]};
                float fa;
                or_eval(nodes, root, p, 1, &fa);
                if (get_sign(fa) * sc <= 0) { found = 1; best[0] = p[0]; best[1] = p[1]; best[2] = p[2]; break; }
            }
        }
        /* :904-1191 */
        float f1 = fc[j], f2;
        or_eval(nodes, root, best, 1, &f2);
        int z2 = fabsf(f2) <= ROOT_TOL, z1 = fabsf(f1) <= ROOT_TOL;
        if (z1) { best[0] = x[0]; best[1] = x[1]; best[2] = x[2]; }
        float* o = out + 3 * j;
        if (found && !(z1 || z2)) {
            float x1[3] = {x[0], x[1], x[2]}, x2[3] = {best[0], best[1], best[2]};
            float fb;
            or_eval(nodes, root, x2, 1, &fb);
            if (fb < -ROOT_TOL) { float t3[3]; memcpy(t3, x1, 12); memcpy(x1, x2, 12); memcpy(x2, t3, 12); }
            /* bisection.hpp:190-378, per point */
            float mid[3] = {x1[0], x1[1], x1[2]};
            for (int it = 0; it < OR_BISECT_CAP; it++) {
                for (int k = 0; k < 3; k++) mid[k] = (float)((double)(x1[k] + x2[k]) / 2.);
                float vm;
                or_eval(nodes, root, mid, 1, &vm);
                if (fabsf(vm) <= ROOT_TOL) break;
                if (vm < -ROOT_TOL) memcpy(x1, mid, 12);
                if (vm > +ROOT_TOL) memcpy(x2, mid, 12);
            }
            o[0] = mid[0]; o[1] = mid[1]; o[2] = mid[2];
        } else if (z1 || z2) {
            o[0] = best[0]; o[1] = best[1]; o[2] = best[2];
        } else {
            o[0] = x[0]; o[1] = x[1]; o[2] = x[2];
        }
    }
    free(alphas); free(fc); free(g); free(pert);
}

/* ------------------------------------------------------------------------------------------ */
/* Eigen 3.3 JacobiSVD<Matrix3f>(A, ComputeFullU|ComputeFullV) restated (Eigen/src/SVD/JacobiSVD.h,
   Eigen/src/Jacobi/Jacobi.h).  Column-major 3x3 float, scalar paths (fixed size 3 is not
   vectorised).  PARITY UNPINNED: the Eigen version the reference used is not recorded. */
typedef struct { float c, s; } jrot;
static inline void rot_rows(float W[3][3], int p, int q, jrot j) {   /* applyOnTheLeft */
    if (j.c == 1.f && j.s == 0.f) return;
    for (int k = 0; k < 3; k++) {
        float xi = W[p][k], yi = W[q][k];
        W[p][k] = j.c * xi + j.s * yi;
        W[q][k] = -j.s * xi + j.c * yi;
    }
}
static inline void rot_cols(float W[3][3], int p, int q, jrot j) {   /* apply_rotation_in_the_plane on columns */
    if (j.c == 1.f && j.s == 0.f) return;
    for (int k = 0; k < 3; k++) {
        float xi = W[k][p], yi = W[k][q];
        W[k][p] = j.c * xi + j.s * yi;
        W[k][q] = -j.s * xi + j.c * yi;
    }
}
static jrot make_jacobi(float x, float y, float z) {
    jrot r;
    float deno = 2.f * fabsf(y);
    if (deno < 1.17549435e-38f) { r.c = 1.f; r.s = 0.f; return r; }
    float tau = (x - z) / deno;
    float w = sqrtf(tau * tau + 1.f);
    float t = (tau > 0.f) ? 1.f / (tau + w) : 1.f / (tau - w);
    float sign_t = t > 0.f ? 1.f : -1.f;
    float n = 1.f / sqrtf(t * t + 1.f);
    r.s = -sign_t * (y / fabsf(y)) * fabsf(t) * n;
    r.c = n;
    return r;
}
static void real_2x2_jacobi_svd(float W[3][3], int p, int q, jrot* jl, jrot* jr) {
    float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
    jrot rot1;
    float t = m00 + m11, d = m10 - m01;
    if (fabsf(d) < 1.17549435e-38f) { rot1.s = 0.f; rot1.c = 1.f; }
    else { float u = t / d; float tmp = sqrtf(1.f + u * u); rot1.s = 1.f / tmp; rot1.c = u / tmp; }
    /* m.applyOnTheLeft(0,1,rot1) */
    if (!(rot1.c == 1.f && rot1.s == 0.f)) {
        float a0 = m00, b0 = m10, a1 = m01, b1 = m11;
        m00 = rot1.c * a0 + rot1.s * b0; m10 = -rot1.s * a0 + rot1.c * b0;
        m01 = rot1.c * a1 + rot1.s * b1; m11 = -rot1.s * a1 + rot1.c * b1;
    }
    *jr = make_jacobi(m00, m01, m11);
    /* j_left = rot1 * j_right.transpose();  (c1 c2 - s1 s2, c1 s2 + s1 c2) with s2 -> -s_r */
    jrot rt = {jr->c, -jr->s};
    jl->c = rot1.c * rt.c - rot1.s * rt.s;
    jl->s = rot1.c * rt.s + rot1.s * rt.c;
}
/* returns rank with threshold; S sorted descending, U, V column-major as W[row][col] */
static int jacobi_svd3(const float A[3][3], float thr, float S[3], float U[3][3], float V[3][3]) {
    const float precision = 2.f * 1.1920929e-07f, consider_zero = 1.17549435e-38f;
    float scale = 0.f;
    for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) { float a = fabsf(A[r][c]); if (a > scale) scale = a; }
    if (scale == 0.f) scale = 1.f;
    float W[3][3];
    for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) { W[r][c] = A[r][c] / scale; U[r][c] = (r == c); V[r][c] = (r == c); }
    float maxd = 0.f;
    for (int i = 0; i < 3; i++) { float a = fabsf(W[i][i]); if (a > maxd) maxd = a; }
    int finished = 0, sweeps = 0;
    while (!finished && sweeps < 100) {
        finished = 1; sweeps++;
        for (int p = 1; p < 3; p++)
            for (int q = 0; q < p; q++) {
                float threshold = consider_zero > precision * maxd ? consider_zero : precision * maxd;
                if (fabsf(W[p][q]) > threshold || fabsf(W[q][p]) > threshold) {
                    finished = 0;
                    jrot jl, jr;
                    real_2x2_jacobi_svd(W, p, q, &jl, &jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, jl);                          /* U.applyOnTheRight(p,q,jl^T) */
                    jrot jrt = {jr.c, -jr.s};
                    rot_cols(W, p, q, jrt);                         /* W.applyOnTheRight(p,q,jr) */
                    rot_cols(V, p, q, jrt);
                    float a = fabsf(W[p][p]), b = fabsf(W[q][q]);
                    float mx = a > b ? a : b;
                    if (mx > maxd) maxd = mx;
                }
            }
    }
    for (int i = 0; i < 3; i++) {
        float a = W[i][i];
        S[i] = fabsf(a);
        if (a < 0.f) for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < 3; i++) S[i] *= scale;
    int nonzero = 3;
    for (int i = 0; i < 3; i++) {
        int pos = i; float mx = S[i];
        for (int k = i + 1; k < 3; k++) if (S[k] > mx) { mx = S[k]; pos = k; }
        if (mx == 0.f) { nonzero = i; break; }
        if (pos != i) {
            float t = S[i]; S[i] = S[pos]; S[pos] = t;
            for (int r = 0; r < 3; r++) { t = U[r][i]; U[r][i] = U[r][pos]; U[r][pos] = t; t = V[r][i]; V[r][i] = V[r][pos]; V[r][pos] = t; }
        }
    }
    float pt = S[0] * thr; if (pt < consider_zero) pt = consider_zero;
    int i = nonzero - 1;
    while (i >= 0 && S[i] < pt) --i;
    return i + 1;
}

/* qem.hpp:256-316 get_A_b and :321-599 vertex_apply_qem for one vertex */
static void qem_vertex(float* v, const int32_t* ul, int64_t deg, const float* C, const float* N, float maxd) {
    float A[3][3] = {{0}}, b[3] = {0, 0, 0};
    const float ox = v[0], oy = v[1], oz = v[2];
    for (int64_t i = 0; i < deg; i++) {
        int32_t ni = ul[i];
        float nx = N[3 * ni], ny = N[3 * ni + 1], nz = N[3 * ni + 2];
        float Px = C[3 * ni] - ox, Py = C[3 * ni + 1] - oy, Pz = C[3 * ni + 2] - oz;
        float nn00 = nx * nx, nn01 = nx * ny, nn02 = nx * nz, nn11 = ny * ny, nn12 = ny * nz, nn22 = nz * nz;
        A[0][0] += nn00; A[0][1] += nn01; A[0][2] += nn02;
        A[1][0] += nn01; A[1][1] += nn11; A[1][2] += nn12;
        A[2][2] += nn22; A[2][0] += nn02; A[2][1] += nn12;
        b[0] -= nn00 * Px + nn01 * Py + nn02 * Pz;
        b[1] -= nn01 * Px + nn11 * Py + nn12 * Pz;
        b[2] -= nn02 * Px + nn12 * Py + nn22 * Pz;
    }
    float S[3], U[3][3], V[3][3];
    int rank = jacobi_svd3((const float(*)[3])A, (float)(1.0 / 680.0), S, U, V);
    /* y = V^T(0) = 0 ; utb = -U^T b  (Eigen coeff-product redux order a0 + (a1 + a2)) */
    float y[3] = {0.f, 0.f, 0.f};
    float utb[3];
    for (int i = 0; i < 3; i++) utb[i] = (-U[0][i]) * b[0] + ((-U[1][i]) * b[1] + (-U[2][i]) * b[2]);
    for (int i = 0; i < rank; i++) y[i] = utb[i] / S[i];
    /* new_x = V * y + origin (Vt^T == matrixV) */
    float nx[3];
    for (int r = 0; r < 3; r++) nx[r] = (V[r][0] * y[0] + (V[r][1] * y[1] + V[r][2] * y[2])) + v[r];
    if (maxd > 0) {
        float dx = nx[0] - v[0], dy = nx[1] - v[1], dz = nx[2] - v[2];
        float dist2 = dx * dx + dy * dy + dz * dz;
        if (dist2 <= maxd * maxd) { v[0] = nx[0]; v[1] = nx[1]; v[2] = nx[2]; }
        else {
            float dist = sqrtf(dist2);
            float len = (float)(maxd * 1.5);
            if (len > dist) len = dist;
            v[0] += dx / dist * len; v[1] += dy / dist * len; v[2] += dz / dist * len;
        }
    } else { v[0] = nx[0]; v[1] = nx[1]; v[2] = nx[2]; }
}

int or_centroids_projection(const or_node* nodes, int root, float* verts, int64_t nv,
                            const int32_t* faces, int64_t nf, int enable_qem,
                            float* centroids_out, float* avg_edge_out) {
    float* C = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    float* FN = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    float* P = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    float* G = (float*)malloc(sizeof(float) * 3 * (size_t)nf + 4);
    int64_t* off = NULL; int32_t* lst = NULL;
    int rc = -1;
    if (!C || !FN || !P || !G) goto done;
    /* compute_average_edge_length centroids_projection.cpp:70-82 (start value defined as 0) */
    float el = 0.f;
    for (int64_t j = 0; j < nf; j++) {
        const float* a = verts + 3 * faces[3 * j]; const float* b = verts + 3 * faces[3 * j + 1];
        const float* c = verts + 3 * faces[3 * j + 2];
        el += norm2f(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
        el += norm2f(a[0] - c[0], a[1] - c[1], a[2] - c[2]);
        el += norm2f(c[0] - b[0], c[1] - b[1], c[2] - b[2]);
    }
    float avg = (float)((double)el / (3. * (double)nf));
    if (avg_edge_out) *avg_edge_out = avg;
    centroids_of(verts, faces, nf, C);
    facet_normals(verts, faces, nf, FN);
    set_centers_on_surface(nodes, root, C, nf, avg, FN, P);
    if (centroids_out) memcpy(centroids_out, P, sizeof(float) * 3 * (size_t)nf);
    if (enable_qem) {
        or_grad(nodes, root, P, nf, G);          /* compute_centroid_gradient :1262 */
        normalize_1111(G, nf);
        if (umbrellas(faces, nf, nv, &off, &lst)) goto done;
        for (int64_t vi = 0; vi < nv; vi++)
            qem_vertex(verts + 3 * vi, lst + off[vi], off[vi + 1] - off[vi], P, G, avg);
    }
    rc = 0;
done:
    free(C); free(FN); free(P); free(G); free(off); free(lst);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* step 3: my_subdiv_ (centroids_projection.cpp:1314-1367).  subdivide_given_faces
   (subdivision/do_subdivision.hpp:26-45) requests every face and returns right after the first
   subdivide_multiple_facets_1to4 (subdiv_1to4.hpp:44-488); randomize_verts (basic_functions.hpp:551-557)
   then adds glibc rand() noise.  The midpoint map (std::map keyed by easy_edge, mesh_algorithms.hpp:46)
   assigns new vertex ids in order of first appearance over (face ascending, e01, e12, e20).
   easy_edge's base 1e6 (configs.hpp:62) makes keys collide beyond 1e6 vertices; the intended
   (min, max) identity is used. */
typedef struct { uint64_t key; int32_t vid; } sub_slot;

static int32_t* sub_lookup(sub_slot* tab, uint64_t mask, uint64_t key, int* inserted) {
    uint64_t s = (key * 0x9E3779B97F4A7C15ull >> 17) & mask;
    while (tab[s].key != ~0ull && tab[s].key != key) s = (s + 1) & mask;
    *inserted = tab[s].key == ~0ull;
    tab[s].key = key;
    return &tab[s].vid;
}

/* Eigen 3.3 lazy 3x3 product T * new_vert_maker (subdiv_1to4.hpp:277-330): coefficient sums are
   reduced as a0 + (a1 + a2) (Redux.h redux_novec_unroller), zero terms included */
static inline float mid3(float a0, float a1, float a2, float w0, float w1, float w2) {
    return a0 * w0 + (a1 * w1 + a2 * w2);
}

int or_subdivide(const float* verts, int64_t nv, const int32_t* faces, int64_t nf, float amplitude,
                 float** vout, int64_t* nv_out, int32_t** fout) {
    uint64_t cap = 1024;
    while (cap < (uint64_t)(4 * nf + 16)) cap <<= 1;
    sub_slot* tab = (sub_slot*)malloc(sizeof(sub_slot) * cap);
    int32_t* mids = (int32_t*)malloc(sizeof(int32_t) * (size_t)(3 * nf + 1));
    unsigned char* ins = (unsigned char*)malloc((size_t)(3 * nf + 1));
    if (!tab || !mids || !ins) { free(tab); free(mids); free(ins); return -1; }
    memset(tab, 0xff, sizeof(sub_slot) * cap);
    int64_t counter = nv;
    for (int64_t fi = 0; fi < nf; fi++) {          /* subdiv_1to4.hpp:147-232 */
        for (int k = 0; k < 3; k++) {
            const uint64_t a = (uint32_t)faces[3 * fi + k], b = (uint32_t)faces[3 * fi + (k + 1) % 3];
            const uint64_t key = a <= b ? (a << 32 | b) : (b << 32 | a);
            int inserted;
            int32_t* vid = sub_lookup(tab, cap - 1, key, &inserted);
            if (inserted) *vid = (int32_t)counter++;
            mids[3 * fi + k] = *vid;
            ins[3 * fi + k] = (unsigned char)inserted;
        }
    }
    float* V = (float*)malloc(sizeof(float) * 3 * (size_t)(counter + 1));
    int32_t* F = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)(4 * nf + 1));
    if (!V || !F) { free(tab); free(mids); free(ins); free(V); free(F); return -1; }
    memcpy(V, verts, sizeof(float) * 3 * (size_t)nv);
    const float H = 0.5f, O = 0.0f;
    /* new_vert_maker << H,O,H, H,H,O, O,H,H: columns m01 = (H,H,O), m12 = (O,H,H), m20 = (H,O,H) */
    const float W[3][3] = {{H, H, O}, {O, H, H}, {H, O, H}};
    int64_t nvt = nv;
    for (int64_t fi = 0; fi < nf; fi++) {          /* :277-330 */
        const float* p0 = verts + 3 * faces[3 * fi];
        const float* p1 = verts + 3 * faces[3 * fi + 1];
        const float* p2 = verts + 3 * faces[3 * fi + 2];
        for (int k = 0; k < 3; k++) {
            if (!ins[3 * fi + k]) continue;
            for (int r = 0; r < 3; r++) V[3 * nvt + r] = mid3(p0[r], p1[r], p2[r], W[k][0], W[k][1], W[k][2]);
            nvt++;
        }
    }
    memcpy(F, faces, sizeof(int32_t) * 3 * (size_t)nf);
    for (int64_t fi = 0; fi < nf; fi++) {          /* :380-470 */
        const int32_t v0 = faces[3 * fi], v1 = faces[3 * fi + 1], v2 = faces[3 * fi + 2];
        const int32_t m01 = mids[3 * fi], m12 = mids[3 * fi + 1], m20 = mids[3 * fi + 2];
        int32_t* o = F + 3 * fi;
        o[0] = m12; o[1] = m20; o[2] = m01;
        o = F + 3 * (nf + 3 * fi);
        o[0] = v0; o[1] = m01; o[2] = m20;
        o[3] = v1; o[4] = m12; o[5] = m01;
        o[6] = v2; o[7] = m20; o[8] = m12;
    }
    /* randomize_verts (basic_functions.hpp:551-557): REAL is float, the 0.5 literal is double */
    for (int64_t i = 0; i < 3 * nvt; i++) {
        const float q = (float)rand() / (float)RAND_MAX;
        V[i] = (float)((double)V[i] + ((double)q - 0.5) * (double)amplitude);
    }
    free(tab); free(mids); free(ins);
    *vout = V; *fout = F; *nv_out = nvt;
    return 0;
}

void or_srand(unsigned seed) { srand(seed); }
int or_rand(void) { return rand(); }
void or_free(void* p) { free(p); }
