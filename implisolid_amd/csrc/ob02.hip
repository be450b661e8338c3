// ob02.hip -- Ohtake-Belyaev mesh refinement (vertex resampling, centroid projection, QEM) on gfx950.
//
// Every reference pass that is vectorised over "all faces" or "all vertices" is independent per
// element, so each becomes one lane per element.  Order-dependent float reductions stay serial
// inside one lane (umbrella sums in ascending face order, the 3-term kij sum); the one global
// serial reduction (compute_average_edge_length) is done in the reference order on the host.
//
// Reference map:
//   topology  make_neighbour_faces_of_vertex  mesh_algorithms.hpp:178-209  -> CSR umbrellas
//             make_edge_lookup / build_faces_of_faces  :50-131             -> hash of (vmin,vmax)
//   step 1    process2_vertex_resampling_relaxation_v1  vertex_resampling.hpp:152-225
//   step 2    compute_average_edge_length cp:70-82; set_centers_on_surface cp:421-1214;
//             bisection bisection.hpp:117-459; vertex_apply_qem qem.hpp:321-599
// (cp = centroids_projection.cpp)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <deque>
#include <future>
#include <limits>
#include <memory>
#include <mutex>
#include <vector>

#include "ifunc_device.hpp"
#include "ob02.hpp"
#include "fold.hpp"
#include "ob02_device.hpp"
#include "jit.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace impli {

using namespace dev;

struct EdgeTab {
    unsigned long long* key;
    uint32_t* first;
    uint32_t* last;
    uint32_t* cnt;
    uint32_t* slot_of;   // 3 * nf
    uint32_t* f2;        // 2 * cap: the faces of an edge's first two insertions (cnt says which hold one)
    uint64_t mask;
};


namespace {

constexpr uint64_t kEmpty = ~0ull;

#define DEPTH_LAUNCH(depth, KERNEL, GRID, BLOCK, STREAM, ...)                              \
    do {                                                                                   \
        if ((depth) <= 4) KERNEL<4><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);        \
        else if ((depth) <= 8) KERNEL<8><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);   \
        else if ((depth) <= 12) KERNEL<12><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__); \
        else KERNEL<16><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);                    \
    } while (0)

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }


// ---- topology --------------------------------------------------------------------------------
__global__ void k_degree(const int32_t* __restrict__ f, int64_t n3, uint32_t* __restrict__ deg) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n3) atomicAdd(&deg[f[i]], 1u);
}

// exclusive scan of n uint32 into out[0..n] (one workgroup of 1024 lanes)
__global__ __launch_bounds__(1024) void k_scan_u32(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int64_t n) {
    __shared__ uint32_t s_w[16];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t chunk = (n + 1023) / 1024;
    const int64_t a = t * chunk, e = (a + chunk < n) ? a + chunk : n;
    uint32_t sum = 0;
    for (int64_t i = a; i < e; ++i) sum += in[i];
    uint32_t x = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
        if (w < wid) pre += s_w[w];
        tot += s_w[w];
    }
    uint32_t run = pre + x - sum;
    for (int64_t i = a; i < e; ++i) {
        const uint32_t v = in[i];
        out[i] = run;
        run += v;
    }
    if (t == 0) out[n] = tot;
}

// multi-block exclusive scan: tiles of 256 x 16 values -> tile sums -> one-block scan of the sums
// (k_scan_u32) -> tiles re-scanned with their offsets.  out[n] = total.
constexpr int kScanPer = 16, kScanTile = 256 * kScanPer;

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* s_w, uint32_t& total) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    uint32_t v = x;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    uint32_t pre = 0;
    total = 0;
    for (int w = 0; w < 4; ++w) {
        pre += (w < wid) ? s_w[w] : 0u;
        total += s_w[w];
    }
    __syncthreads();
    return pre + v - x;
}

__global__ __launch_bounds__(256) void k_scan_tile_sums(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ sums) {
    __shared__ uint32_t s_w[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) a += (base + k < n) ? in[base + k] : 0u;
    uint32_t total;
    (void)block_excl_scan256(a, s_w, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_tiles(const uint32_t* __restrict__ in, int64_t n, const uint32_t* __restrict__ offs,
                                                    uint32_t* __restrict__ out) {
    __shared__ uint32_t s_w[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer], a = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        v[k] = (base + k < n) ? in[base + k] : 0u;
        a += v[k];
    }
    uint32_t total;
    uint32_t run = offs[blockIdx.x] + block_excl_scan256(a, s_w, total);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = offs[blockIdx.x] + total;
}

__global__ void k_fill_umbrella(const int32_t* __restrict__ f, int64_t nf, const uint32_t* __restrict__ off,
                                uint32_t* __restrict__ fill, int32_t* __restrict__ lst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * nf) return;
    const int32_t v = f[i];
    const uint32_t p = atomicAdd(&fill[v], 1u);
    lst[off[v] + p] = (int32_t)(i / 3);
}

// make_neighbour_faces_of_vertex lists faces in ascending order: sort each small umbrella
__global__ void k_sort_umbrella(const uint32_t* __restrict__ off, int32_t* __restrict__ lst, int64_t nv) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= nv) return;
    const uint32_t a = off[v], e = off[v + 1];
    for (uint32_t i = a + 1; i < e; ++i) {
        const int32_t x = lst[i];
        uint32_t j = i;
        while (j > a && lst[j - 1] > x) { lst[j] = lst[j - 1]; --j; }
        lst[j] = x;
    }
}


__global__ void k_edge_insert(const int32_t* __restrict__ f, int64_t nf, int64_t nv, EdgeTab t) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * nf) return;
    const int64_t fi = i / 3;
    const int vj = (int)(i - fi * 3);
    const uint64_t e1 = (uint32_t)f[i], e2 = (uint32_t)f[fi * 3 + (vj + 1) % 3];
    const unsigned long long key = (e2 > e1) ? e1 + e2 * (uint64_t)nv : e2 + e1 * (uint64_t)nv;
    uint64_t s = (key * 0x9E3779B97F4A7C15ull >> 17) & t.mask;
    while (true) {
        const unsigned long long prev = atomicCAS(&t.key[s], kEmpty, key);
        if (prev == kEmpty || prev == key) break;
        s = (s + 1) & t.mask;
    }
    // two atomics per half-edge: the arrival index keeps the first two faces (an edge of a closed
    // manifold mesh has exactly two); min / max over further ones only for non-manifold edges
    const uint32_t k = atomicAdd(&t.cnt[s], 1u);
    if (k < 2) {
        t.f2[2 * s + k] = (uint32_t)fi;
    } else {
        atomicMin(&t.first[s], (uint32_t)fi);
        atomicMax(&t.last[s], (uint32_t)fi);
    }
    t.slot_of[i] = (uint32_t)s;
}

// build_faces_of_faces: fof = first != face ? first : last; "last" of an edge seen once is the
// value-initialised 0 of faces_of_edges (mesh_algorithms.hpp:111-121)
__global__ void k_fof(int64_t nf, EdgeTab t, int32_t* __restrict__ fof) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * nf) return;
    const uint32_t s = t.slot_of[i];
    const uint32_t fi = (uint32_t)(i / 3);
    const uint32_t c = t.cnt[s], a = t.f2[2 * s], b = c >= 2 ? t.f2[2 * s + 1] : a;
    // first / last face of the edge (the min / max words hold only non-manifold extras); every
    // half-edge of the slot stores the same values for the subdivision pass
    const uint32_t first = min(min(a, b), t.first[s]), last = max(max(a, b), t.last[s]);
    t.first[s] = first;
    t.last[s] = last;
    fof[i] = (int32_t)((first != fi) ? first : (c >= 2 ? last : 0u));
}

// ---- step 3: my_subdiv_ (centroids_projection.cpp:1314-1367) -----------------------------------
// subdivide_multiple_facets_1to4 (subdiv_1to4.hpp:147-232) numbers midpoints by first appearance of
// their edge over (face ascending; e01, e12, e20).  The first slot of an edge is in face
// first[edge], at the lowest k of that face holding the edge.
__device__ __forceinline__ bool first_slot(const EdgeTab& t, int64_t fi, int k, uint32_t s[3]) {
    return t.first[s[k]] == (uint32_t)fi && (k < 1 || s[0] != s[k]) && (k < 2 || s[1] != s[k]);
}

__global__ void k_sub_count(int64_t nf, EdgeTab t, uint32_t* __restrict__ cnt) {
    const int64_t fi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (fi >= nf) return;
    uint32_t s[3] = {t.slot_of[3 * fi], t.slot_of[3 * fi + 1], t.slot_of[3 * fi + 2]};
    cnt[fi] = (uint32_t)first_slot(t, fi, 0, s) + (uint32_t)first_slot(t, fi, 1, s) + (uint32_t)first_slot(t, fi, 2, s);
}

// new_vert_maker (subdiv_1to4.hpp:277-330): Eigen's lazy 3x3 product reduces a0 + (a1 + a2)
__device__ __forceinline__ float mid3(float a0, float a1, float a2, float w0, float w1, float w2) {
    return a0 * w0 + (a1 * w1 + a2 * w2);
}

__global__ void k_sub_verts(const float* __restrict__ v, const int32_t* __restrict__ f, int64_t nf, int64_t nv, EdgeTab t,
                            const uint32_t* __restrict__ off, float* __restrict__ vout, uint32_t* __restrict__ tmid) {
    const int64_t fi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (fi >= nf) return;
    uint32_t s[3] = {t.slot_of[3 * fi], t.slot_of[3 * fi + 1], t.slot_of[3 * fi + 2]};
    const float H = 0.5f, O = 0.0f;
    const float W[3][3] = {{H, H, O}, {O, H, H}, {H, O, H}};   // columns m01, m12, m20 of new_vert_maker
    const float* p0 = v + 3 * (int64_t)f[3 * fi];
    const float* p1 = v + 3 * (int64_t)f[3 * fi + 1];
    const float* p2 = v + 3 * (int64_t)f[3 * fi + 2];
    uint32_t id = (uint32_t)nv + off[fi];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (!first_slot(t, fi, k, s)) continue;
        float* o = vout + 3 * (int64_t)id;
#pragma unroll
        for (int r = 0; r < 3; ++r) o[r] = mid3(p0[r], p1[r], p2[r], W[k][0], W[k][1], W[k][2]);
        tmid[s[k]] = id++;
    }
}

// subdiv_1to4.hpp:380-470: face fi becomes (m12, m20, m01); nf + 3 fi + {0,1,2} the corner faces
__global__ void k_sub_faces(const int32_t* __restrict__ f, int64_t nf, EdgeTab t, const uint32_t* __restrict__ tmid,
                            int32_t* __restrict__ fout) {
    const int64_t fi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (fi >= nf) return;
    const int32_t v0 = f[3 * fi], v1 = f[3 * fi + 1], v2 = f[3 * fi + 2];
    const int32_t m01 = (int32_t)tmid[t.slot_of[3 * fi]], m12 = (int32_t)tmid[t.slot_of[3 * fi + 1]],
                  m20 = (int32_t)tmid[t.slot_of[3 * fi + 2]];
    int32_t* o = fout + 3 * fi;
    o[0] = m12; o[1] = m20; o[2] = m01;
    o = fout + 3 * (nf + 3 * fi);
    o[0] = v0; o[1] = m01; o[2] = m20;
    o[3] = v1; o[4] = m12; o[5] = m01;
    o[6] = v2; o[7] = m20; o[8] = m12;
}

// randomize_verts (basic_functions.hpp:551-557) with glibc rand(): lane c produces draws
// [c L, c L + L) of the sequence from its own window x_{m + cL + j} = sum_i Q_c[i] x_{m+i+j},
// Q_c = z^(cL) mod P = qlo[c % 64] * qhi[c / 64] (host.hpp GlibcRand).
constexpr int kRandL = 31 * 8;

__device__ __forceinline__ void poly_mulmod(const uint32_t a[31], const uint32_t b[31], uint32_t out[31]) {
    uint32_t p[61];
#pragma unroll
    for (int k = 0; k < 61; ++k) p[k] = 0;
#pragma unroll
    for (int i = 0; i < 31; ++i)
#pragma unroll
        for (int j = 0; j < 31; ++j) p[i + j] += a[i] * b[j];
#pragma unroll
    for (int k = 60; k >= 31; --k) {
        p[k - 3] += p[k];
        p[k - 31] += p[k];
    }
#pragma unroll
    for (int i = 0; i < 31; ++i) out[i] = p[i];
}

__global__ __launch_bounds__(256) void k_rand_noise(float* __restrict__ v, int64_t n, const uint32_t* __restrict__ xw,
                                                    const uint32_t* __restrict__ qlo, const uint32_t* __restrict__ qhi,
                                                    float amplitude) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n0 = c * kRandL;
    if (n0 >= n) return;
    uint32_t a[31], b[31], q[31], w[31];
#pragma unroll
    for (int i = 0; i < 31; ++i) {
        a[i] = qlo[(c & 63) * 31 + i];
        b[i] = qhi[(c >> 6) * 31 + i];
    }
    poly_mulmod(a, b, q);
#pragma unroll
    for (int j = 0; j < 31; ++j) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 31; ++i) acc += q[i] * xw[i + j];
        w[j] = acc;
    }
    const double amp = (double)amplitude;
    for (int r = 0; r < kRandL / 31; ++r) {
#pragma unroll
        for (int k = 0; k < 31; ++k) {
            const uint32_t x = w[k] + w[(k + 28) % 31];
            w[k] = x;
            const int64_t i = n0 + r * 31 + k;
            if (i < n) {
                // (REAL)rand() / (REAL)RAND_MAX - 0.5 (a double literal), times the float amplitude
                const float u = (float)(int32_t)(x >> 1) / 2147483648.0f;
                v[i] = (float)((double)v[i] + ((double)u - 0.5) * amp);
            }
        }
    }
}

// ---- the tree-evaluating passes over the interpreter (ob02_device.hpp; the JIT point module has
//      the same bodies over tree-specialised code) -------------------------------------------------
using namespace ob;

template <int D>
__global__ __launch_bounds__(256) void k_centroid_normals(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                          const float* __restrict__ v, const int32_t* __restrict__ f,
                                                          int64_t nf, float* __restrict__ C, float* __restrict__ N) {
    centroid_normals_body(InterpPt<D>{prog, tab}, v, f, nf, C, N);
}
template <int D>
__global__ __launch_bounds__(256) void k_project_prep(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      ProjArgs a) {
    project_prep_body(InterpPt<D>{prog, tab}, a);
}
template <int D>
__global__ __launch_bounds__(256) void k_project_early(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                       ProjArgs a) {
    project_early_body(InterpPt<D>{prog, tab}, a);
}
template <int D>
__global__ __launch_bounds__(256) void k_project_late(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      ProjArgs a) {
    project_late_body(InterpPt<D>{prog, tab}, a);
}
template <int D>
__global__ __launch_bounds__(256) void k_normals_at(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                    const float* __restrict__ P, int64_t n, float* __restrict__ G) {
    normals_at_body(InterpPt<D>{prog, tab}, P, n, G);
}

// ---- step 1 ----------------------------------------------------------------------------------
__device__ __forceinline__ float kij(int64_t i, int64_t j, const float* __restrict__ C, const float* __restrict__ N);

// glibc 2.35 e_acosf.c (fdlibm), the libm std::acos(float) of vertex_resampling.hpp:75 resolves to
__device__ __forceinline__ float glibc_acosf(float x) {
    const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
                pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f, pS3 = -4.0055535734e-02f,
                pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f, qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f,
                qS3 = -6.8828397989e-01f, qS4 = 7.7038154006e-02f;
    const int32_t hx = __float_as_int(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return (hx > 0) ? 0.0f : pi + 2.0f * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        const float z = x * x;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {
        const float z = (one + x) * 0.5f;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float s = sqrtf(z);
        const float r = p / q;
        const float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    } else {
        const float z = (one - x) * 0.5f;
        const float s = sqrtf(z);
        const float df = __int_as_float(__float_as_int(s) & (int32_t)0xfffff000);
        const float c = (z - df * df) / (s + df);
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float r = p / q;
        const float w = r * s + c;
        return 2.0f * (df + w);
    }
}

// vertex_resampling.hpp:47-77
__device__ __forceinline__ float kij(int64_t i, int64_t j, const float* __restrict__ C, const float* __restrict__ N) {
    float mimj = N[3 * i] * N[3 * j] + N[3 * i + 1] * N[3 * j + 1] + N[3 * i + 2] * N[3 * j + 2];
    if (mimj > 1.0f) mimj = 1.0f;
    if (mimj < -1.0f) mimj = -1.0f;
    const float pipj = norm2f(C[3 * i] - C[3 * j], C[3 * i + 1] - C[3 * j + 1], C[3 * i + 2] - C[3 * j + 2]);
    if (pipj == 0) return 0;
    return glibc_acosf(mimj) / pipj;
}

__global__ void k_face_weights(const float* __restrict__ C, const float* __restrict__ N, const int32_t* __restrict__ fof,
                               int64_t nf, float c, float* __restrict__ W) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nf) return;
    float ki = 0;   // wi, vertex_resampling.hpp:79-91
    for (int j = 0; j < 3; ++j) ki += kij(i, fof[3 * i + j], C, N);
    W[i] = (float)(1.0 + (double)(c * ki));
}

__global__ void k_resample(const uint32_t* __restrict__ off, const int32_t* __restrict__ lst, const float* __restrict__ W,
                           const float* __restrict__ C, int64_t nv, float* __restrict__ out) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= nv) return;
    const uint32_t a = off[v], e = off[v + 1];
    float sw = 0;   // vertex_resampling_VV1 :108-140
    for (uint32_t k = a; k < e; ++k) sw += W[lst[k]];
    float x = 0, y = 0, z = 0;
    for (uint32_t k = a; k < e; ++k) {
        const int32_t fj = lst[k];
        const float w = W[fj] / sw;
        x += w * C[3 * fj];
        y += w * C[3 * fj + 1];
        z += w * C[3 * fj + 2];
    }
    out[3 * v] = x; out[3 * v + 1] = y; out[3 * v + 2] = z;
}

// ---- step 2 ----------------------------------------------------------------------------------
// compute_average_edge_length cp:70-82 terms, in the reference's order (summed serially on host)
__global__ void k_edge_norms(const float* __restrict__ v, const int32_t* __restrict__ f, int64_t nf, float* __restrict__ o) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nf) return;
    const float* a = v + 3 * f[3 * j];
    const float* b = v + 3 * f[3 * j + 1];
    const float* c = v + 3 * f[3 * j + 2];
    o[3 * j] = norm2f(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
    o[3 * j + 1] = norm2f(a[0] - c[0], a[1] - c[1], a[2] - c[2]);
    o[3 * j + 2] = norm2f(c[0] - b[0], c[1] - b[1], c[2] - b[2]);
}

// the fold's chunk table (fold.hpp), three small passes: each chunk's terms summed in double (one
// wave per chunk); the exclusive prefix of those sums (one block) -> each chunk's binade window;
// the table cells of the window (one wave per chunk, 4 terms per lane, wave sums of the lanes'
// saturating partial sums, flags OR-ed)
__global__ __launch_bounds__(256) void k_fold_chunk_sums(const float* __restrict__ e, int64_t n, double* __restrict__ cs) {
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (c >= fold_chunks(n)) return;   // uniform per wave
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = c * kFoldChunk + q * 64 + lane;
        if (k < n) v += (double)e[k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) cs[c] = v;
}
__global__ __launch_bounds__(1024) void k_fold_bases(const double* __restrict__ cs, int64_t nc, int32_t* __restrict__ base) {
    __shared__ double s_w[16];
    __shared__ double s_carry;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_carry = 0.0;
    __syncthreads();
    for (int64_t i0 = 0; i0 < nc; i0 += 1024) {
        const int64_t i = i0 + t;
        const double v = i < nc ? cs[i] : 0.0;
        double inc = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        double off = s_carry;
        for (int k = 0; k < w; ++k) off += s_w[k];
        if (i < nc) base[i] = fold_base(off + inc - v);   // the estimate of the sum before chunk i
        __syncthreads();
        if (t == 1023) s_carry = off + inc;
        __syncthreads();
    }
}
__global__ __launch_bounds__(256) void k_fold_table(const float* __restrict__ e, int64_t n, const int32_t* __restrict__ base,
                                                    uint32_t* __restrict__ sum, uint8_t* __restrict__ flags) {
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (c >= fold_chunks(n)) return;   // uniform per wave
    uint32_t bits[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = c * kFoldChunk + q * 64 + lane;
        bits[q] = k < n ? __float_as_uint(e[k]) : 0u;   // +0 past the end contributes nothing
    }
    const int E0 = base[c];
#pragma unroll
    for (int b = 0; b < kFoldBinades; ++b) {
        uint32_t s = 0, f = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint8_t fq;
            s = fold_add(s, fold_term(bits[q], E0 + b, fq));
            f |= fq;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s = fold_add(s, (uint32_t)__shfl_xor((int)s, o, 64));
            f |= (uint32_t)__shfl_xor((int)f, o, 64);
        }
        if (lane == 0) {
            sum[c * kFoldBinades + b] = s;
            flags[c * kFoldBinades + b] = (uint8_t)f;
        }
    }
}

// ---- QEM: Eigen 3.3 JacobiSVD<Matrix3f> restated (Eigen/src/SVD/JacobiSVD.h, Jacobi/Jacobi.h) ----
struct JRot { float c, s; };
__device__ __forceinline__ void rot_rows(float W[3][3], int p, int q, JRot j) {
    if (j.c == 1.f && j.s == 0.f) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float xi = W[p][k], yi = W[q][k];
        W[p][k] = j.c * xi + j.s * yi;
        W[q][k] = -j.s * xi + j.c * yi;
    }
}
__device__ __forceinline__ void rot_cols(float W[3][3], int p, int q, JRot j) {
    if (j.c == 1.f && j.s == 0.f) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float xi = W[k][p], yi = W[k][q];
        W[k][p] = j.c * xi + j.s * yi;
        W[k][q] = -j.s * xi + j.c * yi;
    }
}
__device__ __forceinline__ JRot make_jacobi(float x, float y, float z) {
    const float deno = 2.f * fabsf(y);
    if (deno < 1.17549435e-38f) return JRot{1.f, 0.f};
    const float tau = (x - z) / deno;
    const float w = sqrtf(tau * tau + 1.f);
    const float t = (tau > 0.f) ? 1.f / (tau + w) : 1.f / (tau - w);
    const float sign_t = t > 0.f ? 1.f : -1.f;
    const float n = 1.f / sqrtf(t * t + 1.f);
    return JRot{n, -sign_t * (y / fabsf(y)) * fabsf(t) * n};
}
__device__ __forceinline__ void jacobi_2x2(float W[3][3], int p, int q, JRot& jl, JRot& jr) {
    float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
    JRot r1;
    const float t = m00 + m11, d = m10 - m01;
    if (fabsf(d) < 1.17549435e-38f) r1 = JRot{1.f, 0.f};
    else {
        const float u = t / d;
        const float tmp = sqrtf(1.f + u * u);
        r1 = JRot{u / tmp, 1.f / tmp};
    }
    if (!(r1.c == 1.f && r1.s == 0.f)) {
        const float a0 = m00, b0 = m10, a1 = m01, b1 = m11;
        m00 = r1.c * a0 + r1.s * b0; m10 = -r1.s * a0 + r1.c * b0;
        m01 = r1.c * a1 + r1.s * b1; m11 = -r1.s * a1 + r1.c * b1;
    }
    jr = make_jacobi(m00, m01, m11);
    const JRot rt{jr.c, -jr.s};
    jl = JRot{r1.c * rt.c - r1.s * rt.s, r1.c * rt.s + r1.s * rt.c};
}
__device__ int jacobi_svd3(const float A[3][3], float thr, float S[3], float U[3][3], float V[3][3]) {
    const float precision = 2.f * 1.1920929e-07f, consider_zero = 1.17549435e-38f;
    float scale = 0.f;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) { const float a = fabsf(A[r][c]); if (a > scale) scale = a; }
    if (scale == 0.f) scale = 1.f;
    float W[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) { W[r][c] = A[r][c] / scale; U[r][c] = (r == c) ? 1.f : 0.f; V[r][c] = (r == c) ? 1.f : 0.f; }
    float maxd = 0.f;
    for (int i = 0; i < 3; ++i) { const float a = fabsf(W[i][i]); if (a > maxd) maxd = a; }
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const float threshold = consider_zero > precision * maxd ? consider_zero : precision * maxd;
                if (fabsf(W[p][q]) > threshold || fabsf(W[q][p]) > threshold) {
                    finished = false;
                    JRot jl, jr;
                    jacobi_2x2(W, p, q, jl, jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, jl);
                    const JRot jrt{jr.c, -jr.s};
                    rot_cols(W, p, q, jrt);
                    rot_cols(V, p, q, jrt);
                    const float a = fabsf(W[p][p]), b = fabsf(W[q][q]);
                    const float mx = a > b ? a : b;
                    if (mx > maxd) maxd = mx;
                }
            }
    }
    for (int i = 0; i < 3; ++i) {
        const float a = W[i][i];
        S[i] = fabsf(a);
        if (a < 0.f) for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < 3; ++i) S[i] *= scale;
    int nonzero = 3;
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        float mx = S[i];
        for (int k = i + 1; k < 3; ++k) if (S[k] > mx) { mx = S[k]; pos = k; }
        if (mx == 0.f) { nonzero = i; break; }
        if (pos != i) {
            float t = S[i]; S[i] = S[pos]; S[pos] = t;
            for (int r = 0; r < 3; ++r) {
                t = U[r][i]; U[r][i] = U[r][pos]; U[r][pos] = t;
                t = V[r][i]; V[r][i] = V[r][pos]; V[r][pos] = t;
            }
        }
    }
    float pt = S[0] * thr;
    if (pt < consider_zero) pt = consider_zero;
    int i = nonzero - 1;
    while (i >= 0 && S[i] < pt) --i;
    return i + 1;
}

// vertex_apply_qem (qem.hpp:321-599) with get_A_b (:256-316), one lane per vertex
__global__ __launch_bounds__(256) void k_qem(float* __restrict__ verts, int64_t nv, const uint32_t* __restrict__ off,
                                             const int32_t* __restrict__ lst, const float* __restrict__ C,
                                             const float* __restrict__ N, float maxd) {
    const int64_t vi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (vi >= nv) return;
    float* v = verts + 3 * vi;
    const float ox = v[0], oy = v[1], oz = v[2];
    float A[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, b[3] = {0.f, 0.f, 0.f};
    for (uint32_t k = off[vi]; k < off[vi + 1]; ++k) {
        const int32_t ni = lst[k];
        const float nx = N[3 * ni], ny = N[3 * ni + 1], nz = N[3 * ni + 2];
        const float Px = C[3 * ni] - ox, Py = C[3 * ni + 1] - oy, Pz = C[3 * ni + 2] - oz;
        const float nn00 = nx * nx, nn01 = nx * ny, nn02 = nx * nz, nn11 = ny * ny, nn12 = ny * nz, nn22 = nz * nz;
        A[0][0] += nn00; A[0][1] += nn01; A[0][2] += nn02;
        A[1][0] += nn01; A[1][1] += nn11; A[1][2] += nn12;
        A[2][2] += nn22; A[2][0] += nn02; A[2][1] += nn12;
        b[0] -= nn00 * Px + nn01 * Py + nn02 * Pz;
        b[1] -= nn01 * Px + nn11 * Py + nn12 * Pz;
        b[2] -= nn02 * Px + nn12 * Py + nn22 * Pz;
    }
    float S[3], U[3][3], V[3][3];
    const int rank = jacobi_svd3(A, (float)(1.0 / 680.0), S, U, V);
    float y[3] = {0.f, 0.f, 0.f}, utb[3];
    for (int i = 0; i < 3; ++i) utb[i] = (-U[0][i]) * b[0] + ((-U[1][i]) * b[1] + (-U[2][i]) * b[2]);
    for (int i = 0; i < rank; ++i) y[i] = utb[i] / S[i];
    float nx[3];
    for (int r = 0; r < 3; ++r) nx[r] = (V[r][0] * y[0] + (V[r][1] * y[1] + V[r][2] * y[2])) + v[r];
    if (maxd > 0) {
        const float dx = nx[0] - v[0], dy = nx[1] - v[1], dz = nx[2] - v[2];
        const float dist2 = dx * dx + dy * dy + dz * dz;
        if (dist2 <= maxd * maxd) { v[0] = nx[0]; v[1] = nx[1]; v[2] = nx[2]; }
        else {
            const float dist = sqrtf(dist2);
            float len = (float)(maxd * 1.5);
            if (len > dist) len = dist;
            v[0] += dx / dist * len; v[1] += dy / dist * len; v[2] += dz / dist * len;
        }
    } else {
        v[0] = nx[0]; v[1] = nx[1]; v[2] = nx[2];
    }
}

// ---- host helpers ------------------------------------------------------------------------------
// make_alpha_list cp:144-194
std::vector<float> make_alpha_list(float initial_step, float min_step, float max_dist, int max_iter) {
    std::vector<float> a;
    const float unit = max_dist;
    float step = initial_step;
    while (step > min_step) {
        step = (float)(step * 0.5);
        const int total = (int)std::floor((double)(max_dist / std::fabs(step)) + 0.001);
        const int ms = max_iter < total ? max_iter : total;
        for (int i = 1; i < ms + 1; i += 2) {
            const float alpha = (float)i * step;
            a.push_back(alpha / unit);
            a.push_back(-alpha / unit);
        }
        if (a.size() > 100000) break;   // guards a pathological max_dist
    }
    return a;
}

// boost::random::mt11213b (seed 12) + uniform_01<float>: make_random_pm1(n, 3, 1e-6)
// (make_random_pm1.hpp:15-29): the twist in three runs (no index wrap inside), tempering of a
// whole block at once, then uniform_01's rejection of draws that round to 1.0f
std::vector<float> make_random_pm1(int64_t n, float amplitude) {
    constexpr int N = 351, M = 175;
    constexpr uint32_t UM = 0xffffffffu << 19, LM = ~UM, A = 0xccab8ee7u;
    uint32_t x[N], t[N];
    x[0] = 12u;
    for (int i = 1; i < N; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    const float factor = 1.0f / ((float)4294967295u + 1.0f);
    const double amp = (double)amplitude;
    std::vector<float> out((size_t)(3 * n));
    size_t o = 0;
    while (o < out.size()) {
        int k = 0;
        for (; k < N - M; ++k) {
            const uint32_t y = (x[k] & UM) | (x[k + 1] & LM);
            x[k] = x[k + M] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        for (; k < N - 1; ++k) {
            const uint32_t y = (x[k] & UM) | (x[k + 1] & LM);
            x[k] = x[k + M - N] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        const uint32_t y = (x[N - 1] & UM) | (x[0] & LM);
        x[N - 1] = x[M - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        for (int i = 0; i < N; ++i) {
            uint32_t z = x[i];
            z ^= (z >> 11);
            z ^= (z << 7) & 0x31b6ab00u;
            z ^= (z << 15) & 0xffe50000u;
            z ^= (z >> 17);
            t[i] = z;
        }
        for (int i = 0; i < N && o < out.size(); ++i) {
            const float r = (float)t[i] * factor;
            if (!(r < 1.0f)) continue;
            out[o++] = (float)(((double)r * 2.0 - 1.0) * amp);
        }
    }
    return out;
}

// the perturbations depend on the face count alone (seeded afresh on every call): the last few
// face counts' tables are kept, so rebuilding a mesh of the same size does not redraw them
std::shared_ptr<const std::vector<float>> random_pm1_cached(int64_t n) {
    static std::mutex mu;
    static std::deque<std::pair<int64_t, std::shared_ptr<const std::vector<float>>>> cache;
    {
        std::lock_guard<std::mutex> lock(mu);
        for (auto& e : cache)
            if (e.first == n) return e.second;
    }
    auto v = std::make_shared<const std::vector<float>>(make_random_pm1(n, 0.000001f));
    std::lock_guard<std::mutex> lock(mu);
    cache.emplace_front(n, v);
    if (cache.size() > 4) cache.pop_back();
    return v;
}

}  // namespace

Ob02::Ob02(Engine& e, hipStream_t st) : E(e), s(st) {
    misc_.reserve(512);
}

void Ob02::load_mesh(const float* d_verts, int64_t nv_, const int32_t* d_faces, int64_t nf_) {
    nv = nv_;
    nf = nf_;
    for (auto& kv : snaps_) kv.second.buf.release();
    snaps_.clear();
    pointsets_.clear();
    cap_hits_ = 0;
    evals_ = 0;
    jit_launches_ = 0;
    avg_edge_ = 0.f;
    for (double& t : stage_ms_) t = 0.0;
    Stage st(this, kStageTopology);
    IMPLI_HIP(hipMemsetAsync(misc_.p, 0, 64, s));   // (unused), cap hits, evaluations
    verts_.reserve((size_t)(nv + 1) * 12);
    vnew_.reserve((size_t)(nv + 1) * 12);
    faces_.reserve((size_t)(nf + 1) * 12);
    if (nv) IMPLI_HIP(hipMemcpyAsync(verts_.p, d_verts, (size_t)nv * 12, hipMemcpyDeviceToDevice, s));
    if (nf) IMPLI_HIP(hipMemcpyAsync(faces_.p, d_faces, (size_t)nf * 12, hipMemcpyDeviceToDevice, s));
    start_perturbations();   // host thread, overlaps the topology and resampling kernels
    build_topology();
}

EdgeTab Ob02::edge_table() {
    uint64_t cap = 1024;
    while (cap < (uint64_t)(4 * nf + 16)) cap <<= 1;
    etab_.reserve((size_t)cap * (8 + 12 + 8) + (size_t)(3 * nf + 1) * 4);
    EdgeTab t;
    t.key = etab_.as<unsigned long long>();
    t.first = reinterpret_cast<uint32_t*>(t.key + cap);
    t.last = t.first + cap;
    t.cnt = t.last + cap;
    t.slot_of = t.cnt + cap;
    t.f2 = t.slot_of + (3 * nf + 1);
    t.mask = cap - 1;
    return t;
}

void Ob02::build_topology() {
    // umbrellas
    deg_.reserve((size_t)(nv + 1) * 4);
    uoff_.reserve((size_t)(nv + 2) * 4);
    ulst_.reserve((size_t)(3 * nf + 1) * 4);
    IMPLI_HIP(hipMemsetAsync(deg_.p, 0, (size_t)(nv + 1) * 4, s));
    if (nf) k_degree<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, deg_.as<uint32_t>());
    scan(deg_.as<uint32_t>(), uoff_.as<uint32_t>(), nv);
    IMPLI_HIP(hipMemsetAsync(deg_.p, 0, (size_t)(nv + 1) * 4, s));
    if (nf) k_fill_umbrella<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), nf, uoff_.as<uint32_t>(),
                                                             deg_.as<uint32_t>(), ulst_.as<int32_t>());
    if (nv) k_sort_umbrella<<<blocks_for(nv), 256, 0, s>>>(uoff_.as<uint32_t>(), ulst_.as<int32_t>(), nv);
    // faces of faces
    const EdgeTab t = edge_table();
    const uint64_t cap = t.mask + 1;
    IMPLI_HIP(hipMemsetAsync(t.key, 0xff, (size_t)cap * 8, s));
    IMPLI_HIP(hipMemsetAsync(t.first, 0xff, (size_t)cap * 4, s));
    IMPLI_HIP(hipMemsetAsync(t.last, 0, (size_t)cap * 8, s));   // last + cnt
    fof_.reserve((size_t)(3 * nf + 1) * 4);
    if (nf) {
        k_edge_insert<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), nf, nv, t);
        k_fof<<<blocks_for(3 * nf), 256, 0, s>>>(nf, t, fof_.as<int32_t>());
    }
    cen_.reserve((size_t)(nf + 1) * 12);
    nrm_.reserve((size_t)(nf + 1) * 12);
    w_.reserve((size_t)(nf + 1) * 4);
    IMPLI_HIP(hipGetLastError());
    topo_valid_ = true;
}

void Ob02::scan(const uint32_t* in, uint32_t* out, int64_t n) {
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles <= 1) {
        k_scan_u32<<<1, 1024, 0, s>>>(in, out, n);
        return;
    }
    scan_tmp_.reserve((size_t)(2 * tiles + 2) * 4);
    uint32_t* sums = scan_tmp_.as<uint32_t>();
    uint32_t* offs = sums + tiles + 1;
    k_scan_tile_sums<<<(unsigned)tiles, 256, 0, s>>>(in, n, sums);
    k_scan_u32<<<1, 1024, 0, s>>>(sums, offs, tiles);
    k_scan_tiles<<<(unsigned)tiles, 256, 0, s>>>(in, n, offs, out);
}

// STORE_POINTSET: a device snapshot now (stream-ordered, no host sync), copied to the host only
// when pointsets() is asked for
void Ob02::store_pointset(const char* key, const float* d, int64_t n, bool keep_first) {
    if (!capture_pointsets) return;
    if (keep_first && snaps_.count(key)) return;
    Snapshot& e = snaps_[key];
    e.buf.reserve((size_t)(n + 1) * 12);
    e.n = n;
    if (n) IMPLI_HIP(hipMemcpyAsync(e.buf.p, d, (size_t)n * 12, hipMemcpyDeviceToDevice, s));
}

const std::map<std::string, std::vector<float>>& Ob02::pointsets() {
    pointsets_.clear();
    for (auto& kv : snaps_) {
        std::vector<float>& h = pointsets_[kv.first];
        h.resize((size_t)kv.second.n * 3);
        if (kv.second.n) IMPLI_HIP(hipMemcpyAsync(h.data(), kv.second.buf.p, (size_t)kv.second.n * 12, hipMemcpyDeviceToHost, s));
    }
    IMPLI_HIP(hipStreamSynchronize(s));
    return pointsets_;
}

Ob02::~Ob02() {
    if (pert_job_.valid()) pert_job_.wait();
    if (norms_ready_) (void)hipEventDestroy(norms_ready_);
    if (table_done_) (void)hipEventDestroy(table_done_);
    if (copy_s_) (void)hipStreamDestroy(copy_s_);
    host_norms_.release();
    dir_.release();
    evals_buf_.release();
    for (DevBuf* b : {&verts_, &faces_, &vnew_, &cen_, &nrm_, &w_, &fof_, &uoff_, &ulst_, &etab_, &deg_, &proj_, &grad_,
                      &fn_, &norms_, &alphas_, &pert_, &pend_, &misc_, &fnew_, &rtab_, &scan_tmp_, &fold_sum_})
        b->release();
    for (auto& kv : snaps_) kv.second.buf.release();
}

void Ob02::vertex_resampling(float c) {
    if (!nf) return;
    if (!topo_valid_) build_topology();
    Stage st(this, kStageResample);
    store_pointset("pre_resampling_vertices", verts_.as<float>(), nv, true);   // vertex_resampling.hpp:176-180
    if (const TreeJit::PointKernels* pk = E.point_jit()) {
        const float *m = E.d_mats(), *tab = E.d_rabbit(), *v = verts_.as<float>();
        const int32_t* f = faces_.as<int32_t>();
        float *C = cen_.as<float>(), *N = nrm_.as<float>();
        void* args[] = {&m, &tab, &v, &f, &nf, &C, &N};
        TreeJit::launch(pk->cnormals, blocks_for(nf), args, s, "impli_pt_centroid_normals");
        ++jit_launches_;
    } else {
        DEPTH_LAUNCH(E.depth(), k_centroid_normals, blocks_for(nf), 256, s, E.d_program(), E.d_rabbit(), verts_.as<float>(),
                     faces_.as<int32_t>(), nf, cen_.as<float>(), nrm_.as<float>());
    }
    k_face_weights<<<blocks_for(nf), 256, 0, s>>>(cen_.as<float>(), nrm_.as<float>(), fof_.as<int32_t>(), nf, c, w_.as<float>());
    k_resample<<<blocks_for(nv), 256, 0, s>>>(uoff_.as<uint32_t>(), ulst_.as<int32_t>(), w_.as<float>(), cen_.as<float>(),
                                              nv, vnew_.as<float>());
    std::swap(verts_, vnew_);
    IMPLI_HIP(hipGetLastError());
    store_pointset("post_resampling_vertices", verts_.as<float>(), nv, true);   // :207-211
}

// compute_average_edge_length (cp:70-82) is one serial float chain in face order: the terms are
// computed on the device and copied to pinned host memory; the chain runs on the host (one GPU lane
// adds a dependent term every ~4 cycles at 2.4 GHz, slower than a host core) while the GPU runs the
// projection's prep pass, which does not need the average.
void Ob02::start_edge_fold() {
    norms_.reserve((size_t)(nf + 1) * 12);
    k_edge_norms<<<blocks_for(nf), 256, 0, s>>>(verts_.as<float>(), faces_.as<int32_t>(), nf, norms_.as<float>());
    // the chunk table of the serial fold (fold.hpp) and the terms themselves go to pinned memory
    const int64_t chunks = fold_chunks(3 * nf), cells = chunks * kFoldBinades;
    // the table, device and host alike: [sums (cells u32) | bases (chunks i32) | flags (cells u8)],
    // then on the device the chunks' double sums; the host's pinned buffer holds the terms first
    const size_t tab_bytes = (size_t)(cells + chunks) * 4 + (size_t)cells, cs_off = (tab_bytes + 15) & ~(size_t)15;
    fold_sum_.reserve(cs_off + (size_t)(chunks + 1) * 8);
    const size_t terms_bytes = ((size_t)nf * 12 + 15) & ~(size_t)15;
    host_norms_.reserve(terms_bytes + tab_bytes + 16);
    uint32_t* d_sum = fold_sum_.as<uint32_t>();
    int32_t* d_base = reinterpret_cast<int32_t*>(d_sum + cells);
    uint8_t* d_flags = reinterpret_cast<uint8_t*>(d_base + chunks);
    double* d_cs = reinterpret_cast<double*>(fold_sum_.as<char>() + cs_off);
    if (cells) {
        k_fold_chunk_sums<<<blocks_for(chunks * 64), 256, 0, s>>>(norms_.as<float>(), 3 * nf, d_cs);
        k_fold_bases<<<1, 1024, 0, s>>>(d_cs, chunks, d_base);
        k_fold_table<<<blocks_for(chunks * 64), 256, 0, s>>>(norms_.as<float>(), 3 * nf, d_base, d_sum, d_flags);
    }
    // the copies run on their own stream, so the projection's prep pass (next on s) overlaps them
    if (!copy_s_) IMPLI_HIP(hipStreamCreateWithFlags(&copy_s_, hipStreamNonBlocking));
    if (!table_done_) IMPLI_HIP(hipEventCreateWithFlags(&table_done_, hipEventDisableTiming));
    if (!norms_ready_) IMPLI_HIP(hipEventCreateWithFlags(&norms_ready_, hipEventDisableTiming));
    IMPLI_HIP(hipEventRecord(table_done_, s));
    IMPLI_HIP(hipStreamWaitEvent(copy_s_, table_done_, 0));
    if (cells)
        IMPLI_HIP(hipMemcpyAsync(host_norms_.as<char>() + terms_bytes, fold_sum_.p, tab_bytes, hipMemcpyDeviceToHost, copy_s_));
    IMPLI_HIP(hipMemcpyAsync(host_norms_.p, norms_.p, (size_t)nf * 12, hipMemcpyDeviceToHost, copy_s_));
    IMPLI_HIP(hipEventRecord(norms_ready_, copy_s_));
}

float Ob02::finish_edge_fold() {
    IMPLI_HIP(hipEventSynchronize(norms_ready_));
    // the serial chain (the reference starts from an uninitialised float, F8a; defined as 0), from
    // the device's chunk table: bit-identical (fold.hpp, tools/fold_check.cpp), a few chunks term
    // by term
    const int64_t chunks = fold_chunks(3 * nf), cells = chunks * kFoldBinades;
    const uint32_t* sums = reinterpret_cast<const uint32_t*>(host_norms_.as<char>() + (((size_t)nf * 12 + 15) & ~(size_t)15));
    const int32_t* bases = reinterpret_cast<const int32_t*>(sums + cells);
    const float el = fold_walk(host_norms_.as<float>(), 3 * nf, bases, sums, reinterpret_cast<const uint8_t*>(bases + chunks));
    return (float)((double)el / (3. * (double)nf));
}

// make_random_pm1(nf, 3, 1e-6) (centroids_projection.cpp:239-262) is seeded afresh (seed 12) on
// every call, so it depends on nf alone: it is generated once per face count on a host thread,
// started when the mesh is loaded, and uploaded once -- the projection never waits for it unless
// a centroid needs the type-2 directions before the thread is done
void Ob02::start_perturbations() {
    if (pert_nf_ == nf || nf == 0) return;
    if (pert_job_.valid()) pert_job_.wait();
    const int64_t n = nf;
    pert_job_ = std::async(std::launch::async, [n] { return random_pm1_cached(n); });
    pert_nf_ = nf;
    pert_uploaded_ = false;
}

const float* Ob02::perturbations() {
    if (pert_nf_ != nf) start_perturbations();
    if (!pert_uploaded_) {
        pert_host_ = pert_job_.get();
        pert_.reserve(pert_host_->size() * 4 + 16);
        IMPLI_HIP(hipMemcpyAsync(pert_.p, pert_host_->data(), pert_host_->size() * 4, hipMemcpyHostToDevice, s));
        pert_uploaded_ = true;
    }
    return pert_.as<float>();
}

void Ob02::centroids_projection(bool enable_qem) {
    if (!nf) return;
    if (!topo_valid_) build_topology();
    Stage st(this, kStageEdgeFold);
    start_edge_fold();
    proj_.reserve((size_t)(nf + 1) * 12);
    fn_.reserve((size_t)(nf + 1) * 12);
    dir_.reserve((size_t)(nf + 1) * 12);
    pend_.reserve((size_t)(nf + 2) * 4);
    if (profile_) evals_buf_.reserve((size_t)(nf + 1) * 4);
    DevBuf& fcbuf = w_;   // f(centroid) per face; the resampling weights are dead here
    ProjArgs a{};
    a.v = verts_.as<float>();
    a.f = faces_.as<int32_t>();
    a.nf = nf;
    a.out = proj_.as<float>();
    a.fn = fn_.as<float>();
    a.fc = fcbuf.as<float>();
    a.pend = pend_.as<uint32_t>();
    a.pend_count = misc_.as<uint32_t>();
    a.cap_hits = misc_.as<uint32_t>() + 1;
    a.cen = cen_.as<float>();
    a.dir = dir_.as<float>();
    a.evals = profile_ ? evals_buf_.as<uint32_t>() : nullptr;
    const TreeJit::PointKernels* pk = E.point_jit();   // one choice for the whole projection
    const float *jm = E.d_mats(), *jtab = E.d_rabbit();
    void* jargs[] = {&jm, &jtab, &a};
    if (pk) {
        TreeJit::launch(pk->prep, blocks_for(nf), jargs, s, "impli_pt_project_prep");
        ++jit_launches_;
    } else {
        DEPTH_LAUNCH(E.depth(), k_project_prep, blocks_for(nf), 256, s, E.d_program(), E.d_rabbit(), a);
    }
    store_pointset("pre_p_centroids", cen_.as<float>(), nf, false);   // cp:1236-1238: the centroids
    const float avg = finish_edge_fold();
    avg_edge_ = avg;
    alphas_host_ = make_alpha_list((float)(avg * 1.0), (float)(0.001 * 1.0), avg, 20);
    alphas_.reserve((alphas_host_.size() + 1) * 4);
    if (!alphas_host_.empty())
        IMPLI_HIP(hipMemcpyAsync(alphas_.p, alphas_host_.data(), alphas_host_.size() * 4, hipMemcpyHostToDevice, s));
    a.alphas = alphas_.as<float>();
    a.nal = (int)alphas_host_.size();
    a.max_dist = avg;
    st.next(kStageProject);
    const unsigned grid = blocks_for(nf * kProjGroup);
    if (pk) TreeJit::launch(pk->early, grid, jargs, s, "impli_pt_project_early");
    else DEPTH_LAUNCH(E.depth(), k_project_early, grid, 256, s, E.d_program(), E.d_rabbit(), a);
    // centroids left unresolved need the randomised directions (types 2-6): the late pass covers
    // every face and reads the early pass's per-face flags on the device (no host round trip)
    a.pert = perturbations();
    if (pk) TreeJit::launch(pk->late, grid, jargs, s, "impli_pt_project_late");
    else DEPTH_LAUNCH(E.depth(), k_project_late, grid, 256, s, E.d_program(), E.d_rabbit(), a);
    IMPLI_HIP(hipGetLastError());
    if (profile_) {   // the evaluations of this projection, summed on the host
        std::vector<uint32_t> h((size_t)nf);
        IMPLI_HIP(hipMemcpyAsync(h.data(), evals_buf_.p, (size_t)nf * 4, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
        for (uint32_t e : h) evals_ += e;
    }
    store_pointset("post_p_centroids", proj_.as<float>(), nf, false);
    store_pointset("pre_qem_verts", verts_.as<float>(), nv, false);
    if (enable_qem) {
        st.next(kStageQem);
        grad_.reserve((size_t)(nf + 1) * 12);
        if (pk) {
            const float* P = proj_.as<float>();
            float* G = grad_.as<float>();
            void* nargs[] = {&jm, &jtab, &P, &nf, &G};
            TreeJit::launch(pk->normals, blocks_for(nf), nargs, s, "impli_pt_normals_at");
        } else {
            DEPTH_LAUNCH(E.depth(), k_normals_at, blocks_for(nf), 256, s, E.d_program(), E.d_rabbit(), proj_.as<float>(), nf,
                         grad_.as<float>());
        }
        if (nv) k_qem<<<blocks_for(nv), 256, 0, s>>>(verts_.as<float>(), nv, uoff_.as<uint32_t>(), ulst_.as<int32_t>(),
                                                     proj_.as<float>(), grad_.as<float>(), avg);
        IMPLI_HIP(hipGetLastError());
        store_pointset("post_qem_verts", verts_.as<float>(), nv, false);
    }
}

void Ob02::read_counters() {   // cap hits and (profiling) evaluations since load_mesh (blocking)
    uint32_t h[2] = {0, 0};
    IMPLI_HIP(hipMemcpyAsync(h, misc_.p, sizeof h, hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
    cap_hits_ = h[1];
}

// Every stage is a roctx range (SURVEY.md section 5 tracing; rocprofv3 --marker-trace shows them
// beside the kernels).  Profiling (set_profile) adds per-stage wall times, the stream drained at
// every stage boundary.
static const char* const kStageNames[Ob02::kStages] = {"ob02 topology", "ob02 vertex resampling", "ob02 edge-length fold",
                                                       "ob02 projection", "ob02 qem", "ob02 subdivision", "ob02 fetch"};
Ob02::Stage::Stage(Ob02* o, int k) : ob(o), stage(k) {
    roctxRangePush(kStageNames[k]);
    if (ob->profile_) {
        IMPLI_HIP(hipStreamSynchronize(ob->s));
        t0 = std::chrono::steady_clock::now();
    }
}
void Ob02::Stage::next(int k) {
    roctxRangePop();
    roctxRangePush(kStageNames[k]);
    if (!ob->profile_) {
        stage = k;
        return;
    }
    IMPLI_HIP(hipStreamSynchronize(ob->s));
    const auto t1 = std::chrono::steady_clock::now();
    ob->stage_ms_[stage] += std::chrono::duration<double, std::milli>(t1 - t0).count();
    t0 = t1;
    stage = k;
}
Ob02::Stage::~Stage() {
    roctxRangePop();
    if (!ob->profile_) return;
    (void)hipStreamSynchronize(ob->s);
    ob->stage_ms_[stage] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// z^(kL) mod P for k = 0..63 and z^(64 L h) mod P for h = 0..H-1 (constant tables, grown on demand)
void Ob02::rand_tables(int64_t lanes) {
    static std::vector<uint32_t> lo, hi;
    if (lo.empty()) {
        uint32_t step[31];
        rand_jump_poly(kRandL, step);
        lo.assign(64 * 31, 0u);
        lo[0] = 1;
        for (int k = 1; k < 64; ++k) rand_poly_mulmod(&lo[31 * (k - 1)], step, &lo[31 * k]);
    }
    const int64_t H = (lanes + 63) / 64;
    if ((int64_t)hi.size() < 31 * H) {
        uint32_t step[31];
        rand_jump_poly((uint64_t)kRandL * 64, step);
        int64_t h = (int64_t)hi.size() / 31;
        if (h == 0) {
            hi.assign(31, 0u);
            hi[0] = 1;
            h = 1;
        }
        hi.resize((size_t)(31 * H));
        for (; h < H; ++h) rand_poly_mulmod(&hi[31 * (h - 1)], step, &hi[31 * h]);
    }
    if (rand_hi_rows_ < H) {
        rtab_.reserve((size_t)(64 + H) * 31 * 4);
        IMPLI_HIP(hipMemcpyAsync(rtab_.p, lo.data(), lo.size() * 4, hipMemcpyHostToDevice, s));
        IMPLI_HIP(hipMemcpyAsync(rtab_.as<uint32_t>() + 64 * 31, hi.data(), (size_t)H * 31 * 4, hipMemcpyHostToDevice, s));
        IMPLI_HIP(hipStreamSynchronize(s));   // the host vectors may grow (and move) later
        rand_hi_rows_ = H;
    }
}

void Ob02::add_rand_noise(float amplitude) {
    const int64_t n = 3 * nv;
    if (!n) return;
    GlibcRand& g = process_rand();
    uint32_t xw[61];
    g.extended_window(xw);
    const int64_t lanes = (n + kRandL - 1) / kRandL;
    rand_tables(lanes);
    uint32_t* d = misc_.as<uint32_t>() + 16;
    IMPLI_HIP(hipMemcpyAsync(d, xw, sizeof xw, hipMemcpyHostToDevice, s));
    k_rand_noise<<<blocks_for(lanes), 256, 0, s>>>(verts_.as<float>(), n, d, rtab_.as<uint32_t>(),
                                                   rtab_.as<uint32_t>() + 64 * 31, amplitude);
    IMPLI_HIP(hipGetLastError());
    g.skip((uint64_t)n);
    IMPLI_HIP(hipStreamSynchronize(s));   // xw is a stack copy
}

void Ob02::subdivide(float amplitude) {   // my_subdiv_ (centroids_projection.cpp:1314-1367)
    if (!topo_valid_) build_topology();
    Stage st(this, kStageSubdiv);
    int64_t added = 0;
    if (nf) {
        const EdgeTab t = edge_table();
        const uint64_t cap = t.mask + 1;
        DevBuf& cnt = w_;                   // per-face new midpoints (resampling weights are dead here)
        deg_.reserve((size_t)(nf + 2) * 4);
        pend_.reserve((size_t)(cap + 1) * 4);
        k_sub_count<<<blocks_for(nf), 256, 0, s>>>(nf, t, cnt.as<uint32_t>());
        scan(cnt.as<uint32_t>(), deg_.as<uint32_t>(), nf);
        uint32_t tot = 0;
        IMPLI_HIP(hipMemcpyAsync(&tot, deg_.as<uint32_t>() + nf, 4, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
        added = tot;
        const int64_t nvt = nv + added;
        vnew_.reserve((size_t)(nvt + 1) * 12);
        fnew_.reserve((size_t)(4 * nf + 1) * 12);
        if (nv) IMPLI_HIP(hipMemcpyAsync(vnew_.p, verts_.p, (size_t)nv * 12, hipMemcpyDeviceToDevice, s));
        k_sub_verts<<<blocks_for(nf), 256, 0, s>>>(verts_.as<float>(), faces_.as<int32_t>(), nf, nv, t, deg_.as<uint32_t>(),
                                                   vnew_.as<float>(), pend_.as<uint32_t>());
        k_sub_faces<<<blocks_for(nf), 256, 0, s>>>(faces_.as<int32_t>(), nf, t, pend_.as<uint32_t>(), fnew_.as<int32_t>());
        IMPLI_HIP(hipGetLastError());
        std::swap(verts_, vnew_);
        std::swap(faces_, fnew_);
        nv = nvt;
        nf = 4 * nf;
        topo_valid_ = false;
    }
    add_rand_noise(amplitude);
}

void Ob02::fetch(float* verts, int32_t* faces) {
    Stage st(this, kStageFetch);
    if (nv) IMPLI_HIP(hipMemcpyAsync(verts, verts_.p, (size_t)nv * 12, hipMemcpyDeviceToHost, s));
    if (nf) IMPLI_HIP(hipMemcpyAsync(faces, faces_.p, (size_t)nf * 12, hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
}

}  // namespace impli
