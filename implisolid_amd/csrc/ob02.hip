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
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <limits>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ifunc_device.hpp"
#include "ob02.hpp"
#include "fold.hpp"
#include "ob02_device.hpp"
#include "jit.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace impli {

using namespace dev;

// One 32-byte record per slot, so inserting or reading an edge touches one cache line (five
// arrays of one field each made k_edge_insert / k_fof five scattered lines per half-edge).  All
// fields start at 0 (one memset): key holds the edge key + 1 (0 = empty), first_inv the complement
// of the lowest face (so its start value 0 means none and atomicMax takes the minimum).
struct EdgeRec {
    unsigned long long key;
    uint32_t cnt;
    uint32_t f2[2];      // the faces of the edge's first two insertions (cnt says which hold one)
    uint32_t first_inv;  // ~(lowest face): non-manifold extras while inserting, every face after k_fof
    uint32_t last;       // highest face, likewise
    uint32_t pad;
};
static_assert(sizeof(EdgeRec) == 32, "one record per 32 bytes");
struct EdgeTab {
    EdgeRec* rec;        // cap records
    uint32_t* slot_of;   // 3 * nf
    uint64_t mask;
};


namespace {


#define DEPTH_LAUNCH(depth, KERNEL, GRID, BLOCK, STREAM, ...)                              \
    do {                                                                                   \
        if ((depth) <= 4) KERNEL<4><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);        \
        else if ((depth) <= 8) KERNEL<8><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);   \
        else if ((depth) <= 12) KERNEL<12><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__); \
        else KERNEL<16><<<(GRID), (BLOCK), 0, (STREAM)>>>(__VA_ARGS__);                    \
    } while (0)

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }


// ---- topology --------------------------------------------------------------------------------
// Degrees and umbrella slots with the atomics in LDS.  A marching-cubes mesh numbers its faces and
// vertices in cell order, and a face's corners are owned by its cell or the cells one row / one layer
// below, so a block's kWinCorners consecutive corners name vertices inside a window of a few
// thousand ids: the block counts them in LDS and adds each vertex's count to global memory once
// (about a third of the global atomics of one per corner).  A block whose ids spread wider (an
// uploaded or subdivided mesh) takes one global atomic per corner.  The counts are the
// same either way; the slots k_sort_umbrella then orders are the same set.
// PER corners per lane (256 PER per block): 16 on large meshes, 4 on small ones, whose few blocks
// would otherwise leave most of the chip idle
constexpr int kWinSlots = 8192;
struct WinRange { int32_t lo, hi; };
template <int PER>
__device__ __forceinline__ WinRange win_range(const int32_t (&v)[PER], int32_t* s_red) {
    int32_t lo = INT32_MAX, hi = INT32_MIN;
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (v[k] >= 0) { lo = min(lo, v[k]); hi = max(hi, v[k]); }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o, 64));
        hi = max(hi, __shfl_xor(hi, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_red[w] = lo; s_red[4 + w] = hi; }
    __syncthreads();
    WinRange r{min(min(s_red[0], s_red[1]), min(s_red[2], s_red[3])), max(max(s_red[4], s_red[5]), max(s_red[6], s_red[7]))};
    return r;
}
// the block's corners, lane-strided (corner c0 + k 256 + lane); -1 past the end
template <int PER>
__device__ __forceinline__ void win_load(const int32_t* __restrict__ f, int64_t n3, int64_t c0, int32_t (&v)[PER]) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int64_t i = c0 + k * 256 + threadIdx.x;
        v[k] = i < n3 ? f[i] : -1;
    }
}
template <int PER>
__global__ __launch_bounds__(256) void k_degree_win(const int32_t* __restrict__ f, int64_t n3, uint32_t* __restrict__ deg) {
    __shared__ uint32_t cnt[kWinSlots];
    __shared__ int32_t s_red[8];
    const int64_t c0 = (int64_t)blockIdx.x * (256 * PER);
    int32_t v[PER];
    win_load(f, n3, c0, v);
    const WinRange r = win_range(v, s_red);
    if (r.hi < r.lo) return;   // (no corner: never, the grid covers n3)
    const int span = r.hi - r.lo + 1;
    if (r.hi - r.lo >= kWinSlots) {
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if (v[k] >= 0) atomicAdd(&deg[v[k]], 1u);
        return;
    }
    for (int k = threadIdx.x; k < span; k += 256) cnt[k] = 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (v[k] >= 0) atomicAdd(&cnt[v[k] - r.lo], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < span; k += 256)
        if (cnt[k]) atomicAdd(&deg[r.lo + k], cnt[k]);
}

// exclusive scan of n uint32 into out[0..n] (one workgroup of 1024 lanes); zero_in: in[] is left
// zeroed (read exactly once more by its own thread: the next pass's counters need no memset)
__global__ __launch_bounds__(1024) void k_scan_u32(uint32_t* __restrict__ in, uint32_t* __restrict__ out, int64_t n,
                                                   int zero_in) {
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
        if (zero_in) in[i] = 0u;
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

// each tile's offset is the sum of the tile sums before it, summed by the tile's own block (a few
// hundred values at most for the meshes here: no separate scan launch over the sums)
__global__ __launch_bounds__(256) void k_scan_tiles(uint32_t* __restrict__ in, int64_t n, const uint32_t* __restrict__ sums,
                                                    uint32_t* __restrict__ out, int zero_in) {
    __shared__ uint32_t s_w[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer], a = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        v[k] = (base + k < n) ? in[base + k] : 0u;
        a += v[k];
    }
    uint32_t before = 0, off = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += 256) before += sums[k];
    (void)block_excl_scan256(before, s_w, off);
    uint32_t total;
    uint32_t run = off + block_excl_scan256(a, s_w, total);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (base + k < n) {
            out[base + k] = run;
            if (zero_in) in[base + k] = 0u;
        }
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = off + total;
}

// load_mesh in one launch: the mesh into the refinement state's buffers, the degree counters and
// the misc words zeroed (a memset and two copies were three host launch costs on the sync's heels)
__global__ __launch_bounds__(256) void k_load_mesh(float* __restrict__ v, const float* __restrict__ sv, int64_t nv3,
                                                   int32_t* __restrict__ f, const int32_t* __restrict__ sf, int64_t nf3,
                                                   uint32_t* __restrict__ deg, int64_t ndeg, uint32_t* __restrict__ misc,
                                                   int64_t* __restrict__ rng, int64_t nv, int64_t nf) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nv3) v[i] = sv[i];
    if (i < nf3) f[i] = sf[i];
    if (i < ndeg) deg[i] = 0u;
    if (i < 16) misc[i] = 0u;
    if (i < kRngFields) rng[i] = (i == kRngHalo + 1 || i == kRngOwn + 1) ? nv : (i & 1) ? nf : 0;   // the whole mesh
}

// the range block of one shard: every range the whole mesh, or the owned vertices [v0, v1) with
// the min / max scratch reset for the range passes (k_work_range, k_fof_range, k_face_vertex_range)
__global__ void k_ranges_set(int64_t* __restrict__ rng, int64_t v0, int64_t v1, int64_t nv, int64_t nf, int sharded) {
    const int i = threadIdx.x;
    if (i < kRngFields) rng[i] = (i == kRngHalo + 1 || i == kRngOwn + 1) ? nv : (i & 1) ? nf : 0;
    __syncthreads();
    if (!sharded) return;
    if (i == kRngOwn) rng[i] = v0;
    if (i == kRngOwn + 1) rng[i] = v1;
    if (i >= kRngScratch && i < kRngScratch + 6) rng[i] = (i & 1) ? (int64_t)-1 : INT64_MAX;   // (min, max): empty
    // the umbrella vertices start as the owned ones (an owned vertex in no face has an empty umbrella)
    if (i == kRngScratch + 6) rng[i] = v1 > v0 ? v0 : INT64_MAX;
    if (i == kRngScratch + 7) rng[i] = v1 > v0 ? v1 - 1 : (int64_t)-1;
}

// The umbrellas' face lists, the block's slot claims in LDS (see k_degree_win): each corner's rank among
// the block's corners of its vertex from an LDS atomic, one global atomic per vertex for the block's
// base in that umbrella
template <int PER>
__global__ __launch_bounds__(256) void k_fill_umbrella_win(const int32_t* __restrict__ f, int64_t n3,
                                                           const uint32_t* __restrict__ off, uint32_t* __restrict__ fill,
                                                           int32_t* __restrict__ lst) {
    __shared__ uint32_t cnt[kWinSlots];
    __shared__ int32_t s_red[8];
    const int64_t c0 = (int64_t)blockIdx.x * (256 * PER);
    int32_t v[PER];
    win_load(f, n3, c0, v);
    const WinRange r = win_range(v, s_red);
    if (r.hi < r.lo) return;
    const int span = r.hi - r.lo + 1;
    if (r.hi - r.lo >= kWinSlots) {
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if (v[k] >= 0) {
                const uint32_t p = atomicAdd(&fill[v[k]], 1u);
                lst[off[v[k]] + p] = (int32_t)((c0 + k * 256 + threadIdx.x) / 3);
            }
        return;
    }
    for (int k = threadIdx.x; k < span; k += 256) cnt[k] = 0u;
    __syncthreads();
    uint32_t rank[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) rank[k] = v[k] >= 0 ? atomicAdd(&cnt[v[k] - r.lo], 1u) : 0u;
    __syncthreads();
    for (int k = threadIdx.x; k < span; k += 256)   // counts -> the block's base in each umbrella
        if (cnt[k]) cnt[k] = atomicAdd(&fill[r.lo + k], cnt[k]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (v[k] >= 0) lst[off[v[k]] + cnt[v[k] - r.lo] + rank[k]] = (int32_t)((c0 + k * 256 + threadIdx.x) / 3);
}

// make_neighbour_faces_of_vertex lists faces in ascending order: sort each small umbrella
// (an umbrella of up to kSortRegs faces is sorted in registers: one load and one store per entry,
// where the in-memory insertion sort was a chain of dependent global loads)
constexpr int kSortRegs = 12;
constexpr int kUmbrellaRegs = 8;   // umbrellas up to this size load their faces' data at once (QEM)
__device__ __forceinline__ void sort_umbrella_at(const uint32_t* __restrict__ off, int32_t* __restrict__ lst, int64_t v) {
    const uint32_t a = off[v], e = off[v + 1];
    if (e - a <= (uint32_t)kSortRegs) {
        const int n = (int)(e - a);
        int32_t r[kSortRegs];
#pragma unroll
        for (int k = 0; k < kSortRegs; ++k) r[k] = k < n ? lst[a + k] : 0x7fffffff;
        // odd-even transposition sort of the fixed-size array (the padding sorts last)
#pragma unroll
        for (int pass = 0; pass < kSortRegs; ++pass) {
#pragma unroll
            for (int k = pass & 1; k + 1 < kSortRegs; k += 2) {
                const int32_t lo = min(r[k], r[k + 1]), hi = max(r[k], r[k + 1]);
                r[k] = lo;
                r[k + 1] = hi;
            }
        }
#pragma unroll
        for (int k = 0; k < kSortRegs; ++k)
            if (k < n) lst[a + k] = r[k];
        return;
    }
    for (uint32_t i = a + 1; i < e; ++i) {
        const int32_t x = lst[i];
        uint32_t j = i;
        while (j > a && lst[j - 1] > x) { lst[j] = lst[j - 1]; --j; }
        lst[j] = x;
    }
}
__global__ void k_sort_umbrella(const uint32_t* __restrict__ off, int32_t* __restrict__ lst, int64_t nv) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < nv) sort_umbrella_at(off, lst, v);
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
        const unsigned long long prev = atomicCAS(&t.rec[s].key, 0ull, key + 1ull);
        if (prev == 0ull || prev == key + 1ull) break;
        s = (s + 1) & t.mask;
    }
    // two atomics per half-edge: the arrival index keeps the first two faces (an edge of a closed
    // manifold mesh has exactly two); min / max over further ones only for non-manifold edges
    EdgeRec& r = t.rec[s];
    const uint32_t k = atomicAdd(&r.cnt, 1u);
    if (k < 2) {
        r.f2[k] = (uint32_t)fi;
    } else {
        atomicMax(&r.first_inv, ~(uint32_t)fi);
        atomicMax(&r.last, (uint32_t)fi);
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
    EdgeRec& r = t.rec[s];
    const uint32_t c = r.cnt, a = r.f2[0], b = c >= 2 ? r.f2[1] : a;
    // first / last face of the edge (the min / max words hold only non-manifold extras); every
    // half-edge of the slot stores the same values for the subdivision pass
    const uint32_t first = min(min(a, b), ~r.first_inv), last = max(max(a, b), r.last);
    r.first_inv = ~first;
    r.last = last;
    fof[i] = (int32_t)((first != fi) ? first : (c >= 2 ? last : 0u));
}

// build_faces_of_faces from the umbrellas, no edge table: the faces holding edge {a, b} are the
// faces of a's umbrella (ascending; a face appears once per occurrence of a) that have a half-edge
// {a, b} -- in a triangle any two of its vertices form an edge.  first / last / count are the edge
// table's (k_edge_insert + k_fof: min and max face over the edge's half-edges, and their number), so
// fof is the same for every mesh, degenerate faces included.  One thread per half-edge walks a's
// umbrella (~6 faces): 2 dependent L2 loads per face instead of a hash insert with two atomics per
// half-edge and the table's clear (76 us -> see DESIGN "OB02 on the GPU").
__device__ __forceinline__ int32_t fof_at(const int32_t* __restrict__ f, const uint32_t* __restrict__ off,
                                          const int32_t* __restrict__ lst, int64_t i) {
    const int64_t fi = i / 3;
    const int k = (int)(i - 3 * fi);
    const int32_t a = f[i], b = f[3 * fi + (k == 2 ? 0 : k + 1)];
    uint32_t first = 0xffffffffu, last = 0u, c = 0u;
    int32_t prev = -1;
    const uint32_t p1 = off[a + 1];
    for (uint32_t p = off[a]; p < p1; ++p) {
        const int32_t g = lst[p];
        if (g == prev) continue;   // a degenerate face lists a twice: count its half-edges once
        prev = g;
        const int32_t x = f[3 * (int64_t)g], y = f[3 * (int64_t)g + 1], z = f[3 * (int64_t)g + 2];
        const uint32_t n = (uint32_t)((x == a && y == b) || (x == b && y == a)) +
                           (uint32_t)((y == a && z == b) || (y == b && z == a)) +
                           (uint32_t)((z == a && x == b) || (z == b && x == a));
        if (n) {
            c += n;
            first = min(first, (uint32_t)g);
            last = max(last, (uint32_t)g);
        }
    }
    return (int32_t)((first != (uint32_t)fi) ? first : (c >= 2 ? last : 0u));
}
__global__ __launch_bounds__(256) void k_fof_umbrella(const int32_t* __restrict__ f, int64_t nf,
                                                      const uint32_t* __restrict__ off, const int32_t* __restrict__ lst,
                                                      int32_t* __restrict__ fof) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < 3 * nf) fof[i] = fof_at(f, off, lst, i);
}
// fof_at per vertex: vertex a's lane loads its umbrella's faces once (up to kFofRegs, in
// registers; the loads issue together) and answers fof_at for every half-edge leaving a, where the
// per-half-edge lanes each reloaded the whole umbrella (~6 faces, 18 corner loads, per half-edge).
// A larger umbrella takes fof_at per half-edge.
constexpr int kFofRegs = 12;
__global__ __launch_bounds__(256) void k_fof_vertex(const int32_t* __restrict__ f, int64_t nv,
                                                    const uint32_t* __restrict__ off, const int32_t* __restrict__ lst,
                                                    int32_t* __restrict__ fof) {
    const int64_t a64 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a64 >= nv) return;
    const int32_t a = (int32_t)a64;
    const uint32_t p0 = off[a], p1 = off[a + 1];
    const int n = (int)(p1 - p0);
    if (n <= 0) return;
    if (n > kFofRegs) {
        for (uint32_t p = p0; p < p1; ++p) {
            const int32_t g = lst[p];
            if (p > p0 && lst[p - 1] == g) continue;
            for (int k = 0; k < 3; ++k)
                if (f[3 * (int64_t)g + k] == a) fof[3 * (int64_t)g + k] = fof_at(f, off, lst, 3 * (int64_t)g + k);
        }
        return;
    }
    int32_t G[kFofRegs], V[kFofRegs][3];
#pragma unroll
    for (int j = 0; j < kFofRegs; ++j) G[j] = lst[p0 + (uint32_t)min(j, n - 1)];
#pragma unroll
    for (int j = 0; j < kFofRegs; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) V[j][k] = f[3 * (int64_t)G[j] + k];
#pragma unroll
    for (int j = 0; j < kFofRegs; ++j) {
        if (j >= n || (j > 0 && G[j] == G[j - 1])) continue;   // (a degenerate face lists a twice)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (V[j][k] != a) continue;
            const int32_t b = V[j][k == 2 ? 0 : k + 1];
            uint32_t first = 0xffffffffu, last = 0u, c = 0u;
#pragma unroll
            for (int m = 0; m < kFofRegs; ++m) {
                if (m >= n || (m > 0 && G[m] == G[m - 1])) continue;
                const int32_t x = V[m][0], y = V[m][1], z = V[m][2];
                const uint32_t h = (uint32_t)((x == a && y == b) || (x == b && y == a)) +
                                   (uint32_t)((y == a && z == b) || (y == b && z == a)) +
                                   (uint32_t)((z == a && x == b) || (z == b && x == a));
                if (h) {
                    c += h;
                    first = min(first, (uint32_t)G[m]);
                    last = max(last, (uint32_t)G[m]);
                }
            }
            fof[3 * (int64_t)G[j] + k] = (int32_t)((first != (uint32_t)G[j]) ? first : (c >= 2 ? last : 0u));
        }
    }
}

// ---- step 3: my_subdiv_ (centroids_projection.cpp:1314-1367) -----------------------------------
// subdivide_multiple_facets_1to4 (subdiv_1to4.hpp:147-232) numbers midpoints by first appearance of
// their edge over (face ascending; e01, e12, e20).  The first slot of an edge is in face
// first[edge], at the lowest k of that face holding the edge.
__device__ __forceinline__ bool first_slot(const EdgeTab& t, int64_t fi, int k, uint32_t s[3]) {
    return ~t.rec[s[k]].first_inv == (uint32_t)fi && (k < 1 || s[0] != s[k]) && (k < 2 || s[1] != s[k]);
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
                                                          const int64_t* __restrict__ rng, float* __restrict__ C,
                                                          float* __restrict__ N) {
    centroid_normals_body(InterpPt<D>{prog, tab}, v, f, rng, C, N);
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
                                                    const float* __restrict__ P, const int64_t* __restrict__ rng,
                                                    float* __restrict__ G, const uint32_t* __restrict__ pend, int mode) {
    normals_at_body(InterpPt<D>{prog, tab}, P, rng, G, pend, mode);
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
                               const int64_t* __restrict__ rng, float c, float* __restrict__ W) {   // faces [rng[0], rng[1])
    const int64_t i1 = rng[1];
    for (int64_t i = rng[0] + grid_lane(); i < i1; i += grid_lanes()) {
        float ki = 0;   // wi, vertex_resampling.hpp:79-91
        for (int j = 0; j < 3; ++j) ki += kij(i, fof[3 * i + j], C, N);
        W[i] = (float)(1.0 + (double)(c * ki));
    }
}

__global__ void k_resample(const uint32_t* __restrict__ off, const int32_t* __restrict__ lst, const float* __restrict__ W,
                           const float* __restrict__ C, int64_t nv, float* __restrict__ out) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= nv) return;
    const uint32_t a = off[v], e = off[v + 1];
    float sw = 0;   // vertex_resampling_VV1 :108-140
    float x = 0, y = 0, z = 0;
    for (uint32_t k = a; k < e; ++k) sw += W[lst[k]];
    for (uint32_t k = a; k < e; ++k) {
        const int32_t fj = lst[k];
        const float w = W[fj] / sw;
        x += w * C[3 * fj];
        y += w * C[3 * fj + 1];
        z += w * C[3 * fj + 2];
    }
    out[3 * v] = x; out[3 * v + 1] = y; out[3 * v + 2] = z;
}

// A shard's ranges on the device (Ob02::set_owned_vertices; no host round trip), each pass a
// min / max over the previous pass's range, one atomic pair per wave:
//   k_work_range         the work faces: faces touching an owned vertex = the first and last face
//                        of the owned vertices' umbrellas (sorted ascending)
//   k_fof_range          the faces the work faces' resampling weights read: those and their edge
//                        neighbours
//   k_face_vertex_range  the vertices of those faces (the next resampling's one-ring halo)
//   k_ranges_final       the min / max pairs to half-open ranges (an empty work range: none)
// one atomic pair per workgroup (256 lanes): same-address atomics serialise at ~11 ns each, and one
// pair per wave cost 10-30 us per range pass at 256^3
__device__ __forceinline__ void block_minmax_atomic(long long lo, long long hi, long long* out) {
    __shared__ long long s_lo[4], s_hi[4];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const long long a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    const int w = (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            lo = s_lo[k] < lo ? s_lo[k] : lo;
            hi = s_hi[k] > hi ? s_hi[k] : hi;
        }
        if (lo <= hi) {
            atomicMin(&out[0], lo);
            atomicMax(&out[1], hi);
        }
    }
}
// grid-stride range passes: a bounded grid (each block ends in one atomic pair)
inline unsigned range_blocks(int64_t n, unsigned cap = 256) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap));
}
constexpr long long kNoMin = 0x7fffffffffffffffll;

__global__ __launch_bounds__(256) void k_work_range(const uint32_t* __restrict__ off, const int32_t* __restrict__ lst,
                                                    int64_t* __restrict__ rng) {
    const int64_t v1 = rng[kRngOwn + 1];
    long long lo = kNoMin, hi = -1;
    for (int64_t v = rng[kRngOwn] + grid_lane(); v < v1; v += grid_lanes()) {
        const uint32_t a = off[v], e = off[v + 1];
        if (a < e) {
            lo = min(lo, (long long)lst[a]);
            hi = max(hi, (long long)lst[e - 1]);
        }
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch);
}

__global__ __launch_bounds__(256) void k_fof_range(const int32_t* __restrict__ fof, int64_t* __restrict__ rng) {
    const long long j0 = rng[kRngScratch], j1 = rng[kRngScratch + 1];   // inclusive (j0 > j1: empty)
    if (j0 > j1) return;   // uniform
    long long lo = kNoMin, hi = -1;
    for (long long j = j0 + grid_lane(); j <= j1; j += grid_lanes()) {
        lo = min(lo, j);
        hi = max(hi, j);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int32_t g = fof[3 * j + q];
            if (g >= 0) {
                lo = min(lo, (long long)g);
                hi = max(hi, (long long)g);
            }
        }
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch + 2);
}

__global__ __launch_bounds__(256) void k_face_vertex_range(const int32_t* __restrict__ f, int64_t* __restrict__ rng) {
    const long long j0 = rng[kRngScratch + 2], j1 = rng[kRngScratch + 3];   // inclusive (j0 > j1: empty)
    if (j0 > j1) return;   // uniform
    long long lo = kNoMin, hi = -1;
    for (long long j = j0 + grid_lane(); j <= j1; j += grid_lanes()) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int32_t v = f[3 * j + q];
            if (v >= 0) {
                lo = min(lo, (long long)v);
                hi = max(hi, (long long)v);
            }
        }
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch + 4);
}

__global__ void k_ranges_final(int64_t* __restrict__ rng) {
    if (threadIdx.x != 0) return;
    const int64_t v0 = rng[kRngOwn], v1 = rng[kRngOwn + 1];
    const int64_t* m = rng + kRngScratch;
    if (m[0] > m[1]) {   // no face touches the owned vertices
        rng[kRngWork] = rng[kRngWork + 1] = rng[kRngCen] = rng[kRngCen + 1] = 0;
        rng[kRngHalo] = v0;
        rng[kRngHalo + 1] = v1;
        return;
    }
    rng[kRngWork] = m[0];
    rng[kRngWork + 1] = m[1] + 1;
    rng[kRngCen] = m[2];
    rng[kRngCen + 1] = m[3] + 1;
    rng[kRngHalo] = m[4] < v0 ? m[4] : v0;
    rng[kRngHalo + 1] = m[5] + 1 > v1 ? m[5] + 1 : v1;
}

// ---- a shard's load and topology (Ob02::load_shard) -------------------------------------------
// The umbrellas a shard reads are those of its owned vertices (resampling, QEM) and of the vertices
// of the faces in its work range (their faces of faces): the vertices [u0, u1] (scratch pair 3,
// inclusive).  Degrees, offsets, fills and sorts cover only those, faces of faces only the work
// range; the per-vertex / per-face kernels grid-stride over the device ranges.  (The work range is a
// span: a face inside it need not touch an owned vertex, so its vertices are found from the span.)

// k_load_mesh's copies and zeroing, plus the work range (the first and last face touching an owned
// vertex), one atomic pair per wave
__global__ __launch_bounds__(256) void k_load_shard(float* __restrict__ v, const float* __restrict__ sv, int64_t nv3,
                                                    int32_t* __restrict__ f, const int32_t* __restrict__ sf, int64_t nf,
                                                    uint32_t* __restrict__ deg, int64_t ndeg, uint32_t* __restrict__ misc,
                                                    int64_t* __restrict__ rng) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nv3) v[i] = sv[i];
    if (i < 3 * nf) f[i] = sf[i];
    if (i < ndeg) deg[i] = 0u;
    if (i < 16) misc[i] = 0u;
    const int64_t v0 = rng[kRngOwn], v1 = rng[kRngOwn + 1];
    long long lo = kNoMin, hi = -1;
    if (i < nf) {
        const int32_t a = sf[3 * i], b = sf[3 * i + 1], c = sf[3 * i + 2];
        if ((a >= v0 && a < v1) || (b >= v0 && b < v1) || (c >= v0 && c < v1)) lo = hi = i;
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch);
}

// the vertices of the work range's faces, joined to the owned ones (k_ranges_set's start)
__global__ __launch_bounds__(256) void k_work_vertices(const int32_t* __restrict__ f, int64_t* __restrict__ rng) {
    const long long j0 = rng[kRngScratch], j1 = rng[kRngScratch + 1];   // inclusive (j0 > j1: empty)
    if (j0 > j1) return;   // uniform
    long long lo = kNoMin, hi = -1;
    for (long long j = j0 + grid_lane(); j <= j1; j += grid_lanes()) {
        const int32_t a = f[3 * j], b = f[3 * j + 1], c = f[3 * j + 2];
        lo = min(lo, (long long)min(min(a, b), c));
        hi = max(hi, (long long)max(max(a, b), c));
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch + 6);
}

__global__ __launch_bounds__(256) void k_degree_range(const int32_t* __restrict__ f, int64_t n3, uint32_t* __restrict__ deg,
                                                      const int64_t* __restrict__ rng) {
    const int64_t u0 = rng[kRngScratch + 6], u1 = rng[kRngScratch + 7];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n3) {
        const int32_t x = f[i];
        if (x >= u0 && x <= u1) atomicAdd(&deg[x], 1u);
    }
}

// exclusive scan of in[u0..u1] into out[u0..u1 + 1] (out[u1 + 1] = total), in[] left zeroed (the
// fill's counters): one workgroup, tiles of 8192 values staged through LDS (coalesced loads, then
// 8 consecutive values per lane; one word of padding per 32 keeps the lanes' strided reads on
// distinct banks)
constexpr int kRangeScanThreads = 1024, kRangeScanPer = 8, kRangeScanTile = kRangeScanThreads * kRangeScanPer;
__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 5); }
__global__ __launch_bounds__(kRangeScanThreads) void k_scan_range(uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                                 const int64_t* __restrict__ rng) {
    __shared__ uint32_t s_v[kRangeScanTile + kRangeScanTile / 32];
    __shared__ uint32_t s_w[kRangeScanThreads / 64];
    const int64_t u0 = rng[kRngScratch + 6], u1 = rng[kRngScratch + 7];
    if (u0 > u1) return;   // uniform
    const int64_t n = u1 - u0 + 1;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    uint32_t carry = 0;
    for (int64_t base = 0; base < n; base += kRangeScanTile) {
        const int64_t m = n - base < kRangeScanTile ? n - base : kRangeScanTile;
#pragma unroll
        for (int k = 0; k < kRangeScanPer; ++k) {
            const int i = k * kRangeScanThreads + t;
            uint32_t x = 0u;
            if (i < m) {
                x = in[u0 + base + i];
                in[u0 + base + i] = 0u;
            }
            s_v[scan_pad(i)] = x;
        }
        __syncthreads();
        uint32_t x[kRangeScanPer], sum = 0;
#pragma unroll
        for (int k = 0; k < kRangeScanPer; ++k) {
            x[k] = s_v[scan_pad(t * kRangeScanPer + k)];
            sum += x[k];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kRangeScanThreads / 64; ++w) {
            pre += w < wid ? s_w[w] : 0u;
            tot += s_w[w];
        }
        uint32_t run = carry + pre + incl - sum;
#pragma unroll
        for (int k = 0; k < kRangeScanPer; ++k) {
            s_v[scan_pad(t * kRangeScanPer + k)] = run;
            run += x[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kRangeScanPer; ++k) {
            const int i = k * kRangeScanThreads + t;
            if (i < m) out[u0 + base + i] = s_v[scan_pad(i)];
        }
        carry += tot;
        __syncthreads();   // s_v and s_w are rewritten by the next tile
    }
    if (t == 0) out[u1 + 1] = carry;
}

__global__ __launch_bounds__(256) void k_fill_range(const int32_t* __restrict__ f, int64_t n3, const uint32_t* __restrict__ off,
                                                    uint32_t* __restrict__ fill, int32_t* __restrict__ lst,
                                                    const int64_t* __restrict__ rng) {
    const int64_t u0 = rng[kRngScratch + 6], u1 = rng[kRngScratch + 7];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n3) {
        const int32_t x = f[i];
        if (x >= u0 && x <= u1) lst[off[x] + atomicAdd(&fill[x], 1u)] = (int32_t)(i / 3);
    }
}

__global__ __launch_bounds__(256) void k_sort_range(const uint32_t* __restrict__ off, int32_t* __restrict__ lst,
                                                    const int64_t* __restrict__ rng) {
    const int64_t u0 = rng[kRngScratch + 6], u1 = rng[kRngScratch + 7];
    if (u0 > u1) return;   // uniform (an empty range's start is INT64_MAX)
    for (int64_t v = u0 + grid_lane(); v <= u1; v += grid_lanes()) sort_umbrella_at(off, lst, v);
}

// faces of faces of the work faces, and (as k_fof_range) the span of those faces and their neighbours
__global__ __launch_bounds__(256) void k_fof_work(const int32_t* __restrict__ f, const uint32_t* __restrict__ off,
                                                  const int32_t* __restrict__ lst, int32_t* __restrict__ fof,
                                                  int64_t* __restrict__ rng) {
    const long long j0 = rng[kRngScratch], j1 = rng[kRngScratch + 1];   // inclusive (j0 > j1: empty)
    if (j0 > j1) return;   // uniform
    long long lo = kNoMin, hi = -1;
    for (long long i = 3 * j0 + grid_lane(); i < 3 * j1 + 3; i += grid_lanes()) {
        const int32_t g = fof_at(f, off, lst, i);
        fof[i] = g;
        const long long j = i / 3;
        lo = min(lo, j);
        hi = max(hi, j);
        if (g >= 0) {
            lo = min(lo, (long long)g);
            hi = max(hi, (long long)g);
        }
    }
    block_minmax_atomic(lo, hi, (long long*)rng + kRngScratch + 2);
}

// ---- step 2 ----------------------------------------------------------------------------------

// the fold's chunk table (fold.hpp), two passes: each chunk's terms summed in double (one wave per
// chunk, four chunks per block, the block's sum beside them) -- fused with the terms themselves when
// they are the mesh's edge lengths; then the table (one wave per chunk, 4 terms per lane, wave sums
// of the lanes' saturating partial sums, flags OR-ed), each block first summing the block sums
// before it for its chunks' estimates (the sums of the terms before each chunk) and binade windows.
// The estimates only choose windows and staging hints: the walk checks every step, so any close
// double sum serves.
constexpr int kFoldBlockChunks = 4;   // chunks per 256-thread block
__device__ __forceinline__ void fold_block_sums(double v, int64_t c, int64_t nc, double* __restrict__ cs,
                                                double* __restrict__ bs) {
    __shared__ double s_cs[kFoldBlockChunks];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) {
        if (c < nc) cs[c] = v;
        s_cs[w] = c < nc ? v : 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) bs[blockIdx.x] = ((s_cs[0] + s_cs[1]) + s_cs[2]) + s_cs[3];
}
__global__ __launch_bounds__(256) void k_fold_chunk_sums(const float* __restrict__ e, int64_t n, double* __restrict__ cs,
                                                         double* __restrict__ bs) {
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = c * kFoldChunk + 4 * lane + q;
        if (k < n) v += (double)e[k];
    }
    fold_block_sums(v, c, fold_chunks(n), cs, bs);
}
// compute_average_edge_length cp:70-82 terms, in the reference's order: term 3j + r of face j is
// |a - b|, |a - c|, |c - b| for r = 0, 1, 2; written and summed per chunk in one pass
__global__ __launch_bounds__(256) void k_fold_edge_terms(const float* __restrict__ v, const int32_t* __restrict__ f,
                                                         int64_t nf, float* __restrict__ o, double* __restrict__ cs,
                                                         double* __restrict__ bs) {
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t n = 3 * nf;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = c * kFoldChunk + 4 * lane + q;
        if (k < n) {
            const int64_t j = k / 3;
            const int r = (int)(k - 3 * j);
            const float* pa = v + 3 * f[3 * j + (r == 2 ? 2 : 0)];
            const float* pb = v + 3 * f[3 * j + (r == 1 ? 2 : 1)];
            const float x = norm2f(pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]);
            o[k] = x;
            acc += (double)x;
        }
    }
    fold_block_sums(acc, c, fold_chunks(n), cs, bs);
}

// Inclusive wave scan of u32 through DPP (gfx9: row_shr 1, 2, 4, 8 inside rows of 16 lanes, then
// row_bcast 15 and 31 into the rows above): a few cycles per step, where a ds_bpermute shuffle
// takes a round trip through LDS -- the walk is a chain of such scans
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return x;
}
__device__ __forceinline__ uint32_t lane_value(uint32_t x, int lane) {   // lane: wave-uniform
    return (uint32_t)__builtin_amdgcn_readlane((int)x, lane);
}

// The same scan over FoldPair maps (fold.hpp), in lane order: x_l <- (lanes before) then x_l.
// Lanes a DPP step does not reach read the identity (0, 0).
__device__ __forceinline__ FoldPair dpp_pair(FoldPair x, int ctrl, int row_mask) {
    FoldPair p;
    switch (ctrl) {   // the control word must be a constant of the builtin
        case 0x111: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x111, 0xf, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x111, 0xf, 0xf, false); break;
        case 0x112: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x112, 0xf, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x112, 0xf, 0xf, false); break;
        case 0x114: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x114, 0xf, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x114, 0xf, 0xf, false); break;
        case 0x118: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x118, 0xf, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x118, 0xf, 0xf, false); break;
        case 0x142: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x142, 0xa, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x142, 0xa, 0xf, false); break;
        case 0x143: p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x143, 0xc, 0xf, false);
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x143, 0xc, 0xf, false); break;
        default:    p.c0 = __builtin_amdgcn_update_dpp(0, (int)x.c0, 0x138, 0xf, 0xf, false);   // wave_shr:1
                    p.c1 = __builtin_amdgcn_update_dpp(0, (int)x.c1, 0x138, 0xf, 0xf, false); break;
    }
    (void)row_mask;
    return p;
}
__device__ __forceinline__ FoldPair wave_scan_pairs(FoldPair x) {   // inclusive
    x = fold_compose(dpp_pair(x, 0x111, 0xf), x);
    x = fold_compose(dpp_pair(x, 0x112, 0xf), x);
    x = fold_compose(dpp_pair(x, 0x114, 0xf), x);
    x = fold_compose(dpp_pair(x, 0x118, 0xf), x);
    x = fold_compose(dpp_pair(x, 0x142, 0xa), x);
    x = fold_compose(dpp_pair(x, 0x143, 0xc), x);
    return x;
}
__device__ __forceinline__ FoldPair wave_excl_pairs(FoldPair incl) { return dpp_pair(incl, 0x138, 0xf); }
__device__ __forceinline__ uint32_t pair_apply(FoldPair p, uint32_t x) { return x + ((x & 1u) ? p.c1 : p.c0); }

// hint[c] = 1: the walk will probably need chunk c's terms (the estimate is 0, the estimated sum
// crosses a power of two inside the chunk, with a margin for the float chain's drift from the double
// estimate, or the chunk is flagged in the binades the estimate puts s in) -- k_fold_walk stages
// those chunks' terms in LDS beforehand and adds them serially; the other chunks it takes a run at a
// time.  The margin only trades hinted chunks the sum does not cross in (a serial chunk each, ~2 k
// cycles) against crossings in unhinted ones (a failed run lookup and a scan of the table); the
// chain's relative drift is ~sqrt(n) 2^-25, 2^-15.5 for 500 k terms.  2^-7 hinted six chunks per
// crossing at 256^3, 2^-12 about one.
constexpr double kFoldHintMargin = 0x1p-12;
__global__ __launch_bounds__(256) void k_fold_table(const float* __restrict__ e, int64_t n, const double* __restrict__ cs,
                                                    const double* __restrict__ bs, int32_t* __restrict__ base,
                                                    FoldPair* __restrict__ pairs, uint8_t* __restrict__ flags,
                                                    uint8_t* __restrict__ hint) {
    __shared__ double s_part[4];
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the sum of the terms before this block's chunks: the block sums before it, 8 per lane per step
    // with clamped indices so that the loads issue together (one L2 round trip per 2048 blocks, where
    // a load per iteration behind the loop's bound was one round trip each).  The estimate only picks
    // runs and hints (the walk checks every step), so its summation order is free
    double p = 0.0;
    const int64_t nb = blockIdx.x;
    for (int64_t b0 = 0; b0 < nb; b0 += 256 * 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t b = b0 + u * 256 + threadIdx.x;
            const double x = bs[b < nb ? b : nb - 1];
            v[u] = b < nb ? x : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) p += v[u];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
    if (lane == 0) s_part[w] = p;
    __syncthreads();
    const int64_t nc = fold_chunks(n);
    if (c >= nc) return;   // uniform per wave
    double e0 = ((s_part[0] + s_part[1]) + s_part[2]) + s_part[3];
    for (int q = 0; q < w; ++q) e0 += cs[(int64_t)blockIdx.x * kFoldBlockChunks + q];
    const double est_c = e0, est_c1 = e0 + cs[c];
    if (lane == 0) base[c] = fold_base(est_c);
    uint32_t bits[4];   // lane l: the chunk's terms 4 l .. 4 l + 3 (the maps compose in term order)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = c * kFoldChunk + 4 * lane + q;
        bits[q] = k < n ? __float_as_uint(e[k]) : 0u;   // +0 past the end contributes nothing
    }
    const int E0 = fold_base(est_c);
    uint32_t fl34 = 0;
#pragma unroll
    for (int b = 0; b < kFoldBinades; ++b) {
        FoldPair p{0u, 0u};
        uint32_t f = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint8_t fq;
            p = fold_compose(p, fold_pair_term(bits[q], E0 + b, fq));
            f |= fq;
        }
        const FoldPair all = wave_scan_pairs(p);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o, 64);
        if (lane == 63) {
            pairs[c * kFoldBinades + b] = all;
            flags[c * kFoldBinades + b] = (uint8_t)f;
        }
        if (b == 1 || b == 2) fl34 |= f;   // the binades of the estimate and of twice it
    }
    if (lane == 0) {
        const double lo = est_c * (1.0 - kFoldHintMargin), hi = est_c1 * (1.0 + kFoldHintMargin);
        int elo = 0, ehi = 0;
        (void)frexp(lo, &elo);
        (void)frexp(hi, &ehi);
        hint[c] = (uint8_t)(!(est_c > 0.0) || elo != ehi || fl34 != 0 || !(hi < 0x1p100));
    }
}

// The serial chain itself, walked on the device by one wave (no host round trip): the exact sum s
// advances over whole chunks from the table, 64 chunks per wave step (the lanes' integer sums of the
// binade s is in, prefix-summed; the run stops at the first chunk that is flagged, outside its
// window, or would leave the binade), and inside a chunk the table could not take, over the terms
// up to the next event (a tie, an unusable term, the binade's end: the same prefix over the terms'
// rounded multiples of the spacing), the event term then added as the float add of the chain.  Every
// step either adds exactly what the chain adds (fold.hpp) or is the chain's own float add, so the
// result is the serial chain's bit for bit (fold_walk's semantics: the first NaN term decides the
// result, quieted as x86's addss quiets it; after an inf only a NaN changes the sum).  Then the
// average edge length and make_alpha_list (cp:144-194) for it, into FoldOut.
__device__ __forceinline__ float quiet_nan_of(float x) { return __uint_as_float(__float_as_uint(x) | 0x400000u); }

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// make_alpha_list(avg, 0.001, avg, 20) (cp:144-194) as the host called it: at most kMaxHalvings
// halvings (the reference loops forever on an infinite average; any finite one ends within 140)
__device__ void alpha_list_dev(float avg, FoldOut* o) {
    const float unit = avg, min_step = (float)(0.001 * 1.0);
    float step = (float)(avg * 1.0);
    int n = 0;
    for (int h = 0; h < kMaxHalvings && step > min_step; ++h) {
        step = (float)((double)step * 0.5);
        const double q = floor((double)(avg / fabsf(step)) + 0.001);
        // (int) of a double as x86's cvttsd2si: out of range or NaN gives INT_MIN
        const int total = (q >= -2147483648.0 && q < 2147483648.0) ? (int)q : (int)0x80000000u;
        const int ms = 20 < total ? 20 : total;
        for (int i = 1; i < ms + 1; i += 2) {
            const float alpha = (float)i * step;
            o->alphas[n++] = alpha / unit;
            o->alphas[n++] = -alpha / unit;
        }
    }
    o->nal = n;
}

// One block: its waves stage a window of the table (kWalkWindow chunk rows) and the terms of the
// window's hinted chunks (kWalkSlots of them) in LDS, then wave 0 walks the window from LDS; terms
// of an unhinted chunk the walk needs are read from memory.
constexpr int kWalkThreads = 1024, kWalkWindow = 4096, kWalkSlots = 32;
static_assert(kWalkWindow % 256 == 0, "the window is whole run tiles");

// Run maps (the walk's staging): for every chunk c that is not hinted, the composed map of chunks
// [c, e) in binade base + 1 (the binade of the estimate of the sum before c: where no chunk is hinted
// the estimate stays 2^-12 away from a power of two, 2^3.5 times the chain's drift from it, so the
// sum is in that binade), e = the first hinted chunk after c, the first chunk of another base, or
// the end of c's 256-chunk tile; its flags OR-ed; and the run's length.  The walk takes a whole run
// with one lookup -- exact whenever the run's map keeps the value below 2^24 (every increment is
// >= 0, so no chunk inside left the binade).  One wave per tile, 4 chunks per lane: in-lane suffixes,
// then a segmented scan of the lanes' heads across the wave.
struct FoldRun {
    int32_t base;
    uint16_t len;       // 0: a hinted chunk
    uint8_t flags;      // the run's flags in binade base + 1
    uint8_t pad;
    FoldPair run;       // the run's map in binade base + 1
};
static_assert(sizeof(FoldRun) == 16, "one 16-byte row");
constexpr int kRunTile = 256, kRunBinade = 1;

__device__ __forceinline__ uint32_t dpp_u32(uint32_t x, int ctrl, uint32_t old = 0u) {
    switch (ctrl) {
        case 0x111: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x111, 0xf, 0xf, false);
        case 0x112: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x112, 0xf, 0xf, false);
        case 0x114: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x114, 0xf, 0xf, false);
        case 0x118: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x118, 0xf, 0xf, false);
        case 0x142: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x142, 0xa, 0xf, false);
        case 0x143: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x143, 0xc, 0xf, false);
        default: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x138, 0xf, 0xf, false);   // wave_shr:1
    }
}

// One step of a segmented scan in lane order whose lower lanes hold LATER chunks (the lanes own the
// tile's chunks in reverse): a lane still open (no run end yet) appends what the lanes below it
// gathered -- their map after its own, their flags, their openness and their end.  A lane with no
// source reads the identity: the identity map, no flags, and open (so it stays open).
template <int Ctrl>
__device__ __forceinline__ void runs_step(FoldPair& x, uint32_t& f, uint32_t& open) {
    const FoldPair l = dpp_pair(x, Ctrl, 0);
    const uint32_t lf = dpp_u32(f, Ctrl), lo = dpp_u32(open, Ctrl, 1u);
    if (open) {
        x = fold_compose(x, l);
        f |= lf;
        open = lo;
    }
}
template <int Ctrl>
__device__ __forceinline__ void runs_end_step(uint32_t& end, uint32_t& open) {
    const uint32_t le = dpp_u32(end, Ctrl), lo = dpp_u32(open, Ctrl, 1u);
    if (open && !lo) end = le;   // the first run end below: kept once found
    if (open) open = lo;
}

// One wave: the run records of one 256-chunk tile (tile * kRunTile < nc), stored through `put(c, rec)`.
template <class Put>
__device__ __forceinline__ void fold_runs_tile(const FoldPair* __restrict__ pairs, const uint8_t* __restrict__ flags,
                                               const int32_t* __restrict__ base, const uint8_t* __restrict__ hint, int nc,
                                               int tile, const Put& put) {
    const int lane = threadIdx.x & 63;
    // lane l owns the tile's chunks 4 (63 - l) .. 4 (63 - l) + 3, so the DPP scans, which move data
    // up the lanes, carry the later chunks' maps to the earlier ones
    const int c0 = tile * kRunTile + 4 * (63 - lane);
    bool in[5], hin[5];
    int bs[5];
    // every load first (one round trip): the chunks' pairs and flags in binade base + 1
    FoldPair pv[4];
    uint32_t fv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = c0 + j < nc ? c0 + j : nc - 1;
        pv[j] = pairs[(int64_t)c * kFoldBinades + kRunBinade];
        fv[j] = flags[(int64_t)c * kFoldBinades + kRunBinade];
    }
    // the lane's chunks and the one after them: loaded unconditionally (a clamped index), so the
    // compiler issues the ten loads together instead of one round trip per short-circuited load
    uint32_t hv[5];
    int32_t bv[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int c = c0 + j;
        in[j] = c < nc && (j < 4 || lane > 0);
        const int cq = in[j] ? c : 0;
        hv[j] = hint[cq];
        bv[j] = base[cq];
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {   // bitwise, no short circuit
        hin[j] = in[j] & (hv[j] != 0u);
        bs[j] = bv[j] & -(int32_t)in[j];
    }
    bool bnd[4];   // a run ends after chunk j
#pragma unroll
    for (int j = 0; j < 4; ++j) bnd[j] = !in[j] || !in[j + 1] || hin[j] || hin[j + 1] || bs[j + 1] != bs[j];
    int nextb[4];   // the first run end at or after j in the lane (4: none)
    nextb[3] = bnd[3] ? 3 : 4;
#pragma unroll
    for (int j = 2; j >= 0; --j) nextb[j] = bnd[j] ? j : nextb[j + 1];
    const uint32_t lane_open = nextb[0] == 4 ? 1u : 0u;
    // where the run that leaves this lane ends: the first run end in the later lanes
    uint32_t end = lane_open ? 0u : (uint32_t)(c0 + nextb[0]), eo = lane_open;
    runs_end_step<0x111>(end, eo);
    runs_end_step<0x112>(end, eo);
    runs_end_step<0x114>(end, eo);
    runs_end_step<0x118>(end, eo);
    runs_end_step<0x142>(end, eo);
    runs_end_step<0x143>(end, eo);
    const int tail_end = (int)dpp_u32(end, 0x138);   // gathered by the lanes holding the later chunks
    FoldPair v[4];
    uint32_t f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool use = in[j] && !hin[j];
        v[j] = use ? pv[j] : FoldPair{0u, 0u};
        f[j] = use ? fv[j] : 0u;
    }
    FoldPair acc[4];   // in-lane: from chunk j to the first run end at or after it
    uint32_t fa[4];
    acc[3] = v[3];
    fa[3] = f[3];
#pragma unroll
    for (int j = 2; j >= 0; --j) {
        acc[j] = bnd[j] ? v[j] : fold_compose(v[j], acc[j + 1]);
        fa[j] = bnd[j] ? f[j] : (f[j] | fa[j + 1]);
    }
    // the lanes' heads: each lane's map from its first chunk to the end of its run
    FoldPair x = acc[0];
    uint32_t xf = fa[0], open = lane_open;
    runs_step<0x111>(x, xf, open);
    runs_step<0x112>(x, xf, open);
    runs_step<0x114>(x, xf, open);
    runs_step<0x118>(x, xf, open);
    runs_step<0x142>(x, xf, open);
    runs_step<0x143>(x, xf, open);
    const FoldPair tail = dpp_pair(x, 0x138, 0);
    const uint32_t tailf = dpp_u32(xf, 0x138);
    FoldRun rec[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool cont = nextb[j] == 4;   // the run goes on past this lane
        rec[j].base = bs[j];
        rec[j].len = (uint16_t)((!in[j] || hin[j]) ? 0 : (cont ? tail_end - (c0 + j) + 1 : nextb[j] - j + 1));
        rec[j].flags = (uint8_t)(cont ? (fa[j] | tailf) : fa[j]);
        rec[j].pad = 0;
        rec[j].run = cont ? fold_compose(acc[j], tail) : acc[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (in[j]) put(c0 + j, rec[j]);
}

// kCycles: the clock64 split of the walk and its step counts (diagnostics, implisolid_debug_fold
// with IMPLISOLID_FOLD_STATS): each reading is an s_memtime whose wait also drains the wave's LDS
// operations, and the counters hold scalar registers the walk needs, so the production walk is
// compiled without them
template <bool kCycles>
__device__ __forceinline__ long long walk_clock() {
    if constexpr (kCycles) return clock64();
    return 0;
}

// One block.  Its waves stage a window of the run maps (kWalkWindow chunks) and the terms of the
// window's hinted chunks (up to kWalkSlots) in LDS; wave 0 walks the window:
//   - at a chunk boundary, the run map of the chunk in the binade the sum is in: one lookup takes
//     the chunks up to the next hinted one;
//   - a hinted chunk, or one inside a run whose map does not hold (the sum crossed a binade where
//     the estimate did not), goes term by term: its terms added serially, the chain's own float
//     adds (256 dependent adds); a run that failed is first re-entered by a scan of the
//     chunk table (64 lanes x 4 chunks) that finds the chunk where it failed;
//   - a chunk holding a NaN or an infinity goes in segments (its terms as maps of the current
//     binade up to each event, the event term as the chain's own add).
// Every step adds exactly what the chain adds, so the sum is the serial chain's bit for bit
// (fold_walk's semantics: the first NaN term decides the result, quieted as x86's addss quiets it;
// after an inf only a NaN changes the sum).  Then the average edge length and make_alpha_list
// (cp:144-194) for it, into FoldOut.
template <bool kCycles>
__global__ __launch_bounds__(kWalkThreads) void k_fold_walk(const float* __restrict__ e, int64_t n64,
                                                            const int32_t* __restrict__ base, const FoldPair* __restrict__ pairs,
                                                            const uint8_t* __restrict__ flags, const uint8_t* __restrict__ hint,
                                                            int64_t nf, FoldOut* __restrict__ out) {
    __shared__ uint4 w_rec[kWalkWindow];   // the chunks' FoldRun records
    __shared__ int16_t w_slot[kWalkWindow];
    __shared__ int16_t w_slot_chunk[kWalkSlots];
    __shared__ uint4 w_terms[kWalkSlots][64];   // a staged chunk's terms (bits), 4 per lane
    __shared__ int w_nslots;
    __shared__ int w_wcnt[kWalkThreads / 64];
    __shared__ int w_ready[kWalkSlots];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = (int)n64;   // < 2^31 (launch_fold checks)
    const int nc = (int)fold_chunks(n64);
    float s = 0.f;       // wave 0: the chain's exact value after term k - 1
    int k = 0;
    int table_chunks = 0;
    bool done = false;   // wave 0: a NaN or an inf decided the result
    int st_zero = 0, st_lookup = 0, st_scan = 0, st_terms = 0, st_serial = 0, st_global = 0;
    long long cyc_stage = 0, cyc_walk = 0, cyc_lookup = 0, cyc_scan = 0, cyc_serial = 0, cyc_seg = 0, cyc_wait = 0;
    for (int c0 = 0; c0 < nc; c0 += kWalkWindow) {
        const long long tc0 = walk_clock<kCycles>();
        const int wn = nc - c0 < kWalkWindow ? nc - c0 : kWalkWindow;
        if (t < kWalkSlots) w_ready[t] = 0;
        __syncthreads();   // the previous window's walk is over
        // the window's run records, a wave per 256-chunk tile (the window is whole tiles), and the
        // tiles' hinted-chunk counts
        static_assert(kWalkWindow / kRunTile <= kWalkThreads / 64, "a tile per wave");
        if (wid * kRunTile < wn) {
            fold_runs_tile(pairs, flags, base, hint, nc, c0 / kRunTile + wid, [&](int c, const FoldRun& r) {
                w_rec[c - c0] = *reinterpret_cast<const uint4*>(&r);
            });
        }
        __syncthreads();
        // slots for the window's hinted chunks (len 0) in chunk order: a tile's lanes hold its chunks
        // in reverse (fold_runs_tile), so a chunk's rank counts the hinted chunks of the higher lanes
        int tile_hinted = 0, before = 0, total = 0;
        uint64_t hb[4];
        const int ct = wid * kRunTile + 4 * (63 - lane);   // this lane's first chunk in the window
        if (wid * kRunTile < wn) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                hb[j] = __ballot(ct + j < wn && (w_rec[ct + j < wn ? ct + j : 0].y & 0xffffu) == 0u);
#pragma unroll
            for (int j = 0; j < 4; ++j) tile_hinted += (int)__popcll((unsigned long long)hb[j]);
        }
        if (lane == 0) w_wcnt[wid] = tile_hinted;
        __syncthreads();
        for (int w = 0; w < kWalkThreads / 64; ++w) {
            before += w < wid ? w_wcnt[w] : 0;
            total += w_wcnt[w];
        }
        if (wid * kRunTile < wn) {
            const uint64_t above = lane < 63 ? ~0ull << (lane + 1) : 0ull;
            int rank = before;
#pragma unroll
            for (int j = 0; j < 4; ++j) rank += (int)__popcll((unsigned long long)(hb[j] & above));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool h = (hb[j] >> lane) & 1ull;
                if (ct + j < wn) w_slot[ct + j] = (int16_t)(h && rank < kWalkSlots ? rank : -1);
                if (h && rank < kWalkSlots) w_slot_chunk[rank] = (int16_t)(ct + j);
                rank += h ? 1 : 0;
            }
        }
        if (t == 0) w_nslots = total;
        __syncthreads();
        const int ns = w_nslots < kWalkSlots ? w_nslots : kWalkSlots;
        if constexpr (kCycles) cyc_stage += walk_clock<kCycles>() - tc0;
        if (wid != 0) {
            // waves 1.. stage the slots' terms while wave 0 walks, each then its ready flag (the walk
            // waits for it)
            for (int sl = wid - 1; sl < ns; sl += kWalkThreads / 64 - 1) {
                const int kk0 = (c0 + w_slot_chunk[sl]) * kFoldChunk + 4 * lane;
                uint4 tb;
                tb.x = kk0 + 0 < n ? __float_as_uint(e[kk0 + 0]) : 0u;
                tb.y = kk0 + 1 < n ? __float_as_uint(e[kk0 + 1]) : 0u;
                tb.z = kk0 + 2 < n ? __float_as_uint(e[kk0 + 2]) : 0u;
                tb.w = kk0 + 3 < n ? __float_as_uint(e[kk0 + 3]) : 0u;
                w_terms[sl][lane] = tb;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(&w_ready[sl], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            continue;
        }
        const long long tc1 = walk_clock<kCycles>();
        const int kend_w = (c0 + wn) * kFoldChunk < n ? (c0 + wn) * kFoldChunk : n;
        while (!done && k < kend_w) {   // uniform over wave 0
            // the walk's state is wave-uniform: kept in scalar registers, so its branches are scalar
            k = __builtin_amdgcn_readfirstlane(k);
            s = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s)));
            if (!(s >= 0x1p-100f && s <= 0x1p100f)) {
                if constexpr (kCycles) ++st_zero;
                if (s == 0.f) {   // 0 + (+-0) = +0: on to the first term of nonzero magnitude (or NaN)
                    const int kk = k + lane;
                    const bool in = kk < kend_w;
                    const uint64_t m = __ballot(in && (__float_as_uint(e[in ? kk : k]) & 0x7fffffffu) != 0u);
                    if (!m) {
                        k = k + 64 < kend_w ? k + 64 : kend_w;
                        continue;
                    }
                    k += __ffsll((unsigned long long)m) - 1;
                } else if (s == INFINITY) {   // only a NaN term changes it: the first one decides
                    for (; k < n; k += 64) {
                        const int kk = k + lane;
                        const float x = e[kk < n ? kk : 0];
                        const uint64_t m = __ballot(kk < n && x != x);
                        if (m) {
                            s = quiet_nan_of(e[k + __ffsll((unsigned long long)m) - 1]);
                            break;
                        }
                    }
                    done = true;
                    break;
                }
                // tiny, huge or negative, or the first nonzero term after zeros: one float add
                const float x = e[k];
                if (x != x) { s = quiet_nan_of(x); done = true; break; }
                s = s + x;
                ++k;
                continue;
            }
            int E = 0;
            // s in [2^(E-1), 2^E), spacing 2^(E-24), and su = s / 2^(E-24) in [2^23, 2^24): from the
            // bits (s is normal here), scalar
            const uint32_t sb = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s));
            E = (int)((sb >> 23) & 0xffu) - 126;
            uint32_t su = (sb & 0x7fffffu) | 0x800000u;
            const long long tA = walk_clock<kCycles>();
            int ic = k / kFoldChunk - c0;
            bool failed = false;   // a run map that did not hold: the table scan below re-enters it
            if ((k & (kFoldChunk - 1)) == 0) {
                // runs, one lookup each, while their maps keep the value in this binade (E and the
                // integer su carry the exact value; s is formed once at the end)
                for (;;) {
                    uint4 r0 = w_rec[ic];   // FoldRun: base, len | flags << 16, run map
                    // the whole record in one LDS read: without this the compiler reads len first
                    // and the rest behind the len test, two round trips per lookup
                    asm volatile("" : "+v"(r0.x), "+v"(r0.y), "+v"(r0.z), "+v"(r0.w));
                    r0.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0.x);   // uniform: scalar branches
                    r0.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0.y);
                    r0.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0.z);
                    r0.w = (uint32_t)__builtin_amdgcn_readfirstlane((int)r0.w);
                    const int len = (int)(r0.y & 0xffffu);
                    if (len == 0) break;   // a hinted chunk: its terms
                    if constexpr (kCycles) ++st_lookup;
                    const bool fb = E - (int)r0.x != kRunBinade || ((r0.y >> 16) & 0xffu) != 0u;
                    const uint32_t x2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)pair_apply(FoldPair{r0.z, r0.w}, su));
                    if (fb || x2 >= kFoldCap) {
                        failed = true;
                        break;
                    }
                    su = x2;   // exact: the run's map kept it in this binade
                    table_chunks += len;
                    k += len * kFoldChunk;
                    ic += len;
                    if (k >= kend_w) break;
                }
                s = __uint_as_float(((uint32_t)(E + 126) << 23) | (su & 0x7fffffu));   // su in [2^23, 2^24)
                if (k >= kend_w) {
                    if (k > n) k = n;
                    if constexpr (kCycles) cyc_lookup += walk_clock<kCycles>() - tA;
                    continue;
                }
                if constexpr (kCycles) cyc_lookup += walk_clock<kCycles>() - tA;
            }
            if (failed) {
                // the run does not hold: a scan of the chunk table from here (64 lanes x 4 chunks,
                // the lanes' maps in the binade s is in, prefix-composed) finds the chunk where the
                // value first reaches 2^24 or meets a flagged chunk; the chunks before it are exact
                if constexpr (kCycles) ++st_scan;
                const int cc = k / kFoldChunk;
                FoldPair tp[4];
                bool ok[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = cc + 4 * lane + j;
                    const int cq = c < nc ? c : nc - 1;
                    const int bb = E - base[cq];
                    const bool inb = c < nc && c < c0 + wn && bb >= 0 && bb < kFoldBinades;
                    const int64_t cell = (int64_t)cq * kFoldBinades + (inb ? bb : 0);
                    tp[j] = pairs[cell];
                    ok[j] = inb & (flags[cell] == 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (!ok[j]) tp[j] = FoldPair{0u, 0u};
                FoldPair p{0u, 0u};
#pragma unroll
                for (int j = 0; j < 4; ++j) p = fold_compose(p, tp[j]);
                const FoldPair incl = wave_scan_pairs(p), excl = wave_excl_pairs(incl);
                uint32_t v = pair_apply(excl, su), before = v;
                int first = 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) {   // selects, no branches (one wave's dependent chain)
                    const uint32_t v2 = pair_apply(tp[j], v);
                    const bool live = first == 4, stop = live && (!ok[j] || v2 >= kFoldCap);
                    before = stop ? v : before;
                    first = stop ? j : first;
                    v = (live && !stop) ? v2 : v;
                }
                const uint64_t lm = __ballot(first < 4);
                const int L = lm ? __ffsll((unsigned long long)lm) - 1 : 63;
                const int fbk = lm ? 4 * L + (int)lane_value((uint32_t)first, L) : 256;
                if (fbk > 0) {
                    const uint32_t tt = lm ? lane_value(before, L) : pair_apply(FoldPair{lane_value(incl.c0, 63),
                                                                                           lane_value(incl.c1, 63)}, su);
                    s = ldexpf((float)tt, E - 24);   // < 2^24: exact in this binade
                    table_chunks += fbk;
                    k += fbk * kFoldChunk;
                    if (k >= kend_w || !lm) {   // the window's end, or the scan's reach: go on from there
                        if (k > n) k = n;
                        if constexpr (kCycles) cyc_scan += walk_clock<kCycles>() - tA;
                        continue;
                    }
                    k = __builtin_amdgcn_readfirstlane(k);
                    ic = k / kFoldChunk - c0;
                }
                if constexpr (kCycles) cyc_scan += walk_clock<kCycles>() - tA;
            }
            // the chunk the runs could not take (hinted, or the sum crosses a binade in it), from k on
            const long long tB = walk_clock<kCycles>();
            if constexpr (kCycles) ++st_terms;
            const int kc = k & ~(kFoldChunk - 1);
            const int kend = kc + kFoldChunk < n ? kc + kFoldChunk : n;
            // its terms: from LDS if staged (a hinted chunk; uniform: one chunk), else from memory
            uint32_t xb[4];
            const int sl = __builtin_amdgcn_readfirstlane((int)w_slot[ic]);
            if (sl >= 0) {
                const long long tw = walk_clock<kCycles>();
                while (__hip_atomic_load(&w_ready[sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                    __builtin_amdgcn_s_sleep(1);
                if constexpr (kCycles) cyc_wait += walk_clock<kCycles>() - tw;
                const uint4 tb = w_terms[sl][lane];
                xb[0] = tb.x; xb[1] = tb.y; xb[2] = tb.z; xb[3] = tb.w;
            } else {
                if constexpr (kCycles) ++st_global;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kk = kc + 4 * lane + j;
                    xb[j] = __float_as_uint(e[kk < n ? kk : kc]);
                }
            }
            // Added serially, the chain's own float adds: every lane runs the same chain over the
            // wave's terms read lane by lane (v_readlane, eight reads ahead of their adds; the terms
            // outside [k, kend) masked to -0 in their lanes, which adds nothing to any value): 256
            // dependent adds, ~2.2 k cycles, less than locating a crossing in the chunk (a scan of
            // the lanes' term maps, ~3.3 k cycles with the maps staged).  Unless a NaN or an infinity
            // is among the terms from k on: then in segments below.
            {
                uint32_t m[4];
                bool special = false;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kk = kc + 4 * lane + j;
                    const bool act = kk >= k && kk < kend;
                    special = special || (act && (xb[j] & 0x7f800000u) == 0x7f800000u);
                    m[j] = act ? xb[j] : 0x80000000u;
                }
                if (!__ballot(special)) {
                    if constexpr (kCycles) ++st_serial;
                    float sv = s;
#pragma unroll
                    for (int l = 0; l < 64; l += 2) {
                        uint32_t r[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) r[i] = (uint32_t)__builtin_amdgcn_readlane((int)m[i & 3], l + (i >> 2));
#pragma unroll
                        for (int i = 0; i < 8; ++i) sv = sv + __uint_as_float(r[i]);
                    }
                    s = sv;
                    k = kend;
                    if constexpr (kCycles) cyc_serial += walk_clock<kCycles>() - tB;
                    continue;
                }
            }
            for (; !done && k < kend;) {   // segments of the chunk, each ending at an event
                if (!(s >= 0x1p-100f && s <= 0x1p100f)) break;   // the outer loop's term-by-term paths
                const uint32_t sb = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s));
                E = (int)((sb >> 23) & 0xffu) - 126;   // as above
                su = (sb & 0x7fffffu) | 0x800000u;
                FoldPair tp[4], p{0u, 0u};
                bool bad[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kk = kc + 4 * lane + j;
                    uint8_t fl = 0;
                    const bool act = kk >= k && kk < kend;
                    tp[j] = fold_pair_term(act ? xb[j] : 0u, E, fl);
                    bad[j] = act && fl != 0;
                    p = fold_compose(p, tp[j]);
                }
                const FoldPair incl = wave_scan_pairs(p), excl = wave_excl_pairs(incl);
                uint32_t v = pair_apply(excl, su), before = v, xe = 0;
                int first = 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) {   // selects, no branches
                    const uint32_t v2 = pair_apply(tp[j], v);
                    const bool live = first == 4, stop = live && (bad[j] || v2 >= kFoldCap);
                    before = stop ? v : before;
                    xe = stop ? xb[j] : xe;
                    first = stop ? j : first;
                    v = (live && !stop) ? v2 : v;
                }
                const uint64_t lm = __ballot(first < 4);
                if (!lm) {
                    s = ldexpf((float)pair_apply(FoldPair{lane_value(incl.c0, 63), lane_value(incl.c1, 63)}, su), E - 24);
                    k = kend;
                    break;
                }
                const int L = __ffsll((unsigned long long)lm) - 1;
                const int jf = (int)lane_value((uint32_t)first, L);
                s = ldexpf((float)lane_value(before, L), E - 24);   // exact: the chain before the event
                const float x = __uint_as_float(lane_value(xe, L));
                k = kc + 4 * L + jf + 1;
                if (x != x) { s = quiet_nan_of(x); done = true; break; }
                s = s + x;   // the event term: the chain's own float add
                if (k >= kend) break;
            }
            if constexpr (kCycles) cyc_seg += walk_clock<kCycles>() - tB;
        }
        if constexpr (kCycles) cyc_walk += walk_clock<kCycles>() - tc1;
    }
    if (t == 0) {
        out->sum = s;
        out->table_chunks = table_chunks;
        out->steps[0] = st_zero; out->steps[1] = st_lookup; out->steps[2] = st_scan; out->steps[3] = st_terms;
        out->steps[4] = st_serial; out->steps[5] = st_global; out->steps[6] = 0;
        out->cycles[0] = cyc_stage; out->cycles[1] = cyc_walk; out->cycles[2] = cyc_lookup; out->cycles[3] = cyc_scan;
        out->cycles[4] = cyc_serial; out->cycles[5] = cyc_seg; out->cycles[6] = cyc_wait;
        const float avg = (float)((double)s / (3. * (double)nf));
        out->avg = avg;
        alpha_list_dev(avg, out);
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
                                             const float* __restrict__ N, const FoldOut* __restrict__ fo) {
    const int64_t vi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (vi >= nv) return;
    const float maxd = fo->avg;   // the average edge length (k_fold_walk), in stream order
    float* v = verts + 3 * vi;
    const float ox = v[0], oy = v[1], oz = v[2];
    float A[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, b[3] = {0.f, 0.f, 0.f};
    auto accum = [&](float nx, float ny, float nz, float cx, float cy, float cz) {
        const float Px = cx - ox, Py = cy - oy, Pz = cz - oz;
        const float nn00 = nx * nx, nn01 = nx * ny, nn02 = nx * nz, nn11 = ny * ny, nn12 = ny * nz, nn22 = nz * nz;
        A[0][0] += nn00; A[0][1] += nn01; A[0][2] += nn02;
        A[1][0] += nn01; A[1][1] += nn11; A[1][2] += nn12;
        A[2][2] += nn22; A[2][0] += nn02; A[2][1] += nn12;
        b[0] -= nn00 * Px + nn01 * Py + nn02 * Pz;
        b[1] -= nn01 * Px + nn11 * Py + nn12 * Pz;
        b[2] -= nn02 * Px + nn12 * Py + nn22 * Pz;
    };
    const uint32_t a0 = off[vi], a1 = off[vi + 1];
    if (a1 > a0 && a1 - a0 <= (uint32_t)kUmbrellaRegs) {
        // a small umbrella's loads all in flight at once (indices, then normals and centroids;
        // past its end the last face is loaded again and not summed), summed in the same order
        const int n = (int)(a1 - a0);
        int32_t id[kUmbrellaRegs];
#pragma unroll
        for (int k = 0; k < kUmbrellaRegs; ++k) id[k] = lst[a0 + (k < n ? k : n - 1)];
        float q[kUmbrellaRegs][6];
#pragma unroll
        for (int k = 0; k < kUmbrellaRegs; ++k) {
            q[k][0] = N[3 * id[k]]; q[k][1] = N[3 * id[k] + 1]; q[k][2] = N[3 * id[k] + 2];
            q[k][3] = C[3 * id[k]]; q[k][4] = C[3 * id[k] + 1]; q[k][5] = C[3 * id[k] + 2];
        }
#pragma unroll
        for (int k = 0; k < kUmbrellaRegs; ++k)
            if (k < n) accum(q[k][0], q[k][1], q[k][2], q[k][3], q[k][4], q[k][5]);
    } else {
        for (uint32_t k = a0; k < a1; ++k) {
            const int32_t ni = lst[k];
            accum(N[3 * ni], N[3 * ni + 1], N[3 * ni + 2], C[3 * ni], C[3 * ni + 1], C[3 * ni + 2]);
        }
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
// boost::random::mt11213b (seed 12) + uniform_01<float>: make_random_pm1(n, 3, 1e-6)
// (make_random_pm1.hpp:15-29): the twist in three runs (no index wrap inside), tempering of a
// whole block at once, then uniform_01's rejection of draws that round to 1.0f (pert_prefix)
// make_random_pm1(n, 3, 1e-6) draws its 3 n values in order from a generator seeded afresh (12) on
// every call: the table of n faces is the first 3 n values of one sequence, whatever n.  One
// process-wide prefix of that sequence is kept and grown on demand (the generator's state carries
// over; a grown table is a new immutable snapshot, so readers of an older one are undisturbed), and
// the first Ob02 of a process starts drawing kPertAhead faces' worth on a host thread, so a later
// build of a new face count finds its table drawn.  (Round 5 drew each face count's table afresh.)
constexpr int64_t kPertAhead = int64_t(1) << 20;
struct PertSeq {
    std::mutex mu;
    uint32_t x[351], t[351];
    int next = 351;   // the next tempered word of t (351: twist first)
    bool seeded = false;
    std::shared_ptr<const std::vector<float>> vals;
};
PertSeq& pert_seq() {   // never destroyed: a draw-ahead thread may still use it while the process exits
    static PertSeq* S = new PertSeq();
    return *S;
}
std::shared_ptr<const std::vector<float>> pert_prefix(int64_t n, bool only_if_ready = false) {
    constexpr int N = 351, M = 175;
    constexpr uint32_t UM = 0xffffffffu << 19, LM = ~UM, A = 0xccab8ee7u;
    PertSeq& S = pert_seq();
    std::lock_guard<std::mutex> lock(S.mu);
    const size_t want = (size_t)(3 * n);
    if (S.vals && S.vals->size() >= want) return S.vals;
    if (only_if_ready) return nullptr;
    if (!S.seeded) {
        S.x[0] = 12u;
        for (int i = 1; i < N; ++i) S.x[i] = 1812433253u * (S.x[i - 1] ^ (S.x[i - 1] >> 30)) + (uint32_t)i;
        S.seeded = true;
    }
    auto v = std::make_shared<std::vector<float>>();
    const size_t have = S.vals ? S.vals->size() : 0;
    const size_t target = std::max(want, 2 * have);
    v->reserve(target);
    if (S.vals) v->assign(S.vals->begin(), S.vals->end());
    const float factor = 1.0f / ((float)4294967295u + 1.0f);
    const double amp = (double)0.000001f;
    uint32_t* x = S.x;
    while (v->size() < target) {
        if (S.next == N) {   // the twist in three runs (no index wrap inside), then a block's tempering
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
                S.t[i] = z;
            }
            S.next = 0;
        }
        const float r = (float)S.t[S.next++] * factor;
        if (!(r < 1.0f)) continue;   // uniform_01's rejection of draws that round to 1.0f
        v->push_back((float)(((double)r * 2.0 - 1.0) * amp));
    }
    S.vals = v;
    return S.vals;
}
// the draw ahead, started once per process on a thread of its own, never joined: it touches only
// the never-destroyed sequence (no HIP call, nothing a static destructor frees), so a process that
// exits while it draws needs no wait for it (a static future's destructor would have blocked exit)
void pert_draw_ahead() {
    static std::once_flag once;
    std::call_once(once, [] { std::thread([] { (void)pert_prefix(kPertAhead); }).detach(); });
}

}  // namespace

// The perturbation table of a face count on one device, shared by every Ob02 of the process
// (the shards of one process, the builds of one engine): drawn once on a host thread, copied once
// into pinned memory and uploaded once, on the stream of the Ob02 that first needs it; `ready`
// orders every other stream after that upload.  The last few (device, face count) tables are kept.
struct PertDev {
    int device = -1;
    int64_t nf = -1;
    HostBuf pinned;
    DevBuf buf;
    hipEvent_t ready = nullptr;
    ~PertDev() {
        if (ready) (void)hipEventSynchronize(ready);
        if (ready) (void)hipEventDestroy(ready);
        buf.release();
        pinned.release();
    }
};

namespace {
std::shared_ptr<PertDev> pert_device_table(int64_t nf, std::future<std::shared_ptr<const std::vector<float>>>& job,
                                           hipStream_t s, bool& uploaded_here) {
    // never destroyed: the tables' HIP resources are left to the process's exit (a static
    // destructor's hipEventSynchronize / hipHostFree would run while the runtime shuts down)
    static std::mutex mu;
    static auto& cache = *new std::deque<std::shared_ptr<PertDev>>();
    int device = 0;
    IMPLI_HIP(hipGetDevice(&device));
    std::lock_guard<std::mutex> lock(mu);
    uploaded_here = false;
    for (auto& e : cache)   // any table of this device at least nf faces long: its prefix is nf's
        if (e->device == device && e->nf >= nf) return e;
    auto host = job.get();
    auto e = std::make_shared<PertDev>();
    e->device = device;
    // the upload: the next power of two of faces the drawn prefix holds (a later, larger mesh
    // uploads a longer table; a smaller one reads this one's prefix)
    int64_t up = 1;
    while (up < nf) up <<= 1;
    e->nf = std::min<int64_t>(up, (int64_t)(host->size() / 3));
    const size_t bytes = (size_t)e->nf * 3 * 4;
    e->pinned.reserve(bytes + 16);
    std::memcpy(e->pinned.p, host->data(), bytes);
    e->buf.reserve(bytes + 16);
    IMPLI_HIP(hipEventCreateWithFlags(&e->ready, hipEventDisableTiming));
    IMPLI_HIP(hipMemcpyAsync(e->buf.p, e->pinned.p, bytes, hipMemcpyHostToDevice, s));
    IMPLI_HIP(hipEventRecord(e->ready, s));
    uploaded_here = true;
    cache.emplace_front(e);
    if (cache.size() > 8) cache.pop_back();   // a table still in use lives on in its Ob02s
    return e;
}
}  // namespace

Ob02::Ob02(Engine& e, hipStream_t st) : E(e), s(st) {
    misc_.reserve(512);
}

void Ob02::begin_load(const float*& d_verts, int64_t nv_, int64_t nf_, float* d_work) {
    normals_ahead_ = false;
    nv = nv_;
    nf = nf_;
    if (d_work) {   // the caller's vertex array is the working one (sharded loop): no copy
        verts_.attach(d_work, (size_t)nv * 12);   // exactly the caller's 3 nv floats
        d_verts = d_work;
    } else if (verts_.ext) {
        verts_.release();   // a previous attach: own buffer again
    }
    if (vnew_.ext) vnew_.release();   // (a subdivision's swap left a caller's array here)
    // the snapshots' device buffers are kept for the next build's stores (a hipFree per set per
    // build cost 80-380 us of device-wide synchronisation)
    for (auto& kv : snaps_) kv.second.valid = false;
    pointsets_.clear();
    cap_hits_ = 0;
    evals_ = 0;
    jit_launches_ = 0;
    avg_edge_ = 0.f;
    avg_valid_ = true;
    for (double& t : stage_ms_) t = 0.0;
    if (!verts_.ext) verts_.reserve((size_t)(nv + 1) * 12);
    faces_.reserve((size_t)(nf + 1) * 12);
    deg_.reserve((size_t)(nv + 1) * 4);
    rng_.reserve(kRngFields * sizeof(int64_t));
}

// the meshes whose first centroid normals run beside their topology (load_mesh)
constexpr int64_t kNormalsAheadFaces = 400000;

void Ob02::load_mesh(const float* d_verts, int64_t nv_, const int32_t* d_faces, int64_t nf_, float* d_work,
                     bool normals_ahead) {
    begin_load(d_verts, nv_, nf_, d_work);
    Stage st(this, kStageTopology);
    // the mesh copied, the degree counters and misc ((unused), cap hits, evaluations) zeroed, the
    // range block set to the whole mesh
    const int64_t nmax = std::max<int64_t>(std::max<int64_t>(3 * nv, 3 * nf), nv + 1);
    k_load_mesh<<<blocks_for(std::max<int64_t>(nmax, 16)), 256, 0, s>>>(verts_.as<float>(), d_verts,
                                                                       verts_.as<float>() == d_verts ? 0 : 3 * nv, faces_.as<int32_t>(),
                                                                       d_faces, 3 * nf, deg_.as<uint32_t>(), nv + 1,
                                                                       misc_.as<uint32_t>(), rng_.as<int64_t>(), nv, nf);
    start_perturbations();   // host thread, overlaps the topology and resampling kernels
    // the first resampling's centroid normals need no topology: with the caller's word that a
    // resampling comes next, they run on the side stream beside the topology passes (not while
    // profiling, whose stages are drained one by one)
    // (large meshes only: on a small one the side stream's event costs more latency than the
    // overlap saves, 0.70 -> 0.72 ms at 128^3, profiles/r06t_normals_ahead_ab.txt)
    if (normals_ahead && nf >= kNormalsAheadFaces && !profile_) {
        reserve_topology();   // cen_ / nrm_ sized before the side stream writes them
        est_cen_ = nf;        // the whole mesh (whole_ranges below)
        if (!side_s_) IMPLI_HIP(hipStreamCreateWithFlags(&side_s_, hipStreamNonBlocking));
        if (!mesh_ready_) IMPLI_HIP(hipEventCreateWithFlags(&mesh_ready_, hipEventDisableTiming));
        if (!cnormals_done_) IMPLI_HIP(hipEventCreateWithFlags(&cnormals_done_, hipEventDisableTiming));
        IMPLI_HIP(hipEventRecord(mesh_ready_, s));
        IMPLI_HIP(hipStreamWaitEvent(side_s_, mesh_ready_, 0));
        launch_centroid_normals(side_s_);
        IMPLI_HIP(hipEventRecord(cnormals_done_, side_s_));
        normals_ahead_ = true;
    }
    build_topology(true);
    whole_ranges();
}

void Ob02::load_shard(const float* d_verts, int64_t nv_, const int32_t* d_faces, int64_t nf_, float* d_work, int64_t v0,
                      int64_t v1) {
    if (v0 < 0 || v1 < v0 || v1 > nv_) throw InputError("ob02: owned vertex range outside the mesh");
    if (v0 == 0 && v1 == nv_) {
        load_mesh(d_verts, nv_, d_faces, nf_, d_work);
        set_owned_vertices(0, nv_);
        return;
    }
    begin_load(d_verts, nv_, nf_, d_work);
    Stage st(this, kStageTopology);
    reserve_topology();
    int64_t* r = rng_.as<int64_t>();
    k_ranges_set<<<1, 64, 0, s>>>(r, v0, v1, nv, nf, 1);
    const int64_t nmax = std::max<int64_t>(std::max<int64_t>(3 * nv, 3 * nf), nv + 1);
    k_load_shard<<<blocks_for(std::max<int64_t>(nmax, 16)), 256, 0, s>>>(verts_.as<float>(), d_verts,
                                                                        verts_.as<float>() == d_verts ? 0 : 3 * nv,
                                                                        faces_.as<int32_t>(), d_faces, nf, deg_.as<uint32_t>(),
                                                                        nv + 1, misc_.as<uint32_t>(), r);
    start_perturbations();   // host thread, overlaps the kernels below
    own_v0_ = v0;
    own_v1_ = v1;
    sharded_ = true;
    hrng_valid_ = false;
    const int64_t nown = v1 - v0;
    est_work_ = std::min<int64_t>(nf, 2 * nown + nown / 4 + 4096);
    est_cen_ = std::min<int64_t>(nf, est_work_ + 4096);
    const int64_t est_umb = std::min<int64_t>(nv, nown + nown / 4 + 4096);
    uint32_t* deg = deg_.as<uint32_t>();
    uint32_t* off = uoff_.as<uint32_t>();
    int32_t* lst = ulst_.as<int32_t>();
    if (nf) {
        k_work_vertices<<<range_blocks(est_work_), 256, 0, s>>>(faces_.as<int32_t>(), r);
        k_degree_range<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, deg, r);
        k_scan_range<<<1, kRangeScanThreads, 0, s>>>(deg, off, r);
        k_fill_range<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, off, deg, lst, r);
        k_sort_range<<<blocks_for(est_umb), 256, 0, s>>>(off, lst, r);
        k_fof_work<<<range_blocks(3 * est_work_, 512), 256, 0, s>>>(faces_.as<int32_t>(), off, lst, fof_.as<int32_t>(), r);
        k_face_vertex_range<<<range_blocks(est_cen_), 256, 0, s>>>(faces_.as<int32_t>(), r);
    } else {
        // no faces: every umbrella empty
        k_scan_range<<<1, kRangeScanThreads, 0, s>>>(deg, off, r);
    }
    k_ranges_final<<<1, 64, 0, s>>>(r);
    IMPLI_HIP(hipGetLastError());
    etab_valid_ = false;
    topo_valid_ = true;
    topo_partial_ = true;
}

void Ob02::whole_ranges() {   // host side of the range block's whole-mesh state
    own_v0_ = 0;
    own_v1_ = nv;
    const int64_t h[8] = {0, nv, 0, nf, 0, nf, 0, nv};
    std::memcpy(hrng_, h, sizeof h);
    hrng_valid_ = true;
    est_work_ = est_cen_ = nf;
    sharded_ = false;
}

// The shard's ranges are found on the device, in stream order (k_work_range -> k_fof_range ->
// k_face_vertex_range -> k_ranges_final), and the per-face passes read them there: no host round
// trip (the three read-backs of round 4 cost 0.3-0.5 ms per shard).  Their grids are sized by an
// estimate -- a mesh has about two faces per vertex, plus a layer of faces at the slab's boundary --
// and grid-stride over whatever the range turns out to be.
void Ob02::set_owned_vertices(int64_t v0, int64_t v1) {
    normals_ahead_ = false;
    if (v0 < 0 || v1 < v0 || v1 > nv) throw InputError("ob02: owned vertex range outside the mesh");
    if (!topo_valid_ || topo_partial_) build_topology();
    rng_.reserve(kRngFields * sizeof(int64_t));
    const bool sharded = !(v0 == 0 && v1 == nv);
    k_ranges_set<<<1, 64, 0, s>>>(rng_.as<int64_t>(), v0, v1, nv, nf, sharded ? 1 : 0);
    if (!sharded) {
        whole_ranges();
        IMPLI_HIP(hipGetLastError());
        return;
    }
    own_v0_ = v0;
    own_v1_ = v1;
    sharded_ = true;
    hrng_valid_ = false;
    const int64_t nown = v1 - v0;
    est_work_ = std::min<int64_t>(nf, 2 * nown + nown / 4 + 4096);
    est_cen_ = std::min<int64_t>(nf, est_work_ + 4096);
    int64_t* r = rng_.as<int64_t>();
    if (nown) k_work_range<<<range_blocks(nown), 256, 0, s>>>(uoff_.as<uint32_t>(), ulst_.as<int32_t>(), r);
    if (est_work_) k_fof_range<<<range_blocks(est_work_), 256, 0, s>>>(fof_.as<int32_t>(), r);
    if (est_cen_) k_face_vertex_range<<<range_blocks(est_cen_), 256, 0, s>>>(faces_.as<int32_t>(), r);
    k_ranges_final<<<1, 64, 0, s>>>(r);
    IMPLI_HIP(hipGetLastError());
}

// every rank's owned range, all-gathered into equal padded rows (row r: rank r's 3 (v1 - v0)
// floats), unpacked into this rank's vertex array except its own range (one kernel on the stream;
// the offsets travel as a kernel argument, so nothing is staged in host memory)
constexpr int kMaxUnpackRanks = 64;
struct UnpackOffsets {
    int64_t o[kMaxUnpackRanks + 1];
};
__global__ void k_unpack_ranges(float* __restrict__ v, const float* __restrict__ rows, int64_t row_len, UnpackOffsets voff,
                                int self) {
    const int r = blockIdx.y;
    if (r == self) return;
    const int64_t n = 3 * (voff.o[r + 1] - voff.o[r]);
    float* dst = v + 3 * voff.o[r];
    const float* src = rows + (int64_t)r * row_len;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

void Ob02::unpack_ranges(const float* d_rows, int64_t row_len, const std::vector<int64_t>& voff, int self) {
    normals_ahead_ = false;
    const int world = (int)voff.size() - 1;
    if (world < 1 || voff.back() != nv || self < 0 || self >= world) throw InputError("ob02: bad owned ranges");
    if (world > kMaxUnpackRanks) throw InputError("ob02: more than 64 ranks in one unpack");
    UnpackOffsets o{};
    int64_t longest = 0;
    for (int r = 0; r < world; ++r) {
        if (voff[r + 1] < voff[r] || 3 * (voff[r + 1] - voff[r]) > row_len) throw InputError("ob02: bad owned ranges");
        longest = std::max<int64_t>(longest, voff[r + 1] - voff[r]);
    }
    for (int r = 0; r <= world; ++r) o.o[r] = voff[r];
    const unsigned bx = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (3 * longest + 255) / 256), 1024);
    k_unpack_ranges<<<dim3(bx, (unsigned)world), 256, 0, s>>>(verts_.as<float>(), d_rows, row_len, o, self);
    IMPLI_HIP(hipGetLastError());
}

void Ob02::ranges(int64_t out[8]) {
    if (!hrng_valid_) {   // blocking: read the device's range block back once
        int64_t h[kRngFields];
        IMPLI_HIP(hipMemcpyAsync(h, rng_.p, sizeof h, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
        const int64_t m[8] = {h[kRngOwn], h[kRngOwn + 1], h[kRngWork], h[kRngWork + 1], h[kRngCen], h[kRngCen + 1],
                              h[kRngHalo], h[kRngHalo + 1]};
        const bool ok = 0 <= m[0] && m[0] <= m[1] && m[1] <= nv && 0 <= m[2] && m[2] <= m[3] && m[3] <= nf &&
                        0 <= m[4] && m[4] <= m[5] && m[5] <= nf && (m[2] == m[3] || (m[4] <= m[2] && m[3] <= m[5])) &&
                        0 <= m[6] && m[6] <= m[0] && m[1] <= m[7] && m[7] <= nv;
        if (!ok) throw HipError("ob02: the device's shard ranges are inconsistent");
        std::memcpy(hrng_, m, sizeof m);
        hrng_valid_ = true;
    }
    std::memcpy(out, hrng_, sizeof hrng_);
}

EdgeTab Ob02::edge_table() {
    uint64_t cap = 1024;
    while (cap < (uint64_t)(4 * nf + 16)) cap <<= 1;
    etab_.reserve((size_t)cap * sizeof(EdgeRec) + (size_t)(3 * nf + 1) * 4);
    EdgeTab t;
    t.rec = etab_.as<EdgeRec>();
    t.slot_of = reinterpret_cast<uint32_t*>(t.rec + cap);
    t.mask = cap - 1;
    return t;
}

void Ob02::reserve_topology() {
    deg_.reserve((size_t)(nv + 1) * 4);
    uoff_.reserve((size_t)(nv + 2) * 4);
    ulst_.reserve((size_t)(3 * nf + 1) * 4);
    fof_.reserve((size_t)(3 * nf + 1) * 4);
    cen_.reserve((size_t)(nf + 1) * 12);
    nrm_.reserve((size_t)(nf + 1) * 12);
    w_.reserve((size_t)(nf + 1) * 4);
}

void Ob02::build_topology(bool deg_zeroed) {
    // umbrellas
    reserve_topology();
    if (!deg_zeroed) IMPLI_HIP(hipMemsetAsync(deg_.p, 0, (size_t)(nv + 1) * 4, s));
    // 16 corners per lane from 1.5 M corners (512^3: 2.2 M), else 4 (at 128^3, 340 k corners, the
    // 16-corner blocks were 83: slower than the per-corner atomics of round 5)
    const bool big = 3 * nf >= 1500000;
    const int64_t per_block = big ? 256 * 16 : 256 * 4;
    const unsigned wblocks = (unsigned)((3 * nf + per_block - 1) / per_block);
    if (nf && big) k_degree_win<16><<<wblocks, 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, deg_.as<uint32_t>());
    else if (nf) k_degree_win<4><<<wblocks, 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, deg_.as<uint32_t>());
    scan(deg_.as<uint32_t>(), uoff_.as<uint32_t>(), nv, true);   // deg_ left zeroed: the fill counters
    if (nf && big) k_fill_umbrella_win<16><<<wblocks, 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, uoff_.as<uint32_t>(),
                                                        deg_.as<uint32_t>(), ulst_.as<int32_t>());
    else if (nf) k_fill_umbrella_win<4><<<wblocks, 256, 0, s>>>(faces_.as<int32_t>(), 3 * nf, uoff_.as<uint32_t>(),
                                                        deg_.as<uint32_t>(), ulst_.as<int32_t>());
    if (nv) k_sort_umbrella<<<blocks_for(nv), 256, 0, s>>>(uoff_.as<uint32_t>(), ulst_.as<int32_t>(), nv);
    // faces of faces, from the umbrellas (the edge table is built only for subdivision)
    // per vertex on large meshes; per half-edge on small ones (more lanes in flight)
    if (nf && nv && big)
        k_fof_vertex<<<blocks_for(nv), 256, 0, s>>>(faces_.as<int32_t>(), nv, uoff_.as<uint32_t>(), ulst_.as<int32_t>(),
                                                    fof_.as<int32_t>());
    else if (nf)
        k_fof_umbrella<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), nf, uoff_.as<uint32_t>(), ulst_.as<int32_t>(),
                                                          fof_.as<int32_t>());
    etab_valid_ = false;
    IMPLI_HIP(hipGetLastError());
    topo_valid_ = true;
    topo_partial_ = false;
}

void Ob02::scan(uint32_t* in, uint32_t* out, int64_t n, bool zero_in) {
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles <= 1) {
        k_scan_u32<<<1, 1024, 0, s>>>(in, out, n, zero_in ? 1 : 0);
        return;
    }
    scan_tmp_.reserve((size_t)(tiles + 1) * 4);
    uint32_t* sums = scan_tmp_.as<uint32_t>();
    k_scan_tile_sums<<<(unsigned)tiles, 256, 0, s>>>(in, n, sums);
    k_scan_tiles<<<(unsigned)tiles, 256, 0, s>>>(in, n, sums, out, zero_in ? 1 : 0);
}

// STORE_POINTSET: a device snapshot now (stream-ordered, no host sync), copied to the host only
// when pointsets() is asked for
void Ob02::store_pointset(const char* key, const float* d, int64_t n, bool keep_first) {
    if (!capture_pointsets) return;
    auto it = snaps_.find(key);
    const bool stored = it != snaps_.end() && it->second.valid;
    if (keep_first ? stored : !capture_replace) return;
    Snapshot& e = snaps_[key];
    e.buf.reserve((size_t)(n + 1) * 12);
    e.n = n;
    e.valid = true;
    if (n) IMPLI_HIP(hipMemcpyAsync(e.buf.p, d, (size_t)n * 12, hipMemcpyDeviceToDevice, s));
}

const std::map<std::string, std::vector<float>>& Ob02::pointsets() {
    pointsets_.clear();
    for (auto& kv : snaps_) {
        if (!kv.second.valid) continue;
        std::vector<float>& h = pointsets_[kv.first];
        h.resize((size_t)kv.second.n * 3);
        if (kv.second.n) IMPLI_HIP(hipMemcpyAsync(h.data(), kv.second.buf.p, (size_t)kv.second.n * 12, hipMemcpyDeviceToHost, s));
    }
    IMPLI_HIP(hipStreamSynchronize(s));
    return pointsets_;
}

Ob02::~Ob02() {
    if (pert_job_.valid()) pert_job_.wait();
    if (prep_done_) (void)hipEventDestroy(prep_done_);
    if (early_done_) (void)hipEventDestroy(early_done_);
    if (normals_done_) (void)hipEventDestroy(normals_done_);
    if (mesh_ready_) (void)hipEventDestroy(mesh_ready_);
    if (cnormals_done_) (void)hipEventDestroy(cnormals_done_);
    if (side_s_) (void)hipStreamDestroy(side_s_);
    dir_.release();
    evals_buf_.release();
    for (DevBuf* b : {&verts_, &faces_, &vnew_, &cen_, &nrm_, &w_, &fof_, &uoff_, &ulst_, &etab_, &deg_, &proj_, &grad_,
                      &fn_, &norms_, &pend_, &misc_, &fnew_, &rtab_, &scan_tmp_, &fold_sum_, &fold_out_})
        b->release();
    for (auto& kv : snaps_) kv.second.buf.release();
}

// f and normalised grad f at the centroids of the centroid faces (the range block's kRngCen) on q
void Ob02::launch_centroid_normals(hipStream_t q) {
    const int64_t* rng = rng_.as<int64_t>();
    if (const TreeJit::PointKernels* pk = E.point_jit(s)) {
        const float *m = E.d_mats(), *tab = E.d_rabbit(), *v = verts_.as<float>();
        const int32_t* f = faces_.as<int32_t>();
        const int64_t* rc = rng + kRngCen;
        float *C = cen_.as<float>(), *N = nrm_.as<float>();
        void* args[] = {&m, &tab, &v, &f, &rc, &C, &N};
        TreeJit::launch(pk->cnormals, blocks_for(est_cen_), args, q, "impli_pt_centroid_normals");
        ++jit_launches_;
    } else {
        DEPTH_LAUNCH(E.depth(), k_centroid_normals, blocks_for(est_cen_), 256, q, E.d_program(), E.d_rabbit(),
                     verts_.as<float>(), faces_.as<int32_t>(), rng + kRngCen, cen_.as<float>(), nrm_.as<float>());
    }
}

void Ob02::vertex_resampling(float c) {
    if (!nf) return;
    const bool ahead = normals_ahead_;   // this mesh's centroid normals, computed beside its topology
    normals_ahead_ = false;
    if (!topo_valid_) build_topology();
    Stage st(this, kStageResample);
    store_pointset("pre_resampling_vertices", verts_.as<float>(), nv, true);   // vertex_resampling.hpp:176-180
    // centroids and normals of the centroid faces, weights of the work faces, vertices [v0, v1) (the
    // whole mesh unless sharded); the face ranges are read on the device (the range block)
    const int64_t* rng = rng_.as<int64_t>();
    if (ahead) IMPLI_HIP(hipStreamWaitEvent(s, cnormals_done_, 0));
    else if (est_cen_ > 0) launch_centroid_normals(s);
    if (est_work_ > 0)
        k_face_weights<<<blocks_for(est_work_), 256, 0, s>>>(cen_.as<float>(), nrm_.as<float>(), fof_.as<int32_t>(),
                                                              rng + kRngWork, c, w_.as<float>());
    // in place: the new positions are weighted sums of the centroids alone (vertex_resampling.hpp
    // :93-141), which were computed above, so nothing reads the old positions any more and the
    // vertex buffer stays the same (a sharded caller's exchange writes into it directly)
    if (own_v1_ > own_v0_)
        k_resample<<<blocks_for(own_v1_ - own_v0_), 256, 0, s>>>(uoff_.as<uint32_t>() + own_v0_, ulst_.as<int32_t>(),
                                                                  w_.as<float>(), cen_.as<float>(), own_v1_ - own_v0_,
                                                                  verts_.as<float>() + 3 * own_v0_);
    IMPLI_HIP(hipGetLastError());
    store_pointset("post_resampling_vertices", verts_.as<float>(), nv, true);   // :207-211
}

// the fold's device buffers in one allocation: [pairs (cells) | bases i32 (chunks) | flags u8
// (cells) | hints u8 (chunks)], then the chunks' double sums and the estimates (chunks + 1 each)
struct FoldLayout {
    int64_t chunks, cells;
    size_t cs_off, est_off, bytes;
    explicit FoldLayout(int64_t n) : chunks(fold_chunks(n)), cells(fold_chunks(n) * kFoldBinades) {
        const size_t tab = (size_t)cells * sizeof(FoldPair) + (size_t)chunks * 4 + (size_t)cells + (size_t)chunks;
        cs_off = (tab + 15) & ~(size_t)15;
        est_off = cs_off + (size_t)(chunks + 1) * 8;
        bytes = est_off + (size_t)(chunks + 1) * 8;
    }
};
// the terms array of a fold: n terms, padded to whole chunks (the walk reads a chunk's terms with
// scalar loads of the whole chunk)
inline size_t fold_terms_bytes(int64_t n) { return (size_t)(fold_chunks(n) + 1) * kFoldChunk * sizeof(float); }

// the table passes on `ts`, then the walk on `ws` after them (ws may be ts); with d_verts the terms
// are the mesh's edge lengths, computed into d_terms by the first pass
void launch_fold(float* d_terms, int64_t n, int64_t nf, const float* d_verts, const int32_t* d_faces, char* d_tab,
                 FoldOut* d_out, hipStream_t ts, hipStream_t ws, hipEvent_t table_done, bool cycles = false) {
    if (n >= ((int64_t)1 << 31) - kFoldChunk) throw InputError("edge-length fold: more than 2^31 terms");
    const FoldLayout L(n);
    FoldPair* d_pair = reinterpret_cast<FoldPair*>(d_tab);
    int32_t* d_base = reinterpret_cast<int32_t*>(d_pair + L.cells);
    uint8_t* d_flags = reinterpret_cast<uint8_t*>(d_base + L.chunks);
    uint8_t* d_hint = d_flags + L.cells;
    double* d_cs = reinterpret_cast<double*>(d_tab + L.cs_off);
    double* d_bs = reinterpret_cast<double*>(d_tab + L.est_off);   // block sums (chunks / 4 + 1)
    if (L.cells) {
        const unsigned blocks = blocks_for(L.chunks * 64);
        if (d_verts) k_fold_edge_terms<<<blocks, 256, 0, ts>>>(d_verts, d_faces, nf, d_terms, d_cs, d_bs);
        else k_fold_chunk_sums<<<blocks, 256, 0, ts>>>(d_terms, n, d_cs, d_bs);
        k_fold_table<<<blocks, 256, 0, ts>>>(d_terms, n, d_cs, d_bs, d_base, d_pair, d_flags, d_hint);
    }
    if (ws != ts) {
        IMPLI_HIP(hipEventRecord(table_done, ts));
        IMPLI_HIP(hipStreamWaitEvent(ws, table_done, 0));
    }
    const int64_t nfa = nf > 0 ? nf : 1;
    if (cycles)
        k_fold_walk<true><<<1, kWalkThreads, 0, ws>>>(d_terms, n, d_base, d_pair, d_flags, d_hint, nfa, d_out);
    else
        k_fold_walk<false><<<1, kWalkThreads, 0, ws>>>(d_terms, n, d_base, d_pair, d_flags, d_hint, nfa, d_out);
}

// compute_average_edge_length (cp:70-82) is one serial float chain in face order.  The terms, the
// fold's chunk table (fold.hpp) and the walk (k_fold_walk, one wave) run on s, back to back; the
// projection's prep pass, which does not need the average, runs meanwhile on a side stream (from
// the mesh as s left it), and s waits for it before the searches.  The walk is the long one, so
// the searches follow it in s's own order (a wait on the walk from another stream cost ~13 us of
// cross-stream signalling per repeat).  No host round trip: the average and the alpha list stay in
// device memory (FoldOut) for the searches and QEM.
hipStream_t Ob02::start_edge_fold() {
    norms_.reserve(std::max<size_t>((size_t)(nf + 1) * 12, fold_terms_bytes(3 * nf)));
    const FoldLayout L(3 * nf);
    fold_sum_.reserve(L.bytes);
    fold_out_.reserve(sizeof(FoldOut));
    if (!side_s_) IMPLI_HIP(hipStreamCreateWithFlags(&side_s_, hipStreamNonBlocking));
    if (!mesh_ready_) IMPLI_HIP(hipEventCreateWithFlags(&mesh_ready_, hipEventDisableTiming));
    if (!prep_done_) IMPLI_HIP(hipEventCreateWithFlags(&prep_done_, hipEventDisableTiming));
    IMPLI_HIP(hipEventRecord(mesh_ready_, s));
    IMPLI_HIP(hipStreamWaitEvent(side_s_, mesh_ready_, 0));
    launch_fold(norms_.as<float>(), 3 * nf, nf, verts_.as<float>(), faces_.as<int32_t>(), fold_sum_.as<char>(),
                fold_out_.as<FoldOut>(), s, s, nullptr);
    avg_valid_ = false;
    return side_s_;   // the prep pass goes here
}

void Ob02::finish_edge_fold() {   // s waits for the prep pass (stream order, no host sync)
    IMPLI_HIP(hipEventRecord(prep_done_, side_s_));
    IMPLI_HIP(hipStreamWaitEvent(s, prep_done_, 0));
}

// the fold alone on given terms (diagnostics / tests): the same table kernels and walk as a
// projection, on the null stream; returns the chain's sum and the chunks taken from the table
float debug_fold(const float* h_terms, int64_t n, int* table_chunks, long long* stats, int* trace) {
    const FoldLayout L(n);
    DevBuf terms, tab, fo;
    terms.reserve(fold_terms_bytes(n));
    tab.reserve(L.bytes);
    fo.reserve(sizeof(FoldOut));
    if (n) IMPLI_HIP(hipMemcpy(terms.p, h_terms, (size_t)n * 4, hipMemcpyHostToDevice));
    launch_fold(terms.as<float>(), n, n, nullptr, nullptr, tab.as<char>(), fo.as<FoldOut>(), 0, 0, nullptr,
                stats != nullptr && std::getenv("IMPLISOLID_FOLD_STATS") != nullptr);
    IMPLI_HIP(hipGetLastError());
    FoldOut h;
    IMPLI_HIP(hipMemcpy(&h, fo.p, offsetof(FoldOut, alphas), hipMemcpyDeviceToHost));
    if (trace) std::memcpy(trace, h.trace, sizeof h.trace);
    terms.release();
    tab.release();
    fo.release();
    if (table_chunks) *table_chunks = h.table_chunks;
    if (stats) {   // steps: zero / single adds, run lookups, scans, term steps, serial chunks, global term loads;
                   // cycles: staging, walk, lookups, scans, serial chunks, segments
        for (int i = 0; i < 4; ++i) stats[i] = h.steps[i];
        stats[4] = h.cycles[0];
        stats[5] = h.cycles[1];
        stats[6] = h.cycles[2];
        stats[7] = h.cycles[3];
        stats[8] = h.cycles[4];
        stats[9] = h.cycles[5];
        stats[10] = h.steps[4];
        stats[11] = h.steps[5];
        stats[12] = h.cycles[6];
    }
    return h.sum;
}

float Ob02::last_average_edge() {   // blocking: the last fold's average, read back once
    if (!avg_valid_ && fold_out_.p) {
        FoldOut h;
        IMPLI_HIP(hipMemcpyAsync(&h, fold_out_.p, offsetof(FoldOut, alphas), hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
        avg_edge_ = h.avg;
        avg_valid_ = true;
    }
    return avg_edge_;
}

// make_random_pm1(nf, 3, 1e-6) (centroids_projection.cpp:239-262) is seeded afresh (seed 12) on
// every call, so its table is a prefix of one sequence (pert_prefix): drawn on a host thread when the
// loaded mesh needs more of it than is drawn, and uploaded once per device and length -- the
// projection never waits for it unless a centroid needs the type-2 directions before the thread is
// done
void Ob02::start_perturbations() {
    if (pert_nf_ == nf || nf == 0) return;
    if (pert_job_.valid()) pert_job_.wait();
    const int64_t n = nf;
    if (auto ready = pert_prefix(n, true)) {   // drawn already: no thread
        std::promise<std::shared_ptr<const std::vector<float>>> p;
        p.set_value(ready);
        pert_job_ = p.get_future();
        pert_draw_ahead();
    } else {   // this mesh's table first, then the draw ahead behind it
        pert_job_ = std::async(std::launch::async, [n] {
            auto v = pert_prefix(n);
            pert_draw_ahead();
            return v;
        });
    }
    pert_nf_ = nf;
    pert_dev_.reset();
}

const float* Ob02::perturbations() {
    if (pert_nf_ != nf) start_perturbations();
    if (!pert_dev_) {
        bool mine = false;
        pert_dev_ = pert_device_table(nf, pert_job_, s, mine);
        // another Ob02's upload (on its stream): order this stream after it, once
        if (!mine) IMPLI_HIP(hipStreamWaitEvent(s, pert_dev_->ready, 0));
    }
    return pert_dev_->buf.as<float>();
}

// the late pass's group widths (A/B switches, read once): IMPLISOLID_LATE_WMAX (4..64),
// IMPLISOLID_LATE_FLAT (0/1)
static int late_wmax() {
    static const int w = [] {
        const char* e = std::getenv("IMPLISOLID_LATE_WMAX");
        const int v = e ? std::atoi(e) : 64;
        return v >= 64 ? 64 : v >= 32 ? 32 : v >= 16 ? 16 : v >= 8 ? 8 : 4;
    }();
    return w;
}
static int late_flat() {
    static const int f = [] {
        const char* e = std::getenv("IMPLISOLID_LATE_FLAT");
        return e ? (std::atoi(e) ? 1 : 0) : 1;
    }();
    return f;
}

// the work faces from which the point module's early search runs with 2 lanes per face
constexpr int64_t kEarly2Faces = 400000;

void Ob02::centroids_projection(bool enable_qem) {
    normals_ahead_ = false;   // (vertex_resampling: the first step after load_mesh only)
    if (!nf) return;
    if (!topo_valid_) build_topology();
    Stage st(this, kStageEdgeFold);
    const hipStream_t ps = start_edge_fold();   // the prep pass's stream
    proj_.reserve((size_t)(nf + 1) * 12);
    fn_.reserve((size_t)(nf + 1) * 12);
    dir_.reserve((size_t)(nf + 1) * 12);
    pend_.reserve((size_t)(nf + 2) * 4);
    if (profile_) evals_buf_.reserve((size_t)(nf + 1) * 4);
    DevBuf& fcbuf = w_;   // f(centroid) per face; the resampling weights are dead here
    // the work faces (every face unless sharded; the range block on the device), grids sized by
    // the estimate
    const int64_t nw = est_work_;
    ProjArgs a{};
    a.v = verts_.as<float>();
    a.f = faces_.as<int32_t>();
    a.rng = rng_.as<int64_t>() + kRngWork;
    a.out = proj_.as<float>();
    a.fn = fn_.as<float>();
    a.fc = fcbuf.as<float>();
    a.pend = pend_.as<uint32_t>();
    a.early_chunk = early_chunk();
    a.late_wmax = late_wmax();
    a.late_flat = late_flat();
    a.cap_hits = misc_.as<uint32_t>() + 1;
    a.cen = cen_.as<float>();
    a.dir = dir_.as<float>();
    a.evals = profile_ ? evals_buf_.as<uint32_t>() : nullptr;
    const TreeJit::PointKernels* pk = E.point_jit(s);   // one choice for the whole projection
    const float *jm = E.d_mats(), *jtab = E.d_rabbit();
    void* jargs[] = {&jm, &jtab, &a};
    if (nw <= 0) {
        // no face touches this rank's vertices: nothing to project (the fold still ran, as on
        // every rank)
    } else if (pk) {
        TreeJit::launch(pk->prep, blocks_for(nw), jargs, ps, "impli_pt_project_prep");
        ++jit_launches_;
    } else {
        DEPTH_LAUNCH(E.depth(), k_project_prep, blocks_for(nw), 256, ps, E.d_program(), E.d_rabbit(), a);
    }
    finish_edge_fold();
    store_pointset("pre_p_centroids", cen_.as<float>(), nf, false);   // cp:1236-1238: the centroids
    a.fold = fold_out_.as<FoldOut>();
    st.next(kStageProject);
    // lanes per face of the point module's searches (kProjGroup; IMPLISOLID_PROJ_GROUP experiments)
    static const int pgroup = [] {
        const char* e = std::getenv("IMPLISOLID_PROJ_GROUP");
        const int v = e ? std::atoi(e) : 0;
        return v == 2 || v == 8 ? v : kProjGroup;
    }();
    // large meshes: the point module's 2-lane early search (project_early_body<2>); the late pass
    // keeps 4 lanes per face
    const bool early2 = pk && pgroup == kProjGroup && nw >= kEarly2Faces;
    const unsigned grid = blocks_for(nw * (pk ? pgroup : kProjGroup));
    const unsigned late_grid = blocks_for(nw * kProjGroup);
    // centroids left unresolved need the randomised directions (types 2-6): the late pass covers
    // every face and reads the early pass's per-face flags on the device (no host round trip)
    a.pert = perturbations();
    // the QEM normals of the faces the early pass resolved run on the side stream beside the late
    // pass (latency-bound: a few pending faces with long chains leave the chip idle), the pending
    // faces' after it (not while profiling: its stages are drained one by one)
    const bool split_normals = enable_qem && nw > 0 && !profile_;
    if (enable_qem) grad_.reserve((size_t)(nf + 1) * 12);
    auto launch_normals = [&](hipStream_t q, int mode) {
        const float* P = proj_.as<float>();
        float* G = grad_.as<float>();
        const int64_t* rw = a.rng;
        const uint32_t* pd = pend_.as<uint32_t>();
        if (pk) {
            void* nargs[] = {&jm, &jtab, &P, &rw, &G, &pd, &mode};
            TreeJit::launch(pk->normals, blocks_for(nw), nargs, q, "impli_pt_normals_at");
        } else {
            DEPTH_LAUNCH(E.depth(), k_normals_at, blocks_for(nw), 256, q, E.d_program(), E.d_rabbit(), P, rw, G, pd, mode);
        }
    };
    if (nw > 0) {
        // the point module's single-loop early pass: a wave per chunk of early_chunk faces
        const unsigned egrid = early_single_loop() ? blocks_for((nw + a.early_chunk - 1) / a.early_chunk * 64)
                               : early2                ? blocks_for(nw * 2)
                                                       : grid;
        if (pk && early2) TreeJit::launch(pk->early2, egrid, jargs, s, "impli_pt_project_early2");
        else if (pk) TreeJit::launch(pk->early, egrid, jargs, s, "impli_pt_project_early");
        else DEPTH_LAUNCH(E.depth(), k_project_early, grid, 256, s, E.d_program(), E.d_rabbit(), a);
        if (split_normals) {
            if (!early_done_) IMPLI_HIP(hipEventCreateWithFlags(&early_done_, hipEventDisableTiming));
            if (!normals_done_) IMPLI_HIP(hipEventCreateWithFlags(&normals_done_, hipEventDisableTiming));
            IMPLI_HIP(hipEventRecord(early_done_, s));
            IMPLI_HIP(hipStreamWaitEvent(side_s_, early_done_, 0));
            launch_normals(side_s_, 1);
            IMPLI_HIP(hipEventRecord(normals_done_, side_s_));
        }
        if (pk) TreeJit::launch(pk->late, late_grid, jargs, s, "impli_pt_project_late");
        else DEPTH_LAUNCH(E.depth(), k_project_late, late_grid, 256, s, E.d_program(), E.d_rabbit(), a);
    }
    IMPLI_HIP(hipGetLastError());
    if (profile_ && nw > 0) {   // the evaluations of this projection, summed on the host
        int64_t r[8];
        ranges(r);
        std::vector<uint32_t> h((size_t)(r[3] - r[2])), pend(h.size());
        if (!h.empty()) {
            IMPLI_HIP(hipMemcpyAsync(h.data(), evals_buf_.as<uint32_t>() + r[2], h.size() * 4, hipMemcpyDeviceToHost, s));
            IMPLI_HIP(hipMemcpyAsync(pend.data(), pend_.as<uint32_t>() + r[2], h.size() * 4, hipMemcpyDeviceToHost, s));
        }
        IMPLI_HIP(hipStreamSynchronize(s));
        for (uint32_t e : h) evals_ += e;
        if (std::getenv("IMPLISOLID_PROJ_STATS")) {   // diagnostics: the searches' balance per wave
            // (16 faces per wave of 4-lane groups: a wave runs as long as its longest face)
            uint64_t sum = 0, wmax = 0, npend = 0;
            for (size_t w0 = 0; w0 < h.size(); w0 += 16) {
                uint32_t m = 0;
                for (size_t j = w0; j < std::min(h.size(), w0 + 16); ++j) m = std::max(m, h[j]);
                wmax += (uint64_t)m * std::min<size_t>(16, h.size() - w0);
            }
            for (size_t j = 0; j < h.size(); ++j) {
                sum += h[j];
                npend += pend[j] ? 1 : 0;
            }
            std::fprintf(stderr, "projection faces %zu evals %llu (per face %.2f) wave-max-bound %llu (balance %.3f) "
                         "pending after the early pass %llu\n", h.size(), (unsigned long long)sum,
                         (double)sum / (double)h.size(), (unsigned long long)wmax, (double)sum / (double)wmax,
                         (unsigned long long)npend);
        }
    }
    store_pointset("post_p_centroids", proj_.as<float>(), nf, false);
    store_pointset("pre_qem_verts", verts_.as<float>(), nv, false);
    if (enable_qem) {
        st.next(kStageQem);
        if (split_normals) {
            launch_normals(s, 2);   // the faces the late pass resolved
            IMPLI_HIP(hipStreamWaitEvent(s, normals_done_, 0));
        } else if (nw > 0) {
            launch_normals(s, 0);
        }
        // QEM of the owned vertices (all unless sharded), in place
        const int64_t nov = own_v1_ - own_v0_;
        if (nov > 0)
            k_qem<<<blocks_for(nov), 256, 0, s>>>(verts_.as<float>() + 3 * own_v0_, nov, uoff_.as<uint32_t>() + own_v0_,
                                                  ulst_.as<int32_t>(), proj_.as<float>(), grad_.as<float>(),
                                                  fold_out_.as<FoldOut>());
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
    normals_ahead_ = false;
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
    normals_ahead_ = false;
    if (!topo_valid_) build_topology();
    Stage st(this, kStageSubdiv);
    int64_t added = 0;
    if (nf) {
        const EdgeTab t = edge_table();
        const uint64_t cap = t.mask + 1;
        if (!etab_valid_) {   // the edge table of the current faces: half-edge slots, first / last faces
            IMPLI_HIP(hipMemsetAsync(t.rec, 0, (size_t)cap * sizeof(EdgeRec), s));
            k_edge_insert<<<blocks_for(3 * nf), 256, 0, s>>>(faces_.as<int32_t>(), nf, nv, t);
            k_fof<<<blocks_for(3 * nf), 256, 0, s>>>(nf, t, fof_.as<int32_t>());   // fof unchanged: same values
            etab_valid_ = true;
        }
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
        if (vnew_.ext) vnew_.release();   // never reuse a caller's attached array as scratch
        nv = nvt;
        nf = 4 * nf;
        topo_valid_ = false;
        etab_valid_ = false;
        // the new vertices and faces are covered by later steps: the ranges become the whole mesh
        // (a sharded caller sets its owned vertices of the subdivided mesh again)
        rng_.reserve(kRngFields * sizeof(int64_t));
        k_ranges_set<<<1, 64, 0, s>>>(rng_.as<int64_t>(), 0, nv, nv, nf, 0);
        whole_ranges();
    }
    add_rand_noise(amplitude);
}

void Ob02::fetch(float* verts, int32_t* faces) {
    Stage st(this, kStageFetch);
    if (nv) IMPLI_HIP(hipMemcpyAsync(verts, verts_.p, (size_t)nv * 12, hipMemcpyDeviceToHost, s));
    if (nf && faces) IMPLI_HIP(hipMemcpyAsync(faces, faces_.p, (size_t)nf * 12, hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
}

}  // namespace impli
