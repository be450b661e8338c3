// ob02_device.hpp -- device side of the OB02 steps that evaluate the implicit tree, written over an
// evaluator `ev` (ev.f(x, y, z) -> f, ev.fg(x, y, z, g) -> f with the gradient), so the same code is
// compiled twice: over the node-program interpreter (ob02.hip, any tree at once) and over the
// tree-specialised point code of the JIT point module (jit.cpp; generated per tree shape).
//   centroid_normals_body  vertex_resampling.hpp:185-188 (step 1's normals)
//   project_*_body         set_centers_on_surface cp:421-1214 + bisection bisection.hpp:117-459
//   normals_at_body        the QEM normals at the projected centroids (qem.hpp:256-316)
//   points_body            direct evaluation (mcc2.cpp:815-911)
#pragma once
#include "ifunc_device.hpp"

namespace impli {
namespace ob {

using dev::V3;

constexpr float kRootTol = (float)(0.001 / 10.0);   // configs.hpp:33
constexpr int kBisectCap = 200;                      // the reference has no cap (bisection.hpp:360-372)

__device__ __forceinline__ float norm2f(float x, float y, float z) { return sqrtf(x * x + y * y + z * z); }

// the node-program interpreter (ifunc_device.hpp, stack capacity D) as an evaluator
template <int D>
struct InterpPt {
    const Program* prog;
    const float* tab;
    __device__ __forceinline__ float f(float x, float y, float z) const { return dev::eval_f<D>(prog, tab, x, y, z); }
    __device__ __forceinline__ float fg(float x, float y, float z, V3& g) const {
        return dev::eval_fg<D>(prog, tab, x, y, z, g);
    }
};

__device__ __forceinline__ V3 centroid(const float* __restrict__ v, const int32_t* __restrict__ f, int64_t j) {
    const int32_t a = f[3 * j], b = f[3 * j + 1], c = f[3 * j + 2];
    // compute_centroids implicit_vectorised_algorithms.hpp:161-171
    return V3{(v[3 * a] + v[3 * b] + v[3 * c]) / (float)(3.0), (v[3 * a + 1] + v[3 * b + 1] + v[3 * c + 1]) / (float)(3.0),
              (v[3 * a + 2] + v[3 * b + 2] + v[3 * c + 2]) / (float)(3.0)};
}

// Face ranges live in device memory: a pass over faces [rng[0], rng[1]) reads them in stream order
// (a Z-slab shard's work faces are found on the device, Ob02::set_owned_vertices, with no host
// round trip), its grid sized by an estimate on the host and grid-striding over the range.
__device__ __forceinline__ int64_t grid_lane() { return (int64_t)blockIdx.x * 256 + threadIdx.x; }
__device__ __forceinline__ int64_t grid_lanes() { return (int64_t)gridDim.x * 256; }

// vertex_resampling.hpp:185-188: f and normalize_1111(grad) at the face centroids
template <class Ev>
__device__ __forceinline__ void centroid_normals_body(const Ev& ev, const float* __restrict__ v,
                                                      const int32_t* __restrict__ f, const int64_t* __restrict__ rng,
                                                      float* __restrict__ C, float* __restrict__ N) {
    const int64_t j1 = rng[1];
    for (int64_t j = rng[0] + grid_lane(); j < j1; j += grid_lanes()) {
        const V3 c = centroid(v, f, j);
        V3 g;
        (void)ev.fg(c.x, c.y, c.z, g);
        const float nm = norm2f(g.x, g.y, g.z);   // normalize_1111 normalise_inplace.hpp:60-70
        C[3 * j] = c.x; C[3 * j + 1] = c.y; C[3 * j + 2] = c.z;
        N[3 * j] = g.x / nm; N[3 * j + 1] = g.y / nm; N[3 * j + 2] = g.z / nm;
    }
}

__device__ __forceinline__ float get_sign(float v) { return (v > kRootTol) ? 1.f : (v < -kRootTol) ? -1.f : 0.f; }

// normalise_inplace (normalise_inplace.hpp:26-54)
__device__ __forceinline__ V3 normalise_min(V3 a, float min_norm) {
    float nm = norm2f(a.x, a.y, a.z);
    nm = (nm < min_norm) ? 1.0f : nm;
    const float factor = (float)(1.0 / (double)nm);
    return V3{a.x * factor, a.y * factor, a.z * factor};
}

__device__ __forceinline__ V3 cross3(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// produce_facet_normals (implicit_vectorised_algorithms.hpp:52-133)
__device__ __forceinline__ V3 facet_normal(const float* __restrict__ v, const int32_t* __restrict__ f, int64_t j) {
    const float* p0 = v + 3 * f[3 * j];
    const float* p1 = v + 3 * f[3 * j + 1];
    const float* p2 = v + 3 * f[3 * j + 2];
    const float x1 = p1[0] - p0[0], y1 = p1[1] - p0[1], z1 = p1[2] - p0[2];
    const float x2 = p2[0] - p0[0], y2 = p2[1] - p0[1], z2 = p2[2] - p0[2];
    float x = y1 * z2 - z1 * y2, y = z1 * x2 - x1 * z2, z = x1 * y2 - y1 * x2;
    const float micro = (float)(1.0 / 1000.0), nano = (float)((double)micro / 1000.0);
    const float min_area = (30 * nano) * (30 * nano);
    const float n2 = x * x + y * y + z * z;
    if (n2 < min_area * min_area) {
        const float o = (float)(1.0 / (double)sqrtf(3.0f));
        return V3{o, o, o};
    }
    const float n = sqrtf(n2);
    return V3{x / n, y / n, z / n};
}

// The edge-length fold's result, written on the device by k_fold_walk (ob02.hip) and read by the
// projection and QEM kernels in stream order (no host round trip): the serial sum, the average edge
// length (compute_average_edge_length, cp:70-82) and make_alpha_list's list for it (cp:144-194;
// at most 20 alphas per halving of the step, and at most kMaxHalvings halvings).
constexpr int kMaxHalvings = 200;
constexpr int kMaxAlphas = 20 * kMaxHalvings;
struct FoldOut {
    float sum;          // the serial float chain of the 3F edge lengths
    float avg;          // (float)((double)sum / (3. * nf)): max_dist of the searches and QEM's clamp
    int nal;            // alphas in the list
    int table_chunks;   // chunks taken from the chunk table (statistics)
    int steps[8];       // walk steps (statistics): zero-skip / serial terms, table runs, term runs, global term
                        // loads, fast crossings, fast crossings that finished their chunk, serial chunks, (spare)
    long long cycles[8];   // staging, walking, table steps, term steps, term preamble, fast path, serial chunks
                           // (clock64)
    int trace[256];        // the walk's first steps (diagnostics): kind << 28 | term index
    float alphas[kMaxAlphas];
};

struct ProjArgs {
    const float* v;
    const int32_t* f;
    const int64_t* rng;     // the faces to project: [rng[0], rng[1]) (device memory; per-face arrays absolute)
    const FoldOut* fold;    // alphas, their count and max_dist (the average edge length)
    const float* pert;      // type-2 perturbations (3 per centroid), only for the late pass
    float* out;             // projected centroids
    float* fn;              // facet normals (written by the early pass)
    float* fc;              // f(centroid) (written by the early pass)
    uint32_t* pend;         // early pass: per face, 1 if its centroid is unresolved (the late pass's)
    int early_chunk;        // the early pass as one loop (project_early_sm_body): faces per wave chunk
    int late_wmax;          // the late pass's widest group (4..64 lanes, a power of two)
    int late_flat;          // 1: a round of the late searches may cross directions; 0: one direction per round
    uint32_t* cap_hits;     // bisections that reached kBisectCap (accumulated over the build)
    float* cen;             // centroids (written by the prep pass)
    float* dir;             // the type-0 direction per face (prep pass)
    uint32_t* evals;        // profiling: implicit evaluations per face (null: not counted)
};

// Lanes per centroid.  The reference's searches are sequential per centroid (first alpha of the list
// whose sign differs, then bisection); one lane per centroid left ~2 waves per SIMD, each waiting on
// its slowest centroid's chain of evaluations.  A group of kProjGroup lanes evaluates kProjGroup
// alphas at once (the first hit in list order wins) and kBisLevels bisection levels at once (the
// decision tree of the next levels, then the serial path through it), so the chains are shorter and
// the wave is filled: the result is the serial one exactly.  Group size (round 3, A/B on config 2 /
// 3 / 3s with tools/ab_ob02_variants.sh, two alternating rounds): 4 lanes and 2 levels per round
// 1.51-1.52 ms for config3s against 1.66-1.76 with 8 and 3 (fewer evaluations past the hit, and
// 3 instead of 7 per two levels), 2 and 1 1.72-1.74, 16 and 4 1.88; configs 2 and 3 within noise.
// The searches are throughput-bound at this size (90 k faces), not chain-bound.
#ifndef IMPLI_PROJ_GROUP   // (experiments: a point module built with IMPLISOLID_PROJ_GROUP=2 / 8)
#define IMPLI_PROJ_GROUP 4
#endif
constexpr int kProjGroup = IMPLI_PROJ_GROUP;
constexpr int kBisLevels = kProjGroup >= 8 ? 3 : kProjGroup >= 4 ? 2 : 1;
static_assert((1 << kBisLevels) - 1 <= kProjGroup && 64 % kProjGroup == 0, "bisection tree fits the group");

template <int W>
struct GrpW {   // a centroid's W lanes inside the wave (control flow is uniform per group)
    static constexpr int kWidth = W;
    int sub, base;
    __device__ GrpW() {
        const int lane = (int)(threadIdx.x & 63);
        sub = lane & (W - 1);
        base = lane - sub;
    }
    __device__ uint64_t bits(bool p) const {
        if constexpr (W == 64) return (uint64_t)__ballot(p);
        else return (uint64_t)((__ballot(p) >> base) & ((1ull << W) - 1ull));
    }
    __device__ float from(float v, int k) const { return __shfl(v, base + k, 64); }
    __device__ V3 from(V3 v, int k) const { return V3{from(v.x, k), from(v.y, k), from(v.z, k)}; }
};
using Grp = GrpW<kProjGroup>;

struct GrpR {   // a group of w lanes (w a power of two, 4..64, uniform over the wave), chosen at run time
    int sub, base, w;
    uint64_t mask;
    __device__ explicit GrpR(int width) : w(width) {
        const int lane = (int)(threadIdx.x & 63);
        sub = lane & (w - 1);
        base = lane - sub;
        mask = w == 64 ? ~0ull : (1ull << w) - 1ull;
    }
    __device__ uint64_t bits(bool p) const { return ((uint64_t)__ballot(p) >> base) & mask; }
    __device__ float from(float v, int k) const { return __shfl(v, base + k, 64); }
    __device__ V3 from(V3 v, int k) const { return V3{from(v.x, k), from(v.y, k), from(v.z, k)}; }
};

// cp:904-1191 for one centroid: zero tests, swap (x1 outside), vectorised bisection restated per point
__device__ __forceinline__ V3 bis_mid(V3 a, V3 b) {   // bisection.hpp:225-231: (x1 + x2) / 2. in double
    return V3{(float)((double)(a.x + b.x) / 2.), (float)((double)(a.y + b.y) / 2.), (float)((double)(a.z + b.z) / 2.)};
}

// bisection.hpp:190-378 per point: mid, stop at |f(mid)| <= tol, x1 <- mid where f < -tol, x2 <- mid
// where f > tol (a NaN moves neither: the serial loop repeats that mid until the cap).  Lane k < 2^L - 1
// evaluates node k of the next L levels' decision tree (heap order: child 2k+1 after f < -tol, 2k+2
// after f > tol); the group then walks the path the serial loop takes through those levels.
// nodes < 2^L - 1: only the first `nodes` heap nodes are evaluated (a group too narrow for the
// whole tree, e.g. 2 lanes over 2 levels: the mid and the child after f < -tol); the walk stops
// early where its next node was not evaluated.  The mids are the serial loop's either way.
template <class G, class Ev>
__device__ V3 bisect_g(const G& g, const int L, const Ev& ev, V3 x1, V3 x2, uint32_t* cap_hits, uint32_t& evals,
                       int nodes = 0) {
    int it = 0;
    if (nodes <= 0 || nodes > (1 << L) - 1) nodes = (1 << L) - 1;
    const int node = g.sub < nodes ? g.sub : 0;
    int depth = 0, bits = 0;   // node's path from the root, first decision in the lowest bit (1: x1 <- mid)
    for (int n = node; n > 0; n = (n - 1) >> 1) bits = (bits << 1) | ((n & 1) ? 1 : 0), ++depth;
    for (;;) {
        V3 a = x1, b = x2;
        for (int k = 0; k < depth; ++k) {
            const V3 m = bis_mid(a, b);
            if ((bits >> k) & 1) a = m;
            else b = m;
        }
        const V3 mid = bis_mid(a, b);
        const float vm = ev.f(mid.x, mid.y, mid.z);
        evals += nodes;
        int cur = 0;
        for (int lvl = 0; lvl < L; ++lvl) {
            const float v = g.from(vm, cur);
            ++it;
            if (fabsf(v) <= kRootTol) return g.from(mid, cur);
            const bool lo = v < -kRootTol, hi = v > kRootTol;
            if (!(lo || hi) || it == kBisectCap) {
                if (g.sub == 0) atomicAdd(cap_hits, 1u);
                return g.from(mid, cur);
            }
            const int next = lo ? 2 * cur + 1 : 2 * cur + 2;
            if (lvl + 1 < L && next < nodes) {
                cur = next;
            } else {   // the state after this level: node cur's interval with its outcome applied
                const V3 na = g.from(a, cur), nb = g.from(b, cur), nm = g.from(mid, cur);
                x1 = lo ? nm : na;
                x2 = lo ? nb : nm;
                break;
            }
        }
    }
}

// f2 = f(best) (cp:904-951) is known: the search evaluated f at the point it returned, and
// best == x when nothing was found (f(x) = fcv: eval_fg's value is eval_f's)
template <class G, class Ev>
__device__ void finalize_g(const G& g, const int L, const Ev& ev, V3 x, float fcv, bool found, V3 best,
                           float f2, float* out, const ProjArgs& a, uint32_t& evals, int nodes = 0) {
    const bool z2 = fabsf(f2) <= kRootTol, z1 = fabsf(fcv) <= kRootTol;
    if (z1) best = x;
    V3 r;
    if (found && !(z1 || z2)) {
        V3 x1 = x, x2 = best;
        if (f2 < -kRootTol) { const V3 t = x1; x1 = x2; x2 = t; }
        r = bisect_g(g, L, ev, x1, x2, a.cap_hits, evals, nodes);
    } else if (z1 || z2) {
        r = best;
    } else {
        r = x;
    }
    if (g.sub == 0) { out[0] = r.x; out[1] = r.y; out[2] = r.z; }
}

// make_alpha_list's alphas along d, kProjGroup at a time; the first in list order whose sign
// differs from the centroid's (cp:595-903)
template <class G, class Ev>
__device__ __forceinline__ bool try_direction(const G& g, const Ev& ev, V3 x, V3 d, float sc,
                                              const float* alphas, int na, float max_dist, V3& best,
                                              float& best_f, uint32_t& evals) {
    constexpr int kW = G::kWidth;
    for (int a0 = 0; a0 < na; a0 += kW) {
        const int ai = a0 + g.sub;
        V3 p = x;
        float fa = 0.f;
        bool hit = false;
        if (ai < na) {
            const float cc = max_dist * alphas[ai];   // (length_factor * alpha) * 4.0 / 4.0 is exact
            p = V3{x.x + cc * d.x, x.y + cc * d.y, x.z + cc * d.z};
            fa = ev.f(p.x, p.y, p.z);
            hit = get_sign(fa) * sc <= 0;
        }
        evals += na - a0 < kW ? na - a0 : kW;
        const uint32_t m = (uint32_t)g.bits(hit);
        if (m) {
            best = g.from(p, __ffs(m) - 1);
            best_f = g.from(fa, __ffs(m) - 1);
            return true;
        }
    }
    return false;
}

// set_centers_on_surface (cp:421-594), the part before the searches: centroid, facet normal,
// f(centroid) and the type-0 direction -normalise(grad) s_c; one lane per face.  Nothing here needs
// the average edge length, so it runs while k_fold_walk folds the edge lengths.
template <class Ev>
__device__ __forceinline__ void project_prep_face(const Ev& ev, const ProjArgs& a, int64_t j) {
    const V3 x = centroid(a.v, a.f, j);
    const V3 fnv = facet_normal(a.v, a.f, j);
    V3 gr;
    const float fcv = ev.fg(x.x, x.y, x.z, gr);
    V3 gd = normalise_min(gr, 0.000001f);
    const float sc = get_sign(fcv);
    if (sc < 0.0f) { gd.x = -gd.x; gd.y = -gd.y; gd.z = -gd.z; }
    a.cen[3 * j] = x.x; a.cen[3 * j + 1] = x.y; a.cen[3 * j + 2] = x.z;
    a.fn[3 * j] = fnv.x; a.fn[3 * j + 1] = fnv.y; a.fn[3 * j + 2] = fnv.z;
    a.fc[j] = fcv;
    a.dir[3 * j] = -gd.x * sc; a.dir[3 * j + 1] = -gd.y * sc; a.dir[3 * j + 2] = -gd.z * sc;
    if (a.evals) a.evals[j] = 1;
}

template <class Ev>
__device__ __forceinline__ void project_prep_body(const Ev& ev, const ProjArgs& a) {
    const int64_t j1 = a.rng[1];
    for (int64_t j = a.rng[0] + grid_lane(); j < j1; j += grid_lanes()) project_prep_face(ev, a, j);
}

// direction types 0 (gradient) and 1 (mesh normal); W lanes per face (kProjGroup, or 2 on large
// meshes: see project_early_body)
template <int W, class Ev>
__device__ __forceinline__ void project_early_face(const Ev& ev, const ProjArgs& a, const GrpW<W>& g, int64_t j) {
    // bisection levels per evaluation round and the nodes evaluated: the whole tree of 3 / 2 levels
    // for 8 / 4 lanes; 2 lanes evaluate the mid and its child after f < -tol (2 levels when the walk
    // goes that way, 1 otherwise).  (Every lane a node for 4 lanes too, 3 levels with the first node
    // of the third, measured 1-2 % slower at 256^3 and even at 512^3: profiles/r06v_*.)
    constexpr int kLevels = W >= 8 ? 3 : 2;
    constexpr int kNodes = W >= 8 ? 7 : W >= 4 ? 3 : 2;
    const V3 x{a.cen[3 * j], a.cen[3 * j + 1], a.cen[3 * j + 2]};
    const V3 fnv{a.fn[3 * j], a.fn[3 * j + 1], a.fn[3 * j + 2]};
    const V3 d0{a.dir[3 * j], a.dir[3 * j + 1], a.dir[3 * j + 2]};
    const float fcv = a.fc[j];
    const float sc = get_sign(fcv);
    const int nal = a.fold->nal;
    const float max_dist = a.fold->avg;
    const float* alphas = a.fold->alphas;
    uint32_t evals = 0;
    V3 best = x;
    float bf = fcv;
    bool found = try_direction(g, ev, x, d0, sc, alphas, nal, max_dist, best, bf, evals);
    if (!found) found = try_direction(g, ev, x, fnv, sc, alphas, nal < 10 ? nal : 10, max_dist, best, bf, evals);
    if (found) finalize_g(g, kLevels, ev, x, fcv, true, best, bf, a.out + 3 * j, a, evals, kNodes);
    // unresolved faces are flagged for the late pass (a compacted list cost one same-address atomic
    // per wave: 258 us per pass when every face pends, as with a non-finite average edge length)
    if (g.sub == 0) a.pend[j] = found ? 0u : 1u;
    if (a.evals && g.sub == 0) a.evals[j] += evals;
}

// W = kProjGroup (4) everywhere but the point modules' second entry (W = 2), which the host picks
// for large meshes: there the pass is throughput-bound (tens of thousands of waves) and 2 lanes
// evaluate fewer alphas past the hit and fewer tree nodes per bisection level (config 4s at 512^3:
// 184 -> 162 us per call), where on a 180 k-face mesh the longer chains of 2 lanes cost more (69 ->
// 75 us, profiles/r05zy_*)
template <int W = kProjGroup, class Ev>
__device__ __forceinline__ void project_early_body(const Ev& ev, const ProjArgs& a) {
    const GrpW<W> g;
    const int64_t j1 = a.rng[1];
    for (int64_t j = a.rng[0] + grid_lane() / W; j < j1; j += grid_lanes() / W)   // uniform per group
        project_early_face<W>(ev, a, g, j);
}

// The early pass as one loop with one tree evaluation per iteration.  project_early_face runs the
// searches and the bisection as separate loops, each with its own inlined copy of the tree code, and
// a wave's 16 faces in step: a group whose face is done idles until the wave's longest face ends
// (0.76-0.84 of the evaluations' bound, IMPLISOLID_PROJ_STATS), and groups in different phases take
// turns through the two copies.  Here every group is in one of three phases -- searching (4 alphas
// of the current direction per iteration), bisecting (2 levels per iteration), idle -- and each
// iteration computes the group's point for its phase, evaluates the tree once for every lane, and
// then advances each group by the same rules as try_direction / finalize_g / bisect_g (the shuffles
// they need are taken for every group before the phase-specific update, so none runs in divergent
// code).  A group that finishes takes the next face of its wave's chunk of early_chunk faces (rank
// among the finishing groups by ballot: no atomics).  The result of every face is the serial one.
template <class Ev>
__device__ __forceinline__ void project_early_sm_body(const Ev& ev, const ProjArgs& a) {
    constexpr int kSearch = 0, kBisect = 1, kIdle = 2;
    static_assert(kBisLevels == 2, "the single-loop form walks two bisection levels per iteration");
    const Grp g;
    const int64_t j1 = a.rng[1];
    const int nal = a.fold->nal;
    const int n10 = nal < 10 ? nal : 10;
    const float max_dist = a.fold->avg;
    const float* alphas = a.fold->alphas;
    const int chunk = a.early_chunk;
    // this lane's node of the 2-level bisection tree (bisect_g)
    const int node = g.sub < (1 << kBisLevels) - 1 ? g.sub : 0;
    int depth = 0, bits = 0;
    for (int n = node; n > 0; n = (n - 1) >> 1) bits = (bits << 1) | ((n & 1) ? 1 : 0), ++depth;
    for (int64_t c0 = a.rng[0] + (grid_lane() >> 6) * chunk; c0 < j1; c0 += (grid_lanes() >> 6) * chunk) {
        const int cn = (int)(j1 - c0 < chunk ? j1 - c0 : chunk);
        int next = 0;   // the chunk's next face (wave-uniform)
        int phase = kIdle;
        int64_t j = 0;
        V3 x{0.f, 0.f, 0.f}, fnv = x, d = x, best = x, x1 = x, x2 = x;
        float fcv = 0.f, sc = 0.f, bf = 0.f;
        int na = 0, a0 = 0, dir = 0, it = 0;
        uint32_t evals = 0;
        auto finish = [&](bool found, V3 r) {
            if (g.sub == 0) {
                if (found) { a.out[3 * j] = r.x; a.out[3 * j + 1] = r.y; a.out[3 * j + 2] = r.z; }
                a.pend[j] = found ? 0u : 1u;
                if (a.evals) a.evals[j] += evals;
            }
            phase = kIdle;
        };
        auto settle = [&]() {   // a direction with no alpha left: the next direction, or pending
            while (phase == kSearch && a0 >= na) {
                if (dir == 0) {
                    dir = 1;
                    d = fnv;
                    na = n10;
                    a0 = 0;
                } else {
                    finish(false, x);
                }
            }
        };
        for (;;) {
            // idle groups take the chunk's next faces in group order
            const uint64_t idle = __ballot(g.sub == 0 && phase == kIdle);
            if (phase == kIdle) {
                const int f = next + __popcll(idle & ((1ull << g.base) - 1ull));   // idle leaders before ours
                if (f < cn) {
                    j = c0 + f;
                    x = V3{a.cen[3 * j], a.cen[3 * j + 1], a.cen[3 * j + 2]};
                    fnv = V3{a.fn[3 * j], a.fn[3 * j + 1], a.fn[3 * j + 2]};
                    d = V3{a.dir[3 * j], a.dir[3 * j + 1], a.dir[3 * j + 2]};
                    fcv = a.fc[j];
                    sc = get_sign(fcv);
                    best = x;
                    bf = fcv;
                    na = nal;
                    a0 = 0;
                    dir = 0;
                    evals = 0;
                    phase = kSearch;
                    settle();
                }
            }
            next += __popcll(idle);
            if (__ballot(phase != kIdle) == 0) {
                if (next >= cn) break;
                continue;   // every new face settled at once (empty alpha lists): hand out more
            }
            // this iteration's point: an alpha of the current direction, or this lane's bisection node
            V3 p = x, ba = x1, bb = x2;
            bool valid = false;
            if (phase == kSearch) {
                const int ai = a0 + g.sub;
                valid = ai < na;
                if (valid) {
                    const float cc = max_dist * alphas[ai];   // (length_factor * alpha) * 4.0 / 4.0 is exact
                    p = V3{x.x + cc * d.x, x.y + cc * d.y, x.z + cc * d.z};
                }
            } else if (phase == kBisect) {
                for (int k = 0; k < depth; ++k) {
                    const V3 m = bis_mid(ba, bb);
                    if ((bits >> k) & 1) ba = m;
                    else bb = m;
                }
                p = bis_mid(ba, bb);
                valid = true;
            }
            float fv = 0.f;
            if (valid) fv = ev.f(p.x, p.y, p.z);
            // every group's shuffles, in uniform control flow
            const bool hit = phase == kSearch && valid && get_sign(fv) * sc <= 0;
            const uint32_t m = (uint32_t)g.bits(hit);
            const int k = m ? __ffs(m) - 1 : 0;
            const V3 pk = g.from(p, k);
            const float fk = g.from(fv, k);
            const float v0 = g.from(fv, 0);
            const int cur1 = v0 < -kRootTol ? 1 : 2;
            const float v1 = g.from(fv, cur1);
            const V3 pc0 = g.from(p, 0), pc1 = g.from(p, cur1), a1 = g.from(ba, cur1), b1 = g.from(bb, cur1);
            if (phase == kSearch) {   // try_direction's round, then finalize_g
                evals += na - a0 < kProjGroup ? na - a0 : kProjGroup;
                if (m) {
                    best = pk;
                    bf = fk;
                    const bool z2 = fabsf(bf) <= kRootTol, z1 = fabsf(fcv) <= kRootTol;
                    if (z1) best = x;
                    if (!(z1 || z2)) {
                        x1 = x;
                        x2 = best;
                        if (bf < -kRootTol) { const V3 t = x1; x1 = x2; x2 = t; }
                        it = 0;
                        phase = kBisect;
                    } else {
                        finish(true, best);
                    }
                } else {
                    a0 += kProjGroup;
                    settle();
                }
            } else if (phase == kBisect) {   // bisect_g's two levels
                evals += (1 << kBisLevels) - 1;
                const bool lo0 = v0 < -kRootTol, hi0 = v0 > kRootTol;
                const bool lo1 = v1 < -kRootTol, hi1 = v1 > kRootTol;
                if (fabsf(v0) <= kRootTol) {
                    finish(true, pc0);
                } else if (!(lo0 || hi0) || it + 1 == kBisectCap) {
                    if (g.sub == 0) atomicAdd(a.cap_hits, 1u);
                    finish(true, pc0);
                } else if (fabsf(v1) <= kRootTol) {
                    finish(true, pc1);
                } else if (!(lo1 || hi1) || it + 2 == kBisectCap) {
                    if (g.sub == 0) atomicAdd(a.cap_hits, 1u);
                    finish(true, pc1);
                } else {
                    x1 = lo1 ? pc1 : a1;
                    x2 = lo1 ? b1 : pc1;
                    it += 2;
                }
            }
        }
    }
}

// types 2 (cross with a perturbation), 3 (cross of that with the mesh normal), 4-6 (axes), with a
// group of g.w lanes.  The five searches' (direction, alpha) pairs in serial order (cp:1000-1150) are
// taken g.w at a time -- a round may cross from one direction to the next -- and the first hit in that
// order wins, as in the serial loop; the bisection then takes log2(g.w) levels per round.
template <class Ev>
__device__ __forceinline__ void project_late_face(const Ev& ev, const ProjArgs& a, const GrpR& g, int64_t j) {
    const V3 x{a.cen[3 * j], a.cen[3 * j + 1], a.cen[3 * j + 2]};
    const V3 fnv{a.fn[3 * j], a.fn[3 * j + 1], a.fn[3 * j + 2]};
    const float fcv = a.fc[j];
    const float sc = get_sign(fcv);
    const float max_dist = a.fold->avg;
    const float* alphas = a.fold->alphas;
    const int n10 = a.fold->nal < 10 ? a.fold->nal : 10;
    const V3 pv{a.pert[3 * j], a.pert[3 * j + 1], a.pert[3 * j + 2]};
    V3 z = cross3(fnv, pv);               // cp:250-259, add_inplace is a no-op (F9)
    const float nz = norm2f(z.x, z.y, z.z);
    z = V3{z.x / nz, z.y / nz, z.z / nz};  // normalize_1111
    const V3 z2 = normalise_min(cross3(fnv, z), 0.000001f);   // cp:297-312
    uint32_t evals = 0;
    V3 best = x;
    float bf = fcv;
    bool found = false;
    const int n = 5 * n10;
    for (int c0 = 0; c0 < n;) {
        const int cend = a.late_flat ? n : (c0 / n10 + 1) * n10;   // this round's last pair + 1
        const int c = c0 + g.sub;
        const int di = c / n10, ai = c - di * n10;
        V3 p = x;
        float fa = 0.f;
        bool hit = false;
        if (c < cend) {
            const V3 d = di == 0 ? z : di == 1 ? z2 : V3{di == 2 ? 1.f : 0.f, di == 3 ? 1.f : 0.f, di == 4 ? 1.f : 0.f};
            const float cc = max_dist * alphas[ai];   // try_direction's point
            p = V3{x.x + cc * d.x, x.y + cc * d.y, x.z + cc * d.z};
            fa = ev.f(p.x, p.y, p.z);
            hit = get_sign(fa) * sc <= 0;
        }
        const int nxt = cend - c0 < g.w ? cend : c0 + g.w;
        evals += nxt - c0;
        c0 = nxt;
        const uint64_t m = g.bits(hit);
        if (m) {
            const int k = __ffsll((unsigned long long)m) - 1;
            best = g.from(p, k);
            bf = g.from(fa, k);
            found = true;
            break;
        }
    }
    finalize_g(g, 31 - __clz(g.w), ev, x, fcv, found, best, bf, a.out + 3 * j, a, evals);
    if (a.evals && g.sub == 0) a.evals[j] += evals;
}

// The late pass is latency-bound: a few faces in 10^3..10^5 pend, and with 4 lanes each waited on a
// chain of ~15 search rounds and 2 bisection levels per round.  Each wave takes chunks of 16 faces
// (the early pass's faces per wave), reads their flags at once and gives each pending face of the
// chunk 64 / p lanes (p pending, rounded up to a power of two; at least 4): a lone face gets the whole
// wave (its five searches in one round, 6 bisection levels per round), a chunk where every face pends
// (as when the average edge length is not finite) 4 lanes per face.  (Chunks of 64 faces, up to 4
// rounds of 16 faces per wave: a quarter of the waves, 31 -> 55 us on config 2.)
constexpr int kLateChunk = 16;   // faces per wave chunk (the late grid: 4 lanes per face)

template <class Ev>
__device__ __forceinline__ void project_late_body(const Ev& ev, const ProjArgs& a) {
    const int lane = (int)(threadIdx.x & 63);
    const int64_t j1 = a.rng[1];
    for (int64_t c0 = a.rng[0] + (grid_lane() >> 6) * kLateChunk; c0 < j1; c0 += (grid_lanes() >> 6) * kLateChunk) {
        const uint64_t m = (uint64_t)__ballot(lane < kLateChunk && c0 + lane < j1 && a.pend[c0 + lane] != 0u);
        const int np = __popcll(m);
        if (!np) continue;
        int w = np == 1 ? 64 : np == 2 ? 32 : np <= 4 ? 16 : np <= 8 ? 8 : 4;
        w = w < a.late_wmax ? w : a.late_wmax;
        // lane r learns the chunk position of the r-th pending face (a scalar walk over the set bits)
        int pos = 0;
        uint64_t mm = m;
        for (int r = 0; r < np; ++r) {
            const int b = __ffsll((unsigned long long)mm) - 1;
            mm &= mm - 1;
            pos = lane == r ? b : pos;
        }
        const GrpR g(w);
        for (int r0 = 0; r0 < np; r0 += 64 / w) {   // one round unless the width is capped
            const int r = r0 + lane / w;
            const int at = __shfl(pos, r < np ? r : 0, 64);
            if (r < np) project_late_face(ev, a, g, c0 + at);   // uniform per group
        }
    }
}

// normalize_1111(grad) at arbitrary points (the QEM normals at the projected centroids, qem.hpp:256-316)
// over the faces [rng[0], rng[1]) (P, G absolute).  pend (the early pass's flags) splits the pass:
// mode 1 the faces the early pass resolved (run beside the late pass), mode 2 the others (after it),
// mode 0 every face
template <class Ev>
__device__ __forceinline__ void normals_at_body(const Ev& ev, const float* __restrict__ P, const int64_t* __restrict__ rng,
                                                float* __restrict__ G, const uint32_t* __restrict__ pend = nullptr,
                                                int mode = 0) {
    const int64_t j1 = rng[1];
    for (int64_t j = rng[0] + grid_lane(); j < j1; j += grid_lanes()) {
        if (mode != 0 && (pend[j] != 0u) != (mode == 2)) continue;
        V3 g;
        (void)ev.fg(P[3 * j], P[3 * j + 1], P[3 * j + 2], g);
        const float nm = norm2f(g.x, g.y, g.z);
        G[3 * j] = g.x / nm; G[3 * j + 1] = g.y / nm; G[3 * j + 2] = g.z / nm;
    }
}


// direct evaluation of n points (mcc2.cpp:815-911): f, and the gradient when grad != null
template <class Ev>
__device__ __forceinline__ void points_body(const Ev& ev, const float* __restrict__ xyz, int64_t n, float* __restrict__ f,
                                            float* __restrict__ grad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (grad) {
        V3 g;
        const float v = ev.fg(x, y, z, g);
        if (f) f[i] = v;
        grad[3 * i] = g.x; grad[3 * i + 1] = g.y; grad[3 * i + 2] = g.z;
    } else {
        f[i] = ev.f(x, y, z);
    }
}

}  // namespace ob
}  // namespace impli
