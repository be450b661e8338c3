// eval_bricks.hpp -- device side of the brick-pruned field evaluation, shared by the static
// interpreter kernels (eval.hip) and the JIT-compiled tree kernels (jit.cpp).
#pragma once
#include "grid.hpp"

// evaluate a brick's two layers as one straight-line block (measured 57 -> 45 us at 512^3 on the
// config-4 tree); IMPLISOLID_EVAL_PAIR=0 in the environment compiles the JIT kernels without it.
// eval_bricks_body's Pair parameter chooses per kernel (the merged interpreter launch: off)
#ifndef IMPLI_EVAL_PAIR
#define IMPLI_EVAL_PAIR 1
#endif

namespace impli {

// one brick row of sign bits
template <int W> struct SignPiece;
template <> struct SignPiece<8> { typedef uint8_t type; };
template <> struct SignPiece<16> { typedef uint16_t type; };
template <> struct SignPiece<32> { typedef uint32_t type; };
typedef SignPiece<kBX>::type sign_piece_t;

// sample coordinate of stored index i (sample i + 1) along an axis (prepare_grid,
// marching_cubes.hpp:1691-1693: x * factor + min - 2 * width)
__device__ __forceinline__ float sample_xy(const GridDesc& g, int axis, int i) {
    return ((float)(i + 1) * g.w[axis] + g.lo[axis]) - 2.f * g.w[axis];
}
__device__ __forceinline__ float sample_z(const GridDesc& g, int layer) {
    return ((float)(g.fz0 + layer) * g.w[2] + g.lo[2]) - 2.f * g.w[2];
}
// seal_exterior (:895-963): samples 1 and res-2 of any axis hold -1e7
__device__ __forceinline__ bool sealed_xy(const GridDesc& g, int i) { return i == 0 || i == g.n - 1; }
__device__ __forceinline__ bool sealed_z(const GridDesc& g, int layer) {
    const int sz = g.fz0 + layer;
    return sz == 1 || sz == g.res - 2;
}
constexpr float kSealed = -10000000.0f;

__device__ __forceinline__ void brick_of(int b, const BrickGrid& bg, int& bx, int& by, int& bz) {
    bx = b % bg.nbx;
    const int t = b / bg.nbx;
    by = t % bg.nby;
    bz = t / bg.nby;
}

// One wave per listed brick (kBX x kBY lanes, kBZ layers each; grid-stride over the list built by
// k_brick_fill, modes[i] the listed brick's pruning modes): every sample is evaluated with
// `ev(modes, x, y, z)`, stored, and its sign bit set (wave ballot: 64 bits = kBY rows x kBX
// samples).  Sign-filled bricks never reach this kernel -- k_brick_fill wrote their constant sign
// bits -- except claimed candidates (grid.hpp ClaimCtx), evaluated by the wave of the mixed brick
// that claimed them, values only (their sign pieces are constant and already written).
// both layers of a column: the evaluator's pair() when it has one (the JIT tree: one pass of the
// tree code for both samples), else two calls
template <class Eval>
__device__ __forceinline__ auto eval_pair(const Eval& ev, uint64_t m, float x, float y, float z0, float z1, float& f0,
                                          float& f1, int) -> decltype(ev.pair(m, x, y, z0, z1, f0, f1), void()) {
    ev.pair(m, x, y, z0, z1, f0, f1);
}
template <class Eval>
__device__ __forceinline__ void eval_pair(const Eval& ev, uint64_t m, float x, float y, float z0, float z1, float& f0,
                                          float& f1, long) {
    f0 = ev(m, x, y, z0);
    f1 = ev(m, x, y, z1);
}

// one brick (b, its modes m) by the calling wave; neg[k]: layer k's sign bits, valid: the lanes
// inside the grid
template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>
__device__ __forceinline__ void eval_one_brick(const Eval& ev, const GridDesc& g, const BrickGrid& bg, int b, uint64_t m64,
                                               float* __restrict__ field, sign_piece_t* __restrict__ signs,
                                               bool write_signs, uint64_t neg[kBZ], uint64_t& valid) {
    const int lane = threadIdx.x & 63;
    const int n = g.n;
    const int layers = g.fz1 - g.fz0;
    const int row_pieces = (64 / kBX) * sign_row_words(g);
    int bx, by, bz;
    brick_of(b, bg, bx, by, bz);
    const int sx = bx * kBX + (lane % kBX), sy = by * kBY + (lane / kBX);
    const bool ok = sx < n && sy < n;
    valid = __ballot(ok);
    const bool sealed_col = sealed_xy(g, sx) || sealed_xy(g, sy);
    // brick-major field (grid.hpp field_index): the brick's layer k is 64 consecutive floats, one
    // per lane -- the wave stores two whole lines (lanes past the grid edge fill the padding)
    float* out = field + (size_t)b * kBrickSamples + lane;
    const uint64_t m = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m64 >> 32)) << 32) |
                       (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)m64);
    const float x = sample_xy(g, 0, ok ? sx : 0), y = sample_xy(g, 1, ok ? sy : 0);
#pragma unroll
    for (int k = 0; k < kBZ; ++k) neg[k] = 0;
    if constexpr (Pair) {
        // both layers' tree evaluations in one straight-line block: two independent dependency
        // chains per lane (a layer past the slab is evaluated at a clamped z and not stored)
        static_assert(!Pair || kBZ == 2, "the layer pair needs two layers per brick");
        const int l0 = bz * kBZ, l1 = l0 + 1;
        float f0, f1;
        eval_pair(ev, m, x, y, sample_z(g, l0), sample_z(g, l1 < layers ? l1 : l0), f0, f1, 0);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int layer = l0 + k;
            if (layer >= layers) break;
            const float v = (sealed_col || sealed_z(g, layer)) ? kSealed : 0.f + (k ? f1 : f0);
            out[k * kBX * kBY] = v;
            neg[k] = __ballot(v < 0.f);
            if (write_signs && lane < kBY) {
                const int yy = by * kBY + lane;
                if (yy < n) signs[((size_t)layer * n + yy) * row_pieces + bx] = (sign_piece_t)(neg[k] >> (kBX * lane));
            }
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < kBZ; ++k) {
            const int layer = bz * kBZ + k;
            if (layer >= layers) break;
            const float f = ev(m, x, y, sample_z(g, layer));
            const float v = (sealed_col || sealed_z(g, layer)) ? kSealed : 0.f + f;
            out[k * kBX * kBY] = v;
            const uint64_t nk = __ballot(v < 0.f);
            neg[k] = nk;
            if (write_signs && lane < kBY) {
                const int yy = by * kBY + lane;
                if (yy < n) signs[((size_t)layer * n + yy) * row_pieces + bx] = (sign_piece_t)(nk >> (kBX * lane));
            }
        }
    }
}

// The face neighbours of a just evaluated mixed brick that it claims (bit d: direction d = -x, +x,
// -y, +y, -z, +z): candidates (grid.hpp) of sign s such that some sample of this brick on the
// shared face has the other sign -- a cell edge across the face changes sign there, so marching
// cubes reads the candidate's value -- and that no other wave claimed first (atomic on the fill
// byte).  Face samples are the lanes of the face column / row in both layers, or a whole layer.
__device__ __forceinline__ uint32_t claim_neighbours(const GridDesc& g, const BrickGrid& bg, const ClaimCtx& cc, int b,
                                                     const uint64_t neg[kBZ], uint64_t valid) {
    static_assert(kBZ == 2, "face masks of two-layer bricks");
    int bx, by, bz;
    brick_of(b, bg, bx, by, bz);
    const int layers = g.fz1 - g.fz0;
    const bool has1 = bz * kBZ + 1 < layers;
    uint64_t col0 = 0, row0 = (1ull << kBX) - 1ull;
#pragma unroll
    for (int r = 0; r < kBY; ++r) col0 |= 1ull << (r * kBX);
    const uint64_t colL = col0 << (kBX - 1), rowL = row0 << (kBX * (kBY - 1));
    // the six neighbours' fill bytes, loaded together (a neighbour outside the grid reads the
    // brick's own byte, which is never a candidate: it is listed); one memory round trip instead of
    // one per direction
    int an[6];
    uint32_t fa[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        const int ax = d >> 1, up = d & 1;
        const int c = ax == 0 ? bx : ax == 1 ? by : bz;
        const int lim = ax == 0 ? bg.nbx : ax == 1 ? bg.nby : bg.nbz;
        const int step = ax == 0 ? 1 : ax == 1 ? bg.nbx : bg.nbx * bg.nby;
        const bool in = up ? c + 1 < lim : c > 0;
        an[d] = in ? (up ? b + step : b - step) : b;
        fa[d] = cc.fill[an[d]];
    }
    // the directions to claim: a candidate neighbour with a differing sample on the shared face
    uint32_t want = 0;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        const int ax = d >> 1, up = d & 1;
        uint64_t f0, f1;
        if (ax == 0) f0 = f1 = up ? colL : col0;
        else if (ax == 1) f0 = f1 = up ? rowL : row0;
        else { f0 = up ? 0ull : ~0ull; f1 = up ? ~0ull : 0ull; }
        f0 &= valid;
        f1 = has1 ? (f1 & valid) : 0ull;
        const bool aneg = (fa[d] & 3u) == kBrickNeg;
        const uint64_t differ = aneg ? ((~neg[0] & f0) | (~neg[1] & f1)) : ((neg[0] & f0) | (neg[1] & f1));
        if ((fa[d] & kBrickCandidate) && an[d] != b && differ) want |= 1u << d;
    }
    want = __builtin_amdgcn_readfirstlane(want);
    if (!want) return 0u;
    // the claims' atomics issued together by lane 0, their results read after (first claimer wins)
    uint32_t old[6];
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        old[d] = 0u;
        if (((want >> d) & 1u) && (threadIdx.x & 63) == 0)
            old[d] = atomicOr(reinterpret_cast<uint32_t*>(cc.fill + (an[d] & ~3)), (uint32_t)kBrickClaimed << (8 * (an[d] & 3)));
    }
    uint32_t claimed = 0;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        const uint32_t o = __builtin_amdgcn_readfirstlane(old[d]);
        if (((want >> d) & 1u) && !((o >> (8 * (an[d] & 3))) & kBrickClaimed)) claimed |= 1u << d;
    }
    return claimed;
}

// a listed entry: the brick, then (mixed bricks) the candidates it claimed, with their own modes --
// one loop around a single copy of the tree code
template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>
__device__ __forceinline__ void eval_listed(const Eval& ev, const GridDesc& g, const BrickGrid& bg, const ClaimCtx& cc,
                                            uint32_t entry, uint64_t m64, float* __restrict__ field,
                                            sign_piece_t* __restrict__ signs) {
    const int b = (int)(entry & ~kListCheck);
    const bool check = (entry & kListCheck) && cc.fill;
    int cur = b;
    uint64_t mcur = m64;
    uint32_t claimed = 0;
    for (bool first = true;; first = false) {
        uint64_t neg[kBZ], valid;
        eval_one_brick<Eval, Pair>(ev, g, bg, cur, mcur, field, signs, first, neg, valid);
        if (first && check) claimed = claim_neighbours(g, bg, cc, b, neg, valid);
        if (!claimed) break;
        const int d = __builtin_ctz(claimed);
        claimed &= claimed - 1u;
        const int ax = d >> 1, up = d & 1;
        const int step = ax == 0 ? 1 : ax == 1 ? bg.nbx : bg.nbx * bg.nby;
        cur = up ? b + step : b - step;
        int cx, cy, cz;
        brick_of(cur, bg, cx, cy, cz);
        const int cb = cx + cy * cc.cnbx + (cz / kCZ) * cc.cplane;
        mcur = cc.ccls[cb] == kBrickMixed ? cc.bmodes[cur] : cc.cmodes[cb];
    }
}

// The same entry without evaluating the claimed candidates in this wave: they are appended to
// `claimed` (one atomic per claiming wave) for a second pass (eval.hip k_eval_claimed_b).  The
// merged object-stream eval runs the interpreter, whose candidate loop kept its state live across a
// second tree evaluation: 227 -> 196 VGPRs without it at stack depth 12, and at depth 9 168 -- three
// waves per SIMD instead of two.
template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>
__device__ __forceinline__ void eval_listed_deferred(const Eval& ev, const GridDesc& g, const BrickGrid& bg,
                                                     const ClaimCtx& cc, uint32_t entry, uint64_t m64,
                                                     float* __restrict__ field, sign_piece_t* __restrict__ signs,
                                                     uint32_t* __restrict__ claimed_list, uint32_t* __restrict__ claimed_count,
                                                     uint32_t claimed_cap) {
    const int b = (int)(entry & ~kListCheck);
    const bool check = (entry & kListCheck) && cc.fill;
    uint64_t neg[kBZ], valid;
    eval_one_brick<Eval, Pair>(ev, g, bg, b, m64, field, signs, true, neg, valid);
    if (!check) return;
    const uint32_t claimed = claim_neighbours(g, bg, cc, b, neg, valid);
    if (!claimed) return;   // uniform
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(claimed_count, (uint32_t)__popc(claimed));
    base = __builtin_amdgcn_readfirstlane(base);
    // lane d < 6 writes direction d's neighbour if claimed, at its rank among the claimed ones
    if (lane < 6 && ((claimed >> lane) & 1u)) {
        int bx, by, bz;
        brick_of(b, bg, bx, by, bz);
        const int ax = lane >> 1, up = lane & 1;
        const int step = ax == 0 ? 1 : ax == 1 ? bg.nbx : bg.nbx * bg.nby;
        const uint32_t at = base + (uint32_t)__popc(claimed & ((1u << lane) - 1u));
        if (at < claimed_cap) claimed_list[at] = (uint32_t)(up ? b + step : b - step);
    }
}

template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>
__device__ __forceinline__ void eval_bricks_body(const Eval& ev, const GridDesc& g, const BrickGrid& bg,
                                                 const ClaimCtx& cc, const uint64_t* __restrict__ modes,
                                                 const uint32_t* __restrict__ list, const uint32_t* __restrict__ count,
                                                 float* __restrict__ field, void* __restrict__ signs_raw) {
    sign_piece_t* signs = static_cast<sign_piece_t*>(signs_raw);
    const uint32_t nb = *count;
    const uint32_t wpb = blockDim.x >> 6;   // waves per block
    const uint32_t stride = gridDim.x * wpb;
    uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
    // the next brick's list entry and modes are loaded while this brick is evaluated
    uint32_t b_next = i < nb ? list[i] : 0u;
    uint64_t m_next = i < nb ? modes[i] : 0ull;
    for (; i < nb; i += stride) {
        const uint32_t e = __builtin_amdgcn_readfirstlane(b_next);
        const uint64_t m64 = m_next;
        if (i + stride < nb) {
            b_next = list[i + stride];
            m_next = modes[i + stride];
        }
        eval_listed<Eval, Pair>(ev, g, bg, cc, e, m64, field, signs);
    }
}

}  // namespace impli
