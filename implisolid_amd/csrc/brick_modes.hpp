// brick_modes.hpp -- device side of the interval pass (per-brick pruning modes and sign classes),
// shared by the static interpreter kernels (eval.hip) and the JIT-compiled tree kernels (jit.cpp).
//
// Two levels: a coarse box is kBX x kBY x (kCZ kBZ) samples, a brick kBX x kBY x kBZ.  Coarse
// boxes are bounded first; bricks of sign-definite boxes inherit the box's modes and class
// (k_brick_inherit, eval.hip); the listed mixed boxes are refined brick by brick, starting from
// the box's modes (an operand pruned over the box stays pruned over any sub-box).
#pragma once
#include "grid.hpp"
#include "eval_bricks.hpp"
#include "ifunc_interval.hpp"

namespace impli {

// Interval box of the samples [x0, x1] x [y0, y1] x layers [z0, z1]: the sample coordinate is
// monotone in the index, so the end samples bound the box.
__device__ __forceinline__ dev::Box sample_box(const GridDesc& g, int x0, int x1, int y0, int y1, int z0, int z1) {
    return dev::Box{dev::Iv{sample_xy(g, 0, x0), sample_xy(g, 0, x1)}, dev::Iv{sample_xy(g, 1, y0), sample_xy(g, 1, y1)},
                    dev::Iv{sample_z(g, z0), sample_z(g, z1)}};
}

__device__ __forceinline__ uint8_t sign_class(dev::Iv root) {   // MC sets a cube-index bit iff f < 0
    return (root.lo >= 0.f) ? kBrickPos : (root.hi < 0.f) ? kBrickNeg : kBrickMixed;
}

// block-aggregated append of `b` to list (order irrelevant): one atomic per block -- same-address
// atomics serialise (per-wave appends measured slower).  Every thread of the block must call it.
// cap: list capacity (entries past it are dropped -- never reached when the count starts at 0)
template <int kBlock>
__device__ __forceinline__ void block_append(bool take, uint32_t b, uint32_t* __restrict__ list,
                                             uint32_t* __restrict__ count, uint32_t cap) {
    __shared__ uint32_t s_cnt[kBlock / 64], s_base[kBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t mask = __ballot(take);
    if (lane == 0) s_cnt[w] = (uint32_t)__popcll((unsigned long long)mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < kBlock / 64; ++k) { s_base[k] = t; t += s_cnt[k]; }
        const uint32_t base = t ? atomicAdd(count, t) : 0u;
        for (int k = 0; k < kBlock / 64; ++k) s_base[k] += base;
    }
    __syncthreads();
    const uint32_t at = s_base[w] + (uint32_t)__popcll((unsigned long long)(mask & ((1ull << lane) - 1ull)));
    if (take && at < cap) list[at] = b;
}

// the brick's class, adjusted for sealed samples (the neighbours' fill test uses it): sealed
// samples (-1e7) only neighbour unsealed samples of the same brick -- unless the brick is nothing
// but the sealed layer, which is negative.  A positive brick holding sealed samples has crossing
// edges inside: kBrickNoFill.
__device__ __forceinline__ uint8_t sealed_class(const GridDesc& g, uint8_t c, int x0, int x1, int y0, int y1, int z0,
                                                int z1) {
    const bool has_sealed = x0 == 0 || x1 == g.n - 1 || y0 == 0 || y1 == g.n - 1 ||
                            g.fz0 + z0 <= 1 || g.fz0 + z1 >= g.res - 2;
    const bool only_sealed = x0 == g.n - 1 || y0 == g.n - 1 || (z0 == z1 && (g.fz0 + z0 <= 1 || g.fz0 + z0 >= g.res - 2));
    if (only_sealed) c = kBrickNeg;
    if (has_sealed && c == kBrickPos) c |= kBrickNoFill;
    return c;
}

struct BrickBox { int x0, x1, y0, y1, z0, z1; };
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ BrickBox brick_box(const GridDesc& g, int bx, int by, int bz, int zlen) {
    const int layers = g.fz1 - g.fz0;
    const int x0 = bx * kBX, y0 = by * kBY, z0 = bz * zlen;
    return BrickBox{x0, imin(x0 + kBX - 1, g.n - 1), y0, imin(y0 + kBY - 1, g.n - 1), z0, imin(z0 + zlen - 1, layers - 1)};
}

// class of brick (bx, by, bz) from its coarse box's class c and its refined class r: the
// sign-definite box's class (sealed-adjusted for the brick), or r for a brick of a mixed box
__device__ __forceinline__ uint32_t brick_class_of(const GridDesc& g, uint8_t c, uint8_t r, int bx, int by, int bz) {
    const BrickBox q = brick_box(g, bx, by, bz, kBZ);
    return c == kBrickMixed ? (uint32_t)r : (uint32_t)sealed_class(g, c, q.x0, q.x1, q.y0, q.y1, q.z0, q.z1);
}

// The neighbour rule (k_brick_fill, eval.hip): a brick needs exact values only if one of its
// samples can be the end of a sign-changing cell edge.  Edges are axis aligned, so that requires the
// brick or a face neighbour to differ in sign class.  Neighbours outside the stored grid hold no
// sample any cell of this slab reads (clamped to the brick itself).

// Coarse pass: one thread per coarse box -> modes, sign class; mixed boxes are listed.
// IvEval: Iv operator()(Box p, uint64_t modes_in, uint64_t& modes) const.
// counters = the engine's counter block (grid.hpp): block 0 clears it except the list length.
template <class IvEval>
__device__ __forceinline__ void coarse_modes_body(const IvEval& ev, const GridDesc& g, const BrickGrid& cg,
                                                  uint64_t* __restrict__ cmodes, uint8_t* __restrict__ ccls,
                                                  uint32_t* __restrict__ clist, uint32_t* __restrict__ counters) {
    uint32_t* ccount = counters + kCoarseListWord;
    if (blockIdx.x == 0 && threadIdx.x < kCounterWords && threadIdx.x != kCoarseListWord) counters[threadIdx.x] = 0u;
    const int b = blockIdx.x * 256 + threadIdx.x;
    uint8_t c = kBrickPos;
    if (b < cg.n_bricks) {
        int bx, by, bz;
        brick_of(b, cg, bx, by, bz);
        const BrickBox q = brick_box(g, bx, by, bz, kBZ * kCZ);
        uint64_t m;
        c = sign_class(ev(sample_box(g, q.x0, q.x1, q.y0, q.y1, q.z0, q.z1), 0ull, m));
        cmodes[b] = m;
        ccls[b] = c;
    }
    block_append<256>(b < cg.n_bricks && c == kBrickMixed, (uint32_t)b, clist, ccount, (uint32_t)cg.n_bricks);
}

// Bricks of the listed mixed coarse boxes, kRefineSplit = kBZ lanes per brick: item i is sample
// layer i % kBZ of brick (i / kBZ) % kCZ of listed box i / (kBZ kCZ).  A layer's box is flat in z,
// so z-piecewise primitives pick their pieces exactly (the double mushroom's caps r - z: over the
// whole brick the cap piece's bound spans the layer below the cap and reaches above 0, a false
// mixed class for every brick along the cap plane).  Interval arithmetic is inclusion-monotone, so
// each layer's bound is at least as tight as the brick's: the brick is of a definite class iff its
// layers are of that class, and a CSG operand pruned over all layers is pruned over the brick
// (modes agreeing over the layers are kept, the others reset to both operands -- never less
// pruning than the brick's own interval).
//
// WaveModes (merged object streams, whose waves each hold one object): the interval program starts
// from the modes every live lane of the wave agrees on (the others reset to both operands), so the
// interpreter's skips -- and with them its instruction fetch -- are wave-uniform.  Starting from
// fewer skips never changes the field: a mode is only ever derived from the brick's own interval,
// and a skipped operand's select would have returned the kept one exactly.
constexpr int kRefineSplit = kBZ;
#ifndef IMPLI_REFINE_WAVE_MODES   // the tree module's refine pass (JIT): per-lane modes measured as fast
#define IMPLI_REFINE_WAVE_MODES 0
#endif
__device__ __forceinline__ uint64_t agreeing_modes(uint64_t m_and, uint64_t m_or) {
    const uint64_t d = m_and ^ m_or;
    return m_and & ~(((d | (d >> 1)) & 0x5555555555555555ull) * 3ull);
}
template <class IvEval, bool WaveModes = false>
__device__ __forceinline__ void brick_refine_item(const IvEval& ev, const GridDesc& g, const BrickGrid& bg,
                                                  const BrickGrid& cg, const uint64_t* __restrict__ cmodes,
                                                  const uint32_t* __restrict__ clist, uint64_t* __restrict__ modes,
                                                  uint8_t* __restrict__ cls, uint32_t i, bool live) {
    static_assert((kRefineSplit & (kRefineSplit - 1)) == 0 && 64 % kRefineSplit == 0, "lane groups in a wave");
    const uint32_t bi = i / kRefineSplit, qd = i % kRefineSplit;
    const uint32_t cb = live ? clist[bi / kCZ] : 0u;
    int cx, cy, cz;
    brick_of((int)cb, cg, cx, cy, cz);
    const int bz = cz * kCZ + (int)(bi % kCZ);
    const bool ok = live && bz < bg.nbz;
    const BrickBox q = brick_box(g, cx, cy, ok ? bz : 0, kBZ);
    // the lane's layer (a brick past the slab's last layer repeats its last one)
    const int lz = min(q.z0 + (int)qd, q.z1);
    uint64_t m = cmodes[cb];
    if constexpr (WaveModes) {
        uint64_t wa = live ? m : ~0ull, wo = live ? m : 0ull;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            wa &= __shfl_xor(wa, o, 64);
            wo |= __shfl_xor(wo, o, 64);
        }
        m = agreeing_modes(wa, wo);
        m = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
            (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)m);
    }
    uint8_t c = sign_class(ev(sample_box(g, q.x0, q.x1, q.y0, q.y1, lz, lz), m, m));
    // combine the brick's lanes (consecutive lanes of one wave)
    uint64_t m_and = m, m_or = m;
    uint32_t c_and = c, c_or = c;
#pragma unroll
    for (int o = 1; o < kRefineSplit; o <<= 1) {
        const uint64_t a = __shfl_xor(m_and, o, 64), b = __shfl_xor(m_or, o, 64);
        m_and &= a;
        m_or |= b;
        c_and &= (uint32_t)__shfl_xor((int)c_and, o, 64);
        c_or |= (uint32_t)__shfl_xor((int)c_or, o, 64);
    }
    m = agreeing_modes(m_and, m_or);
    c = c_and == c_or ? (uint8_t)c_and : (uint8_t)kBrickMixed;
    if (!ok || qd != 0) return;
    const int b = cx + cy * bg.nbx + bz * bg.nbx * bg.nby;
    modes[b] = m;
    cls[b] = sealed_class(g, c, q.x0, q.x1, q.y0, q.y1, q.z0, q.z1);
}
template <class IvEval, bool WaveModes = IMPLI_REFINE_WAVE_MODES != 0>
__device__ __forceinline__ void brick_refine_body(const IvEval& ev, const GridDesc& g, const BrickGrid& bg,
                                                  const BrickGrid& cg, const uint64_t* __restrict__ cmodes,
                                                  const uint32_t* __restrict__ clist,
                                                  const uint32_t* __restrict__ ccount, uint64_t* __restrict__ modes,
                                                  uint8_t* __restrict__ cls) {
    const uint32_t total = min(*ccount, (uint32_t)cg.n_bricks) * kCZ * kRefineSplit;
    // the loop runs while any lane of the wave has an item: a brick's layer lanes shuffle together
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < total; i0 += gridDim.x * 256) {
        const uint32_t i = i0 + (threadIdx.x & 63u);
        brick_refine_item<IvEval, WaveModes>(ev, g, bg, cg, cmodes, clist, modes, cls, i, i < total);
    }
}

}  // namespace impli
