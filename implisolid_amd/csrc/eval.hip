// eval.hip -- implicit-function field evaluation on gfx950.
//
// k_eval_field : one lane per stored (interior) sample of the slab; the node program is
//                interpreted in lock step by the whole wave (uniform scalar loads of the
//                program and matrices), the result is written once, coalesced, x fastest.
//                Replaces prepare_grid + eval_shape (marching_cubes.hpp:1662-1725) -- the
//                reference's res^3 x 12 B point grid and its per-node batch copies never exist.
// k_brick_modes / k_eval_field_pruned: the same field, computed per brick of kBX x kBY x kBZ
//                samples.  A first pass bounds every node of the program over each brick
//                (ifunc_interval.hpp), records which CSG operands provably win and the brick's
//                sign class; the second pass (one wave per brick) skips the losing subtrees.
//                Level 1: bit-identical to k_eval_field (test_pruned_field_identical).
//                Level 2 (sign_fill): bricks that are sign-definite together with their face
//                neighbours get +-1 instead of exact values -- no cell edge touching them changes
//                sign, so marching cubes reads only their sign and the mesh is bit-identical
//                (test_sign_fill_field_equivalent + every MC parity test).
// k_eval_points: arbitrary points (direct-eval ABI, mcc2.cpp:815-911) with optional gradient.
#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include "ifunc_device.hpp"
#include "ifunc_interval.hpp"
#include "eval_bricks.hpp"
#include "brick_modes.hpp"
#include "kernels.hpp"
#include "jit.hpp"

namespace impli {

using namespace dev;

template <int D>
__global__ __launch_bounds__(256) void k_eval_field(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                    GridDesc g, float* __restrict__ field) {
    const uint32_t n = (uint32_t)g.n;
    const uint32_t plane = n * n;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= plane) return;
    const uint32_t sy = i / n, sx = i - sy * n;
    const int layer = (int)blockIdx.y;
    float f = kSealed;
    if (!(sealed_xy(g, (int)sx) || sealed_xy(g, (int)sy) || sealed_z(g, layer)))
        f = 0.f + eval_f<D>(prog, tab, sample_xy(g, 0, (int)sx), sample_xy(g, 1, (int)sy), sample_z(g, layer));
    field[(size_t)layer * plane + i] = f;   // eval_shape: field (zero) += value
}

template <int D>
struct InterpIv {   // the interval interpreter (ifunc_interval.hpp eval_iv)
    const Program* prog;
    const float* tab;
    float2 tab_range;
    __device__ __forceinline__ Iv operator()(Box p, uint64_t modes_in, uint64_t& modes) const {
        return eval_iv<D>(prog, tab, tab_range, p, modes_in, modes);
    }
};

template <int D>
__global__ __launch_bounds__(256) void k_coarse_modes(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      float2 tab_range, GridDesc g, BrickGrid cg,
                                                      uint64_t* __restrict__ cmodes, uint8_t* __restrict__ ccls,
                                                      uint32_t* __restrict__ clist, uint32_t* __restrict__ ccount) {
    coarse_modes_body(InterpIv<D>{prog, tab, tab_range}, g, cg, cmodes, ccls, clist, ccount);
}

// Bricks of sign-definite coarse boxes inherit the box's modes and class (valid on any sub-box).
__global__ __launch_bounds__(256) void k_brick_inherit(GridDesc g, BrickGrid bg, BrickGrid cg,
                                                       const uint64_t* __restrict__ cmodes,
                                                       const uint8_t* __restrict__ ccls, uint64_t* __restrict__ modes,
                                                       uint8_t* __restrict__ cls) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= bg.n_bricks) return;
    int bx, by, bz;
    brick_of(b, bg, bx, by, bz);
    const int cb = bx + by * cg.nbx + (bz / kCZ) * cg.nbx * cg.nby;
    const uint8_t c = ccls[cb];
    if (c == kBrickMixed) return;   // refined by k_brick_refine
    modes[b] = cmodes[cb];
    const BrickBox q = brick_box(g, bx, by, bz, kBZ);
    cls[b] = sealed_class(g, c, q.x0, q.x1, q.y0, q.y1, q.z0, q.z1);
}

template <int D>
__global__ __launch_bounds__(256) void k_brick_refine(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      float2 tab_range, GridDesc g, BrickGrid bg, BrickGrid cg,
                                                      const uint64_t* __restrict__ cmodes,
                                                      const uint32_t* __restrict__ clist,
                                                      const uint32_t* __restrict__ ccount, uint64_t* __restrict__ modes,
                                                      uint8_t* __restrict__ cls) {
    brick_refine_body(InterpIv<D>{prog, tab, tab_range}, g, bg, cg, cmodes, clist, ccount, modes, cls);
}

template <int D>
struct InterpEval {   // the node-program interpreter with per-brick operand skipping
    const Program* prog;
    const float* tab;
    __device__ __forceinline__ float operator()(uint64_t m, float x, float y, float z) const {
        return eval_f_pruned<D>(prog, tab, m, x, y, z);
    }
};

template <int D>
__global__ __launch_bounds__(256) void k_eval_field_pruned(const Program* __restrict__ prog,
                                                           const float* __restrict__ tab, GridDesc g, BrickGrid bg,
                                                           const uint64_t* __restrict__ modes,
                                                           const uint32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ count,
                                                           float* __restrict__ field, void* __restrict__ signs) {
    eval_bricks_body(InterpEval<D>{prog, tab}, g, bg, modes, list, count, field, signs);
}

// Neighbour rule per brick (brick_fill_class): fill[b], and the list of bricks to evaluate
// (mixed, or next to a brick of another class).  Wave-aggregated appends, order irrelevant.
__global__ __launch_bounds__(256) void k_brick_fill(const uint8_t* __restrict__ cls, BrickGrid bg, int sign_fill,
                                                    uint8_t* __restrict__ fill, uint32_t* __restrict__ list,
                                                    uint32_t* __restrict__ count) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint32_t fc = kBrickMixed;
    if (b < bg.n_bricks) {
        int bx, by, bz;
        brick_of(b, bg, bx, by, bz);
        fc = sign_fill ? brick_fill_class(cls, bg, b, bx, by, bz) : (uint32_t)kBrickMixed;
        fill[b] = (uint8_t)fc;
    }
    const bool eval = b < bg.n_bricks && fc == kBrickMixed;
    const uint64_t mask = __ballot(eval);
    uint32_t base = 0;
    if (lane == __ffsll((unsigned long long)mask) - 1) base = atomicAdd(count, (uint32_t)__popcll(mask));
    base = __shfl(base, __ffsll((unsigned long long)mask) - 1, 64);
    if (eval) list[base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))] = (uint32_t)b;
}

// Constant sign bits of the sign-filled bricks: one thread per 64-bit word of the bitmap (pieces
// of evaluated bricks are rewritten by the eval kernel afterwards).
__global__ __launch_bounds__(256) void k_sign_fill(GridDesc g, BrickGrid bg, const uint8_t* __restrict__ fill,
                                                   uint64_t* __restrict__ signs) {
    const int rw = sign_row_words(g);
    const int64_t rows = (int64_t)g.n * (g.fz1 - g.fz0);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rows * rw) return;
    const int64_t row = i / rw;
    const int c = (int)(i - row * rw);
    const int layer = (int)(row / g.n), y = (int)(row - (int64_t)layer * g.n);
    constexpr int P = 64 / kBX;   // pieces per word
    const uint8_t* f = fill + (size_t)((layer / kBZ) * bg.nby + y / kBY) * bg.nbx;
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int bx = c * P + j;
        if (bx < bg.nbx && f[bx] == kBrickNeg) w |= (kBX == 64 ? ~0ull : ((1ull << kBX) - 1ull)) << (kBX * j);
    }
    signs[i] = w;
}

// sign bitmap of a fully evaluated field (unpruned path): one thread per 64-bit word
__global__ __launch_bounds__(256) void k_signs_from_field(GridDesc g, const float* __restrict__ field,
                                                          uint64_t* __restrict__ signs) {
    const int rw = sign_row_words(g);
    const int64_t rows = (int64_t)g.n * (g.fz1 - g.fz0);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rows * rw) return;
    const int64_t row = i / rw;
    const int w = (int)(i - row * rw);
    const float* f = field + row * g.n;
    uint64_t bits = 0;
    for (int k = 0; k < 64; ++k) {
        const int x = 64 * w + k;
        if (x < g.n && f[x] < 0.f) bits |= 1ull << k;
    }
    signs[i] = bits;
}

template <int D>
__global__ __launch_bounds__(256) void k_eval_points(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                     const float* __restrict__ xyz, int64_t n, float* __restrict__ f,
                                                     float* __restrict__ grad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (grad) {
        V3 g;
        const float v = eval_fg<D>(prog, tab, x, y, z, g);
        if (f) f[i] = v;
        grad[3 * i] = g.x; grad[3 * i + 1] = g.y; grad[3 * i + 2] = g.z;
    } else {
        f[i] = eval_f<D>(prog, tab, x, y, z);
    }
}

// Stack capacity actually instantiated.  Below 12 slots LLVM lowers the uniform-index stack
// accesses to v_cndmask select chains (8 compares + 8 selects per access); from 12 slots on it
// uses VGPR index mode (s_set_gpr_idx_on + one v_mov), measured 1.7x faster on the config-4 tree.
// IMPLISOLID_EVAL_DEPTH overrides the floor (experiments).
static int eval_depth(int depth) {
    static int floor_d = [] {
        const char* s = std::getenv("IMPLISOLID_EVAL_DEPTH");
        return s ? std::atoi(s) : 12;
    }();
    return depth > floor_d ? depth : floor_d;
}

void launch_eval_field(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g, float* d_field,
                       hipStream_t s) {
    const uint32_t plane = (uint32_t)g.n * (uint32_t)g.n;
    const int layers = g.fz1 - g.fz0;
    if (layers <= 0) return;
    dim3 grid((plane + 255) / 256, layers);
    depth = eval_depth(depth);
    if (depth <= 4) k_eval_field<4><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, d_field);
    else if (depth <= 8) k_eval_field<8><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, d_field);
    else if (depth <= 12) k_eval_field<12><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, d_field);
    else k_eval_field<16><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, d_field);
}

BrickGrid brick_grid(const GridDesc& g) {
    BrickGrid bg;
    bg.nbx = (g.n + kBX - 1) / kBX;
    bg.nby = (g.n + kBY - 1) / kBY;
    bg.nbz = (g.fz1 - g.fz0 + kBZ - 1) / kBZ;
    if (bg.nbz < 0) bg.nbz = 0;
    bg.n_bricks = bg.nbx * bg.nby * bg.nbz;
    return bg;
}

BrickGrid coarse_grid(const GridDesc& g) {
    BrickGrid cg = brick_grid(g);
    cg.nbz = (g.fz1 - g.fz0 + kBZ * kCZ - 1) / (kBZ * kCZ);
    if (cg.nbz < 0) cg.nbz = 0;
    cg.n_bricks = cg.nbx * cg.nby * cg.nbz;
    return cg;
}

void launch_brick_modes(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                        uint64_t* d_cmodes, uint8_t* d_ccls, uint32_t* d_clist, uint32_t* d_ccount, uint64_t* d_modes,
                        uint8_t* d_cls, hipStream_t s, const JitIntervalKernels* jit) {
    BrickGrid bg = brick_grid(g), cg = coarse_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    (void)hipMemsetAsync(d_ccount, 0, sizeof(uint32_t), s);
    const unsigned tc = (unsigned)((cg.n_bricks + 255) / 256), tb = (unsigned)((bg.n_bricks + 255) / 256);
    const unsigned tr = (unsigned)std::min<int64_t>(((int64_t)cg.n_bricks * kCZ + 255) / 256, 2048);
    if (jit && jit->coarse && jit->refine) {
        GridDesc gg = g;
        const float* d_mats = reinterpret_cast<const float*>(reinterpret_cast<const char*>(d_prog) + offsetof(Program, mats));
        void* ca[] = {&d_mats, &d_rabbit, &tab_range, &gg, &cg, &d_cmodes, &d_ccls, &d_clist, &d_ccount};
        TreeJit::launch(jit->coarse, tc, ca, s, "impli_coarse_modes");
        k_brick_inherit<<<tb, 256, 0, s>>>(g, bg, cg, d_cmodes, d_ccls, d_modes, d_cls);
        void* ra[] = {&d_mats, &d_rabbit, &tab_range, &gg, &bg, &cg, &d_cmodes, &d_clist, &d_ccount, &d_modes, &d_cls};
        TreeJit::launch(jit->refine, tr, ra, s, "impli_brick_refine");
        return;
    }
#define IMPLI_MODES(DD)                                                                                           \
    do {                                                                                                          \
        k_coarse_modes<DD><<<tc, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, cg, d_cmodes, d_ccls, d_clist,     \
                                              d_ccount);                                                          \
        k_brick_inherit<<<tb, 256, 0, s>>>(g, bg, cg, d_cmodes, d_ccls, d_modes, d_cls);                          \
        k_brick_refine<DD><<<tr, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, cg, d_cmodes, d_clist, d_ccount, \
                                              d_modes, d_cls);                                                    \
    } while (0)
    if (depth <= 4) IMPLI_MODES(4);
    else if (depth <= 8) IMPLI_MODES(8);
    else if (depth <= 12) IMPLI_MODES(12);
    else IMPLI_MODES(16);
#undef IMPLI_MODES
}

void launch_signs_from_field(const GridDesc& g, const float* d_field, uint64_t* d_signs, hipStream_t s) {
    const int64_t words = (int64_t)g.n * (g.fz1 - g.fz0) * sign_row_words(g);
    if (words <= 0) return;
    k_signs_from_field<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(g, d_field, d_signs);
}

void launch_brick_fill(const uint8_t* d_cls, const GridDesc& g, int sign_fill, uint8_t* d_fill, uint32_t* d_list,
                       uint32_t* d_count, uint64_t* d_signs, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    (void)hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
    k_brick_fill<<<(unsigned)((bg.n_bricks + 255) / 256), 256, 0, s>>>(d_cls, bg, sign_fill, d_fill, d_list, d_count);
    const int64_t words = (int64_t)g.n * (g.fz1 - g.fz0) * sign_row_words(g);
    k_sign_fill<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(g, bg, d_fill, d_signs);
}

unsigned eval_bricks_grid(const GridDesc& g) {
    const int nb = brick_grid(g).n_bricks;
    const unsigned want = (unsigned)((nb + 3) / 4);
    return want < 4096u ? (want ? want : 1u) : 4096u;   // grid-stride over the list
}

void launch_eval_bricks_interp(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g,
                               const uint64_t* d_modes, const uint32_t* d_list, const uint32_t* d_count,
                               float* d_field, void* d_signs, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    const unsigned eb = eval_bricks_grid(g);
    if (depth <= 4) k_eval_field_pruned<4><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list, d_count, d_field, d_signs);
    else if (depth <= 8) k_eval_field_pruned<8><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list, d_count, d_field, d_signs);
    else if (depth <= 12) k_eval_field_pruned<12><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list, d_count, d_field, d_signs);
    else k_eval_field_pruned<16><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list, d_count, d_field, d_signs);
}

void launch_eval_points(const Program* d_prog, int depth, const float* d_rabbit, const float* d_xyz, int64_t n,
                        float* d_f, float* d_grad, hipStream_t s) {
    if (n <= 0) return;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    depth = eval_depth(depth);
    if (depth <= 4) k_eval_points<4><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else if (depth <= 8) k_eval_points<8><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else if (depth <= 12) k_eval_points<12><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else k_eval_points<16><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
}

}  // namespace impli
