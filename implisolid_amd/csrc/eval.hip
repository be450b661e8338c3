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
#include <cstdlib>

#include "ifunc_device.hpp"
#include "ifunc_interval.hpp"
#include "eval_bricks.hpp"
#include "kernels.hpp"

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
__global__ __launch_bounds__(256) void k_brick_modes(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                     float2 tab_range, GridDesc g, BrickGrid bg,
                                                     uint64_t* __restrict__ modes, uint8_t* __restrict__ cls) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= bg.n_bricks) return;
    int bx, by, bz;
    brick_of(b, bg, bx, by, bz);
    const int layers = g.fz1 - g.fz0;
    const int x0 = bx * kBX, x1 = min(x0 + kBX - 1, g.n - 1);
    const int y0 = by * kBY, y1 = min(y0 + kBY - 1, g.n - 1);
    const int z0 = bz * kBZ, z1 = min(z0 + kBZ - 1, layers - 1);
    // the sample coordinate is monotone in the index, so the end samples bound the brick
    const Box p{Iv{sample_xy(g, 0, x0), sample_xy(g, 0, x1)}, Iv{sample_xy(g, 1, y0), sample_xy(g, 1, y1)},
                Iv{sample_z(g, z0), sample_z(g, z1)}};
    uint64_t m;
    const Iv root = eval_iv<D>(prog, tab, tab_range, p, m);
    modes[b] = m;
    // Sign class of the brick's evaluated samples (MC sets a cube-index bit iff f < 0); the
    // neighbours' fill test uses it.  Sealed samples (-1e7) only neighbour unsealed samples of
    // the same brick -- unless the brick is nothing but the sealed layer, which is negative.
    // A positive brick holding sealed samples has crossing edges inside: kBrickNoFill.
    const bool has_sealed = x0 == 0 || x1 == g.n - 1 || y0 == 0 || y1 == g.n - 1 ||
                            g.fz0 + z0 <= 1 || g.fz0 + z1 >= g.res - 2;
    const bool only_sealed = x0 == g.n - 1 || y0 == g.n - 1 || (z0 == z1 && (g.fz0 + z0 <= 1 || g.fz0 + z0 >= g.res - 2));
    uint8_t c = (root.lo >= 0.f) ? kBrickPos : (root.hi < 0.f) ? kBrickNeg : kBrickMixed;
    if (only_sealed) c = kBrickNeg;
    if (has_sealed && c == kBrickPos) c |= kBrickNoFill;
    cls[b] = c;
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
                                                           const uint8_t* __restrict__ cls,
                                                           uint8_t* __restrict__ fill, int sign_fill,
                                                           float* __restrict__ field, void* __restrict__ signs) {
    eval_bricks_body(InterpEval<D>{prog, tab}, g, bg, modes, cls, fill, sign_fill, field, signs);
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

void launch_brick_modes(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                        uint64_t* d_modes, uint8_t* d_cls, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    const unsigned tb = (unsigned)((bg.n_bricks + 255) / 256);
    if (depth <= 4) k_brick_modes<4><<<tb, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, d_modes, d_cls);
    else if (depth <= 8) k_brick_modes<8><<<tb, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, d_modes, d_cls);
    else if (depth <= 12) k_brick_modes<12><<<tb, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, d_modes, d_cls);
    else k_brick_modes<16><<<tb, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, d_modes, d_cls);
}

void launch_signs_from_field(const GridDesc& g, const float* d_field, uint64_t* d_signs, hipStream_t s) {
    const int64_t words = (int64_t)g.n * (g.fz1 - g.fz0) * sign_row_words(g);
    if (words <= 0) return;
    k_signs_from_field<<<(unsigned)((words + 255) / 256), 256, 0, s>>>(g, d_field, d_signs);
}

void launch_eval_bricks_interp(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g,
                               const uint64_t* d_modes, const uint8_t* d_cls, uint8_t* d_fill, int sign_fill,
                               float* d_field, void* d_signs, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    const unsigned eb = (unsigned)((bg.n_bricks + 3) / 4);
    if (depth <= 4) k_eval_field_pruned<4><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_cls, d_fill, sign_fill, d_field, d_signs);
    else if (depth <= 8) k_eval_field_pruned<8><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_cls, d_fill, sign_fill, d_field, d_signs);
    else if (depth <= 12) k_eval_field_pruned<12><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_cls, d_fill, sign_fill, d_field, d_signs);
    else k_eval_field_pruned<16><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_cls, d_fill, sign_fill, d_field, d_signs);
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
