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
#include "kernels.hpp"

namespace impli {

using namespace dev;

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

__device__ __forceinline__ void brick_of(int b, const BrickGrid& bg, int& bx, int& by, int& bz) {
    bx = b % bg.nbx;
    const int t = b / bg.nbx;
    by = t % bg.nby;
    bz = t / bg.nby;
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

// A brick needs exact values only if one of its samples can be the end of a sign-changing cell
// edge.  Edges are axis aligned, so that requires the brick or a face neighbour to differ in
// sign class.  Neighbours outside the stored grid hold no sample any cell of this slab reads.
__device__ __forceinline__ uint32_t brick_fill_class(const uint8_t* __restrict__ cls, const BrickGrid& bg, int b,
                                                     int bx, int by, int bz) {
    const uint32_t cb = cls[b], c = cb & 3u;
    if (c == kBrickMixed || (cb & kBrickNoFill)) return kBrickMixed;
    const int sy = bg.nbx, sz = bg.nbx * bg.nby;
    const uint32_t xm = bx > 0 ? cls[b - 1] & 3u : c, xp = bx + 1 < bg.nbx ? cls[b + 1] & 3u : c;
    const uint32_t ym = by > 0 ? cls[b - sy] & 3u : c, yp = by + 1 < bg.nby ? cls[b + sy] & 3u : c;
    const uint32_t zm = bz > 0 ? cls[b - sz] & 3u : c, zp = bz + 1 < bg.nbz ? cls[b + sz] & 3u : c;
    return (xm == c && xp == c && ym == c && yp == c && zm == c && zp == c) ? c : (uint32_t)kBrickMixed;
}

template <int D>
__global__ __launch_bounds__(256) void k_eval_field_pruned(const Program* __restrict__ prog,
                                                           const float* __restrict__ tab, GridDesc g, BrickGrid bg,
                                                           const uint64_t* __restrict__ modes,
                                                           const uint8_t* __restrict__ cls,
                                                           uint8_t* __restrict__ fill, int sign_fill,
                                                           float* __restrict__ field) {
    const int b = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
    if (b >= bg.n_bricks) return;
    const int lane = threadIdx.x & 63;
    int bx, by, bz;
    brick_of(b, bg, bx, by, bz);
    const int n = g.n;
    const int sx = bx * kBX + (lane % kBX), sy = by * kBY + (lane / kBX);
    const bool ok = sx < n && sy < n;
    const bool sealed_col = sealed_xy(g, sx) || sealed_xy(g, sy);
    const int layers = g.fz1 - g.fz0;
    const size_t plane = (size_t)n * n;
    float* out = field + (size_t)sy * n + sx;
    const uint32_t fc = sign_fill ? brick_fill_class(cls, bg, b, bx, by, bz) : (uint32_t)kBrickMixed;
    if (lane == 0) fill[b] = (uint8_t)fc;
    if (fc != kBrickMixed) {   // only the sign is ever read: any value of that sign will do
        const float v = (fc == kBrickPos) ? 1.f : -1.f;
        for (int k = 0; k < kBZ; ++k) {
            const int layer = bz * kBZ + k;
            if (layer >= layers) break;
            if (ok) out[(size_t)layer * plane] = (sealed_col || sealed_z(g, layer)) ? kSealed : v;
        }
        return;
    }
    const uint64_t m64 = modes[b];
    const uint64_t m = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m64 >> 32)) << 32) |
                       (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)m64);
    const float x = sample_xy(g, 0, ok ? sx : 0), y = sample_xy(g, 1, ok ? sy : 0);
#pragma unroll 1
    for (int k = 0; k < kBZ; ++k) {
        const int layer = bz * kBZ + k;
        if (layer >= layers) break;
        const float f = eval_f_pruned<D>(prog, tab, m, x, y, sample_z(g, layer));
        if (ok) out[(size_t)layer * plane] = (sealed_col || sealed_z(g, layer)) ? kSealed : 0.f + f;
    }
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

void launch_eval_field_pruned(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range,
                              const GridDesc& g, uint64_t* d_modes, uint8_t* d_cls, uint8_t* d_fill, int sign_fill,
                              float* d_field, hipStream_t s, hipEvent_t mid) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    const unsigned tb = (unsigned)((bg.n_bricks + 255) / 256), eb = (unsigned)((bg.n_bricks + 3) / 4);
#define IMPLI_PRUNED(DD)                                                                             \
    do {                                                                                             \
        k_brick_modes<DD><<<tb, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, d_modes, d_cls);    \
        if (mid) (void)hipEventRecord(mid, s);                                                       \
        k_eval_field_pruned<DD><<<eb, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_cls, d_fill,    \
                                                   sign_fill, d_field);                              \
    } while (0)
    if (depth <= 4) IMPLI_PRUNED(4);
    else if (depth <= 8) IMPLI_PRUNED(8);
    else if (depth <= 12) IMPLI_PRUNED(12);
    else IMPLI_PRUNED(16);
#undef IMPLI_PRUNED
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
