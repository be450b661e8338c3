// eval.hip -- implicit-function field evaluation on gfx950.
//
// k_eval_field : one lane per stored (interior) sample of the slab; the node program is
//                interpreted in lock step by the whole wave (uniform scalar loads of the
//                program and matrices), the result is written once, coalesced, x fastest.
//                Replaces prepare_grid + eval_shape (marching_cubes.hpp:1662-1725) -- the
//                reference's res^3 x 12 B point grid and its per-node batch copies never exist.
// k_eval_points: arbitrary points (direct-eval ABI, mcc2.cpp:815-911) with optional gradient.
#include <cstdlib>

#include "ifunc_device.hpp"
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
    const int sz = g.fz0 + (int)blockIdx.y;
    // prepare_grid (marching_cubes.hpp:1691-1693): x * factor + min - 2 * width
    const float x = ((float)(int)(sx + 2) * g.w[0] + g.lo[0]) - 2.f * g.w[0];
    const float y = ((float)(int)(sy + 2) * g.w[1] + g.lo[1]) - 2.f * g.w[1];
    const float z = ((float)sz * g.w[2] + g.lo[2]) - 2.f * g.w[2];
    const float f = eval_f<D>(prog, tab, x, y, z);
    field[(size_t)blockIdx.y * plane + i] = 0.f + f;   // eval_shape: field (zero) += value
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
