// batch_device.hpp -- device helpers of the merged object-stream launches (ObjArgs, kernels.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace impli {

// The per-object work of the merged passes differs by orders of magnitude between objects (their
// listed boxes, bricks, unit parts, records), so the merged grid-stride kernels spread one flat
// index over every object's items: each block loads the n list lengths, forms their exclusive prefix in LDS, and a
// thread (refine) or wave (eval) finds the object of its item by binary search.
constexpr int kMaxBatchObjects = 1024;
// align: each object's range rounded up to a multiple of it (64: every wave holds one object)
__device__ __forceinline__ uint32_t batch_prefix(const ObjArgs* __restrict__ objs, int n, int word, uint32_t mult,
                                                 uint32_t cap, uint32_t* s_pre, uint32_t align = 1u) {
    __shared__ uint32_t s_part[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;   // 256 threads, up to 4 objects each
    uint32_t v[4], c[4] = {0u, 0u, 0u, 0u}, sum = 0;
    if (n > 0) {   // uniform; the four loads unconditional (a clamped index), so they issue together
                   // instead of one round trip per guarded load
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = objs[4 * t + k < n ? 4 * t + k : n - 1].counters[word];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int o = 4 * t + k;
        v[k] = o < n ? (min(c[k], cap) * mult + align - 1u) / align * align : 0u;
        sum += v[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) s_part[w] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (int k = 0; k < w; ++k) run += s_part[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (4 * t + k <= n) s_pre[4 * t + k] = run;   // s_pre[n] = total
        run += v[k];
    }
    __syncthreads();
    return s_pre[n];
}
__device__ __forceinline__ int batch_object_of(const uint32_t* s_pre, int n, uint32_t i) {   // last o: pre[o] <= i
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

}  // namespace impli
