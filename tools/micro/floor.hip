// Kernel floors on one MI355X (diagnostics only, not part of the library): the in-stream cost of a
// launch that does almost nothing, and of a chain of k dependent global loads, at the block counts
// the per-slab kernels run with.  Each row: 200 back-to-back launches between two HIP events.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/floor.hip -o /tmp/floor && /tmp/floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_empty(uint32_t* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1u;
}
// k dependent loads (pointer chase through a small table that stays in L2 / MALL), one store
template <int K>
__global__ __launch_bounds__(256) void k_chain(const uint32_t* __restrict__ next, uint32_t* out) {
    uint32_t p = (blockIdx.x * 256u + threadIdx.x) & 4095u;
#pragma unroll
    for (int k = 0; k < K; ++k) p = next[p];
    out[blockIdx.x * 256u + threadIdx.x] = p;
}
// one block-aggregated append: __syncthreads, one atomic per block, the result broadcast, a store
__global__ __launch_bounds__(256) void k_append(uint32_t* count, uint32_t* out) {
    __shared__ uint32_t base;
    __syncthreads();
    if (threadIdx.x == 0) base = atomicAdd(count, 256u);
    __syncthreads();
    out[(base + threadIdx.x) & 0xfffffu] = threadIdx.x;
}

int main() {
    uint32_t *next, *out, *cnt;
    CK(hipMalloc(&next, 4096 * 4));
    CK(hipMalloc(&out, (size_t)64 << 20));
    CK(hipMalloc(&cnt, 64));
    std::vector<uint32_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (uint32_t)((i * 2654435761u + 17u) & 4095u);
    CK(hipMemcpy(next, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(cnt, 0, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200;
    auto run = [&](const char* name, int blocks, auto launch) -> int {
        for (int i = 0; i < 20; ++i) launch(blocks);
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; ++i) launch(blocks);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\": \"%s\", \"blocks\": %d, \"us_per_launch\": %.3f}\n", name, blocks, ms * 1e3f / reps);
        return 0;
    };
    for (int b : {1, 64, 256, 1024, 4096}) {
        run("empty", b, [&](int n) { k_empty<<<n, 256, 0, s>>>(out); });
        run("chain1", b, [&](int n) { k_chain<1><<<n, 256, 0, s>>>(next, out); });
        run("chain2", b, [&](int n) { k_chain<2><<<n, 256, 0, s>>>(next, out); });
        run("chain4", b, [&](int n) { k_chain<4><<<n, 256, 0, s>>>(next, out); });
        run("chain8", b, [&](int n) { k_chain<8><<<n, 256, 0, s>>>(next, out); });
        run("append", b, [&](int n) { k_append<<<n, 256, 0, s>>>(cnt, out); });
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
