// Micro-benchmarks for the count kernel's regime (diagnostics only, not part of the library).
// hipcc -O3 --offload-arch=gfx950 tools/micro/mb.hip -o tools/micro/mb && ./tools/micro/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_empty(uint4* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = make_uint4(blockIdx.x, 0, 0, 0);
}
// streaming read: each thread 4 floats (dwordx4), sum -> one store per block
__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ in, size_t n4, float* out) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    float s = 0;
    for (; i < n4; i += (size_t)gridDim.x * 256) { float4 v = in[i]; s += v.x + v.y + v.z + v.w; }
    if (s == 12345.f) out[0] = s;
}
// count-like pattern: 1024-cell unit per block, 4 cells/thread, 20 loads (4 rows x 5), byte-ish store
__global__ __launch_bounds__(256) void k_countlike(const float* __restrict__ f, int n, int m, long ncells, unsigned* ci, uint4* cnt) {
    const unsigned L0 = blockIdx.x * 1024u + 4u * threadIdx.x;
    unsigned c = 0;
    if (L0 + 3 < ncells) {
        const unsigned mm = (unsigned)m * m;
        const unsigned zr = L0 / mm, rem = L0 - zr * mm, yr = rem / m, xr = rem - yr * m;
        const float* q = f + (xr + (size_t)yr * n + (size_t)zr * n * n);
        const size_t nn = (size_t)n * n;
        #pragma unroll
        for (int k = 0; k < 5; ++k) {
            c |= (q[k] < 0.f) << k;
            c |= (q[n + k] < 0.f) << (k + 5);
            c |= (q[nn + k] < 0.f) << (k + 10);
            c |= (q[nn + n + k] < 0.f) << (k + 15);
        }
        ci[L0 / 4] = c;
    }
    __shared__ unsigned s[4];
    unsigned v = c & 1;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = make_uint4(s[0] + s[1] + s[2] + s[3], 0, 0, 0);
}

int main() {
    const int R = 512, n = R + 3, m = R + 2;
    const long ncells = (long)m * m * m;
    const size_t nf = (size_t)n * n * (m + 1) + 1024;
    float* f; unsigned* ci; uint4* cnt; float* out;
    CK(hipMalloc(&f, nf * 4)); CK(hipMalloc(&ci, ncells + 4096)); CK(hipMalloc(&cnt, (ncells / 1024 + 2) * 16)); CK(hipMalloc(&out, 64));
    CK(hipMemset(f, 0, nf * 4));
    const unsigned nu = (unsigned)((ncells + 1023) / 1024);
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto time = [&](const char* name, auto launch, double bytes) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); ms /= 20;
        printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    time("empty 132k blocks", [&] { k_empty<<<nu, 256>>>(cnt); }, 16.0 * nu);
    time("stream read field (2048 blk)", [&] { k_stream<<<2048 * 4, 256>>>((const float4*)f, nf / 4, out); }, nf * 4.0);
    time("stream read field (full grid)", [&] { k_stream<<<(unsigned)(nf / 4 / 256), 256>>>((const float4*)f, nf / 4, out); }, nf * 4.0);
    time("countlike 4 cells/thread", [&] { k_countlike<<<nu, 256>>>(f, n, m, ncells, ci, cnt); }, nf * 4.0 + ncells);
    return 0;
}
