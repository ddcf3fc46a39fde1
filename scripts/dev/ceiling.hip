// Dev-only: HBM ceilings on this box for the decode's traffic shape (round 5, verdict r4 item 1a).
// Copy (1:1), read-only, write-only, and a "decode-shaped" stream that reads R and writes W bytes
// (R:W = 5:8, the p = 0.5 decode's P:U), each as a persistent grid with UNR 16-B accesses in flight
// per lane. 4 GiB of writes, buffers far beyond the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNR, int NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * UNR;
    for (size_t i = (size_t)blockIdx.x * 256 * UNR + threadIdx.x; i < n; i += stride) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = (i + u * 256 < n) ? __builtin_nontemporal_load(a + i + u * 256) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            if (i + u * 256 < n) {
                if (NT) __builtin_nontemporal_store(v[u], b + i + u * 256);
                else b[i + u * 256] = v[u];
            }
    }
}
template <int UNR>
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * UNR;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 * UNR + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) if (i + u * 256 < n) acc ^= __builtin_nontemporal_load(a + i + u * 256);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) b[0] = acc;
}
template <int UNR>
__global__ __launch_bounds__(256) void write_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * UNR;
    for (size_t i = (size_t)blockIdx.x * 256 * UNR + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            if (i + u * 256 < n) __builtin_nontemporal_store(u32x4{1, 2, 3, (uint32_t)i}, b + i + u * 256);
    }
}
// decode-shaped: per 256-thread block step, read 5 x 4 KiB, write 8 x 4 KiB (P:U = 0.625)
__global__ __launch_bounds__(256) void dshape_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t nsteps) {
    for (size_t s = blockIdx.x; s < nsteps; s += gridDim.x) {
        const u32x4* src = a + s * 5 * 256 + threadIdx.x;
        u32x4* dst = b + s * 8 * 256 + threadIdx.x;
        u32x4 v[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) v[u] = __builtin_nontemporal_load(src + u * 256);
        u32x4 x = v[0] ^ v[1] ^ v[2] ^ v[3] ^ v[4];
#pragma unroll
        for (int u = 0; u < 8; ++u) __builtin_nontemporal_store(x + (uint32_t)u, dst + u * 256);
    }
}
template <typename K, typename A>
static float timeit(K k, int grid, const u32x4* a, u32x4* b, A n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<<<grid, 256>>>(a, b, n);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<<<grid, 256>>>(a, b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0); hipEventDestroy(e1);
    return ms / 5;
}
int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    u32x4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
    const size_t nsteps = bytes / (8 * 4096);  // 4 GiB written, 2.5 GiB read
    for (int grid : {1024, 2048, 4096, 8192, 65536, 262144}) {
        float c1 = timeit(copy_k<1, 1>, grid, a, b, n), c4 = timeit(copy_k<4, 1>, grid, a, b, n);
        float c8 = timeit(copy_k<8, 1>, grid, a, b, n), c4p = timeit(copy_k<4, 0>, grid, a, b, n);
        float r4 = timeit(read_k<4>, grid, a, b, n), r8 = timeit(read_k<8>, grid, a, b, n);
        float w4 = timeit(write_k<4>, grid, a, b, n);
        float ds = timeit(dshape_k, grid, a, b, nsteps);
        printf("grid %6d copy-nt x1 %.0f x4 %.0f x8 %.0f | copy x4 plain-store %.0f | read x4 %.0f x8 %.0f | "
               "write-nt x4 %.0f | decode-shaped (R 2.5 + W 4 GiB) %.0f GB/s\n",
               grid, 2 * bytes / c1 / 1e6, 2 * bytes / c4 / 1e6, 2 * bytes / c8 / 1e6, 2 * bytes / c4p / 1e6,
               bytes / r4 / 1e6, bytes / r8 / 1e6, bytes / w4 / 1e6, (bytes * 1.625) / ds / 1e6);
    }
    return 0;
}
