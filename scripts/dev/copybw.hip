// Dev-only: device copy / read / write bandwidth ceilings on this box (4 GiB buffers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int NT, int UNR>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 * UNR + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256 * UNR;
    for (; i < n; i += stride) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = (i + u * 256 < n) ? a[i + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNR; ++u)
            if (i + u * 256 < n) {
                if (NT) __builtin_nontemporal_store(v[u], b + i + u * 256);
                else b[i + u * 256] = v[u];
            }
    }
}
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    for (; i < n; i += (size_t)gridDim.x * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) b[0] = acc;
}
__global__ __launch_bounds__(256) void write_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * 256) __builtin_nontemporal_store(u32x4{1, 2, 3, (uint32_t)i}, b + i);
}
template <typename K>
static float timeit(K k, int grid, const u32x4* a, u32x4* b, size_t n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k<<<grid, 256>>>(a, b, n);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<<<grid, 256>>>(a, b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}
int main() {
    const size_t bytes = 4ull << 30, n = bytes / 16;
    u32x4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
    for (int grid : {2048, 4096, 8192, 16384, 65536}) {
        float t0 = timeit(copy_k<0, 1>, grid, a, b, n), t1 = timeit(copy_k<1, 1>, grid, a, b, n);
        float t2 = timeit(copy_k<1, 4>, grid, a, b, n);
        float tr = timeit(read_k, grid, a, b, n), tw = timeit(write_k, grid, a, b, n);
        printf("grid %6d copy %.0f GB/s  copy-nt %.0f  copy-nt-x4 %.0f  read %.0f  write-nt %.0f\n", grid,
               2 * bytes / t0 / 1e6, 2 * bytes / t1 / 1e6, 2 * bytes / t2 / 1e6, bytes / tr / 1e6, bytes / tw / 1e6);
    }
    return 0;
}
