// Dev-only: what FETCH_SIZE counts on gfx950 for the read patterns of the codec's kernels.
// Each kernel reads a 256 MiB buffer (N bytes) once in a different pattern; run under
// `rocprofv3 --pmc FETCH_SIZE` and compare the per-kernel KB with N / 1024:
//   stream16   lane i reads bytes [16 i, 16 i + 16): a wave reads 1 KiB contiguous per load
//   lane512    lane l owns the 512-B unit l and reads it 16 B per step over 32 steps (the small
//              kernels' pattern: per step a wave touches 64 units, 64 different lines)
//   sparse16   only the first 16 B of every 128-B line, one load each (N / 8 useful bytes)
// Build: hipcc --offload-arch=gfx950 -O3 -o fetchprobe fetchprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void stream16(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void lane512(const uint4* __restrict__ p, uint64_t units, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < units; u += (uint64_t)gridDim.x * blockDim.x) {
        const uint4* q = p + 32 * u;
        for (int k = 0; k < 32; ++k) {
            const uint4 v = q[k];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void sparse16(const uint4* __restrict__ p, uint64_t lines, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[8 * i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t N = 256ull << 20;
    uint4* p = nullptr;
    uint32_t* o = nullptr;
    if (hipMalloc(&p, N) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    if (hipMemset(p, 1, N) != hipSuccess) return 1;
    for (int r = 0; r < 2; ++r) {
        stream16<<<4096, 256>>>(p, N / 16, o);
        lane512<<<2048, 256>>>(p, N / 512, o);
        sparse16<<<4096, 256>>>(p, N / 128, o);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("N = %llu bytes = %llu KB; sparse16 useful = %llu KB\n", (unsigned long long)N,
           (unsigned long long)(N / 1024), (unsigned long long)(N / 8 / 1024));
    hipFree(p);
    hipFree(o);
    return 0;
}
