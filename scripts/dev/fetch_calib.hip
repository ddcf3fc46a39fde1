// Dev probe (round 5): what FETCH_SIZE reports for the small kernels' read shapes, against a
// known footprint (MI355X_MICROARCH.md §HBM: only wide coalesced 16-B-per-lane reads are
// calibrated, at 1/2). Each kernel reads a 1 GiB buffer exactly once:
//   k0  coalesced: lane l of a wave reads 16 B at 16 l (1 KiB per instruction)
//   k1  lane per 128-B line, the line's 8 pieces by 8 consecutive instructions
//   k2  lane per 512-B span (a small unit), its 32 pieces by consecutive instructions
//   k3  lane per 64-B half line, 4 pieces
// Run under rocprofv3 --pmc FETCH_SIZE; prints the footprint per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int SPAN>  // bytes per lane, read 16 B at a time
__global__ __launch_bounds__(256) void rd(const u32x4* __restrict__ a, uint32_t* __restrict__ sink, size_t bytes) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    if (SPAN == 16) {
        for (size_t i = t; i < bytes / 16; i += (size_t)gridDim.x * 256) {
            const u32x4 v = a[i];
            acc ^= v.x ^ v.w;
        }
    } else {
        const size_t lanes = bytes / SPAN;
        for (size_t l = t; l < lanes; l += (size_t)gridDim.x * 256)
            for (int p = 0; p < SPAN / 16; ++p) {
                const u32x4 v = a[l * (SPAN / 16) + p];
                acc ^= v.x ^ v.w;
            }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const size_t bytes = 1ull << 30;
    u32x4* a;
    uint32_t* sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipDeviceSynchronize();
    rd<16><<<16384, 256>>>(a, sink, bytes);
    rd<128><<<(bytes / 128 + 255) / 256, 256>>>(a, sink, bytes);
    rd<512><<<(bytes / 512 + 255) / 256, 256>>>(a, sink, bytes);
    rd<64><<<(bytes / 64 + 255) / 256, 256>>>(a, sink, bytes);
    (void)hipDeviceSynchronize();
    printf("each kernel read %zu bytes (1 GiB): k<16> coalesced, k<128>, k<512>, k<64> lane-per-span\n", bytes);
    return 0;
}
