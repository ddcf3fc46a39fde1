// Dev probe (round 5): write bandwidth of the store shapes a lane-per-unit decoder can issue.
// A wave owns 64 "units" of 4 KiB output each (1M units = 4 GiB); it writes them in 64 sub-rounds
// of 64 B per unit, as:
//   mode 0  quads, 16 units per instruction, each unit's 64 B at an 8-B offset (run starts at 8 (mod 64))
//   mode 1  quads, 16 units per instruction, each unit's 64 B 64-B aligned
//   mode 2  each lane its own unit, 4 x 16 B (16-B aligned), 64 units per instruction
//   mode 3  8 lanes per unit, 128 B (a whole line) every second sub-round, 8 units per instruction
//   mode 4  the whole wave one unit: 1 KiB contiguous per instruction (the fill pass's shape)
//   +8      non-temporal stores
// Prints GB/s per mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void store_k(uint8_t* out, uint32_t nwaves) {
    const uint32_t wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wv >= nwaves) return;
    uint8_t* base = out + (uint64_t)wv * 64 * 4096;  // 64 units x 4 KiB
    const u32x4 v = {lane, wv, 1u, 2u};
    auto st = [&](uint8_t* p) {
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
        else asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    };
    if (MODE == 0 || MODE == 1) {
        const uint32_t off0 = MODE == 0 ? 8 : 0;
        for (uint32_t r = 0; r < 63; ++r)
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t u = 16 * m + lane / 4, q = lane & 3;
                st(base + (uint64_t)u * 4096 + off0 + 64 * r + 16 * q);
            }
    } else if (MODE == 2) {
        for (uint32_t r = 0; r < 64; ++r)
            for (uint32_t j = 0; j < 4; ++j) st(base + (uint64_t)lane * 4096 + 64 * r + 16 * j);
    } else if (MODE == 3) {
        for (uint32_t r = 0; r < 32; ++r)
            for (uint32_t m = 0; m < 8; ++m) {
                const uint32_t u = 8 * m + lane / 8, q = lane & 7;
                st(base + (uint64_t)u * 4096 + 128 * r + 16 * q);
            }
    } else {
        for (uint32_t u = 0; u < 64; ++u)
            for (uint32_t c = 0; c < 4; ++c) st(base + (uint64_t)u * 4096 + 1024 * c + 16 * lane);
    }
}

template <typename K>
static float timeit(K k, int grid, uint8_t* out, uint32_t nw) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<<<grid, 256>>>(out, nw);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<<<grid, 256>>>(out, nw);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    const uint64_t units = 1u << 20, bytes = units * 4096;
    uint8_t* out;
    if (hipMalloc(&out, bytes + 4096) != hipSuccess) return 1;
    const uint32_t nw = units / 64, grid = nw / 4;
    const char* names[] = {"quads 64B @8-B offset", "quads 64B aligned", "lane 4x16B", "8 lanes 128B lines",
                           "wave 1KiB contiguous"};
    float t[10];
    t[0] = timeit(store_k<0, false>, grid, out, nw);
    t[1] = timeit(store_k<1, false>, grid, out, nw);
    t[2] = timeit(store_k<2, false>, grid, out, nw);
    t[3] = timeit(store_k<3, false>, grid, out, nw);
    t[4] = timeit(store_k<4, false>, grid, out, nw);
    t[5] = timeit(store_k<0, true>, grid, out, nw);
    t[6] = timeit(store_k<1, true>, grid, out, nw);
    t[7] = timeit(store_k<2, true>, grid, out, nw);
    t[8] = timeit(store_k<3, true>, grid, out, nw);
    t[9] = timeit(store_k<4, true>, grid, out, nw);
    for (int i = 0; i < 5; ++i)
        printf("%-24s plain %6.0f GB/s   nt %6.0f GB/s\n", names[i], bytes / t[i] / 1e6, bytes / t[5 + i] / 1e6);
    return 0;
}
