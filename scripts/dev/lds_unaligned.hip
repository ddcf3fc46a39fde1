// Dev probe (round 5): does gfx950 LDS serve ds_read_b64 / ds_read_b128 / ds_write_b64 at byte
// alignment, and at what cost? Checks every byte offset 0..15 against the expected bytes and times
// 4096 independent reads per lane at aligned and unaligned addresses (s_memtime ticks per read).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void probe(uint64_t* out, uint32_t* bad, uint64_t* ticks) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[8192];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 8192; i += 64) lds[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    uint32_t nbad = 0;
    for (uint32_t off = 0; off < 16; ++off) {
        const uint32_t a = (uint32_t)(uintptr_t)lds + lane * 80 + off;
        uint64_t v;
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        uint64_t e = 0;
        for (int k = 0; k < 8; ++k) e |= (uint64_t)(uint8_t)((lane * 80 + off + k) * 7 + 3) << (8 * k);
        nbad += v != e;
        u32x4 w;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a) : "memory");
        uint32_t ew[4] = {0, 0, 0, 0};
        for (int k = 0; k < 16; ++k) ew[k / 4] |= (uint32_t)(uint8_t)((lane * 80 + off + k) * 7 + 3) << (8 * (k & 3));
        nbad += (w.x != ew[0]) + (w.y != ew[1]) + (w.z != ew[2]) + (w.w != ew[3]);
    }
    bad[lane] = nbad;
    // timing: independent reads, aligned (offset 0) vs unaligned (offset 3), lane stride 80 B
    for (int mode = 0; mode < 3; ++mode) {
        const uint32_t a = (uint32_t)(uintptr_t)lds + lane * 80 + (mode == 0 ? 0 : mode == 1 ? 3 : 5);
        uint64_t acc = 0;
        __syncthreads();
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < 1024; ++r) {
            uint64_t v0, v1, v2, v3;
            asm volatile("ds_read_b64 %0, %4\n ds_read_b64 %1, %4 offset:8\n ds_read_b64 %2, %4 offset:16\n"
                         " ds_read_b64 %3, %4 offset:24\n s_waitcnt lgkmcnt(0)"
                         : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3) : "v"(a) : "memory");
            acc += v0 ^ v1 ^ v2 ^ v3;
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) ticks[mode] = t1 - t0;
        out[lane + 64 * mode] = acc;
    }
}

int main() {
    uint64_t *out, *ticks;
    uint32_t* bad;
    hipMalloc(&out, 64 * 3 * 8);
    hipMalloc(&bad, 64 * 4);
    hipMalloc(&ticks, 3 * 8);
    probe<<<1, 64>>>(out, bad, ticks);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    uint32_t hb[64];
    uint64_t ht[3];
    hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
    hipMemcpy(ht, ticks, sizeof ht, hipMemcpyDeviceToHost);
    uint32_t tot = 0;
    for (int i = 0; i < 64; ++i) tot += hb[i];
    printf("unaligned ds_read_b64/b128 mismatches: %u (of %d checks)\n", tot, 64 * 16 * 5);
    printf("ticks per 4 x ds_read_b64 (one wave, lane stride 80 B): aligned %.1f, +3 %.1f, +5 %.1f\n",
           ht[0] / 1024.0, ht[1] / 1024.0, ht[2] / 1024.0);
    return 0;
}
