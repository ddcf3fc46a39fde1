// Dev probe (round 5): how many 128-thread blocks with a given dynamic LDS size the hardware keeps
// resident per CU at once (census: each block bumps a per-CU counter through its lifetime and
// records the peak). XCC_ID and CU_ID come from the HW_ID registers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(128) void census(unsigned* cur, unsigned* peak, unsigned spin) {
    extern __shared__ uint8_t dyn[];
    if (threadIdx.x == 0) {
        unsigned hw = 0, xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        const unsigned id = ((xcc & 7) * 8 + se) * 32 + sh * 16 + cu;
        const unsigned c = atomicAdd(&cur[id], 1u) + 1;
        atomicMax(&peak[id], c);
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < spin) dyn[0] = (uint8_t)t0;
        atomicSub(&cur[id], 1u);
    }
}

int main() {
    unsigned *cur, *peak;
    const int N = 8 * 8 * 32;
    (void)hipMalloc(&cur, N * 4);
    (void)hipMalloc(&peak, N * 4);
    for (int kb : {8192, 16384, 20480, 24576, 26624, 27136, 27264, 27648, 28672, 30720, 30848, 32000, 32512, 32768,
                   40832, 40960}) {
        (void)hipFuncSetAttribute((const void*)census, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        (void)hipMemset(cur, 0, N * 4);
        (void)hipMemset(peak, 0, N * 4);
        census<<<256 * 24, 128, kb>>>(cur, peak, 200000);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed at %d\n", kb); return 1; }
        unsigned h[N];
        (void)hipMemcpy(h, peak, sizeof h, hipMemcpyDeviceToHost);
        unsigned mx = 0, mn = 1000, cus = 0;
        for (int i = 0; i < N; ++i)
            if (h[i]) { mx = h[i] > mx ? h[i] : mx; mn = h[i] < mn ? h[i] : mn; ++cus; }
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, census, 128, kb);
        printf("LDS %6d B/block: resident blocks per CU min %u max %u over %u CUs (API %d)\n", kb, mn, mx, cus, occ);
    }
    return 0;
}
