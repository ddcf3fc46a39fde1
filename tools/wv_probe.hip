// wv_probe.hip — phase timing probe for decode_wave_kernel (diagnostics only).
// Builds the kernels with CPK_WV_PROF so every unit records cycle stamps after
// each phase (stage, walk A, walk B, rounds, count, expand) and counters
// (verification rounds, expand iterations, windows). Prints per-phase means.
// Usage: wv_probe [units=262144] [zero_thresh=128] [unit_bytes=4096]
#define CPK_WV_PROF 1
#include "../capnp-zig_amd/csrc/packed_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 262144;
    const uint32_t thr = argc > 2 ? atoi(argv[2]) : 128;
    const uint64_t ub = argc > 3 ? atoll(argv[3]) : 4096;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;  // 0 wave, 1 checkpoint pass + fast path, 2 stream
    const bool ck = mode == 1;
    const uint64_t slot = 10 * (ub / 8);
    std::vector<uint64_t> h_uoff(n), h_ulen(n, ub), h_poff(n), h_pcap(n, slot);
    for (uint32_t i = 0; i < n; ++i) { h_uoff[i] = i * ub; h_poff[i] = i * slot; }
    uint8_t *d_u, *d_p, *d_o;
    uint64_t *uoff, *ulen, *poff, *pcap, *plen, *olen, *prof;
    int32_t* st;
    CK(hipMalloc(&d_u, n * ub)); CK(hipMalloc(&d_o, n * ub)); CK(hipMalloc(&d_p, n * slot));
    CK(hipMalloc(&uoff, 8 * n)); CK(hipMalloc(&ulen, 8 * n)); CK(hipMalloc(&poff, 8 * n));
    CK(hipMalloc(&pcap, 8 * n)); CK(hipMalloc(&plen, 8 * n)); CK(hipMalloc(&olen, 8 * n));
    CK(hipMalloc(&st, 4 * n)); CK(hipMalloc(&prof, 16 * 8 * (size_t)n));
    CK(hipMemcpy(uoff, h_uoff.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(ulen, h_ulen.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(poff, h_poff.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(pcap, h_pcap.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(cpk::cpk_wv_prof), &prof, sizeof(prof)));
    CK(cpk::launch_generate(d_u, n, ub, 0, 0xC0DE0003ull, thr, 0));
    CK(cpk::launch_encode(d_u, uoff, ulen, n, d_p, poff, pcap, plen, st, true, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(prof, 0, 16 * 8 * (size_t)n));
        CK(hipEventRecord(a, 0));
        const uint32_t blocks = (n + cpk::kWvWaves - 1) / cpk::kWvWaves;
        if (mode == 2) {
            cpk::decode_stream_kernel<16, 2><<<(n + 127) / 128, 128, 0, 0>>>(d_p, poff, plen, n, d_o, uoff, ulen, olen, st);
        } else if (ck) {
            cpk::decode_ckpt_kernel<<<(n + cpk::kCkBlock - 1) / cpk::kCkBlock, cpk::kCkBlock, 0, 0>>>(
                d_p, poff, plen, n, d_o, uoff, ulen, olen, st);
            cpk::decode_wave_kernel<true><<<blocks, cpk::kWvBlock, 0, 0>>>(d_p, poff, plen, n, d_o, uoff, ulen, olen, st);
        } else {
            cpk::decode_wave_kernel<false><<<blocks, cpk::kWvBlock, 0, 0>>>(d_p, poff, plen, n, d_o, uoff, ulen, olen, st);
        }
        CK(hipGetLastError());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
    }
    std::vector<uint64_t> hp(16 * (size_t)n);
    CK(hipMemcpy(hp.data(), prof, 16 * 8 * (size_t)n, hipMemcpyDeviceToHost));
    std::vector<uint8_t> hu(n * ub), ho(n * ub);
    CK(hipMemcpy(hu.data(), d_u, n * ub, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ho.data(), d_o, n * ub, hipMemcpyDeviceToHost));
    const bool ok = hu == ho;
    const char* names[] = {"stage", "walkA", "walkB", "rounds", "count", "expand"};
    printf("{\"units\": %u, \"thr\": %u, \"ms\": %.4f, \"roundtrip_ok\": %s", n, thr, ms, ok ? "true" : "false");
    for (int k = 0; k < 6; ++k) {
        std::vector<double> v(n);
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t a = hp[16ull * i + k], b = hp[16ull * i + k + 1];
            v[i] = (a && b) ? (double)(int64_t)(b - a) : 0.0;
        }
        std::sort(v.begin(), v.end());
        double s = 0; for (double x : v) s += x;
        printf(", \"%s\": [%.0f, %.0f, %.0f]", names[k], s / n, v[n / 2], v[(size_t)(n * 0.99)]);
    }
    const char* cn[] = {"rounds", "expand_iters", "windows"};
    for (int k = 0; k < 3; ++k) {
        std::vector<double> v(n);
        for (uint32_t i = 0; i < n; ++i) v[i] = (double)hp[16ull * i + 8 + k];
        std::sort(v.begin(), v.end());
        double s = 0; for (double x : v) s += x;
        printf(", \"%s\": [%.2f, %.0f, %.0f, %.0f]", cn[k], s / n, v[n / 2], v[(size_t)(n * 0.99)], v[n - 1]);
    }
    printf("}\n");
    return ok ? 0 : 1;
}
