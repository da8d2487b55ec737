// Does a wave64 VALU instruction cost less when one 32-lane half of EXEC is empty?  (Design input for
// the sphere-tracing loop: divergent exits narrow EXEC, a predicated loop keeps it full.)
// Every wave runs the same FMA loop (8 independent chains) under an EXEC pattern chosen per launch;
// the chip is filled with waves; kernel time by HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int CHAINS>
__global__ __launch_bounds__(64) void valu_loop(float* out, int iters, uint64_t pattern) {
    const int lane = threadIdx.x & 63;
    if (!((pattern >> lane) & 1ull)) return;   // EXEC for the loop = pattern
    float a0 = lane * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 0.999f, c = 1e-4f;
    for (int i = 0; i < iters; ++i) {
        a0 = __builtin_fmaf(a0, m, c);
        if (CHAINS > 1) { a1 = __builtin_fmaf(a1, m, c); a2 = __builtin_fmaf(a2, m, c); a3 = __builtin_fmaf(a3, m, c); }
        if (CHAINS > 4) { a4 = __builtin_fmaf(a4, m, c); a5 = __builtin_fmaf(a5, m, c); a6 = __builtin_fmaf(a6, m, c); a7 = __builtin_fmaf(a7, m, c); }
    }
    out[blockIdx.x * 64 + lane] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
}

int main() {
    const int iters = 4096;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 4 * 8 * 4 * 64);
    struct { const char* name; uint64_t p; } pats[] = {
        {"64 lanes", ~0ull}, {"32: lanes 0-31", 0xffffffffull}, {"32: lanes 0-15+32-47", 0x0000ffff0000ffffull},
        {"16: lanes 0-15", 0xffffull}, {"8: lanes 0-7", 0xffull}, {"4: lanes 0-3", 0xfull}, {"2: lanes 0-1", 0x3ull},
        {"1: lane 0", 1ull}, {"1: lane 5", 1ull << 5}, {"1: lane 40", 1ull << 40}, {"2: lanes 0,32", 0x100000001ull},
        {"4: lanes 0,16,32,48", 0x0001000100010001ull}, {"8: every 8th", 0x0101010101010101ull},
        {"16: every 4th", 0x1111111111111111ull}, {"32: every 2nd", 0x5555555555555555ull}};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int chains : {8, 1}) {
        // 8 chains: issue-bound with 8 waves/SIMD; 1 chain, 1 wave/SIMD: dependent-latency-bound
        const int blocks = chains == 8 ? 256 * 4 * 8 * 4 : 256 * 4;
        for (auto& p : pats) {
            float best = 1e9f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                if (chains == 8) hipLaunchKernelGGL(valu_loop<8>, dim3(blocks), dim3(64), 0, 0, out, iters, p.p);
                else hipLaunchKernelGGL(valu_loop<1>, dim3(blocks), dim3(64), 0, 0, out, iters * 4, p.p);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep) best = ms < best ? ms : best;
            }
            const double winst = (double)blocks * (chains == 8 ? iters * 8 : iters * 4);
            printf("chains %d %-24s %8.3f ms  %7.1f G wave-instr/s  %6.2f cyc/instr/wave@2.4GHz\n", chains, p.name, best,
                   winst / (best * 1e-3) / 1e9, best * 1e-3 * 2.4e9 / ((double)(chains == 8 ? iters * 8 : iters * 4) * blocks / (chains == 8 ? 8192.0 : 1024.0)));
        }
    }
    (void)hipFree(out);
    return 0;
}
