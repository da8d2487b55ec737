// Does a wave64 VALU instruction cost less when one 32-lane half of EXEC is empty?  (Design input for
// the sphere-tracing loop: divergent exits narrow EXEC, a predicated loop keeps it full.)
// Every wave runs the same FMA loop (8 independent chains) under an EXEC pattern chosen per launch;
// the chip is filled with waves; kernel time by HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(64) void valu_loop(float* out, int iters, uint64_t pattern) {
    const int lane = threadIdx.x & 63;
    if (!((pattern >> lane) & 1ull)) return;   // EXEC for the loop = pattern
    float a0 = lane * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 0.999f, c = 1e-4f;
    for (int i = 0; i < iters; ++i) {
        a0 = __builtin_fmaf(a0, m, c); a1 = __builtin_fmaf(a1, m, c); a2 = __builtin_fmaf(a2, m, c); a3 = __builtin_fmaf(a3, m, c);
        a4 = __builtin_fmaf(a4, m, c); a5 = __builtin_fmaf(a5, m, c); a6 = __builtin_fmaf(a6, m, c); a7 = __builtin_fmaf(a7, m, c);
    }
    out[blockIdx.x * 64 + lane] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
}

int main() {
    const int blocks = 256 * 4 * 8 * 4;  // 4 rounds of 8 waves per SIMD on 256 CUs
    const int iters = 4096;
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * 64);
    struct { const char* name; uint64_t p; } pats[] = {
        {"all 64 lanes", ~0ull}, {"lanes 0-31 (upper half empty)", 0xffffffffull},
        {"lanes 32-63 (lower half empty)", 0xffffffff00000000ull}, {"lanes 0 and 32 (both halves)", 0x100000001ull},
        {"lane 0 only", 1ull}, {"lanes 0-15 + 32-47", 0x0000ffff0000ffffull}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep)
        for (auto& p : pats) {
            hipLaunchKernelGGL(valu_loop, dim3(blocks), dim3(64), 0, 0, out, iters, p.p);  // warm
            hipEventRecord(e0);
            hipLaunchKernelGGL(valu_loop, dim3(blocks), dim3(64), 0, 0, out, iters, p.p);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * iters * 8;  // wave-level FMA instructions
            printf("%-34s %8.3f ms  %7.1f G wave-instr/s\n", p.name, ms, winst / (ms * 1e-3) / 1e9);
        }
    hipFree(out);
    return 0;
}
