// VALU issue-rate microbenchmark for gfx950: how many wave64 VALU instructions per second the chip
// retires for the instruction kinds the ray kernels are made of (v_fma_f32, v_add_f32, v_mul_f32,
// v_pk_fma_f32, v_pk_add_f32, v_cndmask_b32, v_sqrt_f32), with 8 independent chains per lane and the
// grid filling every SIMD with `waves` waves.  Settles the VALU roofline bench.py prices against.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_peak tools/valu_peak.hip
// run:   tools/valu_peak [waves_per_simd=8]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int kIters = 2048;  // loop trips; 8 instructions per trip

#define OP8(ASM, T, ...)                                                                              \
    asm volatile(ASM : "+v"(a0) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a1) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a2) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a3) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a4) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a5) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a6) : "v"(m), "v"(c) : __VA_ARGS__);                                      \
    asm volatile(ASM : "+v"(a7) : "v"(m), "v"(c) : __VA_ARGS__);

#define KERNEL(NAME, T, ASM)                                                                          \
    __global__ __launch_bounds__(256) void NAME(T* out, T m, T c) {                                   \
        T a0 = out[0] + (T)threadIdx.x, a1 = a0 + (T)1, a2 = a0 + (T)2, a3 = a0 + (T)3;               \
        T a4 = a0 + (T)4, a5 = a0 + (T)5, a6 = a0 + (T)6, a7 = a0 + (T)7;                             \
        for (int i = 0; i < kIters; ++i) { OP8(ASM, T, "memory") }                                              \
        T s = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));                                     \
        if (s[0] == (float)-1.2345f) out[blockIdx.x * 256 + threadIdx.x] = s;                         \
    }

// scalar kinds operate on .x of a float2 so every kernel has the same shape
#define SK(NAME, ASM, ...)                                                                              \
    __global__ __launch_bounds__(256) void NAME(float* out, float m, float c) {                       \
        float a0 = out[0] + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;                       \
        float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                     \
        for (int i = 0; i < kIters; ++i) { OP8(ASM, float, __VA_ARGS__) }                                          \
        float s = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));                                  \
        if (s == -1.2345f) out[blockIdx.x * 256 + threadIdx.x] = s;                                   \
    }

SK(k_fma, "v_fma_f32 %0, %1, %2, %0", "memory")
SK(k_add, "v_add_f32 %0, %1, %0", "memory")
SK(k_mul, "v_mul_f32 %0, %1, %0", "memory")
SK(k_cnd, "v_cndmask_b32 %0, %1, %0, vcc", "memory")
SK(k_sqrt, "v_sqrt_f32 %0, %0", "memory")
SK(k_max, "v_max_f32 %0, %1, %0", "memory")
SK(k_cmp, "v_cmp_lt_f32 vcc, %1, %0", "vcc")
// a compare writing an SGPR pair followed by a select reading it (the pattern compilers emit)
SK(k_cmpsel, "v_cmp_lt_f32_e64 s[20:21], %1, %0\n\tv_cndmask_b32_e64 %0, %0, %1, s[20:21]", "s20", "s21")
// the e32 select reading VCC written by an e32 compare (what the compiler emits most)
SK(k_cmpsel32, "v_cmp_lt_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc", "vcc")
// e64 select reading an SGPR pair nobody writes in the loop (compare with k_cnd's VCC)
SK(k_cnd64s, "v_cndmask_b32_e64 %0, %1, %0, s[20:21]", "s20", "s21")
// e64 select reading VCC
SK(k_cnd64v, "v_cndmask_b32_e64 %0, %1, %0, vcc", "vcc")
// integer ops of the value-noise lattice hash (device_scene.hpp lattice)
SK(k_mullo, "v_mul_lo_u32 %0, %1, %0", "memory")
SK(k_mul24, "v_mul_u32_u24 %0, %1, %0", "memory")
SK(k_xor, "v_xor_b32 %0, %1, %0", "memory")
SK(k_lshr, "v_lshrrev_b32 %0, 16, %0", "memory")
SK(k_cvt, "v_cvt_f32_u32 %0, %0", "memory")
KERNEL(k_pkfma, f2, "v_pk_fma_f32 %0, %1, %2, %0")
KERNEL(k_pkadd, f2, "v_pk_add_f32 %0, %1, %0")
KERNEL(k_pkmul, f2, "v_pk_mul_f32 %0, %1, %0")

template <class K, class T>
static void run(const char* name, K k, T m, T c, int blocks, void* buf, int lane_flops) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, (decltype(m)*)buf, m, c);  // warm-up
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, (decltype(m)*)buf, m, c);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double waves = blocks * 4.0;
    const double instr = waves * kIters * 8.0;
    const double rate = instr / (best * 1e-3);
    // per SIMD cycle at 2.4 GHz: 256 CUs x 4 SIMDs
    const double cyc = 256.0 * 4 * 2.4e9 / rate;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"wave_instr_per_s\": %.4g, \"simd_cycles_per_wave_instr\": %.3f, "
           "\"tflops\": %.2f}\n",
           name, best, rate, cyc, rate * 64.0 * lane_flops / 1e12);
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const int waves_per_simd = argc > 1 ? atoi(argv[1]) : 8;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * waves_per_simd;  // 4 waves per block = 1 per SIMD
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"waves_per_simd\": %d, \"blocks\": %d}\n",
           prop.gcnArchName, prop.multiProcessorCount, prop.clockRate, waves_per_simd, blocks);
    void* buf;
    CHK(hipMalloc(&buf, (size_t)blocks * 256 * sizeof(f2)));
    CHK(hipMemset(buf, 0, (size_t)blocks * 256 * sizeof(f2)));
    f2 m2 = {1.0000001f, 0.9999999f}, c2 = {1e-7f, -1e-7f};
    run("v_fma_f32", k_fma, 1.0000001f, 1e-7f, blocks, buf, 2);
    run("v_add_f32", k_add, 1e-7f, 0.0f, blocks, buf, 1);
    run("v_mul_f32", k_mul, 1.0000001f, 0.0f, blocks, buf, 1);
    run("v_cndmask_b32", k_cnd, 1.0f, 0.0f, blocks, buf, 0);
    run("v_sqrt_f32", k_sqrt, 1.0f, 0.0f, blocks, buf, 1);
    run("v_max_f32", k_max, 1.0f, 0.0f, blocks, buf, 1);
    run("v_cmp_lt_f32(vcc)", k_cmp, 1.0f, 0.0f, blocks, buf, 0);
    run("v_cmp_e64+v_cndmask_e64 (pair, counted as 1)", k_cmpsel, 1.0f, 0.0f, blocks, buf, 0);
    run("v_cmp_e32+v_cndmask_e32 vcc (pair, counted as 1)", k_cmpsel32, 1.0f, 0.0f, blocks, buf, 0);
    run("v_cndmask_b32_e64 s[20:21]", k_cnd64s, 1.0f, 0.0f, blocks, buf, 0);
    run("v_cndmask_b32_e64 vcc", k_cnd64v, 1.0f, 0.0f, blocks, buf, 0);
    run("v_mul_lo_u32", k_mullo, 1.0f, 0.0f, blocks, buf, 0);
    run("v_mul_u32_u24", k_mul24, 1.0f, 0.0f, blocks, buf, 0);
    run("v_xor_b32", k_xor, 1.0f, 2.0f, blocks, buf, 0);
    run("v_lshrrev_b32", k_lshr, 1.0f, 0.0f, blocks, buf, 0);
    run("v_cvt_f32_u32", k_cvt, 1.0f, 0.0f, blocks, buf, 0);
    run("v_pk_fma_f32", k_pkfma, m2, c2, blocks, buf, 4);
    run("v_pk_add_f32", k_pkadd, c2, c2, blocks, buf, 2);
    run("v_pk_mul_f32", k_pkmul, m2, c2, blocks, buf, 2);
    CHK(hipFree(buf));
    return 0;
}
