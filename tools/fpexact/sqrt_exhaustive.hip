// Exhaustive characterisation of gfx950 v_sqrt_f32 against the correctly rounded sqrt, and of
// shorter correction sequences, over all 2^32 f32 bit patterns.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float bits_f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t f_bits(float f) { return __float_as_uint(f); }

__device__ __forceinline__ float cand_two(float x) {   // two-sided, no scaling, no class fixup
    float s = __builtin_amdgcn_sqrtf(x);
    float lo = bits_f(f_bits(s) - 1u), hi = bits_f(f_bits(s) + 1u);
    float elo = __builtin_fmaf(-lo, s, x), ehi = __builtin_fmaf(-hi, s, x);
    s = (elo <= 0.0f) ? lo : s;
    s = (ehi > 0.0f) ? hi : s;
    return s;
}
__device__ __forceinline__ float cand_up(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    float hi = bits_f(f_bits(s) + 1u);
    return (__builtin_fmaf(-hi, s, x) > 0.0f) ? hi : s;
}
__device__ __forceinline__ float cand_down(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    float lo = bits_f(f_bits(s) - 1u);
    return (__builtin_fmaf(-lo, s, x) <= 0.0f) ? lo : s;
}

// sqrt of the predecessor pattern (biases the hardware error low), then one upward correction
__device__ __forceinline__ float cand_prev_up(float x) {
    uint32_t xb = f_bits(x);
    float s = __builtin_amdgcn_sqrtf(bits_f(xb ? xb - 1u : 0u));
    float hi = bits_f(f_bits(s) + 1u);
    return (__builtin_fmaf(-hi, s, x) > 0.0f) ? hi : s;
}
// two-sided correction on the raw hardware result, tiny non-zero magnitudes (< 2^-96) excluded
// from the count (they take the scaled path)
__device__ __forceinline__ bool tiny(float x) { return fabsf(x) < 0x1.0p-96f && x != 0.0f; }

struct Acc {
    unsigned long long hw_exact, hw_up, hw_down, hw_other;        // v_sqrt vs correctly rounded
    unsigned long long bad[5];                                   // cand_two, cand_up, cand_down mismatches
    unsigned int bad_min[5], bad_max[5];                         // smallest / largest failing pattern
};

__device__ __forceinline__ bool same(float a, float b) {
    return (a != a && b != b) || f_bits(a) == f_bits(b);
}

__global__ void sweep(uint32_t hi16, Acc* acc) {
    uint32_t x = (hi16 << 16) | (blockIdx.x * 256u + threadIdx.x) ;  // 65536 patterns per launch
    float f = bits_f(x);
    float r = __builtin_sqrtf(f);           // correctly rounded (LLVM expansion)
    float s = __builtin_amdgcn_sqrtf(f);
    int cls;
    if (same(s, r)) cls = 0;
    else if (f_bits(s) == f_bits(r) + 1u) cls = 1;
    else if (f_bits(s) == f_bits(r) - 1u) cls = 2;
    else cls = 3;
    unsigned long long* h = &acc->hw_exact;
    if (cls != 0) atomicAdd(&h[cls], 1ull);  // hw_exact = 2^32 - the rest (host)
    float c[5] = {cand_two(f), cand_up(f), cand_down(f), cand_prev_up(f), tiny(f) ? r : cand_two(f)};
    for (int k = 0; k < 5; ++k) {
        if (!same(c[k], r)) {
            atomicAdd(&acc->bad[k], 1ull);
            atomicMin(&acc->bad_min[k], x & 0x7fffffffu);
            atomicMax(&acc->bad_max[k], x & 0x7fffffffu);
        }
    }
}

int main() {
    Acc h{};
    for (int k = 0; k < 5; ++k) { h.bad_min[k] = 0xffffffffu; h.bad_max[k] = 0; }
    Acc* d;
    (void)hipMalloc(&d, sizeof(Acc));
    (void)hipMemcpy(d, &h, sizeof(Acc), hipMemcpyHostToDevice);
    for (uint32_t hi = 0; hi < 65536u; ++hi) hipLaunchKernelGGL(sweep, dim3(256), dim3(256), 0, 0, hi, d);
    if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"kernel\"}\n"); return 1; }
    (void)hipMemcpy(&h, d, sizeof(Acc), hipMemcpyDeviceToHost);
    h.hw_exact = (1ull << 32) - h.hw_up - h.hw_down - h.hw_other;
    printf("{\"hw_exact\": %llu, \"hw_up\": %llu, \"hw_down\": %llu, \"hw_other\": %llu", h.hw_exact, h.hw_up,
           h.hw_down, h.hw_other);
    const char* nm[5] = {"two", "up", "down", "prev_up", "two_guarded"};
    for (int k = 0; k < 5; ++k) {
        float mn, mx;
        memcpy(&mn, &h.bad_min[k], 4);
        memcpy(&mx, &h.bad_max[k], 4);
        printf(", \"%s\": {\"bad\": %llu, \"min\": \"0x%08x\", \"min_f\": %g, \"max\": \"0x%08x\", \"max_f\": %g}", nm[k],
               h.bad[k], h.bad_min[k], mn, h.bad_max[k], mx);
    }
    printf("}\n");
    return 0;
}
