// Exhaustive check of a short correctly rounded reciprocal on gfx950: v_rcp_f32 + one fma
// Newton step, against the compiler's full 1.0f / x, over all 2^32 f32 bit patterns.
// Prints one JSON line: mismatches per candidate with the smallest / largest failing |x|.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float bits_f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t f_bits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ bool same(float a, float b) { return (a != a && b != b) || f_bits(a) == f_bits(b); }

__device__ __forceinline__ float cand_newton(float b) {
    float y = __builtin_amdgcn_rcpf(b);
    float e = __builtin_fmaf(-b, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
// Newton step, then the neighbour test on the (exact) residual: 1/b lies above y + u/2 iff
// 1 - b*y > b*u/2.
__device__ __forceinline__ float cand_newton_fix(float b) {
    float y = cand_newton(b);
    float hi = bits_f(f_bits(y) + 1u), lo = bits_f(f_bits(y) - 1u);
    float ehi = __builtin_fmaf(-b, hi, 1.0f), elo = __builtin_fmaf(-b, lo, 1.0f);
    float e = __builtin_fmaf(-b, y, 1.0f);
    // pick the candidate with the smallest |residual| (ties impossible away from powers of two)
    float r = y, best = fabsf(e);
    if (fabsf(ehi) < best) { r = hi; best = fabsf(ehi); }
    if (fabsf(elo) < best) { r = lo; }
    return r;
}
__device__ __forceinline__ bool guard(float b) {  // magnitudes outside [2^-126, 2^126] or non-finite
    float a = fabsf(b);
    return !(a >= 0x1.0p-126f && a <= 0x1.0p+126f);
}

struct Acc {
    unsigned long long hw_bad, bad[3];
    unsigned int bad_min[3], bad_max[3];
};

__global__ void sweep(uint32_t hi16, Acc* acc) {
    uint32_t x = (hi16 << 16) | (blockIdx.x * 256u + threadIdx.x);
    float f = bits_f(x);
    float r = 1.0f / f;  // correctly rounded (compiler's div expansion)
    if (!same(__builtin_amdgcn_rcpf(f), r)) atomicAdd(&acc->hw_bad, 1ull);
    float c[3] = {cand_newton(f), cand_newton_fix(f), guard(f) ? r : cand_newton(f)};
    for (int k = 0; k < 3; ++k) {
        if (!same(c[k], r)) {
            atomicAdd(&acc->bad[k], 1ull);
            atomicMin(&acc->bad_min[k], x & 0x7fffffffu);
            atomicMax(&acc->bad_max[k], x & 0x7fffffffu);
        }
    }
}

int main() {
    Acc h{};
    for (int k = 0; k < 3; ++k) { h.bad_min[k] = 0xffffffffu; h.bad_max[k] = 0; }
    Acc* d;
    (void)hipMalloc(&d, sizeof(Acc));
    (void)hipMemcpy(d, &h, sizeof(Acc), hipMemcpyHostToDevice);
    for (uint32_t hi = 0; hi < 65536u; ++hi) hipLaunchKernelGGL(sweep, dim3(256), dim3(256), 0, 0, hi, d);
    if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"kernel\"}\n"); return 1; }
    (void)hipMemcpy(&h, d, sizeof(Acc), hipMemcpyDeviceToHost);
    printf("{\"hw_bad\": %llu", h.hw_bad);
    const char* nm[3] = {"newton", "newton_fix", "newton_guarded"};
    for (int k = 0; k < 3; ++k) {
        float mn, mx;
        memcpy(&mn, &h.bad_min[k], 4);
        memcpy(&mx, &h.bad_max[k], 4);
        printf(", \"%s\": {\"bad\": %llu, \"min\": \"0x%08x\", \"min_f\": %g, \"max\": \"0x%08x\", \"max_f\": %g}", nm[k],
               h.bad[k], h.bad_min[k], mn, h.bad_max[k], mx);
    }
    printf("}\n");
    return 0;
}
