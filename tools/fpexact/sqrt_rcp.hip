// Exhaustive check (all 2^32 f32 bit patterns) of normalize's (s, 1/s) pair from one v_rsq_f32
// against (sqrtf(x), 1.0f / sqrtf(x)); prints the mismatch count and the first failing patterns,
// with the two candidate reciprocals (one / two Newton steps from y = rsq(x)).
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o sqrt_rcp sqrt_rcp.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

struct Acc {
    unsigned long long bad[3];
    unsigned int nfirst;
    unsigned int first[16][4];
};

__global__ __launch_bounds__(256) void sweep(uint32_t hi16, Acc* acc) {
    const uint32_t xb = (hi16 << 16) | (blockIdx.x * 256u + threadIdx.x);
    const float x = __uint_as_float(xb);
    if (!(xb >= 0x0F800000u && xb < 0x7F800000u)) return;  // the guarded range
    const float want = __builtin_sqrtf(x), winv = 1.0f / want;
    const float y = __builtin_amdgcn_rsqf(x), s0 = x * y;
    const float s = __builtin_fmaf(__builtin_fmaf(-s0, s0, x), 0.5f * y, s0);
    const float r1 = __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
    const float r2 = __builtin_fmaf(__builtin_fmaf(-s, r1, 1.0f), r1, r1);
    const bool bs = __float_as_uint(s) != __float_as_uint(want);
    const bool b1 = __float_as_uint(r1) != __float_as_uint(winv);
    const bool b2 = __float_as_uint(r2) != __float_as_uint(winv);
    if (bs) atomicAdd(&acc->bad[0], 1ull);
    if (b1) atomicAdd(&acc->bad[1], 1ull);
    if (b2) atomicAdd(&acc->bad[2], 1ull);
    if (bs || b1 || b2) {
        const unsigned int n = atomicAdd(&acc->nfirst, 1u);
        if (n < 16u) {
            acc->first[n][0] = xb;
            acc->first[n][1] = __float_as_uint(s);
            acc->first[n][2] = __float_as_uint(r1);
            acc->first[n][3] = __float_as_uint(winv);
        }
    }
}

int main() {
    Acc* d = nullptr;
    if (hipMalloc(&d, sizeof(Acc)) != hipSuccess || hipMemset(d, 0, sizeof(Acc)) != hipSuccess) return 1;
    for (uint32_t hi = 0; hi < 65536u; ++hi) hipLaunchKernelGGL(sweep, dim3(256), dim3(256), 0, 0, hi, d);
    Acc h;
    if (hipMemcpy(&h, d, sizeof(Acc), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"sqrt_bad\": %llu, \"rcp1_bad\": %llu, \"rcp2_bad\": %llu, \"first\": [", h.bad[0], h.bad[1], h.bad[2]);
    for (unsigned i = 0; i < 16 && i < h.nfirst; ++i)
        printf("%s[\"0x%08x\", \"0x%08x\", \"0x%08x\", \"0x%08x\"]", i ? ", " : "", h.first[i][0], h.first[i][1], h.first[i][2], h.first[i][3]);
    printf("]}\n");
    return hipFree(d) == hipSuccess ? 0 : 1;
}
