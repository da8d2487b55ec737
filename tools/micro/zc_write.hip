// Design input for the zero-copy blocking path: a kernel storing a 1920x1080 RGBA8 frame straight
// into pinned host memory, one wave per tile, for the tile shapes a render could use -- 8x8 (the
// render's: 8 rows x 32 B per wave), 16x4 (4 x 64 B) and 32x2 (2 x 128 B, whole cache lines) -- into
// memory registered with hipHostRegister (default, coarse-grained) and hipHostMalloc'd memory, against
// the same stores into device memory.  A little arithmetic per pixel stands in for the render.
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/zc_write.hip -o tools/micro/zc_write
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

// heavy = 0: every tile does `iters`; 1: only the first half of the grid (dispatched first) does, the
// rest store at once; 2: only the second half does -- if stores into host memory leave while the heavy waves compute, the launch
// takes max(work, transfer), if they are held back to the kernel's end, the sum
// ST: 0 plain store, 1 non-temporal store, 2 relaxed store at system scope (write-through cache policy)
template <int TW, int ST = 0>
__global__ __launch_bounds__(64) void tile_store(uint32_t* out, uint32_t W, uint32_t H, uint32_t iters, uint32_t heavy) {
    constexpr int TH = 64 / TW;
    const uint32_t tiles_x = (W + TW - 1) / TW;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t lane = threadIdx.x;
    const uint32_t x = tx * TW + lane % TW, y = ty * TH + lane / TW;
    float v = (float)(x ^ y);
    const uint32_t n = (heavy == 1 && blockIdx.x >= gridDim.x / 2) || (heavy == 2 && blockIdx.x < gridDim.x / 2) ? 0u : iters;
    for (uint32_t i = 0; i < n; ++i) v = v * 1.0000001f + 0.5f;  // stand-in work
    if (x < W && y < H) {
        const uint32_t px = (uint32_t)v | 0xFF000000u;
        uint32_t* p = out + (size_t)y * W + x;
        if constexpr (ST == 1) __builtin_nontemporal_store(px, p);
        else if constexpr (ST == 2) __hip_atomic_store(p, px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else *p = px;
    }
}

template <int TW, int ST = 0>
float run(uint32_t* out, uint32_t W, uint32_t H, uint32_t iters, int reps, uint32_t heavy = 0) {
    constexpr int TH = 64 / TW;
    const uint32_t blocks = ((W + TW - 1) / TW) * ((H + TH - 1) / TH);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    tile_store<TW, ST><<<blocks, 64>>>(out, W, H, iters, heavy);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r) tile_store<TW, ST><<<blocks, 64>>>(out, W, H, iters, heavy);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const uint32_t W = 1920, H = 1080;
    const size_t bytes = (size_t)W * H * 4;
    uint32_t* dev = nullptr;
    (void)hipMalloc(&dev, bytes);
    uint32_t* hm = nullptr;
    (void)hipHostMalloc(&hm, bytes, hipHostMallocDefault);
    uint32_t* hm_dev = nullptr;
    (void)hipHostGetDevicePointer((void**)&hm_dev, hm, 0);
    std::vector<uint32_t> reg(W * H);
    (void)hipHostRegister(reg.data(), bytes, hipHostRegisterMapped);
    uint32_t* reg_dev = nullptr;
    (void)hipHostGetDevicePointer((void**)&reg_dev, reg.data(), 0);
    std::vector<uint32_t> regc(W * H);
    (void)hipHostRegister(regc.data(), bytes, hipHostRegisterMapped | hipExtHostRegisterCoarseGrained);
    uint32_t* regc_dev = nullptr;
    (void)hipHostGetDevicePointer((void**)&regc_dev, regc.data(), 0);
    struct { const char* name; uint32_t* p; } dst[] = {
        {"device", dev}, {"hipHostMalloc", hm_dev}, {"hostRegister", reg_dev}, {"hostRegister_coarse", regc_dev}};
    for (uint32_t iters : {0u, 2000u}) {
        for (auto& d : dst) {
            const float t8 = run<8>(d.p, W, H, iters, 10), t16 = run<16>(d.p, W, H, iters, 10),
                        t32 = run<32>(d.p, W, H, iters, 10), t64 = run<64>(d.p, W, H, iters, 10);
            printf("{\"dst\": \"%s\", \"work_iters\": %u, \"ms_8x8\": %.4f, \"ms_16x4\": %.4f, \"ms_32x2\": %.4f, "
                   "\"ms_64x1\": %.4f, \"GBps_8x8\": %.1f, \"GBps_32x2\": %.1f}\n",
                   d.name, iters, t8, t16, t32, t64, bytes / t8 / 1e6, bytes / t32 / 1e6);
        }
    }
    // overlap test: half the tiles (dispatched first) compute, the other half store at once
    uint32_t* hc = nullptr;
    (void)hipHostMalloc(&hc, bytes, hipHostMallocCoherent);
    uint32_t* hc_dev = nullptr;
    (void)hipHostGetDevicePointer((void**)&hc_dev, hc, 0);
    uint32_t* hn = nullptr;
    (void)hipHostMalloc(&hn, bytes, hipHostMallocNonCoherent);
    uint32_t* hn_dev = nullptr;
    (void)hipHostGetDevicePointer((void**)&hn_dev, hn, 0);
    struct { const char* name; uint32_t* p; } dst2[] = {{"device", dev}, {"hipHostMalloc", hm_dev},
        {"hipHostMalloc_coherent", hc_dev}, {"hipHostMalloc_noncoherent", hn_dev}, {"hostRegister", reg_dev},
        {"hostRegister_coarse", regc_dev}};
    // heavy 1: the heavy half first (the light half's stores wait for slots: end of kernel either way);
    // heavy 2: the light half first -- its 4.1 MB leave at once if stores go out while waves compute
    for (uint32_t heavy : {1u, 2u})
        for (uint32_t iters : {4000u, 8000u})
            for (auto& d : dst2)
                printf("{\"overlap\": \"%s\", \"heavy\": %u, \"heavy_half_iters\": %u, \"ms_32x2\": %.4f}\n",
                       d.name, heavy, iters, run<32>(d.p, W, H, iters, 10, heavy));
    for (auto& d : dst2)
        printf("{\"store_kind\": \"%s\", \"light_first_iters\": 4000, \"ms_plain\": %.4f, \"ms_nontemporal\": %.4f, "
               "\"ms_system_scope\": %.4f, \"no_work_nontemporal\": %.4f, \"no_work_system_scope\": %.4f}\n",
               d.name, run<32, 0>(d.p, W, H, 4000, 10, 2), run<32, 1>(d.p, W, H, 4000, 10, 2),
               run<32, 2>(d.p, W, H, 4000, 10, 2), run<32, 1>(d.p, W, H, 0, 10), run<32, 2>(d.p, W, H, 0, 10));
    bool ok = reg[5] == regc[5] && reg[W * H - 1] != 0u && hm[7] != 0u;
    printf("{\"host_values_written\": %s}\n", ok ? "true" : "false");
    return 0;
}
