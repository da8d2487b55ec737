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

template <int TW>
__global__ __launch_bounds__(64) void tile_store(uint32_t* out, uint32_t W, uint32_t H, uint32_t iters) {
    constexpr int TH = 64 / TW;
    const uint32_t tiles_x = (W + TW - 1) / TW;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t lane = threadIdx.x;
    const uint32_t x = tx * TW + lane % TW, y = ty * TH + lane / TW;
    float v = (float)(x ^ y);
    for (uint32_t i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;  // stand-in work
    if (x < W && y < H) out[(size_t)y * W + x] = (uint32_t)v | 0xFF000000u;
}

template <int TW>
float run(uint32_t* out, uint32_t W, uint32_t H, uint32_t iters, int reps) {
    constexpr int TH = 64 / TW;
    const uint32_t blocks = ((W + TW - 1) / TW) * ((H + TH - 1) / TH);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    tile_store<TW><<<blocks, 64>>>(out, W, H, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r) tile_store<TW><<<blocks, 64>>>(out, W, H, iters);
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
    bool ok = reg[5] == regc[5] && reg[W * H - 1] != 0u && hm[7] != 0u;
    printf("{\"host_values_written\": %s}\n", ok ? "true" : "false");
    return 0;
}
