// Design input for the blocking drop-in path (rrte_hip_render into a host buffer): how fast can an
// 8.3 MB RGBA8 1080p frame reach host memory?  (a) hipMemcpy D2H into pageable memory, (b) into
// pinned memory (SDMA), (c) SDMA split over 2 / 4 streams, (d) a blit kernel storing dwordx4 into
// pinned host memory mapped to the device, (e) host memcpy pinned -> pageable with 1/2/4/8 threads,
// into a reused and into a freshly allocated buffer.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__global__ void blit(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t bytes = 1920ull * 1080 * 4;
    void* d;
    (void)hipMalloc(&d, bytes);
    (void)hipMemset(d, 7, bytes);
    void* pinned;
    (void)hipHostMalloc(&pinned, bytes, hipHostMallocDefault);
    void* mapped;  // coherent pinned + device pointer for the blit kernel
    (void)hipHostMalloc(&mapped, bytes, hipHostMallocMapped);
    void* mapped_d;
    (void)hipHostGetDevicePointer(&mapped_d, mapped, 0);
    std::vector<char> pageable(bytes, 1);
    hipStream_t st[4];
    for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    auto timeit = [&](const char* name, auto fn) {
        double best = 1e9;
        for (int r = 0; r < 12; ++r) {
            (void)hipDeviceSynchronize();
            const double t0 = now_ms();
            fn();
            best = std::min(best, now_ms() - t0);
        }
        printf("%-52s %7.3f ms  %6.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    };
    timeit("(a) hipMemcpy D2H pageable (reused)", [&] { (void)hipMemcpy(pageable.data(), d, bytes, hipMemcpyDeviceToHost); });
    timeit("(a') hipMemcpy D2H pageable (fresh buffer)", [&] {
        char* f = (char*)calloc(bytes, 1);
        (void)hipMemcpy(f, d, bytes, hipMemcpyDeviceToHost);
        free(f);
    });
    timeit("(b) hipMemcpy D2H pinned", [&] { (void)hipMemcpy(pinned, d, bytes, hipMemcpyDeviceToHost); });
    for (int ns : {2, 4}) {
        char name[64];
        snprintf(name, sizeof name, "(c) D2H pinned split over %d streams", ns);
        timeit(name, [&] {
            const size_t part = bytes / ns;
            for (int i = 0; i < ns; ++i)
                (void)hipMemcpyAsync((char*)pinned + i * part, (char*)d + i * part, part, hipMemcpyDeviceToHost, st[i]);
            for (int i = 0; i < ns; ++i) (void)hipStreamSynchronize(st[i]);
        });
    }
    for (int blocks : {256, 1024, 4096}) {
        char name[64];
        snprintf(name, sizeof name, "(d) blit kernel -> mapped pinned, %d blocks", blocks);
        timeit(name, [&] {
            hipLaunchKernelGGL(blit, dim3(blocks), dim3(256), 0, st[0], (const uint4*)d, (uint4*)mapped_d, bytes / 16);
            (void)hipStreamSynchronize(st[0]);
        });
    }
    for (int nt : {1, 2, 4, 8}) {
        for (int fresh = 0; fresh < 2; ++fresh) {
            char name[64];
            snprintf(name, sizeof name, "(e) host memcpy pinned->%s, %d threads", fresh ? "fresh" : "reused", nt);
            timeit(name, [&] {
                char* dst = fresh ? (char*)calloc(bytes, 1) : pageable.data();
                std::vector<std::thread> th;
                const size_t part = (bytes + nt - 1) / nt;
                for (int i = 0; i < nt; ++i)
                    th.emplace_back([&, i] {
                        const size_t a = i * part, b = std::min(bytes, a + part);
                        memcpy(dst + a, (char*)pinned + a, b - a);
                    });
                for (auto& t : th) t.join();
                if (fresh) free(dst);
            });
        }
    }
    timeit("(f) calloc + first touch of 8.3 MB (page faults)", [&] {
        char* f = (char*)calloc(bytes, 1);
        for (size_t i = 0; i < bytes; i += 4096) f[i] = 1;
        free(f);
    });
    return 0;
}
