// kernarg_cost.hip -- host cost of one kernel launch against the size of its argument block (is the
// 3.4 KB KParams block a measurable part of a small frame's launch?).  Launches an almost empty kernel
// (one 64-thread workgroup that reads one word of its arguments) N times per size on one stream, the
// enqueue loop timed alone and with the drain.  Diagnostics only.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/kernarg_cost tools/kernarg_cost.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int BYTES>
struct Args {
    unsigned int w[BYTES / 4];
};

template <int BYTES>
__global__ void touch(Args<BYTES> a, unsigned int* out) {
    if (threadIdx.x == 0 && a.w[BYTES / 4 - 1] == 0xdeadbeefu) out[0] = a.w[0];  // (never true: a read only)
}

template <int BYTES>
void run(hipStream_t st, unsigned int* d, int n) {
    Args<BYTES> a{};
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(touch<BYTES>, dim3(1), dim3(64), 0, st, a, d);
    (void)hipStreamSynchronize(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(touch<BYTES>, dim3(1), dim3(64), 0, st, a, d);
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    const auto t2 = std::chrono::steady_clock::now();
    std::printf("args %5d B  enqueue %.3f us/launch  enqueue+drain %.3f us/launch\n", BYTES,
                std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
}

int main() {
    hipStream_t st;
    unsigned int* d = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipMalloc(&d, 64) != hipSuccess) return 1;
    const int n = 5000;
    for (int rep = 0; rep < 2; ++rep) {
        run<64>(st, d, n);
        run<512>(st, d, n);
        run<1024>(st, d, n);
        run<1536>(st, d, n);
        run<2048>(st, d, n);
        run<3072>(st, d, n);
        run<3584>(st, d, n);
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(st);
    return 0;
}
