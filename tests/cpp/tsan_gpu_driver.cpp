// tsan_gpu_driver — the library's own worker threads under ThreadSanitizer, on a GPU (tools/tsan.sh
// gpu; host code instrumented, device code not).  Two host threads, each with a context of its own,
// render blocking frames through the C ABI while the contexts' workers run beside them: the AUTO
// policy's background hiprtc compile (rrte_hip.hip jit_pending, std::async; RRTE_JIT_CACHE=0 so it
// really compiles) and the tile-order planner after every profiled launch (tp.work, std::async;
// RRTE_TEST_RECYCLE=1 re-profiles every launch).  Each thread alternates two scenes / launch shapes
// every 8 frames, and every frame must equal the first frame of its scene on that context (the
// generic and the specialised kernels are bit-identical).  Exits non-zero on a mismatch or an error;
// TSan reports races on stderr.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../rrte_amd/cpp/examples.hpp"

using namespace rrte_renderer;

static std::atomic<int> failures{0};
#define CHECK(cond, ...)                                 \
    do {                                                 \
        if (!(cond)) {                                   \
            std::fprintf(stderr, "FAIL: " __VA_ARGS__);  \
            std::fprintf(stderr, "\n");                  \
            ++failures;                                  \
        }                                                \
    } while (0)

struct Job {
    std::string name;
    uint32_t w, h;
};

static void worker(int id, Job a, Job b, int frames) {
    rrte_ctx* ctx = nullptr;
    if (rrte_hip_create(0, &ctx) != RRTE_OK) {
        CHECK(false, "thread %d: create", id);
        return;
    }
    CHECK(rrte_hip_set_jit(ctx, RRTE_JIT_AUTO) == RRTE_OK, "set_jit");
    const auto sa = rrte_examples::by_name(a.name, a.w, a.h, Mode::LambertShadow);
    const auto sb = rrte_examples::by_name(b.name, b.w, b.h, Mode::LambertShadow);
    const LoweredScene la(sa.objects, sa.lights, sa.camera), lb(sb.objects, sb.lights, sb.camera);
    const rrte_render_params pa = sa.config.lower(), pb = sb.config.lower();
    std::vector<uint8_t> ref[2], out;
    uint32_t jit_seen = 0;
    for (int f = 0; f < frames; ++f) {
        const int k = (f / 8) & 1;
        const Job& j = k ? b : a;
        out.assign((size_t)j.w * j.h * 4, 0);
        const rrte_status st = rrte_hip_render(ctx, &(k ? lb : la).ir(), k ? &pb : &pa, out.data());
        if (st != RRTE_OK) {
            CHECK(false, "thread %d frame %d: render %d (%s)", id, f, (int)st, rrte_hip_last_error(ctx));
            break;
        }
        rrte_stats s{};
        CHECK(rrte_hip_stats(ctx, &s) == RRTE_OK, "stats");
        jit_seen |= 1u << s.jit_active;
        if (ref[k].empty()) ref[k] = out;
        else CHECK(out == ref[k], "thread %d frame %d (%s): differs from the scene's first frame (jit %u)", id, f,
                   j.name.c_str(), s.jit_active);
    }
    // then scene A alone until the background compile lands and the context switches kernels (the
    // adoption path: the worker's future collected, the module loaded), bounded by time, and 16 frames past it
    int extra = 0, after = -1;
    const auto t0 = std::chrono::steady_clock::now();
    out.assign((size_t)a.w * a.h * 4, 0);
    while (after < 16 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60)) {
        if (rrte_hip_render(ctx, &la.ir(), &pa, out.data()) != RRTE_OK) {
            CHECK(false, "thread %d: render (%s)", id, rrte_hip_last_error(ctx));
            break;
        }
        rrte_stats s{};
        CHECK(rrte_hip_stats(ctx, &s) == RRTE_OK, "stats");
        jit_seen |= 1u << s.jit_active;
        CHECK(out == ref[0], "thread %d: frame %d of the settled scene differs (jit %u)", id, extra, s.jit_active);
        ++extra;
        if (s.jit_active != 0 || after >= 0) ++after;
    }
    CHECK(after >= 16, "thread %d: the specialised kernel never became active", id);
    CHECK(rrte_hip_synchronize(ctx) == RRTE_OK, "synchronize");
    std::printf("thread %d: %d + %d frames, kernels seen (bit per jit kind) 0x%x\n", id, frames, extra, jit_seen);
    rrte_hip_destroy(ctx);
}

int main(int argc, char** argv) {
    const int frames = argc > 1 ? std::atoi(argv[1]) : 160;
    std::thread t0(worker, 0, Job{"sdf-showcase", 160, 90}, Job{"sdf-showcase", 96, 64}, frames);
    std::thread t1(worker, 1, Job{"advanced-demo", 128, 72}, Job{"basic-demo", 64, 48}, frames);
    t0.join();
    t1.join();
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "tsan_gpu_driver: all checks passed", failures.load());
    return failures ? 1 : 0;
}
