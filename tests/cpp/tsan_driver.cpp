// tsan_driver — the host code that runs on more than one thread, under ThreadSanitizer (SURVEY §5
// "race detection"; VERDICT r05 §5: no TSan run of the host threads).  Built by tools/tsan.sh with
// clang's TSan runtime from the CPU oracle, the C++ mirror and the host parts of librrte_hip; device
// code is never instrumented.  What runs concurrently, the way the library and its callers run it:
//  * the scene-specialised kernel's source generation and hiprtc compile (what a context's background
//    JIT worker does, rrte_hip.hip jit_pending / std::async) for two scenes at once, plus the lowering,
//    BVH build and CSG-guard analysis in front of it (rrte_hip_jit_check);
//  * tile-order planning from a profile (the context's tile-order worker, rrte_hip.hip tp.work);
//  * SceneIR dump / load (RRTE_DUMP_SCENE from every render entry point) into separate files;
//  * the JIT cache key / build id (a process-wide digest initialised on first use);
//  * the oracle's own row-chunk thread pool (the checker every parity test and the bench's CPU leg use).
// The context's own workers need a device; what they call is exactly the functions above, with inputs
// they own.  Exits non-zero on a mismatch; TSan reports races on stderr (tests/test_sanitize.py fails
// on any report).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <unistd.h>

#include "../../oracle/rrte_oracle.h"
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

static void jit_worker(const char* name, uint32_t w, uint32_t h) {
    const auto sc = rrte_examples::by_name(name, w, h, Mode::LambertShadow);
    const LoweredScene ls(sc.objects, sc.lights, sc.camera);
    char log[4096] = {0};
    const rrte_status st = rrte_hip_jit_check(&ls.ir(), (int)sc.config.lower().mode, log, sizeof log);
    CHECK(st == RRTE_OK, "%s: jit_check %d: %s", name, (int)st, log);
}

static void plan_worker(uint32_t seed) {
    const uint32_t tx = 240, n = 240 * 135;
    std::vector<uint32_t> costs(n), slots(n), again(n);
    for (uint32_t i = 0; i < n; ++i) costs[i] = 200u + ((i + seed) * 2654435761u >> 20) % 3000u;
    uint32_t a = 0, b = 0;
    CHECK(rrte_hip_tile_order_plan(costs.data(), n, tx, slots.data(), n, &a) == RRTE_OK, "plan");
    CHECK(rrte_hip_tile_order_plan(costs.data(), n, tx, again.data(), n, &b) == RRTE_OK, "plan again");
    CHECK(a == n && b == n && slots == again, "tile order not a pure function of its profile");
}

static void io_worker(int k) {
    const auto sc = rrte_examples::by_name("kitchen-sink", 32, 24, Mode::LambertShadow);
    const LoweredScene ls(sc.objects, sc.lights, sc.camera);
    const rrte_render_params p = sc.config.lower();
    const std::string path = "/tmp/rrte_tsan_" + std::to_string((long)getpid()) + "_" + std::to_string(k) + ".rrtesir";
    for (int it = 0; it < 4; ++it) {
        CHECK(rrte_hip_scene_dump(&ls.ir(), &p, path.c_str()) == RRTE_OK, "scene dump");
        rrte_scene_ir ir{};
        rrte_render_params q{};
        void* storage = nullptr;
        CHECK(rrte_hip_scene_load(path.c_str(), &ir, &q, &storage) == RRTE_OK, "scene load");
        CHECK(ir.num_prims == ls.ir().num_prims && !memcmp(&q, &p, sizeof p), "scene round trip");
        rrte_hip_scene_free(storage);
    }
    std::remove(path.c_str());
}

static void key_worker() {
    char id[40], k[40];
    for (int it = 0; it < 8; ++it) {
        CHECK(rrte_hip_build_id(id, sizeof id) == RRTE_OK, "build id");
        CHECK(rrte_hip_jit_cache_key("src", nullptr, k, sizeof k) == RRTE_OK, "cache key");
    }
}

static void oracle_worker() {
    const uint32_t w = 96, h = 54;
    const auto sc = rrte_examples::by_name("sdf-showcase", w, h, Mode::LambertShadow);
    const LoweredScene ls(sc.objects, sc.lights, sc.camera);
    const rrte_render_params p = sc.config.lower();
    std::vector<uint8_t> a(w * h * 4), b(w * h * 4);
    std::vector<float> fa(w * h * 4), fb(w * h * 4);
    uint64_t sa = 0, sb = 0;
    rrte_oracle_render(&ls.ir(), &p, a.data(), fa.data(), &sa, 4, 0, h);
    rrte_oracle_render(&ls.ir(), &p, b.data(), fb.data(), &sb, 1, 0, h);
    CHECK(a == b && sa == sb, "oracle output depends on its thread count");
}

int main() {
    const bool jit = std::getenv("RRTE_SANITIZE_JIT") == nullptr || std::strcmp(std::getenv("RRTE_SANITIZE_JIT"), "0");
    std::vector<std::thread> ts;
    if (jit) {
        ts.emplace_back(jit_worker, "sdf-showcase", 64, 36);
        ts.emplace_back(jit_worker, "basic-demo", 64, 48);
    }
    ts.emplace_back(plan_worker, 1u);
    ts.emplace_back(plan_worker, 2u);
    ts.emplace_back(io_worker, 0);
    ts.emplace_back(io_worker, 1);
    ts.emplace_back(key_worker);
    ts.emplace_back(key_worker);
    ts.emplace_back(oracle_worker);
    for (auto& t : ts) t.join();
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "tsan_driver: all checks passed", failures.load());
    return failures ? 1 : 0;
}
