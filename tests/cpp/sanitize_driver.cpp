// sanitize_driver — the host-only code paths under AddressSanitizer + UndefinedBehaviorSanitizer
// (SURVEY §5 "race detection / sanitizers").  Built by tools/sanitize.sh with clang's
// sanitizer runtime from: the CPU oracle (oracle/rrte_oracle.c), the C++ mirror of the renderer API
// (rrte_amd/cpp/), and the host parts of librrte_hip (scene validation + lowering, the BVH builder,
// the CSG-guard analysis, the scene-specialised kernel source generator and its hiprtc compile) --
// device code is never instrumented (GPU sanitizers are not available).  Exits non-zero on any
// mismatch; the sanitizers abort on any memory or UB error.
#include <cstdio>
#include <unistd.h>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../oracle/rrte_oracle.h"
#include "../../rrte_amd/cpp/examples.hpp"

using namespace rrte_renderer;

static int failures = 0;
#define CHECK(cond, ...)                                 \
    do {                                                 \
        if (!(cond)) {                                   \
            std::fprintf(stderr, "FAIL: " __VA_ARGS__);  \
            std::fprintf(stderr, "\n");                  \
            ++failures;                                  \
        }                                                \
    } while (0)

static void run_scene(const char* name, uint32_t w, uint32_t h, Mode mode, bool jit) {
    const auto sc = rrte_examples::by_name(name, w, h, mode);
    const LoweredScene ls(sc.objects, sc.lights, sc.camera);
    const rrte_scene_ir& ir = ls.ir();
    const rrte_render_params p = sc.config.lower();
    // the oracle, multi-threaded (its row-chunk pool) and single-threaded: identical bytes
    std::vector<uint8_t> a(w * h * 4), b(w * h * 4);
    std::vector<float> fa(w * h * 4), fb(w * h * 4);
    uint64_t sa = 0, sb = 0;
    rrte_oracle_render(&ir, &p, a.data(), fa.data(), &sa, 4, 0, h);
    rrte_oracle_render(&ir, &p, b.data(), fb.data(), &sb, 1, 0, h);
    CHECK(a == b && sa == sb, "%s: oracle output depends on the thread count", name);
    // CSG guard analysis on every SDF program (host only)
    for (uint32_t i = 0; i < ir.num_prims; ++i) {
        const rrte_prim& pr = ir.prims[i];
        if (pr.kind != RRTE_PRIM_SDF) continue;
        std::vector<rrte_sdf_node> out(pr.sdf_count);
        uint32_t guards = 0;
        for (uint32_t ml : {0u, 1u, 2u, 3u}) {
            const rrte_status st = rrte_hip_sdf_guards(ir.sdf_nodes + pr.sdf_first, pr.sdf_count, ml, out.data(), &guards);
            CHECK(st == RRTE_OK, "%s: sdf_guards prim %u status %d", name, i, (int)st);
        }
    }
    // lowering, BVH build, kernel source generation and the hiprtc compile of the specialised kernel
    if (jit) {
        char log[4096] = {0};
        const rrte_status st = rrte_hip_jit_check(&ir, (int)p.mode, log, sizeof log);
        CHECK(st == RRTE_OK, "%s: jit_check %d: %s", name, (int)st, log);
    }
    std::printf("%s %ux%u mode %u: ok (shadow rays %llu)\n", name, w, h, p.mode, (unsigned long long)sa);
}

int main() {
    // error paths of the ABI and the mirror (no device needed)
    CHECK(rrte_hip_sdf_guards(nullptr, 1, 2, nullptr, nullptr) == RRTE_INVALID_ARG, "sdf_guards null");
    {
        rrte_sdf_node bad[2] = {};
        bad[0].op = RRTE_SDF_UNION;  // pops two values from an empty stack
        rrte_sdf_node out[2];
        uint32_t g = 0;
        CHECK(rrte_hip_sdf_guards(bad, 2, 2, out, &g) == RRTE_UNSUPPORTED_PRIM, "malformed program accepted");
    }
    CHECK(rrte_hip_jit_check(nullptr, 1, nullptr, 0) == RRTE_INVALID_ARG, "jit_check null");
    CHECK(rrte_hip_band_rows_for_rank(1080, 16, 8, 3) == 136u, "band rows (8 full bands + the 8-row last)");
    CHECK(rrte_hip_band_rows_for_rank(1080, 16, 8, 7) == 128u, "band rows last rank");
    {
        // tile-order planning (the host code a context runs after a profile): every tile, slowest
        // first, on a 240 x 135 frame with a silhouette-like tail; the JIT cache key with and without
        // a header override
        const uint32_t tx = 240, n = 240 * 135;
        std::vector<uint32_t> costs(n), slots(n + 16);
        for (uint32_t i = 0; i < n; ++i) costs[i] = 200u + (i * 2654435761u >> 20) % 3000u + (i % 97 == 0 ? 9000u : 0u);
        uint32_t got = 0;
        CHECK(rrte_hip_tile_order_plan(costs.data(), n, tx, slots.data(), (uint32_t)slots.size(), &got) == RRTE_OK,
              "tile order plan");
        CHECK(got == n, "tile order slot count %u", got);
        CHECK(rrte_hip_tile_order_plan(costs.data(), n, tx, slots.data(), 16, &got) == RRTE_INVALID_ARG,
              "tile order plan into a small buffer");
        char k1[40], k2[40];
        CHECK(rrte_hip_jit_cache_key("src", nullptr, k1, sizeof k1) == RRTE_OK &&
                  rrte_hip_jit_cache_key("src", "hdr", k2, sizeof k2) == RRTE_OK && strcmp(k1, k2) != 0,
              "jit cache key");
    }
    {
        // SceneIR dump / load (scene_io.hip): a mirror-lowered scene round trip, and a truncated file
        const auto sc = rrte_examples::by_name("kitchen-sink", 32, 24, Mode::LambertShadow);
        const LoweredScene ls(sc.objects, sc.lights, sc.camera);
        const rrte_render_params p = sc.config.lower();
        const char* path = "/tmp/rrte_sanitize_scene.rrtesir";
        CHECK(rrte_hip_scene_dump(&ls.ir(), &p, path) == RRTE_OK, "scene dump");
        rrte_scene_ir ir{};
        rrte_render_params q{};
        void* storage = nullptr;
        CHECK(rrte_hip_scene_load(path, &ir, &q, &storage) == RRTE_OK, "scene load");
        CHECK(ir.num_prims == ls.ir().num_prims && ir.num_sdf_nodes == ls.ir().num_sdf_nodes &&
                  !memcmp(ir.prims, ls.ir().prims, sizeof(rrte_prim) * ir.num_prims) && !memcmp(&q, &p, sizeof p),
              "scene round trip");
        rrte_hip_scene_free(storage);
        if (FILE* f = std::fopen(path, "r+b")) {  // truncate: refused, nothing allocated
            std::fseek(f, 0, SEEK_END);
            const long n = std::ftell(f);
            std::fclose(f);
            (void)!truncate(path, n - 3);
        }
        storage = nullptr;
        CHECK(rrte_hip_scene_load(path, &ir, &q, &storage) == RRTE_INVALID_ARG && storage == nullptr,
              "truncated dump refused");
        std::remove(path);
    }
    try {
        twist(Vec3(1.0f, 1.0f, 0.0f), 1.0f);
        CHECK(false, "non-axis deformer accepted");
    } catch (const Error&) {
    }
    const bool jit = std::getenv("RRTE_SANITIZE_JIT") == nullptr || std::strcmp(std::getenv("RRTE_SANITIZE_JIT"), "0");
    for (Mode m : {Mode::LambertShadow, Mode::RefCompat}) {
        run_scene("basic-demo", 64, 48, m, jit && m == Mode::LambertShadow);
        run_scene("advanced-demo", 64, 36, m, false);
        run_scene("sdf-showcase", 64, 36, m, jit && m == Mode::LambertShadow);
        run_scene("kitchen-sink", 48, 32, m, jit && m == Mode::LambertShadow);
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "sanitize_driver: all checks passed", failures);
    return failures ? 1 : 0;
}
