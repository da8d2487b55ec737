// cpp_mirror_tool — drives the C++ mirror for tests/test_cpp_mirror.py.
//   cpp_mirror_tool ir <scene> <w> <h> <mode> <out.bin>       lowered IR bytes + render params (no GPU)
//   cpp_mirror_tool render <scene> <w> <h> <mode> <out.bin>    Raytracer::render_f32(linear): u8 then f32 (GPU)
//   cpp_mirror_tool engine <scene> <w> <h> <mode> <out.bin> [frames]
//                                                              Engine::render_frame's loop: one reused
//                                                              buffer through Raytracer::render_into (pinned
//                                                              once); every frame compared with render();
//                                                              the last frame written; ms per frame printed (GPU)
//   cpp_mirror_tool errors                                     error behaviour checks (no GPU needed)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>

#include "../../rrte_amd/cpp/examples.hpp"

using namespace rrte_renderer;

static Mode parse_mode(const char* m) { return std::strcmp(m, "refcompat") == 0 ? Mode::RefCompat : Mode::LambertShadow; }

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string cmd = argv[1];
    try {
        if (cmd == "errors") {
            int bad = 0;
            try {  // deformer axes must be coordinate axes
                twist(Vec3(1.0f, 1.0f, 0.0f), 1.0f);
                bad |= 1;
            } catch (const Error& e) {
                if (e.status != RRTE_UNSUPPORTED_PRIM) bad |= 2;
            }
            try {
                Mesh m({0.0f, 0.0f, 0.0f}, {0u, 1u, 2u});
                bad |= 4;
            } catch (const Error& e) {
                if (e.status != RRTE_INVALID_ARG) bad |= 8;
            }
            try {
                noise(1.0f, 1.0f, rrte_math::ZERO, 0u, RRTE_SDF_MAX_OCTAVES + 1u);
                bad |= 16;
            } catch (const Error&) {
            }
            std::printf("errors %d\n", bad);
            return bad ? 1 : 0;
        }
        if (argc < 7) return 2;
        const auto sc = rrte_examples::by_name(argv[2], (uint32_t)std::atoi(argv[3]), (uint32_t)std::atoi(argv[4]),
                                               parse_mode(argv[5]));
        std::ofstream out(argv[6], std::ios::binary);
        if (cmd == "ir") {
            const LoweredScene ls(sc.objects, sc.lights, sc.camera);
            const auto b = ls.bytes();
            const rrte_render_params p = sc.config.lower();
            out.write(reinterpret_cast<const char*>(b.data()), (std::streamsize)b.size());
            out.write(reinterpret_cast<const char*>(&p), sizeof p);
            return 0;
        }
        if (cmd == "render") {
            Raytracer rt(sc.config, 0);
            const auto u8 = rt.render(sc.objects, sc.lights, {}, sc.camera);
            const auto pr = rt.render_f32(sc.objects, sc.lights, sc.camera, /*linear=*/true);
            out.write(reinterpret_cast<const char*>(u8.data()), (std::streamsize)u8.size());
            out.write(reinterpret_cast<const char*>(pr.second.data()), (std::streamsize)(pr.second.size() * 4));
            const rrte_stats st = rt.stats();
            std::printf("shadow_rays %llu\n", (unsigned long long)st.shadow_rays);
            return 0;
        }
        if (cmd == "engine") {
            const int frames = argc > 7 ? std::atoi(argv[7]) : 20;
            Raytracer rt(sc.config, 0);
            const auto want = rt.render(sc.objects, sc.lights, {}, sc.camera);
            std::vector<uint8_t> frame_buffer(16, 7);  // the engine's buffer (resized on the first frame)
            int mismatched = 0;
            // warm-up: the library's default JIT policy (AUTO) moves to the scene-specialised kernel once
            // its background compile (or code-object cache load) lands
            // (and past the launch shape's first frames: its tile profile, the worker's slowest-first list
            // and that list's first upload -- one-time work of a new shape)
            // (bounded by time, not frames: on a cold code-object cache the compile takes ~1-2 s)
            // then 20 more frames: the new kernel is a new launch shape for the tile order (its profile,
            // the worker's list and that list's upload land over the next few frames)
            const auto w0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 20 || (!rt.stats().jit_active &&
                                       std::chrono::steady_clock::now() - w0 < std::chrono::seconds(20)); ++i)
                rt.render_into(sc.objects, sc.lights, {}, sc.camera, frame_buffer);
            for (int i = 0; i < 20; ++i) rt.render_into(sc.objects, sc.lights, {}, sc.camera, frame_buffer);
            mismatched += frame_buffer != want;  // (the last warm-up frame; the compares stay out of the timing)
            std::fill(frame_buffer.begin(), frame_buffer.end(), (uint8_t)7);
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < frames; ++i) rt.render_into(sc.objects, sc.lights, {}, sc.camera, frame_buffer);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            mismatched += frame_buffer != want;
            const rrte_stats lst = rt.stats();
            std::printf("engine_loop_last_frame upload_ms %.4f jit %u frames %llu\n", lst.upload_ms, lst.jit_active,
                        (unsigned long long)lst.frames);
            out.write(reinterpret_cast<const char*>(frame_buffer.data()), (std::streamsize)frame_buffer.size());
            // of which: lowering the scene objects to the IR each frame (LoweredScene, host only)
            const auto l0 = std::chrono::steady_clock::now();
            size_t sink = 0;
            for (int i = 0; i < frames; ++i) sink += LoweredScene(sc.objects, sc.lights, sc.camera).ir().num_prims;
            const double lms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - l0).count();
            // diagnostics: the same frames through the C ABI with the scene lowered once
            const LoweredScene once(sc.objects, sc.lights, sc.camera);
            const rrte_render_params prm = sc.config.lower();
            const auto c0 = std::chrono::steady_clock::now();
            for (int i = 0; i < frames; ++i) rt.render_raw(once.ir(), prm, frame_buffer.data());
            const double cms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
            std::printf("abi_same_buffer_ms_per_frame %.4f\n", cms / frames);
            const rrte_stats est = rt.stats();
            std::printf("engine_loop_ms_per_frame %.4f mismatched %d lower_ms_per_frame %.4f (%zu) jit %u kernel_ms %.4f\n",
                        ms / frames, mismatched, lms / frames, sink, est.jit_active, est.kernel_ms);
            return mismatched ? 1 : 0;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 2;
}
