// examples.hpp — the BASELINE scenes built through the C++ mirror (ports of rrte_amd/scenes.py,
// which follows examples/*/src/main.rs), plus a scene exercising every object/light/material kind.
#pragma once

#include <string>

#include "../../include/rrte/rrte_renderer.hpp"

namespace rrte_examples {

struct Scene {
    rrte_renderer::Objects objects;
    rrte_renderer::Lights lights;
    rrte_renderer::Camera camera;
    rrte_renderer::RaytracerConfig config;
};

Scene basic_demo(uint32_t w, uint32_t h, rrte_renderer::Mode mode);     // examples/basic-demo/src/main.rs:174-257
Scene advanced_demo(uint32_t w, uint32_t h, rrte_renderer::Mode mode);  // examples/advanced-demo/src/main.rs:238-322
Scene sdf_showcase(uint32_t w, uint32_t h, rrte_renderer::Mode mode);   // sdf-showcase layout with real SDFs
Scene kitchen_sink(uint32_t w, uint32_t h, rrte_renderer::Mode mode);   // every kind (tests/test_cpp_mirror.py twin)
Scene by_name(const std::string& name, uint32_t w, uint32_t h, rrte_renderer::Mode mode);

}  // namespace rrte_examples
