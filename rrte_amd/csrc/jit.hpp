// jit.hpp — scene-specialised kernel compilation (see jit.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "device_scene.hpp"

namespace rrte {

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
    double compile_ms = 0.0;
    size_t code_bytes = 0;
    bool from_cache = false;
    bool topology = false;  // a topology kernel (jit_source with JitTopo)
};

// The host's structural decisions for a TOPOLOGY kernel (ray_kernels.hpp TopoPrim / TopoLight):
// per object, whether its SDF program is convex (sdf_convex); per light, whether shadow culling may
// cull for it (light_record_cullable).
struct JitTopo {
    std::vector<uint8_t> convex;    // one per object
    std::vector<uint8_t> cullable;  // one per light
};

// HIP source for one scene + shading mode and an extern "C" rrte_jit_kernel instantiating
// ray_kernel_body<mode, Scene, single, cull> (single: one sample, one bounce -> straight-line code;
// else runtime sample/bounce loops).  topo == nullptr: a FULL kernel, the whole scene as static
// constexpr arrays.  Otherwise a TOPOLOGY kernel: only the structure is compiled in and the values
// come from the uploaded records (kernel argument rrte::SceneValues); its source -- and so its code
// object -- depends on the scene's topology only (jit_topology_key).
std::string jit_source(const DPrim* prims, uint32_t np, const DMaterial* mats, uint32_t nm, const DLight* lights,
                       uint32_t nl, const rrte_sdf_node* nodes, uint32_t nn, int mode, bool cull, bool single,
                       const JitTopo* topo = nullptr);

// A compiled code object (hiprtc only: no device API, safe on a background thread).
struct JitCode {
    bool ok = false;
    std::vector<char> code;
    std::string log;
    double compile_ms = 0.0;
    bool from_cache = false;  // loaded from the persistent code-object cache (jit.hip)
};
JitCode jit_compile_code(const std::string& src);  // compiles are serialised internally

// Load a compiled code object on the current device.
bool jit_load(const JitCode& jc, JitKernel& out, std::string& log);

// hiprtc compile for gfx950 + module load.  On failure `log` holds the reason.
bool jit_compile(const std::string& src, JitKernel& out, std::string& log);

void jit_release(JitKernel& k);

// hiprtc compile only (no module load, no device needed): diagnostics / CPU tests.
bool jit_compile_only(const std::string& src, std::string& log);

// The persistent cache's file name for `src` (32 hex digits): a hash of the source, the embedded
// device headers (or `hdr_override` in their place, tests), the hiprtc options and version.
std::string jit_cache_name(const std::string& src, const char* hdr_override);

}  // namespace rrte
