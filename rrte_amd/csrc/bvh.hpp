// bvh.hpp — host-side BVH build for triangle meshes (RRTE_PRIM_MESH); see bvh.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/rrte_hip.h"
#include "device_scene.hpp"

namespace rrte {

// Device-ready mesh data for the whole scene (layout: MeshView in ray_kernels.hpp).
struct MeshData {
    std::vector<float4> nodes;   // 4 per interior record: child 0 box (w link), child 1 box (w link)
    std::vector<float4> tris;    // 3 per triangle slot: v0 (w = index within the mesh), e1, e2
    std::vector<float4> norms;   // 3 per triangle slot: n0, n1, n2
    std::vector<uint32_t> perm;  // mesh's first slot + original index -> slot
    uint32_t max_depth = 0;
    bool too_deep = false;       // a subtree hit the depth cap with > 128 triangles (build refused)
};

// Builds one BVH per RRTE_PRIM_MESH object of `s`, appending to `out`, and fills the mesh
// objects' DPrim: sdf_first = root link, sdf_count = triangles, p[0] = first triangle slot.
// `bounds` (one float4 per object, may be null) receives each mesh's bounding sphere.
void build_mesh_bvhs(const rrte_scene_ir* s, DPrim* prims, MeshData& out, float4* bounds);

}  // namespace rrte
