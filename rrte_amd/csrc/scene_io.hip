// scene_io.hip — SceneIR dump / load for repro (SURVEY §5 "SceneIR dump/load"): one frame's lowered
// scene and render parameters in a self-checking binary file, so a frame that misbehaves on the device
// can be replayed bit for bit -- on the GPU through rrte_hip_render*, or on the CPU oracle
// (tests/test_scene_io.py).  Host code only.
//
// File layout (little endian, no padding between fields):
//   magic "RRTESIR\0" | u32 format version (1) | u32 ABI version (RRTE_ABI_VERSION) |
//   u32 sizeof(rrte_prim), sizeof(rrte_material), sizeof(rrte_light), sizeof(rrte_sdf_node),
//       sizeof(rrte_camera), sizeof(rrte_render_params), sizeof(rrte_mesh_vertex) |
//   u32 num_prims, num_materials, num_lights, num_sdf_nodes, num_mesh_vertices, num_mesh_indices |
//   u64 mesh_version | camera | params | prims | materials | lights | sdf_nodes | mesh vertices |
//   mesh indices | u64 FNV-1a of every byte before it.
// Environment: RRTE_DUMP_SCENE=<path> makes every render entry point dump the frame it was given
// before rendering it (rrte_hip.hip, dump_if_asked), overwriting the file atomically, so the last
// frame of a process that fails is on disk.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/rrte_hip.h"

namespace {

constexpr char kMagic[8] = {'R', 'R', 'T', 'E', 'S', 'I', 'R', '\0'};
constexpr uint32_t kFormat = 1;

uint64_t fnv1a64(const unsigned char* p, size_t n, uint64_t h = 1469598103934665603ull) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

struct Writer {
    std::vector<unsigned char> b;
    void put(const void* p, size_t n) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        b.insert(b.end(), c, c + n);
    }
    void u32(uint32_t v) { put(&v, 4); }
};

struct Reader {
    const unsigned char* p;
    size_t n, at = 0;
    bool get(void* out, size_t k) {
        if (k > n - at) return false;
        memcpy(out, p + at, k);
        at += k;
        return true;
    }
    bool u32(uint32_t& v) { return get(&v, 4); }
};

// The storage a loaded scene points into (rrte_hip_scene_load / rrte_hip_scene_free).
struct Loaded {
    std::vector<rrte_prim> prims;
    std::vector<rrte_material> mats;
    std::vector<rrte_light> lights;
    std::vector<rrte_sdf_node> nodes;
    std::vector<rrte_mesh_vertex> verts;
    std::vector<uint32_t> idx;
};

const uint32_t kSizes[7] = {sizeof(rrte_prim), sizeof(rrte_material), sizeof(rrte_light), sizeof(rrte_sdf_node),
                            sizeof(rrte_camera), sizeof(rrte_render_params), sizeof(rrte_mesh_vertex)};

}  // namespace

extern "C" {

rrte_status rrte_hip_scene_dump(const rrte_scene_ir* s, const rrte_render_params* p, const char* path) {
    if (!s || !p || !path) return RRTE_INVALID_ARG;
    if ((s->num_prims && !s->prims) || (s->num_materials && !s->materials) || (s->num_lights && !s->lights) ||
        (s->num_sdf_nodes && !s->sdf_nodes) || (s->num_mesh_vertices && !s->mesh_vertices) ||
        (s->num_mesh_indices && !s->mesh_indices))
        return RRTE_INVALID_ARG;
    Writer w;
    w.put(kMagic, sizeof kMagic);
    w.u32(kFormat);
    w.u32(RRTE_ABI_VERSION);
    for (uint32_t v : kSizes) w.u32(v);
    const uint32_t counts[6] = {s->num_prims, s->num_materials, s->num_lights, s->num_sdf_nodes, s->num_mesh_vertices,
                                s->num_mesh_indices};
    for (uint32_t v : counts) w.u32(v);
    w.put(&s->mesh_version, 8);
    w.put(&s->camera, sizeof s->camera);
    w.put(p, sizeof *p);
    w.put(s->prims, sizeof(rrte_prim) * s->num_prims);
    w.put(s->materials, sizeof(rrte_material) * s->num_materials);
    w.put(s->lights, sizeof(rrte_light) * s->num_lights);
    w.put(s->sdf_nodes, sizeof(rrte_sdf_node) * s->num_sdf_nodes);
    w.put(s->mesh_vertices, sizeof(rrte_mesh_vertex) * s->num_mesh_vertices);
    w.put(s->mesh_indices, sizeof(uint32_t) * s->num_mesh_indices);
    const uint64_t h = fnv1a64(w.b.data(), w.b.size());
    w.put(&h, 8);
    // written under a temporary name and renamed: a reader (or a crash) never sees half a file
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return RRTE_INVALID_ARG;
    const bool ok = fwrite(w.b.data(), 1, w.b.size(), f) == w.b.size();
    if (fclose(f) != 0 || !ok || rename(tmp.c_str(), path) != 0) {
        remove(tmp.c_str());
        return RRTE_INVALID_ARG;
    }
    return RRTE_OK;
}

rrte_status rrte_hip_scene_load(const char* path, rrte_scene_ir* s, rrte_render_params* p, void** storage) {
    if (!path || !s || !p || !storage) return RRTE_INVALID_ARG;
    *storage = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return RRTE_INVALID_ARG;
    std::vector<unsigned char> b;
    unsigned char buf[1 << 16];
    for (size_t k; (k = fread(buf, 1, sizeof buf, f)) > 0;) b.insert(b.end(), buf, buf + k);
    fclose(f);
    if (b.size() < sizeof kMagic + 8 || memcmp(b.data(), kMagic, sizeof kMagic) != 0) return RRTE_INVALID_ARG;
    uint64_t h = 0;
    memcpy(&h, b.data() + b.size() - 8, 8);
    if (fnv1a64(b.data(), b.size() - 8) != h) return RRTE_INVALID_ARG;  // truncated or altered
    Reader r{b.data() + sizeof kMagic, b.size() - sizeof kMagic - 8};
    uint32_t fmt = 0, abi = 0, sizes[7] = {}, counts[6] = {};
    if (!r.u32(fmt) || !r.u32(abi) || fmt != kFormat || abi != RRTE_ABI_VERSION) return RRTE_INVALID_ARG;
    for (uint32_t& v : sizes)
        if (!r.u32(v)) return RRTE_INVALID_ARG;
    if (memcmp(sizes, kSizes, sizeof kSizes) != 0) return RRTE_INVALID_ARG;  // another record layout
    for (uint32_t& v : counts)
        if (!r.u32(v)) return RRTE_INVALID_ARG;
    Loaded* L = new Loaded;
    L->prims.resize(counts[0]);
    L->mats.resize(counts[1]);
    L->lights.resize(counts[2]);
    L->nodes.resize(counts[3]);
    L->verts.resize(counts[4]);
    L->idx.resize(counts[5]);
    rrte_scene_ir ir{};
    const bool ok = r.get(&ir.mesh_version, 8) && r.get(&ir.camera, sizeof ir.camera) && r.get(p, sizeof *p) &&
                    r.get(L->prims.data(), sizeof(rrte_prim) * counts[0]) &&
                    r.get(L->mats.data(), sizeof(rrte_material) * counts[1]) &&
                    r.get(L->lights.data(), sizeof(rrte_light) * counts[2]) &&
                    r.get(L->nodes.data(), sizeof(rrte_sdf_node) * counts[3]) &&
                    r.get(L->verts.data(), sizeof(rrte_mesh_vertex) * counts[4]) &&
                    r.get(L->idx.data(), sizeof(uint32_t) * counts[5]) && r.at == r.n;
    if (!ok) {
        delete L;
        return RRTE_INVALID_ARG;
    }
    ir.prims = L->prims.data();
    ir.num_prims = counts[0];
    ir.materials = L->mats.data();
    ir.num_materials = counts[1];
    ir.lights = L->lights.data();
    ir.num_lights = counts[2];
    ir.sdf_nodes = L->nodes.data();
    ir.num_sdf_nodes = counts[3];
    ir.mesh_vertices = L->verts.data();
    ir.num_mesh_vertices = counts[4];
    ir.mesh_indices = L->idx.data();
    ir.num_mesh_indices = counts[5];
    *s = ir;
    *storage = L;
    return RRTE_OK;
}

void rrte_hip_scene_free(void* storage) { delete static_cast<Loaded*>(storage); }

}  // extern "C"
