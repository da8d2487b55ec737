// bvh.hip — host-side BVH build for triangle meshes (RRTE_PRIM_MESH).
//
// A mesh is defined as the Vec<Triangle> it stands for (include/rrte_hip.h): closest hit over
// its triangles in index order.  The device finds the same hit through a BVH: binned-SAH build
// (16 bins per axis, leaves of <= 4 triangles; index-median splits below depth 20, depth < 32 =
// the device stack), one 64-byte record per interior node holding BOTH children's boxes and links
// (the traversal tests the two children together and descends into the nearer), boxes inflated
// so that a triangle's Moller-Trumbore hit point -- which f32 rounding can put marginally outside
// the triangle -- always lies inside every box on its path, and ties broken by the original index.  Triangles are stored in leaf order with
// e1 = v1 - v0 and e2 = v2 - v0 precomputed (the same f32 subtractions the test performs).
#include "bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace rrte {
namespace {

constexpr int kBins = 16;
constexpr uint32_t kLeafMax = 4;

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const {
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = std::max(0.0f, hi[k] - lo[k]);
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct BTri {
    Box box;
    float c[3];
    uint32_t orig;
};

// Links: interior record index (bit 31 clear), or a leaf: bit 31 set, triangle count - 1 in bits
// 24-30 (1..128 triangles), first triangle slot (mesh-local) in bits 0-23.
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kSahDepth = 20;     // SAH splits above this depth, index-median splits below
constexpr uint32_t kMaxDepth = 31;     // < kMeshStack (32) in ray_kernels.hpp
constexpr uint32_t kBigLeaf = 128;

struct Builder {
    std::vector<BTri>& t;
    struct Rec { Box b[2]; uint32_t link[2]; uint32_t axis; };
    std::vector<Rec> recs;
    uint32_t depth_max = 0;
    bool too_deep = false;

    explicit Builder(std::vector<BTri>& tris) : t(tris) {}

    // Inflation: 1 % of the leaf's extent plus a relative term on its coordinates.
    static Box inflate(Box b) {
        float ext = 0.0f, mag = 0.0f;
        for (int k = 0; k < 3; ++k) {
            ext = std::max(ext, b.hi[k] - b.lo[k]);
            mag = std::max(mag, std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k])));
        }
        const float d = 1e-2f * ext + 1e-5f * mag + 1e-6f;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = std::nextafter(b.lo[k] - d, -INFINITY);
            b.hi[k] = std::nextafter(b.hi[k] + d, INFINITY);
        }
        return b;
    }

    // Builds the subtree over t[b, e); returns its link and (inflated) box.
    std::pair<uint32_t, Box> build(uint32_t b, uint32_t e, uint32_t depth) {
        depth_max = std::max(depth_max, depth);
        Box cb, nb;
        for (uint32_t i = b; i < e; ++i) {
            cb.grow(t[i].c);
            nb.grow(t[i].box);
        }
        const uint32_t n = e - b;
        if (n <= kLeafMax || (depth >= kMaxDepth && n <= kBigLeaf)) return {kLeafBit | ((n - 1) << 24) | b, inflate(nb)};
        if (depth >= kMaxDepth) {  // cannot happen for SAH-then-median trees below 2^24 triangles
            too_deep = true;
            return {kLeafBit | ((kBigLeaf - 1) << 24) | b, inflate(nb)};
        }
        int axis = -1, best_bin = -1;
        if (depth < kSahDepth) {  // binned SAH
            float best_cost = INFINITY;
            for (int ax = 0; ax < 3; ++ax) {
                const float lo = cb.lo[ax], ext = cb.hi[ax] - cb.lo[ax];
                if (!(ext > 0.0f)) continue;
                Box bb[kBins];
                uint32_t cnt[kBins] = {};
                for (uint32_t i = b; i < e; ++i) {
                    int k = (int)((t[i].c[ax] - lo) / ext * kBins);
                    k = std::min(std::max(k, 0), kBins - 1);
                    bb[k].grow(t[i].box);
                    ++cnt[k];
                }
                Box left[kBins];
                uint32_t lc[kBins];
                Box acc;
                uint32_t ac = 0;
                for (int k = 0; k < kBins; ++k) {
                    acc.grow(bb[k]);
                    ac += cnt[k];
                    left[k] = acc;
                    lc[k] = ac;
                }
                Box racc;
                uint32_t rc = 0;
                for (int k = kBins - 1; k > 0; --k) {
                    racc.grow(bb[k]);
                    rc += cnt[k];
                    const uint32_t l = lc[k - 1];
                    if (l == 0 || rc == 0) continue;
                    const float cost = left[k - 1].area() * (float)l + racc.area() * (float)rc;
                    if (cost < best_cost) {
                        best_cost = cost;
                        axis = ax;
                        best_bin = k;
                    }
                }
            }
        }
        uint32_t mid = b + n / 2;
        if (axis >= 0) {
            const float lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
            auto it = std::partition(t.begin() + b, t.begin() + e, [&](const BTri& x) {
                int k = (int)((x.c[axis] - lo) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                return k < best_bin;
            });
            mid = (uint32_t)(it - t.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        } else {  // index-median split along the widest centroid axis
            axis = 0;
            for (int ax = 1; ax < 3; ++ax)
                if (cb.hi[ax] - cb.lo[ax] > cb.hi[axis] - cb.lo[axis]) axis = ax;
            std::nth_element(t.begin() + b, t.begin() + mid, t.begin() + e,
                             [&](const BTri& x, const BTri& y) { return x.c[axis] < y.c[axis]; });
        }
        const uint32_t r = (uint32_t)recs.size();
        recs.emplace_back();
        auto L = build(b, mid, depth + 1);
        auto R = build(mid, e, depth + 1);
        Rec& rec = recs[r];
        rec.b[0] = L.second;
        rec.b[1] = R.second;
        rec.link[0] = L.first;
        rec.link[1] = R.first;
        rec.axis = (uint32_t)axis;
        Box u = L.second;
        u.grow(R.second);
        return {r, u};
    }
};

inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
inline float bits_f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

}  // namespace

void build_mesh_bvhs(const rrte_scene_ir* s, DPrim* prims, MeshData& out, float4* bounds) {
    for (uint32_t pi = 0; pi < s->num_prims; ++pi) {
        const rrte_prim& in = s->prims[pi];
        if (in.kind != RRTE_PRIM_MESH) continue;
        const uint32_t ntri = in.sdf_count;
        const uint32_t* ix = s->mesh_indices + (size_t)in.sdf_first * 3;
        const rrte_mesh_vertex* vx = s->mesh_vertices;
        std::vector<BTri> tris(ntri);
        for (uint32_t k = 0; k < ntri; ++k) {
            BTri& bt = tris[k];
            for (int j = 0; j < 3; ++j) bt.box.grow(vx[ix[3 * k + j]].position);
            for (int a = 0; a < 3; ++a) bt.c[a] = 0.5f * (bt.box.lo[a] + bt.box.hi[a]);
            bt.orig = k;
        }
        const uint32_t rec_base = (uint32_t)(out.nodes.size() / 4);
        const uint32_t slot_base = (uint32_t)(out.tris.size() / 3);
        Builder bd(tris);
        std::pair<uint32_t, Box> root{kLeafBit, Box()};  // empty mesh: a leaf with no triangles (count field unused)
        if (ntri) root = bd.build(0, ntri, 0);
        out.max_depth = std::max(out.max_depth, bd.depth_max);
        out.too_deep = out.too_deep || bd.too_deep;
        // globalise links: interior -> rec_base + r; leaf -> slot_base + first
        auto glob = [&](uint32_t link) { return (link & kLeafBit) ? link + slot_base : link + rec_base; };
        for (const auto& rc : bd.recs) {
            // record: child 0 box (w = child 0 link), child 1 box (w = child 1 link), 4 x float4
            out.nodes.push_back(f4(rc.b[0].lo[0], rc.b[0].lo[1], rc.b[0].lo[2], bits_f(glob(rc.link[0]))));
            out.nodes.push_back(f4(rc.b[0].hi[0], rc.b[0].hi[1], rc.b[0].hi[2], bits_f(rc.axis)));
            out.nodes.push_back(f4(rc.b[1].lo[0], rc.b[1].lo[1], rc.b[1].lo[2], bits_f(glob(rc.link[1]))));
            out.nodes.push_back(f4(rc.b[1].hi[0], rc.b[1].hi[1], rc.b[1].hi[2], 0.0f));
        }
        out.perm.resize(slot_base + ntri);
        for (uint32_t k = 0; k < ntri; ++k) {
            const uint32_t o = tris[k].orig;
            const rrte_mesh_vertex& v0 = vx[ix[3 * o]];
            const rrte_mesh_vertex& v1 = vx[ix[3 * o + 1]];
            const rrte_mesh_vertex& v2 = vx[ix[3 * o + 2]];
            const float* p0 = v0.position;
            out.tris.push_back(f4(p0[0], p0[1], p0[2], bits_f(o)));
            out.tris.push_back(f4(v1.position[0] - p0[0], v1.position[1] - p0[1], v1.position[2] - p0[2], 0.0f));
            out.tris.push_back(f4(v2.position[0] - p0[0], v2.position[1] - p0[1], v2.position[2] - p0[2], 0.0f));
            out.norms.push_back(f4(v0.normal[0], v0.normal[1], v0.normal[2], 0.0f));
            out.norms.push_back(f4(v1.normal[0], v1.normal[1], v1.normal[2], 0.0f));
            out.norms.push_back(f4(v2.normal[0], v2.normal[1], v2.normal[2], 0.0f));
            out.perm[slot_base + o] = slot_base + k;
        }
        DPrim& d = prims[pi];
        d.sdf_first = ntri ? glob(root.first) : kLeafBit;  // root link (an empty mesh: no triangles at all)
        d.sdf_count = ntri;
        d.p[0] = (float)slot_base;
        if (bounds) {
            const Box& b = root.second;
            double c[3], r2 = 0.0;
            for (int a = 0; a < 3; ++a) {
                c[a] = 0.5 * ((double)b.lo[a] + b.hi[a]);
                const double h = 0.5 * ((double)b.hi[a] - b.lo[a]);
                r2 += h * h;
            }
            const double r = ntri ? std::sqrt(r2) * 1.001 + 1e-3 : 0.0;
            bounds[pi] = (ntri && std::isfinite(r)) ? f4((float)c[0], (float)c[1], (float)c[2], std::nextafter((float)r, INFINITY))
                                                     : f4(0.0f, 0.0f, 0.0f, ntri ? INFINITY : 0.0f);
        }
    }
}

}  // namespace rrte
