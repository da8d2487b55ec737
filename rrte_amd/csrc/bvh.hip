// bvh.hip — host-side BVH build for triangle meshes (RRTE_PRIM_MESH).
//
// A mesh is defined as the Vec<Triangle> it stands for (include/rrte_hip.h): closest hit over
// its triangles in index order.  The device finds the same hit through a BVH: binned-SAH build
// (16 bins per axis, leaves of <= 4 triangles, depth < kMeshStack), children of a node stored
// next to each other, node boxes inflated so that a triangle's Moller-Trumbore hit point -- which
// f32 rounding can put marginally outside the triangle -- always lies inside every box on its
// path, and ties broken by the original triangle index.  Triangles are stored in leaf order with
// e1 = v1 - v0 and e2 = v2 - v0 precomputed (the same f32 subtractions the test performs).
#include "bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace rrte {
namespace {

constexpr int kBins = 16;
constexpr uint32_t kLeafMax = 4;
constexpr uint32_t kMaxDepth = 28;  // < kMeshStack (32) in ray_kernels.hpp

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

struct Builder {
    std::vector<BTri>& t;
    std::vector<Box> boxes;       // per node (inflated), filled bottom-up
    std::vector<uint32_t> meta;   // per node: leaf count or 0x80000000 | axis
    std::vector<uint32_t> first;  // per node: first child / first triangle (local)
    uint32_t depth_max = 0;

    explicit Builder(std::vector<BTri>& tris) : t(tris) {}

    uint32_t alloc() {
        boxes.emplace_back();
        meta.push_back(0);
        first.push_back(0);
        return (uint32_t)boxes.size() - 1;
    }

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

    void build(uint32_t node, uint32_t b, uint32_t e, uint32_t depth) {
        depth_max = std::max(depth_max, depth);
        Box cb;  // centroid bounds
        Box nb;
        for (uint32_t i = b; i < e; ++i) {
            cb.grow(t[i].c);
            nb.grow(t[i].box);
        }
        const uint32_t n = e - b;
        auto make_leaf = [&]() {
            boxes[node] = inflate(nb);
            meta[node] = n;
            first[node] = b;
        };
        if (n <= kLeafMax || depth >= kMaxDepth) {
            if (n > kLeafMax && depth >= kMaxDepth) {  // depth cap: split by index into a leaf chain is not
                make_leaf();                          // possible without more depth; keep one big leaf
                return;
            }
            make_leaf();
            return;
        }
        // binned SAH
        float best_cost = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int axis = 0; axis < 3; ++axis) {
            const float lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
            if (!(ext > 0.0f)) continue;
            Box bb[kBins];
            uint32_t cnt[kBins] = {};
            for (uint32_t i = b; i < e; ++i) {
                int k = (int)((t[i].c[axis] - lo) / ext * kBins);
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
                    best_axis = axis;
                    best_bin = k;
                }
            }
        }
        uint32_t mid;
        int axis = best_axis;
        if (axis < 0) {  // all centroids coincide: split by index
            axis = 0;
            mid = b + n / 2;
        } else {
            const float lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
            auto it = std::partition(t.begin() + b, t.begin() + e, [&](const BTri& x) {
                int k = (int)((x.c[axis] - lo) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                return k < best_bin;
            });
            mid = (uint32_t)(it - t.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        const uint32_t l = alloc();
        const uint32_t r = alloc();
        (void)r;
        meta[node] = 0x80000000u | (uint32_t)axis;
        first[node] = l;
        build(l, b, mid, depth + 1);
        build(l + 1, mid, e, depth + 1);
        Box u = boxes[l];
        u.grow(boxes[l + 1]);
        boxes[node] = u;  // children are inflated already
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
        const uint32_t node_base = (uint32_t)(out.nodes.size() / 2);
        const uint32_t slot_base = (uint32_t)(out.tris.size() / 3);
        Builder bd(tris);
        const uint32_t root = bd.alloc();
        if (ntri) {
            bd.build(root, 0, ntri, 0);
        } else {
            bd.boxes[root] = Box();  // empty: a box no ray enters
            bd.meta[root] = 0;
        }
        out.max_depth = std::max(out.max_depth, bd.depth_max);
        for (size_t k = 0; k < bd.boxes.size(); ++k) {
            const Box& b = bd.boxes[k];
            const bool leaf = !(bd.meta[k] & 0x80000000u);
            const uint32_t a = leaf ? slot_base + bd.first[k] : node_base + bd.first[k];
            out.nodes.push_back(f4(b.lo[0], b.lo[1], b.lo[2], bits_f(a)));
            out.nodes.push_back(f4(b.hi[0], b.hi[1], b.hi[2], bits_f(bd.meta[k])));
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
        d.sdf_first = node_base + root;
        d.sdf_count = ntri;
        d.p[0] = (float)slot_base;
        if (bounds) {
            const Box& b = bd.boxes[root];
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
