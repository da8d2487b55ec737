// ray_kernels.hpp — the per-pixel ray->scene loop for gfx950 (CDNA4).
//
// One wave64 lane per pixel, one wave per 8x8 pixel tile (rays in a wave are
// spatially coherent, so the wave-uniform object loop and the sphere-tracing
// loop diverge little), one wave per 64-thread workgroup.  Scene records are
// read with wave-uniform indices -> scalar loads into SGPRs; no MFMA (there is
// no dense contraction on this path).  Operation order mirrors the reference
// (file:line cited per function, paths relative to Melthizar/RRTE).
#pragma once

#include "device_scene.hpp"

namespace rrte {

constexpr float kInf = __builtin_huge_valf();
constexpr uint32_t kCounterShards = 256;  // shadow-ray counter shards (power of two)
constexpr uint32_t kCounterStride = 16;   // u64 per shard: one 128-B line each

// Runtime scene: device pointers + counts (the generic kernel).  A
// scene-specialised kernel (jit.cpp, hiprtc) instead passes a struct whose
// members are static constexpr arrays and counts: the same device code below
// then fully unrolls its object / node / light loops and folds every scene
// constant into the instruction stream.
// Triangle-mesh data (RRTE_PRIM_MESH), built once per scene on the host (bvh.hip).  A link is an
// interior record index (bit 31 clear) or a leaf (bit 31 set, triangle count - 1 in bits 24-30,
// first triangle slot in bits 0-23).  Interior record k = nodes[4k..4k+3]: child 0 box min (w =
// child 0 link), child 0 box max (w = split axis), child 1 box min (w = child 1 link), child 1 box
// max.  Triangle slot k = tris[3k..3k+2]: v0 (w = the triangle's index within its mesh), e1 = v1-v0,
// e2 = v2-v0; norms[3k..3k+2] = vertex normals.  perm maps (mesh's first slot + original index) ->
// slot, for the original-order scan.
struct MeshView {
    const float4* __restrict__ nodes;
    const float4* __restrict__ tris;
    const float4* __restrict__ norms;
    const uint32_t* __restrict__ perm;
};

// Scene features the generic kernel is compiled for (SceneView::kFeat): the host picks the smallest
// precompiled variant whose features cover the scene (rrte_hip.hip generic_kernel), so a scene without
// meshes, deformers or non-sphere analytic objects runs a kernel without their code -- fewer live
// registers, a higher occupancy, no traversal stack in LDS.  Spheres are always compiled in.
constexpr uint32_t kFeatMesh = 1u;      // RRTE_PRIM_MESH objects (BVH traversal, LDS stack)
constexpr uint32_t kFeatDeform = 2u;    // SDF programs with deformers (bend, twist, taper, noise, wave)
constexpr uint32_t kFeatAnalytic = 4u;  // plane, triangle, cube, cylinder, cone, capsule
constexpr uint32_t kFeatSdf = 8u;       // SDF objects
constexpr uint32_t kFeatAll = 15u;

struct SceneView {
    static constexpr bool kStatic = false;
    static constexpr bool kTopo = false;
    static constexpr uint32_t kFeat = kFeatAll;
    const DPrim* __restrict__ prims;
    const DMaterial* __restrict__ mats;
    const DLight* __restrict__ lights;
    const rrte_sdf_node* __restrict__ nodes;
    uint32_t num_prims, num_lights, num_materials;
    MeshView mesh;
};
template <uint32_t F>
struct SceneViewF : SceneView {
    static constexpr uint32_t kFeat = F;
};

// Loop over objects / lights: a plain loop for the runtime scene, compile-time
// recursion (every index a constant) for a static scene, so that the object's
// record, kind and SDF program fold into the code.
template <uint32_t V>
struct UC {
    static constexpr uint32_t value = V;
    __device__ __forceinline__ constexpr operator uint32_t() const { return V; }
};
template <uint32_t I, uint32_t N, class F>
__device__ __forceinline__ void static_for(F& f) {
    if constexpr (I < N) {
        f(UC<I>{});
        static_for<I + 1, N>(f);
    }
}
// The ten SDF leaf kinds (RRTE_SDF_SPHERE .. RRTE_SDF_ELLIPSOID) as compile-time constants.
template <class F>
__device__ __forceinline__ void static_for_leaves(F& f) {
    static_for<RRTE_SDF_SPHERE, RRTE_SDF_ELLIPSOID + 1u>(f);
}
template <class S, class F>
__device__ __forceinline__ void for_each_prim(const S& sc, F&& f) {
    if constexpr (S::kStatic) {
        static_for<0, S::num_prims>(f);
    } else {
        for (uint32_t i = 0; i < sc.num_prims; ++i) f(i);
    }
}
#ifndef RRTE_EXP_PRIM_ORDER
#define RRTE_EXP_PRIM_ORDER 0
#endif
template <uint32_t I, uint32_t N, class F>
__device__ __forceinline__ void static_for_rev(F& f) {
    if constexpr (I < N) {
        f(UC<N - 1u - I>{});
        static_for_rev<I + 1, N>(f);
    }
}
// EXPERIMENT: object order of the closest-hit (bit 0) / any-hit (bit 1) searches, reversed.
template <int BIT, class S, class F>
__device__ __forceinline__ void for_each_prim_exp(const S& sc, F&& f) {
    if constexpr (S::kStatic && (RRTE_EXP_PRIM_ORDER & BIT)) static_for_rev<0, S::num_prims>(f);
    else for_each_prim(sc, f);
}
// Scene-specialised kernels come in two kinds (jit.hip).  FULL (S::kTopo false): every scene record
// is a static constexpr array, so all scene constants fold into the code.  TOPOLOGY (S::kTopo true):
// only the scene's structure is compile-time -- object kinds, materials and SDF node ranges, node
// ops, integer arguments and CSG-guard links, light kinds, the convexity and cullability decisions
// (TopoPrim / TopoNode / TopoLight) -- while positions, sizes, matrices, colours and intensities are
// read from the uploaded scene records with wave-uniform (scalar) loads, so moving or recolouring an
// object needs no recompile.  The accessors below give both kinds the same interface.
struct TopoPrim { uint32_t kind; uint32_t sdf_first, sdf_count; bool convex; };
struct TopoNode { uint32_t op; uint32_t i[3]; };
struct TopoLight { uint32_t kind; bool cullable; };
// The uploaded records a topology kernel reads (a kernel argument).
struct SceneValues {
    const DPrim* prims;
    const DMaterial* mats;
    const DLight* lights;
    const rrte_sdf_node* nodes;
};

// A record of the uploaded scene read through the constant address space: a topology kernel's records
// are wave-uniform and read-only, but the compiler cannot prove that for plain global loads in a kernel
// that also stores (it issued them as vector loads: 0.10 -> 0.72 M VMEM reads per 1080p launch against
// the full kernel); loads from address space 4 at a uniform address are scalar loads.  Word-wise, so
// that only the words used are loaded.
template <class T>
__device__ __forceinline__ T load_uniform(const T* p) {
    static_assert(sizeof(T) % 4u == 0u, "records are whole dwords");
    typedef const __attribute__((address_space(4))) uint32_t CWord;
    CWord* w = (CWord*)p;
    T v;
    uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(T) / 4u; ++k) d[k] = w[k];
    return v;
}
struct NodeArgs { float f[12]; };

// Scene record accessors.  For a full static scene the record is copied in a
// constexpr-expression context (constexpr local): device-side copies of
// constexpr globals may be emitted as externally-initialised memory whose
// loads do not fold, while a constexpr copy always does.  For a topology scene
// the record is loaded and its structural fields replaced by their compile-time values.
template <class S>
__device__ __forceinline__ const DPrim& prim_at(const S& sc, uint32_t i) { return sc.prims[i]; }
template <class S, uint32_t I>
constexpr uint32_t prim_kind() {
    if constexpr (S::kTopo) return S::topo_prims[I].kind;
    else return S::prims[I].kind;
}
template <class S, uint32_t I>
constexpr uint32_t prim_first() {
    if constexpr (S::kTopo) return S::topo_prims[I].sdf_first;
    else return S::prims[I].sdf_first;
}
template <class S, uint32_t I>
constexpr uint32_t prim_count() {
    if constexpr (S::kTopo) return S::topo_prims[I].sdf_count;
    else return S::prims[I].sdf_count;
}
template <class S, uint32_t I>
__device__ __forceinline__ DPrim prim_at(const S& sc, UC<I>) {
    if constexpr (S::kTopo) {
        constexpr TopoPrim tp = S::topo_prims[I];
        DPrim v = load_uniform(sc.prims + I);
        v.kind = tp.kind;
        v.sdf_first = tp.sdf_first;
        v.sdf_count = tp.sdf_count;
        return v;
    } else {
        constexpr DPrim v = S::prims[I];
        return v;
    }
}
template <class S>
__device__ __forceinline__ const DLight& light_at(const S& sc, uint32_t i) { return sc.lights[i]; }
template <class S, uint32_t I>
constexpr uint32_t light_kind() {
    if constexpr (S::kTopo) return S::topo_lights[I].kind;
    else return S::lights[I].kind;
}
template <class S, uint32_t I>
__device__ __forceinline__ DLight light_at(const S& sc, UC<I>) {
    if constexpr (S::kTopo) {
        DLight v = load_uniform(sc.lights + I);
        v.kind = light_kind<S, I>();
        return v;
    } else {
        constexpr DLight v = S::lights[I];
        return v;
    }
}

template <class S, class F>
__device__ __forceinline__ void for_each_light(const S& sc, F&& f) {
    if constexpr (S::kStatic) {
        static_for<0, S::num_lights>(f);
    } else {
#pragma unroll 1
        for (uint32_t i = 0; i < sc.num_lights; ++i) f(i);
    }
}

// ------------------------------------------------------------- SDF program
// The SDF evaluation is templated on its guard policy G (device_scene.hpp: GuardNow / GuardDefer /
// GuardSlow) for its square roots and constant divides; every policy returns the same bits.
template <class G>
__device__ __forceinline__ float len2f(G& g, float a, float b) { return g.sqrt(a * a + b * b); }
template <class G>
__device__ __forceinline__ float len3f(G& g, float a, float b, float c) { return g.sqrt((a * a + b * b) + c * c); }

template <class G>
__device__ __forceinline__ float sdf_leaf(G& g, uint32_t op, const float* __restrict__ f, f3 p) {
    f3 q = vsub(p, V(f[0], f[1], f[2]));
    switch (op) {
    case RRTE_SDF_SPHERE:
        return len3f(g, q.x, q.y, q.z) - f[3];
    case RRTE_SDF_BOX: {
        float dx = fabsf(q.x) - f[4] * 0.5f, dy = fabsf(q.y) - f[5] * 0.5f, dz = fabsf(q.z) - f[6] * 0.5f;
        float outside = len3f(g, smx(dx, 0.0f), smx(dy, 0.0f), smx(dz, 0.0f));
        float inside = smn(smx(dx, smx(dy, dz)), 0.0f);
        return outside + inside;
    }
    case RRTE_SDF_CYLINDER: {
        float dx = len2f(g, q.x, q.z) - f[3], dy = fabsf(q.y) - f[4] * 0.5f;
        return smn(smx(dx, dy), 0.0f) + len2f(g, smx(dx, 0.0f), smx(dy, 0.0f));
    }
    case RRTE_SDF_PRISM: {
        float a = smx(fabsf(q.x) * 0.866025f + q.y * 0.5f, -q.y) - f[5] * 0.25f;
        return smx(fabsf(q.z) - f[6] * 0.5f, a);
    }
    case RRTE_SDF_TORUS: {
        float qx = len2f(g, q.x, q.z) - f[3];
        return len2f(g, qx, q.y) - f[4];
    }
    case RRTE_SDF_TUBE: {
        float rad = len2f(g, q.x, q.z);
        float mid = (f[3] + f[4]) * 0.5f, half = (f[3] - f[4]) * 0.5f;
        float dx = fabsf(rad - mid) - half, dy = fabsf(q.y) - f[5] * 0.5f;
        return smn(smx(dx, dy), 0.0f) + len2f(g, smx(dx, 0.0f), smx(dy, 0.0f));
    }
    case RRTE_SDF_RING: {
        float qx = len2f(g, q.x, q.y) - f[3];
        return len2f(g, qx, q.z) - f[4];
    }
    case RRTE_SDF_CONE: {
        float r1 = f[3], hh = f[4] * 0.5f;
        float qx = len2f(g, q.x, q.z), qy = q.y;
        float k2x = -r1, k2y = hh * 2.0f;
        float cax = qx - smn(qx, (qy < 0.0f) ? r1 : 0.0f);
        float cay = fabsf(qy) - hh;
        float k1mqx = 0.0f - qx, k1mqy = hh - qy;
        float tnum = k1mqx * k2x + k1mqy * k2y;
        float tden = k2x * k2x + k2y * k2y;
        float t = sclamp(g.div(tnum, tden), 0.0f, 1.0f);
        float cbx = (qx - 0.0f) + k2x * t;
        float cby = (qy - hh) + k2y * t;
        float s = (cbx < 0.0f && cay < 0.0f) ? -1.0f : 1.0f;
        float da = cax * cax + cay * cay, db = cbx * cbx + cby * cby;
        return s * g.sqrt(smn(da, db));
    }
    case RRTE_SDF_CAPSULE: {
        float hh = f[4] * 0.5f;
        float y = q.y - sclamp(q.y, -hh, hh);
        return len3f(g, q.x, y, q.z) - f[3];
    }
    case RRTE_SDF_ELLIPSOID: {
        float rx = f[4], ry = f[5], rz = f[6];
        float k0 = len3f(g, g.div(q.x, rx), g.div(q.y, ry), g.div(q.z, rz));
        float k1 = len3f(g, g.div(q.x, rx * rx), g.div(q.y, ry * ry), g.div(q.z, rz * rz));
        if (!(k1 > 0.0f)) return -smn(rx, smn(ry, rz));
        return k0 * (k0 - 1.0f) / k1;
    }
    default:
        return kInf;
    }
}

// smooth_min (README.md:485-488)
template <class G>
__device__ __forceinline__ float smin(G& g, float a, float b, float k) {
    float h = sclamp(0.5f + g.div(0.5f * (b - a), k), 0.0f, 1.0f);
    float om = 1.0f - h;
    return (a * h + b * om) - (k * h) * om;
}

template <class G>
__device__ __forceinline__ f3 sdf_deform(G& g, uint32_t op, const uint32_t* __restrict__ iarg,
                                         const float* __restrict__ f, f3 p) {
    f3 c = V(f[0], f[1], f[2]);
    f3 q = vsub(p, c);
    switch (op) {
    case RRTE_SDF_TWIST:
    case RRTE_SDF_BEND: {
        uint32_t ax = iarg[0];
        uint32_t drive = (op == RRTE_SDF_TWIST) ? ax : iarg[1];
        uint32_t u = (ax + 1) % 3, w = (ax + 2) % 3;
        float s, co;
        sincos_rrte(f[3] * comp(q, drive), s, co);
        float qu = comp(q, u), qw = comp(q, w);
        q = setcomp(q, u, co * qu - s * qw);
        q = setcomp(q, w, s * qu + co * qw);
        break;
    }
    case RRTE_SDF_TAPER: {
        uint32_t ax = iarg[0];
        uint32_t u = (ax + 1) % 3, w = (ax + 2) % 3;
        float t = sclamp(g.div(comp(q, ax) + f[5] * 0.5f, f[5]), 0.0f, 1.0f);
        float s = f[3] + (f[4] - f[3]) * t;
        q = setcomp(q, u, comp(q, u) / s);
        q = setcomp(q, w, comp(q, w) / s);
        break;
    }
    case RRTE_SDF_NOISE: {
        uint32_t oct = iarg[0], seed = iarg[1];
        f3 x = vmuls(q, f[3]);
        // q += amplitude * sum_o persistence^o * noise3(x * 2^o, seed + o * 0x85ebca6b)
        float acc[3] = {0.0f, 0.0f, 0.0f};
#if defined(RRTE_ABLATE_NOISE)  // (timing only, wrong images: the noise deformer's cost, tools/stress_ab.sh)
        (void)oct; (void)seed; (void)x;
#else
        float amp = 1.0f, fr = 1.0f;
        for (uint32_t o = 0; o < oct; ++o) {
            float nv[3];
            value_noise3(x.x * fr, x.y * fr, x.z * fr, seed + o * 0x85ebca6bu, nv);
#pragma unroll
            for (int k = 0; k < 3; ++k) acc[k] = acc[k] + amp * nv[k];
            amp = amp * f[5];
            fr = fr * 2.0f;
        }
#endif
        q = V(q.x + f[4] * acc[0], q.y + f[4] * acc[1], q.z + f[4] * acc[2]);
        break;
    }
    case RRTE_SDF_WAVE: {
        uint32_t ax = iarg[0], disp = iarg[1];
        float s, co;
        sincos_rrte(f[4] * comp(q, ax), s, co);
        q = setcomp(q, disp, comp(q, disp) + f[3] * s);
        break;
    }
    default:
        break;
    }
    return vadd(q, c);
}

// One postfix node applied to the value / point stacks (leaves push a
// distance, CSG ops pop two and push one, deformers push the point and
// replace it, POP_POINT restores it).
// (op and the integer arguments separately from the float arguments: a topology kernel has the
// first two at compile time and reads the third.)
template <class G, bool DEFORM = true>
__device__ __forceinline__ void sdf_node_step(G& g, uint32_t op, const uint32_t* iargs, const float* fargs, float* vs,
                                              f3* ps, uint32_t& sp, uint32_t& pp, f3& p) {
    if (op < 32) {
        vs[sp] = sdf_leaf(g, op, fargs, p);
        ++sp;
    } else if (op < 64) {
        float b = vs[sp - 1], a = vs[sp - 2], r;
        float k = fargs[0];
        switch (op) {
        case RRTE_SDF_UNION: r = smn(a, b); break;
        case RRTE_SDF_DIFFERENCE: r = smx(a, -b); break;
        case RRTE_SDF_INTERSECTION: r = smx(a, b); break;
        case RRTE_SDF_SMOOTH_UNION: r = smin(g, a, b, k); break;
        case RRTE_SDF_SMOOTH_DIFFERENCE: r = -smin(g, -a, b, k); break;
        default: r = -smin(g, -a, -b, k); break;
        }
        sp -= 2;
        vs[sp] = r;
        ++sp;
    } else if constexpr (DEFORM) {  // (a program of a scene without deformers has none: kFeatDeform)
        if (op < 96) {
            ps[pp] = p;
            ++pp;
            p = sdf_deform(g, op, iargs, fargs, p);
        } else {
            --pp;
            p = ps[pp];
        }
    }
}

// Exact CSG early-out (host analysis: sdf_guard.hip).  g = the CSG op node whose right operand B
// starts here, a = its left operand's value (top of the value stack).  Inside the guard's range
// |p - c| in [R, smax], B >= L = lambda (|p - c| - R) (inflated bound), and when L alone decides
// the op its result is exactly a (union: b >= L >= a; difference: -b <= -L <= a; smooth union /
// difference: h computed with L is 1, so h(b) is 1 by monotone rounding, and with b >= L >= 0 the
// formula reduces to a + 0 / -(-a + 0)).  Wave-uniform: taken only when every active lane may take
// it, so the result never depends on the guard.
template <class G>
__device__ __forceinline__ bool sdf_guard(G& gp, uint32_t gop, const float* gf, float a, f3 p, float& r) {
    const float dx = p.x - gf[4], dy = p.y - gf[5], dz = p.z - gf[6];
    const float s = __builtin_amdgcn_sqrtf((dx * dx + dy * dy) + dz * dz);
    const float L = gf[8] * (s - gf[7]);
    bool ok = s >= gf[7] && s <= gf[9];
    switch (gop) {
    case RRTE_SDF_UNION:
        ok = ok && L >= a;
        r = a;
        break;
    case RRTE_SDF_DIFFERENCE:
        ok = ok && -L <= a;  // a NaN left operand fails the guard (smx(NaN, -b) is -b, not a)
        r = a;
        break;
    case RRTE_SDF_SMOOTH_UNION:
        ok = ok && sclamp(0.5f + gp.div(0.5f * (L - a), gf[0]), 0.0f, 1.0f) == 1.0f;
        r = a + 0.0f;
        break;
    default: {  // RRTE_SDF_SMOOTH_DIFFERENCE: -smin(-a, b, k)
        const float na = -a;
        ok = ok && sclamp(0.5f + gp.div(0.5f * (L - na), gf[0]), 0.0f, 1.0f) == 1.0f;
        r = -(na + 0.0f);
        break;
    }
    }
    return __all(ok);
}

// Runtime program: the program counter, op and stack pointers are
// wave-uniform (every lane runs the same program), so the stacks stay in
// registers indexed by SGPR values.  A guarded operand is skipped when its
// guard holds for the whole wave.
#ifndef RRTE_SDF_FASTPATH
#define RRTE_SDF_FASTPATH 1  // generic kernel: one-leaf / leaf-leaf-op programs off the stack machine (A/B)
#endif
template <uint32_t F = kFeatAll>
struct SdfProgramT {
    static constexpr bool kSmall = false;
    static constexpr int kPlan = 0;  // (sdf_parts_plan: no part-wise secant exit)
    const rrte_sdf_node* __restrict__ nodes;
    uint32_t count;
    template <class G>
    __device__ __forceinline__ float eval(f3 p, G& g) const {
        // The two shapes most objects have -- one leaf, or two leaves under one CSG op (no deformer,
        // no guard: guards need operands of >= 2 leaves) -- evaluate without the stack machine: no
        // per-node loop, no dynamically indexed stack, and the nodes' scalar loads do not depend on
        // a loop counter (the march loop around this call can keep them in SGPRs).  Same operations
        // in the same order as the loop below, so the same bits.
        // (the program's nodes are wave-uniform: read through load_uniform, scalar loads)
        const rrte_sdf_node n0 = load_uniform(nodes);
        const uint32_t op0 = n0.op;
        if (RRTE_SDF_FASTPATH && count == 1u && op0 < 32u) return sdf_leaf(g, op0, n0.f, p);
        const rrte_sdf_node n1 = load_uniform(nodes + (count > 1u ? 1u : 0u));
        const rrte_sdf_node n2 = load_uniform(nodes + (count > 2u ? 2u : 0u));
        if (RRTE_SDF_FASTPATH && count == 3u && op0 < 32u && n1.op < 32u && n2.op >= 32u && n2.op < 64u && n1.i[2] == 0u) {
            const float a = sdf_leaf(g, op0, n0.f, p);
            const float b = sdf_leaf(g, n1.op, n1.f, p);
            const float k = n2.f[0];
            switch (n2.op) {
            case RRTE_SDF_UNION: return smn(a, b);
            case RRTE_SDF_DIFFERENCE: return smx(a, -b);
            case RRTE_SDF_INTERSECTION: return smx(a, b);
            case RRTE_SDF_SMOOTH_UNION: return smin(g, a, b, k);
            case RRTE_SDF_SMOOTH_DIFFERENCE: return -smin(g, -a, b, k);
            default: return -smin(g, -a, -b, k);
            }
        }
        float vs[RRTE_SDF_MAX_STACK];
        f3 ps[(F & kFeatDeform) ? RRTE_SDF_MAX_POINT_STACK : 1];
        uint32_t sp = 0, pp = 0;
        for (uint32_t i = 0; i < count; ++i) {
            const rrte_sdf_node ni = load_uniform(nodes + i);
            const uint32_t link = ni.i[2];
            float r;
            if (link != 0u) {
                const rrte_sdf_node gn = load_uniform(nodes + (link - 1u));
                if (sdf_guard(g, gn.op, gn.f, vs[sp - 1], p, r)) {
                    vs[sp - 1] = r;
                    i = link - 1u;  // continue after the op
                    continue;
                }
            }
            sdf_node_step<G, (F & kFeatDeform) != 0u>(g, ni.op, ni.i, ni.f, vs, ps, sp, pp, p);
        }
        return vs[0];
    }
    __device__ __forceinline__ float operator()(f3 p) const {
        GuardNow g;
        return eval(p, g);
    }
};
using SdfProgram = SdfProgramT<kFeatAll>;

#ifndef RRTE_SDF_LEAF_DISPATCH
#define RRTE_SDF_LEAF_DISPATCH 1  // generic kernel: one-leaf objects march with a compile-time leaf kind (A/B)
#endif
// A one-leaf program of the generic kernel with its leaf kind known at compile time: the runtime
// scene dispatches on the leaf once per object (intersect_at), so the sphere-tracing loop runs that
// leaf's straight-line distance, as a scene-specialised kernel does, with only the leaf's sizes read
// (through scalar loads, hoisted out of the loop).  leaf_scale is sdf_leaf_scale of the one node.
template <uint32_t OP>
struct SdfLeafProgram {
    static constexpr bool kSmall = true;
    static constexpr int kPlan = 0;  // (sdf_parts_plan: no part-wise secant exit)
    NodeArgs a;  // the node's arguments (load_uniform)
    __device__ __forceinline__ float leaf_scale() const {
        float k = 0.0f;
#pragma unroll
        for (int j = 0; j < 7; ++j) k += a.f[j] < 0.0f ? -a.f[j] : a.f[j];
        return k;
    }
    template <class G>
    __device__ __forceinline__ float eval(f3 p, G& g) const { return sdf_leaf(g, OP, a.f, p); }
    __device__ __forceinline__ float operator()(f3 p) const {
        GuardNow g;
        return eval(p, g);
    }
};
// Leaves whose one-leaf program is convex and 1-Lipschitz whatever their sizes (sdf_convex; the cone
// only for radius and height > 0, a runtime fact, so not here): the secant early miss applies.
template <uint32_t OP>
constexpr bool leaf_convex() {
    return OP == RRTE_SDF_SPHERE || OP == RRTE_SDF_BOX || OP == RRTE_SDF_CYLINDER || OP == RRTE_SDF_PRISM ||
           OP == RRTE_SDF_CAPSULE;
}

// Is the postfix program a convex, 1-Lipschitz function of p?  Convex leaves (exact SDFs of convex
// solids -- the signed distance of a convex set is a supremum of affine functions -- and the prism's
// max of 1-Lipschitz convex terms) and intersections (max) of such; union, difference, smooth ops,
// the other leaves and every deformer are not.  Evaluated at compile time for the scene-specialised
// kernels (sdf_march CONVEX).
#ifndef RRTE_SECANT_EXIT
#define RRTE_SECANT_EXIT 2
#endif
constexpr int kSecantExit = RRTE_SECANT_EXIT;  // 0 off, 1 any-hit marches, 2 closest-hit marches too
constexpr bool sdf_convex(const rrte_sdf_node* n, uint32_t count) {
    bool st[RRTE_SDF_MAX_STACK] = {};
    uint32_t sp = 0;
    for (uint32_t i = 0; i < count; ++i) {
        const uint32_t op = n[i].op;
        if (op < 32u) {
            if (sp >= RRTE_SDF_MAX_STACK) return false;
            // (box, cylinder and capsule stay convex for any sizes: a degenerate one drops the
            // inside term; the cone formula is the exact SDF only for radius, height > 0)
            st[sp++] = op == RRTE_SDF_SPHERE || op == RRTE_SDF_BOX || op == RRTE_SDF_CYLINDER ||
                       op == RRTE_SDF_PRISM || op == RRTE_SDF_CAPSULE ||
                       (op == RRTE_SDF_CONE && n[i].f[3] > 0.0f && n[i].f[4] > 0.0f);
        } else if (op < 64u) {
            if (sp < 2u) return false;
            // max, and the smooth max -smin(-a, -b, k) = (a + b)/2 + phi(a - b) with phi(u) = k/4 + u^2/(4k)
            // for |u| <= k, |u|/2 beyond (convex, nondecreasing in a and b, 1-Lipschitz), k > 0
            const bool c = (op == RRTE_SDF_INTERSECTION || (op == RRTE_SDF_SMOOTH_INTERSECTION && n[i].f[0] > 0.0f)) &&
                           st[sp - 1] && st[sp - 2];
            sp -= 2;
            st[sp++] = c;
        } else {
            return false;  // deformers (and their point-stack pops)
        }
    }
    return sp == 1u && st[0];
}
// Scale of a program's leaves for sdf_march's error bound: max over leaves of |center|_1 + the sum
// of |size parameters| (an intersection's leaves may reach far outside the object's bound), plus
// every smooth op's |k|.
constexpr float sdf_leaf_scale(const rrte_sdf_node* n, uint32_t count) {
    float k = 0.0f, ks = 0.0f;
    for (uint32_t i = 0; i < count; ++i) {
        if (n[i].op >= 32u) {
            if (n[i].op < 64u) ks += n[i].f[0] < 0.0f ? -n[i].f[0] : n[i].f[0];
            continue;
        }
        float s = 0.0f;
        for (int j = 0; j < 7; ++j) s += n[i].f[j] < 0.0f ? -n[i].f[j] : n[i].f[j];
        k = s > k ? s : k;
    }
    return k + ks;
}

// Static program (scene-specialised kernel): nodes [FIRST, FIRST+COUNT) of a
// constexpr scene, unrolled at compile time; ops fold, stack slots become
// fixed registers.  A guarded operand [I, J) becomes a uniform branch around
// its straight-line code.
template <class S, uint32_t K>
constexpr TopoNode node_topo() {
    if constexpr (S::kTopo) return S::topo_nodes[K];
    else return TopoNode{S::nodes[K].op, {S::nodes[K].i[0], S::nodes[K].i[1], S::nodes[K].i[2]}};
}
template <class S, uint32_t FIRST, uint32_t I, uint32_t END, bool CHECK, class G>
__device__ __forceinline__ void sdf_static_range(const S& sc, G& gp, float* vs, f3* ps, uint32_t& sp, uint32_t& pp,
                                                 f3& p) {
    if constexpr (I < END) {
        constexpr TopoNode tn = node_topo<S, FIRST + I>();
        constexpr uint32_t link = tn.i[2];
        if constexpr (CHECK && link != 0u) {
            constexpr uint32_t gop = node_topo<S, FIRST + link - 1u>().op;
            float r;
            bool taken;
            if constexpr (S::kTopo) {
                const NodeArgs na = load_uniform(reinterpret_cast<const NodeArgs*>(sc.nodes[FIRST + link - 1u].f));
                taken = sdf_guard(gp, gop, na.f, vs[sp - 1], p, r);
            } else {
                constexpr rrte_sdf_node g = S::nodes[FIRST + link - 1u];
                taken = sdf_guard(gp, gop, g.f, vs[sp - 1], p, r);
            }
            if (taken) vs[sp - 1] = r;
            else sdf_static_range<S, FIRST, I, link, false>(sc, gp, vs, ps, sp, pp, p);
            sdf_static_range<S, FIRST, link, END, true>(sc, gp, vs, ps, sp, pp, p);
        } else {
            if constexpr (S::kTopo) {
                const NodeArgs na = load_uniform(reinterpret_cast<const NodeArgs*>(sc.nodes[FIRST + I].f));
                sdf_node_step(gp, tn.op, tn.i, na.f, vs, ps, sp, pp, p);
            } else {
                constexpr rrte_sdf_node n = S::nodes[FIRST + I];
                sdf_node_step(gp, n.op, n.i, n.f, vs, ps, sp, pp, p);
            }
            sdf_static_range<S, FIRST, I + 1u, END, true>(sc, gp, vs, ps, sp, pp, p);
        }
    }
}

template <class S, uint32_t FIRST, uint32_t COUNT>
struct SdfStaticProgram {
    const S& sc;
    static constexpr bool kSmall = COUNT <= 8u;
    static constexpr int kPlan = 0;
    // the secant exit's leaf scale (sdf_leaf_scale): folded for a full scene, the host's value in the
    // program's first node's spare slot f[11] for a topology scene (rrte_hip.hip upload_scene)
    __device__ __forceinline__ float leaf_scale() const {
        if constexpr (S::kTopo) {
            return load_uniform(reinterpret_cast<const NodeArgs*>(sc.nodes[FIRST].f)).f[11];
        } else {
            constexpr float k = sdf_leaf_scale(S::nodes + FIRST, COUNT);
            return k;
        }
    }
    template <class G>
    __device__ __forceinline__ float eval(f3 p, G& g) const {
        float vs[RRTE_SDF_MAX_STACK];
        f3 ps[RRTE_SDF_MAX_POINT_STACK];
        uint32_t sp = 0, pp = 0;
        sdf_static_range<S, FIRST, 0u, COUNT, true>(sc, g, vs, ps, sp, pp, p);
        return vs[0];
    }
    __device__ __forceinline__ float operator()(f3 p) const {
        GuardNow g;
        return eval(p, g);
    }
};

// Part-wise secant early miss (round 6): two convex 1-Lipschitz leaves under one CSG op whose result is
// bounded below by its parts.  f = min(a, b) (union) >= the smaller part; the smooth union
// smin(a, b, k) = a h + b (1 - h) - k h (1 - h) >= min(a, b) - k/4 for every h in [0, 1] (so whatever
// h the rounding produced); the difference max(a, -b) >= a; the smooth difference -smin(-a, b, k) >=
// max(a, -b) >= a (smin <= min; with the computed h within rounding of the exact one).  So once every
// needed part is proven to stay >= E t (+ k/4 for the smooth union) by the convex secant argument of
// sdf_march, no later step can hit.  Plans: 2 = both parts (union, smooth union), 3 = the left part
// (difference, smooth difference); 0 = none.  Three-node programs of a full scene-specialised kernel
// only (leaf, leaf, op, no CSG guard: guards need operands of >= 2 leaves); intersections of convex
// leaves are convex as a whole (sdf_convex, plan 1 there).
constexpr bool leaf_node_convex(const rrte_sdf_node& n) {
    return n.op == RRTE_SDF_SPHERE || n.op == RRTE_SDF_BOX || n.op == RRTE_SDF_CYLINDER || n.op == RRTE_SDF_PRISM ||
           n.op == RRTE_SDF_CAPSULE || (n.op == RRTE_SDF_CONE && n.f[3] > 0.0f && n.f[4] > 0.0f);
}
constexpr int sdf_parts_plan(const rrte_sdf_node* n, uint32_t count) {
    if (count != 3u || n[0].op >= 32u || n[1].op >= 32u || n[2].op < 32u || n[2].op >= 64u) return 0;
    if (n[0].i[2] != 0u || n[1].i[2] != 0u || n[2].i[2] != 0u) return 0;
    const uint32_t op = n[2].op;
    const bool smooth_ok = n[2].f[0] > 0.0f;
    if ((op == RRTE_SDF_UNION || (op == RRTE_SDF_SMOOTH_UNION && smooth_ok)) && leaf_node_convex(n[0]) &&
        leaf_node_convex(n[1]))
        return 2;
    if ((op == RRTE_SDF_DIFFERENCE || (op == RRTE_SDF_SMOOTH_DIFFERENCE && smooth_ok)) && leaf_node_convex(n[0]))
        return 3;
    return 0;
}
// Measured (tools/policy_ab.sh, two interleaved rounds, the headline): exact, a lone launch ~2 % shorter
// (0.1022-0.1044 -> 0.1003-0.1024 ms), but the frame stream ~3 % slower (20 steps 0.0670-0.0675 ->
// 0.0687-0.0696 ms, 200 steps 0.0626-0.0627 -> 0.0647-0.0654): the per-part tests on every step cost
// more issue slots than the shortened marches save (profiles/r06_parts_exit_ab.log).  Off by default;
// tests/test_gpu_parity.py keeps it exact (-DRRTE_PARTS_EXIT=1 against the plain march).
#ifndef RRTE_PARTS_EXIT
#define RRTE_PARTS_EXIT 0  // the part-wise secant exit (A/B switch)
#endif

// A full scene's three-node program (leaf A, leaf B, op) with a part-wise plan: the same operations in
// the same order as the stack machine (sdf_node_step), plus the parts' values for the march's test.
template <class S, uint32_t FIRST>
struct SdfPartsProgram {
    const S& sc;
    static constexpr bool kSmall = true;
    static constexpr int kPlan = sdf_parts_plan(S::nodes + FIRST, 3u);
    static constexpr uint32_t kOp = S::nodes[FIRST + 2].op;
    // extra margin of the parts' test: the smooth ops' rounding (<= D, see sdf_march) and the smooth
    // union's k/4
    static constexpr bool kSmooth = kOp == RRTE_SDF_SMOOTH_UNION || kOp == RRTE_SDF_SMOOTH_DIFFERENCE;
    static constexpr float kQuarterK = kOp == RRTE_SDF_SMOOTH_UNION ? S::nodes[FIRST + 2].f[0] * 0.25f : 0.0f;
    __device__ __forceinline__ float leaf_scale() const {
        constexpr float k = sdf_leaf_scale(S::nodes + FIRST, 3u);
        return k;
    }
    template <class G>
    __device__ __forceinline__ float eval_parts(f3 p, G& g, float& a, float& b) const {
        constexpr rrte_sdf_node na = S::nodes[FIRST], nb = S::nodes[FIRST + 1], no = S::nodes[FIRST + 2];
        a = sdf_leaf(g, na.op, na.f, p);
        b = sdf_leaf(g, nb.op, nb.f, p);
        const float k = no.f[0];
        if constexpr (kOp == RRTE_SDF_UNION) return smn(a, b);
        else if constexpr (kOp == RRTE_SDF_DIFFERENCE) return smx(a, -b);
        else if constexpr (kOp == RRTE_SDF_SMOOTH_UNION) return smin(g, a, b, k);
        else return -smin(g, -a, b, k);  // RRTE_SDF_SMOOTH_DIFFERENCE
    }
    template <class G>
    __device__ __forceinline__ float eval(f3 p, G& g) const {
        float a, b;
        return eval_parts(p, g, a, b);
    }
    __device__ __forceinline__ float operator()(f3 p) const {
        GuardNow g;
        return eval(p, g);
    }
};

// Exact "ray leaves the sphere" early-out for any-hit (shadow) rays: origin outside the sphere
// (cc = |oc|^2 - r^2 > 0) moving away from its centre (hb = oc.d > 0), |d|^2 >= 1/4, t_min >= 2^-57.
// Then the full test finds nothing in [t_min, t_max]: disc = RN(RN(hb^2) - RN(a cc)) <= RN(hb^2), so
// sq = RN(sqrt(disc)) <= RN(sqrt(RN(hb^2))), which is hb when hb >= 2^-60 (fl(sqrt(fl(x*x))) = |x| in
// binary f32 with round-to-nearest, no under/overflow) and <= 2^-60 otherwise; hence -hb + sq <= 2^-60,
// both roots (-hb -/+ sq)/a are <= 2^-58 < t_min, and the sphere / bounding-sphere test rejects.
// Skips the sqrt and divides of, e.g., every shadow ray's test against the ground sphere.
__device__ __forceinline__ bool leaves_sphere(float hb, float cc, float a, float t_min) {
    return hb > 0.0f && cc > 0.0f && a >= 0.25f && t_min >= 0x1p-57f;
}

// SDFObject::intersect, search part -- sphere tracing inside the object's
// bounding sphere (build-defined).  Only t is produced here;
// the closest-hit search keeps (t, object) and the hit attributes are
// computed once for the winner.  The per-lane trip count diverges; the wave
// leaves the loop when its EXEC mask drains.
//
// CONVEX (marches of objects whose SDF program is a convex, 1-Lipschitz function of p: a convex leaf
// or an intersection of such, no deformers; sdf_convex) adds an exact early miss.  Along
// the ray, f(t) = sdf(o + t d) is convex, so for t >= t_k it lies above the secant through the last
// two march points: f(t) >= f(t_k) + s (t - t_k), s = (f(t_k) - f(t_k-1)) / (t_k - t_k-1).  Every
// computed value d~ is within D of f at the exact point: D = 2^-17 (|o|_1 + tend + |c|_1 + 4 R + K),
// K = sdf_leaf_scale (the largest leaf's |center|_1 + |sizes|).  The rounding of p = o + t d moves
// p by <= 2^-24 (|o|_1 + 2t), which f (1-Lipschitz) passes on unchanged, and each leaf's evaluation
// errs by <= 24 * 2^-24 (|q| + sizes), the cone's being the longest (its clamped projection
// parameter's error times the side length stays <= 8 * 2^-24 (|q| + h)), a smooth max adds
// <= 6 * 2^-24 (|a| + |b| + k) and passes its operands' errors on unscaled; together <= 64 * 2^-24
// (...) against 2^-17 = 128 * 2^-24.  Hence if d~_k - E t_k >= 3D and (d~_k - d~_k-1) - E (t_k - t_k-1) >= 3D with
// E = eps (1 + 2^-20) >= fl(eps t) / t, every later step has d~ >= f - D >= E t >= fl(eps t): no
// later step can hit, and the march's answer is "miss" whether it ends at tend or at max_steps.  A
// NaN anywhere fails both tests.  Shadow rays leaving the object they start on exit after ~3 steps
// instead of marching out of the bound; camera and shadow rays that pass an object exit once they
// recede from it.  (A miss's t is never used, so closest-hit marches take it too.)
// Unroll factor of the sphere-tracing loops (RRTE_MARCH_UNROLL, A/B experiments through
// RRTE_JIT_EXTRA_OPTS; the per-lane exit keeps every unrolled copy exact).
#ifndef RRTE_MARCH_UNROLL
#define RRTE_MARCH_UNROLL 1
#endif
// RRTE_MARCH_PRED (A/B switch, bit-exact at every level; tools/jit_ab.sh): 0 divergent-exit march loops
// (default); 1 the predicated loop (sdf_march_loop) after the divergent bound test; 2 + a predicated
// bound test (the loop runs under the caller's EXEC); 3 + predicated shadow rays (every lane of the
// wave runs every any-hit test).  Measured on the headline (two interleaved rounds each): 1 = lone
// launch -6 %, frame stream +1.5 %; 3 = frame stream +9 %, lone launch unchanged.
#ifndef RRTE_MARCH_PRED
#define RRTE_MARCH_PRED 0
#endif
#ifndef RRTE_MARCH_PAIR
#define RRTE_MARCH_PAIR 0  // sphere-tracing loops exit every second step (A/B)
#endif
#define RRTE_PRAGMA_(x) _Pragma(#x)
#define RRTE_UNROLL_(n) RRTE_PRAGMA_(unroll n)
// One SDF evaluation with deferred guards: the short sequences for every lane, one wave-uniform test
// of the folded range checks, and the compiler's full sequences only when some lane needs them.
#ifndef RRTE_DEFER_GUARDS
#define RRTE_DEFER_GUARDS 0
#endif
template <class EVAL>
__device__ __forceinline__ float eval_deferred(const EVAL& eval, f3 p) {
#if RRTE_DEFER_GUARDS
    GuardDefer g;
    float d = eval.eval(p, g);
    const uint64_t bad = __builtin_amdgcn_ballot_w64(g.bad());
    if (__builtin_expect(bad != 0ull, 0)) {
        GuardSlow gs;
        const float ds = eval.eval(p, gs);
        d = mask_select(bad, d, ds);
    }
    return d;
#else
    return eval(p);
#endif
}

// The predicated sphere-tracing loop (RRTE_MARCH_PRED): the lanes of `live` (an SGPR lane mask) march
// from t to tend under the caller's EXEC; a lane that has stopped keeps its state through selects on
// that mask, the step counter is wave-uniform (SGPR), and the loop ends when no lane is left -- the
// same t sequence and result per lane as the divergent-exit loops of sdf_march, without their per-step
// EXEC save / restore chains on the scalar unit.
template <class EVAL, bool CONVEX>
__device__ __forceinline__ bool sdf_march_loop(const DPrim& pr, const EVAL& eval, const Ray& r, float t, float tend,
                                               uint64_t live, float& t_hit) {
    const f3 bc = V(pr.p[0], pr.p[1], pr.p[2]);
    const float br = pr.p[3];
    const float eps = pr.sdf_hit_eps, scale = pr.sdf_step_scale;
    const uint32_t steps = pr.sdf_max_steps;
    [[maybe_unused]] float E = 0.0f, D3 = 0.0f, dp = __builtin_nanf(""), tp = t;
    if constexpr (CONVEX) {
        E = eps * (1.0f + 0x1p-20f);
        const float K = eval.leaf_scale();
        D3 = 3.0f * 0x1p-17f *
             ((((fabsf(r.o.x) + fabsf(r.o.y)) + fabsf(r.o.z)) + tend) +
              ((((fabsf(bc.x) + fabsf(bc.y)) + fabsf(bc.z)) + 4.0f * br) + K));
    }
    // every condition as a wave mask (one v_cmp each, combined on the scalar unit)
    uint64_t hitm = 0ull;
    uint32_t left = steps;
    if (left != 0u) {
        for (;;) {
            const f3 p = ray_at(r, t);
            const float d = eval_deferred(eval, p);
            const float tn = t + d * scale;
            const uint64_t hm = __builtin_amdgcn_ballot_w64(d < eps * t);
            uint64_t sm = hm | __builtin_amdgcn_ballot_w64(tn > tend);
            if constexpr (CONVEX) {
                sm |= __builtin_amdgcn_ballot_w64(d - E * t >= D3) &
                      __builtin_amdgcn_ballot_w64((d - dp) - E * (t - tp) >= D3);
                dp = d;
                tp = t;
            }
            hitm |= hm & live;
            t = mask_select(live & ~hm, t, tn);
            live &= ~sm;
            left = __builtin_amdgcn_readfirstlane(left - 1u);
            if ((left == 0u) | (live == 0ull)) break;
        }
    }
    t_hit = t;
    return mask_lane(hitm);
}

template <class EVAL, bool ANY = false, bool CONVEX = false>
__device__ __forceinline__ bool sdf_march(const DPrim& pr, const EVAL& eval, const Ray& r, float t_min, float t_max,
                                          float& t_hit) {
    f3 bc = V(pr.p[0], pr.p[1], pr.p[2]);
    float br = pr.p[3];
    f3 oc = vsub(r.o, bc);
    float b = vdot(oc, r.d);
    float cc = vdot(oc, oc) - br * br;
#if RRTE_MARCH_PRED >= 2
    // Predicated bound test: no divergent early return -- every lane of the caller's EXEC computes the
    // entry and exit parameters, `enter` says whether it marches (the same decisions as the branches
    // below), and the march loop runs under the caller's EXEC with the marching lanes in `live`.
    // Lanes that do not enter get a benign t (their points stay finite, so no guard fallback runs).
    {
        const float disc = b * b - cc;
        bool enter = !(disc < 0.0f);
        if constexpr (ANY) enter = enter & !(t_max == t_max && leaves_sphere(b, cc, 1.0f, t_min));
        const float sq = sqrt_rn(disc < 0.0f ? 1.0f : disc);
        float t = mx(t_min, -b - sq);
        const float tend = mn(t_max, -b + sq);
        enter = enter & !(t > tend);
        uint64_t live = __builtin_amdgcn_ballot_w64(enter);
        if (live == 0ull) return false;
        t = enter ? t : 1.0f;
        return sdf_march_loop<EVAL, CONVEX>(pr, eval, r, t, tend, live, t_hit);
    }
#endif
    // the bound test below has no divide (roots -b -/+ sq): leaves_sphere's argument with a = 1, which
    // leaves tend = mn(t_max, -b + sq) <= 2^-60 < t_min <= t unless t_max is NaN (tend NaN marches on)
    if (ANY && t_max == t_max && leaves_sphere(b, cc, 1.0f, t_min)) return false;
    float disc = b * b - cc;
    if (disc < 0.0f) return false;
    float sq = sqrt_rn(disc);
    float t = mx(t_min, -b - sq);
    float tend = mn(t_max, -b + sq);
    if (t > tend) return false;
    const float eps = pr.sdf_hit_eps, scale = pr.sdf_step_scale;
    const uint32_t steps = pr.sdf_max_steps;
#if RRTE_MARCH_PRED == 1
    // the predicated loop under the EXEC of the lanes that passed the bound test
    return sdf_march_loop<EVAL, CONVEX>(pr, eval, r, t, tend, __builtin_amdgcn_ballot_w64(true), t_hit);
#endif
    // One divergent exit per step (hit, or the next t leaves the bound) instead of three: same
    // t sequence and result as "if (d < eps*t) hit; t += d*scale; if (t > tend) miss" (NaN
    // included).  (A fully predicated form with a wave-uniform exit was measured slower.)
    bool hit = false;
    if constexpr (EVAL::kPlan >= 2 && RRTE_PARTS_EXIT && !RRTE_MARCH_PAIR && !RRTE_DEFER_GUARDS) {
        // part-wise secant early miss (SdfPartsProgram): every needed part proven to stay above
        // E t + margin by its own secant; D as below (the parts are leaves of the same program)
        const float E = eps * (1.0f + 0x1p-20f);
        const float K = eval.leaf_scale();
        const float D = 0x1p-17f * ((((fabsf(r.o.x) + fabsf(r.o.y)) + fabsf(r.o.z)) + tend) +
                                    ((((fabsf(bc.x) + fabsf(bc.y)) + fabsf(bc.z)) + 4.0f * br) + K));
        const float D3 = 3.0f * D;
        const float D3M = EVAL::kSmooth ? (D3 + D) + EVAL::kQuarterK : D3;
        float ap = __builtin_nanf(""), bp = __builtin_nanf(""), tp = t;
RRTE_UNROLL_(RRTE_MARCH_UNROLL)
        for (uint32_t i = 0; i < steps; ++i) {
            f3 p = ray_at(r, t);
            GuardNow g;
            float a, b;
            float d = eval.eval_parts(p, g, a, b);
            hit = d < eps * t;
            const float tn = t + d * scale;
            bool safe = (a - E * t >= D3M) && ((a - ap) - E * (t - tp) >= D3);
            if constexpr (EVAL::kPlan == 2) safe = safe && (b - E * t >= D3M) && ((b - bp) - E * (t - tp) >= D3);
            const bool stop = hit || tn > tend || safe;
            ap = a;
            bp = b;
            tp = t;
            t = hit ? t : tn;
            if (stop) break;
        }
        t_hit = t;
        return hit;
    }
    if constexpr (CONVEX) {
        const float E = eps * (1.0f + 0x1p-20f);
        const float K = eval.leaf_scale();
        const float D3 = 3.0f * 0x1p-17f *
                         ((((fabsf(r.o.x) + fabsf(r.o.y)) + fabsf(r.o.z)) + tend) +
                          ((((fabsf(bc.x) + fabsf(bc.y)) + fabsf(bc.z)) + 4.0f * br) + K));
        float dp = __builtin_nanf(""), tp = t;
#if RRTE_MARCH_PAIR
        // two steps per loop exit (see below)
        for (uint32_t i = 0; i < steps; i += 2u) {
            const float dA = eval_deferred(eval, ray_at(r, t));
            const bool hitA = dA < eps * t;
            const float tnA = t + dA * scale;
            const bool stopA = hitA || tnA > tend || ((dA - E * t >= D3) && ((dA - dp) - E * (t - tp) >= D3));
            const float tA = hitA ? t : tnA;
            if (i + 1u >= steps) {  // (uniform: an odd step cap ends on a single step)
                hit = hitA;
                t = tA;
                break;
            }
            const float dB = eval_deferred(eval, ray_at(r, tA));
            const bool hitB = dB < eps * tA;
            const float tnB = tA + dB * scale;
            const bool stopB = hitB || tnB > tend || ((dB - E * tA >= D3) && ((dB - dA) - E * (tA - t) >= D3));
            hit = stopA ? hitA : hitB;
            dp = stopA ? dA : dB;
            tp = stopA ? t : tA;
            t = stopA ? tA : (hitB ? tA : tnB);
            if (stopA || stopB) break;
        }
#else
RRTE_UNROLL_(RRTE_MARCH_UNROLL)
        for (uint32_t i = 0; i < steps; ++i) {
            f3 p = ray_at(r, t);
            float d = eval_deferred(eval, p);
            hit = d < eps * t;
            const float tn = t + d * scale;
            const bool safe = (d - E * t >= D3) && ((d - dp) - E * (t - tp) >= D3);
            const bool stop = hit || tn > tend || safe;
            dp = d;
            tp = t;
            t = hit ? t : tn;
            if (stop) break;
        }
#endif
        t_hit = t;
        return hit;
    }
#if RRTE_MARCH_PAIR
    // Two march steps per loop exit: the second step runs on every lane that entered the iteration,
    // and a lane whose first step stopped keeps that step's result through selects -- the same t
    // sequence and result per lane as one exit per step, with half the divergent-exit bookkeeping on
    // the scalar unit (a wave whose last lanes stop on a first step pays one extra step).
    for (uint32_t i = 0; i < steps; i += 2u) {
        const float dA = eval_deferred(eval, ray_at(r, t));
        const bool hitA = dA < eps * t;
        const float tnA = t + dA * scale;
        const bool stopA = hitA || tnA > tend;
        const float tA = hitA ? t : tnA;
        if (i + 1u >= steps) {
            hit = hitA;
            t = tA;
            break;
        }
        const float dB = eval_deferred(eval, ray_at(r, tA));
        const bool hitB = dB < eps * tA;
        const float tnB = tA + dB * scale;
        hit = stopA ? hitA : hitB;
        t = stopA ? tA : (hitB ? tA : tnB);
        if (stopA || hitB || tnB > tend) break;
    }
    t_hit = t;
    return hit;
#endif
RRTE_UNROLL_(RRTE_MARCH_UNROLL)
    for (uint32_t i = 0; i < steps; ++i) {
        f3 p = ray_at(r, t);
        float d = eval_deferred(eval, p);
        hit = d < eps * t;
        const float tn = t + d * scale;
        const bool stop = hit || tn > tend;
        t = hit ? t : tn;
        if (stop) break;
    }
    t_hit = t;
    return hit;
}

// Hit attributes of an SDF hit at t: p = Ray::at(t) and the tetrahedral
// normal n = sum_k k_i f(p + k_i h), h = 1e-3, accumulated in the oracle's
// order: k0=(+,-,-) k1=(-,-,+) k2=(-,+,-) k3=(+,+,+).  One evaluation site.
template <class EVAL>
__device__ __forceinline__ void sdf_hit_attributes(const EVAL& eval, const Ray& r, float t, Hit& out) {
    const float h = 1e-3f;
    const f3 p = ray_at(r, t);
    auto taps = [&](auto& g) {
        f3 n = V(0.0f, 0.0f, 0.0f);
        auto tap = [&](uint32_t k) {
            bool sx = (k == 0) || (k == 3), sy = (k >= 2), sz = (k == 1) || (k == 3);
            f3 q = V(sx ? p.x + h : p.x - h, sy ? p.y + h : p.y - h, sz ? p.z + h : p.z - h);
            float d = eval.eval(q, g);
            if (k == 0) { n.x = d; n.y = -d; n.z = -d; }
            else if (k == 1) { n.x = n.x - d; n.y = n.y - d; n.z = n.z + d; }
            else if (k == 2) { n.x = n.x - d; n.y = n.y + d; n.z = n.z - d; }
            else { n.x = n.x + d; n.y = n.y + d; n.z = n.z + d; }
        };
        if constexpr (EVAL::kSmall) {
            // short programs (scene-specialised, <= 8 nodes): four straight-line taps, no per-tap selects
            // or loop control (-1.3 % per headline frame; long programs keep the loop for code size)
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) tap(k);
        } else {
#pragma unroll 1
            for (uint32_t k = 0; k < 4; ++k) tap(k);
        }
        return n;
    };
#if RRTE_DEFER_GUARDS
    // deferred guards over the four taps: one wave-uniform test, the full sequences only if needed
    GuardDefer g;
    f3 n = taps(g);
    const uint64_t bad = __builtin_amdgcn_ballot_w64(g.bad());
    if (__builtin_expect(bad != 0ull, 0)) {
        GuardSlow gs;
        const f3 ns = taps(gs);
        n = V(mask_select(bad, n.x, ns.x), mask_select(bad, n.y, ns.y), mask_select(bad, n.z, ns.z));
    }
#else
    GuardNow g;
    const f3 n = taps(g);
#endif
    hit_new(out, t, p, vnorm(n), r);
}

// ----------------------------------------------------- analytic intersectors
__device__ __forceinline__ void local_ray(const DPrim& pr, const Ray& r, Ray& lr) {
    // inverse_matrix() applied to the ray, then Ray::new (primitives.rs:303-307)
    lr = ray_new(m_point(pr.inv, r.o), vnorm(m_vector(pr.inv, r.d)));
}

// ----------------------------------------------------- analytic intersectors
// SceneObject::intersect for the seven primitive kinds (primitives.rs:57-725).
// t is always written to out.t; point/normal only matter when NEED_HIT.
template <bool NEED_HIT, bool ANY = false>
__device__ __forceinline__ bool isect_sphere(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:57-81
    f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]);
    float rad = pr.p[3];
    f3 oc = vsub(r.o, ctr);
    float a = vlen2(r.d);
    float hb = vdot(oc, r.d);
    float cc = vlen2(oc) - rad * rad;
    if (ANY && leaves_sphere(hb, cc, a, t_min)) return false;
    float disc = hb * hb - a * cc;
    if (disc < 0.0f) return false;
    float sq = sqrt_rn(disc);
    float root = (-hb - sq) / a;
    if (root < t_min || t_max < root) {
        root = (-hb + sq) / a;
        if (root < t_min || t_max < root) return false;
    }
    f3 p = ray_at(r, root);
    hit_new(out, root, p, vdivs(vsub(p, ctr), rad), r);
    return true;
}

// Hit attributes of a sphere hit found by the search at t (= the root isect_sphere returns for the same
// ray with t_max = INFINITY): the point and normal exactly as isect_sphere builds them, without
// solving the quadratic again.
__device__ __forceinline__ void sphere_attributes(const DPrim& pr, const Ray& r, float t, Hit& out) {
    const f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]);
    const f3 p = ray_at(r, t);
    hit_new(out, t, p, vdivs(vsub(p, ctr), pr.p[3]), r);
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_plane(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:133-149
    f3 pt = V(pr.p[0], pr.p[1], pr.p[2]), n = V(pr.p[4], pr.p[5], pr.p[6]);
    float denom = vdot(n, r.d);
    if (fabsf(denom) < 1e-6f) return false;
    float t = vdot(vsub(pt, r.o), n) / denom;
    if (t < t_min || t > t_max) return false;
    f3 p = ray_at(r, t);
    hit_new(out, t, p, denom < 0.0f ? n : vneg(n), r);
    return true;
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_triangle(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:208-244
    f3 v0 = V(pr.p[0], pr.p[1], pr.p[2]), v1 = V(pr.p[3], pr.p[4], pr.p[5]), v2 = V(pr.p[6], pr.p[7], pr.p[8]);
    f3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    f3 h = vcross(r.d, e2);
    float a = vdot(e1, h);
    if (a > -1e-6f && a < 1e-6f) return false;
    float f = rcp_rn(a);
    f3 s = vsub(r.o, v0);
    float u = f * vdot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    f3 q = vcross(s, e1);
    float v = f * vdot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = f * vdot(e2, q);
    if (t < t_min || t > t_max) return false;
    f3 p = ray_at(r, t);
    float w = 1.0f - u - v;
    f3 n0 = V(pr.p[9], pr.p[10], pr.p[11]), n1 = V(pr.p[12], pr.p[13], pr.p[14]),
       n2 = V(pr.p[15], pr.p[16], pr.p[17]);
    f3 n = vnorm(vadd(vadd(vmuls(n0, w), vmuls(n1, u)), vmuls(n2, v)));
    hit_new(out, t, p, n, r);
    return true;
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_cube(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:301-364
    Ray lr;
    local_ray(pr, r, lr);
    f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]), size = V(pr.p[4], pr.p[5], pr.p[6]);
    f3 half = vmuls(size, 0.5f);
    f3 mnb = vsub(ctr, half), mxb = vadd(ctr, half);
    float t_near = t_min, t_far = t_max;
    f3 normal = V(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (uint32_t i = 0; i < 3; ++i) {
        f3 axis = setcomp(V(0.0f, 0.0f, 0.0f), i, 1.0f);
        float oc = vdot(lr.o, axis), dc = vdot(lr.d, axis);
        float lo = vdot(mnb, axis), hi = vdot(mxb, axis);
        if (fabsf(dc) < 1e-6f) {
            if (oc < lo || oc > hi) return false;
        } else {
            float t1 = (lo - oc) / dc, t2 = (hi - oc) / dc;
            float tsn = t1 < t2 ? t1 : t2, tsf = t1 < t2 ? t2 : t1;
            if (tsn > t_near) {
                t_near = tsn;
                normal = t1 < t2 ? vneg(axis) : axis;
            }
            if (tsf < t_far) t_far = tsf;
            if (t_near > t_far) return false;
        }
    }
    float t = (t_near >= t_min) ? t_near : t_far;
    if (t < t_min || t > t_max) return false;
    f3 lp = ray_at(lr, t);
    hit_new(out, t, m_point(pr.xf, lp), vnorm(m_vector(pr.xf, normal)), r);
    return true;
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_cylinder(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:419-465
    Ray lr;
    local_ray(pr, r, lr);
    f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]);
    float rad = pr.p[3], hh = pr.p[4] * 0.5f;
    f3 oc = vsub(lr.o, ctr);
    float a = lr.d.x * lr.d.x + lr.d.z * lr.d.z;
    float b = 2.0f * (oc.x * lr.d.x + oc.z * lr.d.z);
    float cc = oc.x * oc.x + oc.z * oc.z - rad * rad;
    float disc = b * b - 4.0f * a * cc;
    if (disc < 0.0f) return false;
    float sq = sqrt_rn(disc);
    float ts0 = (-b - sq) / (2.0f * a), ts1 = (-b + sq) / (2.0f * a);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        float t = k == 0 ? ts0 : ts1;
        if (t >= t_min && t <= t_max) {
            f3 p = ray_at(lr, t);
            if (fabsf(p.y - ctr.y) <= hh) {
                f3 ln = V((p.x - ctr.x) / rad, 0.0f, (p.z - ctr.z) / rad);
                hit_new(out, t, m_point(pr.xf, p), vnorm(m_vector(pr.xf, ln)), r);
                return true;
            }
        }
    }
    return false;
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_cone(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:520-571
    Ray lr;
    local_ray(pr, r, lr);
    f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]);
    float rad = pr.p[3], ht = pr.p[4], hh = ht * 0.5f;
    f3 oc = vsub(lr.o, ctr);
    float k = rad / ht, k2 = k * k;
    f3 d = lr.d;
    float a = d.x * d.x + d.z * d.z - k2 * d.y * d.y;
    float b = 2.0f * (oc.x * d.x + oc.z * d.z - k2 * (oc.y - hh) * d.y);
    float cc = oc.x * oc.x + oc.z * oc.z - k2 * (oc.y - hh) * (oc.y - hh);
    float disc = b * b - 4.0f * a * cc;
    if (disc < 0.0f) return false;
    float sq = sqrt_rn(disc);
    float ts0 = (-b - sq) / (2.0f * a), ts1 = (-b + sq) / (2.0f * a);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        float t = kk == 0 ? ts0 : ts1;
        if (t >= t_min && t <= t_max) {
            f3 p = ray_at(lr, t);
            float yl = p.y - ctr.y;
            if (yl >= -hh && yl <= hh) {
                float rr = sqrt_rn(p.x * p.x + p.z * p.z);
                f3 ln = vnorm(V(p.x / rr, k, p.z / rr));
                hit_new(out, t, m_point(pr.xf, p), vnorm(m_vector(pr.xf, ln)), r);
                return true;
            }
        }
    }
    return false;
}

template <bool NEED_HIT>
__device__ __forceinline__ bool isect_capsule(const DPrim& pr, const Ray& r, float t_min, float t_max, Hit& out) {  // primitives.rs:626-725
    Ray lr;
    local_ray(pr, r, lr);
    f3 ctr = V(pr.p[0], pr.p[1], pr.p[2]);
    float rad = pr.p[3], hh = pr.p[4] * 0.5f;
    float closest = kInf;
    bool found = false;
    float a = vlen2(lr.d);
#pragma unroll
    for (int cap = 0; cap < 2; ++cap) {
        f3 cc_ = cap == 0 ? vadd(ctr, V(0.0f, hh, 0.0f)) : vsub(ctr, V(0.0f, hh, 0.0f));
        f3 oc = vsub(lr.o, cc_);
        float hb = vdot(oc, lr.d);
        float cc = vlen2(oc) - rad * rad;
        float disc = hb * hb - a * cc;
        if (disc >= 0.0f) {
            float sq = sqrt_rn(disc);
            float ts0 = (-hb - sq) / a, ts1 = (-hb + sq) / a;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                float t = k == 0 ? ts0 : ts1;
                if (t >= t_min && t <= t_max && t < closest) {
                    f3 p = ray_at(lr, t);
                    bool ok = cap == 0 ? (p.y >= ctr.y) : (p.y <= ctr.y);
                    if (ok) {
                        f3 ln = vnorm(vsub(p, cc_));
                        closest = t;
                        hit_new(out, t, m_point(pr.xf, p), vnorm(m_vector(pr.xf, ln)), r);
                        found = true;
                    }
                }
            }
        }
    }
    f3 oc = vsub(lr.o, ctr);
    float ac = lr.d.x * lr.d.x + lr.d.z * lr.d.z;
    float bc = 2.0f * (oc.x * lr.d.x + oc.z * lr.d.z);
    float ccy = oc.x * oc.x + oc.z * oc.z - rad * rad;
    float disc = bc * bc - 4.0f * ac * ccy;
    if (disc >= 0.0f) {
        float sq = sqrt_rn(disc);
        float ts0 = (-bc - sq) / (2.0f * ac), ts1 = (-bc + sq) / (2.0f * ac);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float t = k == 0 ? ts0 : ts1;
            if (t >= t_min && t <= t_max && t < closest) {
                f3 p = ray_at(lr, t);
                if (fabsf(p.y - ctr.y) <= hh) {
                    f3 ln = V((p.x - ctr.x) / rad, 0.0f, (p.z - ctr.z) / rad);
                    closest = t;
                    hit_new(out, t, m_point(pr.xf, p), vnorm(m_vector(pr.xf, ln)), r);
                    found = true;
                }
            }
        }
    }
    return found;
}

template <bool NEED_HIT, class EVAL, bool ANY = false, bool CONVEX = false>
__device__ __forceinline__ bool isect_sdf(const DPrim& pr, const EVAL& eval, const Ray& r, float t_min, float t_max,
                                          Hit& out) {
    float t;
    if (!sdf_march<EVAL, ANY, CONVEX>(pr, eval, r, t_min, t_max, t)) return false;
    if (NEED_HIT) sdf_hit_attributes(eval, r, t, out);
    else out.t = t;
    return true;
}

// ---------------------------------------------------------------- meshes
// Moller-Trumbore exactly as Triangle::intersect (primitives.rs:208-244), with e1 = v1-v0 and
// e2 = v2-v0 precomputed on the host (the same f32 subtractions).
__device__ __forceinline__ bool mt_test(f3 v0, f3 e1, f3 e2, const Ray& r, float t_min, float t_max, float& t,
                                        float& u, float& v) {
    f3 h = vcross(r.d, e2);
    float a = vdot(e1, h);
    if (a > -1e-6f && a < 1e-6f) return false;
    float f = rcp_rn(a);
    f3 s = vsub(r.o, v0);
    u = f * vdot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    f3 q = vcross(s, e1);
    v = f * vdot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    t = f * vdot(e2, q);
    if (t < t_min || t > t_max) return false;
    return true;
}

__device__ __forceinline__ f3 xyz(float4 a) { return V(a.x, a.y, a.z); }

// Hit attributes of triangle slot k: re-run the test for (u, v), barycentric normal
// (primitives.rs:240-243), HitInfo::new.
__device__ __forceinline__ bool mesh_tri_hit(const MeshView& mv, uint32_t k, const Ray& r, float t_min, float t_max,
                                             Hit& out) {
    float t, u, v;
    if (!mt_test(xyz(mv.tris[3 * k]), xyz(mv.tris[3 * k + 1]), xyz(mv.tris[3 * k + 2]), r, t_min, t_max, t, u, v))
        return false;
    f3 p = ray_at(r, t);
    float w = 1.0f - u - v;
    f3 n = vnorm(vadd(vadd(vmuls(xyz(mv.norms[3 * k]), w), vmuls(xyz(mv.norms[3 * k + 1]), u)),
                      vmuls(xyz(mv.norms[3 * k + 2]), v)));
    hit_new(out, t, p, n, r);
    out.sub = k;
    return true;
}

// Workgroup geometry: one wave per workgroup, one 8x8 pixel tile each (kBlockThreads = 64).  A
// workgroup's waves must start together on one CU and a 4-wave workgroup needs a free slot on every
// SIMD, so with a few long-running (grazing-ray) waves resident, 256-thread workgroups of 16x16 pixels
// left slots idle that single waves fill: -9 % per frame.  RRTE_WG256 (defined by the
// host for RRTE_WG64=0, an A/B switch for the specialised kernels) restores the 256-thread layout.
#ifdef RRTE_WG256
constexpr bool kWg64 = false;
#else
constexpr bool kWg64 = true;
#endif
constexpr uint32_t kBlockThreads = kWg64 ? 64u : 256u;

constexpr int kMeshStack = 32;  // BVH depth is capped below this at build time
__device__ __forceinline__ uint32_t* mesh_stack() {
    __shared__ uint32_t stk[kMeshStack * kBlockThreads];  // [depth][lane of the workgroup]
    return stk + threadIdx.x;
}

// Slab test against an (inflated) node box, clipped to [t_min, t_max]: the entry t, or +inf.
__device__ __forceinline__ float box_entry(float4 lo, float4 hi, f3 o, f3 inv, float t_min, float t_max) {
    float tx0 = (lo.x - o.x) * inv.x, tx1 = (hi.x - o.x) * inv.x;
    float ty0 = (lo.y - o.y) * inv.y, ty1 = (hi.y - o.y) * inv.y;
    float tz0 = (lo.z - o.z) * inv.z, tz1 = (hi.z - o.z) * inv.z;
    float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), t_min));
    float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), t_max));
    return tn <= tf ? tn : kInf;
}

// The mesh as a Vec<Triangle>: closest hit over its triangles in index order (strict '<', the
// lower index wins a tie) or, with ANY, whether any triangle is hit.  The BVH visits the near
// child first and prunes boxes entered beyond the current best; boxes are inflated at build time
// so the pruning never drops a triangle the test would accept (meshes).  Rays with
// a non-finite component take the original-order scan (every test then "hits" with t = NaN, as
// in the reference, and the lowest index wins).  Writes t and the triangle slot (out.sub).
template <bool ANY>
__device__ __forceinline__ bool isect_mesh(const DPrim& pr, const MeshView& mv, const Ray& r, float t_min,
                                           float t_max, Hit& out) {
    const uint32_t count = pr.sdf_count, base = (uint32_t)pr.p[0];
    bool found = false;
    float best = kInf;
    uint32_t best_k = 0u, best_orig = 0u;
    if (!(finite3(r.o) && finite3(r.d))) {
        for (uint32_t i = 0; i < count; ++i) {
            const uint32_t k = mv.perm[base + i];
            float t, u, v;
            if (mt_test(xyz(mv.tris[3 * k]), xyz(mv.tris[3 * k + 1]), xyz(mv.tris[3 * k + 2]), r, t_min, t_max, t, u, v)) {
                if (!found || t < best) {
                    best = t;
                    best_k = k;
                    found = true;
                    if (ANY) break;
                }
            }
        }
    } else {
        const f3 inv = V(rcp_rn(r.d.x), rcp_rn(r.d.y), rcp_rn(r.d.z));
        uint32_t* stk = mesh_stack();
        int sp = 0;
        uint32_t link = count ? pr.sdf_first : 0u;
        while (count) {
            if (!(link & 0x80000000u)) {
                // interior: test both children, descend into the nearer, keep the farther
                const float4* rec = mv.nodes + 4u * link;
                const float4 l0 = rec[0], h0 = rec[1], l1 = rec[2], h1 = rec[3];
                const float cap = found ? fminf(best, t_max) : t_max;
                const float t0 = box_entry(l0, h0, r.o, inv, t_min, cap);
                const float t1 = box_entry(l1, h1, r.o, inv, t_min, cap);
                const uint32_t c0 = __float_as_uint(l0.w), c1 = __float_as_uint(l1.w);
                if (t0 != kInf && t1 != kInf) {
                    const bool near0 = t0 <= t1;
                    stk[(sp++) * kBlockThreads] = near0 ? c1 : c0;
                    link = near0 ? c0 : c1;
                    continue;
                }
                if (t0 != kInf) {
                    link = c0;
                    continue;
                }
                if (t1 != kInf) {
                    link = c1;
                    continue;
                }
            } else {
                const uint32_t a = link & 0xFFFFFFu, n = ((link >> 24) & 0x7Fu) + 1u;
                for (uint32_t k = a; k < a + n; ++k) {
                    const float4 A = mv.tris[3 * k];
                    float t, u, v;
                    if (mt_test(xyz(A), xyz(mv.tris[3 * k + 1]), xyz(mv.tris[3 * k + 2]), r, t_min, t_max, t, u, v)) {
                        const uint32_t orig = __float_as_uint(A.w);
                        if (!found || t < best || (t == best && orig < best_orig)) {
                            best = t;
                            best_k = k;
                            best_orig = orig;
                            found = true;
                        }
                        if (ANY) break;
                    }
                }
                if (ANY && found) break;
            }
            if (sp == 0) break;
            link = stk[(--sp) * kBlockThreads];
        }
    }
    out.t = best;
    out.sub = best_k;
    return found;
}

// SceneObject::intersect dispatch, runtime object index: switch on the kind
// (wave-uniform -> scalar branches).
template <bool NEED_HIT, class S, bool ANY = false>
__device__ __forceinline__ bool intersect_at(const S& sc, uint32_t i, const Ray& r, float t_min, float t_max,
                                             Hit& out) {
    const DPrim pr = load_uniform(sc.prims + i);  // (i is wave-uniform: scalar loads)
    constexpr uint32_t F = S::kFeat;
    // (a kind outside the variant's features cannot occur: the host picked the variant from the scene)
    if (pr.kind == RRTE_PRIM_SPHERE) return isect_sphere<NEED_HIT, ANY>(pr, r, t_min, t_max, out);
    if constexpr ((F & kFeatSdf) != 0u)
        if (pr.kind == RRTE_PRIM_SDF) {
            const rrte_sdf_node* nd = sc.nodes + pr.sdf_first;
            if (RRTE_SDF_LEAF_DISPATCH && pr.sdf_count == 1u) {
                bool hit = false;
                const rrte_sdf_node n = load_uniform(nd);
                auto leaf = [&](auto opc) {
                    constexpr uint32_t OP = decltype(opc)::value;
                    if (n.op == OP)
                        hit = isect_sdf<NEED_HIT, SdfLeafProgram<OP>, ANY,
                                        (ANY ? kSecantExit >= 1 : kSecantExit >= 2) && leaf_convex<OP>()>(
                            pr, SdfLeafProgram<OP>{load_uniform(reinterpret_cast<const NodeArgs*>(nd->f))}, r, t_min,
                            t_max, out);
                };
                static_for_leaves(leaf);
                return hit;
            }
            return isect_sdf<NEED_HIT, SdfProgramT<F>, ANY>(pr, SdfProgramT<F>{nd, pr.sdf_count}, r, t_min, t_max, out);
        }
    if constexpr ((F & kFeatAnalytic) != 0u) {
        switch (pr.kind) {
        case RRTE_PRIM_PLANE: return isect_plane<NEED_HIT>(pr, r, t_min, t_max, out);
        case RRTE_PRIM_TRIANGLE: return isect_triangle<NEED_HIT>(pr, r, t_min, t_max, out);
        case RRTE_PRIM_CUBE: return isect_cube<NEED_HIT>(pr, r, t_min, t_max, out);
        case RRTE_PRIM_CYLINDER: return isect_cylinder<NEED_HIT>(pr, r, t_min, t_max, out);
        case RRTE_PRIM_CONE: return isect_cone<NEED_HIT>(pr, r, t_min, t_max, out);
        case RRTE_PRIM_CAPSULE: return isect_capsule<NEED_HIT>(pr, r, t_min, t_max, out);
        default: break;
        }
    }
    if constexpr ((F & kFeatMesh) != 0u)
        if (pr.kind == RRTE_PRIM_MESH) return isect_mesh<ANY>(pr, sc.mesh, r, t_min, t_max, out);
    return false;
}

// Compile-time object index (scene-specialised kernel): only the object's
// own intersector is instantiated.
// Convexity of object I's SDF program for the secant early miss (sdf_convex): decided at compile time
// from the constant program for a full scene, by the host for a topology scene (its topology key).
template <class S, uint32_t I>
constexpr bool prim_convex() {
    if constexpr (S::kTopo) return S::topo_prims[I].convex;
    else return sdf_convex(S::nodes + S::prims[I].sdf_first, S::prims[I].sdf_count);
}
// Part-wise secant plan of object I (sdf_parts_plan): full scenes only (a topology kernel keeps the
// whole-program convexity its host computed), and only with the default march loops.
template <class S, uint32_t I>
constexpr int prim_parts_plan() {
    if constexpr (S::kTopo || !RRTE_PARTS_EXIT || RRTE_MARCH_PAIR || RRTE_MARCH_PRED != 0 || RRTE_DEFER_GUARDS)
        return 0;
    else if constexpr (S::prims[I].kind != RRTE_PRIM_SDF || S::prims[I].sdf_count != 3u)
        return 0;
    else
        return sdf_parts_plan(S::nodes + S::prims[I].sdf_first, 3u);
}
template <bool NEED_HIT, class S, uint32_t I, bool ANY = false>
__device__ __forceinline__ bool intersect_at(const S& sc, UC<I> ii, const Ray& r, float t_min, float t_max, Hit& out) {
    const DPrim pr = prim_at(sc, ii);
    constexpr uint32_t kind = prim_kind<S, I>();
    if constexpr (kind == RRTE_PRIM_SPHERE) return isect_sphere<NEED_HIT, ANY>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_PLANE) return isect_plane<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_TRIANGLE) return isect_triangle<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_CUBE) return isect_cube<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_CYLINDER) return isect_cylinder<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_CONE) return isect_cone<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_CAPSULE) return isect_capsule<NEED_HIT>(pr, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_SDF && prim_parts_plan<S, I>() >= 2 && (ANY ? kSecantExit >= 1 : kSecantExit >= 2))
        return isect_sdf<NEED_HIT, SdfPartsProgram<S, prim_first<S, I>()>, ANY, false>(
            pr, SdfPartsProgram<S, prim_first<S, I>()>{sc}, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_SDF)
        return isect_sdf<NEED_HIT, SdfStaticProgram<S, prim_first<S, I>(), prim_count<S, I>()>, ANY,
                         (ANY ? kSecantExit >= 1 : kSecantExit >= 2) && prim_convex<S, I>()>(
            pr, SdfStaticProgram<S, prim_first<S, I>(), prim_count<S, I>()>{sc}, r, t_min, t_max, out);
    else if constexpr (kind == RRTE_PRIM_MESH) return isect_mesh<ANY>(pr, sc.mesh, r, t_min, t_max, out);
    else return false;
}

// Closest hit over all objects (raytracer.rs:103-113): strict '<' keeps the
// earlier object on ties; analytic objects get t_max = INFINITY as in the
// reference, SDF objects march only up to the current closest hit.  The
// search carries only (t, object); attributes are produced afterwards.
// `pmask` (camera rays): bit i clear = object i's bounding sphere lies outside this workgroup's
// pixel block (KParams::tile_rect), so no lane can hit it and its test is skipped (exact: the
// skipped test would have missed on every lane).
template <class S>
__device__ __forceinline__ int closest_t(const S& sc, const Ray& r, float t_min, float& best_t, uint32_t& best_sub,
                                         uint32_t pmask = ~0u) {
    int idx = -1;
    best_t = kInf;
    best_sub = 0u;
    for_each_prim_exp<1>(sc, [&](auto ii) {
        const uint32_t i = ii;
        if (i < 32u && !((pmask >> i) & 1u)) return;
        Hit h;
        h.sub = 0u;
        float tmax = (prim_at(sc, ii).kind == RRTE_PRIM_SDF && idx >= 0) ? best_t : kInf;
        if (intersect_at<false>(sc, ii, r, t_min, tmax, h)) {
            if (idx < 0 || h.t < best_t || (h.t == best_t && (int)i < idx)) {
                best_t = h.t;
                best_sub = h.sub;
                idx = (int)i;
            }
        }
    });
    return idx;
}

// Hit attributes for the winning object of each lane: analytic objects are
// re-intersected with the search's exact arguments, SDF objects evaluate
// point + normal at the found t -- bit-identical to computing them during the
// search.  Runtime scene: the wave walks its distinct winners (readfirstlane
// -> uniform object index -> scalar loads).  Static scene: every object is
// visited with a compile-time index and skipped unless some lane won it.
template <class S>
__device__ __forceinline__ void attributes_at(const S& sc, uint32_t i, const Ray& r, float t_min, float t,
                                              uint32_t sub, Hit& out) {
    const DPrim pr = load_uniform(sc.prims + i);  // (i is wave-uniform: scalar loads)
    constexpr uint32_t F = S::kFeat;
    if (pr.kind == RRTE_PRIM_SPHERE) {
        sphere_attributes(pr, r, t, out);
        return;
    }
    if constexpr ((F & kFeatSdf) != 0u) {
        if (pr.kind == RRTE_PRIM_SDF) {
            const rrte_sdf_node* nd = sc.nodes + pr.sdf_first;
            if (RRTE_SDF_LEAF_DISPATCH && pr.sdf_count == 1u) {
                const rrte_sdf_node n = load_uniform(nd);
                auto leaf = [&](auto opc) {
                    constexpr uint32_t OP = decltype(opc)::value;
                    if (n.op == OP)
                        sdf_hit_attributes(SdfLeafProgram<OP>{load_uniform(reinterpret_cast<const NodeArgs*>(nd->f))}, r,
                                           t, out);
                };
                static_for_leaves(leaf);
                return;
            }
            sdf_hit_attributes(SdfProgramT<F>{nd, pr.sdf_count}, r, t, out);
            return;
        }
    }
    if constexpr ((F & kFeatMesh) != 0u) {
        if (pr.kind == RRTE_PRIM_MESH) {
            mesh_tri_hit(sc.mesh, sub, r, t_min, kInf, out);
            return;
        }
    }
    if constexpr ((F & kFeatAnalytic) != 0u) intersect_at<true>(sc, i, r, t_min, kInf, out);
}
template <class S, uint32_t I>
__device__ __forceinline__ void attributes_at(const S& sc, UC<I> ii, const Ray& r, float t_min, float t, uint32_t sub,
                                              Hit& out) {
    constexpr uint32_t kind = prim_kind<S, I>();
    if constexpr (kind == RRTE_PRIM_SDF)
        sdf_hit_attributes(SdfStaticProgram<S, prim_first<S, I>(), prim_count<S, I>()>{sc}, r, t, out);
    else if constexpr (kind == RRTE_PRIM_MESH)
        mesh_tri_hit(sc.mesh, sub, r, t_min, kInf, out);
    else if constexpr (kind == RRTE_PRIM_SPHERE)
        sphere_attributes(prim_at(sc, ii), r, t, out);
    else
        intersect_at<true>(sc, ii, r, t_min, kInf, out);
}

template <class S>
__device__ __forceinline__ void hit_attributes(const S& sc, const Ray& r, float t_min, int idx, float t, uint32_t sub,
                                               Hit& out) {
    if constexpr (S::kStatic) {
        for_each_prim(sc, [&](auto ii) {
            const uint32_t i = ii;
            if (__any((uint32_t)idx == i)) {
                if ((uint32_t)idx == i) attributes_at(sc, ii, r, t_min, t, sub, out);
            }
        });
    } else {
        bool pending = idx >= 0;
        while (pending) {
            const uint32_t i = __builtin_amdgcn_readfirstlane((uint32_t)idx);
            if ((uint32_t)idx == i) {
                attributes_at(sc, i, r, t_min, t, sub, out);
                pending = false;
            }
        }
    }
}

template <class S>
__device__ __forceinline__ int closest_hit(const S& sc, const Ray& r, float t_min, Hit& best, uint32_t pmask = ~0u,
                                           bool attributes = true) {
    float t;
    uint32_t sub;
    int idx = closest_t(sc, r, t_min, t, sub, pmask);
    if (attributes) hit_attributes(sc, r, t_min, idx, t, sub, best);
    return idx;
}

// Any-hit form of intersect_at (meshes stop at their first triangle hit).
template <class S>
__device__ __forceinline__ bool any_hit_at(const S& sc, uint32_t i, const Ray& r, float t_min, float t_max, Hit& h) {
    return intersect_at<false, S, true>(sc, i, r, t_min, t_max, h);
}
template <class S, uint32_t I>
__device__ __forceinline__ bool any_hit_at(const S& sc, UC<I> ii, const Ray& r, float t_min, float t_max, Hit& h) {
    return intersect_at<false, S, I, true>(sc, ii, r, t_min, t_max, h);
}

// Any hit in [t_min, t_max] (LAMBERT_SHADOW shadow rays).
template <class S>
__device__ __forceinline__ bool occluded(const S& sc, const Ray& r, float t_min, float t_max, uint64_t mask,
                                         int self = -1) {
    bool hit_any = false;
    for_each_prim_exp<2>(sc, [&](auto ii) {
        const uint32_t i = ii;
        // one wave-uniform skip test: culled, or every lane already occluded (mask cleared)
        if (mask == 0 || (i < 64u && !((mask >> i) & 1ull))) return;
        Hit h;
#if RRTE_MARCH_PRED >= 3
        // predicated: every lane of the caller's EXEC runs the test (marches stay wide, see
        // sdf_march_loop); lanes that are already occluded or that cast no ray (t_max = -inf) get an
        // empty interval, for which every intersector reports no hit
        const float tm = (hit_any || (int)i == self) ? -kInf : t_max;
        const bool hi = any_hit_at(sc, ii, r, t_min, tm, h);
        hit_any = hit_any | hi;
        if (__all(hit_any | !(t_max != -kInf))) mask = 0;
#else
        if (!hit_any && (int)i != self && any_hit_at(sc, ii, r, t_min, t_max, h)) hit_any = true;
        if (__all(hit_any)) mask = 0;
#endif
    });
    return hit_any;
}

// --------------------------------------------------------------- culling
// Shadow-ray culling.  Conservative per-object bounding spheres (host-
// computed, inflated; radius +inf = never culled) let a wave drop the objects
// none of its shadow rays towards a light can reach.  The 64 object tests run
// lane-parallel (lane j tests object j) and __ballot turns them into a
// wave-uniform candidate mask, so occluded() skips culled objects with scalar
// branches.  An object that is not culled runs its exact intersector: culling
// never changes a result.  (Culling primary rays against the tile's view cone
// was measured too and did not pay: a miss is already a cheap bound test.)
struct Cull {
    const float4* __restrict__ bounds;  // one per object; nullptr = culling off
    uint32_t n;                         // objects with a bound (culling needs n <= 64)
};

// Wave-wide min / max as a wave-uniform value, on order-preserving integer keys of the floats
// (key(f) = bits ^ ((bits >> 31) & 0x7fffffff): signed-integer order = float order, -0 < +0, and the
// map is its own inverse): four DPP steps reduce each 16-lane row (quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_half_mirror, row_mirror -- each a v_min_i32 / v_max_i32 with its DPP source, where
// a float min needs a canonicalising v_max_f32 per operand and a separate v_mov_b32_dpp), then the
// four rows' lanes 0, 16, 32, 48 are read into SGPRs and combined on the scalar unit.  No LDS round
// trips (the ds_bpermute butterfly of __shfl_xor took six dependent ones).  Call with all 64 lanes
// active; NaN-free inputs (the callers select +/-inf for unused lanes).
__device__ __forceinline__ int fkey(float f) {
    const int b = __float_as_int(f);
    return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float funkey(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
template <bool MAX>
__device__ __forceinline__ int wave_reduce_key(int v) {
    auto op = [](int a, int b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));
    v = op(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));
    const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ float wave_min(float v) { return funkey(wave_reduce_key<false>(fkey(v))); }
__device__ __forceinline__ float wave_max(float v) { return funkey(wave_reduce_key<true>(fkey(v))); }
__device__ __forceinline__ bool cull_on(const Cull& cl) { return cl.bounds != nullptr && cl.n <= 64u; }

// Bounding sphere of the wave's shading points (lanes with `hit`) grown by each lane's shadow-origin
// offset |n|*bias (normals need not be unit): centred on one used lane's point (the tile's centre
// lane 36 when it is used, else the first used lane), radius = max over used lanes of
// |p - c| + offset -- one wave reduction (the bounding box took seven: min and max of three
// coordinates and the largest offset).  `ext` stays 0 (folded into r).
struct HitBound { f3 c; float r, ext; bool any, unsafe; };
__device__ __forceinline__ HitBound wave_hit_bound(bool hit, f3 p, f3 n, float bias) {
    // the pre-pass only has to be conservative, so it uses cheap bounds: one finiteness test on a sum
    // (a NaN or infinite term, or an overflowing sum, marks the lane unusable -- the wave is then
    // not culled), the 1-ulp hardware square root scaled up by 2^-20, and the offset bound
    // bias * |n|_1 >= bias * |n|_2; the cull margin (1e-3 + 1e-4 * scale) dwarfs their rounding
    const bool use = hit && __builtin_isfinite(((p.x + p.y) + (p.z + n.x)) + (n.y + n.z));
    HitBound b;
    b.ext = 0.0f;
    b.unsafe = __any(hit && !use);
    const uint64_t used = __ballot(use);
    b.any = used != 0ull;
    if (!b.any) {
        b.c = V(0.0f, 0.0f, 0.0f);
        b.r = 0.0f;
        return b;
    }
    const int src = ((used >> 36) & 1ull) ? 36 : (int)__builtin_ctzll(used);
    b.c = V(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), src)),
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), src)),
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), src)));
    const f3 d = vsub(p, b.c);
    const float reach = __builtin_amdgcn_sqrtf(vdot(d, d)) * 1.000001f +
                        bias * ((fabsf(n.x) + fabsf(n.y)) + fabsf(n.z));  // >= 0, NaN-free on used lanes
    b.r = __int_as_float(wave_reduce_key<true>(use ? __float_as_int(reach) : 0));  // keys of floats >= 0 = bits
    return b;
}

// Shadow rays of one light: every ray runs from within `hb` (grown by the
// origin offset) to the light (point/spot; the segment ends at the light plus
// the same offset) or towards -direction (directional), so all of them lie in
// the capsule of radius hb.r + hb.ext around the axis from hb.c.  Waves with
// a non-finite hit point or normal, and directional lights whose direction is
// not unit length (the sphere tracer's bound test assumes |d| = 1), are not
// culled.  Wave-uniform inputs only: call with all 64 lanes active.
// `bnd`: lane j's object bound (load_bound, once per wave for every light).  The projection
// parameter uses the approximate reciprocal of |AB|^2: a relative error of ~1 ulp in t moves the
// capsule point by ~|AB| t 2^-23, far inside the 1e-3 + 1e-4 * scale margin.
__device__ __forceinline__ float4 load_bound(const Cull& cl) {
    const uint32_t j = threadIdx.x & 63u;
    return cl.bounds[j < cl.n ? j : 0u];
}
__device__ __forceinline__ uint64_t shadow_cull(const Cull& cl, const HitBound& hb, const DLight& l, float4 b) {
    if (!cull_on(cl) || hb.unsafe || l.kind == RRTE_LIGHT_AMBIENT) return ~0ull;
    if (!hb.any) return 0ull;
    const bool directional = l.kind == RRTE_LIGHT_DIRECTIONAL;
    const f3 ld = V(l.direction[0], l.direction[1], l.direction[2]);
    if (directional && !(fabsf(vdot(ld, ld) - 1.0f) <= 1e-3f)) return ~0ull;
    const f3 A = hb.c;
    const f3 B = directional ? vsub(A, ld) : V(l.position[0], l.position[1], l.position[2]);
    const f3 AB = vsub(B, A);
    const float ab2 = vdot(AB, AB);
    const float inv_ab2 = __builtin_amdgcn_rcpf(ab2);
    const float scale = fmaxf(fmaxf(fabsf(A.x), fabsf(A.y)), fmaxf(fabsf(A.z), fmaxf(fmaxf(fabsf(B.x), fabsf(B.y)), fabsf(B.z))));
    const float R = hb.r + hb.ext + 1e-3f + 1e-4f * scale;
    const uint32_t j = threadIdx.x & 63u;
    const f3 P = V(b.x, b.y, b.z);
    float t = vdot(vsub(P, A), AB) * inv_ab2;
    t = directional ? fmaxf(t, 0.0f) : clampf_(t, 0.0f, 1.0f);
    const f3 q = vsub(P, vadd(A, vmuls(AB, t)));
    const float rr = R + b.w;
    const bool near = vdot(q, q) <= rr * rr * 1.0001f;
    const bool cand = j < cl.n && (!(__builtin_isfinite(b.w) && ab2 > 0.0f) || near);
    return __ballot(cand);
}

// All lights' masks in one lane-parallel pass (scene-specialised kernels with objects x lights <= 64):
// lane L tests object j = L mod n against light l = L div n's capsule -- the same test as
// shadow_cull, whose per-light wave-uniform prologue (capsule axis, |AB|^2, its reciprocal, the
// margin) every light repeated on all 64 lanes -- and one ballot carries every light's n bits.
// Lights shadow_cull never culls (ambient; directional with a non-unit direction) get all-ones.
// Whether shadow_cull may cull for light I (not ambient; a directional light only with a unit
// direction): from the constant record of a full scene, by the host for a topology scene.
constexpr bool light_record_cullable(const DLight& L) {
#pragma clang fp contract(off)
    if (L.kind == RRTE_LIGHT_AMBIENT) return false;
    if (L.kind != RRTE_LIGHT_DIRECTIONAL) return true;
    const float d2 = (L.direction[0] * L.direction[0] + L.direction[1] * L.direction[1]) + L.direction[2] * L.direction[2];
    return (d2 - 1.0f <= 1e-3f) && (1.0f - d2 <= 1e-3f);
}
template <class S, uint32_t I>
constexpr bool light_cullable() {
    if constexpr (S::kTopo) {
        return S::topo_lights[I].cullable;
    } else {
        constexpr bool c = light_record_cullable(S::lights[I]);
        return c;
    }
}
template <class S>
__device__ __forceinline__ void shadow_cull_lanes(const S& sc, const Cull& cl, const HitBound& hb, uint64_t* smask) {
    constexpr uint32_t n = S::num_prims, nl = S::num_lights;
    static_assert(n * nl <= 64u && n > 0u, "one lane per (light, object)");
    auto cullable = [](auto lii) { return light_cullable<S, (uint32_t)decltype(lii)::value>(); };
    if (!cull_on(cl) || hb.unsafe || !hb.any) {
        auto fill = [&](auto lii) { smask[(uint32_t)lii] = (cullable(lii) && cull_on(cl) && !hb.unsafe) ? 0ull : ~0ull; };
        static_for<0, nl>(fill);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane / n, j = lane - l * n;
    const f3 A = hb.c;
    f3 B = A;
    bool directional = false;
    auto pick = [&](auto lii) {
        const DLight L = light_at(sc, lii);
        if (l == (uint32_t)lii) {
            if constexpr (light_kind<S, (uint32_t)decltype(lii)::value>() == RRTE_LIGHT_DIRECTIONAL) {
                B = vsub(A, V(L.direction[0], L.direction[1], L.direction[2]));
                directional = true;
            } else {
                B = V(L.position[0], L.position[1], L.position[2]);
            }
        }
    };
    static_for<0, nl>(pick);
    const f3 AB = vsub(B, A);
    const float ab2 = vdot(AB, AB);
    const float inv_ab2 = __builtin_amdgcn_rcpf(ab2);
    const float scale = fmaxf(fmaxf(fabsf(A.x), fabsf(A.y)), fmaxf(fabsf(A.z), fmaxf(fmaxf(fabsf(B.x), fabsf(B.y)), fabsf(B.z))));
    const float R = hb.r + hb.ext + 1e-3f + 1e-4f * scale;
    const float4 b = cl.bounds[j < cl.n ? j : 0u];
    const f3 P = V(b.x, b.y, b.z);
    float t = vdot(vsub(P, A), AB) * inv_ab2;
    t = directional ? fmaxf(t, 0.0f) : clampf_(t, 0.0f, 1.0f);
    const f3 q = vsub(P, vadd(A, vmuls(AB, t)));
    const float rr = R + b.w;
    const bool near = vdot(q, q) <= rr * rr * 1.0001f;
    const bool cand = l < nl && j < cl.n && (!(__builtin_isfinite(b.w) && ab2 > 0.0f) || near);
    const uint64_t m = __ballot(cand);
    constexpr uint64_t kBits = n >= 64u ? ~0ull : ((1ull << n) - 1ull);
    auto split = [&](auto lii) {
        constexpr uint32_t li = (uint32_t)lii;
        smask[li] = cullable(lii) ? ((m >> (li * n)) & kBits) : ~0ull;
    };
    static_for<0, nl>(split);
}

// --------------------------------------------------------------- lighting
struct Contrib { float cr, cg, cb, ca; f3 dir; float dist, att; };

// PointLight::calculate_attenuation (light.rs:170-178)
__device__ __forceinline__ float point_att(const DLight& l, float d) {
    if (d > l.range) return 0.0f;
    float a = rcp_rn((1.0f + l.linear * d) + (l.quadratic * d) * d);
    return mx(a, 0.0f);
}

// Light::illuminate (light.rs:87-94, 182-194, 289-304, 365-372)
__device__ __forceinline__ Contrib illuminate(const DLight& l, f3 p) {
    Contrib k;
    k.cr = l.cI[0]; k.cg = l.cI[1]; k.cb = l.cI[2]; k.ca = l.cI[3];
    switch (l.kind) {
    case RRTE_LIGHT_POINT: {
        f3 lv = vsub(V(l.position[0], l.position[1], l.position[2]), p);
        k.dist = vlen(lv);
        k.dir = vnorm(lv);
        k.att = point_att(l, k.dist);
        break;
    }
    case RRTE_LIGHT_DIRECTIONAL:
        k.dir = vneg(V(l.direction[0], l.direction[1], l.direction[2]));
        k.dist = kInf;
        k.att = 1.0f;
        break;
    case RRTE_LIGHT_SPOT: {
        f3 lv = vsub(V(l.position[0], l.position[1], l.position[2]), p);
        k.dist = vlen(lv);
        k.dir = vnorm(lv);
        float da = point_att(l, k.dist);
        float ang = acosf(vdot(V(l.direction[0], l.direction[1], l.direction[2]), vneg(k.dir)));
        float aa;
        if (ang > l.outer_angle) aa = 0.0f;
        else if (ang < l.inner_angle) aa = 1.0f;
        else {
            float fo = (l.outer_angle - ang) / (l.outer_angle - l.inner_angle);
            aa = fo * fo;
        }
        k.att = da * aa;
        break;
    }
    default:
        k.dir = V(0.0f, 0.0f, 0.0f);
        k.dist = 0.0f;
        k.att = 1.0f;
        break;
    }
    return k;
}

__device__ __forceinline__ f3 rand_in_unit_sphere(uint32_t& st) {  // vector.rs:35-46
    for (;;) {
        float x = rng_f32(st) * 2.0f - 1.0f;
        float y = rng_f32(st) * 2.0f - 1.0f;
        float z = rng_f32(st) * 2.0f - 1.0f;
        f3 p = V(x, y, z);
        if (vlen2(p) < 1.0f) return p;
    }
}
__device__ __forceinline__ f3 reflect3(f3 v, f3 n) { return vsub(v, vmuls(n, 2.0f * vdot(v, n))); }

// Material::scatter (material.rs:60-72, 99-110, 147-170, 200-202)
__device__ __forceinline__ bool scatter(const DMaterial& m, const Ray& rin, const Hit& h, uint32_t& st, Ray& out) {
    switch (m.kind) {
    case RRTE_MAT_LAMBERTIAN: {
        f3 sd = vadd(h.n, vnorm(rand_in_unit_sphere(st)));
        f3 dir = vlen2(sd) < 1e-8f ? h.n : sd;
        out = ray_new(h.p, dir);
        return true;
    }
    case RRTE_MAT_METAL: {
        f3 refl = reflect3(vnorm(rin.d), h.n);
        f3 s = vadd(refl, vmuls(rand_in_unit_sphere(st), m.fuzz));
        if (vdot(s, h.n) > 0.0f) { out = ray_new(h.p, s); return true; }
        return false;
    }
    case RRTE_MAT_DIELECTRIC: {
        float ratio = h.front ? rcp_rn(m.ior) : m.ior;
        f3 ud = vnorm(rin.d);
        float cos_t = mn(vdot(vneg(ud), h.n), 1.0f);
        float sin_t = sqrt_rn(1.0f - cos_t * cos_t);
        bool cannot = ratio * sin_t > 1.0f;
        float r0 = (1.0f - ratio) / (1.0f + ratio);
        r0 = r0 * r0;
        float x = 1.0f - cos_t;
        float x2 = x * x;
        float refl = r0 + (1.0f - r0) * (x * (x2 * x2));
        bool do_reflect = cannot;
        if (!do_reflect) do_reflect = refl > rng_f32(st);
        f3 dir;
        if (do_reflect) {
            dir = reflect3(ud, h.n);
        } else {
            float ct = mn(vdot(vneg(ud), h.n), 1.0f);
            f3 perp = vmuls(vadd(ud, vmuls(h.n, ct)), ratio);
            float l2 = vlen2(perp);
            f3 par = vmuls(h.n, -sqrt_rn(fabsf(1.0f - l2)));
            dir = (l2 < 1.0f) ? vadd(perp, par) : reflect3(ud, h.n);
        }
        out = ray_new(h.p, dir);
        return true;
    }
    default:
        return false;
    }
}

// ----------------------------------------------------------------- pixel
struct Col { float r, g, b, a; };

// Camera::generate_ray (camera.rs:98-133)
__device__ __forceinline__ Ray generate_ray(const FrameCam& cm, float u, float v) {
    float ndc_x = 2.0f * u - 1.0f;
    float ndc_y = 1.0f - 2.0f * v;
    if (cm.projection == RRTE_PERSPECTIVE) {
        float half_w = cm.aspect * cm.half_h;
        f3 cd = vnorm(V(ndc_x * half_w, ndc_y * cm.half_h, -1.0f));
        f3 wd = quat_rotate(cm.cam_rot, cd);
        return ray_new_unit(V(cm.cam_pos[0], cm.cam_pos[1], cm.cam_pos[2]), wd);
    }
    float wx = cm.ortho_l + (cm.ortho_r - cm.ortho_l) * u;
    float wy = cm.ortho_b + (cm.ortho_t - cm.ortho_b) * v;
    f3 o = m_point(cm.cam_xf, V(wx, wy, 0.0f));
    f3 wd = quat_rotate(cm.cam_rot, V(0.0f, 0.0f, -1.0f));
    return ray_new_unit(o, wd);
}

// Raytracer::ray_color (raytracer.rs:92-148) for one camera sample.
// REFCOMPAT: ambient + sum(light.color*I*att) + albedo * ray_color(scatter).
// The reference recursion color_d = local_d + albedo_d * color_{d+1} is
// evaluated forward with a running albedo product; that is bit-identical to
// the recursion for max_depth <= 2 (the parity configs use 1) and differs by
// rounding only beyond.
// Material record of a hit (nullptr = no material -> BLACK, raytracer.rs:139-143).
template <class S>
__device__ __forceinline__ const DMaterial* material_of(const S& sc, int idx) {
    const int mi = sc.prims[idx].material;
    return (mi < 0 || (uint32_t)mi >= sc.num_materials) ? nullptr : &sc.mats[mi];
}

// REFCOMPAT: Raytracer::ray_color (raytracer.rs:92-148) for one camera ray:
// ambient + sum(light.color*I*att) + albedo * ray_color(scatter).  The
// reference recursion color_d = local_d + albedo_d * color_{d+1} is evaluated
// forward with a running albedo product: bit-identical to the recursion for
// max_depth <= 2 (the parity configs use 1), rounding-level beyond.  A path is
// advanced one bounce at a time (path_step) so that the kernel can start a
// lane's next sample as soon as its current path ends (see ray_kernel_body).
struct PathState {
    Ray r;
    Col out;
    float tr, tg, tb;  // running albedo product
    uint32_t depth;
};

__device__ __forceinline__ void path_begin(PathState& ps, const Ray& r) {
    ps.r = r;
    ps.out = Col{0.0f, 0.0f, 0.0f, 1.0f};
    ps.tr = ps.tg = ps.tb = 1.0f;
    ps.depth = 0;
}

// One bounce of ray_color (kp.max_depth >= 1); true when the path has ended.  pmask: camera-ray
// tile culling mask (only for the camera ray, ~0u otherwise).
template <class S>
__device__ __forceinline__ bool path_step(const S& sc, const KParams& kp, PathState& ps, uint32_t& st,
                                          uint32_t pmask = ~0u) {
    Hit h;
    const int idx = closest_hit(sc, ps.r, kp.t_min, h, pmask);
    const uint32_t depth = ps.depth;
    if (idx < 0) {
        if (depth == 0) {
            ps.out = Col{kp.bg[0], kp.bg[1], kp.bg[2], kp.bg[3]};
        } else {
            ps.out.r = ps.out.r + ps.tr * kp.bg[0];
            ps.out.g = ps.out.g + ps.tg * kp.bg[1];
            ps.out.b = ps.out.b + ps.tb * kp.bg[2];
        }
        return true;
    }
    const DMaterial* m = material_of(sc, idx);
    if (!m) return true;  // BLACK
    float ar = m->albedo[0], ag = m->albedo[1], ab = m->albedo[2], aa = m->albedo[3];
    // BLACK + ambient_color()*0.1 (raytracer.rs:124, material.rs:10-12)
    float cr = 0.0f + (ar * 0.1f) * 0.1f;
    float cg = 0.0f + (ag * 0.1f) * 0.1f;
    float cb = 0.0f + (ab * 0.1f) * 0.1f;
    float ca = 1.0f + (aa * 0.1f) * 0.1f;
    for_each_light(sc, [&](auto lii) {
        Contrib k = illuminate(light_at(sc, lii), h.p);
        cr = cr + k.cr * k.att;
        cg = cg + k.cg * k.att;
        cb = cb + k.cb * k.att;
        ca = ca + k.ca * k.att;
    });
    if (depth == 0) {
        ps.out = Col{cr, cg, cb, ca};
    } else {
        ps.out.r = ps.out.r + ps.tr * cr;
        ps.out.g = ps.out.g + ps.tg * cg;
        ps.out.b = ps.out.b + ps.tb * cb;
    }
    Ray sc_ray;
    if (!scatter(*m, ps.r, h, st, sc_ray)) return true;
    if (depth == 0) ps.out.a = ps.out.a + 1.0f;  // Color::from(Vec3) has alpha 1 (color.rs:78-82)
    if (depth + 1 >= kp.max_depth) return true;   // ray_color(depth 0) == BLACK: adds 0
    ps.tr = ps.tr * ar;
    ps.tg = ps.tg * ag;
    ps.tb = ps.tb * ab;
    ps.r = sc_ray;
    ps.depth = depth + 1;
    return false;
}

// The whole path of one camera ray.  SINGLE (scene-specialised straight-line kernels): one
// bounce only (max_depth <= 1).
template <class S, bool SINGLE>
__device__ __forceinline__ Col ray_color_ref(const S& sc, const KParams& kp, Ray r, uint32_t& st,
                                             uint32_t pmask = ~0u) {
    PathState ps;
    path_begin(ps, r);
    if (kp.max_depth == 0) return ps.out;
    if constexpr (SINGLE) {
        path_step(sc, kp, ps, st, pmask);
    } else {
#pragma unroll 1
        while (!path_step(sc, kp, ps, st)) {
        }
    }
    return ps.out;
}

// LAMBERT_SHADOW (build-defined) for one camera ray.  Called by
// all 64 lanes of the wave (`live` marks the lanes that own a pixel): with
// CULL the hit-point bound and the per-light shadow culls are wave reductions.
constexpr bool kShadeAll = RRTE_MARCH_PRED >= 3;  // shade every lane (predicated), or only hit lanes
template <class S, bool CULL>
__device__ __forceinline__ Col shade_lambert(const S& sc, const KParams& kp, const Cull& cl, const Ray& r, bool live,
                                             uint32_t& nshadow, uint32_t pmask) {
    Col out{0.0f, 0.0f, 0.0f, 1.0f};
    if (kp.max_depth == 0) return out;
    Hit h;
    h.t = 0.0f;  // lanes without a hit keep a benign point and normal (predicated shading, RRTE_MARCH_PRED)
    h.p = V(0.0f, 0.0f, 0.0f);
    h.n = V(0.0f, 1.0f, 0.0f);
    h.front = true;
    h.sub = 0u;
    // RRTE_DEBUG bit 7 (timing diagnostics only, with bit 1): the closest-hit search without hit attributes
    const int idx = closest_hit(sc, r, live ? kp.t_min : kInf, h, pmask, !(kp.debug & 128u));  // idle lanes find nothing
    const DMaterial* m = idx >= 0 ? material_of(sc, idx) : nullptr;
    const bool hit = m != nullptr;
    if (idx < 0) out = Col{kp.bg[0], kp.bg[1], kp.bg[2], kp.bg[3]};
    if (kp.debug & 2u) {  // diagnostics: primary visibility only
        if (idx >= 0) out = Col{h.t * 0.01f, 0.0f, 0.0f, 1.0f};
        return out;
    }
    float ar = 0.0f, ag = 0.0f, ab = 0.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f, ca = 1.0f;
    if (hit) {
        ar = m->albedo[0]; ag = m->albedo[1]; ab = m->albedo[2];
        // BLACK + ambient_color()*0.1 (raytracer.rs:124, material.rs:10-12)
        cr = 0.0f + (ar * 0.1f) * 0.1f;
        cg = 0.0f + (ag * 0.1f) * 0.1f;
        cb = 0.0f + (ab * 0.1f) * 0.1f;
        ca = 1.0f + (m->albedo[3] * 0.1f) * 0.1f;
    }
    const float bias = kp.bias;
    // contribution of one light to a hit lane (light.rs illuminate + N.L + shadow ray)
    // RRTE_DEBUG bit 8 (timing diagnostics only, wrong images): shadow tests for light (debug >> 9) & 7 only
    auto shade = [&](const DLight& l, uint64_t smask, uint32_t li) {
        Contrib k = illuminate(l, h.p);
        if (l.kind == RRTE_LIGHT_AMBIENT) {
            if (hit) {
                cr = cr + ar * k.cr;
                cg = cg + ag * k.cg;
                cb = cb + ab * k.cb;
            }
            return;
        }
        const float ndl = vdot(h.n, k.dir);
#if RRTE_MARCH_PRED >= 3
        // predicated over every lane (hit or not): a lane that casts no shadow ray tests the empty
        // interval (t_max = -inf) along a benign direction, so the any-hit marches run wide
        const bool cast = hit && ndl > 0.0f && k.att > 0.0f;
        nshadow += cast ? 1u : 0u;
        {
            const Ray sr = ray_new_unit(vadd(h.p, vmuls(h.n, bias)), cast ? k.dir : V(0.0f, 1.0f, 0.0f));
            const bool skip = (kp.debug & 1u) || ((kp.debug & 256u) && li != ((kp.debug >> 9) & 7u));
            const bool occ = !skip && occluded(sc, sr, bias, cast ? k.dist : -kInf, smask, (kp.debug & 64u) ? idx : -1);
            if (cast && !occ) {
                float f = k.att * ndl;
                cr = cr + ar * (k.cr * f);
                cg = cg + ag * (k.cg * f);
                cb = cb + ab * (k.cb * f);
            }
        }
        if (false) {
#else
        if (ndl > 0.0f && k.att > 0.0f) {
#endif
            ++nshadow;
            Ray sr = ray_new_unit(vadd(h.p, vmuls(h.n, bias)), k.dir);
            // RRTE_DEBUG bit 6 (timing diagnostics only, wrong images): skip the object the ray starts on
            if ((kp.debug & 1u) || ((kp.debug & 256u) && li != ((kp.debug >> 9) & 7u)) ||
                !occluded(sc, sr, bias, k.dist, smask, (kp.debug & 64u) ? idx : -1)) {
                float f = k.att * ndl;
                cr = cr + ar * (k.cr * f);
                cg = cg + ag * (k.cg * f);
                cb = cb + ab * (k.cb * f);
            }
        }
    };
    if constexpr (!CULL) {
        if (kShadeAll || hit) for_each_light(sc, [&](auto lii) { shade(light_at(sc, lii), ~0ull, (uint32_t)lii); });
    } else {
        HitBound hb{};
        hb.unsafe = true;  // no bounds table: every mask all-ones
        if (cull_on(cl)) hb = wave_hit_bound(hit, h.p, h.n, bias);
        if constexpr (S::kStatic) {
            // all light masks first, at one converged point, then the shading
            uint64_t smask[S::num_lights ? S::num_lights : 1];
            if constexpr (S::num_lights > 0 && S::num_prims * S::num_lights <= 64u) {
                shadow_cull_lanes<S>(sc, cl, hb, smask);
            } else {
                const float4 bnd = cull_on(cl) ? load_bound(cl) : float4{};
                auto cull_one = [&](auto lii) { smask[(uint32_t)lii] = shadow_cull(cl, hb, light_at(sc, lii), bnd); };
                static_for<0, S::num_lights>(cull_one);
            }
            auto shade_one = [&](auto lii) { if (kShadeAll || hit) shade(light_at(sc, lii), smask[(uint32_t)lii], (uint32_t)lii); };
            static_for<0, S::num_lights>(shade_one);
        } else {
            const float4 bnd = cull_on(cl) ? load_bound(cl) : float4{};
#pragma unroll 1
            for (uint32_t li = 0; li < sc.num_lights; ++li) {
                const DLight lt = load_uniform(sc.lights + li);  // (li uniform: scalar loads)
                const uint64_t sm = shadow_cull(cl, hb, lt, bnd);
                if (kShadeAll || hit) shade(lt, sm, li);
            }
        }
    }
    if (hit) out = Col{cr, cg, cb, ca};
    return out;
}

// Rust `(x * 255.0) as u8` (raytracer.rs:82-85) and f32::clamp (color.rs:48-55)
__device__ __forceinline__ uint32_t to_u8(float c) {
    float v = c * 255.0f;
    if (!(v > 0.0f)) return 0u;
    if (v >= 255.0f) return 255u;
    return (uint32_t)v;
}
__device__ __forceinline__ float rclamp(float x) {
    if (x < 0.0f) return 0.0f;
    if (x > 1.0f) return 1.0f;
    return x;
}

// One channel of the reference's fixed to_gamma(2.2) -> clamp -> truncating u8 (raytracer.rs:79-85,
// color.rs:58-65) without powf in the common case.  The compiler's powf is a ~100-instruction
// double-float sequence, a tenth of the headline kernel with three per pixel.  y = exp2(log2(c)/2.2)
// from v_log_f32 / v_exp_f32 is within a few ulp of it; RN(p*255) and the clamp are monotone in p,
// so when y(1 - m) and y(1 + m) quantise to the same byte every p in between -- powf's result
// included -- does too, and that byte is the answer.  Lanes near a byte boundary, +inf and -inf
// take powf.  Bit-identical to to_u8(rclamp(powf(c, RN(1/2.2)))) for all 2^32 inputs
// (rrte_hip_fpcheck RRTE_FPCHECK_GAMMA_U8, tests/test_gpu_fpexact.py).
constexpr float kInvGamma22 = 1.0f / 2.2f;
constexpr float kGammaMargin = 0x1p-20f;  // relative, ~8 ulp
__device__ __forceinline__ uint32_t gamma22_u8(float c) {
    const float y = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(c) * kInvGamma22);
    const float m = y * kGammaMargin;
    const uint32_t a = to_u8(rclamp(y - m)), b = to_u8(rclamp(y + m));
    // c = -inf: log2 gives NaN (byte 0) but powf(-inf, 1/2.2) = +inf (byte 255)
    if (__builtin_expect(a == b && c != -kInf, 1)) return a;
    return to_u8(rclamp(powf(c, kInvGamma22)));
}

// Map this launch's local row to the image row (band interleave, §8e).
__device__ __forceinline__ uint32_t image_row(const KParams& kp, uint32_t r) {
    if (kp.band_rows == 0) return r + kp.row0;
    const uint32_t b = r / kp.band_rows, w = r - b * kp.band_rows;
    const BandMap m{kp.band_rows, kp.nranks, kp.sky_bands, kp.root_bands, kp.peer_bands};
    return band_of_local(m, kp.rank, b) * kp.band_rows + w;
}

// Camera-ray tile culling mask of this wave's 8x8 tile (kp.tile_cull = 3) or the 16x16
// block (4) (KParams::tile_rect): lane j tests object j's rectangle and a ballot makes the mask
// wave-uniform (one load and a handful of VALU ops per wave; a scalar loop over the objects cost ~8
// SALU ops and a scalar load each).  Call with all 64 lanes active.  The host enables it only when
// a tile's local rows are consecutive image rows (no band mapping, or bands of a multiple of the
// tile height).
__device__ __forceinline__ uint32_t camera_tile_mask(const KParams& kp, const FrameCam& cm, uint32_t tx,
                                                     uint32_t ty) {
    const uint32_t sh = cm.tile_cull;
    if (!sh) return ~0u;
    uint32_t bx, bx1, by;
    if (kWg64) {  // one tile per workgroup: (1 << tile_shift) x (64 >> tile_shift) pixels
        // (its rows lie in one 8-row block of consecutive image rows: 64 >> tile_shift divides 8 and
        // band heights are multiples of 8)
        bx = (tx << kp.tile_shift) >> sh;
        bx1 = ((tx << kp.tile_shift) + (1u << kp.tile_shift) - 1u) >> sh;
        by = image_row(kp, ty * (64u >> kp.tile_shift)) >> sh;
    } else {
        const uint32_t wave = sh == 3u ? (threadIdx.x >> 6) : 0u;
        bx = (blockIdx.x * 16u + (wave & 1u) * 8u) >> sh;
        bx1 = bx;
        by = image_row(kp, blockIdx.y * 16u + (wave >> 1) * 8u) >> sh;
    }
    const uint32_t j = threadIdx.x & 63u;
    bool in = false;
    if (j < cm.tile_n) {  // the rectangle meets the tile's blocks [bx, bx1] x by
        const uint32_t t = cm.tile_rect[j];
        in = bx1 >= (t & 255u) && bx <= ((t >> 8) & 255u) && by >= ((t >> 16) & 255u) && by <= (t >> 24);
    }
    const uint32_t m = (uint32_t)__ballot(in);
    return m | (cm.tile_n < 32u ? (~0u << cm.tile_n) : 0u);  // objects past the table: never culled
}

// The tile (x, y in workgroup units) and frame of this workgroup: with a tile list (KParams::hot,
// measured-cost order) slot k = blockIdx.z * tiles_x + blockIdx.x renders tile hot[k] (a wave-uniform
// index: one scalar load); run = false for the unused slots of the last slot row.
struct LaunchTile { uint32_t x, y, z; bool run; };
__device__ __forceinline__ LaunchTile launch_tile(const KParams& kp) {
    if (!kWg64) return LaunchTile{blockIdx.x, blockIdx.y, blockIdx.z, true};
    LaunchTile t{blockIdx.x, blockIdx.z, blockIdx.y, true};
    if (kp.hot) {
        const uint32_t k = blockIdx.z * kp.tiles_x + blockIdx.x;
        t.run = k < kp.hot_n;
        const uint32_t h = kp.hot[t.run ? (k & 7u) * kp.hot_stride + (k >> 3) : 0u];
        t.x = hot_x(h);
        t.y = hot_y(h);
    }
    return t;
}

// RRTE_DEBUG bit 2: the launch's derived indices, checked before any memory access that uses them.
// Check-word bits: 1 list slot out of range, 2 decoded tile outside the launch's tiles, 4 frame index
// >= nframes, 8 an output row outside the frame.
__device__ __forceinline__ bool launch_indices_ok(const KParams& kp, unsigned long long* counters) {
    uint32_t bad = 0u;
    const uint32_t th = 64u >> kp.tile_shift, gy = (kp.rows + th - 1u) / th;
    const uint32_t k = blockIdx.z * kp.tiles_x + blockIdx.x;
    if (blockIdx.y >= kp.nframes || blockIdx.y >= kMaxLaunchFrames) bad |= 4u;
    if (kp.hot) {
        if (k < kp.hot_n) {
            const uint32_t at = (k & 7u) * kp.hot_stride + (k >> 3);
            if (kp.hot_stride * 8u < kp.hot_n || at >= kp.hot_stride * 8u) bad |= 1u;
            else {
                const uint32_t h = kp.hot[at];
                if (hot_x(h) >= kp.tiles_x || hot_y(h) >= gy) bad |= 2u;
            }
        }
    } else if (blockIdx.x >= kp.tiles_x || blockIdx.z >= gy) {
        bad |= 2u;
    }
    if (!bad && kp.rows && kp.band_rows == 0u && kp.row0 + kp.rows > kp.height) bad |= 8u;
    if (bad && (threadIdx.x & 63u) == 0u) atomicOr(counters + 1, (unsigned long long)bad);
    return bad == 0u;
}

// One lane per pixel; wave = workgroup = 8x8 tile (RRTE_WG256: 16x16-pixel workgroups).  Every lane
// of a wave runs the sample loop (lanes past the image edge are idle but
// present) so the culling reductions see converged waves.  CULL selects the
// shadow-culled LAMBERT_SHADOW variant (the host picks it per scene).
template <int MODE, class S, bool SINGLE = false, bool CULL = false>
__device__ __forceinline__ void ray_kernel_body(const KParams& kp, const S& sc, const Cull& cl,
                                                uint32_t* __restrict__ out_rgba8, float4* __restrict__ out_f32,
                                                unsigned long long* __restrict__ counters) {
    const uint32_t lane = threadIdx.x & 63u, wave = kWg64 ? 0u : threadIdx.x >> 6;
    // RRTE_DEBUG bit 2 (diagnostics): every index this wave derives from the launch (list slot, tile,
    // frame) is range-checked before use; a violation sets a bit in the check word (counters[1], an
    // unused word of shard 0; rrte_hip_check_word) and the wave stops instead of touching memory
    if ((kp.debug & 4u) && kWg64 && !launch_indices_ok(kp, counters)) return;
    const LaunchTile tile = launch_tile(kp);
    if (!tile.run) return;
    // frame tile.z of the launch: its camera, its output (multi-frame launches have no f32 output)
    const FrameCam& cm = kp.cam[tile.z];
    if (kp.out_image_rows)
        out_rgba8 = cm.out;
    else if (out_rgba8 && tile.z)
        out_rgba8 = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(out_rgba8) + tile.z * kp.frame_stride);
    // RRTE_DEBUG bit 4 (diagnostics, tools/wave_times.py): per-wave start / duration from the 100 MHz
    // wall clock into the f32 buffer instead of colours
    const bool stamps = (kp.debug & 16u) && out_f32;
    const uint32_t tiles_x = kWg64 ? kp.tiles_x : gridDim.x;
    // bit 5: only workgroup (debug >> 16) runs (its waves' durations alone on the GPU)
    const uint32_t brow = tile.y;
    if ((kp.debug & 32u) && brow * tiles_x + tile.x != (kp.debug >> 16)) return;
    const bool timed = stamps || (kp.tile_cost && tile.z == 0u);
    const uint64_t t_wave0 = timed ? wall_clock64() : 0ull;
    const uint32_t ts = kp.tile_shift;  // (kWg64: tile 1 << ts wide, 64 >> ts rows)
    const uint32_t x = kWg64 ? (tile.x << ts) + (lane & ((1u << ts) - 1u)) : tile.x * 16u + (wave & 1u) * 8u + (lane & 7u);
    const uint32_t lr = kWg64 ? brow * (64u >> ts) + (lane >> ts) : brow * 16u + (wave >> 1) * 8u + (lane >> 3);
    bool live = x < kp.width && lr < kp.rows;
    const uint32_t xc = live ? x : 0u;
    const uint32_t y = image_row(kp, live ? lr : 0u);
    if ((kp.debug & 4u) && live && y >= kp.height) {  // (bit 2: a band mapping past the frame)
        atomicOr(counters + 1, 8ull);
        live = false;
    }
    const uint32_t pix = y * kp.width + xc;
    uint32_t nshadow = 0;
    Col acc{0.0f, 0.0f, 0.0f, 1.0f};  // BLACK
    const uint32_t nsamples = SINGLE ? 1u : kp.spp;
    const uint32_t pmask = camera_tile_mask(kp, cm, tile.x, tile.y);
    // camera ray of sample s (raytracer.rs:66-70): per-(pixel, sample) RNG stream, jitter, generate_ray
    auto camera_ray = [&](uint32_t s, uint32_t& st) {
        st = pcg_hash(pcg_hash(pcg_hash(kp.seed) ^ pix) ^ s);
        float jx = 0.5f, jy = 0.5f;
        if (kp.jitter == RRTE_JITTER_RANDOM) {
            jx = rng_f32(st);
            jy = rng_f32(st);
        }
        float u = ((float)xc + jx) / (float)kp.width;
        float v = ((float)y + jy) / (float)kp.height;
        return generate_ray(cm, u, v);
    };
    auto accumulate = [&](const Col& c) {
        acc.r = acc.r + c.r;
        acc.g = acc.g + c.g;
        acc.b = acc.b + c.b;
        acc.a = acc.a + c.a;
    };
    if constexpr (MODE == RRTE_MODE_REFCOMPAT && !SINGLE) {
        // Path regeneration: one loop advances every lane's current path by one bounce; a lane
        // whose path ends adds its colour and starts its next sample at once.  A wave then costs
        // the largest per-lane total of bounces instead of the sum over samples of each sample's
        // longest path.  Same per-sample RNG streams and accumulation order as the nested loops.
        if (kp.max_depth == 0) {
            for (uint32_t s = 0; s < nsamples; ++s) accumulate(Col{0.0f, 0.0f, 0.0f, 1.0f});
        } else {
            uint32_t s = 0, st = 0;
            bool active = false;
            PathState ps;
#pragma unroll 1
            for (;;) {
                if (!active && live && s < nsamples) {
                    path_begin(ps, camera_ray(s, st));
                    active = true;
                }
                if (!__any(active)) break;
                // (camera-ray tile culling while every active lane is on its camera ray was measured
                // slower, 0.94 -> 1.00 ms on the stock config: the runtime mask costs every bounce)
                if (active && path_step(sc, kp, ps, st)) {
                    accumulate(ps.out);
                    active = false;
                    ++s;
                }
            }
        }
    } else {
        for (uint32_t s = 0; s < nsamples; ++s) {
            uint32_t st;
            Ray r = camera_ray(s, st);
            Col c{0.0f, 0.0f, 0.0f, 1.0f};
            if (MODE == RRTE_MODE_LAMBERT_SHADOW) {
                c = shade_lambert<S, CULL>(sc, kp, cl, r, live, nshadow, pmask);
            } else if (live) {
                c = ray_color_ref<S, SINGLE>(sc, kp, r, st, SINGLE ? pmask : ~0u);
            }
            accumulate(c);
        }
    }
    if (live) {
        acc.r = acc.r * kp.inv_spp;
        acc.g = acc.g * kp.inv_spp;
        acc.b = acc.b * kp.inv_spp;
        acc.a = acc.a * kp.inv_spp;
        const float ig = kp.inv_gamma;
        const float ga = rclamp(acc.a);
        const size_t o = (size_t)(kp.out_image_rows ? y : lr) * kp.width + x;  // packed local rows, or image rows
        // the parity float buffer (or a gamma other than the reference's 2.2) needs powf itself
        const bool exact_pow = (out_f32 && !stamps) || ig != kInvGamma22;
        float gr = 0.0f, gg = 0.0f, gb = 0.0f;
        if (exact_pow) {
            gr = rclamp(powf(acc.r, ig));
            gg = rclamp(powf(acc.g, ig));
            gb = rclamp(powf(acc.b, ig));
        }
        if (out_rgba8) {
            const uint32_t px = exact_pow ? (to_u8(gr) | (to_u8(gg) << 8) | (to_u8(gb) << 16) | (to_u8(ga) << 24))
                                          : (gamma22_u8(acc.r) | (gamma22_u8(acc.g) << 8) | (gamma22_u8(acc.b) << 16) |
                                             (to_u8(ga) << 24));
            if (kp.flags & kFlagSlabRgb24) {  // gather slab, alpha proven 255: 3 bytes per pixel
                uint8_t* b = reinterpret_cast<uint8_t*>(out_rgba8) + 3u * o;
                b[0] = (uint8_t)px;
                b[1] = (uint8_t)(px >> 8);
                b[2] = (uint8_t)(px >> 16);
            } else if (kp.flags & kFlagHostStore) {  // zero-copy frame: out now, not at the kernel's end
                __hip_atomic_store(out_rgba8 + o, px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                out_rgba8[o] = px;
            }
        }
        if (out_f32 && !stamps) {
            if (kp.flags & RRTE_FLAG_F32_LINEAR)
                out_f32[o] = make_float4(acc.r, acc.g, acc.b, acc.a);
            else
                out_f32[o] = make_float4(gr, gg, gb, ga);
        }
    }
    if (MODE != RRTE_MODE_REFCOMPAT) {
        // wave-reduce the shadow-ray count, one atomic per wave
        uint32_t v = nshadow;  // (DPP row sums, then the four rows' lanes: as wave_min)
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
        v = (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
            (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
        // 256 counter shards, one 128-B line each: same-address atomics from
        // every wave of the grid would serialise at the memory side.
        if (lane == 0 && v) {
            const uint32_t shard = (tile.x + tile.y * tiles_x + threadIdx.x / 64u * 61u) & (kCounterShards - 1u);
            atomicAdd(counters + shard * kCounterStride, (unsigned long long)v);
        }
    }
    if (kWg64 && kp.tile_cost && tile.z == 0u && lane == 0)  // tile profile (TileProfile, rrte_hip.hip)
        kp.tile_cost[brow * tiles_x + tile.x] = (uint32_t)(wall_clock64() - t_wave0);
    if (stamps && lane == 0) {
        const uint64_t t1 = wall_clock64();
        const uint32_t wid = (brow * tiles_x + tile.x) * 4u + wave;
        uint32_t* s = reinterpret_cast<uint32_t*>(out_f32) + 4u * wid;
        s[0] = (uint32_t)t_wave0;
        s[1] = (uint32_t)(t_wave0 >> 32);
        s[2] = (uint32_t)(t1 - t_wave0);
        s[3] = __smid();
    }
}

// Generic kernel: the scene is read from HBM through wave-uniform (scalar) loads; F = the features
// compiled in (kFeat*, a superset of the scene's).
// Register budget of the generic kernel (waves per SIMD it must fit): 5 (<= 96 VGPRs, a few spills)
// instead of the compiler's 4 -- frames in a stream 0.172 -> 0.164 ms per 1080p showcase frame, a lone
// launch +13 % -- and, once the scene records were scalar loads, 6 (<= 80 VGPRs) for LAMBERT_SHADOW
// variants without meshes or deformers: 0.139 -> 0.131 ms; with meshes (+39 %) or deformers (+5 %) 6 waves
// lose, so those keep 5, as do the REFCOMPAT variants (6 waves: one sample -3 %, the reference's stock config
// spp 4 / depth 50 +6 %; DESIGN.md §13, tools/mw_check.sh, tools/refc_check.sh)
#ifndef RRTE_GENERIC_MINWAVES
#define RRTE_GENERIC_MINWAVES 5
#endif
#ifndef RRTE_GENERIC_MINWAVES_PLAIN
#define RRTE_GENERIC_MINWAVES_PLAIN 6
#endif
template <int MODE, uint32_t F>
constexpr int generic_min_waves() {
    return MODE == RRTE_MODE_LAMBERT_SHADOW && (F & (kFeatMesh | kFeatDeform)) == 0u ? RRTE_GENERIC_MINWAVES_PLAIN
                                                                                        : RRTE_GENERIC_MINWAVES;
}
template <int MODE, bool CULL, uint32_t F = kFeatAll>
__global__ __launch_bounds__(kBlockThreads, (generic_min_waves<MODE, F>())) void ray_kernel(KParams kp, SceneView sc, Cull cl, uint32_t* __restrict__ out_rgba8,
                                                  float4* __restrict__ out_f32,
                                                  unsigned long long* __restrict__ counters) {
    SceneViewF<F> s;
    static_cast<SceneView&>(s) = sc;
    ray_kernel_body<MODE, SceneViewF<F>, false, CULL>(kp, s, cl, out_rgba8, out_f32, counters);
}

// Root-side de-interleave after the RCCL gather: the gathered buffer holds, per rank (rank_stride
// bytes each; rank `skip_rank`'s rows -- the root's, rendered in place -- are skipped, ~0u for none),
// that rank's packed rows of `gridDim.z` frames back to back (frame_stride bytes each,
// `rows_cap` rows of RGBA8 or RGB24 per frame); frame z goes to full[z] (one frame per launch for
// per-frame gathers, a batch's frames for rrte_hip_set_gather_batch).  RGB24 slabs are expanded
// with alpha 255 (the host proved every alpha byte is 255).  VEC4: each lane moves 4 pixels (three
// dword loads for RGB24 or one dwordx4, one dwordx4 store) instead of 4 byte-wise pixels -- the
// host picks it when the width is a multiple of 4 and every target is 16-byte aligned (the slab
// strides are 256-byte aligned).  One workgroup row per image row, blockIdx.x strides the row.
struct DeinterleaveTargets {
    uint32_t* full[16];
};
template <bool RGB24, bool VEC4>
__global__ __launch_bounds__(256) void deinterleave_batch_kernel(const uint8_t* __restrict__ gathered,
                                                                 DeinterleaveTargets t, uint32_t width,
                                                                 BandMap bm, size_t rank_stride, size_t frame_stride,
                                                                 uint32_t skip_rank) {
    const uint32_t y = blockIdx.y;
    const uint32_t band_rows = bm.band_rows;
    const uint32_t band = y / band_rows, w = y - band * band_rows;
    uint32_t local_band = 0;
    const uint32_t rank = band_owner(bm, band, local_band);
    if (rank == skip_rank) return;  // the root's own bands: rendered into the frame in place
    const uint32_t lr = local_band * band_rows + w;
    constexpr uint32_t bpp = RGB24 ? 3u : 4u;
    const uint8_t* src = gathered + (size_t)rank * rank_stride + (size_t)blockIdx.z * frame_stride +
                         (size_t)lr * width * bpp;
    uint32_t* dst = t.full[blockIdx.z] + (size_t)y * width;
    const uint32_t step = gridDim.x * blockDim.x;
    if constexpr (VEC4) {
        const uint32_t n4 = width >> 2;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += step) {
            uint4 o;
            if constexpr (RGB24) {
                // pixels 4i..4i+3 = bytes 12i..12i+11 = dwords 3i..3i+2 (little endian)
                const uint32_t* q = reinterpret_cast<const uint32_t*>(src) + 3u * i;
                const uint32_t d0 = __builtin_nontemporal_load(q), d1 = __builtin_nontemporal_load(q + 1),
                               d2 = __builtin_nontemporal_load(q + 2);
                o.x = d0 | 0xFF000000u;
                o.y = (d0 >> 24) | (d1 << 8) | 0xFF000000u;
                o.z = (d1 >> 16) | (d2 << 16) | 0xFF000000u;
                o.w = (d2 >> 8) | 0xFF000000u;
            } else {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
                o = make_uint4(v.x, v.y, v.z, v.w);
            }
            reinterpret_cast<uint4*>(dst)[i] = o;
        }
    } else {
        for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < width; x += step) {
            if constexpr (RGB24) {
                const uint8_t* q = src + 3u * x;
                dst[x] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | 0xFF000000u;
            } else {
                dst[x] = reinterpret_cast<const uint32_t*>(src)[x];
            }
        }
    }
}

}  // namespace rrte
