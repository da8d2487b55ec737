// device_scene.hpp — device-side scene records and f32 math for the gfx950
// ray kernels.  Every arithmetic expression below keeps the operation order
// of the reference (cited file:line, paths relative to Melthizar/RRTE) so the
// kernel is bit-identical to the reference algorithm wherever the reference
// is deterministic; the library is compiled with -ffp-contract=off and the
// HIP default correctly-rounded f32 divide/sqrt.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "../../include/rrte_hip.h"

namespace rrte {

// ------------------------------------------------------------------ records
// Device copy of one SceneObject.  Read with wave-uniform indices, so the
// compiler serves it from the scalar cache into SGPRs (s_load_dwordx*):
// every lane of a wave tests the same object at the same time.
struct alignas(16) DPrim {
    uint32_t kind;
    int32_t material;
    uint32_t sdf_first;
    uint32_t sdf_count;
    uint32_t sdf_max_steps;
    float sdf_step_scale;
    float sdf_hit_eps;
    uint32_t flags;          // bit0: transform is identity
    float p[20];
    float xf[12];            // Transform::to_matrix, columns x,y,z,w (xyz each)
    float inv[12];           // Transform::inverse_matrix
    float _pad[12];
};
static_assert(sizeof(DPrim) == 256, "DPrim layout");

enum : uint32_t { DPRIM_IDENTITY_XF = 1u };

struct alignas(16) DMaterial {
    uint32_t kind;
    float fuzz;
    float ior;
    float _pad0;
    float albedo[4];
};
static_assert(sizeof(DMaterial) == 32, "DMaterial layout");

struct alignas(16) DLight {
    uint32_t kind;
    float intensity, range, linear, quadratic, inner_angle, outer_angle, _pad0;
    float position[4];
    float direction[4];
    float color[4];
    float cI[4];             // color * intensity (light.rs:189), 4 channels
};
static_assert(sizeof(DLight) == 96, "DLight layout");

// The camera of one frame (camera.rs:24-31 after Camera::look_at; the per-frame part of the launch
// constants) with its camera-ray tile-culling table.
struct FrameCam {
    uint32_t projection;
    float cam_pos[3];
    float cam_rot[4];
    float half_h, aspect;
    float ortho_l, ortho_r, ortho_b, ortho_t;
    float cam_xf[12];
    // Camera-ray tile culling (perspective frames, objects [0, tile_n), tile_n <= 32): object i's
    // bounding sphere projects inside the tile rectangle tile_rect[i] = bx0 | bx1 << 8 | by0 << 16 |
    // by1 << 24 (inclusive, conservative; tiles of 1 << tile_cull pixels: 3 = 8x8 per wave,
    // 4 = 16x16, four 8x8 workgroups); a tile outside it cannot hit object i with a camera ray.  0: off.
    uint32_t tile_cull, tile_n;
    uint32_t tile_rect[32];
    // KParams::out_image_rows launches: this frame's RGBA8 frame buffer (the batched multi-GPU root
    // renders its own bands straight into each frame's caller buffer)
    uint32_t* out;
};

// A launch renders up to kMaxLaunchFrames frames of one scene with the same parameters and their own
// cameras (blockIdx.y = frame; batched multi-GPU frames, rrte_hip_set_gather_batch).
constexpr uint32_t kMaxLaunchFrames = 8;

// Measured-cost tile order (KParams::hot): slot k of a launch renders the tile packed in hot[k] as
// y << 16 | x (tile columns and rows < 65536).  A list covers every tile of the launch shape once.
__host__ __device__ constexpr uint32_t hot_pack(uint32_t x, uint32_t y) { return (y << 16) | x; }
__host__ __device__ constexpr uint32_t hot_x(uint32_t h) { return h & 0xffffu; }
__host__ __device__ constexpr uint32_t hot_y(uint32_t h) { return h >> 16; }

// Multi-GPU row-band partition (DESIGN.md §5 "Band partition").  The image is cut into
// bands of `band_rows` rows.  The first `sky` bands -- rows no object can reach, judged on the host
// from the camera and the objects' culling spheres, so every camera ray there misses (the cheapest
// rows of the frame) -- belong to rank 0 (the root: its rows never cross a link).  The remaining
// bands go round robin in cycles of L = root_bands + (nranks - 1) peer_bands bands: first
// `root_bands` for the root, then `peer_bands` rounds of one band per peer.  sky = 0, root_bands =
// peer_bands = 1 is the plain interleave band % nranks == rank; a smaller root share frees the root
// for the expansion of the peers' rows it does per frame.  Which rank renders a band never changes a
// pixel.
struct BandMap {
    uint32_t band_rows, nranks, sky, root_bands, peer_bands;
};
__host__ __device__ constexpr uint32_t band_cycle(const BandMap& m) {
    return m.root_bands + (m.nranks - 1u) * m.peer_bands;
}
// The image band of `rank`'s local band lb.
__host__ __device__ constexpr uint32_t band_of_local(const BandMap& m, uint32_t rank, uint32_t lb) {
    const uint32_t L = band_cycle(m);
    if (rank == 0u) {
        if (lb < m.sky) return lb;
        const uint32_t t = lb - m.sky;
        return m.sky + (t / m.root_bands) * L + t % m.root_bands;
    }
    return m.sky + (lb / m.peer_bands) * L + m.root_bands + (rank - 1u) + (lb % m.peer_bands) * (m.nranks - 1u);
}
// The rank owning image band b and its local band index there.
__host__ __device__ constexpr uint32_t band_owner(const BandMap& m, uint32_t b, uint32_t& lb) {
    if (b < m.sky || m.nranks <= 1u) {
        lb = b;
        return 0u;
    }
    const uint32_t L = band_cycle(m), q = b - m.sky, cyc = q / L, slot = q % L;
    if (slot < m.root_bands) {
        lb = m.sky + cyc * m.root_bands + slot;
        return 0u;
    }
    const uint32_t s = slot - m.root_bands;
    lb = cyc * m.peer_bands + s / (m.nranks - 1u);
    return 1u + s % (m.nranks - 1u);
}

// Per-launch constants, passed by value (kernel arguments land in SGPRs).
struct KParams {
    uint32_t width, height;
    uint32_t spp, max_depth;
    uint32_t jitter, seed, flags;
    uint32_t num_prims, num_lights, num_materials;
    // row mapping: local row r -> image row (band interleave for multi-GPU)
    uint32_t rows;           // rows this launch renders
    uint32_t band_rows;      // 0 = identity mapping (+ row0)
    uint32_t nranks, rank;
    uint32_t sky_bands, root_bands, peer_bands;  // band partition (BandMap) of multi-GPU frames
    uint32_t row0;           // first image row of this launch (row-chunked blocking renders; band_rows == 0)
    float bg[4];
    float t_min, bias, inv_gamma, inv_spp;
    uint32_t debug;          // RRTE_DEBUG ablation bits (diagnostics only, 0 in production)
    uint32_t nframes;        // frames of this launch (gridDim.y), cam[0 .. nframes)
    uint64_t frame_stride;   // bytes between consecutive frames' RGBA8 / slab outputs
    // Tile order of 64-thread-workgroup launches: grid (tiles_x, nframes, tile rows).  With a list
    // (hot != nullptr) workgroup slot k = blockIdx.z * tiles_x + blockIdx.x renders tile hot[k] of its
    // frame -- every tile, slowest first as an earlier launch of the same shape measured them
    // (rrte_hip.hip, TileProfile); without one, tile (blockIdx.x, blockIdx.z).  Pixels are
    // independent (raytracer.rs:57-60), so any order renders the same bytes; this one starts the
    // frame's longest waves first instead of wherever image order puts them.
    uint32_t* tile_cost;     // non-null: frame 0's workgroups store their duration (100 MHz ticks) at [y * tiles_x + x]
    const uint32_t* hot;     // device tile list (immutable while launches use it)
    uint32_t tiles_x, hot_n;
    // The list is stored XCD-major: slot k at hot[(k & 7) * hot_stride + (k >> 3)].  Workgroups are
    // dispatched round-robin over the 8 XCDs (slot k on XCD k mod 8 when the slot rows are a multiple
    // of 8 tiles wide), and each XCD has its own L2: in slot order every 64-B line of the list held
    // slots of all 8 XCDs, so every XCD fetched the whole list (~1 MB of HBM reads per 1080p launch,
    // PMC FETCH_SIZE); XCD-major, each XCD reads only its own eighth.
    uint32_t hot_stride;
    // Tile shape of 64-thread workgroups: 1 << tile_shift pixels wide, 64 >> tile_shift rows (3: the 8x8
    // tiles of every frame path; 5: 32x2, each wave storing two whole 128-B lines of RGBA8 -- the
    // blocking path's zero-copy stores into pinned host memory cross PCIe as full lines)
    uint32_t tile_shift;
    // Output rows: 0 = this launch's rows packed (row r at r * width, frame z at out + z * frame_stride),
    // 1 = at their image rows of frame z's own buffer cam[z].out (image_row(r) * width: a multi-GPU
    // root renders its own bands straight into the final frames; RGBA8 only)
    uint32_t out_image_rows;
    FrameCam cam[kMaxLaunchFrames];
};
static_assert(sizeof(KParams) <= 3584, "kernel arguments stay below the 4 KB kernarg limit");

// Internal KParams::flags bit (never in the public rrte_render_params::flags): the launch writes
// a gather slab of packed RGB24 pixels (3 B, alpha dropped) instead of RGBA8.  The host sets it
// only when it has proved every pixel's alpha byte is 255 (rrte_hip.hip, slab_rgb24), and the
// root's de-interleave puts the 255 back.
constexpr uint32_t kFlagSlabRgb24 = 1u << 31;
// Internal: the RGBA8 output is pinned HOST memory (the blocking entry point's zero-copy frame).  Its
// pixel stores go out at system scope (write-through cache policy): plain stores into host memory
// were measured to leave only at the kernel's end (tools/micro/zc_write.hip: no overlap with the
// compute of waves still running), system-scope ones while the frame renders.
constexpr uint32_t kFlagHostStore = 1u << 30;


// ---------------------------------------------------------------- f32 vec3
struct f3 { float x, y, z; };

__device__ __forceinline__ f3 V(float x, float y, float z) { return f3{x, y, z}; }
// Out-of-range fallback of the short correctly rounded sequences below: a divergent branch around the
// compiler's full sequence (an EXEC save, branch and restore on the scalar unit per call), or with
// RRTE_GUARD_UNIFORM a wave-uniform branch on the ballot of the out-of-range lanes that runs the full
// sequence on every lane and selects it for the flagged ones (bit-identical either way).
#ifndef RRTE_GUARD_UNIFORM
#define RRTE_GUARD_UNIFORM 0
#endif
#define RRTE_FALLBACK(bad, r, full)                                                            \
    do {                                                                                       \
        if (RRTE_GUARD_UNIFORM) {                                                              \
            const uint64_t m_ = __builtin_amdgcn_ballot_w64(bad);                              \
            if (__builtin_expect(m_ != 0ull, 0)) r = mask_select(m_, r, (full));               \
        } else if (__builtin_expect((bad), 0)) {                                               \
            r = (full);                                                                        \
        }                                                                                      \
    } while (0)
// Lane select on a wave mask held in SGPRs: lane i gets `b` if bit i of m is set, else `a` -- one
// v_cndmask_b32 reading the mask directly (what __builtin_amdgcn_inverse_ballot_w64 lowers to; the
// hiprtc front end of this ROCm does not know that builtin).
__device__ __forceinline__ float mask_select(uint64_t m, float a, float b) {
    float r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ __forceinline__ bool mask_lane(uint64_t m) { return mask_select(m, 0.0f, 1.0f) != 0.0f; }

// Correctly rounded f32 sqrt (Rust f32::sqrt), 7 VALU ops with its guard instead of the compiler's 16.
// Verified bit-identical to __builtin_sqrtf over all 2^32 inputs on gfx950 (rrte_hip_fpcheck,
// tests/test_gpu_fpexact.py).  (Round 1's form -- the neighbour of v_sqrt_f32 whose residual
// x - s*(s -/+ ulp) changes sign, guarded below 2^-96 -- took 11.)
// RRTE_ABLATE_FAST_SQRT swaps in the bare 1-ulp v_sqrt_f32 -- a timing experiment only
// (breaks parity), never a build setting.
// Branch-free form of the same residual correction (RRTE_FPCHECK_SQRT_BF sweeps it over all 2^32
// inputs): x below 2^-96 is scaled by 2^64 first and the root by 2^-32 after (both exact: the scaled
// x is a normal in [2^-85, 2^-32), its root a normal); +-0 and +inf, where rsq gives inf / 0 and
// s = x * y is NaN, return x through one v_cmp_class; negatives and NaNs come out NaN from rsq.  No
// EXEC save / restore, so neighbouring roots share basic blocks (and v_pk_mul / v_pk_fma pairs).
__device__ __forceinline__ float sqrt_rn_branchfree(float x) {
    const bool tiny = x < 0x1p-96f;
    const float xs = x * (tiny ? 0x1p+64f : 1.0f);
    const float y = __builtin_amdgcn_rsqf(xs);
    const float s = xs * y;
    const float e = __builtin_fmaf(-s, s, xs);
    const float r = __builtin_fmaf(e, 0.5f * y, s) * (tiny ? 0x1p-32f : 1.0f);
    return __builtin_amdgcn_classf(xs, 0x060 | 0x200) ? xs : r;  // +-0 (0x20, 0x40), +inf (0x200)
}
// The guarded form: one residual correction from a single transcendental: y = v_rsq_f32(x),
// s = x * y (faithful), e = x - s*s exactly (one fma), r = RN(s + e * h) with h = 0.5 * y ~
// 1/(2 sqrt x): 5 VALU ops, ONE of them transcendental (8 issue cycles against 4 for an fma; s from
// v_sqrt_f32 plus h from v_rsq_f32 took two).  Correctly rounded for every x in [2^-96, FLT_MAX]
// (tools/fpexact/sqrt_markstein.hip, candidate M3: only 0 and inf fail, both outside; below 2^-96 the
// residual underflows); every other x -- tiny, zero, denormal, negative, infinite, NaN -- takes the
// compiler's sequence in a divergent branch no real scene takes, chosen by one unsigned range test on
// the bits (positive floats order like their bit patterns; negatives and NaNs fall outside).
__device__ __forceinline__ float sqrt_rn_guarded(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float e = __builtin_fmaf(-s, s, x);
    float r = __builtin_fmaf(e, 0.5f * y, s);
    // (a single v_cmp_class guard -- every x but a positive normal -- is not enough: 10.2 M normal
    // inputs below 2^-96 come out wrong, tests/test_gpu_fpexact.py)
    constexpr uint32_t kLo = 0x0F800000u, kInf = 0x7F800000u;  // bits of 2^-96 and +inf
#ifndef RRTE_ABLATE_NO_GUARDS  // timing experiment only: drops the out-of-range fallback branches
    RRTE_FALLBACK(__float_as_uint(x) - kLo >= kInf - kLo, r, __builtin_sqrtf(x));
#endif
    return r;
}
// Correctly rounded f32 sqrt (Rust f32::sqrt).  Both forms are verified bit-identical to
// __builtin_sqrtf over all 2^32 inputs on gfx950 (rrte_hip_fpcheck, tests/test_gpu_fpexact.py).
// RRTE_SQRT_GUARDED selects the guarded form (A/B); RRTE_ABLATE_FAST_SQRT swaps in the bare 1-ulp
// v_sqrt_f32 -- a timing experiment only (breaks parity), never a build setting.
#ifdef RRTE_ABLATE_FAST_SQRT
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_amdgcn_sqrtf(x); }
#elif defined(RRTE_SQRT_BRANCHFREE)
__device__ __forceinline__ float sqrt_rn(float x) { return sqrt_rn_branchfree(x); }
#else
__device__ __forceinline__ float sqrt_rn(float x) { return sqrt_rn_guarded(x); }
#endif
// Correctly rounded 1/b: v_rcp_f32 and one Newton fma step is exact for every b with
// |b| in [2^-126, 2^126] (rrte_hip_fpcheck: all 2^32 inputs on gfx950); zeros,
// denormals, huge values, inf and NaN take the compiler's full divide.  5 VALU ops instead of 11.
__device__ __forceinline__ float rcp_rn(float b) {
    if (__builtin_constant_p(b)) return 1.0f / b;
    float y = __builtin_amdgcn_rcpf(b);
    y = __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
#ifndef RRTE_ABLATE_NO_GUARDS
    RRTE_FALLBACK(!(__builtin_fabsf(b) >= 0x1.0p-126f && __builtin_fabsf(b) <= 0x1.0p+126f), y, 1.0f / b);
#endif
    return y;
}
// Correctly rounded a/b.  When b folds to a constant (scene-specialised kernels: SDF and
// primitive parameters), y = RN(1/b) is a constant and q = RN(a*y), r = a - b*q (exact fma),
// RN(q + r*y) is the correctly rounded quotient for every a with |a| in [2^-60, 2^60] and
// |b| in [2^-60, 2^60] (Markstein; checked over all 2^46 significand pairs on gfx950,
// rrte_hip_fpcheck -- the steps are correctly rounded, so the result is
// exponent-invariant inside that range).  Other a take the full divide.  Runtime divisors
// keep the compiler's sequence (a guarded short form would not be shorter).
__device__ __forceinline__ float div_by_rcp(float a, float b, float y) {  // y = RN(1/b)
    const float q = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ float div_rn(float a, float b) {
    if (__builtin_constant_p(b) && __builtin_fabsf(b) >= 0x1.0p-60f && __builtin_fabsf(b) <= 0x1.0p+60f) {
        float r = div_by_rcp(a, b, 1.0f / b);
#ifndef RRTE_ABLATE_NO_GUARDS
        RRTE_FALLBACK(!(__builtin_fabsf(a) >= 0x1.0p-60f && __builtin_fabsf(a) <= 0x1.0p+60f), r, a / b);
#endif
        return r;
    }
    return a / b;
}
// Guard policies of the SDF evaluation (ray_kernels.hpp: sdf_leaf ... SdfStaticProgram::eval).
// GuardNow: sqrt_rn / div_rn as above, each with its own divergent fallback branch (an EXEC save,
// branch and restore on the scalar unit per call).  GuardDefer: the same short sequences, but each
// range test only folds into a running unsigned max of (bits - lower bound) -- one v_sub + v_max_u32,
// nothing on the scalar unit -- and the caller tests bad() once per evaluation and re-evaluates the
// flagged lanes with GuardSlow (the compiler's full sequences: bit-identical to the short ones
// wherever those are in range, so any lane may take it).  A value is in range iff bits(x) - LO
// <= SPAN as unsigned integers (positive floats order like their bit patterns; negatives and NaNs
// wrap above), exactly the tests of sqrt_rn / div_rn.
struct GuardNow {
    __device__ __forceinline__ float sqrt(float x) { return sqrt_rn(x); }
    __device__ __forceinline__ float div(float a, float b) { return div_rn(a, b); }
};
struct GuardSlow {
    __device__ __forceinline__ float sqrt(float x) { return __builtin_sqrtf(x); }
    __device__ __forceinline__ float div(float a, float b) { return a / b; }
};
struct GuardDefer {
    static constexpr uint32_t kSqrtLo = 0x0F800000u, kSqrtSpan = 0x7F800000u - 0x0F800000u - 1u;  // [2^-96, FLT_MAX]
    static constexpr uint32_t kDivLo = 0x21800000u, kDivSpan = 0x5D800000u - 0x21800000u;          // |a| in [2^-60, 2^60]
    uint32_t sq = 0u, dv = 0u;
    __device__ __forceinline__ float sqrt(float x) {
        const float y = __builtin_amdgcn_rsqf(x);
        const float s = x * y;
        const float e = __builtin_fmaf(-s, s, x);
        sq = __builtin_elementwise_max(sq, __float_as_uint(x) - kSqrtLo);
        return __builtin_fmaf(e, 0.5f * y, s);
    }
    __device__ __forceinline__ float div(float a, float b) {
        if (__builtin_constant_p(b) && __builtin_fabsf(b) >= 0x1.0p-60f && __builtin_fabsf(b) <= 0x1.0p+60f) {
            dv = __builtin_elementwise_max(dv, __float_as_uint(__builtin_fabsf(a)) - kDivLo);
            return div_by_rcp(a, b, 1.0f / b);
        }
        return a / b;
    }
    __device__ __forceinline__ bool bad() const { return sq > kSqrtSpan || dv > kDivSpan; }
};

__device__ __forceinline__ f3 vadd(f3 a, f3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 vsub(f3 a, f3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 vneg(f3 a) { return V(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 vmuls(f3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 vdivs(f3 a, float s) { return V(div_rn(a.x, s), div_rn(a.y, s), div_rn(a.z, s)); }
// glam Vec3::dot, left to right
__device__ __forceinline__ float vdot(f3 a, f3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
__device__ __forceinline__ float vlen2(f3 a) { return vdot(a, a); }
__device__ __forceinline__ float vlen(f3 a) { return sqrt_rn(vdot(a, a)); }
// glam Vec3::normalize: self * (1 / length())
__device__ __forceinline__ f3 vnorm(f3 a) { return vmuls(a, rcp_rn(sqrt_rn(vdot(a, a)))); }
__device__ __forceinline__ f3 vcross(f3 a, f3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
__device__ __forceinline__ f3 vld(const float* p) { return V(p[0], p[1], p[2]); }
__device__ __forceinline__ float comp(f3 a, uint32_t i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ f3 setcomp(f3 a, uint32_t i, float s) {
    if (i == 0) a.x = s; else if (i == 1) a.y = s; else a.z = s;
    return a;
}
__device__ __forceinline__ float mn(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float mx(float a, float b) { return (b > a) ? b : a; }
__device__ __forceinline__ float clampf_(float x, float lo, float hi) { return mn(mx(x, lo), hi); }
// SDF min/max (build-defined): IEEE-754 minNum/maxNum (a NaN operand yields the other),
// one v_min_f32 / v_max_f32 / v_max3_f32 / v_med3_f32 each instead of a compare + select; the oracle's
// smn/smx are fminf/fmaxf.  Zero-sign of a +-0 tie unspecified (no SDF output depends on it).
__device__ __forceinline__ float smn(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float smx(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float sclamp(float x, float lo, float hi) { return smn(smx(x, lo), hi); }

// vnorm for a vector already normalised once (|w|^2 within a few ulp of 1: a light direction, a
// rotated unit camera direction), bit-identical to vnorm: with x = fl(w.w) and k = bits(x) -
// bits(1.0f), RN(1 / RN(sqrt(x))) has the bits 0x3F800000 - (k >= 0 ? k & ~1 : k >> 2) for every
// |k| <= 1024 (sqrt(1 + d) = 1 + d/2 - d^2/8: RN keeps 1 + floor(k/2) ulp above 1 or rounds half an ulp
// below 1 away from it, and the reciprocal folds back the same way; checked exhaustively,
// tests/test_fpexact_cpu.py, first failure at |k| = 2898).  Five integer ops replace the sqrt and
// reciprocal sequences (12 VALU ops, two guards); other x take vnorm in a divergent branch.
__device__ __forceinline__ f3 vnorm_unit(f3 w) {
    const float x = vdot(w, w);
    const int k = (int)__float_as_uint(x) - 0x3F800000;
    float r = __int_as_float(0x3F800000 - (k >= 0 ? (k & ~1) : (k >> 2)));
#ifndef RRTE_ABLATE_NO_GUARDS
    if (__builtin_expect((uint32_t)(k + 1024) > 2048u, 0)) r = rcp_rn(sqrt_rn(x));
#endif
    return vmuls(w, r);
}

struct Ray { f3 o, d; };
// Ray::new normalises (ray.rs:13-18); Ray::at (ray.rs:21-23)
__device__ __forceinline__ Ray ray_new(f3 o, f3 d) { return Ray{o, vnorm(d)}; }
// Ray::new for a direction already of unit length up to rounding (vnorm_unit)
__device__ __forceinline__ Ray ray_new_unit(f3 o, f3 d) { return Ray{o, vnorm_unit(d)}; }
__device__ __forceinline__ f3 ray_at(const Ray& r, float t) { return vadd(r.o, vmuls(r.d, t)); }

__device__ __forceinline__ bool finite3(f3 a) {
    return __builtin_isfinite(a.x) && __builtin_isfinite(a.y) && __builtin_isfinite(a.z);
}

struct Hit { float t; f3 p, n; bool front; uint32_t sub; };  // sub: mesh triangle slot of the hit
// HitInfo::new (ray.rs:45-56)
__device__ __forceinline__ void hit_new(Hit& h, float t, f3 p, f3 outward, const Ray& r) {
    h.t = t;
    h.p = p;
    h.front = vdot(r.d, outward) < 0.0f;
    h.n = h.front ? outward : vneg(outward);
}

// Mat4 (3x4 affine part, columns x,y,z,w) transform_point3 / transform_vector3
__device__ __forceinline__ f3 m_point(const float* m, f3 p) {
    return V(((m[0] * p.x + m[3] * p.y) + m[6] * p.z) + m[9],
             ((m[1] * p.x + m[4] * p.y) + m[7] * p.z) + m[10],
             ((m[2] * p.x + m[5] * p.y) + m[8] * p.z) + m[11]);
}
__device__ __forceinline__ f3 m_vector(const float* m, f3 p) {
    return V((m[0] * p.x + m[3] * p.y) + m[6] * p.z,
             (m[1] * p.x + m[4] * p.y) + m[7] * p.z,
             (m[2] * p.x + m[5] * p.y) + m[8] * p.z);
}

// Quat * Vec3 (glam mul_vec3a): v*(w*w - b.b) + b*((v.b)*2) + (b x v)*(w*2)
__device__ __forceinline__ f3 quat_rotate(const float* q, f3 v) {
    f3 b = V(q[0], q[1], q[2]);
    float w = q[3];
    float b2 = vdot(b, b);
    float k0 = w * w - b2;
    float k1 = vdot(v, b) * 2.0f;
    float k2 = w * 2.0f;
    f3 c = vcross(b, v);
    return vadd(vadd(vmuls(v, k0), vmuls(b, k1)), vmuls(c, k2));
}

// ------------------------------------------------------ build-defined trig
// Deterministic sin/cos shared bit-for-bit with the oracle.
__device__ __forceinline__ void sincos_rrte(float x, float& so, float& co) {
    float k = floorf(x * 0.636619772f + 0.5f);
    float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.549789948768648e-8f;
    float r2 = r * r;
    float s = r + (r * r2) * (-1.6666654611e-1f + r2 * (8.3321608736e-3f + r2 * -1.9515295891e-4f));
    float c = (1.0f - 0.5f * r2) +
              (r2 * r2) * (4.166664568298827e-2f + r2 * (-1.388731625493765e-3f + r2 * 2.443315711809948e-5f));
    int q = ((int)k) & 3;
    float s_ = s, c_ = c;
    so = (q == 0) ? s_ : (q == 1) ? c_ : (q == 2) ? -s_ : -c_;
    co = (q == 0) ? c_ : (q == 1) ? -s_ : (q == 2) ? -c_ : s_;
}

// Three-channel value noise (build-defined, DESIGN.md §6 'Deformers'; oracle rrte_oracle_value_noise3):
// every lattice corner has ONE 32-bit hash of (seed, corner) whose bits give its three values in
// [-1, 1) -- bits 0-10 and 11-21 (step 2^-10), bits 22-31 (step 2^-9) -- each channel interpolated
// trilinearly with the smoothstep fade.  (Rounds 1-5 hashed each channel separately: three times the
// integer work, ~45 % of the deformation-stress frame)
// The corner's seed-independent part of the hash (xor is associative and commutative, so
// seed ^ corner_key is the word seed ^ ix*A ^ iy*B ^ iz*C of the oracle in any grouping).
__device__ __forceinline__ uint32_t corner_key(int32_t ix, int32_t iy, int32_t iz) {
    return ((uint32_t)ix * 0x8da6b343u ^ (uint32_t)iy * 0xd8163841u) ^ (uint32_t)iz * 0xcb1ab31fu;
}
__device__ __forceinline__ uint32_t lattice_mix(uint32_t h) {
    h = (h ^ (h >> 16)) * 0x7feb352du;
    h = (h ^ (h >> 15)) * 0x846ca68bu;
    return h ^ (h >> 16);
}
__device__ __forceinline__ float lerpf_(float a, float b, float t) { return a + (b - a) * t; }
__device__ __forceinline__ void value_noise3(float x, float y, float z, uint32_t seed, float out[3]) {
    float fx0 = floorf(x), fy0 = floorf(y), fz0 = floorf(z);
    int32_t ix = (int32_t)fx0, iy = (int32_t)fy0, iz = (int32_t)fz0;
    float fx = x - fx0, fy = y - fy0, fz = z - fz0;
    const float ux = fx * fx * (3.0f - 2.0f * fx);
    const float uy = fy * fy * (3.0f - 2.0f * fy);
    const float uz = fz * fz * (3.0f - 2.0f * fz);
    float v[3][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t h = lattice_mix(seed ^ corner_key(ix + (j & 1), iy + ((j >> 1) & 1), iz + ((j >> 2) & 1)));
        v[0][j] = (float)(h & 0x7ffu) * 0x1p-10f - 1.0f;
        v[1][j] = (float)((h >> 11) & 0x7ffu) * 0x1p-10f - 1.0f;
        v[2][j] = (float)(h >> 22) * 0x1p-9f - 1.0f;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x00 = lerpf_(v[k][0], v[k][1], ux), x10 = lerpf_(v[k][2], v[k][3], ux);
        float x01 = lerpf_(v[k][4], v[k][5], ux), x11 = lerpf_(v[k][6], v[k][7], ux);
        float y0 = lerpf_(x00, x10, uy), y1 = lerpf_(x01, x11, uy);
        out[k] = lerpf_(y0, y1, uz);
    }
}

// ---------------------------------------------------------------- RNG
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
__device__ __forceinline__ float rng_f32(uint32_t& st) {
    st = st * 747796405u + 2891336453u;
    uint32_t s = st;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    w = (w >> 22u) ^ w;
    return (float)(w >> 8) * 5.9604644775390625e-8f;
}

}  // namespace rrte
