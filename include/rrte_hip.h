/*
 * rrte_hip.h — C ABI of the MI355X-native replacement for rrte-renderer's
 * per-pixel ray->scene loop.
 *
 * Replaces (reference paths relative to Melthizar/RRTE @ 2025-06-14):
 *   Raytracer::new / update_config / render
 *       crates/rrte-renderer/src/raytracer.rs:35-51 (render 45-89, ray_color 92-148)
 *   SceneObject::intersect for Sphere/Plane/Triangle/Cube/Cylinder/Cone/Capsule
 *       crates/rrte-renderer/src/primitives.rs:6-18, 57-725
 *   Light::illuminate (PointLight / Directional / Spot / Ambient)
 *       crates/rrte-renderer/src/light.rs:5-26, 87-121, 182-194, 288-338, 364-397
 *   Material::albedo / ambient_color
 *       crates/rrte-renderer/src/material.rs:5-19, 55-81
 *   Camera::generate_ray   crates/rrte-renderer/src/camera.rs:98-133
 *   SDF / CSGOperation / Deformer (README-only in the reference:
 *       README.md:458-510; build-defined here)
 *
 * Conventions
 *   - Plain C, POD structs, caller owns every buffer it passes in.
 *   - A context owns device memory and its HIP stream; one context per
 *     host thread (not internally synchronised).  Multi-GPU composition is
 *     internal to a context once rrte_hip_comm_init has been called.
 *   - No exceptions, panics or aborts cross this ABI: every entry point
 *     returns an rrte_status; rrte_hip_last_error() has the message.
 *   - Output images are RGBA8, row-major, row 0 = top of the image
 *     (v = 0 -> ndc_y = +1, camera.rs:101), exactly the layout of the
 *     Vec<u8> returned by Raytracer::render (raytracer.rs:54-88).
 */
#ifndef RRTE_HIP_H
#define RRTE_HIP_H

#ifndef __HIPCC_RTC__ /* hiprtc (scene-specialised kernels) provides the fixed-width types itself */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define RRTE_ABI_VERSION 2u

/* ------------------------------------------------------------------ status */
typedef enum rrte_status {
    RRTE_OK = 0,
    RRTE_INVALID_ARG = 1,      /* null pointer, zero size, malformed SDF program, ... */
    RRTE_HIP_ERROR = 2,        /* any HIP runtime failure (message in last_error)     */
    RRTE_RCCL_ERROR = 3,       /* RCCL failure during multi-GPU composition            */
    RRTE_UNSUPPORTED_PRIM = 4, /* unknown prim kind / light kind / SDF op              */
    RRTE_NO_DEVICE = 5         /* no HIP device visible / device index out of range    */
} rrte_status;

/* --------------------------------------------------------------- prim kinds */
typedef enum rrte_prim_kind {
    RRTE_PRIM_SPHERE = 0,   /* primitives.rs:57-81   p: center[0..2], radius[3]            */
    RRTE_PRIM_PLANE = 1,    /* primitives.rs:133-149 p: point[0..2], unit normal[4..6]     */
    RRTE_PRIM_TRIANGLE = 2, /* primitives.rs:208-244 p: v0,v1,v2 [0..8], n0,n1,n2 [9..17]  */
    RRTE_PRIM_CUBE = 3,     /* primitives.rs:301-364 p: center[0..2], size[4..6] (full)    */
    RRTE_PRIM_CYLINDER = 4, /* primitives.rs:419-465 p: center[0..2], radius[3], height[4] */
    RRTE_PRIM_CONE = 5,     /* primitives.rs:520-571 p: center[0..2], radius[3], height[4] */
    RRTE_PRIM_CAPSULE = 6,  /* primitives.rs:626-725 p: center[0..2], radius[3], height[4] */
    RRTE_PRIM_SDF = 7,      /* build-defined SDFObject: sphere-traced node program;
                               p: bounding sphere center[0..2], radius[3]                 */
    RRTE_PRIM_MESH = 8      /* triangle mesh (rrte-assets MeshAsset, asset.rs:53-65): triangles
                               sdf_first .. sdf_first+sdf_count-1 of rrte_scene_ir.mesh_indices
                               (3 vertex indices each).  Every triangle is Triangle::intersect
                               (primitives.rs:208-244) with set_normals(n0,n1,n2) -- the vertex
                               normals, already normalised by the caller -- and the mesh is the
                               closest hit over its triangles in index order (strict '<': the
                               lower index wins a tie), i.e. exactly a Vec<Triangle> in the
                               object list.  Like Triangle it ignores trs (bake the entity
                               transform into the vertices).  The device traverses a BVH built
                               once per scene; see DESIGN.md §5.                          */
} rrte_prim_kind;

/* One SceneObject lowered to POD (192 bytes).  trs is the object's
 * rrte_math::Transform {position, rotation quat (x,y,z,w), scale}
 * (transform.rs:6-10); Cube/Cylinder/Cone/Capsule apply it exactly as the
 * reference does (local ray through inverse_matrix, hit back through
 * to_matrix); Sphere/Plane/Triangle ignore it, as the reference does. */
typedef struct rrte_prim {
    uint32_t kind;           /* rrte_prim_kind                                      */
    int32_t material;        /* index into rrte_scene_ir.materials; -1 = none
                                (ray_color returns BLACK, raytracer.rs:139-143)     */
    uint32_t sdf_first;      /* SDF: index of this object's first node             */
    uint32_t sdf_count;      /* SDF: number of nodes in its postfix program        */
    uint32_t sdf_max_steps;  /* SDF: sphere-tracing step cap                        */
    float sdf_step_scale;    /* SDF: step multiplier (<1 for non-Lipschitz deformers) */
    float sdf_hit_eps;       /* SDF: relative hit epsilon: hit when d < eps * t     */
    uint32_t flags;          /* reserved, 0                                         */
    float p[20];             /* geometry, per kind (see rrte_prim_kind)             */
    float trs[10];           /* position[3], rotation quat xyzw[4], scale[3]        */
    float _pad[10];
} rrte_prim;

/* ----------------------------------------------------------------- materials */
typedef enum rrte_material_kind {
    RRTE_MAT_LAMBERTIAN = 0, /* material.rs:45-81   */
    RRTE_MAT_METAL = 1,      /* material.rs:85-120  */
    RRTE_MAT_DIELECTRIC = 2, /* material.rs:124-183 */
    RRTE_MAT_EMISSIVE = 3    /* material.rs:187-213 */
} rrte_material_kind;

typedef struct rrte_material {
    uint32_t kind;       /* rrte_material_kind                               */
    float fuzz;          /* metal roughness                                  */
    float ior;           /* dielectric index of refraction                   */
    float _pad0;
    float albedo[4];     /* Material::albedo() as rrte_math::Color (r,g,b,a) */
} rrte_material;         /* 32 bytes */

/* -------------------------------------------------------------------- lights */
typedef enum rrte_light_kind {
    RRTE_LIGHT_POINT = 0,       /* light.rs:123-220 */
    RRTE_LIGHT_DIRECTIONAL = 1, /* light.rs:57-121  */
    RRTE_LIGHT_SPOT = 2,        /* light.rs:222-338 */
    RRTE_LIGHT_AMBIENT = 3      /* light.rs:340-397 */
} rrte_light_kind;

typedef struct rrte_light {
    uint32_t kind;        /* rrte_light_kind                                   */
    float intensity;
    float range;          /* PointLight/SpotLight (default 100, light.rs:142)  */
    float linear;         /* linear_attenuation   (default 0.09)               */
    float quadratic;      /* quadratic_attenuation (default 0.032)             */
    float inner_angle;    /* SpotLight, radians                                */
    float outer_angle;    /* SpotLight, radians                                */
    float _pad0;
    float position[4];    /* xyz, w unused                                     */
    float direction[4];   /* Directional/Spot unit direction xyz               */
    float color[4];       /* rrte_math::Color (r,g,b,a)                        */
} rrte_light;             /* 80 bytes */

/* ---------------------------------------------------------- SDF node program */
/* An SDFObject's tree is flattened to postfix order.  Leaves push a distance
 * evaluated at the current point; CSG ops pop b, pop a, push op(a, b);
 * deformers save the current point and replace it with deform(point);
 * POP_POINT restores the saved point.  A Deformer chain d1.chain(d2)
 * (README.md:496-502) is emitted as d1, d2, <subtree>, POP_POINT, POP_POINT.
 * Value stack <= RRTE_SDF_MAX_STACK, point stack <= RRTE_SDF_MAX_POINT_STACK.
 * Formulas: DESIGN.md §SDF (build-defined; the reference has no SDF code). */
typedef enum rrte_sdf_op {
    RRTE_SDF_SPHERE = 1,    /* f: center[0..2], radius[3]                     */
    RRTE_SDF_BOX = 2,       /* f: center[0..2], size[4..6] (full extents)     */
    RRTE_SDF_CYLINDER = 3,  /* f: center, radius[3], height[4]  (Y axis)      */
    RRTE_SDF_PRISM = 4,     /* f: center, size[4..6] (triangle in XY, depth Z)*/
    RRTE_SDF_TORUS = 5,     /* f: center, major[3], minor[4]   (XZ plane)     */
    RRTE_SDF_TUBE = 6,      /* f: center, outer[3], inner[4], height[5]       */
    RRTE_SDF_RING = 7,      /* f: center, major[3], minor[4]   (XY plane)     */
    RRTE_SDF_CONE = 8,      /* f: center, radius[3], height[4] (apex +Y)      */
    RRTE_SDF_CAPSULE = 9,   /* f: center, radius[3], height[4] (Y axis)       */
    RRTE_SDF_ELLIPSOID = 10,/* f: center, radii[4..6]                         */

    RRTE_SDF_UNION = 32,
    RRTE_SDF_DIFFERENCE = 33,
    RRTE_SDF_INTERSECTION = 34,
    RRTE_SDF_SMOOTH_UNION = 35,        /* f[0] = k */
    RRTE_SDF_SMOOTH_DIFFERENCE = 36,   /* f[0] = k */
    RRTE_SDF_SMOOTH_INTERSECTION = 37, /* f[0] = k */

    RRTE_SDF_BEND = 64,  /* f: pivot[0..2], amount[3]; i: plane-normal axis[0], driving axis[1] */
    RRTE_SDF_TWIST = 65, /* f: pivot[0..2], rate[3];   i: axis[0]                            */
    RRTE_SDF_TAPER = 66, /* f: pivot[0..2], start[3], end[4], length[5]; i: axis[0]          */
    RRTE_SDF_NOISE = 67, /* f: pivot[0..2], frequency[3], amplitude[4], persistence[5];
                            i: octaves[0], seed[1]                                         */
    RRTE_SDF_WAVE = 68,  /* f: pivot[0..2], amplitude[3], frequency[4]; i: axis[0], displaced axis[1] */

    RRTE_SDF_POP_POINT = 96
} rrte_sdf_op;

#define RRTE_SDF_MAX_STACK 8
#define RRTE_SDF_MAX_POINT_STACK 4
#define RRTE_SDF_MAX_OCTAVES 8

typedef struct rrte_sdf_node {
    uint32_t op;      /* rrte_sdf_op */
    uint32_t i[3];    /* integer args (axes 0=X 1=Y 2=Z, octaves, seed) */
    float f[12];      /* float args */
} rrte_sdf_node;      /* 64 bytes */

/* -------------------------------------------------------------------- camera */
typedef enum rrte_projection { RRTE_PERSPECTIVE = 0, RRTE_ORTHOGRAPHIC = 1 } rrte_projection;

/* rrte_renderer::Camera (camera.rs:24-31): transform + projection. */
typedef struct rrte_camera {
    float position[3];
    uint32_t projection;   /* rrte_projection */
    float rotation[4];     /* quat x,y,z,w (Camera::look_at, camera.rs:85-95) */
    float scale[3];
    float fov;             /* radians */
    float aspect_ratio;
    float near_plane;
    float far_plane;
    float left, right, bottom, top; /* orthographic */
    float _pad[1];
} rrte_camera;             /* 80 bytes */

/* ------------------------------------------------------------ render params */
typedef enum rrte_mode {
    /* Reference formula (raytracer.rs:92-148): ambient albedo*0.01 + sum of
     * light.color*intensity*attenuation (no N.L, no shadows) + albedo *
     * ray_color(scatter, depth-1). */
    RRTE_MODE_REFCOMPAT = 0,
    /* north_star Lambert/shadow pass: ambient albedo*0.01 + sum over lights of
     * albedo * color*intensity * att * max(0, N.L) * visibility(shadow ray). */
    RRTE_MODE_LAMBERT_SHADOW = 1
} rrte_mode;

typedef enum rrte_jitter {
    RRTE_JITTER_CENTER = 0, /* xi = 0.5: deterministic parity config           */
    RRTE_JITTER_RANDOM = 1  /* counter-based RNG keyed by (seed, pixel, sample) */
} rrte_jitter;

#define RRTE_FLAG_F32_LINEAR 1u  /* f32 output holds the averaged linear colour (pre-gamma, unclamped) */
/* Accepted and ignored (ABI v2 compatibility).  It used to move each frame's gather onto a comm
 * stream; frames now overlap through per-frame gathers on the caller's own streams, or through
 * batched gathers (rrte_hip_set_gather_batch), both of which measured faster. */
#define RRTE_FLAG_GATHER_OVERLAP 2u

typedef struct rrte_render_params {
    uint32_t width, height;
    uint32_t samples_per_pixel; /* RaytracerConfig::samples_per_pixel */
    uint32_t max_depth;         /* RaytracerConfig::max_depth         */
    uint32_t mode;              /* rrte_mode                          */
    uint32_t jitter;            /* rrte_jitter                        */
    uint32_t seed;
    uint32_t flags;             /* RRTE_FLAG_*                        */
    float background[4];        /* RaytracerConfig::background_color  */
    float t_min;                /* closest-hit lower bound (raytracer.rs:107: 0.001) */
    float shadow_bias;          /* LAMBERT_SHADOW: origin offset along N and t_min    */
    float gamma;                /* 2.2 (raytracer.rs:79)              */
    uint32_t band_rows;         /* multi-GPU interleave: rows per band (0 = whole image) */
} rrte_render_params;           /* 64 bytes */

/* ---------------------------------------------------------------- scene IR */
/* MeshAsset::Vertex (asset.rs:60-65) position + normal; uv and colour do not
 * enter the ray loop. */
typedef struct rrte_mesh_vertex {
    float position[3];
    float normal[3];
} rrte_mesh_vertex;        /* 24 bytes */

typedef struct rrte_scene_ir {
    const rrte_prim* prims;         uint32_t num_prims;
    const rrte_material* materials; uint32_t num_materials;
    const rrte_light* lights;       uint32_t num_lights;
    const rrte_sdf_node* sdf_nodes; uint32_t num_sdf_nodes;
    rrte_camera camera;
    /* triangle meshes (RRTE_PRIM_MESH): shared vertex pool, 3 indices per triangle */
    const rrte_mesh_vertex* mesh_vertices; uint32_t num_mesh_vertices;
    const uint32_t* mesh_indices;          uint32_t num_mesh_indices;
    /* Mesh data version (the analogue of Scene::is_dirty, crates/rrte-scene/src/lib.rs:310-312):
     * nonzero = caller-maintained stamp, the device copy and BVH are rebuilt when the stamp,
     * the array addresses or the counts change; 0 = compare the mesh arrays byte by byte. */
    uint64_t mesh_version;
} rrte_scene_ir;

typedef struct rrte_stats {
    uint64_t primary_rays;   /* W*H*spp of the last frame (this rank's rows)   */
    uint64_t shadow_rays;    /* shadow rays actually cast in the last frame    */
    double kernel_ms;        /* ray kernel time of the last frame (HIP events) */
    double gather_ms;        /* RCCL gather + de-interleave time               */
    double upload_ms;        /* host time to lower + enqueue a changed scene (0 when cached; the copy is async) */
    uint64_t frames;         /* frames rendered by this context                */
    uint32_t jit_active;     /* last frame's kernel: 0 generic, 1 full, 2 topology specialisation */
    uint32_t hot_tiles;      /* hot slots the last launch dispatched first: the tiles an earlier launch of
                                the same shape measured slowest (0: image order; env RRTE_TILE_ORDER=0
                                forces image order).  Never changes a pixel, only when each tile starts. */
    double jit_compile_ms;   /* hiprtc compile time of the last specialised kernel */
} rrte_stats;

typedef struct rrte_ctx rrte_ctx;

/* ------------------------------------------------------------- entry points */
uint32_t rrte_hip_abi_version(void);

/* Create a context on HIP device `device` (>= 0). */
rrte_status rrte_hip_create(int device, rrte_ctx** out);
void rrte_hip_destroy(rrte_ctx* ctx);
const char* rrte_hip_last_error(const rrte_ctx* ctx);

/* Raytracer::render: blocking; writes W*H*4 bytes to host `out_rgba8`.  When `out_rgba8` is pinned
 * host memory (hipHostMalloc'd, or a range registered with rrte_hip_host_register) the kernel stores
 * the frame straight into it while it renders (system-scope, write-through stores); pageable memory
 * gets one D2H copy after the render.  Returns when the frame is complete; the frame's statistics
 * (shadow-ray count) are read back behind it and rrte_hip_stats waits for them.  params->flags takes
 * only the RRTE_FLAG_* bits (others: RRTE_INVALID_ARG). */
rrte_status rrte_hip_render(rrte_ctx* ctx, const rrte_scene_ir* scene,
                            const rrte_render_params* params, uint8_t* out_rgba8);

/* Parity variant: also writes W*H*4 floats (post-gamma, post-clamp, pre-
 * quantisation; or linear if RRTE_FLAG_F32_LINEAR).  Either pointer may be null. */
rrte_status rrte_hip_render_f32(rrte_ctx* ctx, const rrte_scene_ir* scene,
                                const rrte_render_params* params, uint8_t* out_rgba8,
                                float* out_rgba32f);

/* Device-resident variant for throughput measurement and display: enqueue
 * one frame on `stream` (a hipStream_t, or null for the context's stream)
 * writing to device buffers (either may be null).  Returns without
 * synchronising; shadow-ray counts accumulate on the device and are folded
 * into rrte_hip_stats at the next synchronising call.  A stream passed here (or to
 * rrte_hip_render_gather_async) must stay valid until the next rrte_hip_synchronize: the context
 * records events on it when a scene or tile-list version it read is retired.  Scene changes never
 * drain the device: the scene is kept in a ring of versions. */
rrte_status rrte_hip_render_async(rrte_ctx* ctx, const rrte_scene_ir* scene,
                                  const rrte_render_params* params, void* d_out_rgba8,
                                  void* d_out_rgba32f, void* stream);
/* Waits for every frame of the context.  With a communicator the wait is bounded by the comm timeout
 * (below); without one by env RRTE_NOCOMM_WAIT_MS (default 600000 = 10 minutes, far above any queue
 * of frames; 0 = no limit): a kernel that never completes returns RRTE_HIP_ERROR instead of hanging.
 * The same bound applies to rrte_hip_host_unregister's drain. */
rrte_status rrte_hip_synchronize(rrte_ctx* ctx);
/* Non-blocking completion test of the work queued on the context's OWN streams (its default stream
 * and the batched-gather render / comm streams; caller streams are the caller's to query): *busy = 1
 * while any of it is still running, else 0.  Does not flush an open gather batch. */
rrte_status rrte_hip_query(rrte_ctx* ctx, uint32_t* busy);

/* The last frame's statistics (after a blocking frame: waits for its counter read-back). */
rrte_status rrte_hip_stats(rrte_ctx* ctx, rrte_stats* out);

/* Scene-specialised kernels (hiprtc).  OFF: always the
 * generic kernel.  ON: specialise a scene on its first frame.  AUTO (default):
 * specialise once the same scene is rendered a second time.  Results are
 * bit-identical either way; env RRTE_JIT=0/1/2 overrides the default.
 * A specialisation is FULL (every scene value compiled in) or TOPOLOGY (object kinds, SDF
 * programs' ops and structure, light kinds compiled in; positions, sizes, colours, intensities
 * read from the uploaded scene), so moving, resizing or recolouring objects and lights reuses one
 * compiled kernel.  Which: env RRTE_JIT_TOPO=0 full only, =1 topology only, unset/2 adaptive --
 * topology once a scene change kept the previous scene's topology (an animation), full once a
 * scene has been rendered unchanged for 16 frames.  Compiled code objects persist on disk
 * (RRTE_JIT_CACHE_DIR, default $XDG_CACHE_HOME/rrte-jit or ~/.cache/rrte-jit; RRTE_JIT_CACHE=0 off). */
typedef enum rrte_jit_mode { RRTE_JIT_OFF = 0, RRTE_JIT_ON = 1, RRTE_JIT_AUTO = 2 } rrte_jit_mode;
rrte_status rrte_hip_set_jit(rrte_ctx* ctx, int mode);
/* Diagnostic: generate + hiprtc-compile the specialised kernel for `scene` (the full one; the
 * topology one with env RRTE_JIT_TOPO=1) -- no device needed.  RRTE_OK if it compiles; otherwise
 * the log is copied out. */
rrte_status rrte_hip_jit_check(const rrte_scene_ir* scene, int mode, char* log, size_t log_len);
/* Diagnostic: run the kernels' short correctly rounded f32 sequences (device_scene.hpp
 * sqrt_rn / rcp_rn / the constant-divisor step of div_rn) on `device` against the
 * compiler's full sequences and count bit mismatches (any NaN matches any NaN):
 *   RRTE_FPCHECK_SQRT, RRTE_FPCHECK_RCP: every f32 bit pattern in [lo, hi) (hi <= 2^32);
 *   RRTE_FPCHECK_DIV: a/b for every significand of a in [1, 2) and every b = 1 + k*2^-23,
 *                     k in [lo, hi) (hi <= 2^23), with y = rcp_rn(b).  Synchronous. */
/*   RRTE_FPCHECK_SQRT_HW: control -- the bare v_sqrt_f32 against the correctly rounded sqrt
 *                         (the sweep must find its 1-ulp errors).
 *   RRTE_FPCHECK_GAMMA_U8: every f32 bit pattern in [lo, hi): the kernels' gamma-2.2 byte
 *                          (ray_kernels.hpp gamma22_u8) against to_u8(clamp(powf(c, 1/2.2))).
 *   RRTE_FPCHECK_SQRT_BF: as RRTE_FPCHECK_SQRT for the branch-free form (sqrt_rn_branchfree);
 *                         RRTE_FPCHECK_SQRT sweeps the guarded form (sqrt_rn_guarded). */
typedef enum rrte_fpcheck {
    RRTE_FPCHECK_SQRT = 0, RRTE_FPCHECK_RCP = 1, RRTE_FPCHECK_DIV = 2, RRTE_FPCHECK_SQRT_HW = 3,
    RRTE_FPCHECK_GAMMA_U8 = 4, RRTE_FPCHECK_SQRT_BF = 5
} rrte_fpcheck;
rrte_status rrte_hip_fpcheck(int device, int kind, uint64_t lo, uint64_t hi, uint64_t* mismatches);
/* Diagnostic (host only): the CSG early-out decoration the renderer applies to one SDF program
 * (DESIGN.md §5 CSG guards).  Copies in[0..count) to out with, for every guarded right operand B
 * of a union / difference op j: out[first node of B].i[2] = j + 1 and out[j].f[4..9] = B's bound
 * (centre xyz, radius R, slope lambda, usable range): B >= lambda (|p - centre| - R) wherever
 * R <= |p - centre| <= f[9].  min_leaves: 1 = guard every operand, 2 = the renderer's default
 * (operands of >= 2 leaves and single leaves of the long formulas), N = operands of >= N leaves,
 * 0 = none.  *guards = number of guards.  The program must pass the renderer's validation. */
rrte_status rrte_hip_sdf_guards(const rrte_sdf_node* in, uint32_t count, uint32_t min_leaves, rrte_sdf_node* out,
                                uint32_t* guards);
/* Diagnostic (host only): the measured-cost tile order a context dispatches after a profile with
 * per-tile durations costs[0..tiles) (tiles_x tiles per row): every tile once, slowest first (a
 * counting sort on 65536 cost buckets, ties in tile order).  Writes *n_slots = tiles slots
 * (y << 16 | x) to slots[0..cap); RRTE_INVALID_ARG if they do not fit. */
rrte_status rrte_hip_tile_order_plan(const uint32_t* costs, uint32_t tiles, uint32_t tiles_x, uint32_t* slots,
                                     uint32_t cap, uint32_t* n_slots);
/* Diagnostic: the build id of the device code (32 hex digits): a hash of the embedded device headers,
 * every hiprtc option (RRTE_JIT_EXTRA_OPTS included) and the hiprtc version.  Profiles record it
 * (tools/prof.sh) and bench.py takes counters only from a profile of the same build. */
rrte_status rrte_hip_build_id(char* out, size_t out_len);
/* Diagnostic (host only): the persistent JIT cache's file name (32 hex digits + NUL, out_len >= 33)
 * for a generated kernel `source`: a hash of the source, the device headers embedded in this library
 * (or `headers_override` in their place, to show that a rebuilt library's headers change the key),
 * the hiprtc options (RRTE_JIT_EXTRA_OPTS included) and the hiprtc version. */
rrte_status rrte_hip_jit_cache_key(const char* source, const char* headers_override, char* out, size_t out_len);
/* Diagnostic: with env RRTE_DEBUG bit 2 (value 4) set when the context was created, every wave
 * range-checks the indices it derives from its launch (tile-list slot, decoded tile, frame, output
 * row) before using them and ORs a code into a device check word instead of an out-of-range access
 * (1 list slot, 2 tile, 4 frame, 8 output row), and every scene upload checks the device copy's
 * object kinds, SDF node ranges and CSG-guard links (16 kind, 32 node range, 64 guard link).  Drains
 * the context's work, returns the word in *word and clears it.  0 = no violation. */
rrte_status rrte_hip_check_word(rrte_ctx* ctx, uint64_t* word);

/* ------------------------------------------------ SceneIR dump / load (repro) */
/* A frame's lowered scene and parameters in one self-checking file (rrte_amd/csrc/scene_io.hip: magic,
 * format and ABI version, record sizes, counts, the arrays, an FNV-1a trailer), so a frame can be
 * replayed bit for bit on the device or on the CPU oracle.  env RRTE_DUMP_SCENE=<path>: every render
 * entry point dumps the scene and parameters it was given before rendering (atomic rename), so the
 * last frame of a failing process is on disk.  Host only; no device work. */
rrte_status rrte_hip_scene_dump(const rrte_scene_ir* scene, const rrte_render_params* params, const char* path);
/* Loads a dump: *scene's arrays point into *storage (release it with rrte_hip_scene_free).
 * RRTE_INVALID_ARG for a missing, truncated or altered file, or one of another ABI / record layout. */
rrte_status rrte_hip_scene_load(const char* path, rrte_scene_ir* scene, rrte_render_params* params, void** storage);
void rrte_hip_scene_free(void* storage);

/* ----------------------------------------------------- multi-GPU (RCCL/xGMI) */
/* Row-band partition: band b (band_rows rows) belongs to rank b % nranks.
 * rrte_hip_render_gather renders this rank's bands and gathers every rank's
 * bands to `root`, which de-interleaves them into the full image. */
#define RRTE_UNIQUE_ID_BYTES 128
rrte_status rrte_hip_comm_unique_id(uint8_t out_id[RRTE_UNIQUE_ID_BYTES]);
rrte_status rrte_hip_comm_init(rrte_ctx* ctx, int nranks, int rank,
                               const uint8_t id[RRTE_UNIQUE_ID_BYTES]);
/* Blocking: on the root writes the full W*H*4 image to host out_rgba8 (may be
 * null to keep it on the device); non-root ranks ignore out_rgba8. */
rrte_status rrte_hip_render_gather(rrte_ctx* ctx, const rrte_scene_ir* scene,
                                   const rrte_render_params* params, int root,
                                   uint8_t* out_rgba8);
/* Async device variant: d_full_rgba8 (root only, W*H*4 bytes) receives the frame.  With gather batch 1
 * (the default) all of the frame's work is ordered on `stream`; a frame on another stream than the
 * previous frame's gather waits for that gather (collectives run in issue order on every rank).
 * Every rank must issue the same frames in the same order. */
rrte_status rrte_hip_render_gather_async(rrte_ctx* ctx, const rrte_scene_ir* scene,
                                         const rrte_render_params* params, int root,
                                         void* d_full_rgba8, void* stream);

/* Collective failure detection (the reference has none: examples/basic-demo/src/main.rs:145-150
 * only stops its loop).  Every host wait that covers a gather -- rrte_hip_synchronize, the blocking
 * rrte_hip_render_gather, rrte_hip_comm_init's drain -- polls the work and ncclCommGetAsyncError
 * instead of blocking; a gather that reports an error or does not complete within `ms` (default
 * 30000; env RRTE_COMM_TIMEOUT_MS) aborts the communicator (ncclCommAbort) and returns
 * RRTE_RCCL_ERROR with the reason in rrte_hip_last_error.  A failed gather of either form leaves the
 * communicator aborted: every later gather call returns RRTE_RCCL_ERROR until rrte_hip_comm_init.
 * (Fault injection for tests: env RRTE_FAULT_STALL_GATHER=N stalls the N-th collective of a context
 * on the device until the host gives up on it -- a stalled peer seen from this rank.) */
rrte_status rrte_hip_set_comm_timeout(rrte_ctx* ctx, uint32_t ms);

/* Batched gather (throughput mode, SURVEY §8e "fewer, larger collectives"): with frames > 1 each
 * rrte_hip_render_gather_async only records the frame (its camera is read, the scene uploaded if it
 * changed) into the open batch; every `frames` frames the batch renders in multi-frame launches (up
 * to 8 frames per launch) on the context's render streams, after the work already queued on the
 * frames' streams, and ONE ncclGather on the context's comm stream moves all of them to the root,
 * which de-interleaves each into its d_full_rgba8.  A frame's d_full_rgba8 is then complete only
 * after rrte_hip_flush + a synchronisation (rrte_hip_synchronize, or of the device).  Only gather-path
 * calls every rank makes close a batch (collective): a full batch, rrte_hip_flush, rrte_hip_set_gather_batch,
 * rrte_hip_comm_init, a blocking rrte_hip_render_gather, and a gather frame of another size, band
 * height, root, slab format, mode or sampling setup.  Local calls never do: rrte_hip_synchronize and a
 * scene change through rrte_hip_render / render_f32 / render_async only RENDER the open batch's
 * frames (with the scene they were issued with) and leave its gather for the next collective close,
 * so one rank may poll or render a preview on its own.  frames in [1, 16]; every rank must use the
 * same setting.  Flushing with no open batch does nothing. */
rrte_status rrte_hip_set_gather_batch(rrte_ctx* ctx, uint32_t frames);
rrte_status rrte_hip_flush(rrte_ctx* ctx);
/* Diagnostic: the collectives this context has issued on its communicator since rrte_hip_comm_init
 * (per-frame gathers and batch exchanges) and the frames of the open gather batch.  A local call
 * (rrte_hip_synchronize, a scene change) renders the open batch but never issues a collective, so
 * neither count may move on one rank alone. */
rrte_status rrte_hip_gather_info(rrte_ctx* ctx, uint64_t* collectives, uint32_t* open_frames);
/* Pin a host range the caller keeps alive (e.g. the frame buffer an engine reuses every frame) so
 * rrte_hip_render writes into it directly.  Unregister (or destroy the context) before freeing it;
 * rrte_hip_host_unregister waits for the context's frames first. */
rrte_status rrte_hip_host_register(rrte_ctx* ctx, void* host, size_t bytes);
rrte_status rrte_hip_host_unregister(rrte_ctx* ctx, void* host);

/* Host-side helpers exported for the bindings (no device work). */
/* Rows owned by `rank` under the plain band interleave (band b on rank b % nranks). */
uint32_t rrte_hip_band_rows_for_rank(uint32_t height, uint32_t band_rows, int nranks, int rank);
/* The band partition a multi-GPU frame of `scene` / `params` uses (DESIGN.md §5 "Band partition"): the
 * first *sky_bands bands (bands no object can reach, judged from the camera and the objects' culling
 * spheres: every camera ray there misses) belong to rank 0; the remaining bands go round robin in
 * cycles of L = R + (nranks - 1) P bands, R = *root_bands in [0, 8] for rank 0 first, then P =
 * *peer_bands in [1, 8] rounds of one band per peer.  Band b then belongs to: b < sky -> 0; else with
 * s = (b - sky) % L: s < R -> 0, otherwise 1 + (s - R) % (nranks - 1).  R:P is chosen by a work model
 * (sky rows are cheap; the root receives and expands the peers' rows).  Computed identically on every
 * rank; host only.  (env RRTE_BAND_SKY=0: sky 0, 1:1 -- the plain interleave.)  Rank 0 must be the
 * root for a root-biased partition (otherwise the plain interleave). */
rrte_status rrte_hip_band_layout(const rrte_scene_ir* scene, const rrte_render_params* params, int nranks, int root,
                                 uint32_t* sky_bands, uint32_t* root_bands, uint32_t* peer_bands);
/* Rows owned by `rank` under that partition, in the order they are packed (0 outside the ranges
 * above, or for root_bands = sky_bands = 0). */
uint32_t rrte_hip_band_rows_for_rank_ex(uint32_t height, uint32_t band_rows, int nranks, int rank, uint32_t sky_bands,
                                        uint32_t root_bands, uint32_t peer_bands);

#ifdef __cplusplus
}
#endif

#endif /* RRTE_HIP_H */
