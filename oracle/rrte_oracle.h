/*
 * rrte_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-pixel ray->scene loop
 * (Melthizar/RRTE crates/rrte-renderer/src/raytracer.rs:45-148 and the
 * functions it calls).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the
 * CPU baseline — never as the product path.
 *
 * Parity status:
 *   - The reference is Rust; no cargo/rustc exists in this image and the
 *     reference ships no tests, fixtures or golden vectors (SURVEY.md §4,
 *     §8c).  The restatement is therefore pinned only by hand-derived
 *     known-answer tests written from the reference source and by an
 *     independent numpy restatement (tests/): "parity unpinned" against
 *     the Rust binary itself.
 *   - glam 0.24.2 arithmetic (Vec3 normalize/dot/cross, Quat::from_rotation_arc,
 *     Quat*Vec3, Mat4 SRT + inverse) is restated from glam's published
 *     algorithms; unpinned.
 *   - SDF / CSG / deformers / LAMBERT_SHADOW are build-defined (README-only
 *     in the reference); the formulas in DESIGN.md §SDF are the spec.
 */
#ifndef RRTE_ORACLE_H
#define RRTE_ORACLE_H

#include "../include/rrte_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_hit {
    float t;
    float point[3];
    float normal[3];
    int32_t front_face;
} oracle_hit;

/* Render rows [row_begin, row_end) of the frame (whole image when both 0).
 * out_rgba8 / out_f32 are full-frame W*H*4 buffers (either may be null).
 * Returns 0 on success, nonzero on malformed input. */
int rrte_oracle_render(const rrte_scene_ir* scene, const rrte_render_params* params,
                       uint8_t* out_rgba8, float* out_f32, uint64_t* shadow_rays,
                       int nthreads, uint32_t row_begin, uint32_t row_end);

/* Instrumented event counts of one render (SURVEY.md §8d "flops per ray = sum over
 * evaluations of fixed per-op counts tabulated by the oracle").  Filled only by the
 * counting build (librrte_oracle_count.so, -DRRTE_ORACLE_COUNT); the timed oracle
 * carries no instrumentation. */
typedef struct rrte_oracle_counts {
    uint64_t samples;            /* camera rays generated (pixels * spp)              */
    uint64_t pixels;             /* pixels finalised (average, gamma, clamp, u8)      */
    uint64_t isect_calls[16];    /* intersector entries by RRTE_PRIM_* kind           */
    uint64_t isect_hits[16];     /* hit-attribute computations by kind                */
    uint64_t mesh_tri_tests;     /* Moller-Trumbore tests inside meshes (linear scan)   */
    uint64_t root_checks;        /* candidate roots tested (ray_at + range) in cyl/cone/capsule */
    uint64_t sdf_steps;          /* sphere-tracing steps (one program evaluation each)  */
    uint64_t sdf_normals;        /* tetrahedral normal estimates (4 evaluations each)  */
    uint64_t sdf_nodes[128];     /* program node evaluations by op (all evaluations)   */
    uint64_t noise_octaves;      /* 3-channel value-noise evaluations (1 per octave per NOISE node) */
    uint64_t light_evals[4];     /* Light::illuminate by RRTE_LIGHT_* kind            */
    uint64_t shaded_hits;        /* hits with a material (base colour)                */
    uint64_t lambert_lights;     /* LAMBERT_SHADOW: N.L evaluations (non-ambient)     */
    uint64_t shadow_rays;        /* shadow rays built and traced                       */
    uint64_t lambert_terms;      /* unoccluded diffuse terms added                     */
    uint64_t ref_light_terms;    /* REFCOMPAT: colour*att terms added                  */
    uint64_t scatters[4];        /* Material::scatter by RRTE_MAT_* kind               */
    uint64_t sphere_samples;     /* rand_in_unit_sphere rejection tries                */
} rrte_oracle_counts;

/* Counting build only: render like rrte_oracle_render and accumulate event counts. */
int rrte_oracle_render_counted(const rrte_scene_ir* scene, const rrte_render_params* params,
                               rrte_oracle_counts* counts, int nthreads, uint32_t row_begin, uint32_t row_end);

/* Algorithmic FP32 operations of a count set (weights tabulated in rrte_oracle.c:
 * add, sub, mul, div, sqrt, min, max and each transcendental = 1; abs/neg/compare = 0). */
double rrte_oracle_flops(const rrte_oracle_counts* counts);

/* Known-answer-test hooks. */
int rrte_oracle_intersect(const rrte_scene_ir* scene, uint32_t prim_index,
                          const float origin[3], const float direction[3],
                          float t_min, float t_max, oracle_hit* out);
void rrte_oracle_generate_ray(const rrte_camera* cam, float u, float v,
                              float origin_out[3], float dir_out[3]);
void rrte_oracle_look_at(const float position[3], const float target[3],
                         float quat_out[4]);
float rrte_oracle_sdf_eval(const rrte_scene_ir* scene, uint32_t prim_index,
                           const float p[3]);
void rrte_oracle_mat4_srt(const float trs[10], float m_out[16]);
void rrte_oracle_mat4_inverse(const float m[16], float inv_out[16]);
float rrte_oracle_sinf(float x);
float rrte_oracle_cosf(float x);
void rrte_oracle_value_noise3(float x, float y, float z, uint32_t seed, float out[3]);

#ifdef __cplusplus
}
#endif

#endif
