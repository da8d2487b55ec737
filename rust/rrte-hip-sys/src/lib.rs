//! rrte-hip-sys — raw FFI to librrte_hip (include/rrte_hip.h), the MI355X replacement of
//! `rrte_renderer::Raytracer::render` (crates/rrte-renderer/src/raytracer.rs:45-148).
//!
//! Mirrors include/rrte_hip.h: `#[repr(C)]` records in the header's field order, its constants and
//! every entry point.  `unsafe` lives here only; the renderer keeps `unsafe_code = "forbid"`
//! (Cargo.toml:18-19 workspace lint) and calls the safe wrapper in rrte-renderer-hip.
//! tests/test_rust_binding.py checks this file mechanically against the header (no cargo in the
//! build image): every struct's field names, order, offsets and size (offsetof/sizeof from a C
//! program compiled with the header), every constant, every extern "C" signature.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub type rrte_status = c_int;
pub const RRTE_OK: rrte_status = 0;
pub const RRTE_INVALID_ARG: rrte_status = 1;
pub const RRTE_HIP_ERROR: rrte_status = 2;
pub const RRTE_RCCL_ERROR: rrte_status = 3;
pub const RRTE_UNSUPPORTED_PRIM: rrte_status = 4;
pub const RRTE_NO_DEVICE: rrte_status = 5;
pub const RRTE_ABI_VERSION: u32 = 2;
pub const RRTE_UNIQUE_ID_BYTES: usize = 128;
pub const RRTE_SDF_MAX_STACK: u32 = 8;
pub const RRTE_SDF_MAX_POINT_STACK: u32 = 4;
pub const RRTE_SDF_MAX_OCTAVES: u32 = 8;
pub const RRTE_FLAG_F32_LINEAR: u32 = 1;
pub const RRTE_PRIM_SPHERE: u32 = 0;
pub const RRTE_PRIM_PLANE: u32 = 1;
pub const RRTE_PRIM_TRIANGLE: u32 = 2;
pub const RRTE_PRIM_CUBE: u32 = 3;
pub const RRTE_PRIM_CYLINDER: u32 = 4;
pub const RRTE_PRIM_CONE: u32 = 5;
pub const RRTE_PRIM_CAPSULE: u32 = 6;
pub const RRTE_PRIM_SDF: u32 = 7;
pub const RRTE_PRIM_MESH: u32 = 8;
pub const RRTE_MAT_LAMBERTIAN: u32 = 0;
pub const RRTE_MAT_METAL: u32 = 1;
pub const RRTE_MAT_DIELECTRIC: u32 = 2;
pub const RRTE_MAT_EMISSIVE: u32 = 3;
pub const RRTE_LIGHT_POINT: u32 = 0;
pub const RRTE_LIGHT_DIRECTIONAL: u32 = 1;
pub const RRTE_LIGHT_SPOT: u32 = 2;
pub const RRTE_LIGHT_AMBIENT: u32 = 3;
pub const RRTE_PERSPECTIVE: u32 = 0;
pub const RRTE_ORTHOGRAPHIC: u32 = 1;
pub const RRTE_MODE_REFCOMPAT: u32 = 0;
pub const RRTE_MODE_LAMBERT_SHADOW: u32 = 1;
pub const RRTE_JITTER_CENTER: u32 = 0;
pub const RRTE_JITTER_RANDOM: u32 = 1;
pub const RRTE_SDF_SPHERE: u32 = 1;
pub const RRTE_SDF_BOX: u32 = 2;
pub const RRTE_SDF_CYLINDER: u32 = 3;
pub const RRTE_SDF_PRISM: u32 = 4;
pub const RRTE_SDF_TORUS: u32 = 5;
pub const RRTE_SDF_TUBE: u32 = 6;
pub const RRTE_SDF_RING: u32 = 7;
pub const RRTE_SDF_CONE: u32 = 8;
pub const RRTE_SDF_CAPSULE: u32 = 9;
pub const RRTE_SDF_ELLIPSOID: u32 = 10;
pub const RRTE_SDF_UNION: u32 = 32;
pub const RRTE_SDF_DIFFERENCE: u32 = 33;
pub const RRTE_SDF_INTERSECTION: u32 = 34;
pub const RRTE_SDF_SMOOTH_UNION: u32 = 35;
pub const RRTE_SDF_SMOOTH_DIFFERENCE: u32 = 36;
pub const RRTE_SDF_SMOOTH_INTERSECTION: u32 = 37;
pub const RRTE_SDF_BEND: u32 = 64;
pub const RRTE_SDF_TWIST: u32 = 65;
pub const RRTE_SDF_TAPER: u32 = 66;
pub const RRTE_SDF_NOISE: u32 = 67;
pub const RRTE_SDF_WAVE: u32 = 68;
pub const RRTE_SDF_POP_POINT: u32 = 96;
pub const RRTE_JIT_OFF: c_int = 0;
pub const RRTE_JIT_ON: c_int = 1;
pub const RRTE_JIT_AUTO: c_int = 2;

#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_prim { pub kind: u32, pub material: i32, pub sdf_first: u32, pub sdf_count: u32,
    pub sdf_max_steps: u32, pub sdf_step_scale: f32, pub sdf_hit_eps: f32, pub flags: u32,
    pub p: [f32; 20], pub trs: [f32; 10], pub _pad: [f32; 10] }                       // 192 B
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_material { pub kind: u32, pub fuzz: f32, pub ior: f32, pub _pad0: f32, pub albedo: [f32; 4] }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_light { pub kind: u32, pub intensity: f32, pub range: f32, pub linear: f32,
    pub quadratic: f32, pub inner_angle: f32, pub outer_angle: f32, pub _pad0: f32,
    pub position: [f32; 4], pub direction: [f32; 4], pub color: [f32; 4] }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_sdf_node { pub op: u32, pub i: [u32; 3], pub f: [f32; 12] }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_camera { pub position: [f32; 3], pub projection: u32, pub rotation: [f32; 4],
    pub scale: [f32; 3], pub fov: f32, pub aspect_ratio: f32, pub near_plane: f32, pub far_plane: f32,
    pub left: f32, pub right: f32, pub bottom: f32, pub top: f32, pub _pad: [f32; 1] }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_render_params { pub width: u32, pub height: u32, pub samples_per_pixel: u32,
    pub max_depth: u32, pub mode: u32, pub jitter: u32, pub seed: u32, pub flags: u32,
    pub background: [f32; 4], pub t_min: f32, pub shadow_bias: f32, pub gamma: f32, pub band_rows: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_mesh_vertex { pub position: [f32; 3], pub normal: [f32; 3] }
#[repr(C)]
pub struct rrte_scene_ir { pub prims: *const rrte_prim, pub num_prims: u32,
    pub materials: *const rrte_material, pub num_materials: u32,
    pub lights: *const rrte_light, pub num_lights: u32,
    pub sdf_nodes: *const rrte_sdf_node, pub num_sdf_nodes: u32, pub camera: rrte_camera,
    pub mesh_vertices: *const rrte_mesh_vertex, pub num_mesh_vertices: u32,
    pub mesh_indices: *const u32, pub num_mesh_indices: u32, pub mesh_version: u64 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct rrte_stats { pub primary_rays: u64, pub shadow_rays: u64, pub kernel_ms: f64, pub gather_ms: f64,
    pub upload_ms: f64, pub frames: u64, pub jit_active: u32, pub hot_tiles: u32, pub jit_compile_ms: f64 }
#[repr(C)] pub struct rrte_ctx { _private: [u8; 0] }

extern "C" {
    pub fn rrte_hip_abi_version() -> u32;
    pub fn rrte_hip_create(device: c_int, out: *mut *mut rrte_ctx) -> rrte_status;
    pub fn rrte_hip_destroy(ctx: *mut rrte_ctx);
    pub fn rrte_hip_last_error(ctx: *const rrte_ctx) -> *const c_char;
    pub fn rrte_hip_render(ctx: *mut rrte_ctx, scene: *const rrte_scene_ir,
                           params: *const rrte_render_params, out_rgba8: *mut u8) -> rrte_status;
    pub fn rrte_hip_render_f32(ctx: *mut rrte_ctx, scene: *const rrte_scene_ir,
                               params: *const rrte_render_params, out_rgba8: *mut u8,
                               out_rgba32f: *mut f32) -> rrte_status;
    pub fn rrte_hip_render_async(ctx: *mut rrte_ctx, scene: *const rrte_scene_ir,
                                 params: *const rrte_render_params, d_out_rgba8: *mut c_void,
                                 d_out_rgba32f: *mut c_void, stream: *mut c_void) -> rrte_status;
    pub fn rrte_hip_synchronize(ctx: *mut rrte_ctx) -> rrte_status;
    pub fn rrte_hip_query(ctx: *mut rrte_ctx, busy: *mut u32) -> rrte_status;
    pub fn rrte_hip_stats(ctx: *mut rrte_ctx, out: *mut rrte_stats) -> rrte_status;
    pub fn rrte_hip_set_jit(ctx: *mut rrte_ctx, mode: c_int) -> rrte_status;
    pub fn rrte_hip_jit_check(scene: *const rrte_scene_ir, mode: c_int, log: *mut c_char,
                              log_len: usize) -> rrte_status;
    pub fn rrte_hip_fpcheck(device: c_int, kind: c_int, lo: u64, hi: u64, mismatches: *mut u64) -> rrte_status;
    pub fn rrte_hip_sdf_guards(input: *const rrte_sdf_node, count: u32, min_leaves: u32,
                               out: *mut rrte_sdf_node, guards: *mut u32) -> rrte_status;
    pub fn rrte_hip_tile_order_plan(costs: *const u32, tiles: u32, tiles_x: u32, slots: *mut u32, cap: u32,
                                    n_slots: *mut u32) -> rrte_status;
    pub fn rrte_hip_jit_cache_key(source: *const c_char, headers_override: *const c_char, out: *mut c_char,
                                  out_len: usize) -> rrte_status;
    pub fn rrte_hip_check_word(ctx: *mut rrte_ctx, word: *mut u64) -> rrte_status;
    pub fn rrte_hip_scene_dump(scene: *const rrte_scene_ir, params: *const rrte_render_params, path: *const c_char)
                               -> rrte_status;
    pub fn rrte_hip_scene_load(path: *const c_char, scene: *mut rrte_scene_ir, params: *mut rrte_render_params,
                               storage: *mut *mut c_void) -> rrte_status;
    pub fn rrte_hip_scene_free(storage: *mut c_void);
    pub fn rrte_hip_comm_unique_id(out_id: *mut u8) -> rrte_status;
    pub fn rrte_hip_comm_init(ctx: *mut rrte_ctx, nranks: c_int, rank: c_int, id: *const u8) -> rrte_status;
    pub fn rrte_hip_render_gather(ctx: *mut rrte_ctx, scene: *const rrte_scene_ir,
                                  params: *const rrte_render_params, root: c_int,
                                  out_rgba8: *mut u8) -> rrte_status;
    pub fn rrte_hip_render_gather_async(ctx: *mut rrte_ctx, scene: *const rrte_scene_ir,
                                        params: *const rrte_render_params, root: c_int,
                                        d_full_rgba8: *mut c_void, stream: *mut c_void) -> rrte_status;
    pub fn rrte_hip_set_comm_timeout(ctx: *mut rrte_ctx, ms: u32) -> rrte_status;
    pub fn rrte_hip_set_gather_batch(ctx: *mut rrte_ctx, frames: u32) -> rrte_status;
    pub fn rrte_hip_flush(ctx: *mut rrte_ctx) -> rrte_status;
    pub fn rrte_hip_gather_info(ctx: *mut rrte_ctx, collectives: *mut u64, open_frames: *mut u32) -> rrte_status;
    pub fn rrte_hip_build_id(out: *mut c_char, out_len: usize) -> rrte_status;
    pub fn rrte_hip_host_register(ctx: *mut rrte_ctx, host: *mut c_void, bytes: usize) -> rrte_status;
    pub fn rrte_hip_host_unregister(ctx: *mut rrte_ctx, host: *mut c_void) -> rrte_status;
    pub fn rrte_hip_band_rows_for_rank(height: u32, band_rows: u32, nranks: c_int, rank: c_int) -> u32;
    pub fn rrte_hip_band_layout(scene: *const rrte_scene_ir, params: *const rrte_render_params, nranks: c_int,
                                root: c_int, sky_bands: *mut u32, root_bands: *mut u32,
                                peer_bands: *mut u32) -> rrte_status;
    pub fn rrte_hip_band_rows_for_rank_ex(height: u32, band_rows: u32, nranks: c_int, rank: c_int, sky_bands: u32,
                                          root_bands: u32, peer_bands: u32) -> u32;
}

pub mod safe;
