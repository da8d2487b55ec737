//! Lowering of the reference's scene types to the rrte_hip scene IR (include/rrte_hip.h): every
//! `SceneObject` (Sphere / Plane / Triangle / Cube / Cylinder / Cone / Capsule, primitives.rs:6-725,
//! and the build-defined `SdfObject`), every `Light` (Point / Directional / Spot / Ambient,
//! light.rs:5-397), every `Material` (Lambertian / Metal / Dielectric / Emissive, material.rs:5-213),
//! the `Camera` (camera.rs:24-133) and `RaytracerConfig` (raytracer.rs:8-25).
//!
//! The objects describe themselves through the `gpu_desc` hook that
//! ../patches/0001-rrte-renderer-gpu-desc.patch adds to the three traits (trait objects cannot cross
//! the ABI and the traits have no `as_any`).  Every record is filled exactly as the C++
//! mirror fills it (rrte_amd/cpp/rrte_renderer.cpp `X::lower`, proven byte-identical to the Python
//! mirror and rendered against the oracle on the GPU); tests/test_rust_binding.py compares the two
//! lowerings call by call (kind constants, argument order, fields assigned).
use crate::sdf::SdfProgram;
use rrte_hip_sys::safe::SceneIr;
use rrte_hip_sys::*;
use rrte_math::{Color, Transform, Vec3};
use rrte_renderer::gpu_desc::{GpuLight, GpuMaterial, GpuShape};
use rrte_renderer::{Camera, Light, Material, ProjectionType, RaytracerConfig, SceneObject};
use std::sync::Arc;

const ZERO: Vec3 = Vec3::ZERO;

/// The shading setup `RaytracerConfig` does not carry (rrte_render_params beyond it).  The default
/// reproduces the reference's own formula (raytracer.rs:92-148) with its random jitter.
#[derive(Debug, Clone, Copy)]
pub struct GpuOptions {
    pub mode: u32,
    pub jitter: u32,
    pub seed: u32,
    pub t_min: f32,
    pub shadow_bias: f32,
    pub gamma: f32,
    pub band_rows: u32,
}

impl Default for GpuOptions {
    fn default() -> Self {
        Self { mode: RRTE_MODE_REFCOMPAT, jitter: RRTE_JITTER_RANDOM, seed: 0, t_min: 0.001, shadow_bias: 1e-3,
               gamma: 2.2, band_rows: 16 }
    }
}

fn prim(kind: u32, p: &[f32], t: &Transform) -> rrte_prim {
    let mut r = rrte_prim::default();
    r.kind = kind;
    r.p[..p.len()].copy_from_slice(p);
    r.trs = [t.position.x, t.position.y, t.position.z, t.rotation.x, t.rotation.y, t.rotation.z, t.rotation.w,
             t.scale.x, t.scale.y, t.scale.z];
    r
}

/// One object's record; an SDF object's program is appended to `nodes`.  None for a `Custom`
/// payload this crate does not know (the caller then renders on the CPU).
pub fn lower_shape(shape: &GpuShape, t: &Transform, nodes: &mut Vec<rrte_sdf_node>) -> Option<rrte_prim> {
    Some(match shape {
        GpuShape::Sphere { center, radius } => prim(RRTE_PRIM_SPHERE, &[center.x, center.y, center.z, *radius], t),
        GpuShape::Plane { point, normal } => {
            prim(RRTE_PRIM_PLANE, &[point.x, point.y, point.z, 0.0, normal.x, normal.y, normal.z], t)
        }
        GpuShape::Triangle { vertices: v, normals: n } => prim(
            RRTE_PRIM_TRIANGLE,
            &[v[0].x, v[0].y, v[0].z, v[1].x, v[1].y, v[1].z, v[2].x, v[2].y, v[2].z,
              n[0].x, n[0].y, n[0].z, n[1].x, n[1].y, n[1].z, n[2].x, n[2].y, n[2].z],
            t,
        ),
        GpuShape::Cube { center, size } => {
            prim(RRTE_PRIM_CUBE, &[center.x, center.y, center.z, 0.0, size.x, size.y, size.z], t)
        }
        GpuShape::Cylinder { center, radius, height } => {
            prim(RRTE_PRIM_CYLINDER, &[center.x, center.y, center.z, *radius, *height], t)
        }
        GpuShape::Cone { center, radius, height } => prim(RRTE_PRIM_CONE, &[center.x, center.y, center.z, *radius, *height], t),
        GpuShape::Capsule { center, radius, height } => {
            prim(RRTE_PRIM_CAPSULE, &[center.x, center.y, center.z, *radius, *height], t)
        }
        GpuShape::Custom(payload) => {
            let sdf = payload.downcast_ref::<SdfProgram>()?;
            let b = &sdf.bound_center;
            let mut p = prim(RRTE_PRIM_SDF, &[b[0], b[1], b[2], sdf.bound_radius], t);
            p.sdf_first = nodes.len() as u32;
            p.sdf_count = sdf.nodes.len() as u32;
            p.sdf_max_steps = sdf.max_steps;
            p.sdf_step_scale = sdf.step_scale;
            p.sdf_hit_eps = sdf.hit_eps;
            nodes.extend_from_slice(&sdf.nodes);
            p
        }
    })
}

#[allow(clippy::too_many_arguments)]
fn light_struct(kind: u32, color: Color, intensity: f32, position: Vec3, direction: Vec3, range: f32, linear: f32,
                quadratic: f32, inner: f32, outer: f32) -> rrte_light {
    let mut l = rrte_light::default();
    l.kind = kind;
    l.intensity = intensity;
    l.range = range;
    l.linear = linear;
    l.quadratic = quadratic;
    l.inner_angle = inner;
    l.outer_angle = outer;
    l.position = [position.x, position.y, position.z, 0.0];
    l.direction = [direction.x, direction.y, direction.z, 0.0];
    l.color = [color.r, color.g, color.b, color.a];
    l
}

/// `Light::gpu_desc` -> rrte_light (light.rs: PointLight 123-220, DirectionalLight 57-121,
/// SpotLight 222-338, AmbientLight 340-397).  Point and spot lights keep their attenuation
/// parameters (range 100, linear 0.09, quadratic 0.032 by default, light.rs:137-147).
pub fn lower_light(l: &GpuLight) -> rrte_light {
    match l {
        GpuLight::Point { position, color, intensity, range, linear_attenuation, quadratic_attenuation } => light_struct(
            RRTE_LIGHT_POINT, *color, *intensity, *position, ZERO, *range, *linear_attenuation,
            *quadratic_attenuation, 0.0, 0.0),
        GpuLight::Directional { direction, color, intensity } => {
            light_struct(RRTE_LIGHT_DIRECTIONAL, *color, *intensity, ZERO, *direction, 100.0, 0.09, 0.032, 0.0, 0.0)
        }
        GpuLight::Spot { position, direction, color, intensity, range, inner_angle, outer_angle, linear_attenuation,
                         quadratic_attenuation } => light_struct(
            RRTE_LIGHT_SPOT, *color, *intensity, *position, *direction, *range, *linear_attenuation,
            *quadratic_attenuation, *inner_angle, *outer_angle),
        GpuLight::Ambient { color, intensity } => {
            light_struct(RRTE_LIGHT_AMBIENT, *color, *intensity, ZERO, ZERO, 100.0, 0.09, 0.032, 0.0, 0.0)
        }
    }
}

fn material_struct(kind: u32, albedo: Color, fuzz: f32, ior: f32) -> rrte_material {
    let mut m = rrte_material::default();
    m.kind = kind;
    m.fuzz = fuzz;
    m.ior = ior;
    m.albedo = [albedo.r, albedo.g, albedo.b, albedo.a];
    m
}

/// `Material::gpu_desc` -> rrte_material (material.rs: Lambertian 45-81, Metal 83-122, Dielectric
/// 124-183, Emissive 185-213; `albedo()` is what ray_color reads, raytracer.rs:124-136).
pub fn lower_material(m: &GpuMaterial) -> rrte_material {
    match m {
        GpuMaterial::Lambertian { albedo } => material_struct(RRTE_MAT_LAMBERTIAN, *albedo, 0.0, 1.0),
        GpuMaterial::Metal { albedo, roughness } => material_struct(RRTE_MAT_METAL, *albedo, *roughness, 1.0),
        GpuMaterial::Dielectric { color, ior } => material_struct(RRTE_MAT_DIELECTRIC, *color, 0.0, *ior),
        GpuMaterial::Emissive { color, intensity: _ } => material_struct(RRTE_MAT_EMISSIVE, *color, 0.0, 1.0),
    }
}

/// `Camera` (camera.rs:24-31) -> rrte_camera: the transform (rotation from Camera::look_at,
/// camera.rs:85-95, `up` ignored as the reference ignores it) and the projection's parameters.
pub fn lower_camera(camera: &Camera) -> rrte_camera {
    let t = &camera.transform;
    let mut c = rrte_camera::default();
    c.position = [t.position.x, t.position.y, t.position.z];
    c.rotation = [t.rotation.x, t.rotation.y, t.rotation.z, t.rotation.w];
    c.scale = [t.scale.x, t.scale.y, t.scale.z];
    match camera.projection {
        ProjectionType::Perspective { fov, aspect_ratio, near, far } => {
            c.projection = RRTE_PERSPECTIVE;
            c.fov = fov;
            c.aspect_ratio = aspect_ratio;
            c.near_plane = near;
            c.far_plane = far;
        }
        ProjectionType::Orthographic { left, right, bottom, top, near, far } => {
            c.projection = RRTE_ORTHOGRAPHIC;
            c.left = left;
            c.right = right;
            c.bottom = bottom;
            c.top = top;
            c.near_plane = near;
            c.far_plane = far;
        }
    }
    c
}

/// `RaytracerConfig` (raytracer.rs:8-25) + the GPU-only options -> rrte_render_params.
pub fn lower_config(config: &RaytracerConfig, opt: &GpuOptions) -> rrte_render_params {
    let mut p = rrte_render_params::default();
    p.width = config.width;
    p.height = config.height;
    p.samples_per_pixel = config.samples_per_pixel;
    p.max_depth = config.max_depth;
    p.mode = opt.mode;
    p.jitter = opt.jitter;
    p.seed = opt.seed;
    let bg = &config.background_color;
    p.background = [bg.r, bg.g, bg.b, bg.a];
    p.t_min = opt.t_min;
    p.shadow_bias = opt.shadow_bias;
    p.gamma = opt.gamma;
    p.band_rows = opt.band_rows;
    p
}

/// Lowers a whole scene (the arguments of Raytracer::render, raytracer.rs:45-51).  None if any
/// object, light or material has no GPU description: the caller keeps the reference's CPU path for
/// that frame (user-defined SceneObjects stay supported).  Materials are deduplicated by identity
/// in order of first use (`Arc::ptr_eq`), as the C++ and Python mirrors do.
pub fn lower_scene(objects: &[Arc<dyn SceneObject>], lights: &[Arc<dyn Light>], camera: &Camera) -> Option<SceneIr> {
    let mut ir = SceneIr::default();
    let mut used: Vec<Arc<dyn Material>> = Vec::new();
    for o in objects {
        let desc = o.gpu_desc()?;
        let mut p = lower_shape(&desc.shape, &desc.transform, &mut ir.sdf_nodes)?;
        p.material = match &desc.material {
            None => -1,
            Some(m) => match used.iter().position(|u| Arc::ptr_eq(u, m)) {
                Some(i) => i as i32,
                None => {
                    used.push(m.clone());
                    (used.len() - 1) as i32
                }
            },
        };
        ir.prims.push(p);
    }
    for m in &used {
        ir.materials.push(lower_material(&m.gpu_desc()?));
    }
    for l in lights {
        ir.lights.push(lower_light(&l.gpu_desc()?));
    }
    ir.camera = lower_camera(camera);
    Some(ir)
}
