"""Generates rust/patches/*.patch: the changes a Melthizar/RRTE checkout needs to render through
rust/rrte-renderer-hip (SURVEY §8b "Lowering (required new hook)", §8f rank 3).

  0001-rrte-renderer-gpu-desc.patch  crates/rrte-renderer: src/gpu_desc.rs (plain-data descriptions
      of objects, lights and materials), a defaulted `gpu_desc` method on SceneObject / Light /
      Material (primitives.rs:6-18, light.rs:5-26, material.rs:5-19) implemented for every
      reference type, and the `RenderBackend` slot of Raytracer (raytracer.rs:28-51): render tries
      the back end first and keeps the rayon path as the fallback.
  0002-rrte-core-hip-backend.patch  crates/rrte-core: Engine::render_frame passes the scene's full
      lists (Scene::get_objects / get_lights, crates/rrte-scene/src/lib.rs:165-196) instead of the
      legacy spheres and point lights, and initialize_renderer installs HipBackend
      when a HIP device is present (engine.rs:120-135, 280-312).

The patches are unified diffs against the reference snapshot; this script rebuilds them from the
reference's files (read-only, RRTE_REFERENCE=/root/reference) so they stay reviewable and
re-generable.  No cargo exists in the build image, so they are not compiled here;
tests/test_rust_binding.py checks that they apply (`patch --dry-run`) when the reference is present
and that every reference type gets a hook.
usage: python tools/make_rust_patches.py
"""
import difflib
import os
import re
from pathlib import Path

REF = Path(os.environ.get("RRTE_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parents[1] / "rust" / "patches"

GPU_DESC_RS = '''//! Plain-data descriptions of scene objects, lights and materials for accelerator back ends
//! (rrte-renderer-hip lowers them to the MI355X kernels' scene records).  Trait objects cannot
//! cross an FFI boundary and the traits have no `as_any`: each type describes itself through the
//! defaulted `gpu_desc` methods instead; `None` keeps an object on the CPU path.
use crate::Material;
use rrte_math::{Color, Transform, Vec3};
use std::any::Any;
use std::sync::Arc;

/// The geometry of a `SceneObject` (primitives.rs).  `Custom` carries a back end's own payload
/// (rrte-renderer-hip: the lowered program of an SDF object).
#[derive(Debug, Clone)]
pub enum GpuShape {
    Sphere { center: Vec3, radius: f32 },
    Plane { point: Vec3, normal: Vec3 },
    Triangle { vertices: [Vec3; 3], normals: [Vec3; 3] },
    Cube { center: Vec3, size: Vec3 },
    Cylinder { center: Vec3, radius: f32, height: f32 },
    Cone { center: Vec3, radius: f32, height: f32 },
    Capsule { center: Vec3, radius: f32, height: f32 },
    Custom(Arc<dyn Any + Send + Sync>),
}

/// A `SceneObject` as a back end sees it: geometry, transform, material.
#[derive(Debug, Clone)]
pub struct GpuObject {
    pub shape: GpuShape,
    pub transform: Transform,
    pub material: Option<Arc<dyn Material>>,
}

/// A `Light` (light.rs).
#[derive(Debug, Clone, Copy)]
pub enum GpuLight {
    Point { position: Vec3, color: Color, intensity: f32, range: f32, linear_attenuation: f32,
            quadratic_attenuation: f32 },
    Directional { direction: Vec3, color: Color, intensity: f32 },
    Spot { position: Vec3, direction: Vec3, color: Color, intensity: f32, range: f32, inner_angle: f32,
           outer_angle: f32, linear_attenuation: f32, quadratic_attenuation: f32 },
    Ambient { color: Color, intensity: f32 },
}

/// A `Material` (material.rs).
#[derive(Debug, Clone, Copy)]
pub enum GpuMaterial {
    Lambertian { albedo: Color },
    Metal { albedo: Color, roughness: f32 },
    Dielectric { color: Color, ior: f32 },
    Emissive { color: Color, intensity: f32 },
}
'''

OBJ = {  # SceneObject impls: the GpuShape built from the reference fields (primitives.rs)
    "Sphere": "GpuShape::Sphere { center: self.center, radius: self.radius }",
    "Plane": "GpuShape::Plane { point: self.point, normal: self.normal }",
    "Triangle": "GpuShape::Triangle { vertices: self.vertices, normals: self.normals }",
    "Cube": "GpuShape::Cube { center: self.center, size: self.size }",
    "Cylinder": "GpuShape::Cylinder { center: self.center, radius: self.radius, height: self.height }",
    "Cone": "GpuShape::Cone { center: self.center, radius: self.radius, height: self.height }",
    "Capsule": "GpuShape::Capsule { center: self.center, radius: self.radius, height: self.height }",
}
LIGHT = {
    "DirectionalLight": "GpuLight::Directional { direction: self.direction, color: self.color, intensity: self.intensity }",
    "PointLight": ("GpuLight::Point { position: self.position, color: self.color, intensity: self.intensity, "
                   "range: self.range, linear_attenuation: self.linear_attenuation, "
                   "quadratic_attenuation: self.quadratic_attenuation }"),
    "SpotLight": ("GpuLight::Spot { position: self.position, direction: self.direction, color: self.color, "
                  "intensity: self.intensity, range: self.range, inner_angle: self.inner_angle, "
                  "outer_angle: self.outer_angle, linear_attenuation: self.linear_attenuation, "
                  "quadratic_attenuation: self.quadratic_attenuation }"),
    "AmbientLight": "GpuLight::Ambient { color: self.color, intensity: self.intensity }",
}
MATERIAL = {
    "LambertianMaterial": "GpuMaterial::Lambertian { albedo: self.albedo }",
    "MetalMaterial": "GpuMaterial::Metal { albedo: self.albedo, roughness: self.roughness }",
    "DielectricMaterial": "GpuMaterial::Dielectric { color: self.color, ior: self.ior }",
    "EmissiveMaterial": "GpuMaterial::Emissive { color: self.color, intensity: self.intensity }",
}


def _hook(trait_line, ret):
    """Insert a defaulted gpu_desc method right after `pub trait X ... {`."""
    return (trait_line + "\n    /// Plain-data description for accelerator back ends (rrte-renderer-hip); None keeps this\n"
            f"    /// one on the CPU path.\n    fn gpu_desc(&self) -> Option<{ret}> {{\n        None\n    }}\n")


def _impls(text, trait, table, ret):
    for name, expr in table.items():
        head = f"impl {trait} for {name} {{"
        assert head in text, head
        if ret == "GpuObject":
            body = (f"    fn gpu_desc(&self) -> Option<GpuObject> {{\n        Some(GpuObject {{ shape: {expr}, "
                    "transform: self.transform.clone(), material: self.material.clone() })\n    }\n\n")
        else:
            body = f"    fn gpu_desc(&self) -> Option<{ret}> {{\n        Some({expr})\n    }}\n\n"
        text = text.replace(head, head + "\n" + body, 1)
    return text


def patch_renderer():
    files = {}
    p = (REF / "crates/rrte-renderer/src/primitives.rs").read_text()
    p = p.replace("use crate::Material;\n", "use crate::Material;\nuse crate::gpu_desc::{GpuObject, GpuShape};\n", 1)
    p = p.replace("pub trait SceneObject: Send + Sync + std::fmt::Debug {",
                  _hook("pub trait SceneObject: Send + Sync + std::fmt::Debug {", "GpuObject"), 1)
    files["crates/rrte-renderer/src/primitives.rs"] = _impls(p, "SceneObject", OBJ, "GpuObject")
    lt = (REF / "crates/rrte-renderer/src/light.rs").read_text()
    lt = lt.replace("use serde::{Deserialize, Serialize};\n",
                    "use serde::{Deserialize, Serialize};\nuse crate::gpu_desc::GpuLight;\n", 1)
    lt = lt.replace("pub trait Light: Send + Sync + std::fmt::Debug {",
                    _hook("pub trait Light: Send + Sync + std::fmt::Debug {", "GpuLight"), 1)
    files["crates/rrte-renderer/src/light.rs"] = _impls(lt, "Light", LIGHT, "GpuLight")
    m = (REF / "crates/rrte-renderer/src/material.rs").read_text()
    m = m.replace("use std::sync::Arc;\n", "use std::sync::Arc;\nuse crate::gpu_desc::GpuMaterial;\n", 1)
    m = m.replace("pub trait Material: Send + Sync + std::fmt::Debug {",
                  _hook("pub trait Material: Send + Sync + std::fmt::Debug {", "GpuMaterial"), 1)
    files["crates/rrte-renderer/src/material.rs"] = _impls(m, "Material", MATERIAL, "GpuMaterial")
    lib = (REF / "crates/rrte-renderer/src/lib.rs").read_text()
    lib = lib.replace("/// Camera types.\npub mod camera;\n",
                      "/// Camera types.\npub mod camera;\n/// Plain-data scene descriptions for accelerator back ends.\npub mod gpu_desc;\n", 1)
    files["crates/rrte-renderer/src/lib.rs"] = lib
    r = (REF / "crates/rrte-renderer/src/raytracer.rs").read_text()
    r = r.replace("/// CPU-based raytracer\npub struct Raytracer {\n    config: RaytracerConfig,\n}\n",
                  "/// An accelerator that renders a frame in place of the CPU loop (rrte-renderer-hip:\n"
                  "/// MI355X).  `None` = this frame stays on the CPU (a scene it cannot lower, a device error).\n"
                  "pub trait RenderBackend: Send + Sync {\n"
                  "    fn render(&self, objects: &[Arc<dyn SceneObject>], lights: &[Arc<dyn Light>],\n"
                  "              materials: &[Arc<dyn Material>], camera: &Camera, config: &RaytracerConfig) -> Option<Vec<u8>>;\n\n"
                  "    /// The frame into a caller buffer reused from frame to frame (Engine::frame_buffer): a back end\n"
                  "    /// may keep it pinned and write into it directly.  false = `out` untouched, CPU path.\n"
                  "    fn render_into(&self, objects: &[Arc<dyn SceneObject>], lights: &[Arc<dyn Light>],\n"
                  "                   materials: &[Arc<dyn Material>], camera: &Camera, config: &RaytracerConfig,\n"
                  "                   out: &mut Vec<u8>) -> bool {\n"
                  "        match self.render(objects, lights, materials, camera, config) {\n"
                  "            Some(frame) => {\n                *out = frame;\n                true\n            }\n"
                  "            None => false,\n        }\n    }\n"
                  "}\n\n"
                  "/// CPU-based raytracer\npub struct Raytracer {\n    config: RaytracerConfig,\n"
                  "    backend: Option<Arc<dyn RenderBackend>>,\n}\n", 1)
    r = r.replace("        Self { config }\n    }\n",
                  "        Self { config, backend: None }\n    }\n\n"
                  "    /// Renders through `backend` first (e.g. rrte_renderer_hip::HipBackend); the CPU loop\n"
                  "    /// below stays the fallback, so `render` keeps its infallible signature.\n"
                  "    pub fn set_backend(&mut self, backend: Option<Arc<dyn RenderBackend>>) {\n"
                  "        self.backend = backend;\n    }\n\n"
                  "    /// `render` into a buffer the caller reuses from frame to frame (Engine::frame_buffer): the\n"
                  "    /// back end may keep it pinned and write the frame into it directly; without one, or when it\n"
                  "    /// declines the frame, the CPU loop's frame replaces the buffer as before.\n"
                  "    pub fn render_into(\n        &self,\n        objects: &[Arc<dyn SceneObject>],\n"
                  "        lights: &[Arc<dyn Light>],\n        materials: &[Arc<dyn Material>],\n        camera: &Camera,\n"
                  "        out: &mut Vec<u8>,\n    ) {\n"
                  "        if let Some(b) = &self.backend {\n"
                  "            if b.render_into(objects, lights, materials, camera, &self.config, out) {\n"
                  "                return;\n            }\n        }\n"
                  "        *out = self.render(objects, lights, materials, camera);\n    }\n", 1)
    anchor = "    ) -> Vec<u8> {\n"
    assert anchor in r
    r = r.replace(anchor, anchor + "        if let Some(b) = &self.backend {\n"
                  "            if let Some(frame) = b.render(objects, lights, materials, camera, &self.config) {\n"
                  "                return frame;\n            }\n        }\n", 1)
    files["crates/rrte-renderer/src/raytracer.rs"] = r
    return files


def patch_core():
    files = {}
    e = (REF / "crates/rrte-core/src/engine.rs").read_text()
    old_objs = re.search(r"                // Convert Vec<Arc<Sphere>>.*?raytracer\.render\(&scene_objects, &scene_lights, &Vec::new\(\), &self\.camera\);\n",
                         e, re.S)
    assert old_objs, "engine.rs render_frame CPU branch"
    e = e.replace(old_objs.group(0),
                  "                // Every object and light of the scene (Scene::get_objects / get_lights), not only\n"
                  "                // the legacy sphere and point-light lists: the HIP back end lowers all of them,\n"
                  "                // and the CPU fallback renders the same scene.\n"
                  "                // The frame into the engine's own buffer, reused every frame (the HIP back end keeps it\n"
                  "                // pinned and the kernel writes into it directly; the CPU path replaces it as before).\n"
                  "                raytracer.render_into(self.scene.get_objects(), self.scene.get_lights(),\n"
                  "                                      self.scene.get_materials(), &self.camera, &mut self.frame_buffer);\n", 1)
    old_init = "                let cpu_renderer = Raytracer::new(self.config.renderer_config.clone());\n"
    assert old_init in e
    e = e.replace(old_init,
                  "                let mut cpu_renderer = Raytracer::new(self.config.renderer_config.clone());\n"
                  "                // MI355X back end when a HIP device is present (rrte-renderer-hip); the rayon loop\n"
                  "                // stays the fallback for scenes it cannot lower\n"
                  "                match rrte_renderer_hip::HipBackend::new(0, rrte_renderer_hip::GpuOptions::default()) {\n"
                  "                    Ok(b) => {\n"
                  "                        cpu_renderer.set_backend(Some(std::sync::Arc::new(b)));\n"
                  "                        info!(\"HIP back end enabled (librrte_hip).\");\n"
                  "                    }\n"
                  "                    Err(e) => info!(\"HIP back end unavailable ({e}); CPU raytracer only.\"),\n"
                  "                }\n", 1)
    files["crates/rrte-core/src/engine.rs"] = e
    c = (REF / "crates/rrte-core/Cargo.toml").read_text()
    anchor = "rrte-renderer = { path = \"../rrte-renderer\" }\n"
    assert anchor in c, "rrte-core Cargo.toml"
    c = c.replace(anchor, anchor + "rrte-renderer-hip = { path = \"../rrte-renderer-hip\" }\n", 1)
    files["crates/rrte-core/Cargo.toml"] = c
    w = (REF / "Cargo.toml").read_text()
    m = re.search(r"members = \[\n", w)
    assert m, "workspace members"
    w = w[:m.end()] + "    \"crates/rrte-hip-sys\",\n    \"crates/rrte-renderer-hip\",\n" + w[m.end():]
    files["Cargo.toml"] = w
    return files


def unified(rel, new, new_file=False):
    old = "" if new_file else (REF / rel).read_text()
    a = old.splitlines(keepends=True)
    b = new.splitlines(keepends=True)
    return "".join(difflib.unified_diff(a, b, "/dev/null" if new_file else f"a/{rel}", f"b/{rel}", n=3))


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    rp = unified("crates/rrte-renderer/src/gpu_desc.rs", GPU_DESC_RS, new_file=True)
    for rel, text in patch_renderer().items():
        rp += unified(rel, text)
    (OUT / "0001-rrte-renderer-gpu-desc.patch").write_text(rp)
    cp = ""
    for rel, text in patch_core().items():
        cp += unified(rel, text)
    (OUT / "0002-rrte-core-hip-backend.patch").write_text(cp)
    print("wrote", sorted(p.name for p in OUT.glob("*.patch")))


if __name__ == "__main__":
    main()
