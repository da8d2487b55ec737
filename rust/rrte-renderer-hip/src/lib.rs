//! rrte-renderer-hip — the MI355X back end of `rrte_renderer::Raytracer::render`
//! (crates/rrte-renderer/src/raytracer.rs:45-148): the same scene arguments lowered to the
//! rrte_hip scene IR (lower.rs) and rendered by librrte_hip's HIP kernels through the safe wrapper
//! of rrte-hip-sys.  This crate keeps the workspace's `unsafe_code = "forbid"` (Cargo.toml:18-19).
//!
//! Wiring (../patches): 0001 adds the defaulted `gpu_desc` hooks and the `RenderBackend` slot to
//! rrte-renderer; 0002 makes `Engine::render_frame` pass the scene's full object and light lists
//! (`get_objects()` / `get_lights()` instead of the legacy sphere/point-light lists)
//! and installs `HipBackend` when a HIP device is present.  Frames whose scene cannot be lowered
//! (a user-defined SceneObject without `gpu_desc`) or whose GPU call fails fall back to the
//! reference's CPU path, so `render` stays infallible.
pub mod lower;
pub mod sdf;

pub use lower::{lower_camera, lower_config, lower_light, lower_material, lower_scene, lower_shape, GpuOptions};
pub use rrte_hip_sys::safe::{Context, Error, SceneIr};
pub use sdf::{SdfObject, SdfRef};

use rrte_renderer::{Camera, Light, Material, RaytracerConfig, RenderBackend, SceneObject};
use std::sync::{Arc, Mutex};

/// The HIP back end a `Raytracer` renders through (`Raytracer::set_backend`).  The context is not
/// internally synchronised, and `Raytracer::render` takes `&self` (concurrent calls are allowed):
/// one mutex serialises the frames of one device.
pub struct HipBackend {
    ctx: Mutex<Context>,
    pub options: GpuOptions,
}

impl HipBackend {
    /// A context on HIP device `device`; Err without a device (the caller keeps the CPU path).
    pub fn new(device: i32, options: GpuOptions) -> Result<Self, Error> {
        Ok(Self { ctx: Mutex::new(Context::new(device)?), options })
    }

    /// Statistics of the last frame (primary and shadow rays, kernel time).
    pub fn stats(&self) -> Option<rrte_hip_sys::rrte_stats> {
        self.ctx.lock().ok()?.stats().ok()
    }
}

impl RenderBackend for HipBackend {
    fn render(&self, objects: &[Arc<dyn SceneObject>], lights: &[Arc<dyn Light>], _materials: &[Arc<dyn Material>],
              camera: &Camera, config: &RaytracerConfig) -> Option<Vec<u8>> {
        // (materials: raytracer.rs passes them through unused; objects carry their own)
        let scene = lower_scene(objects, lights, camera)?;
        let params = lower_config(config, &self.options);
        let mut ctx = self.ctx.lock().ok()?;
        match ctx.render(&scene, &params) {
            Ok(frame) => Some(frame),
            Err(e) => {
                log::warn!("rrte_hip frame failed, rendering on the CPU: {e}");
                None
            }
        }
    }

    /// Engine::render_frame's path (patch 0002): the frame into the engine's reused `frame_buffer`,
    /// which the context pins once so the kernel stores the frame straight into it (no fresh
    /// allocation, no D2H copy; rrte_hip_sys::safe::Context::render_engine_frame).  false = this frame
    /// goes to the CPU path, whose frame then replaces `out`.
    fn render_into(&self, objects: &[Arc<dyn SceneObject>], lights: &[Arc<dyn Light>], _materials: &[Arc<dyn Material>],
                   camera: &Camera, config: &RaytracerConfig, out: &mut Vec<u8>) -> bool {
        let Some(scene) = lower_scene(objects, lights, camera) else { return false };
        let params = lower_config(config, &self.options);
        let Ok(mut ctx) = self.ctx.lock() else { return false };
        match ctx.render_engine_frame(&scene, &params, out) {
            Ok(()) => true,
            Err(e) => {
                log::warn!("rrte_hip frame failed, rendering on the CPU: {e}");
                false
            }
        }
    }
}
