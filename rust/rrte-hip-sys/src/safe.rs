//! Safe wrapper over the C ABI (the only `unsafe` code of the integration): an owned context, an
//! owned lowered scene, owned frames.  rrte-renderer-hip (which keeps the workspace's
//! `unsafe_code = "forbid"`) builds on this module only.
//!
//! Conventions of include/rrte_hip.h: the caller owns every buffer, the context owns device memory
//! and streams, no panic or exception crosses the ABI, one context per thread (not internally
//! synchronised: `&mut self` here), multi-GPU is internal to the context.
use crate::*;
use std::ffi::CStr;
use std::fmt;

/// A failed call: the status and the library's message (rrte_hip_last_error).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Error {
    pub status: rrte_status,
    pub message: String,
}

impl fmt::Display for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        let name = match self.status {
            RRTE_INVALID_ARG => "INVALID_ARG",
            RRTE_HIP_ERROR => "HIP_ERROR",
            RRTE_RCCL_ERROR => "RCCL_ERROR",
            RRTE_UNSUPPORTED_PRIM => "UNSUPPORTED_PRIM",
            RRTE_NO_DEVICE => "NO_DEVICE",
            _ => "UNKNOWN",
        };
        write!(f, "rrte_hip {name}: {}", self.message)
    }
}

impl std::error::Error for Error {}

/// A lowered scene: the arrays an `rrte_scene_ir` points into, owned by Rust.
#[derive(Clone, Default)]
pub struct SceneIr {
    pub prims: Vec<rrte_prim>,
    pub materials: Vec<rrte_material>,
    pub lights: Vec<rrte_light>,
    pub sdf_nodes: Vec<rrte_sdf_node>,
    pub camera: rrte_camera,
    pub mesh_vertices: Vec<rrte_mesh_vertex>,
    pub mesh_indices: Vec<u32>,
    /// Caller-maintained dirty stamp of the mesh arrays (0: compared byte for byte), the analogue of
    /// Scene::is_dirty (crates/rrte-scene/src/lib.rs:310-312).
    pub mesh_version: u64,
}

impl SceneIr {
    /// The C view of the arrays; valid while `self` is neither moved nor modified.
    fn raw(&self) -> rrte_scene_ir {
        rrte_scene_ir {
            prims: self.prims.as_ptr(),
            num_prims: self.prims.len() as u32,
            materials: self.materials.as_ptr(),
            num_materials: self.materials.len() as u32,
            lights: self.lights.as_ptr(),
            num_lights: self.lights.len() as u32,
            sdf_nodes: self.sdf_nodes.as_ptr(),
            num_sdf_nodes: self.sdf_nodes.len() as u32,
            camera: self.camera,
            mesh_vertices: self.mesh_vertices.as_ptr(),
            num_mesh_vertices: self.mesh_vertices.len() as u32,
            mesh_indices: self.mesh_indices.as_ptr(),
            num_mesh_indices: self.mesh_indices.len() as u32,
            mesh_version: self.mesh_version,
        }
    }
}

/// A page-aligned host buffer rounded up to whole pages (hipHostRegister pins whole pages,
/// so a buffer that shares a heap page with another registered range makes the second registration
/// fail; this one shares none).  Owned by the context that pinned it.
struct PageBuf {
    ptr: *mut u8,
    len: usize,
    layout: std::alloc::Layout,
}

const PAGE: usize = 4096;

impl PageBuf {
    fn new(len: usize) -> Option<PageBuf> {
        let size = len.max(1).checked_add(PAGE - 1)? & !(PAGE - 1);
        let layout = std::alloc::Layout::from_size_align(size, PAGE).ok()?;
        let ptr = unsafe { std::alloc::alloc_zeroed(layout) };
        if ptr.is_null() {
            return None;
        }
        Some(PageBuf { ptr, len, layout })
    }
    fn bytes(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl Drop for PageBuf {
    fn drop(&mut self) {
        unsafe { std::alloc::dealloc(self.ptr, self.layout) };
    }
}

/// One rrte_hip context on one HIP device.
pub struct Context {
    ctx: *mut rrte_ctx,
    // a frame buffer the context owns and keeps pinned (rrte_hip_host_register): render_pinned has the
    // kernel store each frame straight into it (no D2H copy after the render)
    frame: Option<PageBuf>,
    // a caller buffer pinned by render_engine_frame: (address, length), or the address of the last
    // buffer that could not be pinned (tried once, then the copy path)
    pinned: Option<(usize, usize)>,
    unpinnable: usize,
}

// A context may move between threads (it is used by one thread at a time: `&mut self`).
unsafe impl Send for Context {}

impl Context {
    /// rrte_hip_create: a context on HIP device `device` (RRTE_NO_DEVICE without one).
    pub fn new(device: i32) -> Result<Self, Error> {
        let mut ctx: *mut rrte_ctx = std::ptr::null_mut();
        let st = unsafe { rrte_hip_create(device, &mut ctx) };
        if st != RRTE_OK || ctx.is_null() {
            return Err(Error { status: st, message: "rrte_hip_create failed (no HIP device?)".into() });
        }
        if unsafe { rrte_hip_abi_version() } != RRTE_ABI_VERSION {
            unsafe { rrte_hip_destroy(ctx) };
            return Err(Error { status: RRTE_INVALID_ARG, message: "librrte_hip ABI version mismatch".into() });
        }
        Ok(Self { ctx, frame: None, pinned: None, unpinnable: 0 })
    }

    fn check(&self, st: rrte_status) -> Result<(), Error> {
        if st == RRTE_OK {
            return Ok(());
        }
        let message = unsafe { CStr::from_ptr(rrte_hip_last_error(self.ctx)) }.to_string_lossy().into_owned();
        Err(Error { status: st, message })
    }

    /// Raytracer::render on the GPU: a new W*H*4 RGBA8 buffer, row 0 = top (raytracer.rs:54-89).
    pub fn render(&mut self, scene: &SceneIr, params: &rrte_render_params) -> Result<Vec<u8>, Error> {
        let mut out = vec![0u8; params.width as usize * params.height as usize * 4];
        self.render_into(scene, params, &mut out)?;
        Ok(out)
    }

    /// The same into a caller buffer of at least W*H*4 bytes (Engine::frame_buffer, reused per frame).
    pub fn render_into(&mut self, scene: &SceneIr, params: &rrte_render_params, out: &mut [u8]) -> Result<(), Error> {
        let need = params.width as usize * params.height as usize * 4;
        if out.len() < need {
            return Err(Error { status: RRTE_INVALID_ARG, message: format!("output buffer {} < {need} bytes", out.len()) });
        }
        let ir = scene.raw();
        let st = unsafe { rrte_hip_render(self.ctx, &ir, params, out.as_mut_ptr()) };
        self.check(st)
    }

    /// Engine::render_frame's loop (engine.rs:82,293): the frame into the engine's own `frame_buffer`,
    /// reused every frame and pinned once (rrte_hip_host_register), so the kernel stores the frame
    /// straight into it (the boundary's fast path; bench.py `boundary.ms_per_frame_engine_loop`).  The
    /// buffer is resized to W*H*4 bytes when needed; a buffer that moved since it was pinned (the
    /// engine reallocated it) is unpinned before the new one is pinned, and a buffer that cannot be
    /// pinned (one of its pages already pinned by someone else) is rendered through the copy path.
    pub fn render_engine_frame(&mut self, scene: &SceneIr, params: &rrte_render_params, out: &mut Vec<u8>)
                               -> Result<(), Error> {
        let need = params.width as usize * params.height as usize * 4;
        let cur = (out.as_ptr() as usize, out.len());
        if self.pinned.is_some() && (self.pinned != Some(cur) || out.len() != need) {
            self.unpin_engine_frame()?;  // (before a resize may move or free it)
        }
        if out.len() != need {
            out.resize(need, 0);
        }
        let addr = out.as_ptr() as usize;
        if self.pinned.is_none() && self.unpinnable != addr {
            let st = unsafe { rrte_hip_host_register(self.ctx, out.as_mut_ptr() as *mut c_void, out.len()) };
            if st == RRTE_OK {
                self.pinned = Some((addr, out.len()));
            } else {
                self.unpinnable = addr;
            }
        }
        self.render_into(scene, params, out)
    }

    /// Unpins the buffer render_engine_frame pinned (after the context's frames have completed).
    pub fn unpin_engine_frame(&mut self) -> Result<(), Error> {
        if let Some((addr, _)) = self.pinned.take() {
            self.check(unsafe { rrte_hip_host_unregister(self.ctx, addr as *mut c_void) })?;
        }
        Ok(())
    }

    /// Gives the context a pinned frame buffer of `len` bytes (at least W*H*4 of the frames to come):
    /// page-aligned, whole pages, registered once (rrte_hip_host_register); `render_pinned` then has the
    /// kernel store each frame straight into it.  A previous buffer is unpinned and freed.
    pub fn set_frame_buffer(&mut self, len: usize) -> Result<(), Error> {
        self.release_frame_buffer()?;
        let buf = PageBuf::new(len)
            .ok_or_else(|| Error { status: RRTE_INVALID_ARG, message: format!("cannot allocate {len} bytes") })?;
        self.check(unsafe { rrte_hip_host_register(self.ctx, buf.ptr as *mut c_void, buf.layout.size()) })?;
        self.frame = Some(buf);
        Ok(())
    }

    /// Unpins and frees the frame buffer (after the context's frames have completed).
    pub fn release_frame_buffer(&mut self) -> Result<(), Error> {
        if let Some(buf) = self.frame.take() {
            let st = unsafe { rrte_hip_host_unregister(self.ctx, buf.ptr as *mut c_void) };
            if st != RRTE_OK {
                self.frame = Some(buf);
                return Err(self.check(st).unwrap_err());
            }
        }
        Ok(())
    }

    /// Raytracer::render into the pinned frame buffer (set_frame_buffer): the frame's W*H*4 bytes.
    pub fn render_pinned(&mut self, scene: &SceneIr, params: &rrte_render_params) -> Result<&[u8], Error> {
        let need = params.width as usize * params.height as usize * 4;
        let ptr = match self.frame.as_ref() {
            Some(b) if b.len >= need => b.ptr,
            _ => return Err(Error { status: RRTE_INVALID_ARG, message: format!("no pinned frame buffer of {need} bytes") }),
        };
        let ir = scene.raw();
        self.check(unsafe { rrte_hip_render(self.ctx, &ir, params, ptr) })?;
        Ok(&self.frame.as_ref().unwrap().bytes()[..need])
    }

    /// The device code's build id (rrte_hip_build_id: device headers, hiprtc options and version).
    pub fn build_id() -> Result<String, Error> {
        let mut buf = [0 as c_char; 64];
        let st = unsafe { rrte_hip_build_id(buf.as_mut_ptr(), buf.len()) };
        if st != RRTE_OK {
            return Err(Error { status: st, message: "rrte_hip_build_id failed".into() });
        }
        Ok(unsafe { CStr::from_ptr(buf.as_ptr()) }.to_string_lossy().into_owned())
    }

    /// Statistics of the last frame (rays cast, kernel time, gather time, upload time).
    pub fn stats(&self) -> Result<rrte_stats, Error> {
        let mut s = rrte_stats::default();
        self.check(unsafe { rrte_hip_stats(self.ctx, &mut s) })?;
        Ok(s)
    }

    /// Scene-specialised kernels: RRTE_JIT_OFF / RRTE_JIT_ON / RRTE_JIT_AUTO (default).
    pub fn set_jit(&mut self, mode: c_int) -> Result<(), Error> {
        self.check(unsafe { rrte_hip_set_jit(self.ctx, mode) })
    }

    /// Multi-GPU: the 128-byte unique id rank 0 creates and broadcasts out of band.
    pub fn comm_unique_id() -> Result<[u8; RRTE_UNIQUE_ID_BYTES], Error> {
        let mut id = [0u8; RRTE_UNIQUE_ID_BYTES];
        let st = unsafe { rrte_hip_comm_unique_id(id.as_mut_ptr()) };
        if st != RRTE_OK {
            return Err(Error { status: st, message: "rrte_hip_comm_unique_id failed".into() });
        }
        Ok(id)
    }

    /// Joins the RCCL communicator (one process per GPU, every rank calls it).
    pub fn comm_init(&mut self, nranks: i32, rank: i32, id: &[u8; RRTE_UNIQUE_ID_BYTES]) -> Result<(), Error> {
        self.check(unsafe { rrte_hip_comm_init(self.ctx, nranks, rank, id.as_ptr()) })
    }

    /// Bounded waits: a gather that does not complete within `ms` aborts the communicator.
    pub fn set_comm_timeout(&mut self, ms: u32) -> Result<(), Error> {
        self.check(unsafe { rrte_hip_set_comm_timeout(self.ctx, ms) })
    }

    /// One frame over every rank: this rank's row bands, gathered to `root`, which gets the frame.
    pub fn render_gather(&mut self, scene: &SceneIr, params: &rrte_render_params, root: i32, is_root: bool)
                         -> Result<Option<Vec<u8>>, Error> {
        let ir = scene.raw();
        if is_root {
            let mut out = vec![0u8; params.width as usize * params.height as usize * 4];
            self.check(unsafe { rrte_hip_render_gather(self.ctx, &ir, params, root, out.as_mut_ptr()) })?;
            Ok(Some(out))
        } else {
            self.check(unsafe { rrte_hip_render_gather(self.ctx, &ir, params, root, std::ptr::null_mut()) })?;
            Ok(None)
        }
    }
}

/// The band partition of a multi-GPU frame (include/rrte_hip.h rrte_hip_band_layout): the number of
/// leading bands rank 0 renders because no object reaches them, then the round-robin ratio -- root
/// bands, then peer bands per peer, per cycle.  Host arithmetic only; every rank gets the same answer.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct BandLayout {
    pub sky_bands: u32,
    pub root_bands: u32,
    pub peer_bands: u32,
}

impl BandLayout {
    pub fn of(scene: &SceneIr, params: &rrte_render_params, nranks: i32, root: i32) -> Result<BandLayout, Error> {
        let ir = scene.raw();
        let (mut sky, mut rb, mut pb) = (0u32, 0u32, 0u32);
        let st = unsafe { rrte_hip_band_layout(&ir, params, nranks, root, &mut sky, &mut rb, &mut pb) };
        if st != RRTE_OK {
            return Err(Error { status: st, message: "rrte_hip_band_layout failed".into() });
        }
        Ok(BandLayout { sky_bands: sky, root_bands: rb, peer_bands: pb })
    }

    /// Rows `rank` renders under this partition (packed in image order).
    pub fn rows_for_rank(&self, height: u32, band_rows: u32, nranks: i32, rank: i32) -> u32 {
        unsafe {
            rrte_hip_band_rows_for_rank_ex(height, band_rows, nranks, rank, self.sky_bands, self.root_bands,
                                           self.peer_bands)
        }
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        // rrte_hip_destroy unregisters every pinned range after its frames; the frame buffer is freed
        // after that (field drop order: `frame` outlives the destroy call)
        unsafe { rrte_hip_destroy(self.ctx) };
    }
}
