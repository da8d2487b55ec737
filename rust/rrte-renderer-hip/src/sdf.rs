//! The SDF / CSG / Deformer surface the reference documents but does not implement
//! (README.md:66-78, 228-244, 303-328, 458-510): signed-distance leaves, the six CSG operations with
//! `smooth_min` (README.md:485-488), chainable deformers, and `SdfObject`, a `SceneObject` that
//! sphere-traces its SDF.  Build-defined semantics, identical to the C++ mirror
//! (rrte_amd/cpp/rrte_renderer.cpp, checked mechanically by tests/test_rust_binding.py), the oracle
//! (oracle/rrte_oracle.c sdf_leaf / sdf_deform / sdf_eval / sdf_intersect) and the device kernels.
//!
//! Every SDF lowers to a postfix program of `rrte_sdf_node`s (leaves push a distance, CSG ops pop
//! two and push one, deformers push the point and replace it, POP_POINT restores it).  The CPU
//! `distance` / `intersect` evaluate that same program in the same f32 operation order, so the CPU
//! fallback and the GPU agree bit for bit on the linear image.
use rrte_hip_sys::*;
use rrte_math::{HitInfo, Ray, Transform, Vec3};
use rrte_renderer::gpu_desc::{GpuObject, GpuShape};
use rrte_renderer::{Material, SceneObject};
use std::fmt;
use std::sync::Arc;

/// Conservative bounding sphere (double precision, like the C++ and Python mirrors).
#[derive(Debug, Clone, Copy)]
pub struct Bound {
    pub c: [f64; 3],
    pub r: f64,
}

fn make_bound(c: Vec3, r: f64) -> Bound {
    Bound { c: [c.x as f64, c.y as f64, c.z as f64], r }
}

fn dist3(a: &[f64; 3], b: &[f64; 3]) -> f64 {
    let (dx, dy, dz) = (a[0] - b[0], a[1] - b[1], a[2] - b[2]);
    (dx * dx + dy * dy + dz * dz).sqrt()
}

fn about_pivot(pivot: Vec3, b: Bound) -> Bound {
    let p = [pivot.x as f64, pivot.y as f64, pivot.z as f64];
    Bound { c: p, r: dist3(&p, &b.c) + b.r }
}

/// An invalid SDF description (the C ABI would return RRTE_UNSUPPORTED_PRIM / RRTE_INVALID_ARG).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct SdfError(pub &'static str);

impl fmt::Display for SdfError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        f.write_str(self.0)
    }
}

impl std::error::Error for SdfError {}

fn axis_index(a: Vec3) -> Result<u32, SdfError> {
    let c = [a.x, a.y, a.z];
    for i in 0..3 {
        if c[i].abs() == 1.0 && (0..3).all(|j| j == i || c[j] == 0.0) {
            return Ok(i as u32);
        }
    }
    Err(SdfError("deformer axis must be a coordinate axis"))
}

fn node(op: u32, f: &[f32], iv: &[u32]) -> rrte_sdf_node {
    let mut n = rrte_sdf_node::default();
    n.op = op;
    n.f[..f.len()].copy_from_slice(f);
    n.i[..iv.len()].copy_from_slice(iv);
    n
}

/// `SDF` (README.md:458-467): a signed distance, lowered to a postfix program.
pub trait Sdf: Send + Sync + fmt::Debug {
    /// Appends this SDF's postfix program.
    fn emit(&self, out: &mut Vec<rrte_sdf_node>);
    /// Conservative bounding sphere of the zero set (where the sphere tracer marches).
    fn bound(&self) -> Bound;
    fn has_deformer(&self) -> bool {
        false
    }
    /// `SDF::distance` on the CPU: the lowered program evaluated at `p`.
    fn distance(&self, p: Vec3) -> f32 {
        let mut prog = Vec::new();
        self.emit(&mut prog);
        eval_program(&prog, p)
    }
}

pub type SdfRef = Arc<dyn Sdf>;

/// `Deformer` (README.md:496-502): a point map applied before the SDF it deforms; `chain` below.
pub trait Deformer: Send + Sync + fmt::Debug {
    fn nodes(&self, out: &mut Vec<rrte_sdf_node>);
    /// The bound of a deformed SDF from the undeformed one.
    fn grow(&self, b: Bound) -> Bound;
    /// `Deformer::deform` on the CPU (the chain's nodes applied in order).
    fn deform(&self, p: Vec3) -> Vec3 {
        let mut ns = Vec::new();
        self.nodes(&mut ns);
        ns.iter().fold(p, |q, n| deform_point(n, q))
    }
}

pub type DeformerRef = Arc<dyn Deformer>;

#[derive(Debug)]
struct Leaf {
    op: u32,
    c: Vec3,
    f: Vec<f32>,
    r: f64,
}

impl Sdf for Leaf {
    fn emit(&self, out: &mut Vec<rrte_sdf_node>) {
        let mut n = node(self.op, &[], &[]);
        n.f[0] = self.c.x;
        n.f[1] = self.c.y;
        n.f[2] = self.c.z;
        for (k, v) in self.f.iter().enumerate() {
            n.f[3 + k] = *v;
        }
        out.push(n);
    }
    fn bound(&self) -> Bound {
        make_bound(self.c, self.r)
    }
}

/// CSG operations (README.md:475-482); the smooth ones blend over `k` (README.md:485-488).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub enum CsgOperation {
    Union = 0,
    Difference = 1,
    Intersection = 2,
    SmoothUnion = 3,
    SmoothDifference = 4,
    SmoothIntersection = 5,
}

#[derive(Debug)]
struct Composite {
    a: SdfRef,
    b: SdfRef,
    op: CsgOperation,
    k: f32,
}

impl Sdf for Composite {
    fn emit(&self, out: &mut Vec<rrte_sdf_node>) {
        self.a.emit(out);
        self.b.emit(out);
        out.push(node(RRTE_SDF_UNION + self.op as u32, &[self.k], &[]));
    }
    fn bound(&self) -> Bound {
        let (ba, bb) = (self.a.bound(), self.b.bound());
        let k = (self.k as f64).abs();
        let mut r = match self.op {
            CsgOperation::Union | CsgOperation::SmoothUnion => {
                let d = dist3(&ba.c, &bb.c);
                if d + bb.r <= ba.r {
                    ba
                } else if d + ba.r <= bb.r {
                    bb
                } else {
                    let rr = (d + ba.r + bb.r) * 0.5;
                    let t = if d > 0.0 { (rr - ba.r) / d } else { 0.0 };
                    Bound {
                        c: [ba.c[0] + (bb.c[0] - ba.c[0]) * t, ba.c[1] + (bb.c[1] - ba.c[1]) * t,
                            ba.c[2] + (bb.c[2] - ba.c[2]) * t],
                        r: rr,
                    }
                }
            }
            CsgOperation::Difference | CsgOperation::SmoothDifference => ba,
            _ => {
                if ba.r <= bb.r {
                    ba
                } else {
                    bb
                }
            }
        };
        r.r += k;
        r
    }
    fn has_deformer(&self) -> bool {
        self.a.has_deformer() || self.b.has_deformer()
    }
}

type GrowFn = fn(&SimpleDeformer, Bound) -> Bound;

struct SimpleDeformer {
    n: rrte_sdf_node,
    pivot: Vec3,
    grow: GrowFn,
    pa: f64,
    pb: f64,
    octaves: u32,
}

impl fmt::Debug for SimpleDeformer {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "Deformer(op {}, pivot {:?})", self.n.op, self.pivot)
    }
}

impl Deformer for SimpleDeformer {
    fn nodes(&self, out: &mut Vec<rrte_sdf_node>) {
        out.push(self.n);
    }
    fn grow(&self, b: Bound) -> Bound {
        (self.grow)(self, b)
    }
}

#[derive(Debug, Default)]
struct Chain {
    parts: Vec<DeformerRef>,
}

impl Deformer for Chain {
    fn nodes(&self, out: &mut Vec<rrte_sdf_node>) {
        for p in &self.parts {
            p.nodes(out);
        }
    }
    fn grow(&self, mut b: Bound) -> Bound {
        for p in self.parts.iter().rev() {
            b = p.grow(b); // innermost first
        }
        b
    }
}

#[derive(Debug)]
struct Deformed {
    s: SdfRef,
    d: DeformerRef,
}

impl Sdf for Deformed {
    fn emit(&self, out: &mut Vec<rrte_sdf_node>) {
        let mut ns = Vec::new();
        self.d.nodes(&mut ns);
        let n = ns.len();
        out.extend(ns);
        self.s.emit(out);
        for _ in 0..n {
            out.push(node(RRTE_SDF_POP_POINT, &[], &[]));
        }
    }
    fn bound(&self) -> Bound {
        self.d.grow(self.s.bound())
    }
    fn has_deformer(&self) -> bool {
        true
    }
}

// ------------------------------------------------------------------ builders (README.md:303-328)
pub fn sdf_sphere(c: Vec3, r: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_SPHERE, c, f: vec![r as f32], r })
}
pub fn sdf_box(c: Vec3, s: Vec3) -> SdfRef {
    let (sx, sy, sz) = (s.x as f64, s.y as f64, s.z as f64);
    Arc::new(Leaf { op: RRTE_SDF_BOX, c, f: vec![0.0, s.x, s.y, s.z], r: 0.5 * (sx * sx + sy * sy + sz * sz).sqrt() })
}
pub fn sdf_cylinder(c: Vec3, r: f64, h: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_CYLINDER, c, f: vec![r as f32, h as f32], r: r.hypot(h * 0.5) })
}
pub fn sdf_prism(c: Vec3, s: Vec3) -> SdfRef {
    let (a, b, d) = (s.y as f64 * 0.5, s.y as f64 * 0.433, s.z as f64 * 0.5);
    Arc::new(Leaf { op: RRTE_SDF_PRISM, c, f: vec![0.0, s.x, s.y, s.z], r: (a * a + b * b + d * d).sqrt() })
}
pub fn sdf_torus(c: Vec3, major: f64, minor: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_TORUS, c, f: vec![major as f32, minor as f32], r: major + minor })
}
pub fn sdf_tube(c: Vec3, ro: f64, ri: f64, h: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_TUBE, c, f: vec![ro as f32, ri as f32, h as f32], r: ro.hypot(h * 0.5) })
}
pub fn sdf_ring(c: Vec3, major: f64, minor: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_RING, c, f: vec![major as f32, minor as f32], r: major + minor })
}
pub fn sdf_cone(c: Vec3, r: f64, h: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_CONE, c, f: vec![r as f32, h as f32], r: r.hypot(h * 0.5) })
}
pub fn sdf_capsule(c: Vec3, r: f64, h: f64) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_CAPSULE, c, f: vec![r as f32, h as f32], r: h * 0.5 + r })
}
pub fn sdf_ellipsoid(c: Vec3, radii: Vec3) -> SdfRef {
    Arc::new(Leaf { op: RRTE_SDF_ELLIPSOID, c, f: vec![0.0, radii.x, radii.y, radii.z],
                    r: radii.x.max(radii.y.max(radii.z)) as f64 })
}
pub fn csg(a: SdfRef, b: SdfRef, op: CsgOperation, k: f32) -> SdfRef {
    Arc::new(Composite { a, b, op, k })
}

pub fn twist(axis: Vec3, rate: f32, pivot: Vec3) -> Result<DeformerRef, SdfError> {
    Ok(Arc::new(SimpleDeformer {
        n: node(RRTE_SDF_TWIST, &[pivot.x, pivot.y, pivot.z, rate], &[axis_index(axis)?]),
        pivot, grow: |d, b| about_pivot(d.pivot, b), pa: 0.0, pb: 0.0, octaves: 0,
    }))
}
pub fn bend(axis: Vec3, direction: Vec3, amount: f32, pivot: Vec3) -> Result<DeformerRef, SdfError> {
    Ok(Arc::new(SimpleDeformer {
        n: node(RRTE_SDF_BEND, &[pivot.x, pivot.y, pivot.z, amount], &[axis_index(axis)?, axis_index(direction)?]),
        pivot, grow: |d, b| about_pivot(d.pivot, b), pa: 0.0, pb: 0.0, octaves: 0,
    }))
}
pub fn taper(axis: Vec3, start: f32, end: f32, length: f32, pivot: Vec3) -> Result<DeformerRef, SdfError> {
    Ok(Arc::new(SimpleDeformer {
        n: node(RRTE_SDF_TAPER, &[pivot.x, pivot.y, pivot.z, start, end, length], &[axis_index(axis)?]),
        pivot,
        grow: |d, b| {
            let mut p = about_pivot(d.pivot, b);
            p.r *= 1.0f64.max(d.pa.abs().max(d.pb.abs()));
            p
        },
        pa: start as f64, pb: end as f64, octaves: 0,
    }))
}
pub fn noise(frequency: f32, amplitude: f32, pivot: Vec3, seed: u32, octaves: u32, persistence: f32)
             -> Result<DeformerRef, SdfError> {
    if octaves > RRTE_SDF_MAX_OCTAVES {
        return Err(SdfError("noise octaves > RRTE_SDF_MAX_OCTAVES"));
    }
    Ok(Arc::new(SimpleDeformer {
        n: node(RRTE_SDF_NOISE, &[pivot.x, pivot.y, pivot.z, frequency, amplitude, persistence], &[octaves, seed]),
        pivot,
        grow: |d, mut b| {
            let total: f64 = (0..d.octaves).map(|o| d.pb.abs().powi(o as i32)).sum();
            b.r += 3f64.sqrt() * d.pa.abs() * total;
            b
        },
        pa: amplitude as f64, pb: persistence as f64, octaves,
    }))
}
pub fn wave(axis: Vec3, amplitude: f32, frequency: f32, displaced_axis: Vec3, pivot: Vec3) -> Result<DeformerRef, SdfError> {
    Ok(Arc::new(SimpleDeformer {
        n: node(RRTE_SDF_WAVE, &[pivot.x, pivot.y, pivot.z, amplitude, frequency],
                &[axis_index(axis)?, axis_index(displaced_axis)?]),
        pivot,
        grow: |d, mut b| {
            b.r += d.pa.abs();
            b
        },
        pa: amplitude as f64, pb: 0.0, octaves: 0,
    }))
}
/// `first.chain(then)` (README.md:496-510): `then(first(p))`; chains flatten.
pub fn chain(first: DeformerRef, then: DeformerRef) -> DeformerRef {
    let mut c = Chain::default();
    c.parts.push(first);
    c.parts.push(then); // (nested chains need no flattening: nodes and grow recurse in order)
    Arc::new(c)
}
pub fn deformed(sdf: SdfRef, d: DeformerRef) -> SdfRef {
    Arc::new(Deformed { s: sdf, d })
}

// ------------------------------------------------------- CPU evaluation (oracle/rrte_oracle.c order)
/// Deterministic sin/cos: 3-part Cody-Waite reduction by pi/2 and cephes minimax polynomials, the
/// device's and the oracle's operation order.
pub fn sincos(x: f32) -> (f32, f32) {
    let k = (x * 0.636619772 + 0.5).floor();
    let r = ((x - k * 1.5703125) - k * 4.837512969970703125e-4) - k * 7.549789948768648e-8;
    let r2 = r * r;
    let s = r + (r * r2) * (-1.6666654611e-1 + r2 * (8.3321608736e-3 + r2 * -1.9515295891e-4));
    let c = (1.0 - 0.5 * r2) + (r2 * r2) * (4.166664568298827e-2 + r2 * (-1.388731625493765e-3 + r2 * 2.443315711809948e-5));
    match (k as i32) & 3 {
        0 => (s, c),
        1 => (c, -s),
        2 => (-s, -c),
        _ => (-c, s),
    }
}

fn lattice(ix: i32, iy: i32, iz: i32, seed: u32) -> f32 {
    let mut h = seed ^ (ix as u32).wrapping_mul(0x8da6b343) ^ (iy as u32).wrapping_mul(0xd8163841)
        ^ (iz as u32).wrapping_mul(0xcb1ab31f);
    h = (h ^ (h >> 16)).wrapping_mul(0x7feb352d);
    h = (h ^ (h >> 15)).wrapping_mul(0x846ca68b);
    h ^= h >> 16;
    (h >> 8) as f32 * 1.1920928955078125e-7 - 1.0
}

fn lerp(a: f32, b: f32, t: f32) -> f32 {
    a + (b - a) * t
}

/// Value noise on the integer lattice with smoothstep fade.
pub fn value_noise(x: f32, y: f32, z: f32, seed: u32) -> f32 {
    let (fx0, fy0, fz0) = (x.floor(), y.floor(), z.floor());
    let (ix, iy, iz) = (fx0 as i32, fy0 as i32, fz0 as i32);
    let (fx, fy, fz) = (x - fx0, y - fy0, z - fz0);
    let ux = fx * fx * (3.0 - 2.0 * fx);
    let uy = fy * fy * (3.0 - 2.0 * fy);
    let uz = fz * fz * (3.0 - 2.0 * fz);
    let l = |a: i32, b: i32, c: i32| lattice(ix.wrapping_add(a), iy.wrapping_add(b), iz.wrapping_add(c), seed);
    let x00 = lerp(l(0, 0, 0), l(1, 0, 0), ux);
    let x10 = lerp(l(0, 1, 0), l(1, 1, 0), ux);
    let x01 = lerp(l(0, 0, 1), l(1, 0, 1), ux);
    let x11 = lerp(l(0, 1, 1), l(1, 1, 1), ux);
    lerp(lerp(x00, x10, uy), lerp(x01, x11, uy), uz)
}

fn len2(a: f32, b: f32) -> f32 {
    (a * a + b * b).sqrt()
}
fn len3(a: f32, b: f32, c: f32) -> f32 {
    ((a * a + b * b) + c * c).sqrt()
}
// IEEE minNum / maxNum (the device's v_min_f32 / v_max_f32; fminf / fmaxf in the oracle)
fn smn(a: f32, b: f32) -> f32 {
    a.min(b)
}
fn smx(a: f32, b: f32) -> f32 {
    a.max(b)
}
fn sclamp(x: f32, lo: f32, hi: f32) -> f32 {
    smn(smx(x, lo), hi)
}

fn leaf_distance(n: &rrte_sdf_node, p: Vec3) -> f32 {
    let f = &n.f;
    let q = Vec3::new(p.x - f[0], p.y - f[1], p.z - f[2]);
    match n.op {
        RRTE_SDF_SPHERE => len3(q.x, q.y, q.z) - f[3],
        RRTE_SDF_BOX => {
            let (dx, dy, dz) = (q.x.abs() - f[4] * 0.5, q.y.abs() - f[5] * 0.5, q.z.abs() - f[6] * 0.5);
            len3(smx(dx, 0.0), smx(dy, 0.0), smx(dz, 0.0)) + smn(smx(dx, smx(dy, dz)), 0.0)
        }
        RRTE_SDF_CYLINDER => {
            let (dx, dy) = (len2(q.x, q.z) - f[3], q.y.abs() - f[4] * 0.5);
            smn(smx(dx, dy), 0.0) + len2(smx(dx, 0.0), smx(dy, 0.0))
        }
        RRTE_SDF_PRISM => {
            let a = smx(q.x.abs() * 0.866025 + q.y * 0.5, -q.y) - f[5] * 0.25;
            smx(q.z.abs() - f[6] * 0.5, a)
        }
        RRTE_SDF_TORUS => len2(len2(q.x, q.z) - f[3], q.y) - f[4],
        RRTE_SDF_TUBE => {
            let rad = len2(q.x, q.z);
            let (mid, half) = ((f[3] + f[4]) * 0.5, (f[3] - f[4]) * 0.5);
            let (dx, dy) = ((rad - mid).abs() - half, q.y.abs() - f[5] * 0.5);
            smn(smx(dx, dy), 0.0) + len2(smx(dx, 0.0), smx(dy, 0.0))
        }
        RRTE_SDF_RING => len2(len2(q.x, q.y) - f[3], q.z) - f[4],
        RRTE_SDF_CONE => {
            let (r1, hh) = (f[3], f[4] * 0.5);
            let (qx, qy) = (len2(q.x, q.z), q.y);
            let (k2x, k2y) = (-r1, hh * 2.0);
            let cax = qx - smn(qx, if qy < 0.0 { r1 } else { 0.0 });
            let cay = qy.abs() - hh;
            let (k1mqx, k1mqy) = (0.0 - qx, hh - qy);
            let t = sclamp((k1mqx * k2x + k1mqy * k2y) / (k2x * k2x + k2y * k2y), 0.0, 1.0);
            let (cbx, cby) = ((qx - 0.0) + k2x * t, (qy - hh) + k2y * t);
            let s = if cbx < 0.0 && cay < 0.0 { -1.0 } else { 1.0 };
            s * smn(cax * cax + cay * cay, cbx * cbx + cby * cby).sqrt()
        }
        RRTE_SDF_CAPSULE => {
            let hh = f[4] * 0.5;
            len3(q.x, q.y - sclamp(q.y, -hh, hh), q.z) - f[3]
        }
        RRTE_SDF_ELLIPSOID => {
            let (rx, ry, rz) = (f[4], f[5], f[6]);
            let k0 = len3(q.x / rx, q.y / ry, q.z / rz);
            let k1 = len3(q.x / (rx * rx), q.y / (ry * ry), q.z / (rz * rz));
            if !(k1 > 0.0) {
                -smn(rx, smn(ry, rz))
            } else {
                k0 * (k0 - 1.0) / k1
            }
        }
        _ => f32::INFINITY,
    }
}

/// README.md:485-488: h = clamp(0.5 + 0.5 (b - a) / k); a h + b (1 - h) - k h (1 - h).
pub fn smooth_min(a: f32, b: f32, k: f32) -> f32 {
    let h = sclamp(0.5 + (0.5 * (b - a)) / k, 0.0, 1.0);
    let om = 1.0 - h;
    (a * h + b * om) - (k * h) * om
}

fn comp(v: Vec3, i: u32) -> f32 {
    match i {
        0 => v.x,
        1 => v.y,
        _ => v.z,
    }
}
fn set_comp(v: &mut Vec3, i: u32, s: f32) {
    match i {
        0 => v.x = s,
        1 => v.y = s,
        _ => v.z = s,
    }
}

fn deform_point(n: &rrte_sdf_node, p: Vec3) -> Vec3 {
    let f = &n.f;
    let c = Vec3::new(f[0], f[1], f[2]);
    let mut q = Vec3::new(p.x - c.x, p.y - c.y, p.z - c.z);
    match n.op {
        RRTE_SDF_TWIST | RRTE_SDF_BEND => {
            let ax = n.i[0];
            let drive = if n.op == RRTE_SDF_TWIST { ax } else { n.i[1] };
            let (u, w) = ((ax + 1) % 3, (ax + 2) % 3);
            let (s, co) = sincos(f[3] * comp(q, drive));
            let (qu, qw) = (comp(q, u), comp(q, w));
            set_comp(&mut q, u, co * qu - s * qw);
            set_comp(&mut q, w, s * qu + co * qw);
        }
        RRTE_SDF_TAPER => {
            let ax = n.i[0];
            let (u, w) = ((ax + 1) % 3, (ax + 2) % 3);
            let t = sclamp((comp(q, ax) + f[5] * 0.5) / f[5], 0.0, 1.0);
            let s = f[3] + (f[4] - f[3]) * t;
            let (qu, qw) = (comp(q, u) / s, comp(q, w) / s);
            set_comp(&mut q, u, qu);
            set_comp(&mut q, w, qw);
        }
        RRTE_SDF_NOISE => {
            let (oct, seed) = (n.i[0], n.i[1]);
            let x = Vec3::new(q.x * f[3], q.y * f[3], q.z * f[3]);
            let mut acc = [0.0f32; 3];
            for (k, a) in acc.iter_mut().enumerate() {
                let (mut amp, mut fr, mut sum) = (1.0f32, 1.0f32, 0.0f32);
                for o in 0..oct {
                    let sd = seed.wrapping_add((k as u32).wrapping_mul(0x9e3779b9)).wrapping_add(o.wrapping_mul(0x85ebca6b));
                    sum = sum + amp * value_noise(x.x * fr, x.y * fr, x.z * fr, sd);
                    amp = amp * f[5];
                    fr = fr * 2.0;
                }
                *a = sum;
            }
            q = Vec3::new(q.x + f[4] * acc[0], q.y + f[4] * acc[1], q.z + f[4] * acc[2]);
        }
        RRTE_SDF_WAVE => {
            let (ax, disp) = (n.i[0], n.i[1]);
            let (s, _) = sincos(f[4] * comp(q, ax));
            let v = comp(q, disp) + f[3] * s;
            set_comp(&mut q, disp, v);
        }
        _ => {}
    }
    Vec3::new(q.x + c.x, q.y + c.y, q.z + c.z)
}

/// Evaluates a postfix SDF program at `p` (oracle/rrte_oracle.c sdf_eval).
pub fn eval_program(nodes: &[rrte_sdf_node], mut p: Vec3) -> f32 {
    let mut vs: Vec<f32> = Vec::with_capacity(RRTE_SDF_MAX_STACK as usize);
    let mut ps: Vec<Vec3> = Vec::with_capacity(RRTE_SDF_MAX_POINT_STACK as usize);
    for n in nodes {
        let op = n.op;
        if op < 32 {
            vs.push(leaf_distance(n, p));
        } else if op < 64 {
            let b = vs.pop().unwrap_or(f32::INFINITY);
            let a = vs.pop().unwrap_or(f32::INFINITY);
            let k = n.f[0];
            vs.push(match op {
                RRTE_SDF_UNION => smn(a, b),
                RRTE_SDF_DIFFERENCE => smx(a, -b),
                RRTE_SDF_INTERSECTION => smx(a, b),
                RRTE_SDF_SMOOTH_UNION => smooth_min(a, b, k),
                RRTE_SDF_SMOOTH_DIFFERENCE => -smooth_min(-a, b, k),
                _ => -smooth_min(-a, -b, k),
            });
        } else if op < 96 {
            ps.push(p);
            p = deform_point(n, p);
        } else if let Some(q) = ps.pop() {
            p = q;
        }
    }
    vs.first().copied().unwrap_or(f32::INFINITY)
}

// ------------------------------------------------------------------------------- SdfObject
/// A lowered SDF program with its march parameters: the payload of `GpuShape::Custom` that
/// lower.rs recognises.
#[derive(Debug, Clone)]
pub struct SdfProgram {
    pub nodes: Vec<rrte_sdf_node>,
    pub bound_center: [f32; 3],
    pub bound_radius: f32,
    pub max_steps: u32,
    pub step_scale: f32,
    pub hit_eps: f32,
}

/// `SDFObject` (README.md:458-467): a SceneObject sphere-tracing an SDF inside its bounding sphere.
#[derive(Debug)]
pub struct SdfObject {
    pub sdf: SdfRef,
    pub material: Option<Arc<dyn Material>>,
    pub transform: Transform,
    program: Arc<SdfProgram>,
}

impl SdfObject {
    /// `step_scale` None: 0.6 when the SDF contains a deformer (not 1-Lipschitz), else 1.0.
    pub fn new(sdf: SdfRef, material: Option<Arc<dyn Material>>, max_steps: u32, step_scale: Option<f32>,
               hit_eps: f32) -> Self {
        let mut nodes = Vec::new();
        sdf.emit(&mut nodes);
        let b = sdf.bound();
        let r = b.r * 1.001 + 1e-3;
        let step_scale = step_scale.unwrap_or(if sdf.has_deformer() { 0.6 } else { 1.0 });
        let program = Arc::new(SdfProgram {
            nodes,
            bound_center: [b.c[0] as f32, b.c[1] as f32, b.c[2] as f32],
            bound_radius: r as f32,
            max_steps,
            step_scale,
            hit_eps,
        });
        Self { sdf, material, transform: Transform::identity(), program }
    }

    /// The defaults of the C++ / Python mirrors: 128 steps, hit when d < 1e-4 t.
    pub fn with_defaults(sdf: SdfRef, material: Option<Arc<dyn Material>>) -> Self {
        Self::new(sdf, material, 128, None, 1e-4)
    }

    pub fn program(&self) -> &SdfProgram {
        &self.program
    }
}

impl SceneObject for SdfObject {
    /// Sphere tracing inside the bounding sphere (oracle/rrte_oracle.c sdf_intersect): from
    /// max(t_min, t_enter) to min(t_max, t_exit), hit when d < hit_eps * t, tetrahedral normal.
    fn intersect(&self, ray: &Ray, t_min: f32, t_max: f32) -> Option<HitInfo> {
        let pr = &self.program;
        let bc = Vec3::from(pr.bound_center);
        let br = pr.bound_radius;
        let oc = Vec3::new(ray.origin.x - bc.x, ray.origin.y - bc.y, ray.origin.z - bc.z);
        let dot = |a: Vec3, b: Vec3| ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z);
        let b = dot(oc, ray.direction);
        let cc = dot(oc, oc) - br * br;
        let disc = b * b - cc;
        if disc < 0.0 {
            return None;
        }
        let sq = disc.sqrt();
        let mut t = if -b - sq > t_min { -b - sq } else { t_min };
        let tend = if -b + sq < t_max { -b + sq } else { t_max };
        if t > tend {
            return None;
        }
        let at = |t: f32| Vec3::new(ray.origin.x + ray.direction.x * t, ray.origin.y + ray.direction.y * t,
                                    ray.origin.z + ray.direction.z * t);
        for _ in 0..pr.max_steps {
            let p = at(t);
            let d = eval_program(&pr.nodes, p);
            if d < pr.hit_eps * t {
                let h = 1e-3f32;
                let f0 = eval_program(&pr.nodes, Vec3::new(p.x + h, p.y - h, p.z - h));
                let f1 = eval_program(&pr.nodes, Vec3::new(p.x - h, p.y - h, p.z + h));
                let f2 = eval_program(&pr.nodes, Vec3::new(p.x - h, p.y + h, p.z - h));
                let f3 = eval_program(&pr.nodes, Vec3::new(p.x + h, p.y + h, p.z + h));
                let n = Vec3::new(((f0 - f1) - f2) + f3, ((-f0 - f1) + f2) + f3, ((-f0 + f1) - f2) + f3);
                return Some(HitInfo::new(t, p, n.normalize(), ray));
            }
            t = t + d * pr.step_scale;
            if t > tend {
                return None;
            }
        }
        None
    }
    fn material(&self) -> Option<Arc<dyn Material>> {
        self.material.clone()
    }
    fn transform(&self) -> &Transform {
        &self.transform
    }
    fn set_transform(&mut self, transform: Transform) {
        self.transform = transform;
    }
    fn gpu_desc(&self) -> Option<GpuObject> {
        Some(GpuObject {
            shape: GpuShape::Custom(self.program.clone()),
            transform: self.transform.clone(),
            material: self.material.clone(),
        })
    }
}
