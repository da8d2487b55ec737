/*
 * rrte_oracle.c — TEST INFRASTRUCTURE ONLY (see rrte_oracle.h header for the
 * parity status).  Plain-C restatement of Melthizar/RRTE's CPU raytracer.
 * Every function cites the reference file:line it restates; paths are
 * relative to the reference root.  Build: oracle/Makefile
 * (-O3 -ffp-contract=off -fno-fast-math: f32 IEEE ops, no FMA contraction,
 * like rustc's codegen for the reference).
 *
 * It restates the reference literally, including its costs: Cube/Cylinder/
 * Cone/Capsule rebuild Transform::to_matrix + inverse per call
 * (primitives.rs:303,421,522,628), objects are scanned linearly per ray
 * (raytracer.rs:106-113), and the frame is split over a work-stealing
 * thread pool of row chunks (the rayon analogue of raytracer.rs:57-60).
 */
#include "rrte_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ glam Vec3 */
typedef struct v3 { float x, y, z; } v3;

/* Event counters (counting build only, see rrte_oracle.h). */
#ifdef RRTE_ORACLE_COUNT
static _Thread_local rrte_oracle_counts* tl_cnt;
#define CNT(f) (++tl_cnt->f)
#else
#define CNT(f) ((void)0)
#endif

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 vmuls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
/* glam Vec3::dot: (x*x') + (y*y') + (z*z'), left to right. */
static inline float vdot(v3 a, v3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
static inline float vlen2(v3 a) { return vdot(a, a); }
static inline float vlen(v3 a) { return sqrtf(vdot(a, a)); }
/* glam Vec3::normalize: self * (1 / length()). */
static inline v3 vnorm(v3 a) { return vmuls(a, 1.0f / sqrtf(vdot(a, a))); }
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }
static inline float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline v3 setcomp(v3 a, int i, float s) {
    if (i == 0) a.x = s; else if (i == 1) a.y = s; else a.z = s;
    return a;
}

/* Explicit min/max so NaN behaviour is pinned (same on the device). */
static inline float mn(float a, float b) { return (b < a) ? b : a; }
static inline float mx(float a, float b) { return (b > a) ? b : a; }
static inline float clampf_(float x, float lo, float hi) { return mn(mx(x, lo), hi); }
/* SDF min/max (build-defined): IEEE-754 minNum/maxNum -- a NaN operand yields the
 * other operand -- which the device evaluates with single v_min_f32/v_max_f32/v_max3_f32/v_med3_f32
 * instructions.  The sign of a zero result when both operands are zeros is unspecified (the device
 * compiler may reassociate); no SDF output depends on it (a distance of +-0 marches and shades alike). */
static inline float smn(float a, float b) { return fminf(a, b); }
static inline float smx(float a, float b) { return fmaxf(a, b); }
static inline float sclamp(float x, float lo, float hi) { return smn(smx(x, lo), hi); }

/* ------------------------------------------------------- rrte_math types */
typedef struct ray { v3 o, d; } ray;
/* Ray::new normalises the direction (rrte-math/src/ray.rs:13-18). */
static inline ray ray_new(v3 o, v3 d) { ray r; r.o = o; r.d = vnorm(d); return r; }
/* Ray::at: origin + t*direction (ray.rs:21-23). */
static inline v3 ray_at(const ray* r, float t) { return vadd(r->o, vmuls(r->d, t)); }

typedef struct hit { float t; v3 p, n; int front; } hit;
/* HitInfo::new: front_face = dot(d, n) < 0, normal flipped to face the ray (ray.rs:45-56). */
static inline hit hit_new(float t, v3 p, v3 outward, const ray* r) {
    hit h;
    h.t = t; h.p = p;
    h.front = vdot(r->d, outward) < 0.0f;
    h.n = h.front ? outward : vneg(outward);
    return h;
}

typedef struct col { float r, g, b, a; } col;
static inline col C4(float r, float g, float b, float a) { col c = {r, g, b, a}; return c; }
static const col BLACK = {0.0f, 0.0f, 0.0f, 1.0f}; /* color.rs:30 */
/* Color add / mul(f32) act on all four channels (color.rs:90-113). */
static inline col cadd(col a, col b) { return C4(a.r + b.r, a.g + b.g, a.b + b.b, a.a + b.a); }
static inline col cmuls(col a, float s) { return C4(a.r * s, a.g * s, a.b * s, a.a * s); }
static inline col cload(const float* p) { return C4(p[0], p[1], p[2], p[3]); }

/* ---------------------------------------------------- glam Quat / Mat4 */
/* Quat * Vec3 (glam mul_vec3a, SSE2): v*(w*w - b.b) + b*((v.b)*2) + (b x v)*(w*2). */
static v3 quat_rotate(const float q[4], v3 v) {
    v3 b = V(q[0], q[1], q[2]);
    float w = q[3];
    float b2 = vdot(b, b);
    float k0 = w * w - b2;
    float k1 = vdot(v, b) * 2.0f;
    float k2 = w * 2.0f;
    v3 c = vcross(b, v);
    return vadd(vadd(vmuls(v, k0), vmuls(b, k1)), vmuls(c, k2));
}

/* Mat4::from_scale_rotation_translation (transform.rs:50-52), column-major m[col*4+row]. */
void rrte_oracle_mat4_srt(const float trs[10], float m[16]) {
    float x = trs[3], y = trs[4], z = trs[5], w = trs[6];
    float x2 = x + x, y2 = y + y, z2 = z + z;
    float xx = x * x2, xy = x * y2, xz = x * z2;
    float yy = y * y2, yz = y * z2, zz = z * z2;
    float wx = w * x2, wy = w * y2, wz = w * z2;
    float sx = trs[7], sy = trs[8], sz = trs[9];
    m[0] = (1.0f - (yy + zz)) * sx; m[1] = (xy + wz) * sx; m[2] = (xz - wy) * sx; m[3] = 0.0f * sx;
    m[4] = (xy - wz) * sy; m[5] = (1.0f - (xx + zz)) * sy; m[6] = (yz + wx) * sy; m[7] = 0.0f * sy;
    m[8] = (xz + wy) * sz; m[9] = (yz - wx) * sz; m[10] = (1.0f - (xx + yy)) * sz; m[11] = 0.0f * sz;
    m[12] = trs[0]; m[13] = trs[1]; m[14] = trs[2]; m[15] = 1.0f;
}

/* Mat4::inverse (transform.rs:55-57): glam's glm-derived cofactor inverse. */
void rrte_oracle_mat4_inverse(const float mm[16], float out[16]) {
#define M(c, r) mm[(c) * 4 + (r)]
    float c00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float c02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float c03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float c04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float c06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float c07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float c08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float c10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float c11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float c12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float c14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float c15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float c16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float c18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float c19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float c20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float c22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float c23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    float f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    float v0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)};
    float v1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    float v2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)};
    float v3_[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    float inv[16];
    for (int i = 0; i < 4; ++i) {
        float sa = (i & 1) ? -1.0f : 1.0f; /* SignA = (+,-,+,-) */
        float sb = -sa;                    /* SignB = (-,+,-,+) */
        inv[0 * 4 + i] = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3_[i] * f2[i]) * sa;
        inv[1 * 4 + i] = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3_[i] * f4[i]) * sb;
        inv[2 * 4 + i] = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3_[i] * f5[i]) * sa;
        inv[3 * 4 + i] = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb;
    }
    float d0 = M(0, 0) * inv[0], d1 = M(0, 1) * inv[4], d2 = M(0, 2) * inv[8], d3 = M(0, 3) * inv[12];
    float det = (d0 + d1) + (d2 + d3);
    float rdet = 1.0f / det;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * rdet;
#undef M
}

/* Mat4::transform_point3 / transform_vector3: ((x*px + y*py) + z*pz) [+ w]. */
static inline v3 m4_point(const float m[16], v3 p) {
    return V(((m[0] * p.x + m[4] * p.y) + m[8] * p.z) + m[12],
             ((m[1] * p.x + m[5] * p.y) + m[9] * p.z) + m[13],
             ((m[2] * p.x + m[6] * p.y) + m[10] * p.z) + m[14]);
}
static inline v3 m4_vector(const float m[16], v3 p) {
    return V((m[0] * p.x + m[4] * p.y) + m[8] * p.z,
             (m[1] * p.x + m[5] * p.y) + m[9] * p.z,
             (m[2] * p.x + m[6] * p.y) + m[10] * p.z);
}

/* Quat::from_rotation_arc(-Z, forward) (camera.rs:85-95 via glam). */
void rrte_oracle_look_at(const float position[3], const float target[3], float q[4]) {
    v3 fwd = vnorm(vsub(vload(target), vload(position)));
    v3 from = V(0.0f, 0.0f, -1.0f);
    const float one_minus_eps = 1.0f - 2.0f * 1.1920929e-7f;
    float d = vdot(from, fwd);
    if (d > one_minus_eps) {
        q[0] = 0.0f; q[1] = 0.0f; q[2] = 0.0f; q[3] = 1.0f;
    } else if (d < -one_minus_eps) {
        /* from_axis_angle(from.any_orthonormal_vector(), PI): axis (1,0,0) for -Z. */
        float half = 3.14159265358979f * 0.5f;
        q[0] = sinf(half); q[1] = 0.0f; q[2] = 0.0f; q[3] = cosf(half);
    } else {
        v3 c = vcross(from, fwd);
        float x = c.x, y = c.y, z = c.z, w = 1.0f + d;
        /* glam Vec4 (SSE2) dot: (x*x + z*z) + (y*y + w*w); normalize divides by length. */
        float len = sqrtf((x * x + z * z) + (y * y + w * w));
        q[0] = x / len; q[1] = y / len; q[2] = z / len; q[3] = w / len;
    }
}

/* Camera::generate_ray (camera.rs:98-133). */
static ray generate_ray(const rrte_camera* cam, float u, float v) {
    float ndc_x = 2.0f * u - 1.0f;
    float ndc_y = 1.0f - 2.0f * v;
    if (cam->projection == RRTE_PERSPECTIVE) {
        float half_h = tanf(cam->fov * 0.5f);
        float half_w = cam->aspect_ratio * half_h;
        v3 cd = vnorm(V(ndc_x * half_w, ndc_y * half_h, -1.0f));
        v3 wd = quat_rotate(cam->rotation, cd);
        return ray_new(vload(cam->position), wd);
    } else {
        float wx = cam->left + (cam->right - cam->left) * u;
        float wy = cam->bottom + (cam->top - cam->bottom) * v;
        float trs[10] = {cam->position[0], cam->position[1], cam->position[2],
                         cam->rotation[0], cam->rotation[1], cam->rotation[2], cam->rotation[3],
                         cam->scale[0], cam->scale[1], cam->scale[2]};
        float m[16];
        rrte_oracle_mat4_srt(trs, m);
        v3 o = m4_point(m, V(wx, wy, 0.0f));
        v3 wd = quat_rotate(cam->rotation, V(0.0f, 0.0f, -1.0f));
        return ray_new(o, wd);
    }
}

void rrte_oracle_generate_ray(const rrte_camera* cam, float u, float v, float o[3], float d[3]) {
    ray r = generate_ray(cam, u, v);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    d[0] = r.d.x; d[1] = r.d.y; d[2] = r.d.z;
}

/* ------------------------------------------------- build-defined math */
/* Deterministic sin/cos (DESIGN.md §SDF "trig"): 3-part Cody-Waite reduction
 * by pi/2 and cephes minimax polynomials; identical op order on the device. */
static inline void sincos_rrte(float x, float* s_out, float* c_out) {
    float k = floorf(x * 0.636619772f + 0.5f);
    float r = ((x - k * 1.5703125f) - k * 4.837512969970703125e-4f) - k * 7.549789948768648e-8f;
    float r2 = r * r;
    float s = r + (r * r2) * (-1.6666654611e-1f + r2 * (8.3321608736e-3f + r2 * -1.9515295891e-4f));
    float c = (1.0f - 0.5f * r2) + (r2 * r2) * (4.166664568298827e-2f + r2 * (-1.388731625493765e-3f + r2 * 2.443315711809948e-5f));
    int q = ((int)k) & 3;
    float so, co;
    if (q == 0) { so = s; co = c; }
    else if (q == 1) { so = c; co = -s; }
    else if (q == 2) { so = -s; co = -c; }
    else { so = -c; co = s; }
    *s_out = so; *c_out = co;
}
float rrte_oracle_sinf(float x) { float s, c; sincos_rrte(x, &s, &c); return s; }
float rrte_oracle_cosf(float x) { float s, c; sincos_rrte(x, &s, &c); return c; }

/* Three-channel value noise (build-defined, DESIGN.md §6 'Deformers'): every lattice corner has ONE
 * 32-bit hash of (seed, corner) -- the xor of per-axis multiplies, then a 32-bit finaliser -- whose
 * bits give the corner's three values in [-1, 1): bits 0-10 and 11-21 (11 bits each, step 2^-10) and
 * bits 22-31 (10 bits, step 2^-9); each channel is interpolated trilinearly with the smoothstep fade
 * 3t^2 - 2t^3.  (Rounds 1-5 hashed each channel separately; one hash per corner is a third of the
 * integer work) */
static inline uint32_t lattice_hash(int32_t ix, int32_t iy, int32_t iz, uint32_t seed) {
    uint32_t h = seed ^ ((uint32_t)ix * 0x8da6b343u) ^ ((uint32_t)iy * 0xd8163841u) ^ ((uint32_t)iz * 0xcb1ab31fu);
    h = (h ^ (h >> 16)) * 0x7feb352du;
    h = (h ^ (h >> 15)) * 0x846ca68bu;
    return h ^ (h >> 16);
}
static inline float lattice_ch(uint32_t h, int k) {
    if (k == 0) return (float)(h & 0x7ffu) * 0x1p-10f - 1.0f;
    if (k == 1) return (float)((h >> 11) & 0x7ffu) * 0x1p-10f - 1.0f;
    return (float)(h >> 22) * 0x1p-9f - 1.0f;
}
static inline float lerpf_(float a, float b, float t) { return a + (b - a) * t; }
void rrte_oracle_value_noise3(float x, float y, float z, uint32_t seed, float out[3]) {
    float fx0 = floorf(x), fy0 = floorf(y), fz0 = floorf(z);
    int32_t ix = (int32_t)fx0, iy = (int32_t)fy0, iz = (int32_t)fz0;
    float fx = x - fx0, fy = y - fy0, fz = z - fz0;
    float ux = fx * fx * (3.0f - 2.0f * fx);
    float uy = fy * fy * (3.0f - 2.0f * fy);
    float uz = fz * fz * (3.0f - 2.0f * fz);
    uint32_t h[8];
    for (int j = 0; j < 8; ++j) h[j] = lattice_hash(ix + (j & 1), iy + ((j >> 1) & 1), iz + ((j >> 2) & 1), seed);
    for (int k = 0; k < 3; ++k) {
        float x00 = lerpf_(lattice_ch(h[0], k), lattice_ch(h[1], k), ux);
        float x10 = lerpf_(lattice_ch(h[2], k), lattice_ch(h[3], k), ux);
        float x01 = lerpf_(lattice_ch(h[4], k), lattice_ch(h[5], k), ux);
        float x11 = lerpf_(lattice_ch(h[6], k), lattice_ch(h[7], k), ux);
        float y0 = lerpf_(x00, x10, uy), y1 = lerpf_(x01, x11, uy);
        out[k] = lerpf_(y0, y1, uz);
    }
}

/* ------------------------------------------------------- SDF evaluator */
static inline float len2f(float a, float b) { return sqrtf(a * a + b * b); }
static inline float len3f(float a, float b, float c) { return sqrtf((a * a + b * b) + c * c); }

static float sdf_leaf(const rrte_sdf_node* n, v3 p) {
    const float* f = n->f;
    v3 q = vsub(p, V(f[0], f[1], f[2]));
    switch (n->op) {
    case RRTE_SDF_SPHERE:
        return len3f(q.x, q.y, q.z) - f[3];
    case RRTE_SDF_BOX: {
        float dx = fabsf(q.x) - f[4] * 0.5f, dy = fabsf(q.y) - f[5] * 0.5f, dz = fabsf(q.z) - f[6] * 0.5f;
        float outside = len3f(smx(dx, 0.0f), smx(dy, 0.0f), smx(dz, 0.0f));
        float inside = smn(smx(dx, smx(dy, dz)), 0.0f);
        return outside + inside;
    }
    case RRTE_SDF_CYLINDER: {
        float dx = len2f(q.x, q.z) - f[3], dy = fabsf(q.y) - f[4] * 0.5f;
        return smn(smx(dx, dy), 0.0f) + len2f(smx(dx, 0.0f), smx(dy, 0.0f));
    }
    case RRTE_SDF_PRISM: {
        float a = smx(fabsf(q.x) * 0.866025f + q.y * 0.5f, -q.y) - f[5] * 0.25f;
        return smx(fabsf(q.z) - f[6] * 0.5f, a);
    }
    case RRTE_SDF_TORUS: {
        float qx = len2f(q.x, q.z) - f[3];
        return len2f(qx, q.y) - f[4];
    }
    case RRTE_SDF_TUBE: {
        float rad = len2f(q.x, q.z);
        float mid = (f[3] + f[4]) * 0.5f, half = (f[3] - f[4]) * 0.5f;
        float dx = fabsf(rad - mid) - half, dy = fabsf(q.y) - f[5] * 0.5f;
        return smn(smx(dx, dy), 0.0f) + len2f(smx(dx, 0.0f), smx(dy, 0.0f));
    }
    case RRTE_SDF_RING: {
        float qx = len2f(q.x, q.y) - f[3];
        return len2f(qx, q.z) - f[4];
    }
    case RRTE_SDF_CONE: {
        /* Capped cone, base radius r at y=-h/2, apex at y=+h/2 (exact distance). */
        float r1 = f[3], hh = f[4] * 0.5f;
        float qx = len2f(q.x, q.z), qy = q.y;
        float k2x = -r1, k2y = hh * 2.0f;
        float cax = qx - smn(qx, (qy < 0.0f) ? r1 : 0.0f);
        float cay = fabsf(qy) - hh;
        float k1mqx = 0.0f - qx, k1mqy = hh - qy;
        float tnum = k1mqx * k2x + k1mqy * k2y;
        float tden = k2x * k2x + k2y * k2y;
        float t = sclamp(tnum / tden, 0.0f, 1.0f);
        float cbx = (qx - 0.0f) + k2x * t;
        float cby = (qy - hh) + k2y * t;
        float s = (cbx < 0.0f && cay < 0.0f) ? -1.0f : 1.0f;
        float da = cax * cax + cay * cay, db = cbx * cbx + cby * cby;
        return s * sqrtf(smn(da, db));
    }
    case RRTE_SDF_CAPSULE: {
        float hh = f[4] * 0.5f;
        float y = q.y - sclamp(q.y, -hh, hh);
        return len3f(q.x, y, q.z) - f[3];
    }
    case RRTE_SDF_ELLIPSOID: {
        float rx = f[4], ry = f[5], rz = f[6];
        float k0 = len3f(q.x / rx, q.y / ry, q.z / rz);
        float k1 = len3f(q.x / (rx * rx), q.y / (ry * ry), q.z / (rz * rz));
        if (!(k1 > 0.0f)) return -smn(rx, smn(ry, rz));
        return k0 * (k0 - 1.0f) / k1;
    }
    default:
        return INFINITY;
    }
}

/* smooth_min (README.md:485-488): h = clamp(0.5 + 0.5 (b-a)/k); a h + b (1-h) - k h (1-h). */
static inline float smin(float a, float b, float k) {
    float h = sclamp(0.5f + (0.5f * (b - a)) / k, 0.0f, 1.0f);
    float om = 1.0f - h;
    return (a * h + b * om) - (k * h) * om;
}

static v3 sdf_deform(const rrte_sdf_node* n, v3 p) {
    const float* f = n->f;
    v3 c = V(f[0], f[1], f[2]);
    v3 q = vsub(p, c);
    switch (n->op) {
    case RRTE_SDF_TWIST:
    case RRTE_SDF_BEND: {
        int ax = (int)n->i[0];
        int drive = (n->op == RRTE_SDF_TWIST) ? ax : (int)n->i[1];
        int u = (ax + 1) % 3, w = (ax + 2) % 3;
        float s, co;
        sincos_rrte(f[3] * comp(q, drive), &s, &co);
        float qu = comp(q, u), qw = comp(q, w);
        q = setcomp(q, u, co * qu - s * qw);
        q = setcomp(q, w, s * qu + co * qw);
        break;
    }
    case RRTE_SDF_TAPER: {
        int ax = (int)n->i[0];
        int u = (ax + 1) % 3, w = (ax + 2) % 3;
        float t = sclamp((comp(q, ax) + f[5] * 0.5f) / f[5], 0.0f, 1.0f);
        float s = f[3] + (f[4] - f[3]) * t;
        q = setcomp(q, u, comp(q, u) / s);
        q = setcomp(q, w, comp(q, w) / s);
        break;
    }
    case RRTE_SDF_NOISE: {
        uint32_t oct = n->i[0], seed = n->i[1];
        v3 x = vmuls(q, f[3]);
        float acc[3] = {0.0f, 0.0f, 0.0f};
        float amp = 1.0f, fr = 1.0f;
        for (uint32_t o = 0; o < oct; ++o) {
            float nv[3];
            CNT(noise_octaves);
            rrte_oracle_value_noise3(x.x * fr, x.y * fr, x.z * fr, seed + o * 0x85ebca6bu, nv);
            for (int k = 0; k < 3; ++k) acc[k] = acc[k] + amp * nv[k];
            amp = amp * f[5];
            fr = fr * 2.0f;
        }
        q = V(q.x + f[4] * acc[0], q.y + f[4] * acc[1], q.z + f[4] * acc[2]);
        break;
    }
    case RRTE_SDF_WAVE: {
        int ax = (int)n->i[0], disp = (int)n->i[1];
        float s = rrte_oracle_sinf(f[4] * comp(q, ax));
        q = setcomp(q, disp, comp(q, disp) + f[3] * s);
        break;
    }
    default:
        break;
    }
    return vadd(q, c);
}

/* Evaluate one SDFObject's postfix program at p. */
static float sdf_eval(const rrte_sdf_node* nodes, uint32_t count, v3 p) {
    float vs[RRTE_SDF_MAX_STACK];
    v3 ps[RRTE_SDF_MAX_POINT_STACK];
    int sp = 0, pp = 0;
    for (uint32_t i = 0; i < count; ++i) {
        const rrte_sdf_node* n = &nodes[i];
        uint32_t op = n->op;
        CNT(sdf_nodes[op & 127u]);
        if (op < 32) {
            vs[sp++] = sdf_leaf(n, p);
        } else if (op < 64) {
            float b = vs[--sp], a = vs[--sp], r;
            switch (op) {
            case RRTE_SDF_UNION: r = smn(a, b); break;
            case RRTE_SDF_DIFFERENCE: r = smx(a, -b); break;
            case RRTE_SDF_INTERSECTION: r = smx(a, b); break;
            case RRTE_SDF_SMOOTH_UNION: r = smin(a, b, n->f[0]); break;
            case RRTE_SDF_SMOOTH_DIFFERENCE: r = -smin(-a, b, n->f[0]); break;
            default: r = -smin(-a, -b, n->f[0]); break; /* SMOOTH_INTERSECTION */
            }
            vs[sp++] = r;
        } else if (op < 96) {
            ps[pp++] = p;
            p = sdf_deform(n, p);
        } else {
            p = ps[--pp];
        }
    }
    return vs[0];
}

/* Validate a postfix program (stack discipline, known ops). */
static int sdf_validate(const rrte_sdf_node* nodes, uint32_t count) {
    int sp = 0, pp = 0;
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t op = nodes[i].op;
        if (op >= RRTE_SDF_SPHERE && op <= RRTE_SDF_ELLIPSOID) {
            if (++sp > RRTE_SDF_MAX_STACK) return 0;
        } else if (op >= RRTE_SDF_UNION && op <= RRTE_SDF_SMOOTH_INTERSECTION) {
            if (sp < 2) return 0;
            --sp;
        } else if (op >= RRTE_SDF_BEND && op <= RRTE_SDF_WAVE) {
            if (++pp > RRTE_SDF_MAX_POINT_STACK) return 0;
            if (op == RRTE_SDF_NOISE && nodes[i].i[0] > RRTE_SDF_MAX_OCTAVES) return 0;
        } else if (op == RRTE_SDF_POP_POINT) {
            if (pp < 1) return 0;
            --pp;
        } else {
            return 0;
        }
    }
    return sp == 1 && pp == 0;
}

/* ----------------------------------------------------- scene context */
typedef struct octx {
    const rrte_scene_ir* s;
    const rrte_render_params* prm;
} octx;

static inline float sdf_obj_eval(const octx* c, const rrte_prim* pr, v3 p) {
    return sdf_eval(c->s->sdf_nodes + pr->sdf_first, pr->sdf_count, p);
}

/* SDFObject::intersect (build-defined sphere tracing). */
static int sdf_intersect(const octx* c, const rrte_prim* pr, const ray* r, float t_min, float t_max, hit* out) {
    v3 bc = vload(pr->p);
    float br = pr->p[3];
    v3 oc = vsub(r->o, bc);
    float b = vdot(oc, r->d);
    float cc = vdot(oc, oc) - br * br;
    float disc = b * b - cc;
    if (disc < 0.0f) return 0;
    float sq = sqrtf(disc);
    float t = mx(t_min, -b - sq);
    float tend = mn(t_max, -b + sq);
    if (t > tend) return 0;
    float eps = pr->sdf_hit_eps, scale = pr->sdf_step_scale;
    for (uint32_t i = 0; i < pr->sdf_max_steps; ++i) {
        CNT(sdf_steps);
        v3 p = ray_at(r, t);
        float d = sdf_obj_eval(c, pr, p);
        if (d < eps * t) {
            CNT(sdf_normals);
            CNT(isect_hits[RRTE_PRIM_SDF]);
            /* tetrahedral normal estimate, h = 1e-3 */
            const float h = 1e-3f;
            float f0 = sdf_obj_eval(c, pr, V(p.x + h, p.y - h, p.z - h));
            float f1 = sdf_obj_eval(c, pr, V(p.x - h, p.y - h, p.z + h));
            float f2 = sdf_obj_eval(c, pr, V(p.x - h, p.y + h, p.z - h));
            float f3 = sdf_obj_eval(c, pr, V(p.x + h, p.y + h, p.z + h));
            v3 n = V(((f0 - f1) - f2) + f3, ((-f0 - f1) + f2) + f3, ((-f0 + f1) - f2) + f3);
            *out = hit_new(t, p, vnorm(n), r);
            return 1;
        }
        t = t + d * scale;
        if (t > tend) return 0;
    }
    return 0;
}

static inline void local_ray(const rrte_prim* pr, const ray* r, ray* lr, float m[16]) {
    float inv[16];
    rrte_oracle_mat4_srt(pr->trs, m);
    rrte_oracle_mat4_inverse(m, inv); /* inverse_matrix() per call (primitives.rs:303) */
    *lr = ray_new(m4_point(inv, r->o), vnorm(m4_vector(inv, r->d)));
}

/* Triangle::intersect (primitives.rs:208-244), Moller-Trumbore: the test part.  On success
 * out->t, out->p and the barycentrics (u, v in out->n.x, out->n.y) are set. */
static int tri_intersect(v3 v0, v3 v1, v3 v2, const ray* r, float t_min, float t_max, hit* out) {
    v3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    v3 h = vcross(r->d, e2);
    float a = vdot(e1, h);
    if (a > -1e-6f && a < 1e-6f) return 0;
    float f = 1.0f / a;
    v3 s = vsub(r->o, v0);
    float u = f * vdot(s, h);
    if (u < 0.0f || u > 1.0f) return 0;
    v3 q = vcross(s, e1);
    float v = f * vdot(r->d, q);
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = f * vdot(e2, q);
    if (t < t_min || t > t_max) return 0;
    out->t = t;
    out->p = ray_at(r, t);
    out->n = V(u, v, 0.0f);
    return 1;
}
/* ... and the attribute part: barycentric normal (primitives.rs:240-243), HitInfo::new. */
static void tri_attributes(v3 n0, v3 n1, v3 n2, const ray* r, hit* io) {
    float u = io->n.x, v = io->n.y;
    float w = 1.0f - u - v;
    v3 n = vnorm(vadd(vadd(vmuls(n0, w), vmuls(n1, u)), vmuls(n2, v)));
    *io = hit_new(io->t, io->p, n, r);
}

/* SceneObject::intersect dispatch (primitives.rs:57-725). */
static int intersect(const octx* c, const rrte_prim* pr, const ray* r, float t_min, float t_max, hit* out) {
    CNT(isect_calls[pr->kind & 15u]);
    switch (pr->kind) {
    case RRTE_PRIM_SPHERE: { /* primitives.rs:57-81 */
        v3 ctr = vload(pr->p);
        float rad = pr->p[3];
        v3 oc = vsub(r->o, ctr);
        float a = vlen2(r->d);
        float hb = vdot(oc, r->d);
        float cc = vlen2(oc) - rad * rad;
        float disc = hb * hb - a * cc;
        if (disc < 0.0f) return 0;
        float sq = sqrtf(disc);
        float root = (-hb - sq) / a;
        if (root < t_min || t_max < root) {
            root = (-hb + sq) / a;
            if (root < t_min || t_max < root) return 0;
        }
        v3 p = ray_at(r, root);
        CNT(isect_hits[pr->kind & 7u]);
        *out = hit_new(root, p, vdivs(vsub(p, ctr), rad), r);
        return 1;
    }
    case RRTE_PRIM_PLANE: { /* primitives.rs:133-149 */
        v3 pt = vload(pr->p), n = vload(pr->p + 4);
        float denom = vdot(n, r->d);
        if (fabsf(denom) < 1e-6f) return 0;
        float t = vdot(vsub(pt, r->o), n) / denom;
        if (t < t_min || t > t_max) return 0;
        v3 p = ray_at(r, t);
        CNT(isect_hits[pr->kind & 7u]);
        *out = hit_new(t, p, denom < 0.0f ? n : vneg(n), r);
        return 1;
    }
    case RRTE_PRIM_TRIANGLE: /* primitives.rs:208-244 (Moller-Trumbore) */
        if (!tri_intersect(vload(pr->p), vload(pr->p + 3), vload(pr->p + 6), r, t_min, t_max, out)) return 0;
        CNT(isect_hits[pr->kind & 15u]);
        tri_attributes(vload(pr->p + 9), vload(pr->p + 12), vload(pr->p + 15), r, out);
        return 1;
    case RRTE_PRIM_MESH: { /* a Vec<Triangle> with set_normals: closest over triangles, strict '<' */
        const rrte_mesh_vertex* vx = c->s->mesh_vertices;
        const uint32_t* ix = c->s->mesh_indices + (size_t)pr->sdf_first * 3;
        int found = 0, win = 0;
        hit best = {0}, h = {0};
        for (uint32_t k = 0; k < pr->sdf_count; ++k) {
            CNT(mesh_tri_tests);
            const rrte_mesh_vertex *a = &vx[ix[3 * k]], *b = &vx[ix[3 * k + 1]], *cc = &vx[ix[3 * k + 2]];
            if (tri_intersect(vload(a->position), vload(b->position), vload(cc->position), r, t_min, t_max, &h)) {
                if (!found || h.t < best.t) { best = h; win = (int)k; found = 1; }
            }
        }
        if (!found) return 0;
        CNT(isect_hits[RRTE_PRIM_MESH]);
        const rrte_mesh_vertex *a = &vx[ix[3 * win]], *b = &vx[ix[3 * win + 1]], *cc = &vx[ix[3 * win + 2]];
        tri_attributes(vload(a->normal), vload(b->normal), vload(cc->normal), r, &best);
        *out = best;
        return 1;
    }
    case RRTE_PRIM_CUBE: { /* primitives.rs:301-364 */
        float m[16];
        ray lr;
        local_ray(pr, r, &lr, m);
        v3 ctr = vload(pr->p), size = vload(pr->p + 4);
        v3 half = vmuls(size, 0.5f);
        v3 mnb = vsub(ctr, half), mxb = vadd(ctr, half);
        float t_near = t_min, t_far = t_max;
        v3 normal = V(0.0f, 0.0f, 0.0f);
        for (int i = 0; i < 3; ++i) {
            v3 axis = setcomp(V(0.0f, 0.0f, 0.0f), i, 1.0f); /* Vec3::X / Y / Z */
            float oc = vdot(lr.o, axis), dc = vdot(lr.d, axis);
            float lo = vdot(mnb, axis), hi = vdot(mxb, axis);
            if (fabsf(dc) < 1e-6f) {
                if (oc < lo || oc > hi) return 0;
            } else {
                float t1 = (lo - oc) / dc, t2 = (hi - oc) / dc;
                float tsn = t1 < t2 ? t1 : t2, tsf = t1 < t2 ? t2 : t1;
                if (tsn > t_near) {
                    t_near = tsn;
                    normal = t1 < t2 ? vneg(axis) : axis;
                }
                if (tsf < t_far) t_far = tsf;
                if (t_near > t_far) return 0;
            }
        }
        float t = (t_near >= t_min) ? t_near : t_far;
        if (t < t_min || t > t_max) return 0;
        v3 lp = ray_at(&lr, t);
        CNT(isect_hits[pr->kind & 7u]);
        *out = hit_new(t, m4_point(m, lp), vnorm(m4_vector(m, normal)), r);
        return 1;
    }
    case RRTE_PRIM_CYLINDER: { /* primitives.rs:419-465 */
        float m[16];
        ray lr;
        local_ray(pr, r, &lr, m);
        v3 ctr = vload(pr->p);
        float rad = pr->p[3], hh = pr->p[4] * 0.5f;
        v3 oc = vsub(lr.o, ctr);
        float a = lr.d.x * lr.d.x + lr.d.z * lr.d.z;
        float b = 2.0f * (oc.x * lr.d.x + oc.z * lr.d.z);
        float cc = oc.x * oc.x + oc.z * oc.z - rad * rad;
        float disc = b * b - 4.0f * a * cc;
        if (disc < 0.0f) return 0;
        float sq = sqrtf(disc);
        float ts[2] = {(-b - sq) / (2.0f * a), (-b + sq) / (2.0f * a)};
        for (int k = 0; k < 2; ++k) {
            float t = ts[k];
            if (t >= t_min && t <= t_max) {
                CNT(root_checks);
                v3 p = ray_at(&lr, t);
                if (fabsf(p.y - ctr.y) <= hh) {
                    v3 ln = V((p.x - ctr.x) / rad, 0.0f, (p.z - ctr.z) / rad);
                    CNT(isect_hits[pr->kind & 7u]);
                    *out = hit_new(t, m4_point(m, p), vnorm(m4_vector(m, ln)), r);
                    return 1;
                }
            }
        }
        return 0;
    }
    case RRTE_PRIM_CONE: { /* primitives.rs:520-571 */
        float m[16];
        ray lr;
        local_ray(pr, r, &lr, m);
        v3 ctr = vload(pr->p);
        float rad = pr->p[3], ht = pr->p[4], hh = ht * 0.5f;
        v3 oc = vsub(lr.o, ctr);
        float k = rad / ht, k2 = k * k;
        v3 d = lr.d;
        float a = d.x * d.x + d.z * d.z - k2 * d.y * d.y;
        float b = 2.0f * (oc.x * d.x + oc.z * d.z - k2 * (oc.y - hh) * d.y);
        float cc = oc.x * oc.x + oc.z * oc.z - k2 * (oc.y - hh) * (oc.y - hh);
        float disc = b * b - 4.0f * a * cc;
        if (disc < 0.0f) return 0;
        float sq = sqrtf(disc);
        float ts[2] = {(-b - sq) / (2.0f * a), (-b + sq) / (2.0f * a)};
        for (int kk = 0; kk < 2; ++kk) {
            float t = ts[kk];
            if (t >= t_min && t <= t_max) {
                CNT(root_checks);
                v3 p = ray_at(&lr, t);
                float yl = p.y - ctr.y;
                if (yl >= -hh && yl <= hh) {
                    float rr = sqrtf(p.x * p.x + p.z * p.z);
                    v3 ln = vnorm(V(p.x / rr, k, p.z / rr));
                    CNT(isect_hits[pr->kind & 7u]);
                    *out = hit_new(t, m4_point(m, p), vnorm(m4_vector(m, ln)), r);
                    return 1;
                }
            }
        }
        return 0;
    }
    case RRTE_PRIM_CAPSULE: { /* primitives.rs:626-725 */
        float m[16];
        ray lr;
        local_ray(pr, r, &lr, m);
        v3 ctr = vload(pr->p);
        float rad = pr->p[3], hh = pr->p[4] * 0.5f;
        v3 top = vadd(ctr, V(0.0f, hh, 0.0f)), bot = vsub(ctr, V(0.0f, hh, 0.0f));
        float closest = INFINITY;
        int found = 0;
        hit best = {0};
        float a = vlen2(lr.d);
        for (int cap = 0; cap < 2; ++cap) {
            v3 cc_ = cap == 0 ? top : bot;
            v3 oc = vsub(lr.o, cc_);
            float hb = vdot(oc, lr.d);
            float cc = vlen2(oc) - rad * rad;
            float disc = hb * hb - a * cc;
            if (disc >= 0.0f) {
                float sq = sqrtf(disc);
                float ts[2] = {(-hb - sq) / a, (-hb + sq) / a};
                for (int k = 0; k < 2; ++k) {
                    float t = ts[k];
                    if (t >= t_min && t <= t_max && t < closest) {
                        CNT(root_checks);
                        v3 p = ray_at(&lr, t);
                        int ok = cap == 0 ? (p.y >= ctr.y) : (p.y <= ctr.y);
                        if (ok) {
                            v3 ln = vnorm(vsub(p, cc_));
                            closest = t;
                            CNT(isect_hits[pr->kind & 7u]);
                            best = hit_new(t, m4_point(m, p), vnorm(m4_vector(m, ln)), r);
                            found = 1;
                        }
                    }
                }
            }
        }
        v3 oc = vsub(lr.o, ctr);
        float ac = lr.d.x * lr.d.x + lr.d.z * lr.d.z;
        float bc = 2.0f * (oc.x * lr.d.x + oc.z * lr.d.z);
        float ccy = oc.x * oc.x + oc.z * oc.z - rad * rad;
        float disc = bc * bc - 4.0f * ac * ccy;
        if (disc >= 0.0f) {
            float sq = sqrtf(disc);
            float ts[2] = {(-bc - sq) / (2.0f * ac), (-bc + sq) / (2.0f * ac)};
            for (int k = 0; k < 2; ++k) {
                float t = ts[k];
                if (t >= t_min && t <= t_max && t < closest) {
                    CNT(root_checks);
                    v3 p = ray_at(&lr, t);
                    if (fabsf(p.y - ctr.y) <= hh) {
                        v3 ln = V((p.x - ctr.x) / rad, 0.0f, (p.z - ctr.z) / rad);
                        closest = t;
                        CNT(isect_hits[pr->kind & 7u]);
                        best = hit_new(t, m4_point(m, p), vnorm(m4_vector(m, ln)), r);
                        found = 1;
                    }
                }
            }
        }
        if (found) *out = best;
        return found;
    }
    case RRTE_PRIM_SDF:
        return sdf_intersect(c, pr, r, t_min, t_max, out);
    default:
        return 0;
    }
}

/* ------------------------------------------------------------- RNG */
/* Counter-based RNG (build-defined replacement for rand::thread_rng, F8). */
static inline uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
static inline float rng_f32(uint32_t* st) {
    *st = *st * 747796405u + 2891336453u;
    uint32_t s = *st;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    w = (w >> 22u) ^ w;
    return (float)(w >> 8) * 5.9604644775390625e-8f;
}
static inline v3 rand_in_unit_sphere(uint32_t* st) { /* vector.rs:35-46 */
    for (;;) {
        CNT(sphere_samples);
        float x = rng_f32(st) * 2.0f - 1.0f;
        float y = rng_f32(st) * 2.0f - 1.0f;
        float z = rng_f32(st) * 2.0f - 1.0f;
        v3 p = V(x, y, z);
        if (vlen2(p) < 1.0f) return p;
    }
}
static inline v3 reflect3(v3 v, v3 n) { return vsub(v, vmuls(n, 2.0f * vdot(v, n))); } /* vector.rs:17-19 */

/* Material::scatter (material.rs:60-72, 99-110, 147-170, 200-202). Returns 0 for None. */
static int scatter(const rrte_material* m, const ray* rin, const hit* h, uint32_t* st, ray* out) {
    CNT(scatters[m->kind & 3u]);
    switch (m->kind) {
    case RRTE_MAT_LAMBERTIAN: {
        v3 sd = vadd(h->n, vnorm(rand_in_unit_sphere(st)));
        v3 dir = vlen2(sd) < 1e-8f ? h->n : sd;
        *out = ray_new(h->p, dir);
        return 1;
    }
    case RRTE_MAT_METAL: {
        v3 refl = reflect3(vnorm(rin->d), h->n);
        v3 sc = vadd(refl, vmuls(rand_in_unit_sphere(st), m->fuzz));
        if (vdot(sc, h->n) > 0.0f) { *out = ray_new(h->p, sc); return 1; }
        return 0;
    }
    case RRTE_MAT_DIELECTRIC: {
        float ratio = h->front ? 1.0f / m->ior : m->ior;
        v3 ud = vnorm(rin->d);
        float cos_t = mn(vdot(vneg(ud), h->n), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        int cannot = ratio * sin_t > 1.0f;
        float r0 = (1.0f - ratio) / (1.0f + ratio);
        r0 = r0 * r0;
        float x = 1.0f - cos_t;
        float x2 = x * x;
        float refl = r0 + (1.0f - r0) * (x * (x2 * x2));
        v3 dir;
        int do_reflect = cannot;
        if (!do_reflect) do_reflect = refl > rng_f32(st);
        if (do_reflect) {
            dir = reflect3(ud, h->n);
        } else {
            float ct = mn(vdot(vneg(ud), h->n), 1.0f);
            v3 perp = vmuls(vadd(ud, vmuls(h->n, ct)), ratio);
            float l2 = vlen2(perp);
            v3 par = vmuls(h->n, -sqrtf(fabsf(1.0f - l2)));
            dir = (l2 < 1.0f) ? vadd(perp, par) : reflect3(ud, h->n);
        }
        *out = ray_new(h->p, dir);
        return 1;
    }
    default: /* emissive */
        return 0;
    }
}

/* --------------------------------------------------------- shading */
static int closest_hit(const octx* c, const ray* r, float t_min, hit* best, int* best_idx) {
    int found = 0;
    for (uint32_t i = 0; i < c->s->num_prims; ++i) {
        const rrte_prim* pr = &c->s->prims[i];
        hit h = {0};
        /* Analytic objects are called with t_max = INFINITY exactly as
         * raytracer.rs:107; SDF objects march only up to the current closest
         * hit (build-defined; equivalent for the strict '<' selection). */
        float tmax = (pr->kind == RRTE_PRIM_SDF && found) ? best->t : INFINITY;
        if (intersect(c, pr, r, t_min, tmax, &h)) {
            if (!found || h.t < best->t) { *best = h; *best_idx = (int)i; found = 1; }
        }
    }
    return found;
}

static int occluded(const octx* c, const ray* r, float t_min, float t_max) {
    for (uint32_t i = 0; i < c->s->num_prims; ++i) {
        hit h = {0};
        if (intersect(c, &c->s->prims[i], r, t_min, t_max, &h)) return 1;
    }
    return 0;
}

/* PointLight::calculate_attenuation (light.rs:170-178). */
static inline float point_att(const rrte_light* l, float d) {
    if (d > l->range) return 0.0f;
    float a = 1.0f / ((1.0f + l->linear * d) + (l->quadratic * d) * d);
    return mx(a, 0.0f);
}

typedef struct contrib { col color; v3 dir; float dist, att; } contrib;

/* Light::illuminate (light.rs:87-94, 182-194, 289-304, 365-372). */
static contrib illuminate(const rrte_light* l, v3 p) {
    contrib k;
    CNT(light_evals[l->kind & 3u]);
    k.color = cmuls(cload(l->color), l->intensity);
    switch (l->kind) {
    case RRTE_LIGHT_POINT: {
        v3 lv = vsub(vload(l->position), p);
        k.dist = vlen(lv);
        k.dir = vnorm(lv);
        k.att = point_att(l, k.dist);
        break;
    }
    case RRTE_LIGHT_DIRECTIONAL:
        k.dir = vneg(vload(l->direction));
        k.dist = INFINITY;
        k.att = 1.0f;
        break;
    case RRTE_LIGHT_SPOT: {
        v3 lv = vsub(vload(l->position), p);
        k.dist = vlen(lv);
        k.dir = vnorm(lv);
        float da = point_att(l, k.dist);
        float ang = acosf(vdot(vload(l->direction), vneg(k.dir)));
        float aa;
        if (ang > l->outer_angle) aa = 0.0f;
        else if (ang < l->inner_angle) aa = 1.0f;
        else {
            float fo = (l->outer_angle - ang) / (l->outer_angle - l->inner_angle);
            aa = fo * fo;
        }
        k.att = da * aa;
        break;
    }
    default: /* ambient */
        k.dir = V(0.0f, 0.0f, 0.0f);
        k.dist = 0.0f;
        k.att = 1.0f;
        break;
    }
    return k;
}

/* Raytracer::ray_color (raytracer.rs:92-148), recursion kept. */
static col ray_color(const octx* c, const ray* r, uint32_t depth, uint32_t* st, uint64_t* nshadow) {
    if (depth == 0) return BLACK;
    hit h = {0};
    int idx = -1;
    if (!closest_hit(c, r, c->prm->t_min, &h, &idx)) return cload(c->prm->background);
    const rrte_prim* pr = &c->s->prims[idx];
    if (pr->material < 0 || (uint32_t)pr->material >= c->s->num_materials) return BLACK;
    const rrte_material* m = &c->s->materials[pr->material];
    col alb = cload(m->albedo);
    col color = cadd(BLACK, cmuls(cmuls(alb, 0.1f), 0.1f));
    CNT(shaded_hits);
    if (c->prm->mode == RRTE_MODE_REFCOMPAT) {
        for (uint32_t i = 0; i < c->s->num_lights; ++i) {
            CNT(ref_light_terms);
            contrib k = illuminate(&c->s->lights[i], h.p);
            color = cadd(color, cmuls(k.color, k.att));
        }
        ray sc;
        if (scatter(m, r, &h, st, &sc)) {
            col s = ray_color(c, &sc, depth - 1, st, nshadow);
            color = cadd(color, C4(alb.r * s.r, alb.g * s.g, alb.b * s.b, 1.0f));
        }
        return color;
    }
    /* LAMBERT_SHADOW (build-defined). */
    float bias = c->prm->shadow_bias;
    for (uint32_t i = 0; i < c->s->num_lights; ++i) {
        const rrte_light* l = &c->s->lights[i];
        contrib k = illuminate(l, h.p);
        if (l->kind == RRTE_LIGHT_AMBIENT) {
            color.r = color.r + alb.r * k.color.r;
            color.g = color.g + alb.g * k.color.g;
            color.b = color.b + alb.b * k.color.b;
            continue;
        }
        CNT(lambert_lights);
        float ndl = vdot(h.n, k.dir);
        if (ndl > 0.0f && k.att > 0.0f) {
            ++*nshadow;
            CNT(shadow_rays);
            ray sr = ray_new(vadd(h.p, vmuls(h.n, bias)), k.dir);
            if (!occluded(c, &sr, bias, k.dist)) {
                CNT(lambert_terms);
                float f = k.att * ndl;
                color.r = color.r + alb.r * (k.color.r * f);
                color.g = color.g + alb.g * (k.color.g * f);
                color.b = color.b + alb.b * (k.color.b * f);
            }
        }
    }
    return color;
}

/* Rust `(x * 255.0) as u8`: truncating, saturating, NaN -> 0 (raytracer.rs:82-85). */
static inline uint8_t to_u8(float c) {
    float v = c * 255.0f;
    if (!(v > 0.0f)) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}
/* f32::clamp keeps NaN (color.rs:48-55). */
static inline float rclamp(float x) { if (x < 0.0f) return 0.0f; if (x > 1.0f) return 1.0f; return x; }

typedef struct job {
    octx c;
    uint8_t* rgba8;
    float* f32;
    uint32_t row_begin, row_end;
    atomic_uint next_row;
    atomic_ullong shadow;
#ifdef RRTE_ORACLE_COUNT
    pthread_mutex_t mu;
    rrte_oracle_counts* counts;
#endif
} job;

enum { ROWS_PER_CHUNK = 2 };

static void render_row(job* jb, uint32_t y, uint64_t* nshadow) {
    const rrte_render_params* prm = jb->c.prm;
    uint32_t W = prm->width, H = prm->height;
    float inv_g = 1.0f / prm->gamma;
    float inv_spp = 1.0f / (float)prm->samples_per_pixel;
    for (uint32_t x = 0; x < W; ++x) {
        uint32_t pix = y * W + x;
        col color = BLACK;
        CNT(pixels);
        for (uint32_t s = 0; s < prm->samples_per_pixel; ++s) {
            CNT(samples);
            uint32_t st = pcg_hash(pcg_hash(pcg_hash(prm->seed) ^ pix) ^ s);
            float jx = 0.5f, jy = 0.5f;
            if (prm->jitter == RRTE_JITTER_RANDOM) { jx = rng_f32(&st); jy = rng_f32(&st); }
            float u = ((float)x + jx) / (float)W;
            float v = ((float)y + jy) / (float)H;
            ray r = generate_ray(&jb->c.s->camera, u, v);
            color = cadd(color, ray_color(&jb->c, &r, prm->max_depth, &st, nshadow));
        }
        color = cmuls(color, inv_spp);
        float* fo = jb->f32 ? jb->f32 + (size_t)pix * 4 : NULL;
        if (fo && (prm->flags & RRTE_FLAG_F32_LINEAR)) {
            fo[0] = color.r; fo[1] = color.g; fo[2] = color.b; fo[3] = color.a;
            fo = NULL;
        }
        col gc = C4(rclamp(powf(color.r, inv_g)), rclamp(powf(color.g, inv_g)),
                    rclamp(powf(color.b, inv_g)), rclamp(color.a));
        if (fo) { fo[0] = gc.r; fo[1] = gc.g; fo[2] = gc.b; fo[3] = gc.a; }
        if (jb->rgba8) {
            uint8_t* o = jb->rgba8 + (size_t)pix * 4;
            o[0] = to_u8(gc.r); o[1] = to_u8(gc.g); o[2] = to_u8(gc.b); o[3] = to_u8(gc.a);
        }
    }
    (void)H;
}

static void* worker(void* arg) {
    job* jb = (job*)arg;
    uint64_t local = 0;
#ifdef RRTE_ORACLE_COUNT
    rrte_oracle_counts* mine = (rrte_oracle_counts*)calloc(1, sizeof(rrte_oracle_counts));
    rrte_oracle_counts scratch;
    tl_cnt = mine ? mine : &scratch;
#endif
    for (;;) {
        uint32_t y0 = atomic_fetch_add(&jb->next_row, ROWS_PER_CHUNK);
        if (y0 >= jb->row_end) break;
        uint32_t y1 = y0 + ROWS_PER_CHUNK < jb->row_end ? y0 + ROWS_PER_CHUNK : jb->row_end;
        for (uint32_t y = y0; y < y1; ++y) render_row(jb, y, &local);
    }
    atomic_fetch_add(&jb->shadow, local);
#ifdef RRTE_ORACLE_COUNT
    if (mine) {
        pthread_mutex_lock(&jb->mu);
        uint64_t* dst = (uint64_t*)jb->counts;
        const uint64_t* src = (const uint64_t*)mine;
        for (size_t i = 0; i < sizeof(rrte_oracle_counts) / sizeof(uint64_t); ++i) dst[i] += src[i];
        pthread_mutex_unlock(&jb->mu);
        free(mine);
    }
    tl_cnt = NULL;
#endif
    return NULL;
}

static int validate_scene(const rrte_scene_ir* s, const rrte_render_params* p) {
    if (!s || !p || p->width == 0 || p->height == 0 || p->samples_per_pixel == 0) return 0;
    if (s->num_prims && !s->prims) return 0;
    if (s->num_lights && !s->lights) return 0;
    if (s->num_materials && !s->materials) return 0;
    for (uint32_t i = 0; i < s->num_prims; ++i) {
        const rrte_prim* pr = &s->prims[i];
        if (pr->kind > RRTE_PRIM_MESH) return 0;
        if (pr->kind == RRTE_PRIM_MESH) {
            if ((uint64_t)(pr->sdf_first + (uint64_t)pr->sdf_count) * 3 > s->num_mesh_indices) return 0;
            if (pr->sdf_count && (!s->mesh_indices || !s->mesh_vertices)) return 0;
            for (uint64_t k = (uint64_t)pr->sdf_first * 3; k < (uint64_t)(pr->sdf_first + (uint64_t)pr->sdf_count) * 3; ++k)
                if (s->mesh_indices[k] >= s->num_mesh_vertices) return 0;
        }
        if (pr->kind == RRTE_PRIM_SDF) {
            if (!s->sdf_nodes || (uint64_t)pr->sdf_first + pr->sdf_count > s->num_sdf_nodes) return 0;
            if (!sdf_validate(s->sdf_nodes + pr->sdf_first, pr->sdf_count)) return 0;
        }
    }
    return 1;
}

static int render_impl(const rrte_scene_ir* scene, const rrte_render_params* params, uint8_t* out_rgba8,
                       float* out_f32, uint64_t* shadow_rays, int nthreads, uint32_t row_begin, uint32_t row_end,
                       rrte_oracle_counts* counts) {
    if (!validate_scene(scene, params)) return 1;
    if (row_begin == 0 && row_end == 0) row_end = params->height;
    if (row_end > params->height || row_begin > row_end) return 1;
    job* jb = (job*)calloc(1, sizeof(job));
    if (!jb) return 2;
    jb->c.s = scene;
    jb->c.prm = params;
    jb->rgba8 = out_rgba8;
    jb->f32 = out_f32;
    jb->row_begin = row_begin;
    jb->row_end = row_end;
    atomic_init(&jb->next_row, row_begin);
    atomic_init(&jb->shadow, 0);
#ifdef RRTE_ORACLE_COUNT
    pthread_mutex_init(&jb->mu, NULL);
    jb->counts = counts;
#else
    (void)counts;
#endif
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    int started = 0;
    for (int i = 1; i < nthreads; ++i) {
        if (pthread_create(&th[started], NULL, worker, jb) == 0) ++started;
    }
    worker(jb);
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
    if (shadow_rays) *shadow_rays = atomic_load(&jb->shadow);
#ifdef RRTE_ORACLE_COUNT
    pthread_mutex_destroy(&jb->mu);
#endif
    free(jb);
    return 0;
}

int rrte_oracle_render(const rrte_scene_ir* scene, const rrte_render_params* params,
                       uint8_t* out_rgba8, float* out_f32, uint64_t* shadow_rays,
                       int nthreads, uint32_t row_begin, uint32_t row_end) {
#ifdef RRTE_ORACLE_COUNT
    rrte_oracle_counts scratch;
    memset(&scratch, 0, sizeof scratch);
    return render_impl(scene, params, out_rgba8, out_f32, shadow_rays, nthreads, row_begin, row_end, &scratch);
#else
    return render_impl(scene, params, out_rgba8, out_f32, shadow_rays, nthreads, row_begin, row_end, NULL);
#endif
}

#ifdef RRTE_ORACLE_COUNT
int rrte_oracle_render_counted(const rrte_scene_ir* scene, const rrte_render_params* params,
                               rrte_oracle_counts* counts, int nthreads, uint32_t row_begin, uint32_t row_end) {
    if (!counts) return 1;
    return render_impl(scene, params, NULL, NULL, NULL, nthreads, row_begin, row_end, counts);
}
#endif

int rrte_oracle_intersect(const rrte_scene_ir* scene, uint32_t idx, const float o[3], const float d[3],
                          float t_min, float t_max, oracle_hit* out) {
    if (!scene || idx >= scene->num_prims) return 0;
    octx c = {scene, NULL};
    ray r = ray_new(vload(o), vload(d));
    hit h = {0};
    if (!intersect(&c, &scene->prims[idx], &r, t_min, t_max, &h)) return 0;
    out->t = h.t;
    out->point[0] = h.p.x; out->point[1] = h.p.y; out->point[2] = h.p.z;
    out->normal[0] = h.n.x; out->normal[1] = h.n.y; out->normal[2] = h.n.z;
    out->front_face = h.front;
    return 1;
}

float rrte_oracle_sdf_eval(const rrte_scene_ir* scene, uint32_t idx, const float p[3]) {
    const rrte_prim* pr = &scene->prims[idx];
    return sdf_eval(scene->sdf_nodes + pr->sdf_first, pr->sdf_count, vload(p));
}

/* ------------------------------------------------ algorithmic flop tally */
/* FP32 operations per counted event, tallied from the code above (add, sub, mul,
 * div, sqrt, min, max and each transcendental = 1; abs, negation and compares = 0).
 * Analytic object transforms are priced with the inverse precomputed once per
 * object (as the device does), not rebuilt per ray as primitives.rs:303 does.
 * Intersector "call" weights price the test up to its usual early exit; the
 * root/attribute work is priced by the hit and root-check events. */
double rrte_oracle_flops(const rrte_oracle_counts* c) {
    if (!c) return 0.0;
    /* u,v (4) + generate_ray: ndc 4, tan/half 3, scale 2, normalize 10, quat*vec 38, Ray::new 10 (67) + accumulate 4 */
    const double w_sample = 75.0;
    const double w_pixel = 11.0;                      /* /spp 4, powf x3, *255 x4 */
    /*                              sphere plane tri  cube cyl  cone caps  sdf(bound test)  mesh */
    static const double w_call[16] = {23.0, 14.0, 30.0, 146.0, 79.0, 91.0, 133.0, 21.0, 0.0};
    static const double w_hit[16] = {22.0, 11.0, 60.0, 54.0, 52.0, 64.0, 60.0, 36.0, 60.0};
    const double w_tri_test = 30.0;                   /* Moller-Trumbore to its usual early exit */
    const double w_root = 7.0, w_step = 9.0;
    double w_node[128] = {0};
    w_node[RRTE_SDF_SPHERE] = 10; w_node[RRTE_SDF_BOX] = 22; w_node[RRTE_SDF_CYLINDER] = 19;
    w_node[RRTE_SDF_PRISM] = 12; w_node[RRTE_SDF_TORUS] = 13; w_node[RRTE_SDF_TUBE] = 24;
    w_node[RRTE_SDF_RING] = 13; w_node[RRTE_SDF_CONE] = 38; w_node[RRTE_SDF_CAPSULE] = 14;
    w_node[RRTE_SDF_ELLIPSOID] = 27;
    w_node[RRTE_SDF_UNION] = 1; w_node[RRTE_SDF_DIFFERENCE] = 1; w_node[RRTE_SDF_INTERSECTION] = 1;
    w_node[RRTE_SDF_SMOOTH_UNION] = 13; w_node[RRTE_SDF_SMOOTH_DIFFERENCE] = 13;
    w_node[RRTE_SDF_SMOOTH_INTERSECTION] = 13;
    w_node[RRTE_SDF_BEND] = 39; w_node[RRTE_SDF_TWIST] = 39; w_node[RRTE_SDF_TAPER] = 16;
    w_node[RRTE_SDF_NOISE] = 15; w_node[RRTE_SDF_WAVE] = 35;
    const double w_octave = 135.0; /* per octave: scale 3, cell 15, 24 corner values 48, 21 lerps 63, accumulate 6 */
    static const double w_light[4] = {29.0, 4.0, 39.0, 4.0};  /* point, directional, spot, ambient */
    const double w_shaded = 12.0, w_ndl = 5.0, w_shadow = 16.0, w_term = 10.0, w_ref_term = 8.0;
    static const double w_scatter[4] = {35.0, 50.0, 77.0, 0.0};  /* + 7 for the recursion combine */
    const double w_sphere_sample = 14.0;

    double f = w_sample * (double)c->samples + w_pixel * (double)c->pixels;
    for (int k = 0; k < 16; ++k) f += w_call[k] * (double)c->isect_calls[k] + w_hit[k] * (double)c->isect_hits[k];
    f += w_tri_test * (double)c->mesh_tri_tests;
    f += w_root * (double)c->root_checks + w_step * (double)c->sdf_steps;
    for (int k = 0; k < 128; ++k) f += w_node[k] * (double)c->sdf_nodes[k];
    f += w_octave * (double)c->noise_octaves;
    for (int k = 0; k < 4; ++k) f += w_light[k] * (double)c->light_evals[k] + w_scatter[k] * (double)c->scatters[k];
    f += w_shaded * (double)c->shaded_hits + w_ndl * (double)c->lambert_lights + w_shadow * (double)c->shadow_rays;
    f += w_term * (double)c->lambert_terms + w_ref_term * (double)c->ref_light_terms;
    f += w_sphere_sample * (double)c->sphere_samples;
    return f;
}
