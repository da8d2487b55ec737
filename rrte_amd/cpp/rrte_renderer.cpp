// rrte_renderer.cpp — C++ mirror of the reference renderer API (include/rrte/rrte_renderer.hpp).
// Lowering follows rrte_amd/renderer.py operation for operation (f32 where it uses numpy f32,
// double where it uses Python floats), so both mirrors produce byte-identical rrte_scene_ir.
#include "../../include/rrte/rrte_renderer.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <map>

namespace rrte_math {

Quat Quat::from_rotation_arc(Vec3 from, Vec3 to) {
    const float one_minus_eps = 1.0f - 2.0f * 1.1920929e-7f;
    const float d = from.dot(to);
    if (d > one_minus_eps) return Quat::identity();
    if (d < -one_minus_eps) {  // from_axis_angle(any_orthonormal_vector = X, PI)
        const float half = 3.14159265358979323846f * 0.5f;
        const float s = (float)std::sin((double)half), c = (float)std::cos((double)half);
        return {1.0f * s, 0.0f * s, 0.0f * s, c};
    }
    const Vec3 c = from.cross(to);
    const float x = c.x, y = c.y, z = c.z, w = 1.0f + d;
    // glam Vec4 (SSE2) dot: (x*x + z*z) + (y*y + w*w); normalize divides by the length
    const float len = std::sqrt((x * x + z * z) + (y * y + w * w));
    return {x / len, y / len, z / len, w / len};
}

}  // namespace rrte_math

namespace rrte_renderer {

namespace {

void fill(float* dst, std::initializer_list<float> v) {
    size_t i = 0;
    for (float f : v) dst[i++] = f;
}

rrte_sdf_node node(uint32_t op, std::initializer_list<float> f = {}, std::initializer_list<uint32_t> iv = {}) {
    rrte_sdf_node n;
    std::memset(&n, 0, sizeof n);
    n.op = op;
    fill(n.f, f);
    size_t k = 0;
    for (uint32_t v : iv) n.i[k++] = v;
    return n;
}

double dist3(const double* a, const double* b) {
    const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return std::sqrt(dx * dx + dy * dy + dz * dz);
}

Bound make_bound(Vec3 c, double r) { return Bound{{(double)c.x, (double)c.y, (double)c.z}, r}; }

uint32_t axis_index(Vec3 a) {
    for (int i = 0; i < 3; ++i) {
        bool ok = std::fabs(a[i]) == 1.0f;
        for (int j = 0; j < 3; ++j)
            if (j != i && a[j] != 0.0f) ok = false;
        if (ok) return (uint32_t)i;
    }
    throw Error(RRTE_UNSUPPORTED_PRIM, "deformer axis must be a coordinate axis");
}

Bound about_pivot(Vec3 pivot, Bound b) {
    const double p[3] = {(double)pivot.x, (double)pivot.y, (double)pivot.z};
    return Bound{{p[0], p[1], p[2]}, dist3(p, b.c) + b.r};
}

rrte_light light_struct(uint32_t kind, Color color, float intensity, Vec3 position = rrte_math::ZERO,
                        Vec3 direction = rrte_math::ZERO, float range = 100.0f, float lin = 0.09f,
                        float quad = 0.032f, float inner = 0.0f, float outer = 0.0f) {
    rrte_light l;
    std::memset(&l, 0, sizeof l);
    l.kind = kind;
    l.intensity = intensity;
    l.range = range;
    l.linear = lin;
    l.quadratic = quad;
    l.inner_angle = inner;
    l.outer_angle = outer;
    fill(l.position, {position.x, position.y, position.z, 0.0f});
    fill(l.direction, {direction.x, direction.y, direction.z, 0.0f});
    fill(l.color, {color.r, color.g, color.b, color.a});
    return l;
}

rrte_material material_struct(uint32_t kind, Color albedo, float fuzz, float ior) {
    rrte_material m;
    std::memset(&m, 0, sizeof m);
    m.kind = kind;
    m.fuzz = fuzz;
    m.ior = ior;
    fill(m.albedo, {albedo.r, albedo.g, albedo.b, albedo.a});
    return m;
}

}  // namespace

// --------------------------------------------------------------------------- materials
Color Material::ambient_color() const {
    const Color a = albedo();
    return {a.r * 0.1f, a.g * 0.1f, a.b * 0.1f, a.a * 0.1f};
}
rrte_material LambertianMaterial::lower() const { return material_struct(RRTE_MAT_LAMBERTIAN, albedo_, 0.0f, 1.0f); }
MetalMaterial::MetalMaterial(Color albedo, float r) : roughness(std::min(std::max(r, 0.0f), 1.0f)), albedo_(albedo) {}
rrte_material MetalMaterial::lower() const { return material_struct(RRTE_MAT_METAL, albedo_, roughness, 1.0f); }
rrte_material DielectricMaterial::lower() const { return material_struct(RRTE_MAT_DIELECTRIC, color, 0.0f, ior); }
rrte_material EmissiveMaterial::lower() const { return material_struct(RRTE_MAT_EMISSIVE, color, 0.0f, 1.0f); }

// ------------------------------------------------------------------------------ lights
std::shared_ptr<PointLight> PointLight::with_attenuation(Vec3 position, Color color, float intensity, float range,
                                                         float linear, float quadratic) {
    auto l = std::make_shared<PointLight>(position, color, intensity);
    l->range = range;
    l->linear_attenuation = linear;
    l->quadratic_attenuation = quadratic;
    return l;
}
rrte_light PointLight::lower() const {
    return light_struct(RRTE_LIGHT_POINT, color, intensity, position, rrte_math::ZERO, range, linear_attenuation,
                        quadratic_attenuation);
}
std::shared_ptr<DirectionalLight> DirectionalLight::sun() {
    return std::make_shared<DirectionalLight>(Vec3(-0.3f, -1.0f, -0.3f).normalize(), Color{1.0f, 0.95f, 0.8f, 1.0f},
                                              5.0f);
}
rrte_light DirectionalLight::lower() const {
    return light_struct(RRTE_LIGHT_DIRECTIONAL, color, intensity, rrte_math::ZERO, direction);
}
rrte_light SpotLight::lower() const {
    return light_struct(RRTE_LIGHT_SPOT, color, intensity, position, direction, range, linear_attenuation,
                        quadratic_attenuation, inner_angle, outer_angle);
}
std::shared_ptr<AmbientLight> AmbientLight::default_ambient() {
    return std::make_shared<AmbientLight>(Color{0.2f, 0.2f, 0.3f, 1.0f}, 0.3f);
}
rrte_light AmbientLight::lower() const { return light_struct(RRTE_LIGHT_AMBIENT, color, intensity); }

// ------------------------------------------------------------------------------ camera
Camera Camera::new_perspective(float fov, float aspect_ratio, float near, float far) {
    Camera c;
    c.projection = Projection::Perspective;
    c.fov = fov;
    c.aspect_ratio = aspect_ratio;
    c.near = near;
    c.far = far;
    return c;
}
Camera Camera::new_orthographic(float left, float right, float bottom, float top, float near, float far) {
    Camera c;
    c.projection = Projection::Orthographic;
    c.left = left;
    c.right = right;
    c.bottom = bottom;
    c.top = top;
    c.near = near;
    c.far = far;
    return c;
}
void Camera::look_at(Vec3 target, Vec3 up) {
    (void)up;  // camera.rs:88-89 computes and discards it
    const Vec3 fwd = (target - transform.position).normalize();
    transform.rotation = Quat::from_rotation_arc(Vec3(0.0f, 0.0f, -1.0f), fwd);
}
rrte_camera Camera::lower() const {
    rrte_camera c;
    std::memset(&c, 0, sizeof c);
    fill(c.position, {transform.position.x, transform.position.y, transform.position.z});
    fill(c.rotation, {transform.rotation.x, transform.rotation.y, transform.rotation.z, transform.rotation.w});
    fill(c.scale, {transform.scale.x, transform.scale.y, transform.scale.z});
    c.projection = projection == Projection::Perspective ? RRTE_PERSPECTIVE : RRTE_ORTHOGRAPHIC;
    c.fov = fov;
    c.aspect_ratio = aspect_ratio;
    c.near_plane = near;
    c.far_plane = far;
    c.left = left;
    c.right = right;
    c.bottom = bottom;
    c.top = top;
    return c;
}

// ---------------------------------------------------------------------------- lowering
class Lowering {
public:
    std::vector<rrte_sdf_node> nodes;
    std::vector<rrte_mesh_vertex> mesh_vertices;
    std::vector<uint32_t> mesh_indices;
    std::pair<uint32_t, uint32_t> add_mesh(const Mesh& m) {
        const uint32_t base = (uint32_t)mesh_vertices.size(), first = (uint32_t)(mesh_indices.size() / 3);
        const size_t nv = m.positions.size() / 3;
        for (size_t i = 0; i < nv; ++i) {
            rrte_mesh_vertex v;
            for (int k = 0; k < 3; ++k) {
                v.position[k] = m.positions[3 * i + k];
                v.normal[k] = m.normals[3 * i + k];
            }
            mesh_vertices.push_back(v);
        }
        for (uint32_t ix : m.indices) mesh_indices.push_back(ix + base);
        return {first, (uint32_t)(m.indices.size() / 3)};
    }
};

// ------------------------------------------------------------------------ scene objects
rrte_prim SceneObject::prim(uint32_t kind, std::initializer_list<float> p) const {
    rrte_prim r;
    std::memset(&r, 0, sizeof r);
    r.kind = kind;
    fill(r.p, p);
    const Transform& t = transform_;
    fill(r.trs, {t.position.x, t.position.y, t.position.z, t.rotation.x, t.rotation.y, t.rotation.z, t.rotation.w,
                 t.scale.x, t.scale.y, t.scale.z});
    return r;
}

Sphere::Sphere(Vec3 c, float r, std::shared_ptr<Material> m) : center(c), radius(r) { material_ = std::move(m); }
rrte_prim Sphere::lower(Lowering&) const {
    return prim(RRTE_PRIM_SPHERE, {center.x, center.y, center.z, radius});
}
Plane::Plane(Vec3 p, Vec3 n, std::shared_ptr<Material> m) : point(p), normal(n.normalize()) { material_ = std::move(m); }
rrte_prim Plane::lower(Lowering&) const {
    return prim(RRTE_PRIM_PLANE, {point.x, point.y, point.z, 0.0f, normal.x, normal.y, normal.z});
}
Triangle::Triangle(Vec3 v0, Vec3 v1, Vec3 v2, std::shared_ptr<Material> m) : vertices{v0, v1, v2} {
    const Vec3 n = (v1 - v0).cross(v2 - v0).normalize();
    normals[0] = normals[1] = normals[2] = n;
    material_ = std::move(m);
}
void Triangle::set_normals(Vec3 n0, Vec3 n1, Vec3 n2) {
    normals[0] = n0.normalize();
    normals[1] = n1.normalize();
    normals[2] = n2.normalize();
}
rrte_prim Triangle::lower(Lowering&) const {
    const Vec3 *v = vertices, *n = normals;
    return prim(RRTE_PRIM_TRIANGLE, {v[0].x, v[0].y, v[0].z, v[1].x, v[1].y, v[1].z, v[2].x, v[2].y, v[2].z,
                                     n[0].x, n[0].y, n[0].z, n[1].x, n[1].y, n[1].z, n[2].x, n[2].y, n[2].z});
}
Cube::Cube(Vec3 c, Vec3 s, std::shared_ptr<Material> m) : center(c), size(s) { material_ = std::move(m); }
rrte_prim Cube::lower(Lowering&) const {
    return prim(RRTE_PRIM_CUBE, {center.x, center.y, center.z, 0.0f, size.x, size.y, size.z});
}
Cylinder::Cylinder(Vec3 c, float r, float h, std::shared_ptr<Material> m) : center(c), radius(r), height(h) {
    material_ = std::move(m);
}
rrte_prim Cylinder::lower(Lowering&) const {
    return prim(RRTE_PRIM_CYLINDER, {center.x, center.y, center.z, radius, height});
}
Cone::Cone(Vec3 c, float r, float h, std::shared_ptr<Material> m) : center(c), radius(r), height(h) {
    material_ = std::move(m);
}
rrte_prim Cone::lower(Lowering&) const { return prim(RRTE_PRIM_CONE, {center.x, center.y, center.z, radius, height}); }
Capsule::Capsule(Vec3 c, float r, float h, std::shared_ptr<Material> m) : center(c), radius(r), height(h) {
    material_ = std::move(m);
}
rrte_prim Capsule::lower(Lowering&) const {
    return prim(RRTE_PRIM_CAPSULE, {center.x, center.y, center.z, radius, height});
}

Mesh::Mesh(std::vector<float> pos, std::vector<uint32_t> idx, std::vector<float> nrm, std::shared_ptr<Material> m)
    : positions(std::move(pos)), indices(std::move(idx)) {
    material_ = std::move(m);
    const size_t nv = positions.size() / 3, nt = indices.size() / 3;
    if (positions.size() % 3 || indices.size() % 3) throw Error(RRTE_INVALID_ARG, "mesh arrays must hold triples");
    for (uint32_t i : indices)
        if (i >= nv) throw Error(RRTE_INVALID_ARG, "mesh index out of range");
    auto P = [&](uint32_t i) { return Vec3(positions[3 * i], positions[3 * i + 1], positions[3 * i + 2]); };
    if (nrm.empty()) {  // face normals summed per vertex (rrte_amd/mesh.py: k-major, face order)
        nrm.assign(3 * nv, 0.0f);
        std::vector<Vec3> fn(nt);
        for (size_t t = 0; t < nt; ++t) {
            const Vec3 a = P(indices[3 * t + 1]) - P(indices[3 * t]), b = P(indices[3 * t + 2]) - P(indices[3 * t]);
            fn[t] = a.cross(b).normalize();
        }
        for (int k = 0; k < 3; ++k)
            for (size_t t = 0; t < nt; ++t) {
                const uint32_t v = indices[3 * t + k];
                nrm[3 * v] = nrm[3 * v] + fn[t].x;
                nrm[3 * v + 1] = nrm[3 * v + 1] + fn[t].y;
                nrm[3 * v + 2] = nrm[3 * v + 2] + fn[t].z;
            }
    }
    normals.resize(3 * nv);
    for (size_t i = 0; i < nv; ++i) {
        const Vec3 n = Vec3(nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]).normalize();
        normals[3 * i] = n.x;
        normals[3 * i + 1] = n.y;
        normals[3 * i + 2] = n.z;
    }
}
rrte_prim Mesh::lower(Lowering& lw) const {
    rrte_prim r = prim(RRTE_PRIM_MESH, {});
    const auto fc = lw.add_mesh(*this);
    r.sdf_first = fc.first;
    r.sdf_count = fc.second;
    return r;
}

// ------------------------------------------------------------------ SDF / CSG / deformers
namespace {

class Leaf : public SDF {
public:
    Leaf(uint32_t op, Vec3 c, std::vector<float> f, double r) : op_(op), c_(c), f_(std::move(f)), r_(r) {}
    void emit(std::vector<rrte_sdf_node>& out) const override {
        rrte_sdf_node n = node(op_);
        n.f[0] = c_.x;
        n.f[1] = c_.y;
        n.f[2] = c_.z;
        for (size_t k = 0; k < f_.size(); ++k) n.f[3 + k] = f_[k];
        out.push_back(n);
    }
    Bound bound() const override { return make_bound(c_, r_); }
private:
    uint32_t op_;
    Vec3 c_;
    std::vector<float> f_;
    double r_;
};

class Composite : public SDF {
public:
    Composite(SDFRef a, SDFRef b, CSGOperation op, float k) : a_(std::move(a)), b_(std::move(b)), op_(op), k_(k) {}
    void emit(std::vector<rrte_sdf_node>& out) const override {
        a_->emit(out);
        b_->emit(out);
        out.push_back(node(RRTE_SDF_UNION + (uint32_t)op_, {k_}));
    }
    Bound bound() const override {
        const Bound ba = a_->bound(), bb = b_->bound();
        const double k = std::fabs((double)k_);
        Bound r;
        if (op_ == CSGOperation::Union || op_ == CSGOperation::SmoothUnion) {
            const double d = dist3(ba.c, bb.c);
            if (d + bb.r <= ba.r) {
                r = ba;
            } else if (d + ba.r <= bb.r) {
                r = bb;
            } else {
                const double rr = (d + ba.r + bb.r) * 0.5;
                const double t = d > 0 ? (rr - ba.r) / d : 0.0;
                r = Bound{{ba.c[0] + (bb.c[0] - ba.c[0]) * t, ba.c[1] + (bb.c[1] - ba.c[1]) * t,
                           ba.c[2] + (bb.c[2] - ba.c[2]) * t},
                          rr};
            }
        } else if (op_ == CSGOperation::Difference || op_ == CSGOperation::SmoothDifference) {
            r = ba;
        } else {
            r = ba.r <= bb.r ? ba : bb;
        }
        r.r = r.r + k;
        return r;
    }
    bool has_deformer() const override { return a_->has_deformer() || b_->has_deformer(); }
private:
    SDFRef a_, b_;
    CSGOperation op_;
    float k_;
};

class SimpleDeformer : public Deformer {
public:
    using GrowFn = Bound (*)(const SimpleDeformer&, Bound);
    SimpleDeformer(rrte_sdf_node n, Vec3 pivot, GrowFn g, double a = 0.0, double b = 0.0, uint32_t oct = 0)
        : n_(n), pivot(pivot), grow_(g), pa(a), pb(b), octaves(oct) {}
    void nodes(std::vector<rrte_sdf_node>& out) const override { out.push_back(n_); }
    Bound grow(Bound b) const override { return grow_(*this, b); }
    rrte_sdf_node n_;
    Vec3 pivot;
    GrowFn grow_;
    double pa, pb;
    uint32_t octaves;
};

class Chain : public Deformer {
public:
    std::vector<DeformerRef> parts;
    void nodes(std::vector<rrte_sdf_node>& out) const override {
        for (const auto& p : parts) p->nodes(out);
    }
    Bound grow(Bound b) const override {  // innermost first
        for (auto it = parts.rbegin(); it != parts.rend(); ++it) b = (*it)->grow(b);
        return b;
    }
};

class Deformed : public SDF {
public:
    Deformed(SDFRef s, DeformerRef d) : s_(std::move(s)), d_(std::move(d)) {}
    void emit(std::vector<rrte_sdf_node>& out) const override {
        std::vector<rrte_sdf_node> ns;
        d_->nodes(ns);
        out.insert(out.end(), ns.begin(), ns.end());
        s_->emit(out);
        for (size_t i = 0; i < ns.size(); ++i) out.push_back(node(RRTE_SDF_POP_POINT));
    }
    Bound bound() const override { return d_->grow(s_->bound()); }
    bool has_deformer() const override { return true; }
private:
    SDFRef s_;
    DeformerRef d_;
};

}  // namespace

SDFRef sdf_sphere(Vec3 c, double r) { return std::make_shared<Leaf>(RRTE_SDF_SPHERE, c, std::vector<float>{(float)r}, r); }
SDFRef sdf_box(Vec3 c, Vec3 s) {
    const double sx = s.x, sy = s.y, sz = s.z;
    return std::make_shared<Leaf>(RRTE_SDF_BOX, c, std::vector<float>{0.0f, s.x, s.y, s.z},
                                  0.5 * std::sqrt(sx * sx + sy * sy + sz * sz));
}
SDFRef sdf_cylinder(Vec3 c, double r, double h) {
    return std::make_shared<Leaf>(RRTE_SDF_CYLINDER, c, std::vector<float>{(float)r, (float)h}, std::hypot(r, h * 0.5));
}
SDFRef sdf_prism(Vec3 c, Vec3 s) {
    const double a = (double)s.y * 0.5, b = (double)s.y * 0.433, d = (double)s.z * 0.5;
    return std::make_shared<Leaf>(RRTE_SDF_PRISM, c, std::vector<float>{0.0f, s.x, s.y, s.z},
                                  std::sqrt(a * a + b * b + d * d));
}
SDFRef sdf_torus(Vec3 c, double R, double r) {
    return std::make_shared<Leaf>(RRTE_SDF_TORUS, c, std::vector<float>{(float)R, (float)r}, R + r);
}
SDFRef sdf_tube(Vec3 c, double ro, double ri, double h) {
    return std::make_shared<Leaf>(RRTE_SDF_TUBE, c, std::vector<float>{(float)ro, (float)ri, (float)h}, std::hypot(ro, h * 0.5));
}
SDFRef sdf_ring(Vec3 c, double R, double r) {
    return std::make_shared<Leaf>(RRTE_SDF_RING, c, std::vector<float>{(float)R, (float)r}, R + r);
}
SDFRef sdf_cone(Vec3 c, double r, double h) {
    return std::make_shared<Leaf>(RRTE_SDF_CONE, c, std::vector<float>{(float)r, (float)h}, std::hypot(r, h * 0.5));
}
SDFRef sdf_capsule(Vec3 c, double r, double h) {
    return std::make_shared<Leaf>(RRTE_SDF_CAPSULE, c, std::vector<float>{(float)r, (float)h}, h * 0.5 + r);
}
SDFRef sdf_ellipsoid(Vec3 c, Vec3 radii) {
    return std::make_shared<Leaf>(RRTE_SDF_ELLIPSOID, c, std::vector<float>{0.0f, radii.x, radii.y, radii.z},
                                  (double)std::max(radii.x, std::max(radii.y, radii.z)));
}
SDFRef csg(SDFRef a, SDFRef b, CSGOperation op, float k) { return std::make_shared<Composite>(a, b, op, k); }

DeformerRef twist(Vec3 axis, float rate, Vec3 pivot) {
    return std::make_shared<SimpleDeformer>(node(RRTE_SDF_TWIST, {pivot.x, pivot.y, pivot.z, rate}, {axis_index(axis)}),
                                            pivot, [](const SimpleDeformer& d, Bound b) { return about_pivot(d.pivot, b); });
}
DeformerRef bend(Vec3 axis, Vec3 direction, float amount, Vec3 pivot) {
    return std::make_shared<SimpleDeformer>(
        node(RRTE_SDF_BEND, {pivot.x, pivot.y, pivot.z, amount}, {axis_index(axis), axis_index(direction)}), pivot,
        [](const SimpleDeformer& d, Bound b) { return about_pivot(d.pivot, b); });
}
DeformerRef taper(Vec3 axis, float start, float end, float length, Vec3 pivot) {
    return std::make_shared<SimpleDeformer>(
        node(RRTE_SDF_TAPER, {pivot.x, pivot.y, pivot.z, start, end, length}, {axis_index(axis)}), pivot,
        [](const SimpleDeformer& d, Bound b) {
            Bound p = about_pivot(d.pivot, b);
            p.r = p.r * std::max(1.0, std::max(std::fabs(d.pa), std::fabs(d.pb)));
            return p;
        },
        (double)start, (double)end);
}
DeformerRef noise(float frequency, float amplitude, Vec3 pivot, uint32_t seed, uint32_t octaves, float persistence) {
    if (octaves > RRTE_SDF_MAX_OCTAVES) throw Error(RRTE_INVALID_ARG, "noise octaves > RRTE_SDF_MAX_OCTAVES");
    return std::make_shared<SimpleDeformer>(
        node(RRTE_SDF_NOISE, {pivot.x, pivot.y, pivot.z, frequency, amplitude, persistence}, {octaves, seed}), pivot,
        [](const SimpleDeformer& d, Bound b) {
            double total = 0.0;
            for (uint32_t o = 0; o < d.octaves; ++o) total = total + std::pow(std::fabs(d.pb), (double)o);
            b.r = b.r + std::sqrt(3.0) * std::fabs(d.pa) * total;
            return b;
        },
        (double)amplitude, (double)persistence, octaves);
}
DeformerRef wave(Vec3 axis, float amplitude, float frequency, Vec3 displaced_axis, Vec3 pivot) {
    return std::make_shared<SimpleDeformer>(
        node(RRTE_SDF_WAVE, {pivot.x, pivot.y, pivot.z, amplitude, frequency},
             {axis_index(axis), axis_index(displaced_axis)}),
        pivot,
        [](const SimpleDeformer& d, Bound b) {
            b.r = b.r + std::fabs(d.pa);
            return b;
        },
        (double)amplitude);
}
DeformerRef chain(DeformerRef first, DeformerRef then) {
    auto c = std::make_shared<Chain>();
    for (const DeformerRef& d : {first, then}) {
        if (auto* ch = dynamic_cast<Chain*>(d.get())) c->parts.insert(c->parts.end(), ch->parts.begin(), ch->parts.end());
        else c->parts.push_back(d);
    }
    return c;
}
SDFRef deformed(SDFRef sdf, DeformerRef d) { return std::make_shared<Deformed>(std::move(sdf), std::move(d)); }

SDFObject::SDFObject(SDFRef s, std::shared_ptr<Material> m, uint32_t max_steps, float step_scale, float hit_eps)
    : sdf(std::move(s)), max_steps(max_steps),
      step_scale(step_scale < 0.0f ? (sdf->has_deformer() ? 0.6f : 1.0f) : step_scale), hit_eps(hit_eps) {
    material_ = std::move(m);
}
rrte_prim SDFObject::lower(Lowering& lw) const {
    std::vector<rrte_sdf_node> ns;
    sdf->emit(ns);
    const Bound b = sdf->bound();
    const double r = b.r * 1.001 + 1e-3;
    rrte_prim p = prim(RRTE_PRIM_SDF, {(float)b.c[0], (float)b.c[1], (float)b.c[2], (float)r});
    p.sdf_first = (uint32_t)lw.nodes.size();
    p.sdf_count = (uint32_t)ns.size();
    p.sdf_max_steps = max_steps;
    p.sdf_step_scale = step_scale;
    p.sdf_hit_eps = hit_eps;
    lw.nodes.insert(lw.nodes.end(), ns.begin(), ns.end());
    return p;
}

// ----------------------------------------------------------------------------- renderer
rrte_render_params RaytracerConfig::lower() const {
    rrte_render_params p;
    std::memset(&p, 0, sizeof p);
    p.width = width;
    p.height = height;
    p.samples_per_pixel = samples_per_pixel;
    p.max_depth = max_depth;
    p.mode = (uint32_t)mode;
    p.jitter = (uint32_t)jitter;
    p.seed = seed;
    fill(p.background, {background_color.r, background_color.g, background_color.b, background_color.a});
    p.t_min = t_min;
    p.shadow_bias = shadow_bias;
    p.gamma = gamma;
    p.band_rows = band_rows;
    return p;
}

LoweredScene::LoweredScene(const Objects& objects, const Lights& lights, const Camera& camera) {
    Lowering lw;
    std::map<const Material*, int32_t> index;
    std::vector<std::shared_ptr<Material>> mats;
    for (const auto& o : objects) {
        rrte_prim p = o->lower(lw);
        const auto m = o->material();
        if (!m) {
            p.material = -1;
        } else {
            auto it = index.find(m.get());
            if (it == index.end()) {  // dedupe by identity, in order of first use
                it = index.emplace(m.get(), (int32_t)mats.size()).first;
                mats.push_back(m);
            }
            p.material = it->second;
        }
        prims_.push_back(p);
    }
    for (const auto& m : mats) mats_.push_back(m->lower());
    for (const auto& l : lights) lights_.push_back(l->lower());
    nodes_ = std::move(lw.nodes);
    mesh_vertices_ = std::move(lw.mesh_vertices);
    mesh_indices_ = std::move(lw.mesh_indices);
    ir_.prims = prims_.data();
    ir_.num_prims = (uint32_t)prims_.size();
    ir_.materials = mats_.data();
    ir_.num_materials = (uint32_t)mats_.size();
    ir_.lights = lights_.data();
    ir_.num_lights = (uint32_t)lights_.size();
    ir_.sdf_nodes = nodes_.data();
    ir_.num_sdf_nodes = (uint32_t)nodes_.size();
    ir_.camera = camera.lower();
    ir_.mesh_vertices = mesh_vertices_.data();
    ir_.num_mesh_vertices = (uint32_t)mesh_vertices_.size();
    ir_.mesh_indices = mesh_indices_.data();
    ir_.num_mesh_indices = (uint32_t)mesh_indices_.size();
    // arrays are immutable for this object's life; the stamp is process-wide and atomic, since scenes
    // may be lowered on several threads and two meshes must never share a stamp (the library keys its
    // BVH cache on it: tools/tsan.sh found the plain counter racing)
    static std::atomic<uint64_t> version{0};
    ir_.mesh_version = mesh_indices_.empty() ? 0 : version.fetch_add(1, std::memory_order_relaxed) + 1;
}

std::vector<uint8_t> LoweredScene::bytes() const {
    std::vector<uint8_t> out;
    auto put = [&](const void* p, size_t n) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        out.insert(out.end(), b, b + n);
    };
    put(prims_.data(), prims_.size() * sizeof(rrte_prim));
    put(mats_.data(), mats_.size() * sizeof(rrte_material));
    put(lights_.data(), lights_.size() * sizeof(rrte_light));
    put(nodes_.data(), nodes_.size() * sizeof(rrte_sdf_node));
    put(&ir_.camera, sizeof(rrte_camera));
    put(mesh_vertices_.data(), mesh_vertices_.size() * sizeof(rrte_mesh_vertex));
    put(mesh_indices_.data(), mesh_indices_.size() * sizeof(uint32_t));
    return out;
}

Raytracer::Raytracer(RaytracerConfig config, int device) : config_(config) {
    const rrte_status st = rrte_hip_create(device, &ctx_);
    if (st != RRTE_OK) throw Error(st, "rrte_hip_create failed (no HIP device?)");
}
Raytracer::~Raytracer() { rrte_hip_destroy(ctx_); }
void Raytracer::check(rrte_status st) const {
    if (st != RRTE_OK) throw Error(st, rrte_hip_last_error(ctx_));
}
void Raytracer::set_jit(int mode) { check(rrte_hip_set_jit(ctx_, mode)); }
std::vector<uint8_t> Raytracer::render(const Objects& objects, const Lights& lights, const Materials& materials,
                                       const Camera& camera) {
    (void)materials;  // raytracer.rs passes it through unused; objects carry their materials
    const LoweredScene sc(objects, lights, camera);
    const rrte_render_params p = config_.lower();
    std::vector<uint8_t> out((size_t)p.width * p.height * 4);
    check(rrte_hip_render(ctx_, &sc.ir(), &p, out.data()));
    return out;
}
void Raytracer::render_into(const Objects& objects, const Lights& lights, const Materials& materials,
                            const Camera& camera, std::vector<uint8_t>& out) {
    (void)materials;
    const LoweredScene sc(objects, lights, camera);
    const rrte_render_params p = config_.lower();
    const size_t need = (size_t)p.width * p.height * 4;
    if (pinned_ && (pinned_ != out.data() || pinned_len_ != out.size() || out.size() != need)) {
        check(rrte_hip_host_unregister(ctx_, pinned_));  // (before a resize may move or free it)
        pinned_ = nullptr;
    }
    out.resize(need);
    if (!pinned_ && unpinnable_ != out.data()) {
        if (rrte_hip_host_register(ctx_, out.data(), out.size()) == RRTE_OK) {
            pinned_ = out.data();
            pinned_len_ = out.size();
        } else {
            unpinnable_ = out.data();
        }
    }
    check(rrte_hip_render(ctx_, &sc.ir(), &p, out.data()));
}
std::pair<std::vector<uint8_t>, std::vector<float>> Raytracer::render_f32(const Objects& objects,
                                                                          const Lights& lights,
                                                                          const Camera& camera, bool linear) {
    const LoweredScene sc(objects, lights, camera);
    rrte_render_params p = config_.lower();
    if (linear) p.flags |= RRTE_FLAG_F32_LINEAR;
    std::vector<uint8_t> out8((size_t)p.width * p.height * 4);
    std::vector<float> outf((size_t)p.width * p.height * 4);
    check(rrte_hip_render_f32(ctx_, &sc.ir(), &p, out8.data(), outf.data()));
    return {std::move(out8), std::move(outf)};
}
rrte_stats Raytracer::stats() const {
    rrte_stats s;
    check(rrte_hip_stats(ctx_, &s));
    return s;
}

}  // namespace rrte_renderer
