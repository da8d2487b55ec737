// rrte_renderer.hpp — C++ mirror of the reference's renderer API above the C ABI.
//
// The reference (Melthizar/RRTE) is Rust: rrte_math::{Vec3, Quat, Color, Transform},
// rrte_renderer::{Raytracer, RaytracerConfig, Camera, SceneObject + Sphere/Plane/Triangle/Cube/
// Cylinder/Cone/Capsule, Light + Point/Directional/Spot/Ambient, Material + Lambertian/Metal/
// Dielectric/Emissive} and the README-only SDF/CSG/Deformer surface.  This image has no Rust
// toolchain, so the host side above include/rrte_hip.h is written in C++ with the same names,
// argument meaning and defaults (Arc<dyn T> -> std::shared_ptr<T>), and Raytracer::render keeps the
// reference signature (raytracer.rs:45-51): objects, lights, materials, camera in; W*H*4 RGBA8 out.
// Every object lowers to the C ABI's POD records exactly as the Python mirror (rrte_amd/) does --
// tests/test_cpp_mirror.py checks the two lowerings byte for byte -- and rendering always runs on
// the GPU through librrte_hip.so: there is no CPU path, so SceneObject has no CPU intersect().
// Errors (infallible `render` in the reference) are thrown as rrte_renderer::Error.
#pragma once

#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../rrte_hip.h"

namespace rrte_math {

// glam::Vec3 with glam 0.24's f32 operation order (dot = (x*x + y*y) + z*z; normalize = v * (1/len)).
struct Vec3 {
    float x = 0.0f, y = 0.0f, z = 0.0f;
    constexpr Vec3() = default;
    constexpr Vec3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
    static constexpr Vec3 splat(float v) { return {v, v, v}; }
    Vec3 operator+(Vec3 o) const { return {x + o.x, y + o.y, z + o.z}; }
    Vec3 operator-(Vec3 o) const { return {x - o.x, y - o.y, z - o.z}; }
    Vec3 operator*(float s) const { return {x * s, y * s, z * s}; }
    Vec3 operator-() const { return {-x, -y, -z}; }
    float dot(Vec3 o) const { return (x * o.x + y * o.y) + z * o.z; }
    Vec3 cross(Vec3 o) const { return {y * o.z - o.y * z, z * o.x - o.z * x, x * o.y - o.x * y}; }
    float length() const { return std::sqrt(dot(*this)); }
    Vec3 normalize() const { return *this * (1.0f / std::sqrt(dot(*this))); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline constexpr Vec3 ZERO{0.0f, 0.0f, 0.0f};
inline constexpr Vec3 ONE{1.0f, 1.0f, 1.0f};

struct Quat {
    float x = 0.0f, y = 0.0f, z = 0.0f, w = 1.0f;
    static constexpr Quat identity() { return {0.0f, 0.0f, 0.0f, 1.0f}; }
    // glam Quat::from_rotation_arc (Camera::look_at, camera.rs:85-95)
    static Quat from_rotation_arc(Vec3 from, Vec3 to);
};

// rrte_math::Color (color.rs:6-11): RGBA f32.
struct Color {
    float r = 0.0f, g = 0.0f, b = 0.0f, a = 1.0f;
    static constexpr Color rgb(float r, float g, float b) { return {r, g, b, 1.0f}; }
    static constexpr Color gray(float v) { return {v, v, v, 1.0f}; }
    static constexpr Color black() { return {0.0f, 0.0f, 0.0f, 1.0f}; }
    static constexpr Color white() { return {1.0f, 1.0f, 1.0f, 1.0f}; }
};

// rrte_math::Transform (transform.rs:6-10).
struct Transform {
    Vec3 position = ZERO;
    Quat rotation = Quat::identity();
    Vec3 scale = ONE;
    static Transform identity() { return {}; }
    static Transform from_position(Vec3 p) {
        Transform t;
        t.position = p;
        return t;
    }
};

// f32::to_radians: deg * (PI / 180) in f32.
inline float to_radians(float deg) { return deg * (3.14159265358979323846f / 180.0f); }

}  // namespace rrte_math

namespace rrte_renderer {

using rrte_math::Color;
using rrte_math::Quat;
using rrte_math::Transform;
using rrte_math::Vec3;

struct Error : std::runtime_error {
    rrte_status status;
    Error(rrte_status s, const std::string& what) : std::runtime_error(what), status(s) {}
};

// ------------------------------------------------------------------ materials (material.rs)
class Material {
public:
    virtual ~Material() = default;
    virtual Color albedo() const = 0;
    Color ambient_color() const;  // albedo * 0.1 (material.rs:10-12)
    virtual rrte_material lower() const = 0;
};
class LambertianMaterial : public Material {
public:
    explicit LambertianMaterial(Color albedo) : albedo_(albedo) {}
    static std::shared_ptr<LambertianMaterial> create(Color albedo) { return std::make_shared<LambertianMaterial>(albedo); }
    Color albedo() const override { return albedo_; }
    rrte_material lower() const override;
private:
    Color albedo_;
};
class MetalMaterial : public Material {
public:
    MetalMaterial(Color albedo, float roughness);  // roughness clamped to [0, 1]
    Color albedo() const override { return albedo_; }
    rrte_material lower() const override;
    float roughness;
private:
    Color albedo_;
};
class DielectricMaterial : public Material {
public:
    explicit DielectricMaterial(float ior, Color color = Color::white()) : ior(ior), color(color) {}
    Color albedo() const override { return color; }
    rrte_material lower() const override;
    float ior;
    Color color;
};
class EmissiveMaterial : public Material {
public:
    EmissiveMaterial(Color color, float intensity) : color(color), intensity(intensity) {}
    Color albedo() const override { return color; }
    rrte_material lower() const override;
    Color color;
    float intensity;
};

// --------------------------------------------------------------------- lights (light.rs)
class Light {
public:
    virtual ~Light() = default;
    virtual rrte_light lower() const = 0;
    Transform transform;
};
class PointLight : public Light {
public:
    PointLight(Vec3 position, Color color, float intensity) : position(position), color(color), intensity(intensity) {}
    static std::shared_ptr<PointLight> with_attenuation(Vec3 position, Color color, float intensity, float range,
                                                        float linear, float quadratic);
    rrte_light lower() const override;
    Vec3 position;
    Color color;
    float intensity, range = 100.0f, linear_attenuation = 0.09f, quadratic_attenuation = 0.032f;
};
class DirectionalLight : public Light {
public:
    DirectionalLight(Vec3 direction, Color color, float intensity)
        : direction(direction.normalize()), color(color), intensity(intensity) {}
    static std::shared_ptr<DirectionalLight> sun();
    rrte_light lower() const override;
    Vec3 direction;
    Color color;
    float intensity;
};
class SpotLight : public Light {
public:
    SpotLight(Vec3 position, Vec3 direction, Color color, float intensity, float inner_angle, float outer_angle)
        : position(position), direction(direction.normalize()), color(color), intensity(intensity),
          inner_angle(inner_angle), outer_angle(outer_angle) {}
    rrte_light lower() const override;
    Vec3 position, direction;
    Color color;
    float intensity, inner_angle, outer_angle, range = 100.0f, linear_attenuation = 0.09f,
                                                quadratic_attenuation = 0.032f;
};
class AmbientLight : public Light {
public:
    AmbientLight(Color color, float intensity) : color(color), intensity(intensity) {}
    static std::shared_ptr<AmbientLight> default_ambient();
    rrte_light lower() const override;
    Color color;
    float intensity;
};

// --------------------------------------------------------------------- camera (camera.rs)
enum class Projection { Perspective, Orthographic };
struct Camera {
    Transform transform;
    Projection projection = Projection::Perspective;
    float fov = 0.0f, aspect_ratio = 1.0f, near = 0.1f, far = 100.0f;
    float left = -1.0f, right = 1.0f, bottom = -1.0f, top = 1.0f;
    static Camera new_perspective(float fov, float aspect_ratio, float near, float far);
    static Camera new_orthographic(float left, float right, float bottom, float top, float near, float far);
    // rotation = Quat::from_rotation_arc(-Z, normalize(target - position)); `up` unused (camera.rs:85-95)
    void look_at(Vec3 target, Vec3 up = Vec3(0.0f, 1.0f, 0.0f));
    rrte_camera lower() const;
};

class Lowering;

// -------------------------------------------------------------- scene objects (primitives.rs)
class SceneObject {
public:
    virtual ~SceneObject() = default;
    std::shared_ptr<Material> material() const { return material_; }
    void set_material(std::shared_ptr<Material> m) { material_ = std::move(m); }
    const Transform& transform() const { return transform_; }
    void set_transform(const Transform& t) { transform_ = t; }
    // the additive lowering hook (gpu_desc): this object as an rrte_prim
    virtual rrte_prim lower(Lowering& lw) const = 0;
protected:
    rrte_prim prim(uint32_t kind, std::initializer_list<float> p) const;
    std::shared_ptr<Material> material_;
    Transform transform_;
};
class Sphere : public SceneObject {
public:
    Sphere(Vec3 center, float radius, std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    Vec3 center;
    float radius;
};
class Plane : public SceneObject {
public:
    Plane(Vec3 point, Vec3 normal, std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    Vec3 point, normal;
};
class Triangle : public SceneObject {
public:
    Triangle(Vec3 v0, Vec3 v1, Vec3 v2, std::shared_ptr<Material> m = nullptr);  // face normal on all vertices
    void set_normals(Vec3 n0, Vec3 n1, Vec3 n2);                                  // normalised
    rrte_prim lower(Lowering&) const override;
    Vec3 vertices[3], normals[3];
};
class Cube : public SceneObject {
public:
    Cube(Vec3 center, Vec3 size, std::shared_ptr<Material> m = nullptr);  // size = full extents
    rrte_prim lower(Lowering&) const override;
    Vec3 center, size;
};
class Cylinder : public SceneObject {
public:
    Cylinder(Vec3 center, float radius, float height, std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    Vec3 center;
    float radius, height;
};
class Cone : public SceneObject {
public:
    Cone(Vec3 center, float radius, float height, std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    Vec3 center;
    float radius, height;
};
class Capsule : public SceneObject {
public:
    Capsule(Vec3 center, float radius, float height, std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    Vec3 center;
    float radius, height;
};

// Triangle mesh (rrte-assets MeshAsset, asset.rs:53-65): a Vec<Triangle> with set_normals.
class Mesh : public SceneObject {
public:
    // positions/normals: 3 floats per vertex; indices: 3 per triangle.  Normals are normalised here;
    // empty normals -> area-weighted face normals.
    Mesh(std::vector<float> positions, std::vector<uint32_t> indices, std::vector<float> normals = {},
         std::shared_ptr<Material> m = nullptr);
    rrte_prim lower(Lowering&) const override;
    std::vector<float> positions, normals;
    std::vector<uint32_t> indices;
};

// ----------------------------------------------------- SDF / CSG / deformers (README.md:458-510)
struct Bound {
    double c[3];
    double r;
};
class SDF {
public:
    virtual ~SDF() = default;
    virtual void emit(std::vector<rrte_sdf_node>& out) const = 0;
    virtual Bound bound() const = 0;  // sphere containing the zero set
    virtual bool has_deformer() const { return false; }
};
using SDFRef = std::shared_ptr<SDF>;

// Scalar sizes are taken in double: the node stores them rounded to f32, the bounding sphere is
// computed from the value as given (as the Python mirror does).
SDFRef sdf_sphere(Vec3 c, double radius);
SDFRef sdf_box(Vec3 c, Vec3 size);                             // full extents
SDFRef sdf_cylinder(Vec3 c, double radius, double height);     // Y axis
SDFRef sdf_prism(Vec3 c, Vec3 size);
SDFRef sdf_torus(Vec3 c, double major, double minor);          // XZ ring
SDFRef sdf_tube(Vec3 c, double outer, double inner, double height);
SDFRef sdf_ring(Vec3 c, double major, double minor);           // XY ring
SDFRef sdf_cone(Vec3 c, double radius, double height);         // apex +Y
SDFRef sdf_capsule(Vec3 c, double radius, double height);
SDFRef sdf_ellipsoid(Vec3 c, Vec3 radii);

enum class CSGOperation { Union, Difference, Intersection, SmoothUnion, SmoothDifference, SmoothIntersection };
SDFRef csg(SDFRef a, SDFRef b, CSGOperation op, float k = 0.0f);

class Deformer {
public:
    virtual ~Deformer() = default;
    virtual void nodes(std::vector<rrte_sdf_node>& out) const = 0;
    virtual Bound grow(Bound b) const = 0;
};
using DeformerRef = std::shared_ptr<Deformer>;
// axes are coordinate axes (unit X/Y/Z, either sign)
DeformerRef twist(Vec3 axis, float rate, Vec3 pivot = rrte_math::ZERO);
DeformerRef bend(Vec3 axis, Vec3 direction, float amount, Vec3 pivot = rrte_math::ZERO);
DeformerRef taper(Vec3 axis, float start, float end, float length, Vec3 pivot = rrte_math::ZERO);
DeformerRef noise(float frequency, float amplitude, Vec3 pivot = rrte_math::ZERO, uint32_t seed = 0,
                  uint32_t octaves = 1, float persistence = 0.5f);
DeformerRef wave(Vec3 axis, float amplitude, float frequency, Vec3 displaced_axis, Vec3 pivot = rrte_math::ZERO);
DeformerRef chain(DeformerRef first, DeformerRef then);  // d1.chain(d2) = d2(d1(p))
SDFRef deformed(SDFRef sdf, DeformerRef deformer);

class SDFObject : public SceneObject {
public:
    SDFObject(SDFRef sdf, std::shared_ptr<Material> m = nullptr, uint32_t max_steps = 128, float step_scale = -1.0f,
              float hit_eps = 1e-4f);  // step_scale < 0: 0.6 with deformers, else 1.0
    rrte_prim lower(Lowering&) const override;
    SDFRef sdf;
    uint32_t max_steps;
    float step_scale, hit_eps;
};

// ------------------------------------------------------------------- renderer (raytracer.rs)
enum class Mode : uint32_t { RefCompat = RRTE_MODE_REFCOMPAT, LambertShadow = RRTE_MODE_LAMBERT_SHADOW };
enum class Jitter : uint32_t { Center = RRTE_JITTER_CENTER, Random = RRTE_JITTER_RANDOM };

struct RaytracerConfig {  // raytracer.rs:8-26 + this path's build-defined knobs
    uint32_t max_depth = 50, samples_per_pixel = 100, width = 800, height = 600;
    Color background_color{0.5f, 0.7f, 1.0f, 1.0f};
    Mode mode = Mode::RefCompat;
    Jitter jitter = Jitter::Random;
    uint32_t seed = 0;
    float t_min = 0.001f, shadow_bias = 1e-3f, gamma = 2.2f;
    uint32_t band_rows = 16;
    rrte_render_params lower() const;
};

using Objects = std::vector<std::shared_ptr<SceneObject>>;
using Lights = std::vector<std::shared_ptr<Light>>;
using Materials = std::vector<std::shared_ptr<Material>>;

// A scene lowered to rrte_scene_ir (owns the arrays the IR points into).
class LoweredScene {
public:
    LoweredScene(const Objects& objects, const Lights& lights, const Camera& camera);
    const rrte_scene_ir& ir() const { return ir_; }
    // the IR's bytes in a fixed order (prims, materials, lights, nodes, camera, mesh vertices, mesh
    // indices), for comparing lowerings
    std::vector<uint8_t> bytes() const;
private:
    std::vector<rrte_prim> prims_;
    std::vector<rrte_material> mats_;
    std::vector<rrte_light> lights_;
    std::vector<rrte_sdf_node> nodes_;
    std::vector<rrte_mesh_vertex> mesh_vertices_;
    std::vector<uint32_t> mesh_indices_;
    rrte_scene_ir ir_{};
};

class Raytracer {
public:
    explicit Raytracer(RaytracerConfig config = {}, int device = 0);
    ~Raytracer();
    Raytracer(const Raytracer&) = delete;
    Raytracer& operator=(const Raytracer&) = delete;
    void update_config(const RaytracerConfig& config) { config_ = config; }
    const RaytracerConfig& config() const { return config_; }
    void set_jit(int mode);  // RRTE_JIT_OFF / ON / AUTO
    // raytracer.rs:45-51: W*H*4 RGBA8, row 0 = top.  `materials` is accepted for signature parity
    // (the reference passes it through unused); objects carry their materials.
    std::vector<uint8_t> render(const Objects& objects, const Lights& lights, const Materials& materials,
                                const Camera& camera);
    // Engine::render_frame's loop (engine.rs:82,293; rust/patches/0002): the frame into the caller's
    // buffer, reused every frame and pinned once (rrte_hip_host_register) so the kernel stores the
    // frame straight into it.  `out` is resized to W*H*4; a buffer that moved since it was pinned is
    // unpinned first, one that cannot be pinned takes the copy path.  Keep `out` alive (and do not
    // reallocate it outside this call) until the next call or the Raytracer's destruction.
    void render_into(const Objects& objects, const Lights& lights, const Materials& materials,
                     const Camera& camera, std::vector<uint8_t>& out);
    // parity variant: RGBA8 plus the float image (post-gamma, or linear pre-gamma)
    std::pair<std::vector<uint8_t>, std::vector<float>> render_f32(const Objects& objects, const Lights& lights,
                                                                   const Camera& camera, bool linear = false);
    rrte_stats stats() const;
    // the C ABI call on an already lowered scene (diagnostics, tests/cpp/cpp_mirror_tool.cpp)
    void render_raw(const rrte_scene_ir& ir, const rrte_render_params& p, uint8_t* out) {
        check(rrte_hip_render(ctx_, &ir, &p, out));
    }
private:
    void check(rrte_status st) const;
    RaytracerConfig config_;
    rrte_ctx* ctx_ = nullptr;
    void* pinned_ = nullptr;      // the buffer render_into pinned
    size_t pinned_len_ = 0;
    const void* unpinnable_ = nullptr;  // the last buffer that could not be pinned (copy path)
};

}  // namespace rrte_renderer
