// examples.cpp — see examples.hpp.
#include "examples.hpp"

#include <cmath>
#include <stdexcept>

using namespace rrte_renderer;
using rrte_math::to_radians;

namespace rrte_examples {
namespace {

Camera camera(uint32_t w, uint32_t h, Vec3 pos, Vec3 target, float fov_deg) {
    // Engine::new: perspective fov 45deg, aspect = w/h (engine.rs:97-98); demos then set fov + look_at
    Camera c = Camera::new_perspective(to_radians(45.0f), (float)w / (float)h, 0.1f, 100.0f);
    c.fov = to_radians(fov_deg);
    c.transform.position = pos;
    c.look_at(target, Vec3(0.0f, 1.0f, 0.0f));
    return c;
}

RaytracerConfig config(uint32_t w, uint32_t h, Color bg, Mode mode) {
    RaytracerConfig c;
    c.max_depth = 1;
    c.samples_per_pixel = 1;
    c.width = w;
    c.height = h;
    c.background_color = bg;
    c.mode = mode;
    c.jitter = Jitter::Center;
    return c;
}

std::shared_ptr<Material> lam(float r, float g, float b) { return std::make_shared<LambertianMaterial>(Color::rgb(r, g, b)); }

Lights showcase_lights() {
    return {std::make_shared<PointLight>(Vec3(-10.0f, 15.0f, 10.0f), Color::rgb(1.0f, 1.0f, 1.0f), 25.0f),
            std::make_shared<PointLight>(Vec3(10.0f, 10.0f, 15.0f), Color::rgb(0.6f, 0.7f, 1.0f), 15.0f),
            std::make_shared<PointLight>(Vec3(0.0f, 5.0f, -15.0f), Color::rgb(1.0f, 0.8f, 0.6f), 10.0f)};
}

}  // namespace

Scene basic_demo(uint32_t w, uint32_t h, Mode mode) {
    Scene s;
    auto ground = lam(0.5f, 0.5f, 0.5f), red = lam(0.7f, 0.3f, 0.3f), blue = lam(0.3f, 0.3f, 0.7f),
         green = lam(0.3f, 0.7f, 0.3f);
    s.objects = {std::make_shared<Sphere>(Vec3(0.0f, -1000.0f, 0.0f), 1000.0f, ground),
                 std::make_shared<Sphere>(Vec3(0.0f, 1.0f, 0.0f), 1.0f, red),
                 std::make_shared<Sphere>(Vec3(-2.5f, 1.0f, 0.0f), 1.0f, blue),
                 std::make_shared<Sphere>(Vec3(2.5f, 1.0f, 0.0f), 1.0f, green)};
    s.lights = {std::make_shared<PointLight>(Vec3(0.0f, 5.0f, 5.0f), Color::rgb(1.0f, 1.0f, 1.0f), 50.0f),
                std::make_shared<PointLight>(Vec3(-5.0f, 3.0f, -2.0f), Color::rgb(0.8f, 0.9f, 1.0f), 30.0f)};
    s.camera = camera(w, h, Vec3(6.0f, 4.0f, 6.0f), Vec3(0.0f, 1.0f, 0.0f), 45.0f);
    s.config = config(w, h, Color{0.5f, 0.7f, 1.0f, 1.0f}, mode);
    return s;
}

Scene advanced_demo(uint32_t w, uint32_t h, Mode mode) {
    Scene s;
    const float cols[5][3] = {{0.3f, 0.05f, 0.05f}, {0.05f, 0.1f, 0.3f}, {0.05f, 0.2f, 0.05f}, {0.2f, 0.05f, 0.2f},
                              {0.3f, 0.15f, 0.02f}};
    const float sph[5][4] = {{-6.0f, 1.0f, 0.0f, 1.2f}, {-3.0f, 1.0f, 0.0f, 0.8f}, {0.0f, 1.0f, 0.0f, 0.8f},
                             {3.0f, 1.0f, 0.0f, 0.9f}, {6.0f, 1.0f, 0.0f, 0.7f}};
    for (int i = 0; i < 5; ++i)
        s.objects.push_back(std::make_shared<Sphere>(Vec3(sph[i][0], sph[i][1], sph[i][2]), sph[i][3],
                                                     lam(cols[i][0], cols[i][1], cols[i][2])));
    s.objects.push_back(std::make_shared<Sphere>(Vec3(0.0f, -1000.0f, 0.0f), 1000.0f, lam(0.1f, 0.1f, 0.1f)));
    const float L[5][7] = {{0.0f, 8.0f, 0.0f, 0.2f, 0.1f, 0.4f, 15.0f}, {-8.0f, 3.0f, 4.0f, 0.4f, 0.1f, 0.05f, 12.0f},
                           {8.0f, 4.0f, -4.0f, 0.05f, 0.2f, 0.3f, 10.0f}, {-2.0f, 1.5f, -8.0f, 0.1f, 0.3f, 0.05f, 8.0f},
                           {4.0f, 6.0f, 6.0f, 0.3f, 0.05f, 0.3f, 6.0f}};
    for (const auto& l : L)
        s.lights.push_back(std::make_shared<PointLight>(Vec3(l[0], l[1], l[2]), Color::rgb(l[3], l[4], l[5]), l[6]));
    s.camera = camera(w, h, Vec3(12.0f, 6.0f, 0.0f), Vec3(0.0f, 1.0f, 0.0f), 60.0f);
    s.config = config(w, h, Color{0.05f, 0.05f, 0.1f, 1.0f}, mode);
    return s;
}

Scene sdf_showcase(uint32_t w, uint32_t h, Mode mode) {
    Scene s;
    auto sl = lam(0.2f, 0.6f, 0.9f), adv = lam(0.9f, 0.4f, 0.2f), cg = lam(0.6f, 0.9f, 0.3f), ground = lam(0.2f, 0.2f, 0.2f);
    const float y = 2.0f;
    using CO = CSGOperation;
    const std::pair<SDFRef, std::shared_ptr<Material>> sdfs[] = {
        {sdf_box(Vec3(-12.0f, y, -8.0f), Vec3(2.0f, 2.0f, 2.0f)), sl},
        {sdf_sphere(Vec3(-8.0f, y, -8.0f), 1.2), sl},
        {sdf_cylinder(Vec3(-4.0f, y, -8.0f), 1.0, 2.0), sl},
        {sdf_prism(Vec3(0.0f, y, -8.0f), Vec3(1.5f, 2.0f, 1.0f)), sl},
        {sdf_torus(Vec3(4.0f, y, -8.0f), 0.8, 0.3), sl},
        {sdf_tube(Vec3(8.0f, y, -8.0f), 1.0, 0.6, 1.5), sl},
        {sdf_ring(Vec3(12.0f, y, -8.0f), 0.8, 0.15), sl},
        {sdf_cone(Vec3(-8.0f, y, 0.0f), 1.2, 2.5), adv},
        {sdf_capsule(Vec3(-4.0f, y, 0.0f), 0.8, 2.0), adv},
        {sdf_ellipsoid(Vec3(0.0f, y, 0.0f), Vec3(1.2f, 0.8f, 1.0f)), adv},
        {csg(sdf_sphere(Vec3(4.0f, y, 0.0f), 0.8), sdf_sphere(Vec3(5.0f, y, 0.0f), 0.8), CO::Union), cg},
        {csg(sdf_sphere(Vec3(8.0f, y, 0.0f), 1.2), sdf_sphere(Vec3(8.5f, y, 0.0f), 0.6), CO::Difference), cg},
        {csg(sdf_sphere(Vec3(12.0f, y, 0.0f), 1.0), sdf_sphere(Vec3(12.5f, y, 0.0f), 1.0), CO::Intersection), cg},
        {csg(sdf_sphere(Vec3(4.0f, y, 4.0f), 0.8), sdf_sphere(Vec3(5.0f, y, 4.0f), 0.8), CO::SmoothUnion, 0.3f), cg},
        {csg(sdf_sphere(Vec3(8.0f, y, 4.0f), 1.2), sdf_sphere(Vec3(8.5f, y, 4.0f), 0.6), CO::SmoothDifference, 0.3f), cg},
        {csg(sdf_sphere(Vec3(12.0f, y, 4.0f), 1.0), sdf_sphere(Vec3(12.5f, y, 4.0f), 1.0), CO::SmoothIntersection, 0.3f), cg},
    };
    s.objects.push_back(std::make_shared<Sphere>(Vec3(0.0f, -1000.0f, 0.0f), 1000.0f, ground));
    for (const auto& p : sdfs) s.objects.push_back(std::make_shared<SDFObject>(p.first, p.second));
    s.lights = showcase_lights();
    s.camera = camera(w, h, Vec3(0.0f, 8.0f, 20.0f), Vec3(0.0f, 2.0f, 0.0f), 45.0f);
    s.config = config(w, h, Color{0.05f, 0.05f, 0.08f, 1.0f}, mode);
    return s;
}

Scene kitchen_sink(uint32_t w, uint32_t h, Mode mode) {
    Scene s;
    auto m0 = lam(0.6f, 0.3f, 0.2f), m1 = lam(0.2f, 0.5f, 0.7f), m2 = lam(0.4f, 0.6f, 0.3f);
    auto metal = std::make_shared<MetalMaterial>(Color::rgb(0.8f, 0.7f, 0.5f), 0.2f);
    auto glass = std::make_shared<DielectricMaterial>(1.5f);
    auto glow = std::make_shared<EmissiveMaterial>(Color::rgb(1.0f, 0.5f, 0.2f), 2.0f);
    auto cube = std::make_shared<Cube>(Vec3(1.5f, 1.0f, 0.0f), Vec3(1.0f, 1.5f, 0.8f), m0);
    Transform t;
    t.position = Vec3(0.1f, 0.0f, 0.2f);
    t.rotation = Quat{0.0f, 0.38268343f, 0.0f, 0.92387953f};
    t.scale = Vec3(1.0f, 1.2f, 1.0f);
    cube->set_transform(t);
    auto tri = std::make_shared<Triangle>(Vec3(-3.0f, 0.1f, -3.0f), Vec3(3.0f, 0.1f, -3.0f), Vec3(0.0f, 3.0f, -3.0f), m2);
    tri->set_normals(Vec3(0.0f, 0.0f, 2.0f), Vec3(0.1f, 0.0f, 1.0f), Vec3(-0.1f, 0.2f, 1.0f));
    // a small mesh: an octahedron with face normals
    std::vector<float> pos = {1.0f, 0.0f, 0.0f, -1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f,
                              0.0f, -1.0f, 0.0f, 0.0f, 0.0f, 1.0f, 0.0f, 0.0f, -1.0f};
    for (size_t i = 0; i < pos.size(); i += 3) {
        pos[i] = pos[i] * 0.6f - 1.5f;
        pos[i + 1] = pos[i + 1] * 0.6f + 1.0f;
        pos[i + 2] = pos[i + 2] * 0.6f + 1.8f;
    }
    std::vector<uint32_t> idx = {0, 2, 4, 2, 1, 4, 1, 3, 4, 3, 0, 4, 2, 0, 5, 1, 2, 5, 3, 1, 5, 0, 3, 5};
    auto oct = std::make_shared<Mesh>(pos, idx, std::vector<float>{}, metal);
    auto twisted = deformed(sdf_torus(Vec3(0.0f, 0.6f, 2.2f), 0.7, 0.25),
                            chain(twist(Vec3(0.0f, 1.0f, 0.0f), 1.5f, Vec3(0.0f, 0.6f, 2.2f)),
                                  noise(2.0f, 0.05f, Vec3(0.0f, 0.6f, 2.2f), 7u, 3u, 0.5f)));
    auto tapered = deformed(sdf_box(Vec3(-2.0f, 1.0f, -1.0f), Vec3(1.0f, 1.6f, 1.0f)),
                            chain(taper(Vec3(0.0f, 1.0f, 0.0f), 1.0f, 0.4f, 1.6f, Vec3(-2.0f, 1.0f, -1.0f)),
                                  wave(Vec3(1.0f, 0.0f, 0.0f), 0.1f, 5.0f, Vec3(0.0f, 1.0f, 0.0f), Vec3(-2.0f, 1.0f, -1.0f))));
    auto bent = deformed(sdf_capsule(Vec3(2.5f, 1.2f, 2.0f), 0.3, 1.2),
                         bend(Vec3(0.0f, 0.0f, 1.0f), Vec3(1.0f, 0.0f, 0.0f), 0.3f, Vec3(2.5f, 1.2f, 2.0f)));
    s.objects = {std::make_shared<Plane>(Vec3(0.0f, 0.0f, 0.0f), Vec3(0.0f, 1.0f, 0.0f), m2),
                 cube,
                 std::make_shared<Cylinder>(Vec3(-1.5f, 1.0f, 0.5f), 0.6f, 1.5f, m1),
                 std::make_shared<Cone>(Vec3(0.0f, 1.2f, -1.5f), 0.8f, 1.6f, m0),
                 std::make_shared<Capsule>(Vec3(0.0f, 1.0f, 1.8f), 0.4f, 1.0f, m1),
                 tri,
                 std::make_shared<Sphere>(Vec3(2.2f, 0.6f, -1.8f), 0.6f, glass),
                 std::make_shared<Sphere>(Vec3(-2.6f, 0.4f, 2.6f), 0.4f, glow),
                 oct,
                 std::make_shared<SDFObject>(twisted, m1),
                 std::make_shared<SDFObject>(tapered, m0, 160u, 0.5f, 2e-4f),
                 std::make_shared<SDFObject>(bent, metal)};
    s.lights = {std::make_shared<PointLight>(Vec3(3.0f, 6.0f, 4.0f), Color::rgb(1.0f, 1.0f, 1.0f), 2.0f),
                std::make_shared<DirectionalLight>(Vec3(-0.3f, -1.0f, -0.3f), Color{1.0f, 0.95f, 0.8f, 1.0f}, 0.6f),
                std::make_shared<SpotLight>(Vec3(0.0f, 5.0f, 0.0f), Vec3(0.0f, -1.0f, 0.0f), Color::rgb(1.0f, 0.8f, 0.6f),
                                            6.0f, 0.3f, 0.6f),
                AmbientLight::default_ambient(),
                PointLight::with_attenuation(Vec3(-4.0f, 3.0f, -1.0f), Color::rgb(0.5f, 0.6f, 1.0f), 2.5f, 50.0f, 0.05f, 0.01f)};
    s.camera = camera(w, h, Vec3(4.0f, 3.5f, 6.0f), Vec3(0.0f, 1.0f, 0.0f), 50.0f);
    s.config = config(w, h, Color{0.1f, 0.1f, 0.15f, 1.0f}, mode);
    return s;
}

Scene by_name(const std::string& name, uint32_t w, uint32_t h, Mode mode) {
    if (name == "basic-demo") return basic_demo(w, h, mode);
    if (name == "advanced-demo") return advanced_demo(w, h, mode);
    if (name == "sdf-showcase") return sdf_showcase(w, h, mode);
    if (name == "kitchen-sink") return kitchen_sink(w, h, mode);
    throw std::invalid_argument("unknown scene " + name);
}

}  // namespace rrte_examples
