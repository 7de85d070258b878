// scene.h — host-side scene graph, scene recipes, and compilation to the flat HBM layout (layout.h).
//
// SceneGraph mirrors the reference's object constructors one for one (sphere, moving_sphere, triangle, xy/xz/yz_rect,
// box, hittable_list, bvh_node, translate, rotate_y, constant_medium; lambertian, metal, dielectric, diffuse_light,
// isotropic; solid_color, checker_texture, noise_texture, image_texture, barycentric_image_texture).  Scene-build
// randomness replays the reference's global mt19937 (utils/tracer_utils.h:27-41) in call order, with g++'s
// right-to-left argument evaluation spelled out, so builtin scenes are bit-identical to the reference's
// (pinned by tests/test_scene.py against tests/golden/scenes.json).  The reference's bvh_node consumes one
// random_int(0,2) per node (primitives/bvh.cpp:9); bvh() replays exactly that many draws and leaves the real
// acceleration structure to the SAH builder (bvh.cpp) — closest-hit results do not depend on BVH topology.
#pragma once
#include <array>
#include <cstdint>
#include <random>
#include <string>
#include <vector>

#include "layout.h"

namespace art {

struct Vec3 {
    double e[3] = {0, 0, 0};
    Vec3() = default;
    Vec3(double a, double b, double c) : e{a, b, c} {}
    double operator[](int i) const { return e[i]; }
    double& operator[](int i) { return e[i]; }
};
// core/vec3.h arithmetic, as written there.
inline Vec3 operator+(const Vec3& u, const Vec3& v) { return {u[0] + v[0], u[1] + v[1], u[2] + v[2]}; }
inline Vec3 operator-(const Vec3& u, const Vec3& v) { return {u[0] - v[0], u[1] - v[1], u[2] - v[2]}; }
inline Vec3 operator*(const Vec3& u, const Vec3& v) { return {u[0] * v[0], u[1] * v[1], u[2] * v[2]}; }
inline Vec3 operator*(double t, const Vec3& v) { return {t * v[0], t * v[1], t * v[2]}; }
inline Vec3 operator/(const Vec3& v, double t) { return (1 / t) * v; }
inline double dot(const Vec3& u, const Vec3& v) { return u[0] * v[0] + u[1] * v[1] + u[2] * v[2]; }
inline Vec3 cross(const Vec3& u, const Vec3& v) {
    return {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
}
Vec3 unit_vector(const Vec3& v);

// The reference's scene-build RNG: std::mt19937 (seed 5489) + libstdc++ generate_canonical<double,53>.
class SceneRng {
public:
    explicit SceneRng(uint32_t seed = 5489u) : mt_(seed) {}
    double d();                                          // random_double()
    double d(double lo, double hi) { return lo + (hi - lo) * d(); }
    int i(int lo, int hi) { return static_cast<int>(d(lo, hi + 1)); }
    Vec3 vec01();                                        // vec3::random(): z, y, x drawn in that order (g++)
    Vec3 vec(double lo, double hi);                      // vec3::random(min,max)
    void skip(uint64_t draws) { for (uint64_t k = 0; k < draws; ++k) d(); }
private:
    std::mt19937 mt_;
};

struct AABBd {
    Vec3 mn, mx;
};

struct Texture {
    TexType type = TEX_SOLID;
    Vec3 c;
    int even = -1, odd = -1, perlin = -1, image = -1;
    double scale = 0;
    double uv[6] = {0, 0, 0, 0, 0, 0};
};
struct Material {
    MatType type = MAT_LAMBERTIAN;
    int tex = -1;
    Vec3 albedo;
    double fuzz = 0, ir = 0;
};
struct Perlin {
    std::array<Vec3, 256> ranvec;
    std::array<std::array<int, 256>, 3> perm;
};
struct Image {
    int w = 0, h = 0, bpp = 0;
    std::vector<uint8_t> data;
};

enum NodeType { N_SPHERE, N_MOVING_SPHERE, N_TRIANGLE, N_RECT, N_BOX, N_LIST, N_BVH, N_TRANSLATE, N_ROTATE_Y, N_MEDIUM };
struct Node {
    NodeType type = N_SPHERE;
    int mat = -1;
    Vec3 a, b, c;             // sphere: a=center; moving: a=c0, b=c1; tri: a,b,c; box: a=min, b=max; translate: a=offset
    double r = 0, t0 = 0, t1 = 0;
    int axis = 0;             // rect: 0 xy, 1 xz, 2 yz
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0;
    double sin_t = 0, cos_t = 0;
    bool hasbox = true;
    AABBd bbox;               // rotate_y / bvh
    int child = -1;           // translate / rotate_y / medium boundary
    double neg_inv_density = 0;
    std::vector<int> items;   // list / bvh
};

inline Node make_node(NodeType t) {
    Node n;
    n.type = t;
    return n;
}

struct SceneGraph {
    std::vector<Texture> textures;
    std::vector<Material> materials;
    std::vector<Perlin> perlins;
    std::vector<Image> images;
    std::vector<Node> nodes;
    std::vector<int> world;
    Vec3 lookfrom, lookat, background;
    double vfov = 40.0, aperture = 0.0;
    SceneRng rng;

    // textures (rendering/texture.h)
    int solid(Vec3 c);
    int checker(int even, int odd);
    int noise(double scale);                       // builds a perlin table from rng (perlin.h:10-19)
    int image(Image img);
    int image_file(const std::string& path);       // our raw texel asset (w,h,bpp header + bytes)
    int bary_image(double ua, double va, double ub, double vb, double uc, double vc, int image_tex);
    // materials (rendering/material.h)
    int lambertian(int tex);
    int lambertian_color(Vec3 c) { return lambertian(solid(c)); }
    int metal(Vec3 albedo, double fuzz);
    int dielectric(double ir);
    int diffuse_light(int tex);
    int isotropic(int tex);
    // hittables
    int sphere(Vec3 c, double r, int mat);
    int moving_sphere(Vec3 c0, Vec3 c1, double t0, double t1, double r, int mat);
    int triangle(Vec3 p1, Vec3 p2, Vec3 p3, int mat);
    int rect(int axis, double a0, double a1, double b0, double b1, double k, int mat);
    int box(Vec3 p0, Vec3 p1, int mat);
    int list(std::vector<int> items);
    int bvh(std::vector<int> items);               // consumes the reference's BVH-build draws
    int translate(int child, Vec3 offset);
    int rotate_y(int child, double degrees);
    int constant_medium(int boundary, double density, int phase_tex);

    bool bounding_box(int node, double time0, double time1, AABBd& out) const;
};

// scene_manager::build equivalents.  Names: "1".."9" or the scene_alias names, "c1" (SURVEY Q7), "cow", "dino"
// (SURVEY Q8).  asset_dir holds cow.tris / dino.tris / earthmap.rgb.  Throws std::runtime_error.
void build_builtin_scene(SceneGraph& g, const std::string& name, const std::string& asset_dir);

// Canonical JSON dump, same schema as oracle/ref_harness `dump` (BVH items in construction order).
std::string dump_scene(const SceneGraph& g);

// Reference-BVH node count for n items (bvh.cpp:3-42): the number of random_int draws bvh() replays.
uint64_t reference_bvh_nodes(uint64_t n);

// ---------------------------------------------------------------------------------------------- compiled scene
struct FlatScene {
    std::vector<SphereRec<double>> spheres;
    std::vector<TriRec<double>> tris;
    std::vector<RectRec<double>> rects;
    std::vector<BoxRec<double>> boxes;
    std::vector<uint32_t> primrefs;      // leaf ranges of all BVHs
    std::vector<BvhNode> nodes;
    std::vector<ObjRec<double>> objs;
    std::vector<int32_t> world;          // top-level objects, in hittable_list order
    std::vector<MatRec<double>> mats;
    std::vector<TexRec<double>> texs;
    std::vector<PerlinRec<double>> perlins;
    std::vector<ImageRec> images;
    std::vector<uint8_t> texels;
    double background[3] = {0, 0, 0};
    bool has_media = false;
    uint32_t features = 0;               // layout.h Feature bits present in the scene
    int max_bvh_depth = 0;               // 4-wide tree depth
    int max_stack = 0;                   // worst-case traversal stack entries (sizes the LDS stack)
};
FlatScene compile_scene(const SceneGraph& g);

// camera.h:8-36 in f64 (the reference's own arithmetic).
CameraRec<double> make_camera(const double lookfrom[3], const double lookat[3], const double vup[3], double vfov, double aspect,
                              double aperture, double focus_dist, double time0, double time1);

}  // namespace art
