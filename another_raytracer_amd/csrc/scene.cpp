// scene.cpp — scene graph builder, builtin scene recipes, canonical dump and compilation (see scene.h).
#include "scene.h"
#include "imagedec.h"
#include "options.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <stdexcept>

#include <zlib.h>

#include "bvh.h"
#include "objmesh.h"

namespace art {

namespace {
const double kInf = std::numeric_limits<double>::infinity();
const double kPi = 3.1415926535897932385;  // tracer_utils.h:11
}  // namespace

Vec3 unit_vector(const Vec3& v) { return v / std::sqrt(dot(v, v)); }

// libstdc++ generate_canonical<double, 53> over mt19937: sum = x0 + x1*2^32 (one rounding), / 2^64, clamp < 1.
double SceneRng::d() {
    double sum = 0.0, tmp = 1.0;
    sum += static_cast<double>(mt_()) * tmp;
    tmp *= 4294967296.0;
    sum += static_cast<double>(mt_()) * tmp;
    tmp *= 4294967296.0;
    double r = sum / tmp;
    if (r >= 1.0) r = std::nextafter(1.0, 0.0);
    return r;
}
Vec3 SceneRng::vec01() {
    Vec3 v;
    v[2] = d();
    v[1] = d();
    v[0] = d();
    return v;
}
Vec3 SceneRng::vec(double lo, double hi) {
    Vec3 v;
    v[2] = d(lo, hi);
    v[1] = d(lo, hi);
    v[0] = d(lo, hi);
    return v;
}

// ------------------------------------------------------------------------------------------------ builder
int SceneGraph::solid(Vec3 c) {
    Texture t;
    t.type = TEX_SOLID;
    t.c = c;
    textures.push_back(t);
    return static_cast<int>(textures.size()) - 1;
}
int SceneGraph::checker(int even, int odd) {
    Texture t;
    t.type = TEX_CHECKER;
    t.even = even;
    t.odd = odd;
    textures.push_back(t);
    return static_cast<int>(textures.size()) - 1;
}
int SceneGraph::noise(double scale) {  // texture.h:52-65 + perlin.h:10-19, :69-81 (draws from the scene RNG)
    Perlin p;
    for (auto& v : p.ranvec) v = unit_vector(rng.vec(-1, 1));
    for (auto& perm : p.perm) {
        for (int i = 0; i < 256; i++) perm[i] = i;
        for (int i = 255; i > 0; i--) {
            int target = rng.i(0, i);
            std::swap(perm[i], perm[target]);
        }
    }
    perlins.push_back(p);
    Texture t;
    t.type = TEX_NOISE;
    t.scale = scale;
    t.perlin = static_cast<int>(perlins.size()) - 1;
    textures.push_back(t);
    return static_cast<int>(textures.size()) - 1;
}
int SceneGraph::image(Image img) {
    images.push_back(std::move(img));
    Texture t;
    t.type = TEX_IMAGE;
    t.image = static_cast<int>(images.size()) - 1;
    textures.push_back(t);
    return static_cast<int>(textures.size()) - 1;
}
int SceneGraph::image_file(const std::string& path) {
    // image_texture(filename) (texture.h:70-72 -> imageio::load_image = stbi_load(path, .., 0)): JPEG / PNG through
    // imagedec.cpp, bytes as stb_image returns them
    const size_t dot = path.find_last_of('.');
    std::string ext = dot == std::string::npos ? std::string() : path.substr(dot);
    for (char& ch : ext) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
    if (ext == ".jpg" || ext == ".jpeg" || ext == ".png") {
        DecodedImage d = load_image_file(path);
        Image img;
        img.w = d.w;
        img.h = d.h;
        img.bpp = d.channels;
        img.data = std::move(d.data);
        return image(std::move(img));
    }
    // otherwise a raw texel file (int32 w, h, bpp + bytes), optionally gzip-compressed; gzread passes plain files through
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open texture asset " + path);
    auto read = [&](void* dst, size_t n) {
        return gzread(f, dst, static_cast<unsigned>(n)) == static_cast<int>(n);
    };
    int32_t hdr[3];
    Image img;
    bool ok = read(hdr, sizeof hdr);
    img.w = hdr[0];
    img.h = hdr[1];
    img.bpp = hdr[2];
    if (!ok || img.w <= 0 || img.h <= 0 || img.bpp < 3 || img.w > (1 << 16) || img.h > (1 << 16) || img.bpp > 4) {
        gzclose(f);
        throw std::runtime_error("bad texture asset " + path);
    }
    img.data.resize(static_cast<size_t>(img.w) * img.h * img.bpp);
    ok = read(img.data.data(), img.data.size());
    gzclose(f);
    if (!ok) throw std::runtime_error("truncated texture asset " + path);
    return image(std::move(img));
}
int SceneGraph::bary_image(double ua, double va, double ub, double vb, double uc, double vc, int image_tex) {
    Texture t;
    t.type = TEX_BARY_IMAGE;
    t.image = textures.at(image_tex).image;
    double uv[6] = {ua, va, ub, vb, uc, vc};
    std::memcpy(t.uv, uv, sizeof uv);
    textures.push_back(t);
    return static_cast<int>(textures.size()) - 1;
}
int SceneGraph::lambertian(int tex) {
    Material m;
    m.type = MAT_LAMBERTIAN;
    m.tex = tex;
    materials.push_back(m);
    return static_cast<int>(materials.size()) - 1;
}
int SceneGraph::metal(Vec3 albedo, double fuzz) {
    Material m;
    m.type = MAT_METAL;
    m.albedo = albedo;
    m.fuzz = fuzz < 1. ? fuzz : 1.;  // material.h:47
    materials.push_back(m);
    return static_cast<int>(materials.size()) - 1;
}
int SceneGraph::dielectric(double ir) {
    Material m;
    m.type = MAT_DIELECTRIC;
    m.ir = ir;
    materials.push_back(m);
    return static_cast<int>(materials.size()) - 1;
}
int SceneGraph::diffuse_light(int tex) {
    Material m;
    m.type = MAT_LIGHT;
    m.tex = tex;
    materials.push_back(m);
    return static_cast<int>(materials.size()) - 1;
}
int SceneGraph::isotropic(int tex) {
    Material m;
    m.type = MAT_ISOTROPIC;
    m.tex = tex;
    materials.push_back(m);
    return static_cast<int>(materials.size()) - 1;
}
int SceneGraph::sphere(Vec3 c, double r, int mat) {
    Node n = make_node(N_SPHERE);
    n.a = c;
    n.r = r;
    n.mat = mat;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::moving_sphere(Vec3 c0, Vec3 c1, double t0, double t1, double r, int mat) {
    Node n = make_node(N_MOVING_SPHERE);
    n.a = c0;
    n.b = c1;
    n.t0 = t0;
    n.t1 = t1;
    n.r = r;
    n.mat = mat;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::triangle(Vec3 p1, Vec3 p2, Vec3 p3, int mat) {
    Node n = make_node(N_TRIANGLE);
    n.a = p1;
    n.b = p2;
    n.c = p3;
    n.mat = mat;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::rect(int axis, double a0, double a1, double b0, double b1, double k, int mat) {
    Node n = make_node(N_RECT);
    n.axis = axis;
    n.a0 = a0;
    n.a1 = a1;
    n.b0 = b0;
    n.b1 = b1;
    n.k = k;
    n.mat = mat;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::box(Vec3 p0, Vec3 p1, int mat) {
    Node n = make_node(N_BOX);
    n.a = p0;
    n.b = p1;
    n.mat = mat;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::list(std::vector<int> items) {
    Node n = make_node(N_LIST);
    n.items = std::move(items);
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
uint64_t reference_bvh_nodes(uint64_t n) {
    if (n <= 2) return 1;
    return 1 + reference_bvh_nodes(n / 2) + reference_bvh_nodes(n - n / 2);
}
int SceneGraph::bvh(std::vector<int> items) {
    if (items.empty()) throw std::runtime_error("bvh over an empty list");
    rng.skip(reference_bvh_nodes(items.size()));  // bvh.cpp:9: random_int(0,2) in every node constructor
    Node n = make_node(N_BVH);
    n.items = std::move(items);
    n.t0 = 0;
    n.t1 = 1;
    AABBd acc, tmp;
    bool first = true;
    for (int it : n.items) {
        if (!bounding_box(it, 0, 1, tmp)) throw std::runtime_error("bvh item without a bounding box");
        if (first) acc = tmp;
        else {
            for (int a = 0; a < 3; ++a) {
                acc.mn[a] = std::min(acc.mn[a], tmp.mn[a]);
                acc.mx[a] = std::max(acc.mx[a], tmp.mx[a]);
            }
        }
        first = false;
    }
    n.bbox = acc;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::translate(int child, Vec3 offset) {
    Node n = make_node(N_TRANSLATE);
    n.child = child;
    n.a = offset;
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::rotate_y(int child, double degrees) {  // hittable.cpp:25-55
    Node n = make_node(N_ROTATE_Y);
    n.child = child;
    double radians = degrees * kPi / 180.0;
    n.sin_t = std::sin(radians);
    n.cos_t = std::cos(radians);
    AABBd bbox;
    n.hasbox = bounding_box(child, 0, 1, bbox);
    Vec3 mn(kInf, kInf, kInf), mx(-kInf, -kInf, -kInf);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                double x = i * bbox.mx[0] + (1 - i) * bbox.mn[0];
                double y = j * bbox.mx[1] + (1 - j) * bbox.mn[1];
                double z = k * bbox.mx[2] + (1 - k) * bbox.mn[2];
                double newx = n.cos_t * x + n.sin_t * z;
                double newz = -n.sin_t * x + n.cos_t * z;
                Vec3 tester(newx, y, newz);
                for (int c = 0; c < 3; c++) {
                    mn[c] = std::fmin(mn[c], tester[c]);
                    mx[c] = std::fmax(mx[c], tester[c]);
                }
            }
    n.bbox = AABBd{mn, mx};
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}
int SceneGraph::constant_medium(int boundary, double density, int phase_tex) {  // constant_medium.h:12-22
    Node n = make_node(N_MEDIUM);
    n.child = boundary;
    n.neg_inv_density = -1 / density;
    n.mat = isotropic(phase_tex);
    nodes.push_back(n);
    return static_cast<int>(nodes.size()) - 1;
}

bool SceneGraph::bounding_box(int idx, double time0, double time1, AABBd& out) const {
    const Node& n = nodes.at(idx);
    auto sphere_box = [](const Vec3& c, double r) {
        Vec3 rr(r, r, r);
        return AABBd{c - rr, c + rr};
    };
    switch (n.type) {
        case N_SPHERE: out = sphere_box(n.a, n.r); return true;
        case N_MOVING_SPHERE: {  // moving_sphere.h:61-70
            auto center = [&](double t) { return n.a + ((t - n.t0) / (n.t1 - n.t0)) * (n.b - n.a); };
            AABBd b0 = sphere_box(center(time0), n.r), b1 = sphere_box(center(time1), n.r);
            for (int a = 0; a < 3; ++a) {
                out.mn[a] = std::min(b0.mn[a], b1.mn[a]);
                out.mx[a] = std::max(b0.mx[a], b1.mx[a]);
            }
            return true;
        }
        case N_TRIANGLE:
            for (int a = 0; a < 3; ++a) {
                out.mn[a] = std::min(n.a[a], std::min(n.b[a], n.c[a]));
                out.mx[a] = std::max(n.a[a], std::max(n.b[a], n.c[a]));
            }
            return true;
        case N_RECT: {  // aarect.h:16-21, :37-42, :58-63
            int ka = n.axis == 0 ? 2 : n.axis == 1 ? 1 : 0;
            int ia = n.axis == 2 ? 1 : 0;
            int ib = n.axis == 0 ? 1 : 2;
            out.mn[ia] = n.a0;
            out.mx[ia] = n.a1;
            out.mn[ib] = n.b0;
            out.mx[ib] = n.b1;
            out.mn[ka] = n.k - 0.0001;
            out.mx[ka] = n.k + 0.0001;
            return true;
        }
        case N_BOX: out = AABBd{n.a, n.b}; return true;
        case N_LIST: {
            if (n.items.empty()) return false;
            AABBd tmp;
            bool first = true;
            for (int it : n.items) {
                if (!bounding_box(it, time0, time1, tmp)) return false;
                if (first) out = tmp;
                else
                    for (int a = 0; a < 3; ++a) {
                        out.mn[a] = std::min(out.mn[a], tmp.mn[a]);
                        out.mx[a] = std::max(out.mx[a], tmp.mx[a]);
                    }
                first = false;
            }
            return true;
        }
        case N_BVH: out = n.bbox; return true;
        case N_TRANSLATE:
            if (!bounding_box(n.child, time0, time1, out)) return false;
            out = AABBd{out.mn + n.a, out.mx + n.a};
            return true;
        case N_ROTATE_Y: out = n.bbox; return n.hasbox;
        case N_MEDIUM: return bounding_box(n.child, time0, time1, out);
    }
    return false;
}

// ------------------------------------------------------------------------------------------------ recipes
namespace {

void random_scene(SceneGraph& g) {  // scene_manager.cpp:13-64
    std::vector<int> objects;
    int ground = g.lambertian(g.checker(g.solid(Vec3(0.2, 0.3, 0.1)), g.solid(Vec3(0.9, 0.9, 0.9))));
    objects.push_back(g.sphere(Vec3(0, -1000, 0), 1000, ground));
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            double choose_mat = g.rng.d();
            double cz = b + 0.9 * g.rng.d();  // point3(a + 0.9*rd(), 0.2, b + 0.9*rd()): g++ draws z first
            double cx = a + 0.9 * g.rng.d();
            Vec3 center(cx, 0.2, cz);
            Vec3 dc = center - Vec3(4, 0.2, 0);
            if (std::sqrt(dot(dc, dc)) > 0.9) {
                if (choose_mat < 0.8) {
                    Vec3 rhs = g.rng.vec01();  // color::random() * color::random(): right operand drawn first
                    Vec3 lhs = g.rng.vec01();
                    int m = g.lambertian_color(lhs * rhs);
                    objects.push_back(g.sphere(center, 0.2, m));
                    Vec3 center2 = center + Vec3(0, g.rng.d(0, .5), 0);
                    objects.push_back(g.moving_sphere(center, center2, 0.0, 1.0, 0.2, m));
                } else if (choose_mat < 0.95) {
                    Vec3 albedo = g.rng.vec(0.5, 1);
                    double fuzz = g.rng.d(0, 0.5);
                    objects.push_back(g.sphere(center, 0.2, g.metal(albedo, fuzz)));
                } else {
                    objects.push_back(g.sphere(center, 0.2, g.dielectric(1.5)));
                }
            }
        }
    }
    objects.push_back(g.sphere(Vec3(0, 1, 0), 1.0, g.dielectric(1.5)));
    objects.push_back(g.sphere(Vec3(-4, 1, 0), 1.0, g.lambertian_color(Vec3(0.4, 0.2, 0.1))));
    objects.push_back(g.sphere(Vec3(4, 1, 0), 1.0, g.metal(Vec3(0.7, 0.6, 0.5), 0.0)));
    g.world.push_back(g.bvh(objects));
}

void cornell(SceneGraph& g, bool smoke) {  // scene_manager.cpp:106-169
    int red = g.lambertian_color(Vec3(.65, .05, .05));
    int white = g.lambertian_color(Vec3(.73, .73, .73));
    int green = g.lambertian_color(Vec3(.12, .45, .15));
    double lv = smoke ? 7 : 15;
    int light = g.diffuse_light(g.solid(Vec3(lv, lv, lv)));
    g.world.push_back(g.rect(2, 0, 555, 0, 555, 555, green));
    g.world.push_back(g.rect(2, 0, 555, 0, 555, 0, red));
    if (!smoke) {
        g.world.push_back(g.rect(1, 213, 343, 227, 332, 554, light));
        g.world.push_back(g.rect(1, 0, 555, 0, 555, 0, white));
        g.world.push_back(g.rect(1, 0, 555, 0, 555, 555, white));
    } else {
        g.world.push_back(g.rect(1, 113, 443, 127, 432, 554, light));
        g.world.push_back(g.rect(1, 0, 555, 0, 555, 555, white));
        g.world.push_back(g.rect(1, 0, 555, 0, 555, 0, white));
    }
    g.world.push_back(g.rect(0, 0, 555, 0, 555, 555, white));
    int box1 = g.box(Vec3(0, 0, 0), Vec3(165, 330, 165), white);
    box1 = g.rotate_y(box1, 15);
    box1 = g.translate(box1, Vec3(265, 0, 295));
    int box2 = g.box(Vec3(0, 0, 0), Vec3(165, 165, 165), white);
    box2 = g.rotate_y(box2, -18);
    box2 = g.translate(box2, Vec3(130, 0, 65));
    if (!smoke) {
        g.world.push_back(box1);
        g.world.push_back(box2);
    } else {
        g.world.push_back(g.constant_medium(box1, 0.01, g.solid(Vec3(0, 0, 0))));
        g.world.push_back(g.constant_medium(box2, 0.01, g.solid(Vec3(1, 1, 1))));
    }
}

void final_scene(SceneGraph& g, const std::string& assets) {  // scene_manager.cpp:171-234
    std::vector<int> boxes1;
    int ground = g.lambertian_color(Vec3(0.48, 0.83, 0.53));
    const int boxes_per_side = 20;
    for (int i = 0; i < boxes_per_side; i++) {
        for (int j = 0; j < boxes_per_side; j++) {
            double w = 100.0;
            double x0 = -1000.0 + i * w;
            double z0 = -1000.0 + j * w;
            double y0 = 0.0;
            double x1 = x0 + w;
            double y1 = g.rng.d(1, 101);
            double z1 = z0 + w;
            boxes1.push_back(g.box(Vec3(x0, y0, z0), Vec3(x1, y1, z1), ground));
        }
    }
    g.world.push_back(g.bvh(boxes1));
    g.world.push_back(g.rect(1, 123, 423, 147, 412, 554, g.diffuse_light(g.solid(Vec3(7, 7, 7)))));
    Vec3 center1(400, 400, 200);
    Vec3 center2 = center1 + Vec3(30, 0, 0);
    g.world.push_back(g.moving_sphere(center1, center2, 0, 1, 50, g.lambertian_color(Vec3(0.7, 0.3, 0.1))));
    g.world.push_back(g.sphere(Vec3(260, 150, 45), 50, g.dielectric(1.5)));
    g.world.push_back(g.sphere(Vec3(0, 150, 145), 50, g.metal(Vec3(0.8, 0.8, 0.9), 1.0)));
    int boundary = g.sphere(Vec3(360, 150, 145), 70, g.dielectric(1.5));
    g.world.push_back(boundary);
    g.world.push_back(g.constant_medium(boundary, 0.2, g.solid(Vec3(0.2, 0.4, 0.9))));
    boundary = g.sphere(Vec3(0, 0, 0), 5000, g.dielectric(1.5));
    g.world.push_back(g.constant_medium(boundary, .0001, g.solid(Vec3(1, 1, 1))));
    g.world.push_back(g.sphere(Vec3(400, 200, 400), 100, g.lambertian(g.image_file(assets + "/earthmap.jpg"))));
    int pertext = g.noise(0.1);
    g.world.push_back(g.sphere(Vec3(220, 280, 300), 80, g.lambertian(pertext)));
    std::vector<int> boxes2;
    int white = g.lambertian_color(Vec3(.73, .73, .73));
    for (int j = 0; j < 1000; j++) boxes2.push_back(g.sphere(g.rng.vec(0, 165), 10, white));
    g.world.push_back(g.translate(g.rotate_y(g.bvh(boxes2), 15), Vec3(-100, 270, 395)));
}

void mesh_scene(SceneGraph& g, const std::string& obj_path) {  // scene_manager.cpp:236-258 (SURVEY Q8 for cow/dino)
    const std::vector<int> tris = build_mesh(g, load_obj(obj_path));  // mesh::parse + mesh::build (mesh.h:31-145)
    g.world.push_back(g.bvh(tris));
    g.world.push_back(g.rect(1, 123, 423, 147, 412, 554, g.diffuse_light(g.solid(Vec3(7, 7, 7)))));
    int boundary = g.sphere(Vec3(0, 0, 0), 5000, g.dielectric(1.5));
    g.world.push_back(g.constant_medium(boundary, .0001, g.solid(Vec3(1, 1, 1))));
}

}  // namespace

void build_builtin_scene(SceneGraph& g, const std::string& name, const std::string& assets) {
    const Vec3 sky(0.70, 0.80, 1.00);
    auto cam = [&](Vec3 from, Vec3 at, double vfov, double aperture, Vec3 bg) {
        g.lookfrom = from;
        g.lookat = at;
        g.vfov = vfov;
        g.aperture = aperture;
        g.background = bg;
    };
    if (name == "c1") {  // build-defined 3-sphere lambertian scene
        g.world.push_back(g.sphere(Vec3(0, -100.5, -1), 100, g.lambertian_color(Vec3(0.8, 0.8, 0.0))));
        g.world.push_back(g.sphere(Vec3(0, 0, -1), 0.5, g.lambertian_color(Vec3(0.7, 0.3, 0.3))));
        g.world.push_back(g.sphere(Vec3(-1, 0, -1), 0.5, g.lambertian_color(Vec3(0.1, 0.2, 0.5))));
        cam(Vec3(0, 0, 0), Vec3(0, 0, -1), 90.0, 0.0, sky);
    } else if (name == "1" || name == "random") {
        random_scene(g);
        cam(Vec3(13, 2, 3), Vec3(0, 0, 0), 20.0, 0.1, sky);
    } else if (name == "2" || name == "two_spheres") {
        int checker = g.checker(g.solid(Vec3(0.2, 0.3, 0.1)), g.solid(Vec3(0.9, 0.9, 0.9)));
        g.world.push_back(g.sphere(Vec3(0, -10, 0), 10, g.lambertian(checker)));
        g.world.push_back(g.sphere(Vec3(0, 10, 0), 10, g.lambertian(checker)));
        cam(Vec3(13, 2, 3), Vec3(0, 0, 0), 20.0, 0.0, sky);
    } else if (name == "3" || name == "two_perlin_spheres") {
        int pertext = g.noise(4);
        g.world.push_back(g.sphere(Vec3(0, -1000, 0), 1000, g.lambertian(pertext)));
        g.world.push_back(g.sphere(Vec3(0, 2, 0), 2, g.lambertian(pertext)));
        cam(Vec3(13, 2, 3), Vec3(0, 0, 0), 20.0, 0.0, sky);
    } else if (name == "4" || name == "earth") {
        g.world.push_back(g.sphere(Vec3(0, 0, 0), 2, g.lambertian(g.image_file(assets + "/earthmap.jpg"))));
        cam(Vec3(13, 2, 3), Vec3(0, 0, 0), 20.0, 0.0, sky);
    } else if (name == "5" || name == "simple_light") {
        int pertext = g.noise(4);
        g.world.push_back(g.sphere(Vec3(0, -1000, 0), 1000, g.lambertian(pertext)));
        g.world.push_back(g.sphere(Vec3(0, 2, 0), 2, g.lambertian(pertext)));
        g.world.push_back(g.rect(0, 3, 5, 1, 3, -2, g.diffuse_light(g.solid(Vec3(4, 4, 4)))));
        cam(Vec3(26, 3, 6), Vec3(0, 2, 0), 20.0, 0.0, Vec3(0, 0, 0));
    } else if (name == "6" || name == "cornell_box") {
        cornell(g, false);
        cam(Vec3(278, 278, -800), Vec3(278, 278, 0), 40.0, 0.0, Vec3(0, 0, 0));
    } else if (name == "7" || name == "cornell_smoke") {
        cornell(g, true);
        cam(Vec3(278, 278, -800), Vec3(278, 278, 0), 40.0, 0.0, Vec3(0, 0, 0));
    } else if (name == "8" || name == "final") {
        final_scene(g, assets);
        cam(Vec3(478, 278, -600), Vec3(278, 278, 0), 40.0, 0.0, Vec3(0, 0, 0));
    } else if (name == "cow") {
        mesh_scene(g, assets + "/models/cow.obj");
        cam(Vec3(4, 2, 6), Vec3(2, 0, 0), 75.0, 0.0, sky);
    } else if (name == "dino") {
        mesh_scene(g, assets + "/models/dino.obj");
        cam(Vec3(0, 15, 25), Vec3(0, 10, 0), 75.0, 0.0, sky);
    } else if (name == "9" || name == "mesh") {  // ressources::capsule_obj_path, the stock _mesh_scene
        mesh_scene(g, assets + "/models/capsule/capsule.obj");
        cam(Vec3(2, 2, 1), Vec3(0, 0, 0), 75.0, 0.0, sky);
    } else {
        throw std::runtime_error("unkwnown scene requested: " + name);  // scene_manager.cpp:351 wording
    }
}

// ------------------------------------------------------------------------------------------------ dump
namespace {
std::string D(double x) {
    char b[64];
    if (std::isinf(x)) return x > 0 ? "\"inf\"" : "\"-inf\"";
    std::snprintf(b, sizeof b, "%.17g", x);
    return b;
}
std::string V(const Vec3& v) { return "[" + D(v[0]) + "," + D(v[1]) + "," + D(v[2]) + "]"; }
uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h;
}

struct Dumper {
    const SceneGraph& g;
    mutable std::vector<std::string> image_dump;  // per image: its dump (the texel hash is computed once)
    std::string tex(int ti) const { return tex_rec(g.textures[ti]); }
    std::string tex_rec(const Texture& t) const {
        switch (t.type) {
            case TEX_SOLID: return "{\"type\":\"solid\",\"c\":" + V(t.c) + "}";
            case TEX_CHECKER: return "{\"type\":\"checker\",\"even\":" + tex(t.even) + ",\"odd\":" + tex(t.odd) + "}";
            case TEX_NOISE: {
                const Perlin& p = g.perlins[t.perlin];
                std::string r = "{\"type\":\"noise\",\"scale\":" + D(t.scale) + ",\"ranvec\":[";
                for (int i = 0; i < 256; ++i) r += (i ? "," : "") + V(p.ranvec[i]);
                auto perm = [](const std::array<int, 256>& q) {
                    std::string x = "[";
                    for (int i = 0; i < 256; ++i) x += (i ? "," : "") + std::to_string(q[i]);
                    return x + "]";
                };
                return r + "],\"perm_x\":" + perm(p.perm[0]) + ",\"perm_y\":" + perm(p.perm[1]) + ",\"perm_z\":" + perm(p.perm[2]) + "}";
            }
            case TEX_IMAGE: {
                if (image_dump.size() < g.images.size()) image_dump.resize(g.images.size());
                std::string& s = image_dump[static_cast<size_t>(t.image)];
                if (s.empty()) {
                    const Image& im = g.images[t.image];
                    char h[32];
                    std::snprintf(h, sizeof h, "%016llx", static_cast<unsigned long long>(fnv1a(im.data.data(), im.data.size())));
                    s = "{\"type\":\"image\",\"w\":" + std::to_string(im.w) + ",\"h\":" + std::to_string(im.h) + ",\"bpp\":" +
                        std::to_string(im.bpp) + ",\"fnv1a\":\"" + h + "\"}";
                }
                return s;
            }
            case TEX_BARY_IMAGE: {  // oracle/ref_harness dump_texture schema
                Texture img;
                img.type = TEX_IMAGE;
                img.image = t.image;
                return "{\"type\":\"bary_image\",\"a\":[" + D(t.uv[0]) + "," + D(t.uv[1]) + "],\"b\":[" + D(t.uv[2]) + "," + D(t.uv[3]) +
                       "],\"c\":[" + D(t.uv[4]) + "," + D(t.uv[5]) + "],\"tex\":" + tex_rec(img) + "}";
            }
        }
        return "{}";
    }
    std::string mat(int mi) const {
        const Material& m = g.materials[mi];
        switch (m.type) {
            case MAT_LAMBERTIAN: return "{\"type\":\"lambertian\",\"tex\":" + tex(m.tex) + "}";
            case MAT_METAL: return "{\"type\":\"metal\",\"albedo\":" + V(m.albedo) + ",\"fuzz\":" + D(m.fuzz) + "}";
            case MAT_DIELECTRIC: return "{\"type\":\"dielectric\",\"ir\":" + D(m.ir) + "}";
            case MAT_LIGHT: return "{\"type\":\"diffuse_light\",\"tex\":" + tex(m.tex) + "}";
            case MAT_ISOTROPIC: return "{\"type\":\"isotropic\",\"tex\":" + tex(m.tex) + "}";
        }
        return "{}";
    }
    std::string rect(const Node& n) const {
        static const char* names[3] = {"xy_rect", "xz_rect", "yz_rect"};
        return std::string("{\"type\":\"") + names[n.axis] + "\",\"a0\":" + D(n.a0) + ",\"a1\":" + D(n.a1) + ",\"b0\":" + D(n.b0) +
               ",\"b1\":" + D(n.b1) + ",\"k\":" + D(n.k) + ",\"mat\":" + mat(n.mat) + "}";
    }
    std::string obj(int idx) const {
        const Node& n = g.nodes[idx];
        switch (n.type) {
            case N_SPHERE: return "{\"type\":\"sphere\",\"center\":" + V(n.a) + ",\"radius\":" + D(n.r) + ",\"mat\":" + mat(n.mat) + "}";
            case N_MOVING_SPHERE:
                return "{\"type\":\"moving_sphere\",\"center0\":" + V(n.a) + ",\"center1\":" + V(n.b) + ",\"time0\":" + D(n.t0) +
                       ",\"time1\":" + D(n.t1) + ",\"radius\":" + D(n.r) + ",\"mat\":" + mat(n.mat) + "}";
            case N_TRIANGLE: return "{\"type\":\"triangle\",\"p\":[" + V(n.a) + "," + V(n.b) + "," + V(n.c) + "],\"mat\":" + mat(n.mat) + "}";
            case N_RECT: return rect(n);
            case N_BOX: {  // box.cpp:8-17 side order
                std::string r = "{\"type\":\"box\",\"min\":" + V(n.a) + ",\"max\":" + V(n.b) + ",\"sides\":[";
                const Vec3 &p0 = n.a, &p1 = n.b;
                Node s = make_node(N_RECT);
                s.mat = n.mat;
                auto side = [&](int axis, double a0, double a1, double b0, double b1, double k) {
                    s.axis = axis; s.a0 = a0; s.a1 = a1; s.b0 = b0; s.b1 = b1; s.k = k;
                    return rect(s);
                };
                r += side(0, p0[0], p1[0], p0[1], p1[1], p1[2]) + "," + side(0, p0[0], p1[0], p0[1], p1[1], p0[2]) + ",";
                r += side(1, p0[0], p1[0], p0[2], p1[2], p1[1]) + "," + side(1, p0[0], p1[0], p0[2], p1[2], p0[1]) + ",";
                r += side(2, p0[1], p1[1], p0[2], p1[2], p1[0]) + "," + side(2, p0[1], p1[1], p0[2], p1[2], p0[0]);
                return r + "]}";
            }
            case N_LIST: {
                std::string r = "{\"type\":\"list\",\"items\":[";
                for (size_t i = 0; i < n.items.size(); ++i) r += (i ? "," : "") + obj(n.items[i]);
                return r + "]}";
            }
            case N_BVH: {
                std::string r = "{\"type\":\"bvh\",\"nodes\":" + std::to_string(reference_bvh_nodes(n.items.size())) + ",\"box\":[" +
                                V(n.bbox.mn) + "," + V(n.bbox.mx) + "],\"items\":[";
                for (size_t i = 0; i < n.items.size(); ++i) r += (i ? ",\n" : "\n") + obj(n.items[i]);
                return r + "]}";
            }
            case N_TRANSLATE: return "{\"type\":\"translate\",\"offset\":" + V(n.a) + ",\"child\":" + obj(n.child) + "}";
            case N_ROTATE_Y:
                return "{\"type\":\"rotate_y\",\"sin\":" + D(n.sin_t) + ",\"cos\":" + D(n.cos_t) + ",\"hasbox\":" + (n.hasbox ? "true" : "false") +
                       ",\"bbox\":[" + V(n.bbox.mn) + "," + V(n.bbox.mx) + "],\"child\":" + obj(n.child) + "}";
            case N_MEDIUM:
                return "{\"type\":\"constant_medium\",\"neg_inv_density\":" + D(n.neg_inv_density) + ",\"phase\":" + mat(n.mat) +
                       ",\"boundary\":" + obj(n.child) + "}";
        }
        return "{}";
    }
};
}  // namespace

std::string dump_scene(const SceneGraph& g) {
    Dumper d{g, {}};
    std::string r = "{\"lookfrom\":" + V(g.lookfrom) + ",\"lookat\":" + V(g.lookat) + ",\"vfov\":" + D(g.vfov) + ",\"aperture\":" + D(g.aperture) +
                    ",\"background\":" + V(g.background) + ",\"objects\":[";
    for (size_t i = 0; i < g.world.size(); ++i) r += (i ? ",\n" : "\n") + d.obj(g.world[i]);
    return r + "]}\n";
}

// ------------------------------------------------------------------------------------------------ compile
namespace {
// BVH primitive hoisting (Compiler::obj, N_BVH): at most kMaxHoist primitives of a BVH of >= kHoistMinPrims whose box
// area is >= kHoistAreaShare of the whole BVH's.  Option compile.hoist = 0 turns it off (builder experiments).
constexpr size_t kHoistMinPrims = 8;
constexpr size_t kMaxHoist = 4;
constexpr double kHoistAreaShare = 0.5;
bool hoist_enabled() { return opt(Opt::Hoist) != 0; }
AABBd box_union(const AABBd& a, const AABBd& b) {
    AABBd r;
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = std::min(a.mn[k], b.mn[k]);
        r.mx[k] = std::max(a.mx[k], b.mx[k]);
    }
    return r;
}
double box_area(const AABBd& b) {
    const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return 2 * (dx * dy + dy * dz + dz * dx);
}

struct Compiler {
    const SceneGraph& g;
    FlatScene& f;

    uint32_t add_prim(int idx, AABBd& box) {
        const Node& n = g.nodes[idx];
        if (!g.bounding_box(idx, 0, 1, box)) throw std::runtime_error("primitive without bounding box");
        switch (n.type) {
            case N_SPHERE:
            case N_MOVING_SPHERE: {
                SphereRec<double> s{};
                for (int a = 0; a < 3; ++a) s.c[a] = n.a[a];
                s.r = n.r;
                s.mat = static_cast<uint32_t>(n.mat);
                if (n.type == N_MOVING_SPHERE) {
                    Vec3 d = n.b - n.a;  // (center1 - center0), moving_sphere.h:38
                    for (int a = 0; a < 3; ++a) s.d[a] = d[a];
                    s.t0 = n.t0;
                    s.dt = n.t1 - n.t0;
                    s.flags = SPH_MOVING;
                }
                f.spheres.push_back(s);
                return make_primref(PRIM_SPHERE, static_cast<uint32_t>(f.spheres.size() - 1));
            }
            case N_TRIANGLE: {
                TriRec<double> t{};
                for (int a = 0; a < 3; ++a) {
                    t.p[a] = n.a[a];
                    t.p[3 + a] = n.b[a];
                    t.p[6 + a] = n.c[a];
                }
                t.mat = static_cast<uint32_t>(n.mat);
                f.tris.push_back(t);
                return make_primref(PRIM_TRIANGLE, static_cast<uint32_t>(f.tris.size() - 1));
            }
            case N_RECT: {
                RectRec<double> r{n.a0, n.a1, n.b0, n.b1, n.k, static_cast<uint32_t>(n.axis), static_cast<uint32_t>(n.mat)};
                f.rects.push_back(r);
                return make_primref(PRIM_RECT, static_cast<uint32_t>(f.rects.size() - 1));
            }
            case N_BOX: {
                BoxRec<double> b{};
                for (int a = 0; a < 3; ++a) {
                    b.mn[a] = n.a[a];
                    b.mx[a] = n.b[a];
                }
                b.mat = static_cast<uint32_t>(n.mat);
                f.boxes.push_back(b);
                return make_primref(PRIM_BOX, static_cast<uint32_t>(f.boxes.size() - 1));
            }
            default: throw std::runtime_error("not a primitive");
        }
    }
    static bool is_prim(NodeType t) { return t == N_SPHERE || t == N_MOVING_SPHERE || t == N_TRIANGLE || t == N_RECT || t == N_BOX; }

    void gather(int idx, std::vector<uint32_t>& refs, std::vector<AABBd>& boxes) {
        const Node& n = g.nodes[idx];
        if (is_prim(n.type)) {
            AABBd b;
            refs.push_back(add_prim(idx, b));
            boxes.push_back(b);
        } else if (n.type == N_LIST || n.type == N_BVH) {
            for (int it : n.items) gather(it, refs, boxes);
        } else {
            throw std::runtime_error("instances and media inside a bvh/list below the top level are not supported");
        }
    }
    int add_obj(const ObjRec<double>& o) {
        f.objs.push_back(o);
        return static_cast<int>(f.objs.size()) - 1;
    }
    // One BVH object over every primitive below the graph items (BVH / list nodes and primitives).
    int bvh_obj(const std::vector<int>& items) {
        std::vector<uint32_t> refs;
        std::vector<AABBd> boxes;
        for (int it : items) gather(it, refs, boxes);
        int depth = 0, stack = 0;
        ObjRec<double> o{};
        o.kind = OBJ_BVH;
        // Hoisted primitives (layout.h ObjRec): a primitive whose box is as large as the whole BVH's (the random
        // scene's r = 1000 ground sphere, scene_manager.cpp:18) is met by nearly every ray, so it leaves the tree and
        // every traversal tests it first, with all its lanes at once
        std::vector<uint32_t> hoist;
        if (hoist_enabled() && refs.size() >= kHoistMinPrims) {
            AABBd all = boxes[0];
            for (const AABBd& b : boxes) all = box_union(all, b);
            const double a_all = box_area(all);
            std::vector<uint32_t> r2;
            std::vector<AABBd> b2;
            for (size_t i = 0; i < refs.size(); ++i) {
                if (hoist.size() < kMaxHoist && box_area(boxes[i]) >= kHoistAreaShare * a_all) hoist.push_back(refs[i]);
                else {
                    r2.push_back(refs[i]);
                    b2.push_back(boxes[i]);
                }
            }
            if (!hoist.empty()) {
                refs.swap(r2);
                boxes.swap(b2);
            }
        }
        // split BVH for meshes: a reference's clipped box is the box of the part of its triangle inside the slab (the
        // polygon clipped by the two planes), or the slab of its box for any other primitive
        const ClipFn clip = [&](uint32_t ref, int axis, double lo, double hi, const AABBd& cur, AABBd& out) -> bool {
            AABBd slab = cur;
            slab.mn[axis] = std::max(cur.mn[axis], lo);
            slab.mx[axis] = std::min(cur.mx[axis], hi);
            if (!(slab.mn[axis] <= slab.mx[axis])) return false;
            if (primref_type(ref) != PRIM_TRIANGLE) {
                out = slab;
                return true;
            }
            const TriRec<double>& t = f.tris[primref_index(ref)];
            Vec3 poly[8], next[8];
            int np = 3;
            for (int v = 0; v < 3; ++v) poly[v] = Vec3(t.p[3 * v], t.p[3 * v + 1], t.p[3 * v + 2]);
            for (int side = 0; side < 2 && np > 0; ++side) {  // keep x >= lo, then x <= hi (Sutherland-Hodgman)
                const double c = side == 0 ? lo : hi;
                auto inside = [&](const Vec3& q) { return side == 0 ? q[axis] >= c : q[axis] <= c; };
                int nn = 0;
                for (int i = 0; i < np; ++i) {
                    const Vec3& a = poly[i];
                    const Vec3& b = poly[(i + 1) % np];
                    const bool ia = inside(a), ib = inside(b);
                    if (ia) next[nn++] = a;
                    if (ia != ib) {
                        const double u = (c - a[axis]) / (b[axis] - a[axis]);
                        Vec3 q = a + u * (b - a);
                        q[axis] = c;
                        next[nn++] = q;
                    }
                }
                np = nn;
                for (int i = 0; i < np; ++i) poly[i] = next[i];
            }
            if (np == 0) return false;
            AABBd pb{poly[0], poly[0]};
            for (int i = 1; i < np; ++i)
                for (int k = 0; k < 3; ++k) {
                    pb.mn[k] = std::min(pb.mn[k], poly[i][k]);
                    pb.mx[k] = std::max(pb.mx[k], poly[i][k]);
                }
            for (int k = 0; k < 3; ++k) {
                out.mn[k] = std::max(pb.mn[k], slab.mn[k]);
                out.mx[k] = std::min(pb.mx[k], slab.mx[k]);
                if (!(out.mn[k] <= out.mx[k])) return false;
            }
            return true;
        };
        bool has_tri = false;
        for (uint32_t r : refs) has_tri |= primref_type(r) == PRIM_TRIANGLE;
        o.a = build_sah_bvh(boxes, refs, f.nodes, f.primrefs, depth, stack, has_tri ? &clip : nullptr);
        o.b = kNodeEmpty;
        if (!hoist.empty()) {
            o.b = make_leaf(static_cast<uint32_t>(f.primrefs.size()), static_cast<uint32_t>(hoist.size()));
            f.primrefs.insert(f.primrefs.end(), hoist.begin(), hoist.end());
        }
        f.max_bvh_depth = std::max(f.max_bvh_depth, depth);
        f.max_stack = std::max(f.max_stack, stack);
        return add_obj(o);
    }
    int obj(int idx) {
        const Node& n = g.nodes[idx];
        ObjRec<double> o{};
        if (is_prim(n.type)) {
            AABBd b;
            o.kind = OBJ_PRIM;
            o.a = static_cast<int32_t>(add_prim(idx, b));
            return add_obj(o);
        }
        switch (n.type) {
            case N_LIST:
            case N_BVH:
                return bvh_obj({idx});
            case N_TRANSLATE:
            case N_ROTATE_Y: {
                int depth = 0;
                for (int c = idx; g.nodes[c].type == N_TRANSLATE || g.nodes[c].type == N_ROTATE_Y; c = g.nodes[c].child) ++depth;
                if (depth > kMaxXformChain) throw std::runtime_error("more than two nested translate/rotate_y instances");
                break;
            }
            default: break;
        }
        switch (n.type) {
            case N_TRANSLATE:
                o.kind = OBJ_TRANSLATE;
                o.a = obj(n.child);
                for (int a = 0; a < 3; ++a) o.p[a] = n.a[a];
                return add_obj(o);
            case N_ROTATE_Y:
                o.kind = OBJ_ROTATE_Y;
                o.a = obj(n.child);
                o.p[0] = n.sin_t;
                o.p[1] = n.cos_t;
                return add_obj(o);
            case N_MEDIUM:
                o.kind = OBJ_MEDIUM;
                o.a = obj(n.child);
                o.b = n.mat;
                o.p[0] = n.neg_inv_density;
                f.has_media = true;
                return add_obj(o);
            default: break;
        }
        throw std::runtime_error("unsupported object");
    }
    void flatten(int idx, std::vector<int>& out) const {
        if (g.nodes[idx].type == N_LIST) {  // a nested hittable_list has the same closest-hit semantics flattened
            for (int it : g.nodes[idx].items) flatten(it, out);
            return;
        }
        out.push_back(idx);
    }
    // The world hittable_list (hittable_list.cpp:5-19).  World merging: a run of consecutive world objects that are
    // untransformed BVHs or primitives, holding at least one BVH, becomes one BVH over all their primitives (the
    // Next-Week final scene's box field + light + four spheres; a mesh + its light).  Its closest hit is theirs (up
    // to exact-t ties, as any BVH); a constant_medium ends a run, so every medium still sees the closest hit of the
    // objects before it when it clips its interval and decides whether to draw (constant_medium.h:37-62): the RNG
    // sequence is unchanged.  The loose primitives are then tested only when a ray enters their boxes instead of
    // once per segment by every lane.  Option compile.world_merge = 0 turns it off, 1 merges BVH runs only (experiments).
    void world(const std::vector<int>& roots) {
        std::vector<int> items;
        for (int w : roots) flatten(w, items);
        const int merge = static_cast<int>(opt(Opt::WorldMerge));
        auto mergeable = [&](int idx) { const NodeType t = g.nodes[idx].type; return t == N_BVH || is_prim(t); };
        for (size_t i = 0; i < items.size();) {
            size_t j = i;
            bool has_bvh = false;
            while (j < items.size() && mergeable(items[j])) has_bvh |= g.nodes[items[j++]].type == N_BVH;
            // mode 2 (default) also merges primitive-only runs of >= 3 objects, or that are the whole world (which can
            // then take the LDS kernel): Cornell box +25..32 %, the two-sphere scenes +6..16 %; a 2-primitive run in a
            // longer world (the Next-Week final's earth + perlin spheres) measured -1.5 % as a BVH and stays as it is
            const bool prims_ok = merge >= 2 && (j - i >= 3 || (i == 0 && j == items.size()));
            if (merge && (has_bvh || prims_ok) && j - i >= 2) {
                f.world.push_back(bvh_obj(std::vector<int>(items.begin() + static_cast<std::ptrdiff_t>(i), items.begin() + static_cast<std::ptrdiff_t>(j))));
                i = j;
            } else {
                f.world.push_back(obj(items[i]));
                ++i;
            }
        }
    }
};
}  // namespace

// Level-major node order: the roots of every BVH first, then all their inner children, level by level (a BFS over all
// roots).  A relabelling only -- the same trees, boxes and child order, so the same traversals and images -- that puts
// the levels every traversal walks next to each other at the front of the array.  (An LDS copy of those levels for
// k_paths_g, read through flat loads, measured -20 % on cow and the Next-Week final scene and +-0 on dino, whose
// whole tree fitted: node fetch latency is not what bounds k_paths_g.)
static void relabel_level_major(FlatScene& f) {
    const size_t n = f.nodes.size();
    if (n == 0) return;
    std::vector<int32_t> order, newid(n, -1);
    order.reserve(n);
    auto visit = [&](int32_t i) {
        if (i >= 0 && newid[static_cast<size_t>(i)] < 0) {
            newid[static_cast<size_t>(i)] = static_cast<int32_t>(order.size());
            order.push_back(i);
        }
    };
    for (const auto& o : f.objs)
        if (o.kind == OBJ_BVH) visit(o.a);
    for (size_t h = 0; h < order.size(); ++h)
        for (int c = 0; c < 4; ++c) visit(f.nodes[static_cast<size_t>(order[h])].child[c]);
    for (size_t i = 0; i < n; ++i) visit(static_cast<int32_t>(i));  // unreachable nodes (none expected) go last
    std::vector<BvhNode> out(n);
    for (size_t k = 0; k < n; ++k) {
        out[k] = f.nodes[static_cast<size_t>(order[k])];
        for (int c = 0; c < 4; ++c)
            if (out[k].child[c] >= 0) out[k].child[c] = newid[static_cast<size_t>(out[k].child[c])];
    }
    f.nodes.swap(out);
    for (auto& o : f.objs)
        if (o.kind == OBJ_BVH && o.a >= 0) o.a = newid[static_cast<size_t>(o.a)];
}

FlatScene compile_scene(const SceneGraph& g) {
    FlatScene f;
    if (g.world.empty()) throw std::runtime_error("Invalid input scene!");  // engine.h:32-36
    // does a texture tree sample u,v? (image / barycentric image, possibly under a checker)
    std::function<bool(int)> uses_uv = [&](int t) -> bool {
        if (t < 0) return false;
        const Texture& x = g.textures[t];
        if (x.type == TEX_IMAGE || x.type == TEX_BARY_IMAGE) return true;
        if (x.type == TEX_CHECKER) return uses_uv(x.even) || uses_uv(x.odd);
        return false;
    };
    for (const Material& m : g.materials) {
        MatRec<double> r{};
        r.type = m.type;
        r.tex = m.tex;
        r.flags = uses_uv(m.tex) ? MATF_NEEDS_UV : 0u;
        for (int a = 0; a < 3; ++a) r.albedo[a] = m.albedo[a];
        r.fuzz = m.fuzz;
        r.ir = m.ir;
        f.mats.push_back(r);
    }
    for (const Texture& t : g.textures) {
        TexRec<double> r{};
        r.type = t.type;
        r.even = t.even;
        r.odd = t.odd;
        r.perlin = t.perlin;
        r.image = t.image;
        for (int a = 0; a < 3; ++a) r.c[a] = t.c[a];
        r.scale = t.scale;
        for (int a = 0; a < 6; ++a) r.uv[a] = t.uv[a];
        f.texs.push_back(r);
    }
    for (const Perlin& p : g.perlins) {
        PerlinRec<double> r{};
        for (int i = 0; i < 256; ++i)
            for (int a = 0; a < 3; ++a) r.ranvec[i][a] = p.ranvec[i][a];
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 256; ++i) r.perm[k][i] = p.perm[k][i];
        f.perlins.push_back(r);
    }
    for (const Image& im : g.images) {
        ImageRec r{};
        r.offset = f.texels.size();
        r.w = im.w;
        r.h = im.h;
        r.bpp = im.bpp;
        f.texels.insert(f.texels.end(), im.data.begin(), im.data.end());
        f.images.push_back(r);
    }
    Compiler c{g, f};
    c.world(g.world);
    for (int a = 0; a < 3; ++a) f.background[a] = g.background[a];
    if (f.max_stack > kMaxStackDepth) throw std::runtime_error("bvh needs a deeper traversal stack than kMaxStackDepth");
    f.features = (f.spheres.empty() ? 0u : F_SPHERE) | (f.tris.empty() ? 0u : F_TRI) | (f.rects.empty() ? 0u : F_RECT) |
                 (f.boxes.empty() ? 0u : F_BOX) | (f.has_media ? F_MEDIA : 0u);
    for (const auto& o : f.objs) {
        if (o.kind == OBJ_TRANSLATE || o.kind == OBJ_ROTATE_Y) f.features |= F_XFORM;
        if (o.kind == OBJ_MEDIUM) {
            const ObjRec<double>& b = f.objs[o.a];
            if (!(b.kind == OBJ_PRIM && primref_type(static_cast<uint32_t>(b.a)) == PRIM_SPHERE)) f.features |= F_MEDIA_G;
        }
    }
    relabel_level_major(f);
    return f;
}

CameraRec<double> make_camera(const double lookfrom[3], const double lookat[3], const double vup_[3], double vfov, double aspect,
                              double aperture, double focus_dist, double time0, double time1) {
    // camera.h:8-36, the reference's own operation order.
    Vec3 from(lookfrom[0], lookfrom[1], lookfrom[2]), at(lookat[0], lookat[1], lookat[2]), vup(vup_[0], vup_[1], vup_[2]);
    double theta = vfov * kPi / 180.0;
    double h = std::tan(theta / 2);
    double vh = 2.0 * h;
    double vw = aspect * vh;
    Vec3 w = unit_vector(from - at);
    Vec3 u = unit_vector(cross(vup, w));
    Vec3 v = cross(w, u);
    Vec3 horizontal = focus_dist * vw * u;
    Vec3 vertical = focus_dist * vh * v;
    Vec3 llc = from - horizontal / 2 - vertical / 2 - focus_dist * w;
    CameraRec<double> c{};
    for (int a = 0; a < 3; ++a) {
        c.origin[a] = from[a];
        c.llc[a] = llc[a];
        c.horizontal[a] = horizontal[a];
        c.vertical[a] = vertical[a];
        c.u[a] = u[a];
        c.v[a] = v[a];
    }
    c.lens_radius = aperture / 2;
    c.time0 = time0;
    c.time1 = time1;
    return c;
}

}  // namespace art
