// oracle/restate.cpp — TEST INFRASTRUCTURE ONLY: the CPU restatement of the reference's hot path.
//
// Restates, from the reference's behaviour (not its code), the ray_color / BVH / scatter loop of
// blackccpie/another_raytracer together with the scene feeders it needs, in IEEE double exactly like the reference
// (compiled with -ffp-contract=off).  Every routine cites the reference function it follows (paths relative to
// /root/reference/src).  Two RNG modes (restate.h):
//   ORC_MT  — bit-exact with the reference (checked against oracle/_ref/ref_harness and tests/golden fixtures):
//             global mt19937 + restated libstdc++ generate_canonical, g++ argument evaluation order spelled out
//             (right-to-left: vec3(rd(),rd(),rd()) draws z, y, x), recursive radiance fold of engine.h:447-466.
//   ORC_PCG — the product's RNG contract (per-(pixel, sample) PCG32, source-order draws) with the iterative
//             fold L += T*e; T *= a, i.e. the GPU algorithm in f64.  This is the checker of the HIP path
//             (tests/) and the `port` CPU baseline (bench.py), nothing else.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library.
#include "restate.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <zlib.h>

namespace {

thread_local std::string g_err;
std::string g_asset_dir = "assets";

const double kInf = std::numeric_limits<double>::infinity();
const double kPi = 3.1415926535897932385;  // tracer_utils.h:11

// ------------------------------------------------------------------------------------------------ vec3
// core/vec3.h: operators evaluated exactly as written there (v/t == (1/t)*v, dot left-to-right).
struct V3 {
    double e[3];
    V3() : e{0, 0, 0} {}
    V3(double a, double b, double c) : e{a, b, c} {}
    double operator[](int i) const { return e[i]; }
    double& operator[](int i) { return e[i]; }
    double x() const { return e[0]; }
    double y() const { return e[1]; }
    double z() const { return e[2]; }
    V3 operator-() const { return V3(-e[0], -e[1], -e[2]); }
    V3& operator+=(const V3& v) { e[0] += v.e[0]; e[1] += v.e[1]; e[2] += v.e[2]; return *this; }
    double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    double length() const { return std::sqrt(length_squared()); }
    bool near_zero() const {
        const double s = 1e-8;
        return std::fabs(e[0]) < s && std::fabs(e[1]) < s && std::fabs(e[2]) < s;
    }
};
inline V3 operator+(const V3& u, const V3& v) { return V3(u.e[0] + v.e[0], u.e[1] + v.e[1], u.e[2] + v.e[2]); }
inline V3 operator-(const V3& u, const V3& v) { return V3(u.e[0] - v.e[0], u.e[1] - v.e[1], u.e[2] - v.e[2]); }
inline V3 operator*(const V3& u, const V3& v) { return V3(u.e[0] * v.e[0], u.e[1] * v.e[1], u.e[2] * v.e[2]); }
inline V3 operator*(double t, const V3& v) { return V3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline V3 operator*(const V3& v, double t) { return t * v; }
inline V3 operator/(const V3& v, double t) { return (1 / t) * v; }
inline double dot(const V3& u, const V3& v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; }
inline V3 cross(const V3& u, const V3& v) {
    return V3(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
inline V3 unit_vector(const V3& v) { return v / v.length(); }
inline V3 vmin(const V3& a, const V3& b) { return V3(std::min(a[0], b[0]), std::min(a[1], b[1]), std::min(a[2], b[2])); }
inline V3 vmax(const V3& a, const V3& b) { return V3(std::max(a[0], b[0]), std::max(a[1], b[1]), std::max(a[2], b[2])); }
inline V3 reflect(const V3& v, const V3& n) { return v - 2 * dot(v, n) * n; }  // vec3.h:145-147
inline V3 refract(const V3& uv, const V3& n, double eta) {                     // vec3.h:149-154
    double cos_theta = std::min(dot(-uv, n), 1.0);
    V3 perp = eta * (uv + cos_theta * n);
    V3 par = -std::sqrt(std::fabs(1.0 - perp.length_squared())) * n;
    return perp + par;
}

struct Ray {  // core/ray.h
    V3 orig, dir;
    double tm = 0;
    V3 at(double t) const { return orig + t * dir; }
};

// ------------------------------------------------------------------------------------------------ RNG
// utils/tracer_utils.h:27-31: static std::mt19937 (seed 5489) + uniform_real_distribution<double>(0,1), i.e.
// libstdc++ generate_canonical<double,53>: two 32-bit outputs, (x0 + x1*2^32) / 2^64, clamped below 1.
struct Rng {
    bool pcg = false;
    std::mt19937 mt;
    uint64_t state = 0;

    double mt_canonical() {
        double sum = 0.0, tmp = 1.0;
        sum += static_cast<double>(mt()) * tmp;
        tmp *= 4294967296.0;
        sum += static_cast<double>(mt()) * tmp;
        tmp *= 4294967296.0;
        double r = sum / tmp;
        if (r >= 1.0) r = std::nextafter(1.0, 0.0);
        return r;
    }
    // The product's PCG32 contract (include/art.h "RNG contract"): 24-bit uniforms, exact in f32 and f64.
    double pcg_uniform() {
        uint64_t old = state;
        state = old * 6364136223846793005ull + 1442695040888963407ull;
        uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = static_cast<uint32_t>(old >> 59u);
        uint32_t x = (xs >> rot) | (xs << ((32u - rot) & 31u));
        return static_cast<double>(x >> 8) * (1.0 / 16777216.0);
    }
    double d() { return pcg ? pcg_uniform() : mt_canonical(); }
    double d(double lo, double hi) { return lo + (hi - lo) * d(); }              // tracer_utils.h:33-36
    int i(int lo, int hi) { return static_cast<int>(d(lo, hi + 1)); }            // tracer_utils.h:38-41

    // vec3::random(min,max) (vec3.h:59-61).  g++ evaluates the three constructor arguments right to left, so
    // mt mode draws z, then y, then x.  pcg mode (the product's contract) draws x, y, z.
    V3 vec(double lo, double hi) {
        V3 r;
        if (pcg) { r[0] = d(lo, hi); r[1] = d(lo, hi); r[2] = d(lo, hi); }
        else { r[2] = d(lo, hi); r[1] = d(lo, hi); r[0] = d(lo, hi); }
        return r;
    }
    V3 vec01() {
        V3 r;
        if (pcg) { r[0] = d(); r[1] = d(); r[2] = d(); }
        else { r[2] = d(); r[1] = d(); r[0] = d(); }
        return r;
    }
    V3 in_unit_sphere() {  // vec3.h:117-123
        while (true) {
            V3 p = vec(-1, 1);
            if (p.length_squared() >= 1) continue;
            return p;
        }
    }
    V3 unit() { return unit_vector(in_unit_sphere()); }  // vec3.h:125-127
    V3 in_unit_disk() {                                   // vec3.h:137-143 (mt: y drawn before x)
        while (true) {
            V3 p;
            if (pcg) { p[0] = d(-1, 1); p[1] = d(-1, 1); }
            else { p[1] = d(-1, 1); p[0] = d(-1, 1); }
            if (p.length_squared() >= 1) continue;
            return p;
        }
    }
};

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
uint64_t pcg_seed(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return splitmix64(((static_cast<uint64_t>(pixel) << 32) | sample) ^ splitmix64(seed));
}

// ------------------------------------------------------------------------------------------------ scene graph
struct AABB {  // primitives/aabb.h
    V3 mn, mx;
    bool hit(const Ray& r, double t_min, double t_max) const {  // aabb.h:16-29 (1.0f/d promoted to double)
        for (int a = 0; a < 3; a++) {
            double invD = 1.0f / r.dir[a];
            double t0 = (mn[a] - r.orig[a]) * invD;
            double t1 = (mx[a] - r.orig[a]) * invD;
            if (invD < 0.0f) std::swap(t0, t1);
            t_min = t0 > t_min ? t0 : t_min;
            t_max = t1 < t_max ? t1 : t_max;
            if (t_max <= t_min) return false;
        }
        return true;
    }
};
AABB surrounding(const AABB& a, const AABB& b) { return AABB{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; }  // aabb.h:35-39

struct Perlin {  // rendering/perlin.h
    V3 ranvec[256];
    int px[256], py[256], pz[256];
};

struct Image {
    int w = 0, h = 0, bpp = 0;
    std::vector<unsigned char> data;
};

enum TexK { T_SOLID, T_CHECKER, T_NOISE, T_IMAGE, T_BARY_IMAGE };
struct Tex {
    TexK k;
    V3 c;
    int even = -1, odd = -1;
    double scale = 0;
    int perlin = -1, image = -1;
    double ua = 0, va = 0, ub = 0, vb = 0, uc = 0, vc = 0;
};
enum MatK { M_LAMB, M_METAL, M_DIEL, M_LIGHT, M_ISO };
struct Mat {
    MatK k;
    int tex = -1;
    V3 albedo;
    double fuzz = 0, ir = 0;
};
enum ObjK { O_SPHERE, O_MSPHERE, O_TRI, O_XY, O_XZ, O_YZ, O_BOX, O_LIST, O_BVH, O_TRANSLATE, O_ROTY, O_MEDIUM };
struct Obj {
    ObjK k;
    int mat = -1;
    V3 c0, c1;  // sphere center / moving centers; translate offset; box min/max; triangle p1, p2
    V3 p3;      // triangle p3
    double r = 0, t0 = 0, t1 = 0;
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0, kk = 0;  // rects
    double sin_t = 0, cos_t = 0;
    bool hasbox = true;
    AABB box;                  // rotate_y / bvh cached box
    int left = -1, right = -1; // bvh children; child for translate/rotate/medium boundary
    double neg_inv_density = 0;
    std::vector<int> items;    // list / box sides
};

struct HitRec {  // engine/hittable.h:9-23
    V3 p, normal;
    int mat = -1;
    double t = 0, u = 0, v = 0;
    bool front_face = false;
    void set_face_normal(const Ray& r, const V3& outward) {
        front_face = dot(r.dir, outward) < 0;
        normal = front_face ? outward : -outward;
    }
};

struct Scene {
    std::vector<Obj> objs;
    std::vector<Mat> mats;
    std::vector<Tex> texs;
    std::vector<Perlin> perlins;
    std::vector<Image> images;
    std::vector<int> world;  // top-level hittable_list
    V3 lookfrom, lookat, background;
    double vfov = 40, aperture = 0;

    int add(const Obj& o) { objs.push_back(o); return static_cast<int>(objs.size()) - 1; }
    int mat(const Mat& m) { mats.push_back(m); return static_cast<int>(mats.size()) - 1; }
    int tex(const Tex& t) { texs.push_back(t); return static_cast<int>(texs.size()) - 1; }
    int solid(V3 c) { Tex t{T_SOLID}; t.c = c; return tex(t); }
    int lambertian(V3 c) { Mat m{M_LAMB}; m.tex = solid(c); return mat(m); }
    int lambertian_tex(int t) { Mat m{M_LAMB}; m.tex = t; return mat(m); }
    int metal(V3 a, double f) { Mat m{M_METAL}; m.albedo = a; m.fuzz = f < 1. ? f : 1.; return mat(m); }  // material.h:47
    int dielectric(double ir) { Mat m{M_DIEL}; m.ir = ir; return mat(m); }
    int light(V3 c) { Mat m{M_LIGHT}; m.tex = solid(c); return mat(m); }
    int isotropic(V3 c) { Mat m{M_ISO}; m.tex = solid(c); return mat(m); }
    int sphere(V3 c, double r, int m) { Obj o{O_SPHERE}; o.c0 = c; o.r = r; o.mat = m; return add(o); }
    int msphere(V3 a, V3 b, double t0, double t1, double r, int m) {
        Obj o{O_MSPHERE}; o.c0 = a; o.c1 = b; o.t0 = t0; o.t1 = t1; o.r = r; o.mat = m; return add(o);
    }
    int rect(ObjK k, double a0, double a1, double b0, double b1, double kk, int m) {
        Obj o{k}; o.a0 = a0; o.a1 = a1; o.b0 = b0; o.b1 = b1; o.kk = kk; o.mat = m; return add(o);
    }
    int box(V3 p0, V3 p1, int m) {  // primitives/box.cpp:3-19
        Obj o{O_BOX}; o.c0 = p0; o.c1 = p1;
        o.items.push_back(rect(O_XY, p0.x(), p1.x(), p0.y(), p1.y(), p1.z(), m));
        o.items.push_back(rect(O_XY, p0.x(), p1.x(), p0.y(), p1.y(), p0.z(), m));
        o.items.push_back(rect(O_XZ, p0.x(), p1.x(), p0.z(), p1.z(), p1.y(), m));
        o.items.push_back(rect(O_XZ, p0.x(), p1.x(), p0.z(), p1.z(), p0.y(), m));
        o.items.push_back(rect(O_YZ, p0.y(), p1.y(), p0.z(), p1.z(), p1.x(), m));
        o.items.push_back(rect(O_YZ, p0.y(), p1.y(), p0.z(), p1.z(), p0.x(), m));
        return add(o);
    }
    int translate(int child, V3 off) { Obj o{O_TRANSLATE}; o.left = child; o.c0 = off; return add(o); }
    int medium(int boundary, double d, V3 c) {  // engine/constant_medium.h:18-22
        Obj o{O_MEDIUM}; o.left = boundary; o.neg_inv_density = -1 / d; o.mat = isotropic(c); return add(o);
    }
};

// Moving sphere centre (moving_sphere.h:37-39).
V3 mcenter(const Obj& o, double time) { return o.c0 + ((time - o.t0) / (o.t1 - o.t0)) * (o.c1 - o.c0); }

bool bounding_box(const Scene& s, int idx, double time0, double time1, AABB& out) {
    const Obj& o = s.objs[idx];
    switch (o.k) {
        case O_SPHERE: {  // sphere.h:67-72
            V3 rr(o.r, o.r, o.r);
            out = AABB{o.c0 - rr, o.c0 + rr};
            return true;
        }
        case O_MSPHERE: {  // moving_sphere.h:61-70
            V3 rr(o.r, o.r, o.r);
            AABB b0{mcenter(o, time0) - rr, mcenter(o, time0) + rr};
            AABB b1{mcenter(o, time1) - rr, mcenter(o, time1) + rr};
            out = surrounding(b0, b1);
            return true;
        }
        case O_TRI:  // triangle.h:90-95
            out = AABB{vmin(o.c0, vmin(o.c1, o.p3)), vmax(o.c0, vmax(o.c1, o.p3))};
            return true;
        case O_XY: out = AABB{V3(o.a0, o.b0, o.kk - 0.0001), V3(o.a1, o.b1, o.kk + 0.0001)}; return true;  // aarect.h:16-21
        case O_XZ: out = AABB{V3(o.a0, o.kk - 0.0001, o.b0), V3(o.a1, o.kk + 0.0001, o.b1)}; return true;
        case O_YZ: out = AABB{V3(o.kk - 0.0001, o.a0, o.b0), V3(o.kk + 0.0001, o.a1, o.b1)}; return true;
        case O_BOX: out = AABB{o.c0, o.c1}; return true;  // box.h:15-18
        case O_LIST: {  // hittable_list.cpp:21-34
            if (o.items.empty()) return false;
            AABB tmp;
            bool first = true;
            for (int it : o.items) {
                if (!bounding_box(s, it, time0, time1, tmp)) return false;
                out = first ? tmp : surrounding(out, tmp);
                first = false;
            }
            return true;
        }
        case O_BVH: out = o.box; return true;
        case O_TRANSLATE: {  // hittable.cpp:14-23
            if (!bounding_box(s, o.left, time0, time1, out)) return false;
            out = AABB{out.mn + o.c0, out.mx + o.c0};
            return true;
        }
        case O_ROTY: out = o.box; return o.hasbox;
        case O_MEDIUM: return bounding_box(s, o.left, time0, time1, out);
    }
    return false;
}

int rotate_y(Scene& s, int child, double angle) {  // hittable.cpp:25-55
    Obj o{O_ROTY};
    o.left = child;
    double radians = angle * kPi / 180.0;
    o.sin_t = std::sin(radians);
    o.cos_t = std::cos(radians);
    AABB bbox;
    o.hasbox = bounding_box(s, child, 0, 1, bbox);
    V3 mn(kInf, kInf, kInf), mx(-kInf, -kInf, -kInf);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                double x = i * bbox.mx.x() + (1 - i) * bbox.mn.x();
                double y = j * bbox.mx.y() + (1 - j) * bbox.mn.y();
                double z = k * bbox.mx.z() + (1 - k) * bbox.mn.z();
                double newx = o.cos_t * x + o.sin_t * z;
                double newz = -o.sin_t * x + o.cos_t * z;
                V3 tester(newx, y, newz);
                for (int c = 0; c < 3; c++) {
                    mn[c] = std::fmin(mn[c], tester[c]);
                    mx[c] = std::fmax(mx[c], tester[c]);
                }
            }
    o.box = AABB{mn, mx};
    return s.add(o);
}

// primitives/bvh.cpp:3-42.  One random_int(0,2) per node in pre-order; std::sort (same comparator, same input
// order => the same permutation as the reference's libstdc++ build); median split; 1-spans alias left == right.
int build_bvh(Scene& s, const std::vector<int>& src, size_t start, size_t end, double time0, double time1, Rng& rng) {
    std::vector<int> objects = src;
    int axis = rng.i(0, 2);
    auto cmp = [&s, axis](int a, int b) {  // bvh.h:30-39
        AABB ba, bb;
        bounding_box(s, a, 0, 0, ba);
        bounding_box(s, b, 0, 0, bb);
        return ba.mn.e[axis] < bb.mn.e[axis];
    };
    Obj node{O_BVH};
    size_t span = end - start;
    if (span == 1) {
        node.left = node.right = objects[start];
    } else if (span == 2) {
        if (cmp(objects[start], objects[start + 1])) { node.left = objects[start]; node.right = objects[start + 1]; }
        else { node.left = objects[start + 1]; node.right = objects[start]; }
    } else {
        std::sort(objects.begin() + static_cast<std::ptrdiff_t>(start), objects.begin() + static_cast<std::ptrdiff_t>(end), cmp);
        size_t mid = start + span / 2;
        node.left = build_bvh(s, objects, start, mid, time0, time1, rng);
        node.right = build_bvh(s, objects, mid, end, time0, time1, rng);
    }
    AABB bl, br;
    bounding_box(s, node.left, time0, time1, bl);
    bounding_box(s, node.right, time0, time1, br);
    node.box = surrounding(bl, br);
    return s.add(node);
}

int make_perlin(Scene& s, Rng& rng) {  // perlin.h:10-19, :69-81
    Perlin p;
    for (auto& v : p.ranvec) v = unit_vector(rng.vec(-1, 1));
    for (int* perm : {p.px, p.py, p.pz}) {
        for (int i = 0; i < 256; i++) perm[i] = i;
        for (int i = 255; i > 0; i--) {
            int target = rng.i(0, i);
            int tmp = perm[i];
            perm[i] = perm[target];
            perm[target] = tmp;
        }
    }
    s.perlins.push_back(p);
    return static_cast<int>(s.perlins.size()) - 1;
}
int noise_tex(Scene& s, double scale, Rng& rng) {
    Tex t{T_NOISE};
    t.scale = scale;
    t.perlin = make_perlin(s, rng);
    return s.tex(t);
}

// The reference's stb_image output as a raw (w, h, bpp + bytes) asset, plain or gzip-compressed.
bool load_image_asset(Image& img, const std::string& name) {
    gzFile f = gzopen((g_asset_dir + "/" + name).c_str(), "rb");
    if (!f) return false;
    int32_t hdr[3];
    bool ok = gzread(f, hdr, sizeof hdr) == static_cast<int>(sizeof hdr);
    img.w = hdr[0]; img.h = hdr[1]; img.bpp = hdr[2];
    ok = ok && img.w > 0 && img.h > 0 && img.bpp >= 3 && img.w <= 65536 && img.h <= 65536 && img.bpp <= 4;
    if (ok) {
        img.data.resize(static_cast<size_t>(img.w) * img.h * img.bpp);
        ok = gzread(f, img.data.data(), static_cast<unsigned>(img.data.size())) == static_cast<int>(img.data.size());
    }
    gzclose(f);
    return ok;
}
int image_tex(Scene& s, const std::string& asset) {
    Image img;
    if (!load_image_asset(img, asset)) throw std::runtime_error("missing texture asset " + asset);
    s.images.push_back(std::move(img));
    Tex t{T_IMAGE};
    t.image = static_cast<int>(s.images.size()) - 1;
    return s.tex(t);
}

// ------------------------------------------------------------------------------------------------ scenes
// scene_manager.cpp:13-64 (_random_scene).  Draw order under g++ spelled out.
void random_scene(Scene& s, Rng& rng) {
    std::vector<int> objects;
    Tex chk{T_CHECKER};
    chk.even = s.solid(V3(0.2, 0.3, 0.1));
    chk.odd = s.solid(V3(0.9, 0.9, 0.9));
    int ground = s.lambertian_tex(s.tex(chk));
    objects.push_back(s.sphere(V3(0, -1000, 0), 1000, ground));
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            double choose_mat = rng.d();
            double cz = b + 0.9 * rng.d();  // point3(a + 0.9*rd(), 0.2, b + 0.9*rd()): z evaluated first
            double cx = a + 0.9 * rng.d();
            V3 center(cx, 0.2, cz);
            if ((center - V3(4, 0.2, 0)).length() > 0.9) {
                if (choose_mat < 0.8) {
                    V3 rhs = rng.vec01();  // color::random() * color::random(): right operand first
                    V3 lhs = rng.vec01();
                    int m = s.lambertian(lhs * rhs);
                    objects.push_back(s.sphere(center, 0.2, m));
                    V3 center2 = center + V3(0, rng.d(0, .5), 0);
                    objects.push_back(s.msphere(center, center2, 0.0, 1.0, 0.2, m));
                } else if (choose_mat < 0.95) {
                    V3 albedo = rng.vec(0.5, 1);
                    double fuzz = rng.d(0, 0.5);
                    objects.push_back(s.sphere(center, 0.2, s.metal(albedo, fuzz)));
                } else {
                    objects.push_back(s.sphere(center, 0.2, s.dielectric(1.5)));
                }
            }
        }
    }
    objects.push_back(s.sphere(V3(0, 1, 0), 1.0, s.dielectric(1.5)));
    objects.push_back(s.sphere(V3(-4, 1, 0), 1.0, s.lambertian(V3(0.4, 0.2, 0.1))));
    objects.push_back(s.sphere(V3(4, 1, 0), 1.0, s.metal(V3(0.7, 0.6, 0.5), 0.0)));
    s.world.push_back(build_bvh(s, objects, 0, objects.size(), 0, 1, rng));
}

void cornell_common(Scene& s, double light_val, bool smoke) {  // scene_manager.cpp:106-169
    int red = s.lambertian(V3(.65, .05, .05));
    int white = s.lambertian(V3(.73, .73, .73));
    int green = s.lambertian(V3(.12, .45, .15));
    int light = s.light(V3(light_val, light_val, light_val));
    s.world.push_back(s.rect(O_YZ, 0, 555, 0, 555, 555, green));
    s.world.push_back(s.rect(O_YZ, 0, 555, 0, 555, 0, red));
    if (!smoke) {
        s.world.push_back(s.rect(O_XZ, 213, 343, 227, 332, 554, light));
        s.world.push_back(s.rect(O_XZ, 0, 555, 0, 555, 0, white));
        s.world.push_back(s.rect(O_XZ, 0, 555, 0, 555, 555, white));
    } else {
        s.world.push_back(s.rect(O_XZ, 113, 443, 127, 432, 554, light));
        s.world.push_back(s.rect(O_XZ, 0, 555, 0, 555, 555, white));
        s.world.push_back(s.rect(O_XZ, 0, 555, 0, 555, 0, white));
    }
    s.world.push_back(s.rect(O_XY, 0, 555, 0, 555, 555, white));
    int box1 = s.box(V3(0, 0, 0), V3(165, 330, 165), white);
    box1 = rotate_y(s, box1, 15);
    box1 = s.translate(box1, V3(265, 0, 295));
    int box2 = s.box(V3(0, 0, 0), V3(165, 165, 165), white);
    box2 = rotate_y(s, box2, -18);
    box2 = s.translate(box2, V3(130, 0, 65));
    if (!smoke) {
        s.world.push_back(box1);
        s.world.push_back(box2);
    } else {
        s.world.push_back(s.medium(box1, 0.01, V3(0, 0, 0)));
        s.world.push_back(s.medium(box2, 0.01, V3(1, 1, 1)));
    }
}

void final_scene(Scene& s, Rng& rng) {  // scene_manager.cpp:171-234
    std::vector<int> boxes1;
    int ground = s.lambertian(V3(0.48, 0.83, 0.53));
    const int boxes_per_side = 20;
    for (int i = 0; i < boxes_per_side; i++) {
        for (int j = 0; j < boxes_per_side; j++) {
            double w = 100.0;
            double x0 = -1000.0 + i * w;
            double z0 = -1000.0 + j * w;
            double y0 = 0.0;
            double x1 = x0 + w;
            double y1 = rng.d(1, 101);
            double z1 = z0 + w;
            boxes1.push_back(s.box(V3(x0, y0, z0), V3(x1, y1, z1), ground));
        }
    }
    s.world.push_back(build_bvh(s, boxes1, 0, boxes1.size(), 0, 1, rng));
    s.world.push_back(s.rect(O_XZ, 123, 423, 147, 412, 554, s.light(V3(7, 7, 7))));
    V3 center1(400, 400, 200);
    V3 center2 = center1 + V3(30, 0, 0);
    s.world.push_back(s.msphere(center1, center2, 0, 1, 50, s.lambertian(V3(0.7, 0.3, 0.1))));
    s.world.push_back(s.sphere(V3(260, 150, 45), 50, s.dielectric(1.5)));
    s.world.push_back(s.sphere(V3(0, 150, 145), 50, s.metal(V3(0.8, 0.8, 0.9), 1.0)));
    int boundary = s.sphere(V3(360, 150, 145), 70, s.dielectric(1.5));
    s.world.push_back(boundary);
    s.world.push_back(s.medium(boundary, 0.2, V3(0.2, 0.4, 0.9)));
    boundary = s.sphere(V3(0, 0, 0), 5000, s.dielectric(1.5));
    s.world.push_back(s.medium(boundary, .0001, V3(1, 1, 1)));
    s.world.push_back(s.sphere(V3(400, 200, 400), 100, s.lambertian_tex(image_tex(s, "earthmap.rgb"))));
    int pertext = noise_tex(s, 0.1, rng);
    s.world.push_back(s.sphere(V3(220, 280, 300), 80, s.lambertian_tex(pertext)));
    std::vector<int> boxes2;
    int white = s.lambertian(V3(.73, .73, .73));
    for (int j = 0; j < 1000; j++) boxes2.push_back(s.sphere(rng.vec(0, 165), 10, white));
    int bvh2 = build_bvh(s, boxes2, 0, boxes2.size(), 0.0, 1.0, rng);
    s.world.push_back(s.translate(rotate_y(s, bvh2, 15), V3(-100, 270, 395)));
}

// The mesh enters as the reference's own post-triangulation triangle list (oracle/ref_harness `mesh`): f32 vertices,
// then per-triangle solid colours (unused: replayed from rng below) and, for a map_Kd mesh, the texture coordinates.
void mesh_scene(Scene& s, Rng& rng, const std::string& asset, const std::string& texture = "") {  // scene_manager.cpp:236-258 + mesh.h:67-145
    std::ifstream f(g_asset_dir + "/" + asset, std::ios::binary);
    if (!f) throw std::runtime_error("missing mesh asset " + asset);
    uint32_t n = 0;
    f.read(reinterpret_cast<char*>(&n), 4);
    std::vector<float> p(static_cast<size_t>(n) * 9);
    f.read(reinterpret_cast<char*>(p.data()), static_cast<std::streamsize>(p.size() * 4));
    std::vector<double> uv;
    int image = -1;
    if (!texture.empty()) {  // mesh.h:98-125: lambertian(barycentric_image_texture(uv1, uv2, uv3, map_Kd image))
        f.seekg(static_cast<std::streamoff>(4 + 36ull * n + 24ull * n));
        uv.resize(static_cast<size_t>(n) * 6);
        f.read(reinterpret_cast<char*>(uv.data()), static_cast<std::streamsize>(uv.size() * 8));
        if (!f) throw std::runtime_error("mesh asset " + asset + " has no texture coordinates");
        image = s.texs[image_tex(s, texture)].image;
    }
    std::vector<int> tris;
    for (uint32_t t = 0; t < n; ++t) {
        Obj o{O_TRI};
        const float* q = &p[static_cast<size_t>(t) * 9];
        o.c0 = V3(q[0], q[1], q[2]);
        o.c1 = V3(q[3], q[4], q[5]);
        o.p3 = V3(q[6], q[7], q[8]);
        if (image >= 0) {
            Tex b{T_BARY_IMAGE};
            b.image = image;
            const double* w = &uv[static_cast<size_t>(t) * 6];
            b.ua = w[0]; b.va = w[1]; b.ub = w[2]; b.vb = w[3]; b.uc = w[4]; b.vc = w[5];
            o.mat = s.lambertian_tex(s.tex(b));
        } else {
            o.mat = s.lambertian(rng.vec01());  // mesh.h:136-141: lambertian(color::random()) when the OBJ has no materials
        }
        tris.push_back(s.add(o));
    }
    s.world.push_back(build_bvh(s, tris, 0, tris.size(), 0.0, 1.0, rng));
    s.world.push_back(s.rect(O_XZ, 123, 423, 147, 412, 554, s.light(V3(7, 7, 7))));
    int boundary = s.sphere(V3(0, 0, 0), 5000, s.dielectric(1.5));
    s.world.push_back(s.medium(boundary, .0001, V3(1, 1, 1)));
}

void build_scene(Scene& s, const std::string& name, Rng& rng) {  // scene_manager.cpp:260-355 (+ SURVEY Q7/Q8)
    const V3 sky(0.70, 0.80, 1.00);
    if (name == "c1") {
        s.world.push_back(s.sphere(V3(0, -100.5, -1), 100, s.lambertian(V3(0.8, 0.8, 0.0))));
        s.world.push_back(s.sphere(V3(0, 0, -1), 0.5, s.lambertian(V3(0.7, 0.3, 0.3))));
        s.world.push_back(s.sphere(V3(-1, 0, -1), 0.5, s.lambertian(V3(0.1, 0.2, 0.5))));
        s.background = sky; s.lookfrom = V3(0, 0, 0); s.lookat = V3(0, 0, -1); s.vfov = 90; s.aperture = 0;
    } else if (name == "1" || name == "random") {
        random_scene(s, rng);
        s.background = sky; s.lookfrom = V3(13, 2, 3); s.lookat = V3(0, 0, 0); s.vfov = 20.0; s.aperture = 0.1;
    } else if (name == "2" || name == "two_spheres") {
        Tex chk{T_CHECKER};
        chk.even = s.solid(V3(0.2, 0.3, 0.1));
        chk.odd = s.solid(V3(0.9, 0.9, 0.9));
        int checker = s.tex(chk);
        s.world.push_back(s.sphere(V3(0, -10, 0), 10, s.lambertian_tex(checker)));
        s.world.push_back(s.sphere(V3(0, 10, 0), 10, s.lambertian_tex(checker)));
        s.background = sky; s.lookfrom = V3(13, 2, 3); s.lookat = V3(0, 0, 0); s.vfov = 20.0;
    } else if (name == "3" || name == "two_perlin_spheres") {
        int pertext = noise_tex(s, 4, rng);
        s.world.push_back(s.sphere(V3(0, -1000, 0), 1000, s.lambertian_tex(pertext)));
        s.world.push_back(s.sphere(V3(0, 2, 0), 2, s.lambertian_tex(pertext)));
        s.background = sky; s.lookfrom = V3(13, 2, 3); s.lookat = V3(0, 0, 0); s.vfov = 20.0;
    } else if (name == "4" || name == "earth") {
        s.world.push_back(s.sphere(V3(0, 0, 0), 2, s.lambertian_tex(image_tex(s, "earthmap.rgb"))));
        s.background = sky; s.lookfrom = V3(13, 2, 3); s.lookat = V3(0, 0, 0); s.vfov = 20.0;
    } else if (name == "5" || name == "simple_light") {
        int pertext = noise_tex(s, 4, rng);
        s.world.push_back(s.sphere(V3(0, -1000, 0), 1000, s.lambertian_tex(pertext)));
        s.world.push_back(s.sphere(V3(0, 2, 0), 2, s.lambertian_tex(pertext)));
        s.world.push_back(s.rect(O_XY, 3, 5, 1, 3, -2, s.light(V3(4, 4, 4))));
        s.background = V3(0, 0, 0); s.lookfrom = V3(26, 3, 6); s.lookat = V3(0, 2, 0); s.vfov = 20.0;
    } else if (name == "6" || name == "cornell_box" || name == "7" || name == "cornell_smoke") {
        bool smoke = name == "7" || name == "cornell_smoke";
        cornell_common(s, smoke ? 7 : 15, smoke);
        s.background = V3(0, 0, 0); s.lookfrom = V3(278, 278, -800); s.lookat = V3(278, 278, 0); s.vfov = 40.0;
    } else if (name == "8" || name == "final") {
        final_scene(s, rng);
        s.background = V3(0, 0, 0); s.lookfrom = V3(478, 278, -600); s.lookat = V3(278, 278, 0); s.vfov = 40.0;
    } else if (name == "cow" || name == "dino") {
        mesh_scene(s, rng, name + ".tris");
        s.background = sky;
        if (name == "cow") { s.lookfrom = V3(4, 2, 6); s.lookat = V3(2, 0, 0); }
        else { s.lookfrom = V3(0, 15, 25); s.lookat = V3(0, 10, 0); }
        s.vfov = 75.0;
    } else if (name == "9" || name == "mesh") {  // the stock _mesh_scene: the textured capsule
        mesh_scene(s, rng, "capsule.tris", "models/capsule/capsule.rgb.gz");
        s.background = sky; s.lookfrom = V3(2, 2, 1); s.lookat = V3(0, 0, 0); s.vfov = 75.0;
    } else {
        throw std::runtime_error("unknown scene " + name);
    }
}

// ------------------------------------------------------------------------------------------------ hit
void sphere_uv(const V3& p, double& u, double& v) {  // sphere.h:24-37
    double theta = std::acos(-p.y());
    double phi = std::atan2(-p.z(), p.x()) + kPi;
    u = phi / (2 * kPi);
    v = theta / kPi;
}

bool hit(const Scene& s, int idx, const Ray& r, double t_min, double t_max, HitRec& rec, Rng& rng);

bool hit_sphere_at(const V3& center, double radius, bool uv, const Ray& r, double t_min, double t_max, HitRec& rec) {
    V3 oc = r.orig - center;  // sphere.h:39-65 / moving_sphere.h:41-58
    double a = r.dir.length_squared();
    double half_b = dot(oc, r.dir);
    double c = oc.length_squared() - radius * radius;
    double disc = half_b * half_b - a * c;
    if (disc < 0) return false;
    double sqrtd = std::sqrt(disc);
    double root = (-half_b - sqrtd) / a;
    if (root < t_min || t_max < root) {
        root = (-half_b + sqrtd) / a;
        if (root < t_min || t_max < root) return false;
    }
    rec.t = root;
    rec.p = r.at(rec.t);
    V3 outward = (rec.p - center) / radius;
    rec.set_face_normal(r, outward);
    if (uv) sphere_uv(outward, rec.u, rec.v);
    return true;
}

bool hit_rect(const Obj& o, const Ray& r, double t_min, double t_max, HitRec& rec) {  // aarect.cpp:3-55
    int ka, a, b;
    V3 n;
    if (o.k == O_XY) { ka = 2; a = 0; b = 1; n = V3(0, 0, 1); }
    else if (o.k == O_XZ) { ka = 1; a = 0; b = 2; n = V3(0, 1, 0); }
    else { ka = 0; a = 1; b = 2; n = V3(1, 0, 0); }
    double t = (o.kk - r.orig[ka]) / r.dir[ka];
    if (t < t_min || t > t_max) return false;
    double x = r.orig[a] + t * r.dir[a];
    double y = r.orig[b] + t * r.dir[b];
    if (x < o.a0 || x > o.a1 || y < o.b0 || y > o.b1) return false;
    rec.u = (x - o.a0) / (o.a1 - o.a0);
    rec.v = (y - o.b0) / (o.b1 - o.b0);
    rec.t = t;
    rec.set_face_normal(r, n);
    rec.mat = o.mat;
    rec.p = r.at(t);
    return true;
}

bool hit_tri(const Obj& o, const Ray& r, double t_min, double t_max, HitRec& rec) {  // triangle.h:22-88
    V3 v1v2 = o.c1 - o.c0;
    V3 v1v3 = o.p3 - o.c0;
    V3 N = cross(v1v2, v1v3);
    double ndd = dot(N, r.dir);
    if (std::fabs(ndd) < DBL_EPSILON) return false;
    double d = -dot(N, o.c0);
    double t = -(dot(N, r.orig) + d) / ndd;
    if (t < t_min || t_max < t) return false;
    V3 p = r.orig + t * r.dir;
    double u, v;
    V3 c = cross(o.c1 - o.c0, p - o.c0);
    if (dot(N, c) < 0) return false;
    c = cross(o.p3 - o.c1, p - o.c1);
    if ((u = dot(N, c)) < 0) return false;
    c = cross(o.c0 - o.p3, p - o.p3);
    if ((v = dot(N, c)) < 0) return false;
    rec.t = t;
    rec.p = p;
    rec.set_face_normal(r, N);
    rec.u = u / N.length_squared();
    rec.v = v / N.length_squared();
    rec.mat = o.mat;
    return true;
}

bool hit_list(const Scene& s, const std::vector<int>& items, const Ray& r, double t_min, double t_max, HitRec& rec, Rng& rng) {
    HitRec temp;  // hittable_list.cpp:5-19 (an equal-t later object replaces)
    bool any = false;
    double closest = t_max;
    for (int it : items) {
        if (hit(s, it, r, t_min, closest, temp, rng)) {
            any = true;
            closest = temp.t;
            rec = temp;
        }
    }
    return any;
}

bool hit(const Scene& s, int idx, const Ray& r, double t_min, double t_max, HitRec& rec, Rng& rng) {
    const Obj& o = s.objs[idx];
    switch (o.k) {
        case O_SPHERE:
            if (!hit_sphere_at(o.c0, o.r, true, r, t_min, t_max, rec)) return false;
            rec.mat = o.mat;
            return true;
        case O_MSPHERE:
            if (!hit_sphere_at(mcenter(o, r.tm), o.r, false, r, t_min, t_max, rec)) return false;
            rec.mat = o.mat;
            return true;
        case O_TRI: return hit_tri(o, r, t_min, t_max, rec);
        case O_XY: case O_XZ: case O_YZ: return hit_rect(o, r, t_min, t_max, rec);
        case O_BOX: case O_LIST: return hit_list(s, o.items, r, t_min, t_max, rec, rng);
        case O_BVH: {  // bvh.cpp:44-52
            if (!o.box.hit(r, t_min, t_max)) return false;
            bool hl = hit(s, o.left, r, t_min, t_max, rec, rng);
            bool hr = hit(s, o.right, r, t_min, hl ? rec.t : t_max, rec, rng);
            return hl || hr;
        }
        case O_TRANSLATE: {  // hittable.cpp:3-12
            Ray moved{r.orig - o.c0, r.dir, r.tm};
            if (!hit(s, o.left, moved, t_min, t_max, rec, rng)) return false;
            rec.p += o.c0;
            rec.set_face_normal(moved, rec.normal);
            return true;
        }
        case O_ROTY: {  // hittable.cpp:57-85
            V3 origin = r.orig, direction = r.dir;
            origin[0] = o.cos_t * r.orig[0] - o.sin_t * r.orig[2];
            origin[2] = o.sin_t * r.orig[0] + o.cos_t * r.orig[2];
            direction[0] = o.cos_t * r.dir[0] - o.sin_t * r.dir[2];
            direction[2] = o.sin_t * r.dir[0] + o.cos_t * r.dir[2];
            Ray rr{origin, direction, r.tm};
            if (!hit(s, o.left, rr, t_min, t_max, rec, rng)) return false;
            V3 p = rec.p, normal = rec.normal;
            p[0] = o.cos_t * rec.p[0] + o.sin_t * rec.p[2];
            p[2] = -o.sin_t * rec.p[0] + o.cos_t * rec.p[2];
            normal[0] = o.cos_t * rec.normal[0] + o.sin_t * rec.normal[2];
            normal[2] = -o.sin_t * rec.normal[0] + o.cos_t * rec.normal[2];
            rec.p = p;
            rec.set_face_normal(rr, normal);
            return true;
        }
        case O_MEDIUM: {  // constant_medium.h:37-82
            HitRec rec1, rec2;
            if (!hit(s, o.left, r, -kInf, kInf, rec1, rng)) return false;
            if (!hit(s, o.left, r, rec1.t + 0.0001, kInf, rec2, rng)) return false;
            if (rec1.t < t_min) rec1.t = t_min;
            if (rec2.t > t_max) rec2.t = t_max;
            if (rec1.t >= rec2.t) return false;
            if (rec1.t < 0) rec1.t = 0;
            const double ray_length = r.dir.length();
            const double distance_inside = (rec2.t - rec1.t) * ray_length;
            const double hit_distance = o.neg_inv_density * std::log(rng.d());
            if (hit_distance > distance_inside) return false;
            rec.t = rec1.t + hit_distance / ray_length;
            rec.p = r.at(rec.t);
            rec.normal = V3(1, 0, 0);
            rec.front_face = true;
            rec.mat = o.mat;
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------------------------------------ shading
double perlin_noise(const Perlin& pn, const V3& p) {  // perlin.h:21-40, :83-97
    double u = p.x() - std::floor(p.x());
    double v = p.y() - std::floor(p.y());
    double w = p.z() - std::floor(p.z());
    int i = static_cast<int>(std::floor(p.x()));
    int j = static_cast<int>(std::floor(p.y()));
    int k = static_cast<int>(std::floor(p.z()));
    V3 c[2][2][2];
    for (int di = 0; di < 2; di++)
        for (int dj = 0; dj < 2; dj++)
            for (int dk = 0; dk < 2; dk++)
                c[di][dj][dk] = pn.ranvec[pn.px[(i + di) & 255] ^ pn.py[(j + dj) & 255] ^ pn.pz[(k + dk) & 255]];
    double uu = u * u * (3 - 2 * u);
    double vv = v * v * (3 - 2 * v);
    double ww = w * w * (3 - 2 * w);
    double accum = 0.0;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int cc = 0; cc < 2; cc++) {
                V3 weight_v(u - a, v - b, w - cc);
                accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) * (cc * ww + (1 - cc) * (1 - ww)) *
                         dot(c[a][b][cc], weight_v);
            }
    return accum;
}

V3 image_value(const Image& im, double u, double v) {  // texture.h:90-117
    if (im.data.empty()) return V3(0, 1, 1);
    u = std::clamp(u, 0.0, 1.0);
    v = 1.0 - std::clamp(v, 0.0, 1.0);
    int i = static_cast<int>(u * im.w);
    int j = static_cast<int>(v * im.h);
    if (i >= im.w) i = im.w - 1;
    if (j >= im.h) j = im.h - 1;
    const double color_scale = 1.0 / 255.0;
    const unsigned char* px = im.data.data() + static_cast<size_t>(j) * im.bpp * im.w + static_cast<size_t>(i) * im.bpp;
    return V3(color_scale * px[0], color_scale * px[1], color_scale * px[2]);
}

V3 tex_value(const Scene& s, int ti, double u, double v, const V3& p) {  // rendering/texture.h
    const Tex& t = s.texs[ti];
    switch (t.k) {
        case T_SOLID: return t.c;
        case T_CHECKER: {
            double sines = std::sin(10 * p.x()) * std::sin(10 * p.y()) * std::sin(10 * p.z());
            return sines < 0 ? tex_value(s, t.odd, u, v, p) : tex_value(s, t.even, u, v, p);
        }
        case T_NOISE: {
            double n = perlin_noise(s.perlins[t.perlin], t.scale * p);
            return V3(1, 1, 1) * 0.5 * (1.0 + n);
        }
        case T_IMAGE: return image_value(s.images[t.image], u, v);
        case T_BARY_IMAGE:  // texture.h:135-154
            return image_value(s.images[t.image], u * t.ua + v * t.ub + (1 - u - v) * t.uc, u * t.va + v * t.vb + (1 - u - v) * t.vc);
    }
    return V3();
}

V3 emitted(const Scene& s, const HitRec& rec) {  // material.h:12-14, :114-116
    const Mat& m = s.mats[rec.mat];
    if (m.k == M_LIGHT) return tex_value(s, m.tex, rec.u, rec.v, rec.p);
    return V3(0, 0, 0);
}

double reflectance(double cosine, double ref_idx) {  // material.h:93-98
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * std::pow((1 - cosine), 5);
}

bool scatter(const Scene& s, const Ray& r_in, const HitRec& rec, V3& att, Ray& scattered, Rng& rng) {
    const Mat& m = s.mats[rec.mat];
    switch (m.k) {
        case M_LAMB: {  // material.h:20-43
            V3 dir = rec.normal + rng.unit();
            if (dir.near_zero()) dir = rec.normal;
            scattered = Ray{rec.p, dir, r_in.tm};
            att = tex_value(s, m.tex, rec.u, rec.v, rec.p);
            return true;
        }
        case M_METAL: {  // material.h:45-61
            V3 reflected = reflect(unit_vector(r_in.dir), rec.normal);
            scattered = Ray{rec.p, reflected + m.fuzz * rng.in_unit_sphere(), r_in.tm};
            att = m.albedo;
            return dot(scattered.dir, rec.normal) > 0;
        }
        case M_DIEL: {  // material.h:63-99
            att = V3(1.0, 1.0, 1.0);
            double ratio = rec.front_face ? (1.0 / m.ir) : m.ir;
            V3 ud = unit_vector(r_in.dir);
            double cos_theta = std::min(dot(-ud, rec.normal), 1.0);
            double sin_theta = std::sqrt(1.0 - cos_theta * cos_theta);
            bool cannot = ratio * sin_theta > 1.0;
            V3 dir;
            if (cannot || reflectance(cos_theta, ratio) > rng.d()) dir = reflect(ud, rec.normal);
            else dir = refract(ud, rec.normal, ratio);
            scattered = Ray{rec.p, dir, r_in.tm};
            return true;
        }
        case M_LIGHT: return false;
        case M_ISO: {  // material.h:120-135
            scattered = Ray{rec.p, rng.in_unit_sphere(), r_in.tm};
            att = tex_value(s, m.tex, rec.u, rec.v, rec.p);
            return true;
        }
    }
    return false;
}

// engine.h:447-466, recursive fold (mt mode).
V3 ray_color_rec(const Scene& s, const Ray& r, int depth, Rng& rng, long long& segs) {
    HitRec rec;
    if (depth <= 0) return V3(0, 0, 0);
    ++segs;
    if (!hit_list(s, s.world, r, 0.001, kInf, rec, rng)) return s.background;
    Ray sc;
    V3 att;
    V3 e = emitted(s, rec);
    if (!scatter(s, r, rec, att, sc, rng)) return e;
    return e + att * ray_color_rec(s, sc, depth - 1, rng, segs);
}

// The same integrator flattened into the product's iterative form (pcg mode): L += T*e; T *= a.
// Path tracing diagnostics: ORC_TRACE="pixel:sample" prints every segment of that one path (orc_render_rows) as bit
// patterns, in the format of the product's ART_TRACE build (kernels.hip k_paths_g), so the two can be diffed.
static thread_local bool g_tracing = false;
static uint64_t bits(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return b;
}
V3 ray_color_iter(const Scene& s, Ray r, int max_depth, Rng& rng, long long& segs) {
    V3 L(0, 0, 0), T(1, 1, 1);
    for (int depth = 0; depth < max_depth; ++depth) {
        HitRec rec;
        ++segs;
        if (g_tracing)
            std::fprintf(stderr, "TRACE d=%d o=%016llx,%016llx,%016llx dir=%016llx,%016llx,%016llx tm=%016llx rng=%016llx\n", depth,
                         (unsigned long long)bits(r.orig[0]), (unsigned long long)bits(r.orig[1]), (unsigned long long)bits(r.orig[2]),
                         (unsigned long long)bits(r.dir[0]), (unsigned long long)bits(r.dir[1]), (unsigned long long)bits(r.dir[2]),
                         (unsigned long long)bits(r.tm), (unsigned long long)rng.state);
        if (!hit_list(s, s.world, r, 0.001, kInf, rec, rng)) {
            if (g_tracing) std::fprintf(stderr, "TRACE miss\n");
            L += T * s.background;
            break;
        }
        if (g_tracing)
            std::fprintf(stderr, "TRACE hit t=%016llx p=%016llx,%016llx,%016llx n=%016llx,%016llx,%016llx ff=%d mat=%d\n",
                         (unsigned long long)bits(rec.t), (unsigned long long)bits(rec.p[0]), (unsigned long long)bits(rec.p[1]),
                         (unsigned long long)bits(rec.p[2]), (unsigned long long)bits(rec.normal[0]), (unsigned long long)bits(rec.normal[1]),
                         (unsigned long long)bits(rec.normal[2]), rec.front_face ? 1 : 0, rec.mat);
        Ray sc;
        V3 att;
        V3 e = emitted(s, rec);
        L += T * e;
        if (!scatter(s, r, rec, att, sc, rng)) break;
        T = T * att;
        r = sc;
    }
    return L;
}

struct Camera {  // engine/camera.h:8-47
    V3 origin, llc, horizontal, vertical, u, v, w;
    double lens_radius = 0, time0 = 0, time1 = 0;
    Camera(V3 lookfrom, V3 lookat, V3 vup, double vfov, double aspect, double aperture, double focus_dist, double t0, double t1) {
        double theta = vfov * kPi / 180.0;
        double h = std::tan(theta / 2);
        double vh = 2.0 * h;
        double vw = aspect * vh;
        w = unit_vector(lookfrom - lookat);
        u = unit_vector(cross(vup, w));
        v = cross(w, u);
        origin = lookfrom;
        horizontal = focus_dist * vw * u;
        vertical = focus_dist * vh * v;
        llc = origin - horizontal / 2 - vertical / 2 - focus_dist * w;
        lens_radius = aperture / 2;
        time0 = t0;
        time1 = t1;
    }
    Ray get_ray(double s, double t, Rng& rng) const {
        V3 rd = lens_radius * rng.in_unit_disk();
        V3 offset = u * rd.x() + v * rd.y();
        Ray r;
        r.orig = origin + offset;
        r.dir = llc + s * horizontal + t * vertical - origin - offset;
        r.tm = rng.d(time0, time1);
        return r;
    }
};

void write_color(uint8_t* out, const V3& c, int spp) {  // core/color.h:6-22
    double scale = 1.0 / spp;
    for (int k = 0; k < 3; ++k) {
        double x = std::sqrt(scale * c[k]);
        out[k] = static_cast<uint8_t>(256 * std::clamp(x, 0.0, 0.999));
    }
}

std::string D(double x) {
    char b[64];
    if (std::isinf(x)) return x > 0 ? "\"inf\"" : "\"-inf\"";
    std::snprintf(b, sizeof b, "%.17g", x);
    return b;
}
std::string Vs(const V3& v) { return "[" + D(v[0]) + "," + D(v[1]) + "," + D(v[2]) + "]"; }
uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
    return h;
}

// Image dumps hash the texels once per image and dump (a textured mesh shares one image over every triangle).
std::vector<std::string> g_image_dump;
std::string dump_image(const Scene& s, int ii) {
    if (g_image_dump.size() < s.images.size()) g_image_dump.resize(s.images.size());
    std::string& r = g_image_dump[static_cast<size_t>(ii)];
    if (r.empty()) {
        const Image& im = s.images[ii];
        char h[32];
        std::snprintf(h, sizeof h, "%016llx", static_cast<unsigned long long>(fnv1a(im.data.data(), im.data.size())));
        r = "{\"type\":\"image\",\"w\":" + std::to_string(im.w) + ",\"h\":" + std::to_string(im.h) + ",\"bpp\":" + std::to_string(im.bpp) +
            ",\"fnv1a\":\"" + h + "\"}";
    }
    return r;
}
std::string dump_tex(const Scene& s, int ti) {
    const Tex& t = s.texs[ti];
    switch (t.k) {
        case T_SOLID: return "{\"type\":\"solid\",\"c\":" + Vs(t.c) + "}";
        case T_CHECKER: return "{\"type\":\"checker\",\"even\":" + dump_tex(s, t.even) + ",\"odd\":" + dump_tex(s, t.odd) + "}";
        case T_NOISE: {
            const Perlin& p = s.perlins[t.perlin];
            std::string r = "{\"type\":\"noise\",\"scale\":" + D(t.scale) + ",\"ranvec\":[";
            for (int i = 0; i < 256; ++i) r += (i ? "," : "") + Vs(p.ranvec[i]);
            auto perm = [](const int* q) {
                std::string x = "[";
                for (int i = 0; i < 256; ++i) x += (i ? "," : "") + std::to_string(q[i]);
                return x + "]";
            };
            return r + "],\"perm_x\":" + perm(p.px) + ",\"perm_y\":" + perm(p.py) + ",\"perm_z\":" + perm(p.pz) + "}";
        }
        case T_IMAGE: return dump_image(s, t.image);
        case T_BARY_IMAGE:  // texture.h:135-154, ref_harness dump_texture schema
            return "{\"type\":\"bary_image\",\"a\":[" + D(t.ua) + "," + D(t.va) + "],\"b\":[" + D(t.ub) + "," + D(t.vb) + "],\"c\":[" +
                   D(t.uc) + "," + D(t.vc) + "],\"tex\":" + dump_image(s, t.image) + "}";
    }
    return "{}";
}
std::string dump_mat(const Scene& s, int mi) {
    const Mat& m = s.mats[mi];
    switch (m.k) {
        case M_LAMB: return "{\"type\":\"lambertian\",\"tex\":" + dump_tex(s, m.tex) + "}";
        case M_METAL: return "{\"type\":\"metal\",\"albedo\":" + Vs(m.albedo) + ",\"fuzz\":" + D(m.fuzz) + "}";
        case M_DIEL: return "{\"type\":\"dielectric\",\"ir\":" + D(m.ir) + "}";
        case M_LIGHT: return "{\"type\":\"diffuse_light\",\"tex\":" + dump_tex(s, m.tex) + "}";
        case M_ISO: return "{\"type\":\"isotropic\",\"tex\":" + dump_tex(s, m.tex) + "}";
    }
    return "{}";
}
void bvh_leaves(const Scene& s, int idx, std::vector<int>& out, int& nodes) {
    const Obj& o = s.objs[idx];
    if (o.k == O_BVH) {
        ++nodes;
        bvh_leaves(s, o.left, out, nodes);
        if (o.right != o.left) bvh_leaves(s, o.right, out, nodes);
        return;
    }
    out.push_back(idx);
}
std::string dump_obj(const Scene& s, int idx) {
    const Obj& o = s.objs[idx];
    auto rect = [&](const char* ty) {
        return std::string("{\"type\":\"") + ty + "\",\"a0\":" + D(o.a0) + ",\"a1\":" + D(o.a1) + ",\"b0\":" + D(o.b0) + ",\"b1\":" + D(o.b1) +
               ",\"k\":" + D(o.kk) + ",\"mat\":" + dump_mat(s, o.mat) + "}";
    };
    switch (o.k) {
        case O_SPHERE: return "{\"type\":\"sphere\",\"center\":" + Vs(o.c0) + ",\"radius\":" + D(o.r) + ",\"mat\":" + dump_mat(s, o.mat) + "}";
        case O_MSPHERE:
            return "{\"type\":\"moving_sphere\",\"center0\":" + Vs(o.c0) + ",\"center1\":" + Vs(o.c1) + ",\"time0\":" + D(o.t0) + ",\"time1\":" + D(o.t1) +
                   ",\"radius\":" + D(o.r) + ",\"mat\":" + dump_mat(s, o.mat) + "}";
        case O_TRI: return "{\"type\":\"triangle\",\"p\":[" + Vs(o.c0) + "," + Vs(o.c1) + "," + Vs(o.p3) + "],\"mat\":" + dump_mat(s, o.mat) + "}";
        case O_XY: return rect("xy_rect");
        case O_XZ: return rect("xz_rect");
        case O_YZ: return rect("yz_rect");
        case O_BOX: {
            std::string r = "{\"type\":\"box\",\"min\":" + Vs(o.c0) + ",\"max\":" + Vs(o.c1) + ",\"sides\":[";
            for (size_t i = 0; i < o.items.size(); ++i) r += (i ? "," : "") + dump_obj(s, o.items[i]);
            return r + "]}";
        }
        case O_LIST: {
            std::string r = "{\"type\":\"list\",\"items\":[";
            for (size_t i = 0; i < o.items.size(); ++i) r += (i ? "," : "") + dump_obj(s, o.items[i]);
            return r + "]}";
        }
        case O_BVH: {
            std::vector<int> leaves;
            int nodes = 0;
            bvh_leaves(s, idx, leaves, nodes);
            std::string r = "{\"type\":\"bvh\",\"nodes\":" + std::to_string(nodes) + ",\"box\":[" + Vs(o.box.mn) + "," + Vs(o.box.mx) + "],\"items\":[";
            for (size_t i = 0; i < leaves.size(); ++i) r += (i ? ",\n" : "\n") + dump_obj(s, leaves[i]);
            return r + "]}";
        }
        case O_TRANSLATE: return "{\"type\":\"translate\",\"offset\":" + Vs(o.c0) + ",\"child\":" + dump_obj(s, o.left) + "}";
        case O_ROTY:
            return "{\"type\":\"rotate_y\",\"sin\":" + D(o.sin_t) + ",\"cos\":" + D(o.cos_t) + ",\"hasbox\":" + (o.hasbox ? "true" : "false") +
                   ",\"bbox\":[" + Vs(o.box.mn) + "," + Vs(o.box.mx) + "],\"child\":" + dump_obj(s, o.left) + "}";
        case O_MEDIUM:
            return "{\"type\":\"constant_medium\",\"neg_inv_density\":" + D(o.neg_inv_density) + ",\"phase\":" + dump_mat(s, o.mat) +
                   ",\"boundary\":" + dump_obj(s, o.left) + "}";
    }
    return "{}";
}

}  // namespace

extern "C" {

void orc_set_asset_dir(const char* dir) { g_asset_dir = dir ? dir : "assets"; }
const char* orc_last_error(void) { return g_err.c_str(); }

int orc_kat(int n, double* out) {
    Rng rng;
    for (int i = 0; i < n; ++i) out[i] = rng.d();
    return 0;
}

int orc_probe(const char* scene, int k, double* out) try {
    Scene s;
    Rng rng;
    build_scene(s, scene, rng);
    for (int i = 0; i < k; ++i) out[i] = rng.d();
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

size_t orc_dump(const char* scene, char* buf, size_t cap) try {
    Scene s;
    Rng rng;
    build_scene(s, scene, rng);
    g_image_dump.clear();
    std::string r = "{\"lookfrom\":" + Vs(s.lookfrom) + ",\"lookat\":" + Vs(s.lookat) + ",\"vfov\":" + D(s.vfov) + ",\"aperture\":" + D(s.aperture) +
                    ",\"background\":" + Vs(s.background) + ",\"objects\":[";
    for (size_t i = 0; i < s.world.size(); ++i) r += (i ? ",\n" : "\n") + dump_obj(s, s.world[i]);
    r += "]}\n";
    if (buf && cap) {
        size_t n = std::min(cap - 1, r.size());
        std::memcpy(buf, r.data(), n);
        buf[n] = 0;
    }
    return r.size() + 1;
} catch (const std::exception& e) {
    g_err = e.what();
    return 0;
}

int orc_render(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed, int row0, int nrows, int threads,
               uint8_t* rgb_out, double* acc_out, long long* segments_out, double* ms_out) try {
    if (W < 2 || H < 2 || spp < 1 || max_depth < 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) {
        g_err = "invalid render arguments";
        return -2;
    }
    Scene s;
    Rng scene_rng;  // scene build always replays the reference's mt19937 (geometry identical in both modes)
    build_scene(s, scene, scene_rng);
    Camera cam(s.lookfrom, s.lookat, V3(0, 1, 0), s.vfov, static_cast<double>(W) / static_cast<double>(H), s.aperture, 10.0, 0.0, 1.0);

    auto t0 = std::chrono::steady_clock::now();
    std::atomic<long long> segs_total{0};
    auto shade_pixel = [&](int i, int j, Rng& rng, long long& segs) {
        V3 pc(0, 0, 0);
        for (int sidx = 0; sidx < spp; ++sidx) {
            if (mode == ORC_PCG) rng.state = pcg_seed(seed, static_cast<uint32_t>(j) * static_cast<uint32_t>(W) + static_cast<uint32_t>(i), static_cast<uint32_t>(sidx));
            double ru = rng.d();
            double rv = rng.d();
            double u = (i + ru) / (W - 1);  // engine.h:62-63
            double v = ((H - 1 - j) + rv) / (H - 1);
            Ray r = cam.get_ray(u, v, rng);
            pc += mode == ORC_PCG ? ray_color_iter(s, r, max_depth, rng, segs) : ray_color_rec(s, r, max_depth, rng, segs);
        }
        size_t o = 3 * (static_cast<size_t>(j - row0) * W + i);
        if (acc_out) { acc_out[o] = pc[0]; acc_out[o + 1] = pc[1]; acc_out[o + 2] = pc[2]; }
        if (rgb_out) write_color(rgb_out + o, pc, spp);
    };

    if (mode == ORC_MT) {
        if (row0 != 0 || nrows != H) { g_err = "mt mode renders whole images only (one sequential RNG)"; return -2; }
        long long segs = 0;
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) shade_pixel(i, j, scene_rng, segs);  // the render continues the scene's stream
        segs_total = segs;
    } else {
        int nt = threads > 0 ? threads : static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
        std::atomic<int> next{row0};
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; ++t)
            pool.emplace_back([&]() {
                Rng rng;
                rng.pcg = true;
                long long segs = 0;
                for (int j = next++; j < row0 + nrows; j = next++)
                    for (int i = 0; i < W; ++i) shade_pixel(i, j, rng, segs);
                segs_total += segs;
            });
        for (auto& th : pool) th.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    if (segments_out) *segments_out = segs_total.load();
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(t1 - t0).count();
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

// engine.h:378-445 (_run_parallel_images), see restate.h.
int orc_render_images(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed, int threads,
                      uint8_t* rgb_out, double* acc_out, long long* segments_out, double* ms_out) try {
    if (W < 2 || H < 2 || spp < 1 || max_depth < 0) {
        g_err = "invalid render arguments";
        return -2;
    }
    Scene s;
    Rng scene_rng;
    build_scene(s, scene, scene_rng);
    Camera cam(s.lookfrom, s.lookat, V3(0, 1, 0), s.vfov, static_cast<double>(W) / static_cast<double>(H), s.aperture, 10.0, 0.0, 1.0);
    const int m = spp / 4;  // tracer_constants::samples_per_pixel / 4 per partial image
    std::vector<float> part(static_cast<size_t>(W) * H * 3 * 4, 0.f);
    auto t0 = std::chrono::steady_clock::now();
    std::atomic<long long> segs_total{0};
    // partial image q of pixel (i, j): run_image's _stochastic_sample (engine.h:395-405) + write_color_raw<float>
    auto partial = [&](int q, int i, int j, Rng& rng, long long& segs) {
        V3 pc(0, 0, 0);
        for (int k = 0; k < m; ++k) {
            if (mode == ORC_PCG)
                rng.state = pcg_seed(seed, static_cast<uint32_t>(j) * static_cast<uint32_t>(W) + static_cast<uint32_t>(i), static_cast<uint32_t>(q * m + k));
            double ru = rng.d();
            double rv = rng.d();
            Ray r = cam.get_ray((i + ru) / (W - 1), ((H - 1 - j) + rv) / (H - 1), rng);
            pc += mode == ORC_PCG ? ray_color_iter(s, r, max_depth, rng, segs) : ray_color_rec(s, r, max_depth, rng, segs);
        }
        float* f = part.data() + (static_cast<size_t>(q) * H * W + static_cast<size_t>(j) * W + i) * 3;
        f[0] = static_cast<float>(pc[0]);
        f[1] = static_cast<float>(pc[1]);
        f[2] = static_cast<float>(pc[2]);
    };
    if (mode == ORC_MT) {
        long long segs = 0;
        for (int q = 0; q < 4; ++q)
            for (int j = 0; j < H; ++j)
                for (int i = 0; i < W; ++i) partial(q, i, j, scene_rng, segs);
        segs_total = segs;
    } else {
        const int nt = threads > 0 ? threads : static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
        std::atomic<int> next{0};
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; ++t)
            pool.emplace_back([&]() {
                Rng rng;
                rng.pcg = true;
                long long segs = 0;
                for (int it = next++; it < 4 * H; it = next++)
                    for (int i = 0; i < W; ++i) partial(it / H, i, it % H, rng, segs);
                segs_total += segs;
            });
        for (auto& th : pool) th.join();
    }
    for (int j = 0; j < H; ++j)  // engine.h:424-440
        for (int i = 0; i < W; ++i) {
            V3 c[4];
            for (int q = 0; q < 4; ++q) {
                const float* f = part.data() + (static_cast<size_t>(q) * H * W + static_cast<size_t>(j) * W + i) * 3;
                c[q] = V3(f[0], f[1], f[2]);
            }
            const V3 acc = c[0] + c[1] + c[2] + c[3];
            const size_t o = 3 * (static_cast<size_t>(j) * W + i);
            if (acc_out) { acc_out[o] = acc[0]; acc_out[o + 1] = acc[1]; acc_out[o + 2] = acc[2]; }
            if (rgb_out) write_color(rgb_out + o, acc, spp);
        }
    auto t1 = std::chrono::steady_clock::now();
    if (segments_out) *segments_out = segs_total.load();
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(t1 - t0).count();
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

int orc_render_rows(const char* scene, int W, int H, int spp, int max_depth, uint64_t seed, const int* rows, int nrows, int threads,
                    uint8_t* rgb_out, double* acc_out, long long* segments_out, double* ms_out) try {
    if (W < 2 || H < 2 || spp < 1 || max_depth < 0 || nrows < 0 || (nrows > 0 && !rows)) {
        g_err = "invalid render arguments";
        return -2;
    }
    for (int k = 0; k < nrows; ++k)
        if (rows[k] < 0 || rows[k] >= H) { g_err = "row out of range"; return -2; }
    Scene s;
    Rng scene_rng;
    build_scene(s, scene, scene_rng);
    Camera cam(s.lookfrom, s.lookat, V3(0, 1, 0), s.vfov, static_cast<double>(W) / static_cast<double>(H), s.aperture, 10.0, 0.0, 1.0);
    constexpr int kChunk = 64;
    const int chunks = (W + kChunk - 1) / kChunk;
    long long trace_pixel = -1, trace_sample = -1;
    if (const char* t = std::getenv("ORC_TRACE")) std::sscanf(t, "%lld:%lld", &trace_pixel, &trace_sample);
    auto t0 = std::chrono::steady_clock::now();
    std::atomic<long long> segs_total{0};
    std::atomic<long long> next{0};
    const long long items = static_cast<long long>(nrows) * chunks;
    const int nt = threads > 0 ? threads : static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&]() {
            Rng rng;
            rng.pcg = true;
            long long segs = 0;
            for (long long it = next++; it < items; it = next++) {
                const int k = static_cast<int>(it / chunks), j = rows[k];
                const int i0 = static_cast<int>(it % chunks) * kChunk, i1 = std::min(W, i0 + kChunk);
                for (int i = i0; i < i1; ++i) {  // the per-pixel loop of orc_render, ORC_PCG
                    V3 pc(0, 0, 0);
                    for (int sidx = 0; sidx < spp; ++sidx) {
                        g_tracing = trace_pixel == static_cast<long long>(j) * W + i && trace_sample == sidx;
                        rng.state = pcg_seed(seed, static_cast<uint32_t>(j) * static_cast<uint32_t>(W) + static_cast<uint32_t>(i), static_cast<uint32_t>(sidx));
                        double ru = rng.d();
                        double rv = rng.d();
                        double u = (i + ru) / (W - 1);  // engine.h:62-63
                        double v = ((H - 1 - j) + rv) / (H - 1);
                        Ray r = cam.get_ray(u, v, rng);
                        pc += ray_color_iter(s, r, max_depth, rng, segs);
                    }
                    const size_t o = 3 * (static_cast<size_t>(k) * W + i);
                    if (acc_out) { acc_out[o] = pc[0]; acc_out[o + 1] = pc[1]; acc_out[o + 2] = pc[2]; }
                    if (rgb_out) write_color(rgb_out + o, pc, spp);
                }
            }
            segs_total += segs;
        });
    for (auto& th : pool) th.join();
    auto t1 = std::chrono::steady_clock::now();
    if (segments_out) *segments_out = segs_total.load();
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(t1 - t0).count();
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

int orc_trace_rays(const char* scene, const double* rays, long long n, double* t_out, double* normal_out) try {
    Scene s;
    Rng scene_rng;
    build_scene(s, scene, scene_rng);
    Rng rng;
    rng.pcg = true;
    for (long long i = 0; i < n; ++i) {
        const double* q = rays + 7 * i;
        Ray r{V3(q[0], q[1], q[2]), V3(q[3], q[4], q[5]), q[6]};
        rng.state = pcg_seed(0, static_cast<uint32_t>(i), 0);
        HitRec rec;
        if (hit_list(s, s.world, r, 0.001, kInf, rec, rng)) {
            t_out[i] = rec.t;
            for (int a = 0; a < 3; ++a) normal_out[3 * i + a] = rec.normal[a];
        } else {
            t_out[i] = kInf;
            for (int a = 0; a < 3; ++a) normal_out[3 * i + a] = 0.0;
        }
    }
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

// engine.h:96-333 (_run_adaptive), the 4 stripes one after another.  ORC_MT replays the reference's draw sequence
// (a corner shared by two levels is traced again, from the continuing stream); ORC_PCG traces every distinct pixel
// once (its (pixel, sample) streams would give the same value again), as the GPU does.
int orc_render_adaptive(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed, int threads,
                        uint8_t* rgb_out, long long* segments_out, double* ms_out) try {
    if (W < 12 || H < 12 || spp < 1 || max_depth < 0) { g_err = "invalid render arguments"; return -2; }
    if (W % 12 != 0 || H % 12 != 0) { g_err = "for adaptive strategy image size should perfectly fit big square size for now!!"; return -3; }
    Scene s;
    Rng scene_rng;
    build_scene(s, scene, scene_rng);
    Camera cam(s.lookfrom, s.lookat, V3(0, 1, 0), s.vfov, static_cast<double>(W) / static_cast<double>(H), s.aperture, 10.0, 0.0, 1.0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<int> work(static_cast<size_t>(W) * H * 3, -1);
    std::vector<uint8_t> traced(static_cast<size_t>(W) * H, 0);
    auto px = [&](int i, int j) { return work.data() + 3 * (static_cast<size_t>(j) * W + i); };
    auto evaluate = [&](int i, int j, Rng& rng, long long& segs) {  // write_color<int>(pixel, _stochastic_sample(i, j))
        const size_t p = static_cast<size_t>(j) * W + i;
        if (mode == ORC_PCG && traced[p]) return;
        traced[p] = 1;
        V3 pc(0, 0, 0);
        for (int sidx = 0; sidx < spp; ++sidx) {
            if (mode == ORC_PCG) rng.state = pcg_seed(seed, static_cast<uint32_t>(p), static_cast<uint32_t>(sidx));
            double ru = rng.d();
            double rv = rng.d();
            Ray r = cam.get_ray((i + ru) / (W - 1), ((H - 1 - j) + rv) / (H - 1), rng);
            pc += mode == ORC_PCG ? ray_color_iter(s, r, max_depth, rng, segs) : ray_color_rec(s, r, max_depth, rng, segs);
        }
        uint8_t c[3];
        write_color(c, pc, spp);
        int* o = px(i, j);
        o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
    };
    auto corners = [&](int i, int j, int L, Rng& rng, long long& segs) {  // engine.h:223-233: ul, ur, bl, br
        evaluate(i, j, rng, segs);
        evaluate(i + L - 1, j, rng, segs);
        evaluate(i, j + L - 1, rng, segs);
        evaluate(i + L - 1, j + L - 1, rng, segs);
    };
    auto subdivide = [&](int i, int j, int L) {  // engine.h:96-136
        const int *c1 = px(i, j), *c2 = px(i + L - 1, j), *c3 = px(i, j + L - 1), *c4 = px(i + L - 1, j + L - 1);
        auto d = [](const int* a, const int* b) { return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]); };
        return d(c1, c2) > 100 || d(c2, c4) > 100 || d(c4, c3) > 100 || d(c3, c1) > 100;
    };
    auto interpolate = [&](int i, int j, int L) {  // engine.h:185-219, _interpolate engine.h:138-149 (v/t == (1/t)*v)
        const int x1 = i, x2 = i + L - 1, y1 = j, y2 = j + L - 1;
        auto col = [&](int x, int y) { const int* p = px(x, y); return V3(p[0], p[1], p[2]); };
        const V3 Q11 = col(x1, y1), Q12 = col(x1, y2), Q21 = col(x2, y1), Q22 = col(x2, y2);
        for (int l = 0; l < L; ++l)
            for (int k = 0; k < L; ++k) {
                int* p = px(i + k, j + l);
                if (p[0] >= 0) continue;
                const int x = i + k, y = j + l;
                const double xdiff = x2 - x1, ydiff = y2 - y1;
                const V3 R1 = (x2 - x) * Q11 / xdiff + (x - x1) * Q21 / xdiff;
                const V3 R2 = (x2 - x) * Q12 / xdiff + (x - x1) * Q22 / xdiff;
                const V3 c = (y2 - y) * R1 / ydiff + (y - y1) * R2 / ydiff;
                p[0] = static_cast<int>(c[0]); p[1] = static_cast<int>(c[1]); p[2] = static_cast<int>(c[2]);  // write_color_raw<int>
            }
    };
    auto square = [&](int i, int j, Rng& rng, long long& segs) {  // engine.h:236-292 process_square
        corners(i, j, 12, rng, segs);
        if (!subdivide(i, j, 12)) { interpolate(i, j, 12); return; }
        for (int l = j; l < j + 12; l += 6)
            for (int k = i; k < i + 12; k += 6) {
                corners(k, l, 6, rng, segs);
                if (!subdivide(k, l, 6)) { interpolate(k, l, 6); continue; }
                for (int n = l; n < l + 6; n += 3)
                    for (int m = k; m < k + 6; m += 3) {
                        corners(m, n, 3, rng, segs);
                        if (!subdivide(m, n, 3)) { interpolate(m, n, 3); continue; }
                        evaluate(m + 1, n, rng, segs);
                        evaluate(m, n + 1, rng, segs);
                        evaluate(m + 1, n + 1, rng, segs);
                        evaluate(m + 2, n + 1, rng, segs);
                        evaluate(m + 1, n + 2, rng, segs);
                    }
            }
    };
    std::atomic<long long> segs_total{0};
    if (mode == ORC_MT) {
        long long segs = 0;
        for (int j = 0; j < H; j += 12)
            for (int i = 0; i < W; i += 12) square(i, j, scene_rng, segs);
        segs_total = segs;
    } else {  // big squares are independent: one row of squares per task
        int nt = threads > 0 ? threads : static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
        std::atomic<int> next{0};
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; ++t)
            pool.emplace_back([&]() {
                Rng rng;
                rng.pcg = true;
                long long segs = 0;
                for (int j = 12 * next++; j < H; j = 12 * next++)
                    for (int i = 0; i < W; i += 12) square(i, j, rng, segs);
                segs_total += segs;
            });
        for (auto& th : pool) th.join();
    }
    if (rgb_out)
        for (size_t k = 0; k < work.size(); ++k) rgb_out[k] = static_cast<uint8_t>(work[k]);
    auto t1 = std::chrono::steady_clock::now();
    if (segments_out) *segments_out = segs_total.load();
    if (ms_out) *ms_out = std::chrono::duration<double, std::milli>(t1 - t0).count();
    return 0;
} catch (const std::exception& e) {
    g_err = e.what();
    return -1;
}

}  // extern "C"
