// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never the measured product).
//
// Headless driver around the UNMODIFIED reference sources in /root/reference/src, compiled where they lie
// by oracle/Makefile into oracle/_ref/ref_harness.  It reproduces the reference's per-pixel-exact run
// modes without the X11 GUI:
//   * `_stochastic_sample`  (/root/reference/src/engine/engine.h:58-68)
//   * `_ray_color`          (/root/reference/src/engine/engine.h:447-466)
//   * `_run_single`         (engine.h:70-94)            -> mode "single"
//   * `_run_parallel_stripes` (engine.h:335-376)        -> mode "stripes" (N threads, shared racy global RNG,
//                                                          exactly like the reference's 4-thread pool)
// and adds a segment counter (one count per `world.hit` call = the BASELINE metric's unit).
// Scenes come from the reference's own `scene_manager::build` (aliases 1..9, scene_manager.cpp:260-355),
// plus three build-defined scenes assembled from reference classes: "c1" (SURVEY Q7 3-sphere scene) and
// "cow"/"dino" (`_mesh_scene` scene_manager.cpp:236-258 with the OBJ path swapped).
//
// Commands:
//   ref_harness kat N                               first N random_double() of a fresh generator
//   ref_harness render SCENE W H SPP OUT [single|stripes T|adaptive|adaptive4|images] [T] [PIN]
//                                                   writes OUT.rgb (u8) and OUT.acc (f64 sums; zero in adaptive
//                                                   mode), prints JSON.  "adaptive" = `_run_adaptive` (engine.h:96-333)
//                                                   with its 4 stripes run one after another (deterministic);
//                                                   "images" = `_run_parallel_images` (engine.h:378-445) with its 4
//                                                   partial images traced one after another (OUT.acc: the pixel_acc
//                                                   sum of the four float images); "adaptive4" = `_run_adaptive`
//                                                   as the reference threads it (engine.h:298-313: four stripes of
//                                                   12 * (H / 48) rows, the last one taking the rest, on 4 threads
//                                                   sharing the global RNG: a timing mode, its image is racy as the
//                                                   reference's).  PIN = 1: worker t (or the one render thread) is
//                                                   pinned to the t-th CPU of the process's affinity set
//                                                   (sched_setaffinity), so a timed baseline does not migrate
//   ref_harness probe SCENE K                       next K random_double() after the scene build (RNG pin)
//   ref_harness dump SCENE OUT.json                 canonical dump of the scene graph (scene pin)
//   ref_harness mesh SCENE|PATH.obj OUT.bin                 post-triangulation triangle list: u32 n, f32 xyz*3*n, f64 rgb*n (solid albedo,
//                                                   else 0), and for a map_Kd mesh f64 (ua,va,ub,vb,uc,vc)*n
//   ref_harness texture PATH OUT.bin                stb-decoded texture bytes (w,h,c header + bytes)

// Pre-include the standard library so the access override below only touches reference classes.
#include <algorithm>
#include <array>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>
#include <vector>
#include <condition_variable>
#include <future>
#include <optional>
#include <variant>
#include <system_error>
#include <string_view>
#include <sched.h>
#include <charconv>
#include <unordered_map>
#include <deque>
#include <list>
#include <queue>
#include <set>
#include <numeric>

// The scene dump needs the private members of a few reference classes (sphere, solid_color, ...).
#define private public
#include "scene_manager.cpp"  // single TU: sphere.h/moving_sphere.h/triangle.h/constant_medium.h define non-inline functions
#include "camera.h"
#include "color.h"
#undef private

namespace {

std::atomic<long long> g_segments{0};

// engine.h:447-466, verbatim semantics, plus the segment counter.
color ray_color(const ray& r, const color& background, const hittable& world, int depth, long long& segs) {
    hit_record rec;
    if (depth <= 0)
        return color(0, 0, 0);
    ++segs;
    if (!world.hit(r, 0.001, infinity, rec))
        return background;
    ray scattered;
    color attenuation;
    color emitted = rec.mat_ptr->emitted(rec.u, rec.v, rec.p);
    if (!rec.mat_ptr->scatter(r, rec, attenuation, scattered))
        return emitted;
    return emitted + attenuation * ray_color(scattered, background, world, depth - 1, segs);
}

struct built_scene {
    scene s;
    double aspect = 0;
};

hittable_list c1_scene() {
    // build-defined 3-sphere lambertian scene (no such scene exists in the reference).
    hittable_list objects;
    objects.add(std::make_shared<sphere>(point3(0, -100.5, -1), 100, std::make_shared<lambertian>(color(0.8, 0.8, 0.0))));
    objects.add(std::make_shared<sphere>(point3(0, 0, -1), 0.5, std::make_shared<lambertian>(color(0.7, 0.3, 0.3))));
    objects.add(std::make_shared<sphere>(point3(-1, 0, -1), 0.5, std::make_shared<lambertian>(color(0.1, 0.2, 0.5))));
    return objects;
}

hittable_list mesh_scene(const std::string& path) {
    // scene_manager.cpp:236-258 with the OBJ path swapped.
    mesh m;
    if (!m.parse(path)) throw std::logic_error("cannot parse input obj file!");
    hittable_list world;
    auto triangles = m.build();
    world.add(std::make_shared<bvh_node>(triangles, 0.0, 1.0));
    auto light = std::make_shared<diffuse_light>(color(7, 7, 7));
    world.add(std::make_shared<xz_rect>(123, 423, 147, 412, 554, light));
    auto boundary = std::make_shared<sphere>(point3(0, 0, 0), 5000, std::make_shared<dielectric>(1.5));
    world.add(std::make_shared<constant_medium>(boundary, .0001, color(1, 1, 1)));
    return world;
}

scene build_scene(const std::string& name) {
    scene world;
    if (name == "c1") {
        world.objects = c1_scene();
        world.background = color(0.70, 0.80, 1.00);
        world.lookfrom = point3(0, 0, 0);
        world.lookat = point3(0, 0, -1);
        world.vfov = 90.0;
        world.aperture = 0.0;
    } else if (name == "cow" || name == "dino") {
        world.objects = mesh_scene(name == "cow" ? ressources::cow_obj_path : ressources::dino_obj_path);
        world.background = color(0.70, 0.80, 1.00);
        if (name == "cow") { world.lookfrom = point3(4, 2, 6); world.lookat = point3(2, 0, 0); }
        else { world.lookfrom = point3(0, 15, 25); world.lookat = point3(0, 10, 0); }
        world.vfov = 75.0;
    } else {
        scene_manager mgr;
        world = mgr.build(static_cast<scene_alias>(std::atoi(name.c_str())));
    }
    return world;
}

// ------------------------------------------------------------------------------------------------
// Canonical scene dump (JSON).  Doubles printed with %.17g (round-trip exact).
std::string D(double x) {
    char b[64];
    if (std::isinf(x)) return x > 0 ? "\"inf\"" : "\"-inf\"";
    std::snprintf(b, sizeof b, "%.17g", x);
    return b;
}
std::string V(const vec3& v) { return "[" + D(v[0]) + "," + D(v[1]) + "," + D(v[2]) + "]"; }

uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
    return h;
}

std::string dump_texture(const std::shared_ptr<texture>& t) {
    if (auto s = std::dynamic_pointer_cast<solid_color>(t)) return "{\"type\":\"solid\",\"c\":" + V(s->color_value) + "}";
    if (auto c = std::dynamic_pointer_cast<checker_texture>(t))
        return "{\"type\":\"checker\",\"even\":" + dump_texture(c->even) + ",\"odd\":" + dump_texture(c->odd) + "}";
    if (auto n = std::dynamic_pointer_cast<noise_texture>(t)) {
        std::string s = "{\"type\":\"noise\",\"scale\":" + D(n->scale) + ",\"ranvec\":[";
        for (size_t i = 0; i < n->noise.ranvec.size(); ++i) s += (i ? "," : "") + V(n->noise.ranvec[i]);
        auto perm = [&](const std::array<int, 256>& p) {
            std::string r = "[";
            for (size_t i = 0; i < p.size(); ++i) r += (i ? "," : "") + std::to_string(p[i]);
            return r + "]";
        };
        s += "],\"perm_x\":" + perm(n->noise.perm_x) + ",\"perm_y\":" + perm(n->noise.perm_y) + ",\"perm_z\":" + perm(n->noise.perm_z) + "}";
        return s;
    }
    if (auto im = std::dynamic_pointer_cast<image_texture>(t)) {
        static std::map<const image_texture*, std::string> cache;  // a textured mesh shares one image over all triangles
        auto it = cache.find(im.get());
        if (it != cache.end()) return it->second;
        size_t n = static_cast<size_t>(im->width) * im->height * im->bytes_per_pixel;
        char h[32];
        std::snprintf(h, sizeof h, "%016llx", (unsigned long long)(im->data ? fnv1a(im->data.get(), n) : 0));
        return cache[im.get()] = "{\"type\":\"image\",\"w\":" + std::to_string(im->width) + ",\"h\":" + std::to_string(im->height) +
               ",\"bpp\":" + std::to_string(im->bytes_per_pixel) + ",\"fnv1a\":\"" + h + "\"}";
    }
    if (auto b = std::dynamic_pointer_cast<barycentric_image_texture>(t))
        return "{\"type\":\"bary_image\",\"a\":[" + D(b->texcoord_a.first) + "," + D(b->texcoord_a.second) + "],\"b\":[" +
               D(b->texcoord_b.first) + "," + D(b->texcoord_b.second) + "],\"c\":[" + D(b->texcoord_c.first) + "," +
               D(b->texcoord_c.second) + "],\"tex\":" + dump_texture(b->tex) + "}";
    return "{\"type\":\"unknown_texture\"}";
}

std::string dump_material(const std::shared_ptr<material>& m) {
    if (auto l = std::dynamic_pointer_cast<lambertian>(m)) return "{\"type\":\"lambertian\",\"tex\":" + dump_texture(l->albedo) + "}";
    if (auto me = std::dynamic_pointer_cast<metal>(m)) return "{\"type\":\"metal\",\"albedo\":" + V(me->albedo) + ",\"fuzz\":" + D(me->fuzz) + "}";
    if (auto d = std::dynamic_pointer_cast<dielectric>(m)) return "{\"type\":\"dielectric\",\"ir\":" + D(d->ir) + "}";
    if (auto dl = std::dynamic_pointer_cast<diffuse_light>(m)) return "{\"type\":\"diffuse_light\",\"tex\":" + dump_texture(dl->emit) + "}";
    if (auto is = std::dynamic_pointer_cast<isotropic>(m)) return "{\"type\":\"isotropic\",\"tex\":" + dump_texture(is->albedo) + "}";
    return "{\"type\":\"unknown_material\"}";
}

void collect_bvh_leaves(const std::shared_ptr<hittable>& h, std::vector<std::shared_ptr<hittable>>& out, int& nodes) {
    if (auto b = std::dynamic_pointer_cast<bvh_node>(h)) {
        ++nodes;
        collect_bvh_leaves(b->left, out, nodes);
        if (b->right != b->left) collect_bvh_leaves(b->right, out, nodes);
        return;
    }
    out.push_back(h);
}

std::string dump_object(const std::shared_ptr<hittable>& h) {
    if (auto s = std::dynamic_pointer_cast<sphere>(h))
        return "{\"type\":\"sphere\",\"center\":" + V(s->center) + ",\"radius\":" + D(s->radius) + ",\"mat\":" + dump_material(s->mat_ptr) + "}";
    if (auto s = std::dynamic_pointer_cast<moving_sphere>(h))
        return "{\"type\":\"moving_sphere\",\"center0\":" + V(s->center0) + ",\"center1\":" + V(s->center1) + ",\"time0\":" + D(s->time0) +
               ",\"time1\":" + D(s->time1) + ",\"radius\":" + D(s->radius) + ",\"mat\":" + dump_material(s->mat_ptr) + "}";
    if (auto t = std::dynamic_pointer_cast<triangle>(h))
        return "{\"type\":\"triangle\",\"p\":[" + V(t->pt1) + "," + V(t->pt2) + "," + V(t->pt3) + "],\"mat\":" + dump_material(t->mat_ptr) + "}";
    if (auto r = std::dynamic_pointer_cast<xy_rect>(h))
        return "{\"type\":\"xy_rect\",\"a0\":" + D(r->x0) + ",\"a1\":" + D(r->x1) + ",\"b0\":" + D(r->y0) + ",\"b1\":" + D(r->y1) + ",\"k\":" + D(r->k) + ",\"mat\":" + dump_material(r->mp) + "}";
    if (auto r = std::dynamic_pointer_cast<xz_rect>(h))
        return "{\"type\":\"xz_rect\",\"a0\":" + D(r->x0) + ",\"a1\":" + D(r->x1) + ",\"b0\":" + D(r->z0) + ",\"b1\":" + D(r->z1) + ",\"k\":" + D(r->k) + ",\"mat\":" + dump_material(r->mp) + "}";
    if (auto r = std::dynamic_pointer_cast<yz_rect>(h))
        return "{\"type\":\"yz_rect\",\"a0\":" + D(r->y0) + ",\"a1\":" + D(r->y1) + ",\"b0\":" + D(r->z0) + ",\"b1\":" + D(r->z1) + ",\"k\":" + D(r->k) + ",\"mat\":" + dump_material(r->mp) + "}";
    if (auto b = std::dynamic_pointer_cast<box>(h)) {
        std::string s = "{\"type\":\"box\",\"min\":" + V(b->box_min) + ",\"max\":" + V(b->box_max) + ",\"sides\":[";
        for (size_t i = 0; i < b->sides.objects.size(); ++i) s += (i ? "," : "") + dump_object(b->sides.objects[i]);
        return s + "]}";
    }
    if (auto t = std::dynamic_pointer_cast<translate>(h))
        return "{\"type\":\"translate\",\"offset\":" + V(t->offset) + ",\"child\":" + dump_object(t->ptr) + "}";
    if (auto r = std::dynamic_pointer_cast<rotate_y>(h))
        return "{\"type\":\"rotate_y\",\"sin\":" + D(r->sin_theta) + ",\"cos\":" + D(r->cos_theta) + ",\"hasbox\":" + (r->hasbox ? "true" : "false") +
               ",\"bbox\":[" + V(r->bbox.minimum) + "," + V(r->bbox.maximum) + "],\"child\":" + dump_object(r->ptr) + "}";
    if (auto c = std::dynamic_pointer_cast<constant_medium>(h))
        return "{\"type\":\"constant_medium\",\"neg_inv_density\":" + D(c->neg_inv_density) + ",\"phase\":" + dump_material(c->phase_function) +
               ",\"boundary\":" + dump_object(c->boundary) + "}";
    if (auto b = std::dynamic_pointer_cast<bvh_node>(h)) {
        std::vector<std::shared_ptr<hittable>> leaves;
        int nodes = 0;
        collect_bvh_leaves(h, leaves, nodes);
        std::string s = "{\"type\":\"bvh\",\"nodes\":" + std::to_string(nodes) + ",\"box\":[" + V(b->box.minimum) + "," + V(b->box.maximum) + "],\"items\":[";
        for (size_t i = 0; i < leaves.size(); ++i) s += (i ? ",\n" : "\n") + dump_object(leaves[i]);
        return s + "]}";
    }
    if (auto l = std::dynamic_pointer_cast<hittable_list>(h)) {
        std::string s = "{\"type\":\"list\",\"items\":[";
        for (size_t i = 0; i < l->objects.size(); ++i) s += (i ? "," : "") + dump_object(l->objects[i]);
        return s + "]}";
    }
    return "{\"type\":\"unknown_object\"}";
}

camera make_camera(const scene& w, int W, int H) {
    // main.cpp:33-35 with aspect = W/H instead of the compile-time 4:3.
    vec3 vup(0, 1, 0);
    auto dist_to_focus = 10.0;
    return camera(w.lookfrom, w.lookat, vup, w.vfov, static_cast<double>(W) / static_cast<double>(H), w.aperture, dist_to_focus, 0.0, 1.0);
}

// Pins the calling thread to the t-th CPU (modulo) of the affinity set the process started with.
void pin_thread(int t) {
    static const std::vector<int> cpus = [] {
        std::vector<int> v;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof set, &set) == 0)
            for (int c = 0; c < CPU_SETSIZE; ++c)
                if (CPU_ISSET(c, &set)) v.push_back(c);
        return v;
    }();
    if (cpus.empty()) return;
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpus[static_cast<size_t>(t) % cpus.size()], &one);
    (void)sched_setaffinity(0, sizeof one, &one);
}

int cmd_render(const std::string& name, int W, int H, int spp, const std::string& out, const std::string& mode, int threads, bool pin) {
    if (pin) pin_thread(0);
    scene world = build_scene(name);
    camera cam = make_camera(world, W, H);
    std::vector<std::uint8_t> rgb(static_cast<size_t>(W) * H * 3);
    std::vector<double> acc(static_cast<size_t>(W) * H * 3);
    const hittable_list& objs = world.objects;

    // engine.h:58-68 (_stochastic_sample) + write_color (color.h:6-22) for one row.
    auto run_row = [&](int j, long long& segs) {
        for (int i = 0; i < W; ++i) {
            color pixel_color(0, 0, 0);
            for (int s = 0; s < spp; ++s) {
                auto u = (i + random_double()) / (W - 1);
                auto v = ((H - 1 - j) + random_double()) / (H - 1);
                ray r = cam.get_ray(u, v);
                pixel_color += ray_color(r, world.background, objs, 50, segs);
            }
            size_t o = 3 * (static_cast<size_t>(j) * W + i);
            acc[o + 0] = pixel_color[0];
            acc[o + 1] = pixel_color[1];
            acc[o + 2] = pixel_color[2];
            write_color(rgb.data() + o, pixel_color, spp);
        }
    };

    // engine.h:96-333 (_run_adaptive) on reference types, its four stripes run one after another on this thread (the
    // reference runs them on 4 threads sharing the global RNG, so its own output is not reproducible).
    auto sample = [&](int i, int j, long long& segs) {
        color pixel_color(0, 0, 0);
        for (int s = 0; s < spp; ++s) {
            auto u = (i + random_double()) / (W - 1);
            auto v = ((H - 1 - j) + random_double()) / (H - 1);
            ray r = cam.get_ray(u, v);
            pixel_color += ray_color(r, world.background, objs, 50, segs);
        }
        return pixel_color;
    };
    std::vector<int> work(static_cast<size_t>(W) * H * 3, -1);
    auto px = [&](int i, int j) { return work.data() + 3 * (static_cast<size_t>(j) * W + i); };
    auto evaluate = [&](int i, int j, long long& segs) { write_color<int>(px(i, j), sample(i, j, segs), spp); };
    auto corners = [&](int i, int j, int L, long long& segs) {  // engine.h:223-233
        evaluate(i, j, segs);
        evaluate(i + L - 1, j, segs);
        evaluate(i, j + L - 1, segs);
        evaluate(i + L - 1, j + L - 1, segs);
    };
    auto subdivide = [&](int i, int j, int L) {  // engine.h:96-136 _compute_corners_heuristic
        const int* c1 = px(i, j);
        const int* c2 = px(i + L - 1, j);
        const int* c3 = px(i, j + L - 1);
        const int* c4 = px(i + L - 1, j + L - 1);
        auto d = [](const int* a, const int* b) { return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]); };
        return d(c1, c2) > 100 || d(c2, c4) > 100 || d(c4, c3) > 100 || d(c3, c1) > 100;
    };
    auto interpolate = [&](int i, int j, int L) {  // engine.h:185-219 + _interpolate engine.h:138-149
        const int x1 = i, x2 = i + L - 1, y1 = j, y2 = j + L - 1;
        auto col = [&](int x, int y) { const int* p = px(x, y); return color{static_cast<double>(p[0]), static_cast<double>(p[1]), static_cast<double>(p[2])}; };
        const color Q11 = col(x1, y1), Q12 = col(x1, y2), Q21 = col(x2, y1), Q22 = col(x2, y2);
        for (int l = 0; l < L; ++l)
            for (int k = 0; k < L; ++k) {
                int* p = px(i + k, j + l);
                if (p[0] >= 0) continue;
                const int x = i + k, y = j + l;
                const auto xdiff = x2 - x1;
                const color R1 = (x2 - x) * Q11 / xdiff + (x - x1) * Q21 / xdiff;
                const color R2 = (x2 - x) * Q12 / xdiff + (x - x1) * Q22 / xdiff;
                const auto ydiff = y2 - y1;
                write_color_raw(p, (y2 - y) * R1 / ydiff + (y - y1) * R2 / ydiff);
            }
    };
    auto run_adaptive_rows = [&](int j0, int j1, long long& segs) {  // engine.h:236-292 process_square, row-major
        for (int j = j0; j < j1; j += 12)
            for (int i = 0; i < W; i += 12) {
                corners(i, j, 12, segs);
                if (!subdivide(i, j, 12)) { interpolate(i, j, 12); continue; }
                for (int l = j; l < j + 12; l += 6)
                    for (int k = i; k < i + 12; k += 6) {
                        corners(k, l, 6, segs);
                        if (!subdivide(k, l, 6)) { interpolate(k, l, 6); continue; }
                        for (int n = l; n < l + 6; n += 3)
                            for (int m = k; m < k + 6; m += 3) {
                                corners(m, n, 3, segs);
                                if (!subdivide(m, n, 3)) { interpolate(m, n, 3); continue; }
                                evaluate(m + 1, n, segs);
                                evaluate(m, n + 1, segs);
                                evaluate(m + 1, n + 1, segs);
                                evaluate(m + 2, n + 1, segs);
                                evaluate(m + 1, n + 2, segs);
                            }
                    }
            }
    };
    auto run_adaptive = [&](long long& segs) {
        run_adaptive_rows(0, H, segs);
        std::transform(work.begin(), work.end(), rgb.begin(), [](int v) { return static_cast<std::uint8_t>(v); });
    };
    auto run_adaptive4 = [&]() {  // engine.h:298-313: tp.add_job(run_stripe(...)) x 4 on thread_pool tp{4}
        const int stripe = 12 * (H / (4 * 12));
        const int bounds[5] = {0, stripe, 2 * stripe, 3 * stripe, H};
        std::vector<std::thread> pool;
        for (int t = 0; t < 4; ++t)
            pool.emplace_back([&, t]() {
                if (pin) pin_thread(t);
                long long segs = 0;
                run_adaptive_rows(bounds[t], bounds[t + 1], segs);
                g_segments += segs;
            });
        for (auto& th : pool) th.join();
        std::transform(work.begin(), work.end(), rgb.begin(), [](int v) { return static_cast<std::uint8_t>(v); });
    };

    // engine.h:378-445 (_run_parallel_images) on reference types: four partial images of spp/4 samples each, stored
    // as float by write_color_raw<float> (no gamma), summed as colors and written with the full spp.  The reference
    // runs the four on 4 threads sharing the global RNG; here they run one after another.
    auto run_images = [&](long long& segs) {
        const int m = spp / 4;
        std::vector<float> part(static_cast<size_t>(W) * H * 3 * 4, 0.f);
        for (int q = 0; q < 4; ++q)
            for (int j = 0; j < H; ++j)
                for (int i = 0; i < W; ++i) {
                    color pixel_color(0, 0, 0);
                    for (int s = 0; s < m; ++s) {
                        auto u = (i + random_double()) / (W - 1);
                        auto v = ((H - 1 - j) + random_double()) / (H - 1);
                        ray r = cam.get_ray(u, v);
                        pixel_color += ray_color(r, world.background, objs, 50, segs);
                    }
                    write_color_raw<float>(part.data() + (static_cast<size_t>(q) * H * W + static_cast<size_t>(j) * W + i) * 3, pixel_color);
                }
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) {
                color c[4];
                for (int q = 0; q < 4; ++q) {
                    const float* f = part.data() + (static_cast<size_t>(q) * H * W + static_cast<size_t>(j) * W + i) * 3;
                    c[q] = color(f[0], f[1], f[2]);
                }
                const color pixel_acc = c[0] + c[1] + c[2] + c[3];
                const size_t o = 3 * (static_cast<size_t>(j) * W + i);
                acc[o + 0] = pixel_acc[0];
                acc[o + 1] = pixel_acc[1];
                acc[o + 2] = pixel_acc[2];
                write_color(rgb.data() + o, pixel_acc, spp);
            }
    };

    const auto start = std::chrono::steady_clock::now();
    if (mode == "images") {
        long long segs = 0;
        run_images(segs);
        g_segments += segs;
    } else if (mode == "adaptive" || mode == "adaptive4") {
        if (W % 12 != 0 || H % 12 != 0) throw std::logic_error("for adaptive strategy image size should perfectly fit big square size for now!!");
        if (mode == "adaptive4") {
            run_adaptive4();
        } else {
            long long segs = 0;
            run_adaptive(segs);
            g_segments += segs;
        }
    } else if (mode == "single") {
        long long segs = 0;
        for (int j = 0; j < H; ++j) run_row(j, segs);
        g_segments += segs;
    } else {
        // engine.h:335-376: contiguous row bands, one per worker, shared (racy) global RNG.
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            int j0 = static_cast<int>(static_cast<long long>(H) * t / threads);
            int j1 = static_cast<int>(static_cast<long long>(H) * (t + 1) / threads);
            pool.emplace_back([&, j0, j1, t]() {
                if (pin) pin_thread(t);
                long long segs = 0;
                for (int j = j0; j < j1; ++j) run_row(j, segs);
                g_segments += segs;
            });
        }
        for (auto& th : pool) th.join();
    }
    const auto end = std::chrono::steady_clock::now();
    double ms = std::chrono::duration<double, std::milli>(end - start).count();

    std::ofstream(out + ".rgb", std::ios::binary).write(reinterpret_cast<const char*>(rgb.data()), static_cast<std::streamsize>(rgb.size()));
    std::ofstream(out + ".acc", std::ios::binary).write(reinterpret_cast<const char*>(acc.data()), static_cast<std::streamsize>(acc.size() * sizeof(double)));
    std::printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"spp\":%d,\"mode\":\"%s\",\"threads\":%d,\"segments\":%lld,\"ms\":%.3f,\"mseg_per_s\":%.6f}\n",
                name.c_str(), W, H, spp, mode.c_str(), mode == "stripes" ? threads : mode == "adaptive4" ? 4 : 1, g_segments.load(), ms,
                g_segments.load() / (ms * 1e3));
    return 0;
}

}  // namespace

int main(int argc, char** argv) try {
    if (argc < 2) { std::fprintf(stderr, "usage: see header\n"); return 2; }
    std::string cmd = argv[1];
    if (cmd == "kat") {
        int n = argc > 2 ? std::atoi(argv[2]) : 16;
        for (int i = 0; i < n; ++i) std::printf("%.17g\n", random_double());
        return 0;
    }
    if (cmd == "render") {
        if (argc < 7) return 2;
        std::string mode = argc > 7 ? argv[7] : "single";
        int threads = argc > 8 ? std::atoi(argv[8]) : 4;
        const bool pin = argc > 9 && std::atoi(argv[9]) != 0;
        return cmd_render(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), argv[6], mode, threads, pin);
    }
    if (cmd == "probe") {
        scene w = build_scene(argv[2]);
        int k = argc > 3 ? std::atoi(argv[3]) : 8;
        for (int i = 0; i < k; ++i) std::printf("%.17g\n", random_double());
        return 0;
    }
    if (cmd == "dump") {
        scene w = build_scene(argv[2]);
        std::ofstream f(argv[3]);
        f << "{\"lookfrom\":" << V(w.lookfrom) << ",\"lookat\":" << V(w.lookat) << ",\"vfov\":" << D(w.vfov) << ",\"aperture\":" << D(w.aperture)
          << ",\"background\":" << V(w.background) << ",\"objects\":[";
        for (size_t i = 0; i < w.objects.objects.size(); ++i) f << (i ? ",\n" : "\n") << dump_object(w.objects.objects[i]);
        f << "]}\n";
        return 0;
    }
    if (cmd == "mesh") {
        // Post-triangulation triangle list of a mesh scene, in leaf order of the BVH is NOT wanted: rebuild from the parser.
        std::string name = argv[2];
        mesh m;
        const bool file = name.size() > 4 && name.compare(name.size() - 4, 4, ".obj") == 0;  // any OBJ path (test meshes)
        if (!m.parse(file ? name : name == "cow" ? ressources::cow_obj_path : name == "dino" ? ressources::dino_obj_path : ressources::capsule_obj_path)) return 1;
        auto tris = m.build();
        std::ofstream f(argv[3], std::ios::binary);
        uint32_t n = static_cast<uint32_t>(tris.objects.size());
        f.write(reinterpret_cast<const char*>(&n), 4);
        for (auto& o : tris.objects) {
            auto t = std::dynamic_pointer_cast<triangle>(o);
            float p[9];
            for (int k = 0; k < 3; ++k) { p[k] = (float)t->pt1[k]; p[3 + k] = (float)t->pt2[k]; p[6 + k] = (float)t->pt3[k]; }
            f.write(reinterpret_cast<const char*>(p), sizeof p);
        }
        bool textured = false;
        for (auto& o : tris.objects) {
            auto t = std::dynamic_pointer_cast<triangle>(o);
            auto l = std::dynamic_pointer_cast<lambertian>(t->mat_ptr);
            double c[3] = {0, 0, 0};
            if (auto s = std::dynamic_pointer_cast<solid_color>(l->albedo)) { c[0] = s->color_value[0]; c[1] = s->color_value[1]; c[2] = s->color_value[2]; }
            textured |= static_cast<bool>(std::dynamic_pointer_cast<barycentric_image_texture>(l->albedo));
            f.write(reinterpret_cast<const char*>(c), sizeof c);
        }
        // textured meshes (map_Kd): per triangle the barycentric_image_texture coordinates a, b, c (f64 u, v each)
        for (auto& o : tris.objects) {
            if (!textured) break;
            auto t = std::dynamic_pointer_cast<triangle>(o);
            auto b = std::dynamic_pointer_cast<barycentric_image_texture>(std::dynamic_pointer_cast<lambertian>(t->mat_ptr)->albedo);
            double uv[6] = {0, 0, 0, 0, 0, 0};
            if (b) {
                uv[0] = b->texcoord_a.first; uv[1] = b->texcoord_a.second; uv[2] = b->texcoord_b.first;
                uv[3] = b->texcoord_b.second; uv[4] = b->texcoord_c.first; uv[5] = b->texcoord_c.second;
            }
            f.write(reinterpret_cast<const char*>(uv), sizeof uv);
        }
        return 0;
    }
    if (cmd == "texture") {
        int w = 0, h = 0, c = 0;
        auto data = imageio::load_image(argv[2], w, h, c);
        if (!data) return 1;
        std::ofstream f(argv[3], std::ios::binary);
        int32_t hdr[3] = {w, h, c};
        f.write(reinterpret_cast<const char*>(hdr), sizeof hdr);
        f.write(reinterpret_cast<const char*>(data.get()), static_cast<std::streamsize>(w) * h * c);
        return 0;
    }
    std::fprintf(stderr, "unknown command\n");
    return 2;
} catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
}
