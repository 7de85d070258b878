// include/art_engine.hpp — C++ host surface of the reference's engine path over the C ABI (include/art.h).
//
// The reference's src/main.cpp (main.cpp:25-60) drives three classes: scene_manager::build (scene_manager.cpp:260),
// camera (camera.h:8-36) and engine<W,H,C> (engine.h:19-54).  This header restates that surface for C++ callers on
// top of libart.so, so a reference-style main() changes its includes and nothing else:
//
//     art::scene_manager sm("assets");                           // asset_dir: earthmap.jpg, models/...
//     art::scene world = sm.build("1");                          // scene_alias::random
//     art::camera cam(world.lookfrom, world.lookat, {0, 1, 0}, world.vfov, double(W) / H, world.aperture, 10.0, 0, 1);
//     art::engine<W, H, 3> eng(cam, art::engine_mode::parallel_stripes);
//     eng.set_scene(world, world.background);
//     std::vector<uint8_t> image(W * H * 3);
//     int ms = eng.run(image.data());                            // -1 on an empty world, like engine.h:32-36
//     art::imageio::save_image("output.png", W, H, 3, image.data());
//
// Header-only; no HIP, torch or ROCm header is needed by the caller (link with -lart).  Errors surface as the
// reference's exceptions: std::logic_error for an adaptive size off the 12-px grid (engine.h:178-179) and for an
// unknown scene (scene_manager.cpp:351), std::runtime_error for everything else (message from rt_last_error()).
#ifndef ART_ENGINE_HPP
#define ART_ENGINE_HPP

#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <exception>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "art.h"

namespace art {

struct vec3 {  // core/vec3.h (storage only: the arithmetic runs inside libart)
    double e[3] = {0, 0, 0};
    double x() const { return e[0]; }
    double y() const { return e[1]; }
    double z() const { return e[2]; }
};
using point3 = vec3;
using color = vec3;

inline void check(int rc, const char* where) {
    if (rc < 0) throw std::runtime_error(std::string(where) + ": " + rt_last_error());
}

enum class engine_mode { single, adaptive, parallel_stripes, parallel_images };  // engine.h:10-16

class camera {  // camera.h:8-36 (the basis is built inside libart from the same nine arguments, in f64)
public:
    camera(point3 lookfrom, point3 lookat, vec3 vup, double vfov, double aspect_ratio, double aperture, double focus_dist,
           double time0 = 0, double time1 = 0) {
        for (int k = 0; k < 3; ++k) {
            c_.lookfrom[k] = lookfrom.e[k];
            c_.lookat[k] = lookat.e[k];
            c_.vup[k] = vup.e[k];
        }
        c_.vfov = vfov;
        c_.aspect = aspect_ratio;
        c_.aperture = aperture;
        c_.focus_dist = focus_dist;
        c_.time0 = time0;
        c_.time1 = time1;
    }
    const rt_camera& raw() const { return c_; }

private:
    rt_camera c_{};
};

struct scene {  // scene_manager.h:6-14; `objects` is the compiled world on one device
    std::shared_ptr<rt_scene> objects;
    color background;
    point3 lookfrom, lookat;
    double vfov = 40.0, aperture = 0.0;
    rt_scene_info info{};
};

class scene_manager {  // scene_manager.h:29-42
public:
    explicit scene_manager(std::string asset_dir, int device = 0) : assets_(std::move(asset_dir)), device_(device) {}
    // aliases "1".."9" or the scene_alias names, plus "c1", "cow", "dino" 
    scene build(const std::string& alias) const {
        rt_scene* raw = nullptr;
        const int rc = rt_scene_build(alias.c_str(), assets_.c_str(), device_, &raw);
        if (rc < 0) {
            const std::string msg = rt_last_error();
            if (msg.find("unkwnown scene requested") != std::string::npos) throw std::logic_error(msg);
            throw std::runtime_error("scene_manager::build(" + alias + "): " + msg);
        }
        return wrap(raw);
    }
    // A scene written by save_scene (rt_scene_load: the flat-scene file, no OBJ parsing, image decoding or BVH build).
    scene load(const std::string& path) const {
        rt_scene* raw = nullptr;
        check(rt_scene_load(path.c_str(), device_, &raw), "scene_manager::load");
        return wrap(raw);
    }

private:
    static scene wrap(rt_scene* raw) {
        scene s;
        s.objects = std::shared_ptr<rt_scene>(raw, rt_scene_destroy);
        check(rt_scene_info_get(raw, &s.info), "rt_scene_info_get");
        for (int k = 0; k < 3; ++k) {
            s.lookfrom.e[k] = s.info.lookfrom[k];
            s.lookat.e[k] = s.info.lookat[k];
            s.background.e[k] = s.info.background[k];
        }
        s.vfov = s.info.vfov;
        s.aperture = s.info.aperture;
        return s;
    }
    std::string assets_;
    int device_;
};

// Writes a built or loaded scene as a versioned flat-scene file (rt_scene_save); scene_manager::load reads it back.
// Process-wide library options (rt_option_set / rt_option_get: builder experiments, the RCCL deadline, test fault points)
inline void set_option(const std::string& name, double value) { check(rt_option_set(name.c_str(), value), "rt_option_set"); }
inline double get_option(const std::string& name) {
    double v = 0;
    check(rt_option_get(name.c_str(), &v), "rt_option_get");
    return v;
}
inline void save_scene(const scene& world, const std::string& path) { check(rt_scene_save(world.objects.get(), path.c_str()), "save_scene"); }

// The engine with a runtime image size (the reference fixes W, H, C at compile time: engine<W,H,C> below); samples
// per pixel and max depth are the reference's tracer_constants (tracer_constants.h:12-13) as arguments with the same
// defaults.
class render_engine {
public:
    render_engine(int width, int height, const camera& cam, engine_mode mode, int samples_per_pixel = 100, int max_depth = 50,
                  uint64_t seed = 0)
        : w_(width), h_(height), cam_(cam), mode_(mode), spp_(samples_per_pixel), max_depth_(max_depth), seed_(seed) {}

    void set_scene(const scene& world, color background) {  // engine.h:24-28
        world_ = world;
        background_ = background;
    }

    // engine.h:30-54: blocking, fills W*H*3 bytes (row 0 = top); returns the elapsed milliseconds, or -1 for an empty
    // world.  single and parallel_stripes compute the same image; adaptive traces corners and interpolates
    // (engine.h:96-333); parallel_images sums four float images of spp/4 samples (engine.h:378-445).
    int run(std::uint8_t* out) {
        if (!world_.objects || world_.info.objects == 0) {
            std::fprintf(stderr, "Invalid input scene!\n");
            return -1;
        }
        const rt_params p = params();
        const int rc = rt_render(world_.objects.get(), &cam_.raw(), &p, out, nullptr, &stats_);
        if (rc == RT_E_INVALID && mode_ == engine_mode::adaptive) throw std::logic_error(rt_last_error());
        check(rc, "engine::run");
        return static_cast<int>(stats_.ms);
    }
    // Progressive rendering (the reference's live preview, gui.cpp:25-58, headless): passes of samples_per_pass samples
    // per pixel (0: spp / 8 rounded up); after each, `on_pass(samples_done, rgb)` sees the frame write_color'ed with the
    // samples so far (in `out`); returning false stops there.  The last snapshot equals run()'s image bit for bit.
    int run_progressive(std::uint8_t* out, const std::function<bool(int samples_done, const std::uint8_t* rgb)>& on_pass,
                        int samples_per_pass = 0) {
        if (!world_.objects || world_.info.objects == 0) {
            std::fprintf(stderr, "Invalid input scene!\n");
            return -1;
        }
        rt_params p = params();
        if (p.flags & (RT_ADAPTIVE | RT_PARALLEL_IMAGES)) throw std::logic_error("engine::run_progressive: adaptive and parallel_images are not progressive");
        p.samples_per_pass = samples_per_pass;
        struct ctx_t {
            const std::function<bool(int, const std::uint8_t*)>* fn;
            std::exception_ptr err;
        } ctx{&on_pass, nullptr};
        auto tramp = [](void* user, int32_t done, int32_t, const std::uint8_t* rgb, const double*) -> int {
            auto* c = static_cast<ctx_t*>(user);
            try {
                return (*c->fn)(done, rgb) ? 0 : 1;
            } catch (...) {  // no exception crosses the C ABI: stop the render, rethrow after it returns
                c->err = std::current_exception();
                return 1;
            }
        };
        const int rc = rt_render_progressive(world_.objects.get(), &cam_.raw(), &p, out, nullptr, tramp, &ctx, &stats_);
        if (ctx.err) std::rethrow_exception(ctx.err);
        check(rc, "engine::run_progressive");
        return static_cast<int>(stats_.ms);
    }
    const rt_stats& stats() const { return stats_; }

private:
    rt_params params() const {
        rt_params p{};
        p.width = w_;
        p.height = h_;
        p.spp = spp_;
        p.max_depth = max_depth_;
        p.seed = seed_;
        p.fp_mode = RT_FP64;
        p.band_rows = h_;
        p.band_count = 1;
        p.band_index = 0;
        p.flags = mode_ == engine_mode::adaptive ? RT_ADAPTIVE : mode_ == engine_mode::parallel_images ? RT_PARALLEL_IMAGES : 0;
        for (int k = 0; k < 3; ++k) p.background[k] = background_.e[k];
        return p;
    }
    int w_, h_;
    camera cam_;
    engine_mode mode_;
    int spp_, max_depth_;
    uint64_t seed_;
    scene world_;
    color background_;
    rt_stats stats_{};
};

template <int W, int H, int C>
class engine : public render_engine {  // engine.h:19-54
    static_assert(C == 3, "libart writes RGB8 (color.h:6-22)");

public:
    engine(const camera& cam, engine_mode mode, int samples_per_pixel = 100, int max_depth = 50, uint64_t seed = 0)
        : render_engine(W, H, cam, mode, samples_per_pixel, max_depth, seed) {}
};

// The reference's CPU-parallel drivers (engine.h:335-376: row stripes on threads) over several GPUs of one process:
// the scene on every device, one RCCL communicator per device, each device rendering its row bands and one
// ncclGather assembling the frame on devices[0] (rt_render_multi).  Same image as engine::run for any device count.
class multi_engine {
public:
    multi_engine(const std::string& alias, const std::string& asset_dir, const std::vector<int>& devices, int width, int height,
                 const camera& cam, int samples_per_pixel = 100, int max_depth = 50, uint64_t seed = 0, int band_rows = 16)
        : w_(width), h_(height), cam_(cam), spp_(samples_per_pixel), max_depth_(max_depth), seed_(seed), band_rows_(band_rows) {
        rt_multi* raw = nullptr;
        check(rt_multi_create(alias.c_str(), asset_dir.c_str(), devices.data(), static_cast<int>(devices.size()), &raw), "multi_engine");
        m_ = std::shared_ptr<rt_multi>(raw, rt_multi_destroy);
    }
    void set_background(color background) { background_ = background; }
    // W*H*3 bytes of host memory, row 0 = top; returns the wall milliseconds of the call
    int run(std::uint8_t* out) {
        rt_params p{};
        p.width = w_;
        p.height = h_;
        p.spp = spp_;
        p.max_depth = max_depth_;
        p.seed = seed_;
        p.fp_mode = RT_FP64;
        p.band_rows = band_rows_;
        p.band_count = 1;
        p.band_index = 0;
        for (int k = 0; k < 3; ++k) p.background[k] = background_.e[k];
        check(rt_render_multi(m_.get(), &cam_.raw(), &p, out, &stats_), "multi_engine::run");
        return static_cast<int>(stats_.ms);
    }
    const rt_stats& stats() const { return stats_; }

private:
    std::shared_ptr<rt_multi> m_;
    int w_, h_;
    camera cam_;
    int spp_, max_depth_;
    uint64_t seed_;
    int band_rows_;
    color background_;
    rt_stats stats_{};
};

namespace imageio {  // utils/imageio.h: save_image writes a PNG (zlib deflate; stb_image_write in the reference)
// imageio::load_image (imageio.cpp:11-15, stbi_load(path, &w, &h, &c, 0)): JPEG / PNG through libart's decoder,
// the bytes stb_image v2.27 returns (rt_image_load); throws std::runtime_error on an unreadable file.
inline std::vector<std::uint8_t> load_image(const std::string& path, int& width, int& height, int& channels) {
    int32_t w = 0, h = 0, c = 0;
    std::uint8_t* px = nullptr;
    check(rt_image_load(path.c_str(), &w, &h, &c, &px), "imageio::load_image");
    std::vector<std::uint8_t> out(px, px + static_cast<size_t>(w) * h * c);
    rt_image_free(px);
    width = w;
    height = h;
    channels = c;
    return out;
}
inline bool save_image(const std::string& path, int width, int height, int bytes_per_pixel, const std::uint8_t* data) {
    const int color_type = bytes_per_pixel == 1 ? 0 : bytes_per_pixel == 2 ? 4 : bytes_per_pixel == 3 ? 2 : 6;
    std::vector<std::uint8_t> raw;
    const size_t stride = static_cast<size_t>(width) * bytes_per_pixel;
    raw.reserve((stride + 1) * height);
    for (int y = 0; y < height; ++y) {
        raw.push_back(0);  // filter: none
        raw.insert(raw.end(), data + y * stride, data + (y + 1) * stride);
    }
    uLongf zlen = compressBound(static_cast<uLong>(raw.size()));
    std::vector<std::uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), static_cast<uLong>(raw.size()), 6) != Z_OK) return false;
    z.resize(zlen);
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    auto be32 = [](std::uint32_t v) {
        return std::vector<std::uint8_t>{std::uint8_t(v >> 24), std::uint8_t(v >> 16), std::uint8_t(v >> 8), std::uint8_t(v)};
    };
    auto chunk = [&](const char* tag, const std::vector<std::uint8_t>& payload) {
        std::vector<std::uint8_t> body(tag, tag + 4);
        body.insert(body.end(), payload.begin(), payload.end());
        const auto len = be32(static_cast<std::uint32_t>(payload.size()));
        const auto crc = be32(static_cast<std::uint32_t>(crc32(0L, body.data(), static_cast<uInt>(body.size()))));
        std::fwrite(len.data(), 1, 4, f);
        std::fwrite(body.data(), 1, body.size(), f);
        std::fwrite(crc.data(), 1, 4, f);
    };
    static const std::uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::fwrite(sig, 1, 8, f);
    std::vector<std::uint8_t> ihdr = be32(static_cast<std::uint32_t>(width));
    const auto h = be32(static_cast<std::uint32_t>(height));
    ihdr.insert(ihdr.end(), h.begin(), h.end());
    ihdr.insert(ihdr.end(), {8, static_cast<std::uint8_t>(color_type), 0, 0, 0});
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
    return std::fclose(f) == 0;
}
}  // namespace imageio

}  // namespace art

#endif  // ART_ENGINE_HPP
