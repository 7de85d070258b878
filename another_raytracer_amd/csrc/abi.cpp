// abi.cpp — the extern "C" boundary (include/art.h).  No exception crosses it.
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "art.h"
#include "imagedec.h"
#include "multi.h"
#include "renderer.h"
#include "scenefile.h"
#include "objmesh.h"
#include "options.h"
#include "scene.h"

namespace art {
int device_count();  // kernels.hip
}

struct rt_scene {
    art::SceneGraph graph;       // empty for a scene loaded from a flat-scene file (has_graph false)
    bool has_graph = true;
    art::FlatScene flat;
    art::SceneView view;         // scene_manager::build's lookfrom / lookat / vfov / aperture
    int device = 0;
    std::unique_ptr<art::Renderer> renderer;  // created on first render (scene build/dump works without a GPU)
};
struct rt_graph {
    art::SceneGraph g;
};
struct rt_multi {
    art::SceneGraph graph;
    art::FlatScene flat;
    std::unique_ptr<art::MultiRenderer> renderer;
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
template <class F>
int guard(int code_on_exception, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return fail(RT_E_INTERNAL, "out of memory");
    } catch (const std::exception& e) {
        return fail(code_on_exception, e.what());
    } catch (...) {
        return fail(RT_E_INTERNAL, "unknown error");
    }
}
art::Vec3 v3(const double* p) { return art::Vec3(p[0], p[1], p[2]); }
bool valid_params(const rt_params* p, std::string& why) {
    if (!p) { why = "params is NULL"; return false; }
    if (p->width < 2 || p->height < 2) { why = "width and height must be >= 2 (u = (i + r)/(W-1), engine.h:62-63)"; return false; }
    if (p->spp < 1) { why = "spp must be >= 1"; return false; }
    if (p->max_depth < 0) { why = "max_depth must be >= 0"; return false; }
    if (p->band_rows < 1 || p->band_count < 1 || p->band_index < 0 || p->band_index >= p->band_count) {
        why = "band partition must satisfy band_rows >= 1, band_count >= 1, 0 <= band_index < band_count";
        return false;
    }
    if (p->fp_mode != RT_FP64) { why = "fp_mode must be RT_FP64 (0): the reference's double arithmetic is the only mode"; return false; }
    if (static_cast<int64_t>(p->width) * p->height > (int64_t(1) << 31)) { why = "image too large"; return false; }
    return true;
}
art::RenderParams render_params(const rt_params* p) {
    art::RenderParams rp;
    rp.width = p->width;
    rp.height = p->height;
    rp.spp = p->spp;
    rp.max_depth = p->max_depth;
    rp.seed = p->seed;
    rp.fp_mode = p->fp_mode;
    rp.band_rows = p->band_rows;
    rp.band_count = p->band_count;
    rp.band_index = p->band_index;
    rp.samples_per_pass = p->samples_per_pass;
    rp.flags = p->flags;
    rp.stream = p->stream;
    for (int c = 0; c < 3; ++c) rp.background[c] = p->background[c];
    return rp;
}
void fill_stats(const art::RenderStats& st, rt_stats* stats) {
    if (!stats) return;
    std::memset(stats, 0, sizeof *stats);
    stats->segments = st.segments;
    stats->primary = st.primary;
    stats->ms = st.ms;
    stats->extend_ms = st.extend_ms;
    stats->shade_ms = st.shade_ms;
    stats->extend_launches = st.extend_launches;
    stats->shade_launches = st.shade_launches;
    stats->passes = st.passes;
    stats->samples_per_pass = st.samples_per_pass;
    stats->local_rows = st.local_rows;
    stats->extend_variant = st.extend_variant;
    stats->kernel_features = st.kernel_features;
    stats->kernel_textures = st.kernel_textures;
    stats->kernel_lds_mode = st.kernel_lds_mode;
}
art::CameraRec<double> camera_of(const rt_camera* cam) {
    return art::make_camera(cam->lookfrom, cam->lookat, cam->vup, cam->vfov, cam->aspect, cam->aperture, cam->focus_dist, cam->time0, cam->time1);
}
int multi_from_graph(art::SceneGraph graph, const int* devices, int ngpus, rt_multi** out) {
    if (!devices || ngpus < 1) return fail(RT_E_INVALID, "devices must list ngpus >= 1 device ids");
    auto m = std::make_unique<rt_multi>();
    m->graph = std::move(graph);
    m->flat = art::compile_scene(m->graph);
    m->renderer = std::make_unique<art::MultiRenderer>(m->flat, std::vector<int>(devices, devices + ngpus));
    *out = m.release();
    return RT_OK;
}
int scene_from_graph(art::SceneGraph graph, int device, rt_scene** out) {
    auto s = std::make_unique<rt_scene>();
    s->graph = std::move(graph);
    s->flat = art::compile_scene(s->graph);
    for (int a = 0; a < 3; ++a) {
        s->view.lookfrom[a] = s->graph.lookfrom[a];
        s->view.lookat[a] = s->graph.lookat[a];
    }
    s->view.vfov = s->graph.vfov;
    s->view.aperture = s->graph.aperture;
    s->device = device;
    *out = s.release();
    return RT_OK;
}
}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
int rt_option_set(const char* name, double value) {
    if (!name) {
        art::opt_reset_all();
        return RT_OK;
    }
    const char* why = "";
    if (!art::opt_set(name, value, &why)) return fail(RT_E_INVALID, std::string("rt_option_set(") + name + "): " + why);
    return RT_OK;
}
int rt_option_get(const char* name, double* value) {
    if (!name || !value) return fail(RT_E_INVALID, "rt_option_get: name and value must be non-NULL");
    if (!art::opt_get(name, value)) return fail(RT_E_INVALID, std::string("rt_option_get(") + name + "): unknown option");
    return RT_OK;
}
const char* rt_last_error(void) { return g_err.c_str(); }
int rt_device_count(void) {
    return guard(RT_E_DEVICE, [] { return art::device_count(); });
}

int rt_scene_build(const char* name, const char* asset_dir, int device, rt_scene** out) {
    if (!name || !out) return fail(RT_E_INVALID, "name and out must be non-NULL");
    *out = nullptr;
    return guard(RT_E_SCENE, [&] {
        art::SceneGraph g;
        art::build_builtin_scene(g, name, asset_dir ? asset_dir : "assets");
        return scene_from_graph(std::move(g), device, out);
    });
}

static void fill_info(const art::SceneView& view, const art::FlatScene& flat, rt_scene_info* info) {
    std::memset(info, 0, sizeof *info);
    for (int a = 0; a < 3; ++a) {
        info->lookfrom[a] = view.lookfrom[a];
        info->lookat[a] = view.lookat[a];
        info->background[a] = flat.background[a];
    }
    info->vfov = view.vfov;
    info->aperture = view.aperture;
    info->spheres = static_cast<int64_t>(flat.spheres.size());
    info->triangles = static_cast<int64_t>(flat.tris.size());
    info->rects = static_cast<int64_t>(flat.rects.size());
    info->boxes = static_cast<int64_t>(flat.boxes.size());
    info->bvh_nodes = static_cast<int64_t>(flat.nodes.size());
    info->objects = static_cast<int64_t>(flat.world.size());
    info->materials = static_cast<int64_t>(flat.mats.size());
    info->textures = static_cast<int64_t>(flat.texs.size());
    info->has_media = flat.has_media ? 1 : 0;
    info->max_bvh_depth = flat.max_bvh_depth;
}

int rt_scene_info_get(const rt_scene* s, rt_scene_info* info) {
    if (!s || !info) return fail(RT_E_INVALID, "scene and info must be non-NULL");
    fill_info(s->view, s->flat, info);
    if (s->renderer) info->device_bytes_f64 = s->renderer->scene_bytes();
    return RT_OK;
}

size_t rt_scene_dump(const rt_scene* s, char* buf, size_t cap) {
    if (!s) {
        fail(RT_E_INVALID, "scene is NULL");
        return 0;
    }
    if (!s->has_graph) {
        fail(RT_E_INVALID, "a scene loaded from a flat-scene file has no object graph to dump");
        return 0;
    }
    try {
        std::string d = art::dump_scene(s->graph);
        if (buf && cap) {
            size_t n = std::min(cap - 1, d.size());
            std::memcpy(buf, d.data(), n);
            buf[n] = 0;
        }
        return d.size() + 1;
    } catch (const std::exception& e) {
        fail(RT_E_INTERNAL, e.what());
        return 0;
    }
}

int rt_scene_save(const rt_scene* s, const char* path) {
    if (!s || !path) return fail(RT_E_INVALID, "scene and path must be non-NULL");
    return guard(RT_E_INVALID, [&] {
        art::save_scene_file(path, s->flat, s->view);
        return RT_OK;
    });
}

int rt_scene_load(const char* path, int device, rt_scene** out) {
    if (!path || !out) return fail(RT_E_INVALID, "path and out must be non-NULL");
    *out = nullptr;
    return guard(RT_E_SCENE, [&] {
        auto s = std::make_unique<rt_scene>();
        art::load_scene_file(path, s->flat, s->view);
        s->has_graph = false;
        s->device = device;
        *out = s.release();
        return RT_OK;
    });
}

void rt_scene_destroy(rt_scene* s) {
    try {
        delete s;
    } catch (...) {
    }
}

int rt_local_rows(const rt_params* p, int32_t* rows_out) {
    if (!p || p->height < 1 || p->band_rows < 1 || p->band_count < 1 || p->band_index < 0 || p->band_index >= p->band_count)
        return fail(RT_E_INVALID, "invalid band partition");
    const int n = art::band_local_rows(p->height, p->band_rows, p->band_count, p->band_index);
    if (rows_out)
        for (int ly = 0; ly < n; ++ly) rows_out[ly] = art::band_global_row(ly, p->band_rows, p->band_count, p->band_index);
    return n;
}

int rt_band_block_rows(int32_t height, int32_t band_rows, int32_t n) {
    if (height < 1 || band_rows < 1 || n < 1) return fail(RT_E_INVALID, "height, band_rows and n must be >= 1");
    return art::band_block_rows(height, band_rows, n);
}

int rt_unpack_bands(const uint8_t* packed, size_t packed_bytes, uint8_t* frame, size_t frame_bytes, int32_t width, int32_t height,
                    int32_t band_rows, int32_t n, int32_t flags, void* stream) {
    if (!packed || !frame) return fail(RT_E_INVALID, "packed and frame must be non-NULL");
    if (width < 1 || height < 1 || band_rows < 1 || n < 1) return fail(RT_E_INVALID, "width, height, band_rows and n must be >= 1");
    if (static_cast<int64_t>(width) * height > (int64_t(1) << 31)) return fail(RT_E_INVALID, "image too large");
    const size_t row_bytes = static_cast<size_t>(width) * 3;
    const size_t want_packed = static_cast<size_t>(n) * static_cast<size_t>(art::band_block_rows(height, band_rows, n)) * row_bytes;
    const size_t want_frame = static_cast<size_t>(height) * row_bytes;
    if (packed_bytes != want_packed)
        return fail(RT_E_INVALID, "packed holds " + std::to_string(packed_bytes) + " bytes, the layout needs n * band_block_rows * width * 3 = " +
                                      std::to_string(want_packed) + " (every rank's padded block)");
    if (frame_bytes != want_frame)
        return fail(RT_E_INVALID, "frame holds " + std::to_string(frame_bytes) + " bytes, height * width * 3 = " + std::to_string(want_frame));
    return guard(RT_E_DEVICE, [&] {
        art::unpack_bands(packed, frame, width, height, band_rows, n, (flags & RT_OUT_DEVICE) != 0, stream);
        return RT_OK;
    });
}

int rt_render(rt_scene* s, const rt_camera* cam, const rt_params* p, uint8_t* out_rgb8, double* out_accum, rt_stats* stats) {
    std::string why;
    if (!s || !cam) return fail(RT_E_INVALID, "scene and camera must be non-NULL");
    if (!valid_params(p, why)) return fail(RT_E_INVALID, why);
    if ((p->flags & RT_ADAPTIVE) && (p->flags & RT_PARALLEL_IMAGES)) return fail(RT_E_INVALID, "RT_ADAPTIVE and RT_PARALLEL_IMAGES are two engine modes");
    if (p->flags & RT_ADAPTIVE) {
        const int rows = rt_local_rows(p, nullptr);
        if (p->width % 12 != 0 || rows % 12 != 0 || (p->band_count > 1 && p->band_rows % 12 != 0))
            return fail(RT_E_INVALID, "for adaptive strategy image size should perfectly fit big square size for now!! (engine.h:178-179: "
                                      "width and local rows multiples of 12, band_rows a multiple of 12 when bands are interleaved)");
        if (out_accum) return fail(RT_E_INVALID, "adaptive mode has no per-pixel radiance sums: out_accum must be NULL");
    }
    return guard(RT_E_DEVICE, [&] {
        if (!s->renderer) s->renderer = std::make_unique<art::Renderer>(s->flat, s->device);
        art::RenderStats st;
        s->renderer->render(camera_of(cam), render_params(p), out_rgb8, out_accum, st);
        fill_stats(st, stats);
        return RT_OK;
    });
}

int rt_render_progressive(rt_scene* s, const rt_camera* cam, const rt_params* p, uint8_t* out_rgb8, double* out_accum, rt_progress_fn cb,
                          void* user, rt_stats* stats) {
    std::string why;
    if (!s || !cam || !cb || !out_rgb8) return fail(RT_E_INVALID, "scene, camera, callback and out_rgb8 must be non-NULL");
    if (!valid_params(p, why)) return fail(RT_E_INVALID, why);
    if (p->flags & (RT_ADAPTIVE | RT_PARALLEL_IMAGES))
        return fail(RT_E_INVALID, "progressive rendering traces whole frames of consecutive samples (no RT_ADAPTIVE or RT_PARALLEL_IMAGES)");
    return guard(RT_E_DEVICE, [&] {
        if (!s->renderer) s->renderer = std::make_unique<art::Renderer>(s->flat, s->device);
        art::RenderParams rp = render_params(p);
        if (rp.samples_per_pass <= 0) rp.samples_per_pass = (rp.spp + 7) / 8;
        const int spp = rp.spp;
        rp.on_pass = [&](int done) { return cb(user, done, spp, out_rgb8, out_accum) == 0; };
        art::RenderStats st;
        s->renderer->render(camera_of(cam), rp, out_rgb8, out_accum, st);
        fill_stats(st, stats);
        return RT_OK;
    });
}

int rt_trace_rays(rt_scene* s, const double* rays, int64_t n, int32_t flags, double* t_out, double* normal_out) {
    if (!s || n < 0 || (n > 0 && (!rays || !t_out))) return fail(RT_E_INVALID, "scene, rays and t_out must be non-NULL, n >= 0");
    return guard(RT_E_DEVICE, [&] {
        if (!s->renderer) s->renderer = std::make_unique<art::Renderer>(s->flat, s->device);
        std::vector<double> nrm(normal_out ? 0 : 3 * static_cast<size_t>(n));
        s->renderer->trace_rays(rays, static_cast<size_t>(n), (flags & RT_GLOBAL_SCENE) != 0, t_out, normal_out ? normal_out : nrm.data());
        return RT_OK;
    });
}

int rt_image_load(const char* path, int32_t* width, int32_t* height, int32_t* channels, uint8_t** pixels) {
    if (!path || !width || !height || !channels || !pixels) return fail(RT_E_INVALID, "NULL argument");
    *pixels = nullptr;
    return guard(RT_E_INVALID, [&] {
        art::DecodedImage d = art::load_image_file(path);
        uint8_t* p = static_cast<uint8_t*>(std::malloc(d.data.size()));
        if (!p) throw std::bad_alloc();
        std::memcpy(p, d.data.data(), d.data.size());
        *width = d.w;
        *height = d.h;
        *channels = d.channels;
        *pixels = p;
        return RT_OK;
    });
}
void rt_image_free(uint8_t* pixels) { std::free(pixels); }

// ---------------------------------------------------------------------------------------------- multi-GPU
int rt_multi_create(const char* name, const char* asset_dir, const int* devices, int ngpus, rt_multi** out) {
    if (!name || !out) return fail(RT_E_INVALID, "name and out must be non-NULL");
    *out = nullptr;
    art::SceneGraph g;
    const int rc = guard(RT_E_SCENE, [&] {
        art::build_builtin_scene(g, name, asset_dir ? asset_dir : "assets");
        return RT_OK;
    });
    if (rc != RT_OK) return rc;
    return guard(RT_E_DEVICE, [&] { return multi_from_graph(std::move(g), devices, ngpus, out); });
}
int rt_multi_from_graph(rt_graph* g, const int* devices, int ngpus, rt_multi** out) {
    if (!g || !out) return fail(RT_E_INVALID, "graph and out must be non-NULL");
    *out = nullptr;
    return guard(RT_E_DEVICE, [&] { return multi_from_graph(g->g, devices, ngpus, out); });
}
void rt_multi_destroy(rt_multi* m) {
    try {
        delete m;
    } catch (...) {
    }
}
int rt_render_multi(rt_multi* m, const rt_camera* cam, const rt_params* p, uint8_t* out_rgb8, rt_stats* stats) {
    std::string why;
    if (!m || !cam || !out_rgb8) return fail(RT_E_INVALID, "multi, camera and out_rgb8 must be non-NULL");
    if (!valid_params(p, why)) return fail(RT_E_INVALID, why);
    if (p->flags & RT_ADAPTIVE) return fail(RT_E_INVALID, "rt_render_multi renders engine_mode::single frames (no RT_ADAPTIVE)");
    return guard(RT_E_DEVICE, [&] {
        art::RenderStats st;
        m->renderer->render(camera_of(cam), render_params(p), out_rgb8, (p->flags & RT_OUT_DEVICE) != 0, st);
        fill_stats(st, stats);
        return RT_OK;
    });
}

int rt_multi_device_stats(const rt_multi* m, int k, rt_stats* stats) {
    if (!m || !stats) return fail(RT_E_INVALID, "multi and stats must be non-NULL");
    art::RenderStats st;
    if (!m->renderer->device_stats(k, st)) return fail(RT_E_INVALID, "no such device index, or no render yet");
    fill_stats(st, stats);
    return RT_OK;
}
int rt_multi_scene_info(const rt_multi* m, rt_scene_info* info) {
    if (!m || !info) return fail(RT_E_INVALID, "multi and info must be non-NULL");
    art::SceneView view;
    for (int a = 0; a < 3; ++a) {
        view.lookfrom[a] = m->graph.lookfrom[a];
        view.lookat[a] = m->graph.lookat[a];
    }
    view.vfov = m->graph.vfov;
    view.aperture = m->graph.aperture;
    fill_info(view, m->flat, info);
    info->device_bytes_f64 = m->renderer->scene_bytes();
    return RT_OK;
}
int rt_multi_times_get(const rt_multi* m, rt_multi_times* out) {
    if (!m || !out) return fail(RT_E_INVALID, "multi and out must be non-NULL");
    const art::MultiTimes& t = m->renderer->times();
    std::memset(out, 0, sizeof *out);
    out->total_ms = t.total_ms;
    out->render_ms_max = t.render_ms_max;
    out->render_ms_min = t.render_ms_min;
    out->gather_ms = t.gather_ms;
    out->unpack_ms = t.unpack_ms;
    out->wait_ms = t.wait_ms;
    out->collectives = t.collectives;
    out->slowest_device = t.slowest_device;
    out->ngpus = t.ngpus;
    return RT_OK;
}
int rt_multi_ngpus(const rt_multi* m) {
    if (!m) return fail(RT_E_INVALID, "multi is NULL");
    return m->renderer->ngpus();
}

// ---------------------------------------------------------------------------------------------- graph builder
rt_graph* rt_graph_new(void) {
    try {
        return new rt_graph();
    } catch (...) {
        fail(RT_E_INTERNAL, "out of memory");
        return nullptr;
    }
}
void rt_graph_free(rt_graph* g) { delete g; }

#define GRAPH_CALL(expr)                                                \
    do {                                                                \
        if (!g) return fail(RT_E_INVALID, "graph is NULL");             \
        return guard(RT_E_INVALID, [&] { return static_cast<int>(expr); }); \
    } while (0)

namespace {
void check_tex(const rt_graph* g, int t) {
    if (t < 0 || t >= static_cast<int>(g->g.textures.size())) throw std::runtime_error("bad texture id");
}
void check_mat(const rt_graph* g, int m) {
    if (m < 0 || m >= static_cast<int>(g->g.materials.size())) throw std::runtime_error("bad material id");
}
void check_obj(const rt_graph* g, int o) {
    if (o < 0 || o >= static_cast<int>(g->g.nodes.size())) throw std::runtime_error("bad object id");
}
std::vector<int> items_of(const rt_graph* g, int n, const int* items) {
    if (n < 0 || (n > 0 && !items)) throw std::runtime_error("bad item list");
    std::vector<int> v(items, items + n);
    for (int o : v) check_obj(g, o);
    return v;
}
}  // namespace

int rt_graph_random_double(rt_graph* g, double* out) {
    if (!g || !out) return fail(RT_E_INVALID, "graph/out is NULL");
    *out = g->g.rng.d();
    return RT_OK;
}
int rt_tex_solid(rt_graph* g, double r, double gr, double b) { GRAPH_CALL(g->g.solid(art::Vec3(r, gr, b))); }
int rt_tex_checker(rt_graph* g, int even, int odd) {
    GRAPH_CALL((check_tex(g, even), check_tex(g, odd), g->g.checker(even, odd)));
}
int rt_tex_noise(rt_graph* g, double scale) { GRAPH_CALL(g->g.noise(scale)); }
int rt_tex_image(rt_graph* g, int w, int h, int bpp, const uint8_t* texels) {
    GRAPH_CALL(([&] {
        if (w <= 0 || h <= 0 || bpp < 3 || !texels) throw std::runtime_error("bad image");
        art::Image im;
        im.w = w;
        im.h = h;
        im.bpp = bpp;
        im.data.assign(texels, texels + static_cast<size_t>(w) * h * bpp);
        return g->g.image(std::move(im));
    }()));
}
int rt_tex_bary_image(rt_graph* g, const double uv[6], int image_tex) {
    GRAPH_CALL(([&] {
        if (!uv) throw std::runtime_error("uv is NULL");
        check_tex(g, image_tex);
        if (g->g.textures[image_tex].type != art::TEX_IMAGE) throw std::runtime_error("image_tex must be an rt_tex_image texture");
        return g->g.bary_image(uv[0], uv[1], uv[2], uv[3], uv[4], uv[5], image_tex);
    }()));
}
int rt_mesh_parse(const char* obj_path, int64_t* triangles, int64_t* shapes) {
    if (!obj_path) return fail(RT_E_INVALID, "obj_path is NULL");
    return guard(RT_E_SCENE, [&] {
        const art::ObjMesh m = art::load_obj(obj_path);
        if (triangles) *triangles = static_cast<int64_t>(m.tri.size() / 3);
        if (shapes) *shapes = static_cast<int64_t>(m.shapes);
        return RT_OK;
    });
}
int rt_mesh_build(rt_graph* g, const char* obj_path, int* first_id) {
    if (!g || !obj_path) return fail(RT_E_INVALID, "graph/obj_path is NULL");
    return guard(RT_E_SCENE, [&] {
        const std::vector<int> ids = art::build_mesh(g->g, art::load_obj(obj_path));
        if (first_id) *first_id = ids.empty() ? static_cast<int>(g->g.nodes.size()) : ids.front();
        return static_cast<int>(ids.size());
    });
}
int rt_mat_lambertian(rt_graph* g, int tex) { GRAPH_CALL((check_tex(g, tex), g->g.lambertian(tex))); }
int rt_mat_metal(rt_graph* g, double r, double gr, double b, double fuzz) { GRAPH_CALL(g->g.metal(art::Vec3(r, gr, b), fuzz)); }
int rt_mat_dielectric(rt_graph* g, double ir) { GRAPH_CALL(g->g.dielectric(ir)); }
int rt_mat_diffuse_light(rt_graph* g, int tex) { GRAPH_CALL((check_tex(g, tex), g->g.diffuse_light(tex))); }
int rt_obj_sphere(rt_graph* g, const double c[3], double r, int mat) { GRAPH_CALL((check_mat(g, mat), g->g.sphere(v3(c), r, mat))); }
int rt_obj_moving_sphere(rt_graph* g, const double c0[3], const double c1[3], double t0, double t1, double r, int mat) {
    GRAPH_CALL((check_mat(g, mat), g->g.moving_sphere(v3(c0), v3(c1), t0, t1, r, mat)));
}
int rt_obj_triangle(rt_graph* g, const double p1[3], const double p2[3], const double p3[3], int mat) {
    GRAPH_CALL((check_mat(g, mat), g->g.triangle(v3(p1), v3(p2), v3(p3), mat)));
}
int rt_obj_rect(rt_graph* g, int axis, double a0, double a1, double b0, double b1, double k, int mat) {
    GRAPH_CALL(([&] {
        if (axis < 0 || axis > 2) throw std::runtime_error("rect axis must be 0 (xy), 1 (xz) or 2 (yz)");
        check_mat(g, mat);
        return g->g.rect(axis, a0, a1, b0, b1, k, mat);
    }()));
}
int rt_obj_box(rt_graph* g, const double p0[3], const double p1[3], int mat) { GRAPH_CALL((check_mat(g, mat), g->g.box(v3(p0), v3(p1), mat))); }
int rt_obj_list(rt_graph* g, int n, const int* items) { GRAPH_CALL(g->g.list(items_of(g, n, items))); }
int rt_obj_bvh(rt_graph* g, int n, const int* items) { GRAPH_CALL(g->g.bvh(items_of(g, n, items))); }
int rt_obj_translate(rt_graph* g, int child, const double offset[3]) { GRAPH_CALL((check_obj(g, child), g->g.translate(child, v3(offset)))); }
int rt_obj_rotate_y(rt_graph* g, int child, double degrees) { GRAPH_CALL((check_obj(g, child), g->g.rotate_y(child, degrees))); }
int rt_obj_constant_medium(rt_graph* g, int boundary, double density, int tex) {
    GRAPH_CALL((check_obj(g, boundary), check_tex(g, tex), g->g.constant_medium(boundary, density, tex)));
}
int rt_graph_add_world(rt_graph* g, int obj) {
    GRAPH_CALL((check_obj(g, obj), g->g.world.push_back(obj), static_cast<int>(g->g.world.size()) - 1));
}
int rt_graph_clear_world(rt_graph* g) {
    if (!g) return fail(RT_E_INVALID, "graph is NULL");
    g->g.world.clear();
    return RT_OK;
}
int rt_graph_set_view(rt_graph* g, const double lookfrom[3], const double lookat[3], double vfov, double aperture, const double background[3]) {
    if (!g || !lookfrom || !lookat || !background) return fail(RT_E_INVALID, "NULL argument");
    g->g.lookfrom = v3(lookfrom);
    g->g.lookat = v3(lookat);
    g->g.vfov = vfov;
    g->g.aperture = aperture;
    g->g.background = v3(background);
    return RT_OK;
}
int rt_graph_compile(rt_graph* g, int device, rt_scene** out) {
    if (!g || !out) return fail(RT_E_INVALID, "graph and out must be non-NULL");
    *out = nullptr;
    return guard(RT_E_SCENE, [&] { return scene_from_graph(g->g, device, out); });
}

}  // extern "C"
