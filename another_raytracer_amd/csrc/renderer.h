// renderer.h — host-side device renderer (implemented in kernels.hip; no HIP types in this header).
#pragma once
#include <cstdint>
#include <functional>

#include "art.h"
#include "layout.h"
#include "scene.h"

namespace art {

struct RenderParams {
    int width = 0, height = 0, spp = 1, max_depth = 50;
    uint64_t seed = 0;
    int fp_mode = RT_FP64;
    int band_rows = 1, band_count = 1, band_index = 0;
    int samples_per_pass = 0;
    int flags = 0;
    void* stream = nullptr;
    double background[3] = {0, 0, 0};
    // Progressive rendering (whole-image traces): called after every pass with the samples traced so far, once the
    // frame write_color'ed with that count (and the sums, when requested) are in the caller's buffers; returning
    // false ends the render there.
    std::function<bool(int samples_done)> on_pass;
};

struct RenderStats {
    uint64_t segments = 0, primary = 0;
    double ms = 0, extend_ms = 0, shade_ms = 0;
    uint64_t extend_launches = 0, shade_launches = 0;
    int passes = 0, samples_per_pass = 0, local_rows = 0;
    int extend_variant = 0;
    uint32_t kernel_features = 0, kernel_textures = 0;  // the persistent kernel: k_paths_g<F, TF, LM> / k_paths (LM 3)
    int kernel_lds_mode = -1;
};

class Renderer {
public:
    struct Impl;
    Renderer(FlatScene flat, int device);
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;
    // Uploads the scene to the device now (render and trace_rays otherwise do it at their first call).
    void upload();
    void render(const CameraRec<double>& cam, const RenderParams& p, uint8_t* out_rgb, double* out_acc, RenderStats& stats);
    // Closest hit of n rays (rays: n x {ox, oy, oz, dx, dy, dz, tm}) through the renderer's traversal: t (inf on a
    // miss) and the face normal (n x 3), host buffers; global_scene forces the HBM traversal on an LDS-image scene.
    void trace_rays(const double* rays, size_t n, bool global_scene, double* t_out, double* n_out);
    size_t scene_bytes() const;
    const FlatScene& flat() const;

private:
    Impl* impl_;
};

}  // namespace art
