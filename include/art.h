/* include/art.h — C ABI of the MI355X path tracer (libart.so).
 *
 * Drop-in boundary for the hot path of blackccpie/another_raytracer: what `src/main.cpp:29-46` does with the
 * reference's scene_manager / camera / engine classes maps onto these calls.  Plain pointers and sizes only; no C++,
 * torch or HIP types cross this boundary (a hipStream_t travels as void*).  No exceptions cross it: every call returns
 * RT_OK (0) or a negative RT_E* code, with a message in rt_last_error() (thread-local).
 *
 *   reference (file:line)                                        replacement
 *   scene scene_manager::build(scene_alias)  scene_manager.cpp:260  rt_scene_build(name, assets, device, &scene)
 *   struct scene {lookfrom, lookat, vfov, aperture, background}   rt_scene_info(scene, &info)
 *     scene_manager.h:6-14
 *   camera::camera(lookfrom, lookat, vup, vfov, aspect, aperture, rt_camera (POD, same 9 arguments)
 *     focus_dist, t0, t1)                camera.h:8-36
 *   engine<W,H,C>(const camera&, engine_mode)  engine.h:22        rt_params (W, H, spp, max_depth are runtime here:
 *   engine::set_scene(hittable_list, color)   engine.h:24-28       tracer_constants.h:6-14 made them compile-time)
 *   int engine::run(uint8_t* out)             engine.h:30-54      rt_render(scene, &cam, &params, out_rgb8, ...)
 *   write_color (gamma 2, clamp, quantize)    color.h:6-22        inside rt_render (f64 sums -> RGB8, row 0 = top)
 *   hittable constructors (sphere.h, moving_sphere.h, triangle.h, rt_graph_* (one call per constructor, same
 *     aarect.h, box.h, hittable_list.h, bvh.h, hittable.h,          arguments); rt_graph_compile -> rt_scene
 *     constant_medium.h, material.h, texture.h)
 *   bool mesh::parse(path)                    mesh.h:31-65        rt_mesh_parse(path, &triangles, &shapes)
 *   hittable_list mesh::build()               mesh.h:67-145       rt_mesh_build(graph, path, &first_id)
 *   imageio::load_image (stbi_load)          imageio.cpp:11-15   rt_image_load(path, &w, &h, &c, &pixels)
 *   engine::_run_parallel_stripes (threads)  engine.h:335-376    rt_multi_create + rt_render_multi (GPUs, RCCL)
 *   dynamic_gui refresh per row / square     gui.cpp:25-58,      rt_render_progressive(..., callback, user, ...)
 *                                            engine.h:88,307,353
 *   hittable_list::hit(r, 0.001, inf, rec)   hittable_list.cpp:5 rt_trace_rays(scene, rays, n, flags, t, normals)
 *   (scene construction every run)           scene_manager.cpp,  rt_scene_save / rt_scene_load (flat-scene files)
 *                                            mesh.h, bvh.cpp
 *
 * RNG contract: the reference draws from one global std::mt19937 (tracer_utils.h:27-31).  Scene construction here
 * replays that generator exactly (seed 5489, same draw order), so scenes are bit-identical.  Rendering draws come
 * from PCG32 streams keyed by (seed, global pixel j*W+i, sample index): results depend on neither the tiling nor the
 * GPU count, and oracle/restate.cpp (ORC_PCG) replays the same streams on the CPU.
 */
#ifndef ART_H
#define ART_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2: rt_params.fp_mode 0 = RT_FP64 (the only arithmetic: the reference's IEEE double), rt_scene_info's f32 byte count
 * dropped, rt_multi_* (multi-GPU render over RCCL), rt_render_progressive, rt_scene_save / rt_scene_load, rt_image_load.
 * ABI 3 (additive): rt_band_block_rows, rt_unpack_bands (the gather layout for callers that move the bands themselves,
 * e.g. one process per GPU over torch.distributed), rt_multi_ngpus, rt_multi_scene_info, rt_multi_device_stats.
 * ABI 4: rt_unpack_bands takes the byte sizes of both buffers and refuses a mismatch with the layout; rt_multi_times
 * (per-phase timing of the last rt_render_multi: renders, gather, unpack); rt_render_multi bounds its wait on the
 * collective (RT_E_DEVICE on an RCCL error or timeout, after which the rt_multi refuses further renders).
 * ABI 5: rt_option_set / rt_option_get (process-wide options; the library reads no environment knobs but the documented
 * ART_MULTI_TIMEOUT_MS); rt_stats.kernel_features / kernel_textures / kernel_lds_mode name the persistent kernel a
 * render ran; rt_multi_create uploads the scene to every device before it returns. */
#define RT_ABI_VERSION 5

/* return codes */
#define RT_OK 0
#define RT_E_INVALID (-1)   /* bad argument */
#define RT_E_SCENE (-2)     /* scene build / compile failure (e.g. "Invalid input scene!", engine.h:32-36) */
#define RT_E_DEVICE (-3)    /* HIP runtime failure or no device */
#define RT_E_INTERNAL (-4)

/* rt_params.fp_mode: arithmetic of the leaf tests and shading.  RT_FP64 (= 0, so a zero-initialised rt_params gets it)
 * is the reference's own IEEE double and the only mode: ABI 1's experimental RT_FP32 self-intersected on the
 * reference's r = 1000 / r = 5000 spheres and is gone (any other value is RT_E_INVALID).  The BVH box tests are
 * conservative f32 in every mode; they never decide a hit. */
#define RT_FP64 0
/* rt_params.flags */
#define RT_OUT_DEVICE 1     /* out_rgb8 / out_accum are device pointers (on the scene's device) */
#define RT_PROFILE 2        /* time every extend/shade launch with HIP events (rt_stats.*_ms) */
#define RT_GLOBAL_SCENE 4   /* never use the LDS-resident scene variant of the extend kernel (A/B and parity tests) */
#define RT_SPLIT_SHADE 8    /* never fuse shading into the extend kernel: one k_shade launch per material (A/B, tests) */
#define RT_ADAPTIVE 16      /* engine_mode::adaptive (engine.h:96-333): trace the corners of 12/6/3-px squares, subdivide
                               where neighbouring corners differ by > 100 (squared gamma-corrected RGB), interpolate
                               the rest.  Width and local rows must be multiples of 12 (the reference throws
                               std::logic_error otherwise: RT_E_INVALID here), band_rows a multiple of 12 when
                               band_count > 1, and out_accum NULL (interpolated pixels have no radiance sums). */
#define RT_WAVEFRONT 32     /* LDS-scene renders: one fused extend launch per bounce depth (paths stored in HBM between
                               bounces) instead of the persistent-path kernel (A/B and parity tests) */
#define RT_PARALLEL_IMAGES 64 /* engine_mode::parallel_images (engine.h:378-445): four partial images of spp/4 samples
                               each (samples [q*spp/4, (q+1)*spp/4) of every pixel's streams), every pixel's partial
                               sum rounded to float (write_color_raw<float>), the four summed in double and written
                               with the full spp -- the reference's float rounding and its spp/4 truncation included.
                               out_accum receives that sum.  Not with RT_ADAPTIVE or progressive rendering. */

typedef struct rt_scene rt_scene;
typedef struct rt_graph rt_graph;

typedef struct rt_camera {      /* camera.h:8-18 constructor arguments */
    double lookfrom[3];
    double lookat[3];
    double vup[3];
    double vfov;                /* vertical field of view, degrees */
    double aspect;              /* aspect ratio (the reference hard-codes 4:3 in main.cpp:35) */
    double aperture;
    double focus_dist;          /* main.cpp:34 uses 10 */
    double time0, time1;        /* shutter; main.cpp:35 uses 0, 1 */
} rt_camera;

typedef struct rt_params {
    int32_t width, height;      /* full image */
    int32_t spp;                /* samples per pixel (tracer_constants.h:12) */
    int32_t max_depth;          /* bounce limit (tracer_constants.h:13; 50) */
    uint64_t seed;              /* render RNG seed */
    int32_t fp_mode;            /* RT_FP64 (0) */
    int32_t band_rows;          /* row-interleaved partition: global row y belongs to band (y / band_rows) and */
    int32_t band_count;         /*   is rendered here when band % band_count == band_index; (H, 1, 0) = whole image */
    int32_t band_index;
    int32_t samples_per_pass;   /* 0 = auto: the largest pass whose path state fits half of the free device memory */
    int32_t flags;              /* RT_OUT_DEVICE | RT_PROFILE | RT_GLOBAL_SCENE */
    void* stream;               /* hipStream_t to run on, or NULL for the scene's own stream */
    double background[3];       /* engine::set_scene(world, background) (engine.h:24-28): returned on a miss */
} rt_params;

typedef struct rt_stats {
    uint64_t segments;          /* rays traced through the world (world.hit calls): the metric's unit */
    uint64_t primary;           /* camera rays = local pixels * spp */
    double ms;                  /* device time, first kernel -> finalized RGB8 (HIP events) */
    double extend_ms, shade_ms; /* RT_PROFILE only: summed launch durations */
    uint64_t extend_launches, shade_launches;
    int32_t passes, samples_per_pass, local_rows;
    int32_t extend_variant;     /* 0: scene read from HBM; 1: LDS-resident scene (spheres-only scene that fits);
                                   2: LDS-resident scene with shading fused into the extend kernel (one launch per
                                   depth); 3: persistent paths (the fused bounce loop in registers, one launch per pass);
                                   4: persistent paths over the HBM scene (every other scene; k_paths_g) */
    uint32_t kernel_features;   /* the persistent kernel that ran (variants 3, 4): k_paths_g<kernel_features, */
    uint32_t kernel_textures;   /*   kernel_textures, kernel_lds_mode> (layout.h feature / texture bits; LDS mode 0: BVH */
    int32_t kernel_lds_mode;    /*   in HBM, 1: whole BVH in LDS, 2: its top levels in LDS), or k_paths (LDS mode 3, the */
                                /*   LDS scene image); -1 for the per-depth wavefront variants */
} rt_stats;

typedef struct rt_scene_info {  /* scene_manager.h:6-14 */
    double lookfrom[3], lookat[3];
    double vfov, aperture;
    double background[3];
    int64_t spheres, triangles, rects, boxes, bvh_nodes, objects, materials, textures;
    int32_t has_media, max_bvh_depth;
    uint64_t device_bytes_f64;  /* scene bytes uploaded to the device (0 before the first render) */
} rt_scene_info;

/* ---- library ---- */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(void);
/* Process-wide options, by name (every one is also readable with rt_option_get).  The library reads no environment
 * variables for them (only multi.timeout_ms falls back to ART_MULTI_TIMEOUT_MS while never set).  Unknown names and
 * values outside an option's range are RT_E_INVALID; name NULL resets every option to its default.
 *   compile.world_merge (2: 0 off, 1 BVH runs only), compile.hoist (1), bvh.collapse (0 greedy, 1 SAH-optimal DP),
 *   bvh.collapse_ci (0.6), bvh.dp_binary_leaf (1), bvh.sah_ci (1.5), bvh.sah_leaf (4), bvh.sbvh (1.5), bvh.sbvh_alpha
 *   (1e-5): scene compilation, for scenes built after the call (builder experiments; the defaults are what was measured
 *   best);
 *   render.codes16 (1; 0 = always the 32-bit-child-code kernels), render.leaf2 (1; 0 = no pair-aligned leaves: a mesh
 *   of more than 8192 references takes the 32-bit-code kernels), render.tex_bary (1; 0 = meshes whose only images are
 *   barycentric take the all-textures kernels), render.lds_nodes_max (diagnostic cap on LDS nodes): uploads and
 *   renders after the call (kernel-selection switches for A/B; images are identical either way);
 *   multi.timeout_ms (the RCCL deadline; inf = none), multi.rccl_blocking (0; 1 = blocking communicators, diagnosis:
 *   gives up the deadline and the error-path protection);
 *   test.fault_workspace_bytes (0 = off; N refuses workspace growth beyond N bytes), test.fault_gather_abort (0; 1 = the
 *   next gather fails in flight), test.fault_rccl_group (0; 1 / 2 = an error inside rt_multi_create's / the gather's
 *   RCCL group): fault points for the tests, each failing a later call exactly as the real fault would. */
int rt_option_set(const char* name, double value);
int rt_option_get(const char* name, double* value);

/* ---- scenes ---- */
/* Builtin scenes = scene_manager::build(alias): "1".."8" or "random", "two_spheres", "two_perlin_spheres", "earth",
 * "simple_light", "cornell_box", "cornell_smoke", "final"; plus "c1" (SURVEY Q7 3-sphere scene), "cow", "dino"
 * (SURVEY Q8 mesh scenes) and "9"/"mesh" (the capsule, the reference's default scene).  asset_dir holds earthmap.jpg
 * and models/{cow.obj, dino.obj, capsule/capsule.obj + .mtl + capsule.jpg}; images are decoded by rt_image_load's
 * decoder. */
int rt_scene_build(const char* name, const char* asset_dir, int device, rt_scene** out);
int rt_scene_info_get(const rt_scene* scene, rt_scene_info* info);
/* Canonical JSON of the scene graph (schema of oracle/ref_harness `dump`); returns the size needed incl. NUL. */
size_t rt_scene_dump(const rt_scene* scene, char* buf, size_t cap);
void rt_scene_destroy(rt_scene* scene);
/* Versioned flat-scene files (csrc/scenefile.h): the compiled scene -- primitive records, SAH BVH4, objects, materials,
 * textures and decoded texels, plus the scene_manager view -- written once and loaded (mmap) without re-parsing OBJ/MTL,
 * re-decoding images or rebuilding the BVH (the reference rebuilds every run: scene_manager.cpp:260-355, mesh.h:31-145,
 * bvh.cpp:3-42).  A loaded scene renders bit-identically to the one saved; it has no object graph (rt_scene_dump
 * fails).  Wrong magic, version, record layout, size or checksum: RT_E_SCENE with the reason. */
int rt_scene_save(const rt_scene* scene, const char* path);
int rt_scene_load(const char* path, int device, rt_scene** out);

/* ---- render (engine::run; the engine_mode is in rt_params.flags: RT_ADAPTIVE, RT_PARALLEL_IMAGES, or neither for
 * single and parallel_stripes, which compute the same image) ----
 * out_rgb8: local_rows * width * 3 bytes (row-major, local row 0 = the first row this band set owns, top-most first);
 * out_accum (optional): local_rows * width * 3 f64 radiance sums (pixel_color before write_color).  Host pointers
 * unless RT_OUT_DEVICE.  Blocking. */
int rt_render(rt_scene* scene, const rt_camera* cam, const rt_params* params, uint8_t* out_rgb8, double* out_accum, rt_stats* stats);
/* Progressive rendering: the headless replacement for the reference's live preview (dynamic_gui_impl refreshed after
 * every row / square, gui.cpp:25-58, engine.h:88,307,353).  The frame is traced in passes of params->samples_per_pass
 * samples per pixel (0: ceil(spp / 8)); after each pass `cb` gets the samples traced so far and the frame write_color'ed
 * with that count, already in out_rgb8 (and the f64 sums in out_accum when non-NULL).  A non-zero return from `cb`
 * stops the render there (RT_OK; stats->primary counts the samples traced).  Every snapshot equals rt_render of that
 * many samples bit for bit, the last one rt_render's whole frame.  No RT_ADAPTIVE. */
typedef int (*rt_progress_fn)(void* user, int32_t samples_done, int32_t spp, const uint8_t* rgb8, const double* accum);
int rt_render_progressive(rt_scene* scene, const rt_camera* cam, const rt_params* params, uint8_t* out_rgb8, double* out_accum,
                          rt_progress_fn cb, void* user, rt_stats* stats);
/* Ray queries: the world's closest hit (hittable_list::hit, hittable_list.cpp:5-19, t in [0.001, inf)) of n rays
 * given as n x {ox, oy, oz, dx, dy, dz, time} doubles, through the renderer's own BVH traversal (the LDS scene image when
 * the scene has one, unless flags has RT_GLOBAL_SCENE).  t_out: n hit distances (+inf on a miss); normal_out (may be
 * NULL): n x 3 face normals as hit_record holds them (set_face_normal, hittable.h:18-22), 0 on a miss.  Ray i draws
 * its constant_medium uniforms from the PCG stream keyed (seed 0, pixel i, sample 0).  Host buffers; blocking. */
int rt_trace_rays(rt_scene* scene, const double* rays, int64_t n, int32_t flags, double* t_out, double* normal_out);
/* Number of rows a band partition owns, and optionally their global indices (rows_out may be NULL).  Global row y
 * belongs to band set (y / band_rows) % band_count; local row ly of set r is global row
 * (ly / band_rows) * band_rows * band_count + r * band_rows + ly % band_rows. */
int rt_local_rows(const rt_params* params, int32_t* rows_out);
/* Gather layout of an n-way band partition (what rt_render_multi's ncclGather moves): every band set sends one block of
 * rt_band_block_rows(height, band_rows, n) rows (the largest set's row count; a shorter set pads after its rows).
 * rt_unpack_bands places the n concatenated blocks (packed: n * block_rows * width * 3 bytes, block r = set r's rows in
 * local order) into the height-row frame (row 0 = top): device pointers and a kernel on `stream` (hipStream_t, NULL =
 * default) with RT_OUT_DEVICE, else host memory.  packed_bytes / frame_bytes are the sizes of the two buffers: unless
 * they are exactly n * block_rows * width * 3 and height * width * 3 the call is refused (RT_E_INVALID) before any byte
 * moves.  Replaces the reference's in-place stripe writes into one frame (engine.h:343-355). */
int rt_band_block_rows(int32_t height, int32_t band_rows, int32_t n);
int rt_unpack_bands(const uint8_t* packed, size_t packed_bytes, uint8_t* frame, size_t frame_bytes, int32_t width, int32_t height,
                    int32_t band_rows, int32_t n, int32_t flags, void* stream);

/* ---- images (imageio::load_image, imageio.cpp:11-15: stbi_load(path, &w, &h, &c, 0) of stb_image v2.27) ----
 * Decodes a JPEG (baseline or progressive) or PNG file to 8-bit samples, native channel count, row 0 = top, the bytes
 * stb_image returns (the JPEG inverse DCT, color transform and chroma upsampling follow its arithmetic).  *pixels is
 * allocated by the library (h * w * channels bytes); release it with rt_image_free.  image_texture (texture.h:67-118)
 * and map_Kd textures load their files through this decoder. */
int rt_image_load(const char* path, int32_t* width, int32_t* height, int32_t* channels, uint8_t** pixels);
void rt_image_free(uint8_t* pixels);

/* ---- multi-GPU (one process, one host thread per GPU, RCCL) ----
 * Replaces the reference's CPU-parallel drivers (engine.h:335-376 _run_parallel_stripes: 4 threads on 4 row stripes;
 * SURVEY.md §8(b) rt_render_multi).  An rt_multi holds the scene uploaded on every listed device and one RCCL
 * communicator per device (one group of ncclCommInitRankConfig, non-blocking), both made at creation: the first
 * rt_render_multi spends no time on the upload (the reference times engine::run only, main.cpp:44-46; the pass
 * workspace, sized by the render's W, H and spp, is still allocated by the first render of a size).
 * rt_render_multi renders the whole frame: device k
 * renders the row bands b (params->band_rows rows each) with b % ngpus == k -- params->band_count / band_index are
 * ignored -- packs them into one buffer, and a single ncclGather moves every device's block to devices[0], whose unpack
 * kernel writes the rows in image order.  out_rgb8: W*H*3 bytes, row 0 = top; host memory, or device memory on
 * devices[0] with RT_OUT_DEVICE.  The image is bit-identical to rt_render's for any device count (the RNG is keyed by
 * (seed, global pixel, sample)).  stats: segments/primary summed over the devices, ms = host wall time of the call.
 * Threading: one rt_multi per process at a time per device set; calls are blocking.
 * Failure behaviour: a device whose render fails makes the call return that error before any collective starts (the
 * rt_multi stays usable).  The communicators are non-blocking (ncclConfig_t.blocking = 0); their creation and the
 * gather are polled (ncclCommGetAsyncError, hipStreamQuery) against a deadline of multi.timeout_ms milliseconds
 * (rt_option_set; while unset, the environment's ART_MULTI_TIMEOUT_MS, default 120000).  An RCCL error or an expired
 * deadline aborts every communicator (ncclCommAbort) and returns RT_E_DEVICE; the rt_multi then refuses renders until
 * it is destroyed and created again.  Both RCCL groups (creation, gather) are closed on every error path and the
 * communicators aborted, so a failure never leaves the calling thread inside an open ncclGroupStart. */
typedef struct rt_multi rt_multi;
int rt_multi_create(const char* name, const char* asset_dir, const int* devices, int ngpus, rt_multi** out);
int rt_multi_from_graph(rt_graph* g, const int* devices, int ngpus, rt_multi** out);
void rt_multi_destroy(rt_multi* m);
int rt_render_multi(rt_multi* m, const rt_camera* cam, const rt_params* params, uint8_t* out_rgb8, rt_stats* stats);
int rt_multi_ngpus(const rt_multi* m);
/* The scene_manager view and sizes of the multi's scene (as rt_scene_info_get; device_bytes_f64 = bytes on each device). */
int rt_multi_scene_info(const rt_multi* m, rt_scene_info* info);
/* Stats of devices[k] alone in the last rt_render_multi: its segments, primaries, rows and (RT_PROFILE) its own kernel
 * times and launches; ms = that device's render time (before the gather). */
int rt_multi_device_stats(const rt_multi* m, int k, rt_stats* stats);
/* Phases of the last rt_render_multi, so a scaling shortfall can be attributed: every device's render (host wall time of
 * its thread: kernels + its own finalize), the gather (HIP events around the ncclGather on devices[0]'s stream) and the
 * unpack (k_unpack_bands + the host copy when out_rgb8 is host memory). */
typedef struct rt_multi_times {
    double total_ms;            /* the whole call (== rt_stats.ms) */
    double render_ms_max;       /* slowest device's render */
    double render_ms_min;       /* fastest device's render */
    double gather_ms;           /* ncclGather, as devices[0]'s stream sees it */
    double unpack_ms;           /* unpack kernel (+ device-to-host copy) */
    double wait_ms;             /* host time spent polling the gather */
    uint64_t collectives;       /* gathers this rt_multi has issued so far (failed renders issue none) */
    int32_t slowest_device;     /* index k (devices[k]) of render_ms_max */
    int32_t ngpus;
} rt_multi_times;
int rt_multi_times_get(const rt_multi* m, rt_multi_times* out);

/* ---- scene graph builder (one call per reference constructor; returns an id >= 0 or a negative code) ----
 * Scene-build randomness (noise textures' perlin tables, rt_graph_bvh's node draws) comes from the graph's own
 * mt19937 (seed 5489), in call order, exactly as the reference's global generator would produce it. */
rt_graph* rt_graph_new(void);
void rt_graph_free(rt_graph* g);
int rt_graph_random_double(rt_graph* g, double* out);              /* random_double() from the graph's generator */
int rt_tex_solid(rt_graph* g, double r, double gr, double b);       /* texture.h:16-29 */
int rt_tex_checker(rt_graph* g, int even, int odd);                 /* texture.h:31-50 */
int rt_tex_noise(rt_graph* g, double scale);                        /* texture.h:52-65 */
int rt_tex_image(rt_graph* g, int w, int h, int bpp, const uint8_t* texels); /* texture.h:67-118 */
/* barycentric_image_texture(a, b, c, image) (texture.h:135-154): uv = {ua, va, ub, vb, uc, vc}; image_tex from rt_tex_image */
int rt_tex_bary_image(rt_graph* g, const double uv[6], int image_tex);
int rt_mat_lambertian(rt_graph* g, int tex);                        /* material.h:20-43 */
int rt_mat_metal(rt_graph* g, double r, double gr, double b, double fuzz); /* material.h:45-61 */
int rt_mat_dielectric(rt_graph* g, double ir);                      /* material.h:63-99 */
int rt_mat_diffuse_light(rt_graph* g, int tex);                     /* material.h:101-118 */
int rt_obj_sphere(rt_graph* g, const double c[3], double r, int mat);                 /* sphere.h */
int rt_obj_moving_sphere(rt_graph* g, const double c0[3], const double c1[3], double t0, double t1, double r, int mat);
int rt_obj_triangle(rt_graph* g, const double p1[3], const double p2[3], const double p3[3], int mat); /* triangle.h */
int rt_obj_rect(rt_graph* g, int axis /*0 xy,1 xz,2 yz*/, double a0, double a1, double b0, double b1, double k, int mat);
int rt_obj_box(rt_graph* g, const double p0[3], const double p1[3], int mat);         /* box.cpp */
int rt_obj_list(rt_graph* g, int n, const int* items);                                /* hittable_list */
int rt_obj_bvh(rt_graph* g, int n, const int* items);                                 /* bvh_node(list, 0, 1) */
int rt_obj_translate(rt_graph* g, int child, const double offset[3]);                 /* hittable.cpp:3-23 */
int rt_obj_rotate_y(rt_graph* g, int child, double degrees);                          /* hittable.cpp:25-85 */
int rt_obj_constant_medium(rt_graph* g, int boundary, double density, int tex);       /* constant_medium.h */
int rt_graph_add_world(rt_graph* g, int obj);                                         /* world.add(obj) */
int rt_graph_clear_world(rt_graph* g);
int rt_graph_set_view(rt_graph* g, const double lookfrom[3], const double lookat[3], double vfov, double aperture,
                      const double background[3]);
/* ---- meshes (Wavefront OBJ + MTL, rapidobj v1.0.1 semantics: objmesh.h) ----
 * rt_mesh_parse = mesh::parse: parses and triangulates; reports the triangle and shape counts (either may be NULL).
 * rt_mesh_build = mesh::parse + mesh::build into the graph: one triangle per post-triangulation face with
 *   lambertian(color::random()) (no MTL; draws from the graph's generator), lambertian(Ka + Kd), or
 *   lambertian(barycentric_image_texture) for a map_Kd material, whose image (JPEG / PNG, next to the MTL) is decoded
 *   as rt_image_load does (stb_image's bytes; a raw texel file <stem>.rgb[.gz] is also accepted).  The triangle ids are
 *   *first_id .. *first_id + n - 1; returns n >= 0 or a negative code. */
int rt_mesh_parse(const char* obj_path, int64_t* triangles, int64_t* shapes);
int rt_mesh_build(rt_graph* g, const char* obj_path, int* first_id);
/* Compiles the graph (flat SoA + SAH BVH) and uploads it to `device`.  The graph stays owned by the caller. */
int rt_graph_compile(rt_graph* g, int device, rt_scene** out);

#ifdef __cplusplus
}
#endif
#endif /* ART_H */
