// oracle/restate.h — TEST INFRASTRUCTURE ONLY.  C API of the CPU restatement (oracle/restate.cpp), loaded by
// tests/ and by bench.py's cpu_baseline leg through ctypes.  Never linked into the product.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// RNG modes.
//   ORC_MT  : one global std::mt19937 (default seed 5489) shared by scene build and render, libstdc++
//             generate_canonical restated, g++ argument-evaluation order made explicit
//             (/root/reference/src/utils/tracer_utils.h:27-41).  Single-threaded.  Bit-exact vs oracle/_ref.
//   ORC_PCG : scene built with mt19937 (identical geometry); render draws come from per-(pixel, sample)
//             PCG32 streams, the product's RNG contract; iterative integrator.  Multi-threaded.
enum { ORC_MT = 0, ORC_PCG = 1 };

// Directory holding assets produced from the reference inputs (cow/dino triangle lists, decoded textures).
void orc_set_asset_dir(const char* dir);

// First n values of random_double() from a fresh generator.
int orc_kat(int n, double* out);

// The k random_double() values that follow the scene build (pins RNG consumption of the scene build).
int orc_probe(const char* scene, int k, double* out);

// Canonical JSON dump of the restated scene graph (same schema as `ref_harness dump`).  Returns the
// required size (including NUL); writes at most cap bytes.
size_t orc_dump(const char* scene, char* buf, size_t cap);

// Render rows [row0, row0+nrows) of a WxH image.  rgb_out: nrows*W*3 u8 (may be NULL);
// acc_out: nrows*W*3 f64 per-pixel radiance sums (may be NULL).  segments_out: world.hit calls.
// threads <= 0 -> hardware_concurrency.  ORC_MT ignores threads and requires row0 == 0, nrows == H.
// Returns 0 on success, <0 on error (orc_last_error()).
int orc_render(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed,
               int row0, int nrows, int threads, uint8_t* rgb_out, double* acc_out,
               long long* segments_out, double* ms_out);

// ORC_PCG render of an arbitrary list of rows (rows[k] = global row of output row k) of a WxH image, spread over
// `threads` host threads (<= 0: hardware_concurrency) in work items of (row, 64-pixel column chunk) taken
// dynamically, so a few expensive rows still use every thread.  Same outputs and arguments as orc_render.
int orc_render_rows(const char* scene, int W, int H, int spp, int max_depth, uint64_t seed, const int* rows, int nrows,
                    int threads, uint8_t* rgb_out, double* acc_out, long long* segments_out, double* ms_out);

// hittable_list::hit (hittable_list.cpp:5-19) of the scene's world for n rays (n x {ox, oy, oz, dx, dy, dz, tm}),
// t in [0.001, inf): t_out (+inf on a miss) and the hit_record normal (normal_out n x 3, 0 on a miss).  Ray i's
// constant_medium draws come from the pcg stream pcg_seed(0, i, 0) -- the product's rt_trace_rays contract.
int orc_trace_rays(const char* scene, const double* rays, long long n, double* t_out, double* normal_out);

// engine_mode::adaptive (engine.h:96-333) over the whole WxH image (W, H multiples of 12).  ORC_MT: the
// reference's draw sequence with its 4 stripes run one after another (bit-exact vs `ref_harness render .. adaptive`);
// ORC_PCG: the product's streams, every distinct pixel traced once.  rgb_out: H*W*3 u8.  Returns -3 on a size the
// reference rejects (its std::logic_error).
int orc_render_adaptive(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed, int threads,
                        uint8_t* rgb_out, long long* segments_out, double* ms_out);

// engine_mode::parallel_images (engine.h:378-445) over the whole WxH image: four partial images of spp/4 samples each,
// each pixel's sum rounded to float (write_color_raw<float>), pixel_acc = ((c1 + c2) + c3) + c4 in double, written
// with the full spp.  ORC_MT: the reference's draw sequence with the four images traced one after another
// (bit-exact vs `ref_harness render .. images`); ORC_PCG: partial image q takes samples [q*spp/4, (q+1)*spp/4) of
// the product's (pixel, sample) streams.  acc_out: the pixel_acc sums (H*W*3 f64, may be NULL).
int orc_render_images(const char* scene, int W, int H, int spp, int max_depth, int mode, uint64_t seed, int threads,
                      uint8_t* rgb_out, double* acc_out, long long* segments_out, double* ms_out);

const char* orc_last_error(void);

#ifdef __cplusplus
}
#endif
