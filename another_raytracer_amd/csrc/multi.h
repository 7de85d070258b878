// multi.h — single-process multi-GPU renderer (implemented in multi.hip; no HIP or RCCL types in this header).
//
// The reference's CPU-parallel mode splits the frame into 4 row stripes on 4 threads (engine.h:335-376,
// _run_parallel_stripes).  Here one host thread per GPU renders the row-interleaved band partition of its device
// (band b of band_rows rows goes to GPU b mod N: sky and object rows spread evenly), each GPU packs its rows into one
// device buffer, and a single RCCL gather (ncclGather, rccl.h) moves them over xGMI to the first device, where an
// unpack kernel writes every row to its place in the frame.  The RCCL communicators (non-blocking, one group) and the per-device
// scene uploads are made once, when the MultiRenderer is built.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "renderer.h"
#include "scene.h"

namespace art {

// Phases of the last render (include/art.h rt_multi_times).
struct MultiTimes {
    double total_ms = 0, render_ms_max = 0, render_ms_min = 0, gather_ms = 0, unpack_ms = 0, wait_ms = 0;
    uint64_t collectives = 0;
    int slowest_device = 0, ngpus = 0;
};

class MultiRenderer {
public:
    struct Impl;
    MultiRenderer(const FlatScene& flat, const std::vector<int>& devices);
    ~MultiRenderer();
    MultiRenderer(const MultiRenderer&) = delete;
    MultiRenderer& operator=(const MultiRenderer&) = delete;
    // Whole frame into out_rgb (W*H*3, row 0 = top): host memory, or device memory on devices[0] when out_device.
    // p.band_rows sets the band height; p.band_count / p.band_index are ignored (the devices are the bands).
    // stats: segments / primary summed over the devices, ms = host wall time of the whole call (renders + gather +
    // unpack + output copy).
    void render(const CameraRec<double>& cam, const RenderParams& p, uint8_t* out_rgb, bool out_device, RenderStats& stats);
    int ngpus() const;
    size_t scene_bytes() const;  // scene bytes on each device
    // Stats of device k (devices[k]) in the last render: its segments, its own kernel times and launches, its rows.
    bool device_stats(int k, RenderStats& out) const;
    const MultiTimes& times() const;

private:
    Impl* impl_;
};

// Places n packed band blocks (block r = band set r's band_block_rows(H, band_rows, n) rows in local order, padding
// rows after its band_local_rows) into the H-row frame.  device: both pointers on the current device, a kernel on
// `stream` (hipStream_t); else host memory, copied on the calling thread.
void unpack_bands(const uint8_t* recv, uint8_t* frame, int W, int H, int band_rows, int n, bool device, void* stream);

}  // namespace art
