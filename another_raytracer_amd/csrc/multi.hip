// multi.hip — MultiRenderer (multi.h): one host thread per GPU, row-interleaved bands, one RCCL gather, an unpack
// kernel on the root device.  Reference ancestor: engine.h:335-376 (_run_parallel_stripes: 4 threads, 4 stripes).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "multi.h"

namespace art {

#define HIP_CHECK(x)                                                                                      \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define RCCL_CHECK(x)                                                                                        \
    do {                                                                                                     \
        ncclResult_t r_ = (x);                                                                               \
        if (r_ != ncclSuccess) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// recv holds n packed blocks of max_rows rows (block r = band set r's rows in local order, padding rows after them);
// one block of threads per (r, ly).  Rows whose byte count and both addresses are 16-B aligned move as uint4.
__global__ void k_unpack_bands(const uint8_t* __restrict__ recv, uint8_t* __restrict__ frame, int W, int H, int band_rows, int n,
                               int max_rows, int wide) {
    const int r = static_cast<int>(blockIdx.x) / max_rows, ly = static_cast<int>(blockIdx.x) % max_rows;
    const int gy = band_global_row(ly, band_rows, n, r);
    if (gy >= H) return;  // padding rows of a shorter band set
    const size_t row_bytes = static_cast<size_t>(W) * 3;
    const uint8_t* src = recv + (static_cast<size_t>(r) * max_rows + ly) * row_bytes;
    uint8_t* dst = frame + static_cast<size_t>(gy) * row_bytes;
    if (wide) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (size_t i = threadIdx.x; i < row_bytes / 16; i += blockDim.x) d4[i] = s4[i];
    } else {
        for (size_t i = threadIdx.x; i < row_bytes; i += blockDim.x) dst[i] = src[i];
    }
}

static void launch_unpack(const uint8_t* recv, uint8_t* frame, int W, int H, int band_rows, int n, int max_rows, hipStream_t stream) {
    if (max_rows <= 0) return;
    const size_t row_bytes = static_cast<size_t>(W) * 3;
    const int wide = (row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(recv) % 16 == 0 && reinterpret_cast<uintptr_t>(frame) % 16 == 0);
    hipLaunchKernelGGL(k_unpack_bands, dim3(static_cast<unsigned>(n * max_rows)), dim3(256), 0, stream, recv, frame, W, H, band_rows, n,
                       max_rows, wide);
    HIP_CHECK(hipGetLastError());
}

void unpack_bands(const uint8_t* recv, uint8_t* frame, int W, int H, int band_rows, int n, bool device, void* stream) {
    if (W < 1 || H < 1 || band_rows < 1 || n < 1) throw std::invalid_argument("unpack_bands: W, H, band_rows, n must be >= 1");
    const int max_rows = band_block_rows(H, band_rows, n);
    if (device) {
        launch_unpack(recv, frame, W, H, band_rows, n, max_rows, static_cast<hipStream_t>(stream));
        return;
    }
    const size_t row_bytes = static_cast<size_t>(W) * 3;
    for (int r = 0; r < n; ++r)
        for (int ly = 0; ly < max_rows; ++ly) {
            const int gy = band_global_row(ly, band_rows, n, r);
            if (gy < H) std::memcpy(frame + static_cast<size_t>(gy) * row_bytes, recv + (static_cast<size_t>(r) * max_rows + ly) * row_bytes, row_bytes);
        }
}

struct DeviceBuf {
    int device = 0;
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t want) {
        if (want <= bytes) return;
        HIP_CHECK(hipSetDevice(device));
        if (p) {
            void* old = p;
            p = nullptr;
            bytes = 0;
            HIP_CHECK(hipFree(old));
        }
        void* q = nullptr;
        HIP_CHECK(hipMalloc(&q, want));
        p = q;
        bytes = want;
    }
    void release() {
        if (p) {
            (void)hipSetDevice(device);
            (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
    }
};

struct MultiRenderer::Impl {
    std::vector<int> devices;
    std::vector<std::unique_ptr<Renderer>> renderers;  // one per device (the scene uploaded on each)
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;                  // gather / unpack streams, one per device
    std::vector<DeviceBuf> send;                       // packed local rows, one per device
    DeviceBuf recv, frame;                             // on devices[0]
    std::vector<RenderStats> last;                     // per-device stats of the last render

    ~Impl() {
        for (auto c : comms)
            if (c) (void)ncclCommDestroy(c);
        for (size_t k = 0; k < streams.size(); ++k)
            if (streams[k]) {
                (void)hipSetDevice(devices[k]);
                (void)hipStreamDestroy(streams[k]);
            }
        for (auto& b : send) b.release();
        recv.release();
        frame.release();
    }
};

MultiRenderer::MultiRenderer(const FlatScene& flat, const std::vector<int>& devices) : impl_(new Impl) {
    std::unique_ptr<Impl> guard(impl_);
    if (devices.empty()) throw std::runtime_error("rt_multi needs at least one device");
    int count = 0;
    HIP_CHECK(hipGetDeviceCount(&count));
    for (size_t a = 0; a < devices.size(); ++a) {
        if (devices[a] < 0 || devices[a] >= count) throw std::runtime_error("device " + std::to_string(devices[a]) + " does not exist");
        for (size_t b = 0; b < a; ++b)
            if (devices[a] == devices[b]) throw std::runtime_error("a device may appear only once (one RCCL rank per GPU)");
    }
    const int n = static_cast<int>(devices.size());
    impl_->devices = devices;
    for (int k = 0; k < n; ++k) impl_->renderers.push_back(std::make_unique<Renderer>(flat, devices[k]));
    impl_->comms.assign(n, nullptr);
    RCCL_CHECK(ncclCommInitAll(impl_->comms.data(), n, devices.data()));
    impl_->streams.assign(n, nullptr);
    impl_->send.resize(n);
    for (int k = 0; k < n; ++k) {
        HIP_CHECK(hipSetDevice(devices[k]));
        HIP_CHECK(hipStreamCreateWithFlags(&impl_->streams[k], hipStreamNonBlocking));
        impl_->send[k].device = devices[k];
    }
    impl_->recv.device = impl_->frame.device = devices[0];
    guard.release();
}

MultiRenderer::~MultiRenderer() { delete impl_; }
int MultiRenderer::ngpus() const { return static_cast<int>(impl_->devices.size()); }
size_t MultiRenderer::scene_bytes() const { return impl_->renderers.empty() ? 0 : impl_->renderers[0]->scene_bytes(); }
bool MultiRenderer::device_stats(int k, RenderStats& out) const {
    if (k < 0 || k >= static_cast<int>(impl_->last.size())) return false;
    out = impl_->last[k];
    return true;
}

void MultiRenderer::render(const CameraRec<double>& cam, const RenderParams& p, uint8_t* out_rgb, bool out_device, RenderStats& stats) {
    Impl& I = *impl_;
    const int n = static_cast<int>(I.devices.size());
    const int W = p.width, H = p.height, band_rows = std::max(1, p.band_rows);
    const int max_rows = band_block_rows(H, band_rows, n);
    const size_t row_bytes = static_cast<size_t>(W) * 3, block = static_cast<size_t>(max_rows) * row_bytes;
    for (int k = 0; k < n; ++k) I.send[k].ensure(std::max<size_t>(block, 1));
    I.recv.ensure(std::max<size_t>(block * n, 1));
    if (!out_device) I.frame.ensure(row_bytes * H);

    const auto t0 = std::chrono::steady_clock::now();
    // phase 1: every device renders its bands into its send buffer (one host thread each; Renderer::render blocks)
    std::vector<RenderStats> st(n);
    std::vector<std::exception_ptr> err(n);
    std::vector<std::thread> pool;
    for (int k = 0; k < n; ++k)
        pool.emplace_back([&, k]() {
            try {
                RenderParams pk = p;
                pk.band_rows = band_rows;
                pk.band_count = n;
                pk.band_index = k;
                pk.flags |= RT_OUT_DEVICE;
                pk.stream = nullptr;  // the renderer's own stream on its device
                I.renderers[k]->render(cam, pk, static_cast<uint8_t*>(I.send[k].p), nullptr, st[k]);
            } catch (...) {
                err[k] = std::current_exception();
            }
        });
    for (auto& t : pool) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);  // no collective was started: every rank stays consistent
    // phase 2: one gather of the equal-sized packed blocks to devices[0] (rows past a band's end are padding)
    RCCL_CHECK(ncclGroupStart());
    for (int k = 0; k < n; ++k) {
        HIP_CHECK(hipSetDevice(I.devices[k]));
        RCCL_CHECK(ncclGather(I.send[k].p, k == 0 ? I.recv.p : nullptr, block, ncclUint8, 0, I.comms[k], I.streams[k]));
    }
    RCCL_CHECK(ncclGroupEnd());
    // phase 3: the root places every row and hands the frame over
    HIP_CHECK(hipSetDevice(I.devices[0]));
    uint8_t* dst = out_device ? out_rgb : static_cast<uint8_t*>(I.frame.p);
    launch_unpack(static_cast<const uint8_t*>(I.recv.p), dst, W, H, band_rows, n, max_rows, I.streams[0]);
    if (!out_device) HIP_CHECK(hipMemcpyAsync(out_rgb, I.frame.p, row_bytes * H, hipMemcpyDeviceToHost, I.streams[0]));
    for (int k = 0; k < n; ++k) {
        HIP_CHECK(hipSetDevice(I.devices[k]));
        HIP_CHECK(hipStreamSynchronize(I.streams[k]));
    }
    const auto t1 = std::chrono::steady_clock::now();

    I.last = st;
    stats = RenderStats{};
    for (int k = 0; k < n; ++k) {
        stats.segments += st[k].segments;
        stats.primary += st[k].primary;
        stats.extend_ms = std::max(stats.extend_ms, st[k].extend_ms);
        stats.shade_ms = std::max(stats.shade_ms, st[k].shade_ms);
        stats.extend_launches += st[k].extend_launches;
        stats.shade_launches += st[k].shade_launches;
        stats.passes = std::max(stats.passes, st[k].passes);
    }
    stats.ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    stats.samples_per_pass = st[0].samples_per_pass;
    stats.local_rows = H;
    stats.extend_variant = st[0].extend_variant;
}

}  // namespace art
