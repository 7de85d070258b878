// multi.hip — MultiRenderer (multi.h): one host thread per GPU, row-interleaved bands, one RCCL gather, an unpack
// kernel on the root device.  Reference ancestor: engine.h:335-376 (_run_parallel_stripes: 4 threads, 4 stripes).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "multi.h"
#include "options.h"

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

// Every RCCL call of a non-blocking communicator may return ncclInProgress: the operation then completes in the
// background and ncclCommGetAsyncError reports its state.
static bool rccl_ok(ncclResult_t r) { return r == ncclSuccess || r == ncclInProgress; }
#define RCCL_ISSUE(x)                                                                                          \
    do {                                                                                                       \
        ncclResult_t r_ = (x);                                                                                 \
        if (!rccl_ok(r_)) throw std::runtime_error(std::string(#x) + ": " + ncclGetErrorString(r_));       \
    } while (0)

using Clock = std::chrono::steady_clock;
static Clock::time_point deadline_from_now() {  // option multi.timeout_ms (default: ART_MULTI_TIMEOUT_MS, else 120 s)
    const double ms = opt(Opt::MultiTimeoutMs);
    // inf (or NaN, or any value whose nanoseconds overflow the clock's int64 ticks: > ~292 years) is "no deadline";
    // the duration_cast of such a value would be undefined behaviour (INT64_MIN on x86: a deadline in the past)
    const Clock::time_point now = Clock::now();
    const double max_ms = std::chrono::duration<double, std::milli>(Clock::time_point::max() - now).count() * 0.5;
    if (!(ms < max_ms)) return Clock::time_point::max();
    return now + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double, std::milli>(ms));
}

// One ncclGroupStart / ncclGroupEnd bracket that is closed on every exit path.  RCCL's group depth is per thread: a
// throw between the two (a failed ncclCommInitRankConfig / ncclGather issue, a failed hipSetDevice) would leave the
// caller's thread inside the group, and its next rt_multi_create or rt_render_multi would have its collectives
// absorbed into that stale group.  end() closes the group and reports ncclGroupEnd's result; the destructor closes a
// group still open during unwinding (its result is moot: the caller aborts the communicators and rethrows).
class RcclGroup {
public:
    RcclGroup() {
        const ncclResult_t r = ncclGroupStart();
        if (!rccl_ok(r)) throw std::runtime_error(std::string("ncclGroupStart: ") + ncclGetErrorString(r));
        open_ = true;
    }
    ~RcclGroup() {
        if (open_) (void)ncclGroupEnd();
    }
    RcclGroup(const RcclGroup&) = delete;
    RcclGroup& operator=(const RcclGroup&) = delete;
    void end() {
        open_ = false;
        const ncclResult_t r = ncclGroupEnd();
        if (!rccl_ok(r)) throw std::runtime_error(std::string("ncclGroupEnd: ") + ncclGetErrorString(r));
    }

private:
    bool open_ = false;
};

struct MultiRenderer::Impl {
    std::vector<int> devices;
    std::vector<std::unique_ptr<Renderer>> renderers;  // one per device (the scene uploaded on each)
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;                  // gather / unpack streams, one per device
    std::vector<DeviceBuf> send;                       // packed local rows, one per device
    DeviceBuf recv, frame;                             // on devices[0]
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};    // on devices[0]: gather start, gather end, unpack end
    std::vector<RenderStats> last;                     // per-device stats of the last render
    MultiTimes times;
    std::string broken;                                // why the communicators were aborted ("" = usable)

    ~Impl() {
        for (size_t k = 0; k < comms.size(); ++k)
            if (comms[k]) {
                (void)hipSetDevice(devices[k]);
                (void)ncclCommDestroy(comms[k]);
            }
        for (size_t k = 0; k < streams.size(); ++k)
            if (streams[k]) {
                (void)hipSetDevice(devices[k]);
                (void)hipStreamDestroy(streams[k]);
            }
        if (!devices.empty()) (void)hipSetDevice(devices[0]);
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& b : send) b.release();
        recv.release();
        frame.release();
    }
    // Aborts every communicator (ncclCommAbort: returns without waiting for peers or pending operations); the
    // MultiRenderer then refuses to render.  Throws the reason.
    [[noreturn]] void abort_all(const std::string& why) {
        for (size_t k = 0; k < comms.size(); ++k)
            if (comms[k]) {
                (void)hipSetDevice(devices[k]);
                (void)ncclCommAbort(comms[k]);
                comms[k] = nullptr;
            }
        broken = why;
        throw std::runtime_error(why + " (RCCL communicators aborted; destroy and re-create the rt_multi)");
    }
    // Polls until every communicator's pending operation (init, group launch) is done, an error shows, or the deadline
    // passes.
    void wait_comms(const char* what, std::chrono::steady_clock::time_point deadline) {
        for (;;) {
            bool pending = false;
            for (size_t k = 0; k < comms.size(); ++k) {
                ncclResult_t st = ncclSuccess;
                const ncclResult_t r = ncclCommGetAsyncError(comms[k], &st);
                if (r != ncclSuccess) abort_all(std::string(what) + ": ncclCommGetAsyncError: " + ncclGetErrorString(r));
                if (st == ncclInProgress) pending = true;
                else if (st != ncclSuccess) abort_all(std::string(what) + " on device " + std::to_string(devices[k]) + ": " + ncclGetErrorString(st));
            }
            if (!pending) return;
            if (std::chrono::steady_clock::now() >= deadline) abort_all(std::string(what) + ": timed out (option multi.timeout_ms)");
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    // Polls the gather streams (hipStreamQuery) and the communicators' asynchronous errors until every stream has
    // drained, or aborts at the deadline: a stuck collective ends the call with RT_E_DEVICE instead of hanging it.
    void wait_streams(const char* what, std::chrono::steady_clock::time_point deadline) {
        std::vector<bool> done(streams.size(), false);
        for (;;) {
            bool all = true;
            for (size_t k = 0; k < streams.size(); ++k) {
                if (done[k]) continue;
                HIP_CHECK(hipSetDevice(devices[k]));
                const hipError_t q = hipStreamQuery(streams[k]);
                if (q == hipSuccess) {
                    done[k] = true;
                    continue;
                }
                if (q != hipErrorNotReady) abort_all(std::string(what) + ": hipStreamQuery: " + hipGetErrorString(q));
                all = false;
                ncclResult_t st = ncclSuccess;
                if (ncclCommGetAsyncError(comms[k], &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
                    abort_all(std::string(what) + " on device " + std::to_string(devices[k]) + ": " + ncclGetErrorString(st));
            }
            if (all) return;
            if (std::chrono::steady_clock::now() >= deadline) abort_all(std::string(what) + ": timed out (option multi.timeout_ms)");
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
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
    // the scene is uploaded to every device here, not at the first render: a timed rt_render_multi is the render (the
    // reference times engine::run only, main.cpp:44-46)
    for (int k = 0; k < n; ++k) {
        impl_->renderers.push_back(std::make_unique<Renderer>(flat, devices[k]));
        impl_->renderers.back()->upload();
    }
    impl_->streams.assign(n, nullptr);
    impl_->send.resize(n);
    for (int k = 0; k < n; ++k) {
        HIP_CHECK(hipSetDevice(devices[k]));
        HIP_CHECK(hipStreamCreateWithFlags(&impl_->streams[k], hipStreamNonBlocking));
        impl_->send[k].device = devices[k];
    }
    HIP_CHECK(hipSetDevice(devices[0]));
    for (auto& e : impl_->ev) HIP_CHECK(hipEventCreate(&e));
    impl_->recv.device = impl_->frame.device = devices[0];
    // one communicator per device, rank k = devices[k], created as one group (what ncclCommInitAll does) but
    // non-blocking, so that a stuck bootstrap ends at the deadline instead of hanging the caller
    ncclUniqueId id;
    RCCL_CHECK(ncclGetUniqueId(&id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = opt(Opt::RcclBlocking) != 0 ? 1 : 0;  // option multi.rccl_blocking (diagnosis)
    impl_->comms.assign(n, nullptr);
    const auto deadline = deadline_from_now();
    try {
        RcclGroup group;
        for (int k = 0; k < n; ++k) {
            HIP_CHECK(hipSetDevice(devices[k]));
            RCCL_ISSUE(ncclCommInitRankConfig(&impl_->comms[k], n, id, k, &cfg));
            if (k == n - 1 && opt(Opt::FaultRcclGroup) == 1)  // fault point (tests): an error inside the init group
                throw std::runtime_error("ncclCommInitRankConfig: injected failure (test.fault_rccl_group = 1)");
        }
        group.end();
    } catch (const std::exception& e) {
        // the group is closed (RcclGroup); half-created communicators are aborted, not destroyed: a destroy would wait
        // for peers that may never come
        impl_->abort_all(std::string("RCCL communicator init: ") + e.what());
    }
    impl_->wait_comms("RCCL communicator init", deadline);
    impl_->times.ngpus = n;
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
const MultiTimes& MultiRenderer::times() const { return impl_->times; }

void MultiRenderer::render(const CameraRec<double>& cam, const RenderParams& p, uint8_t* out_rgb, bool out_device, RenderStats& stats) {
    Impl& I = *impl_;
    if (!I.broken.empty()) throw std::runtime_error("rt_multi unusable: " + I.broken + " (destroy and re-create it)");
    const int n = static_cast<int>(I.devices.size());
    const int W = p.width, H = p.height, band_rows = std::max(1, p.band_rows);
    const int max_rows = band_block_rows(H, band_rows, n);
    const size_t row_bytes = static_cast<size_t>(W) * 3, block = static_cast<size_t>(max_rows) * row_bytes;
    for (int k = 0; k < n; ++k) I.send[k].ensure(std::max<size_t>(block, 1));
    I.recv.ensure(std::max<size_t>(block * n, 1));
    if (!out_device) I.frame.ensure(row_bytes * H);
    MultiTimes tm;
    tm.ngpus = n;
    tm.collectives = I.times.collectives;

    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    // phase 1: every device renders its bands into its send buffer (one host thread each; Renderer::render blocks)
    std::vector<RenderStats> st(n);
    std::vector<double> rms(n, 0.0);
    std::vector<std::exception_ptr> err(n);
    std::vector<std::thread> pool;
    for (int k = 0; k < n; ++k)
        pool.emplace_back([&, k]() {
            try {
                const auto a = clock::now();
                RenderParams pk = p;
                pk.band_rows = band_rows;
                pk.band_count = n;
                pk.band_index = k;
                pk.flags |= RT_OUT_DEVICE;
                pk.stream = nullptr;  // the renderer's own stream on its device
                I.renderers[k]->render(cam, pk, static_cast<uint8_t*>(I.send[k].p), nullptr, st[k]);
                rms[k] = std::chrono::duration<double, std::milli>(clock::now() - a).count();
            } catch (...) {
                err[k] = std::current_exception();
            }
        });
    for (auto& t : pool) t.join();
    for (auto& e : err)
        if (e) {
            I.times = tm;  // no collective was started: every rank stays consistent and the multi usable
            std::rethrow_exception(e);
        }
    tm.render_ms_max = tm.render_ms_min = rms[0];
    for (int k = 1; k < n; ++k) {
        if (rms[k] > tm.render_ms_max) {
            tm.render_ms_max = rms[k];
            tm.slowest_device = k;
        }
        tm.render_ms_min = std::min(tm.render_ms_min, rms[k]);
    }
    // phase 2: one gather of the equal-sized packed blocks to devices[0] (rows past a band's end are padding)
    const auto deadline = deadline_from_now();
    HIP_CHECK(hipSetDevice(I.devices[0]));
    HIP_CHECK(hipEventRecord(I.ev[0], I.streams[0]));
    try {
        RcclGroup group;
        for (int k = 0; k < n; ++k) {
            HIP_CHECK(hipSetDevice(I.devices[k]));
            RCCL_ISSUE(ncclGather(I.send[k].p, k == 0 ? I.recv.p : nullptr, block, ncclUint8, 0, I.comms[k], I.streams[k]));
            if (k == n - 1 && opt(Opt::FaultRcclGroup) == 2)  // fault point (tests): an error inside the gather group
                throw std::runtime_error("ncclGather: injected failure inside the group (test.fault_rccl_group = 2)");
        }
        group.end();
    } catch (const std::exception& e) {
        // part of the group may have been issued to some ranks: the communicators cannot be trusted any more
        I.times = tm;
        I.abort_all(std::string("ncclGather issue: ") + e.what());
    }
    ++I.times.collectives;
    tm.collectives = I.times.collectives;
    I.times = tm;
    // fault point (tests): the collective fails while in flight, as a peer error or an expired deadline would
    if (opt(Opt::FaultGatherAbort) != 0) I.abort_all("ncclGather: injected failure (test.fault_gather_abort)");
    const auto tw = clock::now();
    I.wait_comms("ncclGather launch", deadline);  // non-blocking group: the gathers are enqueued once this returns
    HIP_CHECK(hipSetDevice(I.devices[0]));
    HIP_CHECK(hipEventRecord(I.ev[1], I.streams[0]));
    I.wait_streams("ncclGather", deadline);
    tm.wait_ms = std::chrono::duration<double, std::milli>(clock::now() - tw).count();
    // phase 3: the root places every row and hands the frame over
    HIP_CHECK(hipSetDevice(I.devices[0]));
    uint8_t* dst = out_device ? out_rgb : static_cast<uint8_t*>(I.frame.p);
    launch_unpack(static_cast<const uint8_t*>(I.recv.p), dst, W, H, band_rows, n, max_rows, I.streams[0]);
    if (!out_device) HIP_CHECK(hipMemcpyAsync(out_rgb, I.frame.p, row_bytes * H, hipMemcpyDeviceToHost, I.streams[0]));
    HIP_CHECK(hipEventRecord(I.ev[2], I.streams[0]));
    HIP_CHECK(hipStreamSynchronize(I.streams[0]));
    const auto t1 = clock::now();
    float g_ms = 0.f, u_ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&g_ms, I.ev[0], I.ev[1]));
    HIP_CHECK(hipEventElapsedTime(&u_ms, I.ev[1], I.ev[2]));
    tm.gather_ms = g_ms;
    tm.unpack_ms = u_ms;

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
    stats.kernel_features = st[0].kernel_features;
    stats.kernel_textures = st[0].kernel_textures;
    stats.kernel_lds_mode = st[0].kernel_lds_mode;
    tm.total_ms = stats.ms;
    I.times = tm;
}

}  // namespace art
