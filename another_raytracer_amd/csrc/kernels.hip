// kernels.hip — the wavefront path tracer for gfx950 (MI355X).
//
// The reference's recursive integrator (engine.h:58-68 _stochastic_sample + engine.h:447-466 _ray_color) is
// flattened into an iterative per-ray wavefront loop over a pool of P = k * npix paths (k samples of every local
// pixel per pass).  Per pass:
//   for depth d < max_depth:
//     k_extend<R, F>           closest hit over the world list (LDS-stack BVH traversal, f32 boxes, R leaf tests);
//                              at depth 0 it first generates the camera ray of every (pixel, sample) slot itself
//                              (PCG32 keyed by (seed, pixel, sample)); F = the scene's feature subset (layout.h),
//                              misses finish their path (L += T*background); hits are appended to one of five
//                              material queues (branch sorting for the shade stage)
//     k_shade<R, F, M, TF>     one launch per material type M present: emitted + scatter on that material's queue
//                              (branch-sorted shading); survivors go to the next active queue
//   k_accum                    adds the k per-slot radiances into the f64 pixel sums in sample order
// then k_finalize (write_color, color.h:6-22).  All queue sizes live on the device: extend/shade are persistent
// grids walking their input in a static grid-stride order, and appends go to kShards-way sharded queues, so no
// host round trip and no hot atomic word exists inside a render (see "work distribution").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <unordered_map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "device.h"
#include "options.h"
#include "pass_plan.h"
#include "renderer.h"

#ifndef ART_EXTEND_MIN_WAVES
#define ART_EXTEND_MIN_WAVES 1  // __launch_bounds__ minimum waves per SIMD for k_extend (register budget knob)
#endif

// ART_SPLIT_PATHS (Makefile): unset = one translation unit; 1 = everything but k_paths and its launcher; 2 = only
// k_paths and its launcher (kernels_paths.o, compiled with its own scheduler strategy, measured best for it alone);
// 3 = only the k_paths_g instantiations ART_SPLIT_MESH moves out of the main object (kernels_mesh.o, likewise).
#ifndef ART_SPLIT_PATHS
#define ART_SPLIT_PATHS 0
#endif
namespace art {

#define HIP_OK(x)                                                                                         \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------------------------------------ path records
// One path = one AoS record so that a lane touching a scattered slot reads whole cache lines:
//   f32: 64 B = {o.xyz, time} {d.xyz, -} {T.rgb, L.r} {L.gb, rng}
//   f64: 128 B = line 0 {o.xyz, d.xyz, time, rng} (all extend reads) + line 1 {T.rgb, L.rgb}
template <class R> struct PathRec;
template <> struct PathRec<float> {
    float4 ot, d, tl, lr;
};
template <> struct PathRec<double> {
    double2 a, b, c, e;  // line 0: (ox,oy) (oz,dx) (dy,dz) (tm,rng)
    double2 f, g, h, i;  // line 1: (Tr,Tg) (Tb,Lr) (Lg,Lb) (-,-)
};
template <class R>
struct PathState {
    Ray<R> ray;
    V3<R> T, L;
    uint64_t rng;
};
__device__ __forceinline__ void load_path(const PathRec<float>* P, uint32_t q, PathState<float>& s, bool full) {
    const PathRec<float>& p = P[q];
    const float4 ot = p.ot, d = p.d;
    s.ray.o = mk(ot.x, ot.y, ot.z);
    s.ray.tm = ot.w;
    s.ray.d = mk(d.x, d.y, d.z);
    const float4 lr = p.lr;
    s.rng = (static_cast<uint64_t>(__float_as_uint(lr.w)) << 32) | __float_as_uint(lr.z);
    if (full) {
        const float4 tl = p.tl;
        s.T = mk(tl.x, tl.y, tl.z);
        s.L = mk(tl.w, lr.x, lr.y);
    }
}
__device__ __forceinline__ void store_path(PathRec<float>* P, uint32_t q, const PathState<float>& s) {
    PathRec<float>& p = P[q];
    p.ot = make_float4(s.ray.o.x, s.ray.o.y, s.ray.o.z, s.ray.tm);
    p.d = make_float4(s.ray.d.x, s.ray.d.y, s.ray.d.z, 0.0f);
    p.tl = make_float4(s.T.x, s.T.y, s.T.z, s.L.x);
    p.lr = make_float4(s.L.y, s.L.z, __uint_as_float(static_cast<uint32_t>(s.rng)), __uint_as_float(static_cast<uint32_t>(s.rng >> 32)));
}
__device__ __forceinline__ void store_rng(PathRec<float>* P, uint32_t q, uint64_t rng) {
    float2* p = reinterpret_cast<float2*>(&P[q].lr) + 1;
    *p = make_float2(__uint_as_float(static_cast<uint32_t>(rng)), __uint_as_float(static_cast<uint32_t>(rng >> 32)));
}
__device__ __forceinline__ void load_path(const PathRec<double>* P, uint32_t q, PathState<double>& s, bool full) {
    const PathRec<double>& p = P[q];
    const double2 a = p.a, b = p.b, c = p.c, e = p.e;
    s.ray.o = mk(a.x, a.y, b.x);
    s.ray.d = mk(b.y, c.x, c.y);
    s.ray.tm = e.x;
    s.rng = static_cast<uint64_t>(__double_as_longlong(e.y));
    if (full) {
        const double2 f = p.f, g = p.g, h = p.h;
        s.T = mk(f.x, f.y, g.x);
        s.L = mk(g.y, h.x, h.y);
    }
}
__device__ __forceinline__ void store_path(PathRec<double>* P, uint32_t q, const PathState<double>& s) {
    PathRec<double>& p = P[q];
    p.a = make_double2(s.ray.o.x, s.ray.o.y);
    p.b = make_double2(s.ray.o.z, s.ray.d.x);
    p.c = make_double2(s.ray.d.y, s.ray.d.z);
    p.e = make_double2(s.ray.tm, __longlong_as_double(static_cast<long long>(s.rng)));
    p.f = make_double2(s.T.x, s.T.y);
    p.g = make_double2(s.T.z, s.L.x);
    p.h = make_double2(s.L.y, s.L.z);
}
// throughput and radiance only (line 1 of the f64 record)
__device__ __forceinline__ void load_tl(const PathRec<float>* P, uint32_t q, PathState<float>& s) {
    const float4 tl = P[q].tl, lr = P[q].lr;
    s.T = mk(tl.x, tl.y, tl.z);
    s.L = mk(tl.w, lr.x, lr.y);
}
__device__ __forceinline__ void load_tl(const PathRec<double>* P, uint32_t q, PathState<double>& s) {
    const double2 f = P[q].f, g = P[q].g, h = P[q].h;
    s.T = mk(f.x, f.y, g.x);
    s.L = mk(g.y, h.x, h.y);
}
__device__ __forceinline__ void store_rng(PathRec<double>* P, uint32_t q, uint64_t rng) {
    P[q].e.y = __longlong_as_double(static_cast<long long>(rng));
}

template <class R>
struct HitRecD {  // extend -> shade hand-off, 16 B
    R t;
    uint32_t prim, obj;
};
template <> struct HitRecD<double> {
    double t;
    uint32_t prim, obj;
};

template <class R> struct ResRec;  // final per-slot radiance
template <> struct ResRec<float> { float4 v; };
template <> struct ResRec<double> { double x, y, z; };  // 24 B, unpadded: k_accum streams these at HBM rate
__device__ __forceinline__ void store_res(ResRec<float>* res, uint32_t q, V3<float> L) { res[q].v = make_float4(L.x, L.y, L.z, 0.0f); }
// NT: non-temporal stores (read once, by k_accum after the pass), so the records do not evict k_paths' L2-resident
// camera-ray rings.  Measured (r5c, profiles/r5c_write_traffic.txt, HBM bytes per segment vs the 24-B records' own):
// each 8-B non-temporal store reaches HBM as its own partial write, 2.0x the record bytes (Next-Week final: 12.6 B
// against 6.3); temporal stores merge in L2 first, 1.18x (7.4 B), at equal speed -- so k_paths_g, which has no rings,
// stores temporally.  k_paths keeps NT: its writes are ring lines evicted between laps (27.8 B per segment with NT
// 24-B records, 27.2 with NT 32-B ones), and temporal records evict more of them (32.9 B written + 6.8 B re-read,
// -0.25 %).  32-B records cost k_accum a third more reads and lose 0.8-1.2 %.  r6i: the k_paths_g kernels whose BVH is
// not all in LDS (LM 0 / 2) store non-temporally after all: there the temporal records evict the L2-resident nodes
// and leaf triangles (capsule +1.7 %, cow +0.8 %, profiles/r6i_ab_res_nt.txt).
template <bool NT = true>
__device__ __forceinline__ void store_res(ResRec<double>* res, uint32_t q, V3<double> L) {
    if constexpr (NT) {
        __builtin_nontemporal_store(L.x, &res[q].x);
        __builtin_nontemporal_store(L.y, &res[q].y);
        __builtin_nontemporal_store(L.z, &res[q].z);
    } else {
        res[q].x = L.x;
        res[q].y = L.y;
        res[q].z = L.z;
    }
}
__device__ __forceinline__ void load_res(const ResRec<float>* res, uint32_t q, double& r, double& g, double& b) {
    const float4 v = res[q].v;
    r = v.x; g = v.y; b = v.z;
}
__device__ __forceinline__ void load_res(const ResRec<double>* res, uint32_t q, double& r, double& g, double& b) {
    r = res[q].x; g = res[q].y; b = res[q].z;
}

// ------------------------------------------------------------------------------------------------ work distribution
// Queues are split into kShards shards, each with its own counter on its own 128-B line.  Persistent waves take
// 64-item batches in a static grid-stride order (no claim atomic) and a wave appends only to shard
// (global wave id % kShards): one returning atomic per wave and queue, spread over kShards words instead of one
// (a single word saturates at ~88 atomics/us, MI355X_MICROARCH.md "dequeue").  Static assignment also bounds every
// shard: shard s only receives outputs of the batches b with b % kShards == s, so kShardCap(P) slots suffice.
constexpr int kShards = 32;
constexpr int kCounterStride = 32;                   // words between counters (128 B)
constexpr int kQueueKinds = 1 + kNumMatTypes;        // 0: active (extend input), 1..5: material queues
constexpr int kMatSegs = kNumMatTypes * kShards;     // shade input segments
constexpr uint64_t kMaxPassSlots = 1ull << 31;       // slot ids and batch offsets stay well inside u32
// + 2 batches per material kernel: the kNumMatTypes shade launches of one depth all append to the same next-queue shards
__host__ __device__ inline uint32_t shard_cap(uint32_t P) { return 64u * ((((P + 63u) / 64u) + kShards - 1) / kShards + 2 * kNumMatTypes); }

// n / d for a divisor fixed per launch, as a multiply-high, an add and a shift (Granlund & Montgomery 1994,
// round-up variant): l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, n / d = (mulhi(m, n) + n) >> l, exact for
// every n < 2^31 (the add cannot carry out) -- instead of the ~20-instruction integer division sequence.
struct FastDiv {
    uint32_t d, m, l;
    static FastDiv make(uint32_t d) {
        uint32_t l = 0;
        while (l < 32 && (1ull << l) < d) ++l;
        return FastDiv{d, static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(m, n) + n) >> l; }
};

struct PassGeom {
    int32_t W, H;               // full image
    int32_t rows;               // local rows
    int32_t band_rows, band_count, band_index;
    uint32_t tiles_x, npix_pad; // 8x8 tiles over (W x rows)
    uint32_t k;                 // samples in this pass
    uint32_t sample_base;       // first sample index of the pass
    uint32_t P;                 // k * npix_pad path slots
    uint32_t cap;               // shard capacity
    uint32_t live;              // k * rows * W: slots that are real pixels (depth-0 segments)
    uint32_t stack;             // LDS traversal stack rows per lane (stack_rows)
    int32_t max_depth;
    uint64_t seed;
    uint64_t seed_mix;          // splitmix64(seed): the per-frame half of pcg_seed, hoisted to the host
    FastDiv fd_npix, fd_tiles_x, fd_band_rows, fd_w;  // / npix_pad, / tiles_x, / band_rows, / W
    double inv_w1, inv_h1;      // RN(1 / (W - 1)), RN(1 / (H - 1)) for gen_ray's div_rcp (rt_render rejects W or H < 2)
    const uint32_t* list;       // pixel-list mode (engine_mode::adaptive levels): slot pixel = list[qi] (local ly*W+lx)
    uint32_t nlist;             //   for qi < nlist; nullptr = every local pixel in 8x8 tile order
    uint32_t chunk;             // persistent kernels: slots per claim (path_chunk: a power of two >= 64)
    uint32_t lds_ring;          // k_paths_g LM 1: the camera-ray rings are allocated in LDS (kRing, when they fit)
    // 1: pixel-list mode with the samples of a list entry on consecutive slots (slot = entry * k + sample: a wave's 64
    // lanes trace one pixel's samples, coherent rays, instead of 64 entries scattered over the image) and the entry
    // count on the device at list[-1] (the adaptive levels' lists, appended by k_adapt_level: no host round trip);
    // npix_pad = k then, and the persistent kernels take P = list[-1] * k and nlist = list[-1] at their start
    uint32_t list_mode;
};
template <class R>
struct Work {
    PathRec<R>* paths;
    HitRecD<R>* hits;
    ResRec<R>* res;
    uint32_t* active[2];        // extend input of depth d: active[d & 1], kShards x cap
    uint32_t* mq;               // material queues: (m * kShards + s) * cap
    uint32_t* counters;         // [(depth * kQueueKinds + kind) * kShards + shard] * kCounterStride
    unsigned long long* segments;
    double* acc;                // local pixels * 3
    void* pool;                 // k_paths camera-ray rings: kPoolRing PoolRays per wave
};
template <class R>
__host__ __device__ __forceinline__ uint32_t* counter(const Work<R>& w, int d, int kind, int s) {
    return w.counters + (static_cast<size_t>((d * kQueueKinds + kind) * kShards + s)) * kCounterStride;
}

__device__ __forceinline__ int global_row(const PassGeom& g, int ly) {  // row-interleaved band partition
    const uint32_t b = g.fd_band_rows.div(static_cast<uint32_t>(ly));
    return static_cast<int>(b) * (g.band_rows * g.band_count) + g.band_index * g.band_rows + (ly - static_cast<int>(b) * g.band_rows);
}
// slot -> (qi: tile-order pixel or list entry, j: sample of the pass): sample-major slots (j * npix_pad + qi), or
// entry-major ones in list_mode 1 (qi * k + j, npix_pad == k)
__device__ __forceinline__ void slot_split(const PassGeom& g, uint32_t slot, uint32_t& qi, uint32_t& j) {
    const uint32_t a = g.fd_npix.div(slot), b = slot - a * g.npix_pad;
    qi = g.list_mode ? a : b;
    j = g.list_mode ? b : a;
}
__device__ __forceinline__ bool slot_pixel(const PassGeom& g, uint32_t qi, int& lx, int& ly) {
    if (g.list) {
        if (qi >= g.nlist) return false;
        const uint32_t p = g.list[qi];
        ly = static_cast<int>(g.fd_w.div(p));
        lx = static_cast<int>(p - static_cast<uint32_t>(ly) * static_cast<uint32_t>(g.W));
        return true;
    }
    const uint32_t tile = qi >> 6, within = qi & 63u;
    const uint32_t ty = g.fd_tiles_x.div(tile);
    lx = static_cast<int>((tile - ty * g.tiles_x) * 8 + (within & 7u));
    ly = static_cast<int>(ty * 8 + (within >> 3));
    return lx < g.W && ly < g.rows;
}

// Wave-aggregated append to one shard: one atomic per wave, lanes write in lane order.
__device__ __forceinline__ void wave_append(bool pred, uint32_t val, uint32_t* shard_buf, uint32_t* ctr) {
    const uint64_t mask = __ballot(pred);
    if (mask == 0) return;
    const int leader = __ffsll(static_cast<long long>(mask)) - 1;
    uint32_t base = 0;
    if (static_cast<int>(__lane_id()) == leader) base = atomicAdd(ctr, static_cast<uint32_t>(__popcll(mask)));
    base = __shfl(base, leader);
    if (pred) {
        const uint32_t off = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
        shard_buf[base + off] = val;
    }
}

// Appends every lane with mtype in [0, kNumMatTypes) to its material queue (this wave's shard) with ONE vector atomic:
// lane m reserves the slots of material m, so the wave pays one atomic round trip instead of one per material.
template <class R>
__device__ __forceinline__ void append_by_material(int mtype, uint32_t q, const Work<R>& w, const PassGeom& g, int d, int shard) {
    uint64_t masks[kNumMatTypes];
    uint64_t any = 0;
#pragma unroll
    for (int m = 0; m < kNumMatTypes; ++m) {
        masks[m] = __ballot(mtype == m);
        any |= masks[m];
    }
    if (any == 0) return;
    const int lane = static_cast<int>(__lane_id());
    uint64_t my_mask = 0;
#pragma unroll
    for (int m = 0; m < kNumMatTypes; ++m)
        if (lane == m) my_mask = masks[m];
    uint32_t base = 0;
    if (lane < kNumMatTypes && my_mask != 0) base = atomicAdd(counter(w, d, 1 + lane, shard), static_cast<uint32_t>(__popcll(my_mask)));
    base = __shfl(base, mtype >= 0 ? mtype : 0);  // all lanes: lanes 0..4 own the reservations
    if (mtype >= 0) {
        uint64_t mine = masks[0];
#pragma unroll
        for (int m = 1; m < kNumMatTypes; ++m)
            if (mtype == m) mine = masks[m];
        const uint32_t off = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mine >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mine), 0u));
        w.mq[static_cast<size_t>(mtype * kShards + shard) * g.cap + base + off] = q;
    }
}

// Exclusive prefix of the n <= 64 shard counts v (held by threads 0..n-1) into pre[0..n] (pre[n] = total), by one wave
// scan; independent of the block size.
__device__ __forceinline__ void block_prefix(uint32_t* pre, int n, uint32_t v) {
    const int t = threadIdx.x;
    if (t < 64) {
        uint32_t x = t < n ? v : 0u;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (t >= off) x += y;
        }
        if (t < n) pre[t + 1] = x;
        if (t == 0) pre[0] = 0u;
    }
    __syncthreads();
}
// Segment of item i: largest s with pre[s] <= i (pre strictly describes n segments).
__device__ __forceinline__ int find_segment(const uint32_t* pre, int n, uint32_t i) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// ------------------------------------------------------------------------------------------------ kernels
// engine.h:58-68 + camera.h:38-47 for sample j of the pass at local pixel (lx, ly) (slot_split).
// Runs inside the depth-0 extend: the camera ray never round-trips through HBM.
template <class R>
__device__ __forceinline__ void cam_ray(const PassGeom& g, const CameraRec<R>& cam, uint32_t j, int lx, int ly, Ray<R>& ray, uint64_t& rng_out) {
    const int gy = global_row(g, ly);
    const uint32_t pixel = static_cast<uint32_t>(gy) * static_cast<uint32_t>(g.W) + static_cast<uint32_t>(lx);
    uint64_t rng = splitmix64(((static_cast<uint64_t>(pixel) << 32) | (g.sample_base + j)) ^ g.seed_mix);  // == pcg_seed(g.seed, ...)
    const R ru = uniform<R>(rng);
    const R rv = uniform<R>(rng);
    const R s = div_rcp(R(lx) + ru, R(g.W - 1), static_cast<R>(g.inv_w1));  // == (lx + ru) / (W - 1), same bits
    const R t = div_rcp(R(g.H - 1 - gy) + rv, R(g.H - 1), static_cast<R>(g.inv_h1));
    V3<R> p;
    for (;;) {  // random_in_unit_disk (vec3.h:137-143): x, then y
        p.x = uniform_pm1<R>(rng);
        p.y = uniform_pm1<R>(rng);
        p.z = R(0);
        if (len2(p) >= R(1)) continue;
        break;
    }
    const V3<R> rd = cam.lens_radius * p;
    const V3<R> offset = rd.x * ld3(cam.u) + rd.y * ld3(cam.v);
    ray.o = ld3(cam.origin) + offset;
    ray.d = ld3(cam.llc) + s * ld3(cam.horizontal) + t * ld3(cam.vertical) - ld3(cam.origin) - offset;
    ray.tm = uniform<R>(rng, cam.time0, cam.time1);
    rng_out = rng;
}
template <class R>
__device__ __forceinline__ void gen_ray(const PassGeom& g, const CameraRec<R>& cam, uint32_t j, int lx, int ly, PathState<R>& st) {
    cam_ray(g, cam, j, lx, ly, st.ray, st.rng);
    st.T = mk(R(1), R(1), R(1));
    st.L = mk(R(0), R(0), R(0));
}

// material.h scatter() for one hit of material type M (compile time: one shade kernel per material type, so a wave
// never carries another material's code or registers); returns false when the path ends here.
// Shared steps already taken for the whole wave (k_paths_g), or null:
//   pre    the lane's random_in_unit_sphere() draw (coop_unit_sphere);
//   unitv  unit_vector of that draw (lambertian) or of the ray direction (metal, dielectric);
//   texc   the material's texture value at the hit (lambertian, isotropic).
template <class R, uint32_t M, uint32_t TF>
__device__ __forceinline__ bool scatter(const DevScene<R>& S, const MatRec<R>& m, const Surf<R>& s, PathState<R>& st, V3<R>& att, V3<R>& dir,
                                        const V3<R>* pre = nullptr, const V3<R>* unitv = nullptr, const V3<R>* texc = nullptr) {
    if (M == MAT_LAMBERTIAN) {  // material.h:20-43
        const V3<R> rv = unitv ? *unitv : unit(pre ? *pre : in_unit_sphere<R>(st.rng));
        dir = s.n + rv;
        if (near_zero(dir)) dir = s.n;
        att = texc ? *texc : mat_tex_value<R, TF>(S, m, s.u, s.v, s.p);
        return true;
    } else if (M == MAT_METAL) {  // material.h:45-61
        const V3<R> reflected = reflect(unitv ? *unitv : unit(st.ray.d), s.n);
        dir = reflected + m.fuzz * (pre ? *pre : in_unit_sphere<R>(st.rng));
        att = ld3(m.albedo);
        return dot(dir, s.n) > R(0);
    } else if (M == MAT_DIELECTRIC) {  // material.h:63-99
        att = mk(R(1), R(1), R(1));
        const R ratio = s.ff ? (R(1) / m.ir) : m.ir;
        const V3<R> ud = unitv ? *unitv : unit(st.ray.d);
        const R cos_theta = fmin(dot(-ud, s.n), R(1));
        const R sin_theta = sqrt_rn(R(1) - cos_theta * cos_theta);
        const bool cannot = ratio * sin_theta > R(1);
        bool refl = cannot;
        if (!cannot) {
            R r0 = (R(1) - ratio) / (R(1) + ratio);
            r0 = r0 * r0;
            const R refl_p = r0 + (R(1) - r0) * pow5(R(1) - cos_theta);
            refl = refl_p > uniform<R>(st.rng);
        }
        dir = refl ? reflect(ud, s.n) : refract(ud, s.n, ratio);
        return true;
    } else if (M == MAT_ISOTROPIC) {  // material.h:120-135
        dir = pre ? *pre : in_unit_sphere<R>(st.rng);
        att = texc ? *texc : mat_tex_value<R, TF>(S, m, s.u, s.v, s.p);
        return true;
    }
    return false;  // diffuse_light (material.h:106-110)
}

// Emission + scatter of one hit of the fused extend variant, read entirely from the LDS scene image: the surface
// (sphere.h:57-63 via the slot's centre/radius/motion planes, which are the f64 values the hit test used) and the
// material (the image's shading table, layout.h) -- no dependent global loads after a hit.  The arithmetic and the
// draws are those of prim_surface + scatter<R, M, kTexBasic> (tex_value of a solid or solid/solid checker texture).
// Returns true when the path continues (st then holds the scattered ray and the updated throughput).
__device__ __forceinline__ V3<double> lds_mat_color(const uint8_t* lds, uint32_t e) {
    const double2* m = reinterpret_cast<const double2*>(lds + kLdsOffMat) + 2 * e;
    const double2 a = m[0], b = m[1];
    return mk(a.x, a.y, b.x);
}
// pre_ps: the lane's random_in_unit_sphere() draw, already taken by the wave (coop_unit_sphere) when non-null.
__device__ __forceinline__ bool shade_hit_lds(const uint8_t* lds, uint32_t slot, uint32_t mtype, double t, bool last, PathState<double>& st,
                                              const V3<double>* pre_ps = nullptr) {
    using R = double;
    const double2* sp = reinterpret_cast<const double2*>(lds + kLdsOffSph) + slot;
    const double2 a = sp[0], b = sp[kLdsSlotCap];
    const uint32_t code = reinterpret_cast<const uint32_t*>(lds + kLdsOffRef)[slot];
    const uint32_t mi = reinterpret_cast<const uint16_t*>(lds + kLdsOffMatIdx)[slot];
    V3<R> center{a.x, a.y, b.x};
    center.y = center.y + st.ray.tm * reinterpret_cast<const double*>(lds + kLdsOffMov)[slot];  // dy = -0: static
    (void)code;
    Surf<R> s;
    s.p = st.ray.at(t);
    set_face_normal(s, st.ray, reinterpret_cast<const double*>(lds + kLdsOffInvR)[slot] * (s.p - center));  // (p - c) / r
    const uint32_t e = mi & ~kLdsMatChecker;
    const bool checker = (mi & kLdsMatChecker) != 0;
    if (mtype == MAT_LIGHT) {  // material.h:114-116; diffuse_light never scatters
        st.L = st.L + st.T * lds_mat_color(lds, (checker && checker_odd(s.p)) ? e + 1 : e);
        return false;
    }
    if (last) return false;
    // The three materials of a wave share their costly steps (each lane still draws exactly its own material's
    // sequence): lambertian and metal both start with random_in_unit_sphere() (material.h:33, :55 -- metal's
    // unit_vector(r_in.direction()) draws nothing), and all three need one unit_vector (of that sample for
    // lambertian, of the ray direction for metal and dielectric), so the wave runs one rejection loop and one
    // sqrt + divide sequence instead of one per material present.
    const bool lamb = mtype == MAT_LAMBERTIAN;
    V3<R> ps = mk(R(0), R(0), R(0));
    if (pre_ps) ps = *pre_ps;
    else if (mtype != MAT_DIELECTRIC) ps = in_unit_sphere<R>(st.rng);
    const V3<R> u = unit(lamb ? ps : st.ray.d);
    V3<R> att, dir;
    if (lamb) {  // material.h:20-43
        dir = s.n + u;
        if (near_zero(dir)) dir = s.n;
        att = lds_mat_color(lds, (checker && checker_odd(s.p)) ? e + 1 : e);
    } else if (mtype == MAT_METAL) {  // material.h:45-61
        const double2* m = reinterpret_cast<const double2*>(lds + kLdsOffMat) + 2 * e;
        const double2 ma = m[0], mb = m[1];
        dir = reflect(u, s.n) + mb.y * ps;
        att = mk(ma.x, ma.y, mb.x);
        if (!(dot(dir, s.n) > R(0))) return false;
    } else {  // dielectric, material.h:63-99
        // the table entry holds (1 / ir, r0 of the front face, r0 of the back face, ir), each computed on the host by
        // the same IEEE operations material.h:74 and :93-94 apply (lds_scene_image): no division per hit
        const double2* me = reinterpret_cast<const double2*>(lds + kLdsOffMat) + 2 * e;
        const double2 m0 = me[0], m1 = me[1];
        att = mk(R(1), R(1), R(1));
        const R ratio = s.ff ? m0.x : m1.y;  // front_face ? (1.0 / ir) : ir
        const R cos_theta = fmin(dot(-u, s.n), R(1));
        const R sin_theta = sqrt_rn(R(1) - cos_theta * cos_theta);
        const bool cannot = ratio * sin_theta > R(1);
        bool refl = cannot;
        if (!cannot) {
            const R r0 = s.ff ? m0.y : m1.x;  // ((1 - ratio) / (1 + ratio))^2
            const R refl_p = r0 + (R(1) - r0) * pow5(R(1) - cos_theta);
            refl = refl_p > uniform<R>(st.rng);
        }
        dir = refl ? reflect(u, s.n) : refract(u, s.n, ratio);
    }
    st.T = st.T * att;
    st.ray.o = s.p;
    st.ray.d = dir;
    return true;
}

#ifndef ART_LDS_BLOCK
#define ART_LDS_BLOCK 1024
#endif
// Blocks of the LDS-scene variant: one block per CU holds the scene image once for 16 waves (4 per SIMD).
constexpr int kBlockL = ART_LDS_BLOCK;
// LDS bytes of one k_extend block: scene image (L) + per-lane stack + the shard prefix array.
__host__ __device__ constexpr size_t extend_pre_offset(bool L, uint32_t stack) {
    return ((L ? kLdsImageBytes + sizeof(int16_t) * stack * kBlockL : sizeof(int32_t) * stack * kBlock) + 15u) & ~size_t(15);
}

// Copies the LDS scene image (layout.h) into LDS in one round: every lane issues all of its 16-B loads before its
// first store, so the block pays one global-load latency instead of one per plane.
template <int B>
__device__ __forceinline__ void load_lds_image(const uint8_t* image, uint8_t* lds) {
    constexpr uint32_t n16 = kLdsImageBytes / 16;
    constexpr int per = static_cast<int>((n16 + B - 1) / B);
    const uint4* src = reinterpret_cast<const uint4*>(image);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    uint4 v[per];
#pragma unroll
    for (int j = 0; j < per; ++j) {
        const uint32_t i = threadIdx.x + static_cast<uint32_t>(j) * B;
        if (i < n16) v[j] = src[i];
    }
#pragma unroll
    for (int j = 0; j < per; ++j) {
        const uint32_t i = threadIdx.x + static_cast<uint32_t>(j) * B;
        if (i < n16) dst[i] = v[j];
    }
}

// L: the scene is LDS-resident (DevScene::lds_image, spheres-only f64): nodes and leaf spheres are read from LDS.
// FUSE (L scenes with solid/checker textures, no media): every hit is shaded in place (shade_hit) and goes straight to
// the next depth's active queue -- no hit record, no material queues, no k_shade launches, one path-record round trip
// per bounce.
template <class R, uint32_t F, bool L, bool FUSE>
__global__ __launch_bounds__(L ? kBlockL : kBlock, L ? 1 : ART_EXTEND_MIN_WAVES) void k_extend(DevScene<R> S, PassGeom g, CameraRec<R> cam,
                                                                                                 Work<R> w, int d) {
    constexpr int B = L ? kBlockL : kBlock;
    // dynamic LDS: [scene image (L only)][traversal stack: g.stack entries x B lanes] (sized per scene at launch)
    // dynamic LDS only, so the scene image starts at LDS address 0 (device.h lds_f4)
    extern __shared__ __align__(16) uint8_t smem[];
    uint32_t* pre = reinterpret_cast<uint32_t*>(smem + extend_pre_offset(L, g.stack));
    const uint8_t* lds = smem;
    // row 0 of the stack region is this lane's sentinel (device.h traverse), entries start at row 1
    StackT<L>* stk = reinterpret_cast<StackT<L>*>(smem + (L ? kLdsImageBytes : 0u)) + B + stack_column<L>(threadIdx.x);
    stk[-B] = static_cast<StackT<L>>(kNodeEmpty);

    // input: depth 0 = every slot (identity; padding slots are skipped), deeper = the kShards active shards
    uint32_t count;
    if (d == 0) {
        count = g.P;
    } else {
        block_prefix(pre, kShards, threadIdx.x < kShards ? *counter(w, d, 0, threadIdx.x) : 0u);
        count = pre[kShards];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(w.segments, static_cast<unsigned long long>(d == 0 ? g.live : count));
    if constexpr (L) {
        // deep bounces have few paths: blocks without a batch leave before paying for the image
        if (static_cast<uint64_t>(blockIdx.x) * B >= count) return;
        load_lds_image<B>(S.lds_image, smem);
        __syncthreads();
    }
    const uint32_t* in = w.active[d & 1];
    const uint32_t wave = blockIdx.x * (B / 64) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (B / 64);
    const int shard = static_cast<int>(wave % kShards);
#ifdef ART_STATS
    unsigned long long tm_load = 0, tm_trace = 0, tm_shade = 0, tm_app = 0, tm_prev = __builtin_amdgcn_s_memtime();
#define ART_TICK(acc)                                               \
    do {                                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc += now_ - tm_prev;                                      \
        tm_prev = now_;                                             \
    } while (0)
#else
#define ART_TICK(acc)
#endif
    for (uint32_t b = wave; b * 64u < count; b += nwaves) {
        const uint32_t i = b * 64u + __lane_id();
        int mtype = -1;
        bool cont = false;  // FUSE: the path continues at depth d + 1
        uint32_t q = 0;
        bool live = i < count;
        PathState<R> st;
        if (live) {
            if (d == 0) {
                q = i;
                int lx, ly;
                uint32_t qi, j;
                slot_split(g, i, qi, j);
                live = slot_pixel(g, qi, lx, ly);
                if (live) gen_ray(g, cam, j, lx, ly, st);
            } else {
                const int s = find_segment(pre, kShards, i);
                q = in[s * g.cap + (i - pre[s])];
                // FUSE: the throughput/radiance line is needed after the traversal; issuing it with the ray line
                // puts its HBM latency under the traversal instead of after it
                load_path(w.paths, q, st, FUSE);
            }
        }
        ART_TICK(tm_load);
        if (FUSE) {
            R t;
            HitOut h{0, 0, kMatUnknown};
            const bool hitf = live && trace_world<R, F, B, L>(S, lds, st.ray, stk, st.rng, t, h);
            ART_TICK(tm_trace);
            if (hitf) {
                if constexpr (std::is_same<R, double>::value) cont = shade_hit_lds(lds, h.obj >> 16, h.mt, t, d + 1 >= g.max_depth, st);
                if (cont) store_path(w.paths, q, st);
                else store_res(w.res, q, st.L);
            } else if (live) {  // engine.h:455-456: miss -> background
                st.L = st.L + st.T * mk(S.bg[0], S.bg[1], S.bg[2]);
                store_res(w.res, q, st.L);
            }
            ART_TICK(tm_shade);
        } else if (live) {
            R t;
            HitOut h{0, 0, kMatUnknown};
            if (trace_world<R, F, B, L>(S, lds, st.ray, stk, st.rng, t, h)) {
                w.hits[q] = HitRecD<R>{t, h.prim, h.obj};
                if (L && h.mt != kMatUnknown) {
                    mtype = static_cast<int>(h.mt);  // from the LDS image: no dependent global loads
                } else {
                    uint32_t m;
                    if ((F & F_MEDIA) && h.prim == kMediumHit) {
                        m = static_cast<uint32_t>(S.objs[S.world[h.obj & 0xFFFFu]].b);
                    } else if (F == F_SPHERE) {
                        m = S.spheres[primref_index(h.prim)].mat;
                    } else {
                        const uint32_t idx = primref_index(h.prim);
                        switch (primref_type(h.prim)) {
                            case PRIM_SPHERE: m = S.spheres[idx].mat; break;
                            case PRIM_TRIANGLE: m = S.tris[idx].mat; break;
                            case PRIM_RECT: m = S.rects[idx].mat; break;
                            default: m = S.boxes[idx].mat; break;
                        }
                    }
                    mtype = static_cast<int>(S.mats[m].type);
                }
                if (d == 0) store_path(w.paths, q, st);
                else if (F & F_MEDIA) store_rng(w.paths, q, st.rng);
            } else {  // engine.h:455-456: miss -> background
                if (d != 0) load_path(w.paths, q, st, true);
                st.L = st.L + st.T * mk(S.bg[0], S.bg[1], S.bg[2]);
                store_res(w.res, q, st.L);
            }
        }
        if constexpr (FUSE) wave_append(cont, q, w.active[(d + 1) & 1] + static_cast<size_t>(shard) * g.cap, counter(w, d + 1, 0, shard));
        else append_by_material(mtype, q, w, g, d, shard);
        ART_TICK(tm_app);
    }
#ifdef ART_STATS
    if (__lane_id() == 0) {
        atomicAdd(&g_art_stats[8], tm_load);
        atomicAdd(&g_art_stats[9], tm_trace);
        atomicAdd(&g_art_stats[10], tm_shade);
        atomicAdd(&g_art_stats[11], tm_app);
    }
#endif
}

// Persistent-path variant of the fused LDS scene (EXT_MEGA): one launch traces a whole pass.  Every lane owns one
// path at a time and keeps it in registers from its camera ray to its end (engine.h:447-466 flattened: trace,
// shade_hit_lds, repeat until a miss, an absorption, a light or max_depth), then writes the slot's radiance and takes
// the next slot -- no path records, queues or per-depth launches, and the deep bounces of old paths share the waves
// with the first bounces of new ones instead of running as a tail of nearly empty launches.  Slots are claimed in
// increasing order in wave chunks of PassGeom::chunk from one counter (one atomic per chunk).  The bounce arithmetic
// and the RNG draws are those of the fused k_extend, so images are bit-identical to the wavefront variants.
// The slots a wave claims per atomic on the pass counter: PassGeom::chunk = path_chunk (pass_plan.h).
// Camera-ray pool: a path start is run by the whole wave for however few lanes start a path (~a third
// of them per round), so the camera rays are generated 64 at a time -- one per lane, converged -- into a per-wave ring
// in global memory (L2-resident: 8 KiB per wave), and a starting lane loads the next ring entry instead.  Entry pos
// holds the ray of slot base[(pos / 64) & 1] + pos % 64; tm = NaN marks a padding slot of a partial tile.
// ART_POOL_RING: ring entries per wave.  128: two batches of 64, refilled when a batch's worth is free, so a round's
// takers always find entries; 96 (default): refilled when at most 32 are left, so a round with more takers than
// entries leaves the rest idle for that round.  Measured (r3m, scene 1, PMC per segment; XCD-contiguous rings): HBM
// reads 3.50 B (128) -> 0.10 B (96), writes 33.5 -> 27.9 B: the 3 MiB of rings per XCD stay in its 4 MiB L2 between a
// refill and the takes (the writes left are the 8.9 B of radiance records and dirty ring lines evicted between
// laps); Msamples/s +0.4 % (within the run-to-run spread).
#ifndef ART_POOL_RING
#define ART_POOL_RING 96
#endif
constexpr uint32_t kPoolRing = ART_POOL_RING;
static_assert(kPoolRing >= 96 && kPoolRing <= 128, "a ring holds the unread part of one batch and a whole new one");
// XCD-contiguous rings: measured (r3m, 128-entry rings) HBM reads 11.3 -> 3.5 B per segment against the
// block-major layout, Msamples/s unchanged
constexpr uint32_t kXcds = 8;  // MI355X
constexpr uint32_t kPoolWavesPerCu = 32;  // rings allocated per CU: the most waves a CU holds
struct PoolRay {
    double ox, oy, oz, dx;
    double dy, dz, tm;
    uint64_t rng;
};
// A wave's ring.  Fields other than the pointer are wave-uniform.  refill() is called by the whole wave; take() by
// the idle lanes of a round, before the round's refill (whose stores then go to entries already read).
struct RayRing {
    PoolRay* ring;
    uint32_t head, tail;    // positions consumed / produced
    uint32_t base0, base1;  // first slot of the batch in ring half 0 / 1
    uint32_t cur, end;      // the wave's claimed slot chunk [cur, end)
    bool exhausted;         // every slot of the pass is in a batch
    // wave w of block b: the rings of one XCD's blocks are contiguous (blocks go to the 8 XCDs round
    // robin, block b to XCD b % 8), so each XCD's rings spread over all of its L2's sets instead of every block's
    // chunk landing on the same sets (block-major rings of one XCD lie 8 chunks apart: a power-of-two stride)
    __device__ __forceinline__ void init(void* pool, uint32_t block, uint32_t nblocks, uint32_t waves_per_block, uint32_t w) {
        uint32_t wave = block * waves_per_block + w;
        {
            const uint32_t per_xcd = (nblocks + kXcds - 1) / kXcds;
            wave = ((block % kXcds) * per_xcd + block / kXcds) * waves_per_block + w;
        }
        ring = static_cast<PoolRay*>(pool) + static_cast<size_t>(wave) * kPoolRing;
        head = tail = base0 = base1 = cur = end = 0;
        exhausted = false;
    }
    __device__ __forceinline__ void refill(const PassGeom& sg, const CameraRec<double>& sc, uint32_t* next_slot, uint32_t lane) {
        if (cur == end) {
            const uint32_t chunk = sg.chunk;
            uint32_t nb = 0;
            if (lane == 0) nb = atomicAdd(next_slot, chunk);
            nb = __shfl(nb, 0);
            cur = nb;
            end = nb + chunk;
        }
        const uint32_t b = cur;
        cur += 64;
        const uint32_t slot = b + lane;
        __asm__ volatile("" ::: "memory");  // the LDS camera loads stay here
        PoolRay e;
        e.tm = __builtin_nan("");
        int lx, ly;
        uint32_t qi, j;
        slot_split(sg, slot, qi, j);
        if (slot < sg.P && slot_pixel(sg, qi, lx, ly)) {
            Ray<double> r;
            uint64_t rng;
            cam_ray(sg, sc, j, lx, ly, r, rng);
            e.ox = r.o.x; e.oy = r.o.y; e.oz = r.o.z; e.dx = r.d.x;
            e.dy = r.d.y; e.dz = r.d.z; e.tm = r.tm; e.rng = rng;
        }
        ring[(tail + lane) % kPoolRing] = e;
        if ((tail / 64u) & 1u) base1 = b;
        else base0 = b;
        tail += 64;
        if (b + 64u >= sg.P) exhausted = true;
    }
    // The idle lane of rank `rank`: 1 = a path starts (st, q), 0 = a padding slot (the lane idles a round),
    // 2 = the pass is drained.
    __device__ __forceinline__ int take(uint32_t rank, uint32_t P, PathState<double>& st, uint32_t& q) const {
        const uint32_t pos = head + rank;
        const uint32_t slot = (((pos / 64u) & 1u) ? base1 : base0) + pos % 64u;
        if (pos >= tail) return exhausted ? 2 : 0;  // 0: the ring ran dry this round (kPoolRing < 128 only)
        if (slot >= P) return 2;
        const PoolRay& e = ring[pos % kPoolRing];
        const double tm = e.tm;
        if (tm != tm) return 0;
        st.ray.o = mk(e.ox, e.oy, e.oz);
        st.ray.d = mk(e.dx, e.dy, e.dz);
        st.ray.tm = tm;
        st.rng = e.rng;
        st.T = mk(1.0, 1.0, 1.0);
        st.L = mk(0.0, 0.0, 0.0);
        q = slot;
        return 1;
    }
    // after the round's take(): n entries consumed; refill when a batch's worth is free, so an entry is read at
    // least one round after its stores (ordered by the s_waitcnt vmcnt(0) the path loops place after the trace)
    __device__ __forceinline__ void advance(uint32_t n, const PassGeom& sg, const CameraRec<double>& sc, uint32_t* next_slot, uint32_t lane) {
        head = min(head + n, tail);
        if (!exhausted && tail - head <= kPoolRing - 64u) refill(sg, sc, next_slot, lane);
    }
    __device__ __forceinline__ void start(const PassGeom& sg, const CameraRec<double>& sc, uint32_t* next_slot, uint32_t lane) {
        refill(sg, sc, next_slot, lane);
        if (kPoolRing >= 128 && !exhausted) refill(sg, sc, next_slot, lane);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
};
__host__ __device__ constexpr size_t paths_stack_bytes(uint32_t stack) { return (sizeof(int16_t) * stack * kBlockL + 15u) & ~size_t(15); }
constexpr size_t kJumpBytes = sizeof(JumpEntry) * kJumpEntries;
// The world list and object records, copied into LDS by every k_paths block: each trace walks them, and from global
// memory they were three dependent vector loads (world slot -> object -> hoisted leaf) at the start of every trace
// (vector, not scalar, loads: the kernel stores, so the compiler cannot prove them unclobbered).  The LDS scene
// path requires a world of at most kPathsWorldCap objects (lds_scene_image; after world merging the benchmark scene
// has one).
constexpr uint32_t kPathsWorldCap = 16;
constexpr size_t kPathsWorldBytes = sizeof(int32_t) * kPathsWorldCap + sizeof(ObjRec<double>) * kPathsWorldCap;
__host__ __device__ constexpr size_t paths_lds_head(uint32_t stack) {
    return ((kLdsImageBytes + paths_stack_bytes(stack) + kJumpBytes + sizeof(CameraRec<double>) + sizeof(PassGeom)) + 15u) & ~size_t(15);
}
__host__ __device__ constexpr size_t paths_lds_bytes(uint32_t stack) { return paths_lds_head(stack) + kPathsWorldBytes; }
#if ART_SPLIT_PATHS == 0 || ART_SPLIT_PATHS == 2
__global__ __launch_bounds__(kBlockL, 1) void k_paths(DevScene<double> S0, PassGeom g, CameraRec<double> cam, Work<double> w, uint32_t* next_slot) {
    using R = double;
    constexpr int B = kBlockL;
    // dynamic LDS only (no static __shared__, so the image starts at LDS address 0 and every image offset is an
    // immediate): [scene image][traversal stack][camera][pass geometry] -- the camera and pass geometry are read
    // from LDS where a new path starts instead of being held in registers for the whole kernel (as kernel arguments
    // they pin ~60 SGPRs, which spill)
    extern __shared__ __align__(16) uint8_t smem[];
    const uint8_t* lds = smem;
    StackT<true>* stk = reinterpret_cast<StackT<true>*>(smem + kLdsImageBytes) + B + stack_column<true>(threadIdx.x);
    JumpEntry* jt = reinterpret_cast<JumpEntry*>(smem + kLdsImageBytes + paths_stack_bytes(g.stack));
    CameraRec<double>& s_cam = *reinterpret_cast<CameraRec<double>*>(smem + kLdsImageBytes + paths_stack_bytes(g.stack) + kJumpBytes);
    PassGeom& s_g = *reinterpret_cast<PassGeom*>(smem + kLdsImageBytes + paths_stack_bytes(g.stack) + kJumpBytes + sizeof(CameraRec<double>));
    stk[-B] = static_cast<StackT<true>>(kNodeEmpty);
    load_lds_image<B>(S0.lds_image, smem);
    if (threadIdx.x < static_cast<uint32_t>(kJumpEntries)) jt[threadIdx.x] = pcg_jump(3u * threadIdx.x);
    if (threadIdx.x == 0) {
        s_cam = cam;
        s_g = g;
        if (g.list_mode) {  // the list's entry count, on the device (PassGeom::list_mode)
            const uint32_t n = g.list[-1];
            s_g.nlist = n;
            s_g.P = n * g.k;
        }
    }
    DevScene<double> S = S0;
    {
        uint8_t* wb = smem + paths_lds_head(g.stack);
        uint8_t* ob = wb + sizeof(int32_t) * kPathsWorldCap;
        if (threadIdx.x < static_cast<uint32_t>(S0.nworld)) reinterpret_cast<int32_t*>(wb)[threadIdx.x] = S0.world[threadIdx.x];
        if (threadIdx.x < S0.n_objs * (sizeof(ObjRec<double>) / 16))
            reinterpret_cast<uint4*>(ob)[threadIdx.x] = reinterpret_cast<const uint4*>(S0.objs)[threadIdx.x];
        S.world = reinterpret_cast<const int32_t*>(wb);
        S.objs = reinterpret_cast<const ObjRec<double>*>(ob);
    }
    __syncthreads();
    const uint32_t lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const V3<R> bg = mk(S.bg[0], S.bg[1], S.bg[2]);
    bool busy = false, drained = false;
    uint32_t q = 0;
    int depth = 0;
    PathState<R> st;
    unsigned long long segs = 0;
#ifdef ART_STATS
    unsigned long long tm_load = 0, tm_trace = 0, tm_shade = 0, tm_app = 0, tm_prev = __builtin_amdgcn_s_memtime();
#endif
    RayRing rr;
    rr.init(w.pool, blockIdx.x, gridDim.x, B / 64, threadIdx.x / 64);
    rr.start(s_g, s_cam, next_slot, lane);
    for (;;) {
        // every idle lane takes the next ring entry (a padding slot of a partial tile leaves it idle a round)
        const uint64_t idle = __ballot(!busy && !drained);
        if (idle) {
            const uint32_t n = static_cast<uint32_t>(__popcll(idle));
            const uint32_t rank = static_cast<uint32_t>(__popcll(idle & below));
            if (!busy && !drained) {
                const int got = rr.take(rank, s_g.P, st, q);  // g.P, or the device count's (list_mode): read where used
                drained = got == 2;
                busy = got == 1;
                depth = 0;
            }
            rr.advance(n, s_g, s_cam, next_slot, lane);
        }
        ART_TICK(tm_load);
        if (__ballot(busy) == 0) {
            if (__ballot(!drained) == 0) break;
            continue;
        }
        R t = R(0);
        HitOut h{0, 0, kMatUnknown};
        bool hitw = false;
        if (busy) {
            ++segs;
            hitw = trace_world<R, kFeatSpheres, B, true>(S, lds, st.ray, stk, st.rng, t, h);
#if ART_LDS_LEAF_NOREF
            if (hitw) h.mt = reinterpret_cast<const uint32_t*>(lds + kLdsOffRef)[h.obj >> 16] >> kLdsRefMatShift;
#endif
        }
        // the ring stores of this round's refill (issued before the trace) are complete before the next round's loads
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ART_TICK(tm_trace);
        // the whole wave draws random_in_unit_sphere for its lambertian and metal hits (material.h:33, :55), which
        // scatter with it first; lights and the max_depth bounce draw nothing
        const bool need = busy && hitw && (h.mt == MAT_LAMBERTIAN || h.mt == MAT_METAL) && depth + 1 < g.max_depth;
        const V3<R> ps = coop_unit_sphere<R>(need, st.rng, jt);
        if (busy) {
            bool cont = false;
            if (hitw) {
                cont = shade_hit_lds(lds, h.obj >> 16, h.mt, t, depth + 1 >= g.max_depth, st, &ps);
            } else {  // engine.h:455-456: miss -> background
                st.L = st.L + st.T * bg;
            }
            ART_TICK(tm_shade);
            if (cont) {
                ++depth;
            } else {
                store_res(w.res, q, st.L);
                busy = false;
            }
        }
        ART_TICK(tm_app);
    }
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off);
    if (lane == 0) atomicAdd(w.segments, segs);
#ifdef ART_STATS
    if (lane == 0) {
        atomicAdd(&g_art_stats[8], tm_load);
        atomicAdd(&g_art_stats[9], tm_trace);
        atomicAdd(&g_art_stats[10], tm_shade);
        atomicAdd(&g_art_stats[11], tm_app);
    }
#endif
}

#endif  // ART_SPLIT_PATHS == 0 || ART_SPLIT_PATHS == 2

// Persistent paths over the HBM scene (EXT_MEGA_G): the k_paths loop for every scene that does not fit the LDS
// image (triangles, rects, boxes, transforms, media, noise/image textures).  A lane owns one path from its camera
// ray to its end: trace_world over the global BVHs (the k_extend traversal, LDS stack) and, in place, world_surface +
// the material's scatter (the k_shade arithmetic, one switch over the material type instead of one launch per type),
// so the RNG draws and every f64 operation are those of the wavefront kernels and images are bit-identical to them.
// F / TF: the scene's primitive and texture features (smallest instantiation that covers them).
constexpr uint32_t kLdsPartialMinNodes = 64;
#ifndef ART_PATHS_G_WAVES
#define ART_PATHS_G_WAVES 3  // 3 waves per SIMD (<= 168 VGPRs): measured best over 2 and 4 (cow +22 %, final +18 %, dino +21 % over 2)
#endif
#ifdef ART_TRACE
// Path tracing diagnostics (libart_trace.so builds only): ART_TRACE="pixel:sample" prints every segment of that one
// path from k_paths_g as bit patterns, in the format of the oracle's ORC_TRACE, so the two can be diffed.
__device__ long long g_trace_pixel = -1, g_trace_sample = -1;
#define ART_DBITS(x) static_cast<unsigned long long>(__double_as_longlong(x))
#endif
// LM (LDS BVH): a scene whose BVH nodes and primitive references -- and triangles, for a kernel with triangles --
// fit beside the stacks (small meshes: dino; the Next-Week final's 559 nodes) runs one 768-lane block per CU with
// those arrays copied into LDS: node and triangle fetches at LDS latency instead of L2's.  The other arrays stay in
// HBM.  The copies are plain LDS arrays reached through the DevScene pointers: the compiler infers their address
// space (ds_read, no flat loads).
constexpr int kBlockM = 256 * ART_PATHS_G_WAVES;  // one LM block per CU at the kernel's occupancy
constexpr size_t kPathsGLdsCap = 160 * 1024;
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15u) & ~size_t(15); }
__host__ __device__ constexpr size_t align128(size_t x) { return (x + 127u) & ~size_t(127); }
// s16: 16-bit stack entries (F_CODE16 instantiations, device.h StackF)
__host__ __device__ constexpr size_t paths_g_stack_bytes(uint32_t stack, int block, bool s16) { return (s16 ? 2u : 4u) * stack * block; }
__host__ __device__ constexpr size_t paths_g_head_bytes(uint32_t stack, int block, bool s16) {  // stack, camera, pass geometry, jumps, u,v
    return align16(paths_g_stack_bytes(stack, block, s16) + sizeof(CameraRec<double>) + sizeof(PassGeom)) + kJumpBytes + kUvConstBytes;
}
// LM kernels also hold the world list and the object records (a few KiB): every segment walks them, and a prim
// object's test otherwise waits on three dependent L1 loads (world slot -> object -> primitive).  The textured ones
// (noise / image) also hold the material records when there are at most kMatsLdsCap of them (the Next-Week final: 12):
// every hit's shading reads its material (type, flags, the inlined solid colour) right after the surface, and from
// HBM that is one more dependent L2 round trip per bounce.
constexpr uint32_t kMatsLdsCap = 128;
template <uint32_t TF>
__host__ __device__ constexpr uint32_t lds_mats(uint32_t n_mats) {
    return ((TF & (TF_NOISE | TF_IMAGE)) != 0 && n_mats <= kMatsLdsCap) ? n_mats : 0u;
}
__host__ __device__ constexpr size_t paths_g_world_bytes(int32_t nworld, uint32_t n_objs, uint32_t n_lds_mats) {
    return align16(sizeof(int32_t) * static_cast<uint32_t>(nworld)) + (sizeof(ObjRec<double>) + sizeof(PrimRec80)) * n_objs +
           sizeof(MatRec<double>) * n_lds_mats;
}
// LM 1's LDS copy of the leaf triangle records: TriRec112 (plane precomputed, traverse's PL 2 path)
constexpr size_t kLm1TriBytes = sizeof(TriRec112<double>);
__host__ __device__ constexpr size_t paths_g_mesh_bytes(uint32_t n_nodes, uint32_t n_primrefs, uint32_t n_tris) {  // n_tris: 0 unless F_TRI
    return sizeof(BvhNode) * n_nodes + align16(sizeof(uint32_t) * n_primrefs) + kLm1TriBytes * n_tris;
}
// Camera-ray ring in LDS (k_paths_g LM 1, ART_LDS_RING_G): the camera rays are generated 64 at a time by the whole wave,
// converged, into a per-wave ring of 64 entries in LDS, and the lanes that start a path read the next entries -- instead
// of every round's camera-ray code running diverged for the few lanes that start a path (about a third).  k_paths does
// the same through an L2-resident ring; in k_paths_g that ring's L2 round trip per take cost more than it saved (r3y:
// final -0.8 %), the LDS read does not.  An entry is 64 B: o, d, tm, rng; tm = NaN marks a padding slot of a partial
// tile (the taker idles a round), +inf a slot past the pass (the taker is drained).  Entry k holds slot b0 + k.
#ifndef ART_LDS_RING_G
#define ART_LDS_RING_G 1
#endif
constexpr uint32_t kRingG = 64;  // entries per wave
// Which kernels carry the ring: triangle-free LM 1 kernels (r5d, profiles/r5d_ab_lds_ring.txt: Cornell smoke +3.2 %,
// two perlin spheres +3.6 %, simple light +0.2 %; the mesh kernel, whose leaf triangles share the LDS, dino -1.1 %),
// except the Next-Week final's <189, 15, 1>: there the ring's registers push three loop-carried doubles into scratch
// (6 spilled VGPRs) for +0.5 %, so it keeps its spill-free ring-free form.
__host__ __device__ constexpr bool paths_g_ring(uint32_t F, int LM) {
    return ART_LDS_RING_G && LM == 1 && (F & F_TRI) == 0 && F != ((F_ALL & ~F_TRI & ~F_MEDIA_G) | F_CODE16);
}
__host__ __device__ constexpr size_t paths_g_ring_bytes(int block) { return static_cast<size_t>(block / 64) * kRingG * 64u; }
// A wave's ring is 64 entries of 8 fields (o.xyz, d.xyz, tm, rng) stored field-major (SoA: field f of entry k at
// f * 512 + k * 8 bytes), so a wave's reads and writes of one field are contiguous 8-B words (no bank conflicts; the
// AoS 64-B entries put 4 lanes on the same banks).
struct RingG {
    double* f;  // this wave's 8 x 64 doubles
    __device__ __forceinline__ double& at(uint32_t field, uint32_t k) const { return f[field * kRingG + k]; }
};
// 1 = a path starts (st, q), 0 = a padding slot (idle this round), 2 = the pass is drained
__device__ __forceinline__ int ring_take_g(const RingG& ring, uint32_t k, uint32_t b0, PathState<double>& st, uint32_t& q) {
    const double tm = ring.at(6, k);
    if (tm != tm) return 0;
    if (tm == __builtin_inf()) return 2;
    st.ray.o = mk(ring.at(0, k), ring.at(1, k), ring.at(2, k));
    st.ray.d = mk(ring.at(3, k), ring.at(4, k), ring.at(5, k));
    st.ray.tm = tm;
    st.rng = static_cast<uint64_t>(__double_as_longlong(ring.at(7, k)));
    st.T = mk(1.0, 1.0, 1.0);
    st.L = mk(0.0, 0.0, 0.0);
    q = b0 + k;
    return 1;
}
__device__ __forceinline__ void ring_fill_g(const RingG& ring, uint32_t lane, uint32_t slot, const PassGeom& sg, const CameraRec<double>& sc) {
    double v[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, __builtin_inf(), 0.0};
    if (slot < sg.P) {
        v[6] = __builtin_nan("");
        int lx, ly;
        uint32_t qi, j;
        slot_split(sg, slot, qi, j);
        if (slot_pixel(sg, qi, lx, ly)) {
            Ray<double> r;
            uint64_t rng;
            cam_ray(sg, sc, j, lx, ly, r, rng);
            v[0] = r.o.x; v[1] = r.o.y; v[2] = r.o.z; v[3] = r.d.x;
            v[4] = r.d.y; v[5] = r.d.z; v[6] = r.tm; v[7] = __longlong_as_double(static_cast<long long>(rng));
        }
    }
#pragma unroll
    for (uint32_t f = 0; f < 8; ++f) ring.at(f, lane) = v[f];
}
template <uint32_t F, uint32_t TF, int LM>
__global__ __launch_bounds__(LM ? kBlockM : kBlock, LM ? 1 : ART_PATHS_G_WAVES) void k_paths_g(DevScene<double> S0, PassGeom g, CameraRec<double> cam,
                                                                                     Work<double> w, uint32_t* next_slot) {
    using R = double;
    // explicit-LDS node reads (traverse's PL path): LM 2 for its LDS part; LM 1 for every node (the XOR near/far
    // addressing needs the explicit LDS addresses; through the LDS-inferred pointer it costs more adds)
    constexpr int kLdsNodesPL = LM == 2 ? 1 : LM == 1 ? 2 : 0;
    constexpr int B = LM ? kBlockM : kBlock;
    // dynamic LDS: [traversal stack: g.stack entries x B lanes (+ sentinel row)][camera][pass geometry][LM: nodes,
    // primrefs, triangles] -- as in k_paths, the camera and pass geometry are read from LDS where a path starts (as
    // kernel arguments held in SGPRs for the whole loop they spilled ~100 SGPRs into VGPR lanes)
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr bool S16 = (F & F_CODE16) != 0;
    using ST = StackF<false, F>;
    ST* stk = reinterpret_cast<ST*>(smem) + B + stack_column<S16>(threadIdx.x);
    CameraRec<double>& s_cam = *reinterpret_cast<CameraRec<double>*>(smem + paths_g_stack_bytes(g.stack, B, S16));
    PassGeom& s_g = *reinterpret_cast<PassGeom*>(smem + paths_g_stack_bytes(g.stack, B, S16) + sizeof(CameraRec<double>));
    stk[-B] = static_cast<ST>(kNodeEmpty);
    if (threadIdx.x == 0) {
        s_cam = cam;
        s_g = g;
        if (g.list_mode) {  // the list's entry count, on the device (PassGeom::list_mode)
            const uint32_t n = g.list[-1];
            s_g.nlist = n;
            s_g.P = n * g.k;
        }
    }
    [[maybe_unused]] JumpEntry* jt = reinterpret_cast<JumpEntry*>(smem + align16(paths_g_stack_bytes(g.stack, B, S16) + sizeof(CameraRec<double>) + sizeof(PassGeom)));
    if (threadIdx.x < static_cast<uint32_t>(kJumpEntries)) jt[threadIdx.x] = pcg_jump(3u * threadIdx.x);
    DevScene<double> S = S0;
    [[maybe_unused]] double* uvc = reinterpret_cast<double*>(jt + kJumpEntries);  // sphere u, v constants, LDS copy
    if constexpr ((TF & TF_IMAGE) != 0)
        if (threadIdx.x < static_cast<uint32_t>(kUvConsts)) uvc[threadIdx.x] = uv_table(S0)[threadIdx.x];
    size_t lm_off = paths_g_head_bytes(g.stack, B, S16);  // LM: world list and objects, then the BVH arrays
    if constexpr (LM != 0) {
        uint8_t* wb = smem + lm_off;
        for (int32_t i = static_cast<int32_t>(threadIdx.x); i < S0.nworld; i += B) reinterpret_cast<int32_t*>(wb)[i] = S0.world[i];
        uint8_t* ob = wb + align16(sizeof(int32_t) * static_cast<uint32_t>(S0.nworld));
        const uint4* os = reinterpret_cast<const uint4*>(S0.objs);
        for (uint32_t i = threadIdx.x; i < S0.n_objs * (sizeof(ObjRec<double>) / 16); i += B) reinterpret_cast<uint4*>(ob)[i] = os[i];
        uint8_t* pb = ob + sizeof(ObjRec<double>) * S0.n_objs;
        const uint4* ps = reinterpret_cast<const uint4*>(S0.obj_prims);
        for (uint32_t i = threadIdx.x; i < S0.n_objs * (sizeof(PrimRec80) / 16); i += B) reinterpret_cast<uint4*>(pb)[i] = ps[i];
        S.world = reinterpret_cast<const int32_t*>(wb);
        S.objs = reinterpret_cast<const ObjRec<double>*>(ob);
        S.obj_prims = reinterpret_cast<const PrimRec80*>(pb);
        const uint32_t nm = lds_mats<TF>(S0.n_mats);
        if (nm) {
            uint8_t* mb = pb + sizeof(PrimRec80) * S0.n_objs;
            const uint2* ms = reinterpret_cast<const uint2*>(S0.mats);
            static_assert(sizeof(MatRec<double>) % 8 == 0, "material records copied in 8-B pieces");
            for (uint32_t i = threadIdx.x; i < nm * (sizeof(MatRec<double>) / 8); i += B) reinterpret_cast<uint2*>(mb)[i] = ms[i];
            S.mats = reinterpret_cast<const MatRec<double>*>(mb);
        }
        lm_off += paths_g_world_bytes(S0.nworld, S0.n_objs, nm);
    }
    if constexpr (LM != 0) lm_off = align128(lm_off);  // node addresses multiples of 128 (device.h traverse: near/far planes by XOR)
    if constexpr (LM == 2) {  // the first n_lds_nodes nodes (the top levels of every BVH) into LDS
        BvhNode* m = reinterpret_cast<BvhNode*>(smem + lm_off);
        const uint4* s4 = reinterpret_cast<const uint4*>(S0.nodes);
        uint4* d4 = reinterpret_cast<uint4*>(m);
        for (uint32_t i = threadIdx.x; i < S0.n_lds_nodes * (sizeof(BvhNode) / 16); i += B) d4[i] = s4[i];
        S.nodes_lds = static_cast<uint32_t>(reinterpret_cast<size_t>((__attribute__((address_space(3))) BvhNode*)m));
    }
    if constexpr (LM == 1) {
        uint8_t* m = smem + lm_off;
        const size_t nb = sizeof(BvhNode) * S0.n_nodes, pb = align16(sizeof(uint32_t) * S0.n_primrefs);
        const size_t tb = (F & F_TRI) ? kLm1TriBytes * S0.n_primrefs : 0;
        auto copy = [&](uint8_t* dst, const void* src, size_t bytes) {
            const uint4* s4 = static_cast<const uint4*>(src);
            uint4* d4 = reinterpret_cast<uint4*>(dst);
            for (size_t i = threadIdx.x; i < bytes / 16; i += B) d4[i] = s4[i];
        };
        copy(m, S0.nodes, nb);
        // primrefs: 4-B entries, the tail of the last 16-B word comes from past the array's end -- copy word-wise
        for (uint32_t i = threadIdx.x; i < S0.n_primrefs; i += B) reinterpret_cast<uint32_t*>(m + nb)[i] = S0.primrefs[i];
        S.nodes = reinterpret_cast<const BvhNode*>(m);
        if constexpr (kLdsNodesPL) {  // every node read through the explicit-LDS path (device.h traverse, PL)
            S.nodes_lds = static_cast<uint32_t>(reinterpret_cast<size_t>((__attribute__((address_space(3))) uint8_t*)m));
            S.n_lds_nodes = S0.n_nodes;
        }
        S.primrefs = reinterpret_cast<const uint32_t*>(m + nb);
        if constexpr ((F & F_TRI) != 0) {
            copy(m + nb + pb, S0.leaf_tris112, tb);
            S.leaf_tris112 = reinterpret_cast<const TriRec112<double>*>(m + nb + pb);
        }
        lm_off = align16(lm_off + nb + pb + tb);  // the camera-ray rings follow (kRing)
    }
    // radiance records: non-temporal where the scene's nodes and leaf records come from L2 (LM 0 / 2: the streaming
    // records would evict them; r6i: capsule +1.7 %, cow +0.8 %), temporal where they sit in LDS (LM 1: each 8-B NT
    // store reaches HBM as its own partial write, r5c; Cornell smoke -1.5 % with NT, the final and dino +-0)
    constexpr bool kResNT = LM != 1;
    constexpr bool kRing = paths_g_ring(F, LM);
    const bool use_ring = kRing && g.lds_ring != 0;  // the launch found room for the rings
    [[maybe_unused]] const RingG ring{reinterpret_cast<double*>(smem + lm_off) + (threadIdx.x / 64u) * (8u * kRingG)};
    [[maybe_unused]] uint32_t r_head = 0, r_avail = 0, r_b0 = 0;  // wave-uniform: next entry, entries left, batch slot
    [[maybe_unused]] bool r_exhausted = false;                   // every slot of the pass is in a batch
    const int max_depth = g.max_depth;
    __syncthreads();
    const uint32_t lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const V3<R> bg = mk(S.bg[0], S.bg[1], S.bg[2]);
    uint32_t cur = 0, end = 0;  // this wave's claimed slots [cur, end): wave-uniform
    bool busy = false, drained = false;
    uint32_t q = 0;
    int depth = 0;
    PathState<R> st;
    unsigned long long segs = 0;
    // suspendable BVH traversals (ART_SUSPEND_LANES) where node fetches go to L2 (LM 0, 2); with the whole BVH in LDS
    // (LM 1) a traversal is short and suspending only adds rounds
    // (LM 1, the BVH in LDS: thresholds 4-40 measured -5 % to -22 % on dino and the final scene)
    constexpr int kSuspLanes = LM == 1 ? 0 : ART_SUSPEND_LANES;
    constexpr bool SUSP = kSuspLanes > 0;
    TraceState<R> ts;  // the lane's segment trace, possibly suspended in a BVH
    bool in_trace = false;
#ifdef ART_TRACE
    bool tracing = false;
#endif
#ifdef ART_STATS
    unsigned long long tm_load = 0, tm_trace = 0, tm_shade = 0, tm_app = 0, tm_prev = __builtin_amdgcn_s_memtime();
    unsigned long long tm_surf = 0, tm_coop = 0, tm_tex = 0;  // the shading phase split (k_paths_g)
#endif
    for (;;) {
        const uint64_t idle = __ballot(!busy && !drained);
        if (use_ring && idle) {
            // the idle lanes of rank < first take the ring's remaining entries; when more lanes are idle than entries
            // are left (the ring is then empty) the wave refills it with the next 64 slots, converged, and the rest take
            // from the new batch (LDS operations of one wave complete in order: the refill's writes land after the
            // takes' reads of the old entries, and before the reads of the new ones)
            const uint32_t n = static_cast<uint32_t>(__popcll(idle));
            const uint32_t rank = static_cast<uint32_t>(__popcll(idle & below));
            const bool me = !busy && !drained;
            const uint32_t first = min(n, r_avail);
            int got = 0;
            if (me && rank < first) got = ring_take_g(ring, r_head + rank, r_b0, st, q);
            if (n > r_avail && !r_exhausted) {
                if (cur == end) {
                    const uint32_t chunk = s_g.chunk;
                    uint32_t nb = 0;
                    if (lane == 0) nb = atomicAdd(next_slot, chunk);
                    nb = __shfl(nb, 0);
                    cur = nb;
                    end = nb + chunk;
                }
                const uint32_t b = cur;
                cur += 64;
                __asm__ volatile("" ::: "memory");  // the LDS camera / pass geometry loads stay here (see k_paths)
                ring_fill_g(ring, lane, b + lane, s_g, s_cam);
                __asm__ volatile("" ::: "memory");
                r_b0 = b;
                r_exhausted = b + 64u >= s_g.P;  // g.P, or the device count's (list_mode): read where used
                if (me && rank >= first) got = ring_take_g(ring, rank - first, r_b0, st, q);
                r_head = n - first;
                r_avail = kRingG - r_head;
            } else {
                r_head += first;
                r_avail -= first;
                if (me && rank >= first) got = 2;  // no entries left and no slots: drained
            }
            if (me) {
                busy = got == 1;
                drained = got == 2;
                depth = 0;
#ifdef ART_TRACE
                if (busy) {  // as the ring-free path below: is this the traced (pixel, sample)?
                    int lx = 0, ly = 0;
                    uint32_t qi, j;
                    slot_split(s_g, q, qi, j);
                    slot_pixel(s_g, qi, lx, ly);
                    tracing = static_cast<long long>(global_row(s_g, ly)) * s_g.W + lx == g_trace_pixel &&
                              static_cast<long long>(s_g.sample_base + j) == g_trace_sample;
                }
#endif
            }
        } else if (idle) {
            const uint32_t n = static_cast<uint32_t>(__popcll(idle));
            const uint32_t rank = static_cast<uint32_t>(__popcll(idle & below));
            uint32_t slot;
            if (cur + n > end) {
                const uint32_t chunk = s_g.chunk;
                uint32_t nb = 0;
                if (lane == 0) nb = atomicAdd(next_slot, chunk);
                nb = __shfl(nb, 0);
                const uint32_t left = end - cur;
                slot = rank < left ? cur + rank : nb + (rank - left);
                cur = nb + (n - left);
                end = nb + chunk;
            } else {
                slot = cur + rank;
                cur += n;
            }
            if (!busy && !drained) {
                if (slot >= s_g.P) {
                    drained = true;
                } else {
                    int lx, ly;
                    q = slot;
                    __asm__ volatile("" ::: "memory");  // keep the LDS camera/geometry loads here (see k_paths)
                    uint32_t qi, j;
                    slot_split(s_g, slot, qi, j);
                    if (slot_pixel(s_g, qi, lx, ly)) {
                        gen_ray(s_g, s_cam, j, lx, ly, st);
                        busy = true;
                        depth = 0;
#ifdef ART_TRACE
                        tracing = static_cast<long long>(global_row(s_g, ly)) * s_g.W + lx == g_trace_pixel &&
                                  static_cast<long long>(s_g.sample_base + j) == g_trace_sample;
#endif
                    }
                }
            }
        }
        ART_TICK(tm_load);
        if (__ballot(busy) == 0) {
            if (__ballot(!drained) == 0) break;
            continue;
        }
        const bool allow = SUSP && __ballot(drained) == 0;  // suspend only while there are paths to start
        R t;
        HitOut h{0, 0, kMatUnknown};
        bool hitw = false, susp = false;
        Surf<R> s;
        [[maybe_unused]] uint32_t mtype = MAT_LIGHT;
        if (busy) {
            const bool fresh = !in_trace;
            if (fresh) {
                ++segs;
                if constexpr (SUSP) ts.start();
            }
#ifdef ART_TRACE
            if (tracing && fresh)
                printf("TRACE d=%d o=%016llx,%016llx,%016llx dir=%016llx,%016llx,%016llx tm=%016llx rng=%016llx\n", depth, ART_DBITS(st.ray.o.x),
                       ART_DBITS(st.ray.o.y), ART_DBITS(st.ray.o.z), ART_DBITS(st.ray.d.x), ART_DBITS(st.ray.d.y), ART_DBITS(st.ray.d.z),
                       ART_DBITS(st.ray.tm), static_cast<unsigned long long>(st.rng));
#endif
            if constexpr (SUSP) {
                ts.tr.allow = allow;
                ts.tr.lanes = kSuspLanes;
                in_trace = !trace_world_res<R, F, B, kLdsNodesPL>(S, st.ray, stk, st.rng, ts);
                hitw = ts.any;
                t = ts.closest;
                h = ts.h;
            } else {
                hitw = trace_world<R, F, B, false, kLdsNodesPL>(S, nullptr, st.ray, stk, st.rng, t, h);
            }
            susp = in_trace;  // suspended: nothing to shade this round
            ART_TICK(tm_trace);
            if (!susp && hitw) {
                world_surface<R, F, (TF & TF_IMAGE) != 0, (TF & (TF_IMAGE | TF_BARY)) != 0>(S, h, st.ray, t, s, uvc);
                mtype = S.mats[s.mat].type;
            }
        }
        ART_TICK(tm_surf);
        // the whole wave draws random_in_unit_sphere for its lambertian, metal and isotropic hits (material.h:33, :55,
        // :129: each scatters with it first; metal's unit_vector draws nothing), as k_paths does
        const bool need = busy && !susp && hitw && (mtype == MAT_LAMBERTIAN || mtype == MAT_METAL || mtype == MAT_ISOTROPIC) &&
                          depth + 1 < max_depth;
        const V3<R> ps = coop_unit_sphere<R>(need, st.rng, jt);
        const V3<R>* pre = &ps;
        ART_TICK(tm_coop);
        if (busy) {
            bool cont = false;
            if (susp) {
            } else if (hitw) {
#ifdef ART_TRACE
                if (tracing)
                    printf("TRACE hit t=%016llx p=%016llx,%016llx,%016llx n=%016llx,%016llx,%016llx ff=%d mat=%d prim=%08x obj=%08x\n", ART_DBITS(t),
                           ART_DBITS(s.p.x), ART_DBITS(s.p.y), ART_DBITS(s.p.z), ART_DBITS(s.n.x), ART_DBITS(s.n.y), ART_DBITS(s.n.z), s.ff ? 1 : 0,
                           static_cast<int>(s.mat), h.prim, h.obj);
#endif
                const MatRec<R>& mat = S.mats[s.mat];
                // In kernels with noise or image textures (where a texture value is costly): the
                // steps several materials take, once for the wave instead of once per material branch present -- the
                // texture value (diffuse_light, lambertian, isotropic: no draws) and one unit_vector (of the sphere
                // draw for lambertian, of the ray direction for metal and dielectric).  Measured +1.3 % on the
                // Next-Week final; with solid / checker textures only (cow, dino) the longer live ranges cost 1.5-2 %.
                constexpr bool kShared = (TF & (TF_NOISE | TF_IMAGE)) != 0;
                V3<R> texc = mk(R(0), R(0), R(0)), uv = mk(R(0), R(0), R(0));
                if constexpr (kShared) {
                    const bool scat = depth + 1 < max_depth;
                    if (mat.type == MAT_LIGHT || (scat && (mat.type == MAT_LAMBERTIAN || mat.type == MAT_ISOTROPIC)))
                        texc = mat_tex_value<R, TF>(S, mat, s.u, s.v, s.p);
                    if (scat && (mat.type == MAT_LAMBERTIAN || mat.type == MAT_METAL || mat.type == MAT_DIELECTRIC))
                        uv = unit(mat.type == MAT_LAMBERTIAN ? *pre : st.ray.d);
                }
                const V3<R>* texp = kShared ? &texc : nullptr;
                const V3<R>* uvp = kShared ? &uv : nullptr;
                ART_TICK(tm_tex);
                if (mat.type == MAT_LIGHT) {  // material.h:114-116; diffuse_light never scatters
                    st.L = st.L + st.T * (texp ? *texp : mat_tex_value<R, TF>(S, mat, s.u, s.v, s.p));
                } else if (depth + 1 < max_depth) {
                    V3<R> att, dir;
                    bool sc = false;
                    switch (mat.type) {
                        case MAT_LAMBERTIAN: sc = scatter<R, MAT_LAMBERTIAN, TF>(S, mat, s, st, att, dir, pre, uvp, texp); break;
                        case MAT_METAL: sc = scatter<R, MAT_METAL, TF>(S, mat, s, st, att, dir, pre, uvp); break;
                        case MAT_DIELECTRIC: sc = scatter<R, MAT_DIELECTRIC, TF>(S, mat, s, st, att, dir, nullptr, uvp); break;
                        case MAT_ISOTROPIC: sc = scatter<R, MAT_ISOTROPIC, TF>(S, mat, s, st, att, dir, pre, nullptr, texp); break;
                        default: break;
                    }
                    if (sc) {
                        st.T = st.T * att;
                        st.ray.o = s.p;
                        st.ray.d = dir;
                        cont = true;
                    }
                }
            } else {  // engine.h:455-456: miss -> background
#ifdef ART_TRACE
                if (tracing) printf("TRACE miss\n");
#endif
                st.L = st.L + st.T * bg;
            }
            ART_TICK(tm_shade);
            if (susp) {
            } else if (cont) {
                ++depth;
            } else {
                store_res<kResNT>(w.res, q, st.L);
                busy = false;
            }
        }
        ART_TICK(tm_app);
    }
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off);
    if (lane == 0) atomicAdd(w.segments, segs);
#ifdef ART_STATS
    if (lane == 0) {
        atomicAdd(&g_art_stats[8], tm_load);
        atomicAdd(&g_art_stats[9], tm_trace);
        atomicAdd(&g_art_stats[10], tm_shade);
        atomicAdd(&g_art_stats[11], tm_app);
        atomicAdd(&g_art_stats[24], tm_surf);
        atomicAdd(&g_art_stats[25], tm_coop);
        atomicAdd(&g_art_stats[26], tm_tex);
    }
#endif
}

// k_paths_g instantiations without F_MEDIA_G sort packed keys over 16-bit child codes (F_CODE16); a scene
// whose codes do not fit them (more than 32768 nodes or 8192 primitive references) takes the F_ALL kernel instead
// ART_SPLIT_MESH (Makefile, SPLIT=1): the instantiations for meshes with solid/checker textures whose BVH is not all in
// LDS (LM 0 / 2: cow) are compiled in kernels_mesh.o (ART_SPLIT_PATHS=3) with LLVM's iterative-maxocc scheduler
// (MESH_SCHED): cow +1.3 % to +1.8 % over the default scheduler; dino's LM 1 kernel loses 0.9 % under it and the Next-Week
// final's 4.6 % (its spills double), so they stay in kernels.o (r3z2)
#ifndef ART_SPLIT_MESH
#define ART_SPLIT_MESH 0
#endif
constexpr uint32_t kMeshG = kFeatMesh | F_CODE16;
#if ART_SPLIT_PATHS == 3
template __global__ void k_paths_g<kMeshG, kTexBasic, 0>(DevScene<double>, PassGeom, CameraRec<double>, Work<double>, uint32_t*);
template __global__ void k_paths_g<kMeshG, kTexBasic, 2>(DevScene<double>, PassGeom, CameraRec<double>, Work<double>, uint32_t*);
#elif ART_SPLIT_MESH
extern template __global__ void k_paths_g<kMeshG, kTexBasic, 0>(DevScene<double>, PassGeom, CameraRec<double>, Work<double>, uint32_t*);
extern template __global__ void k_paths_g<kMeshG, kTexBasic, 2>(DevScene<double>, PassGeom, CameraRec<double>, Work<double>, uint32_t*);
#endif

// Input: the kShards shards of material queue M at depth d (the extend stage sorted hits by material type).
template <class R, uint32_t F, uint32_t M, uint32_t TF>
__global__ __launch_bounds__(kBlock) void k_shade(DevScene<R> S, PassGeom g, Work<R> w, int d) {
    __shared__ uint32_t pre[kShards + 1];
    block_prefix(pre, kShards, threadIdx.x < kShards ? *counter(w, d, 1 + static_cast<int>(M), threadIdx.x) : 0u);
    const uint32_t total = pre[kShards];
    const uint32_t* in = w.mq + static_cast<size_t>(M) * kShards * g.cap;
    const bool last = d + 1 >= g.max_depth;
    uint32_t* next = w.active[(d + 1) & 1];
    const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * (kBlock / 64);
    const int shard = static_cast<int>(wave % kShards);
    for (uint32_t b = wave; b * 64u < total; b += nwaves) {
        const uint32_t i = b * 64u + __lane_id();
        bool cont = false;
        uint32_t q = 0;
        if (i < total) {
            const int sg = find_segment(pre, kShards, i);
            q = in[static_cast<size_t>(sg) * g.cap + (i - pre[sg])];
            PathState<R> st;
            load_path(w.paths, q, st, true);
            const HitRecD<R> h = w.hits[q];
            Surf<R> s;
            world_surface<R, F, (TF & TF_IMAGE) != 0>(S, HitOut{h.prim, h.obj, kMatUnknown}, st.ray, h.t, s, uv_table(S));
            const MatRec<R>& mat = S.mats[s.mat];
            if (M == MAT_LIGHT) st.L = st.L + st.T * mat_tex_value<R, TF>(S, mat, s.u, s.v, s.p);  // material.h:114-116
            if (M != MAT_LIGHT && !last) {
                V3<R> att, dir;
                if (scatter<R, M, TF>(S, mat, s, st, att, dir)) {
                    st.T = st.T * att;
                    st.ray.o = s.p;
                    st.ray.d = dir;
                    store_path(w.paths, q, st);
                    cont = true;
                }
            }
            if (!cont) store_res(w.res, q, st.L);
        }
        wave_append(cont, q, next + static_cast<size_t>(shard) * g.cap, counter(w, d + 1, 0, shard));
    }
}

template <class R>
__global__ __launch_bounds__(256) void k_accum(PassGeom g, Work<R> w) {
    const uint32_t qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= g.npix_pad) return;
    int lx, ly;
    if (!slot_pixel(g, qi, lx, ly)) return;
    // pixel sums: per local pixel, or per list entry in pixel-list mode
    double* a = w.acc + 3 * (g.list ? static_cast<size_t>(qi) : static_cast<size_t>(ly) * g.W + lx);
    double r = a[0], gg = a[1], b = a[2];
    for (uint32_t j = 0; j < g.k; ++j) {  // sample order == the reference's `pixel_color +=` order
        double x, y, z;
        load_res(w.res, j * g.npix_pad + qi, x, y, z);
        r += x;
        gg += y;
        b += z;
    }
    a[0] = r;
    a[1] = gg;
    a[2] = b;
}

// engine_mode::parallel_images (engine.h:378-445): sample s of a pixel belongs to partial image s / m (m = spp / 4).
// Its samples are summed in order into the quarter sum q (f64, as the reference's pixel_color); when the quarter's
// last sample is in, write_color_raw<float> rounds q to float and the running image sum takes it:
// acc = ((c1 + c2) + c3) + c4 in double, the reference's `pixel_color1 + ... + pixel_color4`.  q persists across passes.
template <class R>
__global__ __launch_bounds__(256) void k_accum_images(PassGeom g, Work<R> w, double* qsum, uint32_t m) {
    const uint32_t qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= g.npix_pad) return;
    int lx, ly;
    if (!slot_pixel(g, qi, lx, ly)) return;
    const size_t pix = static_cast<size_t>(ly) * g.W + lx;
    double* a = w.acc + 3 * pix;
    double* q = qsum + 3 * pix;
    double ar = a[0], ag = a[1], ab = a[2], qr = q[0], qg = q[1], qb = q[2];
    for (uint32_t j = 0; j < g.k; ++j) {
        double x, y, z;
        load_res(w.res, j * g.npix_pad + qi, x, y, z);
        qr += x;
        qg += y;
        qb += z;
        if ((g.sample_base + j + 1) % m == 0) {
            ar += static_cast<double>(static_cast<float>(qr));
            ag += static_cast<double>(static_cast<float>(qg));
            ab += static_cast<double>(static_cast<float>(qb));
            qr = qg = qb = 0.0;
        }
    }
    a[0] = ar;
    a[1] = ag;
    a[2] = ab;
    q[0] = qr;
    q[1] = qg;
    q[2] = qb;
}

#if ART_SPLIT_PATHS <= 1
// Ray queries (rt_trace_rays): the world's closest hit (hittable_list::hit, hittable_list.cpp:5-19) of n caller-given
// rays through the renderer's own traversal -- the LDS image (L) or the HBM scene -- and the surface normal
// (hit_record::set_face_normal), so traversal edge cases (axis-parallel rays, origins on faces) can be checked one ray
// at a time against the oracle.  Ray i's medium draws come from the PCG stream pcg_seed(0, i, 0).
template <uint32_t F, bool L>
__global__ __launch_bounds__(L ? kBlockL : kBlock) void k_trace_rays(DevScene<double> S, const double* rays, uint32_t n, uint32_t stack_rows,
                                                                       double* t_out, double* n_out) {
    using R = double;
    constexpr int B = L ? kBlockL : kBlock;
    extern __shared__ __align__(16) uint8_t smem[];
    StackT<L>* stk = reinterpret_cast<StackT<L>*>(smem + (L ? kLdsImageBytes : 0u)) + B + stack_column<L>(threadIdx.x);
    stk[-B] = static_cast<StackT<L>>(kNodeEmpty);
    if constexpr (L) {
        load_lds_image<B>(S.lds_image, smem);
        __syncthreads();
    }
    (void)stack_rows;
    const uint32_t i = blockIdx.x * B + threadIdx.x;
    if (i >= n) return;
    const double* q = rays + 7 * static_cast<size_t>(i);
    Ray<R> r;
    r.o = mk(q[0], q[1], q[2]);
    r.d = mk(q[3], q[4], q[5]);
    r.tm = q[6];
    uint64_t rng = pcg_seed(0, i, 0);
    R t = R(0);
    HitOut h{0, 0, kMatUnknown};
    if (trace_world<R, F, B, L>(S, L ? smem : nullptr, r, stk, rng, t, h)) {
        Surf<R> s;
        world_surface<R, F, false>(S, h, r, t, s);
        t_out[i] = t;
        n_out[3 * i] = s.n.x;
        n_out[3 * i + 1] = s.n.y;
        n_out[3 * i + 2] = s.n.z;
    } else {
        t_out[i] = __builtin_inf();
        n_out[3 * i] = n_out[3 * i + 1] = n_out[3 * i + 2] = 0.0;
    }
}

__global__ void k_finalize(const double* acc, uint8_t* rgb, uint32_t n, int spp) {  // color.h:6-22
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double scale = 1.0 / spp;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double x = sqrt(scale * acc[3 * i + c]);
        x = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);
        rgb[3 * i + c] = static_cast<uint8_t>(256 * x);
    }
}

// ------------------------------------------------------------------------------------------------ adaptive mode
// engine_mode::adaptive (engine.h:96-333) as four traced levels over the local image, whose rows group into 12-px
// "big squares" (6-px mid and 3-px small squares inside).  Level 0 traces every big square's 4 corners; level L+1
// traces the new corners (12 per square) of the sub-squares of every level-L square whose corner heuristic fired, and
// level 3 the 5 remaining pixels of each subdivided small square; k_adapt_fill then interpolates every pixel no level
// traced from the corners of the deepest square that was not subdivided.  The work image is the reference's int frame
// (-1 = not yet written); every traced pixel's value depends only on its (pixel, sample) streams, so a corner shared by
// two levels is traced once.
constexpr int kBig = 12, kMid = kBig / 2, kSmall = kMid / 2;

// write_color<int> (color.h:6-22) of list entry e's pixel sums into the work image.
__global__ void k_adapt_store(const uint32_t* list, uint32_t n, const double* acc, int spp, int32_t* work) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const double scale = 1.0 / spp;
    int32_t* o = work + 3 * static_cast<size_t>(list[e]);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double x = sqrt(scale * acc[3 * static_cast<size_t>(e) + c]);
        x = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);
        o[c] = static_cast<int32_t>(256 * x);
    }
}

// list_mode 1 (the device-counted levels): the pixel sums of every list entry -- its k samples on consecutive slots,
// summed in sample order from +0.0 as k_accum sums them into the zeroed accumulator (engine.h:58-68) -- written into
// the work image as k_adapt_store writes them.  The entry count is list[-1].
// One wave per entry (r6o): the entry's k records are consecutive (entry-major slots), so the wave reads 64 of them
// per coalesced load into LDS and lanes 0-2 (one per channel) add them in sample order from LDS.  One thread per
// entry, 100 records each, left every level's accumulation latency-bound at ~62 us whatever its size (rocprofv3
// kernel trace of the default run; 45 us with 20 loads in flight per thread).
constexpr int kAdaptAccumWaves = 4;
__global__ __launch_bounds__(64 * kAdaptAccumWaves) void k_adapt_accum(const uint32_t* list, const ResRec<double>* res, uint32_t k, int spp,
                                                                      int32_t* work) {
    __shared__ double buf[kAdaptAccumWaves][3 * 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t e = blockIdx.x * kAdaptAccumWaves + wv;
    if (e >= list[-1]) return;  // wave-uniform
    double* b = buf[wv];
    double acc = 0.0;  // lane c < 3: channel c
    const ResRec<double>* r = res + static_cast<size_t>(e) * k;
    for (uint32_t j0 = 0; j0 < k; j0 += 64) {
        const uint32_t n = min(64u, k - j0);
        if (lane < n) {
            double x, y, z;
            load_res(r, j0 + lane, x, y, z);
            b[3 * lane] = x;
            b[3 * lane + 1] = y;
            b[3 * lane + 2] = z;
        }
        // one wave: its LDS writes complete before its reads (in-order LDS, the waitcnt), and the compiler keeps them apart
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 3)
            for (uint32_t i = 0; i < n; ++i) acc += b[3 * i + lane];
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next chunk's writes after these reads
    }
    if (lane >= 3) return;
    const double scale = 1.0 / spp;
    double x = sqrt(scale * acc);
    x = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);
    work[3 * static_cast<size_t>(list[e]) + lane] = static_cast<int32_t>(256 * x);
}

// _compute_corners_heuristic (engine.h:96-136): any squared RGB distance between neighbouring corners > 100.
__device__ __forceinline__ bool adapt_subdivide(const int32_t* work, int W, int x, int y, int L) {
    const int32_t* c1 = work + 3 * (static_cast<size_t>(y) * W + x);
    const int32_t* c2 = work + 3 * (static_cast<size_t>(y) * W + x + L - 1);
    const int32_t* c3 = work + 3 * (static_cast<size_t>(y + L - 1) * W + x);
    const int32_t* c4 = work + 3 * (static_cast<size_t>(y + L - 1) * W + x + L - 1);
    auto d = [](const int32_t* a, const int32_t* b) {
        return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
    };
    return d(c1, c2) > 100 || d(c2, c4) > 100 || d(c4, c3) > 100 || d(c3, c1) > 100;
}

// Level-0 list: the four corners of every big square (ul, ur, bl, br: engine.h:223-233).
__global__ void k_adapt_corners(uint32_t* list, int W, int sqx, uint32_t nsq) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0) list[-1] = 4 * nsq;  // the entry count of a device-counted list (PassGeom::list_mode)
    if (s >= nsq) return;
    const uint32_t x = (s % sqx) * kBig, y = (s / sqx) * kBig;
    list[4 * s + 0] = y * W + x;
    list[4 * s + 1] = y * W + x + kBig - 1;
    list[4 * s + 2] = (y + kBig - 1) * W + x;
    list[4 * s + 3] = (y + kBig - 1) * W + x + kBig - 1;
}

// Heuristic of every level-`level` square (0: big, 1: mid, 2: small) whose parent was subdivided, and the list of
// the pixels the next level traces.  flags[level] holds one byte per square: index big, big*4+mid, (big*4+mid)*4+small.
__global__ void k_adapt_level(int level, int32_t* work, int W, int sqx, uint32_t nsq, uint8_t* f0, uint8_t* f1, uint8_t* f2, uint32_t* list,
                              uint32_t* count) {
    const uint32_t per = level == 0 ? 1u : (level == 1 ? 4u : 16u);
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nsq * per) return;
    const uint32_t big = id / per, sub = id % per;
    int x = static_cast<int>((big % sqx) * kBig), y = static_cast<int>((big / sqx) * kBig);
    int L = kBig;
    if (level >= 1) {
        if (!f0[big]) return;
        const uint32_t mid = level == 1 ? sub : sub / 4;
        x += static_cast<int>(mid & 1u) * kMid;
        y += static_cast<int>(mid >> 1) * kMid;
        L = kMid;
        if (level == 2) {
            if (!f1[big * 4 + mid]) return;
            x += static_cast<int>(sub & 1u) * kSmall;
            y += static_cast<int>((sub >> 1) & 1u) * kSmall;
            L = kSmall;
        }
    }
    const bool split = adapt_subdivide(work, W, x, y, L);
    (level == 0 ? f0 : (level == 1 ? f1 : f2))[id] = split ? 1 : 0;
    if (!split) return;
    if (level < 2) {  // the 16 corners of the 4 sub-squares minus this square's own 4 corners
        const int h = L / 2;
        const int xs[4] = {x, x + h - 1, x + h, x + L - 1}, ys[4] = {y, y + h - 1, y + h, y + L - 1};
        const uint32_t base = atomicAdd(count, 12u);
        uint32_t k = 0;
        for (int b = 0; b < 4; ++b)
            for (int a = 0; a < 4; ++a) {
                if ((a == 0 || a == 3) && (b == 0 || b == 3)) continue;
                list[base + k++] = static_cast<uint32_t>(ys[b]) * W + static_cast<uint32_t>(xs[a]);
            }
    } else {  // engine.h:268-278: the 5 non-corner pixels of the 3-px square
        const uint32_t base = atomicAdd(count, 5u);
        list[base + 0] = static_cast<uint32_t>(y) * W + x + 1;
        list[base + 1] = static_cast<uint32_t>(y + 1) * W + x;
        list[base + 2] = static_cast<uint32_t>(y + 1) * W + x + 1;
        list[base + 3] = static_cast<uint32_t>(y + 1) * W + x + 2;
        list[base + 4] = static_cast<uint32_t>(y + 2) * W + x + 1;
    }
}

// interpolate_square (engine.h:185-219) with _interpolate (engine.h:138-149, v/t == (1/t)*v), then the u8 frame.
__global__ void k_adapt_fill(int32_t* work, uint8_t* rgb, int W, int rows, int sqx, const uint8_t* f0, const uint8_t* f1, const uint8_t* f2) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= static_cast<uint32_t>(W) * static_cast<uint32_t>(rows)) return;
    const int x = static_cast<int>(p % W), y = static_cast<int>(p / W);
    int32_t* o = work + 3 * static_cast<size_t>(p);
    if (o[0] < 0) {
        const uint32_t big = static_cast<uint32_t>(y / kBig) * sqx + static_cast<uint32_t>(x / kBig);
        int x1 = (x / kBig) * kBig, y1 = (y / kBig) * kBig, L = kBig;
        if (f0[big]) {
            const uint32_t mid = static_cast<uint32_t>(((y % kBig) / kMid) * 2 + (x % kBig) / kMid);
            x1 += (x % kBig) / kMid * kMid;
            y1 += (y % kBig) / kMid * kMid;
            L = kMid;
            if (f1[big * 4 + mid]) {
                x1 += (x % kMid) / kSmall * kSmall;
                y1 += (y % kMid) / kSmall * kSmall;
                L = kSmall;
            }
        }
        const int x2 = x1 + L - 1, y2 = y1 + L - 1;
        const int32_t* q11 = work + 3 * (static_cast<size_t>(y1) * W + x1);
        const int32_t* q12 = work + 3 * (static_cast<size_t>(y2) * W + x1);
        const int32_t* q21 = work + 3 * (static_cast<size_t>(y1) * W + x2);
        const int32_t* q22 = work + 3 * (static_cast<size_t>(y2) * W + x2);
        const double ix = 1.0 / static_cast<double>(x2 - x1), iy = 1.0 / static_cast<double>(y2 - y1);
        const double ax = x2 - x, bx = x - x1, ay = y2 - y, by = y - y1;
        int32_t v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double r1 = ix * (ax * static_cast<double>(q11[c])) + ix * (bx * static_cast<double>(q21[c]));
            const double r2 = ix * (ax * static_cast<double>(q12[c])) + ix * (bx * static_cast<double>(q22[c]));
            v[c] = static_cast<int32_t>(iy * (ay * r1) + iy * (by * r2));
        }
        // written after all three reads: a neighbour never reads this pixel (only corners, which are traced)
        o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
    }
    (void)f2;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[3 * static_cast<size_t>(p) + c] = static_cast<uint8_t>(o[c]);
}

#endif  // ART_SPLIT_PATHS <= 1

#if ART_SPLIT_PATHS <= 1
// ------------------------------------------------------------------------------------------------ device scene
template <class R>
struct DeviceScene {
    std::vector<void*> allocs;
    DevScene<R> view{};
    bool media = false;
    uint32_t features = F_ALL;
    int max_stack = kMaxStackDepth;
    uint32_t mat_types = (1u << kNumMatTypes) - 1;  // bit m: some material of type m exists
    bool tex_basic = false;                          // only solid and checker textures
    bool lds_scene = false;                          // view.lds_image holds the layout.h LDS scene image
    bool lds_shade = false;                          // ... including a complete shading table (fused variant)
    bool codes16 = false;                            // every node's child codes fit BvhNode::pad's 16-bit form
    uint32_t leaf_shift = 0;                         // 1: 16-bit leaf codes count slot pairs (F_LEAF2; leaves on even slots)
    bool tex_bary = false;                           // image textures are barycentric ones on triangles only (TF_BARY)
    size_t bytes = 0;

    template <class T>
    const T* upload(const std::vector<T>& v) {
        if (v.empty()) return nullptr;
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, v.size() * sizeof(T)));
        HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        allocs.push_back(p);
        bytes += v.size() * sizeof(T);
        return static_cast<const T*>(p);
    }
    void release() {
        for (void* p : allocs) (void)hipFree(p);
        allocs.clear();
    }
};

template <class R, class D>
static void cvt_sphere(const SphereRec<D>& s, SphereRec<R>& o) {
    for (int a = 0; a < 3; ++a) { o.c[a] = R(s.c[a]); o.d[a] = R(s.d[a]); }
    o.r = R(s.r); o.t0 = R(s.t0); o.dt = R(s.dt); o.mat = s.mat; o.flags = s.flags;
}

constexpr size_t kLdsPerCu = 160 * 1024;  // gfx950

// Traversal stack rows per lane: the worst-case depth + the sentinel row + the spare row of branchless pushes.
static uint32_t stack_rows(int max_stack) { return static_cast<uint32_t>(std::max(1, max_stack)) + 2u; }
static size_t extend_lds_bytes(bool L, uint32_t stack) { return extend_pre_offset(L, stack) + 4 * (kShards + 1); }

// Builds the layout.h LDS scene image when the f64 scene qualifies: spheres only, every BVH node and leaf slot within
// the plane capacities, and image + stack within one CU's LDS.  Returns an empty vector otherwise.
static std::vector<uint8_t> lds_scene_image(const FlatScene& f, uint32_t& nmov, bool& shade_ok) {
    std::vector<uint8_t> img;
    nmov = 0;
    shade_ok = false;
    if ((f.features & ~kFeatSpheres) != 0 || f.nodes.empty() || f.nodes.size() > kLdsNodeCap || f.primrefs.size() > kLdsSlotCap ||
        f.world.size() > kPathsWorldCap || f.objs.size() > kPathsWorldCap ||
        f.spheres.size() > kLdsRefIndexMask || std::max(extend_lds_bytes(true, stack_rows(f.max_stack)), paths_lds_bytes(stack_rows(f.max_stack))) > kLdsPerCu)
        return img;
    // k_paths shades a hit by its LDS leaf slot: every world object must be a BVH over the image's slots (a loose
    // OBJ_PRIM object, e.g. with option compile.world_merge = 0 or from a flat-scene file, takes the HBM kernels)
    for (int32_t w : f.world)
        if (w < 0 || static_cast<size_t>(w) >= f.objs.size() || f.objs[w].kind != OBJ_BVH) return img;
    for (uint32_t ref : f.primrefs) {
        if (primref_type(ref) != PRIM_SPHERE) return img;
        const SphereRec<double>& sp = f.spheres[primref_index(ref)];
        if (sp.flags & SPH_MOVING) {
            // the image's moving spheres span the unit shutter (every moving_sphere of the reference scenes,
            // scene_manager.cpp:34-35, :201): their centre fraction is the ray time itself (hit_lds_slot); and they
            // move along y only (scene_manager.cpp:33): the image keeps one dy per leaf slot (layout.h)
            if (sp.t0 != 0.0 || sp.dt != 1.0 || sp.d[0] != 0.0 || sp.d[2] != 0.0) return img;
            ++nmov;
        }
    }
    if (nmov > kLdsMovCap) return img;
    for (const BvhNode& b : f.nodes)
        for (int c = 0; c < 4; ++c)
            if (b.child[c] < 0 && b.child[c] != kNodeEmpty && leaf_count(b.child[c]) > kLdsLeafMaxCount) return img;
    img.assign(kLdsImageBytes, 0);
    auto put = [&](uint32_t off, const void* v, size_t n) { std::memcpy(img.data() + off, v, n); };
    for (size_t n = 0; n < f.nodes.size(); ++n) {
        const BvhNode& b = f.nodes[n];
        float planes[6][4];
        const float* src[6] = {b.lox, b.hix, b.loy, b.hiy, b.loz, b.hiz};
        int32_t child[4];
        for (int c = 0; c < 4; ++c) {
            // an empty slot becomes an empty leaf behind a point box at (3e38, 3e38, 3e38): no slab test of it needs
            // a child check, and the astronomically rare ray whose three slab times coincide there finds no primitives
            const bool empty = b.child[c] == kNodeEmpty;
            for (int j = 0; j < 6; ++j) planes[j][c] = empty ? kLdsEmptyBox : src[j][c];
            // inner nodes by their byte offset in a plane (index * 16: device.h traverse), leaves as lds_leaf codes
            child[c] = empty ? kLdsEmptyChild : b.child[c] >= 0 ? b.child[c] * 16 : lds_leaf(leaf_first(b.child[c]), leaf_count(b.child[c]));
        }
        // per axis: lo, hi, lo (layout.h kLdsNodePlanes), then the child codes as int16
        const int order[9] = {0, 1, 0, 2, 3, 2, 4, 5, 4};
        const uint32_t nn = static_cast<uint32_t>(n);
        for (uint32_t j = 0; j < 9; ++j) put(kLdsOffNodes + (j * kLdsNodeCap + nn) * 16, planes[order[j]], 16);
        const int16_t c16[8] = {static_cast<int16_t>(child[0]), static_cast<int16_t>(child[1]), static_cast<int16_t>(child[2]),
                                static_cast<int16_t>(child[3]), 0, 0, 0, 0};
        put(kLdsOffNodes + (kLdsNodePlaneChild * kLdsNodeCap + nn) * 16, c16, 16);
    }
    // shading table: one entry per material (two for a checker of solid colours); anything else keeps the scene off
    // the fused variant (shade_ok = false), which shades from the global scene records instead
    std::vector<int32_t> entry(f.mats.size(), -1);
    uint32_t nent = 0;
    shade_ok = true;
    auto put_entry = [&](const double c[3], double param) {
        const double v[4] = {c[0], c[1], c[2], param};
        if (nent < kLdsMatCap) put(kLdsOffMat + nent * 32, v, 32);
        return nent++;
    };
    auto solid = [&](int32_t t) { return t >= 0 && static_cast<size_t>(t) < f.texs.size() && f.texs[t].type == TEX_SOLID; };
    uint32_t m = 0;
    for (size_t slot = 0; slot < f.primrefs.size(); ++slot) {
        const uint32_t idx = primref_index(f.primrefs[slot]);
        const auto& sp = f.spheres[idx];
        // a moving sphere's x and z at time tm are c + tm * (+-0) (moving_sphere.h:72-74) == c + d: the image stores
        // that value (it differs from c only for c = -0 and d = +0), and the device adds tm * dy to y alone
        const bool moving = (sp.flags & SPH_MOVING) != 0;
        const double cx = moving ? sp.c[0] + sp.d[0] : sp.c[0], cz = moving ? sp.c[2] + sp.d[2] : sp.c[2];
        const double p0[2] = {cx, sp.c[1]}, p1[2] = {cz, sp.r * sp.r}, inv_r = 1.0 / sp.r;
        const uint32_t sl = static_cast<uint32_t>(slot);
        put(kLdsOffSph + sl * 16, p0, 16);
        put(kLdsOffSph + (kLdsSlotCap + sl) * 16, p1, 16);
        put(kLdsOffInvR + sl * 8, &inv_r, 8);
        uint32_t code = idx | (f.mats[sp.mat].type << kLdsRefMatShift);
        const double dy = moving ? sp.d[1] : -0.0;
        put(kLdsOffMov + sl * 8, &dy, 8);
        if (moving) {
            code |= (m + 1) << kLdsRefMovShift;
            ++m;
        }
        put(kLdsOffRef + sl * 4, &code, 4);
        const auto& mat = f.mats[sp.mat];
        if (entry[sp.mat] < 0) {
            if (mat.type == MAT_LAMBERTIAN || mat.type == MAT_LIGHT) {
                const auto& t = f.texs[mat.tex];
                if (t.type == TEX_SOLID) {
                    entry[sp.mat] = static_cast<int32_t>(put_entry(t.c, 0.0));
                } else if (t.type == TEX_CHECKER && solid(t.even) && solid(t.odd)) {
                    entry[sp.mat] = static_cast<int32_t>(put_entry(f.texs[t.even].c, 0.0)) | static_cast<int32_t>(kLdsMatChecker);
                    put_entry(f.texs[t.odd].c, 0.0);
                } else {
                    shade_ok = false;
                }
            } else if (mat.type == MAT_METAL) {
                entry[sp.mat] = static_cast<int32_t>(put_entry(mat.albedo, mat.fuzz));
            } else if (mat.type == MAT_DIELECTRIC) {
                // dielectric (material.h:63-99): 1 / ir, and reflectance()'s r0 = ((1 - ratio) / (1 + ratio))^2 for
                // both faces, in the device's IEEE double arithmetic (-ffp-contract=off), then ir
                const double inv = 1.0 / mat.ir;
                double r0f = (1.0 - inv) / (1.0 + inv), r0b = (1.0 - mat.ir) / (1.0 + mat.ir);
                r0f = r0f * r0f;
                r0b = r0b * r0b;
                const double d3[3] = {inv, r0f, r0b};
                entry[sp.mat] = static_cast<int32_t>(put_entry(d3, mat.ir));
            } else {
                shade_ok = false;
            }
        }
        const uint16_t mi = static_cast<uint16_t>(entry[sp.mat] < 0 ? 0 : entry[sp.mat]);
        put(kLdsOffMatIdx + sl * 2, &mi, 2);
    }
    if (nent > kLdsMatCap) shade_ok = false;
    return img;
}


// The 16-bit child codes (layout.h make_leaf16) of a BVH whose leaves start past slot 8191 (more than 8192 primitive
// references: the capsule's 10 200 triangles) do not fit; with every leaf moved to an even slot of a padded copy of
// the primitive references they do, as first / 2 (F_LEAF2).  Rewrites the device copies of the leaf codes (nodes and
// hoisted leaves) and returns the padded references (pad[i]: slot i belongs to no leaf, its records stay zero), or
// an empty vector when the leaves overlap or the padded codes still do not fit.  A leaf tests the same primitives in
// the same order, so every closest hit, and the image, is unchanged.
static std::vector<uint32_t> pair_align_leaves(const std::vector<uint32_t>& primrefs, std::vector<BvhNode>& nodes,
                                               std::vector<ObjRec<double>>& objs, std::vector<uint8_t>& pad) {
    std::vector<std::pair<uint32_t, uint32_t>> leaves;  // (first, count)
    for (const BvhNode& b : nodes)
        for (int c = 0; c < 4; ++c)
            if (b.child[c] < 0 && b.child[c] != kNodeEmpty) leaves.emplace_back(leaf_first(b.child[c]), leaf_count(b.child[c]));
    for (const auto& o : objs)
        if (o.kind == OBJ_BVH && o.b != kNodeEmpty) leaves.emplace_back(leaf_first(o.b), leaf_count(o.b));
    std::sort(leaves.begin(), leaves.end());
    leaves.erase(std::unique(leaves.begin(), leaves.end()), leaves.end());
    std::unordered_map<uint32_t, uint32_t> moved;  // old first -> new first
    std::vector<uint32_t> out;
    pad.clear();
    uint32_t next = 0;  // first old slot not yet copied
    for (const auto& lf : leaves) {
        if (lf.first < next || lf.second < 1 || lf.second > 4 || lf.first + lf.second > primrefs.size()) return {};
        for (; next < lf.first; ++next) {  // slots outside every leaf keep their order
            out.push_back(primrefs[next]);
            pad.push_back(0);
        }
        if (out.size() & 1u) {
            out.push_back(0u);
            pad.push_back(1);
        }
        moved[lf.first] = static_cast<uint32_t>(out.size());
        if (!leaf16_ok(static_cast<uint32_t>(out.size()) >> 1, lf.second)) return {};
        for (uint32_t k = 0; k < lf.second; ++k) {
            out.push_back(primrefs[lf.first + k]);
            pad.push_back(0);
        }
        next = lf.first + lf.second;
    }
    for (; next < primrefs.size(); ++next) {
        out.push_back(primrefs[next]);
        pad.push_back(0);
    }
    auto remap = [&](int32_t c) { return make_leaf(moved.at(leaf_first(c)), leaf_count(c)); };
    for (BvhNode& b : nodes)
        for (int c = 0; c < 4; ++c)
            if (b.child[c] < 0 && b.child[c] != kNodeEmpty) b.child[c] = remap(b.child[c]);
    for (auto& o : objs)
        if (o.kind == OBJ_BVH && o.b != kNodeEmpty) o.b = remap(o.b);
    return out;
}

template <class R>
static void build_device_scene(const FlatScene& f0, DeviceScene<R>& ds) {
    // the device copy of the BVH arrays, with leaves pair-aligned where 16-bit codes need it (pair_align_leaves)
    FlatScene f = f0;
    std::vector<uint8_t> slot_pad(f.primrefs.size(), 0);
    {
        bool fit = f.nodes.size() <= 32768u;
        for (const BvhNode& b : f.nodes)
            for (int c = 0; c < 4; ++c)
                if (b.child[c] < 0 && b.child[c] != kNodeEmpty) fit = fit && leaf16_ok(leaf_first(b.child[c]), leaf_count(b.child[c]));
        for (const auto& o : f.objs)
            if (o.kind == OBJ_BVH && o.b != kNodeEmpty) fit = fit && leaf16_ok(leaf_first(o.b), leaf_count(o.b));
        ds.leaf_shift = 0;
        // only where an F_LEAF2 kernel exists (mesh feature sets with triangles: launch_paths_g); other kernels decode
        // 16-bit leaves unshifted
        const bool mesh = (f.features & ~kFeatMesh) == 0 && (f.features & F_TRI) != 0;
        if (!fit && mesh && f.nodes.size() <= 32768u && opt(Opt::Leaf2) != 0) {
            std::vector<BvhNode> nodes = f.nodes;
            std::vector<ObjRec<double>> objs = f.objs;
            std::vector<uint8_t> pad;
            std::vector<uint32_t> refs = pair_align_leaves(f.primrefs, nodes, objs, pad);
            if (!refs.empty()) {
                f.primrefs = std::move(refs);
                f.nodes = std::move(nodes);
                f.objs = std::move(objs);
                slot_pad = std::move(pad);
                ds.leaf_shift = 1;
            }
        }
    }
    std::vector<SphereRec<R>> sph(f.spheres.size());
    for (size_t i = 0; i < sph.size(); ++i) cvt_sphere(f.spheres[i], sph[i]);
    std::vector<TriRec<R>> tri(f.tris.size());
    for (size_t i = 0; i < tri.size(); ++i) {
        for (int a = 0; a < 9; ++a) tri[i].p[a] = R(f.tris[i].p[a]);
        tri[i].mat = f.tris[i].mat;
        tri[i].pad = 0;
    }
    std::vector<RectRec<R>> rect(f.rects.size());
    for (size_t i = 0; i < rect.size(); ++i) {
        const auto& s = f.rects[i];
        rect[i] = RectRec<R>{R(s.a0), R(s.a1), R(s.b0), R(s.b1), R(s.k), s.axis, s.mat};
    }
    std::vector<BoxRec<R>> box(f.boxes.size());
    for (size_t i = 0; i < box.size(); ++i) {
        for (int a = 0; a < 3; ++a) { box[i].mn[a] = R(f.boxes[i].mn[a]); box[i].mx[a] = R(f.boxes[i].mx[a]); }
        box[i].mat = f.boxes[i].mat;
        box[i].pad = 0;
    }
    std::vector<ObjRec<R>> objs(f.objs.size());
    for (size_t i = 0; i < objs.size(); ++i) {
        objs[i].kind = f.objs[i].kind; objs[i].a = f.objs[i].a; objs[i].b = f.objs[i].b; objs[i].pad = 0;
        for (int a = 0; a < 4; ++a) objs[i].p[a] = R(f.objs[i].p[a]);
    }
    std::vector<MatRec<R>> mats(f.mats.size());
    for (size_t i = 0; i < mats.size(); ++i) {
        mats[i].type = f.mats[i].type; mats[i].tex = f.mats[i].tex; mats[i].flags = f.mats[i].flags; mats[i].pad = 0;
        for (int a = 0; a < 3; ++a) mats[i].albedo[a] = R(f.mats[i].albedo[a]);
        mats[i].fuzz = R(f.mats[i].fuzz); mats[i].ir = R(f.mats[i].ir);
        mats[i].flags &= ~static_cast<uint32_t>(MATF_SOLID);
        const int32_t t = f.mats[i].tex;
        const uint32_t ty = f.mats[i].type;
        if ((ty == MAT_LAMBERTIAN || ty == MAT_LIGHT || ty == MAT_ISOTROPIC) && t >= 0 && static_cast<size_t>(t) < f.texs.size() &&
            f.texs[t].type == TEX_SOLID) {
            // the solid colour itself: tex_value's ld3(t.c), the same doubles
            for (int a = 0; a < 3; ++a) mats[i].albedo[a] = R(f.texs[t].c[a]);
            mats[i].flags |= MATF_SOLID;
        }
    }
    std::vector<TexRec<R>> texs(f.texs.size());
    for (size_t i = 0; i < texs.size(); ++i) {
        const auto& s = f.texs[i];
        texs[i].type = s.type; texs[i].even = s.even; texs[i].odd = s.odd; texs[i].perlin = s.perlin; texs[i].image = s.image; texs[i].pad = 0;
        for (int a = 0; a < 3; ++a) texs[i].c[a] = R(s.c[a]);
        texs[i].scale = R(s.scale);
        for (int a = 0; a < 6; ++a) texs[i].uv[a] = R(s.uv[a]);
    }
    std::vector<PerlinRec<R>> per(f.perlins.size());
    for (size_t i = 0; i < per.size(); ++i) {
        for (int v = 0; v < 256; ++v) for (int a = 0; a < 3; ++a) per[i].ranvec[v][a] = R(f.perlins[i].ranvec[v][a]);
        std::memcpy(per[i].perm, f.perlins[i].perm, sizeof per[i].perm);
    }
    ds.view.spheres = ds.upload(sph);
    ds.view.tris = ds.upload(tri);
    ds.view.rects = ds.upload(rect);
    ds.view.boxes = ds.upload(box);
    ds.view.primrefs = ds.upload(f.primrefs);
    {  // every scene with a BVH: any kernel instantiated with triangles reads it, whatever the scene holds
        std::vector<TriRec<R>> lt(f.primrefs.size());
        for (size_t i = 0; i < lt.size(); ++i)
            if (!slot_pad[i] && primref_type(f.primrefs[i]) == PRIM_TRIANGLE) lt[i] = tri[primref_index(f.primrefs[i])];
        ds.view.leaf_tris = ds.upload(lt);
        if constexpr (std::is_same<R, double>::value) {
            // TriRec112: the plane of each leaf triangle by the device's operations in its order (device.h cross, dot;
            // -ffp-contract=off on both sides): n = cross(p2 - p1, p3 - p1), dd = -dot(n, p1), bit for bit
            std::vector<TriRec112<R>> l112(lt.size());
            for (size_t i = 0; i < lt.size(); ++i) {
                const R* q = lt[i].p;
                const R ux = q[3] - q[0], uy = q[4] - q[1], uz = q[5] - q[2];
                const R vx = q[6] - q[0], vy = q[7] - q[1], vz = q[8] - q[2];
                const R nx = uy * vz - uz * vy, ny = uz * vx - ux * vz, nz = ux * vy - uy * vx;
                for (int k = 0; k < 9; ++k) l112[i].p[k] = q[k];
                l112[i].n[0] = nx;
                l112[i].n[1] = ny;
                l112[i].n[2] = nz;
                l112[i].dd = -(nx * q[0] + ny * q[1] + nz * q[2]);
                l112[i].mat = lt[i].mat;
                l112[i].pad = 0;
            }
            ds.view.leaf_tris112 = ds.upload(l112);
        }
        std::vector<PrimRec80> lp(f.primrefs.size());  // every primitive type in leaf order (triangle-free kernels)
        for (size_t i = 0; i < lp.size(); ++i) {
            if (slot_pad[i]) continue;
            const uint32_t ref = f.primrefs[i], idx = primref_index(ref);
            switch (primref_type(ref)) {
                case PRIM_SPHERE: std::memcpy(lp[i].b, &sph[idx], sizeof(sph[idx])); break;
                case PRIM_TRIANGLE: std::memcpy(lp[i].b, &tri[idx], sizeof(tri[idx])); break;
                case PRIM_RECT: std::memcpy(lp[i].b, &rect[idx], sizeof(rect[idx])); break;
                default: std::memcpy(lp[i].b, &box[idx], sizeof(box[idx])); break;
            }
        }
        ds.view.leaf_prims = ds.upload(lp);
    }
    {  // BvhNode::pad: the 16-bit child codes (layout.h make_leaf16), derived here from the 32-bit ones (never read
       // from a scene file); codes16 when every inner index, leaf and hoisted leaf fits them
        std::vector<BvhNode> nodes = f.nodes;
        bool ok = nodes.size() <= 32768u;
        for (BvhNode& b : nodes) {
            int32_t c16[4];
            for (int c = 0; c < 4; ++c) {
                const int32_t x = b.child[c];
                if (x >= 0) {
                    c16[c] = x;
                } else if (x == kNodeEmpty) {
                    c16[c] = kNodeEmpty;
                } else {
                    ok = ok && leaf16_ok(leaf_first(x) >> ds.leaf_shift, leaf_count(x));
                    c16[c] = ok ? make_leaf16(leaf_first(x) >> ds.leaf_shift, leaf_count(x)) : kNodeEmpty;
                }
            }
            b.pad[0] = static_cast<int32_t>((static_cast<uint32_t>(c16[1]) << 16) | (static_cast<uint32_t>(c16[0]) & 0xFFFFu));
            b.pad[1] = static_cast<int32_t>((static_cast<uint32_t>(c16[3]) << 16) | (static_cast<uint32_t>(c16[2]) & 0xFFFFu));
            b.pad[2] = b.pad[3] = 0;
        }
        for (const auto& o : f.objs)
            if (o.kind == OBJ_BVH && o.b != kNodeEmpty) ok = ok && leaf16_ok(leaf_first(o.b) >> ds.leaf_shift, leaf_count(o.b));
        // option render.codes16 = 0 (read per upload; tests): take the 32-bit-code kernels as a scene whose codes do
        // not fit would (a parity probe of that path on scenes that fit)
        if (opt(Opt::Codes16) == 0) ok = false;
        ds.codes16 = ok;
        if (!ok) ds.leaf_shift = 0;  // the 32-bit codes (child[]) address the padded slots directly
        ds.view.nodes = ds.upload(nodes);
    }
    ds.view.objs = ds.upload(objs);
    {  // obj_prims[o]: prim object o's primitive record (device.h hit_object)
        std::vector<PrimRec80> op(objs.size());
        for (size_t i = 0; i < objs.size(); ++i) {
            if (objs[i].kind != OBJ_PRIM) continue;
            const uint32_t ref = static_cast<uint32_t>(objs[i].a), idx = primref_index(ref);
            switch (primref_type(ref)) {
                case PRIM_SPHERE: std::memcpy(op[i].b, &sph[idx], sizeof(sph[idx])); break;
                case PRIM_TRIANGLE: std::memcpy(op[i].b, &tri[idx], sizeof(tri[idx])); break;
                case PRIM_RECT: std::memcpy(op[i].b, &rect[idx], sizeof(rect[idx])); break;
                default: std::memcpy(op[i].b, &box[idx], sizeof(box[idx])); break;
            }
        }
        static_assert(sizeof(SphereRec<R>) <= sizeof(PrimRec80) && sizeof(TriRec<R>) <= sizeof(PrimRec80) &&
                      sizeof(RectRec<R>) <= sizeof(PrimRec80) && sizeof(BoxRec<R>) <= sizeof(PrimRec80), "PrimRec80 holds every record");
        ds.view.obj_prims = ds.upload(op);
    }
    ds.view.world = ds.upload(f.world);
    ds.view.mats = ds.upload(mats);
    ds.view.texs = ds.upload(texs);
    ds.view.perlins = ds.upload(per);
    {  // [sphere_uv.h's table][image records]: device.h uv_table reads the table in front of DevScene::images
        std::vector<uint8_t> ib(kUvTableBytes + sizeof(ImageRec) * f.images.size(), 0);
        std::memcpy(ib.data(), glibc_trig_data::kTrigHost, sizeof(glibc_trig_data::kTrigHost));
        if (!f.images.empty()) std::memcpy(ib.data() + kUvTableBytes, f.images.data(), sizeof(ImageRec) * f.images.size());
        ds.view.images = reinterpret_cast<const ImageRec*>(ds.upload(ib) + kUvTableBytes);
    }
    ds.view.texels = ds.upload(f.texels);
    if (std::is_same<R, double>::value) {
        uint32_t nmov = 0;
        bool shade_ok = false;
        const std::vector<uint8_t> img = ds.leaf_shift ? std::vector<uint8_t>() : lds_scene_image(f, nmov, shade_ok);
        if (!img.empty()) {
            ds.view.lds_image = ds.upload(img);
            ds.lds_scene = true;
            ds.lds_shade = shade_ok;
        }
    }
    ds.view.n_nodes = static_cast<uint32_t>(f.nodes.size());
    ds.view.n_objs = static_cast<uint32_t>(f.objs.size());
    ds.view.n_mats = static_cast<uint32_t>(f.mats.size());
    ds.view.n_primrefs = static_cast<uint32_t>(f.primrefs.size());
    ds.view.n_tris = static_cast<uint32_t>(f.tris.size());
    ds.view.nworld = static_cast<int32_t>(f.world.size());
    for (int a = 0; a < 3; ++a) ds.view.bg[a] = R(f.background[a]);
    ds.media = f.has_media;
    ds.features = f.features;
    ds.max_stack = f.max_stack;
    ds.tex_basic = true;
    for (const auto& t : f.texs) ds.tex_basic = ds.tex_basic && (t.type == TEX_SOLID || t.type == TEX_CHECKER);
    {  // TF_BARY: the texture trees the materials reach hold only solid, checker and barycentric-image nodes (a
       // mesh's bary_image refers to its image texture, which no material samples directly), and no primitive but a
       // triangle samples u, v
        bool bary = !ds.tex_basic;
        std::function<bool(int32_t, int)> tree_ok = [&](int32_t t, int depth) -> bool {
            if (t < 0 || static_cast<size_t>(t) >= f.texs.size()) return true;
            const uint32_t ty = f.texs[t].type;
            if (ty == TEX_SOLID || ty == TEX_BARY_IMAGE) return true;
            return ty == TEX_CHECKER && depth < 4 && tree_ok(f.texs[t].even, depth + 1) && tree_ok(f.texs[t].odd, depth + 1);
        };
        for (const auto& m : f.mats)
            if (m.type == MAT_LAMBERTIAN || m.type == MAT_LIGHT || m.type == MAT_ISOTROPIC) bary = bary && tree_ok(m.tex, 0);
        auto needs_uv = [&](uint32_t m) { return m < f.mats.size() && (f.mats[m].flags & MATF_NEEDS_UV) != 0; };
        for (const auto& p : f.spheres) bary = bary && !needs_uv(p.mat);
        for (const auto& p : f.rects) bary = bary && !needs_uv(p.mat);
        for (const auto& p : f.boxes) bary = bary && !needs_uv(p.mat);
        ds.tex_bary = bary && opt(Opt::TexBary) != 0;
    }
    ds.mat_types = 0;
    for (const auto& m : f.mats) ds.mat_types |= 1u << m.type;
}

// ------------------------------------------------------------------------------------------------ renderer
struct Renderer::Impl {
    int device = 0;
    int num_cu = 256;
    hipStream_t own_stream = nullptr;
    FlatScene flat;
    DeviceScene<double> s64;
    bool up64 = false;
    // workspace (grow-only)
    void* ws = nullptr;
    size_t ws_bytes = 0;
    hipEvent_t ev[2] = {nullptr, nullptr};

    ~Impl() {
        s64.release();
        if (ws) (void)hipFree(ws);
        for (auto& e : ev) if (e) (void)hipEventDestroy(e);
        if (own_stream) (void)hipStreamDestroy(own_stream);
    }
    // Grow-only workspace.  The old buffer is released before the larger one is allocated (both need not fit), and
    // ws / ws_bytes describe a live allocation at every point: a failed hipMalloc leaves them at {nullptr, 0}, so the
    // next render allocates again instead of handing out offsets from a null base.
    void* workspace(size_t bytes) {
        // fault point (tests): option test.fault_workspace_bytes = N > 0 makes every workspace growth beyond N bytes
        // fail as a refused hipMalloc would, after the old buffer is released
        const double lim = opt(Opt::FaultWorkspaceBytes);
        if (bytes > ws_bytes) {
            if (lim > 0 && static_cast<double>(bytes) > lim) {
                if (ws) (void)hipFree(ws);
                ws = nullptr;
                ws_bytes = 0;
                throw std::runtime_error("workspace allocation of " + std::to_string(bytes) + " bytes refused (test.fault_workspace_bytes)");
            }
            if (ws) {
                void* old = ws;
                ws = nullptr;
                ws_bytes = 0;
                HIP_OK(hipFree(old));
            }
            void* p = nullptr;
            HIP_OK(hipMalloc(&p, bytes));
            ws = p;
            ws_bytes = bytes;
        }
        return ws;
    }
};

Renderer::Renderer(FlatScene flat, int device) : impl_(new Impl) {
    impl_->device = device;
    HIP_OK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device));
    impl_->num_cu = prop.multiProcessorCount;
    impl_->flat = std::move(flat);
    HIP_OK(hipStreamCreateWithFlags(&impl_->own_stream, hipStreamNonBlocking));
}
Renderer::~Renderer() {
    if (impl_) {
        (void)hipSetDevice(impl_->device);
        delete impl_;
    }
}
size_t Renderer::scene_bytes() const { return impl_->s64.bytes; }
const FlatScene& Renderer::flat() const { return impl_->flat; }

#endif
// The LDS-scene kernels address the scene image at LDS address 0 (device.h lds_f4): they must declare no static
// __shared__ variables, which would be placed first.
static bool static_lds_is_zero(const void* kernel) {
    hipFuncAttributes a{};
    HIP_OK(hipFuncGetAttributes(&a, kernel));
    if (a.sharedSizeBytes != 0) throw std::runtime_error("LDS-scene kernel has static LDS: the scene image would not start at address 0");
    return true;
}
// Launch configuration per (kernel, device, dynamic LDS bytes): the > 64 KiB dynamic-LDS attribute, which
// hipFuncSetAttribute records per device, and the blocks per CU of a persistent grid (every block the CUs hold at
// once).  Scenes on different devices may render from different host threads, so the cache is
// mutex-guarded instead of living in function-local statics shared by all devices.
struct LaunchKey {
    const void* kernel;
    int device;
    size_t lds;
    bool operator<(const LaunchKey& o) const { return std::tie(kernel, device, lds) < std::tie(o.kernel, o.device, o.lds); }
};
static int blocks_per_cu(const void* kernel, int block, size_t lds) {
    static std::mutex mtx;
    static std::map<LaunchKey, int> cache;
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    const LaunchKey key{kernel, dev, lds};
    std::lock_guard<std::mutex> lock(mtx);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (lds > 64 * 1024) HIP_OK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    cache.emplace(key, per_cu);
    return per_cu;
}
#if ART_SPLIT_PATHS <= 1
template <class R, uint32_t F, uint32_t M, uint32_t TF>
static int shade_blocks(int num_cu) {
    return blocks_per_cu(reinterpret_cast<const void*>(k_shade<R, F, M, TF>), kBlock, 0) * num_cu;
}
// Textured materials get the "solid + checker" instantiation unless the scene holds noise or image textures.
template <class R, uint32_t F, uint32_t M>
static void launch_shade(uint32_t mat_types, bool tex_basic, int num_cu, hipStream_t st, const DevScene<R>& S, const PassGeom& g,
                         const Work<R>& w, int d) {
    if (!(mat_types & (1u << M))) return;
    constexpr bool textured = M == MAT_LAMBERTIAN || M == MAT_LIGHT || M == MAT_ISOTROPIC;
    if (!textured || tex_basic)
        hipLaunchKernelGGL((k_shade<R, F, M, kTexBasic>), dim3(shade_blocks<R, F, M, kTexBasic>(num_cu)), dim3(kBlock), 0, st, S, g, w, d);
    else
        hipLaunchKernelGGL((k_shade<R, F, M, TF_ALL>), dim3(shade_blocks<R, F, M, TF_ALL>(num_cu)), dim3(kBlock), 0, st, S, g, w, d);
}
// One bounce (extend + one shade launch per material type present) of the smallest kernel instantiation that
// covers the scene's features.
template <class R, uint32_t F, bool L, bool FUSE>
static void launch_extend(int num_cu, hipStream_t st, const DevScene<R>& S, const PassGeom& g, const CameraRec<R>& cam, const Work<R>& w, int d) {
    const size_t lds = extend_lds_bytes(L, g.stack);
    static const bool checked = !L || static_lds_is_zero(reinterpret_cast<const void*>(k_extend<R, F, L, FUSE>));
    (void)checked;
    // num_cu (256) is a multiple of 8: the wave count is a multiple of kShards
    const int blocks = blocks_per_cu(reinterpret_cast<const void*>(k_extend<R, F, L, FUSE>), L ? kBlockL : kBlock, lds) * num_cu;
    hipLaunchKernelGGL((k_extend<R, F, L, FUSE>), dim3(blocks), dim3(L ? kBlockL : kBlock), lds, st, S, g, cam, w, d);
}
// Extend variant: 0 = HBM scene, 1 = LDS scene, 2 = LDS scene with fused shading (no k_shade launches), 3 = persistent
// paths (k_paths: the fused LDS bounce loop in registers, one launch per pass).
// 4 = persistent paths over the HBM scene (k_paths_g: every other scene, f64).
enum ExtendVariant { EXT_GLOBAL = 0, EXT_LDS = 1, EXT_FUSED = 2, EXT_MEGA = 3, EXT_MEGA_G = 4 };
// One bounce (extend + one shade launch per material type present, unless fused) of the smallest kernel
// instantiation that covers the scene's features.
template <class R, uint32_t F>
static void launch_bounce(uint32_t mat_types, bool tex_basic, int variant, int num_cu, hipStream_t st, const DevScene<R>& S, const PassGeom& g,
                          const CameraRec<R>& cam, const Work<R>& w, int d, const std::function<void()>& mark) {
    if (mark) mark();
    if constexpr (F == kFeatSpheres && std::is_same<R, double>::value) {
        if (variant == EXT_FUSED) launch_extend<R, F, true, true>(num_cu, st, S, g, cam, w, d);
        else if (variant == EXT_LDS) launch_extend<R, F, true, false>(num_cu, st, S, g, cam, w, d);
        else launch_extend<R, F, false, false>(num_cu, st, S, g, cam, w, d);
    } else {
        launch_extend<R, F, false, false>(num_cu, st, S, g, cam, w, d);
    }
    if (mark) mark();
    if (variant != EXT_FUSED) {
        launch_shade<R, F, MAT_LAMBERTIAN>(mat_types, tex_basic, num_cu, st, S, g, w, d);
        launch_shade<R, F, MAT_METAL>(mat_types, tex_basic, num_cu, st, S, g, w, d);
        launch_shade<R, F, MAT_DIELECTRIC>(mat_types, tex_basic, num_cu, st, S, g, w, d);
        launch_shade<R, F, MAT_LIGHT>(mat_types, tex_basic, num_cu, st, S, g, w, d);
        launch_shade<R, F, MAT_ISOTROPIC>(mat_types, tex_basic, num_cu, st, S, g, w, d);
    }
    if (mark) mark();
}
// Extend variant for this scene and these flags (RT_GLOBAL_SCENE / RT_SPLIT_SHADE / RT_WAVEFRONT force the general
// kernels).
template <class R>
static int extend_variant(const DeviceScene<R>& ds, int flags) {
    if (!ds.lds_scene || (flags & RT_GLOBAL_SCENE) || (ds.features & ~kFeatSpheres) != 0)
        return (std::is_same<R, double>::value && !(flags & RT_WAVEFRONT)) ? EXT_MEGA_G : EXT_GLOBAL;
    // an LDS-image scene whose shading the LDS table cannot hold (noise / image textures: the two perlin spheres) runs
    // the persistent HBM-scene kernel, not the per-depth LDS wavefront one: r5 A/B (profiles/r5c_ab_scene3.txt) scene 3
    // 9 586 -> 23 864 Msamples/s; the wavefront variant stays reachable with RT_SPLIT_SHADE / RT_WAVEFRONT
    if (!ds.lds_shade)
        return (std::is_same<R, double>::value && !(flags & (RT_SPLIT_SHADE | RT_WAVEFRONT))) ? EXT_MEGA_G : EXT_LDS;
    if (flags & RT_SPLIT_SHADE) return EXT_LDS;
    return (flags & RT_WAVEFRONT) ? EXT_FUSED : EXT_MEGA;
}
// The persistent kernels' waves index the camera-ray rings (kPoolWavesPerCu per CU allocated)
static void check_ring_waves(int blocks, int block, int num_cu) {
    const size_t padded = (static_cast<size_t>(blocks) + kXcds - 1) / kXcds * kXcds;  // RayRing::init's XCD-major index
    if (padded * static_cast<size_t>(block / 64) > static_cast<size_t>(num_cu) * kPoolWavesPerCu)
        throw std::runtime_error("internal: persistent grid larger than the camera-ray rings");
}
// Which persistent-path kernel a render ran (rt_stats.kernel_*): k_paths_g<F, TF, LM>, or k_paths as LM 3
struct KernelId {
    uint32_t f = 0, tf = 0;
    int lm = -1;
};
template <uint32_t F, uint32_t TF>
static KernelId launch_paths_g_ft(int num_cu, hipStream_t st, const DevScene<double>& S, const PassGeom& g, const CameraRec<double>& cam,
                              const Work<double>& w, uint32_t* next_slot) {
    // g.stack = stack_rows: sentinel + entries + spare row
    const size_t lm_head = paths_g_head_bytes(g.stack, kBlockM, (F & F_CODE16) != 0) + paths_g_world_bytes(S.nworld, S.n_objs, lds_mats<TF>(S.n_mats));
    const size_t lds_m = align16(align128(lm_head) + paths_g_mesh_bytes(S.n_nodes, S.n_primrefs, (F & F_TRI) ? S.n_primrefs : 0u));
    // LM 1 also for a scene without BVH nodes (the earth scene: one sphere object): its world and objects in LDS and no
    // LM 0 suspend machinery (which spilled the earth's textured kernel)
    if (lds_m <= kPathsGLdsCap) {
        // the camera-ray rings (triangle-free kernels) when they fit too; otherwise the lanes generate their own rays
        const size_t lds_r = lds_m + paths_g_ring_bytes(kBlockM);
        PassGeom gr = g;
        // not for a world without a BVH node (the earth: one sphere): its traces are one primitive test and its paths end
        // after a segment or two, so most lanes start a path every round and the ring only adds LDS traffic (-1.4 %)
        gr.lds_ring = (paths_g_ring(F, 1) && S.n_nodes > 0 && lds_r <= kPathsGLdsCap) ? 1u : 0u;
        const size_t lds = gr.lds_ring ? lds_r : lds_m;
        const int blocks = blocks_per_cu(reinterpret_cast<const void*>(k_paths_g<F, TF, 1>), kBlockM, lds) * num_cu;
        check_ring_waves(blocks, kBlockM, num_cu);
        hipLaunchKernelGGL((k_paths_g<F, TF, 1>), dim3(blocks), dim3(kBlockM), lds, st, S, gr, cam, w, next_slot);
        return {F, TF, 1};
    }
    // too large for LM 1: as many of the first (top-level) nodes as fit beside the stacks
    const size_t head = align128(lm_head);
    const size_t node_bytes = sizeof(BvhNode);
    const uint32_t fit = head < kPathsGLdsCap ? static_cast<uint32_t>((kPathsGLdsCap - head) / node_bytes) : 0u;
    if (S.n_nodes > 0 && fit >= kLdsPartialMinNodes) {
        DevScene<double> SP = S;
        // option render.lds_nodes_max (diagnostic): a cap on the LDS-resident nodes, to measure what each one is worth
        const uint32_t cap = static_cast<uint32_t>(opt(Opt::LdsNodesMax));
        SP.n_lds_nodes = std::min<uint32_t>(std::min<uint32_t>(fit, S.n_nodes), std::max<uint32_t>(cap, kLdsPartialMinNodes));
        const size_t lds_p = head + node_bytes * SP.n_lds_nodes;
        const int blocks = blocks_per_cu(reinterpret_cast<const void*>(k_paths_g<F, TF, 2>), kBlockM, lds_p) * num_cu;
        check_ring_waves(blocks, kBlockM, num_cu);
        hipLaunchKernelGGL((k_paths_g<F, TF, 2>), dim3(blocks), dim3(kBlockM), lds_p, st, SP, g, cam, w, next_slot);
        return {F, TF, 2};
    }
    const size_t lds = paths_g_head_bytes(g.stack, kBlock, (F & F_CODE16) != 0);
    const int blocks = blocks_per_cu(reinterpret_cast<const void*>(k_paths_g<F, TF, 0>), kBlock, lds) * num_cu;
    check_ring_waves(blocks, kBlock, num_cu);
    hipLaunchKernelGGL((k_paths_g<F, TF, 0>), dim3(blocks), dim3(kBlock), lds, st, S, g, cam, w, next_slot);
    return {F, TF, 0};
}
static KernelId launch_paths_g(uint32_t feat, bool tex_basic, bool tex_bary, bool codes16, uint32_t leaf_shift, int num_cu, hipStream_t st,
                               const DevScene<double>& S, const PassGeom& g, const CameraRec<double>& cam, const Work<double>& w,
                               uint32_t* next_slot) {
    constexpr uint32_t C = F_CODE16;
    if (leaf_shift) {
        // pair-aligned leaves (build_device_scene: mesh feature sets with triangles only): the F_LEAF2 mesh kernels
        if (!codes16 || (feat & ~kFeatMesh) != 0 || !(feat & F_TRI)) throw std::runtime_error("internal: pair-aligned leaves outside the F_LEAF2 kernels");
        if (tex_basic) return launch_paths_g_ft<kMeshG | F_LEAF2, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
        if (tex_bary) return launch_paths_g_ft<kMeshG | F_LEAF2, kTexBary>(num_cu, st, S, g, cam, w, next_slot);
        return launch_paths_g_ft<kMeshG | F_LEAF2, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
    }
    if (!codes16 && (feat & F_MEDIA_G) == 0) {
        // 32-bit child codes (more than 32768 nodes or 8192 primitive references): the instantiations without F_CODE16.
        // A mesh scene (the capsule: 10 200 triangles, the reference's default scene) gets the mesh feature set, not
        // F_ALL (whose box, transform and boundary-traversal code spilled 45 VGPRs there); the triangle-free one when
        // the scene has no triangles (no triangle code in the kernel)
        if ((feat & ~kFeatMesh) == 0 && (feat & F_TRI)) {
            if (tex_basic) return launch_paths_g_ft<kFeatMesh, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
            return launch_paths_g_ft<kFeatMesh, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
        }
        if (feat & F_TRI) return launch_paths_g_ft<F_ALL, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
        if (tex_basic) return launch_paths_g_ft<F_ALL & ~F_TRI, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
        return launch_paths_g_ft<F_ALL & ~F_TRI, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
    } else if ((feat & ~kFeatSpheres) == 0) {
        if (tex_basic) return launch_paths_g_ft<kFeatSpheres | C, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
        else return launch_paths_g_ft<kFeatSpheres | C, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
    } else if ((feat & ~kFeatMesh) == 0) {
        // the F_TRI bit of an instantiation <=> the scene has triangles (leaf_tris exists)
        if (feat & F_TRI) {
            if (tex_basic) return launch_paths_g_ft<kFeatMesh | C, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
            if (tex_bary) return launch_paths_g_ft<kFeatMesh | C, kTexBary>(num_cu, st, S, g, cam, w, next_slot);
            else return launch_paths_g_ft<kFeatMesh | C, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
        } else {
            if (tex_basic) return launch_paths_g_ft<(kFeatMesh & ~F_TRI) | C, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
            else return launch_paths_g_ft<(kFeatMesh & ~F_TRI) | C, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
        }
    } else if ((feat & F_TRI) == 0) {  // e.g. the Next-Week final: no triangle code in the kernel
        // a non-sphere medium boundary (F_MEDIA_G: the Cornell smoke boxes) traverses from t = -inf: 32-bit codes
        if (feat & F_MEDIA_G) {
            if (tex_basic) return launch_paths_g_ft<F_ALL & ~F_TRI, kTexBasic>(num_cu, st, S, g, cam, w, next_slot);
            return launch_paths_g_ft<F_ALL & ~F_TRI, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
        }
        else return launch_paths_g_ft<(F_ALL & ~F_TRI & ~F_MEDIA_G) | C, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
    } else {
        return launch_paths_g_ft<F_ALL, TF_ALL>(num_cu, st, S, g, cam, w, next_slot);
    }
}
#endif
#if ART_SPLIT_PATHS == 0
#define ART_PATHS_LINKAGE static
#else
#define ART_PATHS_LINKAGE
#endif
#if ART_SPLIT_PATHS == 0 || ART_SPLIT_PATHS == 2
ART_PATHS_LINKAGE void launch_paths(int num_cu, hipStream_t st, const DevScene<double>& S, const PassGeom& g, const CameraRec<double>& cam,
                         const Work<double>& w, uint32_t* next_slot) {
    const size_t lds = paths_lds_bytes(g.stack);
    static const bool checked = static_lds_is_zero(reinterpret_cast<const void*>(k_paths));
    (void)checked;
    (void)blocks_per_cu(reinterpret_cast<const void*>(k_paths), kBlockL, lds);  // the LDS attribute; the grid is one block per CU
    hipLaunchKernelGGL(k_paths, dim3(num_cu), dim3(kBlockL), lds, st, S, g, cam, w, next_slot);
}
#else
void launch_paths(int num_cu, hipStream_t st, const DevScene<double>& S, const PassGeom& g, const CameraRec<double>& cam,
                  const Work<double>& w, uint32_t* next_slot);  // kernels_paths.o
#endif
#if ART_SPLIT_PATHS <= 1
template <class R>
static void bounce(const DeviceScene<R>& ds, int variant, int num_cu, hipStream_t st, const PassGeom& g, const CameraRec<R>& cam, const Work<R>& w,
                   int d, const std::function<void()>& mark) {
    const uint32_t feat = ds.features;
    if ((feat & ~kFeatSpheres) == 0)
        launch_bounce<R, kFeatSpheres>(ds.mat_types, ds.tex_basic, variant, num_cu, st, ds.view, g, cam, w, d, mark);
    else if ((feat & ~kFeatMesh) == 0)
        launch_bounce<R, kFeatMesh>(ds.mat_types, ds.tex_basic, EXT_GLOBAL, num_cu, st, ds.view, g, cam, w, d, mark);
    else
        launch_bounce<R, F_ALL>(ds.mat_types, ds.tex_basic, EXT_GLOBAL, num_cu, st, ds.view, g, cam, w, d, mark);
}

template <class R>
static void render_impl(Renderer::Impl& I, DeviceScene<R>& ds, const CameraRec<double>& camd, const RenderParams& p, uint8_t* out_rgb,
                        double* out_acc, RenderStats& stats) {
    hipStream_t stream = p.stream ? static_cast<hipStream_t>(p.stream) : I.own_stream;
    for (int a = 0; a < 3; ++a) ds.view.bg[a] = R(p.background[a]);  // engine::set_scene's background
    // local rows of this band partition
    std::vector<int> rows;
    for (int ly = 0;; ++ly) {
        int gy = (ly / p.band_rows) * (p.band_rows * p.band_count) + p.band_index * p.band_rows + (ly % p.band_rows);
        if (gy >= p.height) break;
        rows.push_back(gy);
    }
    const int nrows = static_cast<int>(rows.size());
    stats.local_rows = nrows;
    if (nrows == 0) return;
    PassGeom g{};
    g.W = p.width;
    g.H = p.height;
    g.rows = nrows;
    g.band_rows = p.band_rows;
    g.band_count = p.band_count;
    g.band_index = p.band_index;
    g.tiles_x = static_cast<uint32_t>((p.width + 7) / 8);
    const uint32_t tiles_y = static_cast<uint32_t>((nrows + 7) / 8);
    g.npix_pad = g.tiles_x * tiles_y * 64u;
    g.max_depth = p.max_depth;
    g.seed = p.seed;
    g.seed_mix = splitmix64(p.seed);
    g.fd_tiles_x = FastDiv::make(g.tiles_x);
    g.fd_band_rows = FastDiv::make(static_cast<uint32_t>(p.band_rows));
    g.fd_w = FastDiv::make(static_cast<uint32_t>(p.width));
    g.fd_npix = FastDiv::make(g.npix_pad);
    g.inv_w1 = 1.0 / static_cast<double>(p.width - 1);
    g.inv_h1 = 1.0 / static_cast<double>(p.height - 1);
    g.stack = stack_rows(ds.max_stack);
    const int variant = extend_variant(ds, p.flags);
    KernelId kid;  // the persistent kernel the passes ran (stays {0, 0, -1} for the wavefront variants)
    const bool mega = variant == EXT_MEGA || variant == EXT_MEGA_G;
    // Samples per pass: as many path slots as half of the free HBM holds (plus the workspace this renderer already
    // owns).  Every pass pays max_depth bounces of fixed launch/tail cost whatever its size, so on a 288 GB part the
    // 1080p x 1024 spp frame runs in 3 passes instead of ~40 (5.6 -> 6.9 Gsamples/s measured); spread evenly.
    // (persistent paths keep the path state in registers: a slot is its radiance record only)
    const size_t slot_bytes = mega ? sizeof(ResRec<R>) : sizeof(PathRec<R>) + sizeof(HitRecD<R>) + sizeof(ResRec<R>) + 4u * (2u + kNumMatTypes) + 8u;
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    const uint64_t target = std::min<uint64_t>((free_b + I.ws_bytes) / 2 / slot_bytes, kMaxPassSlots);  // fixed point: no regrowth
    // Slot ids, FastDiv operands and shard capacities are u32 and exact below 2^31: a pass never holds more than
    // kMaxPassSlots slots, whether k comes from free memory or from the caller's samples_per_pass.
    if (g.npix_pad > kMaxPassSlots) throw std::runtime_error("image too large for one pass (more than 2^31 padded pixels)");
    // samples traced per pixel: spp, or parallel_images' 4 * (spp / 4) (engine.h:411-414)
    const bool images = (p.flags & RT_PARALLEL_IMAGES) != 0;
    const int spp_t = images ? 4 * (p.spp / 4) : p.spp;
    const uint64_t k_cap = std::max<uint64_t>(1, kMaxPassSlots / g.npix_pad);
    uint64_t k64 = p.samples_per_pass > 0 ? static_cast<uint64_t>(p.samples_per_pass) : std::max<uint64_t>(1, target / g.npix_pad);
    k64 = std::min<uint64_t>(std::min<uint64_t>(k64, k_cap), static_cast<uint64_t>(std::max(1, spp_t)));
    uint32_t k = static_cast<uint32_t>(k64);
    const int npasses = static_cast<int>((std::max(1, spp_t) + k - 1) / k);
    k = static_cast<uint32_t>((std::max(1, spp_t) + npasses - 1) / npasses);
    const uint64_t Pmax64 = static_cast<uint64_t>(k) * g.npix_pad;
    if (Pmax64 > kMaxPassSlots) throw std::runtime_error("internal: pass larger than 2^31 slots");
    const uint32_t Pmax = static_cast<uint32_t>(Pmax64);
    g.cap = shard_cap(Pmax);
    const int depth_slots = p.max_depth + 1;
    const size_t local_pix = static_cast<size_t>(nrows) * p.width;

    auto al = [](size_t x) { return (x + 255) & ~static_cast<size_t>(255); };
    size_t off = 0;
    const size_t wf = mega ? 0u : 1u;  // wavefront-only buffers
    const size_t o_paths = off; off += wf * al(sizeof(PathRec<R>) * Pmax);
    const size_t o_hits = off; off += wf * al(sizeof(HitRecD<R>) * Pmax);
    const size_t o_res = off; off += al(sizeof(ResRec<R>) * Pmax);
    const size_t o_a0 = off; off += wf * al(4ull * kShards * g.cap);
    const size_t o_a1 = off; off += wf * al(4ull * kShards * g.cap);
    const size_t o_mq = off; off += wf * al(4ull * kMatSegs * g.cap);
    // (at least 4 depth lines: the device-counted adaptive levels take one each)
    const size_t cnt_words = static_cast<size_t>(std::max(depth_slots, 4)) * kQueueKinds * kShards * kCounterStride;
    const size_t o_cnt = off; off += al(4ull * cnt_words);
    const size_t o_seg = off; off += al(sizeof(unsigned long long));
    const size_t o_acc = off; off += al(sizeof(double) * 3 * local_pix);
    const size_t o_rgb = off; off += al(3 * local_pix);
    const size_t o_qsum = off; off += images ? al(sizeof(double) * 3 * local_pix) : 0;  // parallel_images quarter sums
    const size_t o_pool = off; off += (variant == EXT_MEGA) ? al(sizeof(PoolRay) * kPoolRing * kPoolWavesPerCu * static_cast<size_t>(I.num_cu)) : 0;
    // adaptive mode: int work frame, pixel list (<= 80 of every 144 pixels per level), square flags, list counter
    const bool adapt_ws = (p.flags & RT_ADAPTIVE) != 0;
    const size_t nsq_ws = adapt_ws ? local_pix / (kBig * kBig) : 0;
    const size_t o_adw = off; off += adapt_ws ? al(sizeof(int32_t) * 3 * local_pix) : 0;
    // four lists (one per level, at most 4 / 12 / 48 / 80 of every 144 pixels), each after its count word
    const size_t o_adl = off; off += adapt_ws ? al(4 * local_pix + 4 * 4 * 64) : 0;
    const size_t o_adf = off; off += adapt_ws ? al(21 * nsq_ws) : 0;
    const size_t o_adc = off; off += adapt_ws ? al(4) : 0;
    char* base = static_cast<char*>(I.workspace(off));
    int32_t* ad_work = reinterpret_cast<int32_t*>(base + o_adw);
    uint32_t* ad_list = reinterpret_cast<uint32_t*>(base + o_adl) + 64;  // host-counted levels: one list at a time
    uint8_t* ad_f0 = reinterpret_cast<uint8_t*>(base + o_adf);
    uint8_t* ad_f1 = ad_f0 + nsq_ws;
    uint8_t* ad_f2 = ad_f1 + 4 * nsq_ws;
    uint32_t* ad_count = reinterpret_cast<uint32_t*>(base + o_adc);

    Work<R> w{};
    w.paths = reinterpret_cast<PathRec<R>*>(base + o_paths);
    w.hits = reinterpret_cast<HitRecD<R>*>(base + o_hits);
    w.res = reinterpret_cast<ResRec<R>*>(base + o_res);
    w.active[0] = reinterpret_cast<uint32_t*>(base + o_a0);
    w.active[1] = reinterpret_cast<uint32_t*>(base + o_a1);
    w.mq = reinterpret_cast<uint32_t*>(base + o_mq);
    w.counters = reinterpret_cast<uint32_t*>(base + o_cnt);
    w.segments = reinterpret_cast<unsigned long long*>(base + o_seg);
    w.acc = reinterpret_cast<double*>(base + o_acc);
    w.pool = base + o_pool;
    uint8_t* drgb = reinterpret_cast<uint8_t*>(base + o_rgb);
    double* qsum = reinterpret_cast<double*>(base + o_qsum);

    CameraRec<R> cam{};
    for (int a = 0; a < 3; ++a) {
        cam.origin[a] = R(camd.origin[a]); cam.llc[a] = R(camd.llc[a]); cam.horizontal[a] = R(camd.horizontal[a]);
        cam.vertical[a] = R(camd.vertical[a]); cam.u[a] = R(camd.u[a]); cam.v[a] = R(camd.v[a]);
    }
    cam.lens_radius = R(camd.lens_radius);
    cam.time0 = R(camd.time0);
    cam.time1 = R(camd.time1);

    const bool prof = (p.flags & RT_PROFILE) != 0;
    const bool adaptive = (p.flags & RT_ADAPTIVE) != 0;
    const int levels = adaptive ? 4 : 1;
    std::vector<hipEvent_t> evs;
    for (auto& e : I.ev)
        if (!e) HIP_OK(hipEventCreate(&e));
    if (prof) {  // event pool created before the timed region (a pixel-list level never needs more passes than k gives)
        evs.resize(static_cast<size_t>(levels) * npasses * p.max_depth * 3);
        for (auto& e : evs) HIP_OK(hipEventCreate(&e));
    }
    size_t ev_next = 0;
    auto mark = [&]() { HIP_OK(hipEventRecord(evs[ev_next++], stream)); };
    int passes_run = 0;
    uint64_t ext_launches = 0;
    int spp_done = 0;      // samples traced so far (progressive snapshots)
    bool stopped = false;  // the progressive callback ended the render early
    // Traces spp samples of every local pixel (list == nullptr) or of every entry of a device pixel list, into
    // w.acc (per local pixel, or per list entry).
    auto trace = [&](const uint32_t* list, uint32_t nlist) {
        g.list = list;
        g.nlist = nlist;
        uint32_t kk = k, npix = static_cast<uint32_t>(local_pix);
        if (list) {
            npix = nlist;
            g.npix_pad = (nlist + 63u) & ~63u;
            g.fd_npix = FastDiv::make(g.npix_pad);
            kk = std::max<uint32_t>(1, std::min<uint32_t>(static_cast<uint32_t>(p.spp), Pmax / std::max<uint32_t>(g.npix_pad, 64u)));
        }
        HIP_OK(hipMemsetAsync(w.acc, 0, sizeof(double) * 3 * npix, stream));
        if (images) HIP_OK(hipMemsetAsync(qsum, 0, sizeof(double) * 3 * npix, stream));
        for (uint32_t sb = 0; sb < static_cast<uint32_t>(spp_t); sb += kk) {
            g.sample_base = sb;
            g.k = std::min<uint32_t>(kk, static_cast<uint32_t>(spp_t) - sb);
            g.P = g.k * g.npix_pad;
            g.live = g.k * npix;
            // the persistent kernels use one counter (counter(w, 0, 0, 0)): clear its line, not the wavefront queues' 1.25 MB
            HIP_OK(hipMemsetAsync(w.counters, 0, mega ? 4u * kCounterStride : 4ull * cnt_words, stream));
            bool persistent = false;
            if constexpr (std::is_same<R, double>::value) {
                if (mega) {
                    persistent = true;
                    if (p.max_depth > 0) {
                        if (prof) mark();
                        g.chunk = path_chunk(g.P, I.num_cu);
                        if (variant == EXT_MEGA) {
                            launch_paths(I.num_cu, stream, ds.view, g, cam, w, counter(w, 0, 0, 0));
                            kid = KernelId{kFeatSpheres, 0, 3};
                        } else {
                            kid = launch_paths_g(ds.features, ds.tex_basic, ds.tex_bary, ds.codes16, ds.leaf_shift, I.num_cu, stream, ds.view, g, cam, w,
                                                 counter(w, 0, 0, 0));
                        }
                        if (prof) { mark(); mark(); }
                        ++ext_launches;
                    }
                }
            }
            if (!persistent) {
                for (int d = 0; d < p.max_depth; ++d)
                    bounce<R>(ds, variant, I.num_cu, stream, g, cam, w, d, prof ? std::function<void()>(mark) : std::function<void()>());
                ext_launches += static_cast<uint64_t>(p.max_depth);
            }
            if (images) {
                hipLaunchKernelGGL(k_accum_images<R>, dim3((g.npix_pad + 255) / 256), dim3(256), 0, stream, g, w, qsum,
                                   static_cast<uint32_t>(spp_t / 4));
            } else {
                hipLaunchKernelGGL(k_accum<R>, dim3((g.npix_pad + 255) / 256), dim3(256), 0, stream, g, w);
            }
            ++passes_run;
            spp_done = static_cast<int>(sb + g.k);
            // progressive snapshot (whole-image traces only): write_color of the sums so far, with the samples so far
            if (!list && p.on_pass) {
                hipLaunchKernelGGL(k_finalize, dim3((npix + 255) / 256), dim3(256), 0, stream, w.acc, drgb, npix, spp_done);
                const hipMemcpyKind kind = (p.flags & RT_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
                if (out_rgb) HIP_OK(hipMemcpyAsync(out_rgb, drgb, 3ull * npix, kind, stream));
                if (out_acc) HIP_OK(hipMemcpyAsync(out_acc, w.acc, sizeof(double) * 3 * npix, kind, stream));
                HIP_OK(hipStreamSynchronize(stream));
                if (!p.on_pass(spp_done)) {
                    stopped = true;
                    break;
                }
            }
        }
    };
#ifdef ART_TRACE
    {
        long long tp = -1, ts = -1;
        if (const char* t = std::getenv("ART_TRACE")) std::sscanf(t, "%lld:%lld", &tp, &ts);
        HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace_pixel), &tp, sizeof tp));
        HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace_sample), &ts, sizeof ts));
    }
#endif
    HIP_OK(hipEventRecord(I.ev[0], stream));
    HIP_OK(hipMemsetAsync(w.segments, 0, sizeof(unsigned long long), stream));
    if (p.max_depth == 0) HIP_OK(hipMemsetAsync(w.res, 0, sizeof(ResRec<R>) * Pmax, stream));  // engine.h:451-452
    uint64_t traced = local_pix;
    uint32_t ad_counts[4] = {0, 0, 0, 0};  // the device-counted levels' entry counts (read back with the frame)
    bool dev_counted = false;
    if (!adaptive) {
        trace(nullptr, 0);
        const uint32_t npix = static_cast<uint32_t>(local_pix);
        hipLaunchKernelGGL(k_finalize, dim3((npix + 255) / 256), dim3(256), 0, stream, w.acc, drgb, npix, stopped ? spp_done : p.spp);
    } else if (mega && k == static_cast<uint32_t>(spp_t) && !images && !p.on_pass) {
        // engine.h:151-333: levels 0..3 (k_adapt_* above), one pass each, with no host round trip: each level's list
        // count stays on the device (list[-1], PassGeom::list_mode 1), the persistent kernel reads it at its start and
        // the level's samples are entry-major (a wave traces one pixel's samples: coherent rays)
        const int sqx = p.width / kBig;
        const uint32_t nsq = static_cast<uint32_t>(sqx) * static_cast<uint32_t>(nrows / kBig);
        const uint32_t caps[4] = {4 * nsq, 12 * nsq, 48 * nsq, 80 * nsq};
        uint32_t* lists[4];
        {
            uint32_t* at = reinterpret_cast<uint32_t*>(base + o_adl);
            for (int L = 0; L < 4; ++L) {
                lists[L] = at + 64;  // the count word at lists[L][-1]
                at = lists[L] + ((caps[L] + 63u) & ~63u);
            }
        }
        HIP_OK(hipMemsetAsync(base + o_adl, 0, 4 * local_pix + 4 * 4 * 64, stream));  // every count 0
        HIP_OK(hipMemsetAsync(ad_work, 0xFF, sizeof(int32_t) * 3 * local_pix, stream));  // the reference's -1 frame
        hipLaunchKernelGGL(k_adapt_corners, dim3((nsq + 255) / 256), dim3(256), 0, stream, lists[0], p.width, sqx, nsq);
        g.list_mode = 1;
        g.k = k;
        g.npix_pad = k;
        g.fd_npix = FastDiv::make(k);
        g.sample_base = 0;
        // one slot counter line per level (counter(w, level, 0, 0): the wavefront variants' depth lines, unused here),
        // cleared together before level 0 instead of one fill launch per level
        HIP_OK(hipMemsetAsync(w.counters, 0, 4ull * kQueueKinds * kShards * kCounterStride * 4, stream));
        for (int level = 0; level < 4; ++level) {
            g.list = lists[level];
            g.nlist = caps[level];                      // upper bounds: the kernels read the count
            g.P = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(caps[level]) * k, kMaxPassSlots));
            g.live = g.P;
            if (static_cast<uint64_t>(caps[level]) * k > Pmax) throw std::runtime_error("internal: adaptive level larger than the pass workspace");
            if (p.max_depth > 0) {
                if (prof) mark();
                g.chunk = path_chunk(g.P, I.num_cu);
                if (variant == EXT_MEGA) {
                    launch_paths(I.num_cu, stream, ds.view, g, cam, w, counter(w, level, 0, 0));
                    kid = KernelId{kFeatSpheres, 0, 3};
                } else {
                    kid = launch_paths_g(ds.features, ds.tex_basic, ds.tex_bary, ds.codes16, ds.leaf_shift, I.num_cu, stream, ds.view, g, cam, w,
                                         counter(w, level, 0, 0));
                }
                if (prof) { mark(); mark(); }
                ++ext_launches;
            }
            ++passes_run;
            hipLaunchKernelGGL(k_adapt_accum, dim3((caps[level] + kAdaptAccumWaves - 1) / kAdaptAccumWaves), dim3(64 * kAdaptAccumWaves), 0, stream, lists[level],
                               reinterpret_cast<const ResRec<double>*>(w.res), k, p.spp, ad_work);
            if (level == 3) break;
            const uint32_t per = level == 0 ? 1u : (level == 1 ? 4u : 16u);
            hipLaunchKernelGGL(k_adapt_level, dim3((nsq * per + 255) / 256), dim3(256), 0, stream, level, ad_work, p.width, sqx, nsq, ad_f0,
                               ad_f1, ad_f2, lists[level + 1], lists[level + 1] - 1);
        }
        const uint32_t npix = static_cast<uint32_t>(local_pix);
        hipLaunchKernelGGL(k_adapt_fill, dim3((npix + 255) / 256), dim3(256), 0, stream, ad_work, drgb, p.width, nrows, sqx, ad_f0, ad_f1, ad_f2);
        for (int L = 0; L < 4; ++L) HIP_OK(hipMemcpyAsync(&ad_counts[L], lists[L] - 1, 4, hipMemcpyDeviceToHost, stream));
        dev_counted = true;
    } else {
        // engine.h:151-333: levels 0..3 (k_adapt_* above); the list sizes come back to the host between levels
        // (multi-pass levels, the wavefront variants)
        const int sqx = p.width / kBig;
        const uint32_t nsq = static_cast<uint32_t>(sqx) * static_cast<uint32_t>(nrows / kBig);
        HIP_OK(hipMemsetAsync(ad_work, 0xFF, sizeof(int32_t) * 3 * local_pix, stream));  // the reference's -1 frame
        hipLaunchKernelGGL(k_adapt_corners, dim3((nsq + 255) / 256), dim3(256), 0, stream, ad_list, p.width, sqx, nsq);
        uint32_t n = 4 * nsq;
        traced = 0;
        for (int level = 0;; ++level) {
            trace(ad_list, n);
            hipLaunchKernelGGL(k_adapt_store, dim3((n + 255) / 256), dim3(256), 0, stream, ad_list, n, w.acc, p.spp, ad_work);
            traced += n;
            if (level == 3) break;
            const uint32_t per = level == 0 ? 1u : (level == 1 ? 4u : 16u);
            HIP_OK(hipMemsetAsync(ad_count, 0, 4, stream));
            hipLaunchKernelGGL(k_adapt_level, dim3((nsq * per + 255) / 256), dim3(256), 0, stream, level, ad_work, p.width, sqx, nsq, ad_f0,
                               ad_f1, ad_f2, ad_list, ad_count);
            HIP_OK(hipMemcpyAsync(&n, ad_count, 4, hipMemcpyDeviceToHost, stream));
            HIP_OK(hipStreamSynchronize(stream));
            if (n == 0) break;
        }
        const uint32_t npix = static_cast<uint32_t>(local_pix);
        hipLaunchKernelGGL(k_adapt_fill, dim3((npix + 255) / 256), dim3(256), 0, stream, ad_work, drgb, p.width, nrows, sqx, ad_f0, ad_f1, ad_f2);
    }
    HIP_OK(hipGetLastError());
#ifdef ART_STATS
    {
        unsigned long long st[kArtStats] = {0};
        HIP_OK(hipStreamSynchronize(stream));
        HIP_OK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_art_stats), sizeof st));
        std::fprintf(stderr, "ART_STATS node_w %llu node_l %llu (util %.3f) leaf_w %llu leaf_l %llu (util %.3f) outer_w %llu outer_l %llu (util %.3f) "
                     "traversals %llu nodes/trav %.2f leaftests/trav %.2f\n",
                     st[0], st[1], st[1] / (64.0 * st[0]), st[2], st[3], st[3] / (64.0 * st[2]), st[4], st[5], st[5] / (64.0 * st[4]), st[6],
                     double(st[1]) / st[6], double(st[3]) / st[6]);
        std::fprintf(stderr, "ART_STATS dead node visits (LDS scene) %llu (%.3f of visits), stale visits (box entered beyond tmax) %llu (%.3f), "
                     "leaf tests that shorten tmax %llu (%.3f of tests)\n",
                     st[12], double(st[12]) / st[1], st[14], double(st[14]) / st[1], st[13], double(st[13]) / st[3]);
        if (st[15] + st[17] + st[19] + st[21] > 0)
            std::fprintf(stderr, "ART_STATS leaf tests by type (lane tests, wave iterations running it): box %llu %llu sphere %llu %llu triangle %llu %llu rect %llu %llu\n",
                         st[15], st[16], st[17], st[18], st[19], st[20], st[21], st[22]);
        const double tt = double(st[8] + st[9] + st[10] + st[11] + st[24] + st[25] + st[26]);
        if (tt > 0)
            std::fprintf(stderr, "ART_STATS cycles: load/claim %.3f trace %.3f shade %.3f append/store %.3f (k_paths_g shading split: surface %.3f "
                         "coop-sphere %.3f texture+unit %.3f scatter %.3f)\n",
                         st[8] / tt, st[9] / tt, (st[10] + st[24] + st[25] + st[26]) / tt, st[11] / tt, st[24] / tt, st[25] / tt, st[26] / tt, st[10] / tt);
        if (st[28] + st[30] > 0)
            std::fprintf(stderr, "ART_STATS texture evaluations (wave iterations, lanes): noise %llu %llu image %llu %llu\n", st[28], st[29], st[30], st[31]);
        if (st[46] > 0)
            std::fprintf(stderr, "ART_STATS leaf phases %llu: leaf-loop wave iterations %llu, a wave-cooperative leaf test's %llu (%.3f)\n", st[46], st[2],
                         st[47], double(st[47]) / double(st[2]));
        if (st[44] > 0)
            std::fprintf(stderr, "ART_STATS surface branches (wave iterations, lanes): world_surface %llu %llu sphere %llu %llu sphere-uv %llu %llu "
                         "unwind %llu %llu medium %llu %llu box/rect-record %llu %llu box/rect-carried %llu %llu\n",
                         st[44], st[45], st[40], st[41], st[32], st[33], st[34], st[35], st[36], st[37], st[38], st[39], st[42], st[43]);
        std::memset(st, 0, sizeof st);
        HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_art_stats), st, sizeof st));
    }
#endif
    HIP_OK(hipEventRecord(I.ev[1], stream));
    const hipMemcpyKind kind_rgb = (p.flags & RT_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (out_rgb) HIP_OK(hipMemcpyAsync(out_rgb, drgb, 3 * local_pix, kind_rgb, stream));
    if (out_acc && !adaptive) HIP_OK(hipMemcpyAsync(out_acc, w.acc, sizeof(double) * 3 * local_pix, kind_rgb, stream));
    unsigned long long segs = 0;
    HIP_OK(hipMemcpyAsync(&segs, w.segments, sizeof segs, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (dev_counted) traced = static_cast<uint64_t>(ad_counts[0]) + ad_counts[1] + ad_counts[2] + ad_counts[3];
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, I.ev[0], I.ev[1]));
    stats.ms = ms;
    stats.passes = passes_run;
    stats.samples_per_pass = static_cast<int>(k);
    stats.segments = segs;
    stats.extend_variant = variant;
    stats.kernel_features = kid.f;
    stats.kernel_textures = kid.tf;
    stats.kernel_lds_mode = kid.lm;
    stats.primary = traced * static_cast<uint64_t>(stopped ? spp_done : spp_t);
    if (prof) {
        double ext_ms = 0, sh_ms = 0;
        for (size_t e = 0; e + 2 < ev_next; e += 3) {
            float a = 0, b = 0;
            HIP_OK(hipEventElapsedTime(&a, evs[e], evs[e + 1]));
            HIP_OK(hipEventElapsedTime(&b, evs[e + 1], evs[e + 2]));
            ext_ms += a;
            sh_ms += b;
        }
        stats.extend_ms = ext_ms;
        stats.shade_ms = sh_ms;
        stats.extend_launches = ext_launches;
        stats.shade_launches = variant == EXT_GLOBAL || variant == EXT_LDS ? ext_launches : 0;
        for (auto e : evs) (void)hipEventDestroy(e);
    }
}

void Renderer::upload() {
    HIP_OK(hipSetDevice(impl_->device));
    if (!impl_->up64) {
        build_device_scene(impl_->flat, impl_->s64);
        impl_->up64 = true;
    }
}

void Renderer::trace_rays(const double* rays, size_t n, bool global_scene, double* t_out, double* n_out) {
    upload();
    const DeviceScene<double>& ds = impl_->s64;
    if (n == 0) return;
    if (n > (1u << 30)) throw std::runtime_error("too many rays");
    hipStream_t st = impl_->own_stream;
    const size_t in_b = sizeof(double) * 7 * n, t_b = sizeof(double) * n, n_b = sizeof(double) * 3 * n;
    char* base = static_cast<char*>(impl_->workspace(in_b + t_b + n_b));
    double* d_rays = reinterpret_cast<double*>(base);
    double* d_t = reinterpret_cast<double*>(base + in_b);
    double* d_n = reinterpret_cast<double*>(base + in_b + t_b);
    HIP_OK(hipMemcpyAsync(d_rays, rays, in_b, hipMemcpyHostToDevice, st));
    const uint32_t stack = stack_rows(ds.max_stack), nn = static_cast<uint32_t>(n);
    const uint32_t feat = ds.features;
    if (ds.lds_scene && !global_scene && (feat & ~kFeatSpheres) == 0) {
        const size_t lds = kLdsImageBytes + paths_stack_bytes(stack);
        static const bool checked = static_lds_is_zero(reinterpret_cast<const void*>(k_trace_rays<kFeatSpheres, true>));
        (void)checked;
        (void)blocks_per_cu(reinterpret_cast<const void*>(k_trace_rays<kFeatSpheres, true>), kBlockL, lds);
        hipLaunchKernelGGL((k_trace_rays<kFeatSpheres, true>), dim3((nn + kBlockL - 1) / kBlockL), dim3(kBlockL), lds, st, ds.view, d_rays, nn, stack, d_t, d_n);
    } else {
        const size_t lds = sizeof(int32_t) * stack * kBlock;
        const dim3 grid((nn + kBlock - 1) / kBlock);
        if ((feat & ~kFeatSpheres) == 0)
            hipLaunchKernelGGL((k_trace_rays<kFeatSpheres, false>), grid, dim3(kBlock), lds, st, ds.view, d_rays, nn, stack, d_t, d_n);
        else if ((feat & ~kFeatMesh) == 0)
            hipLaunchKernelGGL((k_trace_rays<kFeatMesh, false>), grid, dim3(kBlock), lds, st, ds.view, d_rays, nn, stack, d_t, d_n);
        else
            hipLaunchKernelGGL((k_trace_rays<F_ALL, false>), grid, dim3(kBlock), lds, st, ds.view, d_rays, nn, stack, d_t, d_n);
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(t_out, d_t, t_b, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(n_out, d_n, n_b, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
}

void Renderer::render(const CameraRec<double>& cam, const RenderParams& p, uint8_t* out_rgb, double* out_acc, RenderStats& stats) {
    if (p.fp_mode != RT_FP64) throw std::runtime_error("fp_mode must be RT_FP64");
    upload();
    render_impl<double>(*impl_, impl_->s64, cam, p, out_rgb, out_acc, stats);
}

#endif  // ART_SPLIT_PATHS <= 1
}  // namespace art

#if ART_SPLIT_PATHS <= 1
namespace art {
int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
}  // namespace art
#endif
