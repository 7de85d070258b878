// device.h — device-side math, RNG, intersection and shading routines (templated on the real type R).
//
// Every routine restates the reference function it cites with the SAME operation order (v/t == (1/t)*v, dot summed
// left to right, ...), so that the f64 instantiation reproduces the CPU restatement (oracle/restate.cpp, pcg mode)
// to the last bit up to libm-vs-OCML transcendental ulps.  The f32 instantiation runs the identical code in float.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <type_traits>

#include "glibc_log.h"
#include "layout.h"
#include "sphere_uv.h"

namespace art {

// ------------------------------------------------------------------------------------------------ vec3 (core/vec3.h)
template <class R>
struct V3 {
    R x, y, z;
};
template <class R> __device__ __forceinline__ V3<R> mk(R a, R b, R c) { return V3<R>{a, b, c}; }
template <class R> __device__ __forceinline__ V3<R> operator+(V3<R> u, V3<R> v) { return {u.x + v.x, u.y + v.y, u.z + v.z}; }
template <class R> __device__ __forceinline__ V3<R> operator-(V3<R> u, V3<R> v) { return {u.x - v.x, u.y - v.y, u.z - v.z}; }
template <class R> __device__ __forceinline__ V3<R> operator-(V3<R> u) { return {-u.x, -u.y, -u.z}; }
template <class R> __device__ __forceinline__ V3<R> operator*(V3<R> u, V3<R> v) { return {u.x * v.x, u.y * v.y, u.z * v.z}; }
template <class R> __device__ __forceinline__ V3<R> operator*(R t, V3<R> v) { return {t * v.x, t * v.y, t * v.z}; }
// std::sqrt, correctly rounded (sphere.h:47, vec3.h:42 length, vec3.h:152 refract, material.h:75 and
// constant_medium.h:61).  For x >= 2^-767 this is the compiler's own f64 sqrt expansion (hardware rsq, then two
// Goldschmidt and two Newton fma steps) without its denormal-range scaling and its zero/inf select, which never apply
// there: the same operations on the same values, so the same bits.  Smaller x (and 0), inf and NaN take the
// compiler's full sequence.  Saves 7 VALU per call: the leaf test's root, unit_vector and refraction per bounce.
__device__ __forceinline__ double sqrt_rn(double x) {
    if (!(x >= 0x1p-767 && x < __builtin_inf())) return sqrt(x);
    const double y = __builtin_amdgcn_rsq(x);
    double s = x * y, h = y * 0.5;
    const double r = fma(-h, s, 0.5);
    s = fma(s, r, s);
    h = fma(h, r, h);
    s = fma(fma(-s, s, x), h, s);
    return fma(fma(-s, s, x), h, s);
}
__device__ __forceinline__ float sqrt_rn(float x) { return sqrtf(x); }

template <class R> __device__ __forceinline__ R dot(V3<R> u, V3<R> v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
template <class R> __device__ __forceinline__ R len2(V3<R> v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
template <class R> __device__ __forceinline__ V3<R> cross(V3<R> u, V3<R> v) {
    return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
template <class R> __device__ __forceinline__ V3<R> divs(V3<R> v, R t) { return (R(1) / t) * v; }  // vec3.h:97-99: (1/t) * v
template <class R> __device__ __forceinline__ V3<R> unit(V3<R> v) { return divs(v, sqrt_rn(len2(v))); }
template <class R> __device__ __forceinline__ bool near_zero(V3<R> v) {  // vec3.h:49-53
    const R s = R(1e-8);
    return fabs(v.x) < s && fabs(v.y) < s && fabs(v.z) < s;
}
template <class R> __device__ __forceinline__ V3<R> reflect(V3<R> v, V3<R> n) { return v - (R(2) * dot(v, n)) * n; }
template <class R> __device__ __forceinline__ V3<R> refract(V3<R> uv, V3<R> n, R eta) {  // vec3.h:149-154
    R cos_theta = fmin(dot(-uv, n), R(1));
    V3<R> perp = eta * (uv + cos_theta * n);
    V3<R> par = (-sqrt_rn(fabs(R(1) - len2(perp)))) * n;
    return perp + par;
}
template <class R> __device__ __forceinline__ V3<R> ld3(const R* p) { return {p[0], p[1], p[2]}; }

template <class R>
struct Ray {
    V3<R> o, d;
    R tm;
    __device__ __forceinline__ V3<R> at(R t) const { return o + t * d; }
};

// ------------------------------------------------------------------------------------------------ RNG contract
// PCG32 (O'Neill), one 64-bit state per path, seeded from (seed, global pixel, sample) through splitmix64 so the
// stream depends only on what is rendered, never on tiling or GPU count.  Uniforms carry 24 bits: exact in f32/f64.
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__host__ __device__ inline uint64_t pcg_seed(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return splitmix64(((static_cast<uint64_t>(pixel) << 32) | sample) ^ splitmix64(seed));
}
template <class R>
__device__ __forceinline__ R uniform(uint64_t& s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = static_cast<uint32_t>(old >> 59u);
    const uint32_t x = (xs >> rot) | (xs << ((32u - rot) & 31u));
    return static_cast<R>(x >> 8) * static_cast<R>(1.0 / 16777216.0);
}
template <class R> __device__ __forceinline__ R uniform(uint64_t& s, R lo, R hi) { return lo + (hi - lo) * uniform<R>(s); }
// The 24-bit integer k of the next uniform (uniform<R> == k * 2^-24): the argument of glibc_log in hit_medium.
__device__ __forceinline__ uint32_t uniform_k(uint64_t& s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = static_cast<uint32_t>(old >> 59u);
    return ((xs >> rot) | (xs << ((32u - rot) & 31u))) >> 8;
}
// uniform(s, -1, 1) = -1 + 2 * (k * 2^-24) with k < 2^24: every step is exact, so the single fma k * 2^-23 - 1 is the
// same value
template <class R>
__device__ __forceinline__ R uniform_pm1(uint64_t& s) {
    const uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = static_cast<uint32_t>(old >> 59u);
    const uint32_t x = (xs >> rot) | (xs << ((32u - rot) & 31u));
    return fma(static_cast<R>(x >> 8), static_cast<R>(1.0 / 8388608.0), R(-1));
}
template <class R>
__device__ __forceinline__ V3<R> in_unit_sphere(uint64_t& s) {  // vec3.h:117-123, draws x, y, z
    for (;;) {
        V3<R> p;
        p.x = uniform_pm1<R>(s);
        p.y = uniform_pm1<R>(s);
        p.z = uniform_pm1<R>(s);
        if (len2(p) >= R(1)) continue;
        return p;
    }
}

// PCG32 jump-ahead (Brown 1994, "Random number generation with arbitrary strides"): n steps of s -> A s + C are one
// affine map s -> A_n s + C_n (mod 2^64).  kJumpEntries maps of n = 3 j draws (one random_in_unit_sphere candidate per
// j) let a lane compute the state at another lane's j-th candidate directly.
constexpr int kJumpEntries = 64;  // j = 0..63
struct JumpEntry {
    uint64_t a, c;
};
__host__ __device__ inline JumpEntry pcg_jump(uint32_t steps) {
    uint64_t a = 1, c = 0;
    for (uint32_t i = 0; i < steps; ++i) {
        a = a * 6364136223846793005ull;
        c = c * 6364136223846793005ull + 1442695040888963407ull;
    }
    return JumpEntry{a, c};
}

// random_in_unit_sphere (vec3.h:117-123) for every lane with `need`, the wave cooperating on the rejection loop.  A
// lane's result is the first candidate of its own stream inside the unit ball, and its stream ends right after that
// candidate -- exactly the serial loop's draws -- but the search runs in rounds: round 0 tests every lane's next
// candidate in place; in each later round the R lanes still searching share the 64 lanes, K = 64 / R consecutive
// candidates each (a helper lane jumps the owner's state ahead by 3 j draws and tests candidate j), and the owner
// takes the first accepted one.  A wave needs ~2 rounds instead of the ~6 serial iterations of its unluckiest lane.
// Must be called by the whole wave (the helpers are every lane, active or not in the path loop).  jt: the jump table
// in LDS (kJumpEntries JumpEntry).
template <class R>
__device__ __forceinline__ V3<R> coop_unit_sphere(bool need, uint64_t& rng, const JumpEntry* jt) {
    const uint32_t lane = __lane_id();
    V3<R> p = mk(R(0), R(0), R(0));
    uint64_t s = rng;  // pending lanes: the state at the next untested candidate
    bool pending = false;
    if (need) {
        p.x = uniform_pm1<R>(s);
        p.y = uniform_pm1<R>(s);
        p.z = uniform_pm1<R>(s);
        if (len2(p) >= R(1)) pending = true;
        else rng = s;
    }
    uint64_t mask = __ballot(pending);
    while (mask) {
        const uint32_t nr = static_cast<uint32_t>(__popcll(mask));
        const uint32_t k = 64u / nr;  // candidates per searching lane this round
        const uint32_t rank = static_cast<uint32_t>(__popcll(mask & ((1ull << lane) - 1ull)));
        // owner of rank r -> lane r holds the owner's lane id (push), then helper w reads it from lane w / k
        // (lanes that own nothing push to lane 63, which is read only when all 64 lanes search and then it is
        // pushed by its owner alone)
        const int owner_at_rank = __builtin_amdgcn_ds_permute(static_cast<int>(pending ? rank : 63u) * 4, static_cast<int>(lane));
        // o = floor(lane / k): (lane + 1/2) / k is >= 1/(2k) >= 2^-7 away from an integer, far above the error of a
        // 1-ulp reciprocal
        const uint32_t o = static_cast<uint32_t>((static_cast<float>(lane) + 0.5f) * __builtin_amdgcn_rcpf(static_cast<float>(k)));
        const uint32_t j = lane - o * k;
        const bool helper = o < nr;
        const int owner_lane = __builtin_amdgcn_ds_bpermute(static_cast<int>(helper ? o : 0u) * 4, owner_at_rank);
        const uint32_t slo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(owner_lane * 4, static_cast<int>(static_cast<uint32_t>(s))));
        const uint32_t shi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(owner_lane * 4, static_cast<int>(static_cast<uint32_t>(s >> 32))));
        const JumpEntry e = jt[j];
        uint64_t hs = e.a * ((static_cast<uint64_t>(shi) << 32) | slo) + e.c;
        V3<R> c;
        c.x = uniform_pm1<R>(hs);
        c.y = uniform_pm1<R>(hs);
        c.z = uniform_pm1<R>(hs);
        const uint64_t acc = __ballot(helper && len2(c) < R(1));
        // owners: the first accepted candidate of their k; its helper's state (hs) is the state right after it.
        // With none accepted, the state after the last helper's candidate is where the next round starts.
        const uint64_t mine = k == 64u ? acc : (acc >> (rank * k)) & ((1ull << k) - 1ull);
        const uint32_t jstar = mine ? static_cast<uint32_t>(__ffsll(static_cast<long long>(mine)) - 1) : k - 1u;
        const int src = static_cast<int>(pending ? rank * k + jstar : lane) * 4;
        const uint32_t nlo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(static_cast<uint32_t>(hs))));
        const uint32_t nhi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(static_cast<uint32_t>(hs >> 32))));
        V3<R> got;
        got.x = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(c.x)), __builtin_amdgcn_ds_bpermute(src, __double2loint(c.x)));
        got.y = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(c.y)), __builtin_amdgcn_ds_bpermute(src, __double2loint(c.y)));
        got.z = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(c.z)), __builtin_amdgcn_ds_bpermute(src, __double2loint(c.z)));
        if (pending) {
            const uint64_t next = (static_cast<uint64_t>(nhi) << 32) | nlo;
            if (mine) {
                p = got;
                rng = next;
                pending = false;
            } else {
                s = next;
            }
        }
        mask = __ballot(pending);
    }
    return p;
}

// ------------------------------------------------------------------------------------------------ device scene view
template <class R>
struct DevScene {
    const SphereRec<R>* spheres;
    const TriRec<R>* tris;
    const RectRec<R>* rects;
    const BoxRec<R>* boxes;
    const uint32_t* primrefs;
    const BvhNode* nodes;
    const ObjRec<R>* objs;
    const int32_t* world;
    const MatRec<R>* mats;
    const TexRec<R>* texs;
    const PerlinRec<R>* perlins;
    const ImageRec* images;
    const uint8_t* texels;
    const TriRec<R>* leaf_tris;  // leaf_tris[slot] = tris[index of primrefs[slot]] for triangle refs, zeros otherwise
    const TriRec112<R>* leaf_tris112;  // the same with each triangle's plane (n, dd), for the LM 1 kernels' LDS copy
    const PrimRec80* leaf_prims;  // leaf_prims[slot]: the record of primrefs[slot] of any type (triangle-free kernels)
    const PrimRec80* obj_prims;  // obj_prims[o] = the record of prim object o's primitive (indexed like objs)
    const uint8_t* lds_image;   // layout.h LDS scene image (nullptr unless the scene qualifies)
    uint32_t n_nodes, n_primrefs, n_tris, n_objs, n_mats;  // array lengths (k_paths_g's LDS copies)
    uint32_t nodes_lds;         // k_paths_g LM 2: LDS byte address of the copy of nodes [0, n_lds_nodes) (top levels)
    uint32_t n_lds_nodes;
    int32_t nworld;
    R bg[3];
};

// sphere_uv.h's table (glibc_trig.h's constants, then its acos / atan tables) rides in front of the image records
// (DevScene::images - kUvTableBytes, uploaded with them), so the scene view -- the kernels' argument block -- keeps its layout (a new field moved every later kernel
// argument and cost k_paths 0.3 %)
template <class R>
__device__ __forceinline__ const double* uv_table(const DevScene<R>& S) {
    return reinterpret_cast<const double*>(reinterpret_cast<const uint8_t*>(S.images) - kUvTableBytes);
}

constexpr uint32_t kMediumHit = 0xFFFFFFFFu;  // hit.prim value of a constant_medium scattering event

// ------------------------------------------------------------------------------------------------ primitives
// x / a from a precomputed reciprocal inv_a = RN(1 / a): q = RN(x * inv_a) is within 1 ulp of x / a, the residual
// x - q * a is exact in one fma, and RN(q + residual * inv_a) is then the correctly rounded quotient (Markstein's
// theorem, e.g. Muller et al., Handbook of Floating-Point Arithmetic, 2nd ed., Thm. 4.10) -- the same bits as the
// division, for a, x and the quotient away from the overflow/underflow ranges: 3 FLOPs instead of the ~10-instruction
// scaled division sequence.  Callers guarantee the range (see hit_lds_slot and gen_ray).
template <class R>
__device__ __forceinline__ R div_rcp(R x, R a, R inv_a) {
    const R q = x * inv_a;
    return fma(fma(-q, a, x), inv_a, q);
}

// sphere.h:39-65 / moving_sphere.h:41-58 (root selection only; the surface is rebuilt in shade).  a = |d|^2 of the
// ray; RCP: the two root divisions by a use div_rcp with inv_a = 1 / a (same bits).
template <class R, bool RCP>
__device__ __forceinline__ bool sphere_root(V3<R> center, R r2, const Ray<R>& r, R a, R inv_a, R tmin, R tmax, R& t) {
    const V3<R> oc = r.o - center;
    const R half_b = dot(oc, r.d);
    const R c = len2(oc) - r2;
    const R disc = half_b * half_b - a * c;
    if (disc < R(0)) return false;
    const R sqrtd = sqrt_rn(disc);
    R root = RCP ? div_rcp(-half_b - sqrtd, a, inv_a) : (-half_b - sqrtd) / a;
    if (root < tmin || tmax < root) {
        root = RCP ? div_rcp(-half_b + sqrtd, a, inv_a) : (-half_b + sqrtd) / a;
        if (root < tmin || tmax < root) return false;
    }
    t = root;
    return true;
}
// sphere_root with the reciprocal taken where first needed: inv_a = 0 until a root division of this ray needs it
template <class R>
__device__ __forceinline__ bool sphere_root_lazy(V3<R> center, R r2, const Ray<R>& r, R a, R& inv_a, R tmin, R tmax, R& t) {
    const V3<R> oc = r.o - center;
    const R half_b = dot(oc, r.d);
    const R c = len2(oc) - r2;
    const R disc = half_b * half_b - a * c;
    if (disc < R(0)) return false;
    const R sqrtd = sqrt_rn(disc);
    if (inv_a == R(0)) inv_a = R(1) / a;
    R root = div_rcp(-half_b - sqrtd, a, inv_a);
    if (root < tmin || tmax < root) {
        root = div_rcp(-half_b + sqrtd, a, inv_a);
        if (root < tmin || tmax < root) return false;
    }
    t = root;
    return true;
}
template <class R>
__device__ __forceinline__ bool hit_sphere_r2(V3<R> center, R r2, const Ray<R>& r, R tmin, R tmax, R& t) {  // r2 = radius * radius
    return sphere_root<R, false>(center, r2, r, len2(r.d), R(0), tmin, tmax, t);
}
template <class R>
__device__ __forceinline__ bool hit_sphere_at(V3<R> center, R radius, const Ray<R>& r, R tmin, R tmax, R& t) {
    return hit_sphere_r2(center, radius * radius, r, tmin, tmax, t);
}
// std::pow(x, 5) of material.h:97 (Schlick reflectance).  x^5 is carried as a double-double product (each step's
// rounding error recovered exactly by an fma) and rounded once: the correctly rounded x^5.  glibc's pow is within
// 0.52 ulp of it and differs from it in ~0.09% of arguments (tests/test_pow5.py measures it), but the reflectance
// only feeds the comparison refl_p > u against a uniform on the 2^-24 grid, so the branch taken is the same unless u
// lies within 1 ulp of refl_p (probability < 2^-28 per draw).  Ten FLOPs instead of the generic log/exp pow, whose
// table constants also spilled registers of the persistent kernel.  x = 1 - cos(theta) is 0 or >= 2^-53, so
// nothing underflows.
template <class R>
__host__ __device__ __forceinline__ R pow5(R x) {
    const R p = x * x, pe = fma(x, x, -p);                  // x^2 = p + pe exactly
    const R q = p * p, qe = fma(p, p, -q) + (R(2) * p) * pe;  // x^4 = q + qe (pe^2 dropped: 2^-106 relative)
    const R r = q * x, re = fma(q, x, -r) + qe * x;         // x^5 = r + re
    return r + re;
}
// moving_sphere.h:72-74 center(time) = center0 + ((time - time0) / (time1 - time0)) * (center1 - center0)
// (time - time0) / (time1 - time0): x / 1 == x exactly, so the divide is skipped for the common unit shutter span
// (every moving sphere of the reference scenes) without changing a bit.
template <class R>
__device__ __forceinline__ R motion_fraction(R tm, R t0, R dt) {
    R x = tm - t0;
    if (dt != R(1)) {
        __asm__ volatile("" : "+v"(x));  // keeps the divide inside the branch (no if-conversion into a select)
        x = x / dt;
    }
    return x;
}
template <class R>
__device__ __forceinline__ V3<R> moving_center(V3<R> c0, V3<R> d, R t0, R dt, R tm) { return c0 + motion_fraction(tm, t0, dt) * d; }
template <class R>
__device__ __forceinline__ bool hit_sphere(const SphereRec<R>& s, const Ray<R>& r, R tmin, R tmax, R& t) {
    V3<R> center = ld3(s.c);
    if (s.flags & SPH_MOVING) center = moving_center(center, ld3(s.d), s.t0, s.dt, r.tm);
    return hit_sphere_at(center, s.r, r, tmin, tmax, t);
}

// triangle.h:22-88 (geometric test, unnormalised normal).
template <class R>
__device__ __forceinline__ bool hit_tri_v(V3<R> p1, V3<R> p2, V3<R> p3, const Ray<R>& r, R tmin, R tmax, R& t) {
    const V3<R> N = cross(p2 - p1, p3 - p1);
    const R ndd = dot(N, r.d);
    if (fabs(ndd) < R(DBL_EPSILON)) return false;
    const R dd = -dot(N, p1);
    const R tt = -(dot(N, r.o) + dd) / ndd;
    if (tt < tmin || tmax < tt) return false;
    const V3<R> p = r.o + tt * r.d;
    if (dot(N, cross(p2 - p1, p - p1)) < R(0)) return false;
    if (dot(N, cross(p3 - p2, p - p2)) < R(0)) return false;
    if (dot(N, cross(p1 - p3, p - p3)) < R(0)) return false;
    t = tt;
    return true;
}
// hit_tri_v with the plane (N, dd) precomputed on the host by the same operations (TriRec112)
template <class R>
__device__ __forceinline__ bool hit_tri_pre(V3<R> p1, V3<R> p2, V3<R> p3, V3<R> N, R dd, const Ray<R>& r, R tmin, R tmax, R& t) {
    const R ndd = dot(N, r.d);
    if (fabs(ndd) < R(DBL_EPSILON)) return false;
    const R tt = -(dot(N, r.o) + dd) / ndd;
    if (tt < tmin || tmax < tt) return false;
    const V3<R> p = r.o + tt * r.d;
    if (dot(N, cross(p2 - p1, p - p1)) < R(0)) return false;
    if (dot(N, cross(p3 - p2, p - p2)) < R(0)) return false;
    if (dot(N, cross(p1 - p3, p - p3)) < R(0)) return false;
    t = tt;
    return true;
}
template <class R>
__device__ __forceinline__ bool hit_tri(const TriRec<R>& tr, const Ray<R>& r, R tmin, R tmax, R& t) {
    return hit_tri_v(ld3(tr.p), ld3(tr.p + 3), ld3(tr.p + 6), r, tmin, tmax, t);
}

template <class R> __device__ __forceinline__ R comp(V3<R> v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// aarect.cpp:3-55.  axis 0: xy (k on z), 1: xz (k on y), 2: yz (k on x).
template <class R>
__device__ __forceinline__ bool hit_rect(int axis, R a0, R a1, R b0, R b1, R k, const Ray<R>& r, R tmin, R tmax, R& t) {
    const int ka = axis == 0 ? 2 : (axis == 1 ? 1 : 0);
    const int ia = axis == 2 ? 1 : 0;
    const int ib = axis == 0 ? 1 : 2;
    const R tt = (k - comp(r.o, ka)) / comp(r.d, ka);
    if (tt < tmin || tt > tmax) return false;
    const R x = comp(r.o, ia) + tt * comp(r.d, ia);
    const R y = comp(r.o, ib) + tt * comp(r.d, ib);
    if (x < a0 || x > a1 || y < b0 || y > b1) return false;
    t = tt;
    return true;
}

// box.cpp:3-19: face f of a box, in the reference's side order.
template <class R>
__device__ __forceinline__ void box_face(const BoxRec<R>& b, int f, int& axis, R& a0, R& a1, R& b0, R& b1, R& k) {
    const int pair = f >> 1;       // 0: xy, 1: xz, 2: yz
    const bool hi = (f & 1) == 0;  // even faces sit on p1
    axis = pair;
    if (pair == 0) { a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[1]; b1 = b.mx[1]; k = hi ? b.mx[2] : b.mn[2]; }
    else if (pair == 1) { a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[2]; b1 = b.mx[2]; k = hi ? b.mx[1] : b.mn[1]; }
    else { a0 = b.mn[1]; a1 = b.mx[1]; b0 = b.mn[2]; b1 = b.mx[2]; k = hi ? b.mx[0] : b.mn[0]; }
}
template <class R>
__device__ __forceinline__ bool hit_box(const BoxRec<R>& b, const Ray<R>& r, R tmin, R tmax, R& t, uint32_t& face) {
    bool any = false;  // hittable_list semantics over the six sides: closest wins, a later equal t replaces
    R closest = tmax;
    for (int f = 0; f < 6; ++f) {
        int axis;
        R a0, a1, b0, b1, k, tt;
        box_face(b, f, axis, a0, a1, b0, b1, k);
        const bool h = hit_rect(axis, a0, a1, b0, b1, k, r, tmin, closest, tt);
        if (h) {
            any = true;
            closest = tt;
            face = static_cast<uint32_t>(f);
        }
    }
    t = closest;
    return any;
}

// The test of a primitive given its record (a prim object's copy, DevScene::obj_prims): the same arithmetic as hit_prim.
template <class R, uint32_t F>
__device__ __forceinline__ bool hit_prim_rec(uint32_t type, const PrimRec80& rec, const Ray<R>& r, R tmin, R tmax, R& t, uint32_t& face) {
    if ((F & F_SPHERE) && (fbase(F) == F_SPHERE || type == PRIM_SPHERE)) return hit_sphere(reinterpret_cast<const SphereRec<R>&>(rec), r, tmin, tmax, t);
    if ((F & F_TRI) && (fbase(F) == F_TRI || type == PRIM_TRIANGLE)) return hit_tri(reinterpret_cast<const TriRec<R>&>(rec), r, tmin, tmax, t);
    if ((F & F_RECT) && type == PRIM_RECT) {
        const RectRec<R>& q = reinterpret_cast<const RectRec<R>&>(rec);
        return hit_rect(static_cast<int>(q.axis), q.a0, q.a1, q.b0, q.b1, q.k, r, tmin, tmax, t);
    }
    if ((F & F_BOX) && type == PRIM_BOX) return hit_box(reinterpret_cast<const BoxRec<R>&>(rec), r, tmin, tmax, t, face);
    return false;
}
// F (layout.h Feature bits) prunes the primitive kinds a scene cannot contain, so a kernel instantiated for a
// spheres-only scene carries no triangle/box/transform/medium code and needs far fewer registers.
template <class R, uint32_t F>
__device__ __forceinline__ bool hit_prim(const DevScene<R>& S, uint32_t ref, const Ray<R>& r, R tmin, R tmax, R& t, uint32_t& face) {
    const uint32_t idx = primref_index(ref);
    const uint32_t type = primref_type(ref);
    if ((F & F_SPHERE) && (fbase(F) == F_SPHERE || type == PRIM_SPHERE)) return hit_sphere(S.spheres[idx], r, tmin, tmax, t);
    if ((F & F_TRI) && (fbase(F) == F_TRI || type == PRIM_TRIANGLE)) return hit_tri(S.tris[idx], r, tmin, tmax, t);
    if ((F & F_RECT) && type == PRIM_RECT) {
        const RectRec<R>& q = S.rects[idx];
        return hit_rect(static_cast<int>(q.axis), q.a0, q.a1, q.b0, q.b1, q.k, r, tmin, tmax, t);
    }
    if ((F & F_BOX) && type == PRIM_BOX) return hit_box(S.boxes[idx], r, tmin, tmax, t, face);
    return false;
}

// ------------------------------------------------------------------------------------------------ BVH traversal
// While-while traversal of the 4-wide f32 node array with a per-lane stack in LDS (stk[k * B] is entry k of this
// lane; the stack is a dynamic LDS array of the scene's worst-case depth + 2 rows: stk[-B] is a kNodeEmpty sentinel and
// the last row takes the discarded write of a branchless push).  Each node visit tests its four child
// boxes at once, goes to the nearest hit child and pushes the other hit children far-to-near.  Box tests are f32 and
// conservative (boxes padded at build time, interval widened here); leaves run the exact R tests and shrink tmax, so
// the closest hit equals the reference's bvh_node::hit (bvh.cpp:44-52) up to exact-t ties.
constexpr int kBlock = 256;

__device__ __forceinline__ float f_lo(double t) { return t == -__builtin_inf() ? -__builtin_inff() : static_cast<float>(t) * (1.0f - 2e-6f) - 1e-30f; }
__device__ __forceinline__ float f_lo(float t) { return t * (1.0f - 2e-6f) - 1e-30f; }
__device__ __forceinline__ float f_hi(double t) { return t == __builtin_inf() ? __builtin_inff() : static_cast<float>(t) * (1.0f + 2e-6f) + 1e-30f; }
__device__ __forceinline__ float f_hi(float t) { return t * (1.0f + 2e-6f) + 1e-30f; }

// Slab entry distances of the four child boxes of a node, +inf when a box is missed (or the slot is empty).  The plane
// distances are single-rounding FMAs fma(plane, 1/d, -o/d), two children per v_pk_fma_f32; one rounding is no worse
// than the mul+sub the box padding was sized for, so the test stays conservative.
typedef float f2v __attribute__((ext_vector_type(2)));
// The HBM-scene traversal loads each axis' near and far planes by the direction's sign (as the LDS
// variant does), so a child's entry is max(x0, y0, z0, tmin) and its exit min(x1, y1, z1, tmax) without the per-axis
// min/max.  For 1/d > 0, t(lo) <= t(hi) (the FMA rounding is monotone in the plane), so the selected planes give
// exactly the values the min/max picked (and an empty slot's +-FLT_MAX box stays missed): same keys, 24 fewer VALU per
// node visit.  Measured (r3c): cow +3.6 %, Next-Week final +5.6 %, dino 4096^2 +3.9 %.
__device__ __forceinline__ float slab_key_nf(float x0, float x1, float y0, float y1, float z0, float z1, float tminf, float tmaxf) {
    const float lo = fmaxf(fmaxf(x0, y0), fmaxf(z0, tminf));
    const float hi = fminf(fminf(x1, y1), fminf(z1, tmaxf));
    return lo <= hi ? lo : __builtin_inff();
}
// x0/y0/z0 (lx, ly, lz): near planes, x1/y1/z1 (hx, hy, hz): far planes
__device__ __forceinline__ void slab4_nf(const float4& lx, const float4& hx, const float4& ly, const float4& hy, const float4& lz, const float4& hz,
                                        float ix, float iy, float iz, float oix, float oiy, float oiz, float tminf, float tmaxf, float& k0,
                                        float& k1, float& k2, float& k3) {
    const f2v vx = {ix, ix}, vy = {iy, iy}, vz = {iz, iz};
    const f2v nx = {-oix, -oix}, ny = {-oiy, -oiy}, nz = {-oiz, -oiz};
    const f2v x0a = __builtin_elementwise_fma(f2v{lx.x, lx.y}, vx, nx), x0b = __builtin_elementwise_fma(f2v{lx.z, lx.w}, vx, nx);
    const f2v x1a = __builtin_elementwise_fma(f2v{hx.x, hx.y}, vx, nx), x1b = __builtin_elementwise_fma(f2v{hx.z, hx.w}, vx, nx);
    const f2v y0a = __builtin_elementwise_fma(f2v{ly.x, ly.y}, vy, ny), y0b = __builtin_elementwise_fma(f2v{ly.z, ly.w}, vy, ny);
    const f2v y1a = __builtin_elementwise_fma(f2v{hy.x, hy.y}, vy, ny), y1b = __builtin_elementwise_fma(f2v{hy.z, hy.w}, vy, ny);
    const f2v z0a = __builtin_elementwise_fma(f2v{lz.x, lz.y}, vz, nz), z0b = __builtin_elementwise_fma(f2v{lz.z, lz.w}, vz, nz);
    const f2v z1a = __builtin_elementwise_fma(f2v{hz.x, hz.y}, vz, nz), z1b = __builtin_elementwise_fma(f2v{hz.z, hz.w}, vz, nz);
    k0 = slab_key_nf(x0a.x, x1a.x, y0a.x, y1a.x, z0a.x, z1a.x, tminf, tmaxf);
    k1 = slab_key_nf(x0a.y, x1a.y, y0a.y, y1a.y, z0a.y, z1a.y, tminf, tmaxf);
    k2 = slab_key_nf(x0b.x, x1b.x, y0b.x, y1b.x, z0b.x, z1b.x, tminf, tmaxf);
    k3 = slab_key_nf(x0b.y, x1b.y, y0b.y, y1b.y, z0b.y, z1b.y, tminf, tmaxf);
}
// Packed keys of the LDS variant: the entry distance's f32 bits with the low 16 bits replaced by the 16-bit child
// code.  Entry distances are >= tminf > 0 there (world rays start at t = 0.001; the LDS variant has no media, whose
// boundary tests start at -inf), so unsigned order is distance order to 2^-7 relative -- it only orders the pushes;
// misses get kKeyMiss, above every finite key.
constexpr uint32_t kKeyMiss = 0x7F800000u;
// x0/y0/z0: entry distances at the near planes, x1/y1/z1: exit distances at the far planes (planes picked by the
// direction's sign, so no per-axis min/max; a NaN plane distance (0 * inf) drops out of max/min as before).
template <bool HI = false>
__device__ __forceinline__ uint32_t slab_key_packed(float x0, float x1, float y0, float y1, float z0, float z1, int32_t child, float tminf,
                                                    float tmaxf) {
    const float lo = fmaxf(fmaxf(x0, y0), fmaxf(z0, tminf));
    // min(z1, tmaxf) as the bare instruction: fminf would re-quiet tmaxf (a loop-carried arithmetic result, never a
    // signalling NaN) on every node visit; a NaN z1 (0 * inf plane distance) still drops out (IEEE-mode v_min)
    float zt;
    __asm__("v_min_f32 %0, %1, %2" : "=v"(zt) : "v"(z1), "v"(tmaxf));
    const float hi = fminf(fminf(x1, y1), zt);
    // HI: the code is the high half of `child` (layout.h: child codes as int16): bytes 3, 2 of lo over bytes 3, 2 of child, one v_perm
    const uint32_t key = HI ? __builtin_amdgcn_perm(__float_as_uint(lo), static_cast<uint32_t>(child), 0x07060302u)
                            : (__float_as_uint(lo) & 0xFFFF0000u) | (static_cast<uint32_t>(child) & 0xFFFFu);
    return lo <= hi ? key : kKeyMiss;  // empty slots carry a box no ray enters (layout.h kLdsEmptyChild)
}
__device__ __forceinline__ void slab4_packed(const float4& lx, const float4& hx, const float4& ly, const float4& hy, const float4& lz,
                                             const float4& hz, const int4& ch, float ix, float iy, float iz, float oix, float oiy, float oiz,
                                             float tminf, float tmaxf, uint32_t& q0, uint32_t& q1, uint32_t& q2, uint32_t& q3) {
    const f2v vx = {ix, ix}, vy = {iy, iy}, vz = {iz, iz};
    const f2v nx = {-oix, -oix}, ny = {-oiy, -oiy}, nz = {-oiz, -oiz};
    const f2v x0a = __builtin_elementwise_fma(f2v{lx.x, lx.y}, vx, nx), x0b = __builtin_elementwise_fma(f2v{lx.z, lx.w}, vx, nx);
    const f2v x1a = __builtin_elementwise_fma(f2v{hx.x, hx.y}, vx, nx), x1b = __builtin_elementwise_fma(f2v{hx.z, hx.w}, vx, nx);
    const f2v y0a = __builtin_elementwise_fma(f2v{ly.x, ly.y}, vy, ny), y0b = __builtin_elementwise_fma(f2v{ly.z, ly.w}, vy, ny);
    const f2v y1a = __builtin_elementwise_fma(f2v{hy.x, hy.y}, vy, ny), y1b = __builtin_elementwise_fma(f2v{hy.z, hy.w}, vy, ny);
    const f2v z0a = __builtin_elementwise_fma(f2v{lz.x, lz.y}, vz, nz), z0b = __builtin_elementwise_fma(f2v{lz.z, lz.w}, vz, nz);
    const f2v z1a = __builtin_elementwise_fma(f2v{hz.x, hz.y}, vz, nz), z1b = __builtin_elementwise_fma(f2v{hz.z, hz.w}, vz, nz);
    q0 = slab_key_packed(x0a.x, x1a.x, y0a.x, y1a.x, z0a.x, z1a.x, ch.x, tminf, tmaxf);
    q1 = slab_key_packed<true>(x0a.y, x1a.y, y0a.y, y1a.y, z0a.y, z1a.y, ch.y, tminf, tmaxf);
    q2 = slab_key_packed(x0b.x, x1b.x, y0b.x, y1b.x, z0b.x, z1b.x, ch.z, tminf, tmaxf);
    q3 = slab_key_packed<true>(x0b.y, x1b.y, y0b.y, y1b.y, z0b.y, z1b.y, ch.w, tminf, tmaxf);
}
// The HBM-scene traversal's packed keys (PK): near/far planes as slab4_nf, keys as slab_key_packed (the 16-bit codes of
// children 1 and 3 in the high halves of ch.y / ch.w, as the LDS image's)
__device__ __forceinline__ void slab4_packed_nf(const float4& lx, const float4& hx, const float4& ly, const float4& hy, const float4& lz,
                                                const float4& hz, const int4& ch, float ix, float iy, float iz, float oix, float oiy, float oiz,
                                                float tminf, float tmaxf, uint32_t& q0, uint32_t& q1, uint32_t& q2, uint32_t& q3) {
    const f2v vx = {ix, ix}, vy = {iy, iy}, vz = {iz, iz};
    const f2v nx = {-oix, -oix}, ny = {-oiy, -oiy}, nz = {-oiz, -oiz};
    const f2v x0a = __builtin_elementwise_fma(f2v{lx.x, lx.y}, vx, nx), x0b = __builtin_elementwise_fma(f2v{lx.z, lx.w}, vx, nx);
    const f2v x1a = __builtin_elementwise_fma(f2v{hx.x, hx.y}, vx, nx), x1b = __builtin_elementwise_fma(f2v{hx.z, hx.w}, vx, nx);
    const f2v y0a = __builtin_elementwise_fma(f2v{ly.x, ly.y}, vy, ny), y0b = __builtin_elementwise_fma(f2v{ly.z, ly.w}, vy, ny);
    const f2v y1a = __builtin_elementwise_fma(f2v{hy.x, hy.y}, vy, ny), y1b = __builtin_elementwise_fma(f2v{hy.z, hy.w}, vy, ny);
    const f2v z0a = __builtin_elementwise_fma(f2v{lz.x, lz.y}, vz, nz), z0b = __builtin_elementwise_fma(f2v{lz.z, lz.w}, vz, nz);
    const f2v z1a = __builtin_elementwise_fma(f2v{hz.x, hz.y}, vz, nz), z1b = __builtin_elementwise_fma(f2v{hz.z, hz.w}, vz, nz);
    q0 = slab_key_packed(x0a.x, x1a.x, y0a.x, y1a.x, z0a.x, z1a.x, ch.x, tminf, tmaxf);
    q1 = slab_key_packed<true>(x0a.y, x1a.y, y0a.y, y1a.y, z0a.y, z1a.y, ch.y, tminf, tmaxf);
    q2 = slab_key_packed(x0b.x, x1b.x, y0b.x, y1b.x, z0b.x, z1b.x, ch.z, tminf, tmaxf);
    q3 = slab_key_packed<true>(x0b.y, x1b.y, y0b.y, y1b.y, z0b.y, z1b.y, ch.w, tminf, tmaxf);
}
__device__ __forceinline__ void ucas(uint32_t& a, uint32_t& b) {
    const uint32_t lo = a < b ? a : b;
    b = a < b ? b : a;
    a = lo;
}
__device__ __forceinline__ void cas(float& ka, int32_t& ca, float& kb, int32_t& cb) {
    const bool s = kb < ka;
    const float k = s ? kb : ka;
    const int32_t c = s ? cb : ca;
    kb = s ? ka : kb;
    cb = s ? ca : cb;
    ka = k;
    ca = c;
}

#ifndef ART_LDS_LEAF_NOREF
#define ART_LDS_LEAF_NOREF 0  // 1 (k_paths object, Makefile PATHS_NOREF): the leaf test skips the per-slot code
#endif

// Leaf slot test of the LDS scene image (layout.h): the same root selection as hit_sphere on the same f64 values.
// d_a = |d|^2 and d_inv_a = 1 / d_a come from the traversal (once per ray).  The image sits at LDS address 0, so
// every read takes an integer LDS byte address (one shift-add, the plane offset folded in).  Moving spheres of the
// image span the unit shutter (lds_scene_image checks it): moving_sphere.h:72-74's fraction (tm - 0) / 1 is tm.
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 lds_d2(uint32_t addr) {
    const d2v v = *(__attribute__((address_space(3))) const d2v*)(size_t)addr;
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ double lds_d1(uint32_t addr) { return *(__attribute__((address_space(3))) const double*)(size_t)addr; }
__device__ __forceinline__ uint32_t lds_u1(uint32_t addr) { return *(__attribute__((address_space(3))) const uint32_t*)(size_t)addr; }
__device__ __forceinline__ bool hit_lds_slot(const uint8_t* lds, uint32_t slot, const Ray<double>& r, double d_a, double d_inv_a,
                                             double tmin, double tmax, double& t, uint32_t& prim, uint32_t& mt) {
    const double2 a = lds_d2(kLdsOffSph + slot * 16u), b = lds_d2(kLdsOffSph + (kLdsSlotCap + slot) * 16u);
#if ART_LDS_LEAF_NOREF
    // k_paths (its own object, kernels_paths.o): the hit is shaded by slot, and its material type is read once after
    // the trace, so the leaf test skips the per-slot code
    prim = 0;
    mt = kMatUnknown;
#else
    const uint32_t code = lds_u1(kLdsOffRef + slot * 4u);
#endif
    V3<double> center{a.x, a.y, b.x};
    // y motion only (lds_scene_image): c + tm * (+-0, dy, +-0) leaves x and z as they are; static slots hold dy = -0
    center.y = center.y + r.tm * lds_d1(kLdsOffMov + slot * 8u);
#if !ART_LDS_LEAF_NOREF
    prim = make_primref(PRIM_SPHERE, code & kLdsRefIndexMask);
    mt = code >> kLdsRefMatShift;
#endif
    return sphere_root<double, true>(center, b.y, r, d_a, d_inv_a, tmin, tmax, t);
}

#ifdef ART_STATS
// Divergence statistics (diagnostic builds only): [0] node-loop wave iterations, [1] node visits (lane sum), [2] leaf-
// loop wave iterations, [3] leaf tests (lane sum), [4] outer-loop wave iterations, [5] outer iterations (lane sum),
// [6] traversals, [7] hit_sphere tests with disc >= 0; [32..45] k_paths_g's surface branches (wave iterations, lanes):
// sphere u,v, transform unwinds, medium hits, box/rect record reloads, spheres, box/rect from the carried material,
// world_surface calls; [46] leaf phases (wave), [47] the wave iterations a wave-cooperative leaf test would need
// (sum over leaf phases of ceil(the phase's leaf tests / the lanes still traversing)).
constexpr int kArtStats = 48;
__device__ unsigned long long g_art_stats[kArtStats];
__device__ __forceinline__ void stat_wave(int k) {
    const uint64_t m = __ballot(true);
    if (static_cast<int>(__lane_id()) == __ffsll(static_cast<long long>(m)) - 1) atomicAdd(&g_art_stats[k], 1ull);
}
__device__ __forceinline__ void stat_lane(int k) { atomicAdd(&g_art_stats[k], 1ull); }
#define ART_STAT_WAVE(k) stat_wave(k)
#define ART_STAT_LANE(k) stat_lane(k)
#else
#define ART_STAT_WAVE(k)
#define ART_STAT_LANE(k)
#endif


// The LDS scene image lives at LDS address 0 (k_extend and k_paths allocate LDS dynamically only), so node fetches
// take a plain 32-bit LDS byte address: no base add per load.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_f4(uint32_t addr) {
    const f4v v = *(__attribute__((address_space(3))) const f4v*)(size_t)addr;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 lds_u2(uint32_t addr) {
    typedef unsigned u2v_t __attribute__((ext_vector_type(2)));
    const u2v_t v = *(__attribute__((address_space(3))) const u2v_t*)(size_t)addr;
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ int4 lds_i4(uint32_t addr) {
    const i4v v = *(__attribute__((address_space(3))) const i4v*)(size_t)addr;
    return make_int4(v.x, v.y, v.z, v.w);
}
// Per-lane traversal stack: entry k of a lane is stk[k * B]; stk[-B] holds the kNodeEmpty sentinel, so peek() on an
// empty stack returns kNodeEmpty, and the row above the top takes the discarded write of a branchless push.
template <int B, bool L> struct LaneStack;
template <int B>
struct LaneStack<B, true> {  // LDS-scene variant: 16-bit entries, tracked as the LDS byte address of the top row
    static constexpr uint32_t kRow = 2u * B;
    uint32_t bottom, top;
    __device__ __forceinline__ explicit LaneStack(int16_t* stk)
        : bottom(static_cast<uint32_t>(reinterpret_cast<size_t>((__attribute__((address_space(3))) int16_t*)stk)) - kRow), top(bottom) {}
    __device__ __forceinline__ void push(int32_t v, bool keep) {
        *(__attribute__((address_space(3))) int16_t*)(size_t)(top + kRow) = static_cast<int16_t>(v);
        top += keep ? kRow : 0u;
    }
    __device__ __forceinline__ int32_t peek() const { return *(__attribute__((address_space(3))) const int16_t*)(size_t)top; }
    // the entry under the top (garbage, never used, when the stack holds fewer than one entry: the row below the
    // sentinel is still inside LDS, at the end of the scene image)
    __device__ __forceinline__ int32_t peek_below() const { return *(__attribute__((address_space(3))) const int16_t*)(size_t)(top - kRow); }
    // No empty-stack guard: popping the empty stack yields the sentinel row's kNodeEmpty and leaves top one row below
    // it, but a walk whose node is kNodeEmpty ends without another peek or pop (traverse), so that row is never read;
    // the next walk starts from a fresh LaneStack.
    __device__ __forceinline__ void pop_if(bool c) { top -= c ? kRow : 0u; }
    __device__ __forceinline__ uint32_t save() const { return top; }
    __device__ __forceinline__ void restore(uint32_t t) { top = t; }
};
template <int B>
struct LaneStack<B, false> {  // 32-bit entries; `top` is the LDS byte address of the top entry (the sentinel when empty)
    static constexpr uint32_t kRow = 4u * B;
    uint32_t bottom, top;
    __device__ __forceinline__ explicit LaneStack(int32_t* stk)
        : bottom(static_cast<uint32_t>(reinterpret_cast<size_t>((__attribute__((address_space(3))) int32_t*)stk)) - kRow), top(bottom) {}
    __device__ __forceinline__ void push(int32_t v, bool keep) {
        *(__attribute__((address_space(3))) int32_t*)(size_t)(top + kRow) = v;
        top += keep ? kRow : 0u;
    }
    __device__ __forceinline__ int32_t peek() const { return *(__attribute__((address_space(3))) const int32_t*)(size_t)top; }
    // no empty-stack guard: a walk that pops the sentinel's kNodeEmpty ends without reading on
    __device__ __forceinline__ void pop_if(bool c) { top -= c ? kRow : 0u; }
    // the resumable traversal (TravResume) keeps the top address: the stack stays in this lane's LDS column
    __device__ __forceinline__ uint32_t save() const { return top; }
    __device__ __forceinline__ void restore(uint32_t t) { top = t; }
};
// Traversal stack entry: node/leaf codes, 16 bits in the LDS-scene variant (layout.h lds_leaf), 32 bits otherwise.
template <bool L> using StackT = typename std::conditional<L, int16_t, int32_t>::type;
// k_paths_g instantiations with F_CODE16 keep 16-bit entries as well (the LDS variant's LaneStack and stack columns)
template <bool L, uint32_t F> using StackF = StackT<L || (F & F_CODE16) != 0>;
// Column of lane t in a stack row.  16-bit entries pack two lanes per dword; a row holds a wave's 64 entries in 32
// dwords.  Unswizzled, lanes 2i and 2i+1 share dword i, so a wave64 LDS access (serviced as lanes 0-31, then 32-63)
// puts two lanes on one bank whenever their stack depths differ (a 2-way conflict on most pushes and pops of a
// divergent traversal).  Swizzled, lane t sits in dword t & 31, half t >> 5: lanes 0-31 take 32 distinct dwords, and
// so do lanes 32-63, in every row (rows are 2 KiB = 512 dwords apart, a multiple of the 64 banks).
template <bool L>
__device__ __forceinline__ uint32_t stack_column(uint32_t t) {
    if (!L) return t;
    return (t & ~63u) | ((t & 31u) << 1) | ((t >> 5) & 1u);
}

// f32 direction component for the slab reciprocals: magnitude at least 2^-64, sign of d (-0 stays negative).
__device__ __forceinline__ float f32_dir(double d) {
    const float f = static_cast<float>(d);
    return __builtin_copysignf(fmaxf(__builtin_fabsf(f), 0x1p-64f), f);
}
// Suspendable traversal (k_paths_g, ART_SUSPEND_LANES): a world-level BVH traversal may stop at a phase boundary when
// fewer than ART_SUSPEND_LANES lanes of the wave are still traversing, keeping its node, parked leaf and stack depth
// (the stack stays in LDS) so the wave can shade and restart the lanes that finished and resume it next round with
// them: the lane runs the same sequence of node visits and leaf tests, only spread over rounds.
#ifndef ART_SUSPEND_LANES
#define ART_SUSPEND_LANES 24  // measured over 8-40 on cow and the capsule (24: +8 %; 8: +4 %; 40: +7 %)
#endif
struct TravResume {
    int32_t node, parked;
    uint32_t sp;  // LaneStack::save(): the top entry's LDS address
    int32_t lanes;  // suspend when fewer lanes of the wave are traversing
    bool fresh;     // no traversal in progress: start at the root
    bool allow;     // wave-uniform: suspending is allowed in this round (paths remain to be started)
    bool suspended;
};
// B: lanes per block (LDS stack stride).  L: nodes and leaf spheres come from the LDS scene image at `lds`.
// RES: resumable (rs non-null), HBM-scene variant only.
template <class R, uint32_t F, int B, bool L, int PL = 0, bool RES = false>
__device__ __forceinline__ bool traverse(const DevScene<R>& S, const uint8_t* lds, int32_t root, const Ray<R>& r, R tmin, R tmax,
                                         StackF<L, F>* stk, R& t, uint32_t& prim, uint32_t& face, uint32_t& mt, TravResume* rs = nullptr,
                                         int32_t hoisted = kNodeEmpty) {
    static_assert(!(L && (F & F_MEDIA)), "packed LDS keys need tmin > 0: no medium boundary tests in the LDS variant");
    static_assert(!RES || !L, "resumable traversal: HBM-scene variant only");
    const float ox = static_cast<float>(r.o.x), oy = static_cast<float>(r.o.y), oz = static_cast<float>(r.o.z);
    // hardware reciprocal (1 ulp): the box test is conservative by its 2e-6 relative padding, far above that
    // A direction component that is 0 (or tiny) would give 1/d = inf, and the plane distances fma(plane, 1/d, -o/d)
    // would mix +-inf and NaN (inf - inf): a ray parallel to an axis then missed boxes that hold it (tests/
    // test_gpu_rays.py).  The component is raised to +-2^-64 with its sign, so 1/d, o/d and plane/d stay finite for
    // any coordinate below 1e19 and the slab of a parallel ray holds its origin for t in (-huge, +huge) or for none.
    const float ix = __builtin_amdgcn_rcpf(f32_dir(r.d.x)), iy = __builtin_amdgcn_rcpf(f32_dir(r.d.y)), iz = __builtin_amdgcn_rcpf(f32_dir(r.d.z));
    const float oix = ox * ix, oiy = oy * iy, oiz = oz * iz;
    // LDS variant: the near and far plane of each axis follow from the direction's sign, so the slab test reads them
    // directly (near plane offset per axis; the far plane is always the plane above it, one kLdsPlane away -- an
    // immediate DS offset -- since each axis stores lo, hi, lo) and needs no per-axis min/max
    constexpr uint32_t kLdsPlane = kLdsNodeCap * 16;
    static_assert(kLdsPlane % 256 == 0, "every node plane starts on bank 0");
    const uint32_t off_nx = kLdsOffNodes + (0u + (__float_as_uint(ix) >> 31)) * kLdsPlane;
    const uint32_t off_ny = kLdsOffNodes + (3u + (__float_as_uint(iy) >> 31)) * kLdsPlane;
    const uint32_t off_nz = kLdsOffNodes + (6u + (__float_as_uint(iz) >> 31)) * kLdsPlane;
    const float tminf = f_lo(tmin);
    float tmaxf = f_hi(tmax);
    // L: |d|^2 and its reciprocal for the leaf root divisions (div_rcp).  A traced direction is never zero (camera
    // rays point at the focus plane, scatter directions pass near_zero / dot(d, n) > 0) and its components are 0 or
    // differences of scene-scale doubles, so |d|^2 lies far inside div_rcp's range (> 2^-500, < 2^16).
    // The same for the HBM-scene traversal of triangle-free kernels (leaf spheres: the Next-Week final's
    // cluster, the Cornell and two-sphere scenes); their directions are camera rays and scatter directions too
    constexpr bool kSphPre = !L && (F & F_SPHERE) != 0 && (F & F_TRI) == 0;
    // kSphLazy: the spheres-only kernels (two-sphere, perlin, earth scenes: a few spheres per traversal) take the
    // reciprocal at the traversal's first root division instead of at its start (sphere_root_lazy; measured r4u:
    // two perlin spheres +3.5 %, earth +0.6 %; the Next-Week final's kernel, 1000 leaf spheres, keeps the eager one:
    // lazy -0.4 %)
    constexpr bool kSphLazy = kSphPre && (F & (F_BOX | F_RECT | F_XFORM | F_MEDIA)) == 0;
    const R d_a = (L || kSphPre) ? len2(r.d) : R(0);
    R d_inv_a = (L || (kSphPre && !kSphLazy)) ? R(1) / d_a : R(0);
    bool hit = false;
    // PK (k_paths_g instantiations with F_CODE16): the HBM-scene traversal sorts packed keys as the LDS variant does,
    // with the node's 16-bit child codes (BvhNode::pad, layout.h make_leaf16) in the low half of each key; codes,
    // stack entries (16-bit, the LDS variant's LaneStack) and leaves are then in the 16-bit form throughout the walk
    constexpr bool PK = !L && (F & F_CODE16) != 0;
    // F_LEAF2: a 16-bit leaf code's first slot is in units of two (layout.h; every leaf on an even slot)
    constexpr uint32_t kLeafShift = (PK && (F & F_LEAF2) != 0) ? 1u : 0u;
    static_assert(!PK || (F & F_MEDIA_G) == 0, "packed keys need tmin > 0: no medium boundary traversals");
    LaneStack<B, L || PK> st(stk);
    // kNfHoist: the near-plane offsets computed once per traversal in kernels with every node in LDS (PL 2), instead
    // of 6 VALU per node visit: without instance transforms (dino's LM 1 kernel), and with them where the kernel has
    // no triangles or medium-boundary traversals (the Next-Week final's: +0.8 %, r4y_ab_nf_hoist.txt; in the F_ALL
    // kernels it spilled)
    constexpr bool kNfHoist = !L && PL == 2 && ((F & F_XFORM) == 0 || (F & (F_TRI | F_MEDIA_G)) == 0);
    [[maybe_unused]] const uint32_t nf_hx = (__float_as_uint(ix) >> 31) << 4, nf_hy = (__float_as_uint(iy) >> 31) << 4,
                                    nf_hz = (__float_as_uint(iz) >> 31) << 4;
    // L: inner nodes are coded by their byte offset in a node plane (index * 16, layout.h), so a visit's plane
    // addresses are one add each
    static_assert(kLdsNodeCap * 16 <= 32767, "LDS inner-node codes are 16-bit stack entries");
    const int32_t root_code = L ? root * 16 : root;
    int32_t node = root_code;
#ifdef ART_STATS
    // diagnostic mirror of the LDS variant's stack with each entry's box entry distance: counts stale visits (a
    // popped node whose box is entered beyond the current tmax)
    float dstk[kMaxStackDepth + 2];
    int dsp = 0;
    float cur_d = 0.0f;
#define ART_DPUSH(q, keep) do { if (L) { dstk[dsp] = __uint_as_float(static_cast<uint32_t>(q) & 0xFFFF0000u); dsp += (keep) ? 1 : 0; } } while (0)
#define ART_DPOP(c) do { if (L && (c)) { cur_d = dsp > 0 ? dstk[dsp - 1] : 0.0f; dsp -= dsp > 0 ? 1 : 0; } } while (0)
#else
#define ART_DPUSH(q, keep) do { } while (0)
#define ART_DPOP(c) do { } while (0)
#endif
    // Speculative while-while (Aila & Laine 2009): a lane that reaches a leaf parks it and keeps walking inner nodes
    // until every lane of the wave holds a leaf, so the node loop runs with more lanes active; parked leaves are then
    // tested together.  Nodes visited past a parked leaf used the older (larger) tmax: extra visits, same closest hit.
    int32_t parked = kNodeEmpty;
    // hoisted (wave-uniform: the BVH object's leaf of hoisted primitives, ObjRec::b): every lane tests it in the first
    // leaf phase, at once and before any node visit, so the tree walk starts with its closest hit as tmax.  Speculative
    // walk: it is the parked leaf and the first node loop is skipped (a wave-uniform flag; pushing the root under it
    // instead measured 10 more VGPR spills in k_paths); otherwise the walk starts at it with the root pushed under it
    // (popped before any other push: no extra stack depth).
    [[maybe_unused]] bool skip_nodes = false;
    if (hoisted != kNodeEmpty && (!RES || rs->fresh)) {
        const int32_t h = L ? lds_leaf(leaf_first(hoisted), leaf_count(hoisted)) : PK ? make_leaf16(leaf_first(hoisted) >> kLeafShift, leaf_count(hoisted)) : hoisted;
        parked = h;
        skip_nodes = true;
    }
    if constexpr (RES) {
        if (!rs->fresh) {
            node = rs->node;
            parked = rs->parked;
            st.restore(rs->sp);
        }
    }
    [[maybe_unused]] bool progressed = false;
    ART_STAT_LANE(6);
    for (;;) {
        if constexpr (RES) {
            if (rs->allow && progressed && __popcll(__ballot(true)) < rs->lanes) {
                rs->node = node;
                rs->parked = parked;
                rs->sp = st.save();
                rs->fresh = false;
                rs->suspended = true;
                return hit;
            }
            progressed = true;
        }
        ART_STAT_WAVE(4);
        ART_STAT_LANE(5);
        while (node >= 0 && !skip_nodes) {
            ART_STAT_WAVE(0);
            ART_STAT_LANE(1);
#ifdef ART_STATS
            if (L && cur_d > tmaxf) ART_STAT_LANE(14);
#endif
            float4 lx, hx, ly, hy, lz, hz;  // L: near (lx, ly, lz) and far (hx, hy, hz) planes
            int4 ch;
            if constexpr (L) {
                const uint32_t n16 = static_cast<uint32_t>(node);  // index * 16
                const uint32_t ax = n16 + off_nx, ay = n16 + off_ny, az = n16 + off_nz;
                lx = lds_f4(ax);
                hx = lds_f4(ax + kLdsPlane);
                ly = lds_f4(ay);
                hy = lds_f4(ay + kLdsPlane);
                lz = lds_f4(az);
                hz = lds_f4(az + kLdsPlane);
                {  // four 16-bit child codes in 8 bytes (layout.h): a ds_read_b64 instead of a ds_read_b128; codes 1
                   // and 3 stay in the high halves (slab4_packed builds their keys with one byte permute)
                    typedef unsigned u2v __attribute__((ext_vector_type(2)));
                    const u2v cw = *(__attribute__((address_space(3))) const u2v*)(size_t)(kLdsOffNodes + kLdsNodePlaneChild * kLdsPlane + n16);
                    ch = make_int4(static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.y), static_cast<int32_t>(cw.y));
                }
            }
            // !L: each axis' near plane in a BvhNode is at sign(1/d) * 16 from that axis' lo plane (lo x / y / z at 0 / 32 /
            // 64, its hi plane 16 above) and the far plane is the other one (near ^ 16): the same keys as per-axis min/max
            // (the FMA rounding is monotone in the plane; an empty slot's inverted +-FLT_MAX box stays missed), 24 fewer
            // VALU per node visit.  Recomputed per visit from 1/d (live anyway; the empty asm keeps the compiler from
            // hoisting three more loop-carried VGPRs) unless kNfHoist
            [[maybe_unused]] uint32_t nfx = 0, nfy = 0, nfz = 0;
            if constexpr (!L) {
                if (kNfHoist) {  // the per-ray offsets, loop-invariant (3 VGPRs live over the walk)
                    nfx = nf_hx;
                    nfy = nf_hy;
                    nfz = nf_hz;
                } else {
                    uint32_t sx, sy, sz;  // sign bits of 1/d, extracted in the loop (volatile: not hoisted)
                    __asm__ volatile("v_lshrrev_b32 %0, 31, %1" : "=v"(sx) : "v"(ix));
                    __asm__ volatile("v_lshrrev_b32 %0, 31, %1" : "=v"(sy) : "v"(iy));
                    __asm__ volatile("v_lshrrev_b32 %0, 31, %1" : "=v"(sz) : "v"(iz));
                    nfx = sx << 4;
                    nfy = sy << 4;
                    nfz = sz << 4;
                }
            }
            if constexpr (L) {
            } else if (PL == 2 || (PL == 1 && static_cast<uint32_t>(node) < S.n_lds_nodes)) {  // PL 2: every node in LDS
                // the top levels, copied into LDS: explicit LDS loads (a generic pointer here would be merged with
                // the global branch's into flat loads)
                const uint32_t a = S.nodes_lds + static_cast<uint32_t>(node) * static_cast<uint32_t>(sizeof(BvhNode));
                {
                    // node addresses are multiples of 32 (the LDS node array is 128-aligned): near plane = a + sign * 16,
                    // far plane = near ^ 16, and the y / z planes' +32 / +64 ride in the loads' immediate offsets
                    const uint32_t nx = a + nfx, ny = a + nfy, nz = a + nfz;
                    lx = lds_f4(nx); hx = lds_f4(nx ^ 16u); ly = lds_f4(ny + 32u); hy = lds_f4((ny ^ 16u) + 32u);
                    lz = lds_f4(nz + 64u); hz = lds_f4((nz ^ 16u) + 64u);
                }
                if constexpr (PK) {  // the four 16-bit codes (BvhNode::pad), codes 1 and 3 in the high halves
                    const uint2 cw = lds_u2(a + 112u);
                    ch = make_int4(static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.y), static_cast<int32_t>(cw.y));
                } else {
                    ch = lds_i4(a + 96);
                }
            } else {
                const float4* np = reinterpret_cast<const float4*>(S.nodes + node);
                {  // 32-bit offsets from the node array's base, as above
                    const char* nb = reinterpret_cast<const char*>(S.nodes);
                    const uint32_t o = static_cast<uint32_t>(node) * static_cast<uint32_t>(sizeof(BvhNode));
                    const uint32_t nx = o + nfx, ny = o + nfy, nz = o + nfz;
                    lx = *reinterpret_cast<const float4*>(nb + nx); hx = *reinterpret_cast<const float4*>(nb + (nx ^ 16u));
                    ly = *reinterpret_cast<const float4*>(nb + ny + 32u); hy = *reinterpret_cast<const float4*>(nb + ((ny ^ 16u) + 32u));
                    lz = *reinterpret_cast<const float4*>(nb + nz + 64u); hz = *reinterpret_cast<const float4*>(nb + ((nz ^ 16u) + 64u));
                }
                if constexpr (PK) {
                    const uint2 cw = reinterpret_cast<const uint2*>(np)[14];
                    ch = make_int4(static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.x), static_cast<int32_t>(cw.y), static_cast<int32_t>(cw.y));
                } else {
                    ch = reinterpret_cast<const int4*>(np)[6];
                }
            }
            // branchless pushes (far to near) after a sorting network (ascending entry distance, misses last): every
            // write lands at or below the final top, which the stack's spare row covers; the pop reads the entry under
            // the top, the per-lane sentinel row (kNodeEmpty) when the stack is empty
            bool near;
            int32_t near_child;
            if constexpr (L) {
                // 16-bit child codes ride in the low half of the entry-distance keys: the network is 5 integer
                // min/max pairs and each code comes back with one bit-field extract
                uint32_t q0, q1, q2, q3;
                slab4_packed(lx, hx, ly, hy, lz, hz, ch, ix, iy, iz, oix, oiy, oiz, tminf, tmaxf, q0, q1, q2, q3);
                ucas(q0, q1);
                ucas(q2, q3);
                ucas(q0, q2);
                ucas(q1, q3);
                ucas(q1, q2);
                if (q0 >= kKeyMiss) ART_STAT_LANE(12);  // a dead visit: no child box is entered before tmax
                st.push(static_cast<int32_t>(q3), q3 < kKeyMiss);
                st.push(static_cast<int32_t>(q2), q2 < kKeyMiss);
                st.push(static_cast<int32_t>(q1), q1 < kKeyMiss);
                ART_DPUSH(q3, q3 < kKeyMiss);
                ART_DPUSH(q2, q2 < kKeyMiss);
                ART_DPUSH(q1, q1 < kKeyMiss);
                near = q0 < kKeyMiss;
                near_child = static_cast<int16_t>(q0);
#ifdef ART_STATS
                if (near) cur_d = __uint_as_float(q0 & 0xFFFF0000u);
#endif
            } else if constexpr (PK) {
                // as the LDS variant: 5 integer min/max pairs; each pushed code sign-extended from its key's low half
                uint32_t q0, q1, q2, q3;
                slab4_packed_nf(lx, hx, ly, hy, lz, hz, ch, ix, iy, iz, oix, oiy, oiz, tminf, tmaxf, q0, q1, q2, q3);
                ucas(q0, q1);
                ucas(q2, q3);
                ucas(q0, q2);
                ucas(q1, q3);
                ucas(q1, q2);
                st.push(static_cast<int16_t>(q3), q3 < kKeyMiss);
                st.push(static_cast<int16_t>(q2), q2 < kKeyMiss);
                st.push(static_cast<int16_t>(q1), q1 < kKeyMiss);
                near = q0 < kKeyMiss;
                near_child = static_cast<int16_t>(q0);
            } else {
                float k0, k1, k2, k3;
                slab4_nf(lx, hx, ly, hy, lz, hz, ix, iy, iz, oix, oiy, oiz, tminf, tmaxf, k0, k1, k2, k3);
                int32_t c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
                cas(k0, c0, k1, c1);
                cas(k2, c2, k3, c3);
                cas(k0, c0, k2, c2);
                cas(k1, c1, k3, c3);
                cas(k1, c1, k2, c2);
                const float inf = __builtin_inff();
                st.push(c3, k3 < inf);
                st.push(c2, k2 < inf);
                st.push(c1, k1 < inf);
                near = k0 < inf;
                near_child = c0;
            }
            {
                const int32_t top = st.peek();
                node = near ? near_child : top;
                st.pop_if(!near);
                ART_DPOP(!near);
                if (node < kNodeEmpty && parked == kNodeEmpty) {  // a leaf (codes below -1) and none parked yet: park it
                    parked = node;
                    node = st.peek();
                    st.pop_if(true);
                    ART_DPOP(true);
                }
            }
            if (!__any(parked == kNodeEmpty)) break;  // every lane still walking holds a leaf: test them together
        }
        // leaf phase: the parked leaf, else the current node when it is a leaf (a lane that left the node loop on the
        // wave-wide break still has an inner node to return to).  A lane that left the node loop holding a second leaf
        // (parked + current) tests both in this phase, one leaf phase instead of two (the wave's leaf loop runs over
        // the longer sum, once).  The stack is read once up front and the choices are selects (no dependent read in a
        // divergent branch).
        skip_nodes = false;
        int32_t leaf = parked;
        int32_t leaf2 = kNodeEmpty;
        {
            const bool has = parked != kNodeEmpty;
            if (!has && node == kNodeEmpty) break;
            const int32_t t0 = st.peek();
            const bool take2 = has && node < kNodeEmpty;  // a second leaf in hand: test both in this phase
            const bool pop = take2 || !has;
            leaf = has ? parked : node;
            leaf2 = take2 ? node : kNodeEmpty;
            node = pop ? t0 : node;
            st.pop_if(pop);
            ART_DPOP(pop);
            parked = kNodeEmpty;
        }
        uint32_t first, cnt;
        uint32_t first2 = 0, cnt12 = 0;
#ifdef ART_STATS
        const bool stats_phase = true;
#endif
        if constexpr (L) {
            const uint32_t x = ~static_cast<uint32_t>(leaf);
            first = x & ((1u << kLdsLeafShift) - 1);
            cnt = x >> kLdsLeafShift;
            const uint32_t x2 = leaf2 == kNodeEmpty ? 0u : ~static_cast<uint32_t>(leaf2);
            first2 = (x2 & ((1u << kLdsLeafShift) - 1)) - cnt;  // slot of entry k >= cnt: first2 + k
            cnt12 = cnt + (x2 >> kLdsLeafShift);
        } else if constexpr (PK) {
            first = leaf16_first(leaf) << kLeafShift;
            cnt = leaf16_count(leaf);
            // leaf2 == kNodeEmpty decodes as an empty range (count 0)
            first2 = (leaf16_first(leaf2) << kLeafShift) - cnt;
            cnt12 = cnt + leaf16_count(leaf2);
        } else {
            first = leaf_first(leaf);
            cnt = leaf_count(leaf);
            // leaf2 == kNodeEmpty decodes as an empty range (first 0, count 0)
            first2 = leaf_first(leaf2) - cnt;
            cnt12 = cnt + leaf_count(leaf2);
        }
#ifdef ART_STATS
        if (stats_phase) {  // the cooperative leaf test's iterations: the phase's tests spread over the lanes still here
            uint32_t total = 0;
            for (int b = 0; b < 4; ++b) total += static_cast<uint32_t>(__popcll(__ballot((cnt12 >> b) & 1u))) << b;
            const uint32_t active = static_cast<uint32_t>(__popcll(__ballot(true)));
            if (static_cast<int>(__lane_id()) == __ffsll(static_cast<long long>(__ballot(true))) - 1) {
                atomicAdd(&g_art_stats[46], 1ull);
                atomicAdd(&g_art_stats[47], static_cast<unsigned long long>((total + active - 1) / active));
            }
        }
#endif
        for (uint32_t k = 0; k < cnt12; ++k) {
            ART_STAT_WAVE(2);
            ART_STAT_LANE(3);
            R tt;
            uint32_t fc = 0, ref, m = kMatUnknown;
            bool h;
            if constexpr (L) {
                const uint32_t slot = (k < cnt ? first : first2) + k;
                h = hit_lds_slot(lds, slot, r, d_a, d_inv_a, tmin, tmax, tt, ref, m);
                fc = slot;  // the leaf slot travels in the face field (spheres have no face): LDS shading reads it
            } else {
                const uint32_t slot = (k < cnt ? first : first2) + k;
                if constexpr ((F & F_TRI) != 0 && PL == 2) {
                    // the LM 1 kernels' leaf triangles with their planes (TriRec112, in LDS): no cross product or
                    // plane offset per test
                    const TriRec112<R>& lt = S.leaf_tris112[slot];
                    V3<R> p1 = ld3(lt.p), p2 = ld3(lt.p + 3), p3 = ld3(lt.p + 6), nn = ld3(lt.n);
                    R pdd = lt.dd;
                    ref = S.primrefs[slot];
                    __asm__ volatile("" : "+v"(p1.x), "+v"(p1.y), "+v"(p1.z), "+v"(p2.x), "+v"(p2.y), "+v"(p2.z), "+v"(p3.x), "+v"(p3.y), "+v"(p3.z));
                    __asm__ volatile("" : "+v"(nn.x), "+v"(nn.y), "+v"(nn.z), "+v"(pdd));
                    if (fbase(F) == F_TRI || primref_type(ref) == PRIM_TRIANGLE) h = hit_tri_pre(p1, p2, p3, nn, pdd, r, tmin, tmax, tt);
                    else h = hit_prim<R, F & ~F_TRI>(S, ref, r, tmin, tmax, tt, fc);
                } else if constexpr ((F & F_TRI) != 0) {
                    // the leaf-ordered triangle copy: its address depends on the slot alone, so its loads go out
                    // beside the primref's instead of behind it (one L2 round trip per test instead of two); the
                    // empty asm keeps the compiler from sinking them under the type test
                    const TriRec<R>& lt = S.leaf_tris[slot];
                    V3<R> p1 = ld3(lt.p), p2 = ld3(lt.p + 3), p3 = ld3(lt.p + 6);
                    ref = S.primrefs[slot];
                    __asm__ volatile("" : "+v"(p1.x), "+v"(p1.y), "+v"(p1.z), "+v"(p2.x), "+v"(p2.y), "+v"(p2.z), "+v"(p3.x), "+v"(p3.y), "+v"(p3.z));
                    if (fbase(F) == F_TRI || primref_type(ref) == PRIM_TRIANGLE) h = hit_tri_v(p1, p2, p3, r, tmin, tmax, tt);
                    else h = hit_prim<R, F & ~F_TRI>(S, ref, r, tmin, tmax, tt, fc);
                } else {
                    // the leaf-ordered record copy: its loads go out beside the primref's instead of behind it
                    const uint4* lp = reinterpret_cast<const uint4*>(S.leaf_prims + slot);
                    uint4 v0 = lp[0], v1 = lp[1], v2 = lp[2], v3 = lp[3], v4 = lp[4];
                    ref = S.primrefs[slot];
                    __asm__ volatile("" : "+v"(v0.x), "+v"(v0.y), "+v"(v0.z), "+v"(v0.w), "+v"(v1.x), "+v"(v1.y), "+v"(v1.z), "+v"(v1.w),
                                          "+v"(v2.x), "+v"(v2.y), "+v"(v2.z), "+v"(v2.w), "+v"(v3.x), "+v"(v3.y), "+v"(v3.z), "+v"(v3.w));
                    __asm__ volatile("" : "+v"(v4.x), "+v"(v4.y), "+v"(v4.z), "+v"(v4.w));
                    PrimRec80 rec;
                    uint4* rp = reinterpret_cast<uint4*>(rec.b);
                    rp[0] = v0; rp[1] = v1; rp[2] = v2; rp[3] = v3; rp[4] = v4;
                    if constexpr (kSphPre) {
                        // spheres with the ray's |d|^2 and its reciprocal (div_rcp roots), as the LDS variant
                        if (primref_type(ref) == PRIM_SPHERE) {
                            const SphereRec<R>& sr = reinterpret_cast<const SphereRec<R>&>(rec);
                            V3<R> center = ld3(sr.c);
                            if (sr.flags & SPH_MOVING) center = moving_center(center, ld3(sr.d), sr.t0, sr.dt, r.tm);
                            if constexpr (kSphLazy) h = sphere_root_lazy<R>(center, sr.r * sr.r, r, d_a, d_inv_a, tmin, tmax, tt);
                            else h = sphere_root<R, true>(center, sr.r * sr.r, r, d_a, d_inv_a, tmin, tmax, tt);
                        } else {
                            h = hit_prim_rec<R, F & ~F_SPHERE>(primref_type(ref), rec, r, tmin, tmax, tt, fc);
                        }
                    } else {
                        h = hit_prim_rec<R, F>(primref_type(ref), rec, r, tmin, tmax, tt, fc);
                    }
                    // the record's material index (sphere / box / rect: dword 18 / 12 / 11) and a rect's axis (dword 10,
                    // in the face field): the hit's surface then needs no reload of a box or rect record (prim_surface)
                    const uint32_t ty = primref_type(ref);
                    m = ty == PRIM_SPHERE ? v4.z : ty == PRIM_BOX ? v3.x : v2.w;
                    if (ty == PRIM_RECT) fc = v2.z;
                }
#ifdef ART_STATS
                {  // leaf tests by primitive type: lane tests [15/17/19/21], wave iterations running that type [16/18/20/22]
                    const uint32_t ty = primref_type(ref);
                    if (ty == PRIM_BOX) { ART_STAT_WAVE(16); ART_STAT_LANE(15); }
                    else if (ty == PRIM_SPHERE) { ART_STAT_WAVE(18); ART_STAT_LANE(17); }
                    else if (ty == PRIM_TRIANGLE) { ART_STAT_WAVE(20); ART_STAT_LANE(19); }
                    else { ART_STAT_WAVE(22); ART_STAT_LANE(21); }
                }
#endif
            }
            if (h) {
                ART_STAT_LANE(13);
                tmax = tt;
                t = tt;
                prim = ref;
                face = fc;
                mt = m;
                hit = true;
                tmaxf = f_hi(tt);
            }
        }
    }
    return hit;
}

// ------------------------------------------------------------------------------------------------ objects
template <class R>
__device__ __forceinline__ Ray<R> xform_in(const ObjRec<R>& o, const Ray<R>& r) {
    Ray<R> out = r;
    if (o.kind == OBJ_TRANSLATE) {  // hittable.cpp:4: moved_r(origin - offset, direction, time)
        out.o = r.o - mk(o.p[0], o.p[1], o.p[2]);
    } else {  // hittable.cpp:58-67
        const R s = o.p[0], c = o.p[1];
        out.o.x = c * r.o.x - s * r.o.z;
        out.o.z = s * r.o.x + c * r.o.z;
        out.d.x = c * r.d.x - s * r.d.z;
        out.d.z = s * r.d.x + c * r.d.z;
    }
    return out;
}

// Any non-medium object: prim, BVH, or a translate/rotate_y chain (<= kMaxXformChain) over one of them.
template <class R, uint32_t F, int B, bool L, int PL = 0, bool RES = false>
__device__ __forceinline__ bool hit_object(const DevScene<R>& S, const uint8_t* lds, int32_t oi, Ray<R> r, R tmin, R tmax, StackF<L, F>* stk,
                                           R& t, uint32_t& prim, uint32_t& face, uint32_t& mt, TravResume* rs = nullptr) {
    if (F & F_XFORM) {
#pragma unroll
        for (int c = 0; c < kMaxXformChain; ++c) {
            const ObjRec<R>& o = S.objs[oi];
            if (o.kind != OBJ_TRANSLATE && o.kind != OBJ_ROTATE_Y) break;
            r = xform_in(o, r);
            oi = o.a;
        }
    }
    const ObjRec<R>& o = S.objs[oi];
    if (o.kind == OBJ_PRIM) {
        prim = static_cast<uint32_t>(o.a);
        mt = kMatUnknown;
        // HBM-scene kernels: the primitive's record from obj_prims[oi], whose address does not wait on the object
        if constexpr (!L) {
            const PrimRec80& rec = S.obj_prims[oi];
            const uint32_t ty = primref_type(prim);
            const bool h = hit_prim_rec<R, F>(ty, rec, r, tmin, tmax, t, face);
            if constexpr ((F & F_TRI) == 0) {  // as the leaf records: the material index, a rect's axis in `face`
                const uint32_t* wd = reinterpret_cast<const uint32_t*>(rec.b);
                mt = ty == PRIM_SPHERE ? wd[18] : ty == PRIM_BOX ? wd[12] : wd[11];
                if (ty == PRIM_RECT) face = wd[10];
            }
            return h;
        } else {
            return hit_prim<R, F>(S, prim, r, tmin, tmax, t, face);
        }
    }
    return traverse<R, F, B, L, PL, RES>(S, lds, o.a, r, tmin, tmax, stk, t, prim, face, mt, rs, o.b);
}

// Out of line: measured +0.2 % (cow) to +1.8 % (Next-Week final) over the inlined body, which raised the register
// pressure of the whole path loop for a function most segments do not reach.
static __device__ __noinline__ double glibc_log_call(double x) { return glibc_log(x); }
// get_sphere_uv out of line as well (glibc_trig.h's acos / atan2 are long and run only for image-textured spheres):
// measured r4z2 the earth scene +3.1 % (its kernel: 166 -> 160 VGPRs, SGPR spills 28 -> 12), the Next-Week final +-0
[[maybe_unused]] static __device__ __noinline__ UvPair sphere_uv_call(double x, double y, double z, const double* c, const double* t) {
    return sphere_uv(x, y, z, TrigTab(c, t));
}
// constant_medium.h:37-82.  Consumes one uniform when the clamped interval is non-empty.
template <class R, uint32_t F, int B, bool L, int PL = 0>
__device__ __forceinline__ bool hit_medium(const DevScene<R>& S, const uint8_t* lds, const ObjRec<R>& m, const Ray<R>& r, R tmin, R tmax,
                                           StackF<L, F>* stk, uint64_t& rng, R& t) {
    const R inf = R(__builtin_inf());
    R t1, t2;
    const ObjRec<R>& bo = S.objs[m.a];
    if ((F & F_SPHERE) && bo.kind == OBJ_PRIM && primref_type(static_cast<uint32_t>(bo.a)) == PRIM_SPHERE) {
        // A sphere boundary (every medium of the reference scenes but the Cornell smoke boxes): the two boundary->hit
        // calls (constant_medium.h:43, :46) compute the same oc, half_b, c, discriminant and sqrt (sphere.h:39-47)
        // from the same ray and sphere, so both root selections (sphere.h:49-55) run on one quadratic: the same
        // values, half the arithmetic.
        const SphereRec<R>& sp = [&]() -> const SphereRec<R>& {
            if constexpr (!L) return reinterpret_cast<const SphereRec<R>&>(S.obj_prims[m.a]);
            else return S.spheres[primref_index(static_cast<uint32_t>(bo.a))];
        }();
        V3<R> center = ld3(sp.c);
        if (sp.flags & SPH_MOVING) center = moving_center(center, ld3(sp.d), sp.t0, sp.dt, r.tm);
        const V3<R> oc = r.o - center;
        const R a = len2(r.d);
        const R half_b = dot(oc, r.d);
        const R c = len2(oc) - sp.r * sp.r;
        const R disc = half_b * half_b - a * c;
        if (disc < R(0)) return false;
        const R sqrtd = sqrt_rn(disc);
        const R r_near = (-half_b - sqrtd) / a, r_far = (-half_b + sqrtd) / a;
        t1 = r_near;  // first call, t in [-inf, inf]
        if (t1 < -inf || inf < t1) {
            t1 = r_far;
            if (t1 < -inf || inf < t1) return false;
        }
        const R tmin2 = t1 + R(0.0001);  // second call, t in [t1 + 0.0001, inf]
        t2 = r_near;
        if (t2 < tmin2 || inf < t2) {
            t2 = r_far;
            if (t2 < tmin2 || inf < t2) return false;
        }
    } else if constexpr ((F & F_MEDIA_G) != 0) {
        uint32_t p, f, mt;
        if (!hit_object<R, F, B, L, PL>(S, lds, m.a, r, -inf, inf, stk, t1, p, f, mt)) return false;
        if (!hit_object<R, F, B, L, PL>(S, lds, m.a, r, t1 + R(0.0001), inf, stk, t2, p, f, mt)) return false;
    } else {
        return false;  // unreachable: a scene with a non-sphere medium boundary has F_MEDIA_G
    }
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < R(0)) t1 = R(0);
    const R ray_length = sqrt_rn(len2(r.d));
    const R inside = (t2 - t1) * ray_length;
    // log(random_double()) of constant_medium.h:61 is the C library's log (glibc) in the reference; the device's own
    // f64 log differs from it in the last bit for 445 762 of the 2^24 arguments a uniform can take, which moves a
    // scattering path's t and every sum after it.  glibc_log.h restates glibc's log operation by operation (equal for
    // every k * 2^-24); it replaced a 128 MiB table of glibc's values, whose random reads (an L2 miss per draw) cost 5-10 % on the medium scenes.
    const uint32_t k = uniform_k(rng);
    const R hit_distance = m.p[0] * glibc_log_call(static_cast<double>(k) * 0x1p-24);
    if (hit_distance > inside) return false;
    t = t1 + hit_distance / ray_length;
    return true;
}

// The world hittable_list (hittable_list.cpp:5-19): objects in order, t_max = closest so far.
struct HitOut {
    uint32_t prim, obj;  // obj: world slot | box face << 16
    uint32_t mt;         // LDS scene image: the material type; HBM-scene triangle-free kernels: the material index of a
                         // primitive hit (a rect's axis then rides in obj >> 16); else kMatUnknown
};
template <class R, uint32_t F, int B, bool L, int PL = 0>
__device__ __forceinline__ bool trace_world(const DevScene<R>& S, const uint8_t* lds, const Ray<R>& r, StackF<L, F>* stk, uint64_t& rng, R& t,
                                            HitOut& h) {
    R closest = R(__builtin_inf());
    bool any = false;
    for (int w = 0; w < S.nworld; ++w) {
        const int32_t oi = S.world[w];
        const ObjRec<R>& o = S.objs[oi];
        R tt;
        if ((F & F_MEDIA) && o.kind == OBJ_MEDIUM) {
            if (hit_medium<R, F, B, L, PL>(S, lds, o, r, R(0.001), closest, stk, rng, tt)) {
                closest = tt;
                any = true;
                h.prim = kMediumHit;
                h.obj = static_cast<uint32_t>(w);
                h.mt = kMatUnknown;
            }
        } else {
            uint32_t prim = 0, face = 0, mt = kMatUnknown;
            if (hit_object<R, F, B, L, PL>(S, lds, oi, r, R(0.001), closest, stk, tt, prim, face, mt)) {
                closest = tt;
                any = true;
                h.prim = prim;
                h.obj = static_cast<uint32_t>(w) | (face << 16);
                h.mt = mt;
            }
        }
    }
    t = closest;
    return any;
}

// trace_world with suspendable BVH traversals (ART_SUSPEND_LANES): the world list walk of one segment, resumed at
// world slot w with the closest hit so far.  Returns true when the segment's trace is complete.  Medium boundaries
// and prim objects never suspend.
template <class R>
struct TraceState {
    R closest;
    HitOut h;
    int32_t w;
    bool any;
    TravResume tr;
    __device__ __forceinline__ void start() {
        closest = R(__builtin_inf());
        any = false;
        w = 0;
        tr.fresh = true;
    }
};
template <class R, uint32_t F, int B, int PL>
__device__ __forceinline__ bool trace_world_res(const DevScene<R>& S, const Ray<R>& r, StackF<false, F>* stk, uint64_t& rng, TraceState<R>& ts) {
    ts.tr.suspended = false;
    for (int32_t w = ts.w; w < S.nworld; ++w) {
        const int32_t oi = S.world[w];
        const ObjRec<R>& o = S.objs[oi];
        R tt;
        if ((F & F_MEDIA) && o.kind == OBJ_MEDIUM) {
            if (hit_medium<R, F, B, false, PL>(S, nullptr, o, r, R(0.001), ts.closest, stk, rng, tt)) {
                ts.closest = tt;
                ts.any = true;
                ts.h.prim = kMediumHit;
                ts.h.obj = static_cast<uint32_t>(w);
                ts.h.mt = kMatUnknown;
            }
        } else {
            uint32_t prim = 0, face = 0, mt = kMatUnknown;
            if (hit_object<R, F, B, false, PL, true>(S, nullptr, oi, r, R(0.001), ts.closest, stk, tt, prim, face, mt, &ts.tr)) {
                ts.closest = tt;
                ts.any = true;
                ts.h.prim = prim;
                ts.h.obj = static_cast<uint32_t>(w) | (face << 16);
                ts.h.mt = mt;
            }
            if (ts.tr.suspended) {
                ts.w = w;
                return false;
            }
            ts.tr.fresh = true;
        }
    }
    return true;
}

// ------------------------------------------------------------------------------------------------ surfaces
template <class R>
struct Surf {
    V3<R> p, n;
    R u, v;
    bool ff;
    uint32_t mat;
};
template <class R>
__device__ __forceinline__ void set_face_normal(Surf<R>& s, const Ray<R>& r, V3<R> outward) {  // hittable.h:18-22
    s.ff = dot(r.d, outward) < R(0);
    s.n = s.ff ? outward : -outward;
}
// hittable.h:18-22 into locals (prim_surface)
template <class R>
__device__ __forceinline__ void face_normal(const Ray<R>& r, V3<R> outward, bool& ff, V3<R>& n) {
    ff = dot(r.d, outward) < R(0);
    n = ff ? outward : -outward;
}
// An axis-aligned rect's surface into prim_surface's locals.  prim_surface builds every field in locals and stores s
// once: stores into s in several branches were merged by the compiler into one store through a phi of addresses
// (different fields), which kept parts of Surf in scratch memory.
template <class R, bool UV = true>
__device__ __forceinline__ void rect_surface(V3<R>& p, V3<R>& n, bool& ff, R& su, R& sv, int axis, R a0, R a1, R b0, R b1, const Ray<R>& r,
                                             R t, bool need_uv = true) {
    if (UV && need_uv) {  // u, v feed image textures only (materials without MATF_NEEDS_UV skip the two divisions)
        const int ia = axis == 2 ? 1 : 0;
        const int ib = axis == 0 ? 1 : 2;
        const R x = comp(r.o, ia) + t * comp(r.d, ia);
        const R y = comp(r.o, ib) + t * comp(r.d, ib);
        su = (x - a0) / (a1 - a0);
        sv = (y - b0) / (b1 - b0);
    }
    const V3<R> on = axis == 0 ? mk(R(0), R(0), R(1)) : (axis == 1 ? mk(R(0), R(1), R(0)) : mk(R(1), R(0), R(0)));
    face_normal(r, on, ff, n);
    p = r.at(t);
}
// mat_hint (HitOut::mt of a triangle-free HBM-scene kernel): the hit's material index, kMatUnknown otherwise.  With it,
// a box or rect hit whose material samples no u,v builds its surface from the face / axis alone -- normal, point,
// material -- without reloading the primitive record (its bounds only feed u, v).
// uvc: glibc_trig.h's constants (uv_table(S) or k_paths_g's LDS copy of its head; read only when UV); the tables
// behind them are read from uv_table(S)
// TUV: triangle u, v (barycentric image textures); UV: u, v of every primitive (TF_IMAGE kernels)
template <class R, uint32_t F, bool UV = true, bool TUV = UV>
__device__ __forceinline__ void prim_surface(const DevScene<R>& S, uint32_t ref, uint32_t face, const Ray<R>& r, R t, Surf<R>& s,
                                             uint32_t mat_hint, const double* uvc) {
    const uint32_t idx = primref_index(ref);
    const uint32_t type = (fbase(F) == F_SPHERE) ? PRIM_SPHERE : primref_type(ref);
    V3<R> sp_p = mk(R(0), R(0), R(0)), sp_n = mk(R(0), R(0), R(0));
    bool ff = false;
    R su = R(0), sv = R(0);
    uint32_t mat = 0;
    switch (type) {
        case PRIM_SPHERE: {  // sphere.h:57-63, :24-37
            ART_STAT_WAVE(40);
            ART_STAT_LANE(41);
            const SphereRec<R>& sp = S.spheres[idx];
            V3<R> center = ld3(sp.c);
            const bool moving = (sp.flags & SPH_MOVING) != 0;
            if (moving) center = center + motion_fraction(r.tm, sp.t0, sp.dt) * ld3(sp.d);
            sp_p = r.at(t);
            const V3<R> outward = divs(sp_p - center, sp.r);
            face_normal(r, outward, ff, sp_n);
            // u,v only feed image textures: acos/atan2 are skipped for materials that never sample them
            if (UV && !moving && (S.mats[sp.mat].flags & MATF_NEEDS_UV)) {
                ART_STAT_WAVE(32);
                ART_STAT_LANE(33);
                // get_sphere_uv (sphere.h:24-37) with glibc's acos / atan2 restated (sphere_uv.h; their constants are
                // loaded where used, not hoisted into the path loop's registers)
                const UvPair uv = sphere_uv_call(static_cast<double>(outward.x), static_cast<double>(outward.y), static_cast<double>(outward.z),
                                                 uvc, uv_table(S));
                su = R(uv.u);
                sv = R(uv.v);
            }
            mat = sp.mat;
            break;
        }
        case PRIM_TRIANGLE: {  // triangle.h:57-85
            if (!(F & F_TRI)) break;
            const TriRec<R>& tr = S.tris[idx];
            const V3<R> p1 = ld3(tr.p), p2 = ld3(tr.p + 3), p3 = ld3(tr.p + 6);
            const V3<R> N = cross(p2 - p1, p3 - p1);
            const V3<R> p = r.o + t * r.d;
            sp_p = p;
            face_normal(r, N, ff, sp_n);
            if (TUV && (S.mats[tr.mat].flags & MATF_NEEDS_UV)) {  // barycentric u, v feed image textures only (texture.h:135-154)
                const R u = dot(N, cross(p3 - p2, p - p2));
                const R v = dot(N, cross(p1 - p3, p - p3));
                su = u / len2(N);
                sv = v / len2(N);
            }
            mat = tr.mat;
            break;
        }
        case PRIM_RECT: {
            if (!(F & F_RECT)) break;
            if (mat_hint != kMatUnknown && !(UV && (S.mats[mat_hint].flags & MATF_NEEDS_UV))) {
                ART_STAT_WAVE(42);
                ART_STAT_LANE(43);
                rect_surface<R, false>(sp_p, sp_n, ff, su, sv, static_cast<int>(face), R(0), R(0), R(0), R(0), r, t);
                mat = mat_hint;
                break;
            }
            ART_STAT_WAVE(38);
            ART_STAT_LANE(39);
            const RectRec<R>& q = S.rects[idx];
            rect_surface<R, UV>(sp_p, sp_n, ff, su, sv, static_cast<int>(q.axis), q.a0, q.a1, q.b0, q.b1, r, t, (S.mats[q.mat].flags & MATF_NEEDS_UV) != 0);
            mat = q.mat;
            break;
        }
        default: {
            if (!(F & F_BOX)) break;
            if (mat_hint != kMatUnknown && !(UV && (S.mats[mat_hint].flags & MATF_NEEDS_UV))) {
                ART_STAT_WAVE(42);
                ART_STAT_LANE(43);
                rect_surface<R, false>(sp_p, sp_n, ff, su, sv, static_cast<int>(face >> 1), R(0), R(0), R(0), R(0), r, t);  // box_face: axis = f >> 1
                mat = mat_hint;
                break;
            }
            ART_STAT_WAVE(38);
            ART_STAT_LANE(39);
            const BoxRec<R>& b = S.boxes[idx];
            int axis;
            R a0, a1, b0, b1, k;
            box_face(b, static_cast<int>(face), axis, a0, a1, b0, b1, k);
            rect_surface<R, UV>(sp_p, sp_n, ff, su, sv, axis, a0, a1, b0, b1, r, t, (S.mats[b.mat].flags & MATF_NEEDS_UV) != 0);
            mat = b.mat;
            break;
        }
    }
    s.p = sp_p;
    s.n = sp_n;
    s.ff = ff;
    s.u = su;
    s.v = sv;
    s.mat = mat;
}

// Rebuilds the hit_record of the world object that won (transform chain unwound as translate::hit / rotate_y::hit
// do it: hittable.cpp:7-11, :72-84, including set_face_normal against the transformed ray).
template <class R, uint32_t F, bool UV = true, bool TUV = UV>
__device__ __forceinline__ void world_surface(const DevScene<R>& S, const HitOut& h, const Ray<R>& r, R t, Surf<R>& s, const double* uvc = nullptr) {
    const int32_t w = static_cast<int32_t>(h.obj & 0xFFFFu);
    int32_t oi = S.world[w];
    ART_STAT_WAVE(44);
    ART_STAT_LANE(45);
    if ((F & F_MEDIA) && h.prim == kMediumHit) {  // constant_medium.h:75-79
        ART_STAT_WAVE(36);
        ART_STAT_LANE(37);
        s.p = r.at(t);
        s.n = mk(R(1), R(0), R(0));
        s.ff = true;
        s.u = R(0);
        s.v = R(0);
        s.mat = static_cast<uint32_t>(S.objs[oi].b);
        return;
    }
    static_assert(kMaxXformChain == 2, "world_surface unwinds at most two transforms");
    int32_t o0 = -1, o1 = -1;
    Ray<R> r1 = r, r2 = r;
    if (F & F_XFORM) {
        const ObjRec<R>& o = S.objs[oi];
        if (o.kind == OBJ_TRANSLATE || o.kind == OBJ_ROTATE_Y) {
            o0 = oi;
            r1 = xform_in(o, r);
            oi = o.a;
            const ObjRec<R>& q = S.objs[oi];
            if (q.kind == OBJ_TRANSLATE || q.kind == OBJ_ROTATE_Y) {
                o1 = oi;
                r2 = xform_in(q, r1);
                oi = q.a;
            } else {
                r2 = r1;
            }
        }
    }
    prim_surface<R, F, UV, TUV>(S, h.prim, h.obj >> 16, r2, t, s, (F & F_TRI) == 0 ? h.mt : kMatUnknown, uvc);
    if (!(F & F_XFORM)) return;
#ifdef ART_STATS
    if (o0 >= 0) {
        ART_STAT_WAVE(34);
        ART_STAT_LANE(35);
    }
#endif
    auto unwind = [&](int32_t xo, const Ray<R>& inner) {
        const ObjRec<R>& o = S.objs[xo];
        if (o.kind == OBJ_TRANSLATE) {
            s.p = s.p + mk(o.p[0], o.p[1], o.p[2]);
            set_face_normal(s, inner, s.n);
        } else {
            const R sn = o.p[0], c = o.p[1];
            V3<R> p = s.p, n = s.n;
            p.x = c * s.p.x + sn * s.p.z;
            p.z = -sn * s.p.x + c * s.p.z;
            n.x = c * s.n.x + sn * s.n.z;
            n.z = -sn * s.n.x + c * s.n.z;
            s.p = p;
            set_face_normal(s, inner, n);
        }
    };
    if (o1 >= 0) unwind(o1, r2);
    if (o0 >= 0) unwind(o0, r1);
}

// ------------------------------------------------------------------------------------------------ textures
template <class R>
__device__ __forceinline__ R perlin_noise(const PerlinRec<R>& pn, V3<R> p) {  // perlin.h:21-40, :83-97
    const R u = p.x - floor(p.x), v = p.y - floor(p.y), w = p.z - floor(p.z);
    const int i = static_cast<int>(floor(p.x)), j = static_cast<int>(floor(p.y)), k = static_cast<int>(floor(p.z));
    const R uu = u * u * (R(3) - R(2) * u), vv = v * v * (R(3) - R(2) * v), ww = w * w * (R(3) - R(2) * w);
    // perlin_interp's weights i*uu + (1-i)*(1-uu) with i in {0, 1}: u, v, w lie in [+0, 1), so uu, vv, ww and 1 - uu,
    // ... are >= +0 and finite; 0 * x is then +0, 1 * x is x and x + (+0) is x -- the weight is exactly 1 - uu (i = 0)
    // or uu (i = 1), and u - 0 is exactly u.  Folding them (the compiler may not: 0 * x is not +0 for every double)
    // leaves the same products and sums in the same order.
    const R wx[2] = {R(1) - uu, uu}, wy[2] = {R(1) - vv, vv}, wz[2] = {R(1) - ww, ww};
    const R dx[2] = {u, u - R(1)}, dy[2] = {v, v - R(1)}, dz[2] = {w, w - R(1)};
    const int px[2] = {pn.perm[0][i & 255], pn.perm[0][(i + 1) & 255]};
    const int py[2] = {pn.perm[1][j & 255], pn.perm[1][(j + 1) & 255]};
    const int pz[2] = {pn.perm[2][k & 255], pn.perm[2][(k + 1) & 255]};
    R accum = R(0);
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const V3<R> g = ld3(pn.ranvec[px[a] ^ py[b] ^ pz[c]]);
                accum += wx[a] * wy[b] * wz[c] * dot(g, mk(dx[a], dy[b], dz[c]));
            }
    return accum;
}
// perlin noise out of line, as the medium's log and get_sphere_uv: measured r4z3 the two-perlin-spheres scene +6.5 %,
// the Next-Week final +-0
[[maybe_unused]] static __device__ __noinline__ double perlin_call(const PerlinRec<double>* pn, double x, double y, double z) {
    return perlin_noise(*pn, mk(x, y, z));
}
template <class R>
__device__ __forceinline__ V3<R> image_value(const DevScene<R>& S, int32_t im, R u, R v) {  // texture.h:90-117
    const ImageRec& I = S.images[im];
    u = fmin(fmax(u, R(0)), R(1));
    v = R(1) - fmin(fmax(v, R(0)), R(1));
    int i = static_cast<int>(u * R(I.w));
    int j = static_cast<int>(v * R(I.h));
    if (i >= I.w) i = I.w - 1;
    if (j >= I.h) j = I.h - 1;
    const R cs = R(1.0 / 255.0);
    const uint8_t* px = S.texels + I.offset + static_cast<uint64_t>(j) * static_cast<uint64_t>(I.bpp * I.w) + static_cast<uint64_t>(i) * I.bpp;
    return mk(cs * R(px[0]), cs * R(px[1]), cs * R(px[2]));
}
// checker_texture (texture.h:41-48): sin(10x)*sin(10y)*sin(10z) < 0.  Only the SIGN of the product matters, so it
// is evaluated as a sign parity: sin(y) == 0 exactly iff y == 0 for doubles (pi is irrational), and for y != 0
// sin(y) < 0 iff floor(y / pi) is odd.  Same predicate as the reference's, without the Payne-Hanek reduction of a
// full f64 sin (46 VGPRs in the shade kernel); it can only differ when y is within ~1 ulp of a multiple of pi.
// sin(y) < 0 as a bool (y != 0): floor(y / pi) odd, the parity read in floating point (k / 2 == floor(k / 2) for even
// k; every double >= 2^53 is even, as its integer conversion would say) -- no f64 -> int64 conversion sequence.
template <class R>
__device__ __forceinline__ bool sin_negative(R y) {
    const R k = floor(y * R(0.31830988618379067154));
    return R(0.5) * k != floor(R(0.5) * k);
}
template <class R>
__device__ __forceinline__ bool checker_odd(V3<R> p) {  // sin(10x) * sin(10y) * sin(10z) < 0
    const R x = R(10) * p.x, y = R(10) * p.y, z = R(10) * p.z;
    const bool nonzero = x != R(0) && y != R(0) && z != R(0);
    return nonzero && (sin_negative(x) != (sin_negative(y) != sin_negative(z)));
}

// rendering/texture.h.  TF (layout.h TexFeature bits) prunes the texture kinds a scene cannot contain.
template <class R, uint32_t TF = TF_ALL>
__device__ __forceinline__ V3<R> tex_value(const DevScene<R>& S, int32_t ti, R u, R v, V3<R> p) {
    for (int level = 0; level < 4; ++level) {
        const TexRec<R>& t = S.texs[ti];
        if (TF == TF_SOLID || t.type == TEX_SOLID) return ld3(t.c);
        if ((TF & TF_CHECKER) && t.type == TEX_CHECKER) {
            ti = checker_odd(p) ? t.odd : t.even;
            continue;
        }
        if ((TF & TF_NOISE) && t.type == TEX_NOISE) {
            ART_STAT_WAVE(28);
            ART_STAT_LANE(29);
            const V3<R> q = t.scale * p;
            const R n = perlin_call(&S.perlins[t.perlin], q.x, q.y, q.z);
            const R h = (R(1) + n) * R(0.5);
            return mk(h, h, h);
        }
        if ((TF & TF_IMAGE) && t.type == TEX_IMAGE) {
            ART_STAT_WAVE(30);
            ART_STAT_LANE(31);
            return image_value(S, t.image, u, v);
        }
        if ((TF & (TF_IMAGE | TF_BARY)) && t.type == TEX_BARY_IMAGE) {
            const R w = R(1) - u - v;
            return image_value(S, t.image, u * t.uv[0] + v * t.uv[2] + w * t.uv[4], u * t.uv[1] + v * t.uv[3] + w * t.uv[5]);
        }
        break;
    }
    return mk(R(0), R(1), R(1));
}

// The texture value of material m (lambertian / diffuse_light / isotropic): the inlined solid colour (MATF_SOLID) or
// tex_value of its texture tree -- the same doubles either way.
template <class R, uint32_t TF = TF_ALL>
__device__ __forceinline__ V3<R> mat_tex_value(const DevScene<R>& S, const MatRec<R>& m, R u, R v, V3<R> p) {
    if (m.flags & MATF_SOLID) return ld3(m.albedo);
    return tex_value<R, TF>(S, m.tex, u, v, p);
}

}  // namespace art
