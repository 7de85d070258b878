// layout.h — the flat scene and path-state layout in HBM, shared by host (g++) and device (hipcc) code.
//
// The reference walks an OOP graph of shared_ptr<hittable> with virtual hit()/scatter()/value()
// (engine/hittable.h:25-29, rendering/material.h:10-17, rendering/texture.h:11-14).  Here the same graph is
// compiled (scene.cpp: compile()) into typed arrays:
//   * primitives   per-type AoS records (SphereRec, TriRec, RectRec, BoxRec), addressed by a 32-bit prim ref
//   * BVH          one flat array of 128-B four-child nodes (f32, conservatively rounded boxes) per scene
//   * objects      the top-level hittable_list (world) as ObjRec: PRIM | BVH | XFORM (translate/rotate_y) | MEDIUM
//   * materials    MatRec, textures TexRec, perlin tables, image texel pool
// Every record exists in an f64 and an f32 instantiation (template R); the BVH is always f32.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define ART_HD __host__ __device__ inline
#else
#define ART_HD inline
#endif

namespace art {

// ---------------------------------------------------------------------------------------------- prims
enum PrimType : uint32_t { PRIM_SPHERE = 0, PRIM_TRIANGLE = 1, PRIM_RECT = 2, PRIM_BOX = 3 };
constexpr uint32_t kPrimTypeShift = 30;
constexpr uint32_t kPrimIndexMask = (1u << kPrimTypeShift) - 1;
ART_HD uint32_t make_primref(uint32_t type, uint32_t idx) { return (type << kPrimTypeShift) | idx; }
ART_HD uint32_t primref_type(uint32_t ref) { return ref >> kPrimTypeShift; }
ART_HD uint32_t primref_index(uint32_t ref) { return ref & kPrimIndexMask; }

enum SphereFlags : uint32_t { SPH_MOVING = 1u };  // moving_sphere: centre lerp over [t0, t0+dt], no u,v

template <class R>
struct SphereRec {      // sphere.h / moving_sphere.h
    R c[3];             // center (center0 for moving spheres)
    R r;                // radius
    R d[3];             // center1 - center0 (moving only)
    R t0, dt;           // time0, time1 - time0 (moving only)
    uint32_t mat;
    uint32_t flags;
};
template <class R>
struct TriRec {         // triangle.h: pt1, pt2, pt3
    R p[9];
    uint32_t mat;
    uint32_t pad;
};
// A leaf triangle with its plane precomputed on the host by the device's own operations (the LM 1 kernels'
// LDS copy): n = cross(pt2 - pt1, pt3 - pt1) and dd = -dot(n, pt1), triangle.h:30-41
template <class R>
struct TriRec112 {
    R p[9];
    R n[3];
    R dd;
    uint32_t mat;
    uint32_t pad;
};
// One primitive record of any type (SphereRec, TriRec, RectRec, BoxRec are all <= 80 B): the device copy of a prim
// object's primitive, indexed by object (DevScene::obj_prims)
struct alignas(16) PrimRec80 {
    uint8_t b[80];
};
template <class R>
struct RectRec {        // aarect.h: axis 0 = xy_rect (k on z), 1 = xz_rect (k on y), 2 = yz_rect (k on x)
    R a0, a1, b0, b1, k;
    uint32_t axis;
    uint32_t mat;
};
template <class R>
struct BoxRec {         // box.cpp: six rects in a fixed order (face index 0..5 = box.cpp:8-17 order)
    R mn[3], mx[3];
    uint32_t mat;
    uint32_t pad;
};

// ---------------------------------------------------------------------------------------------- BVH
// Four-child node, 128 B = two cache lines, fetched as eight 16-B loads; the four child boxes are stored SoA so one
// node visit tests all four with float4 arithmetic.  Child boxes are rounded outward to f32 and padded, so f32
// traversal is conservative; leaf tests run in R.
//   child >= 0 : inner node index;   child < 0 : leaf ~((count << 24) | first_primref_slot);   -1 : empty slot
struct alignas(16) BvhNode {
    float lox[4], hix[4];
    float loy[4], hiy[4];
    float loz[4], hiz[4];
    int32_t child[4];
    int32_t pad[4];
};
static_assert(sizeof(BvhNode) == 128, "BvhNode must be two 64-B lines");
constexpr int32_t kNodeEmpty = -1;
ART_HD int32_t make_leaf(uint32_t first, uint32_t count) { return ~static_cast<int32_t>((count << 24) | first); }
ART_HD uint32_t leaf_first(int32_t c) { return static_cast<uint32_t>(~c) & 0xFFFFFFu; }
ART_HD uint32_t leaf_count(int32_t c) { return (static_cast<uint32_t>(~c) >> 24) & 0x7Fu; }
// 16-bit child codes (BvhNode::pad, the packed-key traversal of k_paths_g kernels with F_CODE16): an inner node is its
// index (< 32768), a leaf of 1..4 primitives starting at primitive reference `first` (< 8192) is
// -2 - ((count - 1) << 13 | first), at most -2, so kNodeEmpty (-1) stays apart and `code < kNodeEmpty` marks a leaf.
// leaf16_first / leaf16_count of kNodeEmpty give an empty range.
ART_HD bool leaf16_ok(uint32_t first, uint32_t count) { return count >= 1u && count <= 4u && first < 8192u && (((count - 1u) << 13) | first) <= 32766u; }
ART_HD int32_t make_leaf16(uint32_t first, uint32_t count) { return -2 - static_cast<int32_t>(((count - 1u) << 13) | first); }
ART_HD uint32_t leaf16_first(int32_t c) { return static_cast<uint32_t>(-2 - c) & 0x1FFFu; }
ART_HD uint32_t leaf16_count(int32_t c) { return static_cast<uint32_t>((-2 - c) >> 13) + 1u; }
constexpr int kMaxLeafPrims = 4;
constexpr int kMaxBvhDepth = 30;     // binary SAH tree depth cap
constexpr int kMaxStackDepth = 64;   // per-lane LDS traversal stack entries (sized per scene: FlatScene::max_stack)

// ---------------------------------------------------------------------------------------------- LDS scene image
// A spheres-only f64 scene whose BVH4 and leaf spheres fit one CU's LDS (the random-spheres benchmark scene: 234
// nodes, 874 leaf slots) is traversed entirely out of LDS: k_extend copies this image into LDS once per block, so the
// node and sphere fetches of the traversal never touch the vector-memory (TA/L1) path that bounds the global variant.
// Every plane is an array of 16-B entries, so lanes fetching different nodes/spheres spread over the 16 four-bank slots
// of the ds_read_b128 bank row, and the plane strides are compile-time (DS immediate offsets, no address VALU).
// BVH4 nodes: 10 planes -- per axis (lo, hi, lo again) as float4, so the far plane of either direction sign is one
// plane above the near one (an immediate DS offset); then the four child codes as int16 in the first 8 bytes of the
// child plane.  The boxes are the union over the shutter (y motion planes, the lerp of a child's t = 0 and t = 1 boxes,
// measured 7.6 % fewer node visits but -1.5 % overall: two more loads and FMAs per visit, 21 more VGPR spills).
// LDS node capacity: the random scene's tree without the hoisted ground sphere has 259 nodes (greedy collapse, bvh.cpp;
// 223 with option bvh.collapse = 1).  Every plane stays a multiple of 256 B (bank 0); the 7.5 KiB saved against a 320 cap
// leave room for deeper traversal stacks (the optimal collapse's tree needs 18 entries instead of 15)
#ifndef ART_LDS_NODE_CAP
#define ART_LDS_NODE_CAP 272
#endif
constexpr uint32_t kLdsNodeCap = ART_LDS_NODE_CAP;
constexpr uint32_t kLdsNodePlanes = 10;
constexpr uint32_t kLdsNodePlaneChild = 9;
constexpr uint32_t kLdsSlotCap = 1024;  // leaf slots (= primref array entries): 2 planes (cx, cy), (cz, r) as double2
constexpr uint32_t kLdsMovCap = 512;    // moving spheres (unit shutter, y motion)
// The y motion is a plane of one f64 dy per leaf slot, -0.0 for a static sphere (c.y + tm * -0 == c.y for every c.y
// and tm >= 0, -0 included), so a leaf test loads it beside the sphere planes and runs one branch-free sequence
constexpr uint32_t kLdsOffNodes = 0;
constexpr uint32_t kLdsOffSph = kLdsOffNodes + kLdsNodePlanes * kLdsNodeCap * 16;
constexpr uint32_t kLdsOffMov = kLdsOffSph + 2 * kLdsSlotCap * 16;
// u32 per slot: sphere index (19 bits) | (moving index + 1) << 19 (10 bits) | material type << 29 (3 bits)
constexpr uint32_t kLdsOffRef = kLdsOffMov + kLdsSlotCap * 8;
// Shading table (fused variant): u16 per slot = material entry e | kLdsMatChecker, and kLdsMatCap 32-B entries
// (c.x, c.y), (c.z, param): lambertian / diffuse_light colour (a checker of two solid colours takes entries e = even,
// e + 1 = odd), metal albedo + fuzz, dielectric (-, -, -, ir).  A hit is then shaded without any global load.
constexpr uint32_t kLdsOffMatIdx = kLdsOffRef + kLdsSlotCap * 4;
constexpr uint32_t kLdsMatCap = 512;
constexpr uint32_t kLdsMatChecker = 0x8000u;
constexpr uint32_t kLdsOffMat = kLdsOffMatIdx + kLdsSlotCap * 2;
// 1/r per slot (f64): sphere.h's outward normal (p - c) / r is (1/r) * (p - c) in vec3.h, so the host-side
// reciprocal is the same value the device would compute; the hit test's r*r is precomputed the same way (the
// second sphere plane holds (cz, r*r)).
constexpr uint32_t kLdsOffInvR = kLdsOffMat + kLdsMatCap * 32;
constexpr uint32_t kLdsImageBytes = kLdsOffInvR + kLdsSlotCap * 8;
constexpr uint32_t kLdsRefMovShift = 19;
constexpr uint32_t kLdsRefMatShift = 29;
constexpr uint32_t kMatUnknown = 0xFFu;  // HitOut::mt when the hit did not come from the LDS image
// Child codes in the image: inner node n as 16 * n (its byte offset in a plane), leaf ~((count << 10) | first), empty
// -1 -- all fit the 16-bit LDS
// traversal stack entries of this variant (halving the stack is what lets 1024 lanes share one image).
constexpr uint32_t kLdsLeafShift = 10;
constexpr uint32_t kLdsLeafMaxCount = 31;
ART_HD int32_t lds_leaf(uint32_t first, uint32_t count) { return ~static_cast<int32_t>((count << kLdsLeafShift) | first); }
constexpr uint32_t kLdsRefIndexMask = (1u << kLdsRefMovShift) - 1;
// Empty child slots of the image: a count-0 leaf (distinct from the kNodeEmpty stack sentinel) behind a point box far
// outside any scene, so the traversal needs no per-child empty test.
constexpr int32_t kLdsEmptyChild = ~static_cast<int32_t>(1u);
constexpr float kLdsEmptyBox = 3.0e38f;
static_assert(kLdsMovCap + 1 < (1u << (kLdsRefMatShift - kLdsRefMovShift)), "moving index field");
static_assert(kLdsImageBytes % 16 == 0, "LDS image is copied in 16-B pieces");

// ---------------------------------------------------------------------------------------------- objects
enum ObjKind : int32_t { OBJ_PRIM = 0, OBJ_BVH = 1, OBJ_TRANSLATE = 2, OBJ_ROTATE_Y = 3, OBJ_MEDIUM = 4 };
template <class R>
struct ObjRec {
    int32_t kind;
    int32_t a;      // PRIM: prim ref; BVH: root node; TRANSLATE/ROTATE_Y: child object; MEDIUM: boundary object
    int32_t b;      // MEDIUM: phase material; BVH: leaf code of its hoisted primitives (tested before the tree), or -1
    int32_t pad;
    R p[4];         // TRANSLATE: offset xyz; ROTATE_Y: sin, cos; MEDIUM: neg_inv_density
};
constexpr int kMaxXformChain = 2;  // translate(rotate_y(X)) is the deepest chain in the reference scenes
// Scene features: kernels are instantiated for feature subsets (spheres only / meshes / everything).
// F_MEDIA: constant_medium objects; F_MEDIA_G: one of them has a boundary that is not a sphere primitive (its two
// boundary hits are whole object traversals; a sphere boundary is one quadratic, device.h hit_medium)
enum Feature : uint32_t { F_SPHERE = 1u, F_TRI = 2u, F_RECT = 4u, F_BOX = 8u, F_XFORM = 16u, F_MEDIA = 32u, F_MEDIA_G = 64u, F_ALL = 127u };
// Not a scene feature: an instantiation flag of k_paths_g -- its traversals read the 16-bit child codes and sort packed
// keys (device.h traverse); the scene's codes must all fit (DeviceScene::codes16) and it has no F_MEDIA_G boundary
// traversals (those start at t = -inf, which packed keys cannot order).
constexpr uint32_t F_CODE16 = 128u;
// Not a scene feature either: with F_CODE16, a 16-bit leaf code's `first` counts pairs of primitive references (the
// device copy of the primitive references puts every leaf on an even slot, DeviceScene::leaf_shift 1), so a mesh of up
// to 16384 references -- the capsule, the reference's default scene: 10 200 triangles -- keeps the packed-key
// traversal and the 16-bit stacks instead of the 32-bit-code kernels
constexpr uint32_t F_LEAF2 = 256u;
ART_HD constexpr uint32_t fbase(uint32_t f) { return f & F_ALL; }
constexpr uint32_t kFeatSpheres = F_SPHERE;
constexpr uint32_t kFeatMesh = F_SPHERE | F_TRI | F_RECT | F_MEDIA;

// ---------------------------------------------------------------------------------------------- shading
enum MatType : uint32_t { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_LIGHT = 3, MAT_ISOTROPIC = 4 };
constexpr int kNumMatTypes = 5;
// MATF_NEEDS_UV: its texture tree samples u,v (image / barycentric image).  MATF_SOLID (device records only, set at
// upload): a lambertian / diffuse_light / isotropic whose texture is a solid colour, copied into `albedo` (which only
// metal uses otherwise), so its texture value needs no second dependent load (device.h mat_tex_value)
enum MatFlags : uint32_t { MATF_NEEDS_UV = 1u, MATF_SOLID = 2u };
template <class R>
struct MatRec {
    uint32_t type;
    int32_t tex;    // lambertian / diffuse_light / isotropic
    uint32_t flags;
    uint32_t pad;
    R albedo[3];    // metal
    R fuzz;         // metal (already clamped to <= 1, material.h:47)
    R ir;           // dielectric
};
enum TexType : uint32_t { TEX_SOLID = 0, TEX_CHECKER = 1, TEX_NOISE = 2, TEX_IMAGE = 3, TEX_BARY_IMAGE = 4 };
// Texture kinds present (shade kernels are instantiated for "solid + checker" and "all").
enum TexFeature : uint32_t { TF_SOLID = 1u, TF_CHECKER = 2u, TF_NOISE = 4u, TF_IMAGE = 8u, TF_ALL = 15u };
constexpr uint32_t kTexBasic = TF_SOLID | TF_CHECKER;
// TF_BARY (not in TF_ALL): barycentric image textures on triangles only -- a mesh's map_Kd (mesh.h:9-27,
// texture.h:135-154) -- and no image on any other primitive, so the kernel carries triangle u, v and the texel fetch
// but not get_sphere_uv's acos / atan2 (the capsule's kernel: 20 spilled VGPRs with TF_ALL)
constexpr uint32_t TF_BARY = 16u;
constexpr uint32_t kTexBary = kTexBasic | TF_BARY;
template <class R>
struct TexRec {
    uint32_t type;
    int32_t even, odd;   // checker children
    int32_t perlin;      // noise: perlin table index
    int32_t image;       // image / bary_image: image index
    int32_t pad;
    R c[3];              // solid colour
    R scale;             // noise scale
    R uv[6];             // bary_image texcoords a, b, c
};
template <class R>
struct PerlinRec {       // perlin.h: 256 random unit vectors + 3 permutations
    R ranvec[256][3];
    int32_t perm[3][256];
};
struct ImageRec {
    uint64_t offset;     // into the texel pool
    int32_t w, h, bpp, pad;
};

// ---------------------------------------------------------------------------------------------- camera
template <class R>
struct CameraRec {       // camera.h: precomputed on the host in f64 exactly as camera::camera does
    R origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
    R lens_radius, time0, time1;
};

// ---------------------------------------------------------------------------------------------- band partition
// Row-interleaved bands (the multi-GPU split; ancestor: _run_parallel_stripes' 4 contiguous stripes, engine.h:335-376):
// global row y belongs to band y / band_rows, rendered by band set (y / band_rows) % n.  Local row ly of band set r
// is global row band_global_row(ly, ...); band set r owns band_local_rows(H, ...) rows.  One rule for the kernels
// (kernels.hip global_row), rt_local_rows, the RCCL gather's block size and the unpack (multi.hip).
ART_HD int band_global_row(int ly, int band_rows, int n, int r) {
    return (ly / band_rows) * (band_rows * n) + r * band_rows + (ly % band_rows);
}
ART_HD int band_local_rows(int H, int band_rows, int n, int r) {
    // full cycles of n bands, then the part of band set r's band in the last partial cycle
    const int cycle = band_rows * n, full = H / cycle, rest = H - full * cycle;
    const int tail = rest - r * band_rows;
    return full * band_rows + (tail <= 0 ? 0 : (tail < band_rows ? tail : band_rows));
}
ART_HD int band_block_rows(int H, int band_rows, int n) {  // the largest band set (band set 0 owns the most rows)
    return band_local_rows(H, band_rows, n, 0);
}

}  // namespace art
