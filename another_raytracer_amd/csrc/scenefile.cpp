// scenefile.cpp — flat-scene files (scenefile.h).  The file is mapped read-only (mmap) and every array is copied
// out of the mapping into the FlatScene in one memcpy.
#include "scenefile.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace art {
namespace {

constexpr char kMagic[8] = {'A', 'R', 'T', 'S', 'C', 'N', '\0', '\1'};
enum Array { A_SPHERES, A_TRIS, A_RECTS, A_BOXES, A_PRIMREFS, A_NODES, A_OBJS, A_WORLD, A_MATS, A_TEXS, A_PERLINS, A_IMAGES, A_TEXELS, kArrays };

struct FileHeader {
    char magic[8];
    uint32_t version;
    uint32_t header_bytes;
    uint32_t record_bytes[kArrays];  // sizeof of each array's element: a layout change is refused, not misread
    uint32_t features;
    int32_t has_media, max_bvh_depth, max_stack;
    double background[3];
    double lookfrom[3], lookat[3], vfov, aperture;
    uint64_t offset[kArrays], count[kArrays];
    uint64_t payload_bytes;
    uint64_t checksum;  // FNV-1a 64 over the payload (every byte after the header)
};

template <class T>
constexpr uint32_t rec() { return static_cast<uint32_t>(sizeof(T)); }
const uint32_t kRecordBytes[kArrays] = {rec<SphereRec<double>>(), rec<TriRec<double>>(), rec<RectRec<double>>(), rec<BoxRec<double>>(),
                                        rec<uint32_t>(),          rec<BvhNode>(),        rec<ObjRec<double>>(),  rec<int32_t>(),
                                        rec<MatRec<double>>(),    rec<TexRec<double>>(), rec<PerlinRec<double>>(), rec<ImageRec>(),
                                        rec<uint8_t>()};

uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
inline uint64_t align64(uint64_t x) { return (x + 63) & ~uint64_t(63); }

template <class F>
void for_arrays(FlatScene& f, F&& fn) {  // fn(index, vector&)
    fn(A_SPHERES, f.spheres);
    fn(A_TRIS, f.tris);
    fn(A_RECTS, f.rects);
    fn(A_BOXES, f.boxes);
    fn(A_PRIMREFS, f.primrefs);
    fn(A_NODES, f.nodes);
    fn(A_OBJS, f.objs);
    fn(A_WORLD, f.world);
    fn(A_MATS, f.mats);
    fn(A_TEXS, f.texs);
    fn(A_PERLINS, f.perlins);
    fn(A_IMAGES, f.images);
    fn(A_TEXELS, f.texels);
}

[[noreturn]] void bad(const std::string& path, const char* what) { throw std::runtime_error(path + ": " + what); }

// Every index the renderer follows, checked against the arrays; the derived fields (features, has_media, max_stack,
// max_bvh_depth) recomputed as compile_scene computes them (scene.cpp, bvh.cpp collapse).  Nodes are stored level-major
// (scene.cpp relabel_level_major): an inner child's index is above its parent's, so the tree is acyclic by check.
void validate(const std::string& path, FlatScene& f) {
    const size_t nsph = f.spheres.size(), ntri = f.tris.size(), nrect = f.rects.size(), nbox = f.boxes.size();
    const size_t nmat = f.mats.size(), ntex = f.texs.size(), nobj = f.objs.size(), nref = f.primrefs.size();
    auto ref_ok = [&](uint32_t r) {
        const uint32_t i = primref_index(r);
        switch (primref_type(r)) {
            case PRIM_SPHERE: return i < nsph;
            case PRIM_TRIANGLE: return i < ntri;
            case PRIM_RECT: return i < nrect;
            default: return i < nbox;
        }
    };
    auto leaf_ok = [&](int32_t c) { return c < kNodeEmpty && static_cast<uint64_t>(leaf_first(c)) + leaf_count(c) <= nref; };
    for (uint32_t r : f.primrefs)
        if (!ref_ok(r)) bad(path, "primitive reference out of range");
    for (const auto& s : f.spheres)
        if (s.mat >= nmat) bad(path, "sphere material out of range");
    for (const auto& t : f.tris)
        if (t.mat >= nmat) bad(path, "triangle material out of range");
    for (const auto& r : f.rects)
        if (r.mat >= nmat || r.axis > 2) bad(path, "rect material or axis out of range");
    for (const auto& b : f.boxes)
        if (b.mat >= nmat) bad(path, "box material out of range");
    for (const auto& m : f.mats) {
        if (m.type >= static_cast<uint32_t>(kNumMatTypes)) bad(path, "unknown material type");
        const bool textured = m.type == MAT_LAMBERTIAN || m.type == MAT_LIGHT || m.type == MAT_ISOTROPIC;
        if (textured && (m.tex < 0 || static_cast<size_t>(m.tex) >= ntex)) bad(path, "material texture out of range");
    }
    for (size_t t = 0; t < ntex; ++t) {
        const auto& x = f.texs[t];
        switch (x.type) {
            case TEX_SOLID: break;
            case TEX_CHECKER:  // children are built before the checker (scene.cpp): no texture cycles
                if (x.even < 0 || x.odd < 0 || static_cast<size_t>(x.even) >= t || static_cast<size_t>(x.odd) >= t)
                    bad(path, "checker child out of range");
                break;
            case TEX_NOISE:
                if (x.perlin < 0 || static_cast<size_t>(x.perlin) >= f.perlins.size()) bad(path, "noise table out of range");
                break;
            case TEX_IMAGE:
            case TEX_BARY_IMAGE:
                if (x.image < 0 || static_cast<size_t>(x.image) >= f.images.size()) bad(path, "texture image out of range");
                break;
            default: bad(path, "unknown texture type");
        }
    }
    for (const auto& p : f.perlins)
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 256; ++i)
                if (p.perm[k][i] < 0 || p.perm[k][i] > 255) bad(path, "perlin permutation out of range");
    for (const ImageRec& im : f.images)
        if (im.w <= 0 || im.h <= 0 || im.bpp < 1 || im.bpp > 4 || im.offset > f.texels.size() ||
            static_cast<uint64_t>(im.w) * static_cast<uint64_t>(im.h) * static_cast<uint64_t>(im.bpp) > f.texels.size() - im.offset)
            bad(path, "texture image out of range");
    // BVH: children below their parent in level-major order, leaves within the primrefs; stack and depth bounds
    const size_t nn = f.nodes.size();
    std::vector<int> stack(nn, 0), depth(nn, 0);
    for (size_t k = nn; k-- > 0;) {
        const BvhNode& n = f.nodes[k];
        int kids = 0, cs = 0, cd = 0;
        for (int c = 0; c < 4; ++c) {
            const int32_t ch = n.child[c];
            if (ch == kNodeEmpty) {
                // an empty slot must carry a box no ray enters (lo > hi on every axis: bvh.cpp writes +FLT_MAX /
                // -FLT_MAX): the traversal's key tests have no per-child empty check (device.h slab4_nf, slab4_packed_nf)
                if (!(n.lox[c] > n.hix[c] && n.loy[c] > n.hiy[c] && n.loz[c] > n.hiz[c])) bad(path, "empty BVH slot with an enterable box");
                continue;
            }
            ++kids;
            if (ch >= 0) {
                if (static_cast<size_t>(ch) <= k || static_cast<size_t>(ch) >= nn) bad(path, "BVH child out of range");
                cs = std::max(cs, stack[ch]);
                cd = std::max(cd, depth[ch]);
            } else if (!leaf_ok(ch)) {
                bad(path, "BVH leaf out of range");
            }
        }
        if (kids == 0) bad(path, "BVH node without children");
        stack[k] = kids - 1 + cs;
        depth[k] = 1 + cd;
    }
    // objects: children compiled before their parent (scene.cpp: obj() recursion), so chains are acyclic by check
    f.has_media = false;
    f.max_stack = f.max_bvh_depth = 0;
    uint32_t feat = (nsph ? F_SPHERE : 0u) | (ntri ? F_TRI : 0u) | (nrect ? F_RECT : 0u) | (nbox ? F_BOX : 0u);
    std::vector<int> chain(nobj, 0);
    for (size_t k = 0; k < nobj; ++k) {
        const ObjRec<double>& o = f.objs[k];
        switch (o.kind) {
            case OBJ_PRIM:
                if (!ref_ok(static_cast<uint32_t>(o.a))) bad(path, "primitive object out of range");
                break;
            case OBJ_BVH: {
                // a single-leaf BVH's root node holds one real child and no stack entries (bvh.cpp build_sah_bvh)
                if (o.a < 0 || static_cast<size_t>(o.a) >= nn) bad(path, "BVH object out of range");
                if (o.b != kNodeEmpty && !leaf_ok(o.b)) bad(path, "BVH object out of range (hoisted leaf)");
                f.max_stack = std::max(f.max_stack, stack[o.a]);
                f.max_bvh_depth = std::max(f.max_bvh_depth, depth[o.a]);
                break;
            }
            case OBJ_TRANSLATE:
            case OBJ_ROTATE_Y:
                if (o.a < 0 || static_cast<size_t>(o.a) >= k) bad(path, "instance child out of range");
                if (f.objs[o.a].kind == OBJ_MEDIUM) bad(path, "instance of a medium");
                chain[k] = 1 + chain[o.a];
                if (chain[k] > kMaxXformChain) bad(path, "more than two nested translate/rotate_y instances");
                feat |= F_XFORM;
                break;
            case OBJ_MEDIUM: {
                if (o.a < 0 || static_cast<size_t>(o.a) >= k) bad(path, "medium boundary out of range");
                if (o.b < 0 || static_cast<size_t>(o.b) >= nmat) bad(path, "medium phase material out of range");
                const ObjRec<double>& b = f.objs[o.a];
                if (b.kind == OBJ_MEDIUM) bad(path, "medium boundary is a medium");
                if (!(b.kind == OBJ_PRIM && primref_type(static_cast<uint32_t>(b.a)) == PRIM_SPHERE)) feat |= F_MEDIA_G;
                f.has_media = true;
                break;
            }
            default: bad(path, "unknown object kind");
        }
    }
    if (f.has_media) feat |= F_MEDIA;
    f.features = feat;
    if (f.max_stack > kMaxStackDepth) bad(path, "BVH needs a deeper traversal stack than kMaxStackDepth");
    if (f.world.empty()) bad(path, "empty world");
    for (int32_t w : f.world)
        if (w < 0 || static_cast<size_t>(w) >= nobj) bad(path, "world object out of range");
}

}  // namespace

void save_scene_file(const std::string& path, const FlatScene& flat_in, const SceneView& view) {
    FlatScene& flat = const_cast<FlatScene&>(flat_in);  // for_arrays only reads here
    FileHeader h{};
    std::memcpy(h.magic, kMagic, 8);
    h.version = kSceneFileVersion;
    h.header_bytes = sizeof(FileHeader);
    std::memcpy(h.record_bytes, kRecordBytes, sizeof kRecordBytes);
    h.features = flat.features;
    h.has_media = flat.has_media ? 1 : 0;
    h.max_bvh_depth = flat.max_bvh_depth;
    h.max_stack = flat.max_stack;
    for (int a = 0; a < 3; ++a) {
        h.background[a] = flat.background[a];
        h.lookfrom[a] = view.lookfrom[a];
        h.lookat[a] = view.lookat[a];
    }
    h.vfov = view.vfov;
    h.aperture = view.aperture;
    uint64_t at = align64(sizeof(FileHeader));
    const uint64_t start = at;
    std::vector<uint8_t> payload;
    for_arrays(flat, [&](int i, auto& v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        h.offset[i] = at;
        h.count[i] = v.size();
        const uint64_t bytes = v.size() * sizeof(T);
        payload.resize(at + bytes - start, 0);
        if (bytes) std::memcpy(payload.data() + (at - start), v.data(), bytes);
        at = align64(at + bytes);
        payload.resize(at - start, 0);
    });
    h.payload_bytes = payload.size();
    h.checksum = fnv1a(payload.data(), payload.size());
    std::vector<uint8_t> head(start, 0);
    std::memcpy(head.data(), &h, sizeof h);
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + tmp);
    const bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size() &&
                    std::fwrite(payload.data(), 1, payload.size(), f) == payload.size();
    if (std::fclose(f) != 0 || !ok) {
        std::remove(tmp.c_str());
        throw std::runtime_error("short write to " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp + " to " + path);
}

void load_scene_file(const std::string& path, FlatScene& flat, SceneView& view) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open scene file " + path);
    struct stat st {};
    if (::fstat(fd, &st) != 0 || st.st_size < static_cast<off_t>(sizeof(FileHeader))) {
        ::close(fd);
        throw std::runtime_error(path + ": not a scene file (too short)");
    }
    const size_t size = static_cast<size_t>(st.st_size);
    void* map = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (map == MAP_FAILED) throw std::runtime_error("cannot map scene file " + path);
    const uint8_t* base = static_cast<const uint8_t*>(map);
    struct Unmap {
        void* p;
        size_t n;
        ~Unmap() { ::munmap(p, n); }
    } unmap{map, size};
    FileHeader h;
    std::memcpy(&h, base, sizeof h);
    if (std::memcmp(h.magic, kMagic, 8) != 0) throw std::runtime_error(path + ": not a scene file (bad magic)");
    if (h.version != kSceneFileVersion || h.header_bytes != sizeof(FileHeader))
        throw std::runtime_error(path + ": scene file version " + std::to_string(h.version) + ", this library reads version " +
                                 std::to_string(kSceneFileVersion));
    if (std::memcmp(h.record_bytes, kRecordBytes, sizeof kRecordBytes) != 0)
        throw std::runtime_error(path + ": scene file written with another record layout");
    const uint64_t start = align64(sizeof(FileHeader));
    if (size < start || size - start != h.payload_bytes) throw std::runtime_error(path + ": truncated scene file");
    if (fnv1a(base + start, h.payload_bytes) != h.checksum) throw std::runtime_error(path + ": scene file checksum mismatch");
    FlatScene f;
    for_arrays(f, [&](int i, auto& v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        // the header is outside the checksum: no sum below may wrap
        if (h.offset[i] < start || h.offset[i] % 64 || h.offset[i] > size || h.count[i] > (size - h.offset[i]) / sizeof(T))
            throw std::runtime_error(path + ": corrupt array table");
        const uint64_t bytes = h.count[i] * sizeof(T);
        v.resize(h.count[i]);
        if (bytes) std::memcpy(v.data(), base + h.offset[i], bytes);
    });
    for (int a = 0; a < 3; ++a) {
        f.background[a] = h.background[a];
        view.lookfrom[a] = h.lookfrom[a];
        view.lookat[a] = h.lookat[a];
    }
    view.vfov = h.vfov;
    view.aperture = h.aperture;
    validate(path, f);
    // the header's derived fields must be what the arrays imply (the renderer sizes the LDS traversal stacks by
    // max_stack and instantiates kernels by the feature bits)
    if (h.features != f.features || (h.has_media != 0) != f.has_media || h.max_stack != f.max_stack || h.max_bvh_depth != f.max_bvh_depth)
        throw std::runtime_error(path + ": header fields disagree with the arrays");
    flat = std::move(f);
}

}  // namespace art
