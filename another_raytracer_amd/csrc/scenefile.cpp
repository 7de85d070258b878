// scenefile.cpp — flat-scene files (scenefile.h).  The file is mapped read-only (mmap) and every array is copied
// out of the mapping into the FlatScene in one memcpy.
#include "scenefile.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
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
        const uint64_t bytes = h.count[i] * sizeof(T);
        if (h.offset[i] < start || h.offset[i] % 64 || h.count[i] > size || h.offset[i] + bytes > size)
            throw std::runtime_error(path + ": corrupt array table");
        v.resize(h.count[i]);
        if (bytes) std::memcpy(v.data(), base + h.offset[i], bytes);
    });
    f.features = h.features;
    f.has_media = h.has_media != 0;
    f.max_bvh_depth = h.max_bvh_depth;
    f.max_stack = h.max_stack;
    for (int a = 0; a < 3; ++a) {
        f.background[a] = h.background[a];
        view.lookfrom[a] = h.lookfrom[a];
        view.lookat[a] = h.lookat[a];
    }
    view.vfov = h.vfov;
    view.aperture = h.aperture;
    // structural checks the renderer relies on (indices in range)
    const uint32_t nrefs = static_cast<uint32_t>(f.primrefs.size());
    for (const BvhNode& n : f.nodes)
        for (int c = 0; c < 4; ++c) {
            const int32_t ch = n.child[c];
            if (ch >= 0 && static_cast<size_t>(ch) >= f.nodes.size()) throw std::runtime_error(path + ": BVH child out of range");
            if (ch < kNodeEmpty && leaf_first(ch) + leaf_count(ch) > nrefs) throw std::runtime_error(path + ": BVH leaf out of range");
        }
    for (int32_t w : f.world)
        if (w < 0 || static_cast<size_t>(w) >= f.objs.size()) throw std::runtime_error(path + ": world object out of range");
    for (const ObjRec<double>& o : f.objs)
        if (o.kind == OBJ_BVH && (o.a < 0 || static_cast<size_t>(o.a) >= f.nodes.size() ||
                                  (o.b != kNodeEmpty && (o.b >= 0 || leaf_first(o.b) + leaf_count(o.b) > nrefs))))
            throw std::runtime_error(path + ": BVH object out of range");
    for (const ImageRec& im : f.images)
        if (im.offset + static_cast<uint64_t>(im.w) * im.h * im.bpp > f.texels.size()) throw std::runtime_error(path + ": texture out of range");
    flat = std::move(f);
}

}  // namespace art
