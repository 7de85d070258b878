// objmesh.cpp — OBJ/MTL parsing, rapidobj-equivalent triangulation and mesh::build (see objmesh.h).
#include "objmesh.h"

#include <algorithm>
#include <cfloat>
#include <charconv>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string_view>

namespace art {
namespace {

using sv = std::string_view;

bool is_ws(char c) { return c == ' ' || c == '\t'; }
void trim_left(sv& s) {
    while (!s.empty() && is_ws(s.front())) s.remove_prefix(1);
}
void trim(sv& s) {
    trim_left(s);
    while (!s.empty() && is_ws(s.back())) s.remove_suffix(1);
}
// record keyword followed by a blank ("v ", "usemtl\t", ...), as rapidobj's StartsWith(line, "k ") || "k\t"
bool key(sv s, sv k) { return s.size() > k.size() && s.compare(0, k.size(), k) == 0 && is_ws(s[k.size()]); }

[[noreturn]] void parse_error(const std::string& path, size_t line_num, sv line, const char* what) {
    std::ostringstream os;
    os << "cannot parse mesh file " << path << " (error : " << what << ")\n\t -> on line " << line_num << ": \"" << line << "\"";
    throw std::runtime_error(os.str());
}

// Up to max_count blank-separated f32 values (rapidobj ParseReals with fast_float: correctly rounded, like
// std::from_chars<float>).  Returns the count; *rest receives what follows.
size_t parse_floats(sv text, size_t max_count, float* out, sv* rest = nullptr) {
    size_t n = 0;
    while (n < max_count) {
        trim_left(text);
        if (text.empty()) break;
        float v = 0;
        auto [ptr, ec] = std::from_chars(text.data(), text.data() + text.size(), v, std::chars_format::general);
        if (ec != std::errc()) break;
        out[n++] = v;
        text.remove_prefix(static_cast<size_t>(ptr - text.data()));
    }
    if (rest) *rest = text;
    return n;
}

// One face-vertex index (rapidobj ParseFace, rapidobj.hpp:5468-5600): 1-based, negative = relative to the count so
// far; 0 is an error.
bool parse_index(sv& text, size_t count, int32_t& out) {
    int v = 0;
    auto [ptr, ec] = std::from_chars(text.data(), text.data() + text.size(), v);
    if (ec != std::errc()) return false;
    text.remove_prefix(static_cast<size_t>(ptr - text.data()));
    if (v > 0) out = v - 1;
    else if (v < 0) out = v + static_cast<int>(count);
    else return false;
    return out >= 0 && static_cast<size_t>(out) < count;
}

// ParseMaterialLibrary (rapidobj.hpp:5760-5990), the records mesh.h reads.
std::vector<ObjMaterial> load_mtl(const std::string& path, std::map<std::string, int>& ids) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot parse mesh file (error : material library not found: " + path + ")");
    std::vector<ObjMaterial> mats;
    std::string raw;
    size_t line_num = 0;
    while (std::getline(f, raw)) {
        ++line_num;
        sv line(raw);
        if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
        trim(line);
        if (line.empty() || line.front() == '#') continue;
        if (key(line, "newmtl")) {
            line.remove_prefix(7);
            trim(line);
            ObjMaterial m;
            m.name = std::string(line);
            ids.try_emplace(m.name, static_cast<int>(mats.size()));
            mats.push_back(std::move(m));
        } else if (mats.empty()) {
            continue;  // records before the first newmtl belong to no material
        } else if (key(line, "Ka") || key(line, "Kd")) {
            float* dst = line[1] == 'a' ? mats.back().ka : mats.back().kd;
            if (parse_floats(line.substr(3), 3, dst) != 3) parse_error(path, line_num, line, "bad colour");
        } else if (key(line, "map_Kd")) {
            line.remove_prefix(7);
            trim(line);
            // texture options (-s, -o, ...) precede the file name; the reference's MTL carries none
            if (!line.empty() && line.front() == '-') parse_error(path, line_num, line, "map_Kd options are not supported");
            mats.back().map_kd = std::string(line);
        }
    }
    return mats;
}

// ------------------------------------------------------------------------------------------------ earcut
// mapbox earcut v2.2.4 (rapidobj.hpp:497-1166) for one ring, on an index-linked node pool.  Polygons above 80
// vertices use the z-order hashed ear test there (isEarHashed); it tests the same predicate on the subset of nodes
// inside the ear's bounding box, which contains every node the full test could reject on, so the unhashed test is
// used for every size.
struct Earcut {
    struct Node {
        uint32_t i;
        double x, y;
        int prev, next;
    };
    std::vector<Node> n;
    std::vector<uint32_t> out;

    int construct(uint32_t i, double x, double y) {
        n.push_back(Node{i, x, y, -1, -1});
        return static_cast<int>(n.size()) - 1;
    }
    int insert(uint32_t i, double x, double y, int last) {
        const int p = construct(i, x, y);
        if (last < 0) {
            n[p].prev = n[p].next = p;
        } else {
            n[p].next = n[last].next;
            n[p].prev = last;
            n[n[last].next].prev = p;
            n[last].next = p;
        }
        return p;
    }
    void remove(int p) {
        n[n[p].next].prev = n[p].prev;
        n[n[p].prev].next = n[p].next;
    }
    double area(int p, int q, int r) const {
        return (n[q].y - n[p].y) * (n[r].x - n[q].x) - (n[q].x - n[p].x) * (n[r].y - n[q].y);
    }
    bool equals(int a, int b) const { return n[a].x == n[b].x && n[a].y == n[b].y; }
    static bool in_triangle(double ax, double ay, double bx, double by, double cx, double cy, double px, double py) {
        return (cx - px) * (ay - py) >= (ax - px) * (cy - py) && (ax - px) * (by - py) >= (bx - px) * (ay - py) &&
               (bx - px) * (cy - py) >= (cx - px) * (by - py);
    }
    static int sign(double v) { return (0.0 < v) - (v < 0.0); }
    bool on_segment(int p, int q, int r) const {
        return n[q].x <= std::max(n[p].x, n[r].x) && n[q].x >= std::min(n[p].x, n[r].x) && n[q].y <= std::max(n[p].y, n[r].y) &&
               n[q].y >= std::min(n[p].y, n[r].y);
    }
    bool intersects(int p1, int q1, int p2, int q2) const {
        const int o1 = sign(area(p1, q1, p2)), o2 = sign(area(p1, q1, q2));
        const int o3 = sign(area(p2, q2, p1)), o4 = sign(area(p2, q2, q1));
        if (o1 != o2 && o3 != o4) return true;
        if (o1 == 0 && on_segment(p1, p2, q1)) return true;
        if (o2 == 0 && on_segment(p1, q2, q1)) return true;
        if (o3 == 0 && on_segment(p2, p1, q2)) return true;
        if (o4 == 0 && on_segment(p2, q1, q2)) return true;
        return false;
    }
    bool intersects_polygon(int a, int b) const {
        int p = a;
        do {
            const int q = n[p].next;
            if (n[p].i != n[a].i && n[q].i != n[a].i && n[p].i != n[b].i && n[q].i != n[b].i && intersects(p, q, a, b)) return true;
            p = q;
        } while (p != a);
        return false;
    }
    bool locally_inside(int a, int b) const {
        return area(n[a].prev, a, n[a].next) < 0 ? area(a, b, n[a].next) >= 0 && area(a, n[a].prev, b) >= 0
                                                 : area(a, b, n[a].prev) < 0 || area(a, n[a].next, b) < 0;
    }
    bool middle_inside(int a, int b) const {
        int p = a;
        bool inside = false;
        const double px = (n[a].x + n[b].x) / 2, py = (n[a].y + n[b].y) / 2;
        do {
            const int q = n[p].next;
            if (((n[p].y > py) != (n[q].y > py)) && n[q].y != n[p].y && (px < (n[q].x - n[p].x) * (py - n[p].y) / (n[q].y - n[p].y) + n[p].x))
                inside = !inside;
            p = q;
        } while (p != a);
        return inside;
    }
    bool valid_diagonal(int a, int b) const {
        return n[n[a].next].i != n[b].i && n[n[a].prev].i != n[b].i && !intersects_polygon(a, b) &&
               ((locally_inside(a, b) && locally_inside(b, a) && middle_inside(a, b) &&
                 (area(n[a].prev, a, n[b].prev) != 0.0 || area(a, n[b].prev, b) != 0.0)) ||
                (equals(a, b) && area(n[a].prev, a, n[a].next) > 0 && area(n[b].prev, b, n[b].next) > 0));
    }
    bool is_ear(int ear) const {
        const int a = n[ear].prev, b = ear, c = n[ear].next;
        if (area(a, b, c) >= 0) return false;  // reflex
        for (int p = n[c].next; p != a; p = n[p].next)
            if (in_triangle(n[a].x, n[a].y, n[b].x, n[b].y, n[c].x, n[c].y, n[p].x, n[p].y) && area(n[p].prev, p, n[p].next) >= 0) return false;
        return true;
    }
    int filter_points(int start, int end = -1) {
        if (end < 0) end = start;
        int p = start;
        bool again;
        do {
            again = false;
            if (equals(p, n[p].next) || area(n[p].prev, p, n[p].next) == 0) {
                remove(p);
                p = end = n[p].prev;
                if (p == n[p].next) break;
                again = true;
            } else {
                p = n[p].next;
            }
        } while (again || p != end);
        return end;
    }
    int cure_local_intersections(int start) {
        int p = start;
        do {
            const int a = n[p].prev, b = n[n[p].next].next;
            if (!equals(a, b) && intersects(a, p, n[p].next, b) && locally_inside(a, b) && locally_inside(b, a)) {
                out.push_back(n[a].i);
                out.push_back(n[p].i);
                out.push_back(n[b].i);
                remove(p);
                remove(n[p].next);
                p = start = b;
            }
            p = n[p].next;
        } while (p != start);
        return filter_points(p);
    }
    int split_polygon(int a, int b) {
        const int a2 = construct(n[a].i, n[a].x, n[a].y);
        const int b2 = construct(n[b].i, n[b].x, n[b].y);
        const int an = n[a].next, bp = n[b].prev;
        n[a].next = b;
        n[b].prev = a;
        n[a2].next = an;
        n[an].prev = a2;
        n[b2].next = a2;
        n[a2].prev = b2;
        n[bp].next = b2;
        n[b2].prev = bp;
        return b2;
    }
    void split_earcut(int start) {
        int a = start;
        do {
            int b = n[n[a].next].next;
            while (b != n[a].prev) {
                if (n[a].i != n[b].i && valid_diagonal(a, b)) {
                    int c = split_polygon(a, b);
                    a = filter_points(a, n[a].next);
                    c = filter_points(c, n[c].next);
                    earcut_linked(a, 0);
                    earcut_linked(c, 0);
                    return;
                }
                b = n[b].next;
            }
            a = n[a].next;
        } while (a != start);
    }
    void earcut_linked(int ear, int pass) {
        if (ear < 0) return;
        int stop = ear;
        while (n[ear].prev != n[ear].next) {
            const int prev = n[ear].prev, next = n[ear].next;
            if (is_ear(ear)) {
                out.push_back(n[prev].i);
                out.push_back(n[ear].i);
                out.push_back(n[next].i);
                remove(ear);
                ear = n[next].next;  // skipping the next vertex leads to fewer sliver triangles
                stop = n[next].next;
                continue;
            }
            ear = next;
            if (ear == stop) {
                if (pass == 0) {
                    earcut_linked(filter_points(ear), 1);
                } else if (pass == 1) {
                    ear = cure_local_intersections(filter_points(ear));
                    earcut_linked(ear, 2);
                } else if (pass == 2) {
                    split_earcut(ear);
                }
                break;
            }
        }
    }
};

}  // namespace

std::vector<uint32_t> earcut_ring(const std::vector<double>& xy) {
    Earcut e;
    const size_t len = xy.size() / 2;
    if (len == 0) return {};
    e.n.reserve(len * 3 / 2 + 8);
    // linkedList(points, clockwise = true) (rapidobj.hpp:551-586): orientation from the shoelace sum
    double sum = 0;
    for (size_t i = 0, j = len - 1; i < len; j = i++) sum += (xy[2 * j] - xy[2 * i]) * (xy[2 * i + 1] + xy[2 * j + 1]);
    int last = -1;
    if (sum > 0) {
        for (size_t i = 0; i < len; i++) last = e.insert(static_cast<uint32_t>(i), xy[2 * i], xy[2 * i + 1], last);
    } else {
        for (size_t i = len; i-- > 0;) last = e.insert(static_cast<uint32_t>(i), xy[2 * i], xy[2 * i + 1], last);
    }
    if (last >= 0 && e.equals(last, e.n[last].next)) {
        e.remove(last);
        last = e.n[last].next;
    }
    if (last < 0 || e.n[last].prev == e.n[last].next) return {};
    e.earcut_linked(last, 0);
    return e.out;
}

namespace {

// CalculatePolygonArea (rapidobj.hpp:7118-7133), in f32 as there.
float polygon_area(const float* x, const float* y, size_t size) {
    float area = 0.0f;
    for (size_t i = 1; i != size; ++i) {
        const float avg_height = (y[i - 1] + y[i]) / 2;
        const float width = x[i] - x[i - 1];
        area += width * avg_height;
    }
    const float avg_height = (y[0] + y[size - 1]) / 2;
    const float width = x[0] - x[size - 1];
    area += width * avg_height;
    return std::abs(area);
}

// TriangulateSingleTask (rapidobj.hpp:7137-7302) for one face: appends its triangles to out.
bool triangulate_face(const std::vector<float>& pos, const ObjIndex* f, size_t nv, std::vector<ObjIndex>& out) {
    if (nv == 3) {
        out.insert(out.end(), f, f + 3);
        return true;
    }
    auto P = [&](const ObjIndex& k, int c) { return pos[3 * static_cast<size_t>(k.p) + c]; };
    if (nv == 4) {  // split along the shorter diagonal (f32 squared lengths)
        const float e02x = P(f[0], 0) - P(f[2], 0), e02y = P(f[0], 1) - P(f[2], 1), e02z = P(f[0], 2) - P(f[2], 2);
        const float e13x = P(f[1], 0) - P(f[3], 0), e13y = P(f[1], 1) - P(f[3], 1), e13z = P(f[1], 2) - P(f[3], 2);
        const float d02 = e02x * e02x + e02y * e02y + e02z * e02z;
        const float d13 = e13x * e13x + e13y * e13y + e13z * e13z;
        const bool d02_less = d02 < d13;
        out.push_back(f[0]);
        out.push_back(f[1]);
        out.push_back(d02_less ? f[2] : f[3]);
        out.push_back(d02_less ? f[0] : f[1]);
        out.push_back(f[2]);
        out.push_back(f[3]);
        return true;
    }
    std::vector<float> xs(nv), ys(nv), zs(nv);
    for (size_t k = 0; k < nv; ++k) {
        xs[k] = P(f[k], 0);
        ys[k] = P(f[k], 1);
        zs[k] = P(f[k], 2);
    }
    const float ax = polygon_area(ys.data(), zs.data(), nv);
    const float ay = polygon_area(xs.data(), zs.data(), nv);
    const float az = polygon_area(xs.data(), ys.data(), nv);
    if (FLT_MIN > std::max({ax, ay, az})) return false;
    const int plane = ax > ay ? (ax > az ? 0 : 2) : (ay > az ? 1 : 2);
    std::vector<double> xy(2 * nv);
    for (size_t k = 0; k < nv; ++k) {
        xy[2 * k] = plane == 0 ? ys[k] : xs[k];
        xy[2 * k + 1] = plane == 2 ? ys[k] : zs[k];
    }
    std::vector<uint32_t> r = earcut_ring(xy);
    if (r.empty() || r.size() % 3 != 0) return false;
    for (size_t k = 0; k < r.size(); k += 3) std::swap(r[k], r[k + 1]);
    for (uint32_t idx : r) out.push_back(f[idx]);
    return true;
}

std::string dir_of(const std::string& path) {
    const size_t s = path.find_last_of('/');
    return s == std::string::npos ? std::string(".") : (s == 0 ? std::string("/") : path.substr(0, s));
}

}  // namespace

ObjMesh load_obj(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot parse mesh file " + path + " (error : file not found)");
    ObjMesh m;
    m.dir = dir_of(path);
    size_t ntex = 0, nnorm = 0;
    std::vector<ObjIndex> face_idx;      // all face vertices, file order
    std::vector<uint8_t> face_nv;        // vertices per face
    std::vector<size_t> shape_start{0};  // face index where each shape record starts (record 0: the implicit one)
    std::vector<std::pair<std::string, size_t>> usemtl;  // (name, first face)
    std::string mtllib;
    std::string raw;
    size_t line_num = 0;
    while (std::getline(f, raw)) {
        ++line_num;
        sv line(raw);
        if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
        const sv text = line;
        trim_left(line);
        if (line.empty()) continue;
        switch (line.front()) {
            case 'v': {
                float v[7];
                if (key(line, "v")) {  // ParsePosition: x y z [w | r g b]
                    sv rest;
                    const size_t c = parse_floats(line.substr(2), 7, v, &rest);
                    trim_left(rest);
                    if ((c != 3 && c != 4 && c != 6 && c != 7) || !rest.empty()) parse_error(path, line_num, text, "bad vertex");
                    m.positions.insert(m.positions.end(), v, v + 3);
                } else if (key(line, "vt")) {
                    const size_t c = parse_floats(line.substr(3), 3, v);
                    if (c < 2) parse_error(path, line_num, text, "bad texture vertex");
                    m.texcoords.insert(m.texcoords.end(), v, v + 2);
                    ++ntex;
                } else if (key(line, "vn")) {
                    if (parse_floats(line.substr(3), 3, v) < 3) parse_error(path, line_num, text, "bad normal");
                    ++nnorm;
                } else {
                    parse_error(path, line_num, text, "unknown record");
                }
                break;
            }
            case 'f': {
                if (!key(line, "f")) break;
                sv s = line.substr(2);
                size_t nv = 0;
                const size_t npos_count = m.positions.size() / 3;
                for (;;) {
                    trim_left(s);
                    if (s.empty()) break;
                    ObjIndex k;
                    if (!parse_index(s, npos_count, k.p)) parse_error(path, line_num, text, "bad position index");
                    if (!s.empty() && s.front() == '/') {
                        s.remove_prefix(1);
                        if (s.empty()) parse_error(path, line_num, text, "bad face");
                        if (s.front() != '/' && !parse_index(s, ntex, k.t)) parse_error(path, line_num, text, "bad texcoord index");
                        if (!s.empty() && s.front() == '/') {
                            s.remove_prefix(1);
                            if (!parse_index(s, nnorm, k.n)) parse_error(path, line_num, text, "bad normal index");
                        }
                    }
                    if (!s.empty() && !is_ws(s.front())) parse_error(path, line_num, text, "bad face");
                    face_idx.push_back(k);
                    ++nv;
                }
                if (nv < 3 || nv > 255) parse_error(path, line_num, text, "bad face vertex count");
                face_nv.push_back(static_cast<uint8_t>(nv));
                break;
            }
            case 'g':
            case 'o':
                if (!key(line, "g") && !key(line, "o")) parse_error(path, line_num, text, "unknown record");
                shape_start.push_back(face_nv.size());
                break;
            case 'm':
                if (key(line, "mtllib")) {
                    sv name = line.substr(7);
                    trim(name);
                    if (mtllib.empty()) mtllib = std::string(name);
                    else if (mtllib != name) parse_error(path, line_num, text, "ambiguous material library");
                }
                break;
            case 'u':
                if (key(line, "usemtl")) {
                    sv name = line.substr(7);  // the rest of the line, as rapidobj keeps it (rapidobj.hpp:6696-6701)
                    if (!usemtl.empty() && usemtl.back().second == face_nv.size()) usemtl.pop_back();
                    usemtl.emplace_back(std::string(name), face_nv.size());
                }
                break;
            default:  // comments, smoothing groups, lines, points: nothing mesh.h reads
                break;
        }
    }
    m.faces = face_nv.size();
    shape_start.push_back(face_nv.size());
    for (size_t s = 0; s + 1 < shape_start.size(); ++s) m.shapes += shape_start[s + 1] > shape_start[s];

    // materials per face (Merge, rapidobj.hpp:6266-6296): the last usemtl at or before the face, -1 before any
    std::map<std::string, int> ids;
    if (!mtllib.empty()) m.materials = load_mtl(m.dir + "/" + mtllib, ids);
    std::vector<int32_t> face_mat(face_nv.size(), -1);
    for (size_t r = 0; r < usemtl.size(); ++r) {
        auto it = ids.find(usemtl[r].first);
        if (it == ids.end()) throw std::runtime_error("cannot parse mesh file " + path + " (error : material not found: " + usemtl[r].first + ")");
        const size_t end = r + 1 < usemtl.size() ? usemtl[r + 1].second : face_nv.size();
        for (size_t fi = usemtl[r].second; fi < end; ++fi) face_mat[fi] = it->second;
    }

    // rapidobj::Triangulate
    size_t at = 0;
    for (size_t fi = 0; fi < face_nv.size(); ++fi) {
        const size_t before = m.tri.size();
        if (!triangulate_face(m.positions, &face_idx[at], face_nv[fi], m.tri))
            throw std::runtime_error("cannot triangulate parsed mesh file " + path);
        for (size_t t = before / 3; t < m.tri.size() / 3; ++t) m.tri_mat.push_back(face_mat[fi]);
        at += face_nv[fi];
    }
    return m;
}

std::vector<int> build_mesh(SceneGraph& g, const ObjMesh& m) {
    std::map<std::string, int> maps;  // material_map_handler (mesh.h:9-27): one image texture per map name
    auto vert = [&](const ObjIndex& k) {  // get_vertice_by_index (mesh.h:76-82): f32 -> f64
        const size_t b = 3 * static_cast<size_t>(k.p);
        return Vec3(m.positions[b], m.positions[b + 1], m.positions[b + 2]);
    };
    std::vector<int> ids;
    ids.reserve(m.tri.size() / 3);
    for (size_t t = 0; t < m.tri.size() / 3; ++t) {
        const ObjIndex& a = m.tri[3 * t];
        const ObjIndex& b = m.tri[3 * t + 1];
        const ObjIndex& c = m.tri[3 * t + 2];
        int mat;
        if (!m.materials.empty()) {
            const int32_t id = m.tri_mat[t];
            if (id < 0) throw std::runtime_error("mesh triangle without a material in a mesh with a material library");
            const ObjMaterial& mm = m.materials[static_cast<size_t>(id)];
            if (!mm.map_kd.empty()) {
                auto it = maps.find(mm.map_kd);
                if (it == maps.end()) {
                    // material_map_handler (mesh.h:9-27): image_texture(dir + map_Kd), decoded from the file itself
                    it = maps.emplace(mm.map_kd, g.image_file(m.dir + "/" + mm.map_kd)).first;
                }
                if (a.t < 0 || b.t < 0 || c.t < 0) throw std::runtime_error("textured mesh face without texture coordinates");
                auto uv = [&](const ObjIndex& k, int cpt) { return static_cast<double>(m.texcoords[2 * static_cast<size_t>(k.t) + cpt]); };
                const int tex = g.bary_image(uv(a, 0), uv(a, 1), uv(b, 0), uv(b, 1), uv(c, 0), uv(c, 1), it->second);
                mat = g.lambertian(tex);
            } else {  // color(Ka[0]+Kd[0], ...): f32 sums
                mat = g.lambertian_color(Vec3(mm.ka[0] + mm.kd[0], mm.ka[1] + mm.kd[1], mm.ka[2] + mm.kd[2]));
            }
        } else {
            mat = g.lambertian_color(g.rng.vec01());  // color::random()
        }
        ids.push_back(g.triangle(vert(a), vert(b), vert(c), mat));
    }
    return ids;
}

}  // namespace art
