// bvh.cpp — binned SAH builder (see bvh.h).
#include "bvh.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace art {

namespace {

constexpr int kBins = 16;
constexpr double kCostTraverse = 1.0;
constexpr double kCostIntersect = 1.5;

double area(const AABBd& b) {
    double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0;
    return 2 * (dx * dy + dy * dz + dz * dx);
}
AABBd empty_box() {
    const double inf = std::numeric_limits<double>::infinity();
    return AABBd{Vec3(inf, inf, inf), Vec3(-inf, -inf, -inf)};
}
void grow(AABBd& a, const AABBd& b) {
    for (int k = 0; k < 3; ++k) {
        a.mn[k] = std::min(a.mn[k], b.mn[k]);
        a.mx[k] = std::max(a.mx[k], b.mx[k]);
    }
}

struct Builder {
    const std::vector<AABBd>& boxes;
    const std::vector<uint32_t>& refs;
    std::vector<BvhNode>& nodes;
    std::vector<uint32_t>& primrefs;
    std::vector<uint32_t> idx;
    std::vector<Vec3> cent;
    int max_depth = 0;

    int32_t leaf(int b, int e) {
        if (e - b > 127) throw std::runtime_error("bvh leaf too large (depth limit reached)");
        uint32_t first = static_cast<uint32_t>(primrefs.size());
        if (first + static_cast<uint32_t>(e - b) > 0xFFFFFFu) throw std::runtime_error("too many primitives for the bvh encoding");
        for (int i = b; i < e; ++i) primrefs.push_back(refs[idx[i]]);
        return make_leaf(first, static_cast<uint32_t>(e - b));
    }

    // Returns the child code for idx[b, e) and its box.
    int32_t build(int b, int e, int depth, AABBd& box) {
        box = empty_box();
        AABBd cb = empty_box();
        for (int i = b; i < e; ++i) {
            grow(box, boxes[idx[i]]);
            const Vec3& c = cent[idx[i]];
            grow(cb, AABBd{c, c});
        }
        const int n = e - b;
        if (n == 1) return leaf(b, e);
        if (depth >= kMaxBvhDepth - 1) return leaf(b, e);

        // binned SAH over the widest centroid axis
        int axis = 0;
        double ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = cb.mx[k] - cb.mn[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        int mid = -1;
        double best = std::numeric_limits<double>::infinity();
        if (ext[axis] > 0) {
            AABBd bin_box[kBins];
            int bin_n[kBins] = {0};
            for (auto& bb : bin_box) bb = empty_box();
            const double scale = kBins / ext[axis];
            auto bin_of = [&](uint32_t p) {
                int bi = static_cast<int>((cent[p][axis] - cb.mn[axis]) * scale);
                return std::min(kBins - 1, std::max(0, bi));
            };
            for (int i = b; i < e; ++i) {
                int bi = bin_of(idx[i]);
                bin_n[bi]++;
                grow(bin_box[bi], boxes[idx[i]]);
            }
            double right_area[kBins];
            int right_n[kBins];
            AABBd acc = empty_box();
            int cnt = 0;
            for (int i = kBins - 1; i > 0; --i) {
                grow(acc, bin_box[i]);
                cnt += bin_n[i];
                right_area[i] = area(acc);
                right_n[i] = cnt;
            }
            acc = empty_box();
            cnt = 0;
            int best_split = -1;
            const double parent = std::max(area(box), 1e-300);
            for (int i = 1; i < kBins; ++i) {
                grow(acc, bin_box[i - 1]);
                cnt += bin_n[i - 1];
                if (cnt == 0 || right_n[i] == 0) continue;
                double cost = kCostTraverse + kCostIntersect * (area(acc) * cnt + right_area[i] * right_n[i]) / parent;
                if (cost < best) {
                    best = cost;
                    best_split = i;
                }
            }
            if (best_split > 0) {
                if (n <= kMaxLeafPrims && kCostIntersect * n <= best) return leaf(b, e);
                auto it = std::partition(idx.begin() + b, idx.begin() + e, [&](uint32_t p) { return bin_of(p) < best_split; });
                mid = static_cast<int>(it - idx.begin());
            }
        }
        if (mid <= b || mid >= e) {  // degenerate centroids: object median
            if (n <= kMaxLeafPrims) return leaf(b, e);
            mid = b + n / 2;
            std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e,
                             [&](uint32_t x, uint32_t y) { return cent[x][axis] < cent[y][axis]; });
        }
        const int32_t me = static_cast<int32_t>(nodes.size());
        nodes.push_back(BvhNode{});
        max_depth = std::max(max_depth, depth + 1);
        AABBd lb, rb;
        int32_t l = build(b, mid, depth + 1, lb);
        int32_t r = build(mid, e, depth + 1, rb);
        set_node(me, l, lb, r, rb);
        return me;
    }

    void set_node(int32_t me, int32_t l, const AABBd& lb, int32_t r, const AABBd& rb) {
        float llo[3], lhi[3], rlo[3], rhi[3];
        conservative_box(lb, llo, lhi);
        conservative_box(rb, rlo, rhi);
        BvhNode& nd = nodes[me];
        nd.lx0 = llo[0]; nd.lx1 = lhi[0]; nd.ly0 = llo[1]; nd.ly1 = lhi[1];
        nd.rx0 = rlo[0]; nd.rx1 = rhi[0]; nd.ry0 = rlo[1]; nd.ry1 = rhi[1];
        nd.lz0 = llo[2]; nd.lz1 = lhi[2]; nd.rz0 = rlo[2]; nd.rz1 = rhi[2];
        nd.left = l;
        nd.right = r;
        nd.pad0 = nd.pad1 = 0;
    }
};

}  // namespace

void conservative_box(const AABBd& b, float lo[3], float hi[3]) {
    for (int k = 0; k < 3; ++k) {
        float l = static_cast<float>(b.mn[k]);
        float h = static_cast<float>(b.mx[k]);
        if (static_cast<double>(l) > b.mn[k]) l = std::nextafter(l, -std::numeric_limits<float>::infinity());
        if (static_cast<double>(h) < b.mx[k]) h = std::nextafter(h, std::numeric_limits<float>::infinity());
        // relative pad: covers f32 rounding of the ray origin/direction and of the slab arithmetic
        float pad = 1e-6f * std::max(std::max(std::fabs(l), std::fabs(h)), h - l) + 1e-30f;
        lo[k] = l - pad;
        hi[k] = h + pad;
    }
}

int32_t build_sah_bvh(const std::vector<AABBd>& boxes, const std::vector<uint32_t>& refs, std::vector<BvhNode>& nodes,
                      std::vector<uint32_t>& primrefs, int& max_depth) {
    if (boxes.empty() || boxes.size() != refs.size()) throw std::runtime_error("bad bvh input");
    Builder bl{boxes, refs, nodes, primrefs, {}, {}, 0};
    bl.idx.resize(boxes.size());
    bl.cent.resize(boxes.size());
    for (size_t i = 0; i < boxes.size(); ++i) {
        bl.idx[i] = static_cast<uint32_t>(i);
        for (int k = 0; k < 3; ++k) bl.cent[i][k] = 0.5 * (boxes[i].mn[k] + boxes[i].mx[k]);
    }
    AABBd rootbox;
    const int32_t root_slot = static_cast<int32_t>(nodes.size());
    int32_t c = bl.build(0, static_cast<int>(boxes.size()), 0, rootbox);
    if (c < 0) {  // the whole set is one leaf: root node with the leaf on both sides (tested once per side)
        nodes.push_back(BvhNode{});
        bl.set_node(root_slot, c, rootbox, c, rootbox);
        bl.max_depth = std::max(bl.max_depth, 1);
        c = root_slot;
    }
    max_depth = bl.max_depth;
    return c;
}

}  // namespace art
