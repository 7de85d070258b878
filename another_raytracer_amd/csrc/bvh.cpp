// bvh.cpp — full-sweep SAH binary tree, collapsed into the 4-wide node array of layout.h (see bvh.h).
#include "bvh.h"
#include "options.h"

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <memory>
#include <stdexcept>

namespace art {

namespace {

constexpr double kCostTraverse = 1.0;
// SAH primitive-test cost relative to a (binary) node step and the leaf size: options bvh.sah_ci / bvh.sah_leaf
// (rt_option_set; builder experiments, tools/sah_sweep*.sh)
double sah_ci() { return opt(Opt::SahCi); }
int sah_leaf() { return static_cast<int>(opt(Opt::SahLeaf)); }  // 1..16 (the option's range)

int collapse_mode();
// Leaf size of the binary tree: the wide tree's under the greedy collapse; bvh.dp_binary_leaf (default 1) under the
// SAH-optimal collapse, which then chooses the wide tree's leaves itself (merging binary leaves up to sah_leaf())
int binary_leaf() {
    if (collapse_mode() != 1) return sah_leaf();
    return std::max(1, std::min(sah_leaf(), static_cast<int>(opt(Opt::DpBinaryLeaf))));
}

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

struct BNode {  // binary SAH tree node (host only)
    AABBd box;
    int left = -1, right = -1;   // inner: children in `tree`
    int32_t leaf = 0;            // leaf: encoded primref range (< 0)
    bool is_leaf() const { return left < 0; }
};

struct Builder {
    const std::vector<AABBd>& boxes;
    const std::vector<uint32_t>& refs;
    std::vector<uint32_t>& primrefs;
    std::vector<uint32_t> idx;
    std::vector<Vec3> cent;
    std::vector<BNode> tree;

    int make_leaf_node(int b, int e, const AABBd& box) {
        if (e - b > 127) throw std::runtime_error("bvh leaf too large (depth limit reached)");
        uint32_t first = static_cast<uint32_t>(primrefs.size());
        if (first + static_cast<uint32_t>(e - b) > 0xFFFFFFu) throw std::runtime_error("too many primitives for the bvh encoding");
        for (int i = b; i < e; ++i) primrefs.push_back(refs[idx[i]]);
        BNode n;
        n.box = box;
        n.leaf = make_leaf(first, static_cast<uint32_t>(e - b));
        tree.push_back(n);
        return static_cast<int>(tree.size()) - 1;
    }

    int build(int b, int e, int depth) {
        AABBd box = empty_box(), cb = empty_box();
        for (int i = b; i < e; ++i) {
            grow(box, boxes[idx[i]]);
            const Vec3& c = cent[idx[i]];
            grow(cb, AABBd{c, c});
        }
        const int n = e - b;
        if (n == 1 || depth >= kMaxBvhDepth - 1) return make_leaf_node(b, e, box);

        // full-sweep SAH over all three centroid axes (the scenes are small: ~1e3 - 1e4 primitives)
        int axis = 0;
        double ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = cb.mx[k] - cb.mn[k];
        if (ext[1] > ext[axis]) axis = 1;
        if (ext[2] > ext[axis]) axis = 2;
        int mid = -1;
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_split = -1;
        const double parent = std::max(area(box), 1e-300);
        std::vector<uint32_t> order[3];
        std::vector<double> right_area(static_cast<size_t>(n) + 1);
        for (int k = 0; k < 3; ++k) {
            if (!(ext[k] > 0)) continue;
            order[k].assign(idx.begin() + b, idx.begin() + e);
            std::stable_sort(order[k].begin(), order[k].end(), [&](uint32_t x, uint32_t y) { return cent[x][k] < cent[y][k]; });
            AABBd acc = empty_box();
            for (int i = n - 1; i > 0; --i) {
                grow(acc, boxes[order[k][static_cast<size_t>(i)]]);
                right_area[static_cast<size_t>(i)] = area(acc);
            }
            acc = empty_box();
            for (int i = 1; i < n; ++i) {
                grow(acc, boxes[order[k][static_cast<size_t>(i - 1)]]);
                const double cost = kCostTraverse + sah_ci() * (area(acc) * i + right_area[static_cast<size_t>(i)] * (n - i)) / parent;
                if (cost < best) {
                    best = cost;
                    best_axis = k;
                    best_split = i;
                }
            }
        }
        if (best_axis >= 0) {
            if (n <= binary_leaf() && sah_ci() * n <= best) return make_leaf_node(b, e, box);
            std::copy(order[best_axis].begin(), order[best_axis].end(), idx.begin() + b);
            mid = b + best_split;
        }
        if (mid <= b || mid >= e) {  // degenerate centroids: object median
            if (n <= binary_leaf()) return make_leaf_node(b, e, box);
            mid = b + n / 2;
            std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e,
                             [&](uint32_t x, uint32_t y) { return cent[x][axis] < cent[y][axis]; });
        }
        const int me = static_cast<int>(tree.size());
        tree.push_back(BNode{});
        const int l = build(b, mid, depth + 1);
        const int r = build(mid, e, depth + 1);
        tree[me].box = box;
        tree[me].left = l;
        tree[me].right = r;
        return me;
    }
};

// Split BVH (Stich, Friedrich, Dietrich 2009, "Spatial Splits in Bounding Volume Hierarchies"): each node takes the
// cheaper of the full-sweep object split and a binned spatial split, tried when the object split's children overlap;
// a spatial split references a straddling primitive from both sides with its clipped boxes.  Tighter boxes for meshes
// (fewer node visits and leaf tests), at the price of duplicated references (capped by kSbvhRefBudget).
constexpr double kSbvhRefBudget = 1.5;
double sbvh_alpha() { return opt(Opt::SbvhAlpha); }  // overlap / root area below which no spatial split is tried
constexpr int kSbvhBins = 32;
double sbvh_budget() { return opt(Opt::Sbvh); }  // kSbvhRefBudget by default; < 1: object splits only

struct SItem {
    uint32_t ref;
    AABBd box;
};
AABBd box_of(const std::vector<SItem>& v, size_t b, size_t e) {
    AABBd a = empty_box();
    for (size_t i = b; i < e; ++i) grow(a, v[i].box);
    return a;
}
AABBd box_and(const AABBd& a, const AABBd& b) {
    AABBd r;
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = std::max(a.mn[k], b.mn[k]);
        r.mx[k] = std::min(a.mx[k], b.mx[k]);
    }
    return r;
}
bool box_valid(const AABBd& b) { return b.mn[0] <= b.mx[0] && b.mn[1] <= b.mx[1] && b.mn[2] <= b.mx[2]; }

struct SBuilder {
    const ClipFn& clip;
    std::vector<uint32_t>& primrefs;
    std::vector<BNode> tree;
    double root_area = 0;
    size_t refs_left = 0;  // duplicated references still allowed

    int make_leaf_node(const std::vector<SItem>& items, const AABBd& box) {
        if (items.size() > 127) throw std::runtime_error("bvh leaf too large (depth limit reached)");
        const uint32_t first = static_cast<uint32_t>(primrefs.size());
        if (first + items.size() > 0xFFFFFFu) throw std::runtime_error("too many primitives for the bvh encoding");
        for (const SItem& it : items) primrefs.push_back(it.ref);
        BNode n;
        n.box = box;
        n.leaf = make_leaf(first, static_cast<uint32_t>(items.size()));
        tree.push_back(n);
        return static_cast<int>(tree.size()) - 1;
    }

    int build(std::vector<SItem> items, int depth) {
        const AABBd box = box_of(items, 0, items.size());
        const size_t n = items.size();
        if (n == 1 || depth >= kMaxBvhDepth - 1) return make_leaf_node(items, box);
        const double parent = std::max(area(box), 1e-300);
        auto cent = [](const SItem& it, int k) { return 0.5 * (it.box.mn[k] + it.box.mx[k]); };
        // object split: full sweep over the centroids on each axis
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1;
        size_t best_split = 0;
        AABBd best_l{}, best_r{};
        std::vector<SItem> order;
        std::vector<double> right_area(n + 1);
        std::vector<AABBd> right_box(n + 1);
        for (int k = 0; k < 3; ++k) {
            order = items;
            std::stable_sort(order.begin(), order.end(), [&](const SItem& a, const SItem& b) { return cent(a, k) < cent(b, k); });
            AABBd acc = empty_box();
            for (size_t i = n - 1; i > 0; --i) {
                grow(acc, order[i].box);
                right_area[i] = area(acc);
                right_box[i] = acc;
            }
            acc = empty_box();
            for (size_t i = 1; i < n; ++i) {
                grow(acc, order[i - 1].box);
                const double cost = kCostTraverse + sah_ci() * (area(acc) * double(i) + right_area[i] * double(n - i)) / parent;
                if (cost < best) {
                    best = cost;
                    best_axis = k;
                    best_split = i;
                    best_l = acc;
                    best_r = right_box[i];
                }
            }
        }
        // spatial split: binned, when the object split's children overlap
        int sp_axis = -1;
        double sp_plane = 0, sp_best = best;
        const AABBd ov = box_and(best_l, best_r);
        if (refs_left > 0 && best_axis >= 0 && box_valid(ov) && area(ov) > sbvh_alpha() * root_area) {
            for (int k = 0; k < 3; ++k) {
                const double lo = box.mn[k], ext = box.mx[k] - box.mn[k];
                if (!(ext > 0)) continue;
                AABBd bins[kSbvhBins];
                int enter[kSbvhBins] = {0}, leave[kSbvhBins] = {0};
                for (auto& b : bins) b = empty_box();
                auto bin_of = [&](double x) { return std::min(kSbvhBins - 1, std::max(0, static_cast<int>((x - lo) / ext * kSbvhBins))); };
                auto plane = [&](int i) { return i == kSbvhBins ? box.mx[k] : lo + ext * i / kSbvhBins; };
                for (const SItem& it : items) {
                    const int b0 = bin_of(it.box.mn[k]), b1 = bin_of(it.box.mx[k]);
                    if (b0 == b1) {
                        grow(bins[b0], it.box);
                    } else {
                        for (int b = b0; b <= b1; ++b) {
                            AABBd c;
                            if (clip(it.ref, k, b == b0 ? it.box.mn[k] : plane(b), b == b1 ? it.box.mx[k] : plane(b + 1), it.box, c)) grow(bins[b], c);
                        }
                    }
                    ++enter[b0];
                    ++leave[b1];
                }
                double ra[kSbvhBins];
                int rn[kSbvhBins];
                AABBd acc = empty_box();
                int cnt = 0;
                for (int i = kSbvhBins - 1; i > 0; --i) {
                    grow(acc, bins[i]);
                    cnt += leave[i];
                    ra[i] = box_valid(acc) ? area(acc) : 0;
                    rn[i] = cnt;
                }
                acc = empty_box();
                cnt = 0;
                for (int i = 1; i < kSbvhBins; ++i) {
                    grow(acc, bins[i - 1]);
                    cnt += enter[i - 1];
                    if (cnt == 0 || rn[i] == 0) continue;
                    const double cost = kCostTraverse + sah_ci() * ((box_valid(acc) ? area(acc) : 0) * cnt + ra[i] * rn[i]) / parent;
                    if (cost < sp_best) {
                        sp_best = cost;
                        sp_axis = k;
                        sp_plane = plane(i);
                    }
                }
            }
        }
        const double leaf_cost = sah_ci() * double(n);
        if (n <= static_cast<size_t>(binary_leaf()) && leaf_cost <= std::min(best, sp_best)) return make_leaf_node(items, box);
        std::vector<SItem> left, right;
        if (sp_axis >= 0) {
            const int k = sp_axis;
            for (const SItem& it : items) {
                if (it.box.mx[k] <= sp_plane) {
                    left.push_back(it);
                } else if (it.box.mn[k] >= sp_plane) {
                    right.push_back(it);
                } else {
                    AABBd cl, cr;
                    const bool hl = clip(it.ref, k, it.box.mn[k], sp_plane, it.box, cl);
                    const bool hr = clip(it.ref, k, sp_plane, it.box.mx[k], it.box, cr);
                    if (hl) left.push_back(SItem{it.ref, cl});
                    if (hr) right.push_back(SItem{it.ref, cr});
                    if (!hl && !hr) left.push_back(it);  // degenerate clip: keep the reference whole
                    if (hl && hr) refs_left -= refs_left > 0 ? 1 : 0;
                }
            }
        }
        if (left.empty() || right.empty()) {  // object split (also when the spatial partition degenerated)
            left.clear();
            right.clear();
            if (best_axis < 0) {
                if (n <= 127) return make_leaf_node(items, box);
                best_axis = 0;
                best_split = n / 2;
            }
            order = items;
            const int k = best_axis;
            std::stable_sort(order.begin(), order.end(), [&](const SItem& a, const SItem& b) { return cent(a, k) < cent(b, k); });
            left.assign(order.begin(), order.begin() + static_cast<std::ptrdiff_t>(best_split));
            right.assign(order.begin() + static_cast<std::ptrdiff_t>(best_split), order.end());
        }
        items.clear();
        items.shrink_to_fit();
        const int me = static_cast<int>(tree.size());
        tree.push_back(BNode{});
        const int l = build(std::move(left), depth + 1);
        const int r = build(std::move(right), depth + 1);
        tree[me].box = box;
        tree[me].left = l;
        tree[me].right = r;
        return me;
    }
};

// SAH-optimal collapse of the binary tree into the 4-wide one (Ylitie, Karras, Laine 2017, "Efficient incoherent ray
// traversal on GPUs through compressed wide BVHs", §4.1, for width 4): by dynamic programming over the binary nodes,
// C(n, i) = the least SAH cost of covering n's primitives with at most i wide-node children, each either a wide node
// (cost A·1 + the best spread of its 4 slots over n's two children) or a leaf of n's primitives (cost A·ci·count, when
// they are contiguous in the primref array and at most the leaf size).  The greedy alternative pulls the largest-area
// children up and never merges binary leaves.  bvh.collapse: 0 greedy (default), 1 dp; bvh.collapse_ci: the
// primitive test cost relative to a 4-wide node visit.  Measured (r3k, A/B on one box, Msamples/s): the optimal
// collapse visits fewer nodes (scene 1: 6.21 vs 6.36 per traversal) but diverges more (node-loop lane utilization
// 0.441 vs 0.474) and loses on the GPU: scene 1 -3.4 %, cow -1.2 %, Next-Week final -6.1 %, dino +0.6 % (ci 0.6;
// ci 0.4 / 1.0 and a leaf-size-4 binary tree no better), so the greedy collapse stays the default.
int collapse_mode() { return static_cast<int>(opt(Opt::BvhCollapse)); }
double collapse_ci() { return opt(Opt::CollapseCi); }
struct CollapseDP {
    static constexpr int kW = 4;
    const std::vector<BNode>& tree;
    std::vector<std::array<double, kW + 1>> cost;  // cost[n][i], i = 1..kW
    std::vector<std::array<int8_t, kW + 1>> take;  // cost[n][i] (i >= 2): 0 = n itself as one child, k = k slots to the left
    std::vector<int8_t> leaf_ok, as_leaf, inner_split;
    std::vector<uint32_t> first, count;

    explicit CollapseDP(const std::vector<BNode>& t)
        : tree(t), cost(t.size()), take(t.size()), leaf_ok(t.size(), 0), as_leaf(t.size(), 0), inner_split(t.size(), 0), first(t.size()), count(t.size()) {
        const double inf = std::numeric_limits<double>::infinity();
        // children are pushed after their parent (Builder::build, SBuilder::build): reverse index order is bottom-up
        for (int n = static_cast<int>(t.size()) - 1; n >= 0; --n) {
            const BNode& b = t[static_cast<size_t>(n)];
            const double a = area(b.box);
            if (b.is_leaf()) {
                first[n] = leaf_first(b.leaf);
                count[n] = leaf_count(b.leaf);
                leaf_ok[n] = 1;
                as_leaf[n] = 1;
                for (int i = 1; i <= kW; ++i) {
                    cost[n][i] = a * collapse_ci() * count[n];
                    take[n][i] = 0;
                }
                continue;
            }
            const int l = b.left, r = b.right;
            count[n] = count[l] + count[r];
            first[n] = std::min(first[l], first[r]);
            leaf_ok[n] = leaf_ok[l] && leaf_ok[r] && count[n] <= static_cast<uint32_t>(sah_leaf()) &&
                         (first[r] == first[l] + count[l] || first[l] == first[r] + count[r]);
            double best_inner = inf;
            for (int k = 1; k < kW; ++k) {
                const double c = cost[l][k] + cost[r][kW - k];
                if (c < best_inner) {
                    best_inner = c;
                    inner_split[n] = static_cast<int8_t>(k);
                }
            }
            best_inner += a;
            const double leaf_cost = leaf_ok[n] ? a * collapse_ci() * count[n] : inf;
            as_leaf[n] = leaf_cost <= best_inner;
            cost[n][1] = std::min(leaf_cost, best_inner);
            take[n][1] = 0;
            for (int i = 2; i <= kW; ++i) {
                cost[n][i] = cost[n][1];
                take[n][i] = 0;
                for (int k = 1; k < i; ++k) {
                    const double c = cost[l][k] + cost[r][i - k];
                    if (c < cost[n][i]) {
                        cost[n][i] = c;
                        take[n][i] = static_cast<int8_t>(k);
                    }
                }
            }
        }
    }
    // the wide-node children covering n's primitives with at most i of them
    void gather(int n, int i, std::vector<int>& kids) const {
        const int k = take[n][i];
        if (k == 0) {
            kids.push_back(n);
            return;
        }
        gather(tree[n].left, k, kids);
        gather(tree[n].right, i - k, kids);
    }
    // children of the wide node made from binary inner node n
    std::vector<int> children(int n) const {
        std::vector<int> kids;
        gather(tree[n].left, inner_split[n], kids);
        gather(tree[n].right, kW - inner_split[n], kids);
        return kids;
    }
};

// Emits the 4-wide node for binary inner node `bn` and returns its index; `stack` receives the worst-case traversal
// stack use below and including it.  dp null: children pulled up greedily by largest surface area.
int32_t collapse(const std::vector<BNode>& tree, int bn, std::vector<BvhNode>& out, int& stack, int& depth, const CollapseDP* dp = nullptr) {
    std::vector<int> kids;
    if (dp) {
        kids = dp->children(bn);
    } else {
        kids = {tree[bn].left, tree[bn].right};
        while (kids.size() < 4) {
            int best = -1;
            double best_a = -1;
            for (size_t i = 0; i < kids.size(); ++i)
                if (!tree[kids[i]].is_leaf() && area(tree[kids[i]].box) > best_a) {
                    best_a = area(tree[kids[i]].box);
                    best = static_cast<int>(i);
                }
            if (best < 0) break;
            const int k = kids[best];
            kids[best] = tree[k].left;
            kids.push_back(tree[k].right);
        }
    }
    const int32_t me = static_cast<int32_t>(out.size());
    out.push_back(BvhNode{});
    int child_stack = 0, child_depth = 0;
    int32_t code[4];
    float lo[4][3], hi[4][3];
    for (int c = 0; c < 4; ++c) {
        if (c >= static_cast<int>(kids.size())) {
            code[c] = kNodeEmpty;
            for (int k = 0; k < 3; ++k) {
                lo[c][k] = std::numeric_limits<float>::max();
                hi[c][k] = -std::numeric_limits<float>::max();
            }
            continue;
        }
        const BNode& k = tree[kids[c]];
        conservative_box(k.box, lo[c], hi[c]);
        if (k.is_leaf()) {
            code[c] = k.leaf;
        } else if (dp && dp->as_leaf[kids[c]]) {  // a binary subtree whose primitives form one leaf
            code[c] = make_leaf(dp->first[kids[c]], dp->count[kids[c]]);
        } else {
            int s = 0, dd = 0;
            code[c] = collapse(tree, kids[c], out, s, dd, dp);
            child_stack = std::max(child_stack, s);
            child_depth = std::max(child_depth, dd);
        }
    }
    BvhNode& n = out[me];
    for (int c = 0; c < 4; ++c) {
        n.lox[c] = lo[c][0]; n.hix[c] = hi[c][0];
        n.loy[c] = lo[c][1]; n.hiy[c] = hi[c][1];
        n.loz[c] = lo[c][2]; n.hiz[c] = hi[c][2];
        n.child[c] = code[c];
        n.pad[c] = 0;
    }
    stack = static_cast<int>(kids.size()) - 1 + child_stack;  // pushes on the worst root-to-leaf path
    depth = 1 + child_depth;
    return me;
}

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
                      std::vector<uint32_t>& primrefs, int& max_depth, int& max_stack, const ClipFn* clip) {
    if (boxes.empty() || boxes.size() != refs.size()) throw std::runtime_error("bad bvh input");
    Builder bl{boxes, refs, primrefs, {}, {}, {}};
    SBuilder sb{clip ? *clip : ClipFn{}, primrefs, {}, 0, 0};
    const bool split = clip && sbvh_budget() > 1.0;
    int root;
    if (split) {
        std::vector<SItem> items(boxes.size());
        AABBd all = empty_box();
        for (size_t i = 0; i < boxes.size(); ++i) {
            items[i] = SItem{refs[i], boxes[i]};
            grow(all, boxes[i]);
        }
        sb.root_area = area(all);
        sb.refs_left = static_cast<size_t>((sbvh_budget() - 1.0) * static_cast<double>(boxes.size()));
        root = sb.build(std::move(items), 0);
        bl.tree.swap(sb.tree);
    } else {
        bl.idx.resize(boxes.size());
        bl.cent.resize(boxes.size());
        for (size_t i = 0; i < boxes.size(); ++i) {
            bl.idx[i] = static_cast<uint32_t>(i);
            for (int k = 0; k < 3; ++k) bl.cent[i][k] = 0.5 * (boxes[i].mn[k] + boxes[i].mx[k]);
        }
        root = bl.build(0, static_cast<int>(boxes.size()), 0);
    }
    if (bl.tree[root].is_leaf()) {  // a single leaf: a root node with one real child
        const int32_t me = static_cast<int32_t>(nodes.size());
        nodes.push_back(BvhNode{});
        float lo[3], hi[3];
        conservative_box(bl.tree[root].box, lo, hi);
        BvhNode& n = nodes[me];
        for (int c = 0; c < 4; ++c) {
            const bool real = c == 0;
            n.lox[c] = real ? lo[0] : std::numeric_limits<float>::max(); n.hix[c] = real ? hi[0] : -std::numeric_limits<float>::max();
            n.loy[c] = real ? lo[1] : std::numeric_limits<float>::max(); n.hiy[c] = real ? hi[1] : -std::numeric_limits<float>::max();
            n.loz[c] = real ? lo[2] : std::numeric_limits<float>::max(); n.hiz[c] = real ? hi[2] : -std::numeric_limits<float>::max();
            n.child[c] = real ? bl.tree[root].leaf : kNodeEmpty;
            n.pad[c] = 0;
        }
        max_depth = 1;
        max_stack = 0;
        return me;
    }
    int stack = 0, depth = 0;
    std::unique_ptr<CollapseDP> dp;
    if (collapse_mode() == 1) dp = std::make_unique<CollapseDP>(bl.tree);
    const int32_t r = collapse(bl.tree, root, nodes, stack, depth, dp.get());
    max_depth = depth;
    max_stack = stack;
    return r;
}

}  // namespace art
