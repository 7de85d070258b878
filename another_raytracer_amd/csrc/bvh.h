// bvh.h — full-sweep SAH BVH over primitive boxes, collapsed into the flat 128-B four-child node array of layout.h.
//
// Replaces the reference's bvh_node (primitives/bvh.cpp:3-42: random split axis, median split, O(N^2) object
// copies, 1-spans tested twice).  Closest-hit results do not depend on the tree, so the product builds the tree
// that minimises expected traversal cost instead: full-sweep SAH on centroids (plus binned spatial splits for meshes:
// a split BVH), leaves of <= kMaxLeafPrims, depth
// capped at kMaxBvhDepth (the LDS traversal stack), child boxes rounded outward to f32 and padded so that f32
// traversal never rejects a box the f64 leaf test could hit.
#pragma once
#include <cstdint>
#include <functional>
#include <vector>

#include "layout.h"
#include "scene.h"

namespace art {

// Spatial-split support: the box of the part of primitive `ref` inside the slab lo <= x[axis] <= hi, intersected with
// `cur` (the box of the part already assigned to this reference); false when that part is empty.
using ClipFn = std::function<bool(uint32_t ref, int axis, double lo, double hi, const AABBd& cur, AABBd& out)>;

// Appends nodes/primrefs for one BVH and returns its root node index.  max_depth receives the 4-wide tree depth,
// max_stack the worst-case number of traversal stack entries (sum of (children - 1) along a root-to-leaf path).
// With `clip`, the binary tree is a split BVH (Stich et al. 2009): a node may also split space, referencing a primitive
// that straddles the plane from both children with its clipped boxes (duplicated references, at most
// kSbvhRefBudget x the primitive count).
int32_t build_sah_bvh(const std::vector<AABBd>& boxes, const std::vector<uint32_t>& refs, std::vector<BvhNode>& nodes,
                      std::vector<uint32_t>& primrefs, int& max_depth, int& max_stack, const ClipFn* clip = nullptr);

// f32 box rounded outward + relative pad (the conservative box the traversal tests).
void conservative_box(const AABBd& b, float lo[3], float hi[3]);

}  // namespace art
