// pt_leafbvh.h — exact acceleration of the reference tree's big leaves (host build).
#pragma once
#include <stdint.h>

#include <vector>

#include "pt_layout.h"

namespace pt {

// Chunks of the n entries of the leaf whose records are tris[rec0 .. rec0 + n): a build tree
// groups them (by the axis their normal is closest to, by shape — thin triangles apart, whose
// larger rounding bound would widen their neighbours' boxes — then by splits between position and
// direction); its leaf nodes, up to 8 entries each, are appended to `nodes` as chunks [root, end)
// (LNode), the entries' positions in the leaf to `lidx`.  tree (optional): the whole build tree in
// depth-first order (LNode::skip = the node after its subtree; leaves: info >= 0, in chunk order).
void build_leaf_bvh(const Tri* tris, int32_t rec0, int32_t n, std::vector<LNode>& nodes, std::vector<int32_t>& lidx,
                    int32_t& root, int32_t& end, std::vector<LNode>* tree = nullptr);

}  // namespace pt
