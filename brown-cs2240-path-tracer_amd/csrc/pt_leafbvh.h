// pt_leafbvh.h — exact acceleration of the reference tree's big leaves (host build).
#pragma once
#include <stdint.h>

#include <array>
#include <vector>

#include "pt_layout.h"

namespace pt {

// Chunks of the n entries of the leaf whose records are tris[rec0 .. rec0 + n): a build tree
// groups them (by the axis their normal is closest to, by shape — thin triangles apart, whose
// larger rounding bound would widen their neighbours' boxes — then by splits between position and
// direction); its leaf nodes, up to 8 entries each, are appended to `nodes` as chunks [root, end)
// (LNode), the entries' positions in the leaf to `lidx`.  tree (optional): the whole build tree in
// depth-first order (LNode::skip = the node after its subtree; leaves: info >= 0, in chunk order).
// leaf_max: entries per chunk at most (kChunkMax for the traversal's walks, kPassChunkMax for the
// leaf pass's); merge_max > 0: neighbouring chunks of one normal class merged while their entries
// fit merge_max.
void build_leaf_bvh(const Tri* tris, int32_t rec0, int32_t n, std::vector<LNode>& nodes, std::vector<int32_t>& lidx,
                    int32_t& root, int32_t& end, std::vector<LNode>* tree = nullptr, int leaf_max = kChunkMax,
                    int merge_max = 0);

// How often the rays that pass a big leaf's box filter (its path of child boxes from the root,
// PreLeaf) go on to visit it in the reference traversal, for a render's camera: out[b] = {rays that
// pass leaf b's filter, rays that visit it} over a stand-in of the render's queries — the camera
// rays through the centres of a grid x grid raster of the image, from each hit a shadow ray toward
// a random point of a random light (the NEE query) and one cosine bounce, and from the bounce's hit
// another shadow ray (seeded, so the same scene and camera give the same counts;
// scripts/leaf_visit_stats.c PROBE_GRID replays it through the oracle: CornellBox2 all meshes
// 0.377 of the filtered leaf work visited against 0.335 over the render's own queries, the boat
// 0.999 against ~0.99).  The traversal is the reference's (right child first, a child box skipped
// once the closest hit so far is nearer than its distance; leaves in order, strict <) in plain f32.
// Work is capped at max_tests triangle tests.
struct ProbeCamera {
    float cam[3];
    float M[16];         // cam_to_world, column-major (FrameParams::M)
    float focal, half_h, half_w;  // view plane at z = -focal, half extents
};
void probe_pre_leaves(const std::vector<Node>& nodes, const std::vector<Tri>& tris, const std::vector<Light>& lights,
                      const std::vector<PreLeaf>& pre, const ProbeCamera& cam, int grid, uint64_t max_tests,
                      std::vector<std::array<uint32_t, 2>>& out);

// Leaf remainders (pt_leafskip.cpp; the traversal's exact skip of entries the ray tested in the
// leaf it tested just before, pt_device.h lean_node_unit): for every leaf of fewer than max_leaf
// (<= kLeafSkipMaxLeaf) entries, up to `alts` (kLeafAlt) earlier leaves M are chosen — by a probe of
// the reference traversal (rays from random points of the scene in random directions and toward
// the lights, at most max_tests triangle tests), then by nearness in the visit order — and "the
// leaf minus M" is appended to tris (and tnorm, 3 per record) in entry order.  nalt gets per node
// and side `alts` int2 (M's first record, remainder first record << 7 | count), INT32_MIN: none.
struct LeafSkipStats {
    uint64_t probe_tests = 0;  // the probe's triangle tests
    uint64_t remainders = 0;   // remainders built
    uint64_t skipped = 0;      // entries they leave out, summed
    uint64_t records = 0;      // records appended
};
void build_leaf_skips(const std::vector<Node>& nodes, std::vector<Tri>& tris, std::vector<float4>& tnorm,
                      const std::vector<Light>& lights, int max_leaf, int alts, uint64_t max_tests,
                      std::vector<int2>& nalt, LeafSkipStats* stats = nullptr);

}  // namespace pt
