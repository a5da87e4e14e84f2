// pt_layout.h — device-resident scene layout (HBM), built once by pt_scene_create
// from the reference's packed buffers (packer.ts:4-137 layouts).
//
// The reference walks a float-encoded pre-order tree (17-float nodes + inline
// leaf payloads holding 1-based float vertex indices) and gathers 9 vertex
// floats per triangle test.  Here the same tree is re-encoded for 16-byte
// vector loads:
//   nodes[]  64 B: both child AABBs + two child refs (one node = one traversal
//            step of intersection-logic.wgsl:31-212; the root is node 0 = bvh[6])
//   tris[]   48 B per leaf reference, leaves contiguous in traversal order:
//            v0, e1 = v1 - v0, e2 = v2 - v0 packed in 36 B, material id, uid (f32, exactly the values
//            ray-triangle-intersection.wgsl:6-7 computes per test); scenes with at most
//            64 distinct leaf entries (mailbox scenes) append one record per distinct entry
//   lmask[]  mailbox scenes: per leaf (indexed by its first tris[] record) the 64-bit set
//            of the uids it holds
//   mats[]   64 B: Ns Ni illum | Kd | Ks | Ke (program-raymarch.wgsl:87-102)
//   lights[] 48 B: the Ntri emissive triangles in sample_area_lights' slot order,
//            plus one extra entry k == Ntri for hash1 == 1.0 (the reference's
//            out-of-range else-branch, resolved with Tint's clamped reads).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace pt {

struct alignas(16) Node {
    float lmin[3];
    float lmax[3];
    float rmin[3];
    float rmax[3];
    int32_t lref, rref;  // internal child: node index; leaf child: first tri record
    int32_t lcnt, rcnt;  // < 0: internal child; >= 0: leaf with that many triangles
};
static_assert(sizeof(Node) == 64, "node is 4 x 16 B");

// Mailbox scenes with <= 64 internal nodes and <= 63 distinct entries: the internal nodes again,
// numbered in the reference's visiting order (pre-order, right subtree first), each child's
// payload in one 64-bit word — a leaf child's uid set (bit 63 clear; 0 for an empty leaf) or, for
// an internal child, bit 63 | its pre-order number.  The brute-force replay walks this tree with a
// 64-bit set of pending nodes instead of a stack (pt_wavefront.hip bf_closest).
struct alignas(16) BfNode {
    float lmin[3];
    float lmax[3];
    float rmin[3];
    float rmax[3];
    uint64_t lm, rm;
};
static_assert(sizeof(BfNode) == 64, "bf node is 4 x 16 B");

// The nine floats a triangle test reads fill the first 36 bytes so that a test loads them
// with two ds_read_b128 + one ds_read_b32 (10 LDS cycles per wave); with v0/e1/e2 each in its
// own 16-byte slot the compiler reads three ds_read_b96 (8 cycles each on gfx950: 24).
struct alignas(16) Tri {
    float q0[4];   // v0.x v0.y v0.z e1.x
    float q1[4];   // e1.y e1.z e2.x e2.y
    float e2z;
    int32_t mat;
    int32_t uid;   // id of this (i0, i1, i2, material) entry (distinct entries numbered by first appearance; < 64 on mailbox scenes)
    int32_t lbvh;  // a leaf with a leaf BVH (LNode): its first record holds root + 1, its second the end node (else 0)
};
inline void tri_set(Tri& t, const float v0[3], const float e1[3], const float e2[3]) {
    t.q0[0] = v0[0]; t.q0[1] = v0[1]; t.q0[2] = v0[2]; t.q0[3] = e1[0];
    t.q1[0] = e1[1]; t.q1[1] = e1[2]; t.q1[2] = e2[0]; t.q1[3] = e2[1];
    t.e2z = e2[2];
}
static_assert(sizeof(Tri) == 48, "tri record is 3 x 16 B");

// entries per leaf chunk (LNode; build_leaf_bvh's leaf size, the chunk walks' test loops)
#ifndef PT_LEAF_CHUNK
#define PT_LEAF_CHUNK 8
#endif
constexpr int kChunkMax = PT_LEAF_CHUNK;
// entries per chunk of the leaf pass's own chunking of its leaves (pt_leafpass.hip): twice the
// traversal's — with the pass's second check the tests are cheap and the uniform chunk checks are
// the cost (boat in process +5 %, profiles/r05w_ab_chunk_refine.log), while 16-entry chunks cost the
// traversal's walks 13 % (r05x_ab_chunk16.log)
#ifndef PT_PASS_CHUNK
#define PT_PASS_CHUNK 16
#endif
constexpr int kPassChunkMax = PT_PASS_CHUNK;

// Leaf chunk (pt_leafbvh.cpp): up to 8 entries of one big leaf of the reference tree, grouped by
// position and normal direction.  A chunk is skipped only when none of its entries can report a
// hit at t <= the closest t so far: the ray misses, or enters late, the chunk's box grown by
// delta = (A + B |o|) / cf + 1e-5 |o| + C, where cf > 0 bounds |cos(ray, normal)| from below over
// the chunk's cone of triangle normals (axis a, half-angle with cosine ca and sine sa) — the
// test's rounding bound.
struct alignas(16) LNode {
    float lo[3], ax;
    float hi[3], ay;
    float az, ca, sa, B;
    float A, C;
    int32_t skip;  // builder only
    int32_t info;  // first lidx slot | count << 24
};
static_assert(sizeof(LNode) == 64, "leaf BVH node is 4 x 16 B");

// A big leaf resolved before the traversal (pt_leafpass.hip, k_wf_leafpass): its records, and the
// path from the root to it as (node << 1 | side) per step — the child boxes every visit of the leaf
// must enter (ray_box > 0: a leaf child is tested whenever its parent is visited and its box is hit,
// intersection-logic.wgsl:47-176, and a node is visited only if each box on its path was entered).
constexpr int kMaxPre = 8;        // big leaves resolved per scene (the largest ones)
constexpr int kMaxPrePath = 40;   // > the deepest tree the builders make (reference 16 + 1, SAH 28 + 1)
struct alignas(16) PreLeaf {
    int32_t rec0, n, npath, pad;
    int32_t c0, c1, pad1, pad2;  // the leaf pass's chunks of this leaf: SceneView::pnodes[c0 .. c1) (none: c0 == c1)
    int32_t path[kMaxPrePath];
};
static_assert(offsetof(PreLeaf, c0) == 16 && offsetof(PreLeaf, path) == 32, "k_wf_leafpass reads PreLeaf as ints 4, 5, 8..");

// leaf remainders (pt_leafskip.cpp, SceneView::nalt): per leaf child, kLeafAlt earlier leaves whose
// entries its remainders leave out; leaves of fewer than kLeafSkipMaxLeaf entries have them (the
// count is 7 bits of the descriptor; big-leaf thresholds below it turn the skip off, pt_capi.hip)
#ifndef PT_LEAF_ALT
#define PT_LEAF_ALT 1
#endif
constexpr int kLeafAlt = PT_LEAF_ALT;
static_assert(kLeafAlt == 1 || kLeafAlt == 4, "one or four (prev, remainder) pairs per side");
constexpr int kLeafSkipMaxLeaf = 64;

struct alignas(16) Material {
    float Ns, Ni, illum, phong;  // phong = (Ns + 2) / (2 pi), f32, as program-raymarch.wgsl:271
    float Kd[3], kd_pi0;         // kd_pi* = Kd / pi per channel, f32 (program-raymarch.wgsl:165,279)
    float Ks[3], kd_pi1;
    float Ke[3], kd_pi2;
};
static_assert(sizeof(Material) == 64, "material is 4 x 16 B");

struct alignas(16) Light {
    float p0[3], pad0;
    float p1[3], pad1;
    float p2[3], pad2;
};
static_assert(sizeof(Light) == 48, "light is 3 x 16 B");

// Read-only scene view passed to kernels by value.
struct SceneView {
    const Node* nodes;
    const Tri* tris;
    const Material* mats;
    const Light* lights;
    int32_t n_nodes;
    int32_t n_tris;
    int32_t n_mats;
    int32_t n_lights;   // Ntri (table holds n_lights + 1 entries)
    float f_ntri;       // f32(Ntri)
    float inv_ntri;     // 1.0 / f32(Ntri)
    int32_t max_stack;  // deepest traversal stack the tree can produce
    // byte offsets of each section from `nodes` (one contiguous device allocation), and
    // the span [nodes, end of lights) staged into LDS by kernels when it fits
    uint32_t off_tris, off_mats, off_lights, span_bytes;
    // 1: every triangle has |e1|*|e2| < 2^124, so with unit ray directions |det| < 2^126 and
    // the triangle test may take 1/det from rcp_rn (pt_math.h), bit-identical to the division
    int32_t fast_rcp;
    // lean traversal turn policy: a leaf turn needs leaf lanes >= node_bias * node lanes
    // (1 = plain majority; a leaf turn costs up to K triangle tests, a node turn one node
    // step, so node turns that feed lanes into their leaves pay off); 0 = pipeline default
    int32_t node_bias;
    // node steps per node turn of the lean traversal (option node_steps, 1..8; 0 = the pipeline's
    // default: 4 wavefront, 1 megakernel): lanes still in node
    // state after a step take the next in the same turn, without the loop's bookkeeping in between
    int32_t node_steps;
    // mailbox (SceneView::mailbox != 0 when the scene has <= 64 distinct leaf entries): the
    // record of uid u is tris[mb_base + u]; lmask at byte offset off_lmask (inside the span)
    int32_t mailbox;
    int32_t mb_base;
    uint32_t off_lmask;
    const uint64_t* lmask;
    // BfNode tree (nullptr when the scene does not qualify) and bfmap[i] = the nodes[] index of
    // pre-order node i (its leaf ranges, for the tie-break scan and the counting build); both inside
    // the LDS span at off_bfnode / off_bfmap
    const BfNode* bfnode;
    const int32_t* bfmap;
    uint32_t off_bfnode, off_bfmap;
    // vertex-normal mode (pt_scene_set_vertex_normals; the reference's commented-out branch,
    // intersection-logic.wgsl:81-108): per record (v0n, v1n, v2n) as 3 float4, v0n.w = 1 where
    // i2 < vn_range (the branch applies); global memory, read for the winning record only
    const float4* tnorm;
    int32_t vnormals;
    // big leaves in step (lean traversal, TRAV + 160): the lanes of a wave walk a leaf of at least
    // big_leaf entries in one shared rotated order (lean_leaf_loop; 0 = off)
    int32_t big_leaf;
    // leaf chunks (pt_leafbvh.cpp; nullptr when the scene has none or option leaf_walk=0): chunks,
    // and per chunk slot a copy of its entry's record whose lbvh field holds the entry's position
    // in its leaf (ltris: one load per test, no index indirection)
    const LNode* lnodes;
    const Tri* ltris;
    // the leaf pass's own chunks of the pre-resolved leaves (kPassChunkMax entries at most; PreLeaf
    // c0 / c1), laid out as lnodes / ltris, and per chunk slot its entry's unit normal (x, y, z, 0;
    // zero when degenerate) for the pass's second check of a chunk the cone could not skip
    const LNode* pnodes;
    const Tri* ptris;
    const float4* pnorm;
    // leaf turns of the traversal kernel pool the leaf lanes' entries over the wave (lean_leaf_pool;
    // every tree by default, option leaf_pool).  The value is the run length (2 or 4; 0: off),
    // chosen per scene by pt_capi.hip, option pool_run
    int32_t leaf_pool;
    // the traversal kernel's per-wave LDS keys (64: lean_leaf_pool's per-lane bests, the first
    // kMultiRays of them chunk_turn_multi's; set by k_wf_trace, nullptr in the other kernels)
    uint64_t* lkeys;
    // big leaves resolved before the traversal (k_wf_leafpass; the wavefront's TRAV 26x/27x
    // instances): the npre leaves of pre (device table, the largest first) are exactly the leaves of
    // at least big_leaf entries; pres[b * pres_stride + i] is queue entry i's (t, position) key for
    // leaf b (set by k_wf_trace from its part's WfBuffers; nullptr elsewhere)
    const PreLeaf* pre;
    int32_t npre;
    uint32_t pres_stride;
    const uint64_t* pres;
    int32_t pre_rec0[kMaxPre];  // pre[b].rec0 by value (kernel arguments: the traversal's slot lookup in SGPRs)
    // leaf remainders (pt_leafskip.cpp; nullptr: none or option leaf_skip=0): per node, per side,
    // kLeafAlt pairs (first record of the leaf M the ray tested last, the remainder "this leaf minus
    // M" as first record << 7 | count); the lean node step takes the remainder whose M matches
    // TravLean::last (pt_device.h lean_node_unit).  Global memory, never staged into LDS
    const int4* nalt;
};

// Per-call camera/settings block derived from the reference's 48-float meta
// (program-raymarch.wgsl:11-22, program-raymarch.ts:79-92).
struct FrameParams {
    float W, H;           // meta[0], meta[1]
    float inv_w, inv_h;   // meta[8], meta[9]
    float aspect;         // meta[10]
    float focal;          // meta[2]
    float view_half_h;    // 2 * focal * tan(vfov * 0.5), pinned tan, computed once on host
    float rr_prob;        // meta[45]
    float cam[4];         // meta[4..7]
    float M[16];          // cam_to_world, meta[28..43], column-major
    uint32_t width, height;  // u32(meta[0]), u32(meta[1])
    int32_t direct_only;  // meta[46] > 0
    int32_t max_depth;    // literal 16 in `while(depth <= 16)`, program-raymarch.wgsl:118
};

}  // namespace pt
