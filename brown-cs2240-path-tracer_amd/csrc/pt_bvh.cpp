// pt_bvh.cpp — native BVH build + pack (host C++, no GPU): SURVEY.md §8(f) row 2.
//
// Same algorithm as src/ts-util/bvh.ts:14-188 and src/packer.ts:83-137 (restated in the Node
// host as node/lib/bvh.js + packer.js: pack_bvh), in IEEE double exactly as the JS numbers
// are, so the packed buffer is byte-identical and the traversal (whose order and exit-distance
// pruning depend on the topology) returns the same hits:
//   * node split axis = longest of the node's strides (ties x > y > z) — js-geometry's Bounds fixes
//     its strides when constructed and bvh.ts builds a child box from its PARENT's min/max before
//     moving the split face, so a node's strides are its parent's extent (the root's its own);
//     the reference's own renders decide this semantics;
//   * 18 candidate split fractions s = 0.05, 0.05+0.05, ... accumulated in double while
//     s <= 0.95 (the last is 0.9000000000000002); cost |nL - avg| + |nR - avg| with
//     inclusive box overlap counts, first minimum wins;
//   * a triangle overlapping both halves goes to both children;
//   * a child is a leaf with <= 16 objects or when the split separated nothing; depth 16
//     (root = 1) forces a leaf;
//   * every node but the root keeps axis -1 (bvh.ts never stores the axis it passes down).
// Compiled with -ffp-contract=off: `w0 * hi + w1 * lo` must round twice, as in JS.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>

#include "../../include/pt_hip.h"

namespace {

struct Box {
    double mn[3], mx[3];
};

struct BNode {
    bool leaf = false;
    int axis = -1;
    Box box{};
    double stride[3] = {0, 0, 0};  // js-geometry Bounds.stride_* as constructed: the parent's extent
    std::vector<int32_t> objs;  // indices into the triangle list
    std::unique_ptr<BNode> l, r;
    bool objs_empty() const { return leaf && objs.empty(); }  // an empty leaf keeps its zero box
};

constexpr int kMaxDepth = 16;
constexpr size_t kMaxObjPerNode = 16;

inline bool overlap(const Box& a, const Box& b) {  // math.ts:45-49 (inclusive)
    for (int k = 0; k < 3; ++k)
        if (!(b.mn[k] <= a.mx[k] && a.mn[k] <= b.mx[k])) return false;
    return true;
}

inline Box split_box(const Box& b, int axis, double c, bool low) {
    Box o = b;
    if (low) o.mx[axis] = c; else o.mn[axis] = c;
    return o;
}

struct Builder {
    const std::vector<Box>& tb;  // triangle boxes

    void recurse(BNode& n, int depth) {
        if (depth >= kMaxDepth) { n.leaf = true; return; }
        const Box& nb = n.box;
        const double sx = n.stride[0], sy = n.stride[1], sz = n.stride[2];
        int axis;
        if (sx >= sy && sx >= sz) axis = 0;
        else if (sy >= sx && sy >= sz) axis = 1;
        else axis = 2;
        const double lo = nb.mn[axis], hi = nb.mx[axis];
        double split = 0.5, cost = std::numeric_limits<double>::infinity();
        const double step = 0.05;
        for (double s = step; s <= 1.0 - step; s += step) {
            const double w0 = s, w1 = 1.0 - s;
            const double c = w0 * hi + w1 * lo;
            const Box lb = split_box(nb, axis, c, true), hb = split_box(nb, axis, c, false);
            int nl = 0, nh = 0;
            for (int32_t o : n.objs) {
                if (overlap(tb[o], lb)) ++nl;
                if (overlap(tb[o], hb)) ++nh;
            }
            const double avg = (nl + nh) * 0.5;
            const double cur = std::fabs(nl - avg) + std::fabs(nh - avg);
            if (cur < cost) { split = s; cost = cur; }
        }
        const double c = split * hi + (1.0 - split) * lo;
        n.l = std::make_unique<BNode>();
        n.r = std::make_unique<BNode>();
        n.l->box = split_box(nb, axis, c, true);
        n.r->box = split_box(nb, axis, c, false);
        for (int k = 0; k < 3; ++k) n.l->stride[k] = n.r->stride[k] = nb.mx[k] - nb.mn[k];
        for (int32_t o : n.objs) {
            if (overlap(tb[o], n.l->box)) n.l->objs.push_back(o);
            if (overlap(tb[o], n.r->box)) n.r->objs.push_back(o);
        }
        for (BNode* ch : {n.l.get(), n.r.get()}) {
            if (ch->objs.size() <= kMaxObjPerNode || ch->objs.size() == n.objs.size()) ch->leaf = true;
            else recurse(*ch, depth + 1);
        }
    }
};

// pad (the SAH tree only; the reference's tree is packed as its builder made it): child boxes are
// written as the f32 values one ulp outside the round-to-nearest conversion of their double
// bounds, so every box has a positive extent on every axis.  The slab test
// (ray-bbox-intersection.wgsl:1-31) reports a hit only when tmax > max(tmin, 0): a zero-thickness
// box — a leaf of coplanar axis-aligned triangles such as a Cornell wall or the light — is never
// entered (the synthetic sweep scenes lost their light this way and rendered black).
double pad_lo(double v) { return (double)std::nextafter((float)v, -std::numeric_limits<float>::infinity()); }
double pad_hi(double v) { return (double)std::nextafter((float)v, std::numeric_limits<float>::infinity()); }

void pack(const BNode& n, const int32_t* tris, std::vector<double>& out, bool pad = false) {
    const size_t cur = out.size();
    const size_t nchild = n.leaf ? 4 * n.objs.size() : 0;
    const double z3[3] = {0, 0, 0};
    out.push_back(n.leaf ? 1 : 0);
    out.push_back(n.axis);
    out.push_back(n.leaf ? -1.0 : (double)(cur + 5 + 12 + nchild));
    out.push_back(-1);
    out.push_back(n.leaf ? (double)nchild : -2.0);
    for (const BNode* ch : {n.l.get(), n.r.get()}) {
        const double* mn = ch ? ch->box.mn : z3;
        const double* mx = ch ? ch->box.mx : z3;
        if (pad && ch && !ch->objs_empty()) {
            for (int k = 0; k < 3; ++k) out.push_back(pad_lo(mn[k]));
            for (int k = 0; k < 3; ++k) out.push_back(pad_hi(mx[k]));
        } else {
            out.insert(out.end(), mn, mn + 3);
            out.insert(out.end(), mx, mx + 3);
        }
    }
    if (n.leaf)
        for (int32_t o : n.objs)
            for (int q = 0; q < 4; ++q) out.push_back(tris[4 * (size_t)o + q]);
    if (!n.leaf && n.l) pack(*n.l, tris, out, pad);
    if (!n.leaf && n.r) {
        out[cur + 3] = (double)out.size();
        pack(*n.r, tris, out, pad);
    }
}

}  // namespace

extern "C" int pt_bvh_build(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count,
                            float* bvh_out, size_t bvh_cap, size_t* bvh_len) {
    if (!vertices || !tris || !bvh_len || vertex_count == 0 || tri_count == 0 || (bvh_cap && !bvh_out))
        return PT_ERR_INVALID;
    // object boxes (index.ts:140-147, bounds_of_vec3) and the root box over all vertices
    std::vector<Box> tb(tri_count);
    for (size_t t = 0; t < tri_count; ++t) {
        Box b{};
        for (int v = 0; v < 3; ++v) {
            const int32_t i = tris[4 * t + v];
            if (i < 1 || (size_t)i > vertex_count) return PT_ERR_INVALID;
            const double* p = vertices + 3 * (size_t)(i - 1);
            for (int k = 0; k < 3; ++k) {
                if (v == 0 || p[k] <= b.mn[k]) b.mn[k] = p[k];
                if (v == 0 || p[k] >= b.mx[k]) b.mx[k] = p[k];
            }
        }
        tb[t] = b;
    }
    Box root{};
    for (size_t i = 0; i < vertex_count; ++i)
        for (int k = 0; k < 3; ++k) {
            const double x = vertices[3 * i + k];
            if (i == 0 || x <= root.mn[k]) root.mn[k] = x;
            if (i == 0 || x >= root.mx[k]) root.mx[k] = x;
        }
    BNode top;
    top.axis = 0;
    top.box = root;
    for (int k = 0; k < 3; ++k) top.stride[k] = root.mx[k] - root.mn[k];
    top.objs.resize(tri_count);
    for (size_t t = 0; t < tri_count; ++t) top.objs[t] = (int32_t)t;
    Builder{tb}.recurse(top, 1);
    std::vector<double> out(root.mn, root.mn + 3);
    out.insert(out.end(), root.mx, root.mx + 3);
    pack(top, tris, out);
    *bvh_len = out.size();
    if (bvh_cap < out.size()) return bvh_cap ? PT_ERR_INVALID : PT_OK;  // cap 0: size query
    for (size_t i = 0; i < out.size(); ++i) bvh_out[i] = (float)out[i];
    return PT_OK;
}

// ---------------------------------------------------------------------------------------------
// Fast mode ("gives up topology parity"): a binned surface-area-heuristic
// build over triangle centroids — each triangle in exactly one leaf, child boxes tight around
// their triangles — written in the reference's packed layout, so the same traversal (exit-distance
// pruning and all) runs on it.  Renders differ from the reference's tree only where that pruning
// quirk bites differently; the GPU still equals the oracle on these buffers bit for bit.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kSahBins = 16;
constexpr int kSahMaxLeaf = 8;   // a node above this many triangles is always split
constexpr int kSahMaxDepth = 28; // the device stack (kStackMax 32) and the reference's 64-entry marker stack
constexpr int kSahMinLeaf = 4;    // never split below this
constexpr double kSahTraversal = 2.0;  // cost of a node step relative to one triangle test (a node tests two boxes)

double area(const Box& b) {
    const double x = b.mx[0] - b.mn[0], y = b.mx[1] - b.mn[1], z = b.mx[2] - b.mn[2];
    return (x < 0 || y < 0 || z < 0) ? 0.0 : 2.0 * (x * y + y * z + z * x);
}
Box empty_box() {
    Box b;
    for (int k = 0; k < 3; ++k) { b.mn[k] = std::numeric_limits<double>::infinity(); b.mx[k] = -b.mn[k]; }
    return b;
}
void grow(Box& b, const Box& o) {
    for (int k = 0; k < 3; ++k) { b.mn[k] = std::min(b.mn[k], o.mn[k]); b.mx[k] = std::max(b.mx[k], o.mx[k]); }
}

struct SahBuilder {
    const std::vector<Box>& tb;
    std::vector<double> cen;  // 3 per triangle

    void build(BNode& n, int depth) {
        n.box = empty_box();
        Box cb = empty_box();
        for (int32_t o : n.objs) {
            grow(n.box, tb[o]);
            for (int k = 0; k < 3; ++k) {
                cb.mn[k] = std::min(cb.mn[k], cen[3 * (size_t)o + k]);
                cb.mx[k] = std::max(cb.mx[k], cen[3 * (size_t)o + k]);
            }
        }
        const int cnt = (int)n.objs.size();
        if (cnt <= kSahMinLeaf || depth >= kSahMaxDepth) { n.leaf = true; return; }
        double best = std::numeric_limits<double>::infinity();
        int bax = -1, bsplit = 0;
        for (int ax = 0; ax < 3; ++ax) {
            const double lo = cb.mn[ax], ext = cb.mx[ax] - cb.mn[ax];
            if (!(ext > 0)) continue;
            Box bb[kSahBins];
            int bn[kSahBins] = {};
            for (int i = 0; i < kSahBins; ++i) bb[i] = empty_box();
            for (int32_t o : n.objs) {
                int i = (int)((cen[3 * (size_t)o + ax] - lo) / ext * kSahBins);
                i = std::min(std::max(i, 0), kSahBins - 1);
                bn[i]++;
                grow(bb[i], tb[o]);
            }
            double ra[kSahBins];
            int rn[kSahBins];
            Box acc = empty_box();
            int an = 0;
            for (int i = kSahBins - 1; i > 0; --i) { grow(acc, bb[i]); an += bn[i]; ra[i] = area(acc); rn[i] = an; }
            acc = empty_box();
            an = 0;
            for (int i = 0; i < kSahBins - 1; ++i) {
                grow(acc, bb[i]);
                an += bn[i];
                if (an == 0 || rn[i + 1] == 0) continue;
                const double c = area(acc) * an + ra[i + 1] * rn[i + 1];
                if (c < best) { best = c; bax = ax; bsplit = i + 1; }
            }
        }
        const double leaf_cost = (double)cnt, split_cost = kSahTraversal + best / std::max(area(n.box), 1e-300);
        if (cnt <= kSahMaxLeaf && !(split_cost < leaf_cost)) { n.leaf = true; return; }
        n.l = std::make_unique<BNode>();
        n.r = std::make_unique<BNode>();
        if (bax < 0) {  // every centroid in one point: halve the list
            n.l->objs.assign(n.objs.begin(), n.objs.begin() + cnt / 2);
            n.r->objs.assign(n.objs.begin() + cnt / 2, n.objs.end());
        } else {
            const double lo = cb.mn[bax], ext = cb.mx[bax] - cb.mn[bax];
            for (int32_t o : n.objs) {
                int i = (int)((cen[3 * (size_t)o + bax] - lo) / ext * kSahBins);
                i = std::min(std::max(i, 0), kSahBins - 1);
                (i < bsplit ? n.l : n.r)->objs.push_back(o);
            }
        }
        std::vector<int32_t>().swap(n.objs);
        build(*n.l, depth + 1);
        build(*n.r, depth + 1);
    }
};

}  // namespace

// The fast tree keeps the reference's traversal, and with it the exit-distance pruning quirk
// (intersection-logic.wgsl:178-181 with ray-bbox-intersection.wgsl:22-27): a subtree whose box
// holds the ray's origin is skipped once the closest hit so far is nearer than the box's EXIT.
// With tight SAH boxes that skip can hide the light from every shadow ray (the synthetic 1,000 and
// 12,500-triangle sweep scenes rendered black).  A leaf child of the root is tested whenever the
// ray meets its box (intersection-logic.wgsl:47-176: no pruning for leaf children), so the
// triangles of the flagged materials (the emitters, program-raymarch.wgsl:136's sum(Ke) > 0) go
// into the root's left child as ONE leaf, however many they are, and the rest of the scene into its
// right child.  (Round 4 gave more than kSahMaxLeaf emitters an SAH subtree of their own, whose
// internal nodes the pruning can still skip: a finely meshed light could be hidden, advisor r04.
// A big emitter leaf costs the rays that meet its box more tests; leaves of >= big_leaf entries
// take the traversal's big-leaf path.)
extern "C" int pt_bvh_build_sah2(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count,
                                 const uint8_t* isolate_material, size_t material_count, float* bvh_out,
                                 size_t bvh_cap, size_t* bvh_len) {
    if (!vertices || !tris || !bvh_len || vertex_count == 0 || tri_count == 0 || (bvh_cap && !bvh_out) ||
        (material_count && !isolate_material))
        return PT_ERR_INVALID;
    std::vector<Box> tb(tri_count);
    std::vector<double> cen(3 * tri_count);
    for (size_t t = 0; t < tri_count; ++t) {
        Box b = empty_box();
        for (int v = 0; v < 3; ++v) {
            const int32_t i = tris[4 * t + v];
            if (i < 1 || (size_t)i > vertex_count) return PT_ERR_INVALID;
            const double* p = vertices + 3 * (size_t)(i - 1);
            for (int k = 0; k < 3; ++k) { b.mn[k] = std::min(b.mn[k], p[k]); b.mx[k] = std::max(b.mx[k], p[k]); }
        }
        tb[t] = b;
        for (int k = 0; k < 3; ++k) cen[3 * t + k] = 0.5 * (b.mn[k] + b.mx[k]);
    }
    Box root{};
    for (size_t i = 0; i < vertex_count; ++i)
        for (int k = 0; k < 3; ++k) {
            const double x = vertices[3 * i + k];
            if (i == 0 || x <= root.mn[k]) root.mn[k] = x;
            if (i == 0 || x >= root.mx[k]) root.mx[k] = x;
        }
    std::vector<int32_t> lit, rest;
    for (size_t t = 0; t < tri_count; ++t) {
        const int32_t m = tris[4 * t + 3];
        const bool iso = m >= 0 && (size_t)m < material_count && isolate_material[m];
        (iso ? lit : rest).push_back((int32_t)t);
    }
    SahBuilder sb{tb, std::move(cen)};
    BNode top;
    top.axis = 0;
    if (!lit.empty() && !rest.empty()) {
        top.box = empty_box();
        for (size_t t = 0; t < tri_count; ++t) grow(top.box, tb[t]);
        top.l = std::make_unique<BNode>();
        top.r = std::make_unique<BNode>();
        top.l->objs = std::move(lit);
        top.r->objs = std::move(rest);
        top.l->leaf = true;  // one leaf under the root: never pruned
        top.l->box = empty_box();
        for (int32_t o : top.l->objs) grow(top.l->box, tb[o]);
        sb.build(*top.r, 2);
    } else {
        top.objs.resize(tri_count);
        for (size_t t = 0; t < tri_count; ++t) top.objs[t] = (int32_t)t;
        sb.build(top, 1);
    }
    if (top.leaf) {  // the layout needs an internal root: two leaves under it
        top.leaf = false;
        top.l = std::make_unique<BNode>();
        top.r = std::make_unique<BNode>();
        top.l->leaf = top.r->leaf = true;
        top.l->box = top.r->box = top.box;
        top.l->objs.assign(top.objs.begin(), top.objs.begin() + top.objs.size() / 2);
        top.r->objs.assign(top.objs.begin() + top.objs.size() / 2, top.objs.end());
        if (top.l->objs.empty()) top.l->box = Box{};
    }
    std::vector<double> out(root.mn, root.mn + 3);
    out.insert(out.end(), root.mx, root.mx + 3);
    pack(top, tris, out, true);
    if (out.size() >= (1u << 24)) return PT_ERR_INVALID;  // float offsets exact below 2^24 (packer.ts layout)
    *bvh_len = out.size();
    if (bvh_cap < out.size()) return bvh_cap ? PT_ERR_INVALID : PT_OK;
    for (size_t i = 0; i < out.size(); ++i) bvh_out[i] = (float)out[i];
    return PT_OK;
}

extern "C" int pt_bvh_build_sah(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count,
                                float* bvh_out, size_t bvh_cap, size_t* bvh_len) {
    return pt_bvh_build_sah2(vertices, vertex_count, tris, tri_count, nullptr, 0, bvh_out, bvh_cap, bvh_len);
}
