// pt_leafbvh.cpp — leaf chunks: the entries of each big leaf of the reference tree in chunks of up
// to 8 with a conservative skip test each (pt_layout.h LNode), so that a query tests the chunks
// near its ray instead of every entry (MedievalBoat: one leaf of 7327 entries, half the scene's
// box; pt_device.h chunk_leaf checks 64 chunks per wave step and tests 8 open ones per step).
//
// The reference tests a leaf's entries in order with a strict-< update (intersection-logic.wgsl
// :47-176, ray-triangle-intersection.wgsl:1-42), so a leaf leaves the query with the smallest
// (t, position) over its entries that report a hit, if that t beats the closest t so far.  Any
// walk that visits every entry able to report a hit at t <= the current bound gives exactly
// that.  An entry of a chunk cannot, when the ray misses (or enters after the bound) the
// chunk's box grown by the test's rounding bound: a reported hit (u, v, t) puts o + t d within
//     delta_i = eps (216 |o - v0| + 98 (|e1| + |e2|)) / (s_i |cos(d, n_i)|)
// of the triangle (eps = 2^-24; s_i = |e1 x e2| / (|e1| |e2|); first-order error of the
// reference's single-precision test with FMAs where it writes them, times 2 — DESIGN.md §5.3),
// and |cos(d, n_i)| is bounded from below over the chunk by its normal cone.  Chunks store
// A = max eps (216 |v0| + 98 (|e1| + |e2|)) / s_i and B = max 216 eps / s_i, so delta <=
// (A + B |o|) / cf; the device adds 1e-5 (|o| + max |box coordinate|) for its own slab-test
// rounding.  Degenerate entries (s_i = 0) get an unbounded delta: their chunks are never skipped.
#include <hip/hip_runtime.h>  // pt_layout.h's vector types

#include "pt_leafbvh.h"

#include <algorithm>
#include <cfloat>
#include <cmath>

namespace pt {
namespace {

constexpr double kEps = 5.9604644775390625e-8;  // 2^-24
constexpr double kK1 = 216.0, kK2 = 98.0;       // the rounding bound's coefficients (with the factor 2)
constexpr double kThin = 0.05;                  // s_i below this: the thin group
constexpr int kBins = 16;
#ifndef PT_LEAF_CONE_WEIGHT
#define PT_LEAF_CONE_WEIGHT 2.0  // the split cost's weight of a child without a bound (below)
#endif

struct Item {
    double lo[3], hi[3], c[3], n[3];  // box, centroid, unit normal (zero when degenerate)
    double na[3];                      // the normal's line, aligned to its group's axis
    double A, B;                       // this entry's terms of the node constants
    int32_t k;                         // position in the reference leaf
    int cls;                           // group: normal axis (0..2) + 3 * thin
};

float down(double x) { return std::nextafter((float)x, -FLT_MAX); }
float up(double x) { return x >= (double)FLT_MAX ? FLT_MAX : std::nextafter((float)x, FLT_MAX); }

double area(const double lo[3], const double hi[3]) {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

// node constants over items [b, e): box, cone, A, B, C
LNode make_node(const std::vector<Item>& it, size_t b, size_t e, int axis_cls) {
    LNode nd{};
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    double A = 0.0, B = 0.0, sum[3] = {0.0, 0.0, 0.0};
    bool degenerate = false;
    for (size_t i = b; i < e; ++i) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], it[i].lo[a]); hi[a] = std::max(hi[a], it[i].hi[a]); }
        A = std::max(A, it[i].A);
        B = std::max(B, it[i].B);
        const double* n = it[i].n;
        if (n[0] == 0.0 && n[1] == 0.0 && n[2] == 0.0) degenerate = true;
        const double sg = n[axis_cls] < 0.0 ? -1.0 : 1.0;  // lines, not vectors: align to the group's axis
        for (int a = 0; a < 3; ++a) sum[a] += sg * n[a];
    }
    double bmax = 0.0;
    for (int a = 0; a < 3; ++a) {
        nd.lo[a] = down(lo[a]);
        nd.hi[a] = up(hi[a]);
        bmax = std::max({bmax, std::fabs((double)nd.lo[a]), std::fabs((double)nd.hi[a])});
    }
    // cone: axis = the stored (float) direction, half-angle over the entries' normal lines
    const double ls = std::sqrt(sum[0] * sum[0] + sum[1] * sum[1] + sum[2] * sum[2]);
    double ca = 0.0, sa = 1.0;
    float af[3] = {1.0f, 0.0f, 0.0f};
    if (!degenerate && ls > 0.0) {
        for (int a = 0; a < 3; ++a) af[a] = (float)(sum[a] / ls);
        const double la = std::sqrt((double)af[0] * af[0] + (double)af[1] * af[1] + (double)af[2] * af[2]);
        double cmin = 1.0;
        for (size_t i = b; i < e; ++i) {
            const double* n = it[i].n;
            const double c = std::fabs(n[0] * af[0] + n[1] * af[1] + n[2] * af[2]) / la;
            cmin = std::min(cmin, c);
        }
        const double alpha = std::acos(std::min(1.0, cmin)) + 1e-5;
        if (alpha < 0.5 * M_PI) { ca = std::cos(alpha); sa = std::sin(alpha); }
    }
    nd.ax = af[0]; nd.ay = af[1]; nd.az = af[2];
    nd.ca = ca > 0.0 ? down(ca) : 0.0f;
    nd.sa = sa < 1.0 ? up(sa) : 1.0f;
    nd.A = degenerate ? FLT_MAX : up(A);
    nd.B = degenerate ? FLT_MAX : up(B);
    nd.C = up(1e-5 * bmax);
    nd.skip = 0;
    nd.info = -1;
    return nd;
}

// Splits: binned over centroids (space) or over the aligned normals' components (direction), 3
// axes each, chosen by the expected number of entries below a child that a ray opens: a child
// is opened when its cone admits no bound (probability ~ sin(half-angle) for uniform directions)
// or else when the ray meets its box (~ area ratio, as SAH).  Curved and closed surfaces put
// every direction into a spatially small node, so the upper levels split by direction.
void build(std::vector<Item>& it, size_t b, size_t e, int axis_cls, std::vector<LNode>& nodes, std::vector<int32_t>& lidx,
           int leaf_max) {
    const size_t me = nodes.size();
    nodes.push_back(make_node(it, b, e, axis_cls));
    const size_t n = e - b;
    if (n <= (size_t)leaf_max) {
        nodes[me].info = (int32_t)lidx.size() | (int32_t)(n << 24);
        for (size_t i = b; i < e; ++i) lidx.push_back(it[i].k);
        nodes[me].skip = (int32_t)nodes.size();
        return;
    }
    double plo[3], phi[3];
    for (int a = 0; a < 3; ++a) { plo[a] = nodes[me].lo[a]; phi[a] = nodes[me].hi[a]; }
    const double AN = std::max(area(plo, phi), 1e-300);
    struct Bin { double lo[3], hi[3], sum[3]; size_t cnt; };
    double best = DBL_MAX;
    int bkind = -1, bax = 0, bsplit = 0;
    double bkmin = 0.0, bkext = 1.0;
    std::vector<uint8_t> side(n);
    for (int kind = 0; kind < 2; ++kind)
        for (int ax = 0; ax < 3; ++ax) {
            auto key = [&](const Item& x) { return kind ? x.na[ax] : x.c[ax]; };
            double kmin = DBL_MAX, kmax = -DBL_MAX;
            for (size_t i = b; i < e; ++i) { kmin = std::min(kmin, key(it[i])); kmax = std::max(kmax, key(it[i])); }
            const double kext = kmax - kmin;
            if (!(kext > 0.0)) continue;
            auto bin_of = [&](const Item& x) { return std::min(kBins - 1, (int)((key(x) - kmin) / kext * kBins)); };
            Bin bins[kBins];
            for (auto& bn : bins) {
                for (int a = 0; a < 3; ++a) { bn.lo[a] = DBL_MAX; bn.hi[a] = -DBL_MAX; bn.sum[a] = 0.0; }
                bn.cnt = 0;
            }
            for (size_t i = b; i < e; ++i) {
                Bin& bn = bins[bin_of(it[i])];
                for (int a = 0; a < 3; ++a) {
                    bn.lo[a] = std::min(bn.lo[a], it[i].lo[a]);
                    bn.hi[a] = std::max(bn.hi[a], it[i].hi[a]);
                    bn.sum[a] += it[i].na[a];
                }
                bn.cnt++;
            }
            for (int s = 1; s < kBins; ++s) {
                double lo2[2][3], hi2[2][3], sm[2][3] = {{0, 0, 0}, {0, 0, 0}};
                size_t cnt[2] = {0, 0};
                for (int h = 0; h < 2; ++h)
                    for (int a = 0; a < 3; ++a) { lo2[h][a] = DBL_MAX; hi2[h][a] = -DBL_MAX; }
                for (int j = 0; j < kBins; ++j) {
                    const Bin& bn = bins[j];
                    if (!bn.cnt) continue;
                    const int h = j < s ? 0 : 1;
                    for (int a = 0; a < 3; ++a) {
                        lo2[h][a] = std::min(lo2[h][a], bn.lo[a]);
                        hi2[h][a] = std::max(hi2[h][a], bn.hi[a]);
                        sm[h][a] += bn.sum[a];
                    }
                    cnt[h] += bn.cnt;
                }
                if (!cnt[0] || !cnt[1]) continue;
                double axis[2][3], cmin[2] = {1.0, 1.0};
                for (int h = 0; h < 2; ++h) {
                    const double l = std::sqrt(sm[h][0] * sm[h][0] + sm[h][1] * sm[h][1] + sm[h][2] * sm[h][2]);
                    for (int a = 0; a < 3; ++a) axis[h][a] = l > 0.0 ? sm[h][a] / l : 0.0;
                    if (!(l > 0.0)) cmin[h] = 0.0;
                }
                for (size_t i = b; i < e; ++i) {
                    const int h = bin_of(it[i]) < s ? 0 : 1;
                    const double* v = it[i].na;
                    cmin[h] = std::min(cmin[h], v[0] * axis[h][0] + v[1] * axis[h][1] + v[2] * axis[h][2]);
                }
                double cost = 0.0;
                for (int h = 0; h < 2; ++h) {
                    const double sn = cmin[h] > 0.0 ? std::sqrt(std::max(0.0, 1.0 - cmin[h] * cmin[h])) : 1.0;
                    // a cone without a bound opens the child for every ray that meets the leaf's
                    // box, not just those meeting the child's: weighted 2 (scripts/leafbvh_harness.cpp:
                    // open chunks per ray 264 -> 174 on the boat; 4 and 8 weigh worse)
                    cost += (double)cnt[h] * std::min(1.0, PT_LEAF_CONE_WEIGHT * sn + (1.0 - sn) * std::min(1.0, area(lo2[h], hi2[h]) / AN));
                }
                if (cost < best) { best = cost; bkind = kind; bax = ax; bsplit = s; bkmin = kmin; bkext = kext; }
            }
        }
    size_t mid = b;
    if (bkind >= 0) {
        auto p = std::partition(it.begin() + (std::ptrdiff_t)b, it.begin() + (std::ptrdiff_t)e, [&](const Item& x) {
            const double k = bkind ? x.na[bax] : x.c[bax];
            return std::min(kBins - 1, (int)((k - bkmin) / bkext * kBins)) < bsplit;
        });
        mid = (size_t)(p - it.begin());
    }
    if (mid == b || mid == e) {  // no usable split: halve by centroid order on the widest axis
        double cl[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, ch[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (size_t i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) { cl[a] = std::min(cl[a], it[i].c[a]); ch[a] = std::max(ch[a], it[i].c[a]); }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (ch[a] - cl[a] > ch[ax] - cl[ax]) ax = a;
        mid = b + n / 2;
        std::nth_element(it.begin() + (std::ptrdiff_t)b, it.begin() + (std::ptrdiff_t)mid, it.begin() + (std::ptrdiff_t)e,
                         [&](const Item& x, const Item& y) { return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.k < y.k); });
    }
    build(it, b, mid, axis_cls, nodes, lidx, leaf_max);
    build(it, mid, e, axis_cls, nodes, lidx, leaf_max);
    nodes[me].skip = (int32_t)nodes.size();
}

}  // namespace

void build_leaf_bvh(const Tri* tris, int32_t rec0, int32_t n, std::vector<LNode>& nodes, std::vector<int32_t>& lidx,
                    int32_t& root, int32_t& end, std::vector<LNode>* tree_out, int leaf_max, int merge_max) {
    std::vector<Item> it((size_t)n);
    for (int32_t k = 0; k < n; ++k) {
        const Tri& t = tris[rec0 + k];
        const double v0[3] = {t.q0[0], t.q0[1], t.q0[2]}, e1[3] = {t.q0[3], t.q1[0], t.q1[1]},
                     e2[3] = {t.q1[2], t.q1[3], t.e2z};
        Item& x = it[(size_t)k];
        x.k = k;
        for (int a = 0; a < 3; ++a) {
            // the triangle the test sees: v0, v0 + e1, v0 + e2 (float edges)
            const double p1 = v0[a] + e1[a], p2 = v0[a] + e2[a];
            x.lo[a] = std::min({v0[a], p1, p2});
            x.hi[a] = std::max({v0[a], p1, p2});
            x.c[a] = (v0[a] + p1 + p2) / 3.0;
        }
        const double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double ln = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
        const double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
        const double l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
        const double s = (ln > 0.0 && l1 > 0.0 && l2 > 0.0 && std::isfinite(ln)) ? ln / (l1 * l2) : 0.0;
        const double lv = std::sqrt(v0[0] * v0[0] + v0[1] * v0[1] + v0[2] * v0[2]);
        int cls = 0;
        if (s > 0.0) {
            for (int a = 0; a < 3; ++a) x.n[a] = nv[a] / ln;
            for (int a = 1; a < 3; ++a)
                if (std::fabs(x.n[a]) > std::fabs(x.n[cls])) cls = a;
            x.A = kEps * (kK1 * lv + kK2 * (l1 + l2)) / s;
            x.B = kEps * kK1 / s;
        } else {
            x.n[0] = x.n[1] = x.n[2] = 0.0;
            x.A = x.B = DBL_MAX;
        }
        x.cls = cls + (s < kThin ? 3 : 0);
        const double sg = x.n[cls] < 0.0 ? -1.0 : 1.0;
        for (int a = 0; a < 3; ++a) x.na[a] = sg * x.n[a];
    }
    // groups in a fixed order; within a group the entries keep their leaf order until split
    std::stable_sort(it.begin(), it.end(), [](const Item& a, const Item& b) { return a.cls < b.cls; });
    std::vector<LNode> tree;
    std::vector<size_t> cls_end;  // per class group: the tree's size after it
    for (size_t b = 0; b < it.size();) {
        size_t e = b;
        while (e < it.size() && it[e].cls == it[b].cls) ++e;
        build(it, b, e, it[b].cls % 3, tree, lidx, leaf_max);
        cls_end.push_back(tree.size());
        b = e;
    }
    // the device checks chunks, not the tree: keep its leaf nodes, in depth-first order (a leaf
    // covers the next items of `it`); merge_max > 0: neighbours of one class group merged while
    // their entries fit merge_max (one node over the merged items)
    root = (int32_t)nodes.size();
    size_t ci = 0, item = 0, gb = 0, gcls = 0;
    int32_t ginfo = -1;  // the open merged chunk: first slot | count << 24 (-1: none)
    auto flush = [&]() {
        if (ginfo < 0) return;
        LNode g = make_node(it, gb, gb + (size_t)(ginfo >> 24), it[gb].cls % 3);
        g.info = ginfo;
        g.skip = 0;
        nodes.push_back(g);
        ginfo = -1;
    };
    for (size_t t = 0; t < tree.size(); ++t) {
        while (ci < cls_end.size() && t >= cls_end[ci]) ++ci;
        const LNode& nd = tree[t];
        if (nd.info < 0) continue;
        const int32_t cnt = nd.info >> 24;
        if (merge_max <= 0) {
            nodes.push_back(nd);
        } else {
            if (ginfo >= 0 && (gcls != ci || (ginfo >> 24) + cnt > merge_max)) flush();
            if (ginfo < 0) { ginfo = nd.info; gb = item; gcls = ci; }
            else ginfo += cnt << 24;
        }
        item += (size_t)cnt;
    }
    flush();
    end = (int32_t)nodes.size();
    if (tree_out) *tree_out = tree;
}

namespace {

struct ProbeRay {
    float o[3], d[3], inv[3];
};

// the traversal's slab test (pt_device.h ray_box): the entry distance, the exit one from inside, -1: miss
float probe_box(const ProbeRay& r, const float* mn, const float* mx) {
    float tmin = -3.0e+38f, tmax = 3.0e+38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (mn[a] - r.o[a]) * r.inv[a], t2 = (mx[a] - r.o[a]) * r.inv[a];
        tmin = std::fmax(tmin, std::fmin(t1, t2));
        tmax = std::fmin(tmax, std::fmax(t1, t2));
    }
    return (tmax > std::fmax(tmin, 0.0f)) ? (tmin > 0.0f ? tmin : tmax) : -1.0f;
}

// the triangle test (ray-triangle-intersection.wgsl:1-42; pt_device.h tri_hit)
bool probe_tri(const Tri& tr, const ProbeRay& r, float& t) {
    const float eps = 1e-8f;
    const float v0[3] = {tr.q0[0], tr.q0[1], tr.q0[2]}, e1[3] = {tr.q0[3], tr.q1[0], tr.q1[1]},
                e2[3] = {tr.q1[2], tr.q1[3], tr.e2z};
    auto cross = [](const float* a, const float* b, float* c) {
        c[0] = a[1] * b[2] - a[2] * b[1];
        c[1] = a[2] * b[0] - a[0] * b[2];
        c[2] = a[0] * b[1] - a[1] * b[0];
    };
    auto dot = [](const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    float rce2[3], sce1[3];
    cross(r.d, e2, rce2);
    const float det = dot(e1, rce2);
    if (det > -eps && det < eps) return false;
    const float inv_det = 1.0f / det;
    const float sv[3] = {r.o[0] - v0[0], r.o[1] - v0[1], r.o[2] - v0[2]};
    const float u = inv_det * dot(sv, rce2);
    if (u < 0.0f || u > 1.0f) return false;
    cross(sv, e1, sce1);
    const float v = inv_det * dot(r.d, sce1);
    if (v < 0.0f || u + v > 1.0f) return false;
    t = inv_det * dot(e2, sce1);
    return t > eps;
}

}  // namespace

void probe_pre_leaves(const std::vector<Node>& nodes, const std::vector<Tri>& tris, const std::vector<Light>& lights,
                      const std::vector<PreLeaf>& pre, const ProbeCamera& cam, int grid, uint64_t max_tests,
                      std::vector<std::array<uint32_t, 2>>& out) {
    out.assign(pre.size(), {0u, 0u});
    if (pre.empty() || nodes.empty() || tris.empty()) return;
    uint64_t st = 0x9e3779b97f4a7c15ull;  // xorshift64
    auto next = [&]() {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return st;
    };
    auto unif = [&]() { return (float)((double)(next() >> 40) * (1.0 / 16777216.0)); };
    uint64_t tests = 0;
    std::vector<int32_t> stack;
    // one query: counts the filters passed and the leaves visited; the closest hit (record, t)
    auto query = [&](const float o[3], const float d[3], int32_t& hit, float& hit_t) {
        ProbeRay r;
        for (int c = 0; c < 3; ++c) {
            r.o[c] = o[c];
            r.d[c] = d[c];
            r.inv[c] = 1.0f / d[c];
        }
        for (size_t p = 0; p < pre.size(); ++p) {  // k_wf_leafpass's box filter
            bool pass = true;
            for (int j = 0; j < pre[p].npath && pass; ++j) {
                const int32_t step = pre[p].path[j];
                const Node& nd = nodes[(size_t)(step >> 1)];
                pass = 0.0f < ((step & 1) ? probe_box(r, nd.rmin, nd.rmax) : probe_box(r, nd.lmin, nd.lmax));
            }
            out[p][0] += pass ? 1u : 0u;
        }
        float best_t = -1.0f;
        int32_t best = -1;
        auto leaf = [&](int32_t rec0, int32_t n) {
            for (size_t p = 0; p < pre.size(); ++p) out[p][1] += (pre[p].rec0 == rec0 && pre[p].n == n) ? 1u : 0u;
            for (int32_t i = 0; i < n; ++i) {
                float t = 0.0f;
                if (probe_tri(tris[(size_t)(rec0 + i)], r, t) && (best_t < 0.0f || t < best_t)) {
                    best_t = t;
                    best = rec0 + i;
                }
            }
            tests += (uint64_t)n;
        };
        int32_t node = 0;
        stack.clear();
        for (;;) {
            const Node& nd = nodes[(size_t)node];
            const float ld = probe_box(r, nd.lmin, nd.lmax), rd = probe_box(r, nd.rmin, nd.rmax);
            const bool li = 0.0f < ld, ri = 0.0f < rd, lleaf = nd.lcnt >= 0, rleaf = nd.rcnt >= 0;
            if (li && lleaf && nd.lcnt > 0) leaf(nd.lref, nd.lcnt);
            if (ri && rleaf && nd.rcnt > 0) leaf(nd.rref, nd.rcnt);
            const bool tl = li && !lleaf && !(best_t > 0.0f && ld > best_t);
            const bool tr = ri && !rleaf && !(best_t > 0.0f && rd > best_t);
            if (tl && tr) {
                stack.push_back(nd.lref);
                node = nd.rref;
            } else if (tr || tl) {
                node = tr ? nd.rref : nd.lref;
            } else {
                if (stack.empty()) break;
                node = stack.back();
                stack.pop_back();
            }
        }
        hit = best;
        hit_t = best_t;
    };
    auto normalize = [](float v[3]) {
        const float l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (l > 0.0f) for (int c = 0; c < 3; ++c) v[c] /= l;
    };
    // the hit point and the record's unit normal
    auto hit_frame = [&](const float o[3], const float d[3], int32_t rec, float t, float p[3], float n[3]) {
        const Tri& tr = tris[(size_t)rec];
        const float e1[3] = {tr.q0[3], tr.q1[0], tr.q1[1]}, e2[3] = {tr.q1[2], tr.q1[3], tr.e2z};
        n[0] = e1[1] * e2[2] - e1[2] * e2[1];
        n[1] = e1[2] * e2[0] - e1[0] * e2[2];
        n[2] = e1[0] * e2[1] - e1[1] * e2[0];
        normalize(n);
        for (int c = 0; c < 3; ++c) p[c] = o[c] + t * d[c];
    };
    // the NEE query: toward a random point of a random light, from the hit lifted along its normal
    auto shadow = [&](const float p[3], const float n[3]) {
        if (lights.empty()) return;
        const Light& l = lights[(size_t)(next() % lights.size())];
        float a = unif(), b = unif();
        if (a + b > 1.0f) { a = 1.0f - a; b = 1.0f - b; }
        float o[3], d[3];
        for (int c = 0; c < 3; ++c) {
            o[c] = p[c] + 1e-4f * n[c];
            d[c] = l.p0[c] + a * (l.p1[c] - l.p0[c]) + b * (l.p2[c] - l.p0[c]) - o[c];
        }
        normalize(d);
        int32_t h = -1;
        float t = 0.0f;
        query(o, d, h, t);
    };
    for (int j = 0; j < grid && tests < max_tests; ++j) {
        for (int i = 0; i < grid && tests < max_tests; ++i) {
            const float vx = cam.half_w * ((i + 0.5f) / grid - 0.5f), vy = cam.half_h * (0.5f - (j + 0.5f) / grid);
            const float z = -cam.focal;
            const float* M = cam.M;
            float d[3] = {M[12] + M[8] * z + M[4] * vy + M[0] * vx - cam.cam[0],
                          M[13] + M[9] * z + M[5] * vy + M[1] * vx - cam.cam[1],
                          M[14] + M[10] * z + M[6] * vy + M[2] * vx - cam.cam[2]};
            normalize(d);
            int32_t h = -1;
            float t = 0.0f, p[3], n[3];
            query(cam.cam, d, h, t);
            if (h < 0) continue;
            hit_frame(cam.cam, d, h, t, p, n);
            shadow(p, n);
            // one cosine bounce about the normal facing the ray
            float f[3] = {n[0], n[1], n[2]};
            if (f[0] * d[0] + f[1] * d[1] + f[2] * d[2] > 0.0f) for (int c = 0; c < 3; ++c) f[c] = -f[c];
            const float u1 = unif(), u2 = unif(), rr = std::sqrt(u1), phi = 6.2831853f * u2;
            const float tv[3] = {std::fabs(f[0]) > 0.5f ? 0.0f : 1.0f, std::fabs(f[0]) > 0.5f ? 1.0f : 0.0f, 0.0f};
            float b1[3] = {tv[1] * f[2] - tv[2] * f[1], tv[2] * f[0] - tv[0] * f[2], tv[0] * f[1] - tv[1] * f[0]};
            normalize(b1);
            const float b2[3] = {f[1] * b1[2] - f[2] * b1[1], f[2] * b1[0] - f[0] * b1[2], f[0] * b1[1] - f[1] * b1[0]};
            const float lx = rr * std::cos(phi), ly = rr * std::sin(phi), lz = std::sqrt(std::fmax(0.0f, 1.0f - u1));
            float bd[3], bo[3];
            for (int c = 0; c < 3; ++c) bd[c] = b1[c] * lx + b2[c] * ly + f[c] * lz;
            normalize(bd);
            for (int c = 0; c < 3; ++c) bo[c] = p[c] + 0.001f * bd[c];
            query(bo, bd, h, t);
            if (h < 0) continue;
            hit_frame(bo, bd, h, t, p, n);
            shadow(p, n);
        }
    }
}

}  // namespace pt
