// pt_leafskip.cpp — leaf remainders: an exact skip of the leaf entries a ray tested in the leaf it
// tested just before (host build; device side pt_device.h lean_node_unit, SceneView::nalt).
//
// The reference's builder assigns a triangle whose box straddles a split to both children
// (src/ts-util/bvh.ts:136-137), so one (i0, i1, i2, material) entry sits in several leaves — Glossy:
// 5,436 leaf entries for 1,112 distinct — and a ray tests ~35 % of its entries a second time
// (profiles/r04_glossy_repeats.txt).  A leaf child is tested in full whenever its box is entered
// (intersection-logic.wgsl:58-123), with the strict-< update (:117): once a leaf M is done, every
// entry of M either misses the ray or hits it at t >= the closest t, and the closest t only
// decreases — so testing an entry of M again can never change the closest hit, and skipping it is
// exact (the node pruning reads the same closest t).  Within one leaf the first of equal-t hits in
// entry order wins; a remainder keeps the order of the entries it keeps, and a skipped entry never
// wins, so ties resolve as before.
//
// The per-ray state is one int: the first record of the last non-empty leaf the ray tested
// (TravLean::last).  For a leaf L, `alts` earlier leaves M are chosen, and for each the remainder
// "L minus M" — L's records whose uid M holds removed, order kept — is appended to the records.
// A node step that enters a leaf child L whose ray came from one of its M tests that remainder
// instead (nalt: per node and side, `alts` pairs (M's first record, remainder first record << 7 |
// count)).  scripts/leaf_repeats_ring.py measured the catch on host models of the reference
// traversal: of Glossy's 18.5 repeated tests per ray (52.5 tests), the last leaf holds 15.1; four
// probe-chosen leaves per L catch 14.1, the nearest earlier leaves alone 11.1.
#include <hip/hip_runtime.h>  // pt_layout.h's vector types

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "pt_leafbvh.h"

namespace pt {

namespace {

struct SkipRay {
    float o[3], d[3], inv[3];
};

float skip_box(const SkipRay& r, const float* mn, const float* mx) {
    float tmin = -3.0e+38f, tmax = 3.0e+38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (mn[a] - r.o[a]) * r.inv[a], t2 = (mx[a] - r.o[a]) * r.inv[a];
        tmin = std::fmax(tmin, std::fmin(t1, t2));
        tmax = std::fmin(tmax, std::fmax(t1, t2));
    }
    return (tmax > std::fmax(tmin, 0.0f)) ? (tmin > 0.0f ? tmin : tmax) : -1.0f;
}

bool skip_tri(const Tri& tr, const SkipRay& r, float& t) {
    const float eps = 1e-8f;
    const float v0[3] = {tr.q0[0], tr.q0[1], tr.q0[2]}, e1[3] = {tr.q0[3], tr.q1[0], tr.q1[1]},
                e2[3] = {tr.q1[2], tr.q1[3], tr.e2z};
    const float h[3] = {r.d[1] * e2[2] - r.d[2] * e2[1], r.d[2] * e2[0] - r.d[0] * e2[2], r.d[0] * e2[1] - r.d[1] * e2[0]};
    const float det = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
    if (det > -eps && det < eps) return false;
    const float f = 1.0f / det;
    const float s[3] = {r.o[0] - v0[0], r.o[1] - v0[1], r.o[2] - v0[2]};
    const float u = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
    if (u < 0.0f || u > 1.0f) return false;
    const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = f * (r.d[0] * q[0] + r.d[1] * q[1] + r.d[2] * q[2]);
    if (v < 0.0f || u + v > 1.0f) return false;
    t = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
    return t > eps;
}

}  // namespace

void build_leaf_skips(const std::vector<Node>& nodes, std::vector<Tri>& tris, std::vector<float4>& tnorm,
                      const std::vector<Light>& lights, int max_leaf, int alts, uint64_t max_tests,
                      std::vector<int2>& nalt, LeafSkipStats* stats) {
    nalt.clear();
    if (stats) *stats = LeafSkipStats{};
    if (alts <= 0 || nodes.empty() || tris.empty()) return;
    max_leaf = std::min(max_leaf, kLeafSkipMaxLeaf);
    // the leaves (non-empty leaf children), by first record; their uid sets, sorted
    std::unordered_map<int32_t, int32_t> leaf_of;  // first record -> leaf index
    std::vector<int32_t> rec0, cnt;
    for (const Node& nd : nodes) {
        for (int side = 0; side < 2; ++side) {
            const int32_t c = side ? nd.rcnt : nd.lcnt, ref = side ? nd.rref : nd.lref;
            if (c <= 0 || leaf_of.count(ref)) continue;
            leaf_of.emplace(ref, (int32_t)rec0.size());
            rec0.push_back(ref);
            cnt.push_back(c);
        }
    }
    const size_t nl = rec0.size();
    std::vector<std::vector<int32_t>> uids(nl);
    for (size_t l = 0; l < nl; ++l) {
        for (int32_t k = 0; k < cnt[l]; ++k) uids[l].push_back(tris[(size_t)(rec0[l] + k)].uid);
        std::sort(uids[l].begin(), uids[l].end());
    }
    auto shared = [&](size_t a, size_t b) {
        size_t i = 0, j = 0, n = 0;
        while (i < uids[a].size() && j < uids[b].size()) {
            if (uids[a][i] < uids[b][j]) ++i;
            else if (uids[a][i] > uids[b][j]) ++j;
            else { ++n; ++i; ++j; }
        }
        return n;
    };
    // the fixed visit order of leaves (intersection-logic.wgsl:31-212): a node tests its leaf
    // children, left then right, then visits its internal children, the right one first
    std::vector<int32_t> order, opos(nl, -1);
    {
        std::vector<int32_t> st{0};
        while (!st.empty()) {
            const Node& nd = nodes[(size_t)st.back()];
            st.pop_back();
            if (nd.lcnt > 0) order.push_back(leaf_of[nd.lref]);
            if (nd.rcnt > 0) order.push_back(leaf_of[nd.rref]);
            if (nd.lcnt < 0 && nd.lref > 0 && (size_t)nd.lref < nodes.size()) st.push_back(nd.lref);  // after the right subtree
            if (nd.rcnt < 0 && nd.rref > 0 && (size_t)nd.rref < nodes.size()) st.push_back(nd.rref);
        }
        for (size_t k = 0; k < order.size(); ++k) opos[(size_t)order[k]] = (int32_t)k;
    }
    // the probe: rays from random points of random distinct entries in uniform directions, and from
    // each hit one ray toward a random point of a random light; the reference traversal in f32
    // counts (L, the ray's last leaf before L)
    std::unordered_map<uint64_t, uint32_t> seen_pair;
    {
        std::vector<int32_t> firsts;
        {
            std::vector<char> got;
            for (size_t r = 0; r < tris.size(); ++r) {
                const int32_t u = tris[r].uid;
                if (u < 0) continue;
                if ((size_t)u >= got.size()) got.resize((size_t)u + 1, 0);
                if (!got[(size_t)u]) { got[(size_t)u] = 1; firsts.push_back((int32_t)r); }
            }
        }
        uint64_t st = 0x2545f4914f6cdd1dull;
        auto next = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
        auto unif = [&]() { return (float)((double)(next() >> 40) * (1.0 / 16777216.0)); };
        uint64_t tests = 0;
        std::vector<int32_t> stack;
        auto query = [&](const float o[3], const float d[3], int32_t& hit, float& hit_t) {
            SkipRay r;
            for (int c = 0; c < 3; ++c) { r.o[c] = o[c]; r.d[c] = d[c]; r.inv[c] = 1.0f / d[c]; }
            float best_t = -1.0f;
            int32_t best = -1, last = -1;
            auto leaf = [&](int32_t ref, int32_t n) {
                const int32_t l = leaf_of[ref];
                if (last >= 0) seen_pair[(uint64_t)(uint32_t)l << 32 | (uint32_t)last]++;
                for (int32_t i = 0; i < n; ++i) {
                    float t = 0.0f;
                    if (skip_tri(tris[(size_t)(ref + i)], r, t) && (best_t < 0.0f || t < best_t)) { best_t = t; best = ref + i; }
                }
                tests += (uint64_t)n;
                last = l;
            };
            int32_t node = 0;
            stack.clear();
            for (;;) {
                const Node& nd = nodes[(size_t)node];
                const float ld = skip_box(r, nd.lmin, nd.lmax), rd = skip_box(r, nd.rmin, nd.rmax);
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
        const int kRays = 1 << 15;
        for (int k = 0; k < kRays && tests < max_tests && !firsts.empty(); ++k) {
            const Tri& tr = tris[(size_t)firsts[(size_t)(next() % firsts.size())]];
            float a = unif(), b = unif();
            if (a + b > 1.0f) { a = 1.0f - a; b = 1.0f - b; }
            float d[3];
            do {
                for (int c = 0; c < 3; ++c) d[c] = 2.0f * unif() - 1.0f;
            } while (d[0] * d[0] + d[1] * d[1] + d[2] * d[2] > 1.0f || d[0] * d[0] + d[1] * d[1] + d[2] * d[2] < 1e-4f);
            normalize(d);
            const float e1[3] = {tr.q0[3], tr.q1[0], tr.q1[1]}, e2[3] = {tr.q1[2], tr.q1[3], tr.e2z};
            float o[3];
            for (int c = 0; c < 3; ++c) o[c] = tr.q0[c] + a * e1[c] + b * e2[c] + 1e-4f * d[c];
            int32_t h = -1;
            float t = 0.0f;
            query(o, d, h, t);
            if (h < 0 || lights.empty()) continue;
            const Light& lt = lights[(size_t)(next() % lights.size())];
            float la = unif(), lb = unif();
            if (la + lb > 1.0f) { la = 1.0f - la; lb = 1.0f - lb; }
            float p[3], sd[3];
            for (int c = 0; c < 3; ++c) {
                p[c] = o[c] + t * d[c] - 1e-4f * d[c];
                sd[c] = lt.p0[c] + la * (lt.p1[c] - lt.p0[c]) + lb * (lt.p2[c] - lt.p0[c]) - p[c];
            }
            normalize(sd);
            query(p, sd, h, t);
        }
        if (stats) stats->probe_tests = tests;
    }
    // per leaf L: up to `alts` earlier leaves M sharing entries with it — the probe's most frequent
    // last leaves before L weighted by what they share, then the nearest sharing predecessors in
    // the visit order
    std::vector<std::vector<std::pair<double, int32_t>>> cand(nl);
    for (const auto& kv : seen_pair) {
        const size_t l = (size_t)(kv.first >> 32), m = (size_t)(uint32_t)kv.first;
        const size_t sh = shared(l, m);
        if (sh) cand[l].emplace_back((double)kv.second * (double)sh, (int32_t)m);
    }
    nalt.assign(nodes.size() * 2 * (size_t)alts, make_int2(INT32_MIN, 0));
    std::vector<std::vector<int2>> chosen(nl);  // (M's first record, desc) per leaf
    const size_t cap = tris.size();  // the remainders' records at most double the scene's
    size_t added = 0;
    for (size_t l = 0; l < nl; ++l) {
        if (cnt[l] >= max_leaf) continue;
        auto& c = cand[l];
        std::sort(c.begin(), c.end(), [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) {
            return x.first > y.first || (x.first == y.first && x.second < y.second);
        });
        std::vector<int32_t> ms;
        for (const auto& x : c) {
            if ((int)ms.size() >= alts) break;
            ms.push_back(x.second);
        }
        for (int32_t k = opos[l] - 1, look = 0; k >= 0 && (int)ms.size() < alts && look < 64; --k, ++look) {
            const int32_t m = order[(size_t)k];
            if (std::find(ms.begin(), ms.end(), m) == ms.end() && shared(l, (size_t)m)) ms.push_back(m);
        }
        for (int32_t m : ms) {
            std::vector<int32_t> keep;
            for (int32_t k = 0; k < cnt[l]; ++k) {
                const int32_t u = tris[(size_t)(rec0[l] + k)].uid;
                if (!std::binary_search(uids[(size_t)m].begin(), uids[(size_t)m].end(), u)) keep.push_back(k);
            }
            if ((int32_t)keep.size() == cnt[l]) continue;
            const size_t start = tris.size();
            if (added + keep.size() > cap || start + keep.size() >= ((size_t)1 << 24)) break;
            for (int32_t k : keep) {
                Tri t = tris[(size_t)(rec0[l] + k)];
                t.lbvh = 0;
                tris.push_back(t);
                for (int q = 0; q < 3; ++q) {
                    const float4 vn = tnorm[3 * (size_t)(rec0[l] + k) + q];
                    tnorm.push_back(vn);
                }
            }
            added += keep.size();
            chosen[l].push_back(make_int2(rec0[(size_t)m], (int32_t)(start << 7) | (int32_t)keep.size()));
            if (stats) { stats->remainders++; stats->skipped += (uint64_t)(cnt[l] - (int32_t)keep.size()); }
        }
    }
    for (size_t n = 0; n < nodes.size(); ++n) {
        for (int side = 0; side < 2; ++side) {
            const int32_t c = side ? nodes[n].rcnt : nodes[n].lcnt, ref = side ? nodes[n].rref : nodes[n].lref;
            if (c <= 0) continue;
            const auto& ch = chosen[(size_t)leaf_of[ref]];
            for (size_t a = 0; a < ch.size(); ++a) nalt[(n * 2 + (size_t)side) * (size_t)alts + a] = ch[a];
        }
    }
    if (stats) stats->records = added;
}

}  // namespace pt
