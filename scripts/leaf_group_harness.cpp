// scripts/leaf_group_harness.cpp — two-level chunk checks for the boat's big leaf.
//
// chunk_leaf (pt_device.h) checks every chunk of a big leaf against the ray: 1,521 checks per ray
// on the boat's 7,327-entry leaf, ~24 wave steps of ~45 VALU, against ~15 steps of triangle tests
// (profiles/r04_leaf_order.txt: 173 open chunks, 933 tests).  The build tree above the chunks
// (pt_leafbvh.cpp) has nodes with the same skip rule; a node's rule covers every entry below it, so
// a skipped node skips its chunks exactly.  This harness cuts the tree into groups (the maximal
// subtrees of at most S chunks), checks the groups first and only the chunks of open groups,
// and counts per ray: group checks, chunk checks, open chunks and tests, under today's schedule
// (bound tightened every 64 gathered chunks), with the same ray families as
// scripts/leaf_order_harness.cpp; outcomes are checked against the sequential loop.
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off
//        -I brown-cs2240-path-tracer_amd/csrc scripts/leaf_group_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
// Run:   ./a.out boat_leaf.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "pt_leafbvh.h"

using namespace pt;

static bool tri_hit(const Tri& T, const float o[3], const float d[3], float& t) {
    const float e1[3] = {T.q0[3], T.q1[0], T.q1[1]}, e2[3] = {T.q1[2], T.q1[3], T.e2z}, v0[3] = {T.q0[0], T.q0[1], T.q0[2]};
    auto cross = [](const float a[3], const float b[3], float r[3]) {
        r[0] = std::fmaf(a[1], b[2], -(a[2] * b[1]));
        r[1] = std::fmaf(a[2], b[0], -(a[0] * b[2]));
        r[2] = std::fmaf(a[0], b[1], -(a[1] * b[0]));
    };
    auto dot = [](const float a[3], const float b[3]) { return std::fmaf(a[2], b[2], std::fmaf(a[1], b[1], a[0] * b[0])); };
    float h[3], q[3];
    cross(d, e2, h);
    const float det = dot(e1, h);
    const float inv = 1.0f / det;
    const float s[3] = {o[0] - v0[0], o[1] - v0[1], o[2] - v0[2]};
    const float u = inv * dot(s, h);
    cross(s, e1, q);
    const float v = inv * dot(d, q);
    t = inv * dot(e2, q);
    const bool ok_det = !(det > -1e-8f && det < 1e-8f);
    const float lo = std::fmin(u, v), hi = std::fmax(u, u + v);
    return ok_det && !(lo < 0.0f) && !(hi > 1.0f) && (t > 1e-8f);
}

// pt_device.h chunk_skip: true = skip
static bool skip(const LNode& q, const float o[3], const float d[3], const float inv[3], float on, float bound) {
    const float cb = std::fabs(d[0] * q.ax + d[1] * q.ay + d[2] * q.az);
    const float sb = std::sqrt(std::fmax(0.f, 1 - cb * cb));
    const float cf = cb * q.ca - sb * q.sa - 1e-5f;
    if (!(cf > 1e-4f)) return false;
    const float dl = (q.A + q.B * on) / cf * 1.00001f + 1e-5f * on + q.C;
    if (!(dl < 1e30f)) return false;
    float tn = -3e38f, tf = 3e38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (q.lo[a] - dl - o[a]) * inv[a], t2 = (q.hi[a] + dl - o[a]) * inv[a];
        tn = std::fmax(tn, std::fmin(t1, t2));
        tf = std::fmin(tf, std::fmax(t1, t2));
    }
    return (tf < tn) || (tf < 0) || (tn > bound);
}

struct Group {
    int node;          // tree node (its LNode is the group's check)
    int first, count;  // its chunks [first, first + count) (chunk numbers from 0)
};

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<Tri> tris;
    Tri t;
    while (std::fread(&t, sizeof t, 1, f) == 1) tris.push_back(t);
    std::fclose(f);
    const int n = (int)tris.size();
    std::vector<LNode> ch, tree;
    std::vector<int32_t> lidx;
    int32_t root = 0, end = 0;
    build_leaf_bvh(tris.data(), 0, n, ch, lidx, root, end, &tree);
    const int nc = end - root;
    // chunk ordinal of each tree leaf, and leaves below each node
    std::vector<int> ord(tree.size(), -1), below(tree.size(), 0), first(tree.size(), 0);
    for (int i = 0, k = 0; i < (int)tree.size(); ++i)
        if (tree[(size_t)i].info >= 0) ord[(size_t)i] = k++;
    for (int i = (int)tree.size() - 1; i >= 0; --i) {
        int cnt = 0, fst = 1 << 30;
        for (int j = i; j < tree[(size_t)i].skip; ++j)
            if (ord[(size_t)j] >= 0) { ++cnt; fst = std::min(fst, ord[(size_t)j]); }
        below[(size_t)i] = cnt;
        first[(size_t)i] = fst;
    }
    std::printf("entries %d chunks %d tree nodes %zu\n", n, nc, tree.size());
    for (int S : {1, 4, 8, 16, 32, 64}) {
        std::vector<Group> groups;
        for (int i = 0; i < (int)tree.size();) {
            if (below[(size_t)i] <= S) {
                groups.push_back({i, first[(size_t)i], below[(size_t)i]});
                i = tree[(size_t)i].skip;
            } else {
                ++i;  // descend: the children follow in depth-first order
            }
        }
        for (int family = 0; family < 2; ++family)
            for (int with_prior = 0; with_prior < 2; ++with_prior) {
                std::mt19937 rng(5 + family * 2 + with_prior);
                std::uniform_real_distribution<float> U(0, 1);
                std::normal_distribution<float> N(0, 1);
                const int R = 1000;
                double gchecks = 0, cchecks = 0, open = 0, tests = 0, bad = 0, steps = 0;
                for (int r = 0; r < R; ++r) {
                    const int k = (int)(rng() % (unsigned)n);
                    float bu = U(rng), bv = U(rng);
                    if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
                    const Tri& T = tris[(size_t)k];
                    const float P[3] = {T.q0[0] + bu * T.q0[3] + bv * T.q1[2], T.q0[1] + bu * T.q1[0] + bv * T.q1[3],
                                        T.q0[2] + bu * T.q1[1] + bv * T.e2z};
                    float o[3], d[3];
                    if (family == 0) {
                        for (int a = 0; a < 3; ++a) o[a] = P[a] + 10 * U(rng) - 5;
                        for (int a = 0; a < 3; ++a) d[a] = N(rng);
                    } else {
                        float w[3] = {N(rng), N(rng), N(rng)};
                        const float wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                        const float dist = std::exp2(-10.0f + 14.3f * U(rng));
                        for (int a = 0; a < 3; ++a) { o[a] = P[a] + dist * w[a] / wl; d[a] = P[a] - o[a]; }
                    }
                    const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                    for (int a = 0; a < 3; ++a) d[a] /= l;
                    const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
                    const float on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
                    float lt = INFINITY;
                    for (int j = 0; j < n; ++j) {
                        float tt;
                        if (tri_hit(tris[(size_t)j], o, d, tt) && tt < lt) lt = tt;
                    }
                    const float prior = (with_prior && std::isfinite(lt)) ? lt * (0.05f + 0.95f * U(rng)) : INFINITY;
                    const float answer = std::fmin(prior, lt);
                    // schedule: groups checked 64 per step; the chunks of open groups queued and
                    // checked 64 per step; open chunks gathered and tested 64 at a time (the bound
                    // tightened after each test pass)
                    float bt = INFINITY, bound = prior;
                    std::vector<int> cq, gathered;
                    auto test_gathered = [&]() {
                        steps += 8;  // one test pass: up to 8 entries per lane
                        for (int c : gathered) {
                            const LNode& q = ch[(size_t)(root + c)];
                            const int fst = q.info & 0xffffff, cnt = q.info >> 24;
                            for (int j = 0; j < cnt; ++j) {
                                float tt;
                                tests++;
                                if (tri_hit(tris[(size_t)lidx[(size_t)(fst + j)]], o, d, tt) && tt < bt) bt = tt;
                            }
                        }
                        gathered.clear();
                        bound = std::fmin(prior, bt);
                    };
                    auto check_chunks = [&](size_t upto) {  // check queued chunks, 64 per step
                        while (cq.size() >= upto && !cq.empty()) {
                            const size_t m = std::min<size_t>(64, cq.size());
                            steps += 1;
                            std::vector<int> opened;
                            for (size_t i = 0; i < m; ++i) {
                                cchecks++;
                                if (!skip(ch[(size_t)(root + cq[i])], o, d, inv, on, bound)) opened.push_back(cq[i]);
                            }
                            cq.erase(cq.begin(), cq.begin() + (std::ptrdiff_t)m);
                            open += (double)opened.size();
                            if (gathered.size() + opened.size() > 64) test_gathered();
                            gathered.insert(gathered.end(), opened.begin(), opened.end());
                            if (upto == 0 && cq.empty()) break;
                        }
                    };
                    for (size_t gb = 0; gb < groups.size(); gb += 64) {
                        steps += 1;
                        for (size_t g = gb; g < std::min(groups.size(), gb + 64); ++g) {
                            gchecks++;
                            const Group& G = groups[g];
                            if (G.count == 1) {  // a lone chunk: the group check is the chunk check
                                if (!skip(tree[(size_t)G.node], o, d, inv, on, bound)) {
                                    open++;
                                    if (gathered.size() == 64) test_gathered();
                                    gathered.push_back(G.first);
                                }
                                continue;
                            }
                            if (skip(tree[(size_t)G.node], o, d, inv, on, bound)) continue;
                            for (int c = 0; c < G.count; ++c) cq.push_back(G.first + c);
                        }
                        check_chunks(64);
                    }
                    check_chunks(0);
                    if (!gathered.empty()) test_gathered();
                    const float got = std::fmin(prior, bt);
                    if (!(got == answer || (std::isinf(got) && std::isinf(answer)))) bad++;
                }
                std::printf("S %2d groups %4zu  %-5s rays %-4s prior: group checks %6.1f chunk checks %6.1f open %6.1f tests %6.1f "
                            "wave steps ~%5.1f (checks 1, test pass 8) mismatches %.0f\n",
                            S, groups.size(), family == 0 ? "near" : "aimed", with_prior ? "with" : "no", gchecks / R,
                            cchecks / R, open / R, tests / R, steps / R, bad);
            }
    }
    return 0;
}
