// scripts/leaf_order_harness.cpp — does the ORDER in which chunk_leaf checks a big leaf's chunks
// matter?    Host-side model of pt_device.h chunk_leaf on one leaf's
// records (the boat's 7,327-entry leaf: scripts/dump_boat_leaf.py), for the same two ray families
// as scripts/leafbvh_harness.cpp — origins within 5 units of a random point of an entry with
// uniform directions ("near"), and rays aimed at such a point from 10^-3 .. 20 units ("aimed") —
// each with no prior hit (a camera ray) and with the closest t of an earlier leaf as the prior
// (half the rays, uniform in (0, the leaf's own t]).  Chunks opened per ray under three bounds:
//   built   today's chunk_leaf: build order, 64 checks per block, the bound tightened only when
//           the gathered chunks (> 64) are tested;
//   ideal   every chunk checked against the leaf's final answer from the start (min(prior, the
//           sequential loop's closest t)): no order or flush schedule can open fewer;
//   near    chunks sorted by the entry distance of their grown box, one at a time, the bound
//           tightened after every chunk (the best an ordering with per-chunk flushes reaches).
// and why chunks stay open under the ideal bound: the normal cone admits no bound on |cos(d, n)|
// ("cone") or the ray enters the grown box before the bound ("box").  Outcomes are checked
// against the sequential loop (mismatches must be 0).
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off
//        -I brown-cs2240-path-tracer_amd/csrc scripts/leaf_order_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
// Run:   ./a.out leaf_records.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "pt_leafbvh.h"

using namespace pt;

// the reference's test (ray-triangle-intersection.wgsl:1-42), in float without contraction
static bool tri_hit(const Tri& T, const float o[3], const float d[3], float& t) {
    const float e1[3] = {T.q0[3], T.q1[0], T.q1[1]}, e2[3] = {T.q1[2], T.q1[3], T.e2z}, v0[3] = {T.q0[0], T.q0[1], T.q0[2]};
    const float h[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const float det = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
    if (det > -1e-8f && det < 1e-8f) return false;
    const float inv = 1.0f / det;
    const float s[3] = {o[0] - v0[0], o[1] - v0[1], o[2] - v0[2]};
    const float u = inv * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
    if (u < 0 || u > 1) return false;
    const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = inv * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
    if (v < 0 || u + v > 1) return false;
    t = inv * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
    return t > 1e-8f;
}

// pt_device.h chunk_skip: 0 skipped, 1 open (cone admits no bound), 2 open (box); tn: the grown
// box's entry distance (for the near-to-far order; +inf when the ray misses it)
static int chunk_check(const LNode& q, const float o[3], const float d[3], const float inv[3], float on, float bound,
                       float* tn_out = nullptr) {
    const float cb = std::fabs(d[0] * q.ax + d[1] * q.ay + d[2] * q.az);
    const float sb = std::sqrt(std::fmax(0.f, 1 - cb * cb));
    const float cf = cb * q.ca - sb * q.sa - 1e-5f;
    float dl = INFINITY;
    if (cf > 1e-4f) dl = (q.A + q.B * on) / cf + 1e-5f * on + q.C;
    const bool cone = !(dl < 1e30f);
    const float g = cone ? 0.0f : dl;  // the order key of a cone chunk: its plain box
    float tn = -3e38f, tf = 3e38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (q.lo[a] - g - o[a]) * inv[a], t2 = (q.hi[a] + g - o[a]) * inv[a];
        tn = std::fmax(tn, std::fmin(t1, t2));
        tf = std::fmin(tf, std::fmax(t1, t2));
    }
    if (tn_out) *tn_out = (tf < tn || tf < 0) ? INFINITY : std::fmax(tn, 0.0f);
    if (cone) return 1;
    return ((tf < tn) || (tf < 0) || (tn > bound)) ? 0 : 2;
}

struct Stats {
    double open = 0, tests = 0, cone = 0, box = 0, bad = 0;
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
    std::vector<LNode> ch;
    std::vector<int32_t> lidx;
    int32_t root = 0, end = 0;
    build_leaf_bvh(tris.data(), 0, n, ch, lidx, root, end);
    const int nc = end - root;
    std::printf("entries %d chunks %d\n", n, nc);
    for (int family = 0; family < 2; ++family)
        for (int with_prior = 0; with_prior < 2; ++with_prior) {
            std::mt19937 rng(5 + family * 2 + with_prior);
            std::uniform_real_distribution<float> U(0, 1);
            std::normal_distribution<float> N(0, 1);
            const int R = 2000;
            Stats built, ideal, near;
            int rays = 0;
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
                ++rays;
                auto test_chunk = [&](int c, float& bt, Stats& st) {
                    const int first = ch[(size_t)c].info & 0xffffff, cnt = ch[(size_t)c].info >> 24;
                    for (int j = 0; j < cnt; ++j) {
                        float tt;
                        st.tests++;
                        if (tri_hit(tris[(size_t)lidx[(size_t)(first + j)]], o, d, tt) && tt < bt) bt = tt;
                    }
                };
                auto verdict = [&](float bt, Stats& st) {
                    const float got = std::fmin(prior, bt);
                    if (!(got == answer || (std::isinf(got) && std::isinf(answer)))) st.bad++;
                };
                {  // built: chunk_leaf's schedule
                    float bt = INFINITY, bound = prior;
                    std::vector<int> gathered;
                    for (int cb = root; cb < end; cb += 64) {
                        std::vector<int> opened;
                        for (int c = cb; c < std::min(end, cb + 64); ++c) {
                            const int why = chunk_check(ch[(size_t)c], o, d, inv, on, bound);
                            if (!why) continue;
                            built.open++;
                            (why == 1 ? built.cone : built.box)++;
                            opened.push_back(c);
                        }
                        if (gathered.size() + opened.size() > 64) {
                            for (int c : gathered) test_chunk(c, bt, built);
                            gathered.clear();
                            bound = std::fmin(prior, bt);
                        }
                        gathered.insert(gathered.end(), opened.begin(), opened.end());
                    }
                    for (int c : gathered) test_chunk(c, bt, built);
                    verdict(bt, built);
                }
                {  // ideal: the final answer as the bound from the start
                    float bt = INFINITY;
                    for (int c = root; c < end; ++c) {
                        const int why = chunk_check(ch[(size_t)c], o, d, inv, on, answer);
                        if (!why) continue;
                        ideal.open++;
                        (why == 1 ? ideal.cone : ideal.box)++;
                        test_chunk(c, bt, ideal);
                    }
                    verdict(bt, ideal);
                }
                {  // near-to-far, per-chunk bound
                    std::vector<float> key((size_t)nc);
                    for (int c = root; c < end; ++c) chunk_check(ch[(size_t)c], o, d, inv, on, INFINITY, &key[(size_t)(c - root)]);
                    std::vector<int> order((size_t)nc);
                    std::iota(order.begin(), order.end(), root);
                    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[(size_t)(a - root)] < key[(size_t)(b - root)]; });
                    float bt = INFINITY;
                    for (int c : order) {
                        const int why = chunk_check(ch[(size_t)c], o, d, inv, on, std::fmin(prior, bt));
                        if (!why) continue;
                        near.open++;
                        (why == 1 ? near.cone : near.box)++;
                        test_chunk(c, bt, near);
                    }
                    verdict(bt, near);
                }
            }
            const char* fam = family == 0 ? "near" : "aimed";
            for (auto [name, st] : {std::make_pair("built", &built), std::make_pair("ideal", &ideal), std::make_pair("near-to-far", &near)})
                std::printf("%-6s rays, %-8s prior: %-11s %6.1f open chunks (cone %6.1f, box %5.1f), %7.1f tests, mismatches %.0f\n",
                            fam, with_prior ? "with" : "no", name, st->open / rays, st->cone / rays, st->box / rays,
                            st->tests / rays, st->bad);
        }
    return 0;
}
