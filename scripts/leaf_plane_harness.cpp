// scripts/leaf_plane_harness.cpp — a second skip rule for leaf chunks, by plane distance.
//
// Today's rule (pt_device.h chunk_skip) grows a chunk's box by the triangle test's rounding bound,
// which scales with 1 / |cos(d, n)|: a chunk whose normal cone holds directions perpendicular to
// the ray admits no bound and is always opened (~98 % of the open chunks on the boat's big leaf,
// profiles/r04_leaf_order.txt).  But a grazing ray reports, if anything, a t near the distance
// along the ray to the triangle's PLANE, h / |cos| with h the origin's distance to the plane —
// large for a ray nearly parallel to a plane it is not close to.  In the reference's test
// (ray-triangle-intersection.wgsl:1-42, pt_device.h tri_hit) t = N / det with
//     N   = e2 . ((o - v0) x e1) = +-h |e1 x e2|        computed with |dN|   <= c1 eps |o - v0| |e1| |e2|
//     det = e1 . (d x e2)        = +-cos |e1 x e2|      computed with |ddet| <= c2 eps |e1| |e2|
// so |t_computed| >= (h - c1 eps |o - v0| / s) / (cos + c2 eps / s) (1 - 2 eps), s = |e1 x e2| /
// (|e1| |e2|).  Over a chunk: h >= h_low = the distance of a . o from the chunk's range of a . v0
// (a = cone axis) less |n - a| |o - v0| (|n - a| <= sqrt(2 - 2 cos(half-angle))), |o - v0| <= R =
// the distance to the farthest box corner, s >= s_min, cos <= cos_max = the cone's largest
// |cos| against d.  When that lower bound exceeds the closest t so far, no entry of the chunk can
// report a hit that counts (t <= bound), or it reports t < 0: the chunk is skipped.
//
// This harness measures, on the boat's 7,327-entry leaf (scripts/dump_boat_leaf.py) and the ray
// families of scripts/leaf_order_harness.cpp, the chunks opened per ray with and without the plane
// rule under today's schedule, the ideal bound and a near-to-far order, and checks every outcome
// against the sequential loop (mismatches must be 0).  c1 = c2 = 32 (first-order constants of
// this arithmetic are <= 8).
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off
//        -I brown-cs2240-path-tracer_amd/csrc scripts/leaf_plane_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
// Run:   ./a.out boat_leaf.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "pt_leafbvh.h"

using namespace pt;

// tri_hit's arithmetic (pt_device.h; cross and dot as pt_math.h writes them, 1/det IEEE)
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

// pt_device.h chunk_skip (box rule): 0 skipped, 1 open (cone admits no bound), 2 open (box)
static int box_rule(const LNode& q, const float o[3], const float d[3], const float inv[3], float on, float bound) {
    const float cb = std::fabs(d[0] * q.ax + d[1] * q.ay + d[2] * q.az);
    const float sb = std::sqrt(std::fmax(0.f, 1 - cb * cb));
    const float cf = cb * q.ca - sb * q.sa - 1e-5f;
    if (!(cf > 1e-4f)) return 1;
    const float dl = (q.A + q.B * on) / cf * 1.00001f + 1e-5f * on + q.C;
    if (!(dl < 1e30f)) return 1;
    float tn = -3e38f, tf = 3e38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (q.lo[a] - dl - o[a]) * inv[a], t2 = (q.hi[a] + dl - o[a]) * inv[a];
        tn = std::fmax(tn, std::fmin(t1, t2));
        tf = std::fmin(tf, std::fmax(t1, t2));
    }
    return ((tf < tn) || (tf < 0) || (tn > bound)) ? 0 : 2;
}

struct Plane {  // per chunk: range of a . v0 over its entries, eps constants over s_min, |n - a| bound
    float pmin, pmax, k1, k2, g;
};

// the plane rule in f32, with slack for its own rounding: true = skip
static bool plane_rule(const LNode& q, const Plane& P, const float o[3], const float d[3], float bound) {
    if (!(bound < 3e38f)) return false;
    const float cb = std::fabs(d[0] * q.ax + d[1] * q.ay + d[2] * q.az);
    const float sb = std::sqrt(std::fmax(0.f, 1 - cb * cb));
    const float cmax = cb >= q.ca ? 1.0f : std::fmin(1.0f, cb * q.ca + sb * q.sa + 1e-5f);
    const float ao = o[0] * q.ax + o[1] * q.ay + o[2] * q.az;
    const float gap = std::fmax(P.pmin - ao, ao - P.pmax);
    float r2 = 0.0f;
    for (int a = 0; a < 3; ++a) {
        const float m = std::fmax(std::fabs(o[a] - q.lo[a]), std::fabs(o[a] - q.hi[a]));
        r2 += m * m;
    }
    const float R = std::sqrt(r2) * 1.0001f;
    const float h = gap - P.g * R - 1e-5f * (std::fabs(ao) + std::fabs(P.pmin) + std::fabs(P.pmax));
    const float num = h - P.k1 * R;
    if (!(num > 0.0f)) return false;
    const float tl = num / (cmax + P.k2) * 0.999f;
    return tl > bound;
}

struct Stats {
    double open = 0, tests = 0, bad = 0;
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
    // plane constants per chunk, from its entries in double
    const double eps = 5.9604644775390625e-8, c1 = 32.0, c2 = 32.0;
    std::vector<Plane> pl((size_t)ch.size());
    for (int c = root; c < end; ++c) {
        const LNode& q = ch[(size_t)c];
        const double la = std::sqrt((double)q.ax * q.ax + (double)q.ay * q.ay + (double)q.az * q.az);
        const double a[3] = {q.ax / la, q.ay / la, q.az / la};
        const int first = q.info & 0xffffff, cnt = q.info >> 24;
        double pmin = DBL_MAX, pmax = -DBL_MAX, smin = DBL_MAX;
        for (int j = 0; j < cnt; ++j) {
            const Tri& T = tris[(size_t)lidx[(size_t)(first + j)]];
            const double v0[3] = {T.q0[0], T.q0[1], T.q0[2]}, e1[3] = {T.q0[3], T.q1[0], T.q1[1]}, e2[3] = {T.q1[2], T.q1[3], T.e2z};
            const double pv = a[0] * v0[0] + a[1] * v0[1] + a[2] * v0[2];
            pmin = std::min(pmin, pv);
            pmax = std::max(pmax, pv);
            const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
            const double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
            const double l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
            const double s = (l1 > 0 && l2 > 0) ? std::sqrt(cx * cx + cy * cy + cz * cz) / (l1 * l2) : 0.0;
            smin = std::min(smin, s);
        }
        Plane& P = pl[(size_t)c];
        P.pmin = std::nextafter((float)pmin, -FLT_MAX);
        P.pmax = std::nextafter((float)pmax, FLT_MAX);
        P.k1 = smin > 0 ? (float)(c1 * eps / smin) * 1.01f : FLT_MAX;
        P.k2 = smin > 0 ? (float)(c2 * eps / smin) * 1.01f : FLT_MAX;
        P.g = (float)std::sqrt(std::max(0.0, 2.0 - 2.0 * (double)q.ca)) * 1.001f + 1e-6f;
    }
    std::printf("entries %d chunks %d\n", n, nc);
    for (int family = 0; family < 2; ++family)
        for (int with_prior = 0; with_prior < 2; ++with_prior) {
            std::mt19937 rng(5 + family * 2 + with_prior);
            std::uniform_real_distribution<float> U(0, 1);
            std::normal_distribution<float> N(0, 1);
            const int R = 2000;
            Stats st[6];  // built, ideal, near-to-far; each without / with the plane rule
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
                auto open_chunk = [&](int c, float bound, bool plane) {
                    if (!box_rule(ch[(size_t)c], o, d, inv, on, bound)) return false;
                    return !(plane && plane_rule(ch[(size_t)c], pl[(size_t)c], o, d, bound));
                };
                auto test_chunk = [&](int c, float& bt, Stats& s) {
                    const int first = ch[(size_t)c].info & 0xffffff, cnt = ch[(size_t)c].info >> 24;
                    for (int j = 0; j < cnt; ++j) {
                        float tt;
                        s.tests++;
                        if (tri_hit(tris[(size_t)lidx[(size_t)(first + j)]], o, d, tt) && tt < bt) bt = tt;
                    }
                };
                auto verdict = [&](float bt, Stats& s) {
                    const float got = std::fmin(prior, bt);
                    if (!(got == answer || (std::isinf(got) && std::isinf(answer)))) s.bad++;
                };
                for (int plane = 0; plane < 2; ++plane) {
                    {  // built: chunk_leaf's schedule
                        Stats& s = st[0 + 3 * plane];
                        float bt = INFINITY, bound = prior;
                        std::vector<int> gathered;
                        for (int cb = root; cb < end; cb += 64) {
                            std::vector<int> opened;
                            for (int c = cb; c < std::min(end, cb + 64); ++c)
                                if (open_chunk(c, bound, plane)) { s.open++; opened.push_back(c); }
                            if (gathered.size() + opened.size() > 64) {
                                for (int c : gathered) test_chunk(c, bt, s);
                                gathered.clear();
                                bound = std::fmin(prior, bt);
                            }
                            gathered.insert(gathered.end(), opened.begin(), opened.end());
                        }
                        for (int c : gathered) test_chunk(c, bt, s);
                        verdict(bt, s);
                    }
                    {  // ideal: the final answer as the bound from the start
                        Stats& s = st[1 + 3 * plane];
                        float bt = INFINITY;
                        for (int c = root; c < end; ++c)
                            if (open_chunk(c, answer, plane)) { s.open++; test_chunk(c, bt, s); }
                        verdict(bt, s);
                    }
                    {  // near-to-far by the plain box's entry t, the bound after every chunk
                        Stats& s = st[2 + 3 * plane];
                        std::vector<std::pair<float, int>> key;
                        for (int c = root; c < end; ++c) {
                            const LNode& q = ch[(size_t)c];
                            float tn = -3e38f, tf = 3e38f;
                            for (int a = 0; a < 3; ++a) {
                                const float t1 = (q.lo[a] - o[a]) * inv[a], t2 = (q.hi[a] - o[a]) * inv[a];
                                tn = std::fmax(tn, std::fmin(t1, t2));
                                tf = std::fmin(tf, std::fmax(t1, t2));
                            }
                            key.push_back({(tf < tn || tf < 0) ? INFINITY : std::fmax(tn, 0.0f), c});
                        }
                        std::stable_sort(key.begin(), key.end(), [](auto& x, auto& y) { return x.first < y.first; });
                        float bt = INFINITY;
                        for (auto& kc : key)
                            if (open_chunk(kc.second, std::fmin(prior, bt), plane)) { s.open++; test_chunk(kc.second, bt, s); }
                        verdict(bt, s);
                    }
                }
            }
            const char* fam = family == 0 ? "near" : "aimed";
            const char* nm[3] = {"built", "ideal", "near-to-far"};
            for (int i = 0; i < 3; ++i)
                std::printf("%-6s rays, %-5s prior: %-11s open %7.1f -> %7.1f with the plane rule, tests %7.1f -> %7.1f, mismatches %.0f / %.0f\n",
                            fam, with_prior ? "with" : "no", nm[i], st[i].open / rays, st[i + 3].open / rays,
                            st[i].tests / rays, st[i + 3].tests / rays, st[i].bad, st[i + 3].bad);
        }
    return 0;
}
