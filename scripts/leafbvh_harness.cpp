// scripts/leafbvh_harness.cpp — host-side cost model of the leaf chunks.
// Builds csrc/pt_leafbvh.cpp's chunks over one leaf's records (a file of 48-byte Tri records, e.g.
// the boat's 7327-entry leaf) and replays pt_device.h chunk_skip in float for 2000 random rays
// (origins within 5 units of a random point of an entry, uniform directions): chunks open per ray,
// entries tested, the wave-steps of chunk_leaf (checks: chunks / 64; tests: open chunks / 8) against
// the cooperative turn's entries / 64, why chunks stay open, and the chunk-cone histogram.  Each
// ray's outcome is compared with the sequential loop over all entries (mismatches must be 0).
// Also: the cone-open chunks re-checked with their entries' own normals (the leaf pass's second
// check), and a per-ray walk of the whole build tree.  (Groups of 4 / 8 / 16 consecutive chunks
// checked first were measured here too and removed: 46 / 59 / 67 % of them open per ray, so a
// two-level walk saves only ~29 % of the checks.)
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off
//        -I brown-cs2240-path-tracer_amd/csrc scripts/leafbvh_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
// Run:   ./a.out leaf_records.bin [entries per chunk [merge neighbours up to]]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
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

// pt_device.h chunk_skip; why: 0 skipped, 1 open (cone), 2 open (box)
static int chunk_skip(const LNode& q, const float o[3], const float d[3], const float inv[3], float on, float bound) {
    const float cb = std::fabs(d[0] * q.ax + d[1] * q.ay + d[2] * q.az);
    const float sb = std::sqrt(std::fmax(0.f, 1 - cb * cb));
    const float cf = cb * q.ca - sb * q.sa - 1e-5f;
    if (!(cf > 1e-4f)) return 1;
    const float dl = (q.A + q.B * on) / cf + 1e-5f * on + q.C;
    if (!(dl < 1e30f)) return 1;
    float tn = -3e38f, tf = 3e38f;
    for (int a = 0; a < 3; ++a) {
        const float t1 = (q.lo[a] - dl - o[a]) * inv[a], t2 = (q.hi[a] + dl - o[a]) * inv[a];
        tn = std::fmax(tn, std::fmin(t1, t2));
        tf = std::fmin(tf, std::fmax(t1, t2));
    }
    return ((tf < tn) || (tf < 0) || (tn > bound)) ? 0 : 2;
}

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
    const int lmax = argc > 2 ? std::atoi(argv[2]) : kChunkMax, mmax = argc > 3 ? std::atoi(argv[3]) : 0;
    build_leaf_bvh(tris.data(), 0, n, ch, lidx, root, end, nullptr, lmax, mmax);
    const int nc = end - root;
    std::printf("entries %d chunks %d\n", n, nc);
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(0, 1);
    std::normal_distribution<float> N(0, 1);
    const int R = 2000;
    double open = 0, tests = 0, cone = 0, box = 0, bad = 0;
    for (int r = 0; r < R; ++r) {
        const int k = (int)(rng() % (unsigned)n);
        float bu = U(rng), bv = U(rng);
        if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
        const Tri& T = tris[(size_t)k];
        const float P[3] = {T.q0[0] + bu * T.q0[3] + bv * T.q1[2], T.q0[1] + bu * T.q1[0] + bv * T.q1[3],
                            T.q0[2] + bu * T.q1[1] + bv * T.e2z};
        const float o[3] = {P[0] + 10 * U(rng) - 5, P[1] + 10 * U(rng) - 5, P[2] + 10 * U(rng) - 5};
        float d[3] = {N(rng), N(rng), N(rng)};
        const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (int a = 0; a < 3; ++a) d[a] /= l;
        const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
        const float on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
        float lt = INFINITY;
        for (int j = 0; j < n; ++j) {
            float tt;
            if (tri_hit(tris[(size_t)j], o, d, tt) && tt < lt) lt = tt;
        }
        float bt = INFINITY;
        for (int c = root; c < end; ++c) {  // bound = none, as for a camera ray (checks before tests)
            const int why = chunk_skip(ch[(size_t)c], o, d, inv, on, INFINITY);
            if (!why) continue;
            open++;
            (why == 1 ? cone : box)++;
            const int first = ch[(size_t)c].info & 0xffffff, cnt = ch[(size_t)c].info >> 24;
            for (int j = 0; j < cnt; ++j) {
                float tt;
                tests++;
                if (tri_hit(tris[(size_t)lidx[(size_t)(first + j)]], o, d, tt) && tt < bt) bt = tt;
            }
        }
        if (!(bt == lt || (std::isinf(bt) && std::isinf(lt)))) bad++;
    }
    std::printf("per ray: %.1f open chunks (cone %.1f, box %.1f), %.1f entries tested, mismatches %.0f\n", open / R,
                cone / R, box / R, tests / R, bad);
    std::printf("chunk_leaf wave-steps ~%.0f (checks %d + tests %.1f); cooperative turn %d\n",
                (nc + 63) / 64 + open / R / 8, (nc + 63) / 64, open / R / 8, (n + 63) / 64);
    // a walk of the whole build tree per ray (DFS order, skip links): nodes checked per ray, and the
    // most any ray of a group of 64 checks (a wave walking its 64 rays in lockstep runs that long)
    {
        std::vector<LNode> tch, tree;
        std::vector<int32_t> tl;
        int32_t r0 = 0, r1 = 0;
        build_leaf_bvh(tris.data(), 0, n, tch, tl, r0, r1, &tree);
        std::mt19937 rng2(7);
        double vis = 0, vmax = 0, opened = 0;
        for (int g = 0; g < R / 64; ++g) {
            double gm = 0;
            for (int r = 0; r < 64; ++r) {
                const int k = (int)(rng2() % (unsigned)n);
                float bu = U(rng2), bv = U(rng2);
                if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
                const Tri& T = tris[(size_t)k];
                const float P[3] = {T.q0[0] + bu * T.q0[3] + bv * T.q1[2], T.q0[1] + bu * T.q1[0] + bv * T.q1[3],
                                    T.q0[2] + bu * T.q1[1] + bv * T.e2z};
                const float o[3] = {P[0] + 10 * U(rng2) - 5, P[1] + 10 * U(rng2) - 5, P[2] + 10 * U(rng2) - 5};
                float d[3] = {N(rng2), N(rng2), N(rng2)};
                const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                for (int a = 0; a < 3; ++a) d[a] /= l;
                const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
                const float on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
                int v = 0;
                for (size_t i = 0; i < tree.size();) {
                    const LNode& q = tree[i];
                    ++v;
                    if (!chunk_skip(q, o, d, inv, on, INFINITY)) { i = (size_t)q.skip; continue; }
                    if (q.info >= 0) ++opened;
                    ++i;
                }
                vis += v;
                gm = std::max(gm, (double)v);
            }
            vmax += gm;
        }
        const int G = R / 64;
        std::printf("tree walk: %zu nodes; per ray %.1f checked (%.1f leaves open), max of 64 rays %.1f (flat: %d)\n",
                    tree.size(), vis / (G * 64), opened / (G * 64), vmax / G, nc);
    }
    // the cone-open chunks again with the entries' own normals: cf = min |d . n_i| over the chunk
    // (the bound the cone only approximates), then the same expanded-box test
    {
        std::mt19937 rng3(5);
        double open2 = 0, tests2 = 0, bad2 = 0;
        for (int r = 0; r < R; ++r) {
            const int k = (int)(rng3() % (unsigned)n);
            float bu = U(rng3), bv = U(rng3);
            if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
            const Tri& T = tris[(size_t)k];
            const float P[3] = {T.q0[0] + bu * T.q0[3] + bv * T.q1[2], T.q0[1] + bu * T.q1[0] + bv * T.q1[3],
                                T.q0[2] + bu * T.q1[1] + bv * T.e2z};
            const float o[3] = {P[0] + 10 * U(rng3) - 5, P[1] + 10 * U(rng3) - 5, P[2] + 10 * U(rng3) - 5};
            float d[3] = {N(rng3), N(rng3), N(rng3)};
            const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            for (int a = 0; a < 3; ++a) d[a] /= l;
            const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
            const float on = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
            float lt = INFINITY;
            for (int j = 0; j < n; ++j) {
                float tt;
                if (tri_hit(tris[(size_t)j], o, d, tt) && tt < lt) lt = tt;
            }
            float bt = INFINITY;
            for (int c = root; c < end; ++c) {
                const LNode& q = ch[(size_t)c];
                int why = chunk_skip(q, o, d, inv, on, INFINITY);
                const int first = q.info & 0xffffff, cnt = q.info >> 24;
                if (why == 1) {  // refine: the entries' own normals
                    float cmin = 1.0f;
                    for (int j = 0; j < cnt; ++j) {
                        const Tri& E = tris[(size_t)lidx[(size_t)(first + j)]];
                        const double e1[3] = {E.q0[3], E.q1[0], E.q1[1]}, e2[3] = {E.q1[2], E.q1[3], E.e2z};
                        double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
                        const double ln = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
                        float nf[3] = {0, 0, 0};
                        if (ln > 0) for (int a = 0; a < 3; ++a) nf[a] = (float)(nv[a] / ln);
                        cmin = std::fmin(cmin, std::fabs(d[0] * nf[0] + d[1] * nf[1] + d[2] * nf[2]));
                    }
                    const float cf = cmin - 1e-5f;
                    why = 1;
                    if (cf > 1e-4f) {
                        const float dl = (q.A + q.B * on) / cf + 1e-5f * on + q.C;
                        if (dl < 1e30f) {
                            float tn = -3e38f, tf = 3e38f;
                            for (int a = 0; a < 3; ++a) {
                                const float t1 = (q.lo[a] - dl - o[a]) * inv[a], t2 = (q.hi[a] + dl - o[a]) * inv[a];
                                tn = std::fmax(tn, std::fmin(t1, t2));
                                tf = std::fmin(tf, std::fmax(t1, t2));
                            }
                            why = ((tf < tn) || (tf < 0)) ? 0 : 2;
                        }
                    }
                }
                if (!why) continue;
                open2++;
                for (int j = 0; j < cnt; ++j) {
                    float tt;
                    tests2++;
                    if (tri_hit(tris[(size_t)lidx[(size_t)(first + j)]], o, d, tt) && tt < bt) bt = tt;
                }
            }
            if (!(bt == lt || (std::isinf(bt) && std::isinf(lt)))) bad2++;
        }
        std::printf("entries' own normals for cone-open chunks: per ray %.1f open chunks, %.1f entries tested, mismatches %.0f\n",
                    open2 / R, tests2 / R, bad2);
    }
    int hist[10] = {0};
    for (int c = root; c < end; ++c) hist[std::min(9, (int)(ch[(size_t)c].sa * 10.0f))]++;
    for (int b = 0; b < 10; ++b) std::printf("chunks with cone sine in [%.1f, %.1f): %d\n", b / 10.0, (b + 1) / 10.0, hist[b]);
    return bad == 0 ? 0 : 2;
}
