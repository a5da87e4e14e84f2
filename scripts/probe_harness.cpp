// scripts/probe_harness.cpp — host check of pt_leafbvh.cpp probe_pre_leaves (test infrastructure:
// tests/test_preprobe.py builds and runs it; no GPU).  A hand-made tree: the root's left child is an
// inner node whose left child is a big leaf A (200 small triangles at z = -5); the root's right
// child is a leaf B holding a wall of two triangles.  A camera at the origin looks down -z.
//   wall at z = -2 (covering the view): every camera ray passes A's box filter (root-left box, then
//     the inner node's left box), but the wall is hit first and the inner node's box, entered at
//     t ~ 4, is pruned (the reference's exit-distance rule): A is never visited;
//   wall at z = +10 (behind the camera): every ray that passes A's filter visits A.
// Prints "pass visit" for A in each case.
// Build: hipcc -x hip --offload-arch=gfx950 -O2 -std=c++17 -I brown-cs2240-path-tracer_amd/csrc
//        scripts/probe_harness.cpp brown-cs2240-path-tracer_amd/csrc/pt_leafbvh.cpp
#include <hip/hip_runtime.h>  // pt_layout.h's vector types

#include <algorithm>
#include <cstdio>
#include <vector>

#include "pt_leafbvh.h"

using namespace pt;

static void grow(float lo[3], float hi[3], const float p[3]) {
    for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], p[a]);
        hi[a] = std::max(hi[a], p[a]);
    }
}

static void run(float wall_z) {
    std::vector<Tri> tris;
    float alo[3] = {1e30f, 1e30f, 1e30f}, ahi[3] = {-1e30f, -1e30f, -1e30f};
    for (int i = 0; i < 10; ++i)  // leaf A: 10 x 10 cells, two triangles each
        for (int j = 0; j < 10; ++j)
            for (int h = 0; h < 2; ++h) {
                const float x = -2.0f + 0.4f * (float)i, y = -2.0f + 0.4f * (float)j;
                const float v0[3] = {x, y, -5.0f - 0.05f * (float)h};
                const float e1[3] = {0.4f, 0.0f, 0.0f}, e2[3] = {0.0f, 0.4f, 0.0f};
                Tri t{};
                tri_set(t, v0, e1, e2);
                tris.push_back(t);
                const float p1[3] = {v0[0] + e1[0], v0[1], v0[2]}, p2[3] = {v0[0], v0[1] + e2[1], v0[2]};
                grow(alo, ahi, v0);
                grow(alo, ahi, p1);
                grow(alo, ahi, p2);
            }
    const int32_t nA = (int32_t)tris.size();
    float blo[3] = {1e30f, 1e30f, 1e30f}, bhi[3] = {-1e30f, -1e30f, -1e30f};
    for (int h = 0; h < 2; ++h) {  // leaf B: the wall, a 6 x 6 square at z = wall_z
        const float v0[3] = {h ? 3.0f : -3.0f, h ? 3.0f : -3.0f, wall_z};
        const float e1[3] = {h ? -6.0f : 6.0f, 0.0f, 0.0f}, e2[3] = {0.0f, h ? -6.0f : 6.0f, 0.0f};
        Tri t{};
        tri_set(t, v0, e1, e2);
        tris.push_back(t);
        const float p1[3] = {v0[0] + e1[0], v0[1], v0[2]}, p2[3] = {v0[0], v0[1] + e2[1], v0[2]};
        grow(blo, bhi, v0);
        grow(blo, bhi, p1);
        grow(blo, bhi, p2);
    }
    for (int a = 0; a < 3; ++a) {  // boxes with some thickness
        alo[a] -= 0.01f; ahi[a] += 0.01f;
        blo[a] -= 0.01f; bhi[a] += 0.01f;
    }
    std::vector<Node> nodes(2);
    Node& root = nodes[0];
    Node& inner = nodes[1];
    for (int a = 0; a < 3; ++a) {
        root.lmin[a] = alo[a]; root.lmax[a] = ahi[a];  // left: the inner node (A's box)
        root.rmin[a] = blo[a]; root.rmax[a] = bhi[a];  // right: leaf B
        inner.lmin[a] = alo[a]; inner.lmax[a] = ahi[a];  // left: leaf A
        inner.rmin[a] = 1e6f; inner.rmax[a] = 1e6f + 1.0f;  // right: an empty leaf far away
    }
    root.lref = 1; root.lcnt = -1;
    root.rref = nA; root.rcnt = 2;
    inner.lref = 0; inner.lcnt = nA;
    inner.rref = 0; inner.rcnt = 0;
    std::vector<PreLeaf> pre(1);
    pre[0].rec0 = 0;
    pre[0].n = nA;
    pre[0].npath = 2;
    pre[0].path[0] = 0 << 1 | 0;  // the root's left child
    pre[0].path[1] = 1 << 1 | 0;  // the inner node's left child
    std::vector<Light> lights(1);
    const float lp[3][3] = {{-0.5f, 3.0f, -0.5f}, {0.5f, 3.0f, -0.5f}, {0.0f, 3.0f, 0.5f}};
    for (int a = 0; a < 3; ++a) {
        lights[0].p0[a] = lp[0][a];
        lights[0].p1[a] = lp[1][a];
        lights[0].p2[a] = lp[2][a];
    }
    ProbeCamera cam{};
    for (int c = 0; c < 16; ++c) cam.M[c] = (c % 5 == 0) ? 1.0f : 0.0f;  // identity, column-major
    cam.focal = 1.0f;
    cam.half_h = 1.0f;
    cam.half_w = 1.0f;
    std::vector<std::array<uint32_t, 2>> out;
    probe_pre_leaves(nodes, tris, lights, pre, cam, 32, 1ull << 24, out);
    std::printf("%u %u\n", out[0][0], out[0][1]);
}

int main() {
    run(-2.0f);
    run(10.0f);
    return 0;
}
