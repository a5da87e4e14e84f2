// pt_capi.hip — C ABI (include/pt_hip.h): scene upload/re-encoding, render entry points.
// Host code only; kernels live in pt_kernels.hip.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <array>
#include <cfloat>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: librccl is opened on first multi-device use (pt_render_multi)

#include "../../include/pt_hip.h"
#include "pt_kernels.h"
#include "pt_leafbvh.h"

using namespace pt;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return fail(PT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// WGSL i32(f32): truncate toward zero, saturating.
int32_t wgsl_i32(float f) {
    if (std::isnan(f)) return 0;
    if (f >= 2147483647.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}

// Reads of the packed triangle buffer with Dawn/Tint robustness (index clamped to len-1),
// as the WGSL reads primitive_0 in sample_area_lights (intersection-logic.wgsl:260-279).
struct Packed {
    const float* p;
    size_t n;
    float at(int32_t i) const {
        uint32_t u = (uint32_t)i;
        if (u >= n) u = (uint32_t)(n - 1);
        return p[u];
    }
};

// ---------------------------------------------------------------------------------------------
// Options (pt_set_option): the process-wide table of kernel-selection switches.  Nothing is read
// from the environment; tests and A/B scripts set these explicitly.
// ---------------------------------------------------------------------------------------------
enum OptKind { OPT_BOOL, OPT_INT, OPT_ENUM };
struct OptSpec {
    const char* name;
    OptKind kind;
    const char* choices;  // OPT_ENUM: '|'-separated values
};
constexpr OptSpec kOptSpecs[] = {
    {"kernel", OPT_ENUM, "auto|mega|wavefront|literal"},
    {"trav", OPT_ENUM, "nested|flat1|pred|lean|lean2|lean4|lean8|lean16|lean32"},
    {"lds", OPT_BOOL, nullptr},          {"fastrcp", OPT_BOOL, nullptr},     {"dual", OPT_BOOL, nullptr},
    {"fuse", OPT_BOOL, nullptr},         {"fuse_gen", OPT_BOOL, nullptr},    {"bf", OPT_BOOL, nullptr},
    {"mailbox", OPT_BOOL, nullptr},      {"bf_stackless", OPT_BOOL, nullptr}, {"trace_sparse", OPT_INT, nullptr},
    {"region_perm", OPT_BOOL, nullptr},  {"regen", OPT_INT, nullptr},  {"trace_ring", OPT_INT, nullptr},
    {"parts", OPT_INT, nullptr},         {"sort", OPT_INT, nullptr},
    {"node_bias", OPT_INT, nullptr},     {"node_steps", OPT_INT, nullptr},     {"big_leaf", OPT_INT, nullptr},     {"bf_slots", OPT_INT, nullptr},
    {"leaf_pre", OPT_INT, nullptr},      {"leaf_blocks", OPT_INT, nullptr},  {"leaf_pairs", OPT_INT, nullptr},
    {"pre_ratio", OPT_INT, nullptr},     {"leaf_refine", OPT_BOOL, nullptr},
    {"wf_paths", OPT_INT, nullptr},      {"wf_trace_blocks", OPT_INT, nullptr}, {"trace_watchdog", OPT_INT, nullptr},
    {"leaf_bvh", OPT_INT, nullptr},      {"leaf_walk", OPT_BOOL, nullptr},   {"leaf_pool", OPT_BOOL, nullptr},   {"pool_run", OPT_ENUM, "2|4"},
    {"leaf_skip", OPT_BOOL, nullptr},
    {"mb_uid_order", OPT_ENUM, "forward|reverse"},
    {"reduce", OPT_ENUM, "rccl|ordered"},
};
constexpr int kNumOpts = (int)(sizeof(kOptSpecs) / sizeof(kOptSpecs[0]));

std::mutex g_opt_mu;
std::string g_opt_val[kNumOpts];  // "" = default

int opt_index(const char* name) {
    for (int i = 0; i < kNumOpts; ++i)
        if (!std::strcmp(name, kOptSpecs[i].name)) return i;
    return -1;
}

bool opt_valid(const OptSpec& s, const char* v) {
    if (!*v) return false;
    if (s.kind == OPT_BOOL) return !std::strcmp(v, "0") || !std::strcmp(v, "1");
    if (s.kind == OPT_INT) {
        char* end = nullptr;
        const long long x = std::strtoll(v, &end, 10);
        return *end == 0 && x >= 0 && x <= 0x7fffffffLL;
    }
    const size_t n = std::strlen(v);
    for (const char* c = s.choices; *c;) {
        const char* bar = std::strchr(c, '|');
        const size_t len = bar ? (size_t)(bar - c) : std::strlen(c);
        if (len == n && !std::strncmp(c, v, n)) return true;
        c += len + (bar ? 1 : 0);
    }
    return false;
}

// Snapshot of the table, taken once per call (a concurrent pt_set_option affects later calls only).
struct Opts {
    std::string v[kNumOpts];
    const std::string& get(const char* name) const {
        static const std::string empty;
        const int i = opt_index(name);
        return i >= 0 ? v[i] : empty;
    }
    bool has(const char* name) const { return !get(name).empty(); }
    long num(const char* name, long def) const { return has(name) ? std::atol(get(name).c_str()) : def; }
    int flag(const char* name, int def) const { return has(name) ? (get(name) == "1" ? 1 : 0) : def; }
    bool is(const char* name, const char* val) const { return get(name) == val; }
};
Opts opts_snapshot() {
    std::lock_guard<std::mutex> lk(g_opt_mu);
    Opts o;
    for (int i = 0; i < kNumOpts; ++i) o.v[i] = g_opt_val[i];
    return o;
}

// leaves of at least this many entries get leaf chunks (option leaf_bvh, read by pt_scene_create;
// the big-leaf threshold): exact (tests/test_gpu_leafbvh.py), MedievalBoat +10 % in process
// (DESIGN.md §5.3); 0 = none
constexpr long kLeafBvhDefault = 128;
// the probe of the pre-resolvable leaves (probe_pre_leaves): a 32 x 32 raster (<= 4 Ki queries), at
// most 2^23 triangle tests (MedievalBoat: ~4 k per query, ~30 ms)
constexpr int kPreProbeGrid = 32;
// the leaf pass's chunks: the builder's leaves of at most PT_PASS_LEAF entries, neighbours merged
// while they fit PT_PASS_MERGE (<= kPassChunkMax; 0: no merging)
#ifndef PT_PASS_LEAF
#define PT_PASS_LEAF kPassChunkMax
#endif
#ifndef PT_PASS_MERGE
#define PT_PASS_MERGE kPassChunkMax
#endif
static_assert(PT_PASS_LEAF <= kPassChunkMax && PT_PASS_MERGE <= kPassChunkMax, "pass chunks fit the pass's loops");
constexpr uint64_t kPreProbeTests = 1ull << 23;
// the leaf remainders' probe (build_leaf_skips): at most 2^24 triangle tests (Glossy ~1.7 M, ~20 ms)
constexpr uint64_t kLeafSkipProbeTests = 1ull << 24;

struct HostLayout {
    std::vector<Node> nodes;
    std::vector<Tri> tris;
    std::vector<Material> mats;
    std::vector<Light> lights;
    std::vector<uint64_t> lmask;  // mailbox scenes: uid set per leaf, indexed by first record
    std::vector<float4> tnorm;    // vertex-normal mode: 3 per record (SceneView::tnorm)
    std::vector<BfNode> bfnode;   // mailbox scenes with <= 64 internal nodes, <= 63 entries (SceneView::bfnode)
    std::vector<int32_t> bfmap;
    std::vector<LNode> lnodes;    // leaf BVHs (SceneView::lnodes), and per such leaf (first record, entries, nodes)
    std::vector<int32_t> lidx;
    std::vector<Tri> ltris;       // per chunk slot: its entry's record, lbvh = the entry's position in its leaf
    std::vector<LNode> pnodes;    // the leaf pass's chunks of the pre-resolvable leaves (SceneView::pnodes, PreLeaf c0 / c1)
    std::vector<Tri> ptris;       // per pass chunk slot: its entry's record, lbvh = the entry's position in its leaf
    std::vector<float4> pnorm;    // per pass chunk slot: its entry's unit normal
    std::vector<std::array<int32_t, 3>> lleaves;
    int32_t leaf_min = 0;         // leaves of at least this many entries have one (option leaf_bvh; 0: none)
    std::vector<PreLeaf> pre;     // the kMaxPre largest leaves with their paths (SceneView::pre), largest first
    std::vector<int32_t> leaf_sizes;  // every non-empty leaf's entries, largest first
    std::vector<int2> nalt;       // leaf remainders (SceneView::nalt; empty: none)
    LeafSkipStats skip{};
    int32_t mb_base = 0;          // record of uid 0 (mailbox scenes)
    bool mailbox = false;
    pt_scene_info info{};
    int32_t ntri = 0;
    bool fast_rcp = false;  // SceneView::fast_rcp
};

// Re-encode packer.ts layouts into pt_layout.h.
int build_layout(const float* tri, size_t tri_len, const float* bvh, size_t bvh_len, HostLayout& L) {
    if (tri_len < 16 || tri_len > (size_t)INT32_MAX) return fail(PT_ERR_SCENE, "triangle_data shorter than its 16-float header");
    if (bvh_len < 6 + 17 || bvh_len > (size_t)INT32_MAX) return fail(PT_ERR_SCENE, "bvh_data shorter than bounds + one node");
    Packed P{tri, tri_len};
    const float nverts_f = tri[0], nobj_f = tri[1];
    if (!(nverts_f >= 0 && nverts_f == std::floor(nverts_f)) || !(nobj_f >= 1 && nobj_f == std::floor(nobj_f)))
        return fail(PT_ERR_SCENE, "bad vertex/object counts in triangle_data header");
    const int64_t nverts = (int64_t)nverts_f, nobj = (int64_t)nobj_f;
    const int64_t v_start = wgsl_i32(tri[2]), m_start = wgsl_i32(tri[4]);
    if (v_start < 0 || v_start + 3 * nverts > (int64_t)tri_len) return fail(PT_ERR_SCENE, "vertex section out of range");
    if (m_start < 0 || m_start + 15 * nobj > (int64_t)tri_len) return fail(PT_ERR_SCENE, "material section out of range");
    L.info.vertices = (uint32_t)nverts;

    // materials (program-raymarch.wgsl:87-102): Ns Ni illum Ka Kd Ks Ke
    L.mats.resize((size_t)nobj);
    for (int64_t id = 0; id < nobj; ++id) {
        const float* m = tri + m_start + 15 * id;
        Material& o = L.mats[(size_t)id];
        std::memset(&o, 0, sizeof o);
        o.Ns = m[0]; o.Ni = m[1]; o.illum = m[2];
        for (int c = 0; c < 3; ++c) { o.Kd[c] = m[6 + c]; o.Ks[c] = m[9 + c]; o.Ke[c] = m[12 + c]; }
        // the material's constant quotients, once per scene instead of per path and bounce: the
        // same correctly rounded f32 divisions the device would make (no contraction, no FTZ)
        o.kd_pi0 = o.Kd[0] / kPI; o.kd_pi1 = o.Kd[1] / kPI; o.kd_pi2 = o.Kd[2] / kPI;
        o.phong = (o.Ns + 2.0f) / (2.0f * kPI);
    }
    L.info.materials = (uint32_t)nobj;

    auto vertex = [&](int64_t one_based, float out[3]) -> bool {
        if (one_based < 1 || one_based > nverts) return false;
        const float* v = tri + v_start + 3 * (one_based - 1);
        out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
        return true;
    };

    // BVH: pre-order tree from offset 6 (intersection-logic.wgsl:4-16).
    if (bvh[6] == 1.0f) return fail(PT_ERR_SCENE, "BVH root is a leaf (the reference never builds one)");
    struct Item { int32_t off; int32_t node; int32_t depth; };
    std::vector<Item> work;
    // mailbox bookkeeping: each record's leaf entry (i0, i1, i2, material) and the leaves
    std::vector<std::array<int32_t, 4>> entry;
    std::vector<std::pair<int32_t, int32_t>> leaf_ranges;  // (first record, count)
    L.nodes.push_back(Node{});
    work.push_back({6, 0, 0});
    const size_t node_cap = bvh_len / 17 + 1;
    uint32_t max_depth = 0;
    while (!work.empty()) {
        Item it = work.back();
        work.pop_back();
        const int32_t o = it.off;
        if (o < 0 || (size_t)o + 17 > bvh_len) return fail(PT_ERR_SCENE, "BVH node offset out of range");
        max_depth = std::max<uint32_t>(max_depth, (uint32_t)it.depth);
        Node nd{};
        for (int c = 0; c < 3; ++c) {
            nd.lmin[c] = bvh[o + 5 + c]; nd.lmax[c] = bvh[o + 8 + c];
            nd.rmin[c] = bvh[o + 11 + c]; nd.rmax[c] = bvh[o + 14 + c];
        }
        int32_t child_off[2] = {wgsl_i32(bvh[o + 2]), wgsl_i32(bvh[o + 3])};
        int32_t refs[2], cnts[2];
        for (int side = 0; side < 2; ++side) {
            const int32_t c = child_off[side];
            if (c < 0 || (size_t)c + 17 > bvh_len) return fail(PT_ERR_SCENE, "BVH child pointer out of range");
            if (bvh[c] == 1.0f) {  // leaf: (i0,i1,i2,mat) 1-based entries after the 17-float header
                const float nf = bvh[c + 4];
                if (!(nf >= 0) || std::fmod(nf, 4.0f) != 0.0f || (size_t)c + 17 + (size_t)nf > bvh_len)
                    return fail(PT_ERR_SCENE, "BVH leaf payload malformed");
                const int32_t n = (int32_t)(nf / 4.0f);
                refs[side] = (int32_t)L.tris.size();
                cnts[side] = n;
                for (int32_t k = 0; k < n; ++k) {
                    const float* e = bvh + c + 17 + 4 * k;
                    float v0[3], v1[3], v2[3];
                    if (!vertex(wgsl_i32(e[0]), v0) || !vertex(wgsl_i32(e[1]), v1) || !vertex(wgsl_i32(e[2]), v2))
                        return fail(PT_ERR_SCENE, "BVH leaf references a vertex out of range");
                    const int32_t mat = wgsl_i32(e[3]);
                    if (mat < 0 || mat >= nobj) return fail(PT_ERR_SCENE, "BVH leaf references a material out of range");
                    Tri t{};
                    float e1[3], e2[3];
                    for (int q = 0; q < 3; ++q) {
                        e1[q] = v1[q] - v0[q];  // ray-triangle-intersection.wgsl:6
                        e2[q] = v2[q] - v0[q];  // :7
                    }
                    tri_set(t, v0, e1, e2);
                    t.mat = mat;
                    t.uid = -1;
                    L.tris.push_back(t);
                    {   // vertex normals at vn_start + i (i = (index - 1) * 3, the vertex offsets;
                        // intersection-logic.wgsl:81-97), reads clamped as Tint's
                        const int32_t vi[3] = {(wgsl_i32(e[0]) - 1) * 3, (wgsl_i32(e[1]) - 1) * 3, (wgsl_i32(e[2]) - 1) * 3};
                        const int32_t vn_start = wgsl_i32(tri[5]), vn_range = wgsl_i32(tri[6]);
                        for (int q = 0; q < 3; ++q)
                            L.tnorm.push_back(make_float4(P.at(vn_start + vi[q]), P.at(vn_start + vi[q] + 1),
                                                          P.at(vn_start + vi[q] + 2),
                                                          (q == 0 && vi[2] < vn_range) ? 1.0f : 0.0f));
                    }
                    entry.push_back({wgsl_i32(e[0]), wgsl_i32(e[1]), wgsl_i32(e[2]), mat});
                }
                leaf_ranges.emplace_back(refs[side], n);
                L.info.leaves++;
                L.info.leaf_refs += (uint32_t)n;
                L.info.max_leaf = std::max<uint32_t>(L.info.max_leaf, (uint32_t)n);
            } else {
                if (L.nodes.size() >= node_cap) return fail(PT_ERR_SCENE, "BVH is not a tree (node count exceeds buffer)");
                refs[side] = (int32_t)L.nodes.size();
                cnts[side] = -1;
                L.nodes.push_back(Node{});
                work.push_back({c, refs[side], it.depth + 1});
            }
        }
        nd.lref = refs[0]; nd.rref = refs[1]; nd.lcnt = cnts[0]; nd.rcnt = cnts[1];
        L.nodes[(size_t)it.node] = nd;
    }
    L.info.nodes = (uint32_t)L.nodes.size();
    // Mailboxing: a leaf entry tested twice by one query gives the same t both
    // times and the closest-hit update is strict-<, so repeats never change the result.  With
    // at most 64 distinct entries a query keeps the set it has tested in one 64-bit mask.
    // uids follow first appearance (option mb_uid_order=reverse numbers them backwards: tests
    // use it to exercise the tie-break of the uid-ordered leaf loop).
    {
        std::map<std::array<int32_t, 4>, int32_t> ids;
        std::vector<int32_t> uid(entry.size());
        std::vector<size_t> first;
        for (size_t r = 0; r < entry.size(); ++r) {
            auto it = ids.find(entry[r]);
            if (it == ids.end()) {
                it = ids.emplace(entry[r], (int32_t)first.size()).first;
                first.push_back(r);
            }
            uid[r] = it->second;
        }
        const int32_t U = (int32_t)first.size();
        L.mailbox = U >= 1 && U <= 64;
        // every record carries its entry's uid (the mailbox scenes renumber below)
        for (size_t r = 0; r < entry.size(); ++r) L.tris[r].uid = uid[r];
        if (L.mailbox) {
            const bool rev = opts_snapshot().is("mb_uid_order", "reverse");
            for (auto& u : uid) u = rev ? U - 1 - u : u;
            for (size_t r = 0; r < entry.size(); ++r) L.tris[r].uid = uid[r];
            L.mb_base = (int32_t)L.tris.size();
            std::vector<Tri> uniq((size_t)U);
            for (size_t k = 0; k < first.size(); ++k) uniq[(size_t)uid[first[k]]] = L.tris[first[k]];
            L.tris.insert(L.tris.end(), uniq.begin(), uniq.end());
            std::vector<float4> un(3 * (size_t)U);
            for (size_t k = 0; k < first.size(); ++k)
                for (int q = 0; q < 3; ++q) un[3 * (size_t)uid[first[k]] + q] = L.tnorm[3 * first[k] + q];
            L.tnorm.insert(L.tnorm.end(), un.begin(), un.end());
            L.lmask.assign(std::max<size_t>(1, entry.size()), 0);
            for (const auto& lr : leaf_ranges)
                for (int32_t k = 0; k < lr.second; ++k) L.lmask[(size_t)lr.first] |= 1ull << uid[(size_t)(lr.first + k)];
            // the stackless replay tree (BfNode): internal nodes in the reference's visiting
            // order — pre-order with the right subtree first — so the next node to visit is always
            // the smallest-numbered pending one
            if (U <= 63 && L.nodes.size() <= 64) {
                std::vector<int32_t> pre(L.nodes.size(), -1);
                std::vector<int32_t> st{0};
                int32_t next = 0;
                while (!st.empty()) {
                    const int32_t n = st.back();
                    st.pop_back();
                    pre[(size_t)n] = next++;
                    L.bfmap.push_back(n);
                    const Node& nd = L.nodes[(size_t)n];
                    if (nd.lcnt < 0) st.push_back(nd.lref);  // popped after the right subtree
                    if (nd.rcnt < 0) st.push_back(nd.rref);
                }
                L.bfnode.resize(L.nodes.size());
                for (size_t i = 0; i < L.bfmap.size(); ++i) {
                    const Node& nd = L.nodes[(size_t)L.bfmap[i]];
                    BfNode& b = L.bfnode[i];
                    for (int c = 0; c < 3; ++c) { b.lmin[c] = nd.lmin[c]; b.lmax[c] = nd.lmax[c]; b.rmin[c] = nd.rmin[c]; b.rmax[c] = nd.rmax[c]; }
                    b.lm = nd.lcnt < 0 ? (1ull << 63) | (uint64_t)pre[(size_t)nd.lref] : (nd.lcnt > 0 ? L.lmask[(size_t)nd.lref] : 0ull);
                    b.rm = nd.rcnt < 0 ? (1ull << 63) | (uint64_t)pre[(size_t)nd.rref] : (nd.rcnt > 0 ? L.lmask[(size_t)nd.rref] : 0ull);
                }
            }
        }
    }
    // Leaf BVHs (pt_leafbvh.cpp): every leaf of at least leaf_bvh entries (option, read here;
    // default kLeafBvhDefault, 0 = none).  The leaf's first record holds root + 1, its second the
    // end of its nodes (Tri::lbvh).  The lean traversal's big-leaf step walks them (mailbox scenes:
    // only with option mailbox=0, their default kernels test every entry once per ray anyway).
    {
        const long lmin = opts_snapshot().num("leaf_bvh", kLeafBvhDefault);
        if (lmin >= 2) {
            L.leaf_min = (int32_t)std::min<long>(lmin, INT32_MAX);
            std::sort(leaf_ranges.begin(), leaf_ranges.end());
            for (const auto& lr : leaf_ranges) {
                if (lr.second < L.leaf_min || L.lidx.size() + (size_t)lr.second >= (1u << 24)) continue;
                int32_t root = 0, end = 0;
                const size_t slot0 = L.lidx.size();
                build_leaf_bvh(L.tris.data(), lr.first, lr.second, L.lnodes, L.lidx, root, end);
                for (size_t j = slot0; j < L.lidx.size(); ++j) {
                    Tri t = L.tris[(size_t)(lr.first + L.lidx[j])];
                    t.lbvh = L.lidx[j];
                    L.ltris.push_back(t);
                }
                L.tris[(size_t)lr.first].lbvh = root + 1;
                L.tris[(size_t)lr.first + 1].lbvh = end;
                L.lleaves.push_back({lr.first, lr.second, end - root});
            }
            if (L.lleaves.empty()) L.leaf_min = 0;
        }
    }
    // Leaves that k_wf_leafpass can resolve before the traversal: the kMaxPre largest, each with its
    // path of child boxes from the root (node << 1 | side per step; PreLeaf)
    {
        std::vector<PreLeaf> all;
        // iterative pre-order walk keeping the path: (node, depth) frames, path[depth] = the step in
        std::vector<std::pair<int32_t, std::vector<int32_t>>> st;
        st.push_back({0, {}});
        bool deep = false;
        while (!st.empty()) {
            auto fr = std::move(st.back());
            st.pop_back();
            const Node& nd = L.nodes[(size_t)fr.first];
            for (int side = 1; side >= 0; --side) {
                const int32_t cnt = side ? nd.rcnt : nd.lcnt, ref = side ? nd.rref : nd.lref;
                std::vector<int32_t> p2 = fr.second;
                p2.push_back(fr.first << 1 | side);
                if (cnt >= 0) {
                    if (cnt == 0) continue;
                    L.leaf_sizes.push_back(cnt);
                    if ((int)p2.size() > kMaxPrePath) { deep = true; continue; }
                    PreLeaf pl{};
                    pl.rec0 = ref;
                    pl.n = cnt;
                    pl.npath = (int32_t)p2.size();
                    for (size_t k = 0; k < p2.size(); ++k) pl.path[k] = p2[k];
                    all.push_back(pl);
                } else if (ref >= 0 && (size_t)ref < L.nodes.size()) {
                    st.push_back({ref, std::move(p2)});
                }
            }
        }
        std::sort(L.leaf_sizes.begin(), L.leaf_sizes.end(), std::greater<int32_t>());
        std::sort(all.begin(), all.end(), [](const PreLeaf& a, const PreLeaf& b) { return a.n > b.n || (a.n == b.n && a.rec0 < b.rec0); });
        if (!deep) {  // (a leaf below kMaxPrePath steps could be among the largest: no table then)
            for (size_t k = 0; k < all.size() && k < (size_t)kMaxPre; ++k) L.pre.push_back(all[k]);
        }
        // the leaf pass's own chunks (kPassChunkMax entries) of the leaves that have traversal chunks
        std::vector<int32_t> plidx;
        for (PreLeaf& pl : L.pre) {
            pl.c0 = pl.c1 = 0;
            if (L.leaf_min <= 0 || pl.n < L.leaf_min || L.ptris.size() + (size_t)pl.n >= (1u << 24)) continue;
            const size_t slot0 = plidx.size();
            int32_t root = 0, end = 0;
            build_leaf_bvh(L.tris.data(), pl.rec0, pl.n, L.pnodes, plidx, root, end, nullptr, PT_PASS_LEAF, PT_PASS_MERGE);
            for (size_t j = slot0; j < plidx.size(); ++j) {
                Tri t = L.tris[(size_t)(pl.rec0 + plidx[j])];
                t.lbvh = plidx[j];
                L.ptris.push_back(t);
                // the entry's normal in double, rounded (the pass's check allows 1e-5 for it)
                const double e1[3] = {t.q0[3], t.q1[0], t.q1[1]}, e2[3] = {t.q1[2], t.q1[3], t.e2z};
                const double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                                      e1[0] * e2[1] - e1[1] * e2[0]};
                const double ln = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
                const bool ok = ln > 0.0 && std::isfinite(ln);
                L.pnorm.push_back(make_float4(ok ? (float)(nv[0] / ln) : 0.0f, ok ? (float)(nv[1] / ln) : 0.0f,
                                              ok ? (float)(nv[2] / ln) : 0.0f, 0.0f));
            }
            pl.c0 = root;
            pl.c1 = end;
        }
        // the pass's check takes A and B times 1.00001 (pt_leafpass.hip pass_box_skip), rounded up;
        // a degenerate chunk's FLT_MAX stays (its delta is never bounded)
        for (LNode& nd : L.pnodes) {
            auto up5 = [](float v) {
                return v >= FLT_MAX ? v : std::nextafter((float)((double)v * 1.00001), FLT_MAX);
            };
            nd.A = up5(nd.A);
            nd.B = up5(nd.B);
        }
    }
    // Leaf remainders (pt_leafskip.cpp; option leaf_skip, read here and per render, default on):
    // scenes without mailbox (their kernels test every distinct entry once per ray anyway)
    if (!L.mailbox && opts_snapshot().flag("leaf_skip", 1) != 0)
        build_leaf_skips(L.nodes, L.tris, L.tnorm, L.lights, kLeafSkipMaxLeaf, kLeafAlt, kLeafSkipProbeTests, L.nalt,
                         &L.skip);
    // |det| = |e1 . (d x e2)| <= |e1| |e2| |d| with |d| = 1 (every ray direction is normalised or
    // a reflection/refraction of unit vectors; non-finite ones give no hit on either path)
    double emax = 0.0;
    bool finite = true;
    for (const Tri& t : L.tris) {
        const double e1[3] = {t.q0[3], t.q1[0], t.q1[1]}, e2[3] = {t.q1[2], t.q1[3], t.e2z};
        const double a = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
        const double b = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
        finite = finite && std::isfinite(a) && std::isfinite(b);
        emax = std::max(emax, a * b);
    }
    L.fast_rcp = finite && emax < std::ldexp(1.0, 124);
    // The device stack parks at most one left child per internal ancestor.
    L.info.max_stack = max_depth + 1;
    if (L.info.max_stack >= (uint32_t)kStackMax) return fail(PT_ERR_SCENE, "BVH deeper than the device traversal stack");

    // Light table (intersection-logic.wgsl:217-285): entry k for k in [0, Ntri].
    int32_t es[4], ee[4], n[4];
    int32_t ntri = 0;
    for (int s = 0; s < 4; ++s) {
        es[s] = wgsl_i32(tri[8 + 2 * s]);
        ee[s] = wgsl_i32(tri[9 + 2 * s]);
        n[s] = (es[s] != -1) ? (ee[s] - es[s]) / 4 : 0;
        ntri += n[s];
    }
    if (ntri <= 0) return fail(PT_ERR_SCENE, "scene has no emissive triangles (sample_area_lights needs one)");
    L.ntri = ntri;
    const int32_t vs = wgsl_i32(P.at(2));
    for (int32_t k = 0; k <= ntri; ++k) {
        int32_t idx;
        if (k < n[0]) idx = k * 4 + es[0];
        else if (k < n[0] + n[1]) idx = (k - n[0]) * 4 + es[1];
        else if (k < n[0] + n[1] + n[2]) idx = (k - n[0] - n[1]) * 4 + es[2];
        else idx = (k - n[0] - n[1] - n[2]) * 4 + es[3];
        Light lt{};
        float* dst[3] = {lt.p0, lt.p1, lt.p2};
        for (int j = 0; j < 3; ++j) {
            const int32_t i = (wgsl_i32(P.at(idx + j)) - 1) * 3;
            for (int c = 0; c < 3; ++c) dst[j][c] = P.at(vs + i + c);
        }
        L.lights.push_back(lt);
    }
    L.info.emissive_tris = (uint32_t)ntri;
    return PT_OK;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

extern "C" {

int pt_set_option(const char* name, const char* value) {
    if (!name) return fail(PT_ERR_INVALID, "option name is NULL");
    const int i = opt_index(name);
    if (i < 0) return fail(PT_ERR_INVALID, std::string("unknown option '") + name + "'");
    if (value && !opt_valid(kOptSpecs[i], value))
        return fail(PT_ERR_INVALID, std::string("bad value '") + value + "' for option '" + name + "'");
    std::lock_guard<std::mutex> lk(g_opt_mu);
    g_opt_val[i] = value ? value : "";
    return PT_OK;
}

int pt_get_option(const char* name, char* buf, size_t cap) {
    if (!name || !buf || cap == 0) return fail(PT_ERR_INVALID, "null argument");
    const int i = opt_index(name);
    if (i < 0) return fail(PT_ERR_INVALID, std::string("unknown option '") + name + "'");
    std::lock_guard<std::mutex> lk(g_opt_mu);
    if (g_opt_val[i].size() + 1 > cap) return fail(PT_ERR_INVALID, "buffer too small");
    std::memcpy(buf, g_opt_val[i].c_str(), g_opt_val[i].size() + 1);
    return PT_OK;
}

void pt_reset_options(void) {
    std::lock_guard<std::mutex> lk(g_opt_mu);
    for (auto& v : g_opt_val) v.clear();
}

#ifndef PT_SOURCE_HASH
#define PT_SOURCE_HASH "unknown"
#endif
const char* pt_build_id(void) { return PT_SOURCE_HASH; }

}  // extern "C"


struct pt_scene {
    int device = 0;
    void* d_mem = nullptr;
    SceneView view{};
    pt_scene_info info{};
    hipStream_t stream = nullptr;
    float* d_accum = nullptr;  // scratch for the blocking host-buffer calls
    size_t accum_cap = 0;
    Counters* d_counters = nullptr;
    void* d_wf = nullptr;  // wavefront path state, allocated on first use
    WfBuffers wf{};
    bool prof_on = false;  // pt_profile_enable
    KernelProfiler prof;
    uint8_t* d_rgba = nullptr;  // pt_render_image scratch
    size_t rgba_cap = 0;
    WfStreams ws;  // dual-stream wavefront: aux stream + fork/join events (created with d_wf)
    // pinned mirror of the wavefront control words, copied after every wavefront render on its
    // stream: a watchdog flag set by an asynchronous render surfaces once that copy has landed
    // (next call, pt_scene_check) without a synchronisation of its own
    uint32_t* h_ctl = nullptr;
    float* d_rad = nullptr;  // radiance of finished wavefront paths (ensure_rad)
    uint64_t rad_cap = 0;
    float* d_peer = nullptr;  // pt_render_multi (ordered reduction): another device's partial accumulator
    size_t peer_cap = 0;
    int32_t leaf_min = 0;  // leaf BVHs: leaves of at least this many entries have one (0: none)
    std::vector<std::array<int32_t, 3>> lleaves;  // (first record, entries, nodes) per leaf BVH
    // big leaves resolved before the traversal (k_wf_leafpass): the table (device copy in d_mem at
    // d_pre), every leaf's size (largest first), and the result keys (ensure_pres)
    std::vector<PreLeaf> pre;
    // render_impl's choice of the leaf pass: per leaf of pre, probe queries passing its box filter and
    // visiting it (probe_pre_leaves, once, with the camera of the scene's first render that could
    // use the pass), from host copies of the tree, records and lights kept for it
    std::vector<std::array<uint32_t, 2>> pre_probe;
    bool pre_probed = false;
    ProbeCamera pre_cam{};  // the camera pre_probe was taken with (a render with another probes again)
    std::mutex pre_mu;
    std::vector<Node> h_nodes;
    std::vector<Tri> h_tris;
    std::vector<Light> h_lights;
    std::vector<int32_t> leaf_sizes;
    const PreLeaf* d_pre = nullptr;
    uint64_t* d_pres = nullptr;
    size_t pres_cap = 0;  // keys
};

// Set once any call of this library has touched the HIP runtime (pt_set_hw_queues is then too late).
static bool g_hip_touched = false;

namespace pt {
thread_local KernelProfiler* t_prof = nullptr;

hipEvent_t KernelProfiler::take() {
    hipEvent_t e = nullptr;
    if (!pool.empty()) {
        e = pool.back();
        pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
    }
    return e;
}
void KernelProfiler::start(int kid, hipStream_t st) {
    Rec r{kid, take(), take()};
    if (r.a) hipEventRecord(r.a, st);
    recs.push_back(r);
}
void KernelProfiler::stop(hipStream_t st) {
    if (!recs.empty() && recs.back().b) hipEventRecord(recs.back().b, st);
}
void KernelProfiler::reset() {
    for (auto& r : recs) {
        if (r.a) pool.push_back(r.a);
        if (r.b) pool.push_back(r.b);
    }
    recs.clear();
}
void KernelProfiler::destroy() {
    reset();
    for (auto e : pool) hipEventDestroy(e);
    pool.clear();
}
}  // namespace pt

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_profile_enable(pt_scene* s, int enable) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    s->prof.reset();
    s->prof_on = enable != 0;
    return PT_OK;
}

int pt_profile_select(pt_scene* s, const char* kernel) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    if (!kernel) { s->prof.only = -1; return PT_OK; }
    for (int k = 0; k < KID_COUNT; ++k)
        if (!std::strcmp(kernel, kernel_name(k))) { s->prof.only = k; return PT_OK; }
    return fail(PT_ERR_INVALID, "unknown kernel name");
}

int pt_profile_read(pt_scene* s, pt_kernel_time* out, int max_entries, int* n_out) {
    if (!s || !n_out || (max_entries > 0 && !out)) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(s->device));
    pt_kernel_time acc[KID_COUNT] = {};
    // launch intervals relative to the first record's start event (events of one device compare
    // across streams): their union per kernel is its busy time
    std::vector<std::pair<double, double>> iv[KID_COUNT];
    for (const auto& r : s->prof.recs) {
        if (!r.a || !r.b) return fail(PT_ERR_HIP, "profiling event could not be created");
        HIP_TRY(hipEventSynchronize(r.b));
        float ms = 0.0f, t0 = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        HIP_TRY(hipEventElapsedTime(&t0, s->prof.recs.front().a, r.a));
        pt_kernel_time& k = acc[r.kid];
        k.min_ms = k.launches ? std::min(k.min_ms, (double)ms) : (double)ms;
        k.max_ms = k.launches ? std::max(k.max_ms, (double)ms) : (double)ms;
        k.total_ms += ms;
        k.launches++;
        iv[r.kid].emplace_back((double)t0, (double)t0 + (double)ms);
    }
    for (int k = 0; k < KID_COUNT; ++k) {
        std::sort(iv[k].begin(), iv[k].end());
        double busy = 0.0, lo = 0.0, hi = -1.0;
        for (const auto& x : iv[k]) {
            if (x.first > hi) {
                if (hi > lo) busy += hi - lo;
                lo = x.first;
                hi = x.second;
            } else {
                hi = std::max(hi, x.second);
            }
        }
        if (hi > lo) busy += hi - lo;
        acc[k].busy_ms = busy;
    }
    int n = 0;
    for (int k = 0; k < KID_COUNT; ++k) {
        if (!acc[k].launches) continue;
        if (n < max_entries) {
            out[n] = acc[k];
            std::snprintf(out[n].name, sizeof(out[n].name), "%s", kernel_name(k));
        }
        ++n;
    }
    *n_out = std::min(n, std::max(max_entries, 0));
    return PT_OK;
}

const char* pt_last_error(void) { return g_err.c_str(); }

int pt_set_hw_queues(int n) {
    if (n < 1 || n > 32) return fail(PT_ERR_INVALID, "hardware queue count must be in [1, 32]");
    if (g_hip_touched) return fail(PT_ERR_INVALID, "the HIP runtime is already running in this process");
    char v[16];
    std::snprintf(v, sizeof v, "%d", n);
    setenv("GPU_MAX_HW_QUEUES", v, 1);
    return PT_OK;
}

int pt_device_count(int* count_out) {
    if (!count_out) return fail(PT_ERR_INVALID, "count_out is NULL");
    g_hip_touched = true;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count_out = n;
    return PT_OK;
}

int pt_scene_create(const float* triangle_data, size_t triangle_len, const float* bvh_data, size_t bvh_len, int device,
                    pt_scene** scene_out) {
    if (!triangle_data || !bvh_data || !scene_out) return fail(PT_ERR_INVALID, "null argument");
    *scene_out = nullptr;
    g_hip_touched = true;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PT_ERR_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(PT_ERR_NODEVICE, "device ordinal out of range");
    HostLayout L;
    int rc = build_layout(triangle_data, triangle_len, bvh_data, bvh_len, L);
    if (rc != PT_OK) return rc;
    HIP_TRY(hipSetDevice(device));
    const size_t o_nodes = 0;
    const size_t o_tris = align_up(o_nodes + L.nodes.size() * sizeof(Node), 256);
    const size_t o_mats = align_up(o_tris + std::max<size_t>(1, L.tris.size()) * sizeof(Tri), 256);
    const size_t o_lights = align_up(o_mats + L.mats.size() * sizeof(Material), 256);
    const size_t o_lmask = align_up(o_lights + L.lights.size() * sizeof(Light), 16);
    const size_t o_bfnode = align_up(o_lmask + L.lmask.size() * sizeof(uint64_t), 16);
    const size_t o_bfmap = align_up(o_bfnode + L.bfnode.size() * sizeof(BfNode), 16);
    const size_t o_cnt = align_up(o_bfmap + L.bfmap.size() * sizeof(int32_t), 256);
    const size_t o_tn = align_up(o_cnt + sizeof(Counters), 256);
    const size_t o_lnode = align_up(o_tn + std::max<size_t>(1, L.tnorm.size()) * sizeof(float4), 256);
    const size_t o_lidx = align_up(o_lnode + L.lnodes.size() * sizeof(LNode), 256);
    const size_t o_pnode = align_up(o_lidx + std::max<size_t>(1, L.ltris.size()) * sizeof(Tri), 256);
    const size_t o_ptris = align_up(o_pnode + std::max<size_t>(1, L.pnodes.size()) * sizeof(LNode), 256);
    const size_t o_pnorm = align_up(o_ptris + std::max<size_t>(1, L.ptris.size()) * sizeof(Tri), 256);
    const size_t o_pre = align_up(o_pnorm + std::max<size_t>(1, L.pnorm.size()) * sizeof(float4), 256);
    const size_t o_nalt = align_up(o_pre + std::max<size_t>(1, L.pre.size()) * sizeof(PreLeaf), 256);
    const size_t total = align_up(o_nalt + std::max<size_t>(2, L.nalt.size()) * sizeof(int2), 256);
    pt_scene* s = new pt_scene();
    s->device = device;
    if (hipMalloc(&s->d_mem, total) != hipSuccess) { delete s; return fail(PT_ERR_NOMEM, "hipMalloc scene"); }
    char* base = static_cast<char*>(s->d_mem);
    auto up = [&](size_t off, const void* src, size_t bytes) { return bytes ? hipMemcpy(base + off, src, bytes, hipMemcpyHostToDevice) : hipSuccess; };
    if (up(o_nodes, L.nodes.data(), L.nodes.size() * sizeof(Node)) != hipSuccess ||
        up(o_tris, L.tris.data(), L.tris.size() * sizeof(Tri)) != hipSuccess ||
        up(o_mats, L.mats.data(), L.mats.size() * sizeof(Material)) != hipSuccess ||
        up(o_lights, L.lights.data(), L.lights.size() * sizeof(Light)) != hipSuccess ||
        up(o_lmask, L.lmask.data(), L.lmask.size() * sizeof(uint64_t)) != hipSuccess ||
        up(o_bfnode, L.bfnode.data(), L.bfnode.size() * sizeof(BfNode)) != hipSuccess ||
        up(o_bfmap, L.bfmap.data(), L.bfmap.size() * sizeof(int32_t)) != hipSuccess ||
        up(o_tn, L.tnorm.data(), L.tnorm.size() * sizeof(float4)) != hipSuccess ||
        up(o_lnode, L.lnodes.data(), L.lnodes.size() * sizeof(LNode)) != hipSuccess ||
        up(o_lidx, L.ltris.data(), L.ltris.size() * sizeof(Tri)) != hipSuccess ||
        up(o_pnode, L.pnodes.data(), L.pnodes.size() * sizeof(LNode)) != hipSuccess ||
        up(o_ptris, L.ptris.data(), L.ptris.size() * sizeof(Tri)) != hipSuccess ||
        up(o_pnorm, L.pnorm.data(), L.pnorm.size() * sizeof(float4)) != hipSuccess ||
        up(o_pre, L.pre.data(), L.pre.size() * sizeof(PreLeaf)) != hipSuccess ||
        up(o_nalt, L.nalt.data(), L.nalt.size() * sizeof(int2)) != hipSuccess) {
        pt_scene_destroy(s);
        return fail(PT_ERR_HIP, "scene upload failed");
    }
    s->view.nodes = reinterpret_cast<const Node*>(base + o_nodes);
    s->view.tris = reinterpret_cast<const Tri*>(base + o_tris);
    s->view.mats = reinterpret_cast<const Material*>(base + o_mats);
    s->view.lights = reinterpret_cast<const Light*>(base + o_lights);
    s->view.n_nodes = (int32_t)L.nodes.size();
    s->view.n_tris = (int32_t)L.tris.size();
    s->view.n_mats = (int32_t)L.mats.size();
    s->view.n_lights = L.ntri;
    s->view.f_ntri = (float)L.ntri;
    s->view.inv_ntri = 1.0f / (float)L.ntri;  // intersection-logic.wgsl:284
    s->view.max_stack = (int32_t)L.info.max_stack;
    s->view.fast_rcp = L.fast_rcp ? 1 : 0;
    s->view.node_bias = 0;  // per-pipeline default (launch_wavefront / launch_megakernel)
    s->view.node_steps = 0;  // per-pipeline default (launch_wavefront / launch_megakernel)
    s->view.off_tris = (uint32_t)(o_tris - o_nodes);
    s->view.off_mats = (uint32_t)(o_mats - o_nodes);
    s->view.off_lights = (uint32_t)(o_lights - o_nodes);
    s->view.off_lmask = (uint32_t)(o_lmask - o_nodes);
    s->view.lmask = reinterpret_cast<const uint64_t*>(base + o_lmask);
    s->view.mailbox = L.mailbox ? 1 : 0;
    s->view.tnorm = reinterpret_cast<const float4*>(base + o_tn);
    s->view.vnormals = 0;
    s->view.lnodes = L.lnodes.empty() ? nullptr : reinterpret_cast<const LNode*>(base + o_lnode);
    s->view.ltris = L.lnodes.empty() ? nullptr : reinterpret_cast<const Tri*>(base + o_lidx);
    s->view.pnodes = L.pnodes.empty() ? nullptr : reinterpret_cast<const LNode*>(base + o_pnode);
    s->view.ptris = L.pnodes.empty() ? nullptr : reinterpret_cast<const Tri*>(base + o_ptris);
    s->view.pnorm = L.pnodes.empty() ? nullptr : reinterpret_cast<const float4*>(base + o_pnorm);
    s->view.nalt = L.nalt.empty() ? nullptr : reinterpret_cast<const int4*>(base + o_nalt);
    s->leaf_min = L.leaf_min;
    s->lleaves = L.lleaves;
    s->pre = L.pre;
    if (!L.pre.empty()) {
        s->h_nodes = L.nodes;
        s->h_tris = L.tris;
        s->h_lights.assign(L.lights.begin(), L.lights.begin() + std::min<size_t>(L.lights.size(), L.info.emissive_tris));
    }
    s->leaf_sizes = L.leaf_sizes;
    s->d_pre = L.pre.empty() ? nullptr : reinterpret_cast<const PreLeaf*>(base + o_pre);
    s->view.mb_base = L.mb_base;
    s->view.bfnode = L.bfnode.empty() ? nullptr : reinterpret_cast<const BfNode*>(base + o_bfnode);
    s->view.bfmap = L.bfmap.empty() ? nullptr : reinterpret_cast<const int32_t*>(base + o_bfmap);
    s->view.off_bfnode = (uint32_t)(o_bfnode - o_nodes);
    s->view.off_bfmap = (uint32_t)(o_bfmap - o_nodes);
    s->view.span_bytes = (uint32_t)align_up(o_bfmap + L.bfmap.size() * sizeof(int32_t) - o_nodes, 16);
    s->d_counters = reinterpret_cast<Counters*>(base + o_cnt);
    s->info = L.info;
    s->info.device_bytes = total;
    *scene_out = s;
    return PT_OK;
}

void pt_scene_destroy(pt_scene* s) {
    if (!s) return;
    hipSetDevice(s->device);
    if (s->stream) { hipStreamSynchronize(s->stream); hipStreamDestroy(s->stream); }
    if (s->d_accum) hipFree(s->d_accum);
    if (s->d_wf) hipFree(s->d_wf);
    for (int h = 0; h < kMaxParts; ++h) {
        if (s->ws.aux[h]) { hipStreamSynchronize(s->ws.aux[h]); hipStreamDestroy(s->ws.aux[h]); }
        if (s->ws.join[h]) hipEventDestroy(s->ws.join[h]);
    }
    if (s->ws.fork) hipEventDestroy(s->ws.fork);
    if (s->d_rad) hipFree(s->d_rad);
    if (s->d_pres) hipFree(s->d_pres);
    if (s->d_peer) hipFree(s->d_peer);
    if (s->d_rgba) hipFree(s->d_rgba);
    if (s->h_ctl) hipHostFree(s->h_ctl);
    if (s->d_mem) hipFree(s->d_mem);
    s->prof.destroy();
    delete s;
}

int pt_scene_set_vertex_normals(pt_scene* s, int enable) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    s->view.vnormals = enable ? 1 : 0;
    return PT_OK;
}

int pt_scene_get_info(const pt_scene* s, pt_scene_info* out) {
    if (!s || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = s->info;
    return PT_OK;
}

}  // extern "C"

namespace {

// meta (program-raymarch.ts:79-92) -> FrameParams.  view_half_h uses the pinned tan
// (program-raymarch.wgsl:62); it is uniform, so it is evaluated once here.
int make_params(const float* meta, int max_depth, FrameParams& fp) {
    if (!meta) return fail(PT_ERR_INVALID, "meta is NULL");
    const float W = meta[0], H = meta[1];
    if (!(W >= 1.0f && H >= 1.0f && W <= 32768.0f && H <= 32768.0f) || W != std::floor(W) || H != std::floor(H))
        return fail(PT_ERR_INVALID, "meta[0..1] must be integral resolutions in [1, 32768]");
    if (max_depth < -1 || max_depth > 1024) return fail(PT_ERR_INVALID, "max_depth out of range");
    std::memset(&fp, 0, sizeof fp);
    fp.W = W; fp.H = H;
    fp.inv_w = meta[8]; fp.inv_h = meta[9];
    fp.aspect = meta[10];
    fp.focal = meta[2];
    fp.view_half_h = (2.0f * meta[2]) * tan_p(meta[3] * 0.5f);
    fp.rr_prob = meta[45];
    for (int i = 0; i < 4; ++i) fp.cam[i] = meta[4 + i];
    for (int i = 0; i < 16; ++i) fp.M[i] = meta[28 + i];
    fp.width = (uint32_t)W; fp.height = (uint32_t)H;
    fp.direct_only = meta[46] > 0.0f ? 1 : 0;
    fp.max_depth = max_depth < 0 ? 16 : max_depth;
    return PT_OK;
}

// PT_MODE_* -> pipeline.  A/B overrides (pt_set_option): kernel=literal|mega|wavefront, lds=0|1,
// trav=nested|flat1|pred|lean|lean2|lean4|lean8|lean16|lean32, fastrcp=0|1, ...
// AUTO picks the wavefront pipeline once a call has this many paths: below it the fixed
// cost of its ~2(D+1) launches per batch outweighs its better SIMD utilisation.  Measured per
// scene type (round 2, depth 16, ms megakernel / wavefront): mailbox scenes (the fused kernel)
// gain at every size (CornellBox 128^2 x 1: 1.43 / 0.66), so do scenes with cooperative big
// leaves (MedievalBoat 256^2 x 1: 62 / 35); other scenes from about 2^19 paths (Glossy 512^2 x 1:
// 7.1 / 9.1, 512^2 x 2: 13.1 / 9.6).
constexpr uint64_t kWfAutoMinPaths = 1ull << 19;
// k_wf_trace narrows its windows when 32-entry ones would keep < 1/4 of the waves busy (option
// trace_sparse=n; in-process A/B: MedievalBoat +16 %, Glossy and the synthetic scenes +-0.5 %)
constexpr int kTraceSparseDefault = 4;
// camera batches dealt to the fused kernel's regions by a permutation (option region_perm): a
// block's 8 waves serve 8 neighbouring regions, which in row order hold neighbouring batches — at
// 4096^2, 512 neighbouring pixels of one row (an eighth of it) on one CU; permuted, batches far
// apart: 4096^2 2475 -> 2679 Msamples/s, 1024^2 and Mirror unchanged (profiles/r03h_ab_region_perm.txt)
constexpr int kRegionPermDefault = 1;

LaunchOpts launch_opts(const Opts& o, int mode, uint64_t paths, const SceneView& view) {
    LaunchOpts lo;
    const uint64_t auto_min = (view.mailbox || view.big_leaf > 0) ? 1 : kWfAutoMinPaths;
    lo.wavefront = mode == PT_MODE_WAVEFRONT || (mode == PT_MODE_AUTO && paths >= auto_min);
    if (o.has("kernel")) {
        lo.literal = o.is("kernel", "literal");
        if (o.is("kernel", "wavefront")) lo.wavefront = true;
        if (o.is("kernel", "mega") || lo.literal) lo.wavefront = false;
    }
    lo.lds = o.flag("lds", 1) != 0;
    lo.fast_rcp = o.flag("fastrcp", lo.fast_rcp);
    lo.parts = (int)o.num("parts", lo.parts);
    lo.fuse_gen = o.flag("fuse_gen", lo.fuse_gen);
    lo.dual = o.flag("dual", lo.dual);
    lo.fuse = o.flag("fuse", lo.fuse);
    lo.bf = o.flag("bf", lo.bf);
    lo.mailbox = o.flag("mailbox", lo.mailbox);
    lo.sort = (int)o.num("sort", lo.sort);  // 1 / 8: direction octant; 64: + origin octant; 512: + 4^3 origin cells
    lo.trace_sparse = (int)o.num("trace_sparse", kTraceSparseDefault);
    lo.region_perm = o.flag("region_perm", kRegionPermDefault);
    lo.regen = (int)std::max(0L, std::min(1L << 20, o.num("regen", 0)));
    lo.trace_ring = (int)o.num("trace_ring", 0);
    lo.trace_blocks = (int)o.num("wf_trace_blocks", 0);
    lo.watchdog = (uint32_t)o.num("trace_watchdog", 0);
    lo.bf_slots = (int)o.num("bf_slots", -1);
    lo.leaf_blocks = (int)o.num("leaf_blocks", 0);
    // | 4: the pair walk's second check of the open chunks with the entries' own normals (option
    // leaf_refine, default on; pt_leafpass.hip)
    lo.leaf_pairs = (int)std::max(0L, std::min(2L, o.num("leaf_pairs", 1))) | (o.flag("leaf_refine", 1) != 0 ? 4 : 0);
    if (o.has("trav")) {
        static const char* const names[] = {"nested", "flat1", "pred", "lean", "lean2", "lean4", "lean8", "lean16", "lean32"};
        for (int k = 0; k < 9; ++k)
            if (o.is("trav", names[k])) lo.trav = k;
    }
    return lo;
}

// paths in flight per wavefront batch (kWfBytesPerPath = 188 B of queue state per path: 64 M
// paths ~ 12 GB of the 288 GB, plus the queue slack of the region layout).  Every batch ends in
// launch tails that carry few paths at low occupancy (the last depths); a larger batch pays them
// for more samples: CornellBox 1024^2 x 256 +6 % at 64 M over 8 M, CornellBox-Glossy +28 %
// (probe of option wf_paths)
constexpr uint64_t kWfTargetPaths = 64ull << 20;
constexpr int kBigLeafDefault = 128;
constexpr long kPreRatioDefault = 50;  // render_impl: the leaf pass when >= 50 % of its work is visited

int ensure_rad(pt_scene* s, uint64_t paths) {
    if (s->d_rad && s->rad_cap >= paths) { s->wf.rad = s->d_rad; s->wf.rad_cap = s->rad_cap; return PT_OK; }
    if (s->d_rad) { hipDeviceSynchronize(); hipFree(s->d_rad); s->d_rad = nullptr; s->rad_cap = 0; }
    if (hipMalloc(&s->d_rad, 12 * paths) != hipSuccess) {
        s->d_rad = nullptr;
        (void)hipGetLastError();
        return fail(PT_ERR_NOMEM, "hipMalloc wavefront radiance");
    }
    s->rad_cap = paths;
    s->wf.rad = s->d_rad;
    s->wf.rad_cap = paths;
    return PT_OK;
}

// keys of the pre-resolved big leaves: npre per queue entry of the wavefront buffers
int ensure_pres(pt_scene* s, int npre) {
    const size_t need = (size_t)npre * s->wf.qcap;
    if (s->d_pres && s->pres_cap >= need) { s->wf.pres = s->d_pres; s->wf.pres_stride = s->wf.qcap; return PT_OK; }
    if (s->d_pres) { hipDeviceSynchronize(); hipFree(s->d_pres); s->d_pres = nullptr; s->pres_cap = 0; }
    if (hipMalloc(&s->d_pres, need * sizeof(uint64_t)) != hipSuccess) {
        s->d_pres = nullptr;
        (void)hipGetLastError();
        return fail(PT_ERR_NOMEM, "hipMalloc pre-resolved leaf keys");
    }
    s->pres_cap = need;
    s->wf.pres = s->d_pres;
    s->wf.pres_stride = s->wf.qcap;
    return PT_OK;
}

int ensure_wavefront(pt_scene* s, uint64_t paths) {
    if (s->d_wf && s->wf.capacity >= paths) return PT_OK;
    if (paths > 0x7fffffffull) return fail(PT_ERR_INVALID, "image too large for one wavefront batch");
    if (s->d_wf) { hipDeviceSynchronize(); hipFree(s->d_wf); s->d_wf = nullptr; s->wf.capacity = 0; }
    const size_t n = paths;
    // queue arrays carry slack so that each part can be cut into up to kRegions regions of a whole
    // number of 64-entry batches holding all its paths (k_wf_step_bf)
    const size_t qn = n + 2 * (size_t)kQueueSlackRegions * 64;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
    size_t oq[6];
    for (int k = 0; k < 6; ++k) oq[k] = take((k % 3 == 0 ? 32 : 16) * qn);
    const size_t o_p0 = take(16 * qn), o_p1 = take(16 * qn), o_p2 = take(8 * qn), o_hit = take(8 * qn),
                 o_ctl = take(4 * kMaxParts * WF_CTL_WORDS), o_rcnt = take(4 * kMaxParts * 3 * kRegions),
                 o_cam = take(2 * 64 * sizeof(float4));
    if (hipMalloc(&s->d_wf, off) != hipSuccess) {
        s->d_wf = nullptr;
        (void)hipGetLastError();  // the failed allocation is reported here, not by a later call
        return fail(PT_ERR_NOMEM, "hipMalloc wavefront state");
    }
    char* b = static_cast<char*>(s->d_wf);
    auto f4 = [&](size_t o) { return reinterpret_cast<float4*>(b + o); };
    WfBuffers& w = s->wf;
    w.ext = WfQueue{f4(oq[0]), f4(oq[1]), f4(oq[2])};
    w.shd = WfQueue{f4(oq[3]), f4(oq[4]), f4(oq[5])};
    w.sp0 = f4(o_p0); w.sp1 = f4(o_p1);
    w.sp2 = reinterpret_cast<float2*>(b + o_p2);
    w.hitq = reinterpret_cast<int2*>(b + o_hit);
    w.ctl = reinterpret_cast<uint32_t*>(b + o_ctl);
    w.rcnt = reinterpret_cast<uint32_t*>(b + o_rcnt);
    w.camtab = f4(o_cam);
    if (hipMemset(w.ctl, 0, 4 * kMaxParts * WF_CTL_WORDS) != hipSuccess ||
        hipMemset(w.rcnt, 0, 4 * kMaxParts * 3 * kRegions) != hipSuccess)
        return fail(PT_ERR_HIP, "hipMemset wavefront control words");
    if (!s->ws.aux[0]) {
        bool ok = hipEventCreateWithFlags(&s->ws.fork, hipEventDisableTiming) == hipSuccess;
        for (int h = 0; h < kMaxParts && ok; ++h)
            ok = hipStreamCreateWithFlags(&s->ws.aux[h], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&s->ws.join[h], hipEventDisableTiming) == hipSuccess;
        if (!ok) return fail(PT_ERR_HIP, "creating the wavefront's streams");
    }
    if (!s->h_ctl) {
        if (hipHostMalloc(reinterpret_cast<void**>(&s->h_ctl), 4 * kMaxParts * WF_CTL_WORDS) != hipSuccess) {
            s->h_ctl = nullptr;
            return fail(PT_ERR_NOMEM, "hipHostMalloc wavefront control mirror");
        }
        std::memset(s->h_ctl, 0, 4 * kMaxParts * WF_CTL_WORDS);
    }
    w.capacity = (uint32_t)n;
    w.qcap = (uint32_t)qn;
    w.rq = w.rqi = 1;
    w.rad = s->d_rad;
    w.rad_cap = s->rad_cap;
    return PT_OK;
}

// A trace wave that hit its watchdog (k_wf_trace: kTraceWatchdog iterations or
// kTraceWatchdogTicks) sets ctl[WF_WATCHDOG] and leaves its state in ctl[WF_SNAP..]; later
// launches of the scene skip their work.  The pinned mirror h_ctl receives the control words
// after every wavefront render on its stream; once that copy has landed (the caller synchronised,
// or the blocking calls' own synchronisation) the flag is reported here — by whichever call of
// the scene comes next, megakernel or wavefront — and cleared.  The failure path waits for the
// device first, so no mirror copy still in flight can bring the flag back after the clear and
// report the same failure twice.
int take_watchdog(pt_scene* s) {
    if (!s->h_ctl) return PT_OK;
    int h = 0;
    while (h < kMaxParts && !__atomic_load_n(&s->h_ctl[h * WF_CTL_WORDS + WF_WATCHDOG], __ATOMIC_ACQUIRE)) ++h;
    if (h == kMaxParts) return PT_OK;
    HIP_TRY(hipDeviceSynchronize());  // every pending mirror copy of the scene has landed
    uint32_t v[WF_SNAP_WORDS];
    std::memcpy(v, s->h_ctl + h * WF_CTL_WORDS + WF_SNAP, sizeof v);
    for (int k = 0; k < kMaxParts; ++k)
        HIP_TRY(hipMemset(s->wf.ctl + k * WF_CTL_WORDS + WF_WATCHDOG, 0,
                          (WF_SNAP + WF_SNAP_WORDS - WF_WATCHDOG) * sizeof(uint32_t)));
    std::memset(s->h_ctl, 0, 4 * kMaxParts * WF_CTL_WORDS);
    char msg[360];
    std::snprintf(msg, sizeof(msg),
                  "wavefront trace gave up after its watchdog limit (result invalid); first wave: count=%u "
                  "nwaves=%u w=%u jl=%u wv=%u nv=%u cur=%u flushed=%u in_flight=%u mask=%08x%08x queue=%u",
                  v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[10], v[9], v[11]);
    return fail(PT_ERR_HIP, msg);
}

int render_impl(pt_scene* s, const float* meta, uint32_t frame0, uint32_t nframes, uint32_t stride, int max_depth,
                int mode, bool accum, float* d_out, Counters* d_cnt, hipStream_t stream) {
    FrameParams fp{};
    int rc = make_params(meta, max_depth, fp);
    if (rc != PT_OK) return rc;
    if (mode != PT_MODE_AUTO && mode != PT_MODE_MEGAKERNEL && mode != PT_MODE_WAVEFRONT)
        return fail(PT_ERR_INVALID, "unknown mode");
    if (accum && (uint64_t)frame0 + (uint64_t)(nframes ? nframes - 1 : 0) * stride >= (1ull << 24))
        return fail(PT_ERR_INVALID, "frame index >= 2^24 (t_k = u32(f32(k)) would round)");
    HIP_TRY(hipSetDevice(s->device));
    if (nframes == 0) return PT_OK;
    const uint64_t npix = (uint64_t)fp.width * fp.height;
    struct ProfScope {  // attach the scene's profiler to this thread for the launches below
        explicit ProfScope(KernelProfiler* p) { t_prof = p; }
        ~ProfScope() { t_prof = nullptr; }
    } prof_scope(s->prof_on ? &s->prof : nullptr);
    SceneView view = s->view;
    const Opts o = opts_snapshot();
    if (o.has("node_bias")) view.node_bias = std::max(1L, o.num("node_bias", 1));  // A/B runs
    if (o.has("node_steps")) view.node_steps = (int32_t)std::max(1L, std::min(8L, o.num("node_steps", 1)));
    // big leaves (lean traversal): a ray reaching a leaf of >= big_leaf entries has it tested by the
    // whole wave (pt_device.h big_turn); default 128 (MedievalBoat 2.3x, in-process A/B; 64 is 1.5 %
    // faster there but 12 % slower on the 1M-triangle synthetic scene, whose many 64..127-entry
    // leaves waste half a cooperative step each); option big_leaf=n sets it, 0 turns big-leaf
    // turns and leaf chunks off
    {
        const long big = o.num("big_leaf", kBigLeafDefault);
        view.big_leaf = (big > 0 && s->info.max_leaf >= (uint32_t)big) ? (int32_t)big : 0;
        // leaf BVHs (built at pt_scene_create, option leaf_bvh): lanes park at every leaf that has
        // chunks and test them chunk by chunk (chunk_turn_multi); option leaf_walk=0 keeps them out (A/B)
        if (big > 0 && s->leaf_min > 0 && o.flag("leaf_walk", 1) != 0)
            view.big_leaf = view.big_leaf > 0 ? std::min<int32_t>(view.big_leaf, s->leaf_min) : s->leaf_min;
        else
            view.lnodes = nullptr;
    }
    // pooled leaf turns (pt_device.h lean_leaf_pool) on every tree (option leaf_pool=0: each lane
    // walks its own pairs).  The run length: 2 on trees of short leaves (< 16 entries: the SAH
    // builder's; Glossy +2.9 %, the boat +16.5 %, 100k +26 %, 1M +29 % over unpooled:
    // profiles/r04am_sah_pool.log — runs of 4 there cost Glossy 3.6 %, r04t_configs.jsonl) and
    // where the leaves reference >= 32 Ki triangles and no leaf is big (100k +12 %, 1M +26 % against
    // runs of 4: r04aa_ab_run.log; 12.5k +3.7 % with node bias 1-2: r04ak_run2_bias.log), else 4
    // (Glossy 5 Ki references, 1k, and the boat — 52 Ki references, but big leaves walked in
    // chunks — are 1-2 % faster with 4); option pool_run=2|4.  Round 6, with four node steps per node
    // turn: runs of 2 on every tree without big leaves (Glossy +5 %, 1k +2.2 %, 12.5k +0.8 % over 4;
    // the boat, whose big leaves go to the leaf pass, -0.7 %: profiles/r06ac_ab_*.log)
    {
        const bool pool = o.flag("leaf_pool", 1) != 0;
        const bool run2 = s->info.max_leaf < 16 || view.big_leaf == 0;
        const long run = o.num("pool_run", run2 ? 2 : 4);
        view.leaf_pool = pool ? (int32_t)run : 0;
    }
    // leaf remainders (pt_device.h lean_node_unit): option leaf_skip=0 keeps them out (A/B); a big-leaf
    // threshold below kLeafSkipMaxLeaf too (a leaf the cooperative turns or the leaf pass take by its
    // first record must keep it)
    if (o.flag("leaf_skip", 1) == 0 || (view.big_leaf > 0 && view.big_leaf < kLeafSkipMaxLeaf)) view.nalt = nullptr;
    // the brute-force replay walks the BfNode tree without a stack (bf_stackless=0: the stack walk; A/B)
    if (o.flag("bf_stackless", 1) == 0) view.bfnode = nullptr;
    const LaunchOpts lo = launch_opts(o, mode, npix * (accum ? nframes : 1), view);
    // big leaves resolved before the traversal (k_wf_leafpass, pt_leafpass.hip; option leaf_pre=0:
    // the cooperative turns and chunk walks inside k_wf_trace): the leaves of >= big_leaf entries, at
    // most kMaxPre of them — with more, the threshold rises above the (kMaxPre + 1)-th largest and
    // the rest are ordinary leaves of the pooled turns
    // The leaf pass resolves a leaf for every ray that passes its box filter; the traversal tests it
    // only for the rays that reach it, and a ray whose closest hit so far is nearer than a box on the
    // leaf's path never does.  Where the filter over-predicts — the boat of CornellBox2's all-meshes
    // scene sits inside the box's walls: 0.33 of the filtered leaf work is visited, 65 against 91.6
    // Msamples/s without the pass (profiles/r05d_auto_ab.log) — the pass costs more than it saves;
    // the boat alone visits 0.99 of it (+30 %).  The choice (option leaf_pre absent or 2) follows the
    // scene's probe (pt_scene::pre_probe, pt_leafbvh.h probe_pre_leaves; CornellBox2 all meshes 0.38,
    // the boat 1.00): the pass when the visited entries are at least pre_ratio % (default
    // kPreRatioDefault) of the filtered ones, each leaf weighted by its entries.  leaf_pre=1 always,
    // 0 never.  (The choice changes the kernels, not the image: both paths are exact.)
    view.npre = 0;
    view.pre = nullptr;
    const long pre_opt = o.num("leaf_pre", 2);
    if (lo.wavefront && view.big_leaf > 0 && pre_opt != 0 && !s->pre.empty()) {
        int32_t T = view.big_leaf;
        if (s->leaf_sizes.size() > (size_t)kMaxPre && s->leaf_sizes[kMaxPre] >= T) T = s->leaf_sizes[kMaxPre] + 1;
        int np = 0;
        while (np < (int)s->pre.size() && s->pre[(size_t)np].n >= T) ++np;
        // more big leaves than the table holds: the pass would raise the threshold to T and the big
        // leaves left out (big_leaf <= n < T) would lose their chunk walks and cooperative turns, a
        // cost the probe below does not weigh — AUTO keeps the traversal's own big-leaf machinery then
        // (advisor r05; leaf_pre=1 still forces the pass)
        if (pre_opt != 1 && T > view.big_leaf) np = 0;
        if (np > 0 && pre_opt != 1) {
            std::lock_guard<std::mutex> lk(s->pre_mu);
            ProbeCamera pc{};
            for (int c = 0; c < 3; ++c) pc.cam[c] = fp.cam[c];
            for (int c = 0; c < 16; ++c) pc.M[c] = fp.M[c];
            pc.focal = fp.focal;
            pc.half_h = fp.view_half_h;
            pc.half_w = fp.view_half_h * fp.aspect;
            // probed once per camera: a render whose camera differs from the probe's probes again
            // (advisor r05: the choice is the camera's; both paths give the same bits)
            if (!s->pre_probed || std::memcmp(&pc, &s->pre_cam, sizeof pc) != 0) {
                probe_pre_leaves(s->h_nodes, s->h_tris, s->h_lights, s->pre, pc, kPreProbeGrid, kPreProbeTests,
                                 s->pre_probe);
                s->pre_cam = pc;
                s->pre_probed = true;
            }
        }
        if (np > 0 && pre_opt != 1 && s->pre_probe.size() >= (size_t)np) {
            double filt = 0.0, vis = 0.0;
            for (int b = 0; b < np; ++b) {
                filt += (double)s->pre_probe[(size_t)b][0] * s->pre[(size_t)b].n;
                vis += (double)s->pre_probe[(size_t)b][1] * s->pre[(size_t)b].n;
            }
            if (filt > 0.0 && vis * 100.0 < filt * (double)o.num("pre_ratio", kPreRatioDefault)) np = 0;
        }
        if (np > 0) {
            // pt_device.h pre_slot finds a leaf's key slot by its first record among the first np table
            // entries, and answers slot 0 for any other: every leaf of >= T entries must be among them
            // (the table is the kMaxPre largest, and T was raised above the (kMaxPre + 1)-th; advisor r05)
            for (size_t k = (size_t)np; k < s->pre.size(); ++k)
                if (s->pre[k].n >= T) return fail(PT_ERR_SCENE, "internal: a leaf of >= big_leaf entries outside the pre-resolved table");
            if (s->leaf_sizes.size() > (size_t)np && s->leaf_sizes[(size_t)np] >= T)
                return fail(PT_ERR_SCENE, "internal: more leaves of >= big_leaf entries than the pre-resolved table holds");
            view.big_leaf = T;
            view.npre = np;
            view.pre = s->d_pre;
            for (int b = 0; b < kMaxPre; ++b) view.pre_rec0[b] = b < np ? s->pre[(size_t)b].rec0 : -1;
        }
    }
    if ((rc = take_watchdog(s)) != PT_OK) return rc;  // an earlier asynchronous render failed
    if (lo.wavefront) {
        // the target in whole pairs of frames (a batch's two parts take whole frames each): 4096^2
        // holds 4 frames (67 M paths), not 2 of the 3.8 that 64 M would hold
        const uint64_t target0 = (uint64_t)std::max(1L, o.num("wf_paths", (long)kWfTargetPaths));  // A/B
        const uint64_t pairs = (target0 + 2 * npix - 1) / (2 * npix) * (2 * npix);
        const uint64_t target = o.has("wf_paths") || pairs > 0x7fffffffull ? target0 : pairs;
        // at least two frames per batch when the call has two (images above the target, e.g.
        // 4096^2): the batch's parts run on their own streams and overlap (+29 % at 4096^2)
        const uint64_t all = npix * (accum ? nframes : 1);
        const uint64_t two = 2 * npix <= 0x7fffffffull ? 2 * npix : npix;
        // a call that fits the target runs as one batch: its two parts take whole frames each, so
        // an odd frame count gets one frame of room more (5 frames: 3 + 2, not batches of 4 and 1)
        const uint64_t all_even = accum && nframes > 1 && (nframes & 1) ? all + npix : all;
        const uint64_t want = std::max<uint64_t>(std::min<uint64_t>(all, two), std::min<uint64_t>(all_even, target));
        int rc2 = ensure_wavefront(s, want);
        // the batch's state (~188 B/path: 12 GB at the 64 M-path target) may not fit beside other
        // allocations: halve it down to one frame per batch before giving up
        const uint64_t floor_paths = std::min<uint64_t>(all, npix);
        for (uint64_t w = want; rc2 == PT_ERR_NOMEM && w > floor_paths;)
            rc2 = ensure_wavefront(s, w = std::max<uint64_t>(w / 2, floor_paths));
        if (rc2 != PT_OK) return rc2;
        rc2 = ensure_rad(s, s->wf.capacity);
        if (rc2 != PT_OK) return rc2;
        if (view.npre > 0) {
            if ((rc2 = ensure_pres(s, view.npre)) != PT_OK) return rc2;
        } else {
            s->wf.pres = nullptr;
        }
        HIP_TRY(launch_wavefront(lo, view, fp, s->wf, frame0, nframes, stride, accum, d_cnt != nullptr, d_out, d_cnt,
                                 stream, s->ws));
        HIP_TRY(hipMemcpyAsync(s->h_ctl, s->wf.ctl, 4 * kMaxParts * WF_CTL_WORDS, hipMemcpyDeviceToHost, stream));
        return PT_OK;
    }
    HIP_TRY(launch_megakernel(lo, view, fp, frame0, nframes, stride, accum, d_cnt != nullptr, d_out, d_cnt, stream));
    return PT_OK;
}

int ensure_accum(pt_scene* s, size_t n) {
    if (s->accum_cap >= n) return PT_OK;
    if (s->d_accum) hipFree(s->d_accum);
    s->d_accum = nullptr;
    s->accum_cap = 0;
    if (hipMalloc(&s->d_accum, n * sizeof(float)) != hipSuccess) return fail(PT_ERR_NOMEM, "hipMalloc accumulator");
    s->accum_cap = n;
    return PT_OK;
}

}  // namespace

extern "C" {

int pt_render_async(pt_scene* s, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
                    int max_depth, int mode, float* d_accum, pt_counters* d_counters, void* stream) {
    if (!s || !d_accum) return fail(PT_ERR_INVALID, "null argument");
    return render_impl(s, meta, frame0, nframes, frame_stride, max_depth, mode, true, d_accum,
                       reinterpret_cast<Counters*>(d_counters), static_cast<hipStream_t>(stream));
}

// After a synchronised call: a trace wave that hit kTraceWatchdog left a flag (cleared here).
static int check_watchdog(pt_scene* s) { return take_watchdog(s); }

int pt_scene_check(pt_scene* s) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());  // every render of the scene, on whatever stream, has finished
    return take_watchdog(s);
}

// The blocking calls' own stream, created on first use: asynchronous callers never pay for a
// stream (HIP multiplexes every stream of the process onto GPU_MAX_HW_QUEUES hardware queues,
// and an idle extra stream can push the dual-stream wavefront's two onto one queue).
static int blocking_stream(pt_scene* s) {
    if (!s->stream && hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        s->stream = nullptr;
        return fail(PT_ERR_HIP, "hipStreamCreate");
    }
    return PT_OK;
}

int pt_render(pt_scene* s, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
              int max_depth, int mode, float* accum, pt_counters* counters) {
    if (!s || !accum || !meta) return fail(PT_ERR_INVALID, "null argument");
    FrameParams fp{};
    int rc = make_params(meta, max_depth, fp);
    if (rc != PT_OK) return rc;
    const size_t n = (size_t)fp.width * fp.height * 3;
    HIP_TRY(hipSetDevice(s->device));
    if ((rc = ensure_accum(s, n)) != PT_OK || (rc = blocking_stream(s)) != PT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(s->d_accum, accum, n * sizeof(float), hipMemcpyHostToDevice, s->stream));
    if (counters) HIP_TRY(hipMemsetAsync(s->d_counters, 0, sizeof(Counters), s->stream));
    rc = render_impl(s, meta, frame0, nframes, frame_stride, max_depth, mode, true, s->d_accum,
                     counters ? s->d_counters : nullptr, s->stream);
    if (rc != PT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(accum, s->d_accum, n * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (counters) HIP_TRY(hipMemcpyAsync(counters, s->d_counters, sizeof(Counters), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return check_watchdog(s);
}

int pt_frame_async(pt_scene* s, const float meta[48], uint32_t t, int max_depth, float* d_radiance, void* stream) {
    if (!s || !d_radiance) return fail(PT_ERR_INVALID, "null argument");
    return render_impl(s, meta, t, 1, 1, max_depth, PT_MODE_AUTO, false, d_radiance, nullptr,
                       static_cast<hipStream_t>(stream));
}

int pt_frame(pt_scene* s, const float meta[48], uint32_t t, int max_depth, float* radiance) {
    if (!s || !radiance || !meta) return fail(PT_ERR_INVALID, "null argument");
    FrameParams fp{};
    int rc = make_params(meta, max_depth, fp);
    if (rc != PT_OK) return rc;
    const size_t n = (size_t)fp.width * fp.height * 3;
    HIP_TRY(hipSetDevice(s->device));
    if ((rc = ensure_accum(s, n)) != PT_OK || (rc = blocking_stream(s)) != PT_OK) return rc;
    rc = render_impl(s, meta, t, 1, 1, max_depth, PT_MODE_AUTO, false, s->d_accum, nullptr, s->stream);
    if (rc != PT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(radiance, s->d_accum, n * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return check_watchdog(s);
}

int pt_tonemap_async(pt_scene* s, const float* d_accum, size_t npix, uint32_t sample_runs, uint8_t* d_rgba,
                     void* stream) {
    if (!s || !d_accum || !d_rgba || sample_runs == 0) return fail(PT_ERR_INVALID, "null argument or zero sample_runs");
    HIP_TRY(hipSetDevice(s->device));
    struct ProfScope {
        explicit ProfScope(KernelProfiler* p) { t_prof = p; }
        ~ProfScope() { t_prof = nullptr; }
    } prof_scope(s->prof_on ? &s->prof : nullptr);
    HIP_TRY(launch_tonemap(d_accum, npix, sample_runs, d_rgba, static_cast<hipStream_t>(stream)));
    return PT_OK;
}

int pt_readback_async(pt_scene* s, const float* d_src, size_t n, float* h_dst, void* stream) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    if (n == 0) return PT_OK;
    if (!d_src || !h_dst) return fail(PT_ERR_INVALID, "null argument");
    if (((uintptr_t)d_src | (uintptr_t)h_dst) & 15u) return fail(PT_ERR_INVALID, "buffers must be 16-byte aligned");
    HIP_TRY(hipSetDevice(s->device));
    void* hd = nullptr;  // pinned host memory: its address in the device's view
    if (hipHostGetDevicePointer(&hd, h_dst, 0) != hipSuccess || !hd) {
        (void)hipGetLastError();
        return fail(PT_ERR_INVALID, "h_dst is not pinned (page-locked) host memory");
    }
    HIP_TRY(launch_readback(d_src, static_cast<float*>(hd), n, static_cast<hipStream_t>(stream)));
    return PT_OK;
}

int pt_render_image(pt_scene* s, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
                    int max_depth, int mode, uint8_t* rgba, pt_counters* counters) {
    if (!s || !rgba || !meta) return fail(PT_ERR_INVALID, "null argument");
    if (nframes == 0) return fail(PT_ERR_INVALID, "nframes == 0 (the image divides by the sample count)");
    FrameParams fp{};
    int rc = make_params(meta, max_depth, fp);
    if (rc != PT_OK) return rc;
    const size_t npix = (size_t)fp.width * fp.height;
    HIP_TRY(hipSetDevice(s->device));
    if ((rc = ensure_accum(s, 3 * npix)) != PT_OK || (rc = blocking_stream(s)) != PT_OK) return rc;
    if (s->rgba_cap < 4 * npix) {
        if (s->d_rgba) hipFree(s->d_rgba);
        s->d_rgba = nullptr;
        s->rgba_cap = 0;
        if (hipMalloc(&s->d_rgba, 4 * npix) != hipSuccess) return fail(PT_ERR_NOMEM, "hipMalloc image");
        s->rgba_cap = 4 * npix;
    }
    HIP_TRY(hipMemsetAsync(s->d_accum, 0, 3 * npix * sizeof(float), s->stream));
    if (counters) HIP_TRY(hipMemsetAsync(s->d_counters, 0, sizeof(Counters), s->stream));
    rc = render_impl(s, meta, frame0, nframes, frame_stride, max_depth, mode, true, s->d_accum,
                     counters ? s->d_counters : nullptr, s->stream);
    if (rc != PT_OK) return rc;
    if ((rc = pt_tonemap_async(s, s->d_accum, npix, nframes, s->d_rgba, s->stream)) != PT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(rgba, s->d_rgba, 4 * npix, hipMemcpyDeviceToHost, s->stream));
    if (counters) HIP_TRY(hipMemcpyAsync(counters, s->d_counters, sizeof(Counters), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return check_watchdog(s);
}

int pt_tonemap(const float* acc, size_t npix, uint32_t sample_runs, uint8_t* rgba) {
    if (!acc || !rgba || sample_runs == 0) return fail(PT_ERR_INVALID, "null argument or zero sample_runs");
    auto to_int32 = [](double v) -> int32_t {  // ECMAScript ToInt32
        if (!std::isfinite(v)) return 0;
        double m = std::fmod(std::trunc(v), 4294967296.0);
        if (m < 0) m += 4294967296.0;
        return (int32_t)(uint32_t)m;
    };
    auto u8 = [](int32_t v) -> uint8_t { return v < 0 ? 0 : (v > 255 ? 255 : (uint8_t)v); };
    for (size_t i = 0; i < npix; ++i) {
        const double r = (double)acc[3 * i] / sample_runs, g = (double)acc[3 * i + 1] / sample_runs,
                     b = (double)acc[3 * i + 2] / sample_runs;
        const double lum = (r + g + b) / 3.0;
        const double f = std::pow(lum / (lum + 1.0), 0.01);
        rgba[4 * i] = u8(to_int32(r * f * 255.0));
        rgba[4 * i + 1] = u8(to_int32(g * f * 255.0));
        rgba[4 * i + 2] = u8(to_int32(b * f * 255.0));
        rgba[4 * i + 3] = 255;
    }
    return PT_OK;
}

int pt_selftest_math(int device, int fn, const float* a, const float* b, float* out, size_t n) {
    if (!a || !b || !out || n == 0 || n > (1u << 28)) return fail(PT_ERR_INVALID, "bad argument");
    if (fn < 0 || fn >= PT_MATH_COUNT_) return fail(PT_ERR_INVALID, "unknown math fn");
    HIP_TRY(hipSetDevice(device));
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc(&da, n * 4));
    HIP_TRY(hipMalloc(&db, n * 4));
    HIP_TRY(hipMalloc(&dout, n * 4));
    hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice);
    hipError_t e = launch_selftest_math(fn, da, db, dout, (int)n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(dout);
    if (e != hipSuccess) return fail(PT_ERR_HIP, hipGetErrorString(e));
    return PT_OK;
}

int pt_selftest_valu(int device, int iters, int reps, int packed, double* ms_out, uint64_t* fma_wave_instr_out) {
    if (iters < 1 || reps < 1 || !ms_out) return fail(PT_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(device));
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const int blocks = cus * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
    float* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)blocks * 256 * sizeof(float)));
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e = hipEventCreate(&a);
    if (e == hipSuccess) e = hipEventCreate(&b);
    if (e == hipSuccess) e = launch_selftest_valu(iters, blocks, packed, d, nullptr);  // warm-up (clock ramp)
    if (e == hipSuccess) e = hipEventRecord(a, nullptr);
    for (int r = 0; r < reps && e == hipSuccess; ++r) e = launch_selftest_valu(iters, blocks, packed, d, nullptr);
    if (e == hipSuccess) e = hipEventRecord(b, nullptr);
    if (e == hipSuccess) e = hipEventSynchronize(b);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
    hipFree(d);
    if (e != hipSuccess) return fail(PT_ERR_HIP, hipGetErrorString(e));
    *ms_out = ms;
    // v_fma_f32 / v_pk_fma_f32 wave-instructions of the timed launches: 32 per iteration per wave
    if (fma_wave_instr_out) *fma_wave_instr_out = (uint64_t)reps * blocks * 4 * (uint64_t)iters * 32;
    return PT_OK;
}

int pt_scene_leaf_bvh(const pt_scene* s, int leaf, int32_t* first_record, int32_t* entries, int32_t* nodes) {
    if (!s) return fail(PT_ERR_INVALID, "null scene");
    if (leaf < 0 || (size_t)leaf >= s->lleaves.size()) return fail(PT_ERR_INVALID, "no such leaf BVH");
    const auto& l = s->lleaves[(size_t)leaf];
    if (first_record) *first_record = l[0];
    if (entries) *entries = l[1];
    if (nodes) *nodes = l[2];
    return PT_OK;
}

int pt_selftest_leaf(pt_scene* s, int leaf, int mode, uint32_t seed, uint32_t nrays, int32_t* out) {
    if (!s || !out) return fail(PT_ERR_INVALID, "null argument");
    if (mode < 0 || (mode > 7 && mode < 16) || mode > 31 || nrays == 0 || nrays > (1u << 24))
        return fail(PT_ERR_INVALID, "bad mode or ray count");
    const bool pass = mode >= 16;
    if (!pass && (leaf < 0 || (size_t)leaf >= s->lleaves.size())) return fail(PT_ERR_INVALID, "no such leaf BVH");
    if (pass && (leaf < 0 || (size_t)leaf >= s->pre.size())) return fail(PT_ERR_INVALID, "no such pre-resolvable leaf");
    if (pass && ((mode >> 2) & 3) >= 2 && (!s->view.pnodes || s->pre[(size_t)leaf].c1 <= s->pre[(size_t)leaf].c0))
        return fail(PT_ERR_INVALID, "the leaf has no pass chunks (option leaf_bvh)");
    HIP_TRY(hipSetDevice(s->device));
    int32_t* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)nrays * 6 * sizeof(int32_t)));
    hipError_t e;
    if (pass) {
        SceneView v = s->view;
        v.pre = s->d_pre;
        v.npre = (int32_t)s->pre.size();
        e = launch_selftest_leafpass(v, leaf, mode & 15, seed, nrays, d, nullptr);
    } else {
        const auto& l = s->lleaves[(size_t)leaf];
        e = launch_selftest_leaf(s->view, l[0], l[1], mode, seed, nrays, d, nullptr);
    }
    if (e == hipSuccess) e = hipMemcpy(out, d, (size_t)nrays * 6 * sizeof(int32_t), hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) return fail(PT_ERR_HIP, hipGetErrorString(e));
    return PT_OK;
}

int pt_selftest_rcp(int device, int steps, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches,
                    uint32_t* failing_bits) {
    if (!mismatches || steps < -1 || steps > 2 || lo_bits > hi_bits || hi_bits >= 0x80000000u)
        return fail(PT_ERR_INVALID, "bad argument");
    if (steps < 0) steps = kRcpSteps;
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc(&d, 2 * sizeof(unsigned long long)));
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipMemset(d, 0, sizeof(h));
    if (e == hipSuccess) e = launch_selftest_rcp(steps, lo_bits, hi_bits, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) return fail(PT_ERR_HIP, hipGetErrorString(e));
    *mismatches = h[0];
    if (failing_bits) *failing_bits = (uint32_t)h[1];
    return PT_OK;
}


}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Multi-GPU (pt_render_multi): one host thread per device renders its frames, then ONE reduction
// ---------------------------------------------------------------------------------------------
namespace {

struct RcclApi {
    bool ok = false;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;

// librccl: the copy already in the process (e.g. torch's) if there is one, else the system's.
// Resolved once (a function-local static: thread-safe initialisation).
const RcclApi& rccl_api() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = nullptr;
        for (const char* n : {"librccl.so.1", "librccl.so"})
            if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
        for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
            if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.comm_init_all = reinterpret_cast<decltype(a.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        a.reduce = reinterpret_cast<decltype(a.reduce)>(dlsym(h, "ncclReduce"));
        a.group_start = reinterpret_cast<decltype(a.group_start)>(dlsym(h, "ncclGroupStart"));
        a.group_end = reinterpret_cast<decltype(a.group_end)>(dlsym(h, "ncclGroupEnd"));
        a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
        a.ok = a.comm_init_all && a.comm_destroy && a.reduce && a.group_start && a.group_end && a.error_string;
        return a;
    }();
    return api;
}

// one communicator set per device list, made on first use and kept until pt_release_communicators
// or process exit (an atexit handler registered after the HIP runtime started runs before the
// runtime's own teardown)
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

int destroy_comms_locked() {
    const RcclApi& a = rccl_api();
    ncclResult_t bad = ncclSuccess;
    for (auto& kv : g_comms)
        for (ncclComm_t c : kv.second) {
            const ncclResult_t r = a.comm_destroy(c);
            if (r != ncclSuccess) bad = r;
        }
    g_comms.clear();
    if (bad != ncclSuccess) return fail(PT_ERR_HIP, std::string("ncclCommDestroy: ") + a.error_string(bad));
    return PT_OK;
}

void destroy_comms_at_exit() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_comms.empty()) destroy_comms_locked();
}

int rccl_reduce(pt_scene* const* sc, int n, size_t count) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    const RcclApi& a = rccl_api();
    std::vector<int> devs(n);
    for (int g = 0; g < n; ++g) devs[g] = sc[g]->device;
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        static bool registered = false;
        if (!registered) registered = std::atexit(destroy_comms_at_exit) == 0;
        std::vector<ncclComm_t> c(n);
        const ncclResult_t r = a.comm_init_all(c.data(), n, devs.data());
        if (r != ncclSuccess) return fail(PT_ERR_HIP, std::string("ncclCommInitAll: ") + a.error_string(r));
        it = g_comms.emplace(devs, c).first;
    }
    // Nothing returns between ncclGroupStart and ncclGroupEnd: an open group would stay open for the
    // next RCCL call of the process.  No hipSetDevice inside the group either (each communicator
    // carries its device, and a failing call there was such a return, verdict r04 weak #3): the
    // reduces are issued until one fails, the group is always closed, then the error is reported.
    ncclResult_t r = a.group_start();
    if (r == ncclSuccess) {
        for (int g = 0; g < n && r == ncclSuccess; ++g)
            r = a.reduce(sc[g]->d_accum, sc[g]->d_accum, count, ncclFloat32, ncclSum, 0, it->second[g], sc[g]->stream);
        const ncclResult_t r2 = a.group_end();
        if (r == ncclSuccess) r = r2;
    }
    if (r != ncclSuccess) return fail(PT_ERR_HIP, std::string("ncclReduce: ") + a.error_string(r));
    for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(sc[g]->device));
        HIP_TRY(hipStreamSynchronize(sc[g]->stream));
    }
    return PT_OK;
}

// device order: partials of scenes 1..n-1 copied to device 0 and added there one after another
int ordered_reduce(pt_scene* const* sc, int n, size_t count) {
    pt_scene* s0 = sc[0];
    HIP_TRY(hipSetDevice(s0->device));
    if (s0->peer_cap < count) {
        if (s0->d_peer) hipFree(s0->d_peer);
        s0->d_peer = nullptr;
        s0->peer_cap = 0;
        if (hipMalloc(&s0->d_peer, count * sizeof(float)) != hipSuccess) return fail(PT_ERR_NOMEM, "hipMalloc peer accumulator");
        s0->peer_cap = count;
    }
    for (int g = 1; g < n; ++g) {
        if (sc[g]->device == s0->device)
            HIP_TRY(launch_accum_add(s0->d_accum, sc[g]->d_accum, count, s0->stream));
        else {
            HIP_TRY(hipMemcpyPeerAsync(s0->d_peer, s0->device, sc[g]->d_accum, sc[g]->device, count * sizeof(float),
                                       s0->stream));
            HIP_TRY(launch_accum_add(s0->d_accum, s0->d_peer, count, s0->stream));
        }
    }
    HIP_TRY(hipStreamSynchronize(s0->stream));
    return PT_OK;
}

}  // namespace

extern "C" int pt_render_multi(pt_scene* const* scenes, int n, const float meta[48], uint32_t frame0, uint32_t nframes,
                               uint32_t frame_stride, int max_depth, int mode, float* accum, pt_counters* counters) {
    if (!scenes || n < 1 || n > 64 || !meta || !accum) return fail(PT_ERR_INVALID, "bad argument");
    for (int g = 0; g < n; ++g)
        for (int h = 0; h < g; ++h)
            if (!scenes[g] || scenes[g] == scenes[h]) return fail(PT_ERR_INVALID, "null or repeated scene");
    if (!scenes[0]) return fail(PT_ERR_INVALID, "null scene");
    const Opts o = opts_snapshot();
    // one device is pt_render itself — unless option reduce=rccl asks for the RCCL branch anyway
    // (a one-rank communicator: how a one-GPU machine runs that code, tests/test_gpu_multi.py)
    if (n == 1 && !o.is("reduce", "rccl"))
        return pt_render(scenes[0], meta, frame0, nframes, frame_stride, max_depth, mode, accum, counters);
    FrameParams fp{};
    int rc = make_params(meta, max_depth, fp);
    if (rc != PT_OK) return rc;
    if ((uint64_t)frame0 + (uint64_t)(nframes ? nframes - 1 : 0) * frame_stride >= (1ull << 24))
        return fail(PT_ERR_INVALID, "frame index >= 2^24 (t_k = u32(f32(k)) would round)");
    const size_t count = (size_t)fp.width * fp.height * 3;
    bool distinct = true;
    for (int g = 0; g < n; ++g)
        for (int h = 0; h < g; ++h) distinct &= scenes[g]->device != scenes[h]->device;
    const bool want_rccl = !o.is("reduce", "ordered");
    if (o.is("reduce", "rccl") && (!distinct || !rccl_api().ok))
        return fail(PT_ERR_INVALID, "option reduce=rccl needs distinct devices and librccl.so.1");
    const bool use_rccl = want_rccl && distinct && rccl_api().ok;
    for (int g = 0; g < n; ++g) {  // accumulators: scenes[0]'s from accum, the others zero
        pt_scene* s = scenes[g];
        HIP_TRY(hipSetDevice(s->device));
        if ((rc = ensure_accum(s, count)) != PT_OK || (rc = blocking_stream(s)) != PT_OK) return rc;
        if (g == 0) HIP_TRY(hipMemcpyAsync(s->d_accum, accum, count * sizeof(float), hipMemcpyHostToDevice, s->stream));
        else HIP_TRY(hipMemsetAsync(s->d_accum, 0, count * sizeof(float), s->stream));
        if (counters) HIP_TRY(hipMemsetAsync(s->d_counters, 0, sizeof(Counters), s->stream));
    }
    // frames i = g, g + n, ... on scene g, each device on a host thread of its own (the wavefront's
    // host loop waits on its device; one thread would serialise the devices)
    std::vector<int> rcs(n, PT_OK);
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (int g = 0; g < n; ++g)
        th.emplace_back([&, g]() {
            pt_scene* s = scenes[g];
            const uint32_t cnt = nframes > (uint32_t)g ? (nframes - (uint32_t)g + (uint32_t)n - 1) / (uint32_t)n : 0u;
            int r = hipSetDevice(s->device) == hipSuccess ? PT_OK : fail(PT_ERR_HIP, "hipSetDevice");
            if (r == PT_OK)
                r = render_impl(s, meta, frame0 + (uint32_t)g * frame_stride, cnt, (uint32_t)n * frame_stride, max_depth,
                                mode, true, s->d_accum, counters ? s->d_counters : nullptr, s->stream);
            if (r == PT_OK && hipStreamSynchronize(s->stream) != hipSuccess) r = fail(PT_ERR_HIP, "render stream");
            if (r == PT_OK) r = check_watchdog(s);
            rcs[g] = r;
            if (r != PT_OK) errs[g] = pt_last_error();
        });
    for (auto& t : th) t.join();
    for (int g = 0; g < n; ++g)
        if (rcs[g] != PT_OK) return fail(rcs[g], "device " + std::to_string(scenes[g]->device) + ": " + errs[g]);
    rc = use_rccl ? rccl_reduce(scenes, n, count) : ordered_reduce(scenes, n, count);
    if (rc != PT_OK) return rc;
    pt_scene* s0 = scenes[0];
    HIP_TRY(hipSetDevice(s0->device));
    HIP_TRY(hipMemcpyAsync(accum, s0->d_accum, count * sizeof(float), hipMemcpyDeviceToHost, s0->stream));
    HIP_TRY(hipStreamSynchronize(s0->stream));
    if (counters) {
        pt_counters sum{};
        for (int g = 0; g < n; ++g) {
            pt_counters c{};
            HIP_TRY(hipSetDevice(scenes[g]->device));
            HIP_TRY(hipMemcpy(&c, scenes[g]->d_counters, sizeof c, hipMemcpyDeviceToHost));
            sum.samples += c.samples; sum.ext_queries += c.ext_queries; sum.shadow_queries += c.shadow_queries;
            sum.nodes += c.nodes; sum.tri_tests += c.tri_tests; sum.box_tests += c.box_tests;
        }
        *counters = sum;
    }
    return PT_OK;
}

extern "C" int pt_release_communicators(void) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_comms.empty()) return PT_OK;
    return destroy_comms_locked();
}
