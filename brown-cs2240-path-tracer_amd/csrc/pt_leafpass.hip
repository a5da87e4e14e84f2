// pt_leafpass.hip — big leaves resolved before the traversal (k_wf_leafpass).
//
// The reference tree of MedievalBoat (configs[3]) holds a leaf of 7,327 entries that 54 % of the
// render's ray queries visit (scripts/leaf_visit_stats.c, profiles/r05_leaf_visits.txt); tested
// inside the traversal kernel — by cooperative turns and shared chunk walks — it was ~89 % of the
// render, a chain of L2 round trips at 4 waves per SIMD (verdict r04).  A leaf's outcome does not
// need the traversal: the reference's strict-< loop over the leaf's entries in order leaves the
// query with the first entry of the smallest t among the entries that report a hit, whenever that
// t beats the closest t so far (intersection-logic.wgsl:47-176, ray-triangle-intersection.wgsl
// :1-42).  So before each traversal launch this kernel computes, for every big leaf b and every
// queue entry whose ray enters all the child boxes on b's path from the root (a necessary
// condition of any visit: the same f32 slab test as the traversal, ray-bbox-intersection.wgsl),
// that smallest (t, position) over ALL of b's entries as a key (f32 bits of t << 32 | position),
// and k_wf_trace's lanes apply it in their leaf turns (pt_device.h pre_apply).  Leaf-major and lane = ray: the
// wave tests entry k of the leaf for 64 rays at once, the record uniform (one LDS address), with the
// test's early out when no lane passes the determinant and u tests (bf_closest's phase 1) — full
// lanes, no divergence, no per-lane memory traffic in the loop.  The rays that pass a leaf's
// filter are gathered per wave and leaf in an LDS ring until 64 are waiting.
#include "pt_kernels.h"

#include <map>
#include <mutex>

namespace pt {
namespace {

constexpr uint32_t kLeafPassBlock = 256;  // 4 waves
constexpr uint32_t kLeafRing = 128;       // per wave and leaf: entries passed the filter, not resolved yet

__device__ __forceinline__ uint32_t lp_rank_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// uniform loads through the scalar cache (constant address space: s_load, no VGPRs)
typedef const __attribute__((address_space(4))) float* cfloat_p;
typedef const __attribute__((address_space(4))) int32_t* cint_p;

// ray r enters child `side` of node `node` (step = node << 1 | side): the traversal's test of that box
__device__ __forceinline__ bool enters(const SceneView& sc, int step, const Ray& r) {
    const cfloat_p f = (cfloat_p)(sc.nodes + (step >> 1)) + 6 * (step & 1);
    return 0.0f < ray_box(r, f[0], f[1], f[2], f[3], f[4], f[5]);
}

// The leaf (records rec0 .. rec0 + n - 1) for up to 64 rays: each ray ends with the smallest
// (t, position) over the leaf's entries that report a hit, as a key (f32 bits of t << 32 | position;
// t > 1e-8, so the bits order as t; ~0: none), in every lane that holds it.
// Lanes: 2^lg rays (ray = lane & (2^lg - 1); rvalid: this lane's ray exists) times S = 64 >> lg
// segments (seg = lane >> lg): a lane tests entries seg, seg + S, ... of each block, in order, taking a
// hit when strictly closer than its best (or its first), so its best is the first of its smallest t;
// the S lanes of a ray then take the minimum key — the first entry of the leaf's smallest t.  A full
// batch is one ray per lane (S = 1); a few rays — the last depths, a queue too short to fill the
// chip — spread each ray over S lanes, so a wave walks the leaf in n / S steps.
// Arithmetic: tri_hit's, operation for operation (the same pt_math.h cross/dot, the det test, u and
// v as four compares with NaN passing, t > 1e-8), cut after u when no lane can hit.
// The records pass through the wave's LDS in blocks of kRecBlock (lrec: 3 float4 each, the Tri
// layout): the wave loads block j + 1 into registers (one coalesced float4 load per lane) while it
// tests block j, each record read from LDS at one address for its lanes.  (Scalar loads of each
// record were one L2 round trip per few entries: 18 % of the VALU bound, profiles/r05b_ab_leafpre.log.)
// Measured and not kept (profiles/r05g_ab_leafpass.log, r05h_ab_leafpass.log, same bits): two
// entries per step with their records read ahead and the skip vote taken before the reciprocal
// (-2 %); the test without the vote, branch-free (-21 %: the vote skips v and t for about half the
// entries); a walk of the leaf's chunks that skips the chunks no lane's ray can hit (option
// leaf_cull, -35 %, profiles/r05e_ab_leafpre.log: a wave's 64 rays keep nearly every chunk open).
constexpr int kRecBlock = 16;  // records per LDS block: 48 float4, 768 B per wave
template <bool FAST_RCP>
__device__ __forceinline__ uint64_t resolve_leaf(const SceneView& sc, int rec0, int n, const f3 o, const f3 d, bool rvalid,
                                                 int lg, float4* lrec) {
    const float eps = 1e-8f;
    const uint32_t lane = threadIdx.x & 63u;
    const int S = 64 >> lg, seg = (int)(lane >> lg);
    const float4* __restrict__ g = reinterpret_cast<const float4*>(sc.tris + rec0);
    const int nf4 = 3 * n;
    // (loads under ifs: `c ? g[i] : zero` became a load through a select of pointers, the zero in scratch)
    float4 p0 = make_float4(0, 0, 0, 0);
    if (lane < 3u * kRecBlock && (int)lane < nf4) p0 = g[lane];
    float bt = 0.0f;
    int bk = 0x7fffffff;  // none
    for (int k0 = 0; k0 < n; k0 += kRecBlock) {
        wave_lds_sync();  // every lane is done reading the previous block
        if (lane < 3u * kRecBlock) lrec[lane] = p0;
        wave_lds_sync();
        const int nb = 3 * (k0 + kRecBlock);  // the next block, in flight while this one is tested
        if (lane < 3u * kRecBlock && nb + (int)lane < nf4) p0 = g[nb + lane];
        const int m = min(kRecBlock, n - k0);
        for (int j = 0; j < m; j += S) {  // uniform
            const int e = j + seg;        // this lane's entry of the block
            const bool live = rvalid & (e < m);
            const int ee = min(e, m - 1);
            const float4 a = lrec[3 * ee], b = lrec[3 * ee + 1];
            const float c = lrec[3 * ee + 2].x;
            const f3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, c);
            const f3 rce2 = cross(d, e2);
            const float det = dot(e1, rce2);
            const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
            const f3 sv = o - v0;
            const float u = inv_det * dot(sv, rce2);
            const bool ok_det = !(det > -eps && det < eps), ok_lo = !(u < 0.0f), ok_hi = !(u > 1.0f);
            if ((__builtin_amdgcn_ballot_w64(live) & __builtin_amdgcn_ballot_w64(ok_det) &
                 __builtin_amdgcn_ballot_w64(ok_lo) & __builtin_amdgcn_ballot_w64(ok_hi)) == 0)
                continue;  // wave-uniform: no lane can report a hit
            const f3 sce1 = cross(sv, e1);
            const float v = inv_det * dot(d, sce1);
            const float t = inv_det * dot(e2, sce1);
            const bool hit = live & ok_det & ok_lo & ok_hi & !(v < 0.0f) & !(u + v > 1.0f) & (t > eps);
            const bool take = hit & ((t < bt) | (bk == 0x7fffffff));
            bt = take ? t : bt;
            bk = take ? k0 + e : bk;
        }
    }
    uint64_t key = bk == 0x7fffffff ? ~0ull : ((uint64_t)__builtin_bit_cast(uint32_t, bt) << 32) | (uint32_t)bk;
    for (int off = 1 << lg; off < 64; off <<= 1) {  // uniform: the minimum over the ray's S lanes
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)key, off, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), off, 64);
        const uint64_t other = ((uint64_t)hi << 32) | lo;
        key = other < key ? other : key;
    }
    return key;
}

// The same key for 64 rays (one per lane) of a leaf with chunks (the pass's own: SceneView::pnodes,
// ptris, chunks c0 .. c1 of PreLeaf; pt_leafbvh.cpp), testing only the entries each ray can hit.  Chunk c's node — wave-uniform, in SGPRs
// through the scalar cache, the next one in flight — is checked by every lane against its ray
// and its best so far (pass_chunk_skip: chunk_skip's rule, pt_device.h — no entry of a skipped chunk
// can report a hit at t <= the bound).  The (ray, chunk) pairs that stay open are queued in LDS (chunk << 6 | the ray's lane)
// and every 64 of them a pass tests one pair per lane — the chunk's <= 16 records (ptris, copies in
// chunk order holding the entry's position in the leaf) against the pair's ray (from its lane,
// ds_bpermute) — and lowers the ray's LDS key (f32 bits of t << 32 | position) with ds_min_u64.
// REFINE: a chunk stays open for a ray mostly because its normal cone admits a direction
// perpendicular to the ray (a grazing ray: the rounding bound is infinite) — 171 of the ~174 chunks a
// boat ray opens (scripts/leafbvh_harness.cpp) — although its actual entries' |cos(d, n)| is
// rarely that small.  So open pairs queue first for a second check, one pair per lane, with cf =
// min over the chunk's entries of |d . n_i| (SceneView::pnorm, less the same 1e-5 slack) in place of
// the cone's bound and the pair's ray's current best as the bound (pass_box_skip): the harness
// keeps 4.8 chunks open per ray.  Only the pairs that survive it are tested.
// chunk_leaf_multi's argument (round 4): every entry able to report a hit at t <= its ray's bound at
// check time is tested (cf <= |cos(d, n_i)| for each entry is all the rule needs, whether from the
// cone or from the entries), and the bound (the ray's best so far, +inf first) never drops below the
// leaf's final answer, so each ray ends with the smallest (t, position) over the leaf's hitting
// entries — the key resolve_leaf computes.  Round 4 walked the chunks inside the traversal kernel at
// 4 waves per SIMD, a chain of L2 round trips; here the checks need no memory and the passes have
// the kernel's other waves.
struct PairLds {
    uint32_t* pq;      // [2][kLeafRing]: queued pairs (chunk << 6 | ray lane): to check again, to test
    uint64_t* keys;    // [64]: the rays' keys
};

// The pass's chunk check: chunk_skip's rule (pt_device.h; pt_layout.h LNode) in fewer
// instructions, on the pass's own chunks, whose A and B are stored times 1.00001 rounded up
// (pt_capi.hip), so delta = (A' + B' |o|) / cf + 1e-5 |o| + C takes one FMA beside the reciprocal.
// The grown box is taken in t: on axis x its planes at fma(lo, inv, -o inv) and fma(hi, inv, -o inv),
// moved out by delta |inv| — in exact arithmetic the interval ((lo - delta) - o) inv .. ((hi + delta)
// - o) inv that chunk_skip rounds differently, with roundings of the same size (a few ulps of (|lo| +
// |o| + delta) |inv|), which the rule's 1e-5 |o| + C slack covers ~80 times.  A coordinate of d that
// is 0 (inv infinite) yields NaN or infinite bounds on that axis that only widen the interval (tn
// never +inf, tf never -inf): never a skip the rule would not make.
struct PassRay {
    f3 inv, oi;  // 1 / d (rcp3, as everywhere), o * inv
    float on;    // |o|
};
__device__ __forceinline__ PassRay pass_ray(const f3 o, const f3 d) {
    PassRay r;
    r.inv = rcp3(d);
    r.oi = mk(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    r.on = sqrtf(dot(o, o));
    return r;
}
// the rule for a lower bound cf of |cos(d, n)| over the chunk's entries (a, b, e: the node's first,
// second and fourth float4; Bp: its B')
__device__ __forceinline__ bool pass_box_skip(const float4 a, const float4 b, const float4 e, float Bp, const PassRay& r,
                                              float bound, float cf) {
    const float dl = fmaf(Bp, r.on, e.x) * __builtin_amdgcn_rcpf(cf) + fmaf(1e-5f, r.on, e.y);
    const bool bounded = (cf > 1e-4f) & (dl < 1e30f);
    const float px = fmaf(a.x, r.inv.x, -r.oi.x), qx = fmaf(b.x, r.inv.x, -r.oi.x);
    const float py = fmaf(a.y, r.inv.y, -r.oi.y), qy = fmaf(b.y, r.inv.y, -r.oi.y);
    const float pz = fmaf(a.z, r.inv.z, -r.oi.z), qz = fmaf(b.z, r.inv.z, -r.oi.z);
    const float tn = fmaxf(fmaxf(fmaf(-dl, fabsf(r.inv.x), fminf(px, qx)), fmaf(-dl, fabsf(r.inv.y), fminf(py, qy))),
                           fmaf(-dl, fabsf(r.inv.z), fminf(pz, qz)));
    const float tf = fminf(fminf(fmaf(dl, fabsf(r.inv.x), fmaxf(px, qx)), fmaf(dl, fabsf(r.inv.y), fmaxf(py, qy))),
                           fmaf(dl, fabsf(r.inv.z), fmaxf(pz, qz)));
    return bounded & ((tf < tn) | (tf < 0.0f) | (tn > bound));
}
// the first check: cf from the chunk's normal cone (c: the node's third float4), as chunk_skip
__device__ __forceinline__ bool pass_chunk_skip(const float4 a, const float4 b, const float4 c, const float4 e, const f3 d,
                                                float idl, const PassRay& r, float bound) {
    const float cb = fabsf(fmaf(d.z, c.x, fmaf(d.y, b.w, d.x * a.w))) * idl;
    const float sb = __builtin_amdgcn_sqrtf(fmaxf(0.0f, fmaf(-cb, cb, 1.0f)));
    const float cf = fmaf(cb, c.y, -fmaf(sb, c.z, 1e-5f));
    return pass_box_skip(a, b, e, c.w, r, bound, cf);
}
template <bool FAST_RCP>
__device__ __forceinline__ uint64_t resolve_leaf_pairs(const SceneView& sc, int c0, int c1, const f3 o, const f3 d,
                                                       bool rvalid, const PairLds& L, bool refine) {
    const float eps = 1e-8f;
    const uint32_t lane = threadIdx.x & 63u;
    L.keys[lane] = ~0ull;
    wave_lds_sync();
    const PassRay r = pass_ray(o, d);
    const float idl = 1.0f / sqrtf(dot(d, d));
    float bound = __builtin_inff();
    uint32_t* qa = L.pq;               // pairs to check again (refine)
    uint32_t* qb = L.pq + kLeafRing;   // pairs to test
    uint32_t ha = 0, ta = 0, hb = 0, tb = 0;  // pushed / taken (wave-uniform)
    const float4* __restrict__ lt = reinterpret_cast<const float4*>(sc.ptris);
    const float4* __restrict__ ln4 = reinterpret_cast<const float4*>(sc.pnodes);
    auto bp = [](float v, uint32_t ro) {
        return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute((int)(ro << 2), __builtin_bit_cast(int, v)));
    };
    // one pass: lane l tests queued pair tb + l (l < avail)
    auto pass = [&](uint32_t avail) {
        wave_lds_sync();
        const bool has = lane < avail;
        const uint32_t item = has ? qb[(tb + lane) & (kLeafRing - 1)] : 0u;
        const uint32_t ro = item & 63u;
        int info = 0;
        if (has) info = reinterpret_cast<const int*>(ln4 + 4 * (size_t)(item >> 6) + 3)[3];  // LNode::info
        const int first = info & 0xffffff, cnt = info >> 24;
        const f3 qo = mk(bp(o.x, ro), bp(o.y, ro), bp(o.z, ro));  // the pair's ray, from its lane
        const f3 qd = mk(bp(d.x, ro), bp(d.y, ro), bp(d.z, ro));
        float bt = 0.0f;
        int bk = 0x7fffffff;
#pragma unroll 2
        for (int e = 0; e < kPassChunkMax; ++e) {
            if (e < cnt) {
                const float4* rp = lt + 3 * (size_t)(first + e);
                const float4 a = rp[0], b = rp[1], c = rp[2];
                const f3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, c.x);
                const f3 rce2 = cross(qd, e2);
                const float det = dot(e1, rce2);
                const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
                const f3 sv = qo - v0;
                const float u = inv_det * dot(sv, rce2);
                const f3 sce1 = cross(sv, e1);
                const float v = inv_det * dot(qd, sce1);
                const float t = inv_det * dot(e2, sce1);
                const int k = __builtin_bit_cast(int, c.w);  // Tri::lbvh of a ptris copy: the position in the leaf
                const bool hit = !(det > -eps && det < eps) & !(u < 0.0f) & !(u > 1.0f) & !(v < 0.0f) &
                                 !(u + v > 1.0f) & (t > eps);
                if (hit & ((bk == 0x7fffffff) | (t < bt) | ((t == bt) & (k < bk)))) { bt = t; bk = k; }
            }
        }
        if (bk != 0x7fffffff)  // t > 1e-8: its f32 bits order as t does
            atomicMin(reinterpret_cast<unsigned long long*>(L.keys + ro),
                      ((unsigned long long)__builtin_bit_cast(uint32_t, bt) << 32) | (uint32_t)bk);
        wave_lds_sync();
        const uint64_t mkey = L.keys[lane];  // this lane's ray: checks against its best so far
        if (mkey != ~0ull) bound = __builtin_bit_cast(float, (uint32_t)(mkey >> 32));
        tb += avail;
    };
    // one second check: lane l takes queued pair ta + l (l < avail) and keeps it for a pass only if
    // the chunk's entries' own normals leave it open
    auto check = [&](uint32_t avail) {
        wave_lds_sync();
        const bool has = lane < avail;
        const uint32_t item = has ? qa[(ta + lane) & (kLeafRing - 1)] : 0u;
        const uint32_t ro = item & 63u;
        const size_t c = item >> 6;
        // the pair's ray, from its lane: its direction and the check's terms (no reciprocals here)
        const f3 qd = mk(bp(d.x, ro), bp(d.y, ro), bp(d.z, ro));
        PassRay q;
        q.inv = mk(bp(r.inv.x, ro), bp(r.inv.y, ro), bp(r.inv.z, ro));
        q.oi = mk(bp(r.oi.x, ro), bp(r.oi.y, ro), bp(r.oi.z, ro));
        q.on = bp(r.on, ro);
        const float qidl = bp(idl, ro);
        float4 na = make_float4(0, 0, 0, 0), nb = na, nc = na, ne = na;
        if (has) { na = ln4[4 * c]; nb = ln4[4 * c + 1]; nc = ln4[4 * c + 2]; ne = ln4[4 * c + 3]; }
        const int info = __builtin_bit_cast(int, ne.w);
        const int first = info & 0xffffff, cnt = info >> 24;
        float cmin = 1.0f;
#pragma unroll 2
        for (int e = 0; e < kPassChunkMax; ++e) {
            if (e < cnt) {
                const float4 n = sc.pnorm[first + e];
                cmin = fminf(cmin, fabsf(fmaf(qd.z, n.z, fmaf(qd.y, n.y, qd.x * n.x))));
            }
        }
        const uint64_t qk = L.keys[ro];  // the pair's ray's best so far
        const float qbound = qk != ~0ull ? __builtin_bit_cast(float, (uint32_t)(qk >> 32)) : __builtin_inff();
        const bool keep = has && !pass_box_skip(na, nb, ne, nc.w, q, qbound, fmaf(cmin, qidl, -1e-5f));
        const uint64_t m = __builtin_amdgcn_ballot_w64(keep);
        if (keep) qb[(hb + lp_rank_below(m)) & (kLeafRing - 1)] = item;
        hb += (uint32_t)__popcll(m);
        ta += avail;
        if (hb - tb >= 64) pass(64);  // uniform (never more than 127 queued)
    };
    const cfloat_p nf = (cfloat_p)sc.pnodes;  // chunk nodes, 16 floats each, through the scalar cache
    auto node4 = [&](int q) { return make_float4(nf[4 * q], nf[4 * q + 1], nf[4 * q + 2], nf[4 * q + 3]); };
    float4 na = node4(4 * c0), nb = node4(4 * c0 + 1), nc = node4(4 * c0 + 2), ne = node4(4 * c0 + 3);
    for (int c = c0; c < c1; ++c) {
        const float4 a = na, b = nb, cc = nc, e = ne;
        if (c + 1 < c1) {  // the next chunk's node, in flight while this one is checked
            na = node4(4 * c + 4); nb = node4(4 * c + 5); nc = node4(4 * c + 6); ne = node4(4 * c + 7);
        }
        const bool open = rvalid & !pass_chunk_skip(a, b, cc, e, d, idl, r, bound);
        const uint64_t m = __builtin_amdgcn_ballot_w64(open);
        if (!m) continue;  // uniform
        const uint32_t item = ((uint32_t)c << 6) | lane;
        if (refine) {  // uniform
            if (open) qa[(ha + lp_rank_below(m)) & (kLeafRing - 1)] = item;
            ha += (uint32_t)__popcll(m);
            if (ha - ta >= 64) check(64);  // uniform (never more than 127 queued: kLeafRing)
        } else {
            if (open) qb[(hb + lp_rank_below(m)) & (kLeafRing - 1)] = item;
            hb += (uint32_t)__popcll(m);
            if (hb - tb >= 64) pass(64);
        }
    }
    if (ha != ta) check(ha - ta);
    if (hb != tb) pass(hb - tb);
    wave_lds_sync();
    return L.keys[lane];
}

template <bool FAST_RCP>
__global__ __launch_bounds__(kLeafPassBlock) void k_wf_leafpass(SceneView sc, WfBuffers wb, int in_q, int pairs) {
    __shared__ uint32_t ring[kLeafPassBlock / 64][kMaxPre][kLeafRing];
    __shared__ uint32_t pos[kLeafPassBlock / 64][kMaxPre][2];  // per wave and leaf: head, tail (wave-uniform)
    // per wave: a block of leaf records (resolve_leaf) or the pair walk's two pair rings and its rays'
    // keys (resolve_leaf_pairs), one region for both
    constexpr uint32_t kScratch = 2 * kLeafRing * 4 + 64 * 8;  // 1,536 B >= 3 * kRecBlock * 16
    static_assert(kScratch >= 3 * kRecBlock * 16, "the record block fits the pair walk's region");
    __shared__ __attribute__((aligned(16))) char scratch[kLeafPassBlock / 64][kScratch];
    float4* lrec = reinterpret_cast<float4*>(scratch[threadIdx.x / 64u]);
    const PairLds pl_lds{reinterpret_cast<uint32_t*>(scratch[threadIdx.x / 64u]),
                         reinterpret_cast<uint64_t*>(scratch[threadIdx.x / 64u] + 2 * kLeafRing * 4)};
    const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x & 63u;
    // the queue the next traversal launch reads, as k_wf_trace reads it (a trace that gave up: nothing)
    const uint32_t count = wb.ctl[WF_WATCHDOG] ? 0u : wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];
    const int npre = sc.npre;
    if (lane < (uint32_t)kMaxPre * 2) pos[wv][lane >> 1][lane & 1] = 0;
    wave_lds_sync();
    const float4* __restrict__ q = in_q ? wb.shd.ray : wb.ext.ray;
    const uint32_t nwaves = gridDim.x * (kLeafPassBlock / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (kLeafPassBlock / 64) + wv);
    // resolve the 64 (or `avail`) entries waiting in leaf b's ring from position `tail`: 2^lg >= avail
    // rays, each over 64 >> lg lanes
    auto run = [&](int b, uint32_t tail, uint32_t avail) {
        wave_lds_sync();  // the ring's entries were written by other lanes
        const cint_p pl = (cint_p)(sc.pre + b);
        const int rec0 = pl[0];
        // a batch of >= 32 rays of a leaf with chunks takes the pair walk, one ray per lane (its checks
        // cost the same per wave whatever the batch; fewer rays walk the whole leaf spread over lanes)
        // (option leaf_pairs: 0 never; 2 at every batch size: tests)
        const int pmode = pairs & 3;  // option leaf_pairs; bit 2: the second check (option leaf_refine)
        const int c0 = pl[4], c1 = pl[5];  // PreLeaf::c0, c1
        const bool use_pairs = pmode && sc.pnodes && c1 > c0 && (pmode == 2 || avail >= 32);
        const int lg = use_pairs ? 6 : (avail > 1 ? 32 - __builtin_clz(avail - 1) : 0);  // ceil(log2 avail)
        const uint32_t ri = lane & ((1u << lg) - 1u);
        const bool valid = ri < avail;
        const uint32_t i = valid ? ring[wv][b][(tail + ri) & (kLeafRing - 1)] : 0u;
        float4 a = make_float4(0, 0, 0, 0), c = a;
        if (valid) { a = q[2 * (size_t)i]; c = q[2 * (size_t)i + 1]; }
        // the ray arrives here, before resolve_leaf issues its record prefetches: otherwise the
        // compiler's in-order vmcnt wait for the ray sits inside the entry loop and waits for the
        // prefetch of the next record block too, every block
        asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(c.x), "v"(c.y));
        uint64_t key;
        if (use_pairs)  // uniform
            key = resolve_leaf_pairs<FAST_RCP>(sc, c0, c1, mk(a.x, a.y, a.z), mk(a.w, c.x, c.y), valid, pl_lds,
                                               (pairs & 4) != 0);
        else
            key = resolve_leaf<FAST_RCP>(sc, rec0, pl[1], mk(a.x, a.y, a.z), mk(a.w, c.x, c.y), valid, lg, lrec);
        if (lane < avail) wb.pres[(size_t)b * wb.pres_stride + i] = key;
    };
    // windows of wr queue entries per wave: 64, or fewer when the queue cannot give every other wave a
    // window (the last depths): then each wave's rays are few and each is walked by many lanes.  (The
    // bar is half the waves, not all: a batch of 64 rays in the pair walk costs a wave less than
    // fewer rays walking the whole leaf, as long as the batches still fill the chip.)
    uint32_t wr = 64;
    while (wr > 1 && 2 * (uint64_t)count < (uint64_t)nwaves * wr) wr >>= 1;
    const uint32_t nwin = (count + wr - 1) / wr;
    for (uint32_t win = w; win < nwin; win += nwaves) {
        const uint32_t i = win * wr + lane;
        const bool valid = lane < wr && i < count;
        Ray r;
        {
            float4 a = make_float4(0, 0, 0, 1), c = make_float4(0, 0, 0, 0);
            if (valid) { a = q[2 * (size_t)i]; c = q[2 * (size_t)i + 1]; }
            r.o = mk(a.x, a.y, a.z);
            r.d = mk(a.w, c.x, c.y);
            r.inv = rcp3(r.d);  // = unpack_ray's: the traversal's box tests, bit for bit
        }
        for (int b = 0; b < npre; ++b) {
            const cint_p pl = (cint_p)(sc.pre + b);
            const int npath = pl[2];
            bool pass = valid;
            for (int k = 0; k < npath; ++k) {
                if (!__builtin_amdgcn_ballot_w64(pass)) break;  // uniform
                pass = pass && enters(sc, pl[8 + k], r);  // PreLeaf::path
            }
            const uint64_t m = __builtin_amdgcn_ballot_w64(pass);
            if (!m) continue;
            const uint32_t head = __builtin_amdgcn_readfirstlane(pos[wv][b][0]);
            const uint32_t tail = __builtin_amdgcn_readfirstlane(pos[wv][b][1]);
            if (pass) ring[wv][b][(head + lp_rank_below(m)) & (kLeafRing - 1)] = i;
            const uint32_t nh = head + (uint32_t)__popcll(m);
            uint32_t nt = tail;
            if (nh - tail >= 64) {  // uniform: 64 waiting (never more than 127: kLeafRing holds them)
                run(b, tail, 64);
                nt = tail + 64;
            }
            wave_lds_sync();
            if (lane == 0) { pos[wv][b][0] = nh; pos[wv][b][1] = nt; }
            wave_lds_sync();
        }
    }
    for (int b = 0; b < npre; ++b) {  // the last entries of each leaf
        const uint32_t head = __builtin_amdgcn_readfirstlane(pos[wv][b][0]);
        const uint32_t tail = __builtin_amdgcn_readfirstlane(pos[wv][b][1]);
        if (head != tail) run(b, tail, head - tail);
    }
}

// Leaf pass stress (pt_selftest_leaf, mode 16 + (method << 2 | family)): stress rays (pt_device.h
// stress_ray) against the pre-resolvable leaf b (SceneView::pre), resolved once by the reference's
// sequential strict-< loop over all its entries (tri_hit, each lane its own ray) and once by the
// pass's own code — method 0: resolve_leaf with one ray per lane; 1: resolve_leaf with 8 rays per
// wave, each over 8 lanes (the pass's short batches); 2: resolve_leaf_pairs without its second
// check; 3: with it (pass_chunk_skip, then pass_box_skip with the entries' own normals and each
// ray's running best as the bound).  Row i of out: the loop's (position or -1, t bits), the pass's
// key as (position or -1, t bits), 0, 0.
template <bool FAST_RCP>
__global__ __launch_bounds__(kLeafPassBlock) void k_selftest_leafpass(SceneView sc, int b, int mode, uint32_t seed,
                                                                    uint32_t nrays, int32_t* __restrict__ out) {
    constexpr uint32_t kScratch = 2 * kLeafRing * 4 + 64 * 8;
    __shared__ __attribute__((aligned(16))) char scratch[kLeafPassBlock / 64][kScratch];
    const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x & 63u;
    const int family = mode & 3, method = (mode >> 2) & 3;
    const cint_p pl = (cint_p)(sc.pre + b);
    const int rec0 = pl[0], n = pl[1], c0 = pl[4], c1 = pl[5];
    // method 1: 8 rays per wave (lane & 7), each walked by 8 lanes; else one ray per lane
    const int lg = method == 1 ? 3 : 6;
    const uint32_t wave = blockIdx.x * (kLeafPassBlock / 64) + wv;
    const uint32_t i = (wave << lg) + (lane & ((1u << lg) - 1u));
    const bool valid = i < nrays;
    uint32_t st = 0;
    const Ray r = stress_ray(sc, rec0, n, family, seed, i, st);
    float lt = __builtin_inff();
    int lk = 0x7fffffff;
    for (int k = 0; k < n; ++k) {
        float t;
        if (tri_hit<FAST_RCP>(sc.tris, rec0 + k, r, t) && t < lt) { lt = t; lk = k; }
    }
    uint64_t key;
    if (method >= 2) {
        const PairLds L{reinterpret_cast<uint32_t*>(scratch[wv]), reinterpret_cast<uint64_t*>(scratch[wv] + 2 * kLeafRing * 4)};
        key = resolve_leaf_pairs<FAST_RCP>(sc, c0, c1, r.o, r.d, valid, L, method == 3);
    } else {
        key = resolve_leaf<FAST_RCP>(sc, rec0, n, r.o, r.d, valid, lg, reinterpret_cast<float4*>(scratch[wv]));
    }
    if (!valid || (lane >> lg) != 0) return;  // one lane per ray stores
    int32_t* o = out + 6 * (size_t)i;
    o[0] = lk != 0x7fffffff ? lk : -1;
    o[1] = lk != 0x7fffffff ? __builtin_bit_cast(int32_t, lt) : 0;
    o[2] = key != ~0ull ? (int32_t)(uint32_t)key : -1;
    o[3] = key != ~0ull ? (int32_t)(uint32_t)(key >> 32) : 0;
    o[4] = 0;
    o[5] = 0;
}

int leafpass_blocks(const void* kernel) {
    static std::mutex mu;
    static std::map<const void*, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(kernel);
    if (it != cache.end()) return it->second;
    int per_cu = 0, dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kLeafPassBlock, 0);
    const int b = std::max(1, per_cu) * std::max(1, cus);
    cache.emplace(kernel, b);
    return b;
}

}  // namespace

hipError_t launch_selftest_leafpass(const SceneView& sc, int b, int mode, uint32_t seed, uint32_t nrays, int32_t* out,
                                    hipStream_t stream) {
    const uint32_t per_block = (kLeafPassBlock / 64) << (((mode >> 2) & 3) == 1 ? 3 : 6);
    const dim3 grid((nrays + per_block - 1) / per_block);
    if (sc.fast_rcp)
        hipLaunchKernelGGL(k_selftest_leafpass<true>, grid, dim3(kLeafPassBlock), 0, stream, sc, b, mode, seed, nrays, out);
    else
        hipLaunchKernelGGL(k_selftest_leafpass<false>, grid, dim3(kLeafPassBlock), 0, stream, sc, b, mode, seed, nrays, out);
    return hipGetLastError();
}

hipError_t launch_leafpass(const SceneView& sc, const WfBuffers& wb, int in_q, bool fast_rcp, int blocks, int pairs,
                           hipStream_t stream) {
    if (sc.npre <= 0 || !sc.pre || !wb.pres) return hipErrorInvalidValue;
    const void* k = fast_rcp ? (const void*)k_wf_leafpass<true> : (const void*)k_wf_leafpass<false>;
    const int nb = blocks > 0 ? blocks : leafpass_blocks(k);
    if (fast_rcp)
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<true>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q, pairs);
    else
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<false>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q, pairs);
    return hipSuccess;
}

}  // namespace pt
