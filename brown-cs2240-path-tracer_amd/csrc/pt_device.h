// pt_device.h — device-side building blocks shared by the megakernel and the
// wavefront kernels: ray/box and ray/triangle tests, BVH traversal with a
// per-lane LDS stack, light sampling, hemisphere sampling, camera rays.
// Every function cites the WGSL it restates; numerics follow pt_math.h.
#pragma once
#include "pt_layout.h"
#include "pt_math.h"

namespace pt {

constexpr int kStackMax = 32;  // > max traversal stack of any accepted tree (host checks)

// Per-lane traversal stacks in LDS, lane-minor (the 64 entries of a wave at one level are
// contiguous, so a stack access is conflict-free): entry k of a lane at word k * stride.  (Round
// 4 measured 16-bit entries, two layouts, in k_wf_trace: occupancy 6 -> 8 waves per SIMD on
// Glossy and no faster anywhere but the 1k synthetic scene)
struct LStack32 {
    int32_t* p;
    int stride;
    static __device__ __forceinline__ LStack32 make(char* base, int stride) {
        return LStack32{reinterpret_cast<int32_t*>(base) + threadIdx.x, stride};
    }
    __device__ __forceinline__ void put(int k, int v) const { p[k * stride] = v; }
    __device__ __forceinline__ int get(int k) const { return p[k * stride]; }
};

struct Ray {
    f3 o, d, inv;
};

// Diagnostic build only (make EXTRA=-DPT_TRACE_STATS=1 OUT_DIR=...; scripts/trace_stats.py): the lean
// traversal's turns, timed with s_memtime and counted with their participating lanes, per kind
// (TS_*), summed per wave in Counters::ts and flushed into g_trace_stats by k_wf_trace.
#ifndef PT_TRACE_STATS
#define PT_TRACE_STATS 0
#endif
enum { TS_NODE = 0, TS_LEAF, TS_BIG, TS_NONE, TS_POOLRUN, TS_LOOP, TS_BLOCKED, TS_STARVED, TS_COUNT };
struct Counters {
    uint64_t samples, ext_queries, shadow_queries, nodes, tri_tests, box_tests;
#if PT_TRACE_STATS
    uint64_t ts[TS_COUNT][3];  // [kind][cycles, turns, lanes]
#endif
};
#if PT_TRACE_STATS
__device__ __forceinline__ void ts_add(Counters& c, int kind, uint64_t cyc, uint64_t lanes) {
    c.ts[kind][0] += cyc;
    c.ts[kind][1] += 1;
    c.ts[kind][2] += lanes;
}
#endif

// ray-bbox-intersection.wgsl:1-31 (Tavian's slab test; minNum/maxNum NaN handling)
__device__ __forceinline__ float ray_box(const Ray& r, float mnx, float mny, float mnz, float mxx, float mxy, float mxz) {
    float tmin = -3.0e+38f, tmax = 3.0e+38f;
    float t1 = (mnx - r.o.x) * r.inv.x, t2 = (mxx - r.o.x) * r.inv.x;
    tmin = fmaxf(tmin, fminf(t1, t2));
    tmax = fminf(tmax, fmaxf(t1, t2));
    t1 = (mny - r.o.y) * r.inv.y; t2 = (mxy - r.o.y) * r.inv.y;
    tmin = fmaxf(tmin, fminf(t1, t2));
    tmax = fminf(tmax, fmaxf(t1, t2));
    t1 = (mnz - r.o.z) * r.inv.z; t2 = (mxz - r.o.z) * r.inv.z;
    tmin = fmaxf(tmin, fminf(t1, t2));
    tmax = fminf(tmax, fmaxf(t1, t2));
    return (tmax > fmaxf(tmin, 0.0f)) ? (tmin > 0.0f ? tmin : tmax) : -1.0f;
}

// ray-triangle-intersection.wgsl:1-42 restricted to what the traversal needs (t);
// point and normal are rebuilt for the winning record only (hit_data).
__device__ __forceinline__ void test_tri(const Tri* __restrict__ tris, int i, const Ray& r, float& best_t, int& best) {
    const float eps = 1e-8f;
    const float4* tp = reinterpret_cast<const float4*>(tris + i);
    float4 a = tp[0], b = tp[1];
    float c = tris[i].e2z;
    f3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, c);
    f3 rce2 = cross(r.d, e2);
    float det = dot(e1, rce2);
    if (det > -eps && det < eps) return;
    float inv_det = 1.0f / det;
    f3 s = r.o - v0;
    float u = inv_det * dot(s, rce2);
    if (u < 0.0f || u > 1.0f) return;
    f3 sce1 = cross(s, e1);
    float v = inv_det * dot(r.d, sce1);
    if (v < 0.0f || u + v > 1.0f) return;
    float t = inv_det * dot(e2, sce1);
    if (t > eps && (best_t < 0.0f || t < best_t)) { best_t = t; best = i; }
}

// intersection-logic.wgsl:1-215.  The reference keeps -1 markers on a 64-entry
// private stack; popping skips them, so the live entries behave exactly like
// "pop node, push left then right (right on top)".  Here the right child is
// taken directly and the left one parked on this lane's LDS stack
// (stack.get(k), lane-minor: conflict-free).  Same visit order, same
// pruning with the box's exit distance, same strict-< closest hit.
template <bool COUNT, class ST>
__device__ __forceinline__ int trace(const SceneView& sc, const Ray& r, float& t_out, const ST& stack,
                                     Counters& cnt) {
    float best_t = -1.0f;
    int best = -1;
    int node = 0, sp = 0;
    const float4* __restrict__ nodes4 = reinterpret_cast<const float4*>(sc.nodes);
    while (true) {
        const float4* np = nodes4 + 4 * node;
        float4 a = np[0], b = np[1], c = np[2];
        int4 d = reinterpret_cast<const int4*>(np)[3];
        if (COUNT) { cnt.nodes++; cnt.box_tests += 2; }
        float ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
        float rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
        bool li = 0.0f < ld, ri = 0.0f < rd;
        bool lleaf = d.z >= 0, rleaf = d.w >= 0;
        // leaf children are tested at once, left leaf first (intersection-logic.wgsl:47-176);
        // one loop over both ranges keeps lanes with a left-only and a right-only leaf together
        const int na = (li && lleaf) ? d.z : 0, nb = (ri && rleaf) ? d.w : 0;
        for (int k = 0; k < na + nb; ++k) test_tri(sc.tris, k < na ? d.x + k : d.y + (k - na), r, best_t, best);
        if (COUNT) cnt.tri_tests += na + nb;
        bool tl = li && !lleaf && !(best_t > 0.0f && ld > best_t);
        bool tr = ri && !rleaf && !(best_t > 0.0f && rd > best_t);
        if (tl && tr) {
            stack.put(sp, d.x);
            ++sp;
            node = d.y;
        } else if (tl) {
            node = d.x;
        } else if (tr) {
            node = d.y;
        } else {
            if (sp == 0) break;
            --sp;
            node = stack.get(sp);
        }
    }
    t_out = best_t;
    return best;
}

// Same traversal as trace(), flattened for wave64 SIMT.  trace() nests the leaf loop in
// the node loop, so at every node step a wave runs as many triangle iterations as its
// largest leaf pair (measured lane utilisation ~9% on CornellBox).  Here every lane walks
// its own sequence of units — a node step (two child boxes, classify) or ONE triangle test
// of the pending leaf pair — and each iteration the wave runs the unit type that most of
// its lanes are waiting for (wave-uniform choice from two __ballot popcounts); the other
// lanes wait one iteration.  Each lane still executes its units in exactly the reference
// order (left leaf, right leaf, then the push/pop decision with the updated closest t), so
// the result is bit-identical to trace().  `active` = false lanes only vote.
struct TravState {
    int node, sp, k, na, nt, la, lb, lc, rc;
    float ld, rd, best_t;
    int best;
    bool lint, rint, in_leaf, done;
};

__device__ __forceinline__ void trav_init(TravState& s, bool active) {
    s.node = 0; s.sp = 0; s.k = 0; s.na = 0; s.nt = 0; s.la = 0; s.lb = 0; s.lc = 0; s.rc = 0;
    s.ld = 0.0f; s.rd = 0.0f; s.best_t = -1.0f; s.best = -1;
    s.lint = false; s.rint = false; s.in_leaf = false; s.done = !active;
}

// One scheduling step for the whole wave.  Returns false once no lane has work left.
template <bool COUNT, class ST>
__device__ __forceinline__ bool trav_step(const SceneView& sc, const Ray& r, TravState& s, const ST& stack,
                                          Counters& cnt) {
    const uint64_t want_leaf = __ballot(!s.done && s.in_leaf);
    const uint64_t want_node = __ballot(!s.done && !s.in_leaf);
    if ((want_leaf | want_node) == 0) return false;
    const bool leaf_turn = __popcll(want_leaf) >= __popcll(want_node);  // wave-uniform
    bool decide = false;
    if (leaf_turn) {
        if (!s.done && s.in_leaf) {
            const int idx = s.k < s.na ? s.la + s.k : s.lb + (s.k - s.na);
            test_tri(sc.tris, idx, r, s.best_t, s.best);
            if (COUNT) cnt.tri_tests++;
            if (++s.k == s.nt) { s.in_leaf = false; decide = true; }
        }
    } else if (!s.done && !s.in_leaf) {
        const float4* np = reinterpret_cast<const float4*>(sc.nodes) + 4 * s.node;
        float4 a = np[0], b = np[1], c = np[2];
        int4 d = reinterpret_cast<const int4*>(np)[3];
        if (COUNT) { cnt.nodes++; cnt.box_tests += 2; }
        s.ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
        s.rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
        const bool li = 0.0f < s.ld, ri = 0.0f < s.rd;
        const bool lleaf = d.z >= 0, rleaf = d.w >= 0;
        s.na = (li && lleaf) ? d.z : 0;
        s.nt = s.na + ((ri && rleaf) ? d.w : 0);
        s.la = d.x; s.lb = d.y; s.lc = d.x; s.rc = d.y; s.k = 0;
        s.lint = li && !lleaf;
        s.rint = ri && !rleaf;
        if (s.nt > 0) s.in_leaf = true; else decide = true;
    }
    if (decide) {
        const bool tl = s.lint && !(s.best_t > 0.0f && s.ld > s.best_t);
        const bool tr = s.rint && !(s.best_t > 0.0f && s.rd > s.best_t);
        if (tl && tr) {
            stack.put(s.sp, s.lc);
            ++s.sp;
            s.node = s.rc;
        } else if (tl) {
            s.node = s.lc;
        } else if (tr) {
            s.node = s.rc;
        } else if (s.sp == 0) {
            s.done = true;
        } else {
            --s.sp;
            s.node = stack.get(s.sp);
        }
    }
    return true;
}

// Branch-free triangle test with the exact arithmetic of test_tri: every quantity of the
// reference's early-out chain is computed and the chain becomes one predicate (the values
// skipped by an early return never reach `hit`, so the result is identical).
struct TriRec { float4 a, b; float c; };  // (v0, e1.x), (e1.yz, e2.xy), e2.z
__device__ __forceinline__ TriRec load_tri(const Tri* __restrict__ tris, int i) {
    const float4* tp = reinterpret_cast<const float4*>(tris + i);
    return TriRec{tp[0], tp[1], tris[i].e2z};
}

template <bool FAST_RCP = false>
__device__ __forceinline__ bool tri_hit(const TriRec& tr, const Ray& r, float& t_out) {
    const float eps = 1e-8f;
    const float4 a = tr.a, b = tr.b;
    f3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, tr.c);
    f3 rce2 = cross(r.d, e2);
    float det = dot(e1, rce2);
    // FAST_RCP (SceneView::fast_rcp): |det| < 2^126 for this scene, where rcp_rn is the IEEE
    // 1/det bit for bit; below 2^-126 the det test rejects the triangle whatever inv_det is
    float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
    f3 s = r.o - v0;
    float u = inv_det * dot(s, rce2);
    f3 sce1 = cross(s, e1);
    float v = inv_det * dot(r.d, sce1);
    float t = inv_det * dot(e2, sce1);
    t_out = t;
    const bool ok_det = !(det > -eps && det < eps);
    // !(u < 0) & !(v < 0) & !(u > 1) & !(u + v > 1), NaN passing each test as in the early-out
    // chain: minNum/maxNum return the non-NaN operand, so the folded forms are the same
    // predicate in two compares
    const float lo = fminf(u, v), hi = fmaxf(u, u + v);
    const bool ok_uv = !(lo < 0.0f) & !(hi > 1.0f);
    return ok_det & ok_uv & (t > eps);
}
template <bool FAST_RCP = false>
__device__ __forceinline__ bool tri_hit(const Tri* __restrict__ tris, int i, const Ray& r, float& t_out) {
    return tri_hit<FAST_RCP>(load_tri(tris, i), r, t_out);
}

// trav_step with every per-lane branch replaced by selects (the scalar unit is shared by
// the CU's four SIMDs and the exec-mask bookkeeping of divergent branches was ~0.7 SALU
// per VALU instruction).  All lanes run the chosen unit on a valid record; lanes for which
// the unit is not meant keep their state.  The push/pop decision stores unconditionally
// into stack[sp], the free slot just above the lane's stack top, and reads stack[sp-1].
template <bool COUNT, class ST>
__device__ __forceinline__ bool trav_step_pred(const SceneView& sc, const Ray& r, TravState& s, const ST& stack,
                                               Counters& cnt) {
    const bool is_leaf = !s.done && s.in_leaf;
    const bool is_node = !s.done && !s.in_leaf;
    const uint64_t want_leaf = __ballot(is_leaf);
    const uint64_t want_node = __ballot(is_node);
    if ((want_leaf | want_node) == 0) return false;
    bool decide;
    if (__popcll(want_leaf) >= __popcll(want_node)) {  // wave-uniform
        const int idx = s.k < s.na ? s.la + s.k : s.lb + (s.k - s.na);
        float t;
        const bool hit = tri_hit(sc.tris, is_leaf ? idx : 0, r, t);
        const bool take = is_leaf & hit & ((s.best_t < 0.0f) | (t < s.best_t));
        s.best_t = take ? t : s.best_t;
        s.best = take ? idx : s.best;
        if (COUNT) cnt.tri_tests += is_leaf ? 1 : 0;
        s.k += is_leaf ? 1 : 0;
        decide = is_leaf & (s.k == s.nt);
        s.in_leaf = s.in_leaf & !decide;
    } else {
        const float4* np = reinterpret_cast<const float4*>(sc.nodes) + 4 * (is_node ? s.node : 0);
        float4 a = np[0], b = np[1], c = np[2];
        int4 d = reinterpret_cast<const int4*>(np)[3];
        if (COUNT) { cnt.nodes += is_node ? 1 : 0; cnt.box_tests += is_node ? 2 : 0; }
        const float ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
        const float rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
        const bool li = 0.0f < ld, ri = 0.0f < rd;
        const bool lleaf = d.z >= 0, rleaf = d.w >= 0;
        const int na = (li & lleaf) ? d.z : 0;
        const int nt = na + ((ri & rleaf) ? d.w : 0);
        if (is_node) {  // plain moves; the compiler turns these into selects
            s.ld = ld; s.rd = rd; s.na = na; s.nt = nt;
            s.la = d.x; s.lb = d.y; s.lc = d.x; s.rc = d.y; s.k = 0;
            s.lint = li & !lleaf;
            s.rint = ri & !rleaf;
        }
        decide = is_node & (nt == 0);
        s.in_leaf = is_node ? (nt > 0) : s.in_leaf;
    }
    const bool tl = decide & s.lint & !((s.best_t > 0.0f) & (s.ld > s.best_t));
    const bool tr = decide & s.rint & !((s.best_t > 0.0f) & (s.rd > s.best_t));
    const bool push = tl & tr;
    const bool pop = decide & !tl & !tr;
    stack.put(s.sp, s.lc);  // slot above the top: free unless this is a push
    const int top = stack.get(s.sp > 0 ? s.sp - 1 : 0);
    s.node = tr ? s.rc : (tl ? s.lc : (pop ? top : s.node));
    s.done = s.done | (pop & (s.sp == 0));
    s.sp += push ? 1 : ((pop & (s.sp > 0)) ? -1 : 0);
    return true;
}

// trav_step with its per-lane state laid out for the compiler: loop-carried flags live
// in one VGPR bitfield (a bool carried around the loop becomes an SGPR lane mask that
// needs an s_andn2/s_and/s_or merge at every join; a VGPR written under exec needs none),
// the triangle test is branch-free (its three early-outs can only skip work when all 64
// lanes reject at the same step, which practically never happens), each unit is one exec
// region and the push/pop decision is straight-line (stack[sp] is the free slot above the
// top: max_stack = max depth + 1, pt_capi.hip).  Same units, same order, same arithmetic.
enum : int { TF_LINT = 1, TF_RINT = 2, TF_LEAF = 4, TF_DONE = 8, TF_BCUR = 16, TF_PARK = 32 };
struct TravLean {
    int node, sp, k, na, nt, la, lb, fl, best;
    float ld, rd, best_t;
    uint64_t tested, rem;  // mailbox flavours only: uids tested by this query / left in this pair
    uint32_t qi;           // pre-resolved big leaves only: the query's queue entry (SceneView::pres) ...
    uint64_t pkey;         // ... and the key of the first big leaf of its current leaf pair (pre_node_prefetch)
    int last;              // leaf remainders (SceneView::nalt): first record of the last non-empty leaf tested, -1 none
};
__device__ __forceinline__ void trav_init(TravLean& s, bool active) {
    s.node = 0; s.sp = 0; s.k = 0; s.na = 0; s.nt = 0; s.la = 0; s.lb = 0; s.best = -1; s.qi = 0; s.pkey = ~0ull; s.last = -1;
    s.fl = active ? 0 : TF_DONE;
    s.ld = 0.0f; s.rd = 0.0f; s.best_t = -1.0f;
    s.tested = 0; s.rem = 0;
}
__device__ __forceinline__ bool trav_finished(const TravLean& s) { return (s.fl & TF_DONE) != 0; }
__device__ __forceinline__ bool trav_finished(const TravState& s) { return s.done; }

// K = triangle tests per leaf turn: a lane with at least two triangles of its leaf pair left
// runs two in sequence (same order, each against the closest t so far), which halves the
// per-iteration overhead (scheduling ballots, decision, loop control) per test.
// The three pieces of a lean step, for lanes in the matching state.
// the slot of the pre-resolved leaf whose first record is rec0 (SceneView::pre_rec0; slot 0 when none
// matches — callers ask only for leaves of >= big_leaf entries, which are exactly the table's)
__device__ __forceinline__ int pre_slot(const SceneView& sc, int rec0) {
    int b = 0;
#pragma unroll
    for (int j = 1; j < kMaxPre; ++j) b = (j < sc.npre && sc.pre_rec0[j] == rec0) ? j : b;
    return b;
}

// PRE: a node step whose hit leaf children include a pre-resolved big leaf loads that leaf's key
// now (the first such leaf of the pair), so it arrives behind the next steps' own loads instead of
// stalling the wave in its leaf turn (pre_apply)
// Leaf remainders (SceneView::nalt, pt_leafskip.cpp): the descriptor of the remainder of a leaf
// whose ray tested leaf `prev` last (first record << 7 | count), -1 when the leaf has none for it
__device__ __forceinline__ int alt_pick(const int4 p, const int4 q, int prev) {
    int v = -1;
    v = prev == p.x ? p.y : v;
    v = prev == p.z ? p.w : v;
    v = prev == q.x ? q.y : v;
    v = prev == q.z ? q.w : v;
    return v;
}

template <bool COUNT, bool PRE = false>
__device__ __forceinline__ bool lean_node_unit(const SceneView& sc, const Ray& r, TravLean& s, Counters& cnt) {
    const float4* np = reinterpret_cast<const float4*>(sc.nodes) + 4 * s.node;
    float4 a = np[0], b = np[1], c = np[2];
    int4 d = reinterpret_cast<const int4*>(np)[3];
    // leaf remainders: loaded beside the node (the counting build walks the reference's leaves)
    const bool alt = !COUNT && sc.nalt != nullptr;
    int4 al0{}, al1{}, ar0{}, ar1{};  // kLeafAlt 1: al0 = (prevL, remL, prevR, remR); 4: two int4 per side
    if (alt) {
        if constexpr (kLeafAlt == 1) {
            al0 = sc.nalt[s.node];
        } else {
            const int4* ap = sc.nalt + 4 * s.node;
            al0 = ap[0]; al1 = ap[1]; ar0 = ap[2]; ar1 = ap[3];
        }
    }
    if (COUNT) { cnt.nodes++; cnt.box_tests += 2; }
    s.ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
    s.rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
    const bool li = 0.0f < s.ld, ri = 0.0f < s.rd;
    const bool lleaf = d.z >= 0, rleaf = d.w >= 0;
    int lrec = d.x, rrec = d.y, ln = d.z, rn = d.w;
    if (alt) {
        // a leaf child L entered by a ray whose last tested leaf M is one of L's: the remainder
        // "L minus M" instead (exact: pt_leafskip.cpp); the right leaf's M is the left leaf when the
        // left one is tested too.  The leaves keep their identity (first records) for `last`.
        const bool lt = li & lleaf & (d.z > 0), rt = ri & rleaf & (d.w > 0);
        const int pr = lt ? d.x : s.last;
        int dl, dr;
        if constexpr (kLeafAlt == 1) {
            dl = s.last == al0.x ? al0.y : -1;
            dr = pr == al0.z ? al0.w : -1;
        } else {
            dl = alt_pick(al0, al1, s.last);
            dr = alt_pick(ar0, ar1, pr);
        }
        if (lt & (dl >= 0)) { lrec = dl >> 7; ln = dl & 127; }
        if (rt & (dr >= 0)) { rrec = dr >> 7; rn = dr & 127; }
        s.last = rt ? d.y : pr;
    }
    s.na = (li & lleaf) ? ln : 0;
    s.nt = s.na + ((ri & rleaf) ? rn : 0);
    s.la = lrec; s.lb = rrec; s.k = 0;
    s.fl = ((li & !lleaf) ? TF_LINT : 0) | ((ri & !rleaf) ? TF_RINT : 0) | (s.nt > 0 ? TF_LEAF : 0);
    if constexpr (PRE) {
        const bool lbig = s.na >= sc.big_leaf, rbig = s.nt - s.na >= sc.big_leaf;
        if (lbig | rbig) s.pkey = sc.pres[(size_t)pre_slot(sc, lbig ? d.x : d.y) * sc.pres_stride + s.qi];
    }
    return s.nt == 0;  // no leaf to test: decide now
}

// Big leaves (BIG; SceneView::big_leaf): a lane whose next entry starts a leaf of at least
// big_leaf entries parks there (TF_PARK) instead of walking it alone; the wave then tests that
// leaf for that one ray with all 64 lanes (big_turn).  big_at: the lane stands at the start of a
// big left leaf, or at the start of a big right leaf; big_seg: that leaf (first record, entries).
__device__ __forceinline__ bool big_at(const SceneView& sc, const TravLean& s) {
    return (s.k < s.na) ? (s.k == 0 && s.na >= sc.big_leaf) : (s.k == s.na && s.k < s.nt && s.nt - s.na >= sc.big_leaf);
}
__device__ __forceinline__ void big_seg(const TravLean& s, int& rec0, int& n) {
    const bool left = s.k < s.na;
    rec0 = left ? s.la : s.lb;
    n = left ? s.na : s.nt - s.na;
}

template <bool COUNT>
__device__ __forceinline__ bool pre_apply(const SceneView& sc, TravLean& s, Counters& cnt);

template <int K, bool COUNT, bool FAST_RCP, bool BIG = false, bool PRE = false>
__device__ __forceinline__ bool lean_leaf_loop(const SceneView& sc, const Ray& r, TravLean& s, Counters& cnt) {
    if constexpr (PRE) {  // a big leaf at the lane's position: its key (pre_apply)
        if (pre_apply<COUNT>(sc, s, cnt)) { s.fl &= ~TF_LEAF; return true; }
        if (big_at(sc, s)) return false;  // a big right leaf next: its key in the next turn
    } else if constexpr (BIG) {  // park at a big leaf: now, or where this turn would enter it
        if (big_at(sc, s)) { s.fl |= TF_PARK; return false; }
    }
    // a turn of a lane whose right leaf is big stops at that leaf's start (it parks below)
    const int lim = (BIG && s.k < s.na && s.nt - s.na >= sc.big_leaf) ? s.na : s.nt;
    // test j of the turn is entry k0 + j (a lane stops at lim): the position is not counted
    // up per test (v_cndmask + v_add per test and lane), it follows from k0 once the turn ends
    const int k0 = s.k;
    const int bl = s.la + k0, br = s.lb - s.na + k0;  // record of entry k0 + j: (left ? bl : br) + j
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool live = j == 0 || k0 + j < lim;  // the first test always is
        if (j > 0 && !wave_any(live)) break;        // every lane's leaf pair is done
        const int idx = (k0 + j < s.na ? bl : br) + j;
        float t;
        const bool take = tri_hit<FAST_RCP>(sc.tris, live ? idx : s.la, r, t) & live &
                          ((s.best_t < 0.0f) | (t < s.best_t));
        s.best_t = take ? t : s.best_t;
        s.best = take ? idx : s.best;
        if (COUNT) cnt.tri_tests += live ? 1 : 0;
    }
    // tests made: 1, then one per j >= 1 with k0 + j < lim (a break comes only once every
    // lane has k0 + j >= lim, so the count is the same with or without it)
    s.k = max(k0 + 1, min(k0 + K, lim));
    const bool decide = s.k == s.nt;
    s.fl = decide ? (s.fl & ~TF_LEAF) : s.fl;
    if constexpr (BIG && !PRE) s.fl |= (!decide && big_at(sc, s)) ? TF_PARK : 0;
    return decide;
}

template <class ST>
__device__ __forceinline__ void lean_decide(TravLean& s, const ST& stack) {
    const bool tl = (s.fl & TF_LINT) && !((s.best_t > 0.0f) & (s.ld > s.best_t));
    const bool tr = (s.fl & TF_RINT) && !((s.best_t > 0.0f) & (s.rd > s.best_t));
    const bool pop = !tl & !tr;
    stack.put(s.sp, s.la);  // a push keeps it, anything else leaves the slot free
    const int top = stack.get(max(s.sp - 1, 0));
    s.node = tr ? s.lb : (tl ? s.la : top);
    s.fl |= (pop & (s.sp == 0)) ? TF_DONE : 0;
    s.sp += (tl & tr) ? 1 : (pop ? -1 : 0);  // sp < 0 only once done
}

// One cooperative big-leaf turn for the first parked lane f of the wave: the leaf's n entries are
// dealt to the 64 lanes (lane l tests entries l, l + 64, ... against f's ray, read from f's
// registers; the records of one step are 64 consecutive ones, a coalesced load), each lane keeps
// the first of its smallest-t hits, and a wave reduction picks the smallest (t, entry) — the
// first entry in leaf order among the leaf's smallest-t hits, which is what the reference's
// sequential strict-< loop ends with, when that t beats f's closest t so far (strict <, so an
// equal t from an earlier leaf stays).  The ray's walk over the leaf takes n / 64 steps instead of
// n, and the wave's lanes do all of it instead of idling while one lane walks.
template <bool COUNT, bool FAST_RCP, class ST>
__device__ __forceinline__ void big_turn(const SceneView& sc, const Ray& r, TravLean& s, uint64_t parked, const ST& stack,
                                         Counters& cnt) {
    const int f = (int)__builtin_ctzll(parked);
    int my0 = 0, myn = 0;
    big_seg(s, my0, myn);
    const int rec0 = __builtin_amdgcn_readlane(my0, f), n = __builtin_amdgcn_readlane(myn, f);
    auto bc = [&](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), f)); };
    Ray q;
    q.o = mk(bc(r.o.x), bc(r.o.y), bc(r.o.z));
    q.d = mk(bc(r.d.x), bc(r.d.y), bc(r.d.z));
    q.inv = mk(bc(r.inv.x), bc(r.inv.y), bc(r.inv.z));
    const int lane = (int)(threadIdx.x & 63u);
    // the lanes running this turn: all 64 in the wavefront kernels; the megakernel's paths call the
    // traversal with finished lanes switched off, and the entries are dealt over the lanes that run
    const uint64_t act = __ballot(1);
    const int na = __popcll(act), me = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    float bt = 0.0f;
    int bk = 0x7fffffff;  // none
    for (int c = me; c < n; c += na) {
        float t;
        const bool take = tri_hit<FAST_RCP>(sc.tris, rec0 + c, q, t) & ((bk == 0x7fffffff) | (t < bt));
        bt = take ? t : bt;
        bk = take ? c : bk;
    }
    auto better = [](float ot, int ok, float t, int k) {
        return (ok != 0x7fffffff) & ((k == 0x7fffffff) | (ot < t) | ((ot == t) & (ok < k)));
    };
    if (act == ~0ull) {  // butterfly: every lane ends with the wave's smallest (t, entry)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float ot = __shfl_xor(bt, off, 64);
            const int ok = __shfl_xor(bk, off, 64);
            const bool b = better(ot, ok, bt, bk);
            bt = b ? ot : bt;
            bk = b ? ok : bk;
        }
    } else {  // some lanes off (their registers are stale): read the running lanes one by one
        float rt = 0.0f;
        int rk = 0x7fffffff;
        for (uint64_t m = act; m; m &= m - 1) {
            const int l = (int)__builtin_ctzll(m);
            const float ot = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bt), l));
            const int ok = __builtin_amdgcn_readlane(bk, l);
            const bool b = better(ot, ok, rt, rk);
            rt = b ? ot : rt;
            rk = b ? ok : rk;
        }
        bt = rt;
        bk = rk;
    }
    if (lane == f) {
        const bool take = (bk != 0x7fffffff) & ((s.best_t < 0.0f) | (bt < s.best_t));
        s.best_t = take ? bt : s.best_t;
        s.best = take ? rec0 + bk : s.best;
        if (COUNT) cnt.tri_tests += n;
        s.k += n;
        s.fl &= ~TF_PARK;
        if (s.k == s.nt) {
            s.fl &= ~TF_LEAF;
            lean_decide(s, stack);
        } else if (big_at(sc, s)) {
            s.fl |= TF_PARK;  // its right leaf is big too
        }
    }
}

// The per-wave LDS key slots (lean_leaf_pool, chunk_leaf_multi) are written by one lane, lowered by
// other lanes' ds_min_u64 and read back by the first: a wave barrier plus a wavefront-scope fence
// orders those accesses under the memory model too, not only by wave64 lockstep and in-order LDS
// (advisor r04; neither emits an instruction on gfx950).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Cross-lane minima by DPP (gfx9 lane moves inside the VALU: no LDS round trip, unlike the
// ds_bpermute a __shfl_xor becomes).  dpp_mov: lanes the move does not write keep `old`.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_mov(int v, int old) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xF, false);
}
// the wave's smallest (t, k), lexicographic, returned in every lane (t never NaN; `none` is
// (+inf, 0x7fffffff)): quad_perm [1,0,3,2] and [2,3,0,1], the 8-lane and 16-lane mirrors leave each
// row's minimum in all its lanes; row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry it
// to lane 63, which is read back.  A minimum under a total order: any pairing gives the same.
__device__ __forceinline__ void wave_min_tk(float& t, int& k) {
    constexpr int kInfBits = 0x7f800000, kNone = 0x7fffffff;
    auto step = [&](auto mov) {
        const float ot = __builtin_bit_cast(float, mov(__builtin_bit_cast(int, t), kInfBits));
        const int ok = mov(k, kNone);
        const bool b = (ot < t) | ((ot == t) & (ok < k));
        t = b ? ot : t;
        k = b ? ok : k;
    };
    step([](int v, int o) { return dpp_mov<0xB1, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x4E, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x141, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x140, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x142, 0xA>(v, o); });
    step([](int v, int o) { return dpp_mov<0x143, 0xC>(v, o); });
    t = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), 63));
    k = __builtin_amdgcn_readlane(k, 63);
}
// the wave's smallest t (never NaN; +inf for none), in every lane, the same way
__device__ __forceinline__ float wave_min_t(float t) {
    constexpr int kInfBits = 0x7f800000;
    auto step = [&](auto mov) {
        const float ot = __builtin_bit_cast(float, mov(__builtin_bit_cast(int, t), kInfBits));
        t = ot < t ? ot : t;
    };
    step([](int v, int o) { return dpp_mov<0xB1, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x4E, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x141, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x140, 0xF>(v, o); });
    step([](int v, int o) { return dpp_mov<0x142, 0xA>(v, o); });
    step([](int v, int o) { return dpp_mov<0x143, 0xC>(v, o); });
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), 63));
}

// Leaf chunks (SceneView::lnodes; pt_leafbvh.cpp groups a big leaf's entries into chunks of at
// most 8, pt_layout.h LNode states the skip rule).  chunk_skip: no entry of the chunk (its LNode as
// a, b, c, e) can report a hit at t <= bound for ray r (idl = 1 / |d|, on = |o|).  Branch-free: the
// rule's two escapes (a cone admitting no bound, an unbounded delta) are masks, not early returns,
// so every operand of the check is used unconditionally and the node's four loads issue together
// (with the returns the compiler sank the last load into the branch: two memory round trips per
// check); a lane whose escape holds computes the box on meaningless values and is not skipped.
// chunk_box_skip: the same rule for a given lower bound cf of |cos(d, n)| over the chunk's entries
// (B = c.w of the node); chunk_skip takes cf from the chunk's cone.  (The leaf pass has its own
// form of both, pt_leafpass.hip pass_box_skip.)
__device__ __forceinline__ bool chunk_box_skip(const float4 a, const float4 b, const float4 e, float B, const Ray& r,
                                               float on, float bound, float cf) {
    // delta, rounded up by 1e-5 relative against the approximate reciprocal
    const float dl = (e.x + B * on) * __builtin_amdgcn_rcpf(cf) * 1.00001f + 1e-5f * on + e.y;
    const bool bounded = (cf > 1e-4f) & (dl < 1e30f);
    float tn = -3.0e38f, tf = 3.0e38f;
    float t1 = (a.x - dl - r.o.x) * r.inv.x, t2 = (b.x + dl - r.o.x) * r.inv.x;
    tn = fmaxf(tn, fminf(t1, t2));
    tf = fminf(tf, fmaxf(t1, t2));
    t1 = (a.y - dl - r.o.y) * r.inv.y; t2 = (b.y + dl - r.o.y) * r.inv.y;
    tn = fmaxf(tn, fminf(t1, t2));
    tf = fminf(tf, fmaxf(t1, t2));
    t1 = (a.z - dl - r.o.z) * r.inv.z; t2 = (b.z + dl - r.o.z) * r.inv.z;
    tn = fmaxf(tn, fminf(t1, t2));
    tf = fminf(tf, fmaxf(t1, t2));
    return bounded & ((tf < tn) | (tf < 0.0f) | (tn > bound));
}
__device__ __forceinline__ bool chunk_skip(const float4 a, const float4 b, const float4 c, const float4 e, const Ray& r,
                                           float idl, float on, float bound) {
    // |cos(d, n)| >= cos(angle(d, axis) + half-angle) over the chunk's normals, less a slack for
    // this arithmetic's rounding (the reciprocals here are within 1 ulp; the slack is 1e-5)
    const float cb = fabsf(r.d.x * a.w + r.d.y * b.w + r.d.z * c.x) * idl;
    const float sb = __builtin_amdgcn_sqrtf(fmaxf(0.0f, 1.0f - cb * cb));
    const float cf = cb * c.y - sb * c.z - 1e-5f;
    return chunk_box_skip(a, b, e, c.w, r, on, bound, cf);
}

// The leaf whose records start at rec0, for ONE ray q (wave-uniform: every lane holds it), by
// the whole wave: lane l checks chunk l of each block of 64 (chunk_skip against the closest t so
// far — `prior` or the best found in earlier flushes); the open chunks are gathered one per lane
// (ds_permute: the open lanes' chunks go to lanes filled, filled + 1, ... in rank order, the rest
// of the permutation lands above them and is ignored), and once 64 are gathered — or the leaf is
// done — every lane tests its chunk's up to 8 records, contiguous copies in chunk order (ltris),
// so the loads of a lane's tests are independent of each other and of the tests.  Every entry
// that could report a hit at t <= the bound is tested, so the wave's smallest (t, position) —
// returned in every lane — is the sequential strict-< loop's outcome whenever the loop would take
// one (t < prior).  tests / chunks: work counters (selftest only).  The traversal walks with
// chunk_leaf_multi (below: the same argument for several rays at once); this single-ray walk is
// its reference in pt_selftest_leaf, which checks both against the sequential loop.
template <bool FAST_RCP, bool STATS = false>
__device__ __forceinline__ void chunk_leaf(const SceneView& sc, const Ray& q, int rec0, float prior, float& bt_out,
                                           int& bk_out, int* tests = nullptr, int* chunks = nullptr) {
    const int lane = (int)(threadIdx.x & 63u);
    const int c0 = sc.tris[rec0].lbvh - 1, c1 = sc.tris[rec0 + 1].lbvh;
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(sc.lnodes);
    const float idl = 1.0f / sqrtf(dot(q.d, q.d));
    const float on = sqrtf(dot(q.o, q.o));
    float bt = __builtin_inff();
    int bk = 0x7fffffff;  // none
    float bound = prior;
    int mine = 0;    // the gathered chunk of this lane (first slot | count << 24; count 0: none)
    int filled = 0;  // lanes holding a gathered chunk (wave-uniform)
    auto test_gathered = [&]() {
        const int first = mine & 0xffffff, cnt = lane < filled ? (mine >> 24) : 0;
        // the records' loads stay inside the per-entry branch: loading two entries together (or
        // the next while this one is tested) costs the trace kernel 14 VGPRs and a wave per SIMD,
        // measured slower on the boat (profiles/r04g_ab_chunkwalk.log, r04h_ab_chunkwalk.log)
#pragma unroll 2
        for (int e = 0; e < kChunkMax; ++e) {
            if (e < cnt) {
                const Tri* rec = sc.ltris + first + e;
                const int k = rec->lbvh;
                float t;
                const bool hit = tri_hit<FAST_RCP>(load_tri(rec, 0), q, t);
                if (STATS) ++*tests;
                if (hit & ((t < bt) | ((t == bt) & (k < bk)))) { bt = t; bk = k; }
            }
        }
        bound = fminf(prior, wave_min_t(bt));
        filled = 0;
    };
    const int cl = max(c0, c1 - 1);  // a valid chunk for lanes past the end (their check is off)
    // a block's gathered chunks arrive from ds_permute into lanes [plo, phi); they are merged into
    // `mine` only when the next block has opened chunks (or before a test), so the permute's LDS
    // latency hides behind the next block's loads and checks
    int pgot = 0, plo = 0, phi = 0;
    auto merge = [&]() {
        mine = (lane >= plo && lane < phi) ? pgot : mine;
        phi = plo;
    };
    for (int cb = c0; cb < c1; cb += 64) {
        const int c = cb + lane, cn = min(c, cl);
        const float4 a = nodes[4 * cn], b = nodes[4 * cn + 1], cc = nodes[4 * cn + 2], e = nodes[4 * cn + 3];
        const int info = __builtin_bit_cast(int, e.w);
        const bool open = (c < c1) & !chunk_skip(a, b, cc, e, q, idl, on, bound);
        const uint64_t m = __ballot(open);
        const int cnt = (int)__popcll(m);
        if (STATS) *chunks += cnt;
        if (!cnt) continue;
        merge();
        if (filled + cnt > 64) test_gathered();
        const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const int dest = open ? filled + below : (filled + cnt + (lane - below)) & 63;
        pgot = __builtin_amdgcn_ds_permute(dest << 2, info);
        plo = filled;
        phi = filled + cnt;
        filled += cnt;
    }
    merge();
    if (filled) test_gathered();
    wave_min_tk(bt, bk);  // every lane ends with the wave's smallest (t, position)
    bt_out = bt;
    bk_out = bk;
}
// Several rays at one big leaf (the wavefront kernel's chunk walk; verdict r03 item 3 step 3):
// when a turn starts, ~11 lanes of a wave on average are parked at the SAME big leaf of the boat
// (profiles/r04e_park_diag.log) and a turn served them one walk each (chunk_leaf for the first
// parked lane's ray, round 3).  Here up to kMultiRays
// of them (the first parked lane f and the lanes parked at f's leaf) share ONE walk: each block of
// 64 chunks is loaded once and checked against every ray (its o, d, 1/d, |d|, |o| and bound read
// from the owner lane), the open (chunk, ray) pairs are gathered one per lane in ray order, and a
// test pass tests each lane's chunk against its pair's ray (fetched from the owner lane by
// ds_bpermute).  A ray's best (t, position) is kept as one 64-bit key — the f32 bits of t (t > 0,
// so they order as t) above the position — in its LDS slot, lowered with ds_min_u64; its bound
// after each pass is min(prior, that t).  Per ray this is chunk_leaf's argument unchanged: every
// entry able to report a hit at t <= the ray's bound at check time is tested, the bound never
// drops below the leaf's final answer, so each ray ends with the smallest (t, position) over its
// leaf's hitting entries whenever that beats its prior; and each served lane then takes the leaf
// exactly as the single-ray turn did.
constexpr int kMultiRays = 16;
// The walk for the lanes of `same` (wave-uniform, at most kMultiRays lanes; every lane of the wave
// runs), each with its own ray r and closest t so far `prior` (+inf for none), over the leaf whose
// records start at rec0; keys: kMultiRays LDS slots of this wave.  Each lane of `same` ends with
// its (bt, bk): the smallest (t, position) over the leaf's entries able to beat prior (bk =
// 0x7fffffff: none) — what chunk_leaf gives that ray.
template <bool FAST_RCP>
__device__ __forceinline__ void chunk_leaf_multi(const SceneView& sc, const Ray& r, uint64_t same, int rec0, float prior,
                                                 uint64_t* keys, float& bt_out, int& bk_out) {
    constexpr uint64_t kNoKey = ~0ull;
    const int lane = (int)(threadIdx.x & 63u);
    const bool served = ((same >> lane) & 1ull) != 0;
    const int slot = (int)__popcll(same & ((1ull << lane) - 1ull));  // this lane's slot, when served
    if (served) keys[slot] = kNoKey;
    wave_lds_sync();
    // this lane's ray constants, read by the checks from the owner lane
    const float idl = 1.0f / sqrtf(dot(r.d, r.d));
    const float on = sqrtf(dot(r.o, r.o));
    float bnd = prior;  // this lane's ray's bound
    auto rl = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); };
    auto bp = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(l << 2, __builtin_bit_cast(int, v))); };
    const int c0 = sc.tris[rec0].lbvh - 1, c1 = sc.tris[rec0 + 1].lbvh;
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(sc.lnodes);
    int mine = 0;    // the gathered pair of this lane: its chunk (first slot | count << 24) ...
    int mray = 0;    // ... and the lane that owns its ray
    int filled = 0;  // lanes holding a gathered pair (wave-uniform)
    auto test_pairs = [&]() {
        const int first = mine & 0xffffff, cnt_l = lane < filled ? (mine >> 24) : 0;
        Ray q;  // the pair's ray, from its owner lane
        q.o = mk(bp(r.o.x, mray), bp(r.o.y, mray), bp(r.o.z, mray));
        q.d = mk(bp(r.d.x, mray), bp(r.d.y, mray), bp(r.d.z, mray));
        q.inv = mk(bp(r.inv.x, mray), bp(r.inv.y, mray), bp(r.inv.z, mray));
        float bt = __builtin_inff();
        int bk = 0x7fffffff;
#pragma unroll 2
        for (int e = 0; e < kChunkMax; ++e) {
            if (e < cnt_l) {
                const Tri* rec = sc.ltris + first + e;
                const int k = rec->lbvh;
                float t;
                const bool hit = tri_hit<FAST_RCP>(load_tri(rec, 0), q, t);
                if (hit & ((t < bt) | ((t == bt) & (k < bk)))) { bt = t; bk = k; }
            }
        }
        if (bk != 0x7fffffff) {  // t > 1e-8: its f32 bits order as t does
            const int os = (int)__popcll(same & ((1ull << mray) - 1ull));
            atomicMin(reinterpret_cast<unsigned long long*>(keys + os),
                      ((unsigned long long)__builtin_bit_cast(uint32_t, bt) << 32) | (uint32_t)bk);
        }
        filled = 0;
        wave_lds_sync();
        if (served) {  // the next checks against each ray's best so far
            const uint64_t k = keys[slot];
            if (k != kNoKey) bnd = fminf(prior, __builtin_bit_cast(float, (uint32_t)(k >> 32)));
        }
    };
    const int cl = max(c0, c1 - 1);  // a valid chunk for lanes past the end (their check is off)
    int pgot = 0, pray = 0, plo = 0, phi = 0;  // a gathered run, merged later (chunk_leaf)
    auto merge = [&]() {
        const bool in = lane >= plo && lane < phi;
        mine = in ? pgot : mine;
        mray = in ? pray : mray;
        phi = plo;
    };
    for (int cb = c0; cb < c1; cb += 64) {
        const int c = cb + lane, cn = min(c, cl);
        const float4 a = nodes[4 * cn], b = nodes[4 * cn + 1], cc = nodes[4 * cn + 2], e = nodes[4 * cn + 3];
        const int info = __builtin_bit_cast(int, e.w);
        for (uint64_t m = same; m; m &= m - 1) {  // wave-uniform: every ray of the walk
            const int o = (int)__builtin_ctzll(m);
            Ray qr;
            qr.o = mk(rl(r.o.x, o), rl(r.o.y, o), rl(r.o.z, o));
            qr.d = mk(rl(r.d.x, o), rl(r.d.y, o), rl(r.d.z, o));
            qr.inv = mk(rl(r.inv.x, o), rl(r.inv.y, o), rl(r.inv.z, o));
            const bool open = (c < c1) & !chunk_skip(a, b, cc, e, qr, rl(idl, o), rl(on, o), rl(bnd, o));
            const uint64_t mo = __ballot(open);
            const int cnt_o = (int)__popcll(mo);
            if (!cnt_o) continue;
            merge();
            if (filled + cnt_o > 64) test_pairs();
            const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mo, 0u));
            const int dest = open ? filled + below : (filled + cnt_o + (lane - below)) & 63;
            pgot = __builtin_amdgcn_ds_permute(dest << 2, info);
            pray = o;
            plo = filled;
            phi = filled + cnt_o;
            filled += cnt_o;
        }
    }
    merge();
    if (filled) test_pairs();
    wave_lds_sync();
    const uint64_t k = served ? keys[slot] : kNoKey;
    bt_out = __builtin_bit_cast(float, (uint32_t)(k >> 32));
    bk_out = k == kNoKey ? 0x7fffffff : (int)(uint32_t)k;
}
template <bool COUNT, bool FAST_RCP, class ST>
__device__ __forceinline__ void chunk_turn_multi(const SceneView& sc, const Ray& r, TravLean& s, uint64_t parked,
                                                 const ST& stack, Counters& cnt) {
    const int lane = (int)(threadIdx.x & 63u);
    const int f = (int)__builtin_ctzll(parked);
    int my0 = 0, myn = 0;
    big_seg(s, my0, myn);
    const int rec0 = __builtin_amdgcn_readlane(my0, f), n = __builtin_amdgcn_readlane(myn, f);
    // the rays of this walk: parked lanes at f's leaf, the first kMultiRays of them (f included)
    uint64_t same = __ballot((((parked >> lane) & 1ull) != 0) && my0 == rec0);
    while (__popcll(same) > kMultiRays) same &= ~(1ull << (63 - __builtin_clzll(same)));
    float bt;
    int bk;
    chunk_leaf_multi<FAST_RCP>(sc, r, same, rec0, s.best_t < 0.0f ? __builtin_inff() : s.best_t, sc.lkeys, bt, bk);
    if ((same >> lane) & 1ull) {
        const bool take = (bk != 0x7fffffff) & ((s.best_t < 0.0f) | (bt < s.best_t));
        s.best_t = take ? bt : s.best_t;
        s.best = take ? rec0 + bk : s.best;
        if (COUNT) cnt.tri_tests += n;
        s.k += n;
        s.fl &= ~TF_PARK;
        if (s.k == s.nt) {
            s.fl &= ~TF_LEAF;
            lean_decide(s, stack);
        } else if (big_at(sc, s)) {
            s.fl |= TF_PARK;  // its right leaf is big too
        }
    }
}

// Big leaves resolved before the traversal (k_wf_leafpass, pt_leafpass.hip): a lane whose next
// entry starts a big leaf takes that leaf's precomputed key — the smallest (t, position) over ALL
// the leaf's entries that report a hit (~0: none) — and applies it as the reference's strict-<
// loop over the leaf ends: that loop, started at the closest t so far, keeps the first entry of the
// smallest t when that t is below it, and nothing otherwise, so no test of the leaf is needed here
// (the same argument as the cooperative turns; intersection-logic.wgsl:47-176).  Called by the
// lane's leaf turn, before its other entries; the key of the pair's first big leaf was loaded at the
// node step (lean_node_unit), a second one (a big right leaf after a big left one: the lane's next
// leaf turn) is loaded here.  The lane's position moves past the leaf; true when that ends the pair.
template <bool COUNT>
__device__ __forceinline__ bool pre_apply(const SceneView& sc, TravLean& s, Counters& cnt) {
    if (big_at(sc, s)) {
        int rec0 = 0, n = 0;
        big_seg(s, rec0, n);
        const bool first = !(s.na >= sc.big_leaf && s.k >= s.na);
        const uint64_t key = first ? s.pkey : sc.pres[(size_t)pre_slot(sc, rec0) * sc.pres_stride + s.qi];
        const float bt = __builtin_bit_cast(float, (uint32_t)(key >> 32));
        const bool take = (key != ~0ull) & ((s.best_t < 0.0f) | (bt < s.best_t));
        s.best_t = take ? bt : s.best_t;
        s.best = take ? rec0 + (int)(uint32_t)key : s.best;
        if (COUNT) cnt.tri_tests += n;
        s.k += n;
    }
    return s.k == s.nt;
}

// A leaf turn with the pair's remaining entries pooled over the whole wave (the wavefront
// traversal kernel, every lane running).  lean_leaf_loop has each leaf lane test its own pair K
// entries per turn while the lanes in node state — and those whose pair ends sooner — idle: lane
// use ~0.53 on Glossy (PMC; scripts/wave_model.py models the same).  Here every leaf lane's
// remaining entries [k, lim) are cut into runs of RUN positions, the runs of all leaf lanes —
// and the lanes in node state test too — are dealt one per lane (ds_permute, as chunk_leaf
// gathers chunks) and each lane tests its run against the
// run owner's ray (fetched by ds_bpermute), keeping the smallest (t, position); the owner's best
// is a 64-bit key — the f32 bits of t > 0 order as t — lowered with ds_min_u64 in its LDS slot.
// The pair's smallest (t, position) is what the reference's strict-< loop over the entries in
// order ends with among them; it replaces the lane's closest hit only if strictly closer, as that
// loop's first test of it would.  Returns decide for this lane, as lean_leaf_loop does.  Runs of 4
// (in process against lean16, bit-identical, profiles/r04s_ab_pool.log): Glossy +17 %, synthetic
// 1k +10 %, 12.5k +5 %, 100k +9 %, 1M +22 %, the boat +9 %; runs of 8 and 16 in between.  The run
// length RUN is sc.leaf_pool (2 or 4, set per scene by pt_capi.hip; a k_wf_trace template argument): runs of 2 against 4
// (profiles/r04aa_ab_run.log) are +12 % on 100k and +26 % on 1M — trees whose triangles outgrow
// the L2, where shorter runs put more independent triangle loads in flight — and -1 to -1.5 % on
// Glossy and the boat.  RUN is a template argument: a run-time trip count kept only a third of the
// gain (profiles/r04ab_ab_runtime_run.log: 100k +3 %, 1M +12 %; r04ad_ab_runtime_run.log: the
// same with two entries per iteration), and both runs inlined into one kernel cost Glossy 1.5 %
// (r04ac, r04ad: ablib/tmpl), so each run length is its own k_wf_trace instance.
template <int RUN, bool COUNT, bool FAST_RCP, bool BIG, bool PRE = false>
__device__ __forceinline__ bool lean_leaf_pool(const SceneView& sc, const Ray& r, TravLean& s, bool in_leaf, Counters& cnt) {
    constexpr uint64_t kNoKey = ~0ull;
    const int lane = (int)(threadIdx.x & 63u);
    bool pre_done = false;  // PRE: the pair ended with a big leaf's key
    if constexpr (PRE) {  // a big leaf at the lane's position: its key first
        if (in_leaf) {
            pre_done = pre_apply<COUNT>(sc, s, cnt);
            in_leaf = !pre_done && !big_at(sc, s);  // a big right leaf next: its key in the next turn
        }
    } else if constexpr (BIG) {  // park at a big leaf: now (no tests this turn)
        if (in_leaf && big_at(sc, s)) { s.fl |= TF_PARK; in_leaf = false; }
    }
    // a turn of a lane whose right leaf is big stops at that leaf's start (it parks below)
    const int lim = (BIG && s.k < s.na && s.nt - s.na >= sc.big_leaf) ? s.na : s.nt;
    const int n = in_leaf ? lim - s.k : 0;
    static_assert(RUN == 2 || RUN == 4, "pooled runs of 2 or 4 entries");
    const int runs = (n + RUN - 1) / RUN;
    uint64_t* keys = sc.lkeys;
    keys[lane] = kNoKey;
    wave_lds_sync();
    auto bpi = [](int v, int l) { return __builtin_amdgcn_ds_bpermute(l << 2, v); };
    auto bpf = [](float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(l << 2, __builtin_bit_cast(int, v))); };
    int mine = 0;    // this lane's run: owner lane | run index << 6
    int filled = 0;  // lanes holding a run (wave-uniform)
    auto test_runs = [&]() {
        const int o = mine & 63, j = mine >> 6;
        const bool has = lane < filled;
        // the run owner's pair and ray
        const int k0 = bpi(s.k, o), lo = bpi(lim, o), na = bpi(s.na, o), la = bpi(s.la, o), lb = bpi(s.lb, o);
        Ray q;
        q.o = mk(bpf(r.o.x, o), bpf(r.o.y, o), bpf(r.o.z, o));
        q.d = mk(bpf(r.d.x, o), bpf(r.d.y, o), bpf(r.d.z, o));
        const int p0 = k0 + j * RUN, p1 = has ? min(p0 + RUN, lo) : p0;
        float bt = __builtin_inff();
        int bk = 0x7fffffff;
#pragma unroll 2
        for (int e = 0; e < RUN; ++e) {
            const int pos = p0 + e;
            if (pos < p1) {
                const int rec = pos < na ? la + pos : lb + (pos - na);
                float t;
                // positions ascend: the first of equal t; a first hit is taken whatever its t (a t
                // of +inf, reachable only through overflow, is a hit the reference keeps too)
                if (tri_hit<FAST_RCP>(sc.tris, rec, q, t) & ((t < bt) | (bk == 0x7fffffff))) { bt = t; bk = pos; }
            }
        }
        if (bk != 0x7fffffff)
            atomicMin(reinterpret_cast<unsigned long long*>(keys + o),
                      ((unsigned long long)__builtin_bit_cast(uint32_t, bt) << 32) | (uint32_t)bk);
#if PT_TRACE_STATS
        ts_add(cnt, TS_POOLRUN, 0, (uint64_t)filled);  // lanes with a run in this test round
#endif
        filled = 0;
    };
    int pgot = 0, plo = 0, phi = 0;  // a gathered round, merged later (chunk_leaf)
    auto merge = [&]() {
        mine = (lane >= plo && lane < phi) ? pgot : mine;
        phi = plo;
    };
    for (int j = 0;; ++j) {  // round j: every leaf lane with more than j runs contributes its run j
        const bool give = runs > j;
        const uint64_t m = __ballot(give);
        if (!m) break;
        const int c = (int)__popcll(m);
        merge();
        if (filled + c > 64) test_runs();
        const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const int dest = give ? filled + below : (filled + c + (lane - below)) & 63;
        pgot = __builtin_amdgcn_ds_permute(dest << 2, lane | (j << 6));
        plo = filled;
        phi = filled + c;
        filled += c;
    }
    merge();
    if (filled) test_runs();
    wave_lds_sync();
    bool decide = false;
    if (in_leaf) {
        const uint64_t k = keys[lane];
        const float bt = __builtin_bit_cast(float, (uint32_t)(k >> 32));
        const int pos = (int)(uint32_t)k;
        const bool take = (k != kNoKey) & ((s.best_t < 0.0f) | (bt < s.best_t));
        s.best_t = take ? bt : s.best_t;
        s.best = take ? (pos < s.na ? s.la + pos : s.lb + (pos - s.na)) : s.best;
        if (COUNT) cnt.tri_tests += n;
        s.k = lim;
        decide = s.k == s.nt;
        s.fl = decide ? (s.fl & ~TF_LEAF) : s.fl;
        if constexpr (BIG && !PRE) s.fl |= (!decide && big_at(sc, s)) ? TF_PARK : 0;
    }
    if constexpr (PRE) {
        if (pre_done) s.fl &= ~TF_LEAF;
        decide |= pre_done;
    }
    return decide;
}

// Each iteration runs ONE unit type for the whole wave — a leaf turn (up to K triangle tests)
// when leaf lanes >= node_bias * node lanes, else a node turn — keeping each lane's unit order.
// PRUN: the pooled leaf turns' run length (lean_leaf_pool)
// PRE: the big leaves were resolved before the traversal (pre_apply; TRAV 26x / 27x)
template <int K, bool COUNT, bool FAST_RCP, bool BIG = false, bool CHUNKS = false, int PRUN = 4, bool PRE = false,
          class ST>
__device__ __forceinline__ bool trav_step_lean(const SceneView& sc, const Ray& r, TravLean& s, const ST& stack,
                                               Counters& cnt) {
    const int state = s.fl & (TF_LEAF | TF_DONE | ((BIG && !PRE) ? TF_PARK : 0));
    if constexpr (BIG && !PRE) {  // a parked lane's big leaf goes first: the wave tests it for that ray
        const uint64_t parked = __ballot((state & TF_PARK) != 0);
        if (parked) {  // wave-uniform
            int my0 = 0, myn = 0;  // the first parked lane's leaf (the other lanes' fields may not be a leaf's)
            big_seg(s, my0, myn);
            if (CHUNKS && sc.lnodes && __ballot(1) == ~0ull &&
                sc.tris[__builtin_amdgcn_readlane(my0, (int)__builtin_ctzll(parked))].lbvh > 0) {  // its leaf has chunks
                chunk_turn_multi<COUNT, FAST_RCP>(sc, r, s, parked, stack, cnt);  // sc.lkeys: k_wf_trace's BIG instances
            } else
                big_turn<COUNT, FAST_RCP>(sc, r, s, parked, stack, cnt);
#if PT_TRACE_STATS
            ts_add(cnt, TS_BIG, 0, (uint64_t)__popcll(parked));
#endif
            return true;
        }
    }
    const uint64_t want_leaf = __ballot(state == TF_LEAF);
    const uint64_t want_node = __ballot(state == 0);
    if ((want_leaf | want_node) == 0) return false;
    bool decide = false;
#if PT_TRACE_STATS
    const uint64_t ts0 = __builtin_amdgcn_s_memtime();
    const bool leaf_turn = __popcll(want_leaf) >= sc.node_bias * __popcll(want_node);
#endif
    if (__popcll(want_leaf) >= sc.node_bias * __popcll(want_node)) {  // wave-uniform
        if (CHUNKS && sc.leaf_pool && sc.lkeys && __ballot(1) == ~0ull)  // the wavefront kernel: the leaf entries pooled
            decide = lean_leaf_pool<PRUN, COUNT, FAST_RCP, BIG, PRE>(sc, r, s, state == TF_LEAF, cnt);
        else if (state == TF_LEAF)
            decide = lean_leaf_loop<K, COUNT, FAST_RCP, BIG, PRE>(sc, r, s, cnt);
    } else if (state == 0) {
        decide = lean_node_unit<COUNT, PRE>(sc, r, s, cnt);
        // further steps in the same turn for lanes that stay in node state (SceneView::node_steps)
        for (int k = 1; k < sc.node_steps; ++k) {  // uniform
            if (decide) lean_decide(s, stack);
            decide = false;
            const bool node = (s.fl & (TF_LEAF | TF_DONE | ((BIG && !PRE) ? TF_PARK : 0))) == 0;
            if (!wave_any(node)) break;
            if (node) decide = lean_node_unit<COUNT, PRE>(sc, r, s, cnt);
        }
    }
    if (decide) lean_decide(s, stack);
#if PT_TRACE_STATS
    ts_add(cnt, leaf_turn ? TS_LEAF : TS_NODE, __builtin_amdgcn_s_memtime() - ts0,
           (uint64_t)__popcll(leaf_turn ? want_leaf : want_node));
#endif
    return true;
}

// Mailboxed lean step (SceneView::mailbox: at most 64 distinct leaf entries).  A query keeps
// the set of entries (uids) it has tested; a node step takes the union of its hit leaf
// children's uid sets minus that set, and the leaf turns test only those, one uid per test in
// increasing uid order (ctz), against the appended per-uid records.  Exact: (1) an entry
// tested again yields the same t, and after its first test the closest t is <= that t, so
// the strict-< update can never take it again — skipping it changes nothing, the node
// pruning that reads the closest t included; (2) within one leaf pair the reference keeps
// the FIRST of equal-t hits in its leaf order (left entries, then right), so an equal-t hit
// replaces the current best only when the best came from this pair (TF_BCUR) and the new
// entry comes earlier in that order (mb_first: rare, scanned on demand).  tri_tests counts
// the reference's tests (every entry of every hit leaf), so counters match the oracle.
// true when entry uid `a` comes before entry uid `b` in this pair's reference order (left leaf
// entries, then right); b is the current best, taken from this pair, so the scan ends
__device__ __forceinline__ bool mb_first(const SceneView& sc, const TravLean& s, int a, int b) {
    for (int k = 0; k < s.nt; ++k) {
        const int u = sc.tris[k < s.na ? s.la + k : s.lb + (k - s.na)].uid;
        if (u == a || u == b) return u == a;
    }
    return false;
}

template <bool COUNT>
__device__ __forceinline__ bool mb_node_unit(const SceneView& sc, const Ray& r, TravLean& s, Counters& cnt) {
    const float4* np = reinterpret_cast<const float4*>(sc.nodes) + 4 * s.node;
    float4 a = np[0], b = np[1], c = np[2];
    int4 d = reinterpret_cast<const int4*>(np)[3];
    s.ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
    s.rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
    const bool li = 0.0f < s.ld, ri = 0.0f < s.rd;
    const bool lleaf = d.z >= 0, rleaf = d.w >= 0;
    s.na = (li & lleaf) ? d.z : 0;
    s.nt = s.na + ((ri & rleaf) ? d.w : 0);
    if (COUNT) { cnt.nodes++; cnt.box_tests += 2; cnt.tri_tests += s.nt; }
    const bool lm = s.na > 0, rm = s.nt > s.na;
    const uint64_t ml = sc.lmask[lm ? d.x : 0], mr = sc.lmask[rm ? d.y : 0];
    const uint64_t m = (lm ? ml : 0ull) | (rm ? mr : 0ull);
    s.rem = m & ~s.tested;
    s.tested |= m;
    s.la = d.x; s.lb = d.y;
    s.fl = ((li & !lleaf) ? TF_LINT : 0) | ((ri & !rleaf) ? TF_RINT : 0) | (s.rem ? TF_LEAF : 0);  // clears TF_BCUR
    return s.rem == 0;
}

template <int K, bool FAST_RCP>
__device__ __forceinline__ bool mb_leaf_loop(const SceneView& sc, const Ray& r, TravLean& s) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool live = j == 0 || s.rem != 0;  // the first test always is
        if (j > 0 && !wave_any(live)) break;
        const int uid = live ? (int)__builtin_ctzll(s.rem) : 0;
        s.rem &= s.rem - 1;
        const int rec = sc.mb_base + uid;
        float t;
        const bool hit = tri_hit<FAST_RCP>(sc.tris, rec, r, t) & live;
        bool take = hit & ((s.best_t < 0.0f) | (t < s.best_t));
        if (hit & (t == s.best_t) & ((s.fl & TF_BCUR) != 0))
            take = mb_first(sc, s, uid, s.best - sc.mb_base);
        s.best_t = take ? t : s.best_t;
        s.best = take ? rec : s.best;
        s.fl |= take ? TF_BCUR : 0;
    }
    const bool decide = s.rem == 0;
    s.fl = decide ? (s.fl & ~TF_LEAF) : s.fl;
    return decide;
}

template <int K, bool COUNT, bool FAST_RCP, class ST>
__device__ __forceinline__ bool trav_step_mb(const SceneView& sc, const Ray& r, TravLean& s, const ST& stack,
                                             Counters& cnt) {
    const int state = s.fl & (TF_LEAF | TF_DONE);
    const uint64_t want_leaf = __ballot(state == TF_LEAF);
    const uint64_t want_node = __ballot(state == 0);
    if ((want_leaf | want_node) == 0) return false;
    bool decide = false;
    if (__popcll(want_leaf) >= sc.node_bias * __popcll(want_node)) {  // wave-uniform
        if (state == TF_LEAF) decide = mb_leaf_loop<K, FAST_RCP>(sc, r, s);
    } else if (state == 0) {
        decide = mb_node_unit<COUNT>(sc, r, s, cnt);
    }
    if (decide) lean_decide(s, stack);
    return true;
}

// Traversal flavours (LaunchOpts.trav): 0 nested loops (trace), 1 flattened with per-lane
// branches (trav_step), 2 flattened and predicated (trav_step_pred), 3 lean (trav_step_lean),
// 4 lean with two triangle tests per leaf turn, 5 with four, 6 with eight, 7 with sixteen; +10: the lean
// flavours with 1/det from rcp_rn (scenes with SceneView::fast_rcp); +100: mailboxed lean flavours;
// +160: big leaves (cooperative turns / chunk walks); +260: big leaves resolved before the traversal.
template <int TRAV, bool LEAN = (TRAV >= 3)>
struct TravSel { using type = TravState; };
template <int TRAV>
struct TravSel<TRAV, true> { using type = TravLean; };

// CHUNKS: big leaves with leaf chunks take chunk_turn_multi (the wavefront traversal kernel; the
// megakernel keeps the cooperative turn and its registers)
template <int TRAV, bool COUNT, bool CHUNKS = false, int PRUN = 4, class ST>
__device__ __forceinline__ bool trav_advance(const SceneView& sc, const Ray& r, typename TravSel<TRAV>::type& s,
                                             const ST& stack, Counters& cnt) {
    if constexpr (TRAV >= 100 && TRAV < 160) {  // mailboxed lean<K> (SceneView::mailbox scenes); + 10: fast reciprocal
        constexpr int K = 1 << (TRAV % 10 - 3);
        return trav_step_mb<K, COUNT, ((TRAV / 10) & 1) != 0>(sc, r, s, stack, cnt);
    }
    else if constexpr (TRAV >= 3) {  // TRAV + 10: fast reciprocal; + 160: big-leaf cooperation; + 260: pre-resolved
        constexpr int B = TRAV % 10;
        constexpr int K = 1 << (B - 3);  // lean, lean2, lean4, lean8, lean16, lean32
        return trav_step_lean<K, COUNT, ((TRAV / 10) & 1) != 0, TRAV >= 160, CHUNKS, PRUN, (TRAV >= 260)>(sc, r, s, stack,
                                                                                                           cnt);
    }
    else if constexpr (TRAV == 1) return trav_step<COUNT>(sc, r, s, stack, cnt);
    else return trav_step_pred<COUNT>(sc, r, s, stack, cnt);
}

template <int TRAV, bool COUNT, class ST>
__device__ __forceinline__ int trace_any(const SceneView& sc, const Ray& r, float& t_out, const ST& stack,
                                         Counters& cnt) {
    if (TRAV == 0) return trace<COUNT>(sc, r, t_out, stack, cnt);
    typename TravSel<TRAV>::type s;
    trav_init(s, true);
    while (trav_advance<TRAV, COUNT>(sc, r, s, stack, cnt)) {
    }
    t_out = s.best_t;
    return s.best;
}

struct Hit {
    f3 p, n;
    int mat;
};

// Intersection{point, normal} for the winning record (ray-triangle-intersection.wgsl:30-36)
__device__ __forceinline__ Hit hit_data(const SceneView& sc, const Ray& r, int rec, float t) {
    const TriRec tr = load_tri(sc.tris, rec);
    Hit h;
    h.p = madd(r.o, r.d, t);
    const f3 e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
    h.n = normalize(cross(e1, e2));
    h.mat = sc.tris[rec].mat;
    if (sc.vnormals) {
        const float4 n0 = sc.tnorm[3 * rec];
        if (n0.w != 0.0f) {  // ray-triangle-intersection.wgsl:44-87: the test's u, v, then the blend
            const float4 n1 = sc.tnorm[3 * rec + 1], n2 = sc.tnorm[3 * rec + 2];
            const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z);
            const f3 rce2 = cross(r.d, e2);
            const float inv_det = 1.0f / dot(e1, rce2);
            const f3 s = r.o - v0;
            const float u = inv_det * dot(s, rce2);
            const float v = inv_det * dot(r.d, cross(s, e1));
            const float w = (1.0f - u) - v;
            h.n = normalize(mk(fmaf(v, n2.x, fmaf(u, n1.x, w * n0.x)), fmaf(v, n2.y, fmaf(u, n1.y, w * n0.y)),
                               fmaf(v, n2.z, fmaf(u, n1.z, w * n0.z))));
        }
    }
    return h;
}

struct Mat {
    float Ns, illum;
    f3 Kd, Ks, Ke;
    f3 Kd_pi;     // Kd / kPI (Material::kd_pi*, made by pt_scene_create)
    float phong;  // (Ns + 2) / (2 kPI) (Material::phong)
};
__device__ __forceinline__ Mat load_mat(const SceneView& sc, int id) {
    const float4* mp = reinterpret_cast<const float4*>(sc.mats + id);
    float4 a = mp[0], b = mp[1], c = mp[2], e = mp[3];
    Mat m;
    m.Ns = a.x; m.illum = a.z;
    m.Kd = mk(b.x, b.y, b.z); m.Ks = mk(c.x, c.y, c.z); m.Ke = mk(e.x, e.y, e.z);
    m.Kd_pi = mk(b.w, c.w, e.w); m.phong = a.w;
    return m;
}

// samplers.wgsl:70-80
__device__ __forceinline__ f3 sample_triangle(f3 p0, f3 p1, f3 p2, uint32_t seed) {
    float ux, uy;
    hash2(seed, ux, uy);
    float su0 = sqrtf(ux);
    float bx = 1.0f - su0, by = uy * su0;
    float bz = (1.0f - bx) - by;
    return mk(fmaf(bz, p2.x, fmaf(by, p1.x, bx * p0.x)), fmaf(bz, p2.y, fmaf(by, p1.y, bx * p0.y)),
              fmaf(bz, p2.z, fmaf(by, p1.z, bx * p0.z)));
}

// intersection-logic.wgsl:217-285: uniform emissive triangle, uniform point on it.
// Returns the light direction; the MC weight is sc.inv_ntri.
__device__ __forceinline__ f3 sample_area_lights(const SceneView& sc, f3 x, uint32_t seed) {
    int k = (int)(hash1(seed * 7u + 11u) * sc.f_ntri);
    const float4* lp = reinterpret_cast<const float4*>(sc.lights + k);
    float4 a = lp[0], b = lp[1], c = lp[2];
    f3 pt = sample_triangle(mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(c.x, c.y, c.z), seed * 11u + 17u);
    return normalize(pt - x);
}

// samplers.wgsl:15-46: cosine hemisphere around n (Duff et al. 2017 ONB)
__device__ __forceinline__ f3 sample_hemisphere(f3 N, uint32_t seed, float& pdf) {
    float xi1, xi2;
    hash2(seed * 7u + 11u, xi1, xi2);
    float phi = (2.0f * kPI) * xi1;
    float theta = acos_p(sqrtf(xi2));
    float sp, cp, st, ct;
    sincos_p(phi, sp, cp);
    sincos_p(theta, st, ct);
    float nx = cp * st, ny = sp * st, nz = ct;
    float s = N.z < 0.0f ? -1.0f : 1.0f;
    float a = -1.0f / (s + N.z);
    float b = (N.x * N.y) * a;
    f3 T = mk(fmaf((s * N.x) * N.x, a, 1.0f), s * b, (-s) * N.x);
    f3 B = mk(b, fmaf(N.y * N.y, a, s), -N.y);
    pdf = ct / kPI;
    return mk(fmaf(N.x, nz, fmaf(B.x, ny, T.x * nx)), fmaf(N.y, nz, fmaf(B.y, ny, T.y * nx)),
              fmaf(N.z, nz, fmaf(B.z, ny, T.z * nx)));
}

// ray_with_epsilon, data-structs.wgsl:59-61 (w = 1 / 0 lanes are never read)
__device__ __forceinline__ Ray ray_eps(f3 p, f3 d) {
    Ray r;
    r.o = mk(fmaf(0.001f, d.x, p.x), fmaf(0.001f, d.y, p.y), fmaf(0.001f, d.z, p.z));
    r.d = d;
    r.inv = rcp3(d);
    return r;
}

// program-raymarch.wgsl:50-76: pixel seed chain, jittered pinhole ray, radiance seed.
__device__ __forceinline__ Ray camera_ray(const FrameParams& fp, uint32_t x, uint32_t y, uint32_t t, uint32_t& seed_out) {
    uint32_t index = x + y * fp.width;
    uint32_t ts = index * 16787u + t;
    ts = hash1u(ts);
    ts = hash1u(ts);
    float jx, jy;
    hash2(ts, jx, jy);
    float gx = (float)x + (jx - 0.5f), gy = (float)y + (jy - 0.5f);
    float norm_x = fmaf(gx + 0.5f, fp.inv_w, -0.5f);
    float norm_y = fmaf(((fp.H - 1.0f) - gy) + 0.5f, fp.inv_h, -0.5f);
    float vhw = fp.view_half_h * fp.aspect;
    float vx = vhw * norm_x, vy = fp.view_half_h * norm_y;
    ts = hash1u(ts);
    const float* M = fp.M;
    float pz = -fp.focal;
    float px = fmaf(M[12], 1.0f, fmaf(M[8], pz, fmaf(M[4], vy, M[0] * vx)));
    float py = fmaf(M[13], 1.0f, fmaf(M[9], pz, fmaf(M[5], vy, M[1] * vx)));
    float pzw = fmaf(M[14], 1.0f, fmaf(M[10], pz, fmaf(M[6], vy, M[2] * vx)));
    float pw = fmaf(M[15], 1.0f, fmaf(M[11], pz, fmaf(M[7], vy, M[3] * vx)));
    float dx = px - fp.cam[0], dy = py - fp.cam[1], dz = pzw - fp.cam[2], dw = pw - fp.cam[3];
    float len = sqrtf(fmaf(dw, dw, fmaf(dz, dz, fmaf(dy, dy, dx * dx))));  // vec4 normalize
    Ray r;
    r.o = mk(fp.cam[0], fp.cam[1], fp.cam[2]);
    r.d = mk(dx / len, dy / len, dz / len);
    r.inv = rcp3(r.d);
    seed_out = hash1u(ts + (index * 67u + t));
    return r;
}

// Stress rays of the leaf self-tests (pt_selftest_leaf: k_selftest_leaf, k_selftest_leafpass) for
// ray i against the leaf of records rec0 .. rec0 + n - 1, family `mode`: 0 origins within 5 units of
// a random point of an entry, directions uniform; 1 aimed at such a point from 10^-3 .. 20 units
// away; 2 grazing: along the entry's plane, tilted by 10^-7 .. 10^-1 rad, so the test's rounding is
// at its largest; 3 leaving a surface as the path tracer's bounces do (the point offset by 1e-4 along
// the normal, directions uniform).  st: the generator's state after the ray (callers draw on).
__device__ __forceinline__ uint32_t st_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ Ray stress_ray(const SceneView& sc, int rec0, int n, int mode, uint32_t seed, uint32_t i,
                                          uint32_t& st) {
    st = st_hash(seed * 0x9e3779b9u + i * 0x85ebca6bu + (uint32_t)mode);
    auto u01 = [&]() { st = st_hash(st + 0x6a09e667u); return (float)(st >> 8) * (1.0f / 16777216.0f); };
    auto unit = [&]() {
        const float z = 2.0f * u01() - 1.0f, ph = 6.2831853f * u01(), rr = sqrtf(fmaxf(0.0f, 1.0f - z * z));
        return mk(rr * cosf(ph), rr * sinf(ph), z);
    };
    auto nrm = [](f3 v) { const float l = sqrtf(dot(v, v)); return l > 0.0f ? mk(v.x / l, v.y / l, v.z / l) : mk(0.0f, 1.0f, 0.0f); };
    const int k0 = (int)(st_hash(st) % (uint32_t)n);
    const TriRec tr = load_tri(sc.tris, rec0 + k0);
    const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z), e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
    float bu = u01(), bv = u01();
    if (bu + bv > 1.0f) { bu = 1.0f - bu; bv = 1.0f - bv; }
    const f3 p = mk(v0.x + bu * e1.x + bv * e2.x, v0.y + bu * e1.y + bv * e2.y, v0.z + bu * e1.z + bv * e2.z);
    const f3 nn = nrm(cross(e1, e2));
    Ray r;
    if (mode == 0) {
        r.o = mk(p.x + 10.0f * u01() - 5.0f, p.y + 10.0f * u01() - 5.0f, p.z + 10.0f * u01() - 5.0f);
        r.d = unit();
    } else if (mode == 1) {
        const f3 w = unit();
        const float dist = exp2f(-10.0f + 14.3f * u01());
        r.o = mk(p.x + dist * w.x, p.y + dist * w.y, p.z + dist * w.z);
        r.d = nrm(mk(p.x - r.o.x, p.y - r.o.y, p.z - r.o.z));
    } else if (mode == 2) {
        const f3 t1 = nrm(e1), t2 = nrm(cross(nn, t1));
        const float ph = 6.2831853f * u01(), tilt = exp2f(-23.0f + 19.7f * u01()) * (u01() < 0.5f ? -1.0f : 1.0f);
        const f3 w = mk(cosf(ph) * t1.x + sinf(ph) * t2.x, cosf(ph) * t1.y + sinf(ph) * t2.y, cosf(ph) * t1.z + sinf(ph) * t2.z);
        r.d = nrm(mk(w.x + tilt * nn.x, w.y + tilt * nn.y, w.z + tilt * nn.z));
        const float dist = exp2f(-6.0f + 10.0f * u01());
        r.o = mk(p.x - dist * r.d.x, p.y - dist * r.d.y, p.z - dist * r.d.z);
    } else {
        const float sg = u01() < 0.5f ? -1e-4f : 1e-4f;
        r.o = mk(p.x + sg * nn.x, p.y + sg * nn.y, p.z + sg * nn.z);
        r.d = unit();
    }
    r.inv = rcp3(r.d);
    return r;
}

}  // namespace pt
