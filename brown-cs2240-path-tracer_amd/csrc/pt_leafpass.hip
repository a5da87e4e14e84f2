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
// layout): the wave loads block j + 1 into registers (two coalesced float4 loads per lane) while it
// tests block j, each record read from LDS at one address for its lanes.  (Scalar loads of each
// record were one L2 round trip per few entries: 18 % of the VALU bound, profiles/r05b_ab_leafpre.log.)
constexpr int kRecBlock = 32;  // records per LDS block: 96 float4, 1.5 KB per wave
template <bool FAST_RCP>
__device__ __forceinline__ uint64_t resolve_leaf(const SceneView& sc, int rec0, int n, const f3 o, const f3 d, bool rvalid,
                                                 int lg, float4* lrec) {
    const float eps = 1e-8f;
    const uint32_t lane = threadIdx.x & 63u;
    const int S = 64 >> lg, seg = (int)(lane >> lg);
    const float4* __restrict__ g = reinterpret_cast<const float4*>(sc.tris + rec0);
    const int nf4 = 3 * n;
    // (loads under ifs: `c ? g[i] : zero` became a load through a select of pointers, the zero in scratch)
    float4 p0 = make_float4(0, 0, 0, 0), p1 = p0;
    if ((int)lane < nf4) p0 = g[lane];
    if (lane < 32u && 64 + (int)lane < nf4) p1 = g[64 + lane];
    float bt = 0.0f;
    int bk = 0x7fffffff;  // none
    // One entry (record words a, b, c) for this lane's ray: tri_hit's arithmetic.  The wave skips
    // the entry when no lane can report a hit, decided before the reciprocal: a lane cannot when its
    // determinant fails, or when its u = RN(RN(1 / det) * un) is certainly outside [0, 1] — un and
    // det of opposite signs with |un| >= 2^-100 |det| (u < 0, far above underflow to -0), or |un| >
    // RN(|det| (1 + 2^-20)) (|u| > (1 + 2^-21)(1 - 2^-24)^2 > 1).  NaN operands vote "maybe".
    auto test_entry = [&](const float4 a, const float4 b, const float c, const bool live, const int pos) {
        const f3 v0 = mk(a.x, a.y, a.z), e1 = mk(a.w, b.x, b.y), e2 = mk(b.z, b.w, c);
        const f3 rce2 = cross(d, e2);
        const float det = dot(e1, rce2);
        const f3 sv = o - v0;
        const float un = dot(sv, rce2);
        const bool ok_det = !(det > -eps && det < eps);
        const float ad = fabsf(det), au = fabsf(un);
        const bool out = ((un * det < 0.0f) & (au >= ad * 0x1p-100f)) | (au > ad * 1.00000095367431640625f);
        if ((__builtin_amdgcn_ballot_w64(live) & __builtin_amdgcn_ballot_w64(ok_det) &
             ~__builtin_amdgcn_ballot_w64(out)) == 0)
            return;  // wave-uniform: no lane can report a hit
        const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
        const float u = inv_det * un;
        const f3 sce1 = cross(sv, e1);
        const float v = inv_det * dot(d, sce1);
        const float t = inv_det * dot(e2, sce1);
        const bool hit = live & ok_det & !(u < 0.0f) & !(u > 1.0f) & !(v < 0.0f) & !(u + v > 1.0f) & (t > eps);
        const bool take = hit & ((t < bt) | (bk == 0x7fffffff));
        bt = take ? t : bt;
        bk = take ? pos : bk;
    };
    for (int k0 = 0; k0 < n; k0 += kRecBlock) {
        wave_lds_sync();  // every lane is done reading the previous block
        lrec[lane] = p0;
        if (lane < 32u) lrec[64 + lane] = p1;
        wave_lds_sync();
        const int nb = 3 * (k0 + kRecBlock);  // the next block, in flight while this one is tested
        if (nb + (int)lane < nf4) p0 = g[nb + lane];
        if (lane < 32u && nb + 64 + (int)lane < nf4) p1 = g[nb + 64 + lane];
        const int m = min(kRecBlock, n - k0);
        // two entries per step, both records read from LDS before either is tested (their LDS latency
        // behind one another's arithmetic)
        for (int j = 0; j < m; j += 2 * S) {  // uniform
            const int ea = j + seg, eb = j + S + seg;  // this lane's two entries of the block
            const int xa = min(ea, m - 1), xb = min(eb, m - 1);
            const float4 aa = lrec[3 * xa], ab = lrec[3 * xa + 1], ba = lrec[3 * xb], bb = lrec[3 * xb + 1];
            const float ac = lrec[3 * xa + 2].x, bc = lrec[3 * xb + 2].x;
            test_entry(aa, ab, ac, rvalid & (ea < m), k0 + ea);
            if (j + S < m) test_entry(ba, bb, bc, rvalid & (eb < m), k0 + eb);  // uniform
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

// The same result, walking the leaf's chunks (pt_leafbvh.cpp; SceneView::lnodes / ltris, option
// leaf_cull): chunk c (wave-uniform, its node through the scalar cache, loaded one chunk ahead) is
// checked for every lane's ray against that lane's best so far (chunk_skip, pt_device.h: no entry
// of a skipped chunk can report a hit at t <= the bound), and its entries are tested only when some
// lane opens it — by every lane: a lane whose check held no entry able to beat its bound gains
// nothing it could take.  The records stream through LDS in chunk order (ltris; each carries its
// position in the leaf, so the keys are the same (t, position)).  Pays where a wave's rays are
// coherent enough that most chunks are closed for all of them (camera rays).
template <bool FAST_RCP>
__device__ __forceinline__ uint64_t resolve_leaf_cull(const SceneView& sc, int rec0, const f3 o, const f3 d, bool rvalid,
                                                      int lg, float4* lrec) {
    const float eps = 1e-8f;
    const uint32_t lane = threadIdx.x & 63u;
    const int S = 64 >> lg, seg = (int)(lane >> lg);
    const cint_p tr0 = (cint_p)(sc.tris + rec0);
    const int c0 = tr0[11] - 1, c1 = tr0[12 + 11];  // Tri::lbvh of the leaf's first two records
    const cfloat_p nf = (cfloat_p)sc.lnodes;  // chunk nodes, 16 floats each, through the scalar cache
    auto node4 = [&](int q) { return make_float4(nf[4 * q], nf[4 * q + 1], nf[4 * q + 2], nf[4 * q + 3]); };
    Ray r;
    r.o = o;
    r.d = d;
    r.inv = rcp3(d);
    const float idl = 1.0f / sqrtf(dot(d, d));
    const float on = sqrtf(dot(o, o));
    // the record stream: block [bs, bs + kRecBlock) of ltris in LDS, [bs + kRecBlock, + 2 kRecBlock) in
    // registers; every load stays below the leaf's last record f1 (ltris ends there for the last leaf)
    const float4* __restrict__ g = reinterpret_cast<const float4*>(sc.ltris);
    const int f0 = __builtin_bit_cast(int, nf[16 * c0 + 15]) & 0xffffff;
    const int il = __builtin_bit_cast(int, nf[16 * (c1 - 1) + 15]);
    const int f1 = (il & 0xffffff) + (il >> 24);
    int bs = f0 - kRecBlock;  // nothing staged yet: the registers hold [f0, f0 + kRecBlock)
    float4 p0 = make_float4(0, 0, 0, 0), p1 = p0;
    auto fetch = [&](int base, float4& x0, float4& x1) {  // block at record `base` into registers
        if (3 * base + (int)lane < 3 * f1) x0 = g[3 * base + lane];
        if (lane < 32u && 3 * base + 64 + (int)lane < 3 * f1) x1 = g[3 * base + 64 + lane];
    };
    fetch(f0, p0, p1);
    float bt = 0.0f;
    int bk = 0x7fffffff;  // none
    float4 na = node4(4 * c0), nb = node4(4 * c0 + 1), nc = node4(4 * c0 + 2), ne = node4(4 * c0 + 3);
    for (int c = c0; c < c1; ++c) {
        const float4 a = na, b = nb, cc = nc, e = ne;
        if (c + 1 < c1) {  // the next chunk's node, in flight while this one is checked
            na = node4(4 * c + 4); nb = node4(4 * c + 5); nc = node4(4 * c + 6); ne = node4(4 * c + 7);
        }
        const float bound = bk == 0x7fffffff ? __builtin_inff() : bt;
        const bool open = rvalid & !chunk_skip(a, b, cc, e, r, idl, on, bound);
        if (!__builtin_amdgcn_ballot_w64(open)) continue;  // uniform: closed for every ray
        const int info = __builtin_bit_cast(int, e.w), first = info & 0xffffff, cnt = info >> 24;
        for (int j0 = 0; j0 < cnt; j0 += S) {  // uniform
            const int k = first + j0 + seg;  // this lane's record
            const int kk = min(k, first + cnt - 1);
            const int lo = first + j0, hi = min(first + j0 + S, first + cnt);  // this step's records
            if (lo < bs || hi > bs + kRecBlock) {  // uniform: stage the block that holds them
                wave_lds_sync();
                if (lo >= bs + kRecBlock && hi <= bs + 2 * kRecBlock) {  // the prefetched one
                    bs += kRecBlock;
                    lrec[lane] = p0;
                    if (lane < 32u) lrec[64 + lane] = p1;
                } else {  // further ahead (chunks skipped): load it now
                    bs = lo;
                    float4 x0 = make_float4(0, 0, 0, 0), x1 = x0;
                    fetch(bs, x0, x1);
                    lrec[lane] = x0;
                    if (lane < 32u) lrec[64 + lane] = x1;
                }
                wave_lds_sync();
                fetch(bs + kRecBlock, p0, p1);
            }
            const int o3 = 3 * (kk - bs);
            const float4 ra = lrec[o3], rb = lrec[o3 + 1], rc = lrec[o3 + 2];
            const bool live = rvalid & (k < first + cnt);
            const f3 v0 = mk(ra.x, ra.y, ra.z), e1 = mk(ra.w, rb.x, rb.y), e2 = mk(rb.z, rb.w, rc.x);
            const f3 rce2 = cross(d, e2);
            const float det = dot(e1, rce2);
            const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
            const f3 sv = o - v0;
            const float u = inv_det * dot(sv, rce2);
            const bool ok_det = !(det > -eps && det < eps), ok_lo = !(u < 0.0f), ok_hi = !(u > 1.0f);
            if ((__builtin_amdgcn_ballot_w64(live) & __builtin_amdgcn_ballot_w64(ok_det) &
                 __builtin_amdgcn_ballot_w64(ok_lo) & __builtin_amdgcn_ballot_w64(ok_hi)) == 0)
                continue;
            const f3 sce1 = cross(sv, e1);
            const float v = inv_det * dot(d, sce1);
            const float t = inv_det * dot(e2, sce1);
            const int pos = __builtin_bit_cast(int, rc.w);  // Tri::lbvh of an ltris copy: the position in the leaf
            const bool hit = live & ok_det & ok_lo & ok_hi & !(v < 0.0f) & !(u + v > 1.0f) & (t > eps);
            const bool take = hit & ((bk == 0x7fffffff) | (t < bt) | ((t == bt) & (pos < bk)));
            bt = take ? t : bt;
            bk = take ? pos : bk;
        }
    }
    uint64_t key = bk == 0x7fffffff ? ~0ull : ((uint64_t)__builtin_bit_cast(uint32_t, bt) << 32) | (uint32_t)bk;
    for (int off = 1 << lg; off < 64; off <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)key, off, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), off, 64);
        const uint64_t other = ((uint64_t)hi << 32) | lo;
        key = other < key ? other : key;
    }
    return key;
}

template <bool FAST_RCP>
__global__ __launch_bounds__(kLeafPassBlock) void k_wf_leafpass(SceneView sc, WfBuffers wb, int in_q, int cull) {
    __shared__ uint32_t ring[kLeafPassBlock / 64][kMaxPre][kLeafRing];
    __shared__ uint32_t pos[kLeafPassBlock / 64][kMaxPre][2];  // per wave and leaf: head, tail (wave-uniform)
    __shared__ float4 lrec[kLeafPassBlock / 64][3 * kRecBlock];  // per wave: a block of leaf records
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
        const int lg = avail > 1 ? 32 - __builtin_clz(avail - 1) : 0;  // ceil(log2 avail)
        const uint32_t ri = lane & ((1u << lg) - 1u);
        const bool valid = ri < avail;
        const uint32_t i = valid ? ring[wv][b][(tail + ri) & (kLeafRing - 1)] : 0u;
        float4 a = make_float4(0, 0, 0, 0), c = a;
        if (valid) { a = q[2 * (size_t)i]; c = q[2 * (size_t)i + 1]; }
        const cint_p pl = (cint_p)(sc.pre + b);
        const int rec0 = pl[0];
        uint64_t key;
        if (cull && ((cint_p)(sc.tris + rec0))[11] > 0)  // uniform: the leaf has chunks (Tri::lbvh)
            key = resolve_leaf_cull<FAST_RCP>(sc, rec0, mk(a.x, a.y, a.z), mk(a.w, c.x, c.y), valid, lg, lrec[wv]);
        else
            key = resolve_leaf<FAST_RCP>(sc, rec0, pl[1], mk(a.x, a.y, a.z), mk(a.w, c.x, c.y), valid, lg, lrec[wv]);
        if (lane < avail) wb.pres[(size_t)b * wb.pres_stride + i] = key;
    };
    // windows of wr queue entries per wave: 64, or fewer when the queue cannot give every wave a
    // window of 64 (the last depths): then each wave's rays are few and each is walked by many lanes
    uint32_t wr = 64;
    while (wr > 1 && (uint64_t)count < (uint64_t)nwaves * wr) wr >>= 1;
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
                pass = pass && enters(sc, pl[4 + k], r);
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

hipError_t launch_leafpass(const SceneView& sc, const WfBuffers& wb, int in_q, bool fast_rcp, int blocks, int cull,
                           hipStream_t stream) {
    cull = cull && sc.lnodes && sc.ltris;
    if (sc.npre <= 0 || !sc.pre || !wb.pres) return hipErrorInvalidValue;
    const void* k = fast_rcp ? (const void*)k_wf_leafpass<true> : (const void*)k_wf_leafpass<false>;
    const int nb = blocks > 0 ? blocks : leafpass_blocks(k);
    if (fast_rcp)
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<true>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q, cull);
    else
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<false>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q, cull);
    return hipSuccess;
}

}  // namespace pt
