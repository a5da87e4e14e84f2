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

template <bool FAST_RCP>
__global__ __launch_bounds__(kLeafPassBlock) void k_wf_leafpass(SceneView sc, WfBuffers wb, int in_q) {
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
        // the ray arrives here, before resolve_leaf issues its record prefetches: otherwise the
        // compiler's in-order vmcnt wait for the ray sits inside the entry loop and waits for the
        // prefetch of the next record block too, every block
        asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(c.x), "v"(c.y));
        const cint_p pl = (cint_p)(sc.pre + b);
        const uint64_t key =
            resolve_leaf<FAST_RCP>(sc, pl[0], pl[1], mk(a.x, a.y, a.z), mk(a.w, c.x, c.y), valid, lg, lrec[wv]);
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

hipError_t launch_leafpass(const SceneView& sc, const WfBuffers& wb, int in_q, bool fast_rcp, int blocks,
                           hipStream_t stream) {
    if (sc.npre <= 0 || !sc.pre || !wb.pres) return hipErrorInvalidValue;
    const void* k = fast_rcp ? (const void*)k_wf_leafpass<true> : (const void*)k_wf_leafpass<false>;
    const int nb = blocks > 0 ? blocks : leafpass_blocks(k);
    if (fast_rcp)
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<true>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q);
    else
        PT_LAUNCH(KID_WF_LEAF, stream, k_wf_leafpass<false>, dim3(nb), dim3(kLeafPassBlock), 0, stream, sc, wb, in_q);
    return hipSuccess;
}

}  // namespace pt
