// pt_wavefront.hip — wavefront path tracer for gfx950 (the north-star design).
//
// A batch of P = F*W*H paths (F frames of the image) lives in HBM as DENSE queues of
// entries that carry the ray AND the path state (WfQueue, pt_kernels.h: 64 B per entry,
// +40 B of shading point in the shadow queue).  Survivors are compacted into the other
// queue every iteration, so every kernel streams its queue coalesced and nothing is
// gathered by path index (the radiance of a finished path is the only scatter).  Each
// iteration runs:
//   k_wf_trace   closest-hit traversal of the queue.  Persistent waves, each owning a
//                contiguous chunk of the queue (no atomics).  Rays arrive in LDS windows of
//                32 records (the next window in flight in registers) and hits leave through
//                an LDS ring written back one coalesced window at a time, so the traversal
//                loop issues no global memory operation; a lane takes its next ray the
//                moment its traversal ends.  Traversal is trav_step_lean (per-lane stack in
//                LDS, scene in LDS when it fits).
//   k_wf_shade   the path logic after that traversal (path_after_ext / path_after_shadow,
//                pt_path.h) and compaction of the surviving paths into the next queue with
//                __ballot + mbcnt (one atomicAdd per wave).
// All paths of a batch start together, so a queue holds only extension rays or only
// shadow rays and the two alternate.  k_wf_generate writes the camera rays; k_wf_accum adds
// the batch's finished radiance into the accumulator in frame order, which keeps the result
// bit-identical to the reference's host accumulation.
#include "pt_kernels.h"
#include "pt_path.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

namespace pt {

// Diagnostic build only (make EXTRA=-DPT_PHASE_STATS=1 OUT_DIR=...; scripts/phase_stats.py): the fused
// kernel's waves time their phases with s_memtime and count, per phase, loop iterations and the
// active lanes at each (the mean over iterations of popcount(exec) / 64 is the phase's lane use for a
// loop whose body issues the same instructions every iteration), summed over waves into
// g_phase_stats[EXT][phase][cycles, iterations, lanes] at the end of each wave; read by
// pt_phase_stats_read.  Phases (PH_*): the batch's loads, phase 1 (the entries' tests; PH_P1FULL
// counts its iterations past the vote), the replay (PH_REPLAY: its node iterations; PH_RLEAF the
// leaf-hit iterations), the path logic, the append and stores.
#ifndef PT_PHASE_STATS
#define PT_PHASE_STATS 0
#endif
enum { PH_LOAD = 0, PH_P1, PH_P1FULL, PH_REPLAY, PH_RLEAF, PH_SHADE, PH_APPEND, PH_COUNT };
#if PT_PHASE_STATS
struct PhaseAcc {
    uint64_t v[PH_COUNT + 1][3];  // + a scratch row: the start of phase 1
};
__device__ unsigned long long g_phase_stats[2][PH_COUNT][3];
__device__ __forceinline__ uint64_t ph_now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void ph_iter(PhaseAcc& pa, int ph) {
    pa.v[ph][1] += 1;
    pa.v[ph][2] += (uint64_t)__builtin_popcountll(__builtin_amdgcn_read_exec());
}
#define PH_PARAM , PhaseAcc& pa
#define PH_PASS , pa
#define PH_ITER(ph) ph_iter(pa, ph)
#else
#define PH_PARAM
#define PH_PASS
#define PH_ITER(ph) ((void)0)
#endif
#if PT_TRACE_STATS
__device__ unsigned long long g_trace_stats[2][TS_COUNT][3];  // [shadow queue][kind][cycles, turns, lanes]
#endif

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// number of set bits of m below this lane
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t pack_dspec(const PathState& ps) {
    return (uint32_t)ps.depth | (ps.spec ? 0x10000u : 0u);
}
__device__ __forceinline__ void unpack_dspec(uint32_t dw, PathState& ps) {
    ps.depth = (int)(dw & 0xffffu);
    ps.spec = (dw & 0x10000u) != 0;
}
__device__ __forceinline__ Ray unpack_ray(float4 a, float4 b, uint32_t& p) {
    Ray r;
    r.o = mk(a.x, a.y, a.z);
    r.d = mk(a.w, b.x, b.y);
    r.inv = rcp3(r.d);
    p = __builtin_bit_cast(uint32_t, b.z);
    return r;
}
// queue entry i <- (ray, path index, path state)
__device__ __forceinline__ void store_entry(const WfQueue& Q, uint32_t i, const Ray& r, uint32_t p, const PathState& ps) {
    Q.ray[2 * (size_t)i] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
    Q.ray[2 * (size_t)i + 1] = make_float4(r.d.y, r.d.z, __builtin_bit_cast(float, p), __builtin_bit_cast(float, pack_dspec(ps)));
    Q.q2[i] = make_float4(ps.L.x, ps.L.y, ps.L.z, __builtin_bit_cast(float, ps.seed));
    Q.q3[i] = make_float4(ps.beta.x, ps.beta.y, ps.beta.z, 0.0f);
}
__device__ __forceinline__ Ray load_entry(const WfQueue& Q, uint32_t i, uint32_t& p, PathState& ps) {
    const float4 a = Q.ray[2 * (size_t)i], b = Q.ray[2 * (size_t)i + 1], c = Q.q2[i], d = Q.q3[i];
    unpack_dspec(__builtin_bit_cast(uint32_t, b.w), ps);
    ps.L = mk(c.x, c.y, c.z);
    ps.seed = __builtin_bit_cast(uint32_t, c.w);
    ps.beta = mk(d.x, d.y, d.z);
    return unpack_ray(a, b, p);
}
__device__ __forceinline__ void store_shading_point(const WfBuffers& wb, uint32_t i, const PathState& ps) {
    wb.sp0[i] = make_float4(ps.hp.x, ps.hp.y, ps.hp.z, __builtin_bit_cast(float, ps.mat_id));
    wb.sp1[i] = make_float4(ps.hn.x, ps.hn.y, ps.hn.z, ps.wi.x);
    wb.sp2[i] = make_float2(ps.wi.y, ps.wi.z);
}
__device__ __forceinline__ void load_shading_point(const WfBuffers& wb, uint32_t i, PathState& ps) {
    const float4 a = wb.sp0[i], b = wb.sp1[i];
    const float2 c = wb.sp2[i];
    ps.hp = mk(a.x, a.y, a.z);
    ps.mat_id = __builtin_bit_cast(int, a.w);
    ps.hn = mk(b.x, b.y, b.z);
    ps.wi = mk(b.w, c.x, c.y);
}

// The fused kernels' shadow queue (bf_step_batch, its only writer and reader) holds 88 B per entry
// instead of the 104 B of a ray + path state + shading point: the shadow ray's origin is not
// stored — it is offset = madd(hp, hn, 1e-4), recomputed from the shading point with the very
// operation path_after_ext made it with (the same bits) — and the words are packed into the
// queue's arrays as
//   ray[2i]   = (d.xyz, path)      ray[2i+1] = (depth | spec, L.xyz)   q2 = (seed, beta.xyz)
//   q3        = (hp.xyz, material) sp0      = (hn.xyz, wi.x)          sp2 = (wi.y, wi.z)
// (sp1 unused).  The traversal pipeline (k_wf_trace + k_wf_shade) keeps the full layout above.
__device__ __forceinline__ void store_shadow_packed(const WfBuffers& wb, uint32_t i, const Ray& r, uint32_t p,
                                                    const PathState& ps) {
    const WfQueue& Q = wb.shd;
    Q.ray[2 * (size_t)i] = make_float4(r.d.x, r.d.y, r.d.z, __builtin_bit_cast(float, p));
    Q.ray[2 * (size_t)i + 1] = make_float4(__builtin_bit_cast(float, pack_dspec(ps)), ps.L.x, ps.L.y, ps.L.z);
    Q.q2[i] = make_float4(__builtin_bit_cast(float, ps.seed), ps.beta.x, ps.beta.y, ps.beta.z);
    Q.q3[i] = make_float4(ps.hp.x, ps.hp.y, ps.hp.z, __builtin_bit_cast(float, ps.mat_id));
    wb.sp0[i] = make_float4(ps.hn.x, ps.hn.y, ps.hn.z, ps.wi.x);
    wb.sp2[i] = make_float2(ps.wi.y, ps.wi.z);
}
// the ray of a packed shadow entry from its words (a = ray[2i], h = q3, n = sp0)
__device__ __forceinline__ Ray unpack_shadow_ray(float4 a, float4 h, float4 n, uint32_t& p) {
    Ray r;
    r.o = madd(mk(h.x, h.y, h.z), mk(n.x, n.y, n.z), 1.0e-4f);  // = path_after_ext's offset, bit for bit
    r.d = mk(a.x, a.y, a.z);
    r.inv = rcp3(r.d);
    p = __builtin_bit_cast(uint32_t, a.w);
    return r;
}

// The camera path made for queue slot s (the s-th path of a batch part in generation order): its
// frame f, pixel (x, y) and path id p = f * npix + y * W + x — row-major within its frame, the
// radiance index k_wf_accum reads; slot = path id.
__device__ __forceinline__ uint32_t slot_path(uint32_t s, const FrameParams& fp, uint32_t& x, uint32_t& y, uint32_t& f) {
    const uint32_t W = fp.width, npix = W * fp.height;
    f = s / npix;
    const uint32_t q = s - f * npix;
    y = q / W;
    x = q - y * W;
    return s;
}

template <bool COUNT>
__global__ __launch_bounds__(256) void k_wf_generate(FrameParams fp, WfBuffers wb, uint32_t frame0, uint32_t stride,
                                                     uint32_t fbase, uint32_t P, bool raw_salt, Counters* cnt_out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p == 0) {
        wb.ctl[WF_COUNT0] = P;
        wb.ctl[WF_COUNT1] = 0;
    }
    // region layout (k_wf_step_bf, wb.nreg > 0): 64-path batch j goes to region j % nreg
    const uint32_t R = wb.nreg;
    if (R && p < R) {  // counts of region p: its batches j = t, t + R, ... < ceil(P / 64), t = p rq mod R
        const uint32_t nbat = (P + 63) / 64;
        const uint32_t t = (uint32_t)((uint64_t)p * wb.rq % R);
        const uint32_t n = t < nbat ? (nbat - t + R - 1) / R : 0u;
        const uint32_t last = t + (n - 1) * R;
        wb.rcnt[p] = n == 0 ? 0u : n * 64 - ((last == nbat - 1 && (P & 63)) ? 64 - (P & 63) : 0u);
        wb.rcnt[kRegions + p] = 0;
    }
    Counters c = {};
    if (p < P) {  // p: the queue slot; pid: the path made there (slot_path)
        uint32_t x, y, f;
        const uint32_t pid = slot_path(p, fp, x, y, f);
        const uint32_t t = raw_salt ? frame0 : (uint32_t)(float)(frame0 + (fbase + f) * stride);
        PathState ps;
        Ray r = path_begin(fp, x, y, t, ps);
        const uint32_t j = p / 64;
        const uint32_t i = R ? (uint32_t)((uint64_t)(j % R) * wb.rqi % R) * wb.rstride + (j / R) * 64 + (p & 63) : p;
        store_entry(wb.ext, i, r, pid, ps);
        if (COUNT) { c.samples++; c.ext_queries++; }
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// Per-wave LDS staging for k_wf_trace: the current window of 32 queued rays and a ring of
// hit records.  Keeping both in LDS takes every global load and store out of the traversal
// loop: on gfx9 loads and stores share the wave's in-order vmcnt, so a per-lane global store
// (or prefetch) in the loop makes the next use of any loaded register wait for it.
constexpr uint32_t kWinRays = 32;
// the hit ring: 128 or 256 entries (a power of two, a multiple of kWinRays, >= 2 windows), chosen
// per launch (trace_ring): a larger ring lets a wave take new windows while more of its earlier
// windows' stragglers still trace (Glossy: 64 entries -15 %, 256 +4.3 % in process,
// profiles/r03k_ab_ring*.log), but its LDS can cost a block per CU (the boat: 3 -> 2 blocks, -2.4 %)
constexpr uint32_t kHitRing = 128;
constexpr uint32_t kHitRingMax = 256;
// window ids of the windows between the last flushed and the prefetched one: the ring holds
// RING / kWinRays windows, plus the one in registers (a compile-time size per kernel instance: a
// ring size read at run time measured 10 % slower on the deep synthetic trees)
__host__ __device__ constexpr uint32_t win_tab(uint32_t ring) { return 2 * ring / kWinRays > 8 ? 2 * ring / kWinRays : 8; }
static_assert(win_tab(kHitRingMax) >= kHitRingMax / kWinRays + 2, "wtab must name every window the ring can hold");
static_assert(win_tab(kHitRing) >= kHitRing / kWinRays + 2, "wtab must name every window the ring can hold");
// per wave: the window's rays, the hit ring, the window ids, and 64 keys — one per lane for
// lean_leaf_pool's pooled leaf turns, the first kMultiRays for chunk_turn_multi's shared walks
__host__ __device__ constexpr uint32_t stage_bytes(uint32_t ring) { return kWinRays * 32 + ring * 8 + win_tab(ring) * 4; }
// after the waves' stages, when the scene needs them (pooled leaf turns or leaf chunks: keys_on),
// 64 keys per wave — one per lane for lean_leaf_pool, the first kMultiRays for chunk_turn_multi
constexpr uint32_t kKeyBytes = 64 * 8;
// Only the lean flavours pool leaf turns or walk chunks (trav_step_lean; not the mailboxed 1xx nor
// the flattened 1 / 2), so only their instances reserve the keys (advisor r04: every instance did)
template <int TRAV>
__host__ __device__ constexpr bool lean_flavour() { return TRAV >= 3 && !(TRAV >= 100 && TRAV < 160) && TRAV < 300; }
template <int TRAV>
__host__ __device__ inline bool keys_on(const SceneView& sc) {
    return lean_flavour<TRAV>() && (sc.leaf_pool != 0 || sc.lnodes != nullptr);
}
// the traversal flavours that have a 256-entry-ring instance (the defaults: lean16 + fast rcp, with
// and without big-leaf turns); the others always use 128
constexpr bool has_big_ring(int trav) { return trav == 17 || trav == 177 || trav == 277; }
constexpr uint32_t kTraceBlock = 512;  // 8 waves share one LDS copy of the scene
// LDS of k_wf_trace per block: the lanes' traversal stacks (max_stack entries of 4 B) and per wave
// stage_bytes(ring)

// Work split: the queue is cut into windows of 32 entries; wave w of N takes windows w, w+N,
// w+2N, ... (interleaving, not contiguous chunks, because queue order is spatially coherent —
// camera rays in pixel order, survivors compacted block by block — so a contiguous chunk is an
// image region whose cost differs systematically from the others).  Inside a wave, its j-th
// window's entries have the wave-local sequence numbers 32j .. 32j+31, which index the hit ring;
// wtab keeps the ids of the windows between the last written back and the prefetched one.
// No occupancy attribute: the big-leaf instances take 71 VGPRs (7 waves per SIMD); forcing
// amdgpu_waves_per_eu(7) made them 72 and 11 % slower on the 100k synthetic scene (in process,
// profiles/r03m_ab_trace_occ.log).
// sparse (option trace_sparse=n): when windows of wr entries would keep fewer than 1/n of the waves
// busy (the last depths), windows of wr / 2 .. 1 entries spread the queue over more waves, so each
// wave's traversal is the slowest of fewer rays.  A window still takes kWinRays sequence numbers
// (ring and flush bookkeeping unchanged); only its queue span is wr.
template <bool LDS, int TRAV, bool COUNT, uint32_t RING, int PRUN>
__device__ __forceinline__ void wf_trace_body(SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out, uint32_t watchdog,
                                              int sparse) {
    constexpr uint32_t nring = RING, kWinTab = win_tab(RING);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const LStack32 stack = LStack32::make(smem, blockDim.x);
    char* stage_base = smem + (uint32_t)sc.max_stack * 4u * blockDim.x;
    char* stage = stage_base + (threadIdx.x / 64u) * stage_bytes(nring);
    float4* wray = reinterpret_cast<float4*>(stage);               // [kWinRays][2]
    int2* ring = reinterpret_cast<int2*>(stage + kWinRays * 32);   // [RING]
    uint32_t* wtab = reinterpret_cast<uint32_t*>(stage + kWinRays * 32 + RING * 8);  // [kWinTab] window ids
    char* key_base = stage_base + (blockDim.x / 64u) * stage_bytes(nring);
    const uint32_t key_bytes = keys_on<TRAV>(sc) ? (blockDim.x / 64u) * kKeyBytes : 0u;
    sc.lkeys = key_bytes ? reinterpret_cast<uint64_t*>(key_base + (threadIdx.x / 64u) * kKeyBytes) : nullptr;
    sc.pres = wb.pres;  // this part's pre-resolved big leaves (TRAV 26x / 27x; k_wf_leafpass)
    sc.pres_stride = wb.pres_stride;
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1] = 0;  // shade's output count
    const uint32_t count = wb.ctl[WF_WATCHDOG] ? 0u : wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];  // gave up: skip
    // the wave index is uniform: readfirstlane keeps everything derived from it in SGPRs
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    uint32_t wr = kWinRays;
    if (sparse > 0)
        while (wr > 1 && (uint64_t)count * (uint32_t)sparse < (uint64_t)nwaves * wr) wr >>= 1;
    const uint32_t nwin = (count + wr - 1) / wr;
    if (LDS) stage_scene_lds(sc, key_base + key_bytes);
    const uint32_t lane = lane_id();
    constexpr uint32_t kNone = 0xffffffffu;
    uint32_t nstatic = 0;
    auto fetch = [&]() {  // this wave's next window (wave-uniform), or kNone
        const uint64_t wid = (uint64_t)(nstatic++) * nwaves + w;
        return wid < nwin ? (uint32_t)wid : kNone;
    };
    auto wcount = [&](uint32_t wid) { return min(wr, count - wid * wr); };
    const uint32_t w0 = fetch();
    if (w0 == kNone) return;  // wave-uniform: nothing for this wave
    uint32_t wcur = w0, wnx = kNone;  // ids of window jl (handed out now) and of the one in flight
    // lanes 0..31 load the first halves of a window's ray records, lanes 32..63 the second
    const uint32_t wl = lane & (kWinRays - 1), half = lane / kWinRays;
    const float4* q = in_q ? wb.shd.ray : wb.ext.ray;
    Counters c = {};
    // local window jl (id wtab[jl % kWinTab]) sits in LDS; window jl + 1 is in flight in registers
    uint32_t jl = 0, wv = wcount(w0);
    if (lane == 0) wtab[0] = w0;
    if (wl < wv) wray[2 * wl + half] = q[2 * (size_t)(w0 * wr + wl) + half];
    uint32_t nv = 0;
    float4 na = make_float4(0, 0, 0, 0);
    {
        const uint32_t w1 = fetch();
        wnx = w1;
        if (w1 != kNone) {
            nv = wcount(w1);
            if (lane == 0) wtab[1] = w1;
            if (wl < nv) na = q[2 * (size_t)(w1 * wr + wl) + half];
        }
    }
    uint32_t cur = 0;      // sequence number of the next entry to hand out (in window jl)
    uint32_t flushed = 0;  // sequence numbers below this are written back to wb.hitq
    uint32_t sq = 0, p = 0;
    bool has = false;
    Ray r;
    r.o = r.d = r.inv = mk(0.0f, 0.0f, 0.0f);
    typename TravSel<TRAV>::type s;
    trav_init(s, false);
    const uint64_t t_start = wall_clock64();
#if PT_TRACE_STATS
    uint64_t tl0 = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t guard = 0;; ++guard) {
#if PT_TRACE_STATS
        {
            const uint64_t tl1 = __builtin_amdgcn_s_memtime();
            if (guard) ts_add(c, TS_LOOP, tl1 - tl0, (uint64_t)__popcll(__ballot(has)));
            tl0 = tl1;
        }
#endif
        // every wave reaches an exit: after kTraceWatchdog iterations or kTraceWatchdogTicks of
        // wall clock it reports instead of hanging (and later launches of the render skip)
        if (guard == watchdog ||
            ((guard & 1023u) == 1023u && wall_clock64() - t_start > kTraceWatchdogTicks)) {
            const uint64_t hm = __ballot(has);
            if (lane == 0) {
                atomicOr(&wb.ctl[WF_WATCHDOG], 1u);
                if (atomicCAS(&wb.ctl[WF_SNAP_CLAIM], 0u, 1u) == 0u) {
                    const uint32_t v[WF_SNAP_WORDS] = {count, nwaves, w, jl, wv, nv, cur, flushed,
                                                       (uint32_t)__popcll(hm), (uint32_t)hm, (uint32_t)(hm >> 32),
                                                       (uint32_t)in_q, 0u, 0u, 0u, 0u};
                    for (int i = 0; i < WF_SNAP_WORDS; ++i) wb.ctl[WF_SNAP + i] = v[i];
                }
            }
            break;
        }
        // write back every window whose entries are all handed out and traced (coalesced)
        while (flushed < (jl + 1) * kWinRays) {
            const uint32_t jf = flushed / kWinRays;
            const bool handed = jf < jl || cur == jl * kWinRays + wv;
            if (!handed || wave_any(has && sq < flushed + kWinRays)) break;
            const uint32_t wf = wtab[jf % kWinTab];
            const uint32_t fv = wcount(wf);
            if (lane < fv) wb.hitq[wf * wr + lane] = ring[(flushed + lane) & (nring - 1)];
            flushed += kWinRays;
        }
        // hand the next entries to idle lanes (wave-uniform control)
        const uint64_t need = __ballot(!has);
#if PT_TRACE_STATS
        if (need && cur == jl * kWinRays + wv) {  // idle lanes and the window handed out: why no next one?
            if (nv > 0 && (jl + 2) * kWinRays - flushed > nring) ts_add(c, TS_BLOCKED, 0, (uint64_t)__popcll(need));
            else if (nv == 0) ts_add(c, TS_STARVED, 0, (uint64_t)__popcll(need));
        }
#endif
        if (need) {
            if (cur == jl * kWinRays + wv && nv > 0 && (jl + 2) * kWinRays - flushed <= nring) {
                if (wl < nv) wray[2 * wl + half] = na;  // next window, if the hit ring has room
                ++jl;
                wv = nv;
                cur = jl * kWinRays;
                nv = 0;
                wcur = wnx;
                const uint32_t wn = fetch();
                wnx = wn;
                if (wn != kNone) {
                    nv = wcount(wn);
                    if (lane == 0) wtab[(jl + 1) % kWinTab] = wn;
                    if (wl < nv) na = q[2 * (size_t)(wn * wr + wl) + half];
                }
            }
            const uint32_t wend = jl * kWinRays + wv;
            if (cur < wend) {
                const uint32_t k = cur + rank_below(need);
                if (!has && k < wend) {
                    const uint32_t o = k - jl * kWinRays;
                    r = unpack_ray(wray[2 * o], wray[2 * o + 1], p);
                    sq = k;
                    trav_init(s, true);
                    if constexpr (TRAV >= 260 && TRAV < 300) s.qi = wcur * wr + o;  // its queue entry
                    has = true;
                }
                cur = min(cur + (uint32_t)__popcll(need), wend);
            }
        }
        if (!wave_any(has)) {
            if (nv == 0 && cur == jl * kWinRays + wv && flushed >= (jl + 1) * kWinRays) break;  // all done
            continue;  // ring full with nothing in flight: the flush above frees it
        }
#if PT_TRACE_STATS
        if (!trav_advance<TRAV, COUNT, true, PRUN>(sc, r, s, stack, c)) ts_add(c, TS_NONE, 0, 0);
#else
        trav_advance<TRAV, COUNT, true, PRUN>(sc, r, s, stack, c);
#endif
        if (has && trav_finished(s)) {
            ring[sq & (nring - 1)] = make_int2(s.best, __builtin_bit_cast(int, s.best_t));
            has = false;
        }
    }
    if (COUNT) flush_counters(c, cnt_out);
#if PT_TRACE_STATS
    if (!COUNT && lane == 0)
        for (int k = 0; k < TS_COUNT; ++k)
            for (int f = 0; f < 3; ++f) atomicAdd(&g_trace_stats[in_q ? 1 : 0][k][f], (unsigned long long)c.ts[k][f]);
#endif
}
template <bool LDS, int TRAV, bool COUNT, uint32_t RING = kHitRing, int PRUN = 4>
__global__ __launch_bounds__(kTraceBlock) void k_wf_trace(SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out,
                                                          uint32_t watchdog, int sparse) {
    wf_trace_body<LDS, TRAV, COUNT, RING, PRUN>(sc, wb, in_q, cnt_out, watchdog, sparse);
}
// The instances with pre-resolved big leaves (TRAV 26x / 27x): held to 80 VGPRs, 6 waves per SIMD
// (83 unconstrained: 5 waves)
#ifndef PT_TRACE_PRE_WAVES
#define PT_TRACE_PRE_WAVES 6
#endif
template <bool LDS, int TRAV, bool COUNT, uint32_t RING = kHitRing, int PRUN = 4>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(PT_TRACE_PRE_WAVES, 8))) void k_wf_trace_pre(
    SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out, uint32_t watchdog, int sparse) {
    wf_trace_body<LDS, TRAV, COUNT, RING, PRUN>(sc, wb, in_q, cnt_out, watchdog, sparse);
}

// Brute force + replay: the closest-hit kernel for mailbox scenes (SceneView::mailbox: at most
// 64 distinct leaf entries, e.g. every Cornell box).  The reference's traversal (and the
// mailboxed one, trav_step_mb) tests ~19 of CornellBox's 36 distinct entries per query, in an
// order and number that differ from lane to lane, so SIMT lanes idle in each other's leaf
// loops (~30 % of the issued test slots do work).  Here a wave takes 64 queue entries at once
// and
//   phase 1  runs the triangle test of EVERY distinct entry u for all 64 rays in lockstep
//            (wave-uniform loop; the record is uniform, read through the scalar cache), keeping
//            per ray the set of entries hit and the t of the first kBfSlots hits (LDS);
//   phase 2  replays the reference's traversal per ray — node steps, exit-distance pruning,
//            the mailboxed leaf pairs of trav_step_mb — where a leaf entry costs a mask test
//            and, for entries that hit, a lookup of its t instead of a triangle test.
// Exact: a triangle test is a pure function of (ray, record), so phase 1 computes the same t
// (and hit predicate) the traversal would, and phase 2 applies them in the mailboxed order
// with the same strict-< update, tie-break and pruning; tests of entries the traversal never
// reaches have no effect.  A ray with more than `nslots` (<= kBfSlots) hits recomputes the rest on demand.
constexpr int kBfSlots = 8;
__device__ __forceinline__ TriRec load_tri_scalar(const Tri* tris, int i) {
    // uniform index: constant address space, so the record comes through s_load (no VGPRs)
    const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(tris + i);
    return TriRec{make_float4(f[0], f[1], f[2], f[3]), make_float4(f[4], f[5], f[6], f[7]), f[8]};
}

// Phase 2 without a stack (SceneView::bfnode; scenes of <= 64 internal nodes, <= 63 entries).
// The reference's traversal visits nodes depth first, right child before left (a node with both
// children to visit keeps the left one on its stack), and a child's visit is decided when its
// parent is visited (the exit-distance test against the closest t at that moment).  With the
// internal nodes numbered in that visiting order (pre-order, right subtree first; pt_capi.hip
// build_layout), the node the stack walk takes next is always the smallest-numbered node
// decided but not yet visited: a stacked left child of an ancestor comes after everything below
// that ancestor's right child, and the current node's children come after it but before every
// stacked node.  So a 64-bit set of pending nodes walked by ctz replaces the stack, visiting the
// same nodes in the same order with the same decisions: the same leaf pairs, resolved exactly as
// in the stack walk below (mailbox set, phase 1's t, strict < with the pair's tie-break).
__device__ __forceinline__ bool mb_first_node(const SceneView& sc, int node, bool li, bool ri, int a, int b) {
    const int4 d = reinterpret_cast<const int4*>(sc.nodes)[4 * node + 3];
    const int na = (li & (d.z >= 0)) ? d.z : 0;
    const int nt = na + ((ri & (d.w >= 0)) ? d.w : 0);
    for (int k = 0; k < nt; ++k) {
        const int u = sc.tris[k < na ? d.x + k : d.y + (k - na)].uid;
        if (u == a || u == b) return u == a;
    }
    return false;
}

template <bool FAST_RCP>
__device__ __forceinline__ int bf_replay_stackless(const SceneView& sc, const Ray& r, bool active, uint64_t hits,
                                                   float tmin, const float* slot, int nslots, float& t_out PH_PARAM) {
    constexpr uint64_t kInner = 1ull << 63;
    uint64_t pend = active ? 1ull : 0ull;  // pre-order node 0 = the root
    uint64_t tested = 0;
    int best = -1;
    float best_t = -1.0f;
    while (wave_any(pend != 0)) {
        if (pend != 0) {
            PH_ITER(PH_REPLAY);
            const int n = (int)__builtin_ctzll(pend);
            pend &= pend - 1;
            const BfNode& bn = sc.bfnode[n];
            const float ld = ray_box(r, bn.lmin[0], bn.lmin[1], bn.lmin[2], bn.lmax[0], bn.lmax[1], bn.lmax[2]);
            const float rd = ray_box(r, bn.rmin[0], bn.rmin[1], bn.rmin[2], bn.rmax[0], bn.rmax[1], bn.rmax[2]);
            const bool li = 0.0f < ld, ri = 0.0f < rd;
            const bool lint = (bn.lm & kInner) != 0, rint = (bn.rm & kInner) != 0;
            const uint64_t m = ((li & !lint) ? bn.lm : 0ull) | ((ri & !rint) ? bn.rm : 0ull);
            uint64_t rh = m & ~tested & hits;
            tested |= m;
            bool bcur = false;  // the best came from this leaf pair
            while (rh) {
                PH_ITER(PH_RLEAF);
                const int u = (int)__builtin_ctzll(rh);
                rh &= rh - 1;
                const int k = __popcll(hits & ((1ull << u) - 1));
                const int rec = sc.mb_base + u;
                float t;
                if (k < nslots) t = slot[64 * k];
                else tri_hit<FAST_RCP>(sc.tris, rec, r, t);  // a hit, so the same t as phase 1
                bool take = (best_t < 0.0f) | (t < best_t);
                if ((t == best_t) & bcur) take = mb_first_node(sc, sc.bfmap[n], li, ri, u, best - sc.mb_base);
                best_t = take ? t : best_t;
                best = take ? rec : best;
                bcur |= take;
            }
            if (best_t == tmin) {
                pend = 0;
            } else {
                const bool tl = (li & lint) && !((best_t > 0.0f) & (ld > best_t));
                const bool tr = (ri & rint) && !((best_t > 0.0f) & (rd > best_t));
                pend |= (tl ? 1ull << (uint32_t)(bn.lm & 63u) : 0ull) | (tr ? 1ull << (uint32_t)(bn.rm & 63u) : 0ull);
            }
        }
    }
    t_out = best_t;
    return best;
}

// Camera batches (CAM: every ray of the batch starts at the camera, fp.cam — the fused kernel's GEN
// launch): the parts of the triangle test that depend on the origin and the entry only — s = o - v0,
// s x e1 and e2 . (s x e1) — are the same for every camera ray, so k_wf_camtab computes them once
// per render per entry, with the same functions in the same order (so the same bits), and phase 1
// reads them through the scalar cache: camtab[2u] = (s, e2 . (s x e1)), camtab[2u + 1] = (s x e1, 0).
__global__ void k_wf_camtab(SceneView sc, FrameParams fp, float4* camtab) {
    const int u = (int)threadIdx.x;
    if (u >= sc.n_tris - sc.mb_base) return;
    const TriRec tr = load_tri(sc.tris, sc.mb_base + u);
    const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z), e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
    const f3 o = mk(fp.cam[0], fp.cam[1], fp.cam[2]);  // camera_ray's origin
    const f3 sv = o - v0;
    const f3 sce1 = cross(sv, e1);
    camtab[2 * u] = make_float4(sv.x, sv.y, sv.z, dot(e2, sce1));
    camtab[2 * u + 1] = make_float4(sce1.x, sce1.y, sce1.z, 0.0f);
}

// Closest hit of the 64 rays of one batch (lane = ray; `valid` false lanes give no hit):
// phase 1 + phase 2 above.  Returns the record (or -1) and its t in t_out.
template <bool FAST_RCP, bool COUNT, bool CAM = false>
__device__ __forceinline__ int bf_closest(const SceneView& sc, const Tri* gtris, const Ray& r, bool valid, float* slot,
                                          int nslots, const LStack32& stack, Counters& c, float& t_out,
                                          const float4* camtab PH_PARAM) {
    const int U = sc.n_tris - sc.mb_base;
    // phase 1: every distinct entry against all 64 rays.  The test is tri_hit's arithmetic cut
    // after u: when no lane passes the det and u tests (the early-out chain of
    // ray-triangle-intersection.wgsl:15-24) the rest cannot make a hit and is skipped for the wave
    uint64_t hits = 0;
    int nh = 0;
    const uint64_t vmask = __builtin_amdgcn_ballot_w64(valid);  // loop-invariant part of phase 1's vote
    float tmin = 3.0e38f;  // smallest t of any entry this ray hits
    for (int u = 0; u < U; ++u) {
        PH_ITER(PH_P1);
        const TriRec tr = load_tri_scalar(gtris, sc.mb_base + u);
        const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z), e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
        float4 ca = make_float4(0, 0, 0, 0);
        if constexpr (CAM) {
            const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(camtab + 2 * u);
            ca = make_float4(f[0], f[1], f[2], f[3]);
        }
        const f3 rce2 = cross(r.d, e2);
        const float det = dot(e1, rce2);
        const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
        const f3 sv = CAM ? mk(ca.x, ca.y, ca.z) : r.o - v0;
        const float bu = inv_det * dot(sv, rce2);
        const bool ok_det = !(det > -1e-8f && det < 1e-8f), ok_lo = !(bu < 0.0f), ok_hi = !(bu > 1.0f);
        const bool ok_u = valid & ok_det & ok_lo & ok_hi;
        // the vote as SGPR masks of the single compares (one ballot of the combined bool costs
        // two VALU slots per entry: v_cndmask + v_cmp)
        if ((vmask & __builtin_amdgcn_ballot_w64(ok_det) &
             __builtin_amdgcn_ballot_w64(ok_lo) & __builtin_amdgcn_ballot_w64(ok_hi)) == 0)
            continue;  // wave-uniform
        PH_ITER(PH_P1FULL);
        f3 sce1;
        float tn;
        if constexpr (CAM) {
            const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(camtab + 2 * u + 1);
            sce1 = mk(f[0], f[1], f[2]);
            tn = ca.w;
        } else {
            sce1 = cross(sv, e1);
            tn = dot(e2, sce1);
        }
        const float bv = inv_det * dot(r.d, sce1);
        const float t = inv_det * tn;
        const bool h = ok_u & !(bv < 0.0f) & !(bu + bv > 1.0f) & (t > 1e-8f);
        if (h) {
            if (nh < nslots) slot[64 * nh] = t;
            ++nh;
            hits |= 1ull << u;
            tmin = t < tmin ? t : tmin;  // = fminf here (t > 1e-8, never NaN) without its two canonicalising v_max
        }
    }
    // phase 2: the mailboxed traversal, leaf entries resolved from phase 1.  Without counters a
    // ray stops as soon as its closest t equals tmin: no later entry has a smaller t, and an
    // equal one can only win inside the pair just resolved (strict-< across pairs) — so the
    // result is final; a ray that hits nothing at all is final at once.  The counting build
    // (COUNT) walks on, to count the reference's work.
#if PT_PHASE_STATS
    {
        const uint64_t t1 = ph_now();
        pa.v[PH_P1][0] += t1 - pa.v[PH_COUNT][0];  // (the slot holds phase 1's start: set by the caller)
        pa.v[PH_COUNT][0] = t1;
    }
#endif
    if constexpr (!COUNT) {
        if (sc.bfnode) {  // wave-uniform: the stackless walk (bf_replay_stackless)
            return bf_replay_stackless<FAST_RCP>(sc, r, valid && hits != 0, hits, tmin, slot, nslots, t_out PH_PASS);
        }
    }
    TravLean s;
    trav_init(s, valid && (COUNT || hits != 0));
    while (wave_any(!trav_finished(s))) {
        if (!trav_finished(s)) {
            mb_node_unit<COUNT>(sc, r, s, c);
            uint64_t rh = s.rem & hits;
            while (rh) {
                const int u = (int)__builtin_ctzll(rh);
                rh &= rh - 1;
                const int k = __popcll(hits & ((1ull << u) - 1));
                const int rec = sc.mb_base + u;
                float t;
                if (k < nslots) t = slot[64 * k];
                else tri_hit<FAST_RCP>(sc.tris, rec, r, t);  // a hit, so the same t as phase 1
                bool take = (s.best_t < 0.0f) | (t < s.best_t);
                if ((t == s.best_t) & ((s.fl & TF_BCUR) != 0)) take = mb_first(sc, s, u, s.best - sc.mb_base);
                s.best_t = take ? t : s.best_t;
                s.best = take ? rec : s.best;
                s.fl |= take ? TF_BCUR : 0;
            }
            s.rem = 0;
            s.fl &= ~TF_LEAF;
            if (!COUNT && s.best_t == tmin) s.fl |= TF_DONE;
            else lean_decide(s, stack);
        }
    }
    t_out = s.best_t;
    return s.best;
}

// LDS of the bf kernels: per-lane stacks, then per wave kBfSlots x 64 hit slots, then the scene
struct BfLds {
    LStack32 stack;
    float* slot;
    char* scene;
};
__device__ __forceinline__ BfLds bf_lds(char* smem, const SceneView& sc) {
    BfLds l;
    l.stack = LStack32::make(smem, blockDim.x);
    char* slot_base = smem + (uint32_t)sc.max_stack * blockDim.x * 4u;
    l.slot = reinterpret_cast<float*>(slot_base) + (threadIdx.x / 64u) * (kBfSlots * 64) + lane_id();  // slot k: slot[64k]
    l.scene = slot_base + (blockDim.x / 64u) * (kBfSlots * 64 * 4);
    return l;
}

template <bool LDS, bool FAST_RCP, bool COUNT>
__global__ __launch_bounds__(kTraceBlock) void k_wf_trace_bf(SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out, int nslots) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const BfLds l = bf_lds(smem, sc);
    const uint32_t lane = lane_id();
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1] = 0;  // shade's output count
    const uint32_t count = wb.ctl[WF_WATCHDOG] ? 0u : wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];
    const Tri* gtris = sc.tris;  // global records for phase 1
    if (LDS) stage_scene_lds(sc, l.scene);
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    const uint32_t nb = (count + 63) / 64;
    const float4* q = in_q ? wb.shd.ray : wb.ext.ray;
    Counters c = {};
    for (uint32_t b = w; b < nb; b += nwaves) {  // batches of 64 entries, interleaved over waves
        const uint32_t e = b * 64 + lane;
        const bool valid = e < count;
        uint32_t p;
        const Ray r = unpack_ray(valid ? q[2 * (size_t)e] : make_float4(0, 0, 0, 1),
                                 valid ? q[2 * (size_t)e + 1] : make_float4(0, 0, 0, 0), p);
        float t;
#if PT_PHASE_STATS
        PhaseAcc pa{};
#endif
        const int rec = bf_closest<FAST_RCP, COUNT>(sc, gtris, r, valid, l.slot, nslots, l.stack, c, t, nullptr PH_PASS);
        if (valid) wb.hitq[e] = make_int2(rec, __builtin_bit_cast(int, t));
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// One batch of 64 entries of queue `in` (EXT: extension rays, else shadow rays) at entries
// rbase + b * 64 + lane (valid: b * 64 + lane < count): bf_closest, then the path logic of
// k_wf_shade (pt_path.h, so the same bits) in the same wave — the hit never goes through HBM
// and the ray record is read once — and the survivors appended to region rbase of the other
// queue at offsets from `append(n)` (wave-uniform: called by lane 0, result broadcast).
// GEN (the first extension launch, k_wf_step_bf's GEN): the batch's camera paths are made here
// instead of read from the queue — path p = (b * R + region) * 64 + lane, k_wf_generate's
// layout — and packed into the very words store_entry would have written, so everything after
// reads the same bits as from the queue (the queue write and read of the camera rays saved).
// Camera batches: region rg's k-th camera batch is the 64 paths (k * R + rg) * 64 + lane < P.
struct GenArgs {
    uint32_t frame0, stride, fbase, R, rg, P;
    bool raw_salt;
};
// genk (GEN instances; wave-uniform): >= 0 makes this batch camera batch genk of the region
// instead of queue batch b (the first launch); -1 reads the queue.
// CAM: the batch's rays are camera rays (a fresh batch of the first launch: bf_closest's table)
template <bool EXT, bool FAST_RCP, bool COUNT, bool GEN = false, bool CAM = GEN, class Append>
__device__ __forceinline__ void bf_step_batch(const SceneView& sc, const Tri* gtris, const FrameParams& fp,
                                              const WfBuffers& wb, size_t rbase, uint32_t b, uint32_t count,
                                              const BfLds& l, int nslots, Counters& c, Append append,
                                              const GenArgs& gen, int64_t genk PH_PARAM) {
#if PT_PHASE_STATS
    const uint64_t t0 = ph_now();
#endif
    const WfQueue& in = EXT ? wb.ext : wb.shd;
    const WfQueue& out = EXT ? wb.shd : wb.ext;
    const uint32_t lane = lane_id();
    const bool fresh = GEN && genk >= 0;
    const uint32_t pg = fresh ? ((uint32_t)genk * gen.R + gen.rg) * 64 + lane : 0u;
    const bool valid = fresh ? pg < gen.P : b * 64 + lane < count;
    const size_t e = rbase + ((valid && !fresh) ? b * 64 + lane : 0);
    float4 a0 = make_float4(0, 0, 0, 1), a1 = make_float4(0, 0, 0, 0);
    float4 c2 = make_float4(0, 0, 0, 0), d3 = c2;
    if (fresh) {
        if (valid) {
            uint32_t x, y, f;
            const uint32_t pid = slot_path(pg, fp, x, y, f);  // pg: the generation slot
            const uint32_t tt = gen.raw_salt ? gen.frame0 : (uint32_t)(float)(gen.frame0 + (gen.fbase + f) * gen.stride);
            PathState g;
            const Ray gr = path_begin(fp, x, y, tt, g);
            a0 = make_float4(gr.o.x, gr.o.y, gr.o.z, gr.d.x);
            a1 = make_float4(gr.d.y, gr.d.z, __builtin_bit_cast(float, pid), __builtin_bit_cast(float, pack_dspec(g)));
            c2 = make_float4(g.L.x, g.L.y, g.L.z, __builtin_bit_cast(float, g.seed));
            d3 = make_float4(g.beta.x, g.beta.y, g.beta.z, 0.0f);
            if (COUNT) { c.samples++; c.ext_queries++; }
        }
    } else if (EXT) {
        a0 = in.ray[2 * e];
        a1 = in.ray[2 * e + 1];
        if (!valid) { a0 = make_float4(0, 0, 0, 1); a1 = make_float4(0, 0, 0, 0); }
    }
    uint32_t p;
    Ray r;
    if (EXT || fresh) {
        r = unpack_ray(a0, a1, p);
    } else {  // packed shadow entry (store_shadow_packed): the origin from the shading point (its
              // words are read again after the trace, from cache, rather than held across it)
        a0 = valid ? in.ray[2 * e] : make_float4(0, 0, 1, 0);
        r = unpack_shadow_ray(a0, valid ? in.q3[e] : make_float4(0, 0, 0, 0),
                              valid ? wb.sp0[e] : make_float4(0, 0, 0, 0), p);
    }
    // the path state is loaded before the trace and arrives while it runs (+1.3 %)
    if (!fresh) {
        if (EXT) { c2 = in.q2[e]; d3 = in.q3[e]; }
        else { a1 = in.ray[2 * e + 1]; c2 = in.q2[e]; }
    }
    float t;
#if PT_PHASE_STATS
    {
        const uint64_t t1 = ph_now();
        pa.v[PH_LOAD][0] += t1 - t0;
        pa.v[PH_COUNT][0] = t1;  // phase 1's start, for bf_closest
    }
#endif
    // CAM: a camera batch (the first launch reads no queue: genk >= 0 throughout)
    const int rec = bf_closest<FAST_RCP, COUNT, CAM>(sc, gtris, r, valid, l.slot, nslots, l.stack, c, t, wb.camtab PH_PASS);
#if PT_PHASE_STATS
    uint64_t t3 = ph_now();
    pa.v[PH_REPLAY][0] += t3 - pa.v[PH_COUNT][0];
    PH_ITER(PH_SHADE);  // the lanes entering the path logic (all of the batch's)
#endif
    bool more = false;
    PathState ps;
    if (valid) {
        if (EXT) {
            unpack_dspec(__builtin_bit_cast(uint32_t, a1.w), ps);
            ps.L = mk(c2.x, c2.y, c2.z);
            ps.seed = __builtin_bit_cast(uint32_t, c2.w);
            ps.beta = mk(d3.x, d3.y, d3.z);
            more = path_after_ext(sc, rec, t, r, ps);
            if (more && COUNT) c.shadow_queries++;
        } else {  // packed shadow entry
            unpack_dspec(__builtin_bit_cast(uint32_t, a1.x), ps);
            ps.L = mk(a1.y, a1.z, a1.w);
            ps.seed = __builtin_bit_cast(uint32_t, c2.x);
            ps.beta = mk(c2.y, c2.z, c2.w);
            const float4 h3 = in.q3[e], n4 = wb.sp0[e];
            ps.hp = mk(h3.x, h3.y, h3.z);
            ps.mat_id = __builtin_bit_cast(int, h3.w);
            const float2 w2 = wb.sp2[e];
            ps.hn = mk(n4.x, n4.y, n4.z);
            ps.wi = mk(n4.w, w2.x, w2.y);
            more = path_after_shadow(sc, fp, rec, t, r, ps);
            if (more && COUNT) c.ext_queries++;
        }
        if (!more) {
            float* o = wb.rad + 3 * (size_t)p;
            o[0] = ps.L.x; o[1] = ps.L.y; o[2] = ps.L.z;
        }
    }
#if PT_PHASE_STATS
    {
        const uint64_t t4 = ph_now();
        pa.v[PH_SHADE][0] += t4 - t3;
        t3 = t4;
    }
#endif
    const uint64_t keep = __ballot(more);
    if (keep) {  // wave-uniform
        uint32_t base = 0;
        if (lane == 0) base = append((uint32_t)__popcll(keep));
        base = __shfl(base, 0, 64);
        if (more) {
            PH_ITER(PH_APPEND);
            const uint32_t j = (uint32_t)rbase + base + rank_below(keep);
            if (EXT) store_shadow_packed(wb, j, r, p, ps);
            else store_entry(out, j, r, p, ps);
        }
    }
#if PT_PHASE_STATS
    pa.v[PH_APPEND][0] += ph_now() - t3;
#endif
}

// Trace + shade in one launch per iteration (mailbox scenes): queues are cut
// into wb.nreg regions (64-path batches dealt round-robin: camera batch j to region j mod nreg);
// the waves w ≡ r (mod nreg) serve region r of the input and append to region r of the output,
// one atomicAdd per wave and batch on that region's counter (a counter shared by all waves
// serialises at one memory channel, and each wave waits for its add: measured 2x slower).  A
// region's output never exceeds its input, so every region holds its paths through all
// bounces.  Iteration `it` reads the counts of slot it % 3, appends to slot (it + 1) % 3 and
// zeroes slot (it + 2) % 3 for iteration it + 1 (iteration it - 1 read that slot and it - 2
// wrote it, both finished: stream order).
// amdgpu_waves_per_eu(8): the path logic pushed the kernel to 75 VGPRs (6 waves/SIMD); capped
// at 64 it keeps 8 waves/SIMD with no VGPR spills (a few SGPR spills to VGPR lanes): +7 %
// GEN: the first launch makes the camera paths itself (bf_step_batch GEN; replaces
// k_wf_generate): region counts in closed form, the output counts zeroed by the host.
// GEN 2 (option regen = q): streaming regeneration — every extension launch j = it / 2 also admits
// the region's camera batches j q .. (j + 1) q - 1 behind its queued survivors, so the launches stay
// full until the camera batches run out (the host launches 2 (ceil(max camera batches / q) +
// max_depth) iterations).  Those launches mix queued and camera batches: no camera table.
template <bool EXT, bool LDS, bool FAST_RCP, bool COUNT, int GEN = 0>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_wf_step_bf(SceneView sc, FrameParams fp, WfBuffers wb, int it,
                                                           Counters* cnt_out, int nslots, uint32_t frame0,
                                                           uint32_t stride, uint32_t fbase, uint32_t P, bool raw_salt,
                                                           uint32_t q) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const BfLds l = bf_lds(smem, sc);
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    const uint32_t R = wb.nreg;  // <= nwaves (host)
    const uint32_t rg = w % R, g = w / R, G = (nwaves - rg + R - 1) / R;
    if (g == 0 && lane_id() == 0) wb.rcnt[((it + 2) % 3) * kRegions + rg] = 0;
    const uint32_t nbat = (P + 63) / 64;
    const uint32_t tg = (uint32_t)((uint64_t)rg * wb.rq % R);  // region rg's camera batches: tg, tg + R, ...
    const uint32_t ncam = tg < nbat ? (nbat - tg + R - 1) / R : 0u;
    uint32_t count, nqb, nnew = 0, k0 = 0;
    if constexpr (GEN == 1) {  // the first launch: every camera batch of region rg
        const uint32_t last = tg + (ncam - 1) * R;
        count = ncam == 0 ? 0u : ncam * 64 - ((last == nbat - 1 && (P & 63)) ? 64 - (P & 63) : 0u);
        if (w == 0 && lane_id() == 0) { wb.ctl[WF_COUNT0] = P; wb.ctl[WF_COUNT1] = 0; }
        nqb = 0;
        nnew = ncam;
    } else if constexpr (GEN == 2) {  // queued survivors (none in the first launch), then admissions
        count = it == 0 ? 0u : wb.rcnt[(it % 3) * kRegions + rg];
        nqb = (count + 63) / 64;
        k0 = (uint32_t)(it / 2) * q;
        nnew = ncam > k0 ? min(q, ncam - k0) : 0u;
        if (it == 0 && w == 0 && lane_id() == 0) { wb.ctl[WF_COUNT0] = P; wb.ctl[WF_COUNT1] = 0; }
    } else {
        count = wb.rcnt[(it % 3) * kRegions + rg];
        nqb = (count + 63) / 64;
    }
    uint32_t* out_count = &wb.rcnt[((it + 1) % 3) * kRegions + rg];
    const Tri* gtris = sc.tris;  // global records for phase 1
    if (LDS) stage_scene_lds(sc, l.scene);
    const uint32_t nb = nqb + nnew;
    const GenArgs ga{frame0, stride, fbase, R, tg, P, raw_salt};
    Counters c = {};
#if PT_PHASE_STATS
    PhaseAcc pa{};
#endif
    for (uint32_t b = g; b < nb; b += G)  // this region's batches, interleaved over its waves
        bf_step_batch<EXT, FAST_RCP, COUNT, GEN != 0, GEN == 1>(sc, gtris, fp, wb, (size_t)rg * wb.rstride, b, count, l,
                                                                nslots, c, [&](uint32_t n) { return atomicAdd(out_count, n); },
                                                                ga, b < nqb ? (int64_t)-1 : (int64_t)(k0 + b - nqb) PH_PASS);
    if (COUNT) flush_counters(c, cnt_out);
#if PT_PHASE_STATS
    if (!COUNT && lane_id() == 0) {
        pa.v[PH_COUNT][0] = 0;  // (the scratch slot)
        for (int ph = 0; ph < PH_COUNT; ++ph)
            for (int f = 0; f < 3; ++f) atomicAdd(&g_phase_stats[EXT ? 1 : 0][ph][f], (unsigned long long)pa.v[ph][f]);
    }
#endif
}

// Shade blocks are 1024 threads so that compaction takes one atomicAdd per 1024 entries: all
// atomics on the queue counter serialise at one memory channel, and one per wave (131k per
// 8M-path batch) cost more than the shading itself.
constexpr uint32_t kShadeBlock = 1024;

template <bool EXT, bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void k_wf_shade(SceneView sc, FrameParams fp, WfBuffers wb, Counters* cnt_out,
                                                          int bins) {
    // EXT: extension queue -> shadow queue; else shadow queue -> extension queue
    const uint32_t count = wb.ctl[EXT ? WF_COUNT0 : WF_COUNT1];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x * blockDim.x >= count) return;  // whole block past the queue
    const WfQueue& in = EXT ? wb.ext : wb.shd;
    const WfQueue& out = EXT ? wb.shd : wb.ext;
    uint32_t* out_count = &wb.ctl[EXT ? WF_COUNT1 : WF_COUNT0];
    Counters c = {};
    bool more = false;
    uint32_t p = 0;
    Ray r;
    PathState ps;
    if (i < count) {
        r = load_entry(in, i, p, ps);
        const int2 h = wb.hitq[i];
        const float t = __builtin_bit_cast(float, h.y);
        // a trace that gave up (watchdog, reported by the host) leaves stale records: never
        // let one index outside the triangle array
        const int rec = (uint32_t)h.x < (uint32_t)sc.n_tris ? h.x : -1;
        if (EXT) {
            more = path_after_ext(sc, rec, t, r, ps);
            if (more && COUNT) c.shadow_queries++;
        } else {
            load_shading_point(wb, i, ps);
            more = path_after_shadow(sc, fp, rec, t, r, ps);
            if (more && COUNT) c.ext_queries++;
        }
        if (!more) {
            float* o = wb.rad + 3 * (size_t)p;
            o[0] = ps.L.x; o[1] = ps.L.y; o[2] = ps.L.z;
        }
    }
    // compaction of the surviving paths: wave counts -> LDS prefix -> one atomicAdd per block
    __shared__ uint32_t s_cnt[kShadeBlock / 64];
    const uint64_t keep = __ballot(more);
    const uint32_t wv = threadIdx.x / 64;
    if (bins > 1) {  // block-uniform (kernel argument): the block's survivors grouped by a
        // coherence key (PT_SORT): the octant of the new direction (bins = 8), and with bins = 64
        // also the octant of the origin about the scene box's centre.  The block's output stays
        // one contiguous chunk (one atomicAdd), ordered key by key, so the traversal's 32-entry
        // windows hold similar rays.  Only the queue order changes (ranks within a key come from
        // LDS atomics, in any order): every path's result is the same.
        __shared__ uint32_t s_bin[512];
        for (uint32_t b = threadIdx.x; b < 512; b += blockDim.x) s_bin[b] = 0;
        uint32_t key = (r.d.x < 0.0f ? 1u : 0u) | (r.d.y < 0.0f ? 2u : 0u) | (r.d.z < 0.0f ? 4u : 0u);
        if (bins > 8) {  // the origin's cell: octant of the scene box (64 keys) or 4 x 4 x 4 cells (512)
            const Node& root = sc.nodes[0];
            const float lx = fminf(root.lmin[0], root.rmin[0]), hx = fmaxf(root.lmax[0], root.rmax[0]);
            const float ly = fminf(root.lmin[1], root.rmin[1]), hy = fmaxf(root.lmax[1], root.rmax[1]);
            const float lz = fminf(root.lmin[2], root.rmin[2]), hz = fmaxf(root.lmax[2], root.rmax[2]);
            const float q = bins > 64 ? 4.0f : 2.0f;
            auto cell = [&](float v, float lo, float hi) {
                const float c = (v - lo) / fmaxf(hi - lo, 1e-30f) * q;
                return (uint32_t)fminf(fmaxf(c, 0.0f), q - 1.0f);  // NaN -> 0
            };
            const uint32_t sh = bins > 64 ? 2u : 1u;
            key |= (cell(r.o.x, lx, hx) | (cell(r.o.y, ly, hy) << sh) | (cell(r.o.z, lz, hz) << (2 * sh))) << 3;
        }
        __syncthreads();
        const uint32_t rank = more ? atomicAdd(&s_bin[key], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the key counts, 8 per lane
            uint32_t c8[8], n = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) { c8[i] = s_bin[8 * threadIdx.x + i]; n += c8[i]; }
            uint32_t incl = n;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t v = __shfl_up(incl, off, 64);
                if (lane_id() >= (uint32_t)off) incl += v;
            }
            const uint32_t total = __shfl(incl, 63, 64);
            uint32_t base = 0;
            if (threadIdx.x == 0 && total) base = atomicAdd(out_count, total);
            base = __shfl(base, 0, 64);
            uint32_t run = base + incl - n;
#pragma unroll
            for (int i = 0; i < 8; ++i) { s_bin[8 * threadIdx.x + i] = run; run += c8[i]; }
        }
        __syncthreads();
        if (more) {
            const uint32_t j = s_bin[key] + rank;
            store_entry(out, j, r, p, ps);
            if (EXT) store_shading_point(wb, j, ps);
        }
        if (COUNT) flush_counters(c, cnt_out);
        return;
    }
    if (lane_id() == 0) s_cnt[wv] = (uint32_t)__popcll(keep);
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t n = threadIdx.x < kShadeBlock / 64 ? s_cnt[threadIdx.x] : 0u;
        uint32_t incl = n;  // inclusive scan of the wave counts
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(incl, off, 64);
            if (lane_id() >= (uint32_t)off) incl += v;
        }
        const uint32_t total = __shfl(incl, 63, 64);
        uint32_t base = 0;
        if (threadIdx.x == 0 && total) base = atomicAdd(out_count, total);
        base = __shfl(base, 0, 64);
        if (threadIdx.x < kShadeBlock / 64) s_cnt[threadIdx.x] = base + incl - n;
    }
    __syncthreads();
    if (more) {
        const uint32_t j = s_cnt[wv] + rank_below(keep);
        store_entry(out, j, r, p, ps);
        if (EXT) store_shading_point(wb, j, ps);
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// acc += clamp(radiance) for the batch's frames in order (program-raymarch.ts:283-285)
__global__ __launch_bounds__(256) void k_wf_accum(const float* __restrict__ rad, float* __restrict__ acc, uint32_t npix,
                                                  uint32_t F, bool accumulate) {
    const uint32_t pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= npix) return;
    float* o = acc + 3 * (size_t)pix;
    f3 a = accumulate ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);
    for (uint32_t f = 0; f < F; ++f) {
        const float* r = rad + 3 * ((size_t)f * npix + pix);
        f3 L = mk(r[0], r[1], r[2]);
        a = accumulate ? add_clamped(a, L) : L;
    }
    o[0] = a.x; o[1] = a.y; o[2] = a.z;
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
#define HIP_RETURN_IF(expr)                      \
    do {                                         \
        const hipError_t e_ = (expr);            \
        if (e_ != hipSuccess) return e_;         \
    } while (0)
// TRAV >= 300: the brute-force + replay kernel (k_wf_trace_bf; + 10: fast reciprocal); >= 400: fused
// with the shading (k_wf_step_bf)
template <bool LDS, int TRAV, bool COUNT, uint32_t RING = kHitRing, int PRUN = 4>
constexpr const void* trace_kernel() {
    if constexpr (TRAV >= 400) return (const void*)k_wf_step_bf<false, LDS, ((TRAV / 10) & 1) != 0, COUNT>;
    else if constexpr (TRAV >= 300) return (const void*)k_wf_trace_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>;
    else if constexpr (TRAV >= 260) return (const void*)k_wf_trace_pre<LDS, TRAV, COUNT, RING, PRUN>;
    else return (const void*)k_wf_trace<LDS, TRAV, COUNT, RING, PRUN>;
}
// the k_wf_trace instances with a 256-entry ring and with pooled runs of 2 (SceneView::leaf_pool
// == 2): the default flavours, uncounted (the others pool runs of 4: the same bits and counts)
template <int TRAV, bool COUNT>
constexpr bool has_variants() { return TRAV < 300 && has_big_ring(TRAV) && !COUNT; }
template <bool LDS, int TRAV, bool COUNT>
static const void* trace_instance(uint32_t ring, bool run2) {
    if constexpr (has_variants<TRAV, COUNT>()) {
        if (ring == kHitRingMax)
            return run2 ? trace_kernel<LDS, TRAV, COUNT, kHitRingMax, 2>() : trace_kernel<LDS, TRAV, COUNT, kHitRingMax>();
        if (run2) return trace_kernel<LDS, TRAV, COUNT, kHitRing, 2>();
    }
    (void)ring;
    (void)run2;
    return trace_kernel<LDS, TRAV, COUNT>();
}
template <bool LDS, int TRAV, bool COUNT>
static size_t trace_lds(const SceneView& sc, uint32_t ring = kHitRing) {
    const size_t span = LDS ? sc.span_bytes : 0;
    if (TRAV >= 300) return (size_t)sc.max_stack * kTraceBlock * 4 + (kTraceBlock / 64) * ((size_t)kBfSlots * 64 * 4) + span;
    return (size_t)sc.max_stack * 4 * kTraceBlock + (kTraceBlock / 64) * (stage_bytes(ring) + (keys_on<TRAV>(sc) ? kKeyBytes : 0)) + span;
}
// resident blocks of `kernel` per CU at `lds` bytes of dynamic LDS, times the CUs: the persistent
// grid of the trace and step kernels (cached per kernel instance and LDS size)
static int occupancy_blocks(const void* kernel, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(kernel, lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int per_cu = 0, dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kTraceBlock, lds);
    const int b = std::max(1, per_cu) * std::max(1, cus);
    cache.emplace(key, b);
    return b;
}
static size_t max_block_lds() {
    static const size_t v = [] {
        int dev = 0, x = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&x, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
        return (size_t)x;
    }();
    return v;
}

// Paths [0, P) of part h of nparts of a batch: queue entries from h * qcap/nparts, radiance from
// `rad_off` floats (so the parts' radiance is contiguous in frame order), control words from
// h * WF_CTL_WORDS, region counts from h * 3 * kRegions.
static WfBuffers wb_part(const WfBuffers& wb, int h, int nparts, size_t rad_off) {
    WfBuffers v = wb;
    const size_t e = (size_t)h * (wb.qcap / nparts);
    for (WfQueue* q : {&v.ext, &v.shd}) { q->ray += 2 * e; q->q2 += e; q->q3 += e; }
    v.sp0 += e; v.sp1 += e; v.sp2 += e; v.hitq += e;
    if (v.pres) v.pres += e;  // per leaf b at b * pres_stride (the whole buffer's stride)
    v.rad += rad_off;
    v.ctl += h * WF_CTL_WORDS;
    v.rcnt += h * 3 * kRegions;
    v.capacity = wb.capacity / nparts;
    v.qcap = wb.qcap / nparts;
    return v;
}

// The brute-force kernels without counters replay without a stack when the scene has the BfNode
// tree (bf_replay_stackless): no per-lane stack in their LDS (CornellBox: 14 KB of a 512-thread
// block's 43 KB, so 4 blocks fit a CU's 160 KB instead of 3 — 8 waves per SIMD instead of 6).
template <int TRAV, bool COUNT>
static SceneView bf_view(const SceneView& sc) {
    SceneView v = sc;
    if (TRAV >= 300 && !COUNT && sc.bfnode) v.max_stack = 0;
    return v;
}

template <bool LDS, int TRAV, bool COUNT>
static hipError_t wf_render_t(const SceneView& sc_in, const FrameParams& fp, const WfBuffers& wb, uint32_t frame0,
                              uint32_t nframes, uint32_t stride, bool accum, float* out, Counters* cnt,
                              hipStream_t stream, const WfStreams& ws) {
    SceneView sc = bf_view<TRAV, COUNT>(sc_in);
    const uint32_t npix = fp.width * fp.height;
    // the batch in ws.nparts parts on as many streams when a part holds at least a frame: one
    // part's kernel fills the others' launch tails and boundaries (and, with separate trace and
    // shade kernels, a VALU-bound trace runs beside an HBM-bound shade)
    int np = ws.aux[0] != nullptr ? ws.nparts : 1;
    while (np > 1 && (nframes < (uint32_t)np || wb.capacity / np < npix)) np /= 2;
    const uint32_t F = np * std::max<uint32_t>(1, std::min<uint32_t>((nframes + np - 1) / np, (uint32_t)(wb.capacity / np / npix)));
    // k_wf_trace's instance: the 256-entry hit ring when its extra 8 KB per block cost no block per
    // CU (option trace_ring: 128 / 256 forces one)
    uint32_t nring = kHitRing;
    const bool run2 = sc.leaf_pool == 2;  // pooled runs of 2 (the has_variants instances)
    // turn policy of the lean traversal: 4 since the queues are grouped by coherence keys (in process:
    // Glossy +2.5 %, boat +1 %, 1M synthetic +1.8 % over 8; 1 = majority: -13 % in round 1); 1 for the
    // instances that pool runs of 2 (100k +5.2 %, 1M +5.3 % over 4, both orders:
    // profiles/r04ai_node_bias.log; with runs of 4 the bias is within noise, r04z_ab_node_bias.log).
    // Chosen from the instance launched (advisor r04: the counted and non-default flavours pool runs
    // of 4 whatever sc.leaf_pool says)
    if (sc.node_bias <= 0) sc.node_bias = (run2 && has_variants<TRAV, COUNT>()) ? 1 : 4;
    // node steps per node turn: 4 (in process over 1, same bits: Glossy +4.4 %, Glossy SAH +4.1 %, the boat
    // +4.1 %, boat SAH +10.3 %, synthetic 1k +3.2 %, 100k +1.5 %; 3/6/8 within or below; r06g/r06h_ab_*.log)
    if (sc.node_steps <= 0) sc.node_steps = 4;
    if constexpr (has_variants<TRAV, COUNT>()) {
        const size_t l1 = trace_lds<LDS, TRAV, COUNT>(sc, kHitRing), l2 = trace_lds<LDS, TRAV, COUNT>(sc, kHitRingMax);
        const bool fits = l2 <= max_block_lds() &&
                          (ws.trace_ring == (int)kHitRingMax ||
                           (ws.trace_ring <= 0 && occupancy_blocks(trace_instance<LDS, TRAV, COUNT>(kHitRingMax, run2), l2) >=
                                                      occupancy_blocks(trace_instance<LDS, TRAV, COUNT>(kHitRing, run2), l1)));
        if (fits) nring = kHitRingMax;
    }
    const size_t lds = trace_lds<LDS, TRAV, COUNT>(sc, nring);
    int tblocks = occupancy_blocks(trace_instance<LDS, TRAV, COUNT>(nring, run2), lds);
    if (ws.trace_blocks > 0) tblocks = std::min(tblocks, ws.trace_blocks);  // option wf_trace_blocks (tests)
    const int iters = 2 * (fp.max_depth + 1);
    // option trace_watchdog: tests of the failure report
    const uint32_t watchdog = ws.watchdog > 0 ? ws.watchdog : kTraceWatchdog;
    const int sparse = std::max(0, std::min(ws.trace_sparse, 1 << 20));
    // option bf_slots < kBfSlots: tests of the recompute path
    const int bf_slots = ws.bf_slots >= 0 ? std::min(kBfSlots, ws.bf_slots) : kBfSlots;
    if constexpr (TRAV >= 400) {  // the camera batches' table (k_wf_camtab), before every part's GEN launch
        if (ws.fuse_gen) {
            if (sc.n_tris - sc.mb_base > 64) return hipErrorInvalidValue;  // mailbox scenes: <= 64 entries
            hipLaunchKernelGGL(k_wf_camtab, dim3(1), dim3(64), 0, stream, sc, fp, wb.camtab);
        }
    }
    for (uint32_t fb = 0; fb < nframes; fb += F) {
        const uint32_t Fb = std::min(F, nframes - fb);
        // frames of the batch dealt to the parts in contiguous runs (part h: frames fb + f0[h] ..)
        struct Part { WfBuffers w; uint32_t fbase, P; hipStream_t st; };
        Part pv[kMaxParts];
        int nh = 0;
        uint32_t f0 = 0;
        for (int h = 0; h < np && f0 < Fb; ++h) {
            const uint32_t fh = std::min<uint32_t>((Fb + np - 1) / np, Fb - f0);
            pv[nh].w = np > 1 ? wb_part(wb, h, np, (size_t)f0 * npix * 3) : wb;
            pv[nh].fbase = fb + f0;
            pv[nh].P = fh * npix;
            pv[nh].st = np > 1 ? ws.aux[h] : stream;
            f0 += fh;
            ++nh;
        }
        if constexpr (TRAV >= 400) {  // region-partitioned queues (k_wf_step_bf)
            const uint32_t R = std::min<uint32_t>(kRegions, (uint32_t)tblocks * (kTraceBlock / 64));
            // region_perm: region r takes camera batches r q mod R (q ~ 0.618 R, coprime with R), so
            // the 8 waves of a block (8 neighbouring regions) work on batches far apart in the image
            uint32_t q = 1, qi = 1;
            if (ws.region_perm && R > 2) {
                auto gcd = [](uint32_t a, uint32_t b) { while (b) { const uint32_t t = a % b; a = b; b = t; } return a; };
                q = std::max<uint32_t>(1, (uint32_t)(R * 0.6180339887498949));
                while (gcd(q, R) != 1) ++q;
                qi = 1;
                while ((uint64_t)q * qi % R != 1) ++qi;  // R <= 512
            }
            for (int h = 0; h < nh; ++h) {
                pv[h].w.nreg = R;
                pv[h].w.rstride = pv[h].w.qcap / R / 64 * 64;  // R * rstride >= paths of the part (qcap slack)
                pv[h].w.rq = q;
                pv[h].w.rqi = qi;
            }
        }
        // the fused kernel's first launch makes the camera paths itself (GEN); it appends into
        // count slot 1, zeroed here (k_wf_generate zeroes it otherwise) — on the caller's stream
        // before the fork: on a part's stream the second part's memset waited ~0.5 ms for a CU slot
        // behind the first part's first launch, and the parts ran that far apart (a kernel trace of
        // the bench, r06m)
        const bool fgen = TRAV >= 400 && ws.fuse_gen;
        if (fgen)
            for (int h = 0; h < nh; ++h)
                HIP_RETURN_IF(hipMemsetAsync(pv[h].w.rcnt + kRegions, 0, kRegions * sizeof(uint32_t), stream));
        if (np > 1) {
            HIP_RETURN_IF(hipEventRecord(ws.fork, stream));
            for (int h = 0; h < nh; ++h) HIP_RETURN_IF(hipStreamWaitEvent(pv[h].st, ws.fork, 0));
        }
        // option regen (fused kernel, camera paths made in the kernel): q camera batches per region
        // admitted by each extension launch; regen_cam = the most camera batches of any region
        uint32_t regen_q = 0, regen_cam = 0;
        int iters_b = iters;
        if (TRAV >= 400 && fgen && ws.regen > 0) {
            for (int h = 0; h < nh; ++h) {
                const uint32_t nbat = (pv[h].P + 63) / 64;
                regen_cam = std::max(regen_cam, (nbat + pv[h].w.nreg - 1) / pv[h].w.nreg);
            }
            regen_q = (uint32_t)ws.regen;
            if (regen_q < regen_cam)  // J admitting launches, the last admission's paths need max_depth + 1 more
                iters_b = 2 * ((int)((regen_cam + regen_q - 1) / regen_q) + fp.max_depth);
            else
                regen_q = 0;  // one launch admits them all: the plain first launch
        }
        for (int h = 0; h < nh && !fgen; ++h)
            PT_LAUNCH(KID_WF_GENERATE, pv[h].st, (k_wf_generate<COUNT>),
                      dim3((std::max(pv[h].P, pv[h].w.nreg) + 255) / 256), dim3(256), 0, pv[h].st,
                      fp, pv[h].w, frame0, stride, pv[h].fbase, pv[h].P, !accum, cnt);
        // launch `it` of part h (in_q: the queue the trace kernels read, it & 1)
        auto step = [&](int h, int it) -> hipError_t {
            const int in_q = it & 1;
            const hipStream_t st = pv[h].st;
            const WfBuffers& w = pv[h].w;
            const int sblocks = (int)((pv[h].P + kShadeBlock - 1) / kShadeBlock);
            if constexpr (TRAV >= 400) {  // trace + shade in one launch
                constexpr bool rcp = ((TRAV / 10) & 1) != 0;
#define PT_STEP(E, G) PT_LAUNCH(KID_WF_STEP, st, (k_wf_step_bf<E, LDS, rcp, COUNT, G>), dim3(tblocks), dim3(kTraceBlock), \
                                lds, st, sc, fp, w, it, cnt, bf_slots, frame0, stride, pv[h].fbase, pv[h].P, !accum, regen_q)
                if (regen_q > 0 && (it & 1) == 0 && (uint32_t)(it / 2) * regen_q < regen_cam) PT_STEP(true, 2);
                else if (fgen && it == 0) PT_STEP(true, 1);
                else if ((it & 1) == 0) PT_STEP(true, 0);
                else PT_STEP(false, 0);
#undef PT_STEP
                return hipSuccess;
            } else if constexpr (TRAV >= 300) {
                PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>), dim3(tblocks),
                          dim3(kTraceBlock), lds, st, sc, w, in_q, cnt, bf_slots);
            } else {
                if constexpr (TRAV >= 260 && TRAV < 300)  // the big leaves first (k_wf_leafpass)
                    HIP_RETURN_IF(launch_leafpass(sc, w, in_q, ((TRAV / 10) & 1) != 0, ws.leaf_blocks, ws.leaf_pairs, st));
#define PT_TRACE(RG, PR)                                                                                        \
    do {                                                                                                        \
        if constexpr (TRAV >= 260)                                                                              \
            PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace_pre<LDS, TRAV, COUNT, RG, PR>), dim3(tblocks), dim3(kTraceBlock), \
                      lds, st, sc, w, in_q, cnt, watchdog, sparse);                                             \
        else                                                                                                    \
            PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace<LDS, TRAV, COUNT, RG, PR>), dim3(tblocks), dim3(kTraceBlock), \
                      lds, st, sc, w, in_q, cnt, watchdog, sparse);                                             \
    } while (0)
                if constexpr (has_variants<TRAV, COUNT>()) {
                    if (nring == kHitRingMax && run2) PT_TRACE(kHitRingMax, 2);
                    else if (nring == kHitRingMax) PT_TRACE(kHitRingMax, 4);
                    else if (run2) PT_TRACE(kHitRing, 2);
                    else PT_TRACE(kHitRing, 4);
                } else {
                    PT_TRACE(kHitRing, 4);
                }
#undef PT_TRACE
            }
            if ((it & 1) == 0)
                PT_LAUNCH(KID_WF_SHADE_EXT, st, (k_wf_shade<true, COUNT>), dim3(sblocks), dim3(kShadeBlock), 0, st, sc, fp,
                          w, cnt, ws.sort_bins);
            else
                PT_LAUNCH(KID_WF_SHADE_SHADOW, st, (k_wf_shade<false, COUNT>), dim3(sblocks), dim3(kShadeBlock), 0, st, sc,
                          fp, w, cnt, ws.sort_bins);
            return hipSuccess;
        };
        for (int it = 0; it < iters_b; ++it) {
            for (int h = 0; h < nh; ++h) HIP_RETURN_IF(step(h, it));
            // a launch that cannot run (e.g. a configuration error) fails here, after the first
            // iteration, instead of leaving the later launches to read counts it never wrote
            if (it == 0) HIP_RETURN_IF(hipGetLastError());
        }
        if (np > 1) {
            for (int h = 0; h < nh; ++h) {
                HIP_RETURN_IF(hipEventRecord(ws.join[h], pv[h].st));
                HIP_RETURN_IF(hipStreamWaitEvent(stream, ws.join[h], 0));
            }
        }
        PT_LAUNCH(KID_WF_ACCUM, stream, k_wf_accum, dim3((npix + 255) / 256), dim3(256), 0, stream, wb.rad, out, npix, Fb,
                  accum);
    }
    return hipGetLastError();
}

hipError_t launch_wavefront(const LaunchOpts& lo, const SceneView& scene, const FrameParams& fp, const WfBuffers& wb,
                            uint32_t frame0, uint32_t nframes, uint32_t stride, bool accum, bool count, float* out,
                            Counters* cnt, hipStream_t stream, const WfStreams& ws_in) {
    WfStreams ws = lo.dual != 0 ? ws_in : WfStreams{};  // parts on streams by default: +15 % measured (in-process A/B)
    ws.nparts = std::max(1, std::min(kMaxParts, lo.parts > 0 ? lo.parts : 2));
    ws.fuse_gen = lo.fuse_gen != 0;
    // survivors grouped per shade block by direction octant and origin cell (PT_SORT; default 512
    // keys = 8 octants x 4^3 cells: CornellBox-Glossy +4.7 % with 64 keys, +1.2 % more with 512,
    // MedievalBoat unchanged, in-process A/B)
    const int sort = lo.sort >= 0 ? lo.sort : 512;
    ws.sort_bins = sort > 0 ? (sort >= 512 ? 512 : sort >= 64 ? 64 : 8) : 0;
    ws.trace_blocks = lo.trace_blocks;
    ws.trace_sparse = std::max(0, lo.trace_sparse);
    ws.region_perm = lo.region_perm > 0 ? 1 : 0;
    ws.regen = std::max(0, lo.regen);
    ws.trace_ring = lo.trace_ring;
    ws.bf_slots = lo.bf_slots;
    ws.watchdog = lo.watchdog;
    ws.leaf_blocks = lo.leaf_blocks;
    ws.leaf_pairs = lo.leaf_pairs;
    if (!accum) { nframes = 1; stride = 1; }
    SceneView sc = scene;  // node_bias <= 0: chosen per instance in wf_render_t
    const bool lds = lo.lds && scene_fits_lds(sc);
    // lean16 with the fast reciprocal by default (measured best on gfx950, scripts/perf_variants.py);
    // the wavefront always uses a flattened traversal; lean flavours take the fast reciprocal
    // (+10) when it is exact for the scene
    const int base = lo.trav < 0 ? 7 : (lo.trav == 0 ? 1 : lo.trav);
    const bool fast = lo.fast_rcp != 0 && sc.fast_rcp;
    // mailboxed lean<K> (+100) for scenes with <= 64 distinct leaf entries
    const bool mb = lo.mailbox != 0 && sc.mailbox && base >= 5 && base <= 8;
    // brute force + replay (k_wf_trace_bf) by default for mailbox scenes; an explicit trav option
    // or bf=0 keeps the traversal kernels
    const bool bf = lo.bf != 0 && lo.mailbox != 0 && sc.mailbox && lo.trav < 0;
    // big-leaf cooperation (+160) for lean<4..16> on scenes with leaves of >= big_leaf entries; those
    // leaves resolved before the traversal instead (+260, k_wf_leafpass) when the scene's table of
    // pre-resolved leaves holds them (render_impl: option leaf_pre, default on) and the buffers exist
    const bool big = !bf && !mb && sc.big_leaf > 0 && base >= 5 && base <= 7;
    const bool pre = big && sc.npre > 0 && sc.pre && wb.pres;
    const int trav = bf ? (lo.fuse == 0 ? 300 : 400) + (fast ? 10 : 0)
                   : mb ? 100 + base + (fast ? 10 : 0)
                        : base + ((base >= 3 && fast) ? 10 : 0) + (big ? (pre ? 260 : 160) : 0);
#define WF(L, T)                                                                                               \
    if (trav == T) {                                                                                           \
        if (count) return wf_render_t<L, T, true>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream, ws); \
        return wf_render_t<L, T, false>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream, ws);         \
    }
    if (lds) {
        WF(true, 1) WF(true, 2) WF(true, 3) WF(true, 4) WF(true, 5) WF(true, 6) WF(true, 7) WF(true, 8)
        WF(true, 13) WF(true, 14) WF(true, 15) WF(true, 16) WF(true, 17) WF(true, 18)
        WF(true, 300) WF(true, 310) WF(true, 400) WF(true, 410)
        WF(true, 105) WF(true, 106) WF(true, 107) WF(true, 115) WF(true, 116) WF(true, 117) WF(true, 118)
        WF(true, 165) WF(true, 166) WF(true, 167) WF(true, 175) WF(true, 176) WF(true, 177)
        WF(true, 265) WF(true, 266) WF(true, 267) WF(true, 275) WF(true, 276) WF(true, 277)
    } else {
        WF(false, 1) WF(false, 2) WF(false, 3) WF(false, 4) WF(false, 5) WF(false, 6) WF(false, 7) WF(false, 8)
        WF(false, 13) WF(false, 14) WF(false, 15) WF(false, 16) WF(false, 17) WF(false, 18)
        WF(false, 300) WF(false, 310) WF(false, 400) WF(false, 410)
        WF(false, 105) WF(false, 106) WF(false, 107) WF(false, 115) WF(false, 116) WF(false, 117) WF(false, 118)
        WF(false, 165) WF(false, 166) WF(false, 167) WF(false, 175) WF(false, 176) WF(false, 177)
        WF(false, 265) WF(false, 266) WF(false, 267) WF(false, 275) WF(false, 276) WF(false, 277)
    }
#undef WF
    return hipErrorInvalidValue;
}

}  // namespace pt

#if PT_PHASE_STATS
// diagnostic builds only (not in include/pt_hip.h): the fused kernel's per-phase sums since the last
// reset, [EXT][phase][cycles, iterations, lanes] as 2 x PH_COUNT x 3 u64 (scripts/phase_stats.py)
extern "C" int pt_phase_stats_read(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -4;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(pt::g_phase_stats), sizeof(pt::g_phase_stats)) != hipSuccess) return -4;
    if (reset) {
        static const unsigned long long zero[2][pt::PH_COUNT][3] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pt::g_phase_stats), zero, sizeof zero) != hipSuccess) return -4;
    }
    return 0;
}
#endif

#if PT_TRACE_STATS
// diagnostic builds only: k_wf_trace's turn statistics since the last reset, [queue][kind][cycles,
// turns, lanes] as 2 x TS_COUNT x 3 u64 (scripts/trace_stats.py)
extern "C" int pt_trace_stats_read(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -4;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(pt::g_trace_stats), sizeof(pt::g_trace_stats)) != hipSuccess) return -4;
    if (reset) {
        static const unsigned long long zero[2][pt::TS_COUNT][3] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pt::g_trace_stats), zero, sizeof zero) != hipSuccess) return -4;
    }
    return 0;
}
#endif
