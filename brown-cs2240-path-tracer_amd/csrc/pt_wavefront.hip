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

namespace pt {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// k_wf_trace hands out its 32-entry windows dynamically: wave w takes the next window of group
// w % kTraceGroups from that group's counter (one cache line each, in wb.rfetch: slot in_q of the
// launch; the launch zeroes the other slot for the next trace, k_wf_generate both for a batch's
// first).  A group's windows are one contiguous range of the queue.
constexpr uint32_t kTraceGroups = 64;
__device__ __forceinline__ uint32_t* trace_counter(uint32_t* rfetch, int slot, uint32_t g) {
    return rfetch + ((uint32_t)slot * kRegions + g) * kFetchStride;
}

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
// frame f, pixel (x, y) and path id p = f * npix + y * W + x (row-major within its frame: the
// radiance index k_wf_accum reads).  Row order (fp.tiles == 0): slot = path id.  Tile order
// (fp.tiles != 0): a frame's slots walk 8x8 pixel tiles, so the 64 paths of a generation batch are
// one tile (coherent camera rays in one wave) — the W8 x H8 part of the image (W8, H8 = W, H
// rounded down to multiples of 8) in tiles, then the pixels right of it, then those below it, row
// by row.  Scatter order (fp.tiles == 2, option scatter, opt-in: +7.5 % at 4096^2, -5 % at 1024^2,
// and the default region permutation gives the 4096^2 gain alone): slot q of a frame starts pixel
// (q * fp.scatter_mul) mod npix, a bijection (the multiplier is coprime with npix, ~0.618 npix), so
// a batch's 64 paths are spread over the image.  Only which slot a path starts in changes: every
// path computes the same bits.
__device__ __forceinline__ uint32_t slot_path(uint32_t s, const FrameParams& fp, uint32_t& x, uint32_t& y, uint32_t& f) {
    const uint32_t W = fp.width, npix = W * fp.height;
    f = s / npix;
    uint32_t q = s - f * npix;
    if (fp.tiles == 2) {
        q = (uint32_t)(((uint64_t)q * fp.scatter_mul) % npix);
        y = q / W;
        x = q - y * W;
    } else if (!fp.tiles) {
        y = q / W;
        x = q - y * W;
    } else {
        const uint32_t TW = W >> 3, TH = fp.height >> 3, core = TW * TH * 64;
        if (q < core) {
            const uint32_t t = q >> 6, l = q & 63u, ty = t / TW;
            x = (t - ty * TW) * 8 + (l & 7u);
            y = ty * 8 + (l >> 3);
        } else {
            q -= core;
            const uint32_t rw = W - TW * 8, nr = rw * TH * 8;
            if (q < nr) {
                y = q / rw;
                x = TW * 8 + (q - y * rw);
            } else {
                q -= nr;
                y = TH * 8 + q / W;
                x = q - (y - TH * 8) * W;
            }
        }
    }
    return f * npix + y * W + x;
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
    // k_wf_trace's window counters, both slots, for the batch's first trace (trace_counter)
    if (blockIdx.x == 0 && threadIdx.x < 2 * kTraceGroups)
        wb.rfetch[((threadIdx.x / kTraceGroups) * kRegions + threadIdx.x % kTraceGroups) * kFetchStride] = 0;
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
__host__ __device__ constexpr uint32_t stage_bytes(uint32_t ring) { return kWinRays * 32 + ring * 8 + win_tab(ring) * 4; }
// the traversal flavours that have a 256-entry-ring instance (the defaults: lean16 + fast rcp,
// with and without big-leaf turns); the others always use 128
constexpr bool has_big_ring(int trav) { return trav == 17 || trav == 177; }
constexpr uint32_t kTraceBlock = 512;  // 8 waves share one LDS copy of the scene
// k_wf_trace's block (the traversal scenes): its LDS is per lane (the traversal stack, max_stack
// words) and per wave (kStageBytes), so the block size sets the LDS granularity, not the total
#ifndef PT_TRACE_BLOCK
#define PT_TRACE_BLOCK 512
#endif
constexpr uint32_t kTraceBlockTr = PT_TRACE_BLOCK;
template <int TRAV>
constexpr uint32_t trace_block() { return TRAV >= 300 ? kTraceBlock : kTraceBlockTr; }

// Work split: the queue is cut into windows of 32 entries; wave w of N takes windows w, w+N,
// w+2N, ... (interleaving, not contiguous chunks, because queue order is spatially coherent —
// camera rays in pixel order, survivors compacted block by block — so a contiguous chunk is an
// image region whose cost differs systematically from the others).  dyn (option trace_dyn=1): chunks
// of 8 windows are dealt to kTraceGroups groups of blocks round-robin and a group's waves take
// them one window at a time from its counter, so a wave that drew cheap rays takes more windows
// (one stream: +8 %; two: static 4 % faster).  Inside a wave, its
// j-th window's entries have the wave-local sequence numbers 32j .. 32j+31, which index the hit
// ring; wtab keeps the ids of the windows between the last written back and the prefetched one.
// PT_TRACE_WAVES (build-time A/B): cap the traversal kernel's VGPRs for this many waves per SIMD
#ifndef PT_TRACE_WAVES
#define PT_TRACE_WAVES 0
#endif
#if PT_TRACE_WAVES > 0
#define PT_TRACE_OCC __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES, PT_TRACE_WAVES)))
#else
// no occupancy attribute: the big-leaf instances take 71 VGPRs (7 waves per SIMD); forcing
// amdgpu_waves_per_eu(7) made them 72 and 11 % slower on the 100k synthetic scene (in process,
// profiles/r03m_ab_trace_occ.log)
#define PT_TRACE_OCC
#endif
template <bool LDS, int TRAV, bool COUNT, uint32_t RING = kHitRing>
__global__ __launch_bounds__(kTraceBlockTr) PT_TRACE_OCC void k_wf_trace(SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out,
                                                          uint32_t watchdog, int dyn) {
    constexpr uint32_t nring = RING, kWinTab = win_tab(RING);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int32_t* stack = reinterpret_cast<int32_t*>(smem) + threadIdx.x;
    char* stage_base = smem + (uint32_t)sc.max_stack * blockDim.x * 4u;
    char* stage = stage_base + (threadIdx.x / 64u) * stage_bytes(nring);
    float4* wray = reinterpret_cast<float4*>(stage);               // [kWinRays][2]
    int2* ring = reinterpret_cast<int2*>(stage + kWinRays * 32);   // [RING]
    uint32_t* wtab = reinterpret_cast<uint32_t*>(stage + kWinRays * 32 + RING * 8);  // [kWinTab] window ids
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1] = 0;  // shade's output count
    if (blockIdx.x == 0 && threadIdx.x < kTraceGroups) *trace_counter(wb.rfetch, in_q ^ 1, threadIdx.x) = 0;  // next trace's
    const uint32_t count = wb.ctl[WF_WATCHDOG] ? 0u : wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];  // gave up: skip
    // the wave index is uniform: readfirstlane keeps everything derived from it in SGPRs
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    // sparse windows (dyn >> 1 = n > 0, option trace_sparse=n): when windows of wr entries would
    // keep fewer than 1/n of the waves busy (the last depths), windows of wr / 2 .. 1 entries
    // spread the queue over more waves, so each wave's traversal is the slowest of fewer rays.  A
    // window still takes kWinRays sequence numbers (ring and flush bookkeeping unchanged); only
    // its queue span is wr.
    uint32_t wr = kWinRays;
    if (const uint32_t n = (uint32_t)dyn >> 1)
        while (wr > 1 && (uint64_t)count * n < (uint64_t)nwaves * wr) wr >>= 1;
    const uint32_t nwin = (count + wr - 1) / wr;
    if (LDS) stage_scene_lds(sc, stage_base + (blockDim.x / 64u) * stage_bytes(nring));
    // windows: group g owns windows g, g + G, g + 2G, ... (interleaved over the whole queue, whose
    // order is spatially coherent, so every group's share costs about the same), handed out one
    // at a time from the group's counter to the group's waves
    // groups are made of whole blocks (the 8 waves of a block share a counter and the windows of a
    // chunk of 8 consecutive ones: rays of one chunk are neighbours in the queue, so a CU's waves
    // keep working on similar rays — its L1 then holds what they all read)
    constexpr uint32_t kChunk = kTraceBlockTr / 64;
    const uint32_t nblk = nwaves / kChunk, G = min(kTraceGroups, nblk), g = (w / kChunk) % G;
    uint32_t* ctr = trace_counter(wb.rfetch, in_q, g);
    const uint32_t lane = lane_id();
    constexpr uint32_t kNone = 0xffffffffu;
    // the counter's atomic for the window after next is issued one window ahead, so its latency
    // hides behind the current window instead of stalling the hand-out
    // (dyn = 0, trace_dyn=0: the static split — wave w takes windows w, w + nwaves, ... — for A/B)
    uint32_t ticket = 0;  // lane 0: the group counter's value for the next fetch
    uint32_t nstatic = 0;
    auto issue = [&]() {
        if ((dyn & 1) && lane == 0) ticket = atomicAdd(ctr, 1u);
    };
    auto fetch = [&]() {  // the group's next window (wave-uniform), or kNone; issues the one after
        if (!(dyn & 1)) {
            const uint64_t wid = (uint64_t)(nstatic++) * nwaves + w;
            return wid < nwin ? (uint32_t)wid : kNone;
        }
        const uint32_t i = __builtin_amdgcn_readfirstlane(__shfl(ticket, 0, 64));
        issue();
        const uint64_t wid = ((uint64_t)(i / kChunk) * G + g) * kChunk + i % kChunk;  // chunk (i / 8) of group g
        return wid < nwin ? (uint32_t)wid : kNone;
    };
    auto wcount = [&](uint32_t wid) { return min(wr, count - wid * wr); };
    if (((dyn & 1) ? g * kChunk : w) >= nwin) return;  // wave-uniform: nothing for this wave
    issue();
    const uint32_t w0 = fetch();
    if (w0 == kNone) return;  // wave-uniform
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
    for (uint32_t guard = 0;; ++guard) {
        // every wave reaches an exit: after kTraceWatchdog iterations or kTraceWatchdogTicks of
        // wall clock it reports instead of hanging (and later launches of the render skip)
        if (guard == watchdog ||
            ((guard & 1023u) == 1023u && wall_clock64() - t_start > kTraceWatchdogTicks)) {
            const uint64_t hm = __ballot(has);
            if (lane == 0) {
                atomicOr(&wb.ctl[WF_WATCHDOG], 1u);
                if (atomicCAS(&wb.ctl[WF_SNAP_CLAIM], 0u, 1u) == 0u) {
                    const uint32_t v[WF_SNAP_WORDS] = {count, nwaves, w, g, jl, wv, nv, cur, flushed,
                                                       (uint32_t)__popcll(hm), (uint32_t)hm, (uint32_t)(hm >> 32),
                                                       (uint32_t)in_q, G, 0u, 0u};
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
        if (need) {
            if (cur == jl * kWinRays + wv && nv > 0 && (jl + 2) * kWinRays - flushed <= nring) {
                if (wl < nv) wray[2 * wl + half] = na;  // next window, if the hit ring has room
                ++jl;
                wv = nv;
                cur = jl * kWinRays;
                nv = 0;
                const uint32_t wn = fetch();
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
                    has = true;
                }
                cur = min(cur + (uint32_t)__popcll(need), wend);
            }
        }
        if (!wave_any(has)) {
            if (nv == 0 && cur == jl * kWinRays + wv && flushed >= (jl + 1) * kWinRays) break;  // all done
            continue;  // ring full with nothing in flight: the flush above frees it
        }
        trav_advance<TRAV, COUNT, true>(sc, r, s, stack, blockDim.x, c);
        if (has && trav_finished(s)) {
            ring[sq & (nring - 1)] = make_int2(s.best, __builtin_bit_cast(int, s.best_t));
            has = false;
        }
    }
    if (COUNT) flush_counters(c, cnt_out);
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
// phase 1 in entry pairs with packed f32 (bf_pairs): bit-exact, measured no faster (fused kernel,
// extension rays only: 2598 vs 2607 Msamples/s; both queues: 2446, VGPR spills in the shadow instance)
#ifndef PT_BF_LDSREC
#define PT_BF_LDSREC 0
#endif
#ifndef PT_BF_PACKED
#define PT_BF_PACKED 0
#endif
constexpr bool kBfPacked = PT_BF_PACKED != 0;  // (k_regen_bf, itself opt-in, uses bf_pairs: tests cover it)
constexpr bool kBfPackedShadow = PT_BF_PACKED == 2 || PT_BF_PACKED >= 4;  // the shadow instances too (3: bf_quads, extension only; 4: both)
// Diagnostic build only (EXTRA=-DPT_PHASE_TIMING=1, scripts/phase_timing.py): shader-clock
// cycles per phase of bf_step_batch, summed per wave slot (8 phases x {extension, shadow}).
#ifndef PT_PHASE_TIMING
#define PT_PHASE_TIMING 0
#endif
#if PT_PHASE_TIMING
constexpr int kPhaseSlots = 16;
constexpr int kPhaseWaves = 16384;
__device__ unsigned long long g_phase[kPhaseWaves * kPhaseSlots];
#endif
__device__ __forceinline__ uint64_t phase_clock() {
#if PT_PHASE_TIMING
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
}
// Diagnostic builds only (EXTRA=-DPT_DIAG_VALU_PAD=n, scripts/gpu_ab_valupad.sh): n extra dependent
// v_fmac_f32 per phase-1 entry, on a register nothing reads — the images are unchanged.  If the fused
// kernel is bound by VALU issue, each added wave-instruction costs its full issue time (about 4.2
// SIMD cycles, profiles/valu_calibration.json); if it were bound by memory or latency, the added
// instructions would fill idle issue slots and cost little.
#ifndef PT_DIAG_VALU_PAD
#define PT_DIAG_VALU_PAD 0
#endif
// the same for the scalar ALU (PT_DIAG_SALU_PAD extra s_add_u32 per entry) and for latency
// (PT_DIAG_SLEEP: s_sleep n per entry, the wave idles ~64 n cycles and uses no unit)
#ifndef PT_DIAG_VALU_KIND  // the padding instruction: 0 v_fmac a,b,b; 1 v_fma_f32 (3 sources); 2 v_fmac a,b,c; 3 v_add_u32
#define PT_DIAG_VALU_KIND 0
#endif
#ifndef PT_DIAG_SALU_PAD
#define PT_DIAG_SALU_PAD 0
#endif
#ifndef PT_DIAG_SLEEP
#define PT_DIAG_SLEEP 0
#endif
constexpr bool kBfScalarPrefetch = false;  // phase 1: next record's s_load in flight during a test (measured -2 %)
constexpr bool kBfPrefetch = true;  // bf_step_batch loads q2/q3 before the trace

__device__ __forceinline__ uint32_t sload_u32(const uint32_t* p) {  // uniform address: s_load
    return *(const __attribute__((address_space(4))) uint32_t*)p;
}

__device__ __forceinline__ TriRec load_tri_scalar(const Tri* tris, int i) {
    // uniform index: constant address space, so the record comes through s_load (no VGPRs)
    const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(tris + i);
    return TriRec{make_float4(f[0], f[1], f[2], f[3]), make_float4(f[4], f[5], f[6], f[7]), f[8]};
}

// Entry cull (SceneView::cull; camera rays and their shadow rays, whose batches are coherent):
// lane u tests distinct entry u against the bundle of the wave's valid rays — origins in the box
// [olo, ohi], directions in [dlo, dhi], each axis on its own (a superset of the rays) — and the
// entry is dropped from phase 1 when (a) no ray of the bundle reaches the entry's box grown by
// the margin for t >= 0 and (b) every ray of the bundle has |det| >= tau (|e1 . (d x e2)| =
// |d . (e1 x e2)| bounded by interval arithmetic).  (b) bounds the rounding of the test: a ray
// whose |det| >= 1e-2 |e1| |e2| and whose test reports a hit passes within 2.4e-4 S + 6e-5
// (|e1| + |e2|) of the triangle (S = 2 (|o| + |v0|)); the margin is 4e-3 (S + |e1| + |e2|),
// ~16x that bound, so a ray that the test would report hitting always reaches the grown box, and
// an entry dropped here has no hit for any ray of the wave: the result is unchanged.  Exact, like
// the skipped det/u early-out (phase 1), for every entry the test would not hit.
__device__ __forceinline__ float uniformf(float x) {  // to an SGPR (the value is wave-uniform)
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
}
__device__ __forceinline__ float wave_minf(float x) {
    for (int s = 1; s < 64; s <<= 1) x = fminf(x, __shfl_xor(x, s, 64));
    return uniformf(x);
}
__device__ __forceinline__ float wave_maxf(float x) {
    for (int s = 1; s < 64; s <<= 1) x = fmaxf(x, __shfl_xor(x, s, 64));
    return uniformf(x);
}
__device__ __forceinline__ uint64_t bf_cull_mask(const SceneView& sc, const Ray& r, bool valid, int U) {
    const uint64_t all = U >= 64 ? ~0ull : (1ull << U) - 1;
    if (__ballot(valid) == 0) return 0;  // no ray: nothing can hit
    const float inf = __builtin_inff();
    const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    float olo[3], ohi[3], dlo[3], dhi[3];
    for (int a = 0; a < 3; ++a) {
        olo[a] = wave_minf(valid ? o[a] : inf);
        ohi[a] = wave_maxf(valid ? o[a] : -inf);
        dlo[a] = wave_minf(valid ? d[a] : inf);
        dhi[a] = wave_maxf(valid ? d[a] : -inf);
    }
    const int u = (int)lane_id();
    bool keep = true;
    if (u < U) {
        const float4 c0 = sc.cull[3 * u], c1 = sc.cull[3 * u + 1], c2 = sc.cull[3 * u + 2];
        float omax = 0.0f, dm2 = 0.0f;
        for (int a = 0; a < 3; ++a) {
            omax = fmaxf(omax, fmaxf(fabsf(olo[a]), fabsf(ohi[a])));
            const float dm = fmaxf(fabsf(dlo[a]), fabsf(dhi[a]));
            dm2 += dm * dm;
        }
        const float m = c1.w * (3.4641017f * omax + c2.w);
        const float blo[3] = {c0.x - m, c0.y - m, c0.z - m}, bhi[3] = {c1.x + m, c1.y + m, c1.z + m};
        const float n[3] = {c2.x, c2.y, c2.z};
        float tlo = 0.0f, thi = inf, dlo_n = 0.0f, dhi_n = 0.0f;
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
            // some o + t d inside [blo, bhi] on axis a needs olo + t dlo <= bhi and ohi + t dhi >= blo
            const float A = bhi[a] - olo[a], B = blo[a] - ohi[a];
            if (dlo[a] > 0.0f) thi = fminf(thi, A / dlo[a]);
            else if (dlo[a] < 0.0f) tlo = fmaxf(tlo, A / dlo[a]);
            else ok &= A >= 0.0f;
            if (dhi[a] > 0.0f) tlo = fmaxf(tlo, B / dhi[a]);
            else if (dhi[a] < 0.0f) thi = fminf(thi, B / dhi[a]);
            else ok &= B <= 0.0f;
            dlo_n += fminf(n[a] * dlo[a], n[a] * dhi[a]);
            dhi_n += fmaxf(n[a] * dlo[a], n[a] * dhi[a]);
        }
        const bool reach = ok && tlo <= thi;
        const float tau = c0.w * sqrtf(dm2);
        const bool steady = dlo_n >= tau || dhi_n <= -tau;
        keep = reach || !steady || !(m < inf);
    }
    return __ballot(keep) & all;
}

// Phase 1 over pairs of entries (SceneView::bfpair) with packed f32 arithmetic: each
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 does one operation of the test for both entries of
// the pair — the same IEEE operations, in the same order, as tri_hit's (dot/cross of pt_math.h,
// rcp_rn with kRcpSteps = 1), so the same bits at half the VALU issue.  Hits are recorded in
// entry order, as the one-entry loop does.
typedef float fv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fv2 fma2(fv2 a, fv2 b, fv2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ fv2 sp2(float x) { return fv2{x, x}; }
static_assert(kRcpSteps == 1, "bf_pairs restates rcp_rn with one Newton step");
template <bool FAST_RCP>
__device__ __forceinline__ void bf_pairs(const SceneView& sc, const Ray& r, bool valid, float* slot, int nslots,
                                         uint64_t& hits, int& nh, float& tmin) {
    const int NP = (sc.n_tris - sc.mb_base + 1) >> 1;
    const uint64_t vmask = __builtin_amdgcn_ballot_w64(valid);
    for (int j = 0; j < NP; ++j) {
        const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(sc.bfpair + 20 * j);
        const fv2 v0x = {f[0], f[1]}, v0y = {f[2], f[3]}, v0z = {f[4], f[5]};
        const fv2 e1x = {f[6], f[7]}, e1y = {f[8], f[9]}, e1z = {f[10], f[11]};
        const fv2 e2x = {f[12], f[13]}, e2y = {f[14], f[15]}, e2z = {f[16], f[17]};
        const fv2 dx = sp2(r.d.x), dy = sp2(r.d.y), dz = sp2(r.d.z);
        const fv2 rx = fma2(dy, e2z, -(dz * e2y)), ry = fma2(dz, e2x, -(dx * e2z)), rz = fma2(dx, e2y, -(dy * e2x));
        const fv2 det = fma2(e1z, rz, fma2(e1y, ry, e1x * rx));
        fv2 inv;
        if (FAST_RCP) {
            const fv2 y = {__builtin_amdgcn_rcpf(det.x), __builtin_amdgcn_rcpf(det.y)};
            inv = fma2(fma2(-det, y, sp2(1.0f)), y, y);
        } else {
            inv = fv2{1.0f / det.x, 1.0f / det.y};
        }
        const fv2 sx = sp2(r.o.x) - v0x, sy = sp2(r.o.y) - v0y, sz = sp2(r.o.z) - v0z;
        const fv2 bu = inv * fma2(sz, rz, fma2(sy, ry, sx * rx));
        const bool d0 = !(det.x > -1e-8f && det.x < 1e-8f), l0 = !(bu.x < 0.0f), g0 = !(bu.x > 1.0f);
        const bool d1 = !(det.y > -1e-8f && det.y < 1e-8f), l1 = !(bu.y < 0.0f), g1 = !(bu.y > 1.0f);
        const bool ok0 = valid & d0 & l0 & g0, ok1 = valid & d1 & l1 & g1;
        // the vote on SGPR masks of the single compares (as bf_closest's entry loop)
        const uint64_t any0 = __builtin_amdgcn_ballot_w64(d0) & __builtin_amdgcn_ballot_w64(l0) & __builtin_amdgcn_ballot_w64(g0);
        const uint64_t any1 = __builtin_amdgcn_ballot_w64(d1) & __builtin_amdgcn_ballot_w64(l1) & __builtin_amdgcn_ballot_w64(g1);
        if ((vmask & (any0 | any1)) == 0) continue;  // wave-uniform
        const fv2 cx = fma2(sy, e1z, -(sz * e1y)), cy = fma2(sz, e1x, -(sx * e1z)), cz = fma2(sx, e1y, -(sy * e1x));
        const fv2 bv = inv * fma2(dz, cz, fma2(dy, cy, dx * cx));
        const fv2 t = inv * fma2(e2z, cz, fma2(e2y, cy, e2x * cx));
        const bool h0 = ok0 & !(bv.x < 0.0f) & !(bu.x + bv.x > 1.0f) & (t.x > 1e-8f);
        const bool h1 = ok1 & !(bv.y < 0.0f) & !(bu.y + bv.y > 1.0f) & (t.y > 1e-8f);
        if (h0) {
            if (nh < nslots) slot[64 * nh] = t.x;
            ++nh;
            hits |= 1ull << (2 * j);
            tmin = t.x < tmin ? t.x : tmin;
        }
        if (h1) {
            if (nh < nslots) slot[64 * nh] = t.y;
            ++nh;
            hits |= 1ull << (2 * j + 1);
            tmin = t.y < tmin ? t.y : tmin;
        }
    }
}

// bf_pairs two pairs at a time (PT_BF_PACKED=3 builds): the two pairs' det/u parts are
// independent, so their packed instructions interleave and hide each other's latency (one pair's
// chain alone stalls: PMC of PT_BF_PACKED=1, WAIT_INST_ANY +27 %).  Hits are recorded in entry order.
template <bool FAST_RCP>
__device__ __forceinline__ void bf_quads(const SceneView& sc, const Ray& r, bool valid, float* slot, int nslots,
                                         uint64_t& hits, int& nh, float& tmin) {
    const int NQ = (sc.n_tris - sc.mb_base + 3) >> 2;  // bfpair holds a whole number of quads (host)
    const uint64_t vmask = __builtin_amdgcn_ballot_w64(valid);
    const fv2 dx = sp2(r.d.x), dy = sp2(r.d.y), dz = sp2(r.d.z);
    for (int j = 0; j < NQ; ++j) {
        fv2 bu[2], det[2], inv[2], sx[2], sy[2], sz[2];
        const __attribute__((address_space(4))) float* f0 = (const __attribute__((address_space(4))) float*)(sc.bfpair + 40 * j);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const __attribute__((address_space(4))) float* f = f0 + 20 * h;
            const fv2 v0x = {f[0], f[1]}, v0y = {f[2], f[3]}, v0z = {f[4], f[5]};
            const fv2 e1x = {f[6], f[7]}, e1y = {f[8], f[9]}, e1z = {f[10], f[11]};
            const fv2 e2x = {f[12], f[13]}, e2y = {f[14], f[15]}, e2z = {f[16], f[17]};
            const fv2 rx = fma2(dy, e2z, -(dz * e2y)), ry = fma2(dz, e2x, -(dx * e2z)), rz = fma2(dx, e2y, -(dy * e2x));
            det[h] = fma2(e1z, rz, fma2(e1y, ry, e1x * rx));
            if (FAST_RCP) {
                const fv2 y = {__builtin_amdgcn_rcpf(det[h].x), __builtin_amdgcn_rcpf(det[h].y)};
                inv[h] = fma2(fma2(-det[h], y, sp2(1.0f)), y, y);
            } else {
                inv[h] = fv2{1.0f / det[h].x, 1.0f / det[h].y};
            }
            sx[h] = sp2(r.o.x) - v0x; sy[h] = sp2(r.o.y) - v0y; sz[h] = sp2(r.o.z) - v0z;
            bu[h] = inv[h] * fma2(sz[h], rz, fma2(sy[h], ry, sx[h] * rx));
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool d0 = !(det[h].x > -1e-8f && det[h].x < 1e-8f), l0 = !(bu[h].x < 0.0f), g0 = !(bu[h].x > 1.0f);
            const bool d1 = !(det[h].y > -1e-8f && det[h].y < 1e-8f), l1 = !(bu[h].y < 0.0f), g1 = !(bu[h].y > 1.0f);
            const uint64_t any0 = __builtin_amdgcn_ballot_w64(d0) & __builtin_amdgcn_ballot_w64(l0) & __builtin_amdgcn_ballot_w64(g0);
            const uint64_t any1 = __builtin_amdgcn_ballot_w64(d1) & __builtin_amdgcn_ballot_w64(l1) & __builtin_amdgcn_ballot_w64(g1);
            if ((vmask & (any0 | any1)) == 0) continue;  // wave-uniform
            const bool ok0 = valid & d0 & l0 & g0, ok1 = valid & d1 & l1 & g1;
            const __attribute__((address_space(4))) float* f = f0 + 20 * h;
            const fv2 e1x = {f[6], f[7]}, e1y = {f[8], f[9]}, e1z = {f[10], f[11]};
            const fv2 e2x = {f[12], f[13]}, e2y = {f[14], f[15]}, e2z = {f[16], f[17]};
            const fv2 cx = fma2(sy[h], e1z, -(sz[h] * e1y)), cy = fma2(sz[h], e1x, -(sx[h] * e1z)),
                      cz = fma2(sx[h], e1y, -(sy[h] * e1x));
            const fv2 bv = inv[h] * fma2(dz, cz, fma2(dy, cy, dx * cx));
            const fv2 t = inv[h] * fma2(e2z, cz, fma2(e2y, cy, e2x * cx));
            const bool h0 = ok0 & !(bv.x < 0.0f) & !(bu[h].x + bv.x > 1.0f) & (t.x > 1e-8f);
            const bool h1 = ok1 & !(bv.y < 0.0f) & !(bu[h].y + bv.y > 1.0f) & (t.y > 1e-8f);
            const int u = 4 * j + 2 * h;
            if (h0) {
                if (nh < nslots) slot[64 * nh] = t.x;
                ++nh;
                hits |= 1ull << u;
                tmin = t.x < tmin ? t.x : tmin;
            }
            if (h1) {
                if (nh < nslots) slot[64 * nh] = t.y;
                ++nh;
                hits |= 1ull << (u + 1);
                tmin = t.y < tmin ? t.y : tmin;
            }
        }
    }
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
                                                   float tmin, const float* slot, int nslots, float& t_out) {
    constexpr uint64_t kInner = 1ull << 63;
    uint64_t pend = active ? 1ull : 0ull;  // pre-order node 0 = the root
    uint64_t tested = 0;
    int best = -1;
    float best_t = -1.0f;
    while (wave_any(pend != 0)) {
        if (pend != 0) {
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

// Closest hit of the 64 rays of one batch (lane = ray; `valid` false lanes give no hit):
// phase 1 + phase 2 above.  Returns the record (or -1) and its t in t_out.
template <bool FAST_RCP, bool COUNT, bool PK = kBfPacked>
__device__ __forceinline__ int bf_closest(const SceneView& sc, const Tri* gtris, const Ray& r, bool valid, float* slot,
                                          int nslots, int32_t* stack, int stride, Counters& c, float& t_out,
                                          uint64_t todo = ~0ull,  // todo: entries phase 1 tests (bf_cull_mask)
                                          uint64_t* tmark = nullptr) {  // PT_PHASE_TIMING: end of phase 1
    const int U = sc.n_tris - sc.mb_base;
    // phase 1: every distinct entry against all 64 rays.  The test is tri_hit's arithmetic cut
    // after u: when no lane passes the det and u tests (the early-out chain of
    // ray-triangle-intersection.wgsl:15-24) the rest cannot make a hit and is skipped for the wave
    uint64_t hits = 0;
    int nh = 0;
    const uint64_t vmask = __builtin_amdgcn_ballot_w64(valid);  // loop-invariant part of phase 1's vote
    float tmin = 3.0e38f;  // smallest t of any entry this ray hits
    if (PK && todo == ~0ull) {  // every entry: in pairs, packed f32 (bf_pairs; two pairs at a time: bf_quads)
        if (PT_BF_PACKED >= 3) bf_quads<FAST_RCP>(sc, r, valid, slot, nslots, hits, nh, tmin);
        else bf_pairs<FAST_RCP>(sc, r, valid, slot, nslots, hits, nh, tmin);
        todo = 0;
    }
    // one entry of phase 1 against the wave's 64 rays
    float pad = r.d.x;  // PT_DIAG_VALU_PAD builds only
    auto entry = [&](int u, const TriRec& tr) __attribute__((always_inline)) {
        if constexpr (PT_DIAG_VALU_PAD > 0) {  // diagnostic: PAD extra v_fmac_f32 per entry (results unchanged)
#pragma unroll
            for (int i = 0; i < PT_DIAG_VALU_PAD; ++i) {
                if (PT_DIAG_VALU_KIND == 1) __asm__ volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(pad) : "v"(r.o.x), "v"(r.d.y));
                else if (PT_DIAG_VALU_KIND == 2) __asm__ volatile("v_fmac_f32 %0, %1, %2" : "+v"(pad) : "v"(r.o.x), "v"(r.d.y));
                else if (PT_DIAG_VALU_KIND == 3) __asm__ volatile("v_add_u32 %0, %1, %0" : "+v"(pad) : "v"(r.o.x));
                else __asm__ volatile("v_fmac_f32 %0, %1, %1" : "+v"(pad) : "v"(r.o.x));
            }
        }
        if constexpr (PT_DIAG_SALU_PAD > 0) {  // diagnostic: PAD extra s_add_u32 per entry
            uint32_t sp = (uint32_t)u;
#pragma unroll
            for (int i = 0; i < PT_DIAG_SALU_PAD; ++i) __asm__ volatile("s_add_u32 %0, %0, 1" : "+s"(sp));
        }
        if constexpr (PT_DIAG_SLEEP > 0) __builtin_amdgcn_s_sleep(PT_DIAG_SLEEP);  // diagnostic: ~64 x n idle cycles per entry
        const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z), e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
        const f3 rce2 = cross(r.d, e2);
        const float det = dot(e1, rce2);
        const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
        const f3 sv = r.o - v0;
        const float bu = inv_det * dot(sv, rce2);
        const bool ok_det = !(det > -1e-8f && det < 1e-8f), ok_lo = !(bu < 0.0f), ok_hi = !(bu > 1.0f);
        const bool ok_u = valid & ok_det & ok_lo & ok_hi;
        // the vote as SGPR masks of the single compares (one ballot of the combined bool costs
        // two VALU slots per entry: v_cndmask + v_cmp)
        if ((vmask & __builtin_amdgcn_ballot_w64(ok_det) &
             __builtin_amdgcn_ballot_w64(ok_lo) & __builtin_amdgcn_ballot_w64(ok_hi)) == 0)
            return;  // wave-uniform
        const f3 sce1 = cross(sv, e1);
        const float bv = inv_det * dot(r.d, sce1);
        const float t = inv_det * dot(e2, sce1);
        const bool h = ok_u & !(bv < 0.0f) & !(bu + bv > 1.0f) & (t > 1e-8f);
        if (h) {
            if (nh < nslots) slot[64 * nh] = t;
            ++nh;
            hits |= 1ull << u;
            tmin = t < tmin ? t : tmin;  // = fminf here (t > 1e-8, never NaN) without its two canonicalising v_max
        }
    };
    if (todo == ~0ull) {  // every entry (a constant in the instances without the cull)
        if (kBfScalarPrefetch) {
            // the next record's s_load is issued after this record's wait, so it is in flight
            // while this entry is tested (scalar loads return out of order: lgkmcnt(0) would
            // otherwise wait for both)
            TriRec nxt = load_tri_scalar(gtris, sc.mb_base);
            for (int u = 0; u < U; ++u) {
                const TriRec tr = nxt;
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): tr is here
                __asm__ volatile("" ::: "memory");
                nxt = load_tri_scalar(gtris, sc.mb_base + min(u + 1, U - 1));
                entry(u, tr);
            }
        } else {
            // PT_BF_LDSREC builds (A/B): the record read from the scene's copy (LDS when staged) by
            // every lane at one address (a broadcast ds_read) instead of through the scalar cache
            if (PT_BF_LDSREC) for (int u = 0; u < U; ++u) entry(u, load_tri(sc.tris, sc.mb_base + u));
            else for (int u = 0; u < U; ++u) entry(u, load_tri_scalar(gtris, sc.mb_base + u));
        }
    } else {
        todo &= U >= 64 ? ~0ull : (1ull << U) - 1;  // wave-uniform
        while (todo) {
            const int u = (int)__builtin_ctzll(todo);
            todo &= todo - 1;
            entry(u, load_tri_scalar(gtris, sc.mb_base + u));
        }
    }
    if (PT_PHASE_TIMING && tmark) *tmark = phase_clock();
    // phase 2: the mailboxed traversal, leaf entries resolved from phase 1.  Without counters a
    // ray stops as soon as its closest t equals tmin: no later entry has a smaller t, and an
    // equal one can only win inside the pair just resolved (strict-< across pairs) — so the
    // result is final; a ray that hits nothing at all is final at once.  The counting build
    // (COUNT) walks on, to count the reference's work.
    if constexpr (!COUNT) {
        if (sc.bfnode) {  // wave-uniform: the stackless walk (bf_replay_stackless)
            return bf_replay_stackless<FAST_RCP>(sc, r, valid && hits != 0, hits, tmin, slot, nslots, t_out);
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
            else lean_decide(s, stack, stride);
        }
    }
    t_out = s.best_t;
    return s.best;
}

// LDS of the bf kernels: per-lane stacks, then per wave kBfSlots x 64 hit slots, then the scene
struct BfLds {
    int32_t* stack;
    float* slot;
    char* scene;
};
__device__ __forceinline__ BfLds bf_lds(char* smem, const SceneView& sc) {
    BfLds l;
    l.stack = reinterpret_cast<int32_t*>(smem) + threadIdx.x;
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
        const int rec = bf_closest<FAST_RCP, COUNT>(sc, gtris, r, valid, l.slot, nslots, l.stack, blockDim.x, c, t);
        if (valid) wb.hitq[e] = make_int2(rec, __builtin_bit_cast(int, t));
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// ---------------------------------------------------------------------------------------------
// Packet walk + replay (traversal scenes, option packet; verdict r02 item 3): brute force + replay
// generalised past 64 distinct entries.  A wave takes 64 queue entries and
//   phase 1  walks the reference tree ONCE for all of them as a packet: a node's child is entered
//            when some lane that reached the node has dist > 0 for it (no closest-t pruning), with
//            the mask of those lanes, so the packet visits the union of the lanes' UNPRUNED walks —
//            a superset of every lane's reference walk (pruning only removes nodes).  Each leaf
//            reached is tested wave-uniformly (records through s_load, as bf_closest's phase 1);
//            per lane the hits of the lanes that reached the leaf are kept as (entry uid, t), up
//            to kPkSlots distinct uids, with their smallest t (tmin);
//   phase 2  replays each lane's reference traversal (node steps, exit-distance pruning, strict-<
//            in leaf order) where a leaf entry costs a uid lookup instead of a triangle test.
// Exact: a triangle test is a pure function of (ray, record) and duplicated records of an entry
// hold the same floats, so phase 1's t is the test's t; every leaf of the lane's walk was tested
// for the lane; entries phase 1 did not record are misses.  A lane stops once its closest t equals
// tmin (no later entry is smaller, an equal one loses the strict <); a lane with more distinct
// hits than slots replays with real tests.  A packet whose union exceeds `max_nodes` node visits
// (incoherent rays: the union approaches the whole tree) gives up and every lane walks its own
// tree with real tests (the same replay with the test switched on).
constexpr int kPkSlots = 8;
constexpr int kPkMaxNodes = 96;  // packet node visits before a wave gives up (incoherent rays)
// which launches of a batch take the packet kernel: option packet = 1: the camera rays (launch 0),
// 2: camera and shadow rays, 3: every launch
__host__ __device__ inline bool pk_launch(int mode, int it) {
    return mode >= 3 || (mode >= 1 && it == 0) || (mode == 2 && (it & 1));
}
constexpr int kPkStack = 64;  // (node, lane mask) entries per wave: <= 1 + depth of tree entries
constexpr uint32_t kPkLdsPerWave = kPkStack * 16 + kPkSlots * 64 * 8;
constexpr uint32_t kPkBlock = 256;  // 4 waves: per-lane replay stacks + 5 KB per wave of packet state

__device__ __forceinline__ void load_node_scalar(const Node* nodes, int n, float4& a, float4& b, float4& c, int4& d) {
    const __attribute__((address_space(4))) float* f = (const __attribute__((address_space(4))) float*)(nodes + n);
    a = make_float4(f[0], f[1], f[2], f[3]);
    b = make_float4(f[4], f[5], f[6], f[7]);
    c = make_float4(f[8], f[9], f[10], f[11]);
    const __attribute__((address_space(4))) int* q = (const __attribute__((address_space(4))) int*)(nodes + n);
    d = make_int4(q[12], q[13], q[14], q[15]);
}

// every loop of the kernel is bounded: a wave that exceeds kPkGuard iterations in one loop (a bug,
// never a correct walk: the replay visits each node at most once) reports like k_wf_trace's
// watchdog (ctl[WF_WATCHDOG], state in ctl[WF_SNAP..]) and stops, so the grid always drains
constexpr uint32_t kPkGuard = 1u << 22;
__device__ __forceinline__ void pk_report(const WfBuffers& wb, uint32_t where, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if (lane_id() == 0) {
        atomicOr(&wb.ctl[WF_WATCHDOG], 1u);
        if (atomicCAS(&wb.ctl[WF_SNAP_CLAIM], 0u, 1u) == 0u) {
            const uint32_t v[6] = {0xbad0000u | where, a, b, c, d, 0u};
            for (int i = 0; i < 6; ++i) wb.ctl[WF_SNAP + i] = v[i];
        }
    }
}

template <bool LDS, bool FAST_RCP>
__global__ __launch_bounds__(kPkBlock) void k_wf_trace_pk(SceneView sc, WfBuffers wb, int in_q, int max_nodes) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int32_t* stack = reinterpret_cast<int32_t*>(smem) + threadIdx.x;  // replay: per-lane stack (lane-minor)
    char* wbase = smem + (uint32_t)sc.max_stack * blockDim.x * 4u + (threadIdx.x / 64u) * kPkLdsPerWave;
    int* pnode = reinterpret_cast<int*>(wbase);                                  // [kPkStack] packet stack: node
    uint64_t* pmask = reinterpret_cast<uint64_t*>(wbase + kPkStack * 4);         // [kPkStack] lane mask
    int2* slot = reinterpret_cast<int2*>(wbase + kPkStack * 16) + lane_id();     // slot k: slot[64 k] = (uid, t)
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1] = 0;  // shade's output count
    const uint32_t count = wb.ctl[WF_WATCHDOG] ? 0u : wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];
    const Node* gnodes = sc.nodes;  // global copies for the uniform s_loads of phase 1
    const Tri* gtris = sc.tris;
    if (LDS) stage_scene_lds(sc, smem + (uint32_t)sc.max_stack * blockDim.x * 4u + (blockDim.x / 64u) * kPkLdsPerWave);
    const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    const uint32_t lane = lane_id();
    const uint32_t nb = (count + 63) / 64;
    const float4* q = in_q ? wb.shd.ray : wb.ext.ray;
    for (uint32_t bt = w; bt < nb; bt += nwaves) {  // batches of 64 entries, interleaved over waves
        const uint32_t e = bt * 64 + lane;
        const bool valid = e < count;
        uint32_t p;
        const Ray r = unpack_ray(valid ? q[2 * (size_t)e] : make_float4(0, 0, 0, 1),
                                 valid ? q[2 * (size_t)e + 1] : make_float4(0, 0, 0, 0), p);
        // ---- phase 1: the packet walk
        int nh = 0;
        bool ovf = false;
        uint64_t bloom = 0;  // bit (uid & 63) of every recorded uid
        float tmin = 3.0e38f;
        int sp = 0, visits = 0;
        const uint64_t vm = __builtin_amdgcn_ballot_w64(valid);
        if (lane == 0) { pnode[0] = 0; pmask[0] = vm; }
        sp = vm ? 1 : 0;
        bool gave_up = false;
        while (sp > 0) {  // wave-uniform
            if (visits > (int)kPkGuard) { pk_report(wb, 1, sp, visits, bt, count); return; }
            --sp;
            const int n = __builtin_amdgcn_readfirstlane(pnode[sp]);
            const uint64_t m = pmask[sp];
            if (++visits > max_nodes) { gave_up = true; break; }
            float4 a, b, c;
            int4 d;
            load_node_scalar(gnodes, n, a, b, c, d);
            const bool in = (m >> lane) & 1ull;
            const float ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
            const float rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
            const uint64_t lm = __builtin_amdgcn_ballot_w64(in && 0.0f < ld), rm = __builtin_amdgcn_ballot_w64(in && 0.0f < rd);
            for (int side = 0; side < 2; ++side) {  // uniform
                const uint64_t cm = side ? rm : lm;
                const int ref = side ? d.y : d.x, cnt = side ? d.w : d.z;
                if (!cm) continue;
                if (cnt < 0) {  // internal child: the lanes that enter it
                    if (sp >= kPkStack) { pk_report(wb, 3, sp, visits, bt, count); return; }
                    if (lane == 0) { pnode[sp] = ref; pmask[sp] = cm; }
                    ++sp;
                    continue;
                }
                const bool mine = (cm >> lane) & 1ull;
                for (int k = 0; k < cnt; ++k) {  // the leaf for the lanes in cm
                    const TriRec tr = load_tri_scalar(gtris, ref + k);
                    const f3 v0 = mk(tr.a.x, tr.a.y, tr.a.z), e1 = mk(tr.a.w, tr.b.x, tr.b.y), e2 = mk(tr.b.z, tr.b.w, tr.c);
                    const f3 rce2 = cross(r.d, e2);
                    const float det = dot(e1, rce2);
                    const float inv_det = FAST_RCP ? rcp_rn(det) : 1.0f / det;
                    const f3 sv = r.o - v0;
                    const float bu = inv_det * dot(sv, rce2);
                    const bool ok_det = !(det > -1e-8f && det < 1e-8f), ok_lo = !(bu < 0.0f), ok_hi = !(bu > 1.0f);
                    if ((cm & __builtin_amdgcn_ballot_w64(ok_det) & __builtin_amdgcn_ballot_w64(ok_lo) &
                         __builtin_amdgcn_ballot_w64(ok_hi)) == 0)
                        continue;  // wave-uniform: no lane of the leaf passes det and u
                    const f3 sce1 = cross(sv, e1);
                    const float bv = inv_det * dot(r.d, sce1);
                    const float t = inv_det * dot(e2, sce1);
                    const bool h = mine & ok_det & ok_lo & ok_hi & !(bv < 0.0f) & !(bu + bv > 1.0f) & (t > 1e-8f);
                    if (h) {
                        const int uid = (int)sload_u32(reinterpret_cast<const uint32_t*>(&gtris[ref + k].uid));
                        bool seen = false;
                        if ((bloom >> (uid & 63)) & 1ull)
                            for (int j = 0; j < min(nh, kPkSlots); ++j) seen |= slot[64 * j].x == uid;
                        if (!seen) {
                            if (nh < kPkSlots) slot[64 * nh] = make_int2(uid, __builtin_bit_cast(int, t));
                            else ovf = true;
                            ++nh;
                            bloom |= 1ull << (uid & 63);
                            tmin = t < tmin ? t : tmin;
                        }
                    }
                }
            }
        }
        // ---- phase 2: each lane's reference walk; leaf entries from phase 1 (or real tests when the
        // packet gave up / the lane overflowed its slots)
        const bool real = gave_up || ovf;
        int best = -1;
        float best_t = -1.0f;
        bool go = valid && (real || nh > 0);
        int node = 0, rsp = 0;
        for (uint32_t guard = 0; wave_any(go); ++guard) {
            if (guard > kPkGuard) { pk_report(wb, 2, guard, (uint32_t)node, bt, count); return; }
            if (go) {
                const float4* np = reinterpret_cast<const float4*>(sc.nodes) + 4 * node;
                const float4 a = np[0], b = np[1], c = np[2];
                const int4 d = reinterpret_cast<const int4*>(np)[3];
                const float ld = ray_box(r, a.x, a.y, a.z, a.w, b.x, b.y);
                const float rd = ray_box(r, b.z, b.w, c.x, c.y, c.z, c.w);
                const bool li = 0.0f < ld, ri = 0.0f < rd;
                const bool lleaf = d.z >= 0, rleaf = d.w >= 0;
                const int na = (li && lleaf) ? d.z : 0, nt = na + ((ri && rleaf) ? d.w : 0);
                for (int k = 0; k < nt; ++k) {  // the leaf pair in the reference's order
                    const int idx = k < na ? d.x + k : d.y + (k - na);
                    float t = 0.0f;
                    bool hit = false;
                    if (real) {
                        hit = tri_hit<FAST_RCP>(sc.tris, idx, r, t);
                    } else {
                        const int uid = sc.tris[idx].uid;
                        if ((bloom >> (uid & 63)) & 1ull)
                            for (int j = 0; j < nh; ++j) {
                                const int2 sl = slot[64 * j];
                                if (sl.x == uid) { hit = true; t = __builtin_bit_cast(float, sl.y); }
                            }
                    }
                    if (hit && (best_t < 0.0f || t < best_t)) { best_t = t; best = idx; }
                }
                if (!real && best_t == tmin) {
                    go = false;  // final: no later entry has a smaller t
                } else {
                    const bool tl = li && !lleaf && !(best_t > 0.0f && ld > best_t);
                    const bool tr = ri && !rleaf && !(best_t > 0.0f && rd > best_t);
                    if (tl && tr) {
                        stack[rsp * blockDim.x] = d.x;
                        ++rsp;
                        node = d.y;
                    } else if (tl) {
                        node = d.x;
                    } else if (tr) {
                        node = d.y;
                    } else if (rsp == 0) {
                        go = false;
                    } else {
                        --rsp;
                        node = stack[rsp * blockDim.x];
                    }
                }
            }
        }
        if (valid) wb.hitq[e] = make_int2(best, __builtin_bit_cast(int, best_t));
    }
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
// instead of queue batch b (streaming regeneration and the first launch); -1 reads the queue.
template <bool EXT, bool FAST_RCP, bool COUNT, bool GEN = false, class Append>
__device__ __forceinline__ void bf_step_batch(const SceneView& sc, const Tri* gtris, const FrameParams& fp,
                                              const WfBuffers& wb, size_t rbase, uint32_t b, uint32_t count,
                                              const BfLds& l, int nslots, Counters& c, Append append,
                                              bool cull = false,  // cull: wave-uniform (bf_cull_mask)
                                              const GenArgs& gen = GenArgs{}, int64_t genk = -1) {
    const WfQueue& in = EXT ? wb.ext : wb.shd;
    const WfQueue& out = EXT ? wb.shd : wb.ext;
    const uint32_t lane = lane_id();
    uint64_t tm[6];
    if (PT_PHASE_TIMING) tm[0] = phase_clock();
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
    const uint64_t todo = cull ? bf_cull_mask(sc, r, valid, sc.n_tris - sc.mb_base) : ~0ull;  // before the prefetch: fewer live VGPRs
    // the path state is loaded before the trace and arrives while it runs (kBfPrefetch)
    if (!fresh && kBfPrefetch) {
        if (EXT) { c2 = in.q2[e]; d3 = in.q3[e]; }
        else { a1 = in.ray[2 * e + 1]; c2 = in.q2[e]; }
    }
    float t;
    if (PT_PHASE_TIMING) tm[1] = phase_clock();
    const int rec = bf_closest<FAST_RCP, COUNT, EXT ? kBfPacked : kBfPackedShadow>(sc, gtris, r, valid, l.slot, nslots, l.stack, blockDim.x, c, t, todo,
                                                PT_PHASE_TIMING ? &tm[2] : nullptr);
    if (PT_PHASE_TIMING) tm[3] = phase_clock();
    bool more = false;
    PathState ps;
    if (valid) {
        if (!fresh && !kBfPrefetch) {
            if (EXT) { c2 = in.q2[e]; d3 = in.q3[e]; }
            else { a1 = in.ray[2 * e + 1]; c2 = in.q2[e]; }
        }
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
    const uint64_t keep = __ballot(more);
    if (PT_PHASE_TIMING) tm[4] = phase_clock();
    if (keep) {  // wave-uniform
        uint32_t base = 0;
        if (lane == 0) base = append((uint32_t)__popcll(keep));
        base = __shfl(base, 0, 64);
        if (more) {
            const uint32_t j = (uint32_t)rbase + base + rank_below(keep);
            if (EXT) store_shadow_packed(wb, j, r, p, ps);
            else store_entry(out, j, r, p, ps);
        }
    }
#if PT_PHASE_TIMING
    // slots: 0 load + cull, 1 phase 1, 2 phase 2, 3 shading, 4 append + stores, 5 batches
    tm[5] = phase_clock();
    const uint32_t wv = (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) % kPhaseWaves;
    if (lane == 0) {
        unsigned long long* g = g_phase + (size_t)wv * kPhaseSlots + (EXT ? 0 : 8);
        for (int k = 0; k < 5; ++k) atomicAdd(g + k, (unsigned long long)(tm[k + 1] - tm[k]));
        atomicAdd(g + 5, 1ull);
    }
#endif
}

// Trace + shade in one launch per iteration (mailbox scenes; persist=0): queues are cut
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
// CULL: the entry cull (bf_cull_mask) — its own instance, so the launches without it keep
// their register allocation (the cull code costs VGPR spills at the 64-VGPR cap)
// GEN: the first launch makes the camera paths itself (bf_step_batch GEN; replaces
// k_wf_generate): region counts in closed form, the output counts zeroed by the host.
template <bool EXT, bool LDS, bool FAST_RCP, bool COUNT, bool CULL = false, bool GEN = false>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_wf_step_bf(SceneView sc, FrameParams fp, WfBuffers wb, int it,
                                                           Counters* cnt_out, int nslots, uint32_t frame0,
                                                           uint32_t stride, uint32_t fbase, uint32_t P, bool raw_salt) {
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
    uint32_t count, nqb, nnew = 0;
    if constexpr (GEN) {  // k_wf_generate's closed-form count of region rg
        const uint32_t last = tg + (ncam - 1) * R;
        count = ncam == 0 ? 0u : ncam * 64 - ((last == nbat - 1 && (P & 63)) ? 64 - (P & 63) : 0u);
        if (w == 0 && lane_id() == 0) { wb.ctl[WF_COUNT0] = P; wb.ctl[WF_COUNT1] = 0; }
        nqb = 0;
        nnew = ncam;
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
    for (uint32_t b = g; b < nb; b += G)  // this region's batches, interleaved over its waves
        bf_step_batch<EXT, FAST_RCP, COUNT, GEN>(sc, gtris, fp, wb, (size_t)rg * wb.rstride, b, count, l, nslots, c,
                                                 [&](uint32_t n) { return atomicAdd(out_count, n); }, CULL, ga,
                                                 b < nqb ? (int64_t)-1 : (int64_t)(b - nqb));
    if (COUNT) flush_counters(c, cnt_out);
}

// Streaming path regeneration (the default for the fused kernel): the render's P paths are the
// camera batches of the regions (camera batch k of region r: paths (k R + r) 64 + lane).  Every
// extension launch e = it / 2 tops region r up from its queued count c to wb.target entries with
// the region's next camera batches: after the c queued entries come batches rgen[e % 2][r] ..
// + n_new, made in registers by the wave that traces them (no queue write or read of camera rays),
// and the region's cursor moves to slot (e + 1) % 2.  So the queues stay full until the camera
// batches run out — one per-bounce tail at the end of the render instead of one per batch of
// frames.  Each path writes its radiance to rad[p] when it ends; k_wf_accum adds them in frame
// order afterwards, so the result is bit-identical.
// Scheduling: region r is served by the waves w ≡ r (mod R) (with 8 waves per block and
// R = 512 all of them sit in blocks b ≡ b0 (mod 64), so on one XCD when the dispatcher deals
// blocks round-robin to the 8 XCDs: a region's queue and path state stay in one L2), and those
// waves take the region's batches from the region's counter rfetch[it % 3][r] (one cache line
// per region: device-scope atomics on one line serialise at ~12 ns each) instead of a static
// interleave: a static split of ~16 batches per wave left the slowest of 8192 waves ~25 % behind
// the mean at every launch.  A wave fetches its next batch while it works on the current one.
// Wave g == 0 of each region keeps its books: the next launch's count and fetch slots zeroed,
// the camera cursor, and live[it % kLiveRing] = regions with work left (queued entries or camera
// batches); the host stops launching when a launch saw none.
template <bool EXT, bool LDS, bool FAST_RCP, bool COUNT>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_wf_regen_bf(
    SceneView sc, FrameParams fp, WfBuffers wb, int it, Counters* cnt_out, int nslots, uint32_t frame0,
    uint32_t stride, uint32_t fbase, uint32_t P, bool raw_salt) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const BfLds l = bf_lds(smem, sc);
    const uint32_t lane = lane_id();
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    const uint32_t R = wb.nreg;  // <= waves (host)
    const uint32_t rg = w % R, g = w / R;
    const uint32_t e = (uint32_t)it / 2;
    const uint32_t nbat = (P + 63) / 64;
    const uint32_t ncam = rg < nbat ? (nbat - rg + R - 1) / R : 0u;  // camera batches of region rg
    const uint32_t count = wb.rcnt[(it % 3) * kRegions + rg];
    const uint32_t k0 = wb.rgen[((EXT ? e : e + 1) % 2) * kRegions + rg];
    const uint32_t nnew = EXT && wb.target > count ? min((wb.target - count) / 64, ncam - k0) : 0u;
    const uint32_t nqb = (count + 63) / 64, nb = nqb + nnew;
    if (g == 0 && lane == 0) {  // region rg's books
        wb.rcnt[((it + 2) % 3) * kRegions + rg] = 0;
        wb.rfetch[(((it + 2) % 3) * kRegions + rg) * kFetchStride] = 0;
        if (EXT) wb.rgen[((e + 1) % 2) * kRegions + rg] = k0 + nnew;
        if (count > 0 || k0 < ncam) atomicAdd(&wb.live[it % kLiveRing], 1u);
        if (rg == 0) wb.live[(it + 2) % kLiveRing] = 0;
    }
    uint32_t* out_count = &wb.rcnt[((it + 1) % 3) * kRegions + rg];
    uint32_t* fetch = &wb.rfetch[((it % 3) * kRegions + rg) * kFetchStride];
    const Tri* gtris = sc.tris;  // global records for phase 1
    if (LDS) stage_scene_lds(sc, l.scene);
    const GenArgs ga{frame0, stride, fbase, R, rg, P, raw_salt};
    Counters c = {};
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(fetch, 1u);
    b = __builtin_amdgcn_readfirstlane(b);
    while (b < nb) {
        uint32_t bn = 0;
        if (lane == 0) bn = atomicAdd(fetch, 1u);  // the next batch, in flight while this one runs
        bf_step_batch<EXT, FAST_RCP, COUNT, EXT>(sc, gtris, fp, wb, (size_t)rg * wb.rstride, b, count, l, nslots, c,
                                                 [&](uint32_t n) { return atomicAdd(out_count, n); }, false, ga,
                                                 b < nqb ? (int64_t)-1 : (int64_t)(k0 + (b - nqb)));
        b = __builtin_amdgcn_readfirstlane(bn);
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// One launch per batch of paths (mailbox scenes, the default): workgroup g owns region g of the
// queues — the 64-path batches j ≡ g (mod gridDim.x) of the batch's P paths — and runs all of
// their bounces alone.  Its 8 waves write the camera rays, then in every iteration take the
// region's 64-entry queue batches from an LDS counter, trace + shade them (bf_step_batch) and
// append survivors through another LDS counter; a workgroup barrier ends the iteration (its
// global stores are visible to the workgroup's other waves after it: one CU, one L1).  No
// grid-wide step between bounces: no kernel boundary per bounce, no global atomics, and a
// workgroup waiting at its barrier leaves the CU to the other resident workgroups.
template <bool LDS, bool FAST_RCP, bool COUNT>
__global__ __launch_bounds__(kTraceBlock) void k_wf_persist_bf(SceneView sc, FrameParams fp, WfBuffers wb, uint32_t frame0,
                                                              uint32_t stride, uint32_t fbase, uint32_t P, bool raw_salt,
                                                              int iters, Counters* cnt_out, int nslots) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ uint32_t s_cnt[2], s_next;
    const BfLds l = bf_lds(smem, sc);
    const uint32_t lane = lane_id();
    const uint32_t R = gridDim.x, rg = blockIdx.x;
    const size_t rbase = (size_t)rg * wb.rstride;
    const uint32_t nbat = (P + 63) / 64;
    const uint32_t nmine = rg < nbat ? (nbat - rg + R - 1) / R : 0u;  // this region's 64-path batches
    const Tri* gtris = sc.tris;  // global records for phase 1
    if (LDS) stage_scene_lds(sc, l.scene);
    Counters c = {};
    const uint32_t wv = threadIdx.x / 64, nwv = blockDim.x / 64;
    for (uint32_t k = wv; k < nmine; k += nwv) {  // camera rays: local batch k = global batch rg + k R
        const uint32_t p = (rg + k * R) * 64 + lane;
        if (p < P) {
            uint32_t x, y, f;
            const uint32_t pid = slot_path(p, fp, x, y, f);
            const uint32_t t = raw_salt ? frame0 : (uint32_t)(float)(frame0 + (fbase + f) * stride);
            PathState ps;
            const Ray r = path_begin(fp, x, y, t, ps);
            store_entry(wb.ext, (uint32_t)(rbase + k * 64 + lane), r, pid, ps);
            if (COUNT) { c.samples++; c.ext_queries++; }
        }
    }
    if (threadIdx.x == 0) {
        const uint32_t last = rg + (nmine - 1) * R;
        s_cnt[0] = nmine == 0 ? 0u : nmine * 64 - ((last == nbat - 1 && (P & 63)) ? 64 - (P & 63) : 0u);
        s_cnt[1] = 0;
        s_next = 0;
    }
    __syncthreads();
    for (int it = 0; it < iters; ++it) {
        const uint32_t count = s_cnt[it & 1];
        uint32_t* out_cnt = &s_cnt[(it + 1) & 1];
        const uint32_t nb = (count + 63) / 64;
        while (true) {  // the region's batches, handed to the waves as they come free
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&s_next, 1u);
            b = __shfl(b, 0, 64);
            if (b >= nb) break;
            auto append = [&](uint32_t n) { return atomicAdd(out_cnt, n); };
            if ((it & 1) == 0) bf_step_batch<true, FAST_RCP, COUNT>(sc, gtris, fp, wb, rbase, b, count, l, nslots, c, append);
            else bf_step_batch<false, FAST_RCP, COUNT>(sc, gtris, fp, wb, rbase, b, count, l, nslots, c, append);
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // this input count becomes iteration it + 1's output count
            s_cnt[it & 1] = 0;
            s_next = 0;
        }
        __syncthreads();
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// Megakernel with brute force + replay (mailbox scenes, kernel=mega with regen_bf=1): the
// layout of k_regen — lane = pixel of an 8x8 tile, the pixel's frames in order, a lane whose
// path ended starts its next frame at once, clamp(L) accumulated in registers — with every
// query of the wave resolved by bf_closest.  Extension and shadow rays of different lanes share
// one phase 1 (a triangle test does not care which kind of ray it serves), so there are no
// queues, no compaction and no kernel boundary between bounces.
constexpr int kRegenBfBlock = 256;
template <bool LDS, bool FAST_RCP, bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kRegenBfBlock) __attribute__((amdgpu_waves_per_eu(8, 8)))
void k_regen_bf(SceneView sc, FrameParams fp, uint32_t frame0, uint32_t nframes, uint32_t stride, float* __restrict__ out,
                Counters* cnt_out, int nslots) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const BfLds l = bf_lds(smem, sc);
    const Tri* gtris = sc.tris;
    if (LDS) stage_scene_lds(sc, l.scene);
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7), y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    Counters c = {};
    const bool valid = x < fp.width && y < fp.height;
    float* o = out + 3 * ((size_t)(valid ? y : 0) * fp.width + (valid ? x : 0));
    f3 acc = (ACCUM && valid) ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);
    enum { kIdle = 0, kExt = 1, kShadow = 2 };
    int phase = kIdle;
    uint32_t next = 0;  // next frame of this pixel to start
    Ray ray;
    ray.o = ray.d = ray.inv = mk(0.0f, 0.0f, 0.0f);
    PathState ps;
    while (true) {
        if (phase == kIdle && valid && next < nframes) {
            const uint32_t t = ACCUM ? (uint32_t)(float)(frame0 + next * stride) : frame0;
            ++next;
            ray = path_begin(fp, x, y, t, ps);
            phase = kExt;
            if (COUNT) { c.samples++; c.ext_queries++; }
        }
        const bool live = phase != kIdle;
        if (!wave_any(live)) break;  // wave-uniform: every lane's frames are done
        float t;
        const int rec = bf_closest<FAST_RCP, COUNT, true>(sc, gtris, ray, live, l.slot, nslots, l.stack, blockDim.x, c, t);
        if (live) {
            bool more;
            if (phase == kExt) {
                more = path_after_ext(sc, rec, t, ray, ps);
                if (more) { phase = kShadow; if (COUNT) c.shadow_queries++; }
            } else {
                more = path_after_shadow(sc, fp, rec, t, ray, ps);
                if (more) { phase = kExt; if (COUNT) c.ext_queries++; }
            }
            if (!more) {
                acc = ACCUM ? add_clamped(acc, ps.L) : ps.L;
                phase = kIdle;
            }
        }
    }
    if (valid) { o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; }
    if (COUNT) flush_counters(c, cnt_out);
}

hipError_t launch_regen_bf(const LaunchOpts& lo, const SceneView& sc_in, const FrameParams& fp, uint32_t frame0,
                           uint32_t nframes, uint32_t stride, bool accum, bool count, float* out, Counters* cnt,
                           hipStream_t stream) {
    SceneView sc = sc_in;
    if (!count && sc.bfnode) sc.max_stack = 0;  // the stackless replay (bf_view)
    const bool lds = lo.lds && scene_fits_lds(sc);
    const bool fast = lo.fast_rcp != 0 && sc.fast_rcp;
    const int slots = lo.bf_slots >= 0 ? std::min(kBfSlots, lo.bf_slots) : kBfSlots;  // < kBfSlots: tests of the recompute path
    dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kRegenBfBlock);
    const size_t shm = (size_t)sc.max_stack * kRegenBfBlock * 4 + (kRegenBfBlock / 64) * (kBfSlots * 64 * 4) +
                       (lds ? sc.span_bytes : 0);
#define RB(L, F, A, C)                                                                                          \
    PT_LAUNCH(KID_REGEN, stream, (k_regen_bf<L, F, A, C>), grid, block, shm, stream, sc, fp, frame0, nframes, stride, \
              out, cnt, slots)
#define RB_AC(L, F) \
    if (accum) { if (count) RB(L, F, true, true); else RB(L, F, true, false); } else { if (count) RB(L, F, false, true); else RB(L, F, false, false); }
    if (lds) { if (fast) { RB_AC(true, true) } else { RB_AC(true, false) } }
    else { if (fast) { RB_AC(false, true) } else { RB_AC(false, false) } }
#undef RB_AC
#undef RB
    return hipGetLastError();
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
template <bool LDS, int TRAV, bool COUNT>
constexpr const void* trace_kernel() {
    if constexpr (TRAV >= 500) return (const void*)k_wf_persist_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>;
    else if constexpr (TRAV >= 400) return (const void*)k_wf_step_bf<false, LDS, ((TRAV / 10) & 1) != 0, COUNT>;
    else if constexpr (TRAV >= 300) return (const void*)k_wf_trace_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>;
    else return (const void*)k_wf_trace<LDS, TRAV, COUNT>;
}
template <bool LDS, int TRAV, bool COUNT>
static size_t trace_lds(const SceneView& sc, uint32_t ring = kHitRing) {
    const size_t per_wave = TRAV >= 300 ? (size_t)kBfSlots * 64 * 4 : stage_bytes(ring);
    constexpr uint32_t B = trace_block<TRAV>();
    return (size_t)sc.max_stack * B * 4 + (B / 64) * per_wave + (LDS ? sc.span_bytes : 0);
}
template <bool LDS, int TRAV, bool COUNT>
static int trace_blocks(size_t lds_bytes) {
    static int cached = 0;
    static size_t cached_lds = 0;
    int& b = cached;
    if (b == 0 || cached_lds != lds_bytes) {
        int per_cu = 0, dev = 0, cus = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_kernel<LDS, TRAV, COUNT>(), trace_block<TRAV>(), lds_bytes);
        b = std::max(1, per_cu) * std::max(1, cus);
        cached_lds = lds_bytes;
    }
    return b;
}

// Paths [0, P) of part h of nparts of a batch: queue entries from h * qcap/nparts, radiance from
// `rad_off` floats (so the parts' radiance is contiguous in frame order), control words from
// h * WF_CTL_WORDS, region counts from h * 3 * kRegions.
static WfBuffers wb_part(const WfBuffers& wb, int h, int nparts, size_t rad_off) {
    WfBuffers v = wb;
    const size_t e = (size_t)h * (wb.qcap / nparts);
    for (WfQueue* q : {&v.ext, &v.shd}) { q->ray += 2 * e; q->q2 += e; q->q3 += e; }
    v.sp0 += e; v.sp1 += e; v.sp2 += e; v.hitq += e;
    v.rad += rad_off;
    v.ctl += h * WF_CTL_WORDS;
    v.rcnt += h * 3 * kRegions;
    v.rgen += h * 2 * kRegions;
    v.live += h * kLiveRing;
    v.rfetch += h * 3 * kRegions * kFetchStride;
    v.capacity = wb.capacity / nparts;
    v.qcap = wb.qcap / nparts;
    return v;
}

// Streaming regeneration (k_wf_regen_bf): the call's frames in groups whose radiance
// fits wb.rad_cap paths; a group's frames are dealt to the parts in contiguous runs, each part on
// its own stream runs extension / shadow launches until a launch finds no work left in any
// region (the host polls live[] every kPollChunk launches through pinned memory, one chunk
// ahead, so the stream never waits for the host), then k_wf_accum adds the group's frames in
// order.
constexpr int kPollChunk = 8;
template <bool LDS, int TRAV, bool COUNT>
static hipError_t wf_render_regen(const SceneView& sc, const FrameParams& fp, const WfBuffers& wb, uint32_t frame0,
                                  uint32_t nframes, uint32_t stride, bool accum, float* out, Counters* cnt,
                                  hipStream_t stream, const WfStreams& ws, int tblocks, size_t lds, int bf_slots) {
    constexpr bool rcp = ((TRAV / 10) & 1) != 0;
    const uint32_t npix = fp.width * fp.height;
    const int np = (ws.aux[0] != nullptr && ws.h_poll) ? ws.nparts : 1;
    const uint32_t Fs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nframes, wb.rad_cap / npix));
    const uint32_t R = std::min<uint32_t>(kRegions, (uint32_t)tblocks * (kTraceBlock / 64));
    for (uint32_t fb = 0; fb < nframes; fb += Fs) {
        const uint32_t Fb = std::min(Fs, nframes - fb);
        const int nh = (int)std::min<uint32_t>((uint32_t)np, Fb);
        struct Part { WfBuffers w; uint32_t fbase, P, ncam_max; hipStream_t st; int it, chunk; bool done; };
        Part pv[kMaxParts];
        uint32_t f0 = 0;
        for (int h = 0; h < nh; ++h) {
            const uint32_t fh = (Fb - f0 + (nh - h) - 1) / (nh - h);  // frames left over parts left
            Part& q = pv[h];
            q.w = np > 1 ? wb_part(wb, h, np, (size_t)f0 * npix * 3) : wb;
            q.fbase = fb + f0;
            q.P = fh * npix;
            q.st = np > 1 ? ws.aux[h] : stream;
            q.w.nreg = R;
            q.w.rq = q.w.rqi = 1;
            q.w.rstride = q.w.qcap / R / 64 * 64;  // >= capacity / R (queue slack)
            uint64_t T = q.w.capacity;
            if (ws.regen_target) T = std::min<uint64_t>(T, ws.regen_target / (uint64_t)nh);
            q.w.target = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(64, T / R / 64 * 64), q.w.rstride);
            const uint32_t nbat = (q.P + 63) / 64;
            q.ncam_max = (nbat + R - 1) / R;
            q.it = 0;
            q.chunk = 0;
            q.done = false;
            f0 += fh;
        }
        if (np > 1) {
            HIP_RETURN_IF(hipEventRecord(ws.fork, stream));
            for (int h = 0; h < nh; ++h) HIP_RETURN_IF(hipStreamWaitEvent(pv[h].st, ws.fork, 0));
        }
        for (int h = 0; h < nh; ++h) {  // counts of launches 0 (read) and 1 (appended), camera cursors, liveness
            HIP_RETURN_IF(hipMemsetAsync(pv[h].w.rcnt, 0, 2 * kRegions * sizeof(uint32_t), pv[h].st));
            HIP_RETURN_IF(hipMemsetAsync(pv[h].w.rgen, 0, kRegions * sizeof(uint32_t), pv[h].st));
            HIP_RETURN_IF(hipMemsetAsync(pv[h].w.live, 0, kLiveRing * sizeof(uint32_t), pv[h].st));
            HIP_RETURN_IF(hipMemsetAsync(pv[h].w.rfetch, 0, 2 * kRegions * kFetchStride * sizeof(uint32_t), pv[h].st));
        }
        // a hard bound on the launches (every path at most 2 (D + 1) launches; a region makes at
        // least one camera batch per extension launch while it has room): a bug, never a hang
        int left = nh;
        while (left > 0) {
            for (int h = 0; h < nh; ++h) {
                Part& q = pv[h];
                if (q.done) continue;
                const int cap = 2 * (fp.max_depth + 1) * ((int)q.ncam_max + 2) + 64;
                if (q.it > cap) return hipErrorLaunchFailure;
                for (int k = 0; k < kPollChunk; ++k, ++q.it) {
#define PT_RSTEP(E) PT_LAUNCH(KID_WF_STEP, q.st, (k_wf_regen_bf<E, LDS, rcp, COUNT>), dim3(tblocks), \
                              dim3(kTraceBlock), lds, q.st, sc, fp, q.w, q.it, cnt, bf_slots, frame0, stride, q.fbase, \
                              q.P, !accum)
                    if ((q.it & 1) == 0) PT_RSTEP(true);
                    else PT_RSTEP(false);
#undef PT_RSTEP
                }
                const int slot = q.chunk & 1;
                HIP_RETURN_IF(hipMemcpyAsync(&ws.h_poll[2 * h + slot], q.w.live + (q.it - 1) % kLiveRing, sizeof(uint32_t),
                                             hipMemcpyDeviceToHost, q.st));
                HIP_RETURN_IF(hipEventRecord(ws.poll_ev[h][slot], q.st));
                ++q.chunk;
            }
            for (int h = 0; h < nh; ++h) {  // the chunk before the one just queued: did its last launch find work?
                Part& q = pv[h];
                if (q.done || q.chunk < 2) continue;
                const int slot = (q.chunk - 2) & 1;
                HIP_RETURN_IF(hipEventSynchronize(ws.poll_ev[h][slot]));
                if (__atomic_load_n(&ws.h_poll[2 * h + slot], __ATOMIC_ACQUIRE) == 0) {
                    q.done = true;
                    --left;
                }
            }
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
    const SceneView sc = bf_view<TRAV, COUNT>(sc_in);
    const uint32_t npix = fp.width * fp.height;
    // the batch in ws.nparts parts on as many streams when a part holds at least a frame: one
    // part's kernel fills the others' launch tails and boundaries (and, with separate trace and
    // shade kernels, a VALU-bound trace runs beside an HBM-bound shade)
    int np = ws.aux[0] != nullptr ? ws.nparts : 1;
    while (np > 1 && (nframes < (uint32_t)np || wb.capacity / np < npix)) np /= 2;
    const uint32_t F = np * std::max<uint32_t>(1, std::min<uint32_t>((nframes + np - 1) / np, (uint32_t)(wb.capacity / np / npix)));
    size_t lds = trace_lds<LDS, TRAV, COUNT>(sc);
    int tblocks = trace_blocks<LDS, TRAV, COUNT>(lds);
    // k_wf_trace's hit ring: 256 entries when the extra 8 KB per block cost no block per CU (option
    // trace_ring: 128 / 256 forces one)
    uint32_t nring = kHitRing;
    (void)nring;
    if constexpr (TRAV < 300 && has_big_ring(TRAV)) {
        const size_t lds2 = trace_lds<LDS, TRAV, COUNT>(sc, kHitRingMax);
        static const size_t max_lds = [] {
            int dev = 0, v = 0;
            hipGetDevice(&dev);
            hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
            return (size_t)v;
        }();
        const bool fits = lds2 <= max_lds && (ws.trace_ring == (int)kHitRingMax ||
                                                 (ws.trace_ring <= 0 && trace_blocks<LDS, TRAV, COUNT>(lds2) >= tblocks));
        if (fits) {
            lds = lds2;
            tblocks = trace_blocks<LDS, TRAV, COUNT>(lds2);
            nring = kHitRingMax;
        }
    }
    // k_wf_trace_pk (option packet): its LDS (per-lane replay stacks, per-wave packet stack and hit
    // slots, the scene when it fits) and an occupancy-derived grid
    const size_t pk_lds = (size_t)sc.max_stack * kPkBlock * 4 + (kPkBlock / 64) * kPkLdsPerWave + (LDS ? sc.span_bytes : 0);
    const bool pk_ok = pk_lds <= 64 * 1024;  // a workgroup's LDS limit; else the traversal kernel runs
    auto pk_blocks = [&](size_t bytes) {
        static int cached = 0;
        static size_t cached_bytes = 0;
        if (!cached || cached_bytes != bytes) {
            int per_cu = 0, dev = 0, cus = 0;
            hipGetDevice(&dev);
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_wf_trace_pk<LDS, ((TRAV / 10) & 1) != 0>,
                                                         kPkBlock, bytes);
            cached = std::max(1, per_cu) * std::max(1, cus);
            cached_bytes = bytes;
        }
        return ws.trace_blocks > 0 ? std::min(cached, ws.trace_blocks) : cached;
    };
    if (ws.trace_blocks > 0) tblocks = std::min(tblocks, ws.trace_blocks);  // option wf_trace_blocks (tests)
    const int iters = 2 * (fp.max_depth + 1);
    // option trace_watchdog: tests of the failure report
    const uint32_t watchdog = ws.watchdog > 0 ? ws.watchdog : kTraceWatchdog;
    // option trace_dyn=1: k_wf_trace takes its windows from group counters (opt-in: with two parts the
    // static split is 4 % faster on Glossy and the 100k synthetic scene, the counters 2 % on the boat)
    const int trace_dyn = (ws.trace_dyn ? 1 : 0) | (std::max(0, std::min(ws.trace_sparse, 1 << 20)) << 1);
    // option bf_slots < kBfSlots: tests of the recompute path
    const int bf_slots = ws.bf_slots >= 0 ? std::min(kBfSlots, ws.bf_slots) : kBfSlots;
    if constexpr (TRAV >= 500) {  // one workgroup-local launch per batch (k_wf_persist_bf), one stream
        const uint32_t Fp = std::max<uint32_t>(1, std::min<uint32_t>(nframes, wb.capacity / npix));
        const uint32_t nblk = std::min<uint32_t>((uint32_t)tblocks, kPersistMaxBlocks);
        WfBuffers w = wb;
        w.rstride = w.qcap / nblk / 64 * 64;  // >= ceil(batches / nblk) * 64 (queue slack)
        for (uint32_t fb = 0; fb < nframes; fb += Fp) {
            const uint32_t Fb = std::min(Fp, nframes - fb);
            PT_LAUNCH(KID_WF_STEP, stream, (k_wf_persist_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>), dim3(nblk),
                      dim3(kTraceBlock), lds, stream, sc, fp, w, frame0, stride, fb, Fb * npix, !accum, iters, cnt,
                      bf_slots);
            PT_LAUNCH(KID_WF_ACCUM, stream, k_wf_accum, dim3((npix + 255) / 256), dim3(256), 0, stream, wb.rad, out, npix,
                      Fb, accum);
        }
        return hipGetLastError();
    }
    if constexpr (TRAV >= 400 && TRAV < 500) {
        if (ws.regen)
            return wf_render_regen<LDS, TRAV, COUNT>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream, ws,
                                                     tblocks, lds, bf_slots);
    }
    // Batch pipelining (option batch_pipe, two parts, more than one batch): without it both parts
    // start every batch together behind a fork and the accumulation joins them, so their launch
    // tails (the last depths, few paths each) coincide and leave the machine idle.  With it part 1
    // starts the call half a batch behind part 0 and neither waits for the other again: batches
    // alternate between two radiance buffers, the accumulation of batch b (on the caller's stream)
    // joins the parts' batch b, and a part reuses a buffer only behind the accumulation that read
    // it.  Every path computes the same bits and the accumulation order is unchanged.
    const uint32_t nbatches = (nframes + F - 1) / F;
    const bool pipe = np == 2 && ws.pipeline && !ws.stagger && nbatches > 1 && ws.mid && ws.acc_done[0] &&
                      wb.rad_cap >= 2ull * wb.capacity;
    uint32_t b = 0;
    for (uint32_t fb = 0; fb < nframes; fb += F, ++b) {
        const uint32_t Fb = std::min(F, nframes - fb);
        WfBuffers wbb = wb;
        if (pipe) wbb.rad += (size_t)(b & 1) * wb.capacity * 3;
        // frames of the batch dealt to the parts in contiguous runs (part h: frames fb + f0[h] ..)
        struct Part { WfBuffers w; uint32_t fbase, P; hipStream_t st; };
        Part pv[kMaxParts];
        int nh = 0;
        uint32_t f0 = 0;
        for (int h = 0; h < np && f0 < Fb; ++h) {
            const uint32_t fh = std::min<uint32_t>((Fb + np - 1) / np, Fb - f0);
            pv[nh].w = np > 1 ? wb_part(wbb, h, np, (size_t)f0 * npix * 3) : wbb;
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
        if (np > 1 && (!pipe || b == 0)) {
            HIP_RETURN_IF(hipEventRecord(ws.fork, stream));
            for (int h = 0; h < nh; ++h) HIP_RETURN_IF(hipStreamWaitEvent(pv[h].st, ws.fork, 0));
        } else if (pipe && b >= 2) {  // the radiance buffer of batch b - 2 has been accumulated
            for (int h = 0; h < nh; ++h) HIP_RETURN_IF(hipStreamWaitEvent(pv[h].st, ws.acc_done[b & 1], 0));
        }
        // the fused kernel's first launch makes the camera paths itself (GEN); it appends into
        // count slot 1, zeroed here (k_wf_generate zeroes it otherwise)
        const bool fgen = TRAV >= 400 && TRAV < 500 && ws.fuse_gen;
        for (int h = 0; h < nh; ++h) {
            if (fgen)
                HIP_RETURN_IF(hipMemsetAsync(pv[h].w.rcnt + kRegions, 0, kRegions * sizeof(uint32_t), pv[h].st));
            else
                PT_LAUNCH(KID_WF_GENERATE, pv[h].st, (k_wf_generate<COUNT>),
                          dim3((std::max(pv[h].P, pv[h].w.nreg) + 255) / 256), dim3(256), 0, pv[h].st,
                          fp, pv[h].w, frame0, stride, pv[h].fbase, pv[h].P, !accum, cnt);
        }
        // Optional staggering (option stagger=1, two parts; measured slower: 1026 vs 1231 Msamples/s):
        // part 1's trace i waits for part 0's trace i and part 0's trace i+1 for part 1's trace i,
        // so the persistent trace kernels never share the machine.  Default: parts overlap freely.
        const bool stagger = nh == 2 && ws.stagger;
        // launch `it` of part h (in_q: the queue the trace kernels read, it & 1)
        auto step = [&](int h, int it) -> hipError_t {
            const int in_q = it & 1;
            const hipStream_t st = pv[h].st;
            const WfBuffers& w = pv[h].w;
            const int sblocks = (int)((pv[h].P + kShadeBlock - 1) / kShadeBlock);
            if (stagger && (h == 1 || it > 0)) HIP_RETURN_IF(hipStreamWaitEvent(st, ws.traced[1 - h], 0));
            if constexpr (TRAV >= 400) {  // trace + shade in one launch
                constexpr bool rcp = ((TRAV / 10) & 1) != 0;
                const bool cull = it < sc.cull_its;
                const bool g0 = fgen && it == 0;
#define PT_STEP(E, C, G) PT_LAUNCH(KID_WF_STEP, st, (k_wf_step_bf<E, LDS, rcp, COUNT, C, G>), dim3(tblocks), \
                                   dim3(kTraceBlock), lds, st, sc, fp, w, it, cnt, bf_slots, frame0, stride,   \
                                   pv[h].fbase, pv[h].P, !accum)
                if (g0 && cull) PT_STEP(true, true, true);
                else if (g0) PT_STEP(true, false, true);
                else if ((it & 1) == 0 && cull) PT_STEP(true, true, false);
                else if ((it & 1) == 0) PT_STEP(true, false, false);
                else if (cull) PT_STEP(false, true, false);
                else PT_STEP(false, false, false);
#undef PT_STEP
                return hipSuccess;
            } else if constexpr (TRAV >= 300)
                PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace_bf<LDS, ((TRAV / 10) & 1) != 0, COUNT>), dim3(tblocks),
                          dim3(kTraceBlock), lds, st, sc, w, in_q, cnt, bf_slots);
            else if (!COUNT && pk_ok && pk_launch(ws.packet, it))  // packet walk + replay (option packet)
                PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace_pk<LDS, ((TRAV / 10) & 1) != 0>), dim3(pk_blocks(pk_lds)),
                          dim3(kPkBlock), pk_lds, st, sc, w, in_q, ws.packet_nodes > 0 ? ws.packet_nodes : kPkMaxNodes);
            else
            {
                bool launched = false;
                if constexpr (has_big_ring(TRAV)) {
                    if (nring == kHitRingMax) {
                        PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace<LDS, TRAV, COUNT, kHitRingMax>), dim3(tblocks),
                                  dim3(kTraceBlockTr), lds, st, sc, w, in_q, cnt, watchdog, trace_dyn);
                        launched = true;
                    }
                }
                if (!launched)
                    PT_LAUNCH(KID_WF_TRACE, st, (k_wf_trace<LDS, TRAV, COUNT>), dim3(tblocks), dim3(kTraceBlockTr), lds, st,
                              sc, w, in_q, cnt, watchdog, trace_dyn);
            }
            if (stagger) HIP_RETURN_IF(hipEventRecord(ws.traced[h], st));
            if ((it & 1) == 0)
                PT_LAUNCH(KID_WF_SHADE_EXT, st, (k_wf_shade<true, COUNT>), dim3(sblocks), dim3(kShadeBlock), 0, st, sc, fp,
                          w, cnt, ws.sort_bins);
            else
                PT_LAUNCH(KID_WF_SHADE_SHADOW, st, (k_wf_shade<false, COUNT>), dim3(sblocks), dim3(kShadeBlock), 0, st, sc,
                          fp, w, cnt, ws.sort_bins);
            return hipSuccess;
        };
        if (pipe) {  // part 0's launches, then part 1's (its first batch starts at part 0's midpoint)
            for (int h = 0; h < nh; ++h)
                for (int it = 0; it < iters; ++it) {
                    if (b == 0 && h == 1 && it == 0) HIP_RETURN_IF(hipStreamWaitEvent(pv[1].st, ws.mid, 0));
                    HIP_RETURN_IF(step(h, it));
                    if (b == 0 && h == 0 && it == iters / 2 - 1) HIP_RETURN_IF(hipEventRecord(ws.mid, pv[0].st));
                    if (it == 0) HIP_RETURN_IF(hipGetLastError());
                }
        } else {
            for (int it = 0; it < iters; ++it) {
                for (int h = 0; h < nh; ++h) HIP_RETURN_IF(step(h, it));
                // a launch that cannot run (e.g. a configuration error) fails here, after the first
                // iteration, instead of leaving the later launches to read counts it never wrote
                if (it == 0) HIP_RETURN_IF(hipGetLastError());
            }
        }
        if (np > 1) {
            for (int h = 0; h < nh; ++h) {
                HIP_RETURN_IF(hipEventRecord(ws.join[h], pv[h].st));
                HIP_RETURN_IF(hipStreamWaitEvent(stream, ws.join[h], 0));
            }
        }
        PT_LAUNCH(KID_WF_ACCUM, stream, k_wf_accum, dim3((npix + 255) / 256), dim3(256), 0, stream, wbb.rad, out, npix, Fb,
                  accum);
        if (pipe) HIP_RETURN_IF(hipEventRecord(ws.acc_done[b & 1], stream));
    }
    return hipGetLastError();
}

hipError_t launch_wavefront(const LaunchOpts& lo, const SceneView& scene, const FrameParams& fp, const WfBuffers& wb,
                            uint32_t frame0, uint32_t nframes, uint32_t stride, bool accum, bool count, float* out,
                            Counters* cnt, hipStream_t stream, const WfStreams& ws_in) {
    WfStreams ws = lo.dual != 0 ? ws_in : WfStreams{};  // parts on streams by default: +15 % measured (in-process A/B)
    ws.h_poll = ws_in.h_poll;  // the regeneration loop's polling words, with one stream too
    for (int h = 0; h < kMaxParts; ++h) for (int k = 0; k < 2; ++k) ws.poll_ev[h][k] = ws_in.poll_ev[h][k];
    ws.nparts = std::max(1, std::min(kMaxParts, lo.parts > 0 ? lo.parts : 2));
    ws.stagger = lo.stagger > 0;
    ws.pipeline = lo.pipeline > 0;
    ws.fuse_gen = lo.fuse_gen != 0;
    ws.regen = lo.regen > 0 && ws.h_poll != nullptr;  // option regen=1 (measured slower so far)
    ws.regen_target = lo.regen_target > 0 ? (uint32_t)std::min<long>(lo.regen_target, 0x7fffffffL) : 0u;
    // survivors grouped per shade block by direction octant and origin cell (PT_SORT; default 512
    // keys = 8 octants x 4^3 cells: CornellBox-Glossy +4.7 % with 64 keys, +1.2 % more with 512,
    // MedievalBoat unchanged, in-process A/B)
    const int sort = lo.sort >= 0 ? lo.sort : 512;
    ws.sort_bins = sort > 0 ? (sort >= 512 ? 512 : sort >= 64 ? 64 : 8) : 0;
    ws.trace_blocks = lo.trace_blocks;
    ws.trace_dyn = lo.trace_dyn;
    ws.trace_sparse = std::max(0, lo.trace_sparse);
    ws.region_perm = lo.region_perm > 0 ? 1 : 0;
    ws.trace_ring = lo.trace_ring;
    ws.bf_slots = lo.bf_slots;
    ws.watchdog = lo.watchdog;
    ws.packet = lo.packet > 0 ? lo.packet : 0;
    ws.packet_nodes = lo.packet_nodes;
    if (!accum) { nframes = 1; stride = 1; }
    SceneView sc = scene;
    // turn policy of the lean16 traversal: 4 since the queues are grouped by coherence keys (in
    // process: Glossy +2.5 %, boat +1 %, 1M synthetic +1.8 % over 8; 1 = majority: -13 % in round 1)
    if (sc.node_bias <= 0) sc.node_bias = 4;
    sc.cull_its = lo.cull >= 0 ? lo.cull : 0;  // launches 0 (camera rays) and 1 (their shadow rays)
    const bool lds = lo.lds && scene_fits_lds(sc);
    // lean16 with the fast reciprocal by default (measured best on gfx950, scripts/perf_variants.py);
    // the wavefront always uses a flattened traversal; lean flavours take the fast reciprocal
    // (+10) when it is exact for the scene
    const int base = lo.trav < 0 ? 7 : (lo.trav == 0 ? 1 : lo.trav);
    const bool fast = lo.fast_rcp != 0 && sc.fast_rcp;
    const bool pipe = lo.pipe > 0, ifif = lo.ifif > 0;
    // mailboxed lean<K> (+100) for scenes with <= 64 distinct leaf entries, unless pipelined
    // or if-if steps were asked for (those have no mailboxed form)
    const bool mb = lo.mailbox != 0 && sc.mailbox && base >= 5 && base <= 8 && !pipe && !ifif;
    // brute force + replay (k_wf_trace_bf) by default for mailbox scenes; an explicit PT_TRAV
    // or bf=0 keeps the traversal kernels
    const bool bf = lo.bf != 0 && lo.mailbox != 0 && sc.mailbox && lo.trav < 0;
    // k_wf_persist_bf (option persist=1) measured slower: 1771 vs 2207 Msamples/s (its workgroups idle
    // at the per-iteration barrier once a region's queue is down to a few batches)
    // big-leaf cooperation (+160) for lean<4..16> on scenes with leaves of >= big_leaf entries
    const bool big = !bf && !mb && sc.big_leaf > 0 && base >= 5 && base <= 7 && !pipe && !ifif;
    const int trav = bf ? (lo.fuse == 0 ? 300 : lo.persist > 0 ? 500 : 400) + (fast ? 10 : 0)
                   : mb ? 100 + base + (fast ? 10 : 0)
                        : base + ((base >= 3 && fast) ? 10 : 0) + ((base >= 3 && fast && pipe) ? 20 : 0) +
                              ((base >= 3 && fast && ifif && !pipe) ? 40 : 0) + (big ? 160 : 0);
#define WF(L, T)                                                                                               \
    if (trav == T) {                                                                                           \
        if (count) return wf_render_t<L, T, true>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream, ws); \
        return wf_render_t<L, T, false>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream, ws);         \
    }
    if (lds) {
        WF(true, 1) WF(true, 2) WF(true, 3) WF(true, 4) WF(true, 5) WF(true, 6) WF(true, 7) WF(true, 8)
        WF(true, 13) WF(true, 14) WF(true, 15) WF(true, 16) WF(true, 17) WF(true, 18) WF(true, 35) WF(true, 36) WF(true, 37) WF(true, 55) WF(true, 56) WF(true, 57)
        WF(true, 300) WF(true, 310) WF(true, 400) WF(true, 410) WF(true, 500) WF(true, 510)
        WF(true, 105) WF(true, 106) WF(true, 107) WF(true, 115) WF(true, 116) WF(true, 117) WF(true, 118)
        WF(true, 165) WF(true, 166) WF(true, 167) WF(true, 175) WF(true, 176) WF(true, 177)
    } else {
        WF(false, 1) WF(false, 2) WF(false, 3) WF(false, 4) WF(false, 5) WF(false, 6) WF(false, 7) WF(false, 8)
        WF(false, 13) WF(false, 14) WF(false, 15) WF(false, 16) WF(false, 17) WF(false, 18) WF(false, 35) WF(false, 36) WF(false, 37) WF(false, 55) WF(false, 56) WF(false, 57)
        WF(false, 300) WF(false, 310) WF(false, 400) WF(false, 410) WF(false, 500) WF(false, 510)
        WF(false, 105) WF(false, 106) WF(false, 107) WF(false, 115) WF(false, 116) WF(false, 117) WF(false, 118)
        WF(false, 165) WF(false, 166) WF(false, 167) WF(false, 175) WF(false, 176) WF(false, 177)
    }
#undef WF
    return hipErrorInvalidValue;
}

}  // namespace pt

#if PT_PHASE_TIMING
// diagnostic build only: the phase cycle sums per wave slot (kPhaseWaves x kPhaseSlots u64),
// zeroed after the read
extern "C" __attribute__((visibility("default"))) int pt_debug_phase_read(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pt::g_phase), sizeof(unsigned long long) * pt::kPhaseWaves * pt::kPhaseSlots) != hipSuccess) return -1;
    static unsigned long long zero[pt::kPhaseWaves * pt::kPhaseSlots];
    if (hipMemcpyToSymbol(HIP_SYMBOL(pt::g_phase), zero, sizeof(zero)) != hipSuccess) return -1;
    return pt::kPhaseWaves * pt::kPhaseSlots;
}
#endif
