// pt_kernels.h — launch wrappers between the C-ABI layer (pt_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "pt_device.h"

// ids for k_selftest_math (also used by pt_selftest_math in the C-ABI)
enum {
    PT_MATH_SIN = 0, PT_MATH_COS, PT_MATH_TAN, PT_MATH_ACOS, PT_MATH_LOG2, PT_MATH_EXP2, PT_MATH_POW, PT_MATH_SQRT,
    PT_MATH_DIV, PT_MATH_HASH1U, PT_MATH_HASH1, PT_MATH_HASH2X, PT_MATH_HASH2Y, PT_MATH_MIN, PT_MATH_MAX, PT_MATH_COUNT_
};

namespace pt {

// Kernel timing (pt_profile_enable / pt_profile_read): while a profiler is attached to the
// calling thread, every launch is bracketed by two HIP events on its stream.
enum KernelId : int {
    KID_MEGA = 0, KID_REGEN, KID_WF_GENERATE, KID_WF_TRACE, KID_WF_SHADE_EXT, KID_WF_SHADE_SHADOW, KID_WF_ACCUM,
    KID_TONEMAP, KID_WF_STEP, KID_WF_LEAF, KID_COUNT
};
inline const char* kernel_name(int k) {
    static const char* const n[KID_COUNT] = {"k_mega",         "k_regen",           "k_wf_generate", "k_wf_trace",
                                             "k_wf_shade_ext", "k_wf_shade_shadow", "k_wf_accum",    "k_tonemap",
                                             "k_wf_step",      "k_wf_leafpass"};
    return (k >= 0 && k < KID_COUNT) ? n[k] : "?";
}
struct KernelProfiler {
    struct Rec { int kid; hipEvent_t a, b; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    int only = -1;  // record only this kernel id (pt_profile_select); -1 = all
    bool open = false;  // the last start() recorded (stop() closes it)
    hipEvent_t take();
    void start(int kid, hipStream_t s);
    void stop(hipStream_t s);
    void reset();    // records' events go back to the pool
    void destroy();  // frees every event
};
extern thread_local KernelProfiler* t_prof;
#define PT_LAUNCH(KID, STREAM, ...)                                  \
    do {                                                             \
        ::pt::KernelProfiler* p_ = ::pt::t_prof;                     \
        if (p_ && p_->only >= 0 && p_->only != (KID)) p_ = nullptr;  \
        if (p_) p_->start((KID), (STREAM));                          \
        hipLaunchKernelGGL(__VA_ARGS__);                             \
        if (p_) p_->stop(STREAM);                                    \
    } while (0)

constexpr int kMegaBlock = 256;
// dynamic LDS a workgroup may use for traversal stacks + a staged scene copy
constexpr size_t kLdsSceneBudget = 64 * 1024;

// Kernel selection (pt_set_option overrides for tests and A/B runs; pt_capi.hip launch_opts).
struct LaunchOpts {
    bool wavefront = false;  // wavefront pipeline (pt_wavefront.hip)
    bool literal = false;  // k_mega: the reference's control flow
    bool lds = true;       // stage the scene in LDS when it fits
    int fast_rcp = -1;     // rcp_rn for 1/det where SceneView::fast_rcp says it is exact: -1 per-pipeline default
    int dual = -1;         // wavefront batch split in parts on their own streams: -1 default (on)
    int fuse_gen = 1;      // fused kernel: the first launch makes the camera paths (0: k_wf_generate)
    int parts = -1;        // parts of a wavefront batch on their own streams (1..kMaxParts): -1 default (2)
    int mailbox = -1;      // mailboxed lean traversal where SceneView::mailbox allows it: -1 default (on)
    int bf = -1;           // wavefront, mailbox scenes: brute-force + replay trace kernel: -1 default (on)
    int fuse = -1;         // bf trace fused with the shading (k_wf_step_bf): -1 default (on)
    int trav = -1;         // traversal: -1 per-pipeline default, 0 nested, 1 flat, 2 predicated, 3 lean, 4..8 lean2..lean32
    int sort = -1;         // traversal pipeline: survivors grouped per shade block by 8 / 64 / 512 coherence keys (0 off): -1 default (512)
    int bf_slots = -1;     // brute-force kernels: hit slots per lane (< kBfSlots: tests of the recompute path): -1 default
    int trace_blocks = 0;  // traversal / step kernels: cap on the grid (tests): 0 = occupancy-derived
    int trace_sparse = -1; // k_wf_trace: narrower windows when 32-entry ones keep < 1/n of the waves busy (n; 0 off): -1 default
    int region_perm = -1;  // k_wf_step_bf: camera batches dealt to regions by a permutation (WfBuffers::rq); -1 default
    int trace_ring = 0;    // k_wf_trace's hit ring: 0 auto, 128 or 256
    uint32_t watchdog = 0; // k_wf_trace iterations before a wave gives up (tests of the failure report): 0 default
    int leaf_blocks = 0;   // k_wf_leafpass grid (A/B): 0 = occupancy-derived
    int leaf_pairs = 5;    // k_wf_leafpass walks chunked leaves by (ray, chunk) pairs (option leaf_pairs; | 4: leaf_refine)
    int regen = 0;         // fused kernel: camera batches per region admitted by every extension launch (0: all at once)
};

bool scene_fits_lds(const SceneView& sc);

// Wavefront path state (HBM), `capacity` entries per queue; see pt_wavefront.hip.  Every
// path's state travels with its ray: queue entry i holds the ray AND the path state, and
// a shade kernel writes the surviving path to its compacted slot of the other queue, so no
// kernel gathers by path index.  Iterations alternate extension / shadow queues.
enum { WF_COUNT0 = 0, WF_COUNT1 = 1, WF_WATCHDOG = 2, WF_SNAP_CLAIM = 3, WF_RING = 4, WF_SNAP = 8, WF_SNAP_WORDS = 16, WF_CTL_WORDS = 64 };
// the control block holds WF_CTL_WORDS words per half of a dual-stream batch (wb_half)
// iterations after which a trace wave gives up: it sets ctl[WF_WATCHDOG], the first such wave
// leaves its scheduling state in ctl[WF_SNAP..], and the host reports an error
constexpr uint32_t kTraceWatchdog = 1u << 24;
constexpr uint64_t kTraceWatchdogTicks = 500000000ull;  // 5 s of wall_clock64 (100 MHz)
struct WfQueue {
    float4* ray;  // [i][2]: (o.xyz, d.x), (d.y, d.z, path index bits, depth | spec << 16)
    float4* q2;   // (L.xyz, seed bits)
    float4* q3;   // (beta.xyz, -)
};
struct WfBuffers {
    WfQueue ext;   // extension rays (queue 0)
    WfQueue shd;   // shadow rays (queue 1) ...
    float4* sp0;   // ... and their shading points: (hp.xyz, material id)
    float4* sp1;   // (hn.xyz, wi.x)
    float2* sp2;   // (wi.y, wi.z)
    int2* hitq;    // per queue entry: (leaf record, t bits)
    float* rad;    // per path: radiance when it ended [capacity][3]
    uint32_t* ctl; // queue counts
    uint32_t capacity;  // paths per batch
    uint32_t qcap;      // entries per queue array (capacity + slack for the region layout)
    // region-partitioned queues of the fused kernel (k_wf_step_bf): region r of a queue holds
    // entries [r * rstride, r * rstride + count_r); rcnt[slot * kRegions + r] = count_r for
    // the three rotating count slots
    uint32_t* rcnt;
    uint32_t rstride;
    uint32_t nreg;
    // camera batch j of the fused kernel's regions goes to region (j mod nreg) * rqi mod nreg, so
    // region r holds the batches j = r * rq mod nreg (+ k nreg) (rq * rqi = 1 mod nreg; option
    // region_perm; 1, 1: j mod nreg, neighbouring regions — one block's waves — take neighbouring
    // batches)
    uint32_t rq, rqi;
    uint64_t rad_cap;   // paths whose radiance `rad` holds (>= capacity)
    // big leaves resolved before the traversal (k_wf_leafpass): per leaf b and queue entry i the
    // key (f32 bits of t << 32 | position; ~0: no hit) at pres[b * pres_stride + i] (pres_stride = the
    // whole buffer's qcap: a part's pres is offset like its queues); nullptr when the scene has none
    uint64_t* pres;
    uint32_t pres_stride;
    // per distinct entry, the camera-origin parts of the triangle test (k_wf_camtab; 2 x 64 float4)
    float4* camtab;
};
constexpr uint32_t kRegions = 512;
// queue slack (entries per part = 64 * this): regions of R <= kRegions hold ceil(batches / R)
// 64-entry batches each
constexpr uint32_t kQueueSlackRegions = 4096;
constexpr size_t kWfBytesPerPath = 64 + 64 + 40 + 8 + 12;

// Dual-stream wavefront: two streams owned by the scene, created back to back so that HIP's
// round-robin stream -> hardware-queue mapping puts them on different queues (a shared queue
// serialises the halves), plus fork/join events with the caller's stream.  Null = one stream.
constexpr int kMaxParts = 4;  // parts of a wavefront batch on their own streams (LaunchOpts::parts)
struct WfStreams {
    hipStream_t aux[kMaxParts] = {};
    hipEvent_t fork = nullptr, join[kMaxParts] = {};
    bool fuse_gen = true;  // LaunchOpts::fuse_gen
    int nparts = 2;
    int sort_bins = 0;     // LaunchOpts::sort: k_wf_shade groups a block's survivors by a coherence key of 8 / 64 / 512 values (0: off)
    // per-call launch shape (LaunchOpts, filled by launch_wavefront)
    int trace_blocks = 0;  // cap on the trace / step grid (0: occupancy-derived)
    int trace_sparse = 0;  // k_wf_trace windows below 32 entries for short queues (LaunchOpts::trace_sparse)
    int region_perm = 0;   // LaunchOpts::region_perm
    int trace_ring = 0;    // LaunchOpts::trace_ring
    int bf_slots = -1;     // hit slots per lane of the brute-force kernels (-1: kBfSlots)
    uint32_t watchdog = 0; // k_wf_trace iteration limit (0: kTraceWatchdog)
    int leaf_blocks = 0;   // LaunchOpts::leaf_blocks
    int leaf_pairs = 5;    // LaunchOpts::leaf_pairs
    int regen = 0;         // LaunchOpts::regen
};
hipError_t launch_wavefront(const LaunchOpts& lo, const SceneView& sc, const FrameParams& fp, const WfBuffers& wb,
                            uint32_t frame0, uint32_t nframes, uint32_t stride, bool accum, bool count, float* out,
                            Counters* cnt, hipStream_t stream, const WfStreams& ws);

// Megakernel render (accum=true: frames frame0 + i*stride, i < nframes, added to out) or one
// dispatch (accum=false: raw radiance of salt frame0 written to out).
hipError_t launch_megakernel(const LaunchOpts& lo, const SceneView& sc, const FrameParams& fp, uint32_t frame0,
                             uint32_t nframes, uint32_t stride, bool accum, bool count, float* out, Counters* cnt,
                             hipStream_t stream);

// display transform of program-raymarch.ts:295-316 on device (pt_image.hip)
hipError_t launch_tonemap(const float* acc, size_t npix, uint32_t runs, uint8_t* rgba, hipStream_t stream);
// n floats from device memory to pinned host memory (h_dst_dev: its device address; pt_image.hip)
hipError_t launch_readback(const float* d_src, float* h_dst_dev, size_t n, hipStream_t stream);
// dst[i] += src[i] for i < n (f32; both on the stream's device; pt_image.hip)
hipError_t launch_accum_add(float* dst, const float* src, size_t n, hipStream_t stream);

// k_wf_leafpass (pt_leafpass.hip): every big leaf of sc.pre resolved for the entries of queue in_q
// whose rays enter its path's boxes, into wb.pres; blocks: the persistent grid (0: occupancy)
hipError_t launch_leafpass(const SceneView& sc, const WfBuffers& wb, int in_q, bool fast_rcp, int blocks, int pairs,
                           hipStream_t stream);

hipError_t launch_selftest_rcp(int steps, uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t stream);
hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream);
hipError_t launch_selftest_valu(int iters, int blocks, int packed, float* out, hipStream_t stream);
// the leaf pass's resolve_leaf / resolve_leaf_pairs against the sequential loop (pt_leafpass.hip)
hipError_t launch_selftest_leafpass(const SceneView& sc, int b, int mode, uint32_t seed, uint32_t nrays, int32_t* out,
                                    hipStream_t stream);
hipError_t launch_selftest_leaf(const SceneView& sc, int rec0, int n, int mode, uint32_t seed, uint32_t nrays, int32_t* out,
                                hipStream_t stream);

}  // namespace pt
