// pt_wavefront.hip — wavefront path tracer for gfx950 (the north-star design).
//
// A batch of P = F*W*H paths (F frames of the image) lives in HBM as SoA float4 arrays.
// Each iteration runs two kernels over the queue of live paths:
//   k_wf_trace   persistent waves with dynamic ray fetch: a wave pulls 16..64 path indices
//                at a time from the queue with ONE atomic (wave-aggregated), walks every
//                lane's ray through the BVH with the flattened, ballot-scheduled traversal
//                (trav_step, per-lane stack in LDS, scene in LDS when it fits) and refills
//                lanes as their rays finish, so no lane idles behind a long traversal;
//   k_wf_shade   the path logic after that traversal (path_after_ext / path_after_shadow,
//                pt_path.h) and compaction of the survivors into the next queue with
//                __ballot + mbcnt (one atomicAdd per wave).
// All paths of a batch start together, so every queue holds only extension rays or only
// shadow rays and the two alternate.  k_wf_generate creates the camera paths; k_wf_accum
// adds the finished radiance of the batch into the accumulator in frame order, which keeps
// the result bit-identical to the reference's host accumulation.
#include "pt_kernels.h"
#include "pt_path.h"

#include <algorithm>

namespace pt {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// number of set bits of m below this lane
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void store_ray(const WfBuffers& wb, uint32_t p, const Ray& r) {
    wb.ray0[p] = make_float4(r.o.x, r.o.y, r.o.z, r.d.x);
    wb.ray1[p] = make_float4(r.d.y, r.d.z, 0.0f, 0.0f);
}
__device__ __forceinline__ Ray load_ray(const WfBuffers& wb, uint32_t p) {
    float4 a = wb.ray0[p], b = wb.ray1[p];
    Ray r;
    r.o = mk(a.x, a.y, a.z);
    r.d = mk(a.w, b.x, b.y);
    r.inv = rcp3(r.d);
    return r;
}
__device__ __forceinline__ void store_state(const WfBuffers& wb, uint32_t p, const PathState& ps) {
    wb.st0[p] = make_float4(ps.L.x, ps.L.y, ps.L.z, ps.beta.x);
    wb.st1[p] = make_float4(ps.beta.y, ps.beta.z, __builtin_bit_cast(float, ps.seed),
                            __builtin_bit_cast(float, (uint32_t)ps.depth | (ps.spec ? 0x10000u : 0u)));
}
__device__ __forceinline__ void load_state(const WfBuffers& wb, uint32_t p, PathState& ps) {
    float4 a = wb.st0[p], b = wb.st1[p];
    ps.L = mk(a.x, a.y, a.z);
    ps.beta = mk(a.w, b.x, b.y);
    ps.seed = __builtin_bit_cast(uint32_t, b.z);
    const uint32_t dw = __builtin_bit_cast(uint32_t, b.w);
    ps.depth = (int)(dw & 0xffffu);
    ps.spec = (dw & 0x10000u) != 0;
}
__device__ __forceinline__ void store_shading_point(const WfBuffers& wb, uint32_t p, const PathState& ps) {
    wb.sp0[p] = make_float4(ps.hp.x, ps.hp.y, ps.hp.z, __builtin_bit_cast(float, ps.mat_id));
    wb.sp1[p] = make_float4(ps.hn.x, ps.hn.y, ps.hn.z, 0.0f);
    wb.sp2[p] = make_float4(ps.wi.x, ps.wi.y, ps.wi.z, 0.0f);
}
__device__ __forceinline__ void load_shading_point(const WfBuffers& wb, uint32_t p, PathState& ps) {
    float4 a = wb.sp0[p], b = wb.sp1[p], c = wb.sp2[p];
    ps.hp = mk(a.x, a.y, a.z);
    ps.mat_id = __builtin_bit_cast(int, a.w);
    ps.hn = mk(b.x, b.y, b.z);
    ps.wi = mk(c.x, c.y, c.z);
}

// pixel of path p (row-major within its frame)
__device__ __forceinline__ void path_pixel(uint32_t p, uint32_t npix, uint32_t W, uint32_t& x, uint32_t& y, uint32_t& f) {
    f = p / npix;
    const uint32_t pix = p - f * npix;
    y = pix / W;
    x = pix - y * W;
}

template <bool COUNT>
__global__ __launch_bounds__(256) void k_wf_generate(FrameParams fp, WfBuffers wb, uint32_t frame0, uint32_t stride,
                                                     uint32_t fbase, uint32_t P, bool raw_salt, Counters* cnt_out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p == 0) {
        wb.ctl[WF_COUNT0] = P;
        wb.ctl[WF_COUNT1] = 0;
        wb.ctl[WF_HEAD] = 0;
    }
    Counters c = {};
    if (p < P) {
        uint32_t x, y, f;
        path_pixel(p, fp.width * fp.height, fp.width, x, y, f);
        const uint32_t t = raw_salt ? frame0 : (uint32_t)(float)(frame0 + (fbase + f) * stride);
        PathState ps;
        Ray r = path_begin(fp, x, y, t, ps);
        store_ray(wb, p, r);
        store_state(wb, p, ps);
        wb.q0[p] = p;
        if (COUNT) { c.samples++; c.ext_queries++; }
    }
    if (COUNT) flush_counters(c, cnt_out);
}

template <bool LDS, bool COUNT>
__global__ __launch_bounds__(256) void k_wf_trace(SceneView sc, WfBuffers wb, int in_q, Counters* cnt_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int32_t* stack = reinterpret_cast<int32_t*>(smem) + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1] = 0;  // shade's output count
    if (LDS) stage_scene_lds(sc, smem + (uint32_t)sc.max_stack * blockDim.x * 4u);
    const uint32_t* queue = in_q ? wb.q1 : wb.q0;
    const uint32_t count = __hip_atomic_load(&wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    Counters c = {};
    bool has = false, drained = count == 0;
    uint32_t p = 0;
    Ray r;
    r.o = r.d = r.inv = mk(0.0f, 0.0f, 0.0f);
    TravState s;
    trav_init(s, false);
    while (true) {
        const uint64_t empty = __ballot(!has);
        const uint32_t n_empty = (uint32_t)__popcll(empty);
        if (!drained && (n_empty >= 16 || n_empty == 64)) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(&wb.ctl[WF_HEAD], n_empty);
            base = __shfl(base, 0, 64);
            if (base + n_empty >= count) drained = true;
            if (!has) {
                const uint32_t idx = base + rank_below(empty);
                if (idx < count) {
                    p = queue[idx];
                    r = load_ray(wb, p);
                    trav_init(s, true);
                    has = true;
                }
            }
        }
        if (!trav_step<COUNT>(sc, r, s, stack, blockDim.x, c)) {
            if (drained) break;
            continue;
        }
        if (has && s.done) {
            wb.hit[p] = make_int2(s.best, __builtin_bit_cast(int, s.best_t));
            has = false;
        }
    }
    if (COUNT) flush_counters(c, cnt_out);
}

template <bool EXT, bool COUNT>
__global__ __launch_bounds__(256) void k_wf_shade(SceneView sc, FrameParams fp, WfBuffers wb, int in_q,
                                                  Counters* cnt_out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) wb.ctl[WF_HEAD] = 0;  // for the next trace
    const uint32_t* queue = in_q ? wb.q1 : wb.q0;
    uint32_t* out_q = in_q ? wb.q0 : wb.q1;
    uint32_t* out_count = &wb.ctl[in_q ? WF_COUNT0 : WF_COUNT1];
    const uint32_t count = wb.ctl[in_q ? WF_COUNT1 : WF_COUNT0];
    const uint32_t waves = gridDim.x * (blockDim.x / 64), wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    Counters c = {};
    for (uint32_t chunk = wave; chunk * 64 < count; chunk += waves) {
        const uint32_t i = chunk * 64 + lane_id();
        bool more = false;
        uint32_t p = 0;
        if (i < count) {
            p = queue[i];
            PathState ps;
            load_state(wb, p, ps);
            Ray r = load_ray(wb, p);
            const int2 h = wb.hit[p];
            const float t = __builtin_bit_cast(float, h.y);
            if (EXT) {
                more = path_after_ext(sc, h.x, t, r, ps);
                if (more) {
                    store_shading_point(wb, p, ps);
                    if (COUNT) c.shadow_queries++;
                }
            } else {
                load_shading_point(wb, p, ps);
                more = path_after_shadow(sc, fp, h.x, t, r, ps);
                if (more && COUNT) c.ext_queries++;
            }
            if (more) {
                store_ray(wb, p, r);
                store_state(wb, p, ps);
            } else {
                float* o = wb.rad + 3 * (size_t)p;
                o[0] = ps.L.x; o[1] = ps.L.y; o[2] = ps.L.z;
            }
        }
        // compaction of the survivors: one atomic per wave, lane offsets from mbcnt
        const uint64_t keep = __ballot(more);
        if (keep) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(out_count, (uint32_t)__popcll(keep));
            base = __shfl(base, 0, 64);
            if (more) out_q[base + rank_below(keep)] = p;
        }
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
template <bool LDS, bool COUNT>
static int trace_blocks(size_t lds_bytes) {
    static int cached[2][2] = {{0, 0}, {0, 0}};
    static size_t cached_lds[2][2] = {{0, 0}, {0, 0}};
    int& b = cached[LDS][COUNT];
    if (b == 0 || cached_lds[LDS][COUNT] != lds_bytes) {
        int per_cu = 0, dev = 0, cus = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_wf_trace<LDS, COUNT>, 256, lds_bytes);
        b = std::max(1, per_cu) * std::max(1, cus);
        cached_lds[LDS][COUNT] = lds_bytes;
    }
    return b;
}

template <bool LDS, bool COUNT>
static hipError_t wf_render_t(const SceneView& sc, const FrameParams& fp, const WfBuffers& wb, uint32_t frame0,
                              uint32_t nframes, uint32_t stride, bool accum, float* out, Counters* cnt,
                              hipStream_t stream) {
    const uint32_t npix = fp.width * fp.height;
    const uint32_t F = std::max<uint32_t>(1, std::min<uint32_t>(nframes, wb.capacity / npix));
    const size_t lds = (size_t)sc.max_stack * 256 * 4 + (LDS ? sc.span_bytes : 0);
    const int tblocks = trace_blocks<LDS, COUNT>(lds);
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int sblocks = cus * 8;
    const int iters = 2 * (fp.max_depth + 1);
    for (uint32_t fb = 0; fb < nframes; fb += F) {
        const uint32_t Fb = std::min(F, nframes - fb);
        const uint32_t P = Fb * npix;
        hipLaunchKernelGGL((k_wf_generate<COUNT>), dim3((P + 255) / 256), dim3(256), 0, stream, fp, wb, frame0, stride, fb,
                           P, !accum, cnt);
        int in_q = 0;
        for (int it = 0; it < iters; ++it) {
            hipLaunchKernelGGL((k_wf_trace<LDS, COUNT>), dim3(tblocks), dim3(256), lds, stream, sc, wb, in_q, cnt);
            if ((it & 1) == 0)
                hipLaunchKernelGGL((k_wf_shade<true, COUNT>), dim3(sblocks), dim3(256), 0, stream, sc, fp, wb, in_q, cnt);
            else
                hipLaunchKernelGGL((k_wf_shade<false, COUNT>), dim3(sblocks), dim3(256), 0, stream, sc, fp, wb, in_q, cnt);
            in_q ^= 1;
        }
        hipLaunchKernelGGL(k_wf_accum, dim3((npix + 255) / 256), dim3(256), 0, stream, wb.rad, out, npix, Fb, accum);
    }
    return hipGetLastError();
}

hipError_t launch_wavefront(const LaunchOpts& lo, const SceneView& sc, const FrameParams& fp, const WfBuffers& wb,
                            uint32_t frame0, uint32_t nframes, uint32_t stride, bool accum, bool count, float* out,
                            Counters* cnt, hipStream_t stream) {
    if (!accum) { nframes = 1; stride = 1; }
    const bool lds = lo.lds && scene_fits_lds(sc);
    if (lds) return count ? wf_render_t<true, true>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream)
                          : wf_render_t<true, false>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream);
    return count ? wf_render_t<false, true>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream)
                 : wf_render_t<false, false>(sc, fp, wb, frame0, nframes, stride, accum, out, cnt, stream);
}

}  // namespace pt
