// pt_kernels.hip — HIP kernels for gfx950 (MI355X) replacing program-raymarch.wgsl.
//
//   k_regen<LDS, ACCUM, COUNT>  the production megakernel.  One lane owns one pixel
//       (8x8 pixels per wave, 16x16 per 256-thread workgroup) and runs its frames as a
//       state machine with ONE traversal call site per iteration: a lane is either
//       tracing its extension ray or its shadow ray, and a lane whose path ended starts
//       its next frame's camera path right away (path regeneration), so waves stay full
//       until the last frames instead of idling behind the longest path.  Frames of a
//       pixel still run in order, so clamp(L) is accumulated in f32 registers exactly as
//       the host loop of program-raymarch.ts:281-285 adds them.  LDS=true stages the
//       whole scene (nodes, leaf triangles, materials, light table) in LDS.
//   k_mega<ACCUM, COUNT>   the same integrator written with the reference's control flow
//       (radiance() as one loop per sample); kept as the structural twin for A/B tests.
//   k_selftest_math        exposes pt_math.h on device for the numerics tests.
#include "pt_kernels.h"
#include "pt_path.h"

namespace pt {

template <bool COUNT>
__device__ f3 radiance(const SceneView& sc, const FrameParams& fp, Ray ray, uint32_t seed_in, const LStack32& stack,
                       Counters& cnt) {
    // program-raymarch.wgsl:104-303, literal control flow
    f3 L = mk(0.0f, 0.0f, 0.0f), beta = mk(1.0f, 1.0f, 1.0f);
    int depth = 0;
    bool spec = false;
    uint32_t seed = hash1u(seed_in);
    seed = hash1u(seed);
    while (depth <= fp.max_depth) {
        seed = hash1u(seed);
        if (COUNT) cnt.ext_queries++;
        float t;
        int rec = trace<COUNT>(sc, ray, t, stack, cnt);
        if (rec < 0) break;
        Hit h = hit_data(sc, ray, rec, t);
        Mat m = load_mat(sc, h.mat);
        if (sum3(m.Ke) > 0.0f && (depth == 0 || spec)) {
            L = L + beta * m.Ke;
            break;
        }
        f3 off = madd(h.p, h.n, 1.0e-4f);
        f3 ldir = sample_area_lights(sc, off, seed);
        seed = hash1u(seed + 7u);
        Ray sray;
        sray.o = off; sray.d = ldir; sray.inv = rcp3(ldir);
        if (COUNT) cnt.shadow_queries++;
        float st;
        int srec = trace<COUNT>(sc, sray, st, stack, cnt);
        if (srec >= 0) {
            Hit sh = hit_data(sc, sray, srec, st);
            Mat nm = load_mat(sc, sh.mat);
            if (sum3(nm.Ke) > 0.0f) L = L + nee_contrib(m, ray.d, h.p, h.n, ldir, beta, sh, nm, sc.inv_ntri);
            if (fp.direct_only) break;
        }
        if (hash1(seed) > fp.rr_prob) break;
        bsdf_continue(m, h.p, h.n, ray, beta, spec, seed, depth, fp.rr_prob);
        depth += 1;
    }
    return L;
}

__device__ __forceinline__ void pixel_of(uint32_t& x, uint32_t& y) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
}

template <bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kMegaBlock) void k_mega(SceneView sc, FrameParams fp, uint32_t frame0, uint32_t nframes,
                                                    uint32_t stride, float* __restrict__ out, Counters* cnt_out) {
    __shared__ int32_t s_stack[kStackMax * kMegaBlock];
    const LStack32 stack = LStack32::make(reinterpret_cast<char*>(s_stack), kMegaBlock);
    uint32_t x, y;
    pixel_of(x, y);
    Counters c = {};
    if (x < fp.width && y < fp.height) {
        float* o = out + 3 * ((size_t)y * fp.width + x);
        f3 acc = ACCUM ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);
        for (uint32_t i = 0; i < nframes; ++i) {
            uint32_t t = ACCUM ? (uint32_t)(float)(frame0 + i * stride) : frame0;
            uint32_t seed;
            Ray r = camera_ray(fp, x, y, t, seed);
            if (COUNT) c.samples++;
            f3 L = radiance<COUNT>(sc, fp, r, seed, stack, c);
            acc = ACCUM ? add_clamped(acc, L) : L;
        }
        o[0] = acc.x; o[1] = acc.y; o[2] = acc.z;
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// ---------------------------------------------------------------------------------------
// Megakernel: path regeneration, one traversal site, optional LDS scene, flat traversal
// ---------------------------------------------------------------------------------------
template <bool LDS, int TRAV, bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kMegaBlock) void k_regen(SceneView sc, FrameParams fp, uint32_t frame0, uint32_t nframes,
                                                     uint32_t stride, float* __restrict__ out, Counters* cnt_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const LStack32 stack = LStack32::make(smem, kMegaBlock);  // [max_stack][256] int32, lane-minor
    if (LDS) stage_scene_lds(sc, smem + (uint32_t)sc.max_stack * kMegaBlock * 4u);
    uint32_t x, y;
    pixel_of(x, y);
    Counters c = {};
    const bool valid = x < fp.width && y < fp.height;
    float* o = out + 3 * ((size_t)(valid ? y : 0) * fp.width + (valid ? x : 0));
    f3 acc = (ACCUM && valid) ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);

    enum { kIdle = 0, kExt = 1, kShadow = 2 };
    int phase = kIdle;
    uint32_t next = 0;  // next frame of this pixel to start
    Ray ray;
    PathState ps;
    while (true) {
        if (phase == kIdle) {
            if (!valid || next >= nframes) break;
            const uint32_t t = ACCUM ? (uint32_t)(float)(frame0 + next * stride) : frame0;
            ++next;
            ray = path_begin(fp, x, y, t, ps);
            phase = kExt;
            if (COUNT) { c.samples++; c.ext_queries++; }
        }
        float t;
        const int rec = trace_any<TRAV, COUNT>(sc, ray, t, stack, c);
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
    if (valid) { o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; }
    if (COUNT) flush_counters(c, cnt_out);
}

// Exhaustive check of rcp_rn against the IEEE division over every float x whose magnitude
// bits lie in [lo, hi] (both signs): bad[0] += mismatches, bad[1] = some failing bit pattern.
__global__ void k_selftest_rcp(int steps, uint32_t lo, uint32_t hi, unsigned long long* bad) {
    const uint64_t n = (uint64_t)(hi - lo + 1) * 2;
    unsigned long long mis = 0, first = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (lo + (uint32_t)(k >> 1)) | ((uint32_t)(k & 1) << 31);
        const float x = __builtin_bit_cast(float, u);
        const float want = 1.0f / x;
        const float got = steps == 1 ? rcp_rn(x, 1) : (steps == 2 ? rcp_rn(x, 2) : rcp_rn(x, 0));
        if (__builtin_bit_cast(uint32_t, got) != __builtin_bit_cast(uint32_t, want)) { ++mis; first = u; }
    }
    if (mis) {
        atomicAdd(&bad[0], mis);
        atomicExch(&bad[1], first);
    }
}

hipError_t launch_selftest_rcp(int steps, uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t stream) {
    hipLaunchKernelGGL(k_selftest_rcp, dim3(8192), dim3(256), 0, stream, steps, lo, hi, bad);
    return hipGetLastError();
}

// VALU issue calibration (pt_selftest_valu): every thread runs 8 independent v_fma_f32 chains,
// 32 FMAs per loop iteration and no memory operation in the loop, at 8 waves per SIMD (the host
// sizes the grid from the CU count), so the chains' latency is hidden and the SIMDs issue VALU at
// their peak rate — the known rate against which scripts/summarize_traffic.py's PMC formula for
// `valu_issue` is calibrated (scripts/calibrate_valu.sh).  The sum is stored only if it equals an
// impossible value, so the chains stay live and nothing is written.
__global__ __launch_bounds__(256) void k_selftest_valu(int iters, float seed, float m, float c, float* out) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = seed + (float)(threadIdx.x + k);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = fmaf(a[k], m, c);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    if (s == -1.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the same with packed f32: 8 independent v_pk_fma_f32 chains (two FMAs per lane each)
typedef float fv2s __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_selftest_valu_pk(int iters, float seed, float m, float c, float* out) {
    fv2s a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fv2s{seed + (float)(threadIdx.x + k), seed - (float)(threadIdx.x + k)};
    const fv2s mm = {m, m}, cc = {c, c};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = __builtin_elementwise_fma(a[k], mm, cc);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
    if (s == -1.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// mixed: 4 packed chains and 8 plain chains interleaved (the issue rate of a mix of the two kinds;
// per loop iteration 16 v_pk_fma_f32 + 32 v_fma_f32 = 48 wave-instructions)
__global__ __launch_bounds__(256) void k_selftest_valu_mix(int iters, float seed, float m, float c, float* out) {
    fv2s a[4];
    float b[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = fv2s{seed + (float)(threadIdx.x + k), seed - (float)(threadIdx.x + k)};
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = seed * (float)(threadIdx.x + k);
    const fv2s mm = {m, m}, cc = {c, c};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[k] = __builtin_elementwise_fma(a[k], mm, cc);
                b[2 * k] = fmaf(b[2 * k], m, c);
                b[2 * k + 1] = fmaf(b[2 * k + 1], m, c);
            }
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += a[k].x + a[k].y;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += b[k];
    if (s == -1.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// dependent chains: 2 packed (mode 3) or 2 plain (mode 4) chains per thread, 32 instructions per
// iteration — the issue rate when each wave's next instruction depends on its last but one
__global__ __launch_bounds__(256) void k_selftest_valu_dep(int iters, int pk, float seed, float m, float c, float* out) {
    float s = 0.0f;
    if (pk) {
        fv2s a0 = {seed + threadIdx.x, seed - threadIdx.x}, a1 = {seed * 2.0f, seed * 3.0f};
        const fv2s mm = {m, m}, cc = {c, c};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                a0 = __builtin_elementwise_fma(a0, mm, cc);
                a1 = __builtin_elementwise_fma(a1, mm, cc);
            }
        }
        s = a0.x + a0.y + a1.x + a1.y;
    } else {
        float a0 = seed + threadIdx.x, a1 = seed * 2.0f;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                a0 = fmaf(a0, m, c);
                a1 = fmaf(a1, m, c);
            }
        }
        s = a0 + a1;
    }
    if (s == -1.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

hipError_t launch_selftest_valu(int iters, int blocks, int packed, float* out, hipStream_t stream) {
    if (packed == 3 || packed == 4) {
        hipLaunchKernelGGL(k_selftest_valu_dep, dim3(blocks), dim3(256), 0, stream, iters, packed == 3 ? 1 : 0, 1.0f,
                           0.99999994f, 1.0e-7f, out);
        return hipGetLastError();
    }
    if (packed == 2) {  // 48 instructions per iteration: scale iters so the count below holds (x 32 per iteration)
        hipLaunchKernelGGL(k_selftest_valu_mix, dim3(blocks), dim3(256), 0, stream, iters * 2 / 3, 1.0f, 0.99999994f, 1.0e-7f, out);
        return hipGetLastError();
    }
    // m, c as arguments: the FMAs read them from SGPRs (no literal-constant encodings in the loop)
    if (packed)
        hipLaunchKernelGGL(k_selftest_valu_pk, dim3(blocks), dim3(256), 0, stream, iters, 1.0f, 0.99999994f, 1.0e-7f, out);
    else
        hipLaunchKernelGGL(k_selftest_valu, dim3(blocks), dim3(256), 0, stream, iters, 1.0f, 0.99999994f, 1.0e-7f, out);
    return hipGetLastError();
}

// Leaf chunk stress (pt_selftest_leaf): rays against the leaf whose records start at rec0, tested
// once by the reference's sequential loop over all n entries (each lane its own ray) and once by
// chunk_leaf (the wave on each lane's ray in turn, as round 3's single-ray turn ran it), both against the same
// closest t so far (prior; none for half the rays).  Ray families (mode): pt_device.h stress_ray.  Row i of out: the loop's
// result (position taken or -1, t bits), chunk_leaf's, its entry tests and open chunks.  mode + 4:
// chunk_leaf_multi instead (the walk several rays share; tests and chunks not counted).
__global__ __launch_bounds__(256) void k_selftest_leaf(SceneView sc, int rec0, int n, int mode_in, uint32_t seed,
                                                       uint32_t nrays, int32_t* __restrict__ out) {
    const int mode = mode_in & 3;
    const bool multi = (mode_in & 4) != 0;
    // every lane runs (chunk_leaf needs the whole wave); lanes past nrays store nothing
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t st = 0;
    const Ray r = stress_ray(sc, rec0, n, mode, seed, i, st);
    auto u01 = [&]() { st = st_hash(st + 0x6a09e667u); return (float)(st >> 8) * (1.0f / 16777216.0f); };
    const float prior = u01() < 0.5f ? -1.0f : exp2f(-10.0f + 15.0f * u01());
    const float pb = prior < 0.0f ? __builtin_inff() : prior;
    float lt = __builtin_inff();
    int lk = 0x7fffffff;
    for (int k = 0; k < n; ++k) {
        float t;
        if (tri_hit<false>(sc.tris, rec0 + k, r, t) && t < lt) { lt = t; lk = k; }
    }
    float wt = 0.0f;
    int wk = 0x7fffffff, tests = 0, chunks = 0;
    const int lane = (int)(threadIdx.x & 63u);
    if (multi) {  // chunk_leaf_multi: four walks of 16 interleaved lanes each (lanes g, g + 4, ...)
        __shared__ uint64_t keys[4][kMultiRays];
        for (int g = 0; g < 4; ++g) {
            float bt;
            int bk;
            chunk_leaf_multi<false>(sc, r, 0x1111111111111111ull << g, rec0, pb, keys[threadIdx.x / 64u], bt, bk);
            if ((lane & 3) == g) { wt = bt; wk = bk; }
        }
    }
    for (int f = 0; f < (multi ? 0 : 64); ++f) {
        auto bc = [&](float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), f)); };
        Ray q;
        q.o = mk(bc(r.o.x), bc(r.o.y), bc(r.o.z));
        q.d = mk(bc(r.d.x), bc(r.d.y), bc(r.d.z));
        q.inv = mk(bc(r.inv.x), bc(r.inv.y), bc(r.inv.z));
        float bt;
        int bk, t_lane = 0, c_wave = 0;
        chunk_leaf<false, true>(sc, q, rec0, bc(pb), bt, bk, &t_lane, &c_wave);
        for (int off = 1; off < 64; off <<= 1) t_lane += __shfl_xor(t_lane, off, 64);
        if (lane == f) { wt = bt; wk = bk; tests = t_lane; chunks = c_wave; }
    }
    if (i >= nrays) return;
    const bool ltake = lk != 0x7fffffff && lt < pb, wtake = wk != 0x7fffffff && wt < pb;
    int32_t* o = out + 6 * (size_t)i;
    o[0] = ltake ? lk : -1;
    o[1] = ltake ? __builtin_bit_cast(int32_t, lt) : 0;
    o[2] = wtake ? wk : -1;
    o[3] = wtake ? __builtin_bit_cast(int32_t, wt) : 0;
    o[4] = tests;
    o[5] = chunks;
}

hipError_t launch_selftest_leaf(const SceneView& sc, int rec0, int n, int mode, uint32_t seed, uint32_t nrays, int32_t* out,
                                hipStream_t stream) {
    hipLaunchKernelGGL(k_selftest_leaf, dim3((nrays + 255) / 256), dim3(256), 0, stream, sc, rec0, n, mode, seed, nrays, out);
    return hipGetLastError();
}

__global__ void k_selftest_math(int fn, const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ o,
                                int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i], r = 0.0f, s, c;
    uint32_t u = __builtin_bit_cast(uint32_t, x);
    switch (fn) {
        case PT_MATH_SIN: sincos_p(x, s, c); r = s; break;
        case PT_MATH_COS: sincos_p(x, s, c); r = c; break;
        case PT_MATH_TAN: r = tan_p(x); break;
        case PT_MATH_ACOS: r = acos_p(x); break;
        case PT_MATH_LOG2: r = log2_p(x); break;
        case PT_MATH_EXP2: r = exp2_p(x); break;
        case PT_MATH_POW: r = pow_p(x, y); break;
        case PT_MATH_SQRT: r = sqrtf(x); break;
        case PT_MATH_DIV: r = x / y; break;
        case PT_MATH_HASH1U: r = __builtin_bit_cast(float, hash1u(u)); break;
        case PT_MATH_HASH1: r = hash1(u); break;
        case PT_MATH_HASH2X: hash2(u, r, s); break;
        case PT_MATH_HASH2Y: hash2(u, s, r); break;
        case PT_MATH_MIN: r = fminf(x, y); break;
        case PT_MATH_MAX: r = fmaxf(x, y); break;
        default: r = __builtin_nanf(""); break;
    }
    o[i] = r;
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
bool scene_fits_lds(const SceneView& sc) {
    return (size_t)sc.max_stack * kMegaBlock * 4 + sc.span_bytes <= kLdsSceneBudget;
}

template <bool LDS, int TRAV, bool ACCUM, bool COUNT>
static void launch_regen_t(const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes, uint32_t stride,
                           float* out, Counters* cnt, hipStream_t stream) {
    dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kMegaBlock);
    size_t lds = (size_t)sc.max_stack * kMegaBlock * 4 + (LDS ? sc.span_bytes : 0);
    PT_LAUNCH(KID_REGEN, stream, (k_regen<LDS, TRAV, ACCUM, COUNT>), grid, block, lds, stream, sc, fp, frame0, nframes, stride, out,
                       cnt);
}

template <bool LDS, int TRAV>
static void launch_regen_a(const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes, uint32_t stride,
                           bool accum, bool count, float* out, Counters* cnt, hipStream_t stream) {
    if (accum) {
        if (count) launch_regen_t<LDS, TRAV, true, true>(sc, fp, frame0, nframes, stride, out, cnt, stream);
        else launch_regen_t<LDS, TRAV, true, false>(sc, fp, frame0, nframes, stride, out, cnt, stream);
    } else {
        if (count) launch_regen_t<LDS, TRAV, false, true>(sc, fp, frame0, nframes, stride, out, cnt, stream);
        else launch_regen_t<LDS, TRAV, false, false>(sc, fp, frame0, nframes, stride, out, cnt, stream);
    }
}

constexpr int kMegaNodeBias = 8;  // measured with lean4: 1 -> 8 = +9 %

hipError_t launch_megakernel(const LaunchOpts& lo, const SceneView& scene, const FrameParams& fp, uint32_t frame0,
                             uint32_t nframes, uint32_t stride, bool accum, bool count, float* out, Counters* cnt,
                             hipStream_t stream) {
    SceneView sc = scene;
    if (sc.node_bias <= 0) sc.node_bias = kMegaNodeBias;
    // one node step per turn: more lose in the megakernel (Glossy 256^2: 3 steps -9 %, 8 -15 %,
    // profiles/r06h_ab_glossy_small_mega.log)
    if (sc.node_steps <= 0) sc.node_steps = 1;
    if (!accum) { nframes = 1; stride = 1; }
    if (lo.literal) {
        dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kMegaBlock);
#define LIT(A, C) PT_LAUNCH(KID_MEGA, stream, (k_mega<A, C>), grid, block, 0, stream, sc, fp, frame0, nframes, stride, out, cnt)
        if (accum) { if (count) LIT(true, true); else LIT(true, false); }
        else { if (count) LIT(false, true); else LIT(false, false); }
#undef LIT
        return hipGetLastError();
    }
    const bool lds = lo.lds && scene_fits_lds(sc);
    // lean4 + node bias 8 + fast reciprocal by default (measured at 1024^2 64 spp: 848 vs 611
    // for lean2 with majority turns and the division; scripts/perf_variants.py)
    const int trav0 = lo.trav < 0 ? 5 : std::min(lo.trav, 5);
    const bool fast = lo.fast_rcp != 0 && sc.fast_rcp;
    // + 160: cooperative big-leaf turns (SceneView::big_leaf; lean4 with the fast reciprocal)
    const bool big = sc.big_leaf > 0 && trav0 == 5 && fast;
    const int trav = trav0 + ((trav0 >= 3 && fast) ? 10 : 0) + (big ? 160 : 0);
#define RA(L, T) launch_regen_a<L, T>(sc, fp, frame0, nframes, stride, accum, count, out, cnt, stream)
#define RA_T(L, T) else if (trav == T) RA(L, T);
    if (lds) {
        if (trav == 0) RA(true, 0); RA_T(true, 1) RA_T(true, 2) RA_T(true, 3) RA_T(true, 4) RA_T(true, 5) RA_T(true, 13) RA_T(true, 14) RA_T(true, 15) RA_T(true, 175)
    } else {
        if (trav == 0) RA(false, 0); RA_T(false, 1) RA_T(false, 2) RA_T(false, 3) RA_T(false, 4) RA_T(false, 5) RA_T(false, 13) RA_T(false, 14) RA_T(false, 15) RA_T(false, 175)
    }
#undef RA_T
#undef RA
    return hipGetLastError();
}

hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream) {
    hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, stream, fn, a, b, o, n);
    return hipGetLastError();
}

}  // namespace pt
