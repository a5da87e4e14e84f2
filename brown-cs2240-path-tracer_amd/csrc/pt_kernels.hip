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

namespace pt {

// ---------------------------------------------------------------------------------------
// Shading pieces shared by both kernels (program-raymarch.wgsl:104-303)
// ---------------------------------------------------------------------------------------

// NEE contribution once the shadow ray hit an emitter (program-raymarch.wgsl:154-182).
// m: material at the shading point; wi: incoming direction; hp/hn: shading point/normal.
__device__ __forceinline__ f3 nee_contrib(const Mat& m, f3 wi, f3 hp, f3 hn, f3 ldir, f3 beta, const Hit& sh,
                                          const Mat& nm, float inv_ntri) {
    float att = pow2_lit(length(hp - sh.p));
    f3 brdf;
    if (m.Ns == 40.0f) {
        f3 refl = reflect(wi, hn);
        float q = dot(refl, ldir);
        if (q < 0.0f) {
            brdf = (m.Kd * (-q)) / kPI;
        } else {
            float sf = ((m.Ns + 2.0f) * pow_p(q, m.Ns)) / (2.0f * kPI);
            brdf = m.Ks * sf;
        }
    } else {
        brdf = m.Kd / kPI;
    }
    float d1 = dot(sh.n, -ldir);
    float d2 = dot(hn, ldir);
    f3 c = (beta * nm.Ke) * brdf;
    c = c * d1;
    c = c * d2;
    c = c / att;
    return c * inv_ntri;
}

// BSDF continuation after Russian roulette survived (program-raymarch.wgsl:199-299):
// dielectric (illum 7), mirror (Ns > 500 or Fresnel reflection), Phong-glossy or Lambert.
// In: ray.d = incoming direction.  Out: ray = continuation ray, beta/spec/seed updated.
// The caller increments depth.
__device__ __forceinline__ void bsdf_continue(const Mat& m, f3 hp, f3 hn, Ray& ray, f3& beta, bool& spec,
                                              uint32_t& seed, int depth, float rr) {
    bool fresnel_reflect = false;
    if (m.illum == 7.0f) {
        f3 wi = ray.d;
        float eta_i = 1.0f, eta_t = 2.5f;
        float cos_i = clampf(dot(wi, hn), -1.0f, 1.0f);
        f3 nn = hn;
        if (cos_i < 0.0f) {
            cos_i = -cos_i;
        } else {
            eta_i = 2.5f; eta_t = 1.0f; nn = -nn;
        }
        float q = (eta_i - eta_t) / (eta_i + eta_t);
        float r0 = q * q;
        float r_theta = fmaf(1.0f - r0, pow5_lit(1.0f - cos_i), r0);
        seed = hash1u(seed + 7u);
        if (hash1(seed) < r_theta) {
            fresnel_reflect = true;
        } else {
            float ratio = eta_i / eta_t;
            float k = fmaf(-(ratio * ratio), fmaf(-cos_i, cos_i, 1.0f), 1.0f);
            float cf = fmaf(ratio, cos_i, -sqrtf(clampf(k, 0.0f, 1.0f)));
            f3 nd = mk(fmaf(cf, nn.x, ratio * wi.x), fmaf(cf, nn.y, ratio * wi.y), fmaf(cf, nn.z, ratio * wi.z));
            ray = ray_eps(hp, nd);
            spec = true;
            beta = beta * (1.0f / rr);
            return;
        }
    }
    if (m.Ns > 500.0f || fresnel_reflect) {
        ray = ray_eps(hp, reflect(ray.d, hn));
        spec = true;
        beta = beta * (1.0f / rr);
        return;
    }
    float pdf;
    f3 nd = sample_hemisphere(hn, seed, pdf);
    Ray nr = ray_eps(hp, nd);
    f3 brdf;
    if (sum3(m.Ks) > 0.0f) {
        f3 refl = reflect(ray.d, hn);
        float q = dot(refl, nr.d);
        if (q < 0.0f) {
            brdf = mk(0.0f, 0.0f, 0.0f);
        } else {
            float sf = ((m.Ns + 2.0f) / (2.0f * kPI)) * pow_p(q, m.Ns);
            brdf = m.Ks * sf;
            if (depth == 0) spec = true;
        }
    } else {
        brdf = m.Kd / kPI;
    }
    float cosn = dot(nr.d, hn) + 0.0f;  // vec4 dot: + w*w (= +0)
    f3 f = (brdf * cosn) / (pdf * rr);
    beta = beta * f;
    ray = nr;
}

template <bool COUNT>
__device__ f3 radiance(const SceneView& sc, const FrameParams& fp, Ray ray, uint32_t seed_in, int32_t* stack, int stride,
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
        int rec = trace<COUNT>(sc, ray, t, stack, stride, cnt);
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
        int srec = trace<COUNT>(sc, sray, st, stack, stride, cnt);
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void flush_counters(const Counters& c, Counters* out) {
    uint64_t v[6] = {c.samples, c.ext_queries, c.shadow_queries, c.nodes, c.tri_tests, c.box_tests};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        uint64_t s = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(reinterpret_cast<unsigned long long*>(out) + i, (unsigned long long)s);
    }
}

__device__ __forceinline__ void pixel_of(uint32_t& x, uint32_t& y) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
}

__device__ __forceinline__ f3 add_clamped(f3 acc, f3 L) {
    // program-raymarch.ts:283-285: sample_collector += (v >= 0 ? v : 0)
    return mk(acc.x + (L.x >= 0.0f ? L.x : 0.0f), acc.y + (L.y >= 0.0f ? L.y : 0.0f), acc.z + (L.z >= 0.0f ? L.z : 0.0f));
}

template <bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kMegaBlock) void k_mega(SceneView sc, FrameParams fp, uint32_t frame0, uint32_t nframes,
                                                    uint32_t stride, float* __restrict__ out, Counters* cnt_out) {
    __shared__ int32_t s_stack[kStackMax * kMegaBlock];
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
            f3 L = radiance<COUNT>(sc, fp, r, seed, s_stack + threadIdx.x, kMegaBlock, c);
            acc = ACCUM ? add_clamped(acc, L) : L;
        }
        o[0] = acc.x; o[1] = acc.y; o[2] = acc.z;
    }
    if (COUNT) flush_counters(c, cnt_out);
}

// ---------------------------------------------------------------------------------------
// Production megakernel: path regeneration, one traversal site, optional LDS scene
// ---------------------------------------------------------------------------------------
template <bool LDS, bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kMegaBlock) void k_regen(SceneView g_sc, FrameParams fp, uint32_t frame0, uint32_t nframes,
                                                     uint32_t stride, float* __restrict__ out, Counters* cnt_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    int32_t* stack = reinterpret_cast<int32_t*>(smem) + tid;  // [max_stack][256] int32, lane-minor
    const uint32_t stack_bytes = (uint32_t)g_sc.max_stack * kMegaBlock * 4u;
    SceneView sc = g_sc;
    if (LDS) {
        char* base = smem + stack_bytes;
        const float4* src = reinterpret_cast<const float4*>(g_sc.nodes);
        float4* dst = reinterpret_cast<float4*>(base);
        for (uint32_t k = tid; k < g_sc.span_bytes / 16u; k += kMegaBlock) dst[k] = src[k];
        __syncthreads();
        sc.nodes = reinterpret_cast<const Node*>(base);
        sc.tris = reinterpret_cast<const Tri*>(base + g_sc.off_tris);
        sc.mats = reinterpret_cast<const Material*>(base + g_sc.off_mats);
        sc.lights = reinterpret_cast<const Light*>(base + g_sc.off_lights);
    }
    uint32_t x, y;
    pixel_of(x, y);
    Counters c = {};
    const bool valid = x < fp.width && y < fp.height;
    float* o = out + 3 * ((size_t)(valid ? y : 0) * fp.width + (valid ? x : 0));
    f3 acc = (ACCUM && valid) ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);
    const float rr = fp.rr_prob;

    enum { kIdle = 0, kExt = 1, kShadow = 2 };
    int phase = kIdle;
    uint32_t next = 0;  // next frame of this pixel to start
    Ray ray;
    f3 L, beta, hp, hn, wi;
    uint32_t seed = 0;
    int depth = 0, mat_id = 0;
    bool spec = false;

    while (true) {
        if (phase == kIdle) {
            if (!valid || next >= nframes) break;
            // main(): seed chain + camera ray (program-raymarch.wgsl:50-77)
            const uint32_t t = ACCUM ? (uint32_t)(float)(frame0 + next * stride) : frame0;
            ++next;
            uint32_t s0;
            ray = camera_ray(fp, x, y, t, s0);
            // radiance() prologue + first loop head (:115-123)
            seed = hash1u(hash1u(hash1u(s0)));
            L = mk(0.0f, 0.0f, 0.0f);
            beta = mk(1.0f, 1.0f, 1.0f);
            depth = 0;
            spec = false;
            phase = kExt;
            if (COUNT) { c.samples++; c.ext_queries++; }
        }
        float t;
        const int rec = trace<COUNT>(sc, ray, t, stack, kMegaBlock, c);
        bool done = false;
        if (phase == kExt) {
            if (rec < 0) {
                done = true;
            } else {
                Hit h = hit_data(sc, ray, rec, t);
                Mat m = load_mat(sc, h.mat);
                if (sum3(m.Ke) > 0.0f && (depth == 0 || spec)) {
                    L = L + beta * m.Ke;
                    done = true;
                } else {
                    // NEE: light sample + shadow ray (:146-151)
                    f3 off = madd(h.p, h.n, 1.0e-4f);
                    f3 ldir = sample_area_lights(sc, off, seed);
                    seed = hash1u(seed + 7u);
                    hp = h.p; hn = h.n; wi = ray.d; mat_id = h.mat;
                    ray.o = off; ray.d = ldir; ray.inv = rcp3(ldir);
                    phase = kShadow;
                    if (COUNT) c.shadow_queries++;
                }
            }
        } else {
            const Mat m = load_mat(sc, mat_id);
            if (rec >= 0) {
                Hit sh = hit_data(sc, ray, rec, t);
                Mat nm = load_mat(sc, sh.mat);
                if (sum3(nm.Ke) > 0.0f) L = L + nee_contrib(m, wi, hp, hn, ray.d, beta, sh, nm, sc.inv_ntri);
                if (fp.direct_only) done = true;
            }
            if (!done) {
                if (hash1(seed) > rr) {
                    done = true;
                } else {
                    ray.d = wi;
                    bsdf_continue(m, hp, hn, ray, beta, spec, seed, depth, rr);
                    depth += 1;
                    if (depth > fp.max_depth) {
                        done = true;
                    } else {
                        seed = hash1u(seed);  // loop head (:123)
                        phase = kExt;
                        if (COUNT) c.ext_queries++;
                    }
                }
            }
        }
        if (done) {
            acc = ACCUM ? add_clamped(acc, L) : L;
            phase = kIdle;
        }
    }
    if (valid) { o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; }
    if (COUNT) flush_counters(c, cnt_out);
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

template <bool LDS, bool ACCUM, bool COUNT>
static void launch_regen_t(const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes, uint32_t stride,
                           float* out, Counters* cnt, hipStream_t stream) {
    dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kMegaBlock);
    size_t lds = (size_t)sc.max_stack * kMegaBlock * 4 + (LDS ? sc.span_bytes : 0);
    hipLaunchKernelGGL((k_regen<LDS, ACCUM, COUNT>), grid, block, lds, stream, sc, fp, frame0, nframes, stride, out, cnt);
}

hipError_t launch_render(KernelKind kind, const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes,
                         uint32_t stride, bool accum, bool count, float* out, Counters* cnt, hipStream_t stream) {
    if (!accum) { nframes = 1; stride = 1; }
    if (kind == KernelKind::Literal) {
        dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kMegaBlock);
#define LIT(A, C) hipLaunchKernelGGL((k_mega<A, C>), grid, block, 0, stream, sc, fp, frame0, nframes, stride, out, cnt)
        if (accum) { if (count) LIT(true, true); else LIT(true, false); }
        else { if (count) LIT(false, true); else LIT(false, false); }
#undef LIT
        return hipGetLastError();
    }
    const bool lds = (kind == KernelKind::RegenLds || kind == KernelKind::Auto) && scene_fits_lds(sc);
#define REG(L, A, C) launch_regen_t<L, A, C>(sc, fp, frame0, nframes, stride, out, cnt, stream)
    if (lds) {
        if (accum) { if (count) REG(true, true, true); else REG(true, true, false); }
        else { if (count) REG(true, false, true); else REG(true, false, false); }
    } else {
        if (accum) { if (count) REG(false, true, true); else REG(false, true, false); }
        else { if (count) REG(false, false, true); else REG(false, false, false); }
    }
#undef REG
    return hipGetLastError();
}

hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream) {
    hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, stream, fn, a, b, o, n);
    return hipGetLastError();
}

}  // namespace pt
