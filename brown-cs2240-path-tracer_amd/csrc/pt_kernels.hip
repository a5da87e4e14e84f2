// pt_kernels.hip — HIP kernels for gfx950 (MI355X) replacing program-raymarch.wgsl.
//
//   k_mega<ACCUM, COUNT>  one lane per pixel (8x8 pixels per wave, 16x16 per
//                         256-thread workgroup, the reference's 8x8 tiling per
//                         wave); loops over the requested frames in order and
//                         accumulates clamp(L) in f32 registers exactly like the
//                         host loop of program-raymarch.ts:281-285, so the
//                         accumulator is bit-identical to the reference order.
//                         ACCUM=false is one reference dispatch (raw radiance).
//   k_selftest_math       exposes pt_math.h on device for the numerics tests.
#include "pt_kernels.h"

namespace pt {

template <bool COUNT>
__device__ f3 radiance(const SceneView& sc, const FrameParams& fp, Ray ray, uint32_t seed_in, int32_t* stack, int stride,
                       Counters& cnt) {
    // program-raymarch.wgsl:104-303
    f3 L = mk(0.0f, 0.0f, 0.0f), beta = mk(1.0f, 1.0f, 1.0f);
    int depth = 0;
    bool hit_specular = false;
    uint32_t seed = hash1u(seed_in);
    seed = hash1u(seed);
    const float rr = fp.rr_prob;
    while (depth <= fp.max_depth) {
        seed = hash1u(seed);
        if (COUNT) cnt.ext_queries++;
        float t;
        int rec = trace<COUNT>(sc, ray, t, stack, stride, cnt);
        if (rec < 0) break;
        Hit h = hit_data(sc, ray, rec, t);
        Mat m = load_mat(sc, h.mat);
        // emission (:136-141)
        if (sum3(m.Ke) > 0.0f && (depth == 0 || hit_specular)) {
            L = L + beta * m.Ke;
            break;
        }
        // next-event estimation (:146-187)
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
            if (sum3(nm.Ke) > 0.0f) {
                float att = pow2_lit(length(h.p - sh.p));
                f3 brdf;
                if (m.Ns == 40.0f) {
                    f3 refl = reflect(ray.d, h.n);
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
                float d2 = dot(h.n, ldir);
                f3 c = (beta * nm.Ke) * brdf;
                c = c * d1;
                c = c * d2;
                c = c / att;
                c = c * sc.inv_ntri;
                L = L + c;
            }
            if (fp.direct_only) break;
        }
        // russian roulette (:190-193)
        if (hash1(seed) > rr) break;
        // dielectric (:201-238)
        bool fresnel_reflect = false;
        if (m.illum == 7.0f) {
            f3 wi = ray.d;
            float eta_i = 1.0f, eta_t = 2.5f;
            float cos_i = clampf(dot(wi, h.n), -1.0f, 1.0f);
            f3 nn = h.n;
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
                ray = ray_eps(h.p, nd);
                hit_specular = true;
                beta = beta * (1.0f / rr);
                depth += 1;
                continue;
            }
        }
        // mirror (:241-253)
        if (m.Ns > 500.0f || fresnel_reflect) {
            ray = ray_eps(h.p, reflect(ray.d, h.n));
            hit_specular = true;
            beta = beta * (1.0f / rr);
            depth += 1;
            continue;
        }
        // diffuse / glossy (:255-299)
        float pdf;
        f3 nd = sample_hemisphere(h.n, seed, pdf);
        Ray nr = ray_eps(h.p, nd);
        f3 brdf;
        if (sum3(m.Ks) > 0.0f) {
            f3 refl = reflect(ray.d, h.n);
            float q = dot(refl, nr.d);
            if (q < 0.0f) {
                brdf = mk(0.0f, 0.0f, 0.0f);
            } else {
                float sf = ((m.Ns + 2.0f) / (2.0f * kPI)) * pow_p(q, m.Ns);
                brdf = m.Ks * sf;
                if (depth == 0) hit_specular = true;
            }
        } else {
            brdf = m.Kd / kPI;
        }
        float cosn = dot(nr.d, h.n) + 0.0f;  // vec4 dot: + w*w (= +0)
        f3 f = (brdf * cosn) / (pdf * rr);
        beta = beta * f;
        ray = nr;
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

template <bool ACCUM, bool COUNT>
__global__ __launch_bounds__(kMegaBlock) void k_mega(SceneView sc, FrameParams fp, uint32_t frame0, uint32_t nframes,
                                                    uint32_t stride, float* __restrict__ out, Counters* cnt_out) {
    __shared__ int32_t s_stack[kStackMax * kMegaBlock];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    Counters c = {};
    if (x < fp.width && y < fp.height) {
        float* o = out + 3 * ((size_t)y * fp.width + x);
        f3 acc = ACCUM ? mk(o[0], o[1], o[2]) : mk(0.0f, 0.0f, 0.0f);
        for (uint32_t i = 0; i < nframes; ++i) {
            uint32_t t = ACCUM ? (uint32_t)(float)(frame0 + i * stride) : frame0;
            uint32_t seed;
            Ray r = camera_ray(fp, x, y, t, seed);
            if (COUNT) c.samples++;
            f3 L = radiance<COUNT>(sc, fp, r, seed, s_stack + tid, kMegaBlock, c);
            if (ACCUM) {
                acc.x = acc.x + (L.x >= 0.0f ? L.x : 0.0f);
                acc.y = acc.y + (L.y >= 0.0f ? L.y : 0.0f);
                acc.z = acc.z + (L.z >= 0.0f ? L.z : 0.0f);
            } else {
                acc = L;
            }
        }
        o[0] = acc.x; o[1] = acc.y; o[2] = acc.z;
    }
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

hipError_t launch_mega(const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes, uint32_t stride,
                       bool accum, bool count, float* out, Counters* cnt, hipStream_t stream) {
    dim3 grid((fp.width + 15) / 16, (fp.height + 15) / 16), block(kMegaBlock);
    if (accum) {
        if (count) hipLaunchKernelGGL((k_mega<true, true>), grid, block, 0, stream, sc, fp, frame0, nframes, stride, out, cnt);
        else hipLaunchKernelGGL((k_mega<true, false>), grid, block, 0, stream, sc, fp, frame0, nframes, stride, out, cnt);
    } else {
        if (count) hipLaunchKernelGGL((k_mega<false, true>), grid, block, 0, stream, sc, fp, frame0, 1, 1, out, cnt);
        else hipLaunchKernelGGL((k_mega<false, false>), grid, block, 0, stream, sc, fp, frame0, 1, 1, out, cnt);
    }
    return hipGetLastError();
}

hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream) {
    hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, stream, fn, a, b, o, n);
    return hipGetLastError();
}

}  // namespace pt
