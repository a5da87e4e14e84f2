// pt_path.h — one path of program-raymarch.wgsl:35-303 cut at its two traversal calls.
//
//   path_begin        main() seed chain + camera ray, radiance() prologue and first loop head
//   path_after_ext    after intersect(ray): miss / emission end the path; otherwise NEE
//                     samples a light and the path continues with its SHADOW ray
//   path_after_shadow after intersect(shadow ray): NEE contribution, direct-only exit,
//                     Russian roulette, BSDF; the path continues with its next EXTENSION ray
//
// Both the megakernel (k_regen) and the wavefront kernels call exactly these functions, so
// they execute the same f32 operations in the same order as the oracle's radiance().
#pragma once
#include "pt_device.h"

namespace pt {

struct PathState {
    f3 L, beta;
    f3 hp, hn, wi;  // shading point, its normal, incoming direction (live across the shadow trace)
    uint32_t seed;
    int depth;
    int mat_id;
    bool spec;
};

// NEE contribution once the shadow ray hit an emitter (program-raymarch.wgsl:154-182).
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
        brdf = m.Kd_pi;  // = m.Kd / kPI, bit for bit (precomputed per material)
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
// In: ray.d = incoming direction.  Out: ray = continuation ray; beta/spec/seed updated.
__device__ __forceinline__ void bsdf_continue(const Mat& m, f3 hp, f3 hn, Ray& ray, f3& beta, bool& spec,
                                              uint32_t& seed, int depth, float rr) {
    bool fresnel_reflect = false;
    if (m.illum == 7.0f) {
        f3 wi = ray.d;
        float cos_i = clampf(dot(wi, hn), -1.0f, 1.0f);
        f3 nn = hn;
        // eta_i, eta_t = 1, 2.5 (entering) or 2.5, 1; the quotients of these constants are folded
        // by the compiler with the same IEEE rounding: q = (eta_i - eta_t) / (eta_i + eta_t),
        // ratio = eta_i / eta_t
        constexpr float kQin = (1.0f - 2.5f) / (1.0f + 2.5f), kQout = (2.5f - 1.0f) / (2.5f + 1.0f);
        constexpr float kRatioIn = 1.0f / 2.5f, kRatioOut = 2.5f / 1.0f;
        const bool entering = cos_i < 0.0f;
        if (entering) {
            cos_i = -cos_i;
        } else {
            nn = -nn;
        }
        float q = entering ? kQin : kQout;
        float r0 = q * q;
        float r_theta = fmaf(1.0f - r0, pow5_lit(1.0f - cos_i), r0);
        seed = hash1u(seed + 7u);
        if (hash1(seed) < r_theta) {
            fresnel_reflect = true;
        } else {
            float ratio = entering ? kRatioIn : kRatioOut;
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
            float sf = m.phong * pow_p(q, m.Ns);  // m.phong = (m.Ns + 2) / (2 kPI)
            brdf = m.Ks * sf;
            if (depth == 0) spec = true;
        }
    } else {
        brdf = m.Kd_pi;  // = m.Kd / kPI, bit for bit (precomputed per material)
    }
    float cosn = dot(nr.d, hn) + 0.0f;  // vec4 dot: + w*w (= +0)
    f3 f = (brdf * cosn) / (pdf * rr);
    beta = beta * f;
    ray = nr;
}

// main() (program-raymarch.wgsl:50-77) + radiance() prologue and first loop head (:115-123)
__device__ __forceinline__ Ray path_begin(const FrameParams& fp, uint32_t x, uint32_t y, uint32_t t, PathState& ps) {
    uint32_t s0;
    Ray ray = camera_ray(fp, x, y, t, s0);
    ps.seed = hash1u(hash1u(hash1u(s0)));
    ps.L = mk(0.0f, 0.0f, 0.0f);
    ps.beta = mk(1.0f, 1.0f, 1.0f);
    ps.hp = ps.hn = ps.wi = mk(0.0f, 0.0f, 0.0f);
    ps.depth = 0;
    ps.mat_id = 0;
    ps.spec = false;
    return ray;
}

// :124-151 after the extension trace.  Returns true when the path continues; `ray` then
// holds the shadow ray and ps the shading point.
__device__ __forceinline__ bool path_after_ext(const SceneView& sc, int rec, float t, Ray& ray, PathState& ps) {
    if (rec < 0) return false;
    Hit h = hit_data(sc, ray, rec, t);
    Mat m = load_mat(sc, h.mat);
    if (sum3(m.Ke) > 0.0f && (ps.depth == 0 || ps.spec)) {
        ps.L = ps.L + ps.beta * m.Ke;
        return false;
    }
    f3 off = madd(h.p, h.n, 1.0e-4f);
    f3 ldir = sample_area_lights(sc, off, ps.seed);
    ps.seed = hash1u(ps.seed + 7u);
    ps.hp = h.p; ps.hn = h.n; ps.wi = ray.d; ps.mat_id = h.mat;
    ray.o = off; ray.d = ldir; ray.inv = rcp3(ldir);
    return true;
}

// :152-299 (+ loop test :118 and head :123) after the shadow trace.  Returns true when
// the path continues; `ray` then holds the next extension ray.
__device__ __forceinline__ bool path_after_shadow(const SceneView& sc, const FrameParams& fp, int rec, float t, Ray& ray,
                                                  PathState& ps) {
    const Mat m = load_mat(sc, ps.mat_id);
    if (rec >= 0) {
        Hit sh = hit_data(sc, ray, rec, t);
        Mat nm = load_mat(sc, sh.mat);
        if (sum3(nm.Ke) > 0.0f) ps.L = ps.L + nee_contrib(m, ps.wi, ps.hp, ps.hn, ray.d, ps.beta, sh, nm, sc.inv_ntri);
        if (fp.direct_only) return false;
    }
    if (hash1(ps.seed) > fp.rr_prob) return false;
    ray.d = ps.wi;
    bsdf_continue(m, ps.hp, ps.hn, ray, ps.beta, ps.spec, ps.seed, ps.depth, fp.rr_prob);
    ps.depth += 1;
    if (ps.depth > fp.max_depth) return false;
    ps.seed = hash1u(ps.seed);
    return true;
}

// program-raymarch.ts:283-285: sample_collector += (v >= 0 ? v : 0)
__device__ __forceinline__ f3 add_clamped(f3 acc, f3 L) {
    return mk(acc.x + (L.x >= 0.0f ? L.x : 0.0f), acc.y + (L.y >= 0.0f ? L.y : 0.0f), acc.z + (L.z >= 0.0f ? L.z : 0.0f));
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

// Copy the scene span into LDS at `base` (whole workgroup) and point `sc` at it.
__device__ __forceinline__ void stage_scene_lds(SceneView& sc, char* base) {
    const float4* src = reinterpret_cast<const float4*>(sc.nodes);
    float4* dst = reinterpret_cast<float4*>(base);
    for (uint32_t k = threadIdx.x; k < sc.span_bytes / 16u; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
    sc.nodes = reinterpret_cast<const Node*>(base);
    sc.tris = reinterpret_cast<const Tri*>(base + sc.off_tris);
    sc.mats = reinterpret_cast<const Material*>(base + sc.off_mats);
    sc.lights = reinterpret_cast<const Light*>(base + sc.off_lights);
    sc.lmask = reinterpret_cast<const uint64_t*>(base + sc.off_lmask);
    if (sc.bfnode) {
        sc.bfnode = reinterpret_cast<const BfNode*>(base + sc.off_bfnode);
        sc.bfmap = reinterpret_cast<const int32_t*>(base + sc.off_bfmap);
    }
}

}  // namespace pt
