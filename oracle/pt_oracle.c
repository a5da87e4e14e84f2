/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the reference's per-pixel Monte Carlo path tracer
 * (Kauhentus/brown-cs2240-path-tracer, WGSL megakernel), written to be read side
 * by side with the WGSL.  It consumes the reference's packed buffers verbatim
 * (`primitive_0` = triangle buffer, `bvh_0` = BVH buffer, `meta_data` = 48 f32)
 * and follows the shader's control flow literally: the 64-entry traversal stack
 * with -1 markers, the strict-< closest hit, the exit-distance pruning quirk,
 * the seed algebra, the 1/Ntri NEE estimator, sticky hit_specular, etc.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline.  The product path
 * (brown-cs2240-path-tracer_amd/) never links or calls it.
 *
 * Parity status: the reference WGSL cannot run in this container (no WebGPU
 * adapter), so bit-level parity with the reference is
 * UNPINNED; this restatement is pinned statistically against the reference's
 * own renders (scenes/student_outputs/ PNGs, tests/test_student_outputs.py)
 * and structurally against the survey's independently derived scene counts.
 *
 * Numeric contract: IEEE f32 everywhere, correctly rounded
 * + - * / sqrt, no implicit contraction (build with -ffp-contract=off), FMAs
 * only where written as fmaf() below (the places a GPU compiler contracts
 * a*b+c), min/max with IEEE minNum/maxNum NaN handling, and the WGSL
 * transcendentals pinned to the Cephes single-precision algorithms
 * (po_sincosf/po_acosf/po_log2f/po_exp2f below).  Out-of-bounds storage reads
 * follow Dawn/Tint robustness (index clamped to len-1).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

/* -------------------------------------------------------------------------- */
/* f32 vector helpers (data-structs.wgsl:1-66 types)                           */
/* -------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 xyz(v4 a) { return V3(a.x, a.y, a.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v4 sub4(v4 a, v4 b) { return V4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 divs3(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 div3(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* dot(a,b) = a.x*b.x + a.y*b.y + a.z*b.z, contracted left to right */
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline float dot4(v4 a, v4 b) { return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x))); }
/* cross(a,b).x = a.y*b.z - a.z*b.y, first product fused */
static inline v3 cross3(v3 a, v3 b) {
    return V3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline float length4(v4 a) { return sqrtf(dot4(a, a)); }
static inline v3 normalize3(v3 a) { return divs3(a, length3(a)); }
static inline v4 normalize4(v4 a) {
    float l = length4(a);
    return V4(a.x / l, a.y / l, a.z / l, a.w / l);
}
/* a + b*s contracted: fma(b, s, a) */
static inline v3 madd3(v3 a, v3 b, float s) { return V3(fmaf(b.x, s, a.x), fmaf(b.y, s, a.y), fmaf(b.z, s, a.z)); }

/* -------------------------------------------------------------------------- */
/* Pinned transcendentals (WGSL leaves their precision implementation-defined) */
/* Cephes single-precision algorithms (S. L. Moshier), restated.                */
/* -------------------------------------------------------------------------- */
static inline float as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t as_uint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

EXPORT void po_sincosf(float x, float *s_out, float *c_out) {
    if (isnan(x) || isinf(x)) { *s_out = NAN; *c_out = NAN; return; }
    int sgn_s = 0;
    if (x < 0.0f) { x = -x; sgn_s = 1; }
    int j = (int)(x * 1.27323954473516f); /* 4/pi, truncation */
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    float r = fmaf(-y, 3.77489497744594108e-8f, fmaf(-y, 2.4187564849853515625e-4f, fmaf(-y, 0.78515625f, x)));
    float z = r * r;
    float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float S = fmaf(ps * z, r, r);
    float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float C = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
    float s, c;
    switch (j) {
        case 0: s = S; c = C; break;
        case 2: s = C; c = -S; break;
        case 4: s = -S; c = -C; break;
        default: s = -C; c = S; break; /* 6 */
    }
    *s_out = sgn_s ? -s : s;
    *c_out = c;
}
EXPORT float po_sinf(float x) { float s, c; po_sincosf(x, &s, &c); return s; }
EXPORT float po_cosf(float x) { float s, c; po_sincosf(x, &s, &c); return c; }
EXPORT float po_tanf(float x) { float s, c; po_sincosf(x, &s, &c); return s / c; }

static inline float asin_core(float a) {
    float z = a * a;
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z, 7.4953002686e-2f), z,
                   1.6666752422e-1f);
    return fmaf(p * z, a, a);
}
EXPORT float po_acosf(float x) {
    if (!(x >= -1.0f && x <= 1.0f)) return NAN;
    if (x < -0.5f) return 3.14159265358979323846f - 2.0f * asin_core(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_core(sqrtf(0.5f * (1.0f - x)));
    return 1.57079632679489661923f - asin_core(x);
}

EXPORT float po_log2f(float x) {
    if (isnan(x) || x < 0.0f) return NAN;
    if (x == 0.0f) return -INFINITY;
    if (isinf(x)) return INFINITY;
    int e_adj = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; e_adj = -23; } /* subnormal: scale by 2^23 */
    uint32_t b = as_uint(x);
    int e = (int)((b >> 23) & 0xffu) - 126 + e_adj;
    float m = as_float((b & 0x807fffffu) | 0x3f000000u); /* [0.5, 1) */
    if (m < 0.707106781186547524f) { e -= 1; m = (m + m) - 1.0f; } else { m = m - 1.0f; }
    float z = m * m;
    float p = 7.0376836292e-2f;
    p = fmaf(p, m, -1.1514610310e-1f);
    p = fmaf(p, m, 1.1676998740e-1f);
    p = fmaf(p, m, -1.2420140846e-1f);
    p = fmaf(p, m, 1.4249322787e-1f);
    p = fmaf(p, m, -1.6668057665e-1f);
    p = fmaf(p, m, 2.0000714765e-1f);
    p = fmaf(p, m, -2.4999993993e-1f);
    p = fmaf(p, m, 3.3333331174e-1f);
    float y = m * (z * p);
    y = fmaf(-0.5f, z, y);
    float r = fmaf(m, 0.44269504088896340736f, y * 0.44269504088896340736f);
    r = r + y;
    r = r + m;
    r = r + (float)e;
    return r;
}

static inline float ldexp_pinned(float r, int i) {
    if (i >= -126) return r * as_float((uint32_t)(i + 127) << 23);
    return (r * as_float(1u << 23)) * as_float((uint32_t)(i + 126 + 127) << 23);
}
EXPORT float po_exp2f(float x) {
    if (isnan(x)) return NAN;
    if (x > 127.0f) return INFINITY;
    if (x < -127.0f) return 0.0f;
    float px = floorf(x + 0.5f);
    int i0 = (int)px;
    float f = x - px;
    float p = 1.535336188319500e-4f;
    p = fmaf(p, f, 1.339887440266574e-3f);
    p = fmaf(p, f, 9.618437357674640e-3f);
    p = fmaf(p, f, 5.550332471162809e-2f);
    p = fmaf(p, f, 2.402264791363012e-1f);
    p = fmaf(p, f, 6.931472028550421e-1f);
    float r = 1.0f + p * f;
    return ldexp_pinned(r, i0);
}
/* pow(x, y) for runtime y: exp2(y * log2(x)) (WGSL's own definition of pow's precision) */
EXPORT float po_powf(float x, float y) {
    if (x < 0.0f || isnan(x) || isnan(y)) return NAN;
    if (x == 0.0f) return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : INFINITY);
    return po_exp2f(y * po_log2f(x));
}
/* literal exponents are strength-reduced */
static inline float pow2_lit(float x) { return x * x; }
static inline float pow5_lit(float x) { float x2 = x * x; return (x2 * x2) * x; }

/* -------------------------------------------------------------------------- */
/* RNG: hash.wgsl:1-28 (u32 wrapping arithmetic)                               */
/* -------------------------------------------------------------------------- */
static inline uint32_t mix(uint32_t n) {
    n = (n << 13u) ^ n;
    return n * (n * n * 15731u + 789221u) + 1376312589u;
}
EXPORT uint32_t po_hash1u(uint32_t n) { return mix(n) & 0x7fffffffu; }                         /* hash.wgsl:1-8 */
EXPORT float po_hash1(uint32_t n) { return 1.0f - (float)(mix(n) & 0x7fffffffu) / 2147483648.0f; } /* :10-17 */
EXPORT void po_hash2(uint32_t n, float out[2]) {                                                 /* :19-28 */
    n = mix(n);
    uint32_t kx = n * n, ky = n * (n * 16807u);
    out[0] = (float)(kx & 0x7fffffffu) / 2147483648.0f;
    out[1] = (float)(ky & 0x7fffffffu) / 2147483648.0f;
}

/* -------------------------------------------------------------------------- */
/* Scene view: the two packed buffers, read with Tint's clamped indexing       */
/* -------------------------------------------------------------------------- */
typedef struct {
    const float *tri; uint32_t tri_len;
    const float *bvh; uint32_t bvh_len;
} scene_t;
static inline float P(const scene_t *s, int32_t i) { uint32_t u = (uint32_t)i; if (u >= s->tri_len) u = s->tri_len - 1; return s->tri[u]; }
static inline float B(const scene_t *s, int32_t i) { uint32_t u = (uint32_t)i; if (u >= s->bvh_len) u = s->bvh_len - 1; return s->bvh[u]; }

typedef struct { uint64_t samples, ext_queries, shadow_queries, nodes, tri_tests, box_tests; } po_counters;

typedef struct { v4 p, d, d_inv; } ray_t; /* data-structs.wgsl:1-5 */
typedef struct { v4 point, normal; int intersected; float t; int32_t material_id; } isect_t;
typedef struct { float Ns, Ni, illum; v3 Ka, Kd, Ks, Ke; } material_t;

static inline isect_t null_isect(void) { isect_t r; memset(&r, 0, sizeof r); return r; }
static inline v4 inv4(v4 d) { return V4(1.0f / d.x, 1.0f / d.y, 1.0f / d.z, 1.0f / d.w); }
/* ray_with_epsilon: data-structs.wgsl:59-61, p + 0.001*d contracted */
static inline ray_t ray_with_epsilon(v4 p, v4 d) {
    ray_t r;
    r.p = V4(fmaf(0.001f, d.x, p.x), fmaf(0.001f, d.y, p.y), fmaf(0.001f, d.z, p.z), fmaf(0.001f, d.w, p.w));
    r.d = d; r.d_inv = inv4(d);
    return r;
}

/* ray-bbox-intersection.wgsl:1-31 */
static float ray_bbox(const ray_t *r, v3 mn, v3 mx) {
    float tmin = -3.0e+38f, tmax = 3.0e+38f;
    float t1x = (mn.x - r->p.x) * r->d_inv.x, t2x = (mx.x - r->p.x) * r->d_inv.x;
    tmin = fmaxf(tmin, fminf(t1x, t2x)); tmax = fminf(tmax, fmaxf(t1x, t2x));
    float t1y = (mn.y - r->p.y) * r->d_inv.y, t2y = (mx.y - r->p.y) * r->d_inv.y;
    tmin = fmaxf(tmin, fminf(t1y, t2y)); tmax = fminf(tmax, fmaxf(t1y, t2y));
    float t1z = (mn.z - r->p.z) * r->d_inv.z, t2z = (mx.z - r->p.z) * r->d_inv.z;
    tmin = fmaxf(tmin, fminf(t1z, t2z)); tmax = fminf(tmax, fmaxf(t1z, t2z));
    if (tmax > fmaxf(tmin, 0.0f)) return tmin > 0.0f ? tmin : tmax;
    return -1.0f;
}

/* ray-triangle-intersection.wgsl:1-42 (Moller-Trumbore, eps 1e-8) */
static isect_t ray_tri(const ray_t *r, v3 v0, v3 v1, v3 v2) {
    v3 rd = xyz(r->d), ro = xyz(r->p);
    const float eps = 1e-8f;
    v3 e1 = sub3(v1, v0), e2 = sub3(v2, v0);
    v3 rce2 = cross3(rd, e2);
    float det = dot3(e1, rce2);
    if (det > -eps && det < eps) return null_isect();
    float inv_det = 1.0f / det;
    v3 s = sub3(ro, v0);
    float u = inv_det * dot3(s, rce2);
    if (u < 0.0f || u > 1.0f) return null_isect();
    v3 sce1 = cross3(s, e1);
    float v = inv_det * dot3(rd, sce1);
    if (v < 0.0f || u + v > 1.0f) return null_isect();
    float t = inv_det * dot3(e2, sce1);
    if (t > eps) {
        isect_t h;
        v3 p = madd3(ro, rd, t);
        v3 n = normalize3(cross3(e1, e2));
        h.point = V4(p.x, p.y, p.z, 1.0f);
        h.normal = V4(n.x, n.y, n.z, 0.0f);
        h.intersected = 1; h.t = t; h.material_id = 0;
        return h;
    }
    return null_isect();
}

/* ray-triangle-intersection.wgsl:44-87 (ray_triangle_intersection_vertex_normals): the same test,
 * normal = normalize(w*v0n + u*v1n + v*v2n), w = 1 - u - v.  The reference calls it only from
 * commented-out code (intersection-logic.wgsl:81-108); vertex-normal mode (po_set_vertex_normals)
 * enables that branch.  The a*b+c sites are FMAs, as everywhere in the contract. */
static isect_t ray_tri_vn(const ray_t *r, v3 v0, v3 v1, v3 v2, v3 n0, v3 n1, v3 n2) {
    v3 rd = xyz(r->d), ro = xyz(r->p);
    const float eps = 1e-8f;
    v3 e1 = sub3(v1, v0), e2 = sub3(v2, v0);
    v3 rce2 = cross3(rd, e2);
    float det = dot3(e1, rce2);
    if (det > -eps && det < eps) return null_isect();
    float inv_det = 1.0f / det;
    v3 s = sub3(ro, v0);
    float u = inv_det * dot3(s, rce2);
    if (u < 0.0f || u > 1.0f) return null_isect();
    v3 sce1 = cross3(s, e1);
    float v = inv_det * dot3(rd, sce1);
    if (v < 0.0f || u + v > 1.0f) return null_isect();
    float w = (1.0f - u) - v;
    float t = inv_det * dot3(e2, sce1);
    if (t > eps) {
        isect_t h;
        v3 p = madd3(ro, rd, t);
        v3 nn = V3(fmaf(v, n2.x, fmaf(u, n1.x, w * n0.x)), fmaf(v, n2.y, fmaf(u, n1.y, w * n0.y)),
                   fmaf(v, n2.z, fmaf(u, n1.z, w * n0.z)));
        v3 n = normalize3(nn);
        h.point = V4(p.x, p.y, p.z, 1.0f);
        h.normal = V4(n.x, n.y, n.z, 0.0f);
        h.intersected = 1; h.t = t; h.material_id = 0;
        return h;
    }
    return null_isect();
}

static int g_vertex_normals; /* po_set_vertex_normals */
EXPORT void po_set_vertex_normals(int on) { g_vertex_normals = on != 0; }

static inline v3 vert(const scene_t *s, int32_t v_start, int32_t i) {
    return V3(P(s, v_start + i), P(s, v_start + i + 1), P(s, v_start + i + 2));
}

/* diagnostic hooks (scripts/leaf_visit_stats.c defines them; empty in the oracle build) */
#ifndef PO_LEAF_HOOK
#define PO_LEAF_HOOK(s, ray, lp)
#endif
#ifndef PO_INTERSECT_HOOK
#define PO_INTERSECT_HOOK(s, ray, closest_t)
#endif
static void test_leaf(const scene_t *s, const ray_t *ray, int32_t lp, isect_t *closest, float *closest_t, po_counters *c) {
    PO_LEAF_HOOK(s, ray, lp);
    float num_triangles = B(s, lp + 4);
    int32_t o_start = lp + 5 + 12;
    int32_t o_end = o_start + (int32_t)num_triangles;
    int32_t v_start = (int32_t)P(s, 2);
    int32_t vn_start = (int32_t)P(s, 5), vn_range = (int32_t)P(s, 6);
    for (int32_t i = o_start; i < o_end; i += 4) {
        int32_t i0 = ((int32_t)B(s, i) - 1) * 3, i1 = ((int32_t)B(s, i + 1) - 1) * 3, i2 = ((int32_t)B(s, i + 2) - 1) * 3;
        isect_t h = (g_vertex_normals && i2 < vn_range)
                        ? ray_tri_vn(ray, vert(s, v_start, i0), vert(s, v_start, i1), vert(s, v_start, i2),
                                     vert(s, vn_start, i0), vert(s, vn_start, i1), vert(s, vn_start, i2))
                        : ray_tri(ray, vert(s, v_start, i0), vert(s, v_start, i1), vert(s, v_start, i2));
        if (c) c->tri_tests++;
        if (h.intersected && (*closest_t < 0.0f || h.t < *closest_t)) {
            *closest = h;
            *closest_t = h.t;
            closest->material_id = (int32_t)B(s, i + 3);
        }
    }
}

/* intersection-logic.wgsl:1-215 — closest hit with the 64-entry marker stack.
 * SI: Tint clamps array indices; unreachable here (depth <= 16 => <= 33 entries). */
#define SI(i) ((i) > 63 ? 63 : (i))
static isect_t intersect(const scene_t *s, const ray_t *ray, po_counters *c) {
    int32_t stack[64];
    memset(stack, 0, sizeof stack);
    stack[0] = 6;
    int sp = 0;
    isect_t closest = null_isect();
    float closest_t = -1.0f;
    while (sp > -1) {
        int32_t ptr = stack[sp];
        if (c) { c->nodes++; c->box_tests += 2; }
        v3 lmin = V3(B(s, ptr + 5), B(s, ptr + 6), B(s, ptr + 7));
        v3 lmax = V3(B(s, ptr + 8), B(s, ptr + 9), B(s, ptr + 10));
        v3 rmin = V3(B(s, ptr + 11), B(s, ptr + 12), B(s, ptr + 13));
        v3 rmax = V3(B(s, ptr + 14), B(s, ptr + 15), B(s, ptr + 16));
        float ld = ray_bbox(ray, lmin, lmax), rd = ray_bbox(ray, rmin, rmax);
        int li = 0.0f < ld, ri = 0.0f < rd;
        int l_leaf = 0, r_leaf = 0;
        if (li) {
            int32_t lp = (int32_t)B(s, ptr + 2);
            if (B(s, lp) == 1.0f) { l_leaf = 1; test_leaf(s, ray, lp, &closest, &closest_t, c); }
        }
        if (ri) {
            int32_t rp = (int32_t)B(s, ptr + 3);
            if (B(s, rp) == 1.0f) { r_leaf = 1; test_leaf(s, ray, rp, &closest, &closest_t, c); }
        }
        int tl = li && !l_leaf && !(closest_t > 0.0f && ld > closest_t);
        int tr = ri && !r_leaf && !(closest_t > 0.0f && rd > closest_t);
        if (!tl && !tr) {
            sp -= 1;
            if (sp < 0) break;
            while (stack[sp] == -1) { sp -= 1; if (sp < 0) break; }
        } else {
            stack[sp] = -1;
            if (tl && !tr) { sp += 1; stack[SI(sp)] = (int32_t)B(s, ptr + 2); }
            else if (!tl && tr) { sp += 1; stack[SI(sp)] = (int32_t)B(s, ptr + 3); }
            else { stack[SI(sp + 1)] = (int32_t)B(s, ptr + 2); sp += 2; stack[SI(sp)] = (int32_t)B(s, ptr + 3); }
        }
    }
    PO_INTERSECT_HOOK(s, ray, closest_t);
    return closest;
}

/* program-raymarch.wgsl:87-102 */
static material_t get_material(const scene_t *s, int32_t id) {
    int32_t m = (int32_t)P(s, 4) + id * 15;
    material_t r;
    r.Ns = P(s, m); r.Ni = P(s, m + 1); r.illum = P(s, m + 2);
    r.Ka = V3(P(s, m + 3), P(s, m + 4), P(s, m + 5));
    r.Kd = V3(P(s, m + 6), P(s, m + 7), P(s, m + 8));
    r.Ks = V3(P(s, m + 9), P(s, m + 10), P(s, m + 11));
    r.Ke = V3(P(s, m + 12), P(s, m + 13), P(s, m + 14));
    return r;
}
static inline float sum3(v3 a) { return dot3(a, V3(1.0f, 1.0f, 1.0f)); }

/* samplers.wgsl:70-80 */
static v3 sample_triangle_3D(v3 p0, v3 p1, v3 p2, uint32_t seed) {
    float u[2]; po_hash2(seed, u);
    float su0 = sqrtf(u[0]);
    float bx = 1.0f - su0, by = u[1] * su0;
    float bz = (1.0f - bx) - by;
    return V3(fmaf(bz, p2.x, fmaf(by, p1.x, bx * p0.x)), fmaf(bz, p2.y, fmaf(by, p1.y, bx * p0.y)),
              fmaf(bz, p2.z, fmaf(by, p1.z, bx * p0.z)));
}

/* intersection-logic.wgsl:217-285 */
static v4 sample_area_lights(const scene_t *s, v3 x, int32_t seed) {
    int32_t e1s = (int32_t)P(s, 8), e1e = (int32_t)P(s, 9), e2s = (int32_t)P(s, 10), e2e = (int32_t)P(s, 11);
    int32_t e3s = (int32_t)P(s, 12), e3e = (int32_t)P(s, 13), e4s = (int32_t)P(s, 14), e4e = (int32_t)P(s, 15);
    int32_t n1 = 0, n2 = 0, n3 = 0, n4 = 0;
    if (e1s != -1) n1 += (e1e - e1s) / 4;
    if (e2s != -1) n2 += (e2e - e2s) / 4;
    if (e3s != -1) n3 += (e3e - e3s) / 4;
    if (e4s != -1) n4 += (e4e - e4s) / 4;
    int32_t ntri = n1 + n2 + n3 + n4;
    int32_t k = (int32_t)(po_hash1((uint32_t)seed * 7u + 11u) * (float)ntri);
    int32_t idx;
    if (k < n1) idx = k * 4 + e1s;
    else if (k < n1 + n2) idx = (k - n1) * 4 + e2s;
    else if (k < n1 + n2 + n3) idx = (k - n1 - n2) * 4 + e3s;
    else idx = (k - n1 - n2 - n3) * 4 + e4s;
    int32_t v_start = (int32_t)P(s, 2);
    int32_t i0 = ((int32_t)P(s, idx) - 1) * 3, i1 = ((int32_t)P(s, idx + 1) - 1) * 3, i2 = ((int32_t)P(s, idx + 2) - 1) * 3;
    v3 pt = sample_triangle_3D(vert(s, v_start, i0), vert(s, v_start, i1), vert(s, v_start, i2), (uint32_t)seed * 11u + 17u);
    v3 dir = normalize3(sub3(pt, x));
    return V4(dir.x, dir.y, dir.z, 1.0f / (float)ntri);
}

#define PI_F 3.14159f /* program-raymarch.wgsl:9 */

/* samplers.wgsl:15-46: cosine hemisphere, Duff et al. ONB */
static ray_t sample_hemisphere(v4 x, v4 n, int32_t seed, float *pdf) {
    float xi[2]; po_hash2((uint32_t)seed * 7u + 11u, xi);
    float phi = (2.0f * PI_F) * xi[0];
    float theta = po_acosf(sqrtf(xi[1]));
    float sp, cp, st, ct;
    po_sincosf(phi, &sp, &cp);
    po_sincosf(theta, &st, &ct);
    float nx = cp * st, ny = sp * st, nz = ct;
    v3 N = xyz(n);
    float s = N.z < 0.0f ? -1.0f : 1.0f;
    float a = -1.0f / (s + N.z);
    float b = (N.x * N.y) * a;
    v3 T = V3(fmaf((s * N.x) * N.x, a, 1.0f), s * b, (-s) * N.x);
    v3 Bv = V3(b, fmaf(N.y * N.y, a, s), -N.y);
    v3 d = V3(fmaf(N.x, nz, fmaf(Bv.x, ny, T.x * nx)), fmaf(N.y, nz, fmaf(Bv.y, ny, T.y * nx)),
              fmaf(N.z, nz, fmaf(Bv.z, ny, T.z * nx)));
    *pdf = ct / PI_F;
    return ray_with_epsilon(x, V4(d.x, d.y, d.z, 0.0f));
}

/* reflect: w_i - 2*dot(w_i, n)*n, contracted */
static inline v3 reflect3(v3 wi, v3 n) { float k = -(2.0f * dot3(wi, n)); return V3(fmaf(k, n.x, wi.x), fmaf(k, n.y, wi.y), fmaf(k, n.z, wi.z)); }

/* program-raymarch.wgsl:104-303 */
static v3 radiance(const scene_t *s, ray_t ray, int32_t seed_in, float rr_prob, int direct_only, int max_depth,
                   po_counters *c) {
    v3 L = V3(0, 0, 0), beta = V3(1, 1, 1);
    int depth = 0, hit_specular = 0;
    uint32_t seed = po_hash1u((uint32_t)seed_in);
    seed = po_hash1u(seed);
    while (depth <= max_depth) {
        seed = po_hash1u(seed);
        if (c) c->ext_queries++;
        isect_t hit = intersect(s, &ray, c);
        if (!hit.intersected) break;
        material_t m = get_material(s, hit.material_id);
        v4 n4 = hit.normal, p4 = hit.point;
        v3 n = xyz(n4);
        if (sum3(m.Ke) > 0.0f) {
            if (depth == 0 || hit_specular) { L = add3(L, mul3(beta, m.Ke)); break; }
        }
        /* direct lighting (NEE) */
        v4 off = V4(fmaf(n4.x, 1.0e-4f, p4.x), fmaf(n4.y, 1.0e-4f, p4.y), fmaf(n4.z, 1.0e-4f, p4.z), fmaf(n4.w, 1.0e-4f, p4.w));
        v4 sal = sample_area_lights(s, xyz(off), (int32_t)seed);
        v4 ldir = V4(sal.x, sal.y, sal.z, 0.0f);
        float mc = sal.w;
        seed = po_hash1u(seed + 7u);
        ray_t sray; sray.p = off; sray.d = ldir; sray.d_inv = inv4(ldir);
        if (c) c->shadow_queries++;
        isect_t sh = intersect(s, &sray, c);
        if (sh.intersected) {
            material_t nm = get_material(s, sh.material_id);
            if (sum3(nm.Ke) > 0.0f) {
                v3 ln = xyz(sh.normal);
                float att = pow2_lit(length4(sub4(p4, sh.point)));
                v3 brdf;
                if (m.Ns == 40.0f) {
                    float nn = m.Ns;
                    v3 refl = reflect3(xyz(ray.d), n);
                    float q = dot3(refl, xyz(ldir));
                    if (q < 0.0f) brdf = divs3(muls3(m.Kd, -q), PI_F);
                    else {
                        float sf = ((nn + 2.0f) * po_powf(q, nn)) / (2.0f * PI_F);
                        brdf = muls3(m.Ks, sf);
                    }
                } else {
                    brdf = divs3(m.Kd, PI_F);
                }
                float d1 = dot3(ln, neg3(xyz(ldir)));
                float d2 = dot3(n, xyz(ldir));
                v3 t = mul3(mul3(beta, nm.Ke), brdf);
                t = muls3(t, d1);
                t = muls3(t, d2);
                t = divs3(t, att);
                t = muls3(t, mc);
                L = add3(L, t);
            }
            if (direct_only) break;
        }
        /* russian roulette */
        if (po_hash1(seed) > rr_prob) break;

        int fresnel_reflect = 0;
        if (m.illum == 7.0f) {
            v3 wi = xyz(ray.d), nh = n;
            float eta_i = 1.0f, eta_t = 2.5f;
            float cos_i = fminf(fmaxf(dot3(wi, nh), -1.0f), 1.0f);
            v3 nn = nh;
            if (cos_i < 0.0f) cos_i = -cos_i;
            else { eta_i = 2.5f; eta_t = 1.0f; nn = neg3(nn); }
            float q = (eta_i - eta_t) / (eta_i + eta_t);
            float r0 = q * q;
            float r_theta = fmaf(1.0f - r0, pow5_lit(1.0f - cos_i), r0);
            seed = po_hash1u(seed + 7u);
            if (po_hash1(seed) < r_theta) {
                fresnel_reflect = 1;
            } else {
                float ratio = eta_i / eta_t;
                float k = fmaf(-(ratio * ratio), fmaf(-cos_i, cos_i, 1.0f), 1.0f);
                float kk = fminf(fmaxf(k, 0.0f), 1.0f);
                float cf = fmaf(ratio, cos_i, -sqrtf(kk));
                v3 nd = V3(fmaf(cf, nn.x, ratio * wi.x), fmaf(cf, nn.y, ratio * wi.y), fmaf(cf, nn.z, ratio * wi.z));
                ray = ray_with_epsilon(p4, V4(nd.x, nd.y, nd.z, 0.0f));
                hit_specular = 1;
                beta = muls3(beta, 1.0f / rr_prob);
                depth += 1;
                continue;
            }
        }
        if (m.Ns > 500.0f || fresnel_reflect) {
            v3 r = reflect3(xyz(ray.d), n);
            ray = ray_with_epsilon(p4, V4(r.x, r.y, r.z, 0.0f));
            hit_specular = 1;
            beta = muls3(beta, 1.0f / rr_prob);
            depth += 1;
            continue;
        }
        float pdf;
        ray_t nr = sample_hemisphere(p4, n4, (int32_t)seed, &pdf);
        v3 brdf = V3(0, 0, 0);
        if (sum3(m.Ks) > 0.0f) {
            v3 refl = reflect3(xyz(ray.d), n);
            float nn = m.Ns;
            float q = dot3(refl, xyz(nr.d));
            if (q < 0.0f) brdf = V3(0, 0, 0);
            else {
                float pf = po_powf(dot3(refl, xyz(nr.d)), nn);
                float sf = ((nn + 2.0f) / (2.0f * PI_F)) * pf;
                brdf = muls3(m.Ks, sf);
                if (depth == 0) hit_specular = 1;
            }
        } else {
            brdf = divs3(m.Kd, PI_F);
        }
        float cosn = dot4(nr.d, n4);
        v3 f = divs3(muls3(brdf, cosn), pdf * rr_prob);
        beta = mul3(beta, f);
        ray = nr;
        depth += 1;
    }
    return L;
}

/* program-raymarch.wgsl:35-85 for one (pixel, salt).  meta: 48 f32 (A2). */
static v3 pixel_sample(const scene_t *s, const float *meta, float view_half_h, uint32_t x, uint32_t y, uint32_t t,
                       int max_depth, po_counters *c) {
    float W = meta[0], H = meta[1];
    float focal = meta[2];
    v4 cam = V4(meta[4], meta[5], meta[6], meta[7]);
    float inv_w = meta[8], inv_h = meta[9];
    float aspect = meta[10];
    const float *M = meta + 28; /* cam_to_world, column-major */
    uint32_t index = x + y * (uint32_t)W;
    uint32_t ts = index * 16787u + t;
    ts = po_hash1u(ts);
    ts = po_hash1u(ts);
    float jit[2]; po_hash2(ts, jit);
    float gx = (float)x + (jit[0] - 0.5f), gy = (float)y + (jit[1] - 0.5f);
    float norm_x = fmaf(gx + 0.5f, inv_w, -0.5f);
    float norm_y = fmaf(((H - 1.0f) - gy) + 0.5f, inv_h, -0.5f);
    float view_half_w = view_half_h * aspect;
    float vx = view_half_w * norm_x, vy = view_half_h * norm_y;
    ts = po_hash1u(ts);
    v4 pp = V4(vx, vy, -focal, 1.0f);
    v4 pw;
    pw.x = fmaf(M[12], pp.w, fmaf(M[8], pp.z, fmaf(M[4], pp.y, M[0] * pp.x)));
    pw.y = fmaf(M[13], pp.w, fmaf(M[9], pp.z, fmaf(M[5], pp.y, M[1] * pp.x)));
    pw.z = fmaf(M[14], pp.w, fmaf(M[10], pp.z, fmaf(M[6], pp.y, M[2] * pp.x)));
    pw.w = fmaf(M[15], pp.w, fmaf(M[11], pp.z, fmaf(M[7], pp.y, M[3] * pp.x)));
    v4 dir = normalize4(sub4(pw, cam));
    ray_t ray; ray.p = cam; ray.d = dir; ray.d_inv = inv4(dir);
    /* u32(i + i32(index*67) + i32(t)) with i = 0: two's-complement wrap == u32 wrap */
    ts = po_hash1u(ts + (index * 67u + t));
    if (c) c->samples++;
    return radiance(s, ray, (int32_t)ts, meta[45], meta[46] > 0.0f, max_depth, c);
}

/* view_half_h = 2 * focal * tan(vfov * 0.5), program-raymarch.wgsl:62 */
EXPORT float po_view_half_h(const float *meta) { return (2.0f * meta[2]) * po_tanf(meta[3] * 0.5f); }

/* One dispatch of the reference (1 spp, salt t): out[3*(x+y*W)+c] = radiance. */
EXPORT void po_frame(const float *tri, uint32_t tri_len, const float *bvh, uint32_t bvh_len, const float *meta,
                     uint32_t y0, uint32_t y1, uint32_t t, int max_depth, float *out, po_counters *cnt, int nthreads) {
    scene_t s = {tri, tri_len, bvh, bvh_len};
    uint32_t W = (uint32_t)meta[0];
    float vh = po_view_half_h(meta);
    po_counters total; memset(&total, 0, sizeof total);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        po_counters loc; memset(&loc, 0, sizeof loc);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t y = y0; y < (int64_t)y1; y++)
            for (uint32_t x = 0; x < W; x++) {
                v3 L = pixel_sample(&s, meta, vh, x, (uint32_t)y, t, max_depth, cnt ? &loc : NULL);
                float *o = out + 3 * ((size_t)(y - y0) * W + x);
                o[0] = L.x; o[1] = L.y; o[2] = L.z;
            }
        if (cnt) {
#ifdef _OPENMP
#pragma omp critical
#endif
            {
                total.samples += loc.samples; total.ext_queries += loc.ext_queries; total.shadow_queries += loc.shadow_queries;
                total.nodes += loc.nodes; total.tri_tests += loc.tri_tests; total.box_tests += loc.box_tests;
            }
        }
    }
    (void)nthreads;
    if (cnt) {
        cnt->samples += total.samples; cnt->ext_queries += total.ext_queries; cnt->shadow_queries += total.shadow_queries;
        cnt->nodes += total.nodes; cnt->tri_tests += total.tri_tests; cnt->box_tests += total.box_tests;
    }
}

/* program-raymarch.ts:281-285: sample_collector += (v >= 0 ? v : 0), f32, frame order.
 * Renders frames k = frame0 + i*stride (salt t_k = u32(f32(k))) for rows [y0, y1) into acc (in/out). */
EXPORT void po_render(const float *tri, uint32_t tri_len, const float *bvh, uint32_t bvh_len, const float *meta,
                      uint32_t y0, uint32_t y1, uint32_t frame0, uint32_t nframes, uint32_t stride, int max_depth,
                      float *acc, po_counters *cnt, int nthreads) {
    scene_t s = {tri, tri_len, bvh, bvh_len};
    uint32_t W = (uint32_t)meta[0];
    float vh = po_view_half_h(meta);
    po_counters total; memset(&total, 0, sizeof total);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        po_counters loc; memset(&loc, 0, sizeof loc);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t y = y0; y < (int64_t)y1; y++)
            for (uint32_t x = 0; x < W; x++) {
                float *a = acc + 3 * ((size_t)(y - y0) * W + x);
                for (uint32_t i = 0; i < nframes; i++) {
                    uint32_t k = frame0 + i * stride;
                    uint32_t t = (uint32_t)(float)k;
                    v3 L = pixel_sample(&s, meta, vh, x, (uint32_t)y, t, max_depth, cnt ? &loc : NULL);
                    a[0] = a[0] + (L.x >= 0.0f ? L.x : 0.0f);
                    a[1] = a[1] + (L.y >= 0.0f ? L.y : 0.0f);
                    a[2] = a[2] + (L.z >= 0.0f ? L.z : 0.0f);
                }
            }
        if (cnt) {
#ifdef _OPENMP
#pragma omp critical
#endif
            {
                total.samples += loc.samples; total.ext_queries += loc.ext_queries; total.shadow_queries += loc.shadow_queries;
                total.nodes += loc.nodes; total.tri_tests += loc.tri_tests; total.box_tests += loc.box_tests;
            }
        }
    }
    if (cnt) {
        cnt->samples += total.samples; cnt->ext_queries += total.ext_queries; cnt->shadow_queries += total.shadow_queries;
        cnt->nodes += total.nodes; cnt->tri_tests += total.tri_tests; cnt->box_tests += total.box_tests;
    }
}

/* Single-query entry points for known-answer tests. ray: p[4], d[4]; d_inv computed as 1/d. */
EXPORT float po_ray_bbox(const float *p, const float *d, const float *mn, const float *mx) {
    ray_t r; r.p = V4(p[0], p[1], p[2], p[3]); r.d = V4(d[0], d[1], d[2], d[3]); r.d_inv = inv4(r.d);
    return ray_bbox(&r, V3(mn[0], mn[1], mn[2]), V3(mx[0], mx[1], mx[2]));
}
/* out: point xyz, normal xyz, t, material_id; returns intersected */
EXPORT int po_intersect(const float *tri, uint32_t tri_len, const float *bvh, uint32_t bvh_len, const float *p,
                        const float *d, float *out, po_counters *cnt) {
    scene_t s = {tri, tri_len, bvh, bvh_len};
    ray_t r; r.p = V4(p[0], p[1], p[2], p[3]); r.d = V4(d[0], d[1], d[2], d[3]); r.d_inv = inv4(r.d);
    isect_t h = intersect(&s, &r, cnt);
    out[0] = h.point.x; out[1] = h.point.y; out[2] = h.point.z;
    out[3] = h.normal.x; out[4] = h.normal.y; out[5] = h.normal.z;
    out[6] = h.t; out[7] = (float)h.material_id;
    return h.intersected;
}

/* program-raymarch.ts:295-316 tone map in JS doubles; u8 = ToInt32(final*255) clamped. */
static inline int32_t to_int32(double v) {
    if (!isfinite(v)) return 0;
    double t = trunc(v);
    double m = fmod(t, 4294967296.0);
    if (m < 0) m += 4294967296.0;
    uint32_t u = (uint32_t)m;
    return (int32_t)u;
}
static inline uint8_t clamp_u8(int32_t v) { return v < 0 ? 0 : (v > 255 ? 255 : (uint8_t)v); }
EXPORT void po_tonemap(const float *acc, uint64_t npix, uint32_t sample_runs, uint8_t *rgba) {
    for (uint64_t i = 0; i < npix; i++) {
        double r = (double)acc[3 * i] / sample_runs, g = (double)acc[3 * i + 1] / sample_runs,
               b = (double)acc[3 * i + 2] / sample_runs;
        double lum = (r + g + b) / 3.0;
        double lo = lum / (lum + 1.0);
        double f = pow(lo, 0.01);
        rgba[4 * i] = clamp_u8(to_int32(r * f * 255.0));
        rgba[4 * i + 1] = clamp_u8(to_int32(g * f * 255.0));
        rgba[4 * i + 2] = clamp_u8(to_int32(b * f * 255.0));
        rgba[4 * i + 3] = 255;
    }
}
