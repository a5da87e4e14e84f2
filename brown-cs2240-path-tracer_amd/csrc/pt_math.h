// pt_math.h — f32 numerics of the path-tracing core, host+device.
//
// The reference WGSL leaves tan/acos/cos/sin/pow/normalize precision
// implementation-defined (SURVEY.md §7 "Non-bitwise math").  This header pins
// them ("numeric contract"):
//   * + - * / sqrt are IEEE f32, correctly rounded (hipcc's gfx950 default:
//     v_div_scale/v_div_fmas/v_div_fixup and the corrected v_sqrt sequence);
//     denormals preserved (amdhsa_float_denorm_mode_32 = 3);
//   * no implicit contraction (-ffp-contract=off); an FMA appears exactly
//     where written as fmaf(): the a*b+c sites a GPU compiler contracts;
//   * min/max are IEEE minNum/maxNum (v_min_f32 / v_max_f32);
//   * sin/cos/acos/log2/exp2 follow the Cephes single-precision algorithms
//     (S. L. Moshier); pow(x, y) = exp2(y * log2 x); the literal exponents
//     2.0 and 5.0 are strength-reduced to products.
// The CPU oracle (oracle/pt_oracle.c) restates the same contract independently;
// tests/test_gpu_parity.py checks the two are bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_HD __host__ __device__ __forceinline__

namespace pt {

constexpr float kPI = 3.14159f;  // program-raymarch.wgsl:9 (not M_PI)

struct f3 { float x, y, z; };

PT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
PT_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_HD f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
PT_HD f3 operator/(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
PT_HD f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
// dot(a,b): a.x*b.x + a.y*b.y + a.z*b.z contracted left to right
PT_HD float dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// cross(a,b).x = a.y*b.z - a.z*b.y with the first product fused
PT_HD f3 cross(f3 a, f3 b) {
    return f3{fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x))};
}
PT_HD float sum3(f3 a) { return dot(a, f3{1.0f, 1.0f, 1.0f}); }
PT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
PT_HD f3 normalize(f3 a) { return a / length(a); }
// a + b*s contracted
PT_HD f3 madd(f3 a, f3 b, float s) { return f3{fmaf(b.x, s, a.x), fmaf(b.y, s, a.y), fmaf(b.z, s, a.z)}; }
// w_i - 2*dot(w_i, n)*n contracted
PT_HD f3 reflect(f3 wi, f3 n) {
    float k = -(2.0f * dot(wi, n));
    return f3{fmaf(k, n.x, wi.x), fmaf(k, n.y, wi.y), fmaf(k, n.z, wi.z)};
}
PT_HD f3 rcp3(f3 d) { return f3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z}; }

// Wave vote: true when the predicate holds on any active lane.  The ballot intrinsic keeps a
// compare's lane mask in SGPRs (s_and with exec, branch on SCC); HIP's __any materialises the
// bool in a VGPR and compares it again (v_cndmask + v_cmp: two VALU slots per vote).
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// Correctly rounded 1/x without the IEEE division sequence: the hardware reciprocal
// (v_rcp_f32, about 1 ulp) refined by kRcpSteps Newton steps e = 1 - x*y, y += y*e, each an
// exact-residual FMA pair.  Valid for 2^-126 <= |x| <= kRcpHi, where it equals 1.0f / x bit
// for bit — verified on gfx950 over every float of that range (pt_selftest_rcp,
// tests/test_gpu_parity.py); outside it the callers use the division.
constexpr float kRcpHi = 0x1p125f;
constexpr int kRcpSteps = 1;
__device__ __forceinline__ float rcp_rn(float x, int steps = kRcpSteps) {
    float y = __builtin_amdgcn_rcpf(x);
    for (int i = 0; i < steps; ++i) {
        const float e = fmaf(-x, y, 1.0f);
        y = fmaf(e, y, y);
    }
    return y;
}
PT_HD float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

PT_HD float bits_f(uint32_t u) { return __builtin_bit_cast(float, u); }
PT_HD uint32_t f_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

// ---- RNG: hash.wgsl:1-28 -------------------------------------------------
PT_HD uint32_t hmix(uint32_t n) {
    n = (n << 13u) ^ n;
    return n * (n * n * 15731u + 789221u) + 1376312589u;
}
PT_HD uint32_t hash1u(uint32_t n) { return hmix(n) & 0x7fffffffu; }
PT_HD float hash1(uint32_t n) { return 1.0f - (float)(hmix(n) & 0x7fffffffu) * (1.0f / 2147483648.0f); }
PT_HD void hash2(uint32_t n, float& a, float& b) {
    n = hmix(n);
    a = (float)((n * n) & 0x7fffffffu) * (1.0f / 2147483648.0f);
    b = (float)((n * (n * 16807u)) & 0x7fffffffu) * (1.0f / 2147483648.0f);
}

// ---- Cephes sinf/cosf (range-reduced by pi/4 with a 3-part constant) ------
PT_HD void sincos_p(float x, float& s_out, float& c_out) {
    if (__builtin_isnan(x) || __builtin_isinf(x)) { s_out = __builtin_nanf(""); c_out = s_out; return; }
    bool neg = x < 0.0f;
    x = neg ? -x : x;
    int j = (int)(x * 1.27323954473516f);
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
    if (j == 0) { s = S; c = C; }
    else if (j == 2) { s = C; c = -S; }
    else if (j == 4) { s = -S; c = -C; }
    else { s = -C; c = S; }
    s_out = neg ? -s : s;
    c_out = c;
}
PT_HD float tan_p(float x) { float s, c; sincos_p(x, s, c); return s / c; }

// ---- Cephes asinf/acosf ----------------------------------------------------
PT_HD float asin_core(float a) {
    float z = a * a;
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z, 7.4953002686e-2f), z,
                   1.6666752422e-1f);
    return fmaf(p * z, a, a);
}
PT_HD float acos_p(float x) {
    if (!(x >= -1.0f && x <= 1.0f)) return __builtin_nanf("");
    if (x < -0.5f) return 3.14159265358979323846f - 2.0f * asin_core(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_core(sqrtf(0.5f * (1.0f - x)));
    return 1.57079632679489661923f - asin_core(x);
}

// ---- Cephes log2f / exp2f ------------------------------------------------------
PT_HD float log2_p(float x) {
    if (__builtin_isnan(x) || x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -__builtin_inff();
    if (__builtin_isinf(x)) return __builtin_inff();
    int e_adj = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; e_adj = -23; }
    uint32_t b = f_bits(x);
    int e = (int)((b >> 23) & 0xffu) - 126 + e_adj;
    float m = bits_f((b & 0x807fffffu) | 0x3f000000u);
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
    return r + (float)e;
}
PT_HD float exp2_p(float x) {
    if (__builtin_isnan(x)) return x;
    if (x > 127.0f) return __builtin_inff();
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
    if (i0 >= -126) return r * bits_f((uint32_t)(i0 + 127) << 23);
    return (r * bits_f(1u << 23)) * bits_f((uint32_t)(i0 + 126 + 127) << 23);
}
PT_HD float pow_p(float x, float y) {
    if (x < 0.0f || __builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nanf("");
    if (x == 0.0f) return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : __builtin_inff());
    return exp2_p(y * log2_p(x));
}
PT_HD float pow2_lit(float x) { return x * x; }
PT_HD float pow5_lit(float x) { float x2 = x * x; return (x2 * x2) * x; }

}  // namespace pt
