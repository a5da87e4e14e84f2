// pt_image.hip — on-device display transform.
//
// program-raymarch.ts:295-316 on the accumulator, per pixel, in double like the JS it
// replaces: raw = acc / sample_runs, lum = (r + g + b) / 3, out = raw * (lum / (lum + 1))^0.01,
// u8 = clamp(ToInt32(out * 255)), alpha 255.  The same function as the host pt_tonemap
// (pt_capi.hip); the GPU test checks the two byte for byte.
#include "pt_kernels.h"

namespace pt {

__device__ __forceinline__ int32_t to_int32(double v) {  // ECMAScript ToInt32
    if (!isfinite(v)) return 0;
    double m = fmod(trunc(v), 4294967296.0);
    if (m < 0) m += 4294967296.0;
    return (int32_t)(uint32_t)m;
}
__device__ __forceinline__ uint8_t clamp_u8(int32_t v) { return v < 0 ? 0 : (v > 255 ? 255 : (uint8_t)v); }

__global__ __launch_bounds__(256) void k_tonemap(const float* __restrict__ acc, size_t npix, uint32_t runs,
                                                uchar4* __restrict__ rgba) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const double r = (double)acc[3 * i] / runs, g = (double)acc[3 * i + 1] / runs, b = (double)acc[3 * i + 2] / runs;
    const double lum = (r + g + b) / 3.0;
    const double f = pow(lum / (lum + 1.0), 0.01);
    rgba[i] = make_uchar4(clamp_u8(to_int32(r * f * 255.0)), clamp_u8(to_int32(g * f * 255.0)),
                          clamp_u8(to_int32(b * f * 255.0)), 255);
}

hipError_t launch_tonemap(const float* acc, size_t npix, uint32_t runs, uint8_t* rgba, hipStream_t stream) {
    if (npix == 0) return hipSuccess;
    PT_LAUNCH(KID_TONEMAP, stream, k_tonemap, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, acc, npix,
              runs, reinterpret_cast<uchar4*>(rgba));
    return hipGetLastError();
}

}  // namespace pt
