// pt_image.hip — on-device display transform.
//
// program-raymarch.ts:295-316 on the accumulator, per pixel, in double like the JS it
// replaces: raw = acc / sample_runs, lum = (r + g + b) / 3, out = raw * (lum / (lum + 1))^0.01,
// u8 = clamp(ToInt32(out * 255)), alpha 255.  The same function as the host pt_tonemap
// (pt_capi.hip); the GPU test checks the two byte for byte.
#include "pt_kernels.h"

#include <algorithm>

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

// The accumulator to pinned host memory (pt_readback_async): a copy by a few blocks, each thread
// storing 16-B words straight over PCIe.  The runtime's own copy of a 12 MB accumulator is a blit
// kernel of 512 blocks that holds its CU slots for the whole PCIe transfer (0.2-1.2 ms in a kernel
// trace of the bench, r06m), beside the next step's render; PCIe is the bound either way.
constexpr int kReadbackBlocks = 16;
__global__ __launch_bounds__(256) void k_readback(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4,
                                                  const float* __restrict__ src_tail, float* __restrict__ dst_tail,
                                                  uint32_t ntail) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += step) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < ntail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}
hipError_t launch_readback(const float* d_src, float* h_dst_dev, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t n4 = n / 4;
    const uint32_t ntail = (uint32_t)(n - 4 * n4);
    hipLaunchKernelGGL(k_readback, dim3(kReadbackBlocks), dim3(256), 0, stream, reinterpret_cast<const float4*>(d_src),
                       reinterpret_cast<float4*>(h_dst_dev), n4, d_src + 4 * n4, h_dst_dev + 4 * n4, ntail);
    return hipGetLastError();
}

// dst += src, f32, element-wise (the ordered multi-device reduction of pt_render_multi: partial
// accumulators added onto device 0's in device order)
__global__ __launch_bounds__(256) void k_accum_add(float4* __restrict__ dst, const float4* __restrict__ src, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 a = dst[i];
        const float4 b = src[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        dst[i] = a;
    }
}
__global__ void k_accum_add_tail(float* __restrict__ dst, const float* __restrict__ src, size_t from, size_t n) {
    const size_t i = from + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

hipError_t launch_accum_add(float* dst, const float* src, size_t n, hipStream_t stream) {
    const size_t n4 = n / 4;
    if (n4) {
        const unsigned blocks = (unsigned)std::min<size_t>((n4 + 255) / 256, 8192);
        hipLaunchKernelGGL(k_accum_add, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<float4*>(dst),
                           reinterpret_cast<const float4*>(src), n4);
    }
    if (n % 4) hipLaunchKernelGGL(k_accum_add_tail, dim3(1), dim3(4), 0, stream, dst, src, n4 * 4, n);
    return hipGetLastError();
}

}  // namespace pt
