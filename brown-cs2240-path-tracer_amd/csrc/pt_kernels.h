// pt_kernels.h — launch wrappers between the C-ABI layer (pt_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_device.h"

// ids for k_selftest_math (also used by pt_selftest_math in the C-ABI)
enum {
    PT_MATH_SIN = 0, PT_MATH_COS, PT_MATH_TAN, PT_MATH_ACOS, PT_MATH_LOG2, PT_MATH_EXP2, PT_MATH_POW, PT_MATH_SQRT,
    PT_MATH_DIV, PT_MATH_HASH1U, PT_MATH_HASH1, PT_MATH_HASH2X, PT_MATH_HASH2Y, PT_MATH_MIN, PT_MATH_MAX, PT_MATH_COUNT_
};

namespace pt {

constexpr int kMegaBlock = 256;
// dynamic LDS a workgroup may use for traversal stacks + a staged scene copy
constexpr size_t kLdsSceneBudget = 64 * 1024;

// Kernel selection (PT_KERNEL / PT_LDS / PT_TRAV environment overrides for A/B runs).
struct LaunchOpts {
    bool wavefront = false;  // wavefront pipeline (pt_wavefront.hip)
    bool literal = false;  // k_mega: the reference's control flow
    bool lds = true;       // stage the scene in LDS when it fits
    int trav = 3;          // traversal: 0 nested loops, 1 flattened (trav_step), 2 flattened+predicated, 3 lean
};

bool scene_fits_lds(const SceneView& sc);

// Wavefront path state (SoA, HBM), `capacity` paths; see pt_wavefront.hip.
enum { WF_COUNT0 = 0, WF_COUNT1 = 1, WF_CTL_WORDS = 64 };
struct WfBuffers {
    // ray queues (dense, compacted each iteration; ping-pong): entry i = 2 float4
    // (o.xyz, d.x), (d.y, d.z, path index bits, 0)
    float4* rq0;
    float4* rq1;
    int2* hitq;    // per queue entry: (leaf record, t bits)
    float4* st0;   // per path: (L.xyz, beta.x)
    float4* st1;   // per path: (beta.y, beta.z, seed bits, depth | spec << 16)
    float4* sp0;   // per path: (shading point, material id)
    float4* sp1;   // per path: (normal, -)
    float4* sp2;   // per path: (incoming direction, -)
    float* rad;    // per path: radiance when it ended [capacity][3]
    uint32_t* ctl; // queue counts
    uint32_t capacity;
};
constexpr size_t kWfBytesPerPath = 32 * 2 + 8 + 16 * 5 + 12;

hipError_t launch_wavefront(const LaunchOpts& lo, const SceneView& sc, const FrameParams& fp, const WfBuffers& wb,
                            uint32_t frame0, uint32_t nframes, uint32_t stride, bool accum, bool count, float* out,
                            Counters* cnt, hipStream_t stream);

// Megakernel render (accum=true: frames frame0 + i*stride, i < nframes, added to out) or one
// dispatch (accum=false: raw radiance of salt frame0 written to out).
hipError_t launch_megakernel(const LaunchOpts& lo, const SceneView& sc, const FrameParams& fp, uint32_t frame0,
                             uint32_t nframes, uint32_t stride, bool accum, bool count, float* out, Counters* cnt,
                             hipStream_t stream);

hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream);

}  // namespace pt
