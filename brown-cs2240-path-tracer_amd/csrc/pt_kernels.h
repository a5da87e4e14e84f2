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

enum class KernelKind { Auto, Literal, Regen, RegenLds };

bool scene_fits_lds(const SceneView& sc);

// Render (accum=true: frames frame0 + i*stride, i < nframes, added to out) or one dispatch
// (accum=false: raw radiance of salt frame0 written to out).
hipError_t launch_render(KernelKind kind, const SceneView& sc, const FrameParams& fp, uint32_t frame0, uint32_t nframes,
                         uint32_t stride, bool accum, bool count, float* out, Counters* cnt, hipStream_t stream);

hipError_t launch_selftest_math(int fn, const float* a, const float* b, float* o, int n, hipStream_t stream);

}  // namespace pt
