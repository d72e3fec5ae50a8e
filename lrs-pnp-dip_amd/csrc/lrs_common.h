// Shared device/host definitions for liblrspnp_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lrspnp.h"

namespace lrs {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; the accumulator
// holds C[4*(l>>4) + i][l&15], i = 0..3 (cdna_hip_programming.md §3).
__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__host__ __device__ constexpr int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace lrs

#define LRS_CHECK_LAUNCH()                                       \
    do {                                                         \
        hipError_t e__ = hipGetLastError();                      \
        if (e__ != hipSuccess) return (int)e__;                  \
    } while (0)
