// Shared device/host definitions for liblrspnp_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/lrspnp.h"

namespace lrs {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; the accumulator
// holds C[4*(l>>4) + i][l&15], i = 0..3 (cdna_hip_programming.md §3).
__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) applies per device: set it once per device a
// kernel is launched on (bit d of `done` = device d done; devices >= 64 are set on every call).
inline int lds_opt_in(const void *fn, int bytes, std::atomic<uint64_t> &done) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    const uint64_t bit = dev < 64 ? (uint64_t)1 << dev : 0;
    if (bit && (done.load(std::memory_order_relaxed) & bit)) return 0;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return (int)e;
    done.fetch_or(bit, std::memory_order_relaxed);
    return 0;
}

__host__ __device__ constexpr int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// In-launch hand-off of small partials to a "last arriver" workgroup without fences (gfx950: 8
// XCDs with private L2s; MI355X_MICROARCH.md, visibility table row 1): the payload is stored
// write-through (global_store sc1), the storing wave drains it (s_waitcnt vmcnt(0)), ONE lane then
// adds to an agent-scope counter; the workgroup whose add returned count - 1 reads the payload with
// sc1 loads only (they bypass the stale-able L1).  __threadfence() would instead write back the
// whole XCD L2 per workgroup (buffer_wbl2 sc1): 2.6x slower on the DIP loss head.
typedef __attribute__((address_space(1))) unsigned long long lrs_gu64;
typedef __attribute__((address_space(1))) int lrs_gi32;
__device__ __forceinline__ void wt_store(double *p, double v) {
    __hip_atomic_store((lrs_gu64 *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wt_load(const double *p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((lrs_gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ int agent_add(int *p, int v) {
    return __hip_atomic_fetch_add((lrs_gi32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_store(int *p, int v) {
    __hip_atomic_store((lrs_gi32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace lrs

#define LRS_CHECK_LAUNCH()                                       \
    do {                                                         \
        hipError_t e__ = hipGetLastError();                      \
        if (e__ != hipSuccess) return (int)e__;                  \
    } while (0)
