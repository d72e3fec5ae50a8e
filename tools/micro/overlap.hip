// Microbenchmark: can fp64 VALU work overlap MFMA (f32 16x16x4 / bf16 16x16x32) issued by the
// other wave of the same SIMD?  mode: 0 = both, 1 = MFMA waves only, 2 = VALU waves only.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND, int PAIR>   // 0: f32 mfma, 1: bf16 mfma ; VALU side: 2 = fp64 fma, 3 = fp32 fma
__global__ __launch_bounds__(512, 2) void k(float *out, int iters, int mode, int valu_kind) {
    const int w = threadIdx.x >> 6;
    const bool mfma_wave = PAIR ? (w < 4) : ((w & 1) == 0);   // PAIR: waves w, w+4 share a SIMD
    float acc_out = 0.f;
    if (mfma_wave && mode != 2) {
        floatx4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        float a = threadIdx.x * 1e-3f, b = 1.0f + a;
        bf16x8 A8 = {1, 2, 3, 4, 5, 6, 7, (short)threadIdx.x}, B8 = A8;
        for (int i = 0; i < iters; ++i) {
            if (KIND == 0) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
            } else {
                // 2 bf16 MFMAs = same FLOP count as 32 f32 MFMAs... use 8 per iter to keep time comparable
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, c1, 0, 0, 0);
                    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, c2, 0, 0, 0);
                    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A8, B8, c3, 0, 0, 0);
                }
            }
        }
        acc_out = c0[0] + c1[1] + c2[2] + c3[3];
    }
    if (!mfma_wave && mode != 1) {
        if (valu_kind == 2) {
            double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 0.999999;
            for (int i = 0; i < iters * 8; ++i) {
                x0 = __fma_rn(x0, y, 1e-3); x1 = __fma_rn(x1, y, 1e-3);
                x2 = __fma_rn(x2, y, 1e-3); x3 = __fma_rn(x3, y, 1e-3);
            }
            acc_out = (float)(x0 + x1 + x2 + x3);
        } else {
            float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, y = 0.999999f;
            for (int i = 0; i < iters * 8; ++i) {
                x0 = __fmaf_rn(x0, y, 1e-3f); x1 = __fmaf_rn(x1, y, 1e-3f);
                x2 = __fmaf_rn(x2, y, 1e-3f); x3 = __fmaf_rn(x3, y, 1e-3f);
            }
            acc_out = x0 + x1 + x2 + x3;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc_out;
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 512 * 4 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 20000;
    for (int pair = 0; pair < 2; ++pair)
    for (int kind = 0; kind < 2; ++kind)
        for (int vk = 2; vk <= 3; ++vk)
            for (int mode = 0; mode < 3; ++mode) {
                float best = 1e30f;
                for (int rep = 0; rep < 3; ++rep) {
                    hipEventRecord(e0);
                    if (kind == 0 && pair) hipLaunchKernelGGL((k<0, 1>), dim3(256), dim3(512), 0, 0, out, iters, mode, vk);
                    else if (kind == 0) hipLaunchKernelGGL((k<0, 0>), dim3(256), dim3(512), 0, 0, out, iters, mode, vk);
                    else if (pair) hipLaunchKernelGGL((k<1, 1>), dim3(256), dim3(512), 0, 0, out, iters, mode, vk);
                    else hipLaunchKernelGGL((k<1, 0>), dim3(256), dim3(512), 0, 0, out, iters, mode, vk);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                printf("%s mfma=%s valu=%s mode=%s : %.3f ms\n", pair ? "same-SIMD " : "cross-SIMD", kind ? "bf16x32" : "f32x4", vk == 2 ? "f64fma" : "f32fma",
                       mode == 0 ? "both" : (mode == 1 ? "mfma-only" : "valu-only"), best);
            }
    return 0;
}
