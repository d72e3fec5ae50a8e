// DIP low-rank prox primitives: the layers of the 1-Lipschitz U-Net and its training step.
//
// Reference (shuoli0708/LRS-PnP-DIP):
//   models/my_Lipschitz_Unet.py:21-148        the network (conv / bn / act stack)
//   models/lipschitz_constraint_layer.py:6-22   act(): LeakyReLU(0.2, inplace=True)
//   lipschitz_constraint_layer.py:36-44         SpectralNorm._update_u_v: sigma = svd(W.view(Co,-1))[0],
//                                               W = W_bar / max(1, sigma / ln_lambda)
//   lipschitz_constraint_layer.py:65-78         conv(): ReflectionPad2d((k-1)//2) + Conv2d(pad 0)
//   lipschitz_constraint_layer.py:88-101,113-122  BatchNormSpectralNorm: gamma/c, beta/c with
//                                               c = max(max|gamma_orig|, 1) (no grad through c)
//   main_LRS_PnP_DIP_1-LiP.py:214-237           Adam(lr), MSELoss(target*mask, out*mask)
//
// MI355X design: activations are [C][H][W] fp32 (batch 1, as the reference).  A conv is an
// explicit im2col (reflection pad / stride / nearest x2 upsample folded into the gather) and an
// MFMA f32 GEMM; the backward is the same GEMM transposed (dW = dZ col^T with split-K, dcol =
// Wn^T dZ) plus a deterministic col2im gather that also applies the adjoints of the padding and
// the upsample.  BatchNorm (train-mode batch statistics) + LeakyReLU are one kernel per
// direction, one workgroup per channel, statistics in fp64.  sigma_max of every conv weight is
// computed exactly (not by power iteration): fp64 Gram on the smaller side, then Lanczos with
// the Gram held in registers and a 256-way parallel Sturm multisection for the top eigenvalue.
#include <math.h>

#include "lrs_common.h"
#include "lrs_dip.h"

// Kernel definitions; included by dipnet.hip only (one translation unit).
#pragma once

namespace lrs {

// ------------------------------------------------------------------------------------------
// GEMM  C[M][N] = op(A)[M][K] * op(B)[K][N]   (fp32, v_mfma_f32_16x16x4_f32)
//   TA = 0: A stored [M][K];  TA = 1: A stored [K][M]
//   TB = 0: B stored [K][N];  TB = 1: B stored [N][K]
// 128x128 tile per 256-thread workgroup (2x2 waves of 64x64 = 4x4 MFMA tiles), BK = 16.
// Both operands sit in LDS k-contiguous ([x][BK+4] floats), so each lane fetches the four
// k-steps of an MFMA fragment with one ds_read_b128; two LDS stages, one barrier per k-step,
// the next k-step's global loads in flight during the MFMAs.
// gridDim.z > 1 = split-K: partial z goes to Cpart + z*M*N and k_gemm_reduce finishes.
// ------------------------------------------------------------------------------------------
constexpr int kBM = 128, kBN = 128, kBK = 16, kGemmThreads = 256, kLdsK = kBK + 4;

struct GemmArgs {
    const float *A, *B;
    float *C;            // final output (split == 1) or partial base (split > 1)
    const float *bias;   // [M] or null (split == 1 only)
    const float *div;    // scalar divisor (device) or null (split == 1 only)
    int M, N, K, kchunk;
    int accum;           // final C += result instead of C = result
    // k_gemm_s3 only: ncls > 1 output parity classes of an upsampled conv (gridDim.z = ncls x
    // splits; column n of class cls = 2 i + j is source pixel (a, b) = (n / cls_ws, n % cls_ws),
    // stored at output pixel (2a + i) cls_wo + 2b + j of rows of ldc floats)
    int ncls, cls_ws, cls_wo;
    int64_t ldc;         // output row length (0: N)
};

// A 128(x) x 16(k) operand tile, 8 values per thread, as two float4 of 4 consecutive k.
//  KCONTIG: stored [x][k] (k contiguous): thread -> x = t/2, k = 8 (t&1) + 0..7
//  else   : stored [k][x] (x contiguous): thread -> x = t&127, k = 8 (t>>7) + 0..7
template <bool KCONTIG>
__device__ __forceinline__ void load_tile(const float *__restrict__ S, int ld, int k0, int kend, int x0, int X,
                                          float4 (&r)[2]) {
    const int t = threadIdx.x;
    if (KCONTIG) {
        const int x = x0 + (t >> 1), kb = k0 + 8 * (t & 1);
        const float *src = S + (int64_t)x * ld;
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (x < X && kb + u < kend) ? src[kb + u] : 0.0f;
        r[0] = float4{v[0], v[1], v[2], v[3]};
        r[1] = float4{v[4], v[5], v[6], v[7]};
    } else {
        const int x = x0 + (t & 127), kb = k0 + 8 * (t >> 7);
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (x < X && kb + u < kend) ? S[(int64_t)(kb + u) * ld + x] : 0.0f;
        r[0] = float4{v[0], v[1], v[2], v[3]};
        r[1] = float4{v[4], v[5], v[6], v[7]};
    }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(float (*T)[kLdsK], const float4 (&r)[2]) {
    const int t = threadIdx.x;
    const int x = KCONTIG ? (t >> 1) : (t & 127);
    const int kb = KCONTIG ? 8 * (t & 1) : 8 * (t >> 7);
    *reinterpret_cast<float4 *>(&T[x][kb]) = r[0];
    *reinterpret_cast<float4 *>(&T[x][kb + 4]) = r[1];
}

template <int TA, int TB>
__global__ __launch_bounds__(kGemmThreads) void k_gemm(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float As[2][kBM][kLdsK];
    __shared__ __attribute__((aligned(16))) float Bs[2][kBN][kLdsK];
    const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    const int lda = TA ? g.M : g.K;
    const int ldb = TB ? g.K : g.N;
    floatx4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 ra[2], rb[2];
    load_tile<TA == 0>(g.A, lda, kbeg, kend, m0, g.M, ra);
    load_tile<TB == 1>(g.B, ldb, kbeg, kend, n0, g.N, rb);
    int stage = 0;
    store_tile<TA == 0>(As[0], ra);
    store_tile<TB == 1>(Bs[0], rb);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += kBK) {
        const bool more = k0 + kBK < kend;
        if (more) {
            load_tile<TA == 0>(g.A, lda, k0 + kBK, kend, m0, g.M, ra);
            load_tile<TB == 1>(g.B, ldb, k0 + kBK, kend, n0, g.N, rb);
        }
        float4 fa[4], fb[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) fa[a] = *reinterpret_cast<const float4 *>(&As[stage][wm + 16 * a + jl][4 * gk]);
#pragma unroll
        for (int b = 0; b < 4; ++b) fb[b] = *reinterpret_cast<const float4 *>(&Bs[stage][wn + 16 * b + jl][4 * gk]);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[a][b] = mfma16x16x4(fa[a].x, fb[b].x, acc[a][b]);
                acc[a][b] = mfma16x16x4(fa[a].y, fb[b].y, acc[a][b]);
                acc[a][b] = mfma16x16x4(fa[a].z, fb[b].z, acc[a][b]);
                acc[a][b] = mfma16x16x4(fa[a].w, fb[b].w, acc[a][b]);
            }
        if (more) {
            store_tile<TA == 0>(As[stage ^ 1], ra);   // the other stage: last read one step ago
            store_tile<TB == 1>(Bs[stage ^ 1], rb);
        }
        __syncthreads();
        stage ^= 1;
    }
    float *C = g.C + (int64_t)blockIdx.z * g.M * g.N;
    const bool final_out = gridDim.z == 1;
    const float dv = (final_out && g.div) ? *g.div : 1.0f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int n = n0 + wn + 16 * b + jl;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * a + 4 * gk + r;
                if (m < g.M && n < g.N) {
                    float v = acc[a][b][r];
                    if (final_out) {
                        if (g.bias) v = v + g.bias[m];
                        if (g.div) v = v / dv;
                        if (g.accum) v = C[(int64_t)m * g.N + n] + v;
                    }
                    C[(int64_t)m * g.N + n] = v;
                }
            }
        }
}

// ---- split-bf16 variant of the 128x128 GEMM (BK 32) ---------------------------------------------
// Same tiling and pipeline as k_gemm, but the products run on v_mfma_f32_16x16x32_bf16: every fp32
// operand is split exactly into three bf16 terms (hi + mid + lo) when its fragment leaves LDS and
// the six partial products with i + j <= 4 are accumulated in fp32 (the dropped ones are <= 2^-24
// relative: fp32-GEMM accuracy, the ISTA kernel's scheme).  2.7x fewer matrix-core cycles than the
// f32 MFMA for the same tile.
constexpr int kBK32 = 32, kLdsK32 = kBK32 + 4;
typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));

template <bool KCONTIG>
__device__ __forceinline__ void load_tile32(const float *__restrict__ S, int ld, int k0, int kend, int x0, int X,
                                            float4 (&r)[4]) {
    const int t = threadIdx.x;
    float v[16];
    if (KCONTIG) {
        const int x = x0 + (t >> 1), kb = k0 + 16 * (t & 1);
        const float *src = S + (int64_t)x * ld;
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (x < X && kb + u < kend) ? src[kb + u] : 0.0f;
    } else {
        const int x = x0 + (t & 127), kb = k0 + 16 * (t >> 7);
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (x < X && kb + u < kend) ? S[(int64_t)(kb + u) * ld + x] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = float4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}

__device__ __forceinline__ void store_tile32(float (*T)[kLdsK32], const float4 (&r)[4], bool kcontig) {
    const int t = threadIdx.x;
    const int x = kcontig ? (t >> 1) : (t & 127);
    const int kb = kcontig ? 16 * (t & 1) : 16 * (t >> 7);
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<float4 *>(&T[x][kb + 4 * q]) = r[q];
}

__device__ __forceinline__ void gsplit8(const float4 &a, const float4 &b, gbf16x8 (&f)[3]) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 h = (__bf16)v[e];
        const float r1 = v[e] - (float)h;
        const __bf16 m = (__bf16)r1;
        f[0][e] = h;
        f[1][e] = m;
        f[2][e] = (__bf16)(r1 - (float)m);
    }
}

__device__ __forceinline__ floatx4 gmfma6(const gbf16x8 (&A)[3], const gbf16x8 (&B)[3], floatx4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], acc, 0, 0, 0);
    return acc;
}

template <int TA, int TB>
__global__ __launch_bounds__(kGemmThreads) void k_gemm_b3(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float As[2][kBM][kLdsK32];
    __shared__ __attribute__((aligned(16))) float Bs[2][kBN][kLdsK32];
    const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    const int lda = TA ? g.M : g.K;
    const int ldb = TB ? g.K : g.N;
    floatx4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 ra[4], rb[4];
    load_tile32<TA == 0>(g.A, lda, kbeg, kend, m0, g.M, ra);
    load_tile32<TB == 1>(g.B, ldb, kbeg, kend, n0, g.N, rb);
    int stage = 0;
    store_tile32(As[0], ra, TA == 0);
    store_tile32(Bs[0], rb, TB == 1);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += kBK32) {
        const bool more = k0 + kBK32 < kend;
        if (more) {
            load_tile32<TA == 0>(g.A, lda, k0 + kBK32, kend, m0, g.M, ra);
            load_tile32<TB == 1>(g.B, ldb, k0 + kBK32, kend, n0, g.N, rb);
        }
        // fragments: 8 consecutive k (8 gk .. 8 gk + 7) of row / column 16 a + jl
        gbf16x8 fb[4][3];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float *src = &Bs[stage][wn + 16 * b + jl][8 * gk];
            gsplit8(*reinterpret_cast<const float4 *>(src), *reinterpret_cast<const float4 *>(src + 4), fb[b]);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            gbf16x8 fa[3];
            const float *src = &As[stage][wm + 16 * a + jl][8 * gk];
            gsplit8(*reinterpret_cast<const float4 *>(src), *reinterpret_cast<const float4 *>(src + 4), fa);
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = gmfma6(fa, fb[b], acc[a][b]);
        }
        if (more) {
            store_tile32(As[stage ^ 1], ra, TA == 0);   // the other stage: last read one step ago
            store_tile32(Bs[stage ^ 1], rb, TB == 1);
        }
        __syncthreads();
        stage ^= 1;
    }
    float *C = g.C + (int64_t)blockIdx.z * g.M * g.N;
    const bool final_out = gridDim.z == 1;
    const float dv = (final_out && g.div) ? *g.div : 1.0f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int n = n0 + wn + 16 * b + jl;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * a + 4 * gk + r;
                if (m < g.M && n < g.N) {
                    float v = acc[a][b][r];
                    if (final_out) {
                        if (g.bias) v = v + g.bias[m];
                        if (g.div) v = v / dv;
                        if (g.accum) v = C[(int64_t)m * g.N + n] + v;
                    }
                    C[(int64_t)m * g.N + n] = v;
                }
            }
        }
}

// ---- small-tile variant (64x64, BK 16, 2x2 waves of 32x32) for GEMMs whose 128-tile grid is
// too small to fill the chip (the 36x36 native U-Net layers) ----------------------------------
constexpr int kBM64 = 64, kBN64 = 64, kBK64 = 16;

// Load a 16(k) x 64(x) operand tile into 4 registers per thread.
//  kmajor = stored [k][x] (contiguous along x), else stored [x][k] (contiguous along k).
template <bool KMAJOR>
__device__ __forceinline__ void load_tile64(const float *__restrict__ S, int ld, int k0, int kend, int x0, int X,
                                          float (&r)[4]) {
    const int t = threadIdx.x;
    if (KMAJOR) {
        const int kk = t >> 4, i = (t & 15) * 4;
        const int k = k0 + kk;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int x = x0 + i + u;
            r[u] = (k < kend && x < X) ? S[(int64_t)k * ld + x] : 0.0f;
        }
    } else {
        const int i = t >> 2, kk = (t & 3) * 4;
        const int x = x0 + i;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + kk + u;
            r[u] = (k < kend && x < X) ? S[(int64_t)x * ld + k] : 0.0f;
        }
    }
}

template <bool KMAJOR>
__device__ __forceinline__ void store_tile64(float (*T)[kBM64 + 4], const float (&r)[4]) {
    const int t = threadIdx.x;
    if (KMAJOR) {
        const int kk = t >> 4, i = (t & 15) * 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) T[kk][i + u] = r[u];
    } else {
        const int i = t >> 2, kk = (t & 3) * 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) T[kk + u][i] = r[u];
    }
}

template <int TA, int TB>
__global__ __launch_bounds__(kGemmThreads) void k_gemm64(GemmArgs g) {
    __shared__ float As[kBK64][kBM64 + 4];
    __shared__ float Bs[kBK64][kBN64 + 4];
    const int m0 = blockIdx.y * kBM64, n0 = blockIdx.x * kBN64;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 32, wn = (wv & 1) * 32;
    const int jl = lane & 15, gk = lane >> 4;
    // A: TA=0 stored [M][K] -> contiguous along k (x-major); TA=1 stored [K][M] (k-major)
    const int lda = TA ? g.M : g.K;
    const int ldb = TB ? g.K : g.N;
    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    float ra[4], rb[4];
    load_tile64<TA == 1>(g.A, lda, kbeg, kend, m0, g.M, ra);
    load_tile64<TB == 0>(g.B, ldb, kbeg, kend, n0, g.N, rb);
    for (int k0 = kbeg; k0 < kend; k0 += kBK64) {
        store_tile64<TA == 1>(As, ra);
        store_tile64<TB == 0>(Bs, rb);
        __syncthreads();
        if (k0 + kBK64 < kend) {
            load_tile64<TA == 1>(g.A, lda, k0 + kBK64, kend, m0, g.M, ra);
            load_tile64<TB == 0>(g.B, ldb, k0 + kBK64, kend, n0, g.N, rb);
        }
#pragma unroll
        for (int s = 0; s < kBK64 / 4; ++s) {
            const float a0 = As[4 * s + gk][wm + jl], a1 = As[4 * s + gk][wm + 16 + jl];
            const float b0 = Bs[4 * s + gk][wn + jl], b1 = Bs[4 * s + gk][wn + 16 + jl];
            acc[0][0] = mfma16x16x4(a0, b0, acc[0][0]);
            acc[0][1] = mfma16x16x4(a0, b1, acc[0][1]);
            acc[1][0] = mfma16x16x4(a1, b0, acc[1][0]);
            acc[1][1] = mfma16x16x4(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
    float *C = g.C + (int64_t)blockIdx.z * g.M * g.N;
    const bool final_out = gridDim.z == 1;
    const float dv = (final_out && g.div) ? *g.div : 1.0f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int n = n0 + wn + 16 * b + jl;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * a + 4 * gk + r;
                if (m < g.M && n < g.N) {
                    float v = acc[a][b][r];
                    if (final_out) {
                        if (g.bias) v = v + g.bias[m];
                        if (g.div) v = v / dv;
                        if (g.accum) v = C[(int64_t)m * g.N + n] + v;
                    }
                    C[(int64_t)m * g.N + n] = v;
                }
            }
        }
}

// C = (sum_z part[z]) (+ bias[m]) (/ *div): fixed summation order (deterministic); 8 partial
// chains so the loads of a long split stay in flight
__global__ void k_gemm_reduce(const float *__restrict__ part, int nsplit, int M, int N, const float *bias,
                              const float *div, int accum, float *__restrict__ C) {
    const int64_t MN = (int64_t)M * N;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= MN) return;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= nsplit; z += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(z + u) * MN + i];
    for (; z < nsplit; ++z) acc[z & 7] += part[(int64_t)z * MN + i];
    float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    if (bias) s = s + bias[i / N];
    if (div) s = s / *div;
    if (accum) s = C[i] + s;
    C[i] = s;
}

// ------------------------------------------------------------------------------------------
// im2col / col2im with nearest x2 upsample and reflection / zero padding folded in.
//   source x: [C][Hs][Ws];  upsampled (Hu, Wu) = up ? (2Hs, 2Ws) : (Hs, Ws);
//   padded coordinate iy in [0, Hu + 2 pad);  col[(c*k + ky)*k + kx][oy*Wo + ox] =
//   xsrc(c, iy = oy*stride + ky, ix = ox*stride + kx)   (torch weight order [co][ci][ky][kx])
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int reflect_idx(int u, int n) {   // ReflectionPad2d (no edge repeat)
    if (u < 0) u = -u;
    if (u >= n) u = 2 * (n - 1) - u;
    return u;
}

// One col row r = (c, ky, kx) per blockIdx.y (grid-strided), the output pixels of that row across
// blockIdx.x: 32-bit index arithmetic, c / ky / kx uniform per workgroup.
__global__ __launch_bounds__(256) void k_im2col(const float *__restrict__ x, ConvGeom gm, float *__restrict__ col) {
    const int P = gm.Ho * gm.Wo, kk = gm.k * gm.k, Kc = gm.Cin * kk;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int oy = p / gm.Wo, ox = p - oy * gm.Wo;
    for (int r = blockIdx.y; r < Kc; r += gridDim.y) {
        const int c = r / kk, kyx = r - c * kk, ky = kyx / gm.k, kx = kyx - ky * gm.k;
        int uy = oy * gm.stride + ky - gm.pad, ux = ox * gm.stride + kx - gm.pad;
        float v = 0.0f;
        bool inside = true;
        if (gm.pad_mode == LRS_PAD_REFLECT) {
            uy = reflect_idx(uy, gm.Hu);
            ux = reflect_idx(ux, gm.Wu);
        } else {
            inside = uy >= 0 && uy < gm.Hu && ux >= 0 && ux < gm.Wu;
        }
        if (inside) {
            const int sy = gm.up ? (uy >> 1) : uy, sx = gm.up ? (ux >> 1) : ux;
            v = x[((int64_t)c * gm.Hs + sy) * gm.Ws + sx];
        }
        col[(int64_t)r * P + p] = v;
    }
}

// Padded positions that read upsampled index u (n = upsampled extent): the direct one and, for
// reflection, the top/left mirror (u in [1, pad]) and the bottom/right mirror
// (u in [n-1-pad, n-2]); a tiny extent can have all three.
// kPadClamp (internal, pad 1 only): the border index also takes the position just outside it --
// the source-grid form of an upsampled reflection-padded conv (k_gemm_s3's parity classes)
constexpr int kPadClamp = 2;
__device__ __forceinline__ int padded_sources(int u, int n, int pad, int mode, int (&iy)[3]) {
    int cnt = 0;
    iy[cnt++] = u + pad;
    if (mode == LRS_PAD_REFLECT && pad > 0) {
        if (u >= 1 && u <= pad) iy[cnt++] = pad - u;
        if (u >= n - 1 - pad && u <= n - 2) iy[cnt++] = 2 * (n - 1) - u + pad;
    } else if (mode == kPadClamp) {
        if (u == 0) iy[cnt++] = 0;
        if (u == n - 1) iy[cnt++] = n + 1;
    }
    return cnt;
}

// dx[c][y][x] = sum over every col entry that read it (adjoint of k_im2col), gather form.  One
// channel per blockIdx.y (grid-strided), its pixels across blockIdx.x; 32-bit index arithmetic and
// the stride as a template parameter (1 and 2 are the nets' strides).
template <int STRIDE>
__device__ __forceinline__ float col2im_pixel(const float *__restrict__ dcol, const ConvGeom &gm, int c, int sy,
                                              int sx, int P) {
    const int k = gm.k;
    const int s = STRIDE > 0 ? STRIDE : gm.stride;
    float acc = 0.0f;
    const int nup = gm.up ? 2 : 1;
    for (int a = 0; a < nup; ++a) {
        const int uy = gm.up ? 2 * sy + a : sy;
        int iys[3];
        const int ny = padded_sources(uy, gm.Hu, gm.pad, gm.pad_mode, iys);
        for (int b = 0; b < nup; ++b) {
            const int ux = gm.up ? 2 * sx + b : sx;
            int ixs[3];
            const int nx = padded_sources(ux, gm.Wu, gm.pad, gm.pad_mode, ixs);
            for (int py = 0; py < ny; ++py)
                for (int ky = 0; ky < k; ++ky) {
                    const int ty = iys[py] - ky;
                    if (ty < 0 || ty % s) continue;
                    const int oy = ty / s;
                    if (oy >= gm.Ho) continue;
                    for (int px = 0; px < nx; ++px)
                        for (int kx = 0; kx < k; ++kx) {
                            const int tx = ixs[px] - kx;
                            if (tx < 0 || tx % s) continue;
                            const int ox = tx / s;
                            if (ox >= gm.Wo) continue;
                            acc += dcol[(int64_t)((c * k + ky) * k + kx) * P + oy * gm.Wo + ox];
                        }
                }
        }
    }
    return acc;
}

template <int STRIDE>
__global__ __launch_bounds__(256) void k_col2im(const float *__restrict__ dcol, ConvGeom gm, float *__restrict__ dx,
                                                int accum) {
    const int HW = gm.Hs * gm.Ws, P = gm.Ho * gm.Wo;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= HW) return;
    const int sy = q / gm.Ws, sx = q - sy * gm.Ws;
    for (int c = blockIdx.y; c < gm.Cin; c += gridDim.y) {
        const float acc = col2im_pixel<STRIDE>(dcol, gm, c, sy, sx, P);
        const int64_t i = (int64_t)c * HW + q;
        dx[i] = accum ? dx[i] + acc : acc;
    }
}

// ------------------------------------------------------------------------------------------
// Wave / block reductions.  Doubles go through DPP row operations (no LDS crossbar): after four
// steps every 16-lane row holds its row sum, then readlane gathers the four rows.
// ------------------------------------------------------------------------------------------
// (full-row permutations only: every lane reads a lane of its own row, so no 'old' value is needed
// -- mov_dpp instead of update_dpp(0, ...) saves the zeroing of each destination)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// sum over the 64 lanes, result uniform (fixed order: deterministic)
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);   // row_half_mirror
    v += dpp_d<0x140>(v);   // row_mirror
    return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// block sum; red must hold 2 * (blockDim/64) doubles; `parity` alternates between calls so a
// single barrier suffices (the other half of red is still being read by slow waves)
__device__ __forceinline__ double block_sum_d1(double v, double *red, int &parity) {
    const int nw = blockDim.x >> 6;
    v = wave_sum_d(v);
    double *r = red + parity * nw;
    if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += r[i];
    parity ^= 1;
    return s;
}

__device__ __forceinline__ double block_sum_d(double v, double *red) {
    int parity = 0;
    const double s = block_sum_d1(v, red, parity);
    __syncthreads();
    return s;
}

// Two / three block sums behind ONE barrier (red >= 2 / 3 x blockDim / 64 doubles): each sum is
// formed exactly as block_sum_d1 forms it (wave sums, then the waves' values in wave order from
// 0.0), so the results are bitwise those of consecutive block_sum_d1 calls; every thread gets them.
__device__ __forceinline__ void block_sum2_d(double &a, double &b, double *red) {
    const int nw = blockDim.x >> 6, w = threadIdx.x >> 6;
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    if ((threadIdx.x & 63) == 0) {
        red[w] = a;
        red[nw + w] = b;
    }
    __syncthreads();
    double s0 = 0.0, s1 = 0.0;
    for (int i = 0; i < nw; ++i) {
        s0 += red[i];
        s1 += red[nw + i];
    }
    a = s0;
    b = s1;
}

__device__ __forceinline__ void block_sum3_d(double &a, double &b, double &c, double *red) {
    const int nw = blockDim.x >> 6, w = threadIdx.x >> 6;
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    c = wave_sum_d(c);
    if ((threadIdx.x & 63) == 0) {
        red[w] = a;
        red[nw + w] = b;
        red[2 * nw + w] = c;
    }
    __syncthreads();
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < nw; ++i) {
        s0 += red[i];
        s1 += red[nw + i];
        s2 += red[2 * nw + i];
    }
    a = s0;
    b = s1;
    c = s2;
}

// ------------------------------------------------------------------------------------------
// BatchNorm2d (train mode, batch 1) with the Lipschitz rescale, + activation.
// Each channel is split over S workgroups (grid = S x C).  Statistics: per-workgroup fp64
// partials, the last workgroup of a channel (atomic ticket, fixed summation order) finalises.
// Forward = k_bn_stats + k_bn_apply; backward = k_bn_bwd_stats + k_bn_bwd_apply.
// ------------------------------------------------------------------------------------------
constexpr int kBnThreads = 256;
constexpr int kBn1Threads = 1024;   // one workgroup per channel (S == 1): 16 waves share the channel
// ... and on small maps (P <= 4 * kBn1Small: the 25^2 and smaller maps at 196^2, 18^2 and smaller at
// 36^2), where 1024 threads would leave most lanes idle, 256 threads (bn1_threads, dipnet.hip)
constexpr int kBn1Small = 256;

// element i of a [C][P] tensor summed over nsplit split-K partials (stride MN): acc[e] = the splits
// e, e + 8, ... in increasing order (k_gemm_reduce's order), the loads of one group of 8 predicated.
// (Every load of up to 32 splits issued before the first add measured slower: 36^2 step 0.635 ->
// 0.671 ms, 196^2 1.244 -> 1.272, tuning build, 2 interleaved rounds.)
__device__ __forceinline__ float splitk_sum1(const float *__restrict__ part, int nsplit, int64_t MN, int64_t i) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int z0 = 0; z0 < nsplit; z0 += 8) {
        float p[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) p[e] = z0 + e < nsplit ? part[(int64_t)(z0 + e) * MN + i] : 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (z0 + e < nsplit) acc[e] += p[e];
    }
    return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// c = max(max|gamma_orig|, 1.0) (lipschitz_constraint_layer.py:93-97); whole block, C <= 4 * blockDim
__device__ float bn_lip_scale(const float *gamma, int C, float *redf) {
    float m = 0.0f;
    for (int i = threadIdx.x; i < C; i += blockDim.x) m = fmaxf(m, fabsf(gamma[i]));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) redf[threadIdx.x >> 6] = m;
    __syncthreads();
    float r = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, redf[i]);
    return fmaxf(r, 1.0f);
}

// The same scale computed by every wave on its own (no barrier): the maximum of the same set of
// |gamma|, so bitwise bn_lip_scale's value
__device__ __forceinline__ float bn_lip_scale_w(const float *gamma, int C) {
    float m = 0.0f;
    for (int i = threadIdx.x & 63; i < C; i += 64) m = fmaxf(m, fabsf(gamma[i]));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    return fmaxf(m, 1.0f);
}


__device__ __forceinline__ float act_fwd(float v, int act) {
    if (act == LRS_ACT_LRELU) return v > 0.0f ? v : v * 0.2f;
    if (act == LRS_ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
    return v;
}

__device__ __forceinline__ float act_bwd(float g, float y, int act) {
    if (act == LRS_ACT_LRELU) return y > 0.0f ? g : g * 0.2f;
    if (act == LRS_ACT_SIGMOID) return g * (1.0f - y) * y;
    return g;
}

struct BnArgs {
    const float *z;              // [C][P] conv output
    float *y;                    // [C][P] activation output (may alias z when !bn)
    const float *gamma, *beta;   // bn params (orig), null when !bn
    float *mean, *invstd;        // [C] saved statistics
    float *run_mean, *run_var;   // [C] running statistics (momentum update), nullable
    double *part;                // [C][S][3] partials
    int C, P, S, chunk, bn, act;
    float eps, momentum;
    int lip;                     // BatchNormSpectralNorm rescale (1-Lip) or plain BatchNorm2d
    int vec;                     // float4 path: P, chunk multiples of 4, tensors 16-B aligned
};

// The forward statistics every thread derives from the block sums (thread 0 also stores them):
// the arithmetic k_bn_fwd1's thread 0 used, so bitwise the same mean / invstd
__device__ __forceinline__ void bn_fwd_finish(const BnArgs &a, int c, double K, double s1, double s2, float &m32,
                                              float &is32) {
    const double m = s1 / a.P;
    double var = s2 / a.P - m * m;
    if (var < 0.0) var = 0.0;
    m32 = (float)(K + m);
    is32 = (float)(1.0 / sqrt(var + (double)a.eps));
    if (threadIdx.x == 0) {
        a.mean[c] = m32;
        a.invstd[c] = is32;
        if (a.run_mean) {
            const double unb = a.P > 1 ? var * a.P / (a.P - 1) : var;
            a.run_mean[c] = (1.0f - a.momentum) * a.run_mean[c] + a.momentum * m32;
            a.run_var[c] = (1.0f - a.momentum) * a.run_var[c] + a.momentum * (float)unb;
        }
    }
}

// partial sums of (z - K), (z - K)^2 over this workgroup's slice, K = z[c][0] (stable variance);
// block-reduced (valid in every thread), both sums behind one barrier
__device__ __forceinline__ void bn_stats_body(const BnArgs &a, int c, int sb, double &s1, double &s2, double *red) {
    const float *z = a.z + (int64_t)c * a.P;
    const int i0 = sb * a.chunk, i1 = min(a.P, i0 + a.chunk);
    const double K = (double)z[0];
    s1 = 0.0;
    s2 = 0.0;
    if (a.vec) {   // one float4 per lane per pass: 16-B loads, 4x the bytes in flight
        const float4 *z4 = reinterpret_cast<const float4 *>(z);
        for (int q = (i0 >> 2) + threadIdx.x; q < (i1 >> 2); q += blockDim.x) {
            const float4 v = z4[q];
            const double d0 = (double)v.x - K, d1 = (double)v.y - K, d2 = (double)v.z - K, d3 = (double)v.w - K;
            s1 += d0; s2 += d0 * d0;
            s1 += d1; s2 += d1 * d1;
            s1 += d2; s2 += d2 * d2;
            s1 += d3; s2 += d3 * d3;
        }
    } else {
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
            const double d = (double)z[i] - K;
            s1 += d;
            s2 += d * d;
        }
    }
    block_sum2_d(s1, s2, red);
}

__global__ __launch_bounds__(kBnThreads) void k_bn_stats(BnArgs a) {
    __shared__ double red[2 * kBnThreads / 64];
    const int c = blockIdx.y, sb = blockIdx.x;
    double s1, s2;
    bn_stats_body(a, c, sb, s1, s2, red);
    if (threadIdx.x == 0) {
        double *pp = a.part + ((int64_t)c * a.S + sb) * 3;
        pp[0] = s1;
        pp[1] = s2;
    }
}

// normalise + affine + activation of this workgroup's slice; t1, t2 = the channel's summed
// partials (read by thread 0 only).  ONE (k_bn_fwd1): t1, t2 valid in every thread, which then all
// form the statistics themselves (thread 0's arithmetic) and the Lipschitz scale per wave: no barrier
template <bool ONE = false>
__device__ __forceinline__ void bn_apply_body(const BnArgs &a, int c, int sb, double t1, double t2, float *redf,
                                              float *st_s) {
    const int64_t off = (int64_t)c * a.P;
    const float *z = a.z + off;
    float *y = a.y + off;
    const int i0 = sb * a.chunk, i1 = min(a.P, i0 + a.chunk);
    float cs, m32, is32;
    if constexpr (ONE) {
        cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
        bn_fwd_finish(a, c, (double)a.z[off], t1, t2, m32, is32);
    } else {
        cs = a.lip ? bn_lip_scale(a.gamma, a.C, redf) : 1.0f;
        if (threadIdx.x == 0) {
            const double m = t1 / a.P;
            double var = t2 / a.P - m * m;
            if (var < 0.0) var = 0.0;
            const float m32 = (float)((double)a.z[off] + m);
            const float is32 = (float)(1.0 / sqrt(var + (double)a.eps));
            st_s[0] = m32;
            st_s[1] = is32;
            if (sb == 0) {
                a.mean[c] = m32;
                a.invstd[c] = is32;
                if (a.run_mean) {
                    const double unb = a.P > 1 ? var * a.P / (a.P - 1) : var;
                    a.run_mean[c] = (1.0f - a.momentum) * a.run_mean[c] + a.momentum * m32;
                    a.run_var[c] = (1.0f - a.momentum) * a.run_var[c] + a.momentum * (float)unb;
                }
            }
        }
        __syncthreads();
        m32 = st_s[0];
        is32 = st_s[1];
    }
    const float gm = a.gamma[c] / cs, bt = a.beta[c] / cs;
    if (a.vec) {
        const float4 *z4 = reinterpret_cast<const float4 *>(z);
        float4 *y4 = reinterpret_cast<float4 *>(y);
        for (int q = (i0 >> 2) + threadIdx.x; q < (i1 >> 2); q += blockDim.x) {
            const float4 v = z4[q];
            y4[q] = make_float4(act_fwd((v.x - m32) * is32 * gm + bt, a.act), act_fwd((v.y - m32) * is32 * gm + bt, a.act),
                                act_fwd((v.z - m32) * is32 * gm + bt, a.act), act_fwd((v.w - m32) * is32 * gm + bt, a.act));
        }
        return;
    }
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) y[i] = act_fwd((z[i] - m32) * is32 * gm + bt, a.act);
}

__global__ __launch_bounds__(kBnThreads) void k_bn_apply(BnArgs a) {
    __shared__ float redf[kBnThreads / 64];
    __shared__ float st_s[2];
    const int c = blockIdx.y, sb = blockIdx.x;
    if (!a.bn) {
        const int64_t off = (int64_t)c * a.P;
        const int i0 = sb * a.chunk, i1 = min(a.P, i0 + a.chunk);
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) a.y[off + i] = act_fwd(a.z[off + i], a.act);
        return;
    }
    double t1 = 0.0, t2 = 0.0;
    if (threadIdx.x == 0) {
        const double *q = a.part + (int64_t)c * a.S * 3;
        for (int j = 0; j < a.S; ++j) { t1 += q[3 * j]; t2 += q[3 * j + 1]; }
    }
    bn_apply_body(a, c, sb, t1, t2, redf, st_s);
}

// S == 1 (a channel fits one workgroup): statistics and apply in one launch, the same
// arithmetic as k_bn_stats + k_bn_apply (0 + the single partial)
__global__ __launch_bounds__(kBn1Threads) void k_bn_fwd1(BnArgs a) {
    __shared__ double red[2 * kBn1Threads / 64];
    __shared__ float redf[kBn1Threads / 64];
    __shared__ float st_s[2];
    const int c = blockIdx.y;
    double s1, s2;
    bn_stats_body(a, c, 0, s1, s2, red);
    bn_apply_body<true>(a, c, 0, 0.0 + s1, 0.0 + s2, redf, st_s);
}

// Split-K finish + BatchNorm(+act) of one channel in one launch (a channel fits one workgroup:
// P <= 4 * kBn1Threads): z = sum of the GEMM's split-K partials (k_gemm_reduce's order) + bias,
// stored for the backward, then k_bn_fwd1's statistics / normalisation / activation from the
// values held in registers.  Replaces k_gemm_reduce + k_bn_fwd1 for the small-map convs.
template <int TH = kBn1Threads>
__global__ __launch_bounds__(TH) void k_reduce_bn1(const float *__restrict__ part, int nsplit,
                                                   const float *__restrict__ bias, BnArgs a,
                                                   const float *__restrict__ sdiv = nullptr) {
    __shared__ double red[2 * TH / 64];
    const int c = blockIdx.y, t = threadIdx.x;
    const int64_t MN = (int64_t)a.C * a.P, off = (int64_t)c * a.P;
    auto zsum = [&](int i) {   // sdiv: as k_bn_fwd_r (raw-weight conv)
        float v = splitk_sum1(part, nsplit, MN, off + i);
        if (sdiv) v = v / *sdiv;
        if (bias) v = v + bias[c];
        return v;
    };
    const float cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    float zv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = t + u * TH;
        zv[u] = 0.0f;
        if (i >= a.P) continue;
        zv[u] = zsum(i);
        const_cast<float *>(a.z)[off + i] = zv[u];
    }
    // K = z[c][0], formed again by every thread (the same sum, so the same value) instead of being
    // broadcast from thread 0 behind a barrier
    const double K = (double)zsum(0);
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (t + u * TH < a.P) {
            const double d = (double)zv[u] - K;
            s1 += d;
            s2 += d * d;
        }
    block_sum2_d(s1, s2, red);   // the only barrier
    float m32, is32;
    bn_fwd_finish(a, c, K, s1, s2, m32, is32);
    const float gm = a.gamma[c] / cs, bt = a.beta[c] / cs;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = t + u * TH;
        if (i < a.P) a.y[off + i] = act_fwd((zv[u] - m32) * is32 * gm + bt, a.act);
    }
}

struct BnBwdArgs {
    const float *gy;             // [C][P] dL/dy
    const float *y, *z;          // activation output, conv output
    const float *gamma;          // bn gamma_orig (null when !bn)
    const float *mean, *invstd;
    float *gz;                   // [C][P] dL/dz (may alias gy)
    float *ggamma, *gbeta;       // [C] grads of gamma_orig / beta_orig (null when !bn)
    float *gbias;                // [C] grad of the conv bias = sum_p dL/dz
    double *part;                // [C][S][3] partials
    int C, P, S, chunk, bn, act;
    int lip;                     // BatchNormSpectralNorm rescale (1-Lip) or plain BatchNorm2d
    int accum;                   // gz += instead of gz =
    int vec;                     // float4 path: P, chunk multiples of 4, tensors 16-B aligned
    const float *beta;           // bn beta_orig: with it the LeakyReLU branch is taken from z (bn_act_bwd)
};

// dL/d(pre-activation) of a BN node: for LeakyReLU the branch is decided on pre = x_hat gm + bt, the
// forward's own arithmetic ((z - m) is) gm + bt, so y need not be read (same decisions bitwise: y > 0
// iff pre > 0); a Sigmoid (or no beta) takes y.
__device__ __forceinline__ bool bn_needs_y(const BnBwdArgs &a) { return a.act == LRS_ACT_SIGMOID || !a.beta; }
__device__ __forceinline__ float bn_act_bwd(float g, float xh, float gm, float bt, float y, const BnBwdArgs &a) {
    if (a.act == LRS_ACT_LRELU && a.beta) {
        const float pre = xh * gm + bt;
        return pre > 0.0f ? g : g * 0.2f;
    }
    return act_bwd(g, y, a.act);
}

// redf: the Lipschitz scale's reduction scratch (kBn*Threads / 64 floats); with beta the LeakyReLU
// branch comes from the pre-activation (bn_act_bwd), so y is not read.  The three sums behind one
// barrier (red >= 3 x blockDim / 64 doubles); ONE (k_bn_bwd1): the scale per wave (no barrier)
template <bool ONE = false>
__device__ __forceinline__ void bn_bwd_stats_body(const BnBwdArgs &a, int c, int sb, double (&o)[3], double *red,
                                                  float *redf) {
    const int64_t off = (int64_t)c * a.P;
    const float *gy = a.gy + off, *y = a.y + off, *z = a.z + off;
    const int i0 = sb * a.chunk, i1 = min(a.P, i0 + a.chunk);
    double sg = 0.0, sgx = 0.0, sx = 0.0;
    const bool ldy = bn_needs_y(a);
    float gm = 0.0f, bt = 0.0f;
    if (a.bn && !ldy) {
        float cs = 1.0f;
        if constexpr (ONE) cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
        else cs = a.lip ? bn_lip_scale(a.gamma, a.C, redf) : 1.0f;
        gm = a.gamma[c] / cs;
        bt = a.beta[c] / cs;
    }
    if (a.bn && a.vec) {
        const float m32 = a.mean[c], is32 = a.invstd[c];
        const float4 *gy4 = reinterpret_cast<const float4 *>(gy), *y4 = reinterpret_cast<const float4 *>(y),
                     *z4 = reinterpret_cast<const float4 *>(z);
        for (int q = (i0 >> 2) + threadIdx.x; q < (i1 >> 2); q += blockDim.x) {
            const float4 gv = gy4[q], zv = z4[q];
            const float4 yv = ldy ? y4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float ge[4] = {gv.x, gv.y, gv.z, gv.w}, ye[4] = {yv.x, yv.y, yv.z, yv.w},
                        ze[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float xh = (ze[e] - m32) * is32;
                const float g = ldy ? act_bwd(ge[e], ye[e], a.act) : bn_act_bwd(ge[e], xh, gm, bt, 0.0f, a);
                sg += (double)g;
                sgx += (double)g * (double)xh;
                sx += (double)xh;
            }
        }
    } else if (a.bn) {
        const float m32 = a.mean[c], is32 = a.invstd[c];
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
            const float xh = (z[i] - m32) * is32;
            const float g = ldy ? act_bwd(gy[i], y[i], a.act) : bn_act_bwd(gy[i], xh, gm, bt, 0.0f, a);
            sg += (double)g;
            sgx += (double)g * (double)xh;
            sx += (double)xh;
        }
    } else {
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) sg += (double)act_bwd(gy[i], y[i], a.act);
    }
    block_sum3_d(sg, sgx, sx, red);
    o[0] = sg;
    o[1] = sgx;
    o[2] = sx;
}

__global__ __launch_bounds__(kBnThreads) void k_bn_bwd_stats(BnBwdArgs a) {
    __shared__ double red[3 * kBnThreads / 64];
    __shared__ float redf[kBnThreads / 64];
    const int c = blockIdx.y, sb = blockIdx.x;
    double o[3];
    bn_bwd_stats_body(a, c, sb, o, red, redf);
    if (threadIdx.x == 0) {
        double *pp = a.part + ((int64_t)c * a.S + sb) * 3;
        pp[0] = o[0];
        pp[1] = o[1];
        pp[2] = o[2];
    }
}

// t = the channel's summed partials (read by thread 0 only).  ONE (k_bn_bwd1): t valid in every
// thread, which then all form mean(g), mean(g x_hat) themselves and the scale per wave: no barrier
template <bool ONE = false>
__device__ __forceinline__ void bn_bwd_apply_body(const BnBwdArgs &a, int c, int sb, const double (&t)[3],
                                                  float *redf, float *st_s) {
    const int64_t off = (int64_t)c * a.P;
    const float *gy = a.gy + off, *y = a.y + off, *z = a.z + off;
    float *gz = a.gz + off;
    const int i0 = sb * a.chunk, i1 = min(a.P, i0 + a.chunk);
    if (!a.bn) {
        if (threadIdx.x == 0 && sb == 0 && a.gbias) a.gbias[c] = (float)t[0];
        for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
            const float v = act_bwd(gy[i], y[i], a.act);
            gz[i] = a.accum ? gz[i] + v : v;
        }
        return;
    }
    float cs = 1.0f;
    if constexpr (ONE) cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    else cs = a.lip ? bn_lip_scale(a.gamma, a.C, redf) : 1.0f;
    const float m32 = a.mean[c], is32 = a.invstd[c];
    const float gm = a.gamma[c] / cs;
    const float k = gm * is32;
    const bool ldy = bn_needs_y(a);
    const float bt = ldy ? 0.0f : a.beta[c] / cs;
    float mg, mgx;
    if (ONE || threadIdx.x == 0) {
        mg = (float)(t[0] / a.P);
        mgx = (float)(t[1] / a.P);
        if (!ONE) {
            st_s[0] = mg;
            st_s[1] = mgx;
        }
        if (threadIdx.x == 0 && sb == 0) {
            a.ggamma[c] = (float)t[1] / cs;
            a.gbeta[c] = (float)t[0] / cs;
            // conv bias grad = sum_p gz = k (sg - P mg - mgx sum_p xhat)  (zero in exact arithmetic)
            if (a.gbias) a.gbias[c] = (float)((double)k * (t[0] - (double)a.P * mg - (double)mgx * t[2]));
        }
    }
    if constexpr (!ONE) {
        __syncthreads();
        mg = st_s[0];
        mgx = st_s[1];
    }
    if (a.vec) {
        const float4 *gy4 = reinterpret_cast<const float4 *>(gy), *y4 = reinterpret_cast<const float4 *>(y),
                     *z4 = reinterpret_cast<const float4 *>(z);
        float4 *gz4 = reinterpret_cast<float4 *>(gz);
        for (int q = (i0 >> 2) + threadIdx.x; q < (i1 >> 2); q += blockDim.x) {
            const float4 gv = gy4[q], zv = z4[q];
            const float4 yv = ldy ? y4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float ge[4] = {gv.x, gv.y, gv.z, gv.w}, ye[4] = {yv.x, yv.y, yv.z, yv.w},
                        ze[4] = {zv.x, zv.y, zv.z, zv.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float xh = (ze[e] - m32) * is32;
                const float g = ldy ? act_bwd(ge[e], ye[e], a.act) : bn_act_bwd(ge[e], xh, gm, bt, 0.0f, a);
                o[e] = k * (g - mg - xh * mgx);
            }
            float4 r = make_float4(o[0], o[1], o[2], o[3]);
            if (a.accum) {
                const float4 pv = gz4[q];
                r = make_float4(pv.x + r.x, pv.y + r.y, pv.z + r.z, pv.w + r.w);
            }
            gz4[q] = r;
        }
        return;
    }
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const float xh = (z[i] - m32) * is32;
        const float g = ldy ? act_bwd(gy[i], y[i], a.act) : bn_act_bwd(gy[i], xh, gm, bt, 0.0f, a);
        const float v = k * (g - mg - xh * mgx);
        gz[i] = a.accum ? gz[i] + v : v;
    }
}

__global__ __launch_bounds__(kBnThreads) void k_bn_bwd_apply(BnBwdArgs a) {
    __shared__ float redf[kBnThreads / 64];
    __shared__ float st_s[2];
    const int c = blockIdx.y, sb = blockIdx.x;
    double t[3] = {0.0, 0.0, 0.0};
    if (threadIdx.x == 0 && (a.bn || (sb == 0 && a.gbias))) {
        const double *q = a.part + (int64_t)c * a.S * 3;
        for (int j = 0; j < a.S; ++j)
            for (int e = 0; e < 3; ++e) t[e] += q[3 * j + e];
    }
    bn_bwd_apply_body(a, c, sb, t, redf, st_s);
}

// S == 1: statistics and apply in one launch (same arithmetic as the two-kernel path)
__global__ __launch_bounds__(kBn1Threads) void k_bn_bwd1(BnBwdArgs a) {
    __shared__ double red[3 * kBn1Threads / 64];
    __shared__ float redf[kBn1Threads / 64];
    __shared__ float st_s[2];
    const int c = blockIdx.y;
    double o[3];
    bn_bwd_stats_body<true>(a, c, 0, o, red, redf);
    const double t[3] = {0.0 + o[0], 0.0 + o[1], 0.0 + o[2]};
    bn_bwd_apply_body<true>(a, c, 0, t, redf, st_s);
}

// ---- one workgroup per channel, the channel held in registers (P <= 4096 NQ, float4 path) ----
// For the mid-size maps (98^2, 196^2 in configs[2]) the two-launch S-way split (statistics, then
// apply, each re-reading the channel) costs more than one 1024-thread workgroup per channel that
// reads every value once: thread t holds the float4 quads t + 1024 u, u < NQ.  The statistics are
// the same fp64 shifted sums (K = z[c][0]) as k_bn_stats / k_bn_bwd_stats; only their summation
// order differs.
constexpr int kBnRegMaxQ = 10;   // 40960 pixels

template <int NQ>
__device__ __forceinline__ bool bnr_ok(int P, int u) { return threadIdx.x + u * kBn1Threads < (unsigned)(P >> 2); }
template <int TH>
__device__ __forceinline__ bool bnr_ok_t(int P, int u) { return threadIdx.x + u * TH < (unsigned)(P >> 2); }

// quad q of a [C][P] tensor at channel offset off, summed over nsplit split-K partials (stride MN):
// acc[e] = the splits e, e + 8, ... in increasing order (k_gemm_reduce's order); the loads of one
// group of 8 are predicated, not indexed, so acc stays in registers
__device__ __forceinline__ float4 splitk_sum4(const float *__restrict__ part, int nsplit, int64_t MN, int64_t off, int q) {
    float4 acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z0 = 0; z0 < nsplit; z0 += 8) {
        float4 p[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
            p[e] = z0 + e < nsplit ? reinterpret_cast<const float4 *>(part + (int64_t)(z0 + e) * MN + off)[q]
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (z0 + e < nsplit) {
                acc[e].x += p[e].x; acc[e].y += p[e].y; acc[e].z += p[e].z; acc[e].w += p[e].w;
            }
    }
    float4 v;
    v.x = ((acc[0].x + acc[1].x) + (acc[2].x + acc[3].x)) + ((acc[4].x + acc[5].x) + (acc[6].x + acc[7].x));
    v.y = ((acc[0].y + acc[1].y) + (acc[2].y + acc[3].y)) + ((acc[4].y + acc[5].y) + (acc[6].y + acc[7].y));
    v.z = ((acc[0].z + acc[1].z) + (acc[2].z + acc[3].z)) + ((acc[4].z + acc[5].z) + (acc[6].z + acc[7].z));
    v.w = ((acc[0].w + acc[1].w) + (acc[2].w + acc[3].w)) + ((acc[4].w + acc[5].w) + (acc[6].w + acc[7].w));
    return v;
}

// forward: z = (split-K partials summed in k_gemm_reduce's order + bias) or z as stored; then
// BN statistics, normalisation, affine (Lipschitz rescale), activation.  part == nullptr: z given.
// TH = threads per workgroup (quads t + TH u): 1024 by default; 256 (4 wave slots instead of 16) lets a
// 98^2 map's workgroup fit where one sparse-coding workgroup retires (tuning build, LRS_DIP_BNR_SMALL_WG)
// sdiv (nullable): the conv ran on the raw weights W_bar (the spectral-norm scale not yet known when
// it was launched, dipnet_step's overlapped sigma): z = sum / scale + bias, the same order as the
// scaled path's epilogue (W / scale) x + bias up to the rounding of the quotient's place.
template <int NQ, int TH = kBn1Threads>
__global__ __launch_bounds__(TH) void k_bn_fwd_r(const float *__restrict__ part, int nsplit,
                                                 const float *__restrict__ bias, BnArgs a,
                                                 const float *__restrict__ sdiv = nullptr) {
    __shared__ double red[2 * kBn1Threads / 64];
    const int c = blockIdx.y, t = threadIdx.x;
    const int64_t MN = (int64_t)a.C * a.P, off = (int64_t)c * a.P;
    const float cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    float4 zv[NQ];
    float4 *z4 = reinterpret_cast<float4 *>(const_cast<float *>(a.z) + off);
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
        zv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!bnr_ok_t<TH>(a.P, u)) continue;
        const int q = t + u * TH;
        if (!part) {
            zv[u] = z4[q];
            continue;
        }
        // acc[e] = the splits e, e + 8, ... in increasing order (k_gemm_reduce's order); the loads of
        // one group of 8 are predicated, not indexed, so acc stays in registers
        float4 v = splitk_sum4(part, nsplit, MN, off, q);
        if (sdiv) {
            const float sc = *sdiv;
            v.x = v.x / sc; v.y = v.y / sc; v.z = v.z / sc; v.w = v.w / sc;
        }
        if (bias) {
            const float b = bias[c];
            v.x = v.x + b; v.y = v.y + b; v.z = v.z + b; v.w = v.w + b;
        }
        zv[u] = v;
        z4[q] = v;
    }
    // K = z[c][0] (thread 0's first value), formed again by every thread: no broadcast barrier
    float k0;
    if (part) {
        k0 = splitk_sum4(part, nsplit, MN, off, 0).x;
        if (sdiv) k0 = k0 / *sdiv;
        if (bias) k0 = k0 + bias[c];
    } else {
        k0 = z4[0].x;
    }
    const double K = (double)k0;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int u = 0; u < NQ; ++u)
        if (bnr_ok_t<TH>(a.P, u)) {
            const double d0 = (double)zv[u].x - K, d1 = (double)zv[u].y - K, d2 = (double)zv[u].z - K,
                         d3 = (double)zv[u].w - K;
            s1 += d0; s2 += d0 * d0;
            s1 += d1; s2 += d1 * d1;
            s1 += d2; s2 += d2 * d2;
            s1 += d3; s2 += d3 * d3;
        }
    block_sum2_d(s1, s2, red);   // the only barrier
    float m32, is32;
    bn_fwd_finish(a, c, K, s1, s2, m32, is32);
    const float gm = a.gamma[c] / cs, bt = a.beta[c] / cs;
    float4 *y4 = reinterpret_cast<float4 *>(a.y + off);
#pragma unroll
    for (int u = 0; u < NQ; ++u)
        if (bnr_ok_t<TH>(a.P, u)) {
            const float4 v = zv[u];
            y4[t + u * TH] =
                make_float4(act_fwd((v.x - m32) * is32 * gm + bt, a.act), act_fwd((v.y - m32) * is32 * gm + bt, a.act),
                            act_fwd((v.z - m32) * is32 * gm + bt, a.act), act_fwd((v.w - m32) * is32 * gm + bt, a.act));
        }
}

// Split-K finish + BatchNorm(+act) backward of one channel in one launch (P <= 4096: four values per
// thread, any P): dL/dy = the sum of the data-gradient GEMM's split-K partials (k_gemm_reduce's
// order; dL/dy itself is not stored: only this kernel reads it), then k_bn_bwd_r's arithmetic.
// Replaces k_gemm_reduce + k_bn_bwd1 below a small-map conv's data gradient.
template <int TH = kBn1Threads>
__global__ __launch_bounds__(TH) void k_reduce_bn_bwd1(const float *__restrict__ part, int nsplit, BnBwdArgs a) {
    __shared__ double red[3 * TH / 64];
    const int c = blockIdx.y, t = threadIdx.x;
    const int64_t MN = (int64_t)a.C * a.P, off = (int64_t)c * a.P;
    const float m32 = a.mean[c], is32 = a.invstd[c];
    const float cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    const float gm = a.gamma[c] / cs, bt = a.beta ? a.beta[c] / cs : 0.0f;
    const bool ldy = bn_needs_y(a);
    float g[4], xh[4];
    double sg = 0.0, sgx = 0.0, sx = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = t + u * TH;
        g[u] = xh[u] = 0.0f;
        if (i >= a.P) continue;
        const float gy = splitk_sum1(part, nsplit, MN, off + i);
        xh[u] = (a.z[off + i] - m32) * is32;
        g[u] = bn_act_bwd(gy, xh[u], gm, bt, ldy ? a.y[off + i] : 0.0f, a);
        sg += (double)g[u];
        sgx += (double)g[u] * (double)xh[u];
        sx += (double)xh[u];
    }
    block_sum3_d(sg, sgx, sx, red);   // the only barrier
    const float k = gm * is32;
    const float mg = (float)(sg / a.P), mgx = (float)(sgx / a.P);
    if (t == 0) {
        a.ggamma[c] = (float)sgx / cs;
        a.gbeta[c] = (float)sg / cs;
        if (a.gbias) a.gbias[c] = (float)((double)k * (sg - (double)a.P * mg - (double)mgx * sx));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = t + u * TH;
        if (i >= a.P) continue;
        const float v = k * (g[u] - mg - xh[u] * mgx);
        a.gz[off + i] = a.accum ? a.gz[off + i] + v : v;
    }
}

// backward (a.bn): g = act'(dL/dy) and x_hat held in registers, the three fp64 sums, then
// dL/dz = k (g - mean(g) - x_hat mean(g x_hat)) (+= when accumulating), and the parameter grads
template <int NQ>
__global__ __launch_bounds__(kBn1Threads) void k_bn_bwd_r(BnBwdArgs a) {
    __shared__ double red[3 * kBn1Threads / 64];
    const int c = blockIdx.y, t = threadIdx.x;
    const int64_t off = (int64_t)c * a.P;
    const float4 *gy4 = reinterpret_cast<const float4 *>(a.gy + off), *y4 = reinterpret_cast<const float4 *>(a.y + off),
                 *z4 = reinterpret_cast<const float4 *>(a.z + off);
    const float m32 = a.mean[c], is32 = a.invstd[c];
    const float cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    const float gm = a.gamma[c] / cs, bt = a.beta ? a.beta[c] / cs : 0.0f;
    const bool ldy = bn_needs_y(a);
    float g[NQ][4], xh[NQ][4];
    double sg = 0.0, sgx = 0.0, sx = 0.0;
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
#pragma unroll
        for (int e = 0; e < 4; ++e) g[u][e] = xh[u][e] = 0.0f;
        if (!bnr_ok<NQ>(a.P, u)) continue;
        const int q = t + u * kBn1Threads;
        const float4 gv = gy4[q], yv = ldy ? y4[q] : make_float4(0.f, 0.f, 0.f, 0.f), zv = z4[q];
        const float ge[4] = {gv.x, gv.y, gv.z, gv.w}, ye[4] = {yv.x, yv.y, yv.z, yv.w}, ze[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            xh[u][e] = (ze[e] - m32) * is32;
            g[u][e] = bn_act_bwd(ge[e], xh[u][e], gm, bt, ye[e], a);
            sg += (double)g[u][e];
            sgx += (double)g[u][e] * (double)xh[u][e];
            sx += (double)xh[u][e];
        }
    }
    block_sum3_d(sg, sgx, sx, red);   // the only barrier
    const float k = gm * is32;
    const float mg = (float)(sg / a.P), mgx = (float)(sgx / a.P);
    if (t == 0) {
        a.ggamma[c] = (float)sgx / cs;
        a.gbeta[c] = (float)sg / cs;
        if (a.gbias) a.gbias[c] = (float)((double)k * (sg - (double)a.P * mg - (double)mgx * sx));
    }
    float4 *gz4 = reinterpret_cast<float4 *>(a.gz + off);
#pragma unroll
    for (int u = 0; u < NQ; ++u)
        if (bnr_ok<NQ>(a.P, u)) {
            const int q = t + u * kBn1Threads;
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = k * (g[u][e] - mg - xh[u][e] * mgx);
            float4 r = make_float4(o[0], o[1], o[2], o[3]);
            if (a.accum) {
                const float4 pv = gz4[q];
                r = make_float4(pv.x + r.x, pv.y + r.y, pv.z + r.z, pv.w + r.w);
            }
            gz4[q] = r;
        }
}

// ------------------------------------------------------------------------------------------
// sigma_max of every conv weight W (rows x cols), batched: one conv per blockIdx.y.
// Gram on the smaller side (m = min(rows, cols) <= 128) in fp64, exact products.
// ------------------------------------------------------------------------------------------
constexpr int kSnMaxDim = 128;
constexpr int kSnSplit = 16;  // inner-dimension split of the Gram (partials reduced by k_sn_gram_reduce; 32: slower)
constexpr int kSnPairs = 36;  // upper 16 x 16 tile pairs of a 128 x 128 Gram
// Gram workspace per conv (doubles): the reduced symmetric Gram [128][128], then the split
// partials [kSnSplit][kSnPairs][16 * 16]
constexpr int64_t kSnGramDoubles = (int64_t)kSnMaxDim * kSnMaxDim + (int64_t)kSnSplit * kSnPairs * 256;

typedef double sn_d4 __attribute__((ext_vector_type(4)));

struct SnPairs {
    int a[kSnPairs], b[kSnPairs];
};
__host__ __device__ constexpr SnPairs sn_pairs() {
    SnPairs t{};
    int k = 0;
    for (int a = 0; a < 8; ++a)
        for (int b = a; b < 8; ++b) {
            t.a[k] = a;
            t.b[k] = b;
            ++k;
        }
    return t;
}

template <int W, int... U>
__device__ __forceinline__ void sn_mfmas(const double (&f)[8], sn_d4 (&acc)[9], std::integer_sequence<int, U...>) {
    constexpr SnPairs P = sn_pairs();
    ((acc[U] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[P.a[W + 4 * U]], f[P.b[W + 4 * U]], acc[U], 0, 0, 0)), ...);
}

// grid (kSnSplit, n), 256 threads: partial z of the 36 upper 16 x 16 tile pairs of the fp64 Gram
// (G = W W^T on the smaller side, m <= 128) over the z-th inner range, on v_mfma_f64_16x16x4
// (exact products of float32 values, fp64 sums).  W is staged 32 inner values at a time in LDS as
// [row][k] floats (row stride 36: the 16 rows x 4 k of a fragment read hit 64 distinct banks); a
// lane's A and B fragments are W[16 c + (l & 15)][k + (l >> 4)] (the same form for both
// operands), wave w owns the pairs w, w + 4, ..., w + 32.
template <int WV>
__device__ __forceinline__ void sn_gram_body(const SnConv &cv, float (*Ws)[36], double *out) {
    const bool rowside = cv.rows <= cv.cols;
    const int m = rowside ? cv.rows : cv.cols;
    const int inner = rowside ? cv.cols : cv.rows;
    const int per = (int)round_up((inner + kSnSplit - 1) / kSnSplit, 32);
    const int kb = blockIdx.x * per, ke = min(inner, kb + per);
    const int t = threadIdx.x, lane = t & 63, g = lane >> 4, jl = lane & 15;
    sn_d4 acc[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) acc[u] = sn_d4{0.0, 0.0, 0.0, 0.0};
    // the next chunk's global loads are issued before this chunk's MFMAs
    float v[16];
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = t + 256 * u;
            const int r = rowside ? (e >> 5) : (e & 127), kk = rowside ? (e & 31) : (e >> 7);
            const int k = k0 + kk;
            v[u] = (r < m && k < ke) ? (rowside ? cv.W[(int64_t)r * cv.cols + k] : cv.W[(int64_t)k * cv.cols + r]) : 0.f;
        }
    };
    if (kb < ke) load(kb);
    for (int k0 = kb; k0 < ke; k0 += 32) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = t + 256 * u;
            const int r = rowside ? (e >> 5) : (e & 127), kk = rowside ? (e & 31) : (e >> 7);
            Ws[r][kk] = v[u];
        }
        __syncthreads();
        if (k0 + 32 < ke) load(k0 + 32);
#pragma unroll
        for (int kq = 0; kq < 32; kq += 4) {
            double f[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) f[c] = (double)Ws[16 * c + jl][kq + g];
            sn_mfmas<WV>(f, acc, std::make_integer_sequence<int, 9>{});
        }
    }
    // C/D layout of the f64 MFMA: column l & 15, row (l >> 4) + 4 r
#pragma unroll
    for (int u = 0; u < 9; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(int64_t)(WV + 4 * u) * 256 + (g + 4 * r) * 16 + jl] = acc[u][r];
}

__global__ __launch_bounds__(256) void k_sn_gram(const SnConv *convs, double *gram) {
    __shared__ float Ws[128][36];
    const SnConv cv = convs[blockIdx.y];
    double *out = gram + (int64_t)blockIdx.y * kSnGramDoubles + (int64_t)kSnMaxDim * kSnMaxDim +
                  (int64_t)blockIdx.x * kSnPairs * 256;
    switch (threadIdx.x >> 6) {
    case 0: sn_gram_body<0>(cv, Ws, out); break;
    case 1: sn_gram_body<1>(cv, Ws, out); break;
    case 2: sn_gram_body<2>(cv, Ws, out); break;
    default: sn_gram_body<3>(cv, Ws, out); break;
    }
}

// grid (kSnPairs, n): tile pair p, element q of its 16 x 16 block (coalesced partial reads): the
// sum over z (in order) of the partials, stored at G[i][j] and mirrored to G[j][i]; G is m x m
// inside the 128 x 128 buffer (the staged rows >= m were zero, so entries outside are 0).
__global__ __launch_bounds__(256) void k_sn_gram_reduce(const SnConv *convs, double *gram) {
    constexpr SnPairs PT = sn_pairs();
    const int p = blockIdx.x, q = threadIdx.x;
    const int i = 16 * PT.a[p] + (q >> 4), j = 16 * PT.b[p] + (q & 15);
    double *G = gram + (int64_t)blockIdx.y * kSnGramDoubles;
    const double *part = G + (int64_t)kSnMaxDim * kSnMaxDim + (int64_t)p * 256 + q;
    double pv[kSnSplit];
#pragma unroll
    for (int z = 0; z < kSnSplit; ++z) pv[z] = part[(int64_t)z * kSnPairs * 256];
    double v = 0.0;
#pragma unroll
    for (int z = 0; z < kSnSplit; ++z) v += pv[z];
    G[i * kSnMaxDim + j] = v;
    if (PT.a[p] != PT.b[p]) G[j * kSnMaxDim + i] = v;
}

// number of eigenvalues of the symmetric tridiagonal T_n above x, T_n given as ab[i] = {alpha_i,
// beta_{i-1}^2}: n minus the sign changes of the characteristic-polynomial sequence p_i =
// (alpha_i - x) p_{i-1} - beta_{i-1}^2 p_{i-2} (division-free; rescaled by a power of two every 4
// terms, which changes no sign).
__device__ __forceinline__ void sturm_term(double a, double b2, double x, double &p, double &pm, int &changes) {
    double pn = __fma_rn(a - x, p, -b2 * pm);
    // a zero takes the sign opposite to its predecessor: perturb it to -p * 2^-600 (the usual
    // Sturm-sequence convention; the next term is then -b2 p (1 + O(2^-600)))
    pn = pn != 0.0 ? pn : -p * 0x1p-600;
    changes += (int)((unsigned long long)(__double_as_longlong(pn) ^ __double_as_longlong(p)) >> 63);
    pm = p;
    p = pn;
}

__device__ __noinline__ int sturm_gt_checked(const double2 *ab, int n, double x) {
    double pm = 1.0, p = ab[0].x - x;
    p = p != 0.0 ? p : -0x1p-600;              // p_0 = 1 > 0: a zero p_1 counts as negative
    int changes = p < 0.0;
    int i = 1;
    double2 c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = ab[min(i + j, kSnMaxDim - 1)];
    for (; i + 4 <= n; i += 4) {
        double2 nx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) nx[j] = ab[min(i + 4 + j, kSnMaxDim - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) sturm_term(c[j].x, c[j].y, x, p, pm, changes);
        int e;
        frexp(fabs(p) > fabs(pm) ? p : pm, &e);
        p = ldexp(p, -e);
        pm = ldexp(pm, -e);
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = nx[j];
    }
    for (; i < n; ++i) sturm_term(ab[i].x, ab[i].y, x, p, pm, changes);
    return n - changes;
}

// The same count with the zero test off the recurrence's dependency chain: the terms are
// evaluated unperturbed and any exact zero is only recorded; a sequence that met one (rare) is
// re-evaluated by sturm_gt_checked.  Without a zero both evaluate the same values (the power-of-
// two rescaling, here every 8 terms, is exact), so the count is the checked one.  Eight terms'
// LDS reads are in flight while eight are evaluated.
__device__ __forceinline__ int sturm_gt(const double2 *ab, int n, double x) {
    double pm = 1.0, p = ab[0].x - x;
    if (p == 0.0) return sturm_gt_checked(ab, n, x);
    int changes = p < 0.0;
    bool zero = false;
    int i = 1;
    double2 c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = ab[min(i + j, kSnMaxDim - 1)];
    for (; i + 8 <= n; i += 8) {
        double2 nx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) nx[j] = ab[min(i + 8 + j, kSnMaxDim - 1)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const double pn = __fma_rn(c[j].x - x, p, -c[j].y * pm);
            zero |= pn == 0.0;
            changes += (int)((unsigned long long)(__double_as_longlong(pn) ^ __double_as_longlong(p)) >> 63);
            pm = p;
            p = pn;
        }
        int e;
        frexp(fabs(p) > fabs(pm) ? p : pm, &e);
        p = ldexp(p, -e);
        pm = ldexp(pm, -e);
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = nx[j];
    }
    for (; i < n; ++i) {
        const double pn = __fma_rn(ab[i].x - x, p, -ab[i].y * pm);
        zero |= pn == 0.0;
        changes += (int)((unsigned long long)(__double_as_longlong(pn) ^ __double_as_longlong(p)) >> 63);
        pm = p;
        p = pn;
    }
    return zero ? sturm_gt_checked(ab, n, x) : n - changes;
}

// One 256-point multisection round on T_n: thread t tests x_t = base + step (t + 1); returns (to
// every thread) the largest t with an eigenvalue above x_t, or -1.  So the top eigenvalue lies in
// (x_bt, x_{bt+1}] with x_{-1} = base, recomputed by the caller with sn_grid (the same rounding).
// `best` holds 3 slots used round-robin: a round's slot was reset by thread 0 in the previous
// round, before its barrier, and last read two rounds ago.  One barrier per round.
__device__ __forceinline__ double sn_grid(double base, double step, int t) { return base + step * (double)(t + 1); }

// max over the 64 lanes (uniform): DPP row steps, then the four rows' values by readlane
__device__ __forceinline__ int wave_max_i(int v) {
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));   // row_half_mirror
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));   // row_mirror
    return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
               max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

__device__ __forceinline__ int sn_round(const double2 *ab, int n, double base, double step, int *best, int &rnd) {
    const int t = threadIdx.x;
    int *slot = best + rnd % 3;
    if (t == 0) best[(rnd + 1) % 3] = -1;
    // the wave's largest flagged t by DPP, then one LDS atomic per wave (a per-lane atomicMax
    // compiled to a scalar loop over the flagged lanes)
    const int wmax = wave_max_i(sturm_gt(ab, n, sn_grid(base, step, t)) >= 1 ? t : -1);
    if ((t & 63) == 0 && wmax >= 0) atomicMax(slot, wmax);
    __syncthreads();
    const int bt = *slot;
    ++rnd;
    return bt;
}

// Narrow [lo, hi] (top eigenvalue inside, lo exclusive) by 257x per round until hi - lo <= tol hi
// (at most 12 rounds: 29 decades; tol >= 1e-12 stays far above the rounding of the grid).
__device__ __forceinline__ void sn_multisect(const double2 *ab, int n, double &lo, double &hi, double tol, int *best,
                                             int &rnd) {
    for (int it = 0; it < 12 && hi - lo > tol * hi; ++it) {
        const double step = (hi - lo) * (1.0 / 257.0);
        const int bt = sn_round(ab, n, lo, step, best, rnd);
        const double nlo = bt >= 0 ? sn_grid(lo, step, bt) : lo;
        const double nhi = bt < 255 ? sn_grid(lo, step, bt + 1) : hi;
        lo = nlo;
        hi = fmax(nlo, nhi);
    }
}

// One workgroup (256 threads) per conv: Lanczos (no reorthogonalisation: the extreme Ritz value
// converges regardless, Paige) with the Gram in registers (thread t holds half a row, 64
// doubles).  The Gershgorin bounds of T_k are kept in registers as rows become final.
// Convergence: at step 24 the top Ritz value is bracketed to a cell of width <= 5e-10 of it
// (multisection from the Gershgorin interval); every 4 steps after that ONE round over the 256
// cells of that width above the bracket's low end relocates it (the top Ritz value only grows
// with k, Cauchy interlacing).  Converged when it stayed in its cell for 4 steps (typically 28-40
// steps for these weights instead of m = 128); one more round then narrows the cell 257x.
// A move of more than 256 cells re-brackets from the Gershgorin bound.
// sigma32 = float(sqrt(lambda_max)); scale = max(1, sigma32 / ln_lambda) (float32, as torch).
__global__ __launch_bounds__(256) void k_sn_sigma(const SnConv *convs, const double *gram, float *sigma,
                                                  float *scale, float ln_lambda, long long *prof) {
    if (prof && threadIdx.x == 0) prof[blockIdx.x * 8 + 0] = wall_clock64();
    const SnConv cv = convs[blockIdx.x];
    const int m = cv.rows <= cv.cols ? cv.rows : cv.cols;
    const double *G = gram + (int64_t)blockIdx.x * kSnGramDoubles;
    __shared__ __attribute__((aligned(16))) double q[kSnMaxDim];
    __shared__ __attribute__((aligned(16))) double2 ab[kSnMaxDim];   // {alpha_i, beta_{i-1}^2}
    __shared__ int best_s[3];
    // Matvec blocking: thread t holds the 4 x 16 block of G at rows 4 rb .. 4 rb + 3 (rb = t >> 3),
    // columns 16 cb .. 16 cb + 15 (cb = t & 7), so a step reads 16 values of q from LDS per thread
    // (a quarter of what half rows needed: the LDS return bandwidth was the step's largest cost),
    // and the 8 lanes of a row block sum their partials by DPP.  Vector entries: row = 4 rb +
    // (cb & 3), held by lanes cb and cb + 4 (half = cb >> 2; half 0 contributes and writes q).
    // Column chunk c (2 doubles) of a thread is 2 ((c + cb) & 7): the 8 lanes of a row block read
    // distinct LDS banks.
    const int t = threadIdx.x, rb = t >> 3, cb = t & 7, row = 4 * rb + (cb & 3), half = cb >> 2;
    if (t < 3) best_s[t] = -1;
    // the thread's block of the reduced Gram (k_sn_gram_reduce), straight into registers: 32
    // 16-B loads, all in flight.  (No LDS staging: a kernel that asked for the 129 KB a staged
    // copy needs could not start on any CU that held a sparse-coding workgroup, so the DIP
    // stalled at every step's sigma while the sparse coding ran beside it.)
    double g[64];   // g[16 i + 2 c + e] = G[4 rb + i][16 cb + 2 ((c + cb) & 7) + e]
    {
        double2 pv[32];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 8; ++c)
                pv[8 * i + c] = *reinterpret_cast<const double2 *>(G + (int64_t)(4 * rb + i) * kSnMaxDim + 16 * cb +
                                                                   2 * ((c + cb) & 7));
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            g[2 * u] = pv[u].x;
            g[2 * u + 1] = pv[u].y;
        }
    }
    if (prof && t == 0) prof[blockIdx.x * 8 + 1] = wall_clock64();
    int par = 0, rnd = 0;
    // Lanczos on the unnormalised residual r_k (r_0 = start vector): one matvec u' = G r_k, one
    // two-value reduction (||r_k||^2, r_k.u'), then beta_k = ||r_k||, q_k = r_k / beta_k,
    // alpha_k = r_k.u' / beta_k^2 and r_{k+1} = u'/beta_k - alpha_k q_k - beta_k q_{k-1}.
    // Two barriers per step.
    // (Measured: warm-starting from the previous step's top Ritz vector does not shorten the
    // iteration: with Adam at lr 0.1 the weights change by O(their size) every step.)
    double rr = (row < m) ? 1.0 + 0.5 * sin(0.7 * (double)row + 0.3) : 0.0;
    double qprev = 0.0;
    // uniform: Gershgorin max / min over the final rows of T, the last row's alpha and beta
    double gmax = -1e300, gmin = 1e300, a_last = 0.0, b_last = 0.0;
    double blo = 0.0, bhi = 0.0;                  // bracket of the last check's top Ritz value
    bool have = false, converged = false;
    __shared__ double red2[2][8];
    if (half == 0) q[row] = rr;
    __syncthreads();
    int k = 0;
    long long tcheck = 0, ccheck = 0;
    for (; k < m; ++k) {
        // all 8 b128 reads of this thread's 16 entries of q are issued before the first FMA (left
        // to itself the compiler waited on each read)
        double qv[16];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const double2 v = *reinterpret_cast<const double2 *>(q + 16 * cb + 2 * ((c + cb) & 7));
            qv[2 * c] = v.x;
            qv[2 * c + 1] = v.y;
        }
        __builtin_amdgcn_sched_barrier(0);
        double u4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // two independent FMA chains per row
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int c = 0; c < 16; c += 2) {
                s0 = __fma_rn(g[16 * i + c], qv[c], s0);
                s1 = __fma_rn(g[16 * i + c + 1], qv[c + 1], s1);
            }
            u4[i] = s0 + s1;
        }
        // sum over the row block's 8 lanes (xor 1, xor 2, then lane i + lane 7 - i)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u4[i] += dpp_d<0xB1>(u4[i]);
            u4[i] += dpp_d<0x4E>(u4[i]);
            u4[i] += dpp_d<0x141>(u4[i]);
        }
        const int own = cb & 3;   // (selects, not a branch per lane group)
        const double u01 = (own & 1) ? u4[1] : u4[0], u23 = (own & 1) ? u4[3] : u4[2];
        double u = (own & 2) ? u23 : u01;
        const double w_rr = wave_sum_d(half == 0 ? rr * rr : 0.0);
        const double w_ru = wave_sum_d(half == 0 ? rr * u : 0.0);
        if ((t & 63) == 0) {
            red2[0][(t >> 6) + 4 * par] = w_rr;
            red2[1][(t >> 6) + 4 * par] = w_ru;
        }
        __syncthreads();
        const double s_rr = (red2[0][4 * par] + red2[0][4 * par + 1]) + (red2[0][4 * par + 2] + red2[0][4 * par + 3]);
        const double s_ru = (red2[1][4 * par] + red2[1][4 * par + 1]) + (red2[1][4 * par + 2] + red2[1][4 * par + 3]);
        par ^= 1;
        const double b = sqrt(s_rr);
        if (k > 0 && !(b > 1e-14 * fabs(a_last))) break;   // invariant subspace: T_k is exact
        const double ib = 1.0 / b;
        const double a = s_ru * ib * ib;
        if (t == 0) ab[k] = make_double2(a, s_rr);
        // row k-1 is final now (its off-diagonals beta_{k-1}, beta_k are known); row k so far
        if (k > 0) {
            const double r = b_last + b;
            gmax = fmax(gmax, a_last + r);
            gmin = fmin(gmin, a_last - r);
        }
        a_last = a;
        b_last = k > 0 ? b : 0.0;
        const double qk = rr * ib;
        rr = u * ib - a * qk - (k > 0 ? b : 0.0) * qprev;
        qprev = qk;
        if (k + 1 == m) { ++k; break; }
        if (k + 1 >= 24 && ((k + 1) & 3) == 0) {
            __syncthreads();                      // ab[k] visible
            const long long tc0 = prof ? wall_clock64() : 0, cc0 = prof ? clock64() : 0;
            const int n = k + 1;
            const double ghi = fmax(gmax, a_last + b_last);
            double lo, hi = ghi;
            bool need = true;
            if (have) {
                const double w = bhi - blo;
                const int bt = sn_round(ab, n, blo, w, best_s, rnd);
                if (bt < 0) {
                    converged = true;              // still inside [blo, bhi]
                    need = false;
                } else if (bt < 255) {
                    const double b0 = blo;
                    blo = sn_grid(b0, w, bt);
                    bhi = sn_grid(b0, w, bt + 1);
                    need = false;
                } else {
                    lo = sn_grid(blo, w, 255);
                }
            } else {
                lo = fmax(0.0, fmin(gmin, a_last - b_last));
            }
            if (need) {
                sn_multisect(ab, n, lo, hi, 5e-10, best_s, rnd);
                blo = lo;
                bhi = hi;
                have = true;
            }
            if (prof) { tcheck += wall_clock64() - tc0; ccheck += clock64() - cc0; }
            if (converged) { ++k; break; }
        }
        if (half == 0) q[row] = rr;                   // the matvec reads of q finished before the barrier
        __syncthreads();
    }
    __syncthreads();
    if (prof && t == 0) { prof[blockIdx.x * 8 + 2] = wall_clock64(); prof[blockIdx.x * 8 + 4] = k; prof[blockIdx.x * 8 + 5] = tcheck; prof[blockIdx.x * 8 + 6] = ccheck; }
    double lmax = 0.0;
    if (m > 0) {
        double lo, hi;
        if (converged) {
            // one more round inside the converged cell (width <= 5e-10 lmax -> <= 2e-12)
            lo = blo;
            hi = bhi;
            sn_multisect(ab, k, lo, hi, 0.5 * (bhi - blo) / bhi, best_s, rnd);
        } else {
            // T_k exhausted (k = m) or exact (invariant subspace): from its Gershgorin interval
            lo = fmax(0.0, fmin(gmin, a_last - b_last));
            hi = fmax(gmax, a_last + b_last);
            sn_multisect(ab, k, lo, hi, 1e-12, best_s, rnd);
        }
        lmax = 0.5 * (lo + hi);
    }
    if (prof && t == 0) prof[blockIdx.x * 8 + 3] = wall_clock64();
    if (t == 0) {
        const float s32 = (float)sqrt(fmax(lmax, 0.0));
        sigma[blockIdx.x] = s32;
        scale[blockIdx.x] = fmaxf(1.0f, s32 / ln_lambda);
    }
}

// Wn = W_bar / scale  (all convs; blockIdx.y = conv)
__global__ void k_sn_apply(const SnConv *convs, const float *scale) {
    const SnConv cv = convs[blockIdx.y];
    const int64_t n = (int64_t)cv.rows * cv.cols;
    const float s = scale[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        cv.Wn[i] = cv.W[i] / s;
}

// ------------------------------------------------------------------------------------------
// Loss: mse(target*mask, out*mask) over C*P (main_LRS_PnP_DIP_1-LiP.py:234); gout = dL/dout.
// mask is [P] (broadcast over channels, mask_bkg (1,1,H,W)) or null.
// ------------------------------------------------------------------------------------------
// grid (S, C): workgroup (sb, c) covers pixels [sb*chunk, +chunk) of channel c, so the mask
// index is the pixel (no 64-bit modulo); vec: float4 loads / stores (P, chunk multiples of 4).
__global__ __launch_bounds__(256) void k_masked_mse(const float *__restrict__ out, const float *__restrict__ target,
                                                    const float *__restrict__ mask, int C, int64_t P, int chunk,
                                                    int vec, float *__restrict__ gout, double *loss_acc) {
    __shared__ double red[8];
    const float norm = (float)(2.0 / ((double)C * (double)P));
    const int64_t off = (int64_t)blockIdx.y * P;
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = min(P, i0 + chunk);
    double s = 0.0;
    if (vec) {
        const float4 *o4 = reinterpret_cast<const float4 *>(out + off), *t4 = reinterpret_cast<const float4 *>(target + off);
        const float4 *m4 = reinterpret_cast<const float4 *>(mask);
        float4 *g4 = gout ? reinterpret_cast<float4 *>(gout + off) : nullptr;
        for (int64_t q = (i0 >> 2) + threadIdx.x; q < (i1 >> 2); q += blockDim.x) {
            const float4 ov = o4[q], tv = t4[q];
            const float4 mv = mask ? m4[q] : make_float4(1.0f, 1.0f, 1.0f, 1.0f);
            const float oe[4] = {ov.x, ov.y, ov.z, ov.w}, te[4] = {tv.x, tv.y, tv.z, tv.w},
                        me[4] = {mv.x, mv.y, mv.z, mv.w};
            float ge[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = te[e] * me[e] - oe[e] * me[e];
                s += (double)d * (double)d;
                ge[e] = (-(norm * d)) * me[e];
            }
            if (g4) g4[q] = make_float4(ge[0], ge[1], ge[2], ge[3]);
        }
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
            const float mk = mask ? mask[i] : 1.0f;
            const float a = target[off + i] * mk, b = out[off + i] * mk;
            const float d = a - b;
            s += (double)d * (double)d;
            if (gout) gout[off + i] = (-(norm * d)) * mk;
        }
    }
    s = block_sum_d(s, red);
    if (threadIdx.x == 0) atomicAdd(loss_acc, s);
}

// Loss head of a training step whose last node is a conv without BN (both reference nets): the
// masked MSE (as k_masked_mse: sum d^2, dL/dout = -(2/(C P)) d m) fused with that node's
// activation backward dL/dz = act'(out) dL/dout and its bias gradient sum_p dL/dz: one pass
// instead of masked-MSE + BN-backward statistics + BN-backward apply.  Grid (S, C), S ~ P / 4096
// (a few thousand workgroups: the pass is HBM-bound only with many loads in flight).  Partials
// (fp64) go to part[c][S] (bias) and part[C S + c][S] (loss); the last workgroup of a channel to
// finish (per-channel counter) sums that channel's partials in order, the last channel to finish
// (counter cnt[C]) sums the channel losses in order into loss_acc: bias gradient and loss are both
// deterministic.  Counters are reset by their last arriver.
__global__ __launch_bounds__(256) void k_mse_head(const float *__restrict__ out, const float *__restrict__ target,
                                                  const float *__restrict__ mask, int C, int64_t P, int chunk,
                                                  int vec, int act, float *__restrict__ gz, double *loss_acc,
                                                  double *__restrict__ part, int *__restrict__ cnt,
                                                  float *__restrict__ gbias) {
    __shared__ double red[8];
    __shared__ int last;
    const float norm = (float)(2.0 / ((double)C * (double)P));
    const int c = blockIdx.y, S = gridDim.x;
    const int64_t off = (int64_t)c * P;
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = min(P, i0 + chunk);
    double s = 0.0, sb = 0.0;
    if (vec) {
        // one fp64 accumulator pair per float4 lane: four independent dependency chains
        double s4[4] = {0.0, 0.0, 0.0, 0.0}, sb4[4] = {0.0, 0.0, 0.0, 0.0};
        const float4 *o4 = reinterpret_cast<const float4 *>(out + off), *t4 = reinterpret_cast<const float4 *>(target + off);
        const float4 *m4 = reinterpret_cast<const float4 *>(mask);
        float4 *g4 = reinterpret_cast<float4 *>(gz + off);
        const int q0 = (int)(i0 >> 2), q1 = (int)(i1 >> 2);
        // two float4 per thread per trip: both loads of both in flight together
        for (int q = q0 + threadIdx.x; q < q1; q += 2 * blockDim.x) {
            const bool hb = q + (int)blockDim.x < q1;
            const int qb = hb ? q + (int)blockDim.x : q;   // loads unconditional (all in flight together)
            const float4 ov0 = o4[q], tv0 = t4[q], ov1 = o4[qb], tv1 = t4[qb];
            const float4 one4 = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
            const float4 mv0 = mask ? m4[q] : one4, mv1 = mask ? m4[qb] : one4;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && !hb) break;
                const float4 ov = h ? ov1 : ov0, tv = h ? tv1 : tv0, mv = h ? mv1 : mv0;
                const float oe[4] = {ov.x, ov.y, ov.z, ov.w}, te[4] = {tv.x, tv.y, tv.z, tv.w},
                            me[4] = {mv.x, mv.y, mv.z, mv.w};
                float ge[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = te[e] * me[e] - oe[e] * me[e];
                    s4[e] += (double)d * (double)d;
                    ge[e] = act_bwd((-(norm * d)) * me[e], oe[e], act);
                    sb4[e] += (double)ge[e];
                }
                g4[h ? qb : q] = make_float4(ge[0], ge[1], ge[2], ge[3]);
            }
        }
        s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        sb = (sb4[0] + sb4[1]) + (sb4[2] + sb4[3]);
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
            const float mk = mask ? mask[i] : 1.0f;
            const float o = out[off + i];
            const float d = target[off + i] * mk - o * mk;
            s += (double)d * (double)d;
            const float g = act_bwd((-(norm * d)) * mk, o, act);
            gz[off + i] = g;
            sb += (double)g;
        }
    }
    int parity = 0;
    block_sum2_d(s, sb, red);   // (red is free again after the barrier below)
    double *bp = part + (int64_t)c * S, *lp = part + (int64_t)C * S + (int64_t)c * S;
    double *cl = part + 2 * (int64_t)C * S;   // per-channel losses
    // hand-offs without fences (lrs_common.h, wt_store): write-through partials, drain, count
    if (threadIdx.x == 0) {
        wt_store(bp + blockIdx.x, sb);
        wt_store(lp + blockIdx.x, s);
        wt_drain();
        last = agent_add(cnt + c, 1) == S - 1;
    }
    __syncthreads();
    if (!last) return;
    // the channel's partials, summed by the whole workgroup in a fixed tree (S <= 64): deterministic
    const int t = threadIdx.x;
    double tb = t < S ? wt_load(bp + t) : 0.0, tl = t < S ? wt_load(lp + t) : 0.0;
    block_sum2_d(tb, tl, red);
    if (t == 0) {
        gbias[c] = (float)tb;
        agent_store(cnt + c, 0);
        wt_store(cl + c, tl);
        wt_drain();
        last = agent_add(cnt + C, 1) == C - 1;
    }
    __syncthreads();
    if (!last) return;
    double tot = 0.0;
    for (int k = t; k < C; k += blockDim.x) tot += wt_load(cl + k);
    tot = block_sum_d1(tot, red, parity);
    if (t == 0) {
        *loss_acc += tot;
        agent_store(cnt + C, 0);
    }
}

// ------------------------------------------------------------------------------------------
// Adam (torch.optim.Adam defaults: no weight decay, no amsgrad), flat parameter buffer.
// step is a device counter so a captured step replays correctly.
// ------------------------------------------------------------------------------------------
// A weight gradient whose split-K partials Adam itself finishes (the step's last weight gradient,
// lrs_dipnet_train_steps): parameters [beg, beg + len) take g = (sum of the nsplit partials, in
// k_gemm_reduce's order) / *div, which is also stored to the gradient buffer
struct AdamPend {
    const float *part;
    int nsplit;
    int64_t beg, len;
    const float *div;
    float *gout;
};

__device__ __forceinline__ float adam_pend_grad(const AdamPend &a, int64_t idx) {
    const int64_t i = idx - a.beg;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= a.nsplit; z += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += a.part[(int64_t)(z + u) * a.len + i];
    for (; z < a.nsplit; ++z) acc[z & 7] += a.part[(int64_t)z * a.len + i];
    float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    if (a.div) s = s / *a.div;
    a.gout[idx] = s;
    return s;
}

__global__ void k_adam(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                       float *__restrict__ v, int64_t n, const int *step, float lr, float b1, float b2,
                       float eps, AdamPend pend) {
    __shared__ float sc[2];   // the bias corrections, once per workgroup (fp64 pow is costly)
    const bool vec = ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0);
    const int64_t n4 = vec ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the first float4 of every thread is loaded before thread 0's fp64 pow: the loads' latency and
    // the bias corrections overlap (one float4 per thread covers the whole net at the launch size)
    float4 pv0 = {0.f, 0.f, 0.f, 0.f}, mv0 = pv0, vv0 = pv0, gv0 = pv0;
    if (q0 < n4) {
        pv0 = reinterpret_cast<float4 *>(p)[q0];
        mv0 = reinterpret_cast<float4 *>(m)[q0];
        vv0 = reinterpret_cast<float4 *>(v)[q0];
        gv0 = reinterpret_cast<const float4 *>(g)[q0];
    }
    if (threadIdx.x == 0) {
        const int t = *step;
        const double bc1 = 1.0 - pow((double)b1, (double)t);
        const double bc2 = 1.0 - pow((double)b2, (double)t);
        sc[0] = (float)((double)lr / bc1);
        sc[1] = (float)sqrt(bc2);
    }
    __syncthreads();
    const float step_size = sc[0], bc2s = sc[1];
    // elementwise, so the float4 body (all four buffers 16-B aligned) is bitwise the scalar one
    auto upd = [&](float &pi, float gi, float &mi, float &vi) {
        mi = mi + (1.0f - b1) * (gi - mi);                          // exp_avg.lerp_(grad, 1-b1)
        vi = vi * b2 + (1.0f - b2) * gi * gi;                       // mul_(b2).addcmul_(g, g, 1-b2)
        const float den = sqrtf(vi) / bc2s + eps;
        pi = pi - step_size * (mi / den);
    };
    for (int64_t q = q0; q < n4; q += stride) {
        const bool first = q == q0;
        float4 pv = first ? pv0 : reinterpret_cast<float4 *>(p)[q], mv = first ? mv0 : reinterpret_cast<float4 *>(m)[q],
               vv = first ? vv0 : reinterpret_cast<float4 *>(v)[q];
        float4 gv = first ? gv0 : reinterpret_cast<const float4 *>(g)[q];
        if (pend.part && 4 * q + 3 >= pend.beg && 4 * q < pend.beg + pend.len) {
            if (4 * q >= pend.beg && 4 * q + 3 < pend.beg + pend.len) {
                gv.x = adam_pend_grad(pend, 4 * q); gv.y = adam_pend_grad(pend, 4 * q + 1);
                gv.z = adam_pend_grad(pend, 4 * q + 2); gv.w = adam_pend_grad(pend, 4 * q + 3);
            } else {
                float ge[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * q + e >= pend.beg && 4 * q + e < pend.beg + pend.len) ge[e] = adam_pend_grad(pend, 4 * q + e);
                gv = make_float4(ge[0], ge[1], ge[2], ge[3]);
            }
        }
        upd(pv.x, gv.x, mv.x, vv.x);
        upd(pv.y, gv.y, mv.y, vv.y);
        upd(pv.z, gv.z, mv.z, vv.z);
        upd(pv.w, gv.w, mv.w, vv.w);
        reinterpret_cast<float4 *>(m)[q] = mv;
        reinterpret_cast<float4 *>(v)[q] = vv;
        reinterpret_cast<float4 *>(p)[q] = pv;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float pi = p[i], mi = m[i], vi = v[i];
        const float gi = (pend.part && i >= pend.beg && i < pend.beg + pend.len) ? adam_pend_grad(pend, i) : g[i];
        upd(pi, gi, mi, vi);
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
    }
}

__global__ void k_counter_inc(int *c) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *c += 1;
}

__global__ void k_step_begin(double *loss_acc, int *step) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        *loss_acc = 0.0;
        *step += 1;
    }
}

// ------------------------------------------------------------------------------------------
// Early stopping (main_LRS_PnP_DIP_1-LiP.py:71-99, 244-264), on device.
// The reference's metric each step, once the last `size` outputs are collected (myMetric, :102-103):
//   var = mean_j sum_p (ave_p - img_j,p)^2 / N = (Q2 - sum_p A_p^2 / size) / (N size),
// A_p = sum_j img_j,p over the ring and Q2 = sum_p sum_j img_j,p^2, one scalar (the squares' sum needs
// no per-pixel form).  The buffer (lrs_es_ring_bytes) holds the ring [size][N] floats, then A [N]
// (fp64), the per-workgroup partial sums [2][kEsMaxBlocks] and Q2.  One pass per step (k_es_step)
// writes the new output into its slot and slides A (+ new - the slot's old value), so a step reads the
// ring slot it overwrites and nothing else, and its workgroups sum the change of the squares (exact in
// fp64: new^2 - old^2) and A_p^2; k_es_decide adds both in a fixed order (deterministic), slides Q2
// and forms the variance.  Every kEsRefresh windows (the slot of the last index) A and Q2 are
// re-summed from the whole ring in slot order, bounding the sliding sums' rounding drift (~1e-16 per
// update: after 300 updates still ~1e-12 of the variance).  Traffic 28 B per output element per step
// (round 6 first form: 44 B with a per-pixel B_p and a re-sum every window; round 5: the whole ring read
// twice per step -- 1.8 GB per step at 196 x 196 x 198 -- and workgroup sums added with atomics).
// ------------------------------------------------------------------------------------------
constexpr int kEsMaxBlocks = 1024;
constexpr int kEsRefresh = 10;   // windows between re-sums of A and Q2 from the ring

// this output's epoch c (before k_es_decide increments count) re-sums A and Q2 from the ring
__host__ __device__ inline bool es_refresh(int c, int S) { return (c + 1) % (S * kEsRefresh) == 0; }

__host__ __device__ inline int64_t es_ab_offset_bytes(int size, int64_t N) {   // A after the ring, 16-B aligned
    return ((int64_t)size * N * 4 + 15) / 16 * 16;
}

__global__ __launch_bounds__(256) void k_es_step(const float *__restrict__ out, int64_t N, float *__restrict__ ring,
                                                lrs_es_state *st) {
    __shared__ double red[16];
    const int S = st->size, c = st->count, slot = c % S;   // c: this output's epoch (k_es_decide increments count)
    double *A = reinterpret_cast<double *>(reinterpret_cast<char *>(ring) + es_ab_offset_bytes(S, N));
    double *part = A + N;   // [0 .. kEsMaxBlocks): the squares' change (or sum), then the A^2 sums
    float *dst = ring + (int64_t)slot * N;
    const bool full = c + 1 >= S, refresh = es_refresh(c, S);
    double dq = 0.0, qa = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        const float x = out[i];
        double a;
        if (refresh) {   // the ring in slot order, the new output in the last slot
            dst[i] = x;
            a = 0.0;
            double q = 0.0;
            for (int j = 0; j < S - 1; ++j) {
                const double v = (double)ring[(int64_t)j * N + i];
                a += v;
                q += v * v;
            }
            a += (double)x;
            q += (double)x * (double)x;
            dq += q;
        } else if (c < S) {   // filling: a plain running sum
            dst[i] = x;
            a = c == 0 ? (double)x : A[i] + (double)x;
            dq += (double)x * (double)x;
        } else {              // sliding: the slot's old output leaves the window
            const float o = dst[i];
            dst[i] = x;
            a = A[i] + ((double)x - (double)o);
            dq += (double)x * (double)x - (double)o * (double)o;
        }
        A[i] = a;
        if (full) qa += a * a;
    }
    block_sum2_d(dq, qa, red);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = dq;
        part[kEsMaxBlocks + blockIdx.x] = qa;
    }
}

#ifdef LRS_TUNING
// The round-5 form (tuning build, LRS_DIP_ES_TWO_PASS=1, A/B only): push, then the whole ring read
// twice per step (mean, then squared deviations), workgroup sums into var_acc by atomics.
__global__ void k_es_push_r5(const float *__restrict__ out, int64_t N, float *__restrict__ ring, lrs_es_state *st) {
    const int slot = st->count % st->size;
    float *dst = ring + (int64_t)slot * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = out[i];
}
__global__ void k_es_var_r5(const float *__restrict__ ring, int64_t N, lrs_es_state *st) {
    __shared__ double red[8];
    if (st->count + 1 < st->size) return;
    const int S = st->size;
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        double ave = 0.0;
        for (int j = 0; j < S; ++j) ave += (double)ring[(int64_t)j * N + i];
        ave /= S;
        for (int j = 0; j < S; ++j) {
            const double d = ave - (double)ring[(int64_t)j * N + i];
            s += d * d;
        }
    }
    s = block_sum_d(s, red);
    if (threadIdx.x == 0) atomicAdd(&st->var_acc, s);
}
#endif

// one wave: the nblk partials of k_es_step in a fixed order, then the reference's patience test
// (nblk == 0: the round-5 form's var_acc instead)
__global__ void k_es_decide(const float *ring, int64_t N, int nblk, lrs_es_state *st) {
    const int S = st->size;
    double *part = reinterpret_cast<double *>(reinterpret_cast<char *>(const_cast<float *>(ring)) + es_ab_offset_bytes(S, N)) + N;
    double *q2 = part + 2 * kEsMaxBlocks;   // the window's sum of squares
    double dq = 0.0, qa = 0.0;
    for (int b = threadIdx.x; b < nblk; b += 64) {
        dq += part[b];
        qa += part[kEsMaxBlocks + b];
    }
    dq = wave_sum_d(dq);   // fixed order
    qa = wave_sum_d(qa);
    if (threadIdx.x != 0) return;
    double v;
    if (nblk == 0) {
        v = st->var_acc;
    } else {
        const int c = st->count;
        const double q = (c == 0 || es_refresh(c, S)) ? dq : *q2 + dq;
        *q2 = q;
        v = q - qa / (double)S;
    }
    const int epoch = st->count;           // iteration index i of the reference loop
    st->count += 1;
    if (st->count >= S && !st->stop) {
        const double var = v / (double)N / (double)S;
        st->last_var = var;
        if (var < st->best) {
            st->best = var;
            st->best_epoch = epoch;
            st->wait = 0;
        } else {
            st->wait += 1;
            if (st->wait >= st->patience) {
                st->stop = 1;
                st->stop_epoch = epoch;
            }
        }
    }
    st->var_acc = 0.0;
}

// ------------------------------------------------------------------------------------------
// Concat (models/common.py:11-42): out = cat(a, up2?(b)) along channels, both centre-cropped to
// the smaller H and W (offset (size - target) // 2, :27-37).
// ------------------------------------------------------------------------------------------
struct CatGeom {
    int Ca, Ha, Wa, Cb, Hb, Wb, upb;   // b is (Cb, Hb, Wb) before the optional nearest x2
    int H, W;                          // output spatial size
    int oay, oax, oby, obx;            // crop offsets into a and into up2(b)
};

__global__ void k_concat_fwd(const float *__restrict__ a, const float *__restrict__ b, CatGeom g,
                             float *__restrict__ out) {
    const int64_t HW = (int64_t)g.H * g.W, n = (int64_t)(g.Ca + g.Cb) * HW;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i / HW);
        const int p = (int)(i - (int64_t)c * HW);
        const int y = p / g.W, x = p - y * g.W;
        float v;
        if (c < g.Ca) {
            v = a[((int64_t)c * g.Ha + y + g.oay) * g.Wa + x + g.oax];
        } else {
            int yy = y + g.oby, xx = x + g.obx;
            if (g.upb) { yy >>= 1; xx >>= 1; }
            v = b[((int64_t)(c - g.Ca) * g.Hb + yy) * g.Wb + xx];
        }
        out[i] = v;
    }
}

// The same copies / sums laid out for throughput: grid (row quads, channels), a thread = 4
// consecutive x of one row of one channel; no 64-bit division per element, float4 stores when the
// rows are multiples of 4 (the values and the 2x2 summation order are k_concat_fwd / _bwd's).
__global__ __launch_bounds__(256) void k_concat_fwd4(const float *__restrict__ a, const float *__restrict__ b,
                                                     CatGeom g, float *__restrict__ out) {
    const int W4 = (g.W + 3) >> 2;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= g.H * W4) return;
    const int c = blockIdx.y, y = t / W4, x0 = 4 * (t - y * W4);
    float v[4];
    if (c < g.Ca) {
        const float *src = a + ((int64_t)c * g.Ha + y + g.oay) * g.Wa + g.oax;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = x0 + e < g.W ? src[x0 + e] : 0.0f;
    } else {
        int yy = y + g.oby;
        if (g.upb) yy >>= 1;
        const float *src = b + ((int64_t)(c - g.Ca) * g.Hb + yy) * g.Wb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            int xx = x0 + e + g.obx;
            if (g.upb) xx >>= 1;
            v[e] = x0 + e < g.W ? src[xx] : 0.0f;
        }
    }
    float *dst = out + ((int64_t)c * g.H + y) * g.W + x0;
    if ((g.W & 3) == 0) {
        *reinterpret_cast<float4 *>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (x0 + e < g.W) dst[e] = v[e];
    }
}

// part 0: ga over (Ha rows x Wa), channels Ca; part 1: gb over (Hb x Wb), channels Cb
__global__ __launch_bounds__(256) void k_concat_bwd4(const float *__restrict__ go, CatGeom g, float *__restrict__ gx,
                                                     int acc, int part) {
    const int Hs = part ? g.Hb : g.Ha, Ws = part ? g.Wb : g.Wa;
    const int W4 = (Ws + 3) >> 2;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= Hs * W4) return;
    const int c = blockIdx.y, Y = t / W4, X0 = 4 * (t - Y * W4);
    const int64_t HW = (int64_t)g.H * g.W;
    float v[4];
    if (part == 0) {
        const float *gc = go + (int64_t)c * HW;
        const int y = Y - g.oay;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int x = X0 + e - g.oax;
            v[e] = (y >= 0 && y < g.H && x >= 0 && x < g.W && X0 + e < Ws) ? gc[(int64_t)y * g.W + x] : 0.0f;
        }
    } else {
        const float *gc = go + (int64_t)(g.Ca + c) * HW;
        const int f = g.upb ? 2 : 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float s = 0.0f;
            for (int dy = 0; dy < f; ++dy)
                for (int dx = 0; dx < f; ++dx) {
                    const int y = Y * f + dy - g.oby, x = (X0 + e) * f + dx - g.obx;
                    if (y >= 0 && y < g.H && x >= 0 && x < g.W) s += gc[(int64_t)y * g.W + x];
                }
            v[e] = s;
        }
    }
    float *dst = gx + ((int64_t)c * Hs + Y) * Ws + X0;
    if ((Ws & 3) == 0) {
        float4 r = make_float4(v[0], v[1], v[2], v[3]);
        if (acc) {
            const float4 o = *reinterpret_cast<const float4 *>(dst);
            r = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
        }
        *reinterpret_cast<float4 *>(dst) = r;
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (X0 + e < Ws) dst[e] = acc ? dst[e] + v[e] : v[e];
    }
}

// ga (nullable) / gb (nullable): gather the output gradient back (zeros outside the crop;
// the 2x2 children of an upsampled b pixel are summed); accumulate flags per input
__global__ void k_concat_bwd(const float *__restrict__ go, CatGeom g, float *__restrict__ ga, int acc_a,
                             float *__restrict__ gb, int acc_b) {
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t na = ga ? (int64_t)g.Ca * g.Ha * g.Wa : 0;
    const int64_t nb = gb ? (int64_t)g.Cb * g.Hb * g.Wb : 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i < na) {
            const int64_t hw = (int64_t)g.Ha * g.Wa;
            const int c = (int)(i / hw);
            const int p = (int)(i - (int64_t)c * hw);
            const int y = p / g.Wa - g.oay, x = p % g.Wa - g.oax;
            float v = 0.0f;
            if (y >= 0 && y < g.H && x >= 0 && x < g.W) v = go[(int64_t)c * HW + (int64_t)y * g.W + x];
            ga[i] = acc_a ? ga[i] + v : v;
        } else {
            const int64_t j = i - na;
            const int64_t hw = (int64_t)g.Hb * g.Wb;
            const int c = (int)(j / hw);
            const int p = (int)(j - (int64_t)c * hw);
            const int Y = p / g.Wb, X = p % g.Wb;
            const float *gc = go + (int64_t)(g.Ca + c) * HW;
            float v = 0.0f;
            const int f = g.upb ? 2 : 1;
            for (int dy = 0; dy < f; ++dy)
                for (int dx = 0; dx < f; ++dx) {
                    const int y = Y * f + dy - g.oby, x = X * f + dx - g.obx;
                    if (y >= 0 && y < g.H && x >= 0 && x < g.W) v += gc[(int64_t)y * g.W + x];
                }
            gb[j] = acc_b ? gb[j] + v : v;
        }
    }
}

}  // namespace lrs
