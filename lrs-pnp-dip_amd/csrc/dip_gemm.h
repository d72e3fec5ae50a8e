// Split-bf16 GEMM and implicit-GEMM convolution for the DIP engine (gfx950).
//
// C[M][N] = op(A)[M][K] op(B)[K][N] in fp32 accuracy on the bf16 matrix cores: every fp32 operand
// value is split exactly into three bf16 terms (hi + mid + lo, the remainder after lo is below
// 2^-24 relative) ONCE, when its tile is written to LDS, and each 16x16 output tile accumulates
// the six partial products with i + j <= 2 (A_lo B_hi, A_mid B_mid, A_hi B_lo, A_mid B_hi,
// A_hi B_mid, A_hi B_hi; smallest first) with v_mfma_f32_16x16x32_bf16 into fp32.
//
// Tile: 128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64 = 4 x 4 MFMA tiles), 32 k
// per step.  LDS holds the three bf16 planes of both operands k-contiguous, 64 B rows with the
// 16-B chunk index XOR-swizzled by (row >> 2) & 3, so a lane's 8-k fragment is one conflict-free
// ds_read_b128.  One LDS stage, the next step's global loads in registers during the MFMAs,
// 2-3 workgroups per CU.  gridDim.z > 1 = split-K as in k_gemm.
//
// Operands come from loaders: dense matrices, or the implicit im2col of a conv (reflection /
// zero padding, stride and the nearest x2 upsample folded into the gather), so the forward and
// the weight gradient of a conv never materialise the col matrix (the reference's
// ReflectionPad2d + Conv2d, lipschitz_constraint_layer.py:65-78, common.py:73-121).
#pragma once

#include "lrs_dip.h"

namespace lrs {

constexpr int kS3K = 32;
typedef __bf16 s3bf8 __attribute__((ext_vector_type(8)));
typedef float s3f4 __attribute__((ext_vector_type(4)));

// LDS image of one operand: [plane][row 0..127][32 k] bf16, chunk (8 k) swizzled per row
struct S3Tile {
    __bf16 v[3][128][kS3K];
};

__device__ __forceinline__ int s3_chunk(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// thread -> (row, first k) of the 16 values it loads per step:
//  KC (operand stored k-contiguous): row = t / 2, k = 16 (t & 1) + 0..15
//  else (stored row-contiguous)    : row = t & 127, k = 16 (t >> 7) + 0..15
// (measured: a 2-k x 8-row KC arrangement with 16 lanes per row is slower, 2-20 %)
template <bool KC>
__device__ __forceinline__ int s3_row() { return KC ? (threadIdx.x >> 1) : (threadIdx.x & 127); }
template <bool KC>
__device__ __forceinline__ int s3_kb() { return KC ? 16 * (threadIdx.x & 1) : 16 * (threadIdx.x >> 7); }

struct S3Split {
    __bf16 b0, b1, b2;
};
__device__ __forceinline__ S3Split s3_split(float x) {
    S3Split r;
    r.b0 = (__bf16)x;
    const float r1 = x - (float)r.b0;
    r.b1 = (__bf16)r1;
    r.b2 = (__bf16)(r1 - (float)r.b1);
    return r;
}

template <bool KC>
__device__ __forceinline__ void s3_store(S3Tile &T, const float (&v)[16]) {
    const int row = s3_row<KC>(), c0 = s3_kb<KC>() >> 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        s3bf8 p0, p1, p2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const S3Split q = s3_split(v[8 * h + e]);
            p0[e] = q.b0;
            p1[e] = q.b1;
            p2[e] = q.b2;
        }
        const int ch = s3_chunk(row, c0 + h) * 8;
        *reinterpret_cast<s3bf8 *>(&T.v[0][row][ch]) = p0;
        *reinterpret_cast<s3bf8 *>(&T.v[1][row][ch]) = p1;
        *reinterpret_cast<s3bf8 *>(&T.v[2][row][ch]) = p2;
    }
}

__device__ __forceinline__ void s3_frag(const S3Tile &T, int row, int gk, s3bf8 (&f)[3]) {
    const int ch = s3_chunk(row, gk) * 8;
#pragma unroll
    for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const s3bf8 *>(&T.v[p][row][ch]);
}

__device__ __forceinline__ s3f4 s3_mfma6(const s3bf8 (&A)[3], const s3bf8 (&B)[3], s3f4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], acc, 0, 0, 0);
    return acc;
}

// ---- loaders ---------------------------------------------------------------------------------
// Each provides: static constexpr bool kc; setup(x0, smem) once per workgroup (before the first
// barrier); load(x0, k0, kend, v) the thread's 16 values of the step starting at k0 (zero past
// kend or past the operand's row count).

// Dense operand: KC = stored [x][k] (leading dimension ld), else stored [k][x].
template <bool KC>
struct LdDense {
    static constexpr bool kc = KC;
    const float *S;
    int ld, X;
    __device__ __forceinline__ void setup(int, int *) {}
    __device__ __forceinline__ void load(int x0, int k0, int kend, float (&v)[16]) const {
        const int x = x0 + s3_row<KC>(), kb = k0 + s3_kb<KC>();
        if (KC) {
            const float *src = S + (int64_t)x * ld + kb;
            if (x < X && kb + 16 <= kend && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 f = *reinterpret_cast<const float4 *>(src + 4 * q);
                    v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
                }
            } else {
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = (x < X && kb + u < kend) ? src[u] : 0.0f;
            }
        } else {
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = (x < X && kb + u < kend) ? S[(int64_t)(kb + u) * ld + x] : 0.0f;
        }
    }
};

// source index of padded / upsampled coordinate u (extent n upsampled), -1 for a zero pad
__device__ __forceinline__ int conv_src(int u, int n, int mode, int up) {
    if (mode == LRS_PAD_REFLECT) {
        u = u < 0 ? -u : u;
        u = u >= n ? 2 * (n - 1) - u : u;
    } else if (u < 0 || u >= n) {
        return -1;
    }
    return up ? (u >> 1) : u;
}

// Forward B operand: col[r][p] with r = (c, ky, kx) the k index and p = output pixel the x
// index (stored "[k][x]").  The k*k source offsets of the workgroup's 128 pixels are tabulated
// in LDS once; a step then costs one table read + one gather per value.
struct LdConvFwd {
    static constexpr bool kc = false;
    const float *X;
    ConvGeom g;
    int *tab;   // [k*k][128] source offset in a channel plane, -1 = zero pad / past P
    __device__ __forceinline__ void setup(int x0, int *smem) {
        tab = smem;
        const int kk = g.k * g.k, P = g.Ho * g.Wo;
        for (int i = threadIdx.x; i < kk * 128; i += blockDim.x) {
            const int kyx = i >> 7, p = x0 + (i & 127);
            int o = -1;
            if (p < P) {
                const int oy = p / g.Wo, ox = p - oy * g.Wo, ky = kyx / g.k, kx = kyx - ky * g.k;
                const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
                const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
                if (sy >= 0 && sx >= 0) o = sy * g.Ws + sx;
            }
            tab[i] = o;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int x = s3_row<false>(), r0 = k0 + s3_kb<false>();
        const int kk = g.k * g.k, plane = g.Hs * g.Ws;
        int c = r0 / kk, kyx = r0 - c * kk;
        const float *base = X + (int64_t)c * plane;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int o = tab[kyx * 128 + x];
            v[u] = (r0 + u < kend && o >= 0) ? base[o] : 0.0f;
            if (++kyx == kk) {
                kyx = 0;
                base += plane;
            }
        }
    }
};

// Data-gradient operands (stride 1): gxp[ci][q] over the padded, upsampled domain
// q = (iy, ix) in [0, Hu + 2 pad) x [0, Wu + 2 pad) is the correlation of gy with the kernel,
//   gxp[ci][iy][ix] = sum_{co, ky, kx} W[co][ci][ky][kx] gy[co][iy - ky][ix - kx],
// an implicit GEMM with M = Cin, K = (co, ky, kx), N = q; k_fold_pad then adds the padded
// border back onto the pixels it mirrors and sums the x2 upsample (the adjoint of the gather
// of LdConvFwd), so no Kc x P col gradient is ever written.
// A: W^T, row ci, k index (co, kyx) -> W[co][ci][kyx]
struct LdWT {
    static constexpr bool kc = true;
    const float *W;
    int Cin, kk;
    __device__ __forceinline__ void setup(int, int *) {}
    __device__ __forceinline__ void load(int x0, int k0, int kend, float (&v)[16]) const {
        const int ci = x0 + s3_row<true>(), kb = k0 + s3_kb<true>();
        int co = kb / kk, kyx = kb - co * kk;
        const int Kc = Cin * kk;
        const float *src = W + (int64_t)co * Kc + ci * kk;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            v[u] = (ci < Cin && kb + u < kend) ? src[kyx] : 0.0f;
            if (++kyx == kk) {
                kyx = 0;
                src += Kc;
            }
        }
    }
};

// B: gy gathered at (iy - ky, ix - kx); k index (co, kyx), x index q.  Offsets per (kyx, q) of
// the workgroup's 128 q tabulated once, as in LdConvFwd.
struct LdConvDgrad {
    static constexpr bool kc = false;
    const float *GY;
    ConvGeom g;
    int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem) {
        tab = smem;
        const int kk = g.k * g.k, Wp = g.Wu + 2 * g.pad, Q = (g.Hu + 2 * g.pad) * Wp;
        for (int i = threadIdx.x; i < kk * 128; i += blockDim.x) {
            const int kyx = i >> 7, q = x0 + (i & 127);
            int o = -1;
            if (q < Q) {
                const int iy = q / Wp, ix = q - iy * Wp, ky = kyx / g.k, kx = kyx - ky * g.k;
                const int oy = iy - ky, ox = ix - kx;
                if (oy >= 0 && oy < g.Ho && ox >= 0 && ox < g.Wo) o = oy * g.Wo + ox;
            }
            tab[i] = o;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int x = s3_row<false>(), r0 = k0 + s3_kb<false>();
        const int kk = g.k * g.k, plane = g.Ho * g.Wo;
        int c = r0 / kk, kyx = r0 - c * kk;
        const float *base = GY + (int64_t)c * plane;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int o = tab[kyx * 128 + x];
            v[u] = (r0 + u < kend && o >= 0) ? base[o] : 0.0f;
            if (++kyx == kk) {
                kyx = 0;
                base += plane;
            }
        }
    }
};

// Weight-gradient B operand: col^T, x index r = (c, ky, kx) (an output column of dW), k index p
// = output pixel (stored "[x][k]").  A thread's row r is fixed for the whole kernel; the source
// offsets of the step's 32 pixels for every (ky, kx) are tabulated in LDS one step ahead
// (prepare(), double-buffered), so a value costs one table read and one gather.
struct LdConvWgrad {
    static constexpr bool kc = true;
    static constexpr bool kPrepare = true;
    const float *X;
    ConvGeom g;
    int Kc;
    int *tab;   // [2][k*k][32]
    __device__ __forceinline__ void setup(int, int *smem) { tab = smem; }
    // table of the step starting at k0 into buffer b
    __device__ __forceinline__ void prepare(int k0, int kend, int b) const {
        const int kk = g.k * g.k;
        for (int i = threadIdx.x; i < kk * 32; i += blockDim.x) {
            const int kyx = i >> 5, p = k0 + (i & 31);
            int o = -1;
            if (p < kend) {
                const int oy = p / g.Wo, ox = p - oy * g.Wo, ky = kyx / g.k, kx = kyx - ky * g.k;
                const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
                const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
                if (sy >= 0 && sx >= 0) o = sy * g.Ws + sx;
            }
            tab[b * 9 * 32 + i] = o;
        }
    }
    __device__ __forceinline__ void load(int x0, int k0, int kend, float (&v)[16], int b) const {
        const int r = x0 + s3_row<true>(), kb = s3_kb<true>();
        const int kk = g.k * g.k;
        const int c = r / kk, kyx = r - c * kk;
        const float *pl = X + (int64_t)c * g.Hs * g.Ws;
        const int *t = tab + b * 9 * 32 + (r < Kc ? kyx : 0) * 32 + kb;
        int o[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 f = *reinterpret_cast<const int4 *>(t + 4 * q);
            o[4 * q] = f.x; o[4 * q + 1] = f.y; o[4 * q + 2] = f.z; o[4 * q + 3] = f.w;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = (r < Kc && o[u] >= 0) ? pl[o[u]] : 0.0f;
    }
};

template <class L>
struct HasPrepare {
    static constexpr bool value = false;
};
template <>
struct HasPrepare<LdConvWgrad> {
    static constexpr bool value = true;
};

constexpr int kS3TabInts = 9 * 128;   // k <= 3

template <class LA, class LB>
__global__ __launch_bounds__(256, 2) void k_gemm_s3(GemmArgs g, LA la, LB lb) {
    __shared__ __attribute__((aligned(16))) S3Tile As, Bs;
    __shared__ __attribute__((aligned(16))) int tab[kS3TabInts];
    const int m0 = blockIdx.y * 128, n0 = blockIdx.x * 128;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    constexpr bool PREP = HasPrepare<LB>::value;
    la.setup(m0, tab);
    lb.setup(n0, tab);
    if constexpr (PREP) lb.prepare(kbeg, kend, 0);
    __syncthreads();
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    float va[16], vb[16];
    la.load(m0, kbeg, kend, va);
    if constexpr (PREP) lb.load(n0, kbeg, kend, vb, 0);
    else lb.load(n0, kbeg, kend, vb);
    int tb = 0;
    for (int k0 = kbeg; k0 < kend; k0 += kS3K) {
        s3_store<LA::kc>(As, va);
        s3_store<LB::kc>(Bs, vb);
        if constexpr (PREP) {
            if (k0 + kS3K < kend) lb.prepare(k0 + kS3K, kend, tb ^ 1);
        }
        __syncthreads();
        if (k0 + kS3K < kend) {
            la.load(m0, k0 + kS3K, kend, va);
            if constexpr (PREP) lb.load(n0, k0 + kS3K, kend, vb, tb ^ 1);
            else lb.load(n0, k0 + kS3K, kend, vb);
        }
        tb ^= 1;
        s3bf8 fb[4][3];
#pragma unroll
        for (int b = 0; b < 4; ++b) s3_frag(Bs, wn + 16 * b + jl, gk, fb[b]);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            s3bf8 fa[3];
            s3_frag(As, wm + 16 * a + jl, gk, fa);
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = s3_mfma6(fa, fb[b], acc[a][b]);
        }
        __syncthreads();
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

// gx[c][sy][sx] (+)= sum over the x2 upsample children u of sum over the padded positions that
// read u (direct + reflection mirrors, padded_sources) of gxp[c][iy][ix]
__global__ __launch_bounds__(256) void k_fold_pad(const float *__restrict__ gxp, ConvGeom gm, float *__restrict__ gx,
                                                  int accum) {
    const int HW = gm.Hs * gm.Ws, Wp = gm.Wu + 2 * gm.pad, Qp = (gm.Hu + 2 * gm.pad) * Wp;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= HW) return;
    const int sy = q / gm.Ws, sx = q - sy * gm.Ws;
    const int nup = gm.up ? 2 : 1;
    for (int c = blockIdx.y; c < gm.Cin; c += gridDim.y) {
        const float *src = gxp + (int64_t)c * Qp;
        float acc = 0.0f;
        for (int a = 0; a < nup; ++a) {
            int iys[3];
            const int ny = padded_sources(gm.up ? 2 * sy + a : sy, gm.Hu, gm.pad, gm.pad_mode, iys);
            for (int b = 0; b < nup; ++b) {
                int ixs[3];
                const int nx = padded_sources(gm.up ? 2 * sx + b : sx, gm.Wu, gm.pad, gm.pad_mode, ixs);
                for (int py = 0; py < ny; ++py)
                    for (int px = 0; px < nx; ++px) acc += src[iys[py] * Wp + ixs[px]];
            }
        }
        const int64_t i = (int64_t)c * HW + q;
        gx[i] = accum ? gx[i] + acc : acc;
    }
}

}  // namespace lrs
