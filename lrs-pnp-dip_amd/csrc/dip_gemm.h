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
// 16-B chunk index XOR-swizzled by (row >> 1) & 3, so a lane's 8-k fragment is one conflict-free
// ds_read_b128.  One LDS stage, the next step's global loads in registers during the MFMAs,
// 2-3 workgroups per CU.  gridDim.z > 1 = split-K as in k_gemm.
//
// Operands come from loaders: dense fp32 matrices (split at the LDS store), conv weights
// pre-split into bf16 planes once per step (k_wprep: no split work in the GEMM), or the implicit
// im2col of a conv (reflection / zero padding, stride and the nearest x2 upsample folded into
// LDS offset tables, buffer loads with range-checked zero fill), so no conv direction
// materialises a col matrix (the reference's ReflectionPad2d + Conv2d,
// lipschitz_constraint_layer.py:65-78, common.py:73-121).
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

// chunk ^ ((row >> 1) & 3): conflict-free for the CDNA4 LDS lane groups (MI355X_MICROARCH.md §LDS)
// of both sides -- the fragment reads (ds_read_b128: groups {0-3,12-15,20-27}, ... of 16 lanes over
// 64 banks: rows base + (l & 15), chunk l >> 4) and the tile stores (ds_write_b128: 8 contiguous
// lanes over 32 banks: 8 consecutive rows at one chunk, or 4 rows x 2 chunks).  The previous
// (row >> 2) & 3 was conflict-free only for 16-lane groups {0-15}, ...: measured 8.3M bank-conflict
// cycles per 196^2 forward conv launch (SQ_LDS_BANK_CONFLICT).  Found by exhaustive search over
// f(row mod 16) (tools: DESIGN.md §4).
__device__ __forceinline__ int s3_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 3); }

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
#ifdef LRS_S3_CHEAPSPLIT   // timing experiment only (wrong products): the split's VALU cost
    r.b1 = r.b0;
    r.b2 = r.b0;
    return r;
#endif
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
// Each provides: static constexpr bool kc; setup(x0, smem, cls) once per workgroup (before the first
// barrier); load(x0, k0, kend, v) the thread's 16 values of the step starting at k0 (zero past
// kend or past the operand's row count).

// Dense operand: KC = stored [x][k] (leading dimension ld), else stored [k][x].
template <bool KC>
struct LdDense {
    static constexpr bool kc = KC;
    static constexpr bool pre = false;
    const float *S;
    int ld, X;
    __device__ __forceinline__ void setup(int, int *, int) {}
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
__host__ __device__ __forceinline__ int conv_src(int u, int n, int mode, int up) {
    if (mode == LRS_PAD_REFLECT) {
        u = u < 0 ? -u : u;
        u = u >= n ? 2 * (n - 1) - u : u;
    } else if (u < 0 || u >= n) {
        return -1;
    }
    return up ? (u >> 1) : u;
}

// ---- implicit-GEMM conv operands --------------------------------------------------------------
// The tap tables below are built by k_gemm_s3's 256 threads as thread t -> table column t & 127 (the
// workgroup's pixel), taps t >> 7, t >> 7 + 2, ...: the pixel's coordinates take one division per
// thread, a tap's (ky, kx) none (k <= 4, the effective 4 x 4 data-gradient kernel included; the
// per-entry divisions cost ~1.8 us per workgroup).
__device__ __forceinline__ int s3_tap_y(int kyx, int k) {
    return kyx >= 3 * k ? 3 : (kyx >= 2 * k ? 2 : (kyx >= k ? 1 : 0));
}
// The conv's K index is tap-major, r = kyx * Cp + c (kyx = ky * k + kx, c < Cp = Cin rounded up to
// 16, channels >= Cin are zero), so the 16 consecutive k a thread loads share one tap: their
// source offset is one LDS table entry and the 16 channels are a scalar stride apart.  Sources
// are read through buffer loads (32-bit offsets, range-checked): a table entry kOob marks a zero
// pad / out-of-range pixel and the hardware returns 0 for it, so no per-value select remains.
constexpr int kOob = 0x7FFFFFF0;   // >= every buffer's byte count (host checks < kOob)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t s3_rsrc(const void *p, int bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const void *u = reinterpret_cast<const void *>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(u), 0, __builtin_amdgcn_readfirstlane(bytes),
                                             0x00020000);
}

__device__ __forceinline__ float s3_bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// The NV channel planes c0 .. c0 + NV - 1 (plane stride pb bytes) at one tap's offsets vo, without a
// branch or a mask: every load is issued, a channel c >= nc reads channel nc - 1.  The values that
// are not the operand's -- padding channels, and the k groups past a split's end (whose callers
// read tap 0) -- meet zero weights: every implicit-GEMM B loader is paired with LdPre, whose planes
// are zero at ci >= Cin (co >= Cout) and which reads zeros past kend, so they add exact zeros.
// Written as "c < nc ? load : 0" (or with a mask applied to the loaded bits) the compiler branched
// around each load or waited for it right away, and its wait-count pass, meeting paths with
// different loads in flight at the GEMM's loop head, drained them all there (s_waitcnt vmcnt(0)
// every k-step: the prefetch two steps ahead was lost; tools/micro/gemm_phase).
template <int NV>
__device__ __forceinline__ void s3_bload_chans(__amdgpu_buffer_rsrc_t r, int vo, int c0, int nc, int pb, float (&v)[NV]) {
#pragma unroll
    for (int u = 0; u < NV; ++u) v[u] = s3_bload(r, vo, min(c0 + u, nc - 1) * pb);
}

// Pre-split operand (the conv weights, split into bf16 planes by k_wprep): plane p of row x at
// P + p * pstride + x * ld, k contiguous.  Loads go straight to the LDS image (no split).
struct RegP {
    uint4 h[3][2];
};

struct LdPre {
    static constexpr bool kc = true;
    static constexpr bool pre = true;
    const __bf16 *P;
    int64_t pstride;
    int ld, X;
    int64_t cstride = 0;   // parity-class GEMMs: class cls reads the planes at P + cls * cstride
    __device__ __forceinline__ void setup(int, int *, int cls) { P += cls * cstride; }
    // buffer loads, branch-free (s3_bload_chans): a row past X or a k group past kend reads at kOob
    // (zeros); the planes' bytes are < kOob (k_conv_prep's 2^31 / 3 element limit)
    __device__ __forceinline__ void load(int x0, int k0, int kend, RegP &r) const {
        const int x = x0 + s3_row<true>(), kb = k0 + s3_kb<true>();
        const bool ok = x < X && kb < kend;   // K and kend are multiples of 16
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(P, (int)(6 * pstride));
        const int vo = ok ? 2 * (x * ld + kb) : kOob;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            r.h[p][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (int)(2 * p * pstride), 0));
            r.h[p][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (int)(2 * p * pstride) + 16, 0));
        }
    }
};

__device__ __forceinline__ void s3_store_pre(S3Tile &T, const RegP &r) {
    const int row = s3_row<true>(), c0 = s3_kb<true>() >> 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch = s3_chunk(row, c0 + h) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4 *>(&T.v[p][row][ch]) = r.h[p][h];
    }
}

// Forward B: col[r][p] (k = r tap-major, x = output pixel p).  Table [kk][128] of the
// workgroup's pixels' source byte offsets within a channel plane.
struct LdFwdTM {
    static constexpr bool kc = false;
    static constexpr bool pre = false;
    const float *X;
    int xbytes;
    ConvGeom g;
    int Cp;
    int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem, int) {
        tab = smem;
        const int kk = g.k * g.k, r = threadIdx.x & 127, p = x0 + r;
        const bool in = p < g.Ho * g.Wo;
        const int oy = in ? p / g.Wo : 0, ox = p - oy * g.Wo;
        for (int kyx = threadIdx.x >> 7; kyx < kk; kyx += 2) {
            const int ky = s3_tap_y(kyx, g.k), kx = kyx - ky * g.k;
            const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
            const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
            tab[kyx * 128 + r] = (in && sy >= 0 && sx >= 0) ? 4 * (sy * g.Ws + sx) : kOob;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + s3_kb<false>());
        const int rr = r0 < kend ? r0 : 0,   // past the chunk: tap 0 (meets zero weights)
                  kyx = rr / Cp, c0 = rr - kyx * Cp;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, xbytes);
        s3_bload_chans(rs, tab[kyx * 128 + s3_row<false>()], c0, g.Cin, g.Hs * g.Ws * 4, v);
    }
};

// Data-gradient B (stride 1): gy at (iy - ky, ix - kx) over the padded, upsampled domain
// q = (iy, ix); k = kyx * Cop + co.  Table [kk][128] of the workgroup's q.
struct LdDgradTM {
    static constexpr bool kc = false;
    static constexpr bool pre = false;
    const float *GY;
    int gbytes;
    ConvGeom g;
    int Cout, Cop;
    int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem, int) {
        tab = smem;
        const int kk = g.k * g.k, Wp = g.Wu + 2 * g.pad, r = threadIdx.x & 127, q = x0 + r;
        const bool in = q < (g.Hu + 2 * g.pad) * Wp;
        const int iy = in ? q / Wp : 0, ix = q - iy * Wp;
        for (int kyx = threadIdx.x >> 7; kyx < kk; kyx += 2) {
            const int ky = s3_tap_y(kyx, g.k), kx = kyx - ky * g.k;
            const int oy = iy - ky, ox = ix - kx;
            tab[kyx * 128 + r] = (in && oy >= 0 && oy < g.Ho && ox >= 0 && ox < g.Wo) ? 4 * (oy * g.Wo + ox) : kOob;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + s3_kb<false>());
        const int rr = r0 < kend ? r0 : 0, kyx = rr / Cop, c0 = rr - kyx * Cop;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(GY, gbytes);
        s3_bload_chans(rs, tab[kyx * 128 + s3_row<false>()], c0, Cout, g.Ho * g.Wo * 4, v);
    }
};

// Lane-per-pixel staging of a weight gradient's col^T tile (128 rows r x 32 pixels per k-step):
// wave w owns rows 32 w .. 32 w + 31, lane l pixel l & 31 of rows 32 w + 2 u + (l >> 5), u < 16, so
// each load instruction reads 2 x 32 consecutive pixels of one channel plane (coalesced), and the
// values go to the row-major LDS image as single bf16 writes.  Rows = (channel, tap) pairs, ntap
// taps per channel; tab = the step's [ntap][32] source offsets (kOob = zero).
__device__ __forceinline__ int wlp_row(int u) { return 32 * (threadIdx.x >> 6) + 2 * u + ((threadIdx.x >> 5) & 1); }

__device__ __forceinline__ void wlp_load(const float *X, int xbytes, int plane_bytes, int nrows, int ntap, int x0,
                                         const int *tab, float (&v)[16]) {
    const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, xbytes);
    const int pl = threadIdx.x & 31;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int r = x0 + wlp_row(u), c = r / ntap, tap = r - c * ntap;
        v[u] = s3_bload(rs, tab[tap * 32 + pl] + (r < nrows ? c * plane_bytes : kOob), 0);
    }
}

__device__ __forceinline__ void wlp_store(S3Tile &T, const float (&v)[16]) {
    const int k = threadIdx.x & 31;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int row = wlp_row(u), at = s3_chunk(row, k >> 3) * 8 + (k & 7);
        const S3Split q = s3_split(v[u]);
        T.v[0][row][at] = q.b0;
        T.v[1][row][at] = q.b1;
        T.v[2][row][at] = q.b2;
    }
}

// Weight-gradient B: col^T, x = r = c * kk + kyx (dW's own column order: a wave's 32 rows are
// ~4 channels x all taps, whose gathers share cache lines), k = output pixel.  The thread's row
// is fixed; the step's 32 pixels x kk taps are tabulated one step ahead (prepare,
// double-buffered).  Rows past Cin * kk read at kOob (zeros).
struct LdWgradTM {
    static constexpr bool kc = true;
    static constexpr bool pre = false;
    static constexpr bool lanepix = true;   // wlp_load / wlp_store (coalesced gathers)
    const float *X;
    int xbytes;
    ConvGeom g;
    int *tab;   // [2][kk][32]
    int x0;
    __device__ __forceinline__ void setup(int x0_, int *smem, int) {
        tab = smem;
        x0 = x0_;
    }
    __device__ __forceinline__ void prepare(int k0, int kend, int b) const {
        const int kk = g.k * g.k;
        for (int i = threadIdx.x; i < kk * 32; i += blockDim.x) {
            const int kyx = i >> 5, p = k0 + (i & 31);
            int o = kOob;
            if (p < kend) {
                const int oy = p / g.Wo, ox = p - oy * g.Wo, ky = kyx / g.k, kx = kyx - ky * g.k;
                const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
                const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
                if (sy >= 0 && sx >= 0) o = 4 * (sy * g.Ws + sx);
            }
            tab[b * 9 * 32 + i] = o;
        }
    }
    __device__ __forceinline__ void load(int, int, int, float (&v)[16], int b) const {
        wlp_load(X, xbytes, g.Hs * g.Ws * 4, g.Cin * g.k * g.k, g.k * g.k, x0, tab + b * 9 * 32, v);
    }
};

// ---- upsampled 3 x 3 convs by output parity class -------------------------------------------
// conv3x3(ReflectionPad2d(1)(Upsample2x(x))) (my_Lipschitz_Unet.py:83-94): output pixel
// (2a + i, 2b + j) reads source rows clamp(a + ey + i - 1), ey in {0, 1}, through the tap sets
// T(i, ey) = {0} {1, 2} (i = 0) or {0, 1} {2} (i = 1), and likewise the columns: the reflection of the
// upsampled border is a clamp on the source grid.  Per class the conv is a 2 x 2 conv of x with
// summed ("effective") weights (k_conv_prep's upc planes): 16 / 9 of the taps of one class, so the
// four classes cost 4 / 9 of the direct product over the upsampled grid.

__device__ __forceinline__ int clampi(int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }

// Forward B of class cls = 2 i + j: col[e * Cp + c][n], n = source pixel (a, b), e = 2 ey + ex:
// x[c] at (clamp(a + ey + i - 1), clamp(b + ex + j - 1)).  Table [4][128].
struct LdUpFwdTM {
    static constexpr bool kc = false;
    static constexpr bool pre = false;
    const float *X;
    int xbytes;
    ConvGeom g;
    int Cp;
    int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem, int cls) {
        tab = smem;
        const int i = cls >> 1, j = cls & 1, r = threadIdx.x & 127, n = x0 + r;
        const bool in = n < g.Hs * g.Ws;
        const int a = in ? n / g.Ws : 0, b = n - a * g.Ws;
        for (int e = threadIdx.x >> 7; e < 4; e += 2)
            tab[e * 128 + r] = in ? 4 * (clampi(a + (e >> 1) + i - 1, g.Hs) * g.Ws + clampi(b + (e & 1) + j - 1, g.Ws)) : kOob;
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + s3_kb<false>());
        const int rr = r0 < kend ? r0 : 0, e = rr / Cp, c0 = rr - e * Cp;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, xbytes);
        s3_bload_chans(rs, tab[e * 128 + s3_row<false>()], c0, g.Cin, g.Hs * g.Ws * 4, v);
    }
};

// Data-gradient B of the same conv over the source grid extended by one pixel on each side
// (n = (qy + 1)(Ws + 2) + qx + 1, qy in [-1, Hs], qx in [-1, Ws]; k_fold_pad in kPadClamp mode adds
// the outside ring back onto the border): k = (4 cls + e) Cop + co, dL/dz[co] at
// (2a + i, 2b + j) with a = qy - ey - i + 1, b = qx - ex - j + 1 when inside.  Table [16][128].
struct LdUpDgradTM {
    static constexpr bool kc = false;
    static constexpr bool pre = false;
    const float *GY;
    int gbytes;
    ConvGeom g;
    int Cout, Cop;
    int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem, int) {
        tab = smem;
        const int We = g.Ws + 2, r = threadIdx.x & 127, n = x0 + r;
        const bool in = n < (g.Hs + 2) * We;
        const int qy = (in ? n / We : 0) - 1, qx = n - (qy + 1) * We - 1;
        for (int ce = threadIdx.x >> 7; ce < 16; ce += 2) {
            const int cl = ce >> 2, e = ce & 3, i = cl >> 1, j = cl & 1;
            const int a = qy - (e >> 1) - i + 1, b = qx - (e & 1) - j + 1;
            tab[ce * 128 + r] = (in && a >= 0 && a < g.Hs && b >= 0 && b < g.Ws) ? 4 * ((2 * a + i) * g.Wo + 2 * b + j) : kOob;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, float (&v)[16]) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + s3_kb<false>());
        const int rr = r0 < kend ? r0 : 0, ce = rr / Cop, c0 = rr - ce * Cop;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(GY, gbytes);
        s3_bload_chans(rs, tab[ce * 128 + s3_row<false>()], c0, Cout, g.Ho * g.Wo * 4, v);
    }
};

// Weight gradient of the same conv by output parity class cls (gridDim.z = 4 classes x split-K):
// dWE_cls[co][c * 4 + e] = sum over source pixels (a, b) of dL/dz[co] at (2a + i, 2b + j) times x[c]
// at (clamp(a + ey + i - 1), clamp(b + ex + j - 1)); the classes are stacked in the output
// ([split][cls][Cout][4 Cin], GemmArgs cls_wo = 0) and k_upc_wgrad_combine sums them into dW.
// A: dL/dz at the class's output pixels, k = source pixel (16 consecutive per thread).
struct LdGzCls {
    static constexpr bool kc = true;
    static constexpr bool pre = false;
    static constexpr bool lanepix = true;   // lane = source pixel (wlp_store), as the col^T side
    const float *GZ;
    int Hs, Ws, Wo, M;
    int cls;
    __device__ __forceinline__ void setup(int, int *, int c) { cls = c; }
    __device__ __forceinline__ void load(int x0, int k0, int kend, float (&v)[16]) const {
        const int k = k0 + (threadIdx.x & 31), i = cls >> 1, j = cls & 1;
        const int a = k / Ws, b = k - a * Ws;
        const int po = (2 * a + i) * Wo + 2 * b + j;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(GZ, M * 4 * Hs * Ws * 4);
        // the row offset differs between the wave's two halves: in the VGPR offset, not the SGPR one
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int row = x0 + wlp_row(u);
            v[u] = s3_bload(rs, (k < kend && row < M) ? 4 * po + row * (4 * Hs * Ws * 4) : kOob, 0);
        }
    }
};

// B: col^T of the class, x = r = c * 4 + e, k = source pixel; the step's 32 pixels x 4 taps
// tabulated one step ahead (double-buffered, as LdWgradTM).
struct LdWgradCls {
    static constexpr bool kc = true;
    static constexpr bool pre = false;
    static constexpr bool lanepix = true;
    const float *X;
    int xbytes;
    ConvGeom g;
    int *tab;   // [2][4][32]
    int x0, cls;
    __device__ __forceinline__ void setup(int x0_, int *smem, int c) {
        tab = smem;
        x0 = x0_;
        cls = c;
    }
    __device__ __forceinline__ void prepare(int k0, int kend, int b) const {
        const int i = cls >> 1, j = cls & 1;
        for (int idx = threadIdx.x; idx < 4 * 32; idx += blockDim.x) {
            const int e = idx >> 5, p = k0 + (idx & 31);
            int o = kOob;
            if (p < kend) {
                const int a = p / g.Ws, bb = p - a * g.Ws;
                o = 4 * (clampi(a + (e >> 1) + i - 1, g.Hs) * g.Ws + clampi(bb + (e & 1) + j - 1, g.Ws));
            }
            tab[b * 4 * 32 + idx] = o;
        }
    }
    __device__ __forceinline__ void load(int, int, int, float (&v)[16], int b) const {
        wlp_load(X, xbytes, g.Hs * g.Ws * 4, 4 * g.Cin, 4, x0, tab + b * 4 * 32, v);
    }
};

// dW[co][c][ky][kx] = (sum over the 4 classes of dWE_cls[co][c * 4 + e(cls, ky, kx)], each summed over
// the nsplit splits in k_gemm_reduce's order) / *div: the chain rule through upc_weight's sums.
__global__ void k_upc_wgrad_combine(const float *__restrict__ part, int nsplit, int Cout, int Cin,
                                    const float *div, float *__restrict__ gw) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = (int64_t)Cout * Cin * 9;
    if (idx >= n) return;
    const int tap = (int)(idx % 9), c = (int)((idx / 9) % Cin), co = (int)(idx / (9 * (int64_t)Cin));
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int64_t MN = (int64_t)Cout * 4 * Cin;
    float tot = 0.0f;
    for (int cl = 0; cl < 4; ++cl) {
        const int i = cl >> 1, j = cl & 1;
        const int ey = i == 0 ? (ky == 0 ? 0 : 1) : (ky == 2 ? 1 : 0), ex = j == 0 ? (kx == 0 ? 0 : 1) : (kx == 2 ? 1 : 0);
        const int64_t off = (int64_t)cl * MN + (int64_t)co * 4 * Cin + c * 4 + 2 * ey + ex;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int z0 = 0; z0 < nsplit; z0 += 8) {
            float p[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) p[e] = z0 + e < nsplit ? part[(int64_t)(z0 + e) * 4 * MN + off] : 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (z0 + e < nsplit) acc[e] += p[e];
        }
        tot = tot + (((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7])));
    }
    if (div) tot = tot / *div;
    gw[idx] = tot;
}

template <class L>
struct HasPrepare {
    static constexpr bool value = false;
};
template <class L, class = void>
struct LanePix {
    static constexpr bool value = false;
};
template <class L>
struct LanePix<L, std::void_t<decltype(L::lanepix)>> {
    static constexpr bool value = L::lanepix;
};

template <>
struct HasPrepare<LdWgradTM> {
    static constexpr bool value = true;
};
template <>
struct HasPrepare<LdWgradCls> {
    static constexpr bool value = true;
};

constexpr int kS3TabInts = 16 * 128;  // k <= 4 (the 4 x 4 effective kernel of an upsampled 3 x 3 conv's data gradient)

// The LDS of one k_gemm_s3 workgroup: both operand images (one object: the epilogue reuses them as a
// 4 x 32 x 68-float staging area) and the loaders' tap tables.
struct S3Smem {
    struct {
        S3Tile a, b;
    } ab;
    int tab[kS3TabInts];
};
static_assert(sizeof(S3Tile) * 2 >= 4 * 32 * 68 * sizeof(float), "epilogue staging fits the operand images");

// One workgroup of the split-bf16 GEMM.  (gx, gy, gz): the GEMM's own grid (N tiles, M tiles, classes x
// split-K); L: this workgroup's linear index in it.  L must keep the hardware's XCD (L % 8) of the
// launch's workgroup: k_gemm_s3 passes its own index; k_gemm_s3x2 offsets its second GEMM by a
// multiple of 8.
template <class LA, class LB>
__device__ __forceinline__ void gemm_s3_body(const GemmArgs &g, LA la, LB lb, S3Smem &sm, int L, unsigned gx,
                                             unsigned gy, unsigned gz) {
    auto &ab = sm.ab;
    S3Tile &As = ab.a, &Bs = ab.b;
    int *tab = sm.tab;
    // XCD-aware tile order: the hardware deals workgroup L to XCD L % 8 (placement matters for
    // speed only), so consecutive logical tiles -- neighbouring pixel tiles that share input rows,
    // the N-tiles of one split-K chunk that share its A rows -- are given to one XCD and meet in
    // its L2 instead of being fetched from HBM by all eight
    const int T = gx * gy * gz;
    const int xcd = L & 7, q8 = T >> 3, r8 = T & 7;
    const int j = xcd * q8 + min(xcd, r8) + (L >> 3);
    const int bx = j % gx, byz = j / gx, by = byz % gy, bz = byz / gy;
    const int m0 = by * 128, n0 = bx * 128;
    const int ncls = g.ncls > 1 ? g.ncls : 1, cls = bz % ncls, kz = bz / ncls;   // parity class, split
    const int kbeg = kz * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    constexpr bool PREP = HasPrepare<LB>::value;
    la.setup(m0, tab, cls);
    RegP pa;   // LA::pre: the weight planes
    if constexpr (!PREP && LA::pre) {   // the first weight planes are in flight while the tables are built
        la.load(m0, kbeg, kend, pa);
        __builtin_amdgcn_sched_barrier(0);
    }
    lb.setup(n0, tab, cls);
    if constexpr (PREP) lb.prepare(kbeg, kend, 0);
    __syncthreads();
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    float va[16], vb[16];
    static_assert(!LB::pre, "B is never pre-split");
    auto mma = [&]() {
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
    };
    if constexpr (PREP) {
        if constexpr (LA::pre) la.load(m0, kbeg, kend, pa);
        else la.load(m0, kbeg, kend, va);
        lb.load(n0, kbeg, kend, vb, 0);
        int tb = 0;
        for (int k0 = kbeg; k0 < kend; k0 += kS3K) {
            if constexpr (LA::pre) s3_store_pre(As, pa);
            else if constexpr (LanePix<LA>::value) wlp_store(As, va);
            else s3_store<LA::kc>(As, va);
            if constexpr (LanePix<LB>::value) wlp_store(Bs, vb);
            else s3_store<LB::kc>(Bs, vb);
            if (k0 + kS3K < kend) lb.prepare(k0 + kS3K, kend, tb ^ 1);
            __syncthreads();
            if (k0 + kS3K < kend) {
                if constexpr (LA::pre) la.load(m0, k0 + kS3K, kend, pa);
                else la.load(m0, k0 + kS3K, kend, va);
                lb.load(n0, k0 + kS3K, kend, vb, tb ^ 1);
            }
            tb ^= 1;
            mma();
            __syncthreads();
        }
    } else {
        // the B operand's loads two steps ahead (register sets vb / vb1, the loop unrolled by two),
        // the A operand's one step (the weight planes hit L2; two would spill): with one wave per
        // SIMD a single step of prefetch left the implicit-GEMM gathers exposed behind the MFMAs
        float vb1[16];
        auto ldA = [&](int k0) {
            if constexpr (LA::pre) la.load(m0, k0, kend, pa);
            else la.load(m0, k0, kend, va);
        };
        auto st = [&](const float (&b)[16]) {
            if constexpr (LA::pre) s3_store_pre(As, pa);
            else if constexpr (LanePix<LA>::value) wlp_store(As, va);
            else s3_store<LA::kc>(As, va);
            if constexpr (LanePix<LB>::value) wlp_store(Bs, b);
            else s3_store<LB::kc>(Bs, b);
        };
        // the prefetches are issued unconditionally (past kend the loaders read zeros or discarded
        // values without a branch), so every path through the loop has the same loads in flight and the
        // waits stay counted (s3_bload_chans)
        // (the A loads of a step are kept ahead of the B loads issued with it: the next step's operands
        // are then all but the newest 16 loads, a counted wait; reordered, the wait was vmcnt(0))
        if constexpr (!LA::pre) ldA(kbeg);   // (the weight planes were issued before the tables)
        __builtin_amdgcn_sched_barrier(0);
        lb.load(n0, kbeg, kend, vb);
        lb.load(n0, kbeg + kS3K, kend, vb1);
        for (int k0 = kbeg; k0 < kend; k0 += 2 * kS3K) {
            st(vb);
            __syncthreads();
            ldA(k0 + kS3K);
            __builtin_amdgcn_sched_barrier(0);
            lb.load(n0, k0 + 2 * kS3K, kend, vb);
            mma();
            __syncthreads();
            if (k0 + kS3K >= kend) break;
            st(vb1);
            __syncthreads();
            ldA(k0 + 2 * kS3K);
            __builtin_amdgcn_sched_barrier(0);
            lb.load(n0, k0 + 3 * kS3K, kend, vb1);
            mma();
            __syncthreads();
        }
    }
    const int64_t ldc = g.ldc ? g.ldc : g.N;
    // stacked classes (cls_wo == 0): output [split][cls][M][N]; else the parity scatter below
    const bool stacked = ncls > 1 && g.cls_wo == 0;
    float *C = g.C + (int64_t)(stacked ? kz * ncls + cls : kz) * g.M * ldc;
    const bool final_out = (int)gz == ncls;
    const float dv = (final_out && g.div) ? *g.div : 1.0f;
    if (ncls > 1 && !stacked) {
        // parity class: column n = source pixel (a, b) -> output pixel (2a + i, 2b + j)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int n = n0 + wn + 16 * b + jl;
            const int sa = n / g.cls_ws, sb = n - sa * g.cls_ws;
            const int64_t p = (int64_t)(2 * sa + (cls >> 1)) * g.cls_wo + 2 * sb + (cls & 1);
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + wm + 16 * a + 4 * gk + r;
                    if (m < g.M && n < g.N) {
                        float v = acc[a][b][r];
                        if (final_out) {
                            if (g.bias) v = v + g.bias[m];
                            if (g.div) v = v / dv;
                            if (g.accum) v = C[(int64_t)m * ldc + p] + v;
                        }
                        C[(int64_t)m * ldc + p] = v;
                    }
                }
        }
        return;
    }
    if ((g.N & 3) != 0 || (reinterpret_cast<uintptr_t>(g.C) & 15) != 0) {
        // rows not float4-aligned (odd pixel counts): straight from the MFMA layout, 64-B runs
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
        return;
    }
    // float4-aligned rows: through LDS (the operand images are dead after the last barrier).
    // Each wave writes half of its 64 x 64 sub-tile at a time as [row][col] (row stride 68
    // floats) and reads it back as float4 runs, so 16 lanes store 256 contiguous bytes of a row
    float *E = reinterpret_cast<float *>(&ab) + wv * 32 * 68;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) E[(16 * a2 + 4 * gk + r) * 68 + 16 * b + jl] = acc[2 * hf + a2][b][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's half-tile is in LDS (wave-local)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int idx = lane + 64 * i, rr = idx >> 4, q = 4 * (idx & 15);
            const int m = m0 + wm + 32 * hf + rr, n = n0 + wn + q;
            if (m < g.M && n < g.N) {   // N % 4 == 0: a float4 run is all in or all out
                float4 v = *reinterpret_cast<const float4 *>(E + rr * 68 + q);
                float4 *c = reinterpret_cast<float4 *>(C + (int64_t)m * g.N + n);
                if (final_out) {
                    if (g.bias) {
                        const float bs = g.bias[m];
                        v.x = v.x + bs; v.y = v.y + bs; v.z = v.z + bs; v.w = v.w + bs;
                    }
                    if (g.div) { v.x = v.x / dv; v.y = v.y / dv; v.z = v.z / dv; v.w = v.w / dv; }
                    if (g.accum) {
                        const float4 o = *c;
                        v.x = o.x + v.x; v.y = o.y + v.y; v.z = o.z + v.z; v.w = o.w + v.w;
                    }
                }
                *c = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <class LA, class LB>
__global__ __launch_bounds__(256, 2) void k_gemm_s3(GemmArgs g, LA la, LB lb) {
    __shared__ __attribute__((aligned(16))) S3Smem sm;
    gemm_s3_body(g, la, lb, sm, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gridDim.x, gridDim.y,
                 gridDim.z);
}

// Two independent GEMMs in ONE launch (a conv's data gradient and its weight gradient, which read the
// same dL/dz): a 1-D grid of round_up(T1, 8) + T2 workgroups, the first GEMM's tiles first (they are
// dispatched first: the data gradient is the critical chain), the padding workgroups leave at once.
struct S3Grid {
    unsigned x, y, z;
};
template <class LA1, class LB1, class LA2, class LB2>
__global__ __launch_bounds__(256, 2) void k_gemm_s3x2(GemmArgs g1, LA1 la1, LB1 lb1, S3Grid d1, GemmArgs g2, LA2 la2,
                                                       LB2 lb2, S3Grid d2) {
    __shared__ __attribute__((aligned(16))) S3Smem sm;
    const int T1 = (int)(d1.x * d1.y * d1.z), T1p = (T1 + 7) & ~7, L = blockIdx.x;
    if (L < T1p) {
        if (L < T1) gemm_s3_body(g1, la1, lb1, sm, L, d1.x, d1.y, d1.z);
    } else {
        gemm_s3_body(g2, la2, lb2, sm, L - T1p, d2.x, d2.y, d2.z);
    }
}

// ---- pointwise (1x1, stride 1, unpadded) conv product -----------------------------------------
// C[M][N] (+)= A[M][Kp] B[K][N] (+ bias[M]) for M <= 256 output channels over N pixels: the
// forward (A = the k_wprep forward planes WF, B = x) and the data gradient (A = WD = W^T planes,
// B = dL/dz) of the reference's 1x1 convs (my_Lipschitz_Unet.py:96-103, skip.py's 1x1 skips).
// One workgroup per 64 pixels: their B columns (all K) are read from HBM once and split into the
// three bf16 planes in LDS ([plane][pixel][k], row stride ldsrow bytes = 16 mod 256 so the 16
// pixel rows of a fragment read sit in distinct bank groups); the pre-split A fragments stream
// from L2 (one k-step prefetched), so every C element of the 64 pixels is produced by this one
// workgroup: no split-K, no tile quantisation on M.  Wave w owns rows 16 w + 64 j (j < MT).
struct PwArgs {
    const __bf16 *A;
    int64_t pstride;   // plane stride of A (elements)
    int lda;           // A row length (Kp, multiple of 16; columns >= the valid K are zero)
    const float *B;
    int K;             // valid B rows
    int64_t N;
    float *C;
    const float *bias;
    int M, Kp32, ldsrow, accum;
    int dbg;   // diagnostics only (LRS_PW_DBG): 1 no C stores, 2 no A loads, 4 no B loads
    int act;   // activation applied after the bias (a conv without BN: its act in the epilogue)
    // the masked-MSE head fused into the network's last conv (tgt != NULL; k_mse_head's arithmetic per
    // element): gz = act'(out) * (-norm (tgt m - out m) m) stored beside out, and per output row the
    // workgroup's fp64 sums of gz and of (tgt m - out m)^2 in hpart[0 / 1][row][blockIdx.x]
    const float *tgt = nullptr, *msk = nullptr;
    float *gz = nullptr;
    double *hpart = nullptr;
    float hnorm = 0.0f;
};

inline int pw_ldsrow(int Kp32) {   // bytes; Kp32 * 2 rounded up to 16 mod 256
    int b = Kp32 * 2;
    return b + (((16 - b) % 256) + 256) % 256;
}

// NB = 16-pixel column blocks per workgroup (16 NB pixels): 4, or 5, chosen per launch by
// pw_launch (dipnet.hip) from the rounds of CU slots the grid needs.
template <int MT, int NB = 4>
__global__ __launch_bounds__(256, 2) void k_pw(PwArgs a) {
    extern __shared__ __attribute__((aligned(16))) char pw_smem[];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, jl = lane & 15, gk = lane >> 4;
    constexpr int NPX = 16 * NB;
    const int64_t n0 = (int64_t)blockIdx.x * NPX;
    const int64_t plane = (int64_t)NPX * a.ldsrow;
    if constexpr (NB == 4) {   // stage: thread (n = t & 63) splits k chunks (t >> 6) + 4 i of 8 values each.  Buffer
        // loads, branch-free: k (wave-uniform) goes in the scalar offset, so rows k >= K fall past
        // the buffer's K * N floats and read 0; a pixel n >= N reads at kOob.
        const int n = t & 63;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(a.B, (int)(a.K * a.N * 4));
        const int voff = n0 + n < a.N ? (int)((n0 + n) * 4) : kOob;
        const int nck = a.Kp32 / 8, c0 = __builtin_amdgcn_readfirstlane(t >> 6);
        float v[8][8];   // all of the thread's chunks (<= 8 for K <= 256) in flight together
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = c0 + 4 * i;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t so = (int64_t)(8 * c + u) * a.N * 4;
                v[i][u] = (c < nck && !(a.dbg & 4)) ? s3_bload(rs, voff, so < kOob ? (int)so : kOob) : 0.0f;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = c0 + 4 * i;
            if (c >= nck) break;
            s3bf8 p0, p1, p2;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const S3Split q = s3_split(v[i][u]);
                p0[u] = q.b0;
                p1[u] = q.b1;
                p2[u] = q.b2;
            }
            char *dst = pw_smem + (int64_t)n * a.ldsrow + 16 * c;
            *reinterpret_cast<s3bf8 *>(dst) = p0;
            *reinterpret_cast<s3bf8 *>(dst + plane) = p1;
            *reinterpret_cast<s3bf8 *>(dst + 2 * plane) = p2;
        }
    } else {   // NPX pixels x nck chunks as items it = t + 256 j: pixel it % NPX, chunk it / NPX
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(a.B, (int)(a.K * a.N * 4));
        const int nck = a.Kp32 / 8, items = NPX * nck;
        constexpr int kMaxIt = (NPX * 32 + 255) / 256;   // K <= 256
        float v[kMaxIt][8];
#pragma unroll
        for (int j = 0; j < kMaxIt; ++j) {
            const int it = t + 256 * j, n = it % NPX, c = it / NPX;
            const int voff = n0 + n < a.N ? (int)((n0 + n) * 4) : kOob;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t so = (int64_t)(8 * c + u) * a.N * 4;
                v[j][u] = (it < items && !(a.dbg & 4)) ? s3_bload(rs, voff, so < kOob ? (int)so : kOob) : 0.0f;
            }
        }
#pragma unroll
        for (int j = 0; j < kMaxIt; ++j) {
            const int it = t + 256 * j, n = it % NPX, c = it / NPX;
            if (it >= items) break;
            s3bf8 p0, p1, p2;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const S3Split q = s3_split(v[j][u]);
                p0[u] = q.b0;
                p1[u] = q.b1;
                p2[u] = q.b2;
            }
            char *dst = pw_smem + (int64_t)n * a.ldsrow + 16 * c;
            *reinterpret_cast<s3bf8 *>(dst) = p0;
            *reinterpret_cast<s3bf8 *>(dst + plane) = p1;
            *reinterpret_cast<s3bf8 *>(dst + 2 * plane) = p2;
        }
    }
    s3f4 acc[MT][NB];
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[j][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    const int ksteps = a.Kp32 / 32;
    s3bf8 fa[MT][3], fn[MT][3];
    // A fragments: 16-B buffer loads (L2-resident planes), rows >= M and k >= lda at kOob (zeros)
    const __amdgpu_buffer_rsrc_t ra = s3_rsrc(a.A, (int)(3 * a.pstride * 2));
    auto loadA = [&](int ks, s3bf8 (&f)[MT][3]) {
        const int k = ks * 32 + 8 * gk;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int row = 16 * wv + 64 * j + jl;
            const int vo = (row < a.M && k < a.lda && !(a.dbg & 2)) ? 2 * (row * a.lda + k) : kOob;
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f[j][p] = __builtin_bit_cast(s3bf8, __builtin_amdgcn_raw_buffer_load_b128(ra, vo, (int)(2 * p * a.pstride), 0));
        }
    };
    // NB = 4 prefetches the next k-step's A fragments; NB = 5 has no registers for that (its loads
    // overlap the step's B fragment reads from LDS instead)
    constexpr bool PF = NB == 4;
    loadA(0, fa);
    __syncthreads();
    for (int ks = 0; ks < ksteps; ++ks) {
        if constexpr (PF) {
            if (ks + 1 < ksteps) loadA(ks + 1, fn);
        } else if (ks > 0) {
            loadA(ks, fa);
        }
        s3bf8 fb[NB][3];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const char *s0 = pw_smem + (int64_t)(16 * b + jl) * a.ldsrow + 16 * (4 * ks + gk);
#pragma unroll
            for (int p = 0; p < 3; ++p) fb[b][p] = *reinterpret_cast<const s3bf8 *>(s0 + p * plane);
        }
#pragma unroll
        for (int j = 0; j < MT; ++j)
#pragma unroll
            for (int b = 0; b < NB; ++b) acc[j][b] = s3_mfma6(fa[j], fb[b], acc[j][b]);
        if (PF && ks + 1 < ksteps) {
#pragma unroll
            for (int j = 0; j < MT; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p) fa[j][p] = fn[j][p];
        }
    }
    // epilogue through LDS (the B image is dead after this barrier): wave w writes its 16 x 64 tile
    // of each row block as [row][pixel] and reads it back as float4 rows, so every 16 lanes store
    // one full 256-B pixel run of a channel row (the MFMA layout gives a lane 4 rows of 1 pixel)
    __syncthreads();
    constexpr int ES = NPX + 4;   // staging row stride (floats)
    float *E = reinterpret_cast<float *>(pw_smem) + wv * 16 * ES;
    const bool vec = (a.N & 3) == 0 && ((reinterpret_cast<uintptr_t>(a.C) & 15) == 0);
    const bool head = a.tgt != nullptr;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) E[(4 * gk + r) * ES + 16 * b + jl] = acc[j][b][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes done (wave-local tile)
        __builtin_amdgcn_wave_barrier();
        double hs[NB], hb[NB];   // head: this lane's loss / bias-gradient sums of its run per i
#pragma unroll
        for (int i = 0; i < NB; ++i) {   // 16 rows x NPX / 4 float4 runs
            hs[i] = 0.0;
            hb[i] = 0.0;
            const int idx = lane + 64 * i, rr = idx / (4 * NB), q = 4 * (idx % (4 * NB));
            const int m = 16 * wv + 64 * j + rr;
            const int64_t n = n0 + q;
            if (m >= a.M || (a.dbg & 1)) continue;
            float4 v = *reinterpret_cast<const float4 *>(E + rr * ES + q);
            const float bs = a.bias ? a.bias[m] : 0.0f;
            float *c = a.C + (int64_t)m * a.N + n;
            if (vec && n + 3 < a.N) {
                if (a.bias) { v.x = v.x + bs; v.y = v.y + bs; v.z = v.z + bs; v.w = v.w + bs; }
                if (a.accum) {
                    const float4 o = *reinterpret_cast<const float4 *>(c);
                    v.x = o.x + v.x; v.y = o.y + v.y; v.z = o.z + v.z; v.w = o.w + v.w;
                }
                if (a.act) { v.x = act_fwd(v.x, a.act); v.y = act_fwd(v.y, a.act); v.z = act_fwd(v.z, a.act); v.w = act_fwd(v.w, a.act); }
                *reinterpret_cast<float4 *>(c) = v;
                if (head) {   // k_mse_head's per-element arithmetic, in the same order
                    const float4 tv = *reinterpret_cast<const float4 *>(a.tgt + (int64_t)m * a.N + n);
                    const float4 mv = a.msk ? *reinterpret_cast<const float4 *>(a.msk + n) : make_float4(1.0f, 1.0f, 1.0f, 1.0f);
                    const float oe[4] = {v.x, v.y, v.z, v.w}, te[4] = {tv.x, tv.y, tv.z, tv.w}, me[4] = {mv.x, mv.y, mv.z, mv.w};
                    float ge[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = te[e] * me[e] - oe[e] * me[e];
                        hs[i] += (double)d * (double)d;
                        ge[e] = act_bwd((-(a.hnorm * d)) * me[e], oe[e], a.act);
                        hb[i] += (double)ge[e];
                    }
                    *reinterpret_cast<float4 *>(a.gz + (int64_t)m * a.N + n) = make_float4(ge[0], ge[1], ge[2], ge[3]);
                }
            } else {
                const float vv[4] = {v.x, v.y, v.z, v.w};
                for (int u = 0; u < 4; ++u) {
                    if (n + u >= a.N) break;
                    float x = vv[u];
                    if (a.bias) x = x + bs;
                    if (a.accum) x = c[u] + x;
                    if (a.act) x = act_fwd(x, a.act);
                    c[u] = x;
                    if (head) {
                        const float mk = a.msk ? a.msk[n + u] : 1.0f;
                        const float d = a.tgt[(int64_t)m * a.N + n + u] * mk - x * mk;
                        hs[i] += (double)d * (double)d;
                        const float g = act_bwd((-(a.hnorm * d)) * mk, x, a.act);
                        a.gz[(int64_t)m * a.N + n + u] = g;
                        hb[i] += (double)g;
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (head) {   // each row's sums over the workgroup's runs, in run order, through this wave's LDS
            double2 *R = reinterpret_cast<double2 *>(E);   // [16 rows x 4 NB runs] (fits the wave's E)
            static_assert(16 * 4 * NB * sizeof(double2) <= 16 * ES * sizeof(float), "head sums fit the staging");
#pragma unroll
            for (int i = 0; i < NB; ++i) R[lane + 64 * i] = make_double2(hs[i], hb[i]);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const int m = 16 * wv + 64 * j + lane;
            if (lane < 16 && m < a.M) {
                double sl = 0.0, sg = 0.0;
                for (int k = 0; k < 4 * NB; ++k) {
                    const double2 p = R[lane * 4 * NB + k];
                    sl += p.x;
                    sg += p.y;
                }
                a.hpart[(int64_t)m * gridDim.x + blockIdx.x] = sg;
                a.hpart[((int64_t)a.M + m) * gridDim.x + blockIdx.x] = sl;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// The fused head's sums (k_pw with PwArgs::tgt): per channel c (grid C) the gz sums of the nwg
// workgroups, summed in a fixed order -> the conv's bias gradient, and the loss sums -> closs[c];
// k_head_loss then adds closs in channel order into loss_acc (deterministic, as k_mse_head).
__global__ __launch_bounds__(256) void k_head_reduce(const double *__restrict__ hpart, int C, int nwg, float *gbias,
                                                     double *closs) {
    __shared__ double red[12];
    const int c = blockIdx.x;
    double sg = 0.0, sl = 0.0;
    for (int w = threadIdx.x; w < nwg; w += blockDim.x) {
        sg += hpart[(int64_t)c * nwg + w];
        sl += hpart[((int64_t)C + c) * nwg + w];
    }
    block_sum2_d(sg, sl, red);
    if (threadIdx.x == 0) {
        gbias[c] = (float)sg;
        closs[c] = sl;
    }
}

__global__ void k_head_loss(const double *__restrict__ closs, int C, double *loss_acc) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double s = 0.0;
    for (int c = 0; c < C; ++c) s += closs[c];
    *loss_acc += s;
}

// Per-step weight preparation of every conv of a network in ONE launch (grid (blocks, convs)):
// Wn = W_bar / scale[si] for the spectrally normalised convs (lipschitz_constraint_layer.py:42-44)
// and the bf16 planes the split-bf16 kernels read, from the same W / scale quotient:
//   WF[p][co][kyx * Cp + ci]            forward operand (Cp = Cin rounded up to 16)
//   WD[p][ci][kyx * Cop + co]           data-gradient operand (W^T, Cop = Cout rounded up to 16), or,
//                                       for an upsampled stride-1 conv (ke > 0),
//   WE[p][ci][(ey * ke + ex) * Cop + co] the effective ke x ke kernel of its data gradient as a
//                                       stride-2 conv over dL/dz (conv_bwd): the sum of the taps
//                                       W[a + k-1-ey][b + k-1-ex] over the 2 x 2 upsample children a, b
//   upc: an upsampled reflection-padded 3 x 3 conv run by output parity class (LdUpFwdTM /
//   LdUpDgradTM): instead of WF / WD,
//   WUF[p][cls][co][e * Cp + ci]         the class's 2 x 2 effective weights (e = 2 ey + ex, the sum
//                                        of W[co][ci][ky][kx] over ky in T(i, ey), kx in T(j, ex))
//   WUD[p][ci][(4 cls + e) * Cop + co]   the same, transposed, all classes (the data gradient's K)
struct ConvPrep {
    const float *W;
    float *Wn;          // nullable
    __bf16 *wf, *wd;    // nullable (wd holds WE when ke > 0)
    int Cout, Cin, kk, Cp, Cop, si, k, ke;   // si: scale index, -1 = no spectral norm
    int upc;
};

// effective weight of parity class (i, j), tap (ey, ex): the taps T(i, ey) x T(j, ex) summed in
// increasing ky, kx order (w = the 3 x 3 taps of one (co, ci))
__device__ __forceinline__ float upc_weight(const float *w, int i, int j, int ey, int ex) {
    const int y0 = (i == 0) ? (ey == 0 ? 0 : 1) : (ey == 0 ? 0 : 2), y1 = (i == 0) ? (ey == 0 ? 0 : 2) : (ey == 0 ? 1 : 2);
    const int x0 = (j == 0) ? (ex == 0 ? 0 : 1) : (ex == 0 ? 0 : 2), x1 = (j == 0) ? (ex == 0 ? 0 : 2) : (ex == 0 ? 1 : 2);
    float s = 0.0f;
    for (int ky = y0; ky <= y1; ++ky)
        for (int kx = x0; kx <= x1; ++kx) s = s + w[ky * 3 + kx];
    return s;
}

__device__ __forceinline__ void conv_prep_body(const ConvPrep &c, float s, int64_t i0, int64_t stride) {
    const int64_t nw = (int64_t)c.Cout * c.Cin * c.kk;
    if (c.Wn)
        for (int64_t i = i0; i < nw; i += stride) c.Wn[i] = c.W[i] / s;
    const int ed = c.upc ? 16 : (c.ke > 0 ? c.ke * c.ke : c.kk);
    // 32-bit index arithmetic (lrs_dipnet_create and the lrs_conv2d_* entry points reject a conv whose
    // planes reach 2^31 / 3 elements)
    const int nf = c.wf ? c.Cout * (c.upc ? 16 : c.kk) * c.Cp : 0, nd = c.wd ? c.Cin * ed * c.Cop : 0;
    auto put = [&](__bf16 *dst, int plane, int j, float x) {
        const S3Split q = s3_split(x);
        dst[j] = q.b0;
        dst[plane + j] = q.b1;
        dst[2 * plane + j] = q.b2;
    };
    // forward planes (ci fastest: the W reads of a wave are kk floats apart)
    for (int i = (int)i0; i < nf; i += (int)stride) {
        float x = 0.0f;
        if (c.upc) {   // [cls][co][e * Cp + ci]
            const int cl = i / (c.Cout * 4 * c.Cp), rem = i - cl * c.Cout * 4 * c.Cp;
            const int co = rem / (4 * c.Cp), r = rem - co * 4 * c.Cp, e = r / c.Cp, ci = r - e * c.Cp;
            if (ci < c.Cin) {
                x = upc_weight(c.W + ((int64_t)co * c.Cin + ci) * 9, cl >> 1, cl & 1, e >> 1, e & 1);
                if (c.si >= 0) x = x / s;
            }
        } else {       // [co][kyx * Cp + ci]
            const int co = i / (c.kk * c.Cp), rem = i - co * c.kk * c.Cp, kyx = rem / c.Cp, ci = rem - kyx * c.Cp;
            if (ci < c.Cin) {
                x = c.W[((int64_t)co * c.Cin + ci) * c.kk + kyx];
                if (c.si >= 0) x = x / s;
            }
        }
        put(c.wf, nf, i, x);
    }
    // data-gradient planes [ci][e * Cop + co] (W^T): a wave covers 8 ci x 8 co of one e, so its W reads
    // touch 8 rows of W instead of 64 (co fastest alone put the lanes Cin kk floats apart)
    const int nci8 = (c.Cin + 7) / 8, ncob = c.Cop / 8, ndt = c.wd ? nci8 * 64 * ed * ncob : 0;
    for (int t = (int)i0; t < ndt; t += (int)stride) {
        const int l = t & 63, r = t >> 6;
        const int cob = r % ncob, r2 = r / ncob, e = r2 % ed, cib = r2 / ed;
        const int ci = 8 * cib + (l >> 3), co = 8 * cob + (l & 7);
        if (ci >= c.Cin) continue;
        float x = 0.0f;
        if (co < c.Cout) {
            const float *w = c.W + ((int64_t)co * c.Cin + ci) * c.kk;
            if (c.upc) {   // e = 4 cls + tap
                x = upc_weight(w, (e >> 2) >> 1, (e >> 2) & 1, (e & 3) >> 1, e & 1);
            } else if (c.ke > 0) {
                const int ey = e / c.ke, ex = e - ey * c.ke;
                for (int a = 0; a < 2; ++a)
                    for (int b = 0; b < 2; ++b) {
                        const int ky = a + c.k - 1 - ey, kx = b + c.k - 1 - ex;
                        if (ky >= 0 && ky < c.k && kx >= 0 && kx < c.k) x = x + w[ky * c.k + kx];
                    }
            } else {
                x = w[e];
            }
            if (c.si >= 0) x = x / s;
        }
        put(c.wd, nd, (ci * ed + e) * c.Cop + co, x);
    }
}

__global__ __launch_bounds__(256) void k_conv_prep(const ConvPrep *__restrict__ tab, const float *__restrict__ scale,
                                                   double *loss_acc, int *step) {
    if (loss_acc && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {   // a training step begins
        *loss_acc = 0.0;
        *step += 1;
    }
    const ConvPrep c = tab[blockIdx.y];
    conv_prep_body(c, c.si >= 0 ? scale[c.si] : 1.0f, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
                   (int64_t)gridDim.x * blockDim.x);
}

// one conv, no spectral norm (the standalone lrs_conv2d_* entry points)
__global__ __launch_bounds__(256) void k_conv_prep1(ConvPrep c) {
    conv_prep_body(c, 1.0f, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// Reflection-pad corrections of the effective-kernel data gradient of an upsampled, reflection-
// padded 3 x 3 conv (pad 1).  The stride-2 4 x 4 conv over dL/dz treats the padded border as zeros;
// the reference's ReflectionPad2d(1) also feeds padded row -1 from row 1 and row Hu from Hu - 2
// (same for columns): extra (oy, ky) pairs (0, 0) -> source row 0 and (Hu - 1, 2) -> row Hs - 1,
// and likewise (ox, kx) for the columns.  Four "lines": 0 / 1 = source rows 0 / Hs - 1 take every
// term with a reflected row (any column, reflected or not); 2 / 3 = source columns 0 / Ws - 1 every
// term with a reflected column and an unreflected row, so each term is counted once.  Three wide
// launches (k_up_border_s, _mm, _add), scratch in the conv's col-gradient buffer:
//   S[line][co][j][pos]  = the line's dL/dz summed over the positions that map to source pos via
//                          tap j (j = kx for rows, ky for columns)
//   corr[line][c][pos]   = sum_{co, j} W[co][c][tap(line, j)] S[line][co][j][pos]
// then gx[c][perimeter pixel] += its row-line and column-line corrections.  w = the conv's fp32
// weights (W / sigma) [Cout][Cin][3][3].
constexpr int kUbC = 4, kUbCo = 32;

__device__ __forceinline__ int ub_len(int line, int Hs, int Ws) { return line < 2 ? Ws : Hs; }

__global__ __launch_bounds__(256) void k_up_border_s(const float *__restrict__ gz, int Cout, int Hs, int Ws, int Lmax,
                                                     float *__restrict__ S) {
    const int co = blockIdx.y, e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 4 * 3 * Lmax) return;
    const int line = e / (3 * Lmax), j = (e / Lmax) % 3, pos = e % Lmax;
    const int Hu = 2 * Hs, Wu = 2 * Ws, rows = line < 2, L = ub_len(line, Hs, Ws), Lu = rows ? Wu : Hu;
    float v = 0.0f;
    if (pos < L) {
        const int ofix = (line & 1) == 0 ? 0 : (rows ? Hu - 1 : Wu - 1);
        const float *g = gz + (int64_t)co * Hu * Wu;
        for (int o = max(0, 2 * pos - 2); o <= min(Lu - 1, 2 * pos + 3); ++o) {
            int u = o + j - 1;
            if (rows) u = u < 0 ? -u : (u >= Lu ? 2 * (Lu - 1) - u : u);   // along x: reflected ends included
            else if (u < 0 || u >= Lu) continue;                          // along y: unreflected rows only
            if ((u >> 1) == pos) v += g[rows ? (int64_t)ofix * Wu + o : (int64_t)o * Wu + ofix];
        }
    }
    S[(((int64_t)line * Cout + co) * 3 + j) * Lmax + pos] = v;
}

__global__ __launch_bounds__(256) void k_up_border_mm(const float *__restrict__ S, const float *__restrict__ w, int Cin,
                                                      int Cout, int Hs, int Ws, int Lmax, float *__restrict__ corr) {
    __shared__ float Ss[kUbCo * 3 * 128], Wl[kUbCo * kUbC * 3];
    const int line = blockIdx.x, c0 = blockIdx.y * kUbC, p0 = blockIdx.z * 128;
    const int rows = line < 2, L = ub_len(line, Hs, Ws), tfix = (line & 1) == 0 ? 0 : 2;
    const int cl = threadIdx.x >> 7, pl = threadIdx.x & 127;   // 2 channels x 128 positions per pass
    float acc[2] = {0.0f, 0.0f};
    for (int co0 = 0; co0 < Cout; co0 += kUbCo) {
        __syncthreads();
        float sv[kUbCo * 3 * 128 / 256];   // all 48 loads issued before any LDS store (clamped, then masked)
#pragma unroll
        for (int u = 0; u < kUbCo * 3 * 128 / 256; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int col = e / 384, j = (e >> 7) % 3, pos = p0 + (e & 127), co = co0 + col;
            const int cc = min(co, Cout - 1), pp = min(pos, Lmax - 1);
            sv[u] = S[(((int64_t)line * Cout + cc) * 3 + j) * Lmax + pp];
        }
#pragma unroll
        for (int u = 0; u < kUbCo * 3 * 128 / 256; ++u) {
            const int e = threadIdx.x + 256 * u;
            const int col = e / 384, pos = p0 + (e & 127), co = co0 + col;
            Ss[e] = (co < Cout && pos < L) ? sv[u] : 0.0f;
        }
        for (int e = threadIdx.x; e < kUbCo * kUbC * 3; e += blockDim.x) {
            const int col = e / (kUbC * 3), c = c0 + (e / 3) % kUbC, j = e % 3, co = co0 + col;
            Wl[e] = (co < Cout && c < Cin) ? w[((int64_t)co * Cin + c) * 9 + (rows ? tfix * 3 + j : j * 3 + tfix)] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = 2 * h + cl;
            float a = acc[h];
            for (int col = 0; col < kUbCo; ++col)
#pragma unroll
                for (int j = 0; j < 3; ++j) a = __fmaf_rn(Wl[(col * kUbC + c) * 3 + j], Ss[(col * 3 + j) * 128 + pl], a);
            acc[h] = a;
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int c = c0 + 2 * h + cl, pos = p0 + pl;
        if (c < Cin && pos < L) corr[((int64_t)line * Cin + c) * Lmax + pos] = acc[h];
    }
}

__global__ __launch_bounds__(256) void k_up_border_add(const float *__restrict__ corr, int Cin, int Hs, int Ws,
                                                       int Lmax, float *__restrict__ gx) {
    const int nper = 2 * Ws + 2 * (Hs - 2);
    const int idx = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y;
    if (idx >= nper) return;
    int sy, sx;
    if (idx < Ws) { sy = 0; sx = idx; }
    else if (idx < 2 * Ws) { sy = Hs - 1; sx = idx - Ws; }
    else { const int r = idx - 2 * Ws; sy = 1 + (r >> 1); sx = (r & 1) ? Ws - 1 : 0; }
    float v = 0.0f;
    if (sy == 0) v += corr[((int64_t)0 * Cin + c) * Lmax + sx];
    if (sy == Hs - 1) v += corr[((int64_t)1 * Cin + c) * Lmax + sx];
    if (sx == 0) v += corr[((int64_t)2 * Cin + c) * Lmax + sy];
    if (sx == Ws - 1) v += corr[((int64_t)3 * Cin + c) * Lmax + sy];
    float *o = gx + ((int64_t)c * Hs + sy) * Ws + sx;
    *o = *o + v;
}

// gx[c][sy][sx] (+)= sum over the x2 upsample children u of sum over the padded positions that
// read u (direct + reflection mirrors, padded_sources) of gxp[c][iy][ix], where gxp is the sum of
// nsplit split-K partials (stride zstride floats; the data-gradient GEMM's split-K finished here, in
// k_gemm_reduce's order per position)
__device__ __forceinline__ float fold_term(const float *__restrict__ src, int nsplit, int64_t zstride, int64_t i) {
    if (nsplit == 1) return src[i];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int z0 = 0; z0 < nsplit; z0 += 8) {
        float p[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) p[e] = z0 + e < nsplit ? src[(int64_t)(z0 + e) * zstride + i] : 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (z0 + e < nsplit) acc[e] += p[e];
    }
    return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

__global__ __launch_bounds__(256) void k_fold_pad(const float *__restrict__ gxp, int nsplit, int64_t zstride,
                                                  ConvGeom gm, float *__restrict__ gx, int accum) {
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
                    for (int px = 0; px < nx; ++px) acc += fold_term(src, nsplit, zstride, iys[py] * Wp + ixs[px]);
            }
        }
        const int64_t i = (int64_t)c * HW + q;
        gx[i] = accum ? gx[i] + acc : acc;
    }
}

// k_fold_pad for one partial (nsplit == 1, no upsample; a data-gradient GEMM with enough tiles, e.g.
// the 512^2 layers of configs[3]): grid (row quads, Cin), a thread = 4 consecutive source x of one
// row, float4 stores (Ws % 4 == 0).  Per pixel the same padded sources in the same order as
// k_fold_pad, so the result is bit-identical.
__global__ __launch_bounds__(256) void k_fold_pad1q(const float *__restrict__ gxp, ConvGeom gm, float *__restrict__ gx,
                                                    int accum) {
    const int W4 = gm.Ws >> 2, Wp = gm.Wu + 2 * gm.pad, Qp = (gm.Hu + 2 * gm.pad) * Wp;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= gm.Hs * W4) return;
    const int c = blockIdx.y, sy = t / W4, sx0 = 4 * (t - sy * W4);
    const float *src = gxp + (int64_t)c * Qp;
    int iys[3];
    const int ny = padded_sources(sy, gm.Hu, gm.pad, gm.pad_mode, iys);
    float acc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        int ixs[3];
        const int nx = padded_sources(sx0 + e, gm.Wu, gm.pad, gm.pad_mode, ixs);
        float a = 0.0f;
        for (int py = 0; py < ny; ++py)
            for (int px = 0; px < nx; ++px) a += src[iys[py] * Wp + ixs[px]];
        acc[e] = a;
    }
    float4 *o = reinterpret_cast<float4 *>(gx + ((int64_t)c * gm.Hs + sy) * gm.Ws + sx0);
    float4 r = make_float4(acc[0], acc[1], acc[2], acc[3]);
    if (accum) {
        const float4 p = *o;
        r = make_float4(p.x + r.x, p.y + r.y, p.z + r.z, p.w + r.w);
    }
    *o = r;
}

}  // namespace lrs
