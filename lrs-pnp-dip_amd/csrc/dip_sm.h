// Small-map implicit-GEMM convolution for the DIP engine (gfx950): the U-Net's 49^2 .. 13^2
// layers (my_Lipschitz_Unet.py:40-82 at 196^2 input), whose products are a few hundred MFLOP and
// whose cost is launch and memory latency, not matrix-core time.
//
// C[M][N] (+)= A[M][K] B[K][N] on 64 x 64 tiles (256 threads, 2 x 2 waves of 32 x 32), fp32-accurate
// on the bf16 matrix cores exactly as k_gemm_s3 (three bf16 planes per operand, the six partial
// products with i + j <= 2 on v_mfma_f32_16x16x32_bf16), 64 k per LDS stage with the next stage's
// loads in registers, split-K over gridDim.z (partials as k_gemm_reduce / k_reduce_bn1 expect).
//   forward        : A = the k_conv_prep planes WF [3][Cout][kk Cp], B = the implicit im2col of x
//                    (LDS table of the tile's 64 pixels x kk taps: source offset or kOob), so no
//                    col matrix and no k_im2col launch;
//   data gradient  : A = the planes WD = W^T [3][Cin][kk Cop], B[(tap, co)][q] = the sum of dL/dz
//                    over the output pixels that read input pixel q through that tap (the conv's
//                    adjoint, with reflection, stride and the x2 upsample folded into a table built
//                    on the host, <= 2 terms per dimension): gx directly, no dcol, no col2im and no
//                    fold;
//   weight gradient: A = dL/dz [Cout][P] (fp32, split at the store), B = col^T gathered from x
//                    through a per-conv tap table (SmWgrad), so no col matrix and no k_im2col
//                    launch; without split-K (short K: the 36^2 maps) one launch finishes dW / scale.
#pragma once

#include "dip_gemm.h"

namespace lrs {

constexpr int kSmK = 64;                 // k per LDS stage
constexpr int kSmTabInts = 9 * 64 * 4 + 16;   // k <= 3: [tap][pixel][4 combos] + per-tap flags

struct SmImg {
    __bf16 v[3][64][kSmK];   // [plane][row][k], 128-B rows, 16-B chunks swizzled by sm_chunk
};

// chunk ^ ((row >> 1) & 7): the 16 rows of a fragment read (lanes jl = 0..15 at one chunk) land on
// 16 distinct 16-B bank slots (two rows per 256-B bank line)
__device__ __forceinline__ int sm_chunk(int row, int c) { return c ^ ((row >> 1) & 7); }

// group j (0, 1) of this thread: row = (t + 256 j) & 63, 8-k chunk kg = (t + 256 j) >> 6
__device__ __forceinline__ int sm_row(int j) { return (threadIdx.x + 256 * j) & 63; }
__device__ __forceinline__ int sm_kg(int j) { return (threadIdx.x + 256 * j) >> 6; }

__device__ __forceinline__ void sm_store_pre(SmImg &T, int row, int kg, const uint4 (&h)[3]) {
    const int ch = sm_chunk(row, kg) * 8;
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4 *>(&T.v[p][row][ch]) = h[p];
}

__device__ __forceinline__ void sm_store_f32(SmImg &T, int row, int kg, const float (&v)[8]) {
    s3bf8 p0, p1, p2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const S3Split q = s3_split(v[e]);
        p0[e] = q.b0;
        p1[e] = q.b1;
        p2[e] = q.b2;
    }
    const int ch = sm_chunk(row, kg) * 8;
    *reinterpret_cast<s3bf8 *>(&T.v[0][row][ch]) = p0;
    *reinterpret_cast<s3bf8 *>(&T.v[1][row][ch]) = p1;
    *reinterpret_cast<s3bf8 *>(&T.v[2][row][ch]) = p2;
}

__device__ __forceinline__ void sm_frag(const SmImg &T, int row, int c, s3bf8 (&f)[3]) {
    const int ch = sm_chunk(row, c) * 8;
#pragma unroll
    for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const s3bf8 *>(&T.v[p][row][ch]);
}

// A: pre-split planes, plane p of row x at P + p * pstride + x * ld (k contiguous, K and ld
// multiples of 16); rows >= X and k >= kend read 0.  16-B buffer loads (L2-resident planes).
struct SmPre {
    static constexpr bool pre = true;
    const __bf16 *P;
    int64_t pstride;
    int ld, X;
    __device__ __forceinline__ void load(int x0, int k0, int kend, int j, uint4 (&h)[3]) const {
        const int x = x0 + sm_row(j), k = k0 + 8 * sm_kg(j);
        const __amdgpu_buffer_rsrc_t r = s3_rsrc(P, (int)(3 * pstride * 2));
        const int vo = (x < X && k < kend) ? 2 * (x * ld + k) : kOob;
#pragma unroll
        for (int p = 0; p < 3; ++p)
            h[p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, (int)(2 * p * pstride), 0));
    }
};

// B forward: col[r][p], r = tap * Cp + c (tap-major, Cp = Cin rounded up to 16), p = output pixel.
// Table [kk][64]: the source byte offset of the tile's pixels within a channel plane (kOob = zero).
struct SmFwd {
    const float *X;
    int xbytes;
    ConvGeom g;
    int Cp;
    const int *tab;
    __device__ __forceinline__ void setup(int x0, int *smem) {
        const int kk = g.k * g.k, P = g.Ho * g.Wo;
        for (int i = threadIdx.x; i < kk * 64; i += blockDim.x) {
            const int kyx = i >> 6, p = x0 + (i & 63);
            int o = kOob;
            if (p < P) {
                const int oy = p / g.Wo, ox = p - oy * g.Wo, ky = kyx / g.k, kx = kyx - ky * g.k;
                const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
                const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
                if (sy >= 0 && sx >= 0) o = 4 * (sy * g.Ws + sx);
            }
            smem[i] = o;
        }
        tab = smem;
    }
    __device__ __forceinline__ void load(int, int k0, int kend, int j, float (&v)[8]) const {
        // r0 is wave-uniform (a wave's 64 threads share kg): in an SGPR, the channel offsets below are
        // scalar buffer offsets (a VGPR there would make the compiler loop over every load)
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + 8 * sm_kg(j));
        const int kyx = r0 / Cp, c0 = r0 - kyx * Cp;
        const int pb = g.Hs * g.Ws * 4;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, xbytes);
        const int vo = r0 < kend ? tab[kyx * 64 + sm_row(j)] : kOob;
        s3_bload_chans(rs, vo, c0, g.Cin, pb, v);   // channels >= Cin meet zero weights (SmPre)
    }
};

// B data gradient: B[r][q], r = tap * Cop + co, q = input pixel: the sum of dL/dz[co] over the
// (<= 2 x 2) output pixels o with src(o, tap) = q.  adj = the host's table [kk][Q] of int4 byte
// offsets within a dL/dz plane (kOob = no term; sm_adj_table), staged per tile into LDS
// [kk][64][4] with all of a thread's loads in flight together.
struct SmAdj {
    const float *GZ;
    int gbytes;
    ConvGeom g;
    int Cout, Cop;
    const int4 *adj;
    const int *tab;
    // + one flag per tap after the table: no second term anywhere in the tile -> the single-load path
    __device__ __forceinline__ void setup(int x0, int *smem) {
        const int kk = g.k * g.k, Q = g.Hs * g.Ws;
        int *multi = smem + kk * 64 * 4;
        int4 e[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = threadIdx.x + 256 * u, kyx = i >> 6, q = x0 + (i & 63);
            e[u] = (kyx < kk && q < Q) ? adj[(int64_t)kyx * Q + q] : int4{kOob, kOob, kOob, kOob};
        }
        if (threadIdx.x < kk) multi[threadIdx.x] = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = threadIdx.x + 256 * u;
            if ((i >> 6) < kk) {
                *reinterpret_cast<int4 *>(smem + 4 * i) = e[u];
                if ((e[u].y & e[u].z & e[u].w) != kOob) atomicOr(multi + (i >> 6), 1);
            }
        }
        tab = smem;
    }
    __device__ __forceinline__ void load(int, int k0, int kend, int j, float (&v)[8]) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + 8 * sm_kg(j));   // wave-uniform (as SmFwd)
        const int kyx = r0 / Cop, c0 = r0 - kyx * Cop;
        const int pb = g.Ho * g.Wo * 4;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(GZ, gbytes);
        int4 o = int4{kOob, kOob, kOob, kOob};
        if (r0 < kend) o = *reinterpret_cast<const int4 *>(tab + 4 * (kyx * 64 + sm_row(j)));
        // every load issued before any is used (a channel >= Cout reads channel Cout - 1 and meets zero
        // weights, SmPre): written "c < Cout ? loads : 0", each channel's loads were branched around
        // and waited for in turn (s_waitcnt vmcnt(0) per channel, tools/micro/gemm_phase's finding)
        if (r0 >= kend || !__builtin_amdgcn_readfirstlane(tab[g.k * g.k * 64 * 4 + kyx])) {   // one term per pixel
            s3_bload_chans(rs, o.x, c0, Cout, pb, v);
            return;
        }
        float t[4][8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int so = min(c0 + u, Cout - 1) * pb;
            t[0][u] = s3_bload(rs, o.x, so);
            t[1][u] = s3_bload(rs, o.y, so);
            t[2][u] = s3_bload(rs, o.z, so);
            t[3][u] = s3_bload(rs, o.w, so);
        }
        // fixed order (deterministic); terms past the list read kOob = 0
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ((t[0][u] + t[1][u]) + t[2][u]) + t[3][u];
    }
};

// A: a dense fp32 [X][ld] matrix, k contiguous (dL/dz of the weight gradient, k = output pixel);
// split into the three planes at the LDS store
struct SmDense {
    static constexpr bool pre = false;
    const float *S;
    int ld, X;
    // buffer loads, the zeros by address (kOob) so no load is branched around (host: X ld 4 < kOob)
    __device__ __forceinline__ void load(int x0, int k0, int kend, int j, float (&v)[8]) const {
        const int x = x0 + sm_row(j), k = k0 + 8 * sm_kg(j);
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(S, X * ld * 4);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s3_bload(rs, (x < X && k + u < kend) ? 4 * (x * ld + k + u) : kOob, 0);
    }
};

// B of the weight gradient: col^T[p][r], r = c kk + tap (dW's own column order), p = output pixel:
// x[c] at the source pixel of (p, tap), from the conv's table tw[tap][P] of byte offsets within a
// channel plane (kOob = zero pad; built on the host, sm_wgrad_table).  No LDS table.
struct SmWgrad {
    const float *X;
    int xbytes;
    int Kc, kk, P, plane;   // plane = Hs Ws 4 bytes
    const int *tw;
    __device__ __forceinline__ void setup(int, int *) {}
    __device__ __forceinline__ void load(int x0, int k0, int kend, int j, float (&v)[8]) const {
        const int r = x0 + sm_row(j), p0 = k0 + 8 * sm_kg(j);
        const int c = r / kk, tap = r - c * kk;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, xbytes);
        const int base = r < Kc ? c * plane : kOob;
        // the eight table entries in flight together (clamped index, no branch), then the gathers
        int o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = tw[min(tap, kk - 1) * P + min(p0 + u, kend - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = s3_bload(rs, (p0 + u >= kend || o[u] == kOob || base == kOob) ? kOob : base + o[u], 0);
    }
};

template <class LA>
struct SmAReg {   // the A operand's registers for one load group
    uint4 h[3];
};
template <>
struct SmAReg<SmDense> {
    float v[8];
};

template <class LB, class LA = SmPre>
__global__ __launch_bounds__(256, 2) void k_conv_sm(GemmArgs g, LA la, LB lb) {
    __shared__ __attribute__((aligned(16))) SmImg As, Bs;
    __shared__ __attribute__((aligned(16))) int tab[kSmTabInts];
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 32, wn = (wv & 1) * 32;
    const int jl = lane & 15, gk = lane >> 4;
    lb.setup(n0, tab);
    __syncthreads();
    s3f4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    SmAReg<LA> ha[2];
    float vb[2][8];
    auto lda = [&](int k0, int j) {
        if constexpr (LA::pre) la.load(m0, k0, kend, j, ha[j].h);
        else la.load(m0, k0, kend, j, ha[j].v);
    };
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        lda(kbeg, j);
        lb.load(n0, kbeg, kend, j, vb[j]);
    }
    for (int k0 = kbeg; k0 < kend; k0 += kSmK) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if constexpr (LA::pre) sm_store_pre(As, sm_row(j), sm_kg(j), ha[j].h);
            else sm_store_f32(As, sm_row(j), sm_kg(j), ha[j].v);
            sm_store_f32(Bs, sm_row(j), sm_kg(j), vb[j]);
        }
        __syncthreads();
        if (k0 + kSmK < kend) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                lda(k0 + kSmK, j);
                lb.load(n0, k0 + kSmK, kend, j, vb[j]);
            }
        }
#pragma unroll
        for (int s = 0; s < kSmK / 32; ++s) {
            s3bf8 fa[2][3], fb[2][3];
#pragma unroll
            for (int a = 0; a < 2; ++a) sm_frag(As, wm + 16 * a + jl, 4 * s + gk, fa[a]);
#pragma unroll
            for (int b = 0; b < 2; ++b) sm_frag(Bs, wn + 16 * b + jl, 4 * s + gk, fb[b]);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = s3_mfma6(fa[a], fb[b], acc[a][b]);
        }
        __syncthreads();
    }
    float *C = g.C + (int64_t)blockIdx.z * g.M * g.N;
    const bool final_out = gridDim.z == 1;
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
                        if (g.div) v = v / *g.div;
                        if (g.accum) v = C[(int64_t)m * g.N + n] + v;
                    }
                    C[(int64_t)m * g.N + n] = v;
                }
            }
        }
}

}  // namespace lrs
