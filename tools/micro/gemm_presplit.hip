// Is the B operand's split worth removing? (tools/micro/gemm_presplit)  k_gemm_s3's non-prepared
// loop (dip_gemm.h) on the 98^2 conv with B read from activations stored PRE-SPLIT as three bf16
// planes in a pixel-major layout ([plane][pixel][Cp]: a thread's 16 channels at one pixel are two
// 16-B pieces per plane, stored to LDS without VALU, like the weight planes), against the current
// fp32 [C][P] gathers split per value.  Same products, so the two must agree bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/gemm_presplit tools/micro/gemm_presplit.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "dip_kernels.h"
#include "dip_gemm.h"

using namespace lrs;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// B from pixel-major planes: tab = the source pixel's byte offset in a plane (pixel * Cp * 2) or kOob
struct LdFwdPlanes {
    const __bf16 *X;   // [3][Ps][Cp]
    int plane_bytes;   // Ps * Cp * 2
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
            tab[kyx * 128 + r] = (in && sy >= 0 && sx >= 0) ? (sy * g.Ws + sx) * Cp * 2 : kOob;
        }
    }
    __device__ __forceinline__ void load(int, int k0, int kend, RegP &r) const {
        const int r0 = __builtin_amdgcn_readfirstlane(k0 + s3_kb<false>());
        const int rr = r0 < kend ? r0 : 0, kyx = rr / Cp, c0 = rr - kyx * Cp;
        const __amdgpu_buffer_rsrc_t rs = s3_rsrc(X, 3 * plane_bytes);
        const int vo = tab[kyx * 128 + s3_row<false>()];
        const int v2 = vo == kOob ? kOob : vo + 2 * c0;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            r.h[p][0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, v2, p * plane_bytes, 0));
            r.h[p][1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, v2, p * plane_bytes + 16, 0));
        }
    }
};

__device__ __forceinline__ void store_pre_b(S3Tile &T, const RegP &r) {   // the B (non-KC) thread mapping
    const int row = s3_row<false>(), c0 = s3_kb<false>() >> 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch = s3_chunk(row, c0 + h) * 8;
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4 *>(&T.v[p][row][ch]) = r.h[p][h];
    }
}

__global__ __launch_bounds__(256, 2) void k_presplit(GemmArgs g, LdPre la, LdFwdPlanes lb) {
    __shared__ __attribute__((aligned(16))) struct { S3Tile a, b; } ab;
    S3Tile &As = ab.a, &Bs = ab.b;
    __shared__ __attribute__((aligned(16))) int tab[kS3TabInts];
    const int T = gridDim.x * gridDim.y * gridDim.z;
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = L & 7, q8 = T >> 3, r8 = T & 7;
    const int j = xcd * q8 + min(xcd, r8) + (L >> 3);
    const int bx = j % gridDim.x, byz = j / gridDim.x, by = byz % gridDim.y, bz = byz / gridDim.y;
    const int m0 = by * 128, n0 = bx * 128, kz = bz;
    const int kbeg = kz * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    la.setup(m0, tab, 0);
    RegP pa, b0;
    la.load(m0, kbeg, kend, pa);
    __builtin_amdgcn_sched_barrier(0);
    lb.setup(n0, tab, 0);
    __syncthreads();
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
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
    __builtin_amdgcn_sched_barrier(0);
    lb.load(n0, kbeg, kend, b0);
    for (int k0 = kbeg; k0 < kend; k0 += kS3K) {   // both operands one step ahead: no spill
        s3_store_pre(As, pa);
        store_pre_b(Bs, b0);
        __syncthreads();
        la.load(m0, k0 + kS3K, kend, pa);
        __builtin_amdgcn_sched_barrier(0);
        lb.load(n0, k0 + kS3K, kend, b0);
        mma();
        __syncthreads();
    }
    float *C = g.C + (int64_t)kz * g.M * g.N;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int n = n0 + wn + 16 * b + jl;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * a + 4 * gk + r;
                if (m < g.M && n < g.N) C[(int64_t)m * g.N + n] = acc[a][b][r];
            }
        }
}

// x [C][Ps] fp32 -> [3][Ps][Cp] bf16 planes (s3_split), channels >= C zero
__global__ void k_planes(const float *x, int C, int Ps, int Cp, __bf16 *out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)Ps * Cp) return;
    const int p = (int)(i / Cp), c = (int)(i - (int64_t)p * Cp);
    const S3Split q = s3_split(c < C ? x[(int64_t)c * Ps + p] : 0.0f);
    out[i] = q.b0;
    out[(int64_t)Ps * Cp + i] = q.b1;
    out[2 * (int64_t)Ps * Cp + i] = q.b2;
}

__global__ void k_fill(float *p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (float)(h & 0xFFFF) / 65536.0f - 0.5f;
    }
}

int main() {
    const int H = 98, C = 128, Cp = 128, Ps = H * H, P = H * H, K = 9 * Cp, tiles = (P + 127) / 128;
    float *x, *o1, *o2;
    __bf16 *wp, *xp;
    CK(hipMalloc(&x, (int64_t)C * Ps * 4));
    CK(hipMalloc(&xp, 3LL * Ps * Cp * 2));
    CK(hipMalloc(&o1, 12LL * 128 * P * 4));
    CK(hipMalloc(&o2, 12LL * 128 * P * 4));
    CK(hipMalloc(&wp, 3LL * 128 * 9 * 128 * 2));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, x, (int64_t)C * Ps, 1u);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (float *)wp, 3LL * 128 * 9 * 128 / 2, 2u);
    hipLaunchKernelGGL(k_planes, dim3((Ps * Cp + 255) / 256), dim3(256), 0, 0, x, C, Ps, Cp, xp);
    ConvGeom g{};
    g.Cin = C;
    g.Hs = g.Ws = g.Hu = g.Wu = H;
    g.pad = 1;
    g.pad_mode = LRS_PAD_REFLECT;
    g.k = 3;
    g.stride = 1;
    g.Ho = g.Wo = H;
    LdPre la{wp, (int64_t)128 * 9 * Cp, 9 * Cp, 128};
    LdFwdTM lb{x, C * Ps * 4, g, Cp, nullptr};
    LdFwdPlanes lp{xp, Ps * Cp * 2, g, Cp, nullptr};
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const int Ss[] = {1, 2, 3, 6, 9};
    for (int S : Ss) {
        const int kchunk = ((K + S - 1) / S + 31) / 32 * 32;
        GemmArgs a1{nullptr, nullptr, o1, nullptr, nullptr, 128, P, K, kchunk, 0, 0, 0, 0, 0};
        GemmArgs a2 = a1;
        a2.C = o2;
        const dim3 grid(tiles, 1, S);
        float ms[2];
        for (int v = 0; v < 2; ++v) {
            auto go = [&]() {
                if (v == 0) hipLaunchKernelGGL((k_gemm_s3<LdPre, LdFwdTM>), grid, dim3(256), 0, 0, a1, la, lb);
                else hipLaunchKernelGGL(k_presplit, grid, dim3(256), 0, 0, a2, la, lp);
            };
            for (int w = 0; w < 10; ++w) go();
            CK(hipEventRecord(t0, 0));
            for (int r = 0; r < 200; ++r) go();
            CK(hipEventRecord(t1, 0));
            CK(hipEventSynchronize(t1));
            CK(hipEventElapsedTime(&ms[v], t0, t1));
        }
        const size_t n = (size_t)S * 128 * P;
        std::vector<float> h1(n), h2(n);
        CK(hipMemcpy(h1.data(), o1, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), o2, n * 4, hipMemcpyDeviceToHost));
        printf("98^2 conv S %d (%d k-steps): fp32 gathers + split %7.2f us | pre-split planes %7.2f us | %s\n", S, kchunk / 32,
               ms[0] * 5, ms[1] * 5, memcmp(h1.data(), h2.data(), n * 4) ? "DIFFER" : "bit-identical");
    }
    return 0;
}
