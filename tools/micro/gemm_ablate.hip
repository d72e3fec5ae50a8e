// Ablation of the implicit-GEMM conv main loop (tools/micro/gemm_ablate): a copy of k_gemm_s3's
// non-prepared loop (dip_gemm.h, LdPre x LdFwdTM) with parts switched off by DBG bits -- 1: the A
// (weight plane) loads inside the loop, 2: the B (gather) loads, 4: the MFMAs, 8: the LDS stores,
// 16: the split (B stored as one plane's bits) -- timed on the 98^2 conv at one workgroup per CU
// (S = 1, 36 k-steps) and at the step's split (S = 6).  Results are wrong by design; only the time
// per launch is read: which part the per-step time is made of.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/gemm_ablate tools/micro/gemm_ablate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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

template <int DBG>
__device__ __forceinline__ void ab_store_b(S3Tile &T, const float (&v)[16]) {
    if constexpr (DBG & 16) {   // no split: the fp32 bits' high halves into all three planes
        const int row = s3_row<false>(), c0 = s3_kb<false>() >> 3;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            s3bf8 p;
#pragma unroll
            for (int e = 0; e < 8; ++e) p[e] = __builtin_bit_cast(__bf16, (unsigned short)(__builtin_bit_cast(uint32_t, v[8 * h + e]) >> 16));
            const int ch = s3_chunk(row, c0 + h) * 8;
            *reinterpret_cast<s3bf8 *>(&T.v[0][row][ch]) = p;
            *reinterpret_cast<s3bf8 *>(&T.v[1][row][ch]) = p;
            *reinterpret_cast<s3bf8 *>(&T.v[2][row][ch]) = p;
        }
    } else {
        s3_store<false>(T, v);
    }
}

template <int DBG>
__global__ __launch_bounds__(256, 2) void k_ablate(GemmArgs g, LdPre la, LdFwdTM lb) {
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
    RegP pa;
    la.load(m0, kbeg, kend, pa);
    __builtin_amdgcn_sched_barrier(0);
    lb.setup(n0, tab, 0);
    __syncthreads();
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    float vb[16], vb1[16];
    auto mma = [&]() {
        if constexpr (DBG & 4) return;
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
    auto st = [&](const float (&b)[16]) {
        if constexpr (DBG & 8) return;
        s3_store_pre(As, pa);
        ab_store_b<DBG>(Bs, b);
    };
    auto ldA = [&](int k0) {
        if constexpr (!(DBG & 1)) la.load(m0, k0, kend, pa);
    };
    auto ldB = [&](int k0, float (&b)[16]) {
        if constexpr (!(DBG & 2)) lb.load(n0, k0, kend, b);
    };
    __builtin_amdgcn_sched_barrier(0);
    lb.load(n0, kbeg, kend, vb);
    lb.load(n0, kbeg + kS3K, kend, vb1);
    for (int k0 = kbeg; k0 < kend; k0 += 2 * kS3K) {
        st(vb);
        __syncthreads();
        ldA(k0 + kS3K);
        __builtin_amdgcn_sched_barrier(0);
        ldB(k0 + 2 * kS3K, vb);
        mma();
        __syncthreads();
        if (k0 + kS3K >= kend) break;
        st(vb1);
        __syncthreads();
        ldA(k0 + 2 * kS3K);
        __builtin_amdgcn_sched_barrier(0);
        ldB(k0 + 3 * kS3K, vb1);
        mma();
        __syncthreads();
    }
    // keep every result live: one float per thread
    float s = 0.0f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
    if (DBG & 4) s += vb[0] + vb1[5] + __builtin_bit_cast(float, pa.h[0][0].x);
    g.C[(int64_t)L * 256 + threadIdx.x] = s;
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

template <int DBG>
float run(const GemmArgs &a, const LdPre &la, const LdFwdTM &lb, dim3 grid, int reps) {
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(k_ablate<DBG>, grid, dim3(256), 0, 0, a, la, lb);
    CK(hipEventRecord(t0, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_ablate<DBG>, grid, dim3(256), 0, 0, a, la, lb);
    CK(hipEventRecord(t1, 0));
    CK(hipEventSynchronize(t1));
    float ms;
    CK(hipEventElapsedTime(&ms, t0, t1));
    return 1e3f * ms / reps;
}

int main() {
    float *x, *out;
    __bf16 *wp;
    CK(hipMalloc(&x, 128LL * 98 * 98 * 4));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMalloc(&wp, 3LL * 128 * 9 * 128 * 2));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, x, 128LL * 98 * 98, 1u);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (float *)wp, 3LL * 128 * 9 * 128 / 2, 2u);
    ConvGeom g{};
    g.Cin = 128;
    g.Hs = g.Ws = g.Hu = g.Wu = 98;
    g.pad = 1;
    g.pad_mode = LRS_PAD_REFLECT;
    g.k = 3;
    g.stride = 1;
    g.Ho = g.Wo = 98;
    const int P = 9604, Cp = 128, K = 9 * Cp, tiles = 76;
    LdPre la{wp, (int64_t)128 * 9 * Cp, 9 * Cp, 128};
    LdFwdTM lb{x, g.Cin * g.Hs * g.Ws * 4, g, Cp, nullptr};
    const int Ss[] = {1, 6};
    for (int S : Ss) {
        const int kchunk = ((K + S - 1) / S + 31) / 32 * 32;
        GemmArgs a{nullptr, nullptr, out, nullptr, nullptr, 128, P, K, kchunk, 0, 0, 0, 0, 0};
        const dim3 grid(tiles, 1, S);
        printf("98x98 conv, S %d (%d k-steps per workgroup):\n", S, kchunk / 32);
        printf("  full loop           %7.2f us\n", run<0>(a, la, lb, grid, 200));
        printf("  no A loads          %7.2f us\n", run<1>(a, la, lb, grid, 200));
        printf("  no B loads          %7.2f us\n", run<2>(a, la, lb, grid, 200));
        printf("  no A, B loads       %7.2f us\n", run<3>(a, la, lb, grid, 200));
        printf("  no MFMA             %7.2f us\n", run<4>(a, la, lb, grid, 200));
        printf("  no LDS stores       %7.2f us\n", run<8>(a, la, lb, grid, 200));
        printf("  no split            %7.2f us\n", run<16>(a, la, lb, grid, 200));
        printf("  MFMA only (no loads, stores) %7.2f us\n", run<11>(a, la, lb, grid, 200));
        printf("  loads only (no MFMA, stores) %7.2f us\n", run<12>(a, la, lb, grid, 200));
    }
    return 0;
}
