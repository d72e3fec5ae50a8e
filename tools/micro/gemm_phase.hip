// Per-phase cycle accounting of the implicit-GEMM conv main loop (tools/micro/gemm_phase): an
// instrumented copy of k_gemm_s3's non-prepared path (dip_gemm.h) with s_memtime stamps per wave at
// each phase boundary, run on the 98^2 / 49^2 U-Net conv shapes.  The stamps cost ~10 % of the wave
// cycles (MI355X_MICROARCH.md), so the split between phases is the result, not the totals.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/gemm_phase tools/micro/gemm_phase.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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

enum { kSetup, kFirstLoads, kWait, kStore, kBar1, kIssue, kIssueB, kMma, kBar2, kEpi, kNPh };
static const char *kPhName[kNPh] = {"setup+bar", "first loads", "wait data", "split+store", "barrier 1", "issue A", "issue B", "mma", "barrier 2", "epilogue"};

#define STAMP(ph)                                           \
    do {                                                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
        ph_acc[ph] += t_ - t_last;                          \
        t_last = t_;                                        \
    } while (0)

template <class LA, class LB>
__global__ __launch_bounds__(256, 2) void k_gemm_s3_phase(GemmArgs g, LA la, LB lb, unsigned long long *prof) {
    uint64_t ph_acc[kNPh] = {};
    uint64_t t_last = __builtin_amdgcn_s_memtime();
    const uint64_t t_begin = t_last;
    __shared__ __attribute__((aligned(16))) struct { S3Tile a, b; } ab;
    S3Tile &As = ab.a, &Bs = ab.b;
    __shared__ __attribute__((aligned(16))) int tab[kS3TabInts];
    const int T = gridDim.x * gridDim.y * gridDim.z;
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = L & 7, q8 = T >> 3, r8 = T & 7;
    const int j = xcd * q8 + min(xcd, r8) + (L >> 3);
    const int bx = j % gridDim.x, byz = j / gridDim.x, by = byz % gridDim.y, bz = byz / gridDim.y;
    const int m0 = by * 128, n0 = bx * 128;
    const int kz = bz;
    const int kbeg = kz * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    la.setup(m0, tab, 0);
    lb.setup(n0, tab, 0);
    __syncthreads();
    STAMP(kSetup);
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    float vb[16], vb1[16];
    RegP pa;
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
    auto st = [&](const float (&b)[16]) {
        s3_store_pre(As, pa);
        s3_store<LB::kc>(Bs, b);
    };
    la.load(m0, kbeg, kend, pa);
    lb.load(n0, kbeg, kend, vb);
    if (kbeg + kS3K < kend) lb.load(n0, kbeg + kS3K, kend, vb1);
    __builtin_amdgcn_s_waitcnt(0);   // account the first loads' latency here (instrumentation only)
    STAMP(kFirstLoads);
    for (int k0 = kbeg; k0 < kend; k0 += 2 * kS3K) {
        // vmcnt(16): everything but the newest 16 loads (the B loads of the step after next) has
        // arrived: the wait for this step's operands (near the end of the loop it waits for more)
        __builtin_amdgcn_s_waitcnt(0x4F70);
        STAMP(kWait);
        st(vb);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        STAMP(kStore);
        __syncthreads();
        STAMP(kBar1);
        if (k0 + kS3K < kend) la.load(m0, k0 + kS3K, kend, pa);
        STAMP(kIssue);
        if (k0 + 2 * kS3K < kend) lb.load(n0, k0 + 2 * kS3K, kend, vb);
        STAMP(kIssueB);
        mma();
        __builtin_amdgcn_s_waitcnt(0xc07f);
        STAMP(kMma);
        __syncthreads();
        STAMP(kBar2);
        if (k0 + kS3K >= kend) break;
        __builtin_amdgcn_s_waitcnt(0x4F70);
        STAMP(kWait);
        st(vb1);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        STAMP(kStore);
        __syncthreads();
        STAMP(kBar1);
        if (k0 + 2 * kS3K < kend) la.load(m0, k0 + 2 * kS3K, kend, pa);
        STAMP(kIssue);
        if (k0 + 3 * kS3K < kend) lb.load(n0, k0 + 3 * kS3K, kend, vb1);
        STAMP(kIssueB);
        mma();
        __builtin_amdgcn_s_waitcnt(0xc07f);
        STAMP(kMma);
        __syncthreads();
        STAMP(kBar2);
    }
    float *C = g.C + (int64_t)kz * g.M * g.N;
    float *E = reinterpret_cast<float *>(&ab) + wv * 32 * 68;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) E[(16 * a2 + 4 * gk + r) * 68 + 16 * b + jl] = acc[2 * hf + a2][b][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int idx = lane + 64 * i, rr = idx >> 4, q = 4 * (idx & 15);
            const int m = m0 + wm + 32 * hf + rr, n = n0 + wn + q;
            if (m < g.M && n < g.N) *reinterpret_cast<float4 *>(C + (int64_t)m * g.N + n) = *reinterpret_cast<const float4 *>(E + rr * 68 + q);
        }
        __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(kEpi);
    if (lane == 0) {
        unsigned long long *o = prof + ((int64_t)L * 4 + wv) * (kNPh + 2);
#pragma unroll
        for (int p = 0; p < kNPh; ++p) o[p] = ph_acc[p];
        o[kNPh] = t_begin;
        o[kNPh + 1] = t_last;
    }
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
    float *x, *part;
    __bf16 *wp;
    unsigned long long *prof;
    const int64_t xmax = 128LL * 98 * 98, pmax = 12LL * 128 * 9604;
    CK(hipMalloc(&x, xmax * 4));
    CK(hipMalloc(&part, pmax * 4));
    CK(hipMalloc(&wp, 3LL * 128 * 9 * 128 * 2));
    CK(hipMalloc(&prof, 8192LL * 4 * (kNPh + 2) * 8));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, x, xmax, 1u);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (float *)wp, 3LL * 128 * 9 * 128 / 2, 2u);
    struct Run {
        int H, stride, S;
    } runs[] = {{98, 1, 1}, {98, 1, 3}, {98, 1, 6}, {98, 1, 12}, {49, 1, 1}, {49, 1, 9}, {98, 2, 9}};
    for (const Run &r : runs) {
        ConvGeom g{};
        g.Cin = 128;
        g.Hs = g.Ws = g.Hu = g.Wu = r.H;
        g.pad = 1;
        g.pad_mode = LRS_PAD_REFLECT;
        g.k = 3;
        g.stride = r.stride;
        g.Ho = g.Wo = (r.H + 2 - 3) / r.stride + 1;
        const int P = g.Ho * g.Wo, Cp = 128, K = 9 * Cp, tiles = (P + 127) / 128;
        const int kchunk = ((K + r.S - 1) / r.S + 31) / 32 * 32;
        GemmArgs a{nullptr, nullptr, part, nullptr, nullptr, 128, P, K, kchunk, 0, 0, 0, 0, 0};
        LdPre la{wp, (int64_t)128 * 9 * Cp, 9 * Cp, 128};
        LdFwdTM lb{x, g.Cin * g.Hs * g.Ws * 4, g, Cp, nullptr};
        const int nwg = tiles * r.S;
        for (int w = 0; w < 5; ++w)
            hipLaunchKernelGGL((k_gemm_s3_phase<LdPre, LdFwdTM>), dim3(tiles, 1, r.S), dim3(256), 0, 0, a, la, lb, prof);
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h((size_t)nwg * 4 * (kNPh + 2));
        CK(hipMemcpy(h.data(), prof, h.size() * 8, hipMemcpyDeviceToHost));
        double sum[kNPh] = {0};
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int w = 0; w < nwg * 4; ++w) {
            const unsigned long long *o = &h[(size_t)w * (kNPh + 2)];
            for (int p = 0; p < kNPh; ++p) sum[p] += (double)o[p];
            t0 = std::min(t0, o[kNPh]);
            t1 = std::max(t1, o[kNPh + 1]);
        }
        const int steps = kchunk / 32;
        double tot = 0;
        for (int p = 0; p < kNPh; ++p) tot += sum[p];
        printf("%dx%d s%d S %d: %d WGs x %d k-steps; mean wave cycles %.0f (%.0f per k-step), first-to-last wave span %.0f cycles\n",
               r.H, r.H, r.stride, r.S, nwg, steps, tot / (nwg * 4), tot / (nwg * 4) / steps, (double)(t1 - t0));
        for (int p = 0; p < kNPh; ++p)
            printf("   %-12s %8.0f cycles/wave  %5.1f %%  (%.0f per k-step)\n", kPhName[p], sum[p] / (nwg * 4), 100 * sum[p] / tot,
                   sum[p] / (nwg * 4) / steps);
    }
    return 0;
}
