// Producer / consumer waves for the implicit-GEMM conv, instrumented (tools/micro/gemm_pc): threads
// 0-255 load, split and store the next k-step (k_gemm_s3's 256-thread loader mapping), threads
// 256-511 issue the MFMAs on the other LDS stage; one barrier per step.  Per wave and per step the
// s_memtime cycles of its own work and of its wait at the barrier, so the slower role shows.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/gemm_pc tools/micro/gemm_pc.hip
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

__global__ __launch_bounds__(512, 1) void k_pc(GemmArgs g, LdPre la, LdFwdTM lb, unsigned long long *prof) {
    __shared__ __attribute__((aligned(16))) struct {
        S3Tile a[2], b[2];
        int tab[kS3TabInts];
    } sm;
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int T = gridDim.x * gridDim.y * gridDim.z;
    const int xcd = L & 7, q8 = T >> 3, r8 = T & 7;
    const int j = xcd * q8 + min(xcd, r8) + (L >> 3);
    const int bx = j % gridDim.x, byz = j / gridDim.x, bz = byz / gridDim.y;
    const int m0 = 0, n0 = bx * 128, kz = bz;
    const int kbeg = kz * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
    const bool producer = threadIdx.x < 256;
    const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) & 3;
    const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
    const int jl = lane & 15, gk = lane >> 4;
    uint64_t work = 0, wait = 0, t_last, ph[4] = {0, 0, 0, 0};
    s3f4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = s3f4{0.f, 0.f, 0.f, 0.f};
    RegP pa;
    float vb0[16], vb1[16];
    la.setup(m0, sm.tab, 0);
    if (producer) {
        la.load(m0, kbeg, kend, pa);
        lb.setup(n0, sm.tab, 0);
    }
    __syncthreads();
    if (producer) {
        lb.load(n0, kbeg, kend, vb0);
        lb.load(n0, kbeg + kS3K, kend, vb1);
        s3_store_pre(sm.a[0], pa);
        s3_store<false>(sm.b[0], vb0);
        la.load(m0, kbeg + kS3K, kend, pa);
        __builtin_amdgcn_sched_barrier(0);
        lb.load(n0, kbeg + 2 * kS3K, kend, vb0);
    }
    __syncthreads();
    t_last = __builtin_amdgcn_s_memtime();
    auto step = [&](int k0, int cur, float (&b)[16]) {
        if (producer) {
            __builtin_amdgcn_s_waitcnt(0x4F70);   // vmcnt(16): this step's A and B have arrived
            const uint64_t ta = __builtin_amdgcn_s_memtime();
            ph[0] += ta - t_last;
            s3_store_pre(sm.a[cur ^ 1], pa);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            const uint64_t tb = __builtin_amdgcn_s_memtime();
            ph[1] += tb - ta;
            s3_store<false>(sm.b[cur ^ 1], b);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            const uint64_t tc = __builtin_amdgcn_s_memtime();
            ph[2] += tc - tb;
            la.load(m0, k0 + 2 * kS3K, kend, pa);
            __builtin_amdgcn_sched_barrier(0);
            lb.load(n0, k0 + 3 * kS3K, kend, b);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            ph[3] += __builtin_amdgcn_s_memtime() - tc;
        } else if (k0 < kend) {
            s3bf8 fb[4][3];
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) s3_frag(sm.b[cur], wn + 16 * bb + jl, gk, fb[bb]);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                s3bf8 fa[3];
                s3_frag(sm.a[cur], wm + 16 * a + jl, gk, fa);
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) acc[a][bb] = s3_mfma6(fa, fb[bb], acc[a][bb]);
            }
            // the MFMA results: the wave's work ends when its last MFMA retires
            float s = acc[3][3][3];
            __asm__ volatile("" ::"v"(s));
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        work += t1 - t_last;
        __syncthreads();
        t_last = __builtin_amdgcn_s_memtime();
        wait += t_last - t1;
    };
    for (int k0 = kbeg; k0 < kend; k0 += 2 * kS3K) {
        step(k0, 0, vb1);
        step(k0 + kS3K, 1, vb0);
    }
    if (lane == 0) {
        prof[(L * 8 + (threadIdx.x >> 6)) * 6] = work;
        prof[(L * 8 + (threadIdx.x >> 6)) * 6 + 1] = wait;
        for (int i = 0; i < 4; ++i) prof[(L * 8 + (threadIdx.x >> 6)) * 6 + 2 + i] = ph[i];
    }
    if (!producer) {
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) s += acc[a][b][0];
        g.C[(int64_t)L * 256 + (threadIdx.x - 256)] = s;
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
    float *x, *out;
    __bf16 *wp;
    unsigned long long *prof;
    CK(hipMalloc(&x, 128LL * 98 * 98 * 4));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMalloc(&wp, 3LL * 128 * 9 * 128 * 2));
    CK(hipMalloc(&prof, 1 << 20));
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
    const int S = 1, kchunk = K;
    GemmArgs a{nullptr, nullptr, out, nullptr, nullptr, 128, P, K, kchunk, 0, 0, 0, 0, 0};
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_pc, dim3(tiles, 1, S), dim3(512), 0, 0, a, la, lb, prof);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(tiles * 8 * 6);
    CK(hipMemcpy(h.data(), prof, h.size() * 8, hipMemcpyDeviceToHost));
    double pw = 0, pq = 0, cw = 0, cq = 0, pp[4] = {0, 0, 0, 0};
    for (int l = 0; l < tiles; ++l)
        for (int w = 0; w < 8; ++w) {
            const double wk = h[(l * 8 + w) * 6], wt = h[(l * 8 + w) * 6 + 1];
            if (w < 4) {
                pw += wk; pq += wt;
                for (int i = 0; i < 4; ++i) pp[i] += h[(l * 8 + w) * 6 + 2 + i];
            } else { cw += wk; cq += wt; }
        }
    const double n = tiles * 4.0 * 36;
    printf("98^2 conv, 36 k-steps, producer/consumer waves: cycles per step per wave\n");
    printf("  producers: work %7.0f  barrier wait %7.0f\n", pw / n, pq / n);
    printf("  consumers: work %7.0f  barrier wait %7.0f\n", cw / n, cq / n);
    printf("  producer work: wait for data %7.0f, A store %7.0f, B split+store %7.0f, issue loads %7.0f\n", pp[0] / n, pp[1] / n,
           pp[2] / n, pp[3] / n);
    return 0;
}
