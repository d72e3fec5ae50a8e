// Where the time of one implicit-GEMM conv launch goes (tools/micro/gemm_shape): k_gemm_s3<LdPre,
// LdFwdTM> alone on the 196^2 U-Net's conv shapes, timed over back-to-back launches, for a range of
// split-K counts S and of K truncations, so the per-workgroup fixed cost (tables, first loads,
// epilogue) separates from the per-k-step cost.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/gemm_shape tools/micro/gemm_shape.hip
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

__global__ void k_fill(float *p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (float)(h & 0xFFFF) / 65536.0f - 0.5f;
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    struct Shape {
        const char *name;
        int Cin, H, stride, Cout;
    } shapes[] = {{"98x98 3x3 s1 128->128", 128, 98, 1, 128}, {"98->49 3x3 s2 128->128", 128, 98, 2, 128},
                  {"49x49 3x3 s1 128->128", 128, 49, 1, 128}};
    float *x, *y, *part;
    __bf16 *wp;
    const int64_t xmax = 128LL * 98 * 98, pmax = 64LL * 128 * 9604;
    CK(hipMalloc(&x, xmax * 4));
    CK(hipMalloc(&y, 128LL * 9604 * 4));
    CK(hipMalloc(&part, pmax * 4));
    CK(hipMalloc(&wp, 3LL * 128 * 9 * 128 * 2));
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, x, xmax, 1u);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (float *)wp, 3LL * 128 * 9 * 128 / 2, 2u);
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (const Shape &s : shapes) {
        ConvGeom g{};
        g.Cin = s.Cin;
        g.Hs = g.Ws = g.Hu = g.Wu = s.H;
        g.up = 0;
        g.pad = 1;
        g.pad_mode = LRS_PAD_REFLECT;
        g.k = 3;
        g.stride = s.stride;
        g.Ho = g.Wo = (s.H + 2 - 3) / s.stride + 1;
        const int P = g.Ho * g.Wo, Cp = 128, Kfull = 9 * Cp;
        const int tiles = (P + 127) / 128;
        printf("%s: P %d, %d N-tiles, K %d\n", s.name, P, tiles, Kfull);
        const int Ks[] = {Kfull, Kfull / 2, Kfull / 4, 96, 32};
        for (int K : Ks) {
            const int Ss[] = {1, 2, 3, 4, 6, 9, 12, 18, 36};
            for (int S : Ss) {
                int kchunk = (K + S - 1) / S;
                kchunk = (kchunk + 31) / 32 * 32;
                const int Sr = (K + kchunk - 1) / kchunk;
                if (Sr != S || (int64_t)S * 128 * P > pmax) continue;
                GemmArgs a{nullptr, nullptr, S > 1 ? part : y, nullptr, nullptr, s.Cout, P, K, kchunk, 0, 0, 0, 0, 0};
                LdPre la{wp, (int64_t)128 * 9 * Cp, 9 * Cp, s.Cout};
                LdFwdTM lb{x, g.Cin * g.Hs * g.Ws * 4, g, Cp, nullptr};
                const dim3 grid(tiles, 1, S);
                for (int w = 0; w < 10; ++w) hipLaunchKernelGGL((k_gemm_s3<LdPre, LdFwdTM>), grid, dim3(256), 0, 0, a, la, lb);
                CK(hipEventRecord(t0, 0));
                for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_gemm_s3<LdPre, LdFwdTM>), grid, dim3(256), 0, 0, a, la, lb);
                CK(hipEventRecord(t1, 0));
                CK(hipEventSynchronize(t1));
                float ms;
                CK(hipEventElapsedTime(&ms, t0, t1));
                const double us = 1e3 * ms / reps, flop = 2.0 * s.Cout * P * (double)K;
                printf("  K %4d S %2d: %4d WGs, %3d k-steps/WG: %7.2f us  %6.1f TFLOP/s (fp32-equiv)\n", K, S, tiles * S,
                       kchunk / 32, us, flop / us * 1e-6);
            }
        }
    }
    return 0;
}
