// k_fold_pad alone (tools/micro/fold_alone): the upsampled data gradient's fold of the 196^2 step
// (98^2 source grid extended by one pixel, 128 channels, 7 split-K partials, kPadClamp) and the 98^2
// stride-1 fold (padded 100^2, 6 partials, reflection), timed over back-to-back launches on an idle
// GPU, to separate the kernel's own time from the in-step time (40 / 25 us beside the weight-gradient
// stream).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/fold_alone tools/micro/fold_alone.hip
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

int main() {
    const int C = 128, H = 98, Qe = (H + 2) * (H + 2);
    float *part, *gx;
    CK(hipMalloc(&part, 8LL * C * Qe * 4));
    CK(hipMalloc(&gx, (int64_t)C * H * H * 4));
    CK(hipMemset(part, 0, 8LL * C * Qe * 4));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    struct Case {
        const char *name;
        int nsplit, mode;
    } cases[] = {{"upsampled dgrad fold (kPadClamp), 7 partials", 7, kPadClamp},
                 {"stride-1 dgrad fold (reflect), 6 partials", 6, LRS_PAD_REFLECT},
                 {"stride-1 dgrad fold (reflect), 1 partial", 1, LRS_PAD_REFLECT}};
    for (const Case &k : cases) {
        ConvGeom g{};
        g.Cin = C;
        g.Hs = g.Ws = g.Hu = g.Wu = H;
        g.pad = 1;
        g.pad_mode = k.mode;
        g.k = 3;
        g.stride = 1;
        g.Ho = g.Wo = H;
        const dim3 grid((H * H + 255) / 256, C);
        for (int w = 0; w < 10; ++w)
            hipLaunchKernelGGL(k_fold_pad, grid, dim3(256), 0, 0, part, k.nsplit, (int64_t)C * Qe, g, gx, 0);
        CK(hipEventRecord(t0, 0));
        for (int r = 0; r < 200; ++r)
            hipLaunchKernelGGL(k_fold_pad, grid, dim3(256), 0, 0, part, k.nsplit, (int64_t)C * Qe, g, gx, 0);
        CK(hipEventRecord(t1, 0));
        CK(hipEventSynchronize(t1));
        float ms;
        CK(hipEventElapsedTime(&ms, t0, t1));
        const double us = ms * 5, mb = (k.nsplit * (double)C * H * H + (double)C * H * H) * 4 / 1e6;
        printf("%s: %.2f us per launch, %.1f MB algorithmic -> %.2f TB/s\n", k.name, us, mb, mb / us);
    }
    return 0;
}
