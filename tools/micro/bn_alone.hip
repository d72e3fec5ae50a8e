// The one-workgroup-per-channel BatchNorm kernels alone (tools/micro/bn_alone): k_reduce_bn1 and
// k_bn_fwd_r on the 196^2 U-Net's shapes (128 channels; 49^2 with 9 split-K partials, 98^2 with 6),
// back-to-back launches on an idle GPU, to compare with their duration inside the training step
// (beside the weight-gradient stream): is a BN kernel slow by itself or by sharing the chip?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lrs-pnp-dip_amd/csrc -I include \
//         -o tools/micro/bn_alone tools/micro/bn_alone.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "dip_kernels.h"

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

template <class F>
float timeit(F f, int reps) {
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int w = 0; w < 10; ++w) f();
    CK(hipEventRecord(t0, 0));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(t1, 0));
    CK(hipEventSynchronize(t1));
    float ms;
    CK(hipEventElapsedTime(&ms, t0, t1));
    return 1e3f * ms / reps;
}

__global__ void k_empty(float *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p == nullptr) p[0] = 0.f;
}

int main() {
    const int C = 128;
    float *part, *z, *y, *g, *bt, *m, *is, *rm, *rv, *bias;
    CK(hipMalloc(&part, 9LL * C * 9604 * 4));
    CK(hipMalloc(&z, (int64_t)C * 38416 * 4));
    CK(hipMalloc(&y, (int64_t)C * 38416 * 4));
    for (float **q : {&g, &bt, &m, &is, &rm, &rv, &bias}) CK(hipMalloc(q, C * 4));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, part, 9LL * C * 9604, 1u);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, g, (int64_t)C, 2u);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, bt, (int64_t)C, 3u);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, bias, (int64_t)C, 4u);
    printf("empty kernel, 128 workgroups: %6.2f us\n",
           timeit([&]() { hipLaunchKernelGGL(k_empty, dim3(128), dim3(1024), 0, 0, y); }, 500));
    {
        const int P = 2401, S = 9;
        BnArgs a{z, y, g, bt, m, is, rm, rv, nullptr, C, P, 1, P, 1, LRS_ACT_LRELU, 1e-5f, 0.1f, 1, 0};
        printf("k_reduce_bn1<1024>, 49^2, %d partials: %6.2f us\n", S,
               timeit([&]() { hipLaunchKernelGGL(k_reduce_bn1<1024>, dim3(1, C), dim3(1024), 0, 0, (const float *)part, S, (const float *)bias, a, (const float *)nullptr); }, 500));
    }
    {
        const int P = 625, S = 8;
        BnArgs a{z, y, g, bt, m, is, rm, rv, nullptr, C, P, 1, P, 1, LRS_ACT_LRELU, 1e-5f, 0.1f, 1, 0};
        printf("k_reduce_bn1<1024>, 25^2, %d partials: %6.2f us\n", S,
               timeit([&]() { hipLaunchKernelGGL(k_reduce_bn1<1024>, dim3(1, C), dim3(1024), 0, 0, (const float *)part, S, (const float *)bias, a, (const float *)nullptr); }, 500));
        printf("k_reduce_bn1<256>,  25^2, %d partials: %6.2f us\n", S,
               timeit([&]() { hipLaunchKernelGGL(k_reduce_bn1<256>, dim3(1, C), dim3(256), 0, 0, (const float *)part, S, (const float *)bias, a, (const float *)nullptr); }, 500));
    }
    {
        const int P = 9604, S = 6;
        BnArgs a{z, y, g, bt, m, is, rm, rv, nullptr, C, P, 1, P, 1, LRS_ACT_LRELU, 1e-5f, 0.1f, 1, 1};
        printf("k_bn_fwd_r<3>, 98^2, %d partials: %6.2f us\n", S,
               timeit([&]() { hipLaunchKernelGGL((k_bn_fwd_r<3, 1024>), dim3(1, C), dim3(1024), 0, 0, (const float *)part, S, (const float *)bias, a, (const float *)nullptr); }, 500));
    }
    {
        const int P = 38416;
        BnArgs a{z, y, g, bt, m, is, rm, rv, nullptr, C, P, 1, P, 1, LRS_ACT_LRELU, 1e-5f, 0.1f, 1, 1};
        printf("k_bn_fwd_r<10>, 196^2, z given: %6.2f us\n",
               timeit([&]() { hipLaunchKernelGGL((k_bn_fwd_r<10, 1024>), dim3(1, C), dim3(1024), 0, 0, (const float *)nullptr, 1, (const float *)bias, a, (const float *)nullptr); }, 500));
    }
    return 0;
}
