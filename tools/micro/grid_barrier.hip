// What a grid-wide barrier costs inside one persistent launch on MI355X, against a launch boundary
// (the persistent small-map section of the 36^2 U-Net pays only if a barrier
// is well under the ~10 us a dependent launch pair costs there).  tools/micro/grid_barrier
//
//   launch   : R back-to-back launches of an empty G-workgroup kernel on one stream (per launch), and of
//              a "layer" kernel (each workgroup reads 4 KB written by another workgroup in the previous
//              launch and writes 4 KB): the launch boundary a persistent kernel would replace
//   barrier  : one launch of G workgroups running R rounds of an atomic-counter grid barrier (thread 0
//              adds 1 to a monotonic agent-scope counter and polls it until it reaches G * round),
//              polling with and without s_sleep
//   exchange : the same barrier with the layer's data hand-off around it: each workgroup writes 4 KB,
//              releases (agent scope: its XCD's L2 written back so other XCDs see it), arrives, waits,
//              acquires and reads the 4 KB another workgroup (on another XCD) wrote
// Every poll loop has a cap (1 << 24 polls): a workgroup that hits it records a timeout and leaves, so
// the grid always drains; the run reports any timeout.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/grid_barrier tools/micro/grid_barrier.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int kTh = 256, kWords = 1024;   // 4 KB per workgroup per layer
constexpr unsigned kCap = 1u << 24;

__global__ void k_empty() {}

// one layer of the launch chain: read the 4 KB of workgroup (b + 37) % G written last launch, write own
__global__ void k_layer(const float *in, float *out, int G) {
    const int b = blockIdx.x, src = (b + 37) % G;
    float acc = 0.0f;
    for (int i = threadIdx.x; i < kWords; i += kTh) acc += in[(size_t)src * kWords + i];
    for (int i = threadIdx.x; i < kWords; i += kTh) out[(size_t)b * kWords + i] = acc + (float)i;
}

__device__ __forceinline__ bool grid_wait(unsigned *cnt, unsigned target, bool sleep, unsigned *timeout) {
    unsigned n = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if (++n >= kCap) {
            __hip_atomic_fetch_add(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    return true;
}

// mode 0: barrier only, busy poll; 1: barrier only, s_sleep poll; 2: exchange (data hand-off), s_sleep
__global__ void k_persist(unsigned *cnt, unsigned *timeout, float *buf, int rounds, int mode) {
    const int G = gridDim.x, b = blockIdx.x, src = (b + 37) % G;
    __shared__ int ok;
    float acc = 0.0f;
    for (int r = 1; r <= rounds; ++r) {
        float *cur = buf + (size_t)(r & 1) * G * kWords, *prev = buf + (size_t)((r + 1) & 1) * G * kWords;
        if (mode == 2) {
            for (int i = threadIdx.x; i < kWords; i += kTh) acc += prev[(size_t)src * kWords + i];
            for (int i = threadIdx.x; i < kWords; i += kTh) cur[(size_t)b * kWords + i] = acc + (float)i;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            // release: this workgroup's writes (mode 2) visible at agent scope before the arrival
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            ok = grid_wait(cnt, (unsigned)(G * r), mode != 0, timeout) ? 1 : 0;
        }
        __syncthreads();
        if (!ok) return;   // a timed-out workgroup leaves; the others time out too and drain
    }
    if (acc == 12345.678f) buf[0] = acc;   // keep the loads
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 2000;
    float *buf, *buf2;
    unsigned *cnt, *timeout;
    CK(hipMalloc(&buf, (size_t)2 * 1024 * kWords * sizeof(float)));
    CK(hipMalloc(&buf2, (size_t)2 * 1024 * kWords * sizeof(float)));
    CK(hipMemset(buf, 0, (size_t)2 * 1024 * kWords * sizeof(float)));
    CK(hipMalloc(&cnt, 4));
    CK(hipMalloc(&timeout, 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("R = %d rounds / launches; times in us per round\n", R);
    printf("%6s %12s %12s %14s %14s %16s\n", "G", "launch_empty", "launch_layer", "barrier_spin", "barrier_sleep",
           "barrier_exchange");
    for (int G : {64, 128, 256, 512}) {
        float ms;
        double res[5];
        // launch chains (warm first)
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_empty, dim3(G), dim3(kTh), 0, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
        }
        res[0] = 1e3 * ms / R;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < R; ++r)
                hipLaunchKernelGGL(k_layer, dim3(G), dim3(kTh), 0, st, (r & 1) ? buf2 : buf, (r & 1) ? buf : buf2, G);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
        }
        res[1] = 1e3 * ms / R;
        for (int mode = 0; mode < 3; ++mode) {
            double t[2];
            for (int k = 0; k < 2; ++k) {   // R rounds and 0 rounds: the difference is the barriers
                const int rounds = k == 0 ? R : 0;
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipMemsetAsync(cnt, 0, 4, st));
                    CK(hipMemsetAsync(timeout, 0, 4, st));
                    CK(hipEventRecord(e0, st));
                    hipLaunchKernelGGL(k_persist, dim3(G), dim3(kTh), 0, st, cnt, timeout, buf, rounds, mode);
                    CK(hipEventRecord(e1, st));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    unsigned to = 0;
                    CK(hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost));
                    if (to) {
                        printf("G = %d mode %d: %u workgroups timed out (not all resident?)\n", G, mode, to);
                        return 1;
                    }
                }
                t[k] = ms;
            }
            res[2 + mode] = 1e3 * (t[0] - t[1]) / R;
        }
        printf("%6d %12.2f %12.2f %14.2f %14.2f %16.2f\n", G, res[0], res[1], res[2], res[3], res[4]);
    }
    CK(hipStreamDestroy(st));
    return 0;
}
