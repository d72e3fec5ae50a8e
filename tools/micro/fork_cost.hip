// Cost of a cross-stream fork on the critical (main) stream, native HIP (tools/micro/fork_cost).
// A chain of N short dependent kernels on the main stream (each ~5 us of one-workgroup-per-CU work);
// after every kernel a fork hands a small kernel to a side stream:
//   mode 0: no fork (the chain alone)
//   mode 1: hipEventRecord(main) + hipStreamWaitEvent(side)              (what lrs_dipnet does)
//   mode 2: hipStreamWriteValue32(main) + hipStreamWaitValue32(side)      (stream memory operations)
//   mode 3: the main-stream kernel itself writes the flag (last workgroup, agent-scope release) and
//           the side stream waits with hipStreamWaitValue32: no packet on the main stream at all
//   mode 4: mode 1 with the event created hipEventDisableSystemFence (device-scope fences only: the
//           consumer is a kernel on the same device)
//   mode 5: mode 1 with the event created hipEventReleaseToDevice
// Prints the main-stream time per link; mode k minus mode 0 is the fork's cost to the critical path.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/fork_cost tools/micro/fork_cost.hip
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

// y = a x + b over n floats, a few dependent FMAs per element (a ~5 us kernel at n = 4M)
__global__ void k_work(const float *x, float *y, int n, unsigned *flag, unsigned *count, unsigned ticket) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        float v = x[i];
#pragma unroll
        for (int r = 0; r < 8; ++r) v = v * 1.0001f + 0.5f;
        y[i] = v;
    }
    if (flag) {   // mode 3: the last workgroup publishes the ticket
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();   // this workgroup's stores before its arrival
            const unsigned c = atomicAdd(count, 1u);
            if (c == gridDim.x - 1) {
                __threadfence();
                __hip_atomic_store(flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                *count = 0;
            }
        }
    }
}

__global__ void k_side(float *s, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) s[i] = s[i] * 0.5f + 1.0f;
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 200, n = 1 << 22;
    float *a, *b, *s;
    unsigned *flag, *count;
    CK(hipMalloc(&a, n * sizeof(float)));
    CK(hipMalloc(&b, n * sizeof(float)));
    CK(hipMalloc(&s, 65536 * sizeof(float)));
    CK(hipMalloc(&count, 4));
    CK(hipMemset(count, 0, 4));
    CK(hipMemset(a, 0, n * sizeof(float)));
    CK(hipExtMallocWithFlags((void **)&flag, 8, hipMallocSignalMemory));   // signal memory: 8 bytes
    CK(hipMemset(flag, 0, 8));
    hipStream_t main_s, side;
    CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    hipEvent_t ev, ev_dev, ev_rel, t0, t1;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_dev, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&ev_rel, hipEventDisableTiming | hipEventReleaseToDevice));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    unsigned ticket = 0;
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 6; ++mode) {
            if (mode == 3 && argc < 3) continue;   // (345 us per link: measured round 5; argv[2] runs it)
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, main_s));
            for (int i = 0; i < N; ++i) {
                const float *x = (i & 1) ? b : a;
                float *y = (i & 1) ? a : b;
                ++ticket;
                hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, main_s, x, y, n, mode == 3 ? flag : nullptr,
                                   count, ticket);
                if (mode == 1 || mode == 4 || mode == 5) {
                    hipEvent_t e = mode == 1 ? ev : mode == 4 ? ev_dev : ev_rel;
                    CK(hipEventRecord(e, main_s));
                    CK(hipStreamWaitEvent(side, e, 0));
                } else if (mode == 2) {
                    CK(hipStreamWriteValue32(main_s, flag, ticket, 0));
                    CK(hipStreamWaitValue32(side, flag, ticket, hipStreamWaitValueGte, 0xffffffffu));
                } else if (mode == 3) {
                    CK(hipStreamWaitValue32(side, flag, ticket, hipStreamWaitValueGte, 0xffffffffu));
                }
                if (mode > 0) hipLaunchKernelGGL(k_side, dim3(256), dim3(256), 0, side, s, 65536);
            }
            CK(hipEventRecord(t1, main_s));
            CK(hipStreamSynchronize(main_s));
            CK(hipStreamSynchronize(side));
            float ms;
            CK(hipEventElapsedTime(&ms, t0, t1));
            const char *name[] = {"no fork", "event record + stream wait", "write value + wait value",
                                  "kernel flag + wait value", "event, no system fence", "event, release to device"};
            printf("rep %d mode %d %-28s %8.2f us per link\n", rep, mode, name[mode], 1e3f * ms / N);
        }
    return 0;
}
