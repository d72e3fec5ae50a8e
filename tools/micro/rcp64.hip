// Accuracy of v_rcp_f64 (and one Newton step) against IEEE 1/x over [0.5, 16): prints the max
// relative error in units of 2^-53 for both.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

__global__ void k(const double *x, double *r0, double *r1, double *ref, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    double r = __builtin_amdgcn_rcp(d);
    r0[i] = r;
    const double e = __fma_rn(-d, r, 1.0);
    r1[i] = __fma_rn(r, e, r);
    ref[i] = 1.0 / d;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> hx(n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        hx[i] = 0.5 + 15.5 * ((s >> 11) * (1.0 / 9007199254740992.0));
    }
    double *x, *r0, *r1, *ref;
    hipMalloc(&x, n * 8); hipMalloc(&r0, n * 8); hipMalloc(&r1, n * 8); hipMalloc(&ref, n * 8);
    hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(x, r0, r1, ref, n);
    std::vector<double> h0(n), h1(n), hr(n);
    hipMemcpy(h0.data(), r0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h1.data(), r1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hr.data(), ref, n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0;
    long ex0 = 0, ex1 = 0;
    for (int i = 0; i < n; ++i) {
        m0 = fmax(m0, fabs(h0[i] - hr[i]) / hr[i]);
        m1 = fmax(m1, fabs(h1[i] - hr[i]) / hr[i]);
        ex0 += h0[i] == hr[i]; ex1 += h1[i] == hr[i];
    }
    printf("rcp_f64: max rel err %.3g (= %.2f x 2^-53), exact %.4f\n", m0, m0 * 9007199254740992.0, ex0 / (double)n);
    printf("rcp_f64 + 1 Newton: max rel err %.3g (= %.2f x 2^-53), exact %.4f\n", m1, m1 * 9007199254740992.0, ex1 / (double)n);
    return 0;
}
