// Quality metrics of the reference (not on the timed path): MSSIM of pytorch_ssim.ssim
// (pytorch_ssim/__init__.py:7-37, 65-73), as main_LRS_PnP_DIP_1-LiP.py:480-481 calls it:
// per channel, an 11x11 Gaussian window (sigma 1.5, float32, normalised in float32) applied as a
// zero-padded (padding 5) convolution to x, y, x*x, y*y, x*y; C1 = 0.01^2, C2 = 0.03^2;
//   ssim = ((2 mu1 mu2 + C1)(2 s12 + C2)) / ((mu1^2 + mu2^2 + C1)(s1 + s2 + C2)),  mean over all.
// One thread per output pixel, float32 map (as the reference), fp64 mean.
#include <math.h>

#include "lrs_common.h"

namespace lrs {

struct SsimWin {
    float w[121];
};

__global__ __launch_bounds__(256) void k_ssim(const float *__restrict__ a, const float *__restrict__ b, int C, int H,
                                              int W, SsimWin win, double *acc) {
    __shared__ double red[4];
    const int64_t n = (int64_t)C * H * W;
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % W), y = (int)((i / W) % H);
        const int64_t base = i - (int64_t)y * W - x;
        float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
        for (int dy = 0; dy < 11; ++dy) {
            const int yy = y + dy - 5;
            if (yy < 0 || yy >= H) continue;
            for (int dx = 0; dx < 11; ++dx) {
                const int xx = x + dx - 5;
                if (xx < 0 || xx >= W) continue;
                const float wt = win.w[dy * 11 + dx];
                const float u = a[base + (int64_t)yy * W + xx], v = b[base + (int64_t)yy * W + xx];
                m1 = __fmaf_rn(wt, u, m1);
                m2 = __fmaf_rn(wt, v, m2);
                e11 = __fmaf_rn(wt, u * u, e11);
                e22 = __fmaf_rn(wt, v * v, e22);
                e12 = __fmaf_rn(wt, u * v, e12);
            }
        }
        const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
        const float m1s = m1 * m1, m2s = m2 * m2, m12 = m1 * m2;
        const float s1 = e11 - m1s, s2 = e22 - m2s, s12 = e12 - m12;
        const float v = ((2.f * m12 + C1) * (2.f * s12 + C2)) / ((m1s + m2s + C1) * (s1 + s2 + C2));
        s += (double)v;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(acc, red[0] + red[1] + red[2] + red[3]);
}

}  // namespace lrs

namespace lrs {

// ---- per-band PSNR on the unfolded matrices (main_LRS_PnP.py:379-384; psnr() :40-46) --------
// Stage 1: workgroup s sums (X - C)^2 over its slab of rows for every band (threads over bands,
// coalesced rows, fp64); stage 2: one thread per band reduces the slabs in fixed order and
// applies the reference's 10 log10(255 / sqrt(mse)) (100 when mse < 1e-10, as psnr() does).
constexpr int kPsnrSlabs = 256;

__global__ __launch_bounds__(256) void k_psnr_partial(const float *__restrict__ X, const float *__restrict__ C,
                                                      int64_t P, int B, int64_t rows, double *__restrict__ part) {
    const int64_t r0 = (int64_t)blockIdx.x * rows, r1 = min<int64_t>(P, r0 + rows);
    for (int b = threadIdx.x; b < B; b += 256) {
        double s = 0.0;
        for (int64_t r = r0; r < r1; ++r) {
            const double d = (double)X[r * B + b] - (double)C[r * B + b];
            s = __fma_rn(d, d, s);
        }
        part[(int64_t)blockIdx.x * B + b] = s;
    }
}

__global__ __launch_bounds__(256) void k_psnr_finish(const double *__restrict__ part, int nslab, int64_t P, int B,
                                                     double *__restrict__ psnr) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    double s = 0.0;
    for (int k = 0; k < nslab; ++k) s += part[(int64_t)k * B + b];
    const double mse = s / (double)P;
    psnr[b] = mse < 1.0e-10 ? 100.0 : 10.0 * log10(255.0 / sqrt(mse));
}

}  // namespace lrs

using namespace lrs;

extern "C" size_t lrs_psnr_workspace(int64_t P, int64_t B) {
    if (P <= 0 || B <= 0) return 0;
    return (size_t)kPsnrSlabs * (size_t)B * sizeof(double);
}

// psnr (device, B doubles) <- per-band PSNR of X against C, both P x B float32 (unfolded).
extern "C" int lrs_psnr_bands_f32(const float *X, const float *C, int64_t P, int64_t B, double *psnr, void *ws,
                                  size_t ws_bytes, void *stream) {
    if (!X || !C || !psnr || !ws || P <= 0 || B <= 0) return LRS_E_INVALID;
    if (ws_bytes < lrs_psnr_workspace(P, B)) return LRS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const int64_t rows = (P + kPsnrSlabs - 1) / kPsnrSlabs;
    const int nslab = (int)((P + rows - 1) / rows);
    hipLaunchKernelGGL(k_psnr_partial, dim3((unsigned)nslab), dim3(256), 0, st, X, C, P, (int)B, rows, (double *)ws);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_psnr_finish, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, (const double *)ws, nslab, P,
                       (int)B, psnr);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// acc (device double, zeroed by the call) receives sum of the SSIM map; mssim = acc / (C*H*W).
extern "C" int lrs_ssim_f32(const float *img1, const float *img2, int C, int H, int W, double *acc, void *stream) {
    if (!img1 || !img2 || !acc || C <= 0 || H <= 0 || W <= 0) return LRS_E_INVALID;
    SsimWin win;
    float g[11], gs = 0.0f;
    for (int x = 0; x < 11; ++x) g[x] = (float)exp(-(double)((x - 5) * (x - 5)) / (2.0 * 1.5 * 1.5));
    for (int x = 0; x < 11; ++x) gs += g[x];
    for (int x = 0; x < 11; ++x) g[x] = g[x] / gs;
    for (int i = 0; i < 11; ++i)
        for (int j = 0; j < 11; ++j) win.w[i * 11 + j] = g[i] * g[j];
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(acc, 0, sizeof(double), st);
    if (e != hipSuccess) return (int)e;
    const int64_t n = (int64_t)C * H * W;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_ssim, dim3((unsigned)blocks), dim3(256), 0, st, img1, img2, C, H, W, win, acc);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
