// Block grid, im2col, and the fused col2im + closed-form X + dual update of one ADMM iteration.
//
// Reference: get_image_block (main_LRS_PnP.py:73-107), the col2im / X / lambda block of
// main_LRS_PnP.py:324-362 (…1-LiP.py:420-448) and state_convergence (:23-25).
//
// col2im is a GATHER, not a scatter: every (p, b) element walks the blocks covering it in block
// order (the reference loop order), so IMout, Weight and lambda1_summation are bit-identical to
// the reference's sequential `+=`, deterministic, atomic-free, and the whole update is one
// coalesced pass over the P x B arrays (HBM-bound: DESIGN.md §ADMM).
#include <math.h>

#include <vector>

#include "lrs_common.h"

namespace lrs {

// ---------------------------------------------------------------------------------------------
// Host: block grid (get_image_block corner indicator, F-order enumeration)
// ---------------------------------------------------------------------------------------------
static void axis_starts(int64_t extent, int64_t bb, int64_t sliding, std::vector<int32_t> &out) {
    out.clear();
    const int64_t n = extent - bb + 1;  // idx_Mat size along this axis
    if (n <= 0) return;
    std::vector<char> ind((size_t)n, 0);
    for (int64_t i = 0; i < n; i += sliding) ind[(size_t)i] = 1;  // idx_Mat[0:n+1:s] = 1
    if (extent % bb != 0) ind[(size_t)(n - 1)] = 1;                // appended last row/column
    for (int64_t i = 0; i < n; ++i)
        if (ind[(size_t)i]) out.push_back((int32_t)i);
}

}  // namespace lrs

using namespace lrs;

// The corner indicator of get_image_block is a product of row and column indicators except for
// the appended-column/appended-row rule, which marks the appended entries only at the regular
// positions of the other axis plus the corner — i.e. again the product of the two start sets.
extern "C" int64_t lrs_block_count(int64_t P, int64_t B, int64_t bb, int64_t sliding) {
    if (P <= 0 || B <= 0 || bb <= 0 || sliding <= 0 || bb > P || bb > B) return LRS_E_INVALID;
    std::vector<int32_t> r, c;
    axis_starts(P, bb, sliding, r);
    axis_starts(B, bb, sliding, c);
    return (int64_t)r.size() * (int64_t)c.size();
}

extern "C" int lrs_block_grid(int64_t P, int64_t B, int64_t bb, int64_t sliding, int32_t *rows,
                              int32_t *cols, int64_t nb) {
    if (!rows || !cols) return LRS_E_INVALID;
    const int64_t want = lrs_block_count(P, B, bb, sliding);
    if (want < 0) return (int)want;
    if (nb != want) return LRS_E_INVALID;
    std::vector<int32_t> r, c;
    axis_starts(P, bb, sliding, r);
    axis_starts(B, bb, sliding, c);
    int64_t j = 0;
    for (size_t ic = 0; ic < c.size(); ++ic)      // F-order over the corner matrix: column outer
        for (size_t ir = 0; ir < r.size(); ++ir) {
            rows[j] = r[ir];
            cols[j] = c[ic];
            ++j;
        }
    return LRS_OK;
}

extern "C" int lrs_cover_ranges(int64_t extent, int64_t bb, const int32_t *starts, int64_t nstarts,
                                int32_t *lo, int32_t *hi) {
    if (!starts || !lo || !hi || extent <= 0 || bb <= 0 || nstarts < 0) return LRS_E_INVALID;
    for (int64_t i = 1; i < nstarts; ++i)
        if (starts[i] <= starts[i - 1]) return LRS_E_INVALID;
    // covering starts of x: x - bb < start <= x  (contiguous in the sorted list)
    int64_t a = 0, b = -1;
    for (int64_t x = 0; x < extent; ++x) {
        while (a < nstarts && starts[a] + bb <= x) ++a;
        while (b + 1 < nstarts && starts[b + 1] <= x) ++b;
        lo[x] = (int32_t)a;
        hi[x] = (int32_t)b;
    }
    return LRS_OK;
}

// ---------------------------------------------------------------------------------------------
// Device: im2col of X + L/mu into [nb][n_pad] block vectors (+ observation mask)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_im2col(const float *__restrict__ X, const float *__restrict__ L,
                                                float mu, int64_t B, int bb, const int32_t *__restrict__ rows,
                                                const int32_t *__restrict__ cols, int64_t nb, int n_pad,
                                                float *__restrict__ Yb, uint8_t *__restrict__ obs) {
    const int64_t total = nb * (int64_t)n_pad;
    const int n = bb * bb;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx / n_pad;
        const int r = (int)(idx - j * n_pad);
        float v = 0.0f;
        if (r < n) {
            const int a = r % bb, c = r / bb;  // F-order flatten of the bb x bb block
            const int64_t e = (int64_t)(rows[j] + a) * B + (cols[j] + c);
            v = X[e];
            if (L) v = v + L[e] / mu;           // X + lambda_1/mu_1 (main_LRS_PnP.py:259)
        }
        Yb[idx] = v;
        if (obs) obs[idx] = (r < n && v != 0.0f) ? 1 : 0;  // missing = observed value == 0 (:278)
    }
}

extern "C" int lrs_im2col_f32(const float *X, const float *L, float mu, int64_t P, int64_t B, int64_t bb,
                              const int32_t *rows, const int32_t *cols, int64_t nb, int64_t n_pad, float *Yb,
                              uint8_t *obs, void *stream) {
    if (!X || !rows || !cols || !Yb || P <= 0 || B <= 0 || bb <= 0 || n_pad < bb * bb || nb < 0)
        return LRS_E_INVALID;
    if (nb == 0) return LRS_OK;
    const int64_t total = nb * n_pad;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_im2col, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, X, L, mu, B,
                       (int)bb, rows, cols, nb, (int)n_pad, Yb, obs);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// ---------------------------------------------------------------------------------------------
// Device: fused col2im + X update + dual updates + convergence norms
// ---------------------------------------------------------------------------------------------
struct AdmmParams {
    float *X, *L1, *L2;
    const float *Y, *M, *U, *phi;
    const int32_t *row_starts, *col_starts, *rlo, *rhi, *clo, *chi;
    double *norms;
    float *imout;
    int64_t P, B, nbr;
    int bb, n_pad;
    float gamma, mu1, mu2;
};

constexpr int kAdmmThreads = 256;

__global__ __launch_bounds__(kAdmmThreads) void k_admm_update(AdmmParams a) {
    const int64_t N = a.P * a.B;
    double sx = 0.0, s1 = 0.0, s2 = 0.0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = e / a.B;
        const int b = (int)(e - p * a.B);
        const float l1 = a.L1[e];
        float im = 0.0f, w = 0.0f, ls = 0.0f;
        const int c0 = a.clo[b], c1 = a.chi[b];
        const int r0 = a.rlo[p], r1 = a.rhi[p];
        for (int ic = c0; ic <= c1; ++ic) {            // block order: column-major over corners
            const int cc = b - a.col_starts[ic];
            for (int ir = r0; ir <= r1; ++ir) {
                const int rr = (int)(p - a.row_starts[ir]);
                const int64_t j = (int64_t)ic * a.nbr + ir;
                im = im + a.phi[j * a.n_pad + rr + a.bb * cc];
                w = w + 1.0f;
                ls = ls + l1;
            }
        }
        const float x_old = a.X[e];
        const float u = a.U[e];
        const float l2 = a.L2[e];
        // (gamma*MtY + mu1*IMout + mu2*U - lambda1_sum - lambda_2) / (gamma*MtM + mu1*W + mu2)
        float num = a.gamma * a.Y[e];
        num = num + a.mu1 * im;
        num = num + a.mu2 * u;
        num = num - ls;
        num = num - l2;
        float den = a.gamma * a.M[e];
        den = den + a.mu1 * w;
        den = den + a.mu2;
        const float x = num / den;
        const float l1n = l1 + a.mu1 * (x - im);
        const float l2n = l2 + a.mu2 * (x - u);
        a.X[e] = x;
        a.L1[e] = l1n;
        a.L2[e] = l2n;
        if (a.imout) a.imout[e] = im;
        const double dx = (double)x - (double)x_old, d1 = (double)l1n - (double)l1,
                     d2 = (double)l2n - (double)l2;
        sx += dx * dx;
        s1 += d1 * d1;
        s2 += d2 * d2;
    }
    if (!a.norms) return;
    // wave reduce then one atomic per wave (3 doubles)
    for (int off = 32; off > 0; off >>= 1) {
        sx += __shfl_down(sx, off, 64);
        s1 += __shfl_down(s1, off, 64);
        s2 += __shfl_down(s2, off, 64);
    }
    __shared__ double red[3][kAdmmThreads / 64];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wv] = sx; red[1][wv] = s1; red[2][wv] = s2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
        for (int i = 0; i < kAdmmThreads / 64; ++i) s += red[threadIdx.x][i];
        atomicAdd(&a.norms[threadIdx.x], s);
    }
}

extern "C" int lrs_admm_update_f32(float *X, float *L1, float *L2, const float *Y, const float *M,
                                   const float *U, const float *phi, int64_t P, int64_t B, int64_t bb,
                                   int64_t n_pad, const int32_t *row_starts, const int32_t *col_starts,
                                   int64_t nbr, const int32_t *rlo, const int32_t *rhi, const int32_t *clo,
                                   const int32_t *chi, float gamma, float mu1, float mu2, double *norms,
                                   float *imout, void *stream) {
    if (!X || !L1 || !L2 || !Y || !M || !U || !phi || !row_starts || !col_starts || !rlo || !rhi || !clo ||
        !chi || P <= 0 || B <= 0 || bb <= 0 || n_pad < bb * bb || nbr <= 0)
        return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (norms) {
        hipError_t e = hipMemsetAsync(norms, 0, 3 * sizeof(double), st);
        if (e != hipSuccess) return (int)e;
    }
    AdmmParams a{X, L1, L2, Y, M, U, phi, row_starts, col_starts, rlo, rhi, clo, chi, norms, imout,
                 P, B, nbr, (int)bb, (int)n_pad, gamma, mu1, mu2};
    const int64_t N = P * B;
    const int64_t blocks = std::min<int64_t>((N + kAdmmThreads - 1) / kAdmmThreads, 2048);
    hipLaunchKernelGGL(k_admm_update, dim3((unsigned)blocks), dim3(kAdmmThreads), 0, st, a);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
