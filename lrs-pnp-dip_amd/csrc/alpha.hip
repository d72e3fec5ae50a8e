// ISTA step size alpha and NLM strength h per observation pattern.
//
// Reference: inside ista(), recomputed per block per outer iteration although it depends only
// on the block's missing-row set (fixed by blocks_copy, main_LRS_PnP.py:244) and D:
//   main_LRS_PnP.py:134-146       alpha = np.linalg.norm(H,2)**2, T = 0.1/(2 alpha), h = 0.1 T
//   …1-LiP.py:187-196              alpha = 2(tr(H^T H) + tr(H^T H)), T = 0.1/(2 alpha), h = T
//   ista.m:15-23 (soft variant)    alpha = norm(H)^2, soft threshold T
// with H = D restricted to the observed rows.  Scalars follow numpy>=2 float32 semantics.
//
// ||H||_2^2 = lambda_max of the masked Gram, computed matrix-free in fp64 by Lanczos with full
// (twice-applied classical Gram-Schmidt) reorthogonalisation on the smaller of D_m D_m^T (n_obs)
// and D_m^T D_m (K); the Ritz value of the tridiagonal comes from Sturm bisection.  One
// workgroup per distinct observation pattern (the host deduplicates the patterns).
#include <math.h>

#include "lrs_common.h"

namespace lrs {

constexpr int kAlphaThreads = 256;
constexpr int kLanczosMax = 128;

__device__ __forceinline__ double wg_sum(double v, double *red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kAlphaThreads / 64; ++i) s += red[i];
    return s;
}

// t[a] = sum_k D[rows[a]][k] x[k]  (a < m_obs), one wave per row, lanes over k
__device__ void rows_dot(const float *__restrict__ D, int K, const short *rows, int m_obs, const double *x,
                         double *t) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int a = wv; a < m_obs; a += kAlphaThreads / 64) {
        const float *Dr = D + (int64_t)rows[a] * K;
        double s = 0.0;
        for (int k = lane; k < K; k += 64) s = __fma_rn((double)Dr[k], x[k], s);
        for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
        if (lane == 0) t[a] = s;
    }
}

// y[k] = sum_a D[rows[a]][k] t[a]  (k < K), thread per k
__device__ void cols_sum(const float *__restrict__ D, int K, const short *rows, int m_obs, const double *t,
                         double *y) {
    for (int k = threadIdx.x; k < K; k += kAlphaThreads) {
        double s = 0.0;
        for (int a = 0; a < m_obs; ++a) s = __fma_rn((double)D[(int64_t)rows[a] * K + k], t[a], s);
        y[k] = s;
    }
}

// number of eigenvalues of the symmetric tridiagonal (al, be) greater than x
__device__ int sturm_count_greater(const double *al, const double *be, int k, double x) {
    int neg = 0;
    double d = 1.0;
    for (int i = 0; i < k; ++i) {
        const double b2 = (i > 0) ? be[i - 1] * be[i - 1] : 0.0;
        d = (al[i] - x) - (i > 0 ? b2 / d : 0.0);
        if (d == 0.0) d = -1e-300;
        if (d < 0.0) ++neg;
    }
    return k - neg;  // eigenvalues > x
}

struct AlphaParams {
    const float *D;
    const uint8_t *obs_pat;
    float *alpha_pat;
    double *thr_pat;
    double *ws;  // per pattern: kLanczosMax * K doubles
    int n, K, n_pad, mode;
    float lambda_ista;
};

__global__ __launch_bounds__(kAlphaThreads) void k_alpha(AlphaParams p) {
    extern __shared__ double smem[];
    // layout: q[K] w[K] qprev[K] t[max(n,K)] coef[kLanczosMax] al[kLanczosMax] be[kLanczosMax] red[4]
    const int K = p.K, n = p.n;
    const int tlen = n > K ? n : K;
    double *q = smem, *w = q + K, *qprev = w + K, *t = qprev + K, *coef = t + tlen;
    double *al = coef + kLanczosMax, *be = al + kLanczosMax, *red = be + kLanczosMax;
    short *rows = (short *)(red + 8);
    __shared__ int m_obs_s;
    const int pat = blockIdx.x;
    const uint8_t *ob = p.obs_pat + (int64_t)pat * p.n_pad;
    if (threadIdx.x == 0) {
        int m = 0;
        for (int r = 0; r < n; ++r)
            if (ob[r]) rows[m++] = (short)r;
        m_obs_s = m;
    }
    __syncthreads();
    const int m_obs = m_obs_s;
    float alpha32;
    if (p.mode == LRS_ALPHA_FRO4) {
        // tr(H^T H) = sum over observed rows of ||d_r||^2
        double s = 0.0;
        for (int k = threadIdx.x; k < K; k += kAlphaThreads)
            for (int a = 0; a < m_obs; ++a) {
                const double v = (double)p.D[(int64_t)rows[a] * K + k];
                s = __fma_rn(v, v, s);
            }
        const float tr = (float)wg_sum(s, red);
        alpha32 = 2.0f * (tr + tr);
    } else {
        // Lanczos on A = D_m D_m^T (dim m_obs) if m_obs <= K else A = D_m^T D_m (dim K)
        const bool small = m_obs <= K;
        const int m = small ? m_obs : K;
        double *Q = p.ws + (int64_t)pat * kLanczosMax * K;
        const int kmax = m < kLanczosMax ? m : kLanczosMax;
        for (int i = threadIdx.x; i < m; i += kAlphaThreads) {
            q[i] = 1.0 + 0.5 * sin(0.7 * (double)i + 0.3);   // deterministic start vector
            qprev[i] = 0.0;
        }
        __syncthreads();
        double nrm;
        {
            double s = 0.0;
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) s += q[i] * q[i];
            nrm = sqrt(wg_sum(s, red));
        }
        for (int i = threadIdx.x; i < m; i += kAlphaThreads) q[i] /= nrm;
        __syncthreads();
        int k = 0;
        double beta_prev = 0.0;
        for (; k < kmax; ++k) {
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) Q[(int64_t)k * K + i] = q[i];
            // w = A q
            if (small) {
                cols_sum(p.D, K, rows, m_obs, q, t);   // t[K] = D_m^T q
                __syncthreads();
                rows_dot(p.D, K, rows, m_obs, t, w);   // w[m_obs] = D_m t
            } else {
                rows_dot(p.D, K, rows, m_obs, q, t);   // t[m_obs] = D_m q
                __syncthreads();
                cols_sum(p.D, K, rows, m_obs, t, w);   // w[K] = D_m^T t
            }
            __syncthreads();
            double s = 0.0;
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) s += q[i] * w[i];
            const double a_k = wg_sum(s, red);
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) w[i] = w[i] - a_k * q[i] - beta_prev * qprev[i];
            __syncthreads();
            // full reorthogonalisation, CGS applied twice
            for (int pass = 0; pass < 2; ++pass) {
                const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
                for (int i = wv; i <= k; i += kAlphaThreads / 64) {
                    double d = 0.0;
                    for (int x = lane; x < m; x += 64) d = __fma_rn(Q[(int64_t)i * K + x], w[x], d);
                    for (int off = 32; off > 0; off >>= 1) d += __shfl_down(d, off, 64);
                    if (lane == 0) coef[i] = d;
                }
                __syncthreads();
                for (int x = threadIdx.x; x < m; x += kAlphaThreads) {
                    double v = w[x];
                    for (int i = 0; i <= k; ++i) v -= coef[i] * Q[(int64_t)i * K + x];
                    w[x] = v;
                }
                __syncthreads();
            }
            s = 0.0;
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) s += w[i] * w[i];
            const double b_k = sqrt(wg_sum(s, red));
            if (threadIdx.x == 0) { al[k] = a_k; be[k] = b_k; }
            if (!(b_k > 1e-13 * fabs(a_k)) || k + 1 == kmax) { ++k; break; }
            for (int i = threadIdx.x; i < m; i += kAlphaThreads) {
                qprev[i] = q[i];
                q[i] = w[i] / b_k;
            }
            beta_prev = b_k;
            __syncthreads();
        }
        __syncthreads();
        __shared__ double lmax_s;
        if (threadIdx.x == 0) {
            double lmax = 0.0;
            if (m > 0) {
                double lo = 1e300, hi = -1e300;
                for (int i = 0; i < k; ++i) {
                    const double r = (i > 0 ? fabs(be[i - 1]) : 0.0) + (i + 1 < k ? fabs(be[i]) : 0.0);
                    lo = fmin(lo, al[i] - r);
                    hi = fmax(hi, al[i] + r);
                }
                for (int it = 0; it < 200 && hi - lo > 0.0; ++it) {
                    const double mid = 0.5 * (lo + hi);
                    if (mid <= lo || mid >= hi) break;
                    if (sturm_count_greater(al, be, k, mid) >= 1) lo = mid; else hi = mid;
                }
                lmax = 0.5 * (lo + hi);
            }
            lmax_s = lmax;
        }
        __syncthreads();
        // numpy: sigma = float32 SVD value, alpha = sigma**2 in float32
        const float sigma = (float)sqrt(fmax(lmax_s, 0.0));
        alpha32 = sigma * sigma;
    }
    if (threadIdx.x == 0) {
        const float a = alpha32;
        float T = p.lambda_ista / (2.0f * a);
        double thr;
        if (p.mode == LRS_ALPHA_SPEC2) thr = (double)(T * 0.1f);
        else thr = (double)T;
        if (!(a > 0.0f)) thr = 1.0;   // fully-missing block: the reference divides by zero
        p.alpha_pat[pat] = (a > 0.0f) ? a : 1.0f;
        p.thr_pat[pat] = thr;
    }
}

}  // namespace lrs

using namespace lrs;

extern "C" size_t lrs_ista_alpha_workspace(int64_t n, int64_t K, int64_t npat) {
    (void)n;
    if (K <= 0 || npat < 0) return 0;
    return (size_t)npat * kLanczosMax * K * sizeof(double) + 256;
}

extern "C" int lrs_ista_alpha_f32(const float *D, int64_t n, int64_t K, const uint8_t *obs_pat, int64_t npat,
                                  int64_t n_pad, int alpha_mode, float lambda_ista, float *alpha_pat,
                                  double *thr_pat, void *ws, size_t ws_bytes, void *stream) {
    if (!D || !obs_pat || !alpha_pat || !thr_pat || n <= 0 || K <= 0 || n_pad < n || npat < 0) return LRS_E_INVALID;
    if (alpha_mode != LRS_ALPHA_SPEC2 && alpha_mode != LRS_ALPHA_FRO4 && alpha_mode != LRS_ALPHA_SOFT)
        return LRS_E_INVALID;
    if (n > 32767 || K > 4096) return LRS_E_UNSUPPORTED;
    if (npat == 0) return LRS_OK;
    if (alpha_mode != LRS_ALPHA_FRO4 && (!ws || ws_bytes < lrs_ista_alpha_workspace(n, K, npat)))
        return LRS_E_WORKSPACE;
    const int64_t tlen = n > K ? n : K;
    const size_t smem = sizeof(double) * (3 * K + tlen + 3 * kLanczosMax + 8) + sizeof(short) * n + 16;
    if (smem > 160 * 1024) return LRS_E_UNSUPPORTED;
    AlphaParams p{D, obs_pat, alpha_pat, thr_pat, (double *)ws, (int)n, (int)K, (int)n_pad, alpha_mode, lambda_ista};
    hipLaunchKernelGGL(k_alpha, dim3((unsigned)npat), dim3(kAlphaThreads), smem, (hipStream_t)stream, p);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
