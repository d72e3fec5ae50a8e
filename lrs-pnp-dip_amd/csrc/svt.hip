// SVT low-rank prox: U = SVT(Z, tau), Z = X + c2*L2 (main_LRS_PnP.py:112-124, called at :315 as
// SVT(X + (1/mu_2)*lambda_2, 1/mu_2)).
//
// The reference runs a float32 LAPACK SVD of the P x B matrix.  Here, MI355X-first:
//   1. fp64 Gram Z^T Z over row slabs (many workgroups, coalesced rows) + a fixed-order reduce;
//   2. one workgroup runs a cyclic parallel (round-robin) two-sided Jacobi eigensolver on the
//      B x B Gram in fp64, WARM-STARTED from the previous outer iteration's eigenvectors
//      (A0 = V^T G V is nearly diagonal, so 1-3 sweeps instead of ~8);
//   3. E = V diag(min(tau/s, 1)) V^T and U = Z - Z E (f32 accumulate; E is small, so its
//      float32 rounding costs << 1e-6 relative).  Z V diag((s-tau)_+/s) V^T == U_s (S-tau)_+ V_h.
// The Gram/eig stage runs on its own stream beside the sparse-coding kernel.
#include <math.h>

#include "lrs_common.h"

namespace lrs {

constexpr int kGramTile = 32;
constexpr int kGramRows = 1024;   // rows per slab
constexpr int kGramChunk = 64;    // rows staged per LDS chunk
constexpr int kJacobiThreads = 1024;

struct SvtWs {
    double *partial;  // [nslab][ntile_pairs][32*32]
    double *G;        // [Bp][Bp]
    double *A;        // [Bp][Bp]
    double *V;        // [Bp][Bp]
    double *T;        // [Bp][Bp] scratch
    float *E;         // [B][B]
    int *state;       // [0] = V valid (warm start available), [1] = sweeps used last call
    int64_t nslab, ntp, Bp;
};

static inline int64_t gram_ntiles(int64_t B) { return (B + kGramTile - 1) / kGramTile; }

static SvtWs svt_ws_layout(void *base, int64_t P, int64_t B) {
    SvtWs w;
    const int64_t nt = gram_ntiles(B);
    w.nslab = (P + kGramRows - 1) / kGramRows;
    w.ntp = nt * (nt + 1) / 2;
    w.Bp = B + (B & 1);
    char *p = (char *)base;
    auto take = [&](size_t bytes) {
        char *r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    w.state = (int *)take(256);
    w.partial = (double *)take((size_t)w.nslab * w.ntp * kGramTile * kGramTile * sizeof(double));
    w.G = (double *)take((size_t)w.Bp * w.Bp * sizeof(double));
    w.A = (double *)take((size_t)w.Bp * w.Bp * sizeof(double));
    w.V = (double *)take((size_t)w.Bp * w.Bp * sizeof(double));
    w.T = (double *)take((size_t)w.Bp * w.Bp * sizeof(double));
    w.E = (float *)take((size_t)B * B * sizeof(float));
    return w;
}

static size_t svt_ws_bytes(int64_t P, int64_t B) {
    SvtWs w = svt_ws_layout(nullptr, P, B);
    return (size_t)((char *)(w.E + B * B) - (char *)nullptr) + 256;
}

// ---- 1. partial Gram over a slab of rows, one 32x32 upper-triangular tile pair per workgroup --
__global__ __launch_bounds__(256) void k_gram_partial(const float *__restrict__ X, const float *__restrict__ L2,
                                                      float c2, int64_t P, int B, int ntiles,
                                                      double *__restrict__ partial) {
    const int tp = blockIdx.x;   // tile pair index (ti <= tj)
    const int slab = blockIdx.y;
    int ti = 0, rem = tp;
    while (rem >= ntiles - ti) { rem -= ntiles - ti; ++ti; }
    const int tj = ti + rem;
    __shared__ float Zi[kGramChunk][kGramTile + 1];
    __shared__ float Zj[kGramChunk][kGramTile + 1];
    const int tid = threadIdx.x;
    const int oi = tid / 8;            // output row within tile  (0..31)
    const int oj0 = (tid % 8) * 4;     // 4 output cols
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t r_begin = (int64_t)slab * kGramRows;
    const int64_t r_end = min<int64_t>(r_begin + kGramRows, P);
    for (int64_t r0 = r_begin; r0 < r_end; r0 += kGramChunk) {
        __syncthreads();
        for (int idx = tid; idx < kGramChunk * kGramTile; idx += 256) {
            const int rr = idx / kGramTile, cc = idx % kGramTile;
            const int64_t r = r0 + rr;
            float zi = 0.f, zj = 0.f;
            if (r < r_end) {
                const int ci = ti * kGramTile + cc, cj = tj * kGramTile + cc;
                if (ci < B) {
                    zi = X[r * B + ci];
                    if (L2) zi = zi + c2 * L2[r * B + ci];   // X + (1/mu_2)*lambda_2
                }
                if (cj < B) {
                    zj = X[r * B + cj];
                    if (L2) zj = zj + c2 * L2[r * B + cj];
                }
            }
            Zi[rr][cc] = zi;
            Zj[rr][cc] = zj;
        }
        __syncthreads();
#pragma unroll 8
        for (int rr = 0; rr < kGramChunk; ++rr) {
            const double a = (double)Zi[rr][oi];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = __fma_rn(a, (double)Zj[rr][oj0 + k], acc[k]);
        }
    }
    double *out = partial + ((int64_t)slab * gridDim.x + tp) * (kGramTile * kGramTile);
#pragma unroll
    for (int k = 0; k < 4; ++k) out[oi * kGramTile + oj0 + k] = acc[k];
}

// ---- 1b. fixed-order reduction of the slab partials into the full symmetric Gram ------------
__global__ __launch_bounds__(256) void k_gram_reduce(const double *__restrict__ partial, int64_t nslab, int ntp,
                                                     int ntiles, int B, int Bp, double *__restrict__ G) {
    const int64_t total = (int64_t)ntp * kGramTile * kGramTile;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int tp = (int)(idx / (kGramTile * kGramTile));
        const int e = (int)(idx % (kGramTile * kGramTile));
        int ti = 0, rem = tp;
        while (rem >= ntiles - ti) { rem -= ntiles - ti; ++ti; }
        const int tj = ti + rem;
        const int i = ti * kGramTile + e / kGramTile, j = tj * kGramTile + e % kGramTile;
        double s = 0.0;
        for (int64_t sl = 0; sl < nslab; ++sl) s += partial[(sl * ntp + tp) * (kGramTile * kGramTile) + e];
        if (i < B && j < B) {
            G[(int64_t)i * Bp + j] = s;
            G[(int64_t)j * Bp + i] = s;
        }
    }
}

// ---- 2. one-workgroup cyclic parallel Jacobi + E = V diag(min(tau/s,1)) V^T ------------------
__device__ __forceinline__ double block_sum(double v, double *red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    return s;
}

__global__ __launch_bounds__(kJacobiThreads) void k_jacobi_svt(SvtWs w, int B, double tau, int warm, int max_sweeps,
                                                               double *__restrict__ s_out) {
    const int Bp = (int)w.Bp;  // even
    const int half = Bp / 2;
    const int tid = threadIdx.x;
    __shared__ double red[kJacobiThreads / 64];
    __shared__ double rc[512], rs[512];
    __shared__ int rp[512], rq[512];
    __shared__ double lam[512];
    __shared__ int order[512];
    const int64_t BB = (int64_t)Bp * Bp;
    const bool use_warm = warm && w.state[0] == 1;
    // A0 = V^T G V (warm) or G (cold).  Padding row/col (B odd) is an isolated zero eigenpair.
    if (use_warm) {
        for (int64_t idx = tid; idx < BB; idx += kJacobiThreads) {    // T = G V
            const int i = (int)(idx / Bp), j = (int)(idx % Bp);
            double s = 0.0;
            for (int k = 0; k < Bp; ++k) s = __fma_rn(w.G[(int64_t)i * Bp + k], w.V[(int64_t)k * Bp + j], s);
            w.T[idx] = s;
        }
        __syncthreads();
        for (int64_t idx = tid; idx < BB; idx += kJacobiThreads) {    // A = V^T T
            const int i = (int)(idx / Bp), j = (int)(idx % Bp);
            double s = 0.0;
            for (int k = 0; k < Bp; ++k) s = __fma_rn(w.V[(int64_t)k * Bp + i], w.T[(int64_t)k * Bp + j], s);
            w.A[idx] = s;
        }
    } else {
        for (int64_t idx = tid; idx < BB; idx += kJacobiThreads) {
            const int i = (int)(idx / Bp), j = (int)(idx % Bp);
            w.A[idx] = (i < B && j < B) ? w.G[idx] : 0.0;
            w.V[idx] = (i == j) ? 1.0 : 0.0;
        }
    }
    __syncthreads();
    double diag2 = 0.0;
    for (int i = tid; i < Bp; i += kJacobiThreads) diag2 += w.A[(int64_t)i * Bp + i] * w.A[(int64_t)i * Bp + i];
    double off2 = 0.0;
    for (int64_t idx = tid; idx < BB; idx += kJacobiThreads) {
        const int i = (int)(idx / Bp), j = (int)(idx % Bp);
        if (i != j) off2 += w.A[idx] * w.A[idx];
    }
    double dn = block_sum(diag2, red);
    double of = block_sum(off2, red);
    int sweeps = 0;
    const double tol2 = 1e-30;  // (1e-15)^2 relative
    while (sweeps < max_sweeps && of > tol2 * (dn + of)) {
        for (int r = 0; r < Bp - 1; ++r) {
            // round-robin pairing (circle method) over indices 0..Bp-1
            for (int k = tid; k < half; k += kJacobiThreads) {
                int p, q;
                if (k == 0) { p = Bp - 1; q = r; }
                else { p = (r + k) % (Bp - 1); q = (r - k + (Bp - 1)) % (Bp - 1); }
                if (p > q) { int t = p; p = q; q = t; }
                const double app = w.A[(int64_t)p * Bp + p], aqq = w.A[(int64_t)q * Bp + q];
                const double apq = w.A[(int64_t)p * Bp + q];
                double c = 1.0, s = 0.0;
                if (apq != 0.0 && fabs(apq) > 1e-300) {
                    const double theta = (aqq - app) / (2.0 * apq);
                    const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    c = 1.0 / sqrt(t * t + 1.0);
                    s = t * c;
                }
                rp[k] = p; rq[k] = q; rc[k] = c; rs[k] = s;
            }
            __syncthreads();
            // A <- J^T A J on every 2x2 block (k1,k2); J = [[c, s], [-s, c]] on (p, q)
            for (int idx = tid; idx < half * half; idx += kJacobiThreads) {
                const int k1 = idx / half, k2 = idx % half;
                const int p1 = rp[k1], q1 = rq[k1], p2 = rp[k2], q2 = rq[k2];
                const double c1 = rc[k1], s1 = rs[k1], c2 = rc[k2], s2 = rs[k2];
                double *App = &w.A[(int64_t)p1 * Bp + p2], *Apq = &w.A[(int64_t)p1 * Bp + q2];
                double *Aqp = &w.A[(int64_t)q1 * Bp + p2], *Aqq = &w.A[(int64_t)q1 * Bp + q2];
                const double a = *App, b = *Apq, cc = *Aqp, d = *Aqq;
                // left: rows (p1,q1) by J1^T ; right: cols (p2,q2) by J2
                const double la = c1 * a - s1 * cc, lb = c1 * b - s1 * d;
                const double lc = s1 * a + c1 * cc, ld = s1 * b + c1 * d;
                double na = c2 * la - s2 * lb, nb = s2 * la + c2 * lb;
                double nc = c2 * lc - s2 * ld, nd = s2 * lc + c2 * ld;
                if (k1 == k2) { nb = 0.0; nc = 0.0; }
                *App = na; *Apq = nb; *Aqp = nc; *Aqq = nd;
            }
            for (int idx = tid; idx < Bp * half; idx += kJacobiThreads) {   // V <- V J
                const int i = idx / half, k = idx % half;
                double *vp = &w.V[(int64_t)i * Bp + rp[k]], *vq = &w.V[(int64_t)i * Bp + rq[k]];
                const double a = *vp, b = *vq;
                *vp = rc[k] * a - rs[k] * b;
                *vq = rs[k] * a + rc[k] * b;
            }
            __syncthreads();
        }
        ++sweeps;
        diag2 = 0.0; off2 = 0.0;
        for (int i = tid; i < Bp; i += kJacobiThreads) diag2 += w.A[(int64_t)i * Bp + i] * w.A[(int64_t)i * Bp + i];
        for (int64_t idx = tid; idx < BB; idx += kJacobiThreads) {
            const int i = (int)(idx / Bp), j = (int)(idx % Bp);
            if (i != j) off2 += w.A[idx] * w.A[idx];
        }
        dn = block_sum(diag2, red);
        of = block_sum(off2, red);
    }
    // eigenvalues -> singular values -> shrink factors e_k = min(tau/s_k, 1) (1 - phi)
    for (int i = tid; i < Bp; i += kJacobiThreads) {
        const double l = w.A[(int64_t)i * Bp + i];
        lam[i] = l > 0.0 ? sqrt(l) : 0.0;
    }
    __syncthreads();
    if (s_out && tid == 0) {
        // selection order by descending s (B <= 512, serial is fine, once per call)
        for (int i = 0; i < Bp; ++i) order[i] = i;
        for (int i = 0; i < Bp; ++i)
            for (int k = i + 1; k < Bp; ++k)
                if (lam[order[k]] > lam[order[i]]) { int t = order[i]; order[i] = order[k]; order[k] = t; }
        for (int i = 0; i < B; ++i) s_out[i] = lam[order[i]];
    }
    __syncthreads();
    for (int i = tid; i < Bp; i += kJacobiThreads) {
        const double s = lam[i];
        lam[i] = (s > tau) ? tau / s : 1.0;
    }
    __syncthreads();
    for (int64_t idx = tid; idx < (int64_t)B * B; idx += kJacobiThreads) {
        const int i = (int)(idx / B), j = (int)(idx % B);
        double s = 0.0;
        for (int k = 0; k < Bp; ++k) s = __fma_rn(w.V[(int64_t)i * Bp + k] * lam[k], w.V[(int64_t)j * Bp + k], s);
        w.E[idx] = (float)s;
    }
    if (tid == 0) { w.state[0] = 1; w.state[1] = sweeps; }
}

// ---- 3. U = Z - Z E  (64 x 64 output tile per workgroup, f32) ------------------------------
constexpr int kAT = 64;   // output tile
constexpr int kAK = 16;   // k chunk

__global__ __launch_bounds__(256) void k_svt_apply(const float *__restrict__ X, const float *__restrict__ L2, float c2,
                                                   const float *__restrict__ E, int64_t P, int B,
                                                   float *__restrict__ U) {
    __shared__ float Zs[kAK][kAT + 1];   // [k][row]
    __shared__ float Es[kAK][kAT + 1];   // [k][col]
    const int64_t r0 = (int64_t)blockIdx.x * kAT;
    const int c0 = blockIdx.y * kAT;
    const int tid = threadIdx.x;
    const int tr = tid / 16, tc = tid % 16;  // 4x4 outputs per thread
    float acc[4][4] = {};
    for (int k0 = 0; k0 < B; k0 += kAK) {
        __syncthreads();
        for (int idx = tid; idx < kAK * kAT; idx += 256) {
            const int rr = idx / kAK, kk = idx % kAK;      // Z: row-major, k fastest -> coalesced-ish
            const int64_t r = r0 + rr;
            const int k = k0 + kk;
            float z = 0.f;
            if (r < P && k < B) {
                z = X[r * B + k];
                if (L2) z = z + c2 * L2[r * B + k];
            }
            Zs[kk][rr] = z;
            const int kk2 = idx / kAT, cc = idx % kAT;
            const int k2 = k0 + kk2, c = c0 + cc;
            Es[kk2][cc] = (k2 < B && c < B) ? E[(int64_t)k2 * B + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kAK; ++kk) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = Zs[kk][tr * 4 + i];
#pragma unroll
            for (int i = 0; i < 4; ++i) b[i] = Es[kk][tc * 4 + i];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) acc[i][jj] = __fmaf_rn(a[i], b[jj], acc[i][jj]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t r = r0 + tr * 4 + i;
        if (r >= P) continue;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int c = c0 + tc * 4 + jj;
            if (c >= B) continue;
            float z = X[r * B + c];
            if (L2) z = z + c2 * L2[r * B + c];
            U[r * B + c] = z - acc[i][jj];
        }
    }
}

}  // namespace lrs

using namespace lrs;

extern "C" size_t lrs_svt_workspace(int64_t P, int64_t B) {
    if (P <= 0 || B <= 0) return 0;
    return svt_ws_bytes(P, B);
}

extern "C" int lrs_svt_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau, float *U,
                           double *s_out, int warm, void *ws, size_t ws_bytes, void *stream) {
    if (!X || !U || !ws || P <= 0 || B <= 0 || tau < 0.0) return LRS_E_INVALID;
    if (B > 510) return LRS_E_UNSUPPORTED;
    if (ws_bytes < svt_ws_bytes(P, B)) return LRS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    SvtWs w = svt_ws_layout(ws, P, B);
    if (!warm) {
        hipError_t e = hipMemsetAsync(w.state, 0, sizeof(int) * 2, st);
        if (e != hipSuccess) return (int)e;
    }
    const int nt = (int)gram_ntiles(B);
    hipLaunchKernelGGL(k_gram_partial, dim3((unsigned)w.ntp, (unsigned)w.nslab), dim3(256), 0, st, X, L2, c2, P,
                       (int)B, nt, w.partial);
    LRS_CHECK_LAUNCH();
    const int64_t tot = w.ntp * kGramTile * kGramTile;
    hipLaunchKernelGGL(k_gram_reduce, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 4096)), dim3(256), 0, st,
                       w.partial, w.nslab, (int)w.ntp, nt, (int)B, (int)w.Bp, w.G);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_jacobi_svt, dim3(1), dim3(kJacobiThreads), 0, st, w, (int)B, tau, warm, 30, s_out);
    LRS_CHECK_LAUNCH();
    dim3 grid((unsigned)((P + kAT - 1) / kAT), (unsigned)((B + kAT - 1) / kAT));
    hipLaunchKernelGGL(k_svt_apply, grid, dim3(256), 0, st, X, L2, c2, w.E, P, (int)B, U);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
