// SVT low-rank prox: U = SVT(Z, tau), Z = X + c2*L2 (main_LRS_PnP.py:112-124, called at :315 as
// SVT(X + (1/mu_2)*lambda_2, 1/mu_2)).
//
// The reference runs a float32 LAPACK SVD of the P x B matrix.  Here, MI355X-first:
//   1. fp64 Gram G = Z^T Z over row slabs (many workgroups, coalesced rows), fixed-order reduce;
//   2. warm start: A0 = V^T G V with the previous outer iteration's eigenvectors (tiled fp64
//      GEMMs) — nearly diagonal, so Jacobi needs 1-3 sweeps instead of ~8;
//   3. ONE workgroup runs a cyclic parallel (round-robin) two-sided Jacobi on A held in LDS as a
//      packed fp64 upper triangle (B <= 200: <= 160,800 B), logging each round's rotations;
//   4. the eigenvector update V <- V J_1 ... J_R is replayed from the log row by row in parallel
//      (rows of V evolve independently), off the Jacobi workgroup's critical path;
//   5. E = V diag(min(tau/s, 1)) V^T (fp64 -> f32) and U = Z - Z E.
//      Z V diag((s-tau)_+/s) V^T == U_s (S-tau)_+ V_h, and E is small so its f32 rounding costs
//      << 1e-6 relative in U.
// The whole chain runs on its own stream beside the sparse-coding kernel.
#include <math.h>

#include <algorithm>

#include "lrs_common.h"

namespace lrs {

constexpr int kGramTile = 32;
constexpr int kGramRows = 1024;   // rows per slab
constexpr int kGramChunk = 64;    // rows staged per LDS chunk
constexpr int kJacobiThreads = 1024;
constexpr int kMaxBp = 200;       // packed fp64 triangle of 200 x 200 = 160,800 B of LDS
constexpr int kMaxSweeps = 40;

struct SvtWs {
    double *partial;  // [nslab][ntile_pairs][32*32]
    double *G;        // [Bp][Bp]
    double *A0;       // [Bp][Bp]  V^T G V (warm start)
    double *T;        // [Bp][Bp]  scratch
    double *V[2];     // [Bp][Bp]  eigenvectors, double-buffered
    double *lam;      // [Bp]      eigenvalues (diag of the converged A)
    double *rot;      // [kMaxSweeps*(Bp-1)][Bp/2][2]  (c, s) per round and pair
    double *beta;     // [Bp]      Householder scalars (tridiagonal path)
    double *F;        // [Bp][4][Bp] pivoted LU rows of T - lambda_i I (inverse iteration)
    float *E;         // [B][B]
    int *state;       // [0] V valid, [1] current V buffer, [2] rounds, [3] sweeps,
                      // [4] path of the last solve (1 tridiagonal, 2 Jacobi fallback, 3 Jacobi)
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
    const size_t mat = (size_t)w.Bp * w.Bp * sizeof(double);
    w.state = (int *)take(256);
    w.partial = (double *)take((size_t)w.nslab * w.ntp * kGramTile * kGramTile * sizeof(double));
    w.G = (double *)take(mat);
    w.A0 = (double *)take(mat);
    w.T = (double *)take(mat);
    w.V[0] = (double *)take(mat);
    w.V[1] = (double *)take(mat);
    w.lam = (double *)take((size_t)w.Bp * sizeof(double));
    w.rot = (double *)take((size_t)kMaxSweeps * (w.Bp - 1) * (w.Bp / 2) * 2 * sizeof(double));
    w.beta = (double *)take((size_t)w.Bp * sizeof(double));
    w.F = (double *)take((size_t)4 * mat);
    w.E = (float *)take((size_t)B * B * sizeof(float));
    return w;
}

static size_t svt_ws_bytes(int64_t P, int64_t B) {
    SvtWs w = svt_ws_layout(nullptr, P, B);
    return (size_t)((char *)(w.E + B * B) - (char *)nullptr) + 256;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt) but not
// for its outstanding global stores (the rotation log), unlike __syncthreads().
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Round-robin (circle method) pair k of round r over indices 0..Bp-1, returned with p < q.
__device__ __forceinline__ void rr_pair(int r, int k, int Bp, int &p, int &q) {
    if (k == 0) { p = Bp - 1; q = r; }
    else { p = (r + k) % (Bp - 1); q = (r - k + (Bp - 1)) % (Bp - 1); }
    if (p > q) { int t = p; p = q; q = t; }
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
        if (i < Bp && j < Bp) {
            const double v = (i < B && j < B) ? s : 0.0;   // pad row/col (B odd) is zero
            G[(int64_t)i * Bp + j] = v;
            G[(int64_t)j * Bp + i] = v;
        }
    }
}

// ---- 2. warm start A0 = V^T (G V) with the current V (16 x 16 fp64 tiles) -------------------
// stage 0: T = G V ; stage 1: A0 = V^T T.  The current V buffer index lives on the device.
__global__ __launch_bounds__(256) void k_gemm_f64_state(SvtWs w, int stage) {
    __shared__ double As[16][17], Bs[16][17];
    const int n = (int)w.Bp;
    const double *V = w.V[w.state[1]];
    const double *A = stage == 0 ? w.G : V;
    const double *Bm = stage == 0 ? V : w.T;
    double *C = stage == 0 ? w.T : w.A0;
    const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;
    const int i = blockIdx.y * 16 + ty, j = blockIdx.x * 16 + tx;
    double acc = 0.0;
    for (int k0 = 0; k0 < n; k0 += 16) {
        const int ka = k0 + tx, kb = k0 + ty;
        if (stage == 1) As[ty][tx] = (i < n && ka < n) ? A[(int64_t)ka * n + i] : 0.0;   // (V^T)[i][ka]
        else As[ty][tx] = (i < n && ka < n) ? A[(int64_t)i * n + ka] : 0.0;
        Bs[ty][tx] = (kb < n && j < n) ? Bm[(int64_t)kb * n + j] : 0.0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = __fma_rn(As[ty][k], Bs[k][tx], acc);
        __syncthreads();
    }
    if (i < n && j < n) C[(int64_t)i * n + j] = acc;
}

// ---- 3. one-workgroup Jacobi on the packed upper triangle in LDS -----------------------------
// Table-driven: per round the pair indices (ip, iq) and rotations (rc, rs) go to LDS once, the
// packed index of (i <= j) is rowoff[i] + j, and the 2x2 block updates are mapped on a 32 x 32
// thread grid (shifts, no divisions in the inner loop).
__device__ __forceinline__ double wg_reduce(double v, double *red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kJacobiThreads / 64; ++i) s += red[i];
    return s;
}

// The solve on A = src (packed into LDS), eigenvalues to w.lam, rounds/sweeps to w.state[2..3].
__device__ __noinline__ void jacobi_core(double *sm, SvtWs w, const double *src) {
    const int Bp = (int)w.Bp, half = Bp / 2;
    const int npk = Bp * (Bp + 1) / 2;
    double *A = sm;                      // packed upper triangle
    double *rc = A + npk, *rs = rc + half, *red = rs + half;
    int *ip = (int *)(red + 16), *iq = ip + half, *rowoff = iq + half;
    __shared__ int any_rot;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < Bp; i += kJacobiThreads) rowoff[i] = i * Bp - (i * (i - 1)) / 2 - i;
    __syncthreads();
    for (int i = 0; i < Bp; ++i)
        for (int j = i + tid; j < Bp; j += kJacobiThreads) A[rowoff[i] + j] = src[(int64_t)i * Bp + j];
    __syncthreads();
    int sweeps = 0, rounds = 0;
    // threshold Jacobi: rotate (p,q) only while |a_pq| > tol * sqrt(|a_pp a_qq|); a sweep without
    // any rotation ends the solve (the off-diagonal mass is then below tol relative).
    const double tol = 1e-7;    // residual a_pq perturbs E = f(A) by ~|a_pq| f'(lambda): << 1e-8 relative in U
    while (sweeps < kMaxSweeps) {
        if (tid == 0) any_rot = 0;
        lds_barrier();
        for (int r = 0; r < Bp - 1; ++r) {
            if (tid < half) {
                int p, q;
                rr_pair(r, tid, Bp, p, q);
                const double app = A[rowoff[p] + p], aqq = A[rowoff[q] + q], apq = A[rowoff[p] + q];
                double c = 1.0, s = 0.0;
                if (fabs(apq) > tol * sqrt(fabs(app * aqq)) && apq != 0.0) {
                    const double theta = (aqq - app) / (2.0 * apq);
                    const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    c = 1.0 / sqrt(t * t + 1.0);
                    s = t * c;
                    any_rot = 1;
                }
                ip[tid] = p;
                iq[tid] = q;
                rc[tid] = c;
                rs[tid] = s;
                double *log = w.rot + ((int64_t)rounds * half + tid) * 2;
                log[0] = c;
                log[1] = s;
            }
            lds_barrier();
            // A <- J^T A J on every unordered 2x2 block (k1 <= k2); J = [[c, s], [-s, c]] on (p, q).
            // One wave per k1 (wave-uniform rotation), lanes over k2; identity pairs are skipped.
            for (int k1 = wv; k1 < half; k1 += kJacobiThreads / 64) {
                const double c1 = rc[k1], s1 = rs[k1];
                const bool id1 = (s1 == 0.0);
                const int p1 = ip[k1], q1 = iq[k1];
                const int ro_p1 = rowoff[p1], ro_q1 = rowoff[q1];
                for (int k2 = k1 + lane; k2 < half; k2 += 64) {
                    const double c2 = rc[k2], s2 = rs[k2];
                    if (id1 && s2 == 0.0) continue;
                    if (k1 == k2) {
                        const int ipp = ro_p1 + p1, iqq = ro_q1 + q1, ipq = ro_p1 + q1;
                        const double a = A[ipp], b = A[ipq], d = A[iqq];
                        const double la = c1 * a - s1 * b, lb = c1 * b - s1 * d;
                        const double lc = s1 * a + c1 * b, ld = s1 * b + c1 * d;
                        A[ipp] = c1 * la - s1 * lb;
                        A[iqq] = s1 * lc + c1 * ld;
                        A[ipq] = 0.0;
                    } else {
                        const int p2 = ip[k2], q2 = iq[k2];
                        const int i00 = p1 <= p2 ? ro_p1 + p2 : rowoff[p2] + p1;
                        const int i01 = p1 <= q2 ? ro_p1 + q2 : rowoff[q2] + p1;
                        const int i10 = q1 <= p2 ? ro_q1 + p2 : rowoff[p2] + q1;
                        const int i11 = q1 <= q2 ? ro_q1 + q2 : rowoff[q2] + q1;
                        const double a = A[i00], b = A[i01], cc = A[i10], d = A[i11];
                        const double la = c1 * a - s1 * cc, lb = c1 * b - s1 * d;
                        const double lc = s1 * a + c1 * cc, ld = s1 * b + c1 * d;
                        A[i00] = c2 * la - s2 * lb;
                        A[i01] = s2 * la + c2 * lb;
                        A[i10] = c2 * lc - s2 * ld;
                        A[i11] = s2 * lc + c2 * ld;
                    }
                }
            }
            lds_barrier();
            ++rounds;
        }
        ++sweeps;
        const int rotated = any_rot;
        lds_barrier();   // every thread has read the flag before thread 0 resets it
        if (!rotated) break;
    }
    for (int i = tid; i < Bp; i += kJacobiThreads) w.lam[i] = A[rowoff[i] + i];
    if (tid == 0) {
        w.state[2] = rounds;
        w.state[3] = sweeps;
    }
    __syncthreads();   // rotation log and eigenvalues visible to the workgroup (in-kernel fallback)
}

__global__ __launch_bounds__(kJacobiThreads) void k_jacobi_lds(SvtWs w, int warm) {
    extern __shared__ double sm[];
    const bool use_warm = warm && w.state[0] == 1;
    jacobi_core(sm, w, use_warm ? w.A0 : w.G);
}

// ---- 4. V_new = V_old J_1 ... J_R, 64 rows per 1024-thread workgroup, rows in LDS ------------
// The rotation log is staged kLogRounds rounds at a time (one global-latency per batch); rounds
// are separated by LDS-only barriers.
constexpr int kVRows = 64;
constexpr int kLogRounds = 16;

// Rows i0 .. i0+63 of Vn = Vo J_1 ... J_R (Vo = identity when null); 1024 threads.
__device__ __noinline__ void vrebuild_tile(double *vsm, SvtWs w, const double *Vo, double *Vn, int i0) {
    const int Bp = (int)w.Bp, half = Bp / 2;
    double *vrow = vsm;                                   // [kVRows][Bp]
    double *lcs = vrow + kVRows * Bp;                     // [kLogRounds][half][2]
    short *lpq = (short *)(lcs + kLogRounds * half * 2);  // [kLogRounds][half][2]
    const int nrows = min(kVRows, Bp - i0);
    for (int idx = threadIdx.x; idx < nrows * Bp; idx += 1024) {
        const int rr = idx / Bp, j = idx % Bp, i = i0 + rr;
        vrow[rr * Bp + j] = Vo ? Vo[(int64_t)i * Bp + j] : (i == j ? 1.0 : 0.0);
    }
    const int rounds = w.state[2];
    const int rr = threadIdx.x >> 4, kk = threadIdx.x & 15;
    for (int rb = 0; rb < rounds; rb += kLogRounds) {
        const int nr = min(kLogRounds, rounds - rb);
        __syncthreads();
        for (int idx = threadIdx.x; idx < nr * half; idx += 1024) {
            const int ro = idx / half, k = idx % half;
            const double *log = w.rot + ((int64_t)(rb + ro) * half + k) * 2;
            lcs[2 * idx] = log[0];
            lcs[2 * idx + 1] = log[1];
            int p, q;
            rr_pair((rb + ro) % (Bp - 1), k, Bp, p, q);
            lpq[2 * idx] = (short)p;
            lpq[2 * idx + 1] = (short)q;
        }
        __syncthreads();
        for (int ro = 0; ro < nr; ++ro) {
            if (rr < nrows) {
                double *row = vrow + rr * Bp;
                for (int k = kk; k < half; k += 16) {
                    const int e = ro * half + k;
                    const double sn = lcs[2 * e + 1];
                    if (sn == 0.0) continue;
                    const double c = lcs[2 * e];
                    const int p = lpq[2 * e], q = lpq[2 * e + 1];
                    const double vp = row[p], vq = row[q];
                    row[p] = c * vp - sn * vq;
                    row[q] = sn * vp + c * vq;
                }
            }
            lds_barrier();
        }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nrows * Bp; idx += 1024) {
        const int r2 = idx / Bp, j = idx % Bp;
        Vn[(int64_t)(i0 + r2) * Bp + j] = vrow[r2 * Bp + j];
    }
}

__global__ __launch_bounds__(1024) void k_jacobi_vrebuild(SvtWs w, int warm) {
    extern __shared__ double vsm[];
    const bool use_warm = warm && w.state[0] == 1;
    const int cur = w.state[1];
    vrebuild_tile(vsm, w, use_warm ? w.V[cur] : nullptr, w.V[cur ^ 1], blockIdx.x * kVRows);
}

__global__ void k_svt_finish_state(SvtWs w) {
    // flip the current-V buffer; V is now valid for warm starts
    w.state[1] ^= 1;
    w.state[0] = 1;
    w.state[4] = 3;
}

}  // namespace lrs

#include <float.h>

#include "svt_eig.h"

namespace lrs {

// ---- 3'. the whole eigen chain in one workgroup: tridiagonal path, Jacobi fallback, E ---------
// V -> w.V[state[1]], eigenvalues -> w.lam, E -> w.E; state[0] = 1 (V valid), state[4] = path.
// Certificate of the tridiagonal path (else the Jacobi fallback on the same G):
//   * max |V^T V - I| <= kEigOrth0 before, and <= kEigOrth after <= 3 Newton-Schulz steps;
//   * per vector, ||T w_i - lambda_i w_i|| plus the mixing the orthogonalisation adds,
//     0.5 ||((lambda_j - lambda_i) (S - I)_ji)_j||, at most kEigRes * ||T||.
// E = f(G) then differs from the exact matrix function by O(kEigRes ||T|| max|f'|).
constexpr double kEigOrth0 = 0.05, kEigOrth = 1e-13, kEigRes = 1e-11;
__global__ __launch_bounds__(kEigThreads) void k_svt_eig(SvtWs w, int B, double tau, int dbg) {
    extern __shared__ double sm[];
    __shared__ double shb[2], red[kEigThreads / 64];
    const int n = (int)w.Bp, tid = threadIdx.x;
    unsigned long long *ts = (unsigned long long *)(w.state + 16);   // phase timestamps (100 MHz)
    if (tid == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
    double *A = sm;
    double *pv = A + (size_t)n * (n + 1) / 2;      // [n] p vector, then the eigenvalues
    for (int e0 = tid; e0 < n * n; e0 += 8 * kEigThreads) {
        double g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * kEigThreads;
            g[u] = e < n * n ? w.G[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * kEigThreads, i = e / n, j = e - i * n;
            if (e < n * n && j >= i) A[pk_idx(i, j, n)] = g[u];
        }
    }
    __syncthreads();
    eig_tridiag(A, pv, shb, n, w.beta);
    if (tid == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
    if (dbg)   // diagnostics: the tridiagonal T (d, e) into the Gram partial buffer
        for (int j = tid; j < n; j += kEigThreads) {
            const int idx = pk_idx(j, j, n);
            w.partial[j] = A[idx];
            w.partial[n + j] = (j + 1 < n) ? A[idx + 1] : 0.0;
        }
    // Gershgorin interval and the tridiagonal's scale (every thread, broadcast reads)
    double gl = 1e300, gu = -1e300, emax2 = 0.0;
    {
        int idx = 0;
        double ep = 0.0;
        for (int j = 0; j < n; ++j) {
            const double e = (j + 1 < n) ? fabs(A[idx + 1]) : 0.0;
            gl = fmin(gl, A[idx] - ep - e);
            gu = fmax(gu, A[idx] + ep + e);
            emax2 = fmax(emax2, e * e);
            ep = e;
            if (j + 1 < n) idx += n - j;
        }
    }
    const double tn = fmax(fmax(fabs(gl), fabs(gu)), 1e-300);
    gl -= 4.0 * DBL_EPSILON * tn * n;
    gu += 4.0 * DBL_EPSILON * tn * n;
    const double pivmin = 1e-290 * fmax(1.0, emax2);
    eig_values(A, n, gl, gu, tn, pivmin, pv, w.lam);
    __syncthreads();
    if (tid == 0) ts[2] = __builtin_amdgcn_s_memrealtime();
    const double res = eig_vectors(A, pv, n, tn, w.F, w.T);
    __syncthreads();
    if (tid == 0) ts[3] = __builtin_amdgcn_s_memrealtime();
    for (int k = tid; k < n - 2; k += kEigThreads) pv[k] = w.beta[k];   // the eigenvalues are in w.lam
    __syncthreads();
    eig_backtransform(A, pv, n, w.T, w.V[0]);
    __syncthreads();
    if (tid == 0) ts[4] = __builtin_amdgcn_s_memrealtime();
    // certificate + orthogonalisation (LDS of the reflectors is free from here on)
    int cur = 0;
    double dev = eig_syrk<true, 1>(sm, w.V[0], n, nullptr, 0.0, 0, nullptr, w.A0, red);
    bool bad = !(dev <= kEigOrth0);
    if (!bad) {
        double mix = 0.0;
        if (tid < n) {
            const double li = w.lam[tid];
            for (int j = 0; j < n; ++j) {
                const double m = (w.lam[j] - li) * (w.A0[(int64_t)j * n + tid] - (j == tid ? 1.0 : 0.0));
                mix = __fma_rn(m, m, mix);
            }
        }
        const double bound = res + 0.5 * sqrt(mix);
        bad = __syncthreads_or(!(bound <= kEigRes * tn));
    }
    for (int step = 0; step < 3 && !bad && dev > kEigOrth; ++step) {
        eig_ns_step(sm, w.V[cur], w.A0, n, w.V[cur ^ 1]);
        cur ^= 1;
        dev = eig_syrk<true, 1>(sm, w.V[cur], n, nullptr, 0.0, 0, nullptr, w.A0, red);
    }
    bad = bad || !(dev <= kEigOrth);
    if (tid == 0) ts[5] = __builtin_amdgcn_s_memrealtime();
    if (dbg) {   // diagnostics: keep the tridiagonal path's V (no fallback, no E)
        if (tid == 0) { w.state[1] = cur; w.state[4] = bad ? 2 : 1; }
        return;
    }
    if (bad) {
        // clustered / repeated eigenvalues: the orthogonal Jacobi basis of the same G
        __syncthreads();
        jacobi_core(sm, w, w.G);
        cur = 0;
        for (int i0 = 0; i0 < n; i0 += kVRows) {
            vrebuild_tile(sm, w, nullptr, w.V[0], i0);
            __syncthreads();
        }
    }
    if (tid == 0) {
        w.state[0] = 1;
        w.state[1] = cur;
        w.state[4] = bad ? 2 : 1;
    }
    __syncthreads();
    eig_syrk<false, 0>(sm, w.V[cur], n, w.lam, tau, B, w.E, nullptr, red);
    if (tid == 0) ts[6] = __builtin_amdgcn_s_memrealtime();
}

// ---- 5a. E = V diag(e) V^T, e_k = min(tau/s_k, 1); s_out = sorted singular values -----------
__global__ __launch_bounds__(256) void k_build_E(SvtWs w, int B, double tau) {
    __shared__ double Vi[16][17], Vj[16][17], ek[16];
    const int Bp = (int)w.Bp;
    const double *V = w.V[w.state[1]];
    const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;
    const int i = blockIdx.y * 16 + ty, jrow0 = blockIdx.x * 16;
    const int j = jrow0 + tx;
    double acc = 0.0;
    for (int k0 = 0; k0 < Bp; k0 += 16) {
        Vi[ty][tx] = (i < Bp && k0 + tx < Bp) ? V[(int64_t)i * Bp + k0 + tx] : 0.0;
        Vj[ty][tx] = (jrow0 + ty < Bp && k0 + tx < Bp) ? V[(int64_t)(jrow0 + ty) * Bp + k0 + tx] : 0.0;
        if (threadIdx.x < 16) {
            const int k = k0 + threadIdx.x;
            double e = 0.0;
            if (k < Bp) {
                const double l = w.lam[k];
                const double s = l > 0.0 ? sqrt(l) : 0.0;
                e = (s > tau) ? tau / s : 1.0;
            }
            ek[threadIdx.x] = e;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = __fma_rn(Vi[ty][k] * ek[k], Vj[tx][k], acc);
        __syncthreads();
    }
    if (i < B && j < B) w.E[(int64_t)i * B + j] = (float)acc;
}

__global__ __launch_bounds__(256) void k_sorted_singular_values(SvtWs w, int B, double *__restrict__ s_out) {
    // rank of each eigenvalue (ties broken by index) -> descending order
    const int Bp = (int)w.Bp;
    for (int i = threadIdx.x; i < Bp; i += blockDim.x) {
        const double li = w.lam[i];
        int rank = 0;
        for (int k = 0; k < Bp; ++k) {
            const double lk = w.lam[k];
            rank += (lk > li) || (lk == li && k < i);
        }
        if (rank < B) s_out[rank] = li > 0.0 ? sqrt(li) : 0.0;
    }
}

// ---- 5b'. U = Z - Z E on the bf16 matrix cores (B <= 224) -----------------------------------
// Operands split exactly into three bf16 terms, six partial products (fp32-GEMM accuracy), so
// the product leaves the VALU, which the concurrently running sparse-coding kernel saturates.
// grid (row groups, column chunks of 64): each workgroup stages its 64 columns of E once (three
// bf16 images [col][k], 464-B rows: conflict-free ds_read_b128) and loops over row blocks of 64;
// wave w owns rows 16w..16w+15 of a block, 4 column tiles.
typedef __bf16 sbf16x8 __attribute__((ext_vector_type(8)));
constexpr int kApKMax = 224, kApLd = 232, kApCols = 64;

__device__ __forceinline__ void ap_split3(float v, __bf16 &a, __bf16 &b, __bf16 &c) {
    a = (__bf16)v;
    const float r1 = v - (float)a;
    b = (__bf16)r1;
    c = (__bf16)(r1 - (float)b);
}

__device__ __forceinline__ floatx4 ap_mfma(const sbf16x8 &a, const sbf16x8 &b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void k_svt_apply_b3(const float *__restrict__ X, const float *__restrict__ L2,
                                                      float c2, const float *__restrict__ E, int64_t P, int B,
                                                      float *__restrict__ U) {
    extern __shared__ __align__(16) __bf16 Es[];   // [3][kApCols][kApLd]
    const int c0 = blockIdx.y * kApCols;
    for (int idx = threadIdx.x; idx < kApCols * kApKMax; idx += 256) {
        const int cc = idx / kApKMax, k = idx % kApKMax;
        const int c = c0 + cc;
        const float v = (k < B && c < B) ? E[(int64_t)k * B + c] : 0.0f;
        __bf16 a, b, d;
        ap_split3(v, a, b, d);
        Es[(0 * kApCols + cc) * kApLd + k] = a;
        Es[(1 * kApCols + cc) * kApLd + k] = b;
        Es[(2 * kApCols + cc) * kApLd + k] = d;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int jl = lane & 15, g = lane >> 4;
    const int nks = (B + 31) / 32;
    for (int64_t rb = (int64_t)blockIdx.x * 64; rb < P; rb += (int64_t)gridDim.x * 64) {
        const int64_t row = rb + 16 * w + jl;            // A-operand row of this lane
        floatx4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < nks; ++ks) {
            const int kb = 32 * ks + 8 * g;
            sbf16x8 A[3];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = kb + j;
                float z = 0.0f;
                if (row < P && k < B) {
                    z = X[row * B + k];
                    if (L2) z = z + c2 * L2[row * B + k];
                }
                __bf16 a, b, d;
                ap_split3(z, a, b, d);
                A[0][j] = a; A[1][j] = b; A[2][j] = d;
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int cc = 16 * t + jl;
                sbf16x8 Bf[3];
#pragma unroll
                for (int sp = 0; sp < 3; ++sp)
                    Bf[sp] = *reinterpret_cast<const sbf16x8 *>(&Es[(sp * kApCols + cc) * kApLd + kb]);
                floatx4 a4 = acc[t];
                a4 = ap_mfma(A[2], Bf[0], a4);
                a4 = ap_mfma(A[1], Bf[1], a4);
                a4 = ap_mfma(A[0], Bf[2], a4);
                a4 = ap_mfma(A[1], Bf[0], a4);
                a4 = ap_mfma(A[0], Bf[1], a4);
                a4 = ap_mfma(A[0], Bf[0], a4);
                acc[t] = a4;
            }
        }
        // C layout: rows 4g + i of the wave's 16, column jl of tile t
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = c0 + 16 * t + jl;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = rb + 16 * w + 4 * g + i;
                if (r < P && c < B) {
                    float z = X[r * B + c];
                    if (L2) z = z + c2 * L2[r * B + c];
                    U[r * B + c] = z - acc[t][i];
                }
            }
        }
    }
}

// ---- 5b. U = Z - Z E  (64 x 64 output tile per workgroup, f32) ------------------------------
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
            const int rr = idx / kAK, kk = idx % kAK;
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

// Stage 1 (multi-workgroup, ~0.3 ms): fp64 Gram and, when warm, A0 = V^T G V.
extern "C" int lrs_svt_gram_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, int warm, void *ws,
                                size_t ws_bytes, void *stream) {
    if (!X || !ws || P <= 0 || B <= 0) return LRS_E_INVALID;
    if (B + (B & 1) > kMaxBp) return LRS_E_UNSUPPORTED;
    if (ws_bytes < svt_ws_bytes(P, B)) return LRS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    SvtWs w = svt_ws_layout(ws, P, B);
    if (!warm) {
        hipError_t e = hipMemsetAsync(w.state, 0, sizeof(int) * 4, st);
        if (e != hipSuccess) return (int)e;
    }
    const int nt = (int)gram_ntiles(B);
    const int Bp = (int)w.Bp;
    hipLaunchKernelGGL(k_gram_partial, dim3((unsigned)w.ntp, (unsigned)w.nslab), dim3(256), 0, st, X, L2, c2, P,
                       (int)B, nt, w.partial);
    LRS_CHECK_LAUNCH();
    const int64_t tot = w.ntp * kGramTile * kGramTile;
    hipLaunchKernelGGL(k_gram_reduce, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 4096)), dim3(256), 0, st,
                       w.partial, w.nslab, (int)w.ntp, nt, (int)B, Bp, w.G);
    LRS_CHECK_LAUNCH();
    if ((warm & LRS_SVT_WARM) && (warm & LRS_SVT_JACOBI)) {
        // A0 = V^T (G V) with the current V (unused when V is not valid yet: Jacobi starts from G)
        const dim3 g16((Bp + 15) / 16, (Bp + 15) / 16);
        hipLaunchKernelGGL(k_gemm_f64_state, g16, dim3(256), 0, st, w, 0);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_gemm_f64_state, g16, dim3(256), 0, st, w, 1);
        LRS_CHECK_LAUNCH();
    }
    return LRS_OK;
}

// Stage 2: one-workgroup Jacobi (runs beside the sparse-coding kernel), V replay, E, U.
extern "C" int lrs_svt_finish_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau,
                                  float *U, double *s_out, int warm, void *ws, size_t ws_bytes, void *stream) {
    if (!X || !U || !ws || P <= 0 || B <= 0 || tau < 0.0) return LRS_E_INVALID;
    if (B + (B & 1) > kMaxBp) return LRS_E_UNSUPPORTED;
    if (ws_bytes < svt_ws_bytes(P, B)) return LRS_E_WORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    SvtWs w = svt_ws_layout(ws, P, B);
    const int Bp = (int)w.Bp;
    const size_t smem = sizeof(double) * ((size_t)Bp * (Bp + 1) / 2 + Bp + 16) + sizeof(int) * (2 * Bp);
    const size_t vsmem = sizeof(double) * ((size_t)kVRows * Bp + (size_t)kLogRounds * (Bp / 2) * 2) +
                         sizeof(short) * (size_t)kLogRounds * (Bp / 2) * 2;
    if (warm & LRS_SVT_JACOBI) {
        const int jwarm = warm & LRS_SVT_WARM;
        // dynamic LDS above 64 KiB must be opted into; request exactly what this shape needs
        hipError_t ea = hipFuncSetAttribute((const void *)k_jacobi_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)smem);
        if (ea != hipSuccess) return (int)ea;
        ea = hipFuncSetAttribute((const void *)k_jacobi_vrebuild, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)vsmem);
        if (ea != hipSuccess) return (int)ea;
        hipLaunchKernelGGL(k_jacobi_lds, dim3(1), dim3(kJacobiThreads), smem, st, w, jwarm);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_jacobi_vrebuild, dim3((unsigned)((Bp + kVRows - 1) / kVRows)), dim3(1024), vsmem, st,
                           w, jwarm);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_svt_finish_state, dim3(1), dim3(1), 0, st, w);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_build_E, dim3((unsigned)((B + 15) / 16), (unsigned)((B + 15) / 16)), dim3(256), 0, st,
                           w, (int)B, tau);
        LRS_CHECK_LAUNCH();
    } else {
        const size_t tsmem = sizeof(double) * ((size_t)Bp * (Bp + 1) / 2 + Bp);
        const size_t esmem = sizeof(double) * 2 * kEKc * kELd;
        const size_t lds = std::max(std::max(tsmem, esmem), std::max(smem, vsmem));
        hipError_t ea = hipFuncSetAttribute((const void *)k_svt_eig, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)lds);
        if (ea != hipSuccess) return (int)ea;
        hipLaunchKernelGGL(k_svt_eig, dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau, 0);
        LRS_CHECK_LAUNCH();
    }
    if (s_out) {
        hipLaunchKernelGGL(k_sorted_singular_values, dim3(1), dim3(256), 0, st, w, (int)B, s_out);
        LRS_CHECK_LAUNCH();
    }
    if (B <= kApKMax) {
        const size_t lds = sizeof(__bf16) * 3 * kApCols * kApLd;
        hipError_t e = hipFuncSetAttribute((const void *)k_svt_apply_b3, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return (int)e;
        int64_t rgroups = (P + 63) / 64;
        if (rgroups > 64) rgroups = 64;
        dim3 grid((unsigned)rgroups, (unsigned)((B + kApCols - 1) / kApCols));
        hipLaunchKernelGGL(k_svt_apply_b3, grid, dim3(256), lds, st, X, L2, c2, w.E, P, (int)B, U);
    } else {
        dim3 grid((unsigned)((P + kAT - 1) / kAT), (unsigned)((B + kAT - 1) / kAT));
        hipLaunchKernelGGL(k_svt_apply, grid, dim3(256), 0, st, X, L2, c2, w.E, P, (int)B, U);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_svt_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau, float *U,
                           double *s_out, int warm, void *ws, size_t ws_bytes, void *stream) {
    if (!U || tau < 0.0) return LRS_E_INVALID;
    int rc = lrs_svt_gram_f32(X, L2, c2, P, B, warm, ws, ws_bytes, stream);
    if (rc != LRS_OK) return rc;
    return lrs_svt_finish_f32(X, L2, c2, P, B, tau, U, s_out, warm, ws, ws_bytes, stream);
}

// Diagnostics (not in include/lrspnp.h): state words of the last call (host copy): V valid, V buffer,
// Jacobi rounds, sweeps, path (1 tridiagonal, 2 Jacobi fallback, 3 Jacobi), 11 spare, then 8 u64
// phase timestamps of the tridiagonal path (s_memrealtime, 100 MHz).
extern "C" int lrs_diag_svt_state(void *ws, int64_t P, int64_t B, int *out32) {
    SvtWs w = svt_ws_layout(ws, P, B);
    return (int)hipMemcpy(out32, w.state, 32 * sizeof(int), hipMemcpyDeviceToHost);
}

// Diagnostics: the tridiagonal path on the Gram already in ws (after lrs_svt_gram_f32), no fallback,
// leaving T (d, e) in the partial buffer, eigenvalues in lam, W in T, V in V[state[1]], S in A0.
extern "C" int lrs_diag_svt_eig(void *ws, int64_t P, int64_t B, double *out, void *stream) {
    SvtWs w = svt_ws_layout(ws, P, B);
    const int Bp = (int)w.Bp;
    const size_t smem = std::max(sizeof(double) * ((size_t)Bp * (Bp + 1) / 2 + Bp + 16) + sizeof(int) * (2 * Bp),
                                 sizeof(double) * 2 * kEKc * kELd);
    hipError_t ea = hipFuncSetAttribute((const void *)k_svt_eig, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (ea != hipSuccess) return (int)ea;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_svt_eig, dim3(1), dim3(kEigThreads), smem, st, w, (int)B, 1.0, 1);
    LRS_CHECK_LAUNCH();
    // out: d[Bp], e[Bp], lam[Bp], W[Bp*Bp], V[Bp*Bp], S[Bp*Bp]
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    int state[8];
    e = hipMemcpy(state, w.state, sizeof(state), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return (int)e;
    const size_t m = (size_t)Bp * Bp;
    hipMemcpy(out, w.partial, 2 * Bp * sizeof(double), hipMemcpyDeviceToHost);
    hipMemcpy(out + 2 * Bp, w.lam, Bp * sizeof(double), hipMemcpyDeviceToHost);
    hipMemcpy(out + 3 * Bp, w.T, m * sizeof(double), hipMemcpyDeviceToHost);
    hipMemcpy(out + 3 * Bp + m, w.V[state[1]], m * sizeof(double), hipMemcpyDeviceToHost);
    e = hipMemcpy(out + 3 * Bp + 2 * m, w.A0, m * sizeof(double), hipMemcpyDeviceToHost);
    return e != hipSuccess ? (int)e : state[4];
}
