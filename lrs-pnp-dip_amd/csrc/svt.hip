// SVT low-rank prox: U = SVT(Z, tau), Z = X + c2*L2 (main_LRS_PnP.py:112-124, called at :315 as
// SVT(X + (1/mu_2)*lambda_2, 1/mu_2)).
//
// The reference runs a float32 LAPACK SVD of the P x B matrix.  Here, MI355X-first:
//   1. fp64 Gram G = Z^T Z over row slabs (many workgroups, coalesced rows), fixed-order reduce;
//   2. warm start: A0 = V^T G V with the previous outer iteration's eigenvectors (tiled fp64
//      GEMMs) — nearly diagonal, so Jacobi needs 1-3 sweeps instead of ~8;
//   3. ONE workgroup runs a cyclic parallel (round-robin) two-sided Jacobi on A held in LDS as a
//      packed fp64 upper triangle (B <= 198: <= 157,608 B), logging each round's rotations;
//   4. the eigenvector update V <- V J_1 ... J_R is replayed from the log row by row in parallel
//      (rows of V evolve independently), off the Jacobi workgroup's critical path;
//   5. E = V diag(min(tau/s, 1)) V^T (fp64 -> f32) and U = Z - Z E.
//      Z V diag((s-tau)_+/s) V^T == U_s (S-tau)_+ V_h, and E is small so its f32 rounding costs
//      << 1e-6 relative in U.
// The whole chain runs on its own stream beside the sparse-coding kernel.
#include <math.h>

#include <algorithm>
#include <utility>

#include "lrs_common.h"

namespace lrs {

constexpr int kGramSlabs = 256;
// k-steps of 4 of the SVT apply: 50 up to B = 200, 64 up to 256
__host__ __device__ constexpr int ap_steps(int64_t B) { return B <= 200 ? 50 : 64; }
constexpr int kJacobiThreads = 1024;
// The packed fp64 triangle of 198 x 198 = 157,608 B fits the LDS beside the solver's vectors and
// flags (at Bp = 200 the chain would need 164,128 B > 160 KiB): up to kLdsMaxBp the one-workgroup
// chain keeps it in LDS; above (the 224-band cubes of BASELINE configs[3]/[4]) the same chain runs
// on the packed triangle in the workspace (L2-resident: 224^2/2 x 8 B = 200 KB), with full
// workgroup barriers instead of LDS-only ones.  kMaxBp: every phase's register / lane layout.
constexpr int kLdsMaxBp = 198;
constexpr int kMaxBp = 256;
constexpr int kMaxSweeps = 40;

// Gram column blocks of 16: 13 up to B = 208 (91 tile pairs), 16 up to 256 (136)
__host__ __device__ constexpr int gram_nt(int64_t B) { return B <= 208 ? 13 : 16; }
__host__ __device__ constexpr int gram_npairs(int nt) { return nt * (nt + 1) / 2; }

struct SvtWs {
    double *partial;  // [kGramSlabs][16x16 tile pairs][256]  Gram partials
    double *G;        // [Bp][Bp]
    double *A0;       // [Bp][Bp]  V^T G V (warm start)
    double *T;        // [Bp][Bp]  scratch
    double *V[2];     // [Bp][Bp]  eigenvectors, double-buffered
    double *lam;      // [Bp]      eigenvalues (diag of the converged A)
    double *rot;      // [kMaxSweeps*(Bp-1)][Bp/2][2]  (c, s) per round and pair
    double *beta;     // [Bp]      Householder scalars (tridiagonal path)
    double *F;        // [Bp][4][Bp] pivoted LU rows of T - lambda_i I (inverse iteration)
    float *E;         // [B][B]
    float *Fp;        // [ap_steps(B)][B][4]  I - E in the apply kernel's fragment order
    int *state;       // [0] V valid, [1] current V buffer, [2] rounds, [3] sweeps,
                      // [4] path of the last solve (1 tridiagonal, 2 Jacobi fallback, 3 Jacobi)
    int64_t Bp;
};


static SvtWs svt_ws_layout(void *base, int64_t P, int64_t B) {
    SvtWs w;
    w.Bp = B + (B & 1);
    char *p = (char *)base;
    auto take = [&](size_t bytes) {
        char *r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    const size_t mat = (size_t)w.Bp * w.Bp * sizeof(double);
    w.state = (int *)take(256);
    w.partial = (double *)take((size_t)kGramSlabs * gram_npairs(gram_nt(B)) * 256 * sizeof(double));
    w.G = (double *)take(mat);
    w.A0 = (double *)take(mat);
    w.T = (double *)take(mat);
    w.V[0] = (double *)take(mat);
    w.V[1] = (double *)take(mat);
    w.lam = (double *)take((size_t)w.Bp * sizeof(double));
    w.rot = (double *)take((size_t)kMaxSweeps * (w.Bp - 1) * (w.Bp / 2) * 2 * sizeof(double));
    w.beta = (double *)take((size_t)w.Bp * sizeof(double));
    w.F = (double *)take((size_t)4 * mat);
    w.Fp = (float *)take((size_t)ap_steps(B) * B * 4 * sizeof(float));
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

// ---- 1. Gram G = Z^T Z on the fp64 matrix cores ---------------------------------------------
// Z = X + c2*L2 (float32: exact in fp64).  One workgroup per slab of rows computes every 16 x 16
// tile pair (a <= b) of the nt = ceil(B/16) column blocks, so Z is read from HBM once: rows are
// staged kGramChunk at a time into LDS with float4 loads (Z formed on the way), then per k-step
// of 4 rows a lane reads Z[p0 + (l>>4)][16c + (l&15)] for all nt blocks (the A and B fragments of
// v_mfma_f64_16x16x4 have that same form) and wave w issues the MFMAs of pairs w, w + 4, ...
// (compile-time pair lists: one instantiation per wave).  Partials [slab][pair][16*16] are
// reduced in fixed order, so G is deterministic.
typedef double doublex4 __attribute__((ext_vector_type(4)));
// NT column blocks (B <= 16 NT) over NW waves: 13 / 4 waves (91 pairs) up to B = 208, 16 / 8 waves
// (136 pairs, 17 accumulators per wave) up to 256
constexpr int kGramChunk = 32;   // rows per LDS chunk (row stride 16 NT + 4)
constexpr int kGramBatch = 13;   // loads in flight per thread

template <int NT>
struct GramPairs {
    int a[gram_npairs(NT)], b[gram_npairs(NT)];
};
template <int NT>
__host__ __device__ constexpr GramPairs<NT> gram_pairs() {
    GramPairs<NT> t{};
    int k = 0;
    for (int a = 0; a < NT; ++a)
        for (int b = a; b < NT; ++b) {
            t.a[k] = a;
            t.b[k] = b;
            ++k;
        }
    return t;
}

template <int NT, int PI>
struct GramPair {
    static constexpr int a = gram_pairs<NT>().a[PI], b = gram_pairs<NT>().b[PI];
};

template <int NT, int NW, int W, int... U>
__device__ __forceinline__ void gram_mfmas(const double (&f)[NT], doublex4 (&acc)[sizeof...(U)],
                                           std::integer_sequence<int, U...>) {
    ((acc[U] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[GramPair<NT, W + NW * U>::a], f[GramPair<NT, W + NW * U>::b],
                                                    acc[U], 0, 0, 0)),
     ...);
}

// Whole workgroup body for wave W (every wave runs the same staging and barriers; the pair list,
// the accumulators and their stores are compile-time per wave, so they stay in registers).
template <int NT, int NW, int W>
__device__ __forceinline__ void gram_body(float *Zs, const float *__restrict__ X, const float *__restrict__ L2,
                                          float c2, int B, int64_t pbeg, int64_t pend, double *__restrict__ out) {
    constexpr int kGramPairs = gram_npairs(NT), kGramLd = 16 * NT + 4, NTH = 64 * NW;
    constexpr int NP = (kGramPairs - W + NW - 1) / NW;
    const int lane = threadIdx.x & 63, g = lane >> 4, jl = lane & 15;
    doublex4 acc[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) acc[u] = doublex4{0.0, 0.0, 0.0, 0.0};
    for (int64_t c0 = pbeg; c0 < pend; c0 += kGramChunk) {
        const int rows = (int)min<int64_t>(kGramChunk, pend - c0);
        __syncthreads();
        // rows x B elements, kGramBatch loads in flight per thread, then the LDS stores
        for (int e0 = threadIdx.x; e0 < kGramChunk * B; e0 += NTH * kGramBatch) {
            float z[kGramBatch];
#pragma unroll
            for (int u = 0; u < kGramBatch; ++u) {
                const int e = e0 + NTH * u, rr = e / B;
                z[u] = 0.f;
                if (e < kGramChunk * B && rr < rows) {
                    const int64_t o = c0 * B + e;
                    z[u] = X[o];
                    if (L2) z[u] = z[u] + c2 * L2[o];   // X + (1/mu_2)*lambda_2
                }
            }
#pragma unroll
            for (int u = 0; u < kGramBatch; ++u) {
                const int e = e0 + NTH * u, rr = e / B, c = e - rr * B;
                if (e < kGramChunk * B) Zs[rr * kGramLd + c] = z[u];
            }
        }
        for (int idx = threadIdx.x; idx < kGramChunk * (kGramLd - B); idx += NTH) {   // zero pad columns
            const int rr = idx / (kGramLd - B), c = B + idx % (kGramLd - B);
            Zs[rr * kGramLd + c] = 0.f;
        }
        __syncthreads();
        const int rows4 = (rows + 3) & ~3;
        for (int r = 0; r < rows4; r += 4) {
            double f[NT];
#pragma unroll
            for (int c = 0; c < NT; ++c) f[c] = (double)Zs[(r + g) * kGramLd + 16 * c + jl];
            gram_mfmas<NT, NW, W>(f, acc, std::make_integer_sequence<int, NP>{});
        }
    }
    // C/D layout of the f64 MFMA: column l & 15, row (l >> 4) + 4 r
#pragma unroll
    for (int u = 0; u < NP; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(int64_t)(W + NW * u) * 256 + (g + 4 * r) * 16 + jl] = acc[u][r];
}

template <int NT, int NW, int... W>
__device__ __forceinline__ void gram_dispatch(int wv, float *Zs, const float *X, const float *L2, float c2, int B,
                                              int64_t pbeg, int64_t pend, double *out, std::integer_sequence<int, W...>) {
    ((wv == W ? gram_body<NT, NW, W>(Zs, X, L2, c2, B, pbeg, pend, out) : (void)0), ...);
}

template <int NT, int NW>
__global__ __launch_bounds__(64 * NW, 1) void k_gram_mfma(const float *__restrict__ X, const float *__restrict__ L2,
                                                          float c2, int64_t P, int B, int64_t rows_per_slab,
                                                          double *__restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float Zs[kGramChunk * (16 * NT + 4)];
    const int sl = blockIdx.x, wv = threadIdx.x >> 6;
    const int64_t pbeg = (int64_t)sl * rows_per_slab, pend = min<int64_t>(P, pbeg + rows_per_slab);
    double *out = partial + (int64_t)sl * gram_npairs(NT) * 256;
    gram_dispatch<NT, NW>(wv, Zs, X, L2, c2, B, pbeg, pend, out, std::make_integer_sequence<int, NW>{});
}

// ---- 1b. fixed-order reduction of the slab partials into the full symmetric Gram ------------
__global__ __launch_bounds__(256) void k_gram_reduce16(const double *__restrict__ partial, int nslab, int nt, int B,
                                                       int Bp, double *__restrict__ G) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)Bp * Bp) return;
    const int i = (int)(idx / Bp), j = (int)(idx % Bp);
    if (j < i) return;
    double s = 0.0;
    if (i < B && j < B) {
        const int a = i >> 4, b = j >> 4, npair = gram_npairs(nt);
        const int pi = a * nt - ((a * (a - 1)) >> 1) + (b - a);
        const int e = (i & 15) * 16 + (j & 15);
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int sl = 0;
        for (; sl + 8 <= nslab; sl += 8)
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += partial[((int64_t)(sl + u) * npair + pi) * 256 + e];
        for (; sl < nslab; ++sl) acc[sl & 7] += partial[((int64_t)sl * npair + pi) * 256 + e];
        s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    G[(int64_t)i * Bp + j] = s;   // pad row/col (B odd) is zero
    G[(int64_t)j * Bp + i] = s;
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

// The solve on A = src (packed into LDS, or with GA into Ag in the workspace when the triangle
// exceeds the LDS: B > kLdsMaxBp), eigenvalues to w.lam, rounds/sweeps to w.state[2..3].
template <bool GA>
__device__ __forceinline__ void jac_bar() {
    if (GA) __syncthreads();
    else lds_barrier();
}

template <bool GA>
__device__ __noinline__ void jacobi_core(double *sm, SvtWs w, const double *src, double *Ag = nullptr) {
    const int Bp = (int)w.Bp, half = Bp / 2;
    const int npk = Bp * (Bp + 1) / 2;
    double *A = GA ? Ag : sm;            // packed upper triangle
    double *rc = GA ? sm : A + npk, *rs = rc + half, *red = rs + half;
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
        jac_bar<GA>();
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
            jac_bar<GA>();
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
            jac_bar<GA>();
            ++rounds;
        }
        ++sweeps;
        const int rotated = any_rot;
        jac_bar<GA>();   // every thread has read the flag before thread 0 resets it
        if (!rotated) break;
    }
    for (int i = tid; i < Bp; i += kJacobiThreads) w.lam[i] = A[rowoff[i] + i];
    if (tid == 0) {
        w.state[2] = rounds;
        w.state[3] = sweeps;
    }
    __syncthreads();   // rotation log and eigenvalues visible to the workgroup (in-kernel fallback)
}

// GA: the triangle in w.T (free here: the warm start's G V product is consumed into A0)
template <bool GA>
__global__ __launch_bounds__(kJacobiThreads) void k_jacobi_lds(SvtWs w, int warm) {
    extern __shared__ double sm[];
    const bool use_warm = warm && w.state[0] == 1;
    jacobi_core<GA>(sm, w, use_warm ? w.A0 : w.G, w.T);
}

// ---- 4. V_new = V_old J_1 ... J_R, 64 rows per 1024-thread workgroup, rows in LDS ------------
// The rotation log is staged kLogRounds rounds at a time (one global-latency per batch); rounds
// are separated by LDS-only barriers.
constexpr int kVRows = 64;
constexpr int kLogRounds = 16;

// Rows i0 .. i0 + vrows - 1 of Vn = Vo J_1 ... J_R (Vo = identity when null); 1024 threads.
// vrows = kVRows, or half that where 64 rows of Bp > kLdsMaxBp exceed the LDS (vrebuild_rows).
__host__ __device__ constexpr int vrebuild_rows(int Bp) { return Bp <= kLdsMaxBp ? kVRows : kVRows / 2; }
__host__ __device__ constexpr size_t vrebuild_lds(int Bp) {
    return sizeof(double) * ((size_t)vrebuild_rows(Bp) * Bp + (size_t)kLogRounds * (Bp / 2) * 2) +
           sizeof(short) * (size_t)kLogRounds * (Bp / 2) * 2;
}

__device__ __noinline__ void vrebuild_tile(double *vsm, SvtWs w, const double *Vo, double *Vn, int i0) {
    const int Bp = (int)w.Bp, half = Bp / 2, vrows = vrebuild_rows(Bp);
    double *vrow = vsm;                                   // [vrows][Bp]
    double *lcs = vrow + vrows * Bp;                      // [kLogRounds][half][2]
    short *lpq = (short *)(lcs + kLogRounds * half * 2);  // [kLogRounds][half][2]
    const int nrows = min(vrows, Bp - i0);
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
    vrebuild_tile(vsm, w, use_warm ? w.V[cur] : nullptr, w.V[cur ^ 1], blockIdx.x * vrebuild_rows((int)w.Bp));
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

// packed upper triangle of G (fp64, [n][n] in global) into LDS
__device__ __forceinline__ void eig_load_packed(const double *G, double *A, int n) {
    const int tid = threadIdx.x;
    for (int e0 = tid; e0 < n * n; e0 += 8 * kEigThreads) {
        double g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * kEigThreads;
            g[u] = e < n * n ? G[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + u * kEigThreads, i = e / n, j = e - i * n;
            if (e < n * n && j >= i) A[pk_idx(i, j, n)] = g[u];
        }
    }
}

// Gershgorin interval of T (diagonal / first superdiagonal of the packed A), its scale and the
// Sturm pivot floor (every thread, broadcast reads)
__device__ __forceinline__ void eig_bounds(const double *A, int n, double &gl, double &gu, double &tn, double &pivmin) {
    gl = 1e300;
    gu = -1e300;
    double emax2 = 0.0;
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
    tn = fmax(fmax(fabs(gl), fabs(gu)), 1e-300);
    gl -= 4.0 * DBL_EPSILON * tn * n;
    gu += 4.0 * DBL_EPSILON * tn * n;
    pivmin = 1e-290 * fmax(1.0, emax2);
}

// D + F of the chain (one workgroup): the certificate on V = w.V[0], at most 3 Newton-Schulz
// steps, the Jacobi fallback, then E.  res = this thread's eigenvector residual (thread i < n).
// NB: the fp64 products' block count (eig_nb); GA: the fallback's packed triangle in w.T (free once
// the back-transformation has consumed W) instead of LDS.
template <int NB, bool GA>
__device__ __forceinline__ void eig_certify_finish(double *sm, double *red, const SvtWs &w, int n, int B, double tau,
                                                   double tn, double res, int dbg, unsigned long long *ts) {
    const int tid = threadIdx.x;
    int cur = 0;
    double dev = eig_syrk<true, 1, NB>(sm, w.V[0], n, nullptr, 0.0, 0, nullptr, w.A0, red);
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
        eig_ns_step<NB>(sm, w.V[cur], w.A0, n, w.V[cur ^ 1]);
        cur ^= 1;
        dev = eig_syrk<true, 1, NB>(sm, w.V[cur], n, nullptr, 0.0, 0, nullptr, w.A0, red);
    }
    bad = bad || !(dev <= kEigOrth);
    if (ts && tid == 0) ts[5] = __builtin_amdgcn_s_memrealtime();
    if (dbg) {   // diagnostics: keep the tridiagonal path's V (no fallback, no E)
        if (tid == 0) { w.state[1] = cur; w.state[4] = bad ? 2 : 1; }
        return;
    }
    if (bad) {
        // clustered / repeated eigenvalues: the orthogonal Jacobi basis of the same G
        __syncthreads();
        jacobi_core<GA>(sm, w, w.G, w.T);
        cur = 0;
        for (int i0 = 0; i0 < n; i0 += vrebuild_rows(n)) {
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
    eig_syrk<false, 0, NB>(sm, w.V[cur], n, w.lam, tau, B, w.E, nullptr, red, w.Fp);
    if (ts && tid == 0) ts[6] = __builtin_amdgcn_s_memrealtime();
}

// GA (B > kLdsMaxBp): the packed A (reflectors + T) in w.A0, dead once the back-transformation is
// done (the certificate then writes S there), the LDS holding only the vectors and the products'
// staging
template <int NB, bool GA>
__global__ __launch_bounds__(kEigThreads) void k_svt_eig(SvtWs w, int B, double tau, int dbg) {
    extern __shared__ double sm[];
    __shared__ double shb[2], red[kEigThreads / 64];
    const int n = (int)w.Bp, tid = threadIdx.x;
    unsigned long long *ts = (unsigned long long *)(w.state + 16);   // phase timestamps (100 MHz)
    if (tid == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
    double *A = GA ? w.A0 : sm;
    double *pv = GA ? sm : A + (size_t)n * (n + 1) / 2;   // [n] p vector, then the eigenvalues
    eig_load_packed(w.G, A, n);
    __syncthreads();
    eig_tridiag<GA>(A, pv, shb, n, w.beta);
    if (tid == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
    if (dbg)   // diagnostics: the tridiagonal T (d, e) into the Gram partial buffer
        for (int j = tid; j < n; j += kEigThreads) {
            const int idx = pk_idx(j, j, n);
            w.partial[j] = A[idx];
            w.partial[n + j] = (j + 1 < n) ? A[idx + 1] : 0.0;
        }
    double gl, gu, tn, pivmin;
    eig_bounds(A, n, gl, gu, tn, pivmin);
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
    eig_certify_finish<NB, GA>(sm, red, w, n, B, tau, tn, res, dbg, ts);
}

// ---- 3''. the same chain over several workgroups (LRS_SVT_MULTI_WG) ---------------------------
// Phases B (eigenvalues: 4 threads each), C (inverse iteration: a thread per eigenvector) and E
// (back-transformation: a wave per 4 columns) are independent per eigenvalue / vector / column, so
// they run on many CUs; A (tridiagonalisation) and D + F (certificate, fallback, E) stay on one
// workgroup.  Every phase calls the device function k_svt_eig calls, with its workgroup's offset,
// so the result is bit-identical.  For a caller whose chain is on the critical path (a row-slab
// shard): beside a chip-filling sparse-coding kernel the one-workgroup chain is the
// better choice (each launch here waits for free CUs).  Packed A (reflectors + T) passes through
// w.A0 (free until the certificate), the residuals through w.partial.
template <bool GA>
__global__ __launch_bounds__(kEigThreads) void k_svt_eig_tri(SvtWs w) {
    extern __shared__ double sm[];
    __shared__ double shb[2];
    const int n = (int)w.Bp, tid = threadIdx.x;
    double *A = GA ? w.A0 : sm;   // GA: reduced in place in the workspace
    double *pv = GA ? sm : A + (size_t)n * (n + 1) / 2;
    eig_load_packed(w.G, A, n);
    __syncthreads();
    eig_tridiag<GA>(A, pv, shb, n, w.beta);
    __syncthreads();
    if (GA) return;
    const int np = n * (n + 1) / 2;
    for (int e = tid; e < np; e += kEigThreads) w.A0[e] = A[e];
}

constexpr int kEigMwThreads = 64;   // one wave per workgroup for phases B and C (one per CU)

__global__ __launch_bounds__(kEigMwThreads) void k_svt_eig_vals(SvtWs w) {
    const int n = (int)w.Bp;
    double gl, gu, tn, pivmin;
    eig_bounds(w.A0, n, gl, gu, tn, pivmin);
    eig_values(w.A0, n, gl, gu, tn, pivmin, w.lam, w.lam, kEigMwThreads * blockIdx.x);
}

__global__ __launch_bounds__(kEigMwThreads) void k_svt_eig_vecs(SvtWs w) {
    const int n = (int)w.Bp;
    double gl, gu, tn, pivmin;
    eig_bounds(w.A0, n, gl, gu, tn, pivmin);
    const double r = eig_vectors(w.A0, w.lam, n, tn, w.F, w.T, kEigMwThreads * blockIdx.x);
    const int i = kEigMwThreads * blockIdx.x + threadIdx.x;
    if (i < n) w.partial[i] = r;
}

__global__ __launch_bounds__(256) void k_svt_eig_back(SvtWs w) {
    eig_backtransform(w.A0, w.beta, (int)w.Bp, w.T, w.V[0], 4 * blockIdx.x, 4 * gridDim.x);
}

template <int NB, bool GA>
__global__ __launch_bounds__(kEigThreads) void k_svt_eig_cert(SvtWs w, int B, double tau) {
    extern __shared__ double sm[];
    __shared__ double red[kEigThreads / 64];
    const int n = (int)w.Bp, tid = threadIdx.x;
    const double res = tid < n ? w.partial[tid] : 0.0;
    double gl, gu, tn, pivmin;
    eig_bounds(w.A0, n, gl, gu, tn, pivmin);   // from the packed A, before the certificate reuses A0
    __syncthreads();
    eig_certify_finish<NB, GA>(sm, red, w, n, B, tau, tn, res, 0, nullptr);
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
    if (i < B && j < B) {
        w.E[(int64_t)i * B + j] = (float)acc;
        store_fp(w.Fp, B, i, j, (float)acc);
    }
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

// ---- 5b. U = Z (I - E) on the f32 matrix cores --------------------------------------------------
// One wave per 16 rows and every column (ceil(B/16) <= 13 accumulator tiles), K walked in 50
// k-steps of 4 (B <= 200).  The k-steps are ordered so that a lane's two A values of k-steps 2q,
// 2q+1 are one aligned float2 of its Z row (k = 8q + 2g + h, lane group g = l >> 4), and F = I - E
// was written in that order by the eigensolver (Fp, store_fp): each B fragment is 64 consecutive
// floats out of L2.  No LDS, so several waves per SIMD hide the memory latency; Z is read once and
// U written once.  Exact f32 products, fp32 accumulation.
// Accumulator tiles per wave: 16 kApRows rows x NTL x 16 columns (NTL = 13 up to B = 208, 16 up to
// 256), NST = ap_steps(B) k-steps.
constexpr int kApRows = 1;

template <int RT, int NTL = 13, int NST = 50>
__global__ __launch_bounds__(256) void k_svt_apply_f(const float *__restrict__ X, const float *__restrict__ L2,
                                                     float c2, const float *__restrict__ Fp, int64_t P, int B,
                                                     float *__restrict__ U) {
    constexpr int kApTiles = NTL, kApSteps = NST;
    const int lane = threadIdx.x & 63, g = lane >> 4, jl = lane & 15;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (16 * RT);
    if (r0 >= P) return;
    floatx4 acc[RT][kApTiles];
#pragma unroll
    for (int m = 0; m < RT; ++m)
#pragma unroll
        for (int t = 0; t < kApTiles; ++t) acc[m][t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int q = 0; q < kApSteps / 2; ++q) {
        const int k = 8 * q + 2 * g;
        float2 z[RT];
#pragma unroll
        for (int m = 0; m < RT; ++m) {
            const int64_t row = r0 + 16 * m + jl;
            z[m] = make_float2(0.f, 0.f);
            if (row < P && k < B) {
                if ((B & 1) == 0) {   // even B: 8-byte aligned rows, k + 1 < B
                    z[m] = *reinterpret_cast<const float2 *>(&X[row * B + k]);
                    if (L2) {
                        const float2 l = *reinterpret_cast<const float2 *>(&L2[row * B + k]);
                        z[m].x = z[m].x + c2 * l.x;   // X + (1/mu_2)*lambda_2
                        z[m].y = z[m].y + c2 * l.y;
                    }
                } else {
                    z[m].x = X[row * B + k];
                    if (L2) z[m].x = z[m].x + c2 * L2[row * B + k];
                    if (k + 1 < B) {
                        z[m].y = X[row * B + k + 1];
                        if (L2) z[m].y = z[m].y + c2 * L2[row * B + k + 1];
                    }
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float *fb = Fp + (int64_t)(2 * q + h) * B * 4 + g;
#pragma unroll
            for (int t = 0; t < kApTiles; ++t) {
                const int c = 16 * t + jl;
                // rows k >= B of F are never written (the workspace's zeros): skip them explicitly
                const float b = (c < B && k + h < B) ? fb[c * 4] : 0.0f;
#pragma unroll
                for (int m = 0; m < RT; ++m) acc[m][t] = mfma16x16x4(h ? z[m].y : z[m].x, b, acc[m][t]);
            }
        }
    }
    // acc[m][t][i] = U[r0 + 16m + 4g + i][16t + jl]
#pragma unroll
    for (int m = 0; m < RT; ++m)
#pragma unroll
        for (int t = 0; t < kApTiles; ++t) {
            const int c = 16 * t + jl;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t r = r0 + 16 * m + 4 * g + i;
                if (r < P && c < B) U[r * B + c] = acc[m][t][i];
            }
        }
}

}  // namespace lrs

using namespace lrs;

extern "C" size_t lrs_svt_workspace(int64_t P, int64_t B) {
    if (P <= 0 || B <= 0) return 0;
    return svt_ws_bytes(P, B);
}

extern "C" int lrs_svt_gram_offset(int64_t P, int64_t B, int64_t *offset_bytes, int64_t *ld) {
    if (P <= 0 || B <= 0 || !offset_bytes || !ld) return LRS_E_INVALID;
    if (B + (B & 1) > kMaxBp) return LRS_E_UNSUPPORTED;
    const SvtWs w = svt_ws_layout(nullptr, P, B);
    *offset_bytes = (int64_t)((char *)w.G - (char *)nullptr);
    *ld = w.Bp;
    return LRS_OK;
}

// Stage 1 (multi-workgroup): fp64 Gram on the matrix cores and, for a warm Jacobi, A0 = V^T G V.
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
    const int Bp = (int)w.Bp;
    int64_t rows = ((P + kGramSlabs - 1) / kGramSlabs + 3) / 4 * 4;
    const int nslab = (int)((P + rows - 1) / rows);
    const int nt = gram_nt(B);
    if (nt == 13)
        hipLaunchKernelGGL((k_gram_mfma<13, 4>), dim3((unsigned)nslab), dim3(256), 0, st, X, L2, c2, P, (int)B, rows,
                           w.partial);
    else
        hipLaunchKernelGGL((k_gram_mfma<16, 8>), dim3((unsigned)nslab), dim3(512), 0, st, X, L2, c2, P, (int)B, rows,
                           w.partial);
    LRS_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_gram_reduce16, dim3((unsigned)((Bp * Bp + 255) / 256)), dim3(256), 0, st, w.partial, nslab,
                       nt, (int)B, Bp, w.G);
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
    const bool ga = Bp > kLdsMaxBp;   // the packed triangle in the workspace, not in LDS
    const int nb = eig_nb(Bp);
    // LDS of the Jacobi solve: the packed triangle (unless ga) + its rotation tables
    const size_t jaux = sizeof(double) * ((size_t)Bp + 16) + sizeof(int) * (2 * Bp);
    const size_t smem = (ga ? 0 : sizeof(double) * (size_t)Bp * (Bp + 1) / 2) + jaux;
    const size_t vsmem = vrebuild_lds(Bp);
    if (warm & LRS_SVT_JACOBI) {
        const int jwarm = warm & LRS_SVT_WARM;
        // dynamic LDS above 64 KiB must be opted into; request exactly what this shape needs
        const void *kj = ga ? (const void *)k_jacobi_lds<true> : (const void *)k_jacobi_lds<false>;
        hipError_t ea = hipFuncSetAttribute(kj, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (ea != hipSuccess) return (int)ea;
        ea = hipFuncSetAttribute((const void *)k_jacobi_vrebuild, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)vsmem);
        if (ea != hipSuccess) return (int)ea;
        if (ga) hipLaunchKernelGGL(k_jacobi_lds<true>, dim3(1), dim3(kJacobiThreads), smem, st, w, jwarm);
        else hipLaunchKernelGGL(k_jacobi_lds<false>, dim3(1), dim3(kJacobiThreads), smem, st, w, jwarm);
        LRS_CHECK_LAUNCH();
        const int vr = vrebuild_rows(Bp);
        hipLaunchKernelGGL(k_jacobi_vrebuild, dim3((unsigned)((Bp + vr - 1) / vr)), dim3(1024), vsmem, st, w, jwarm);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_svt_finish_state, dim3(1), dim3(1), 0, st, w);
        LRS_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_build_E, dim3((unsigned)((B + 15) / 16), (unsigned)((B + 15) / 16)), dim3(256), 0, st,
                           w, (int)B, tau);
        LRS_CHECK_LAUNCH();
    } else {
        const size_t tsmem = sizeof(double) * ((ga ? 0 : (size_t)Bp * (Bp + 1) / 2) + Bp);
        const size_t esmem = sizeof(double) * 2 * kEKc * eld(nb);
        const size_t lds = std::max(std::max(tsmem, esmem), std::max(smem, vsmem));
        // the instantiations: (NB, GA) = (7, false) up to kLdsMaxBp, (7, true) up to 224, (8, true) above
        const void *keig = nb == 8 ? (const void *)k_svt_eig<8, true>
                                   : ga ? (const void *)k_svt_eig<7, true> : (const void *)k_svt_eig<7, false>;
        const void *kcert = nb == 8 ? (const void *)k_svt_eig_cert<8, true>
                                    : ga ? (const void *)k_svt_eig_cert<7, true> : (const void *)k_svt_eig_cert<7, false>;
        if (warm & LRS_SVT_MULTI_WG) {
            const void *ktri = ga ? (const void *)k_svt_eig_tri<true> : (const void *)k_svt_eig_tri<false>;
            hipError_t ea = hipFuncSetAttribute(ktri, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tsmem);
            if (ea == hipSuccess) ea = hipFuncSetAttribute(kcert, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (ea != hipSuccess) return (int)ea;
            if (ga) hipLaunchKernelGGL(k_svt_eig_tri<true>, dim3(1), dim3(kEigThreads), tsmem, st, w);
            else hipLaunchKernelGGL(k_svt_eig_tri<false>, dim3(1), dim3(kEigThreads), tsmem, st, w);
            LRS_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_svt_eig_vals, dim3((unsigned)((4 * Bp + kEigMwThreads - 1) / kEigMwThreads)),
                               dim3(kEigMwThreads), 0, st, w);
            LRS_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_svt_eig_vecs, dim3((unsigned)((Bp + kEigMwThreads - 1) / kEigMwThreads)),
                               dim3(kEigMwThreads), 0, st, w);
            LRS_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_svt_eig_back, dim3((unsigned)((Bp + 15) / 16)), dim3(256), 0, st, w);
            LRS_CHECK_LAUNCH();
            if (nb == 8) hipLaunchKernelGGL((k_svt_eig_cert<8, true>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau);
            else if (ga) hipLaunchKernelGGL((k_svt_eig_cert<7, true>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau);
            else hipLaunchKernelGGL((k_svt_eig_cert<7, false>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau);
            LRS_CHECK_LAUNCH();
        } else {
            hipError_t ea = hipFuncSetAttribute(keig, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (ea != hipSuccess) return (int)ea;
            if (nb == 8) hipLaunchKernelGGL((k_svt_eig<8, true>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau, 0);
            else if (ga) hipLaunchKernelGGL((k_svt_eig<7, true>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau, 0);
            else hipLaunchKernelGGL((k_svt_eig<7, false>), dim3(1), dim3(kEigThreads), lds, st, w, (int)B, tau, 0);
            LRS_CHECK_LAUNCH();
        }
    }
    if (s_out) {
        hipLaunchKernelGGL(k_sorted_singular_values, dim3(1), dim3(256), 0, st, w, (int)B, s_out);
        LRS_CHECK_LAUNCH();
    }
    const dim3 agrid((unsigned)((P + 64 * kApRows - 1) / (64 * kApRows)));
    if (B <= 200)
        hipLaunchKernelGGL((k_svt_apply_f<kApRows, 13, 50>), agrid, dim3(256), 0, st, X, L2, c2, w.Fp, P, (int)B, U);
    else
        hipLaunchKernelGGL((k_svt_apply_f<kApRows, 16, 64>), agrid, dim3(256), 0, st, X, L2, c2, w.Fp, P, (int)B, U);
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
    if (Bp > kLdsMaxBp) return LRS_E_UNSUPPORTED;   // diagnostics of the LDS-resident chain only
    const size_t smem = std::max(sizeof(double) * ((size_t)Bp * (Bp + 1) / 2 + Bp + 16) + sizeof(int) * (2 * Bp),
                                 sizeof(double) * 2 * kEKc * kELd);
    hipError_t ea = hipFuncSetAttribute((const void *)k_svt_eig<7, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)smem);
    if (ea != hipSuccess) return (int)ea;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL((k_svt_eig<7, false>), dim3(1), dim3(kEigThreads), smem, st, w, (int)B, 1.0, 1);
    LRS_CHECK_LAUNCH();
    // out: d[Bp], e[Bp], lam[Bp], W[Bp*Bp], V[Bp*Bp], S[Bp*Bp]
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    int state[8];
    e = hipMemcpy(state, w.state, sizeof(state), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return (int)e;
    const size_t m = (size_t)Bp * Bp;
    (void)hipMemcpy(out, w.partial, 2 * Bp * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipMemcpy(out + 2 * Bp, w.lam, Bp * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipMemcpy(out + 3 * Bp, w.T, m * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipMemcpy(out + 3 * Bp + m, w.V[state[1]], m * sizeof(double), hipMemcpyDeviceToHost);
    e = hipMemcpy(out + 3 * Bp + 2 * m, w.A0, m * sizeof(double), hipMemcpyDeviceToHost);
    return e != hipSuccess ? (int)e : state[4];
}

// Diagnostics: the SVT apply alone (F = I - E from the last solve in ws).
extern "C" int lrs_diag_svt_apply(const float *X, const float *L2, float c2, int64_t P, int64_t B, void *ws, float *U,
                                  int dbg, void *stream) {
    SvtWs w = svt_ws_layout(ws, P, B);
    hipStream_t st = (hipStream_t)stream;
    if (B > 200) return LRS_E_UNSUPPORTED;   // diagnostics of the B <= 200 apply variants only
    if (dbg == 1)
        hipLaunchKernelGGL(k_svt_apply_f<1>, dim3((unsigned)((P + 63) / 64)), dim3(256), 0, st, X, L2, c2, w.Fp, P,
                           (int)B, U);
    else if (dbg == 2)
        hipLaunchKernelGGL(k_svt_apply_f<2>, dim3((unsigned)((P + 127) / 128)), dim3(256), 0, st, X, L2, c2, w.Fp, P,
                           (int)B, U);
    else
        hipLaunchKernelGGL(k_svt_apply_f<4>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, X, L2, c2, w.Fp, P,
                           (int)B, U);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
