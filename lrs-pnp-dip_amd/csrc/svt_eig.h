// One-workgroup symmetric eigensolver for the SVT low-rank prox (included by svt.hip).
//
// The SVT needs E = f(G) = V diag(f(lambda)) V^T of the B x B fp64 Gram G = Z^T Z with
// f(lambda) = min(tau / sqrt(lambda), 1) (main_LRS_PnP.py:112-124: U = U_s (S - tau)_+ V_h =
// Z - Z E).  The cyclic Jacobi solver needs ~1,200 rounds of two LDS barriers each on one CU
// (5-7 ms at B = 198); this path does the same job in O(B) barriers:
//   A. Householder tridiagonalisation in LDS (packed upper triangle; reflector k stored in row k
//      with v_{k+1} = 1 implicit, beta_k in global memory): 3 LDS barriers per column;
//   B. all eigenvalues of T by 9-way multisection (4 threads x 2 points per eigenvalue,
//      division-free Sturm counts of the characteristic-polynomial sequence, T in registers);
//   C. inverse iteration, one thread per eigenvector (LU with partial pivoting of T - lambda I,
//      two solves), factors and vectors in global scratch laid out [row][vector] (coalesced);
//   E. back-transformation V = H_0 ... H_{n-3} W, one wave per 4 eigenvectors, DPP reductions;
//   D. a certificate on V (k_svt_eig): inverse iteration without reorthogonalisation loses
//      orthogonality inside tight clusters, so S = V^T V is formed, V is repaired by Newton-Schulz
//      (Loewdin) steps V <- V (3I - S)/2 — which only mixes vectors of nearby eigenvalues, so the
//      residuals stay small, and that growth is bounded explicitly — and repeated eigenvalues
//      (S far from I) or large residuals send the workgroup to the Jacobi solve on the same G;
//   F. E = V f V^T (fp64 accumulation, float32 output, symmetric blocks computed once).
// Everything runs in ONE workgroup so the chain gets its CU once and never waits for a CU again
// while the sparse-coding kernel holds the rest of the chip.  The phases are separate
// (non-inlined) functions so each gets its own register allocation.

namespace lrs {

constexpr int kEigThreads = 1024;

// packed upper-triangle index of (i <= j) in an n x n symmetric matrix
__device__ __forceinline__ int pk_idx(int i, int j, int n) { return i * n - ((i * (i - 1)) >> 1) + (j - i); }

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROWMASK, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// 64-bit value of register v in lane l (l uniform)
__device__ __forceinline__ double rl64(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Sum over the 64 lanes, returned in every lane (bitwise the same in every wave for the same data:
// fixed order row_shr 1/2/4/8 scans, then row_bcast 15/31, lane 63 broadcast).
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_f64<0x111>(v);
    v += dpp_f64<0x112>(v);
    v += dpp_f64<0x114>(v);
    v += dpp_f64<0x118>(v);
    v += dpp_f64<0x142, 0xA>(v);
    v += dpp_f64<0x143, 0xC>(v);
    return rl64(v, 63);
}

// element j (uniform) of a wave-distributed vector r[t] = x[lane + 64 t].  readlane reads the
// source lane's register whatever the EXEC mask, so it must be applied to the registers every lane
// loaded (r[t]) and the choice among them made afterwards: a vector select in front of it would
// leave the inactive lanes' values unwritten.
__device__ __forceinline__ double wdist(const double (&r)[4], int j) {
    const int t = j >> 6, l = j & 63;
    const double v0 = rl64(r[0], l), v1 = rl64(r[1], l), v2 = rl64(r[2], l), v3 = rl64(r[3], l);
    return t == 0 ? v0 : t == 1 ? v1 : t == 2 ? v2 : v3;
}

// Workgroup barrier of the chain: LDS-only while the packed A is in LDS (B <= kLdsMaxBp), a full
// one (global stores drained and visible to the workgroup) when A lives in the workspace.
template <bool GA>
__device__ __forceinline__ void eig_bar() {
    if (GA) __syncthreads();
    else lds_barrier();
}

// ---- A. tridiagonalisation: A (packed) -> T on its diagonal / first superdiagonal ---------------
// Per column k: wave 0 forms the reflector; the matvec p = beta A_sub v runs four threads per row
// with eight loads in flight per thread; the rank-2 update runs one wave per row over absolute
// column lanes (v_j, w_j computed once per lane), two rows per batch.  GA: A is in global memory
// (the workspace, L2-resident: B > kLdsMaxBp, whose packed triangle exceeds the 160 KiB of LDS).
template <bool GA>
__device__ __noinline__ void eig_tridiag(double *A, double *pv, double *shb, int n, double *beta_g) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = kEigThreads / 64;
    for (int k = 0; k < n - 2; ++k) {
        const int rk = pk_idx(k, k, n);   // A(k, j) = A[rk + j - k]
        if (wv == 0) {
            double xv[4], sig = 0.0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = k + 2 + lane + 64 * t;
                xv[t] = (j < n) ? A[rk + j - k] : 0.0;
                sig = __fma_rn(xv[t], xv[t], sig);
            }
            sig = wave_sum_dpp(sig);
            const double x0 = A[rk + 1];
            double beta = 0.0, e = x0;
            if (sig > 0.0) {
                // Golub & Van Loan Alg. 5.1.1: H x = mu e_1, v = [1; x(2:m) / v1]
                const double mu = sqrt(__fma_rn(x0, x0, sig));
                const double v1 = (x0 <= 0.0) ? x0 - mu : -sig / (x0 + mu);
                beta = 2.0 * v1 * v1 / (sig + v1 * v1);
                e = mu;
                const double r = 1.0 / v1;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = k + 2 + lane + 64 * t;
                    if (j < n) A[rk + j - k] = xv[t] * r;
                }
            }
            if (lane == 0) {
                A[rk + 1] = e;
                shb[k & 1] = beta;
                beta_g[k] = beta;
            }
        }
        eig_bar<GA>();
        const double beta = shb[k & 1];
        if (beta == 0.0) continue;   // column already reduced (uniform branch)
        // p = beta * A_sub v, four threads per row, quad reduction
        {
            const int i = k + 1 + (tid >> 2), q = tid & 3;
            double acc = 0.0;
            if (i < n) {
                const int ri = pk_idx(i, i, n) - i;   // A(i, j) = A[ri + j], j >= i
                for (int j0 = k + 1 + q; j0 < n; j0 += 32) {
                    double av[8], vv[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int j = j0 + 4 * u;
                        const int jc = (j < n) ? j : n - 1;
                        const int aa = (jc >= i) ? ri + jc : pk_idx(jc, i, n);
                        av[u] = A[aa];
                        vv[u] = A[rk + jc - k];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int j = j0 + 4 * u;
                        const double vj = (j == k + 1) ? 1.0 : vv[u];
                        if (j < n) acc = __fma_rn(av[u], vj, acc);
                    }
                }
            }
            acc += __shfl_xor(acc, 1, 64);
            acc += __shfl_xor(acc, 2, 64);
            if (i < n && q == 0) pv[i] = beta * acc;
        }
        eig_bar<GA>();
        // K = beta/2 p.v (every wave computes the same value), w = p - K v
        double vj[4], wj[4], kp = 0.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = k + 1 + lane + 64 * t;
            const int jc = (j < n) ? j : n - 1;
            const double a = A[rk + jc - k], pj = pv[jc];
            vj[t] = (j < n) ? ((j == k + 1) ? 1.0 : a) : 0.0;
            wj[t] = (j < n) ? pj : 0.0;
            kp = __fma_rn(wj[t], vj[t], kp);
        }
        const double K = 0.5 * beta * wave_sum_dpp(kp);
#pragma unroll
        for (int t = 0; t < 4; ++t) wj[t] = wj[t] - K * vj[t];
        // A_sub -= v w^T + w v^T on the upper triangle: wave per row, lanes over absolute j
        for (int i0 = k + 1 + wv; i0 < n; i0 += 2 * NW) {
            double a[2][4], vi[2], wi[2];
            int ri[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int i = i0 + r * NW;
                const int ic = (i < n) ? i : n - 1;
                ri[r] = pk_idx(ic, ic, n) - ic;
                const double vr = A[rk + ic - k];
                vi[r] = (ic == k + 1) ? 1.0 : vr;
                wi[r] = pv[ic] - K * vi[r];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = k + 1 + lane + 64 * t;
                    a[r][t] = (i < n && j >= i && j < n) ? A[ri[r] + j] : 0.0;
                }
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int i = i0 + r * NW;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int j = k + 1 + lane + 64 * t;
                    if (i < n && j >= i && j < n) A[ri[r] + j] = a[r][t] - (vi[r] * wj[t] + wi[r] * vj[t]);
                }
            }
        }
        eig_bar<GA>();
    }
}

// bisection tolerance for an eigenvalue bracketed by [lo, hi]
__device__ __forceinline__ double eig_tol(double lo, double hi, double tn) {
    return 4.0 * DBL_EPSILON * fmax(fabs(lo), fabs(hi)) + 2.0 * DBL_EPSILON * tn + 1e-300;
}

// one step of the Sturm sequence p_j = (d_j - x) p_{j-1} - e_{j-1}^2 p_{j-2}; an exact zero is
// replaced by -pivmin * p_{j-1} (the LDL^T form's q_j = -pivmin); counts sign changes
__device__ __forceinline__ void sturm_step(double d, double e2, double x, double pivmin, double &p, double &pm,
                                           int &changes) {
    double pn = __fma_rn(d - x, p, -e2 * pm);
    if (pn == 0.0) pn = -pivmin * p;
    changes += (pn < 0.0) != (p < 0.0);
    pm = p;
    p = pn;
}

__device__ __forceinline__ void sturm_rescale(double &p, double &pm) {
    int ex;
    frexp(fmax(fabs(p), fabs(pm)), &ex);
    p = ldexp(p, -ex);
    pm = ldexp(pm, -ex);
}

// ---- B. all eigenvalues, ascending: 9-way multisection, 4 threads x 2 points per eigenvalue ----
// d_j and e_{j-1}^2 live in registers distributed over the lanes of every wave and reach the
// Sturm chains by readlane (no memory access inside the sequence).  The number of sign changes
// of p_0 = 1, p_1(x), ..., p_n(x) is the number of eigenvalues below x.
__device__ __noinline__ void eig_values(const double *A, int n, double gl, double gu, double tn, double pivmin,
                                        double *lamv, double *lam_g, int tid0 = 0) {
    const int tid = tid0 + (int)threadIdx.x, lane = tid & 63;   // tid0: this workgroup's first thread (multi-WG)
    double dr[4], er[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        dr[t] = (j < n) ? A[pk_idx(j, j, n)] : 0.0;
        const double e = (j >= 1 && j < n) ? A[pk_idx(j - 1, j - 1, n) + 1] : 0.0;
        er[t] = e * e;
        // every lane's copy is read by readlane below, including lanes that leave early: keep the
        // loads ahead of the exit (the compiler may otherwise sink them into the active region)
        __asm__ volatile("" ::"v"(dr[t]), "v"(er[t]));
    }
    const int ev = tid >> 2, s = tid & 3;
    if (ev >= n) return;
    double lo = gl, hi = gu;
    for (int it = 0; it < 64; ++it) {
        if (!(hi - lo > eig_tol(lo, hi, tn))) break;   // uniform within the quad
        const double h9 = (hi - lo) * (1.0 / 9.0);
        const double x1 = lo + h9 * (double)(2 * s + 1), x2 = lo + h9 * (double)(2 * s + 2);
        double p1 = 1.0, pm1 = 0.0, p2 = 1.0, pm2 = 0.0;
        int c1 = 0, c2 = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int jn = min(64, n - 64 * t);
#pragma unroll 4
            for (int l = 0; l < jn; ++l) {
                const double d = rl64(dr[t], l), e2 = rl64(er[t], l);
                sturm_step(d, e2, x1, pivmin, p1, pm1, c1);
                sturm_step(d, e2, x2, pivmin, p2, pm2, c2);
                if ((l & 3) == 3) {
                    sturm_rescale(p1, pm1);
                    sturm_rescale(p2, pm2);
                }
            }
        }
        // lambda_ev < x  <=>  more than ev eigenvalues below x
        const unsigned long long m1 = __ballot(c1 > ev), m2 = __ballot(c2 > ev);
        const unsigned b1 = (unsigned)(m1 >> (lane & ~3)) & 0xFu, b2 = (unsigned)(m2 >> (lane & ~3)) & 0xFu;
        unsigned bits = 0;   // bit m-1 <-> point m = 1..8
#pragma unroll
        for (int q = 0; q < 4; ++q) bits |= (((b1 >> q) & 1u) << (2 * q)) | (((b2 >> q) & 1u) << (2 * q + 1));
        if (bits == 0) {
            lo = lo + h9 * 8.0;
        } else {
            const int m = __builtin_ctz(bits) + 1;
            const double nhi = lo + h9 * (double)m;
            lo = m > 1 ? lo + h9 * (double)(m - 1) : lo;
            hi = nhi;
        }
    }
    if (s == 0) {
        const double l = 0.5 * (lo + hi);
        lamv[ev] = l;
        lam_g[ev] = l;
    }
}

// ---- C. inverse iteration, one thread per eigenvector -------------------------------------------
// F: [n][4][n] (1/u0, u1, u2, rhs of row j of the pivoted LU for vector i), W: [n][n] with
// W[j * n + i] = component j of eigenvector i (coalesced across threads).  d_j, e_j by readlane;
// global loads issued kEigUnroll rows ahead.  Returns ||T w_i - lambda_i w_i|| (0 for i >= n).
constexpr int kEigUnroll = 4;
__device__ __noinline__ double eig_vectors(const double *A, const double *lamv, int n, double tn, double *F,
                                           double *W, int tid0 = 0) {
    const int i = tid0 + (int)threadIdx.x, lane = i & 63;
    double dr[4], er[4];   // d_j, e_j = A(j, j+1)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = lane + 64 * t;
        const int idx = (j < n) ? pk_idx(j, j, n) : 0;
        dr[t] = (j < n) ? A[idx] : 0.0;
        er[t] = (j + 1 < n) ? A[idx + 1] : 0.0;
        __asm__ volatile("" ::"v"(dr[t]), "v"(er[t]));   // loaded by every lane (see eig_values)
    }
    if (i >= n) return 0.0;
    const double lam = lamv[i];
    const double small = fmax(DBL_EPSILON * tn, 1e-290);
    auto at = [&](int j, int f) -> double & { return F[((int64_t)j * 4 + f) * n + i]; };
    // deterministic start vector, distinct per i
    auto start = [&](int j) -> double {
        const unsigned h = (unsigned)(j * 2654435761u) ^ (unsigned)(i * 40503u + 17u);
        return 1.0 + (double)(h % 1021u) * (1.0 / 2048.0);
    };
    auto guard = [&](double u) -> double { return fabs(u) < small ? copysign(small, u) : u; };
    double scale = 1.0;
    for (int iter = 0; iter < 2; ++iter) {
        // factor T - lam I = P L U while applying L^{-1} P to the right-hand side
        double a = wdist(dr, 0) - lam, bs = (n > 1) ? wdist(er, 0) : 0.0;
        double rb = iter == 0 ? start(0) : W[i] * scale;
        for (int j0 = 0; j0 < n - 1; j0 += kEigUnroll) {
            double bnv[kEigUnroll];
#pragma unroll
            for (int u = 0; u < kEigUnroll; ++u) {
                const int j = min(j0 + u, n - 2);
                bnv[u] = iter == 0 ? start(j + 1) : W[(int64_t)(j + 1) * n + i] * scale;
            }
#pragma unroll
            for (int u = 0; u < kEigUnroll; ++u) {
                const int j = j0 + u;
                if (j >= n - 1) break;
                const double sub = wdist(er, j);
                const double dn = wdist(dr, j + 1) - lam;
                const double supn = (j + 2 < n) ? wdist(er, j + 1) : 0.0;
                const double bn = bnv[u];
                if (fabs(a) >= fabs(sub)) {
                    const double r0 = 1.0 / guard(a);
                    const double l = sub * r0;
                    at(j, 0) = r0; at(j, 1) = bs; at(j, 2) = 0.0; at(j, 3) = rb;
                    a = dn - l * bs;
                    bs = supn;
                    rb = bn - l * rb;
                } else {
                    const double r0 = 1.0 / sub;
                    const double l = a * r0;
                    at(j, 0) = r0; at(j, 1) = dn; at(j, 2) = supn; at(j, 3) = bn;
                    a = bs - l * dn;
                    bs = -l * supn;
                    rb = rb - l * bn;
                }
            }
        }
        double x1 = rb / guard(a), x2 = 0.0;
        W[(int64_t)(n - 1) * n + i] = x1;
        double nrm = x1 * x1;
        for (int jt = n - 2; jt >= 0; jt -= kEigUnroll) {
            double f[kEigUnroll][4];
#pragma unroll
            for (int u = 0; u < kEigUnroll; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) f[u][c] = at(max(jt - u, 0), c);
#pragma unroll
            for (int u = 0; u < kEigUnroll; ++u) {
                const int j = jt - u;
                if (j < 0) break;
                const double x = (f[u][3] - f[u][1] * x1 - f[u][2] * x2) * f[u][0];
                W[(int64_t)j * n + i] = x;
                nrm = __fma_rn(x, x, nrm);
                x2 = x1;
                x1 = x;
            }
        }
        scale = 1.0 / sqrt(nrm);
    }
    // normalise and measure the residual ||T w - lam w||
    double r2 = 0.0, xm = 0.0, x0 = W[i] * scale;
    for (int j0 = 0; j0 < n; j0 += kEigUnroll) {
        double xv[kEigUnroll];
#pragma unroll
        for (int u = 0; u < kEigUnroll; ++u) xv[u] = W[(int64_t)min(j0 + u + 1, n - 1) * n + i] * scale;
#pragma unroll
        for (int u = 0; u < kEigUnroll; ++u) {
            const int j = j0 + u;
            if (j >= n) break;
            const double ejm = j > 0 ? wdist(er, j - 1) : 0.0;
            const double ej = (j + 1 < n) ? wdist(er, j) : 0.0;
            const double xp = (j + 1 < n) ? xv[u] : 0.0;
            const double r = (wdist(dr, j) - lam) * x0 + ejm * xm + ej * xp;
            r2 = __fma_rn(r, r, r2);
            W[(int64_t)j * n + i] = x0;
            xm = x0;
            x0 = xp;
        }
    }
    return sqrt(r2);
}

// ---- E. V = H_0 H_1 ... H_{n-3} W (V[j * n + c] = component j of eigenvector c) ----------------
// beta_k from LDS (bl), reflector k from row k of the packed A.
__device__ __noinline__ void eig_backtransform(const double *A, const double *bl, int n, const double *W,
                                               double *V, int wave0 = 0, int nwaves = kEigThreads / 64) {
    const int lane = threadIdx.x & 63, wv = wave0 + (int)(threadIdx.x >> 6);   // wave0 / nwaves: multi-WG
    for (int c0 = 4 * wv; c0 < n; c0 += 4 * nwaves) {
        double x[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = lane + 64 * t;
                x[c][t] = (j < n && c0 + c < n) ? W[(int64_t)j * n + c0 + c] : 0.0;
            }
        for (int k = n - 3; k >= 0; --k) {
            const double beta = bl[k];
            if (beta == 0.0) continue;
            const int rk = pk_idx(k, k, n);
            double v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = lane + 64 * t;
                const int jc = (j > k + 1 && j < n) ? j : k + 1;
                const double a = A[rk + jc - k];
                v[t] = (j == k + 1) ? 1.0 : ((j > k + 1 && j < n) ? a : 0.0);
            }
            double s[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                double acc = 0.0;
#pragma unroll
                for (int t = 0; t < 4; ++t) acc = __fma_rn(v[t], x[c][t], acc);
                s[c] = wave_sum_dpp(acc);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const double bsc = beta * s[c];
#pragma unroll
                for (int t = 0; t < 4; ++t) x[c][t] = x[c][t] - bsc * v[t];
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = lane + 64 * t;
                if (j < n && c0 + c < n) V[(int64_t)j * n + c0 + c] = x[c][t];
            }
    }
}

// F = I - E in the layout of the SVT apply kernel's MFMA B fragments: K is walked in k-steps
// st = 2q + h whose lane group g holds k = 8q + 2g + h (so a lane's two A values of a q are one
// aligned float2 of a Z row); Fp[(st * B + c) * 4 + g] = F[k][c].
__device__ __forceinline__ void store_fp(float *Fp, int B, int k, int c, float e) {
    const int q = k >> 3, g = (k >> 1) & 3, h = k & 1, st = 2 * q + h;
    Fp[((int64_t)st * B + c) * 4 + g] = (k == c ? 1.0f : 0.0f) - e;
}

// ---- one-workgroup fp64 products on a 32 x 32 thread grid -------------------------------------
// Operands staged kEKc values of the summation index at a time as [kk][row] images (row stride
// eld(NB) = 32 NB + 1 doubles: the transposed staging stores hit distinct banks).  Thread (ty, tx)
// owns rows ty + 32a and columns tx + 32b of the n x n result (n <= 32 NB: NB = 7 up to 224, 8 up
// to 256; the sums run over k in the same order either way).
constexpr int kEKc = 16;
__host__ __device__ constexpr int eld(int NB) { return 32 * NB + 1; }
constexpr int kELd = eld(7);
__host__ __device__ constexpr int eig_nb(int n) { return n <= 224 ? 7 : 8; }

// stage X(k0 + kk, r) for kk < kEKc, r < LD (zero outside n): KMAJ: X[k * ld + r], else X[r * ld + k]
template <bool KMAJ, int NB = 7>
__device__ __forceinline__ void eig_stage(double *Xs, const double *X, int ld, int n, int k0) {
    constexpr int kELd = eld(NB);
    constexpr int NIT = (kEKc * kELd + kEigThreads - 1) / kEigThreads;
    double v[NIT];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
        const int idx = threadIdx.x + u * kEigThreads;
        int kk, r;
        if (KMAJ) { kk = idx / kELd; r = idx % kELd; }
        else { r = idx / kEKc; kk = idx % kEKc; }
        const int k = k0 + kk;
        const bool ok = idx < kEKc * kELd && k < n && r < n;
        v[u] = ok ? (KMAJ ? X[(int64_t)k * ld + r] : X[(int64_t)r * ld + k]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
        const int idx = threadIdx.x + u * kEigThreads;
        int kk, r;
        if (KMAJ) { kk = idx / kELd; r = idx % kELd; }
        else { r = idx / kEKc; kk = idx % kEKc; }
        if (idx < kEKc * kELd) Xs[kk * kELd + r] = v[u];
    }
}

// Symmetric product C = X^T diag(f) X over the summation index k (X(k, r) as eig_stage<KMAJ>),
// blocks a <= b only.  MODE 0: f_k = min(tau / sqrt(lam_k), 1), C -> E (float, B x B);
// MODE 1: f = 1, C -> S (double, n x n) and the return value is max |S - I| (uniform).
template <bool KMAJ, int MODE, int NB = 7>
__device__ __noinline__ double eig_syrk(double *sm, const double *X, int n, const double *lam, double tau, int B,
                                        float *E, double *S, double *red, float *Fp = nullptr) {
    constexpr int kELd = eld(NB);
    double *Xs = sm;                   // [kEKc][kELd]
    double *Xf = sm + kEKc * kELd;     // [kEKc][kELd]  X * f  (MODE 0)
    const int tid = threadIdx.x, ty = tid >> 5, tx = tid & 31;
    double acc[NB][NB];
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[a][b] = 0.0;
    for (int k0 = 0; k0 < n; k0 += kEKc) {
        __syncthreads();
        eig_stage<KMAJ, NB>(Xs, X, n, n, k0);
        if (MODE == 0) {
            __syncthreads();
            for (int idx = tid; idx < kEKc * kELd; idx += kEigThreads) {
                const int k = k0 + idx / kELd;
                double f = 0.0;
                if (k < n) {
                    const double l = lam[k];
                    const double sv = l > 0.0 ? sqrt(l) : 0.0;
                    f = (sv > tau) ? tau / sv : 1.0;
                }
                Xf[idx] = Xs[idx] * f;
            }
        }
        __syncthreads();
        const double *Xl = MODE == 0 ? Xf : Xs;
        const int kn = min(kEKc, n - k0);
#pragma unroll 2
        for (int kk = 0; kk < kn; ++kk) {
            double vj[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) vj[b] = Xs[kk * kELd + tx + 32 * b];
#pragma unroll
            for (int a = 0; a < NB; ++a) {
                const double vi = Xl[kk * kELd + ty + 32 * a];
#pragma unroll
                for (int b = a; b < NB; ++b) acc[a][b] = __fma_rn(vi, vj[b], acc[a][b]);
            }
        }
    }
    // block (a, b), a <= b: the (b, a) block takes the transposed sums; diagonal blocks are written
    // by the thread with tx >= ty, so C is bitwise symmetric.
    double dmax = 0.0;
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
        for (int b = a; b < NB; ++b) {
            const int i = ty + 32 * a, j = tx + 32 * b;
            const int lim = MODE == 0 ? B : n;
            if (i < lim && j < lim && (a != b || tx >= ty)) {
                if (MODE == 0) {
                    const float e = (float)acc[a][b];
                    E[(int64_t)i * B + j] = e;
                    E[(int64_t)j * B + i] = e;
                    store_fp(Fp, B, i, j, e);
                    store_fp(Fp, B, j, i, e);
                } else {
                    S[(int64_t)i * n + j] = acc[a][b];
                    S[(int64_t)j * n + i] = acc[a][b];
                    dmax = fmax(dmax, fabs(acc[a][b] - (i == j ? 1.0 : 0.0)));
                }
            }
        }
    if (MODE == 0) return 0.0;
    // workgroup max
    for (int off = 32; off > 0; off >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, off, 64));
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = dmax;
    __syncthreads();
    double m = 0.0;
    for (int q = 0; q < kEigThreads / 64; ++q) m = fmax(m, red[q]);
    __syncthreads();
    return m;
}

// One Newton-Schulz (Loewdin) orthogonalisation step Vn = 1.5 V - 0.5 V S with S = V^T V
// (V[r * n + c], S symmetric).  Two passes over the row blocks keep the accumulators at 4 NB.
template <int NB = 7>
__device__ __noinline__ void eig_ns_step(double *sm, const double *V, const double *S, int n, double *Vn) {
    constexpr int kELd = eld(NB);
    double *As = sm;                   // [kEKc][kELd]  V(r, j) for the chunk of j
    double *Bs = sm + kEKc * kELd;     // [kEKc][kELd]  S(j, c)
    const int tid = threadIdx.x, ty = tid >> 5, tx = tid & 31;
    for (int half = 0; half < 2; ++half) {
        const int a0 = half * 4, na = half == 0 ? 4 : NB - 4;
        double acc[4][NB];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b) acc[a][b] = 0.0;
        for (int k0 = 0; k0 < n; k0 += kEKc) {
            __syncthreads();
            eig_stage<false, NB>(As, V, n, n, k0);
            eig_stage<true, NB>(Bs, S, n, n, k0);
            __syncthreads();
            const int kn = min(kEKc, n - k0);
#pragma unroll 2
            for (int kk = 0; kk < kn; ++kk) {
                double vj[NB];
#pragma unroll
                for (int b = 0; b < NB; ++b) vj[b] = Bs[kk * kELd + tx + 32 * b];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const double vi = (a < na) ? As[kk * kELd + ty + 32 * (a0 + a)] : 0.0;
#pragma unroll
                    for (int b = 0; b < NB; ++b) acc[a][b] = __fma_rn(vi, vj[b], acc[a][b]);
                }
            }
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int r = ty + 32 * (a0 + a), c = tx + 32 * b;
                if (a < na && r < n && c < n) {
                    const int64_t o = (int64_t)r * n + c;
                    Vn[o] = 1.5 * V[o] - 0.5 * acc[a][b];
                }
            }
    }
    __syncthreads();
}

}  // namespace lrs
