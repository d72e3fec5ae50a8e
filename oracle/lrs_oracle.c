/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Plain-C restatement of the LRS-PnP sparse-coding prox and ADMM update of the reference
 * (shuoli0708/LRS-PnP-DIP), one block / one element at a time, in the reference's order of
 * floating-point operations wherever that order is observable:
 *
 *   oracle_ista_block   ista()            main_LRS_PnP.py:131-149 (alpha = ||H||_2^2, h = 0.1 T)
 *                                         main_LRS_PnP_DIP_1-LiP.py:185-198 (alpha = 4||H||_F^2, h = T)
 *                       + delete_element  main_LRS_PnP.py:152-155 / the pruning at :278-289
 *                       + Phi_z[:,jj] = Full_Dictionary @ Coefs   main_LRS_PnP.py:294,302
 *   oracle_admm_update  col2im + closed-form X + dual updates
 *                                         main_LRS_PnP.py:324-362, main_LRS_PnP_DIP_1-LiP.py:420-448
 *
 * alpha and h are computed by the caller (oracle/oracle.py, numpy, exactly the reference
 * expressions) and passed in, because the reference evaluates them with numpy/LAPACK.
 * The GEMVs accumulate in double and round once to float32 at the points where the reference's
 * torch.mm produces a float32 tensor.  Build with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void oracle_nlm_col(const float *g, long K, long ldg, double h, float *out, long ldo);
void oracle_nlm_matlab_col(const float *g, long K, long ldg, double h, float *out, long ldo);

enum { ORACLE_PROX_NLM = 0, ORACLE_PROX_SOFT = 1, ORACLE_PROX_NLM_MATLAB = 2 };

/*
 * One block of the sparse-coding prox.
 *   y     [n]    block of (X + lambda_1/mu_1), F-ordered (get_image_block, main_LRS_PnP.py:105)
 *   obs   [n]    1 where the observed block (blocks_copy, :244) is non-zero, 0 where pruned (:278)
 *   D     [n*K]  Full_Dictionary, row-major (D[r*K + k])
 *   alpha        ISTA step normaliser (float32, as numpy returns it)
 *   thr          NLM h (prox NLM, NLM_MATLAB) or soft threshold T (prox SOFT)
 *   x     [K]    out: Coefs
 *   phi   [n]    out: Full_Dictionary @ Coefs (may be NULL)
 */
void oracle_ista_block(const float *y, const uint8_t *obs, const float *D, long n, long K,
                       float alpha, double thr, int Nit, int prox, float *x, float *phi) {
    long *rows = (long *)malloc(sizeof(long) * (size_t)n);
    float *r = (float *)malloc(sizeof(float) * (size_t)n);
    float *g = (float *)malloc(sizeof(float) * (size_t)K);
    long m = 0;
    for (long i = 0; i < n; ++i)
        if (obs[i]) rows[m++] = i;
    for (long k = 0; k < K; ++k) x[k] = 0.0f;
    for (int it = 0; it < Nit; ++it) {
        /* r = y - H x      (torch.mm(H, x) -> float32, then the float32 subtraction) */
        for (long a = 0; a < m; ++a) {
            const float *Dr = D + rows[a] * K;
            double acc = 0.0;
            for (long k = 0; k < K; ++k) acc += (double)Dr[k] * (double)x[k];
            r[a] = y[rows[a]] - (float)acc;
        }
        /* g = x + (H^T r) / alpha */
        for (long k = 0; k < K; ++k) {
            double acc = 0.0;
            for (long a = 0; a < m; ++a) acc += (double)D[rows[a] * K + k] * (double)r[a];
            float q = (float)acc / alpha;
            g[k] = x[k] + q;
        }
        if (prox == ORACLE_PROX_SOFT) {
            /* soft(g, T) = sign(g) max(|g| - T, 0): ista.m:23, admm_utils.py:72-75 */
            float T = (float)thr;
            for (long k = 0; k < K; ++k) {
                float t = fabsf(g[k]) - T;
                t = t > 0.0f ? t : 0.0f;
                x[k] = g[k] > 0.0f ? t : (g[k] < 0.0f ? -t : 0.0f);
            }
        } else if (prox == ORACLE_PROX_NLM_MATLAB) {
            /* pnp_ista.m:30 NLmeansfilter(gradient, 3, 3, 0.1*T); thr = 0.1*T */
            oracle_nlm_matlab_col(g, K, 1, thr, x, 1);
        } else {
            oracle_nlm_col(g, K, 1, thr, x, 1);
        }
    }
    if (phi) {
        for (long i = 0; i < n; ++i) {
            double acc = 0.0;
            for (long k = 0; k < K; ++k) acc += (double)D[i * K + k] * (double)x[k];
            phi[i] = (float)acc;
        }
    }
    free(rows); free(r); free(g);
}

/* Batched form over nb blocks laid out [nb][n]; OpenMP over blocks when available. */
void oracle_ista_batch(const float *Y, const uint8_t *OBS, const float *D, long n, long K, long nb,
                       const float *alpha, const double *thr, int Nit, int prox, float *X,
                       float *PHI) {
#pragma omp parallel for schedule(dynamic, 4)
    for (long j = 0; j < nb; ++j)
        oracle_ista_block(Y + j * n, OBS + j * n, D, n, K, alpha[j], thr[j], Nit, prox, X + j * K,
                          PHI ? PHI + j * n : NULL);
}

/*
 * col2im + closed-form X update + dual updates (main_LRS_PnP.py:324-362).
 *   all P x B arrays float32 row-major (row = pixel p, column = band);
 *   PHI [nb][bb*bb] F-ordered blocks, brow/bcol [nb] block corners in reference order.
 * Overlapping blocks are accumulated in block order exactly like the reference loop, so
 * IMout, Weight and lambda1_summation are bit-identical to the reference's.
 * Writes X, lambda_1, lambda_2 in place of Xo, L1, L2 (they may alias the inputs).
 */
void oracle_admm_update(long P, long B, long bb, long nb, const long *brow, const long *bcol,
                        const float *PHI, const float *Y, const float *M, const float *U,
                        const float *L1, const float *L2, float gamma, float mu1, float mu2,
                        float *Xo, float *L1o, float *L2o, float *IMo, float *Wo) {
    const size_t N = (size_t)P * B;
    float *IM = (float *)calloc(N, sizeof(float));
    float *W = (float *)calloc(N, sizeof(float));
    float *LS = (float *)calloc(N, sizeof(float));
    for (long j = 0; j < nb; ++j) {
        const float *blk = PHI + j * bb * bb;
        for (long c = 0; c < bb; ++c)
            for (long a = 0; a < bb; ++a) {
                size_t e = (size_t)(brow[j] + a) * B + (bcol[j] + c);
                IM[e] = IM[e] + blk[a + bb * c];
                W[e] = W[e] + 1.0f;
                LS[e] = LS[e] + L1[e];
            }
    }
    for (size_t e = 0; e < N; ++e) {
        float num = gamma * Y[e];
        num = num + mu1 * IM[e];
        num = num + mu2 * U[e];
        num = num - LS[e];
        num = num - L2[e];
        float den = gamma * M[e];
        den = den + mu1 * W[e];
        den = den + mu2;
        float x = num / den;
        float l1 = L1[e] + mu1 * (x - IM[e]);
        float l2 = L2[e] + mu2 * (x - U[e]);
        Xo[e] = x;
        L1o[e] = l1;
        L2o[e] = l2;
        if (IMo) IMo[e] = IM[e];
        if (Wo) Wo[e] = W[e];
    }
    free(IM); free(W); free(LS);
}

/* get_image_block gather (main_LRS_PnP.py:101-105): out[j][a + bb*c] = X[brow[j]+a][bcol[j]+c]. */
void oracle_im2col(long P, long B, long bb, long nb, const long *brow, const long *bcol,
                   const float *X, float *out) {
    (void)P;
    for (long j = 0; j < nb; ++j)
        for (long c = 0; c < bb; ++c)
            for (long a = 0; a < bb; ++a)
                out[j * bb * bb + a + bb * c] = X[(size_t)(brow[j] + a) * B + bcol[j] + c];
}
