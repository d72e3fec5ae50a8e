/*
 * liblrspnp_hip.so — C ABI of the MI355X-native LRS-PnP inner loop (gfx950 / CDNA4).
 *
 * Plain C: pointers, sizes, a `void *stream` (a hipStream_t, NULL = default stream).  Every
 * device pointer is caller-owned; the library never allocates (workspaces are sized by the
 * `*_workspace` queries and passed in).  Calls are stream-ordered and reentrant, never
 * synchronise the host, and return 0 (LRS_OK), a negative LRS_E_* code, or a positive
 * hipError_t.  Arrays are float32 row-major unless noted.
 *
 * Reference interfaces replaced (shuoli0708/LRS-PnP-DIP; file:line):
 *   lrs_nlm_col_f32       skimage.restoration.denoise_nl_means(g, h, fast_mode=True,
 *                         patch_size=3, patch_distance=3) as called at
 *                         main_LRS_PnP_DIP_1-LiP.py:196, main_LRS_PnP.py:146
 *   lrs_block_count/_grid get_image_block corner logic            main_LRS_PnP.py:73-99
 *   lrs_im2col_f32        get_image_block gather of X + lambda_1/mu_1, plus the missing-pixel
 *                         masks of blocks_copy                     main_LRS_PnP.py:101-105,244,259,278
 *   lrs_ista_alpha_f32    alpha / T / h inside ista()              main_LRS_PnP.py:134-146,
 *                                                                  main_LRS_PnP_DIP_1-LiP.py:187-196
 *   lrs_ista_f32          the per-block loop: delete_element + ista + Phi_z = D @ Coefs,
 *                         for all blocks at once               main_LRS_PnP.py:270-303,131-155
 *   lrs_svt_f32           SVT(X + lambda_2/mu_2, 1/mu_2)          main_LRS_PnP.py:112-124,315
 *   lrs_admm_update_f32   col2im, closed-form X update, dual updates, state_convergence norms
 *                                                                  main_LRS_PnP.py:324-366,23-25
 */
#ifndef LRSPNP_H
#define LRSPNP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LRS_OK 0
#define LRS_E_INVALID (-1)     /* bad argument (shape, null pointer, unsupported parameter) */
#define LRS_E_UNSUPPORTED (-2) /* parameter combination not compiled in (e.g. K) */
#define LRS_E_WORKSPACE (-3)   /* workspace too small */
#define LRS_E_NODEVICE (-4)    /* no gfx950 device */

/* ISTA step-size rule (alpha) and prox */
#define LRS_ALPHA_SPEC2 0 /* alpha = ||H||_2^2, NLM h = 0.1*T   main_LRS_PnP.py:134,146      */
#define LRS_ALPHA_FRO4 1  /* alpha = 4||H||_F^2, NLM h = T      …1-LiP.py:187,196           */
#define LRS_ALPHA_SOFT 2  /* alpha = ||H||_2^2, soft threshold T (ista.m:15-23)              */
#define LRS_PROX_NLM 0
#define LRS_PROX_SOFT 1

const char *lrs_version(void);
/* 0 when the current device is gfx950, LRS_E_NODEVICE otherwise. */
int lrs_check_device(void);

/* ---- NLM prox ------------------------------------------------------------------------------
 * out[v*ldo + i] = NLM(g[v*ldg + 0..K-1])[i] for v < nvec.  h_per_vec (device, nvec doubles)
 * overrides h when non-NULL.  Only patch_size = 3, patch_distance = 3 (the reference's call). */
int lrs_nlm_col_f32(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K, int64_t nvec,
                    double h, const double *h_per_vec, int patch_size, int patch_distance,
                    void *stream);

/* ---- Block grid (host-side) ----------------------------------------------------------------
 * Block corners of get_image_block on a P x B unfolded matrix, in the reference's order
 * (column-major over corners).  rows/cols are host arrays of length lrs_block_count(). */
int64_t lrs_block_count(int64_t P, int64_t B, int64_t bb, int64_t sliding);
int lrs_block_grid(int64_t P, int64_t B, int64_t bb, int64_t sliding, int32_t *rows, int32_t *cols,
                   int64_t nb);
/* For every index x in [0, extent): the contiguous range [lo[x], hi[x]] of positions in the
 * sorted `starts` whose bb-window covers x (hi < lo when none).  Host arrays. */
int lrs_cover_ranges(int64_t extent, int64_t bb, const int32_t *starts, int64_t nstarts,
                     int32_t *lo, int32_t *hi);

/* ---- im2col --------------------------------------------------------------------------------
 * Yb[j*n_pad + a + bb*c] = X[rows[j]+a][cols[j]+c] + L[..]/mu   (L may be NULL: X alone);
 * entries n..n_pad-1 are 0.  obs (nullable, u8 [nb][n_pad]) = 1 where that value != 0.
 * rows/cols are DEVICE int32 arrays. */
int lrs_im2col_f32(const float *X, const float *L, float mu, int64_t P, int64_t B, int64_t bb,
                   const int32_t *rows, const int32_t *cols, int64_t nb, int64_t n_pad, float *Yb,
                   uint8_t *obs, void *stream);

/* ---- ISTA step size / threshold per observation pattern ------------------------------------
 * obs_pat: u8 [npat][n_pad] (1 = observed row).  D: n x K.  Writes alpha_pat[npat] (float32,
 * as numpy returns it) and thr_pat[npat] (the NLM h, or the soft threshold T).
 * SPEC2/SOFT run a fp64 Lanczos on the masked Gram in `ws`. */
size_t lrs_ista_alpha_workspace(int64_t n, int64_t K, int64_t npat);
int lrs_ista_alpha_f32(const float *D, int64_t n, int64_t K, const uint8_t *obs_pat, int64_t npat,
                       int64_t n_pad, int alpha_mode, float lambda_ista, float *alpha_pat,
                       double *thr_pat, void *ws, size_t ws_bytes, void *stream);

/* ---- Masked ISTA with PnP prox over all blocks (the hot kernel) ----------------------------
 * Yb, obs: [nb][n_pad]; D: n x K; alpha[nb], thr[nb].  x0 = 0; Nit iterations of
 *   g = x + D^T(obs .* (y - D x)) / alpha ;  x = prox(g)
 * then phi[j*n_pad + r] = (D x_j)[r] for r < n (all rows, the inpainting step).
 * coefs (nullable) receives x [nb][K].  Supported: K = 256, n_pad % 16 == 0. */
int lrs_ista_f32(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad,
                 int64_t K, int64_t nb, const float *alpha, const double *thr, int Nit, int prox,
                 float *coefs, float *phi, void *stream);

/* ---- SVT low-rank prox ---------------------------------------------------------------------
 * U = SVT(Z, tau) with Z = X + c2 * L2 (c2 = float(1/mu_2); L2 may be NULL), via an fp64 Gram
 * Z^T Z, a one-workgroup Jacobi eigensolver (warm-started from the previous call's eigenvectors
 * kept in ws when warm != 0) and U = Z * V diag(max(1 - tau/s, 0)) V^T.  s_out (nullable,
 * device, B doubles) receives the singular values (descending). */
size_t lrs_svt_workspace(int64_t P, int64_t B);
int lrs_svt_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau,
                float *U, double *s_out, int warm, void *ws, size_t ws_bytes, void *stream);
/* The same call split in two stream-ordered halves so the caller can start the sparse-coding
 * kernel between them: _gram (multi-workgroup Gram + warm-start products, ~0.3 ms) and _finish
 * (one-workgroup eigensolver + V update + U, which then runs beside the sparse coding). */
int lrs_svt_gram_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, int warm,
                     void *ws, size_t ws_bytes, void *stream);
int lrs_svt_finish_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau,
                       float *U, double *s_out, int warm, void *ws, size_t ws_bytes, void *stream);

/* ---- col2im + closed-form X update + dual updates ------------------------------------------
 * IMout = sum over covering blocks (block order) of phi, Weight = count, lambda1_sum = repeated
 * sum of lambda_1, then (float32, the reference's operation order)
 *   X  = (g*Y + mu1*IMout + mu2*U - lambda1_sum - L2) / (g*M + mu1*Weight + mu2)
 *   L1 = L1 + mu1*(X - IMout);   L2 = L2 + mu2*(X - U)
 * X, L1, L2 updated in place.  rlo/rhi [P], clo/chi [B]: device cover ranges over the sorted
 * block-row / block-column starts (lrs_cover_ranges); nbr = number of block rows.
 * norms (nullable, device, 3 doubles, zeroed by the call) += ||dX||^2, ||dL1||^2, ||dL2||^2.
 * imout (nullable) receives IMout. */
int lrs_admm_update_f32(float *X, float *L1, float *L2, const float *Y, const float *M,
                        const float *U, const float *phi, int64_t P, int64_t B, int64_t bb,
                        int64_t n_pad, const int32_t *row_starts, const int32_t *col_starts,
                        int64_t nbr, const int32_t *rlo, const int32_t *rhi, const int32_t *clo,
                        const int32_t *chi, float gamma, float mu1, float mu2, double *norms,
                        float *imout, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LRSPNP_H */
