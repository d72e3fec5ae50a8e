/*
 * liblrspnp_hip.so — C ABI of the MI355X-native LRS-PnP inner loop (gfx950 / CDNA4).
 *
 * Plain C: pointers, sizes, a `void *stream` (a hipStream_t, NULL = default stream).  Every
 * device pointer is caller-owned; the library never allocates (workspaces are sized by the
 * `*_workspace` queries and passed in).  Calls are stream-ordered and reentrant, never
 * synchronise the host, and return 0 (LRS_OK), a negative LRS_E_* code, or a positive
 * hipError_t.  Arrays are float32 row-major unless noted.  Modes are per call (lrs_ista_opts,
 * lrs_dip_opts) or per handle; no exported function changes process-wide state.
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
#define LRS_PROX_NLM_MATLAB 2 /* NLmeansfilter(g,3,3,0.1T) of pnp_ista.m:30, fp64        */

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
 * coefs (nullable) receives x [nb][K].  Any n (n_pad % 16 == 0), any K <= 16384 (K > 512 on the
 * generic dense-GEMM path, see lrs_ista_opts), every prox.
 * n_pad <= 64 with K = 256 runs the dictionary-resident kernels (ws unused); everything else runs
 * the row-split kernel, whose fragment-ordered dictionary images live in `ws`
 * (lrs_ista_workspace bytes; LRS_E_WORKSPACE when too small).
 * Replaces the per-block loop of main_LRS_PnP.py:270-303 / main_LRS_PnP_DIP_1-LiP.py:367-392
 * around ista() (main_LRS_PnP.py:131-149, …1-LiP.py:185-198) and delete_element (:201-204). */
/* Per-call options (NULL = defaults); the library keeps no process-wide mode.
 *   precision: arithmetic of the two products of the resident (n_pad <= 64) kernel:
 *     LRS_ISTA_SPLIT_BF16 (default): bf16 matrix cores on operands split exactly into three bf16
 *     terms (six partial products, fp32 accumulation: fp32-GEMM accuracy, not bitwise the f32
 *     MFMA); LRS_ISTA_F32: v_mfma_f32_16x16x4_f32 (exact f32 products).  The NLM prox is identical.
 *   max_workgroups: 0 (default) = one workgroup per 16-block tile; > 0 bounds the row-split
 *     kernel's grid (each workgroup then loops over tiles), so a concurrent launch on another
 *     stream (the DIP training of the …_DIP mains) keeps the rest of the CUs.  Results do not
 *     depend on it. */
#define LRS_ISTA_F32 0
#define LRS_ISTA_SPLIT_BF16 1
#define LRS_ISTA_ALGO_AUTO 0
#define LRS_ISTA_ALGO_GENERIC 1
typedef struct {
    int32_t precision;
    int32_t max_workgroups;
    int32_t algorithm;    /* LRS_ISTA_ALGO_AUTO: the fused kernels for K <= 512, the generic path above;
                             LRS_ISTA_ALGO_GENERIC: every inner iteration as two dense fp32-accurate
                             GEMMs + the prox kernel, chunks of 4096 blocks (any K <= 16384) */
    int32_t warm_start;   /* 1: start from x0 = coefs (on input) instead of 0 and write the result back to
                             coefs, so Nit iterations split over several calls give exactly the
                             iterates of one call (the time-sliced sparse coding beside the DIP, see
                             DESIGN.md §5).  Row-split kernel only (n_pad > 64 or K != 256):
                             LRS_E_UNSUPPORTED elsewhere or without coefs. */
    int32_t reserved[4];
} lrs_ista_opts;
size_t lrs_ista_workspace(int64_t n, int64_t K, int prox, const lrs_ista_opts *opts);
int lrs_ista_f32(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad,
                 int64_t K, int64_t nb, const float *alpha, const double *thr, int Nit, int prox,
                 float *coefs, float *phi, const lrs_ista_opts *opts, void *ws, size_t ws_bytes,
                 void *stream);
/* ---- Masked ISTA on per-pattern Grams --------------------------------------------------------
 * The same sparse coding as lrs_ista_f32 for blocks that share observation patterns.  ista()'s
 * gradient H^T (y - H x) (main_LRS_PnP.py:131-149, …1-LiP.py:185-198, H = D pruned to the observed
 * rows by delete_element :201-204) is expanded as b - Q_p x with Q_p = D^T diag(obs_pat[p]) D
 * (fp64 sums of exact products, rounded to float32; formed once per call and pattern) and
 * b = D^T (obs .* y) (once per block), so an inner iteration costs 2 K^2 instead of 4 n K FLOP per
 * block.  Products on f32 matrix cores, the prox and the quotient as lrs_ista_f32: the results
 * differ from it by rounding only.  K <= 512, any n (n_pad % 16 == 0), every prox; opts as
 * lrs_ista_f32 (max_workgroups bounds the grid over tiles, warm_start continues from coefs;
 * algorithm must be AUTO).
 *   lrs_ista_pat_plan (host): groups the blocks by pattern.  pat: host int32 [nb], block j's row of
 *     obs_pat (as lrs_ista_alpha_f32's patterns); plan: host int32 [cap >= lrs_ista_pat_plan_len]
 *     = the blocks ordered by pattern (ascending within one), then per tile {first position,
 *     pattern * 32 + count (1..16)}.  Returns the tile count (< 0: error).  Upload it as is.
 *   lrs_ista_pat_preferred (host): 1 when this path does less matrix-core work than lrs_ista_f32's
 *     row-split kernel for these sizes (few patterns, n > K / 2).
 *   lrs_ista_pat_prepare: forms the dictionary images and every pattern's Q_p in ws
 *     (lrs_ista_pat_workspace bytes), once per D and set of patterns (both fixed for a solve);
 *     obs_pat DEVICE u8 [npat][n_pad].
 *   lrs_ista_pat_f32: the sparse coding on the images ws holds (prepare first, again whenever D or
 *     obs_pat change); plan DEVICE int32 (lrs_ista_pat_plan's); Yb [nb][n_pad], alpha/thr [nb] per
 *     block. */
int64_t lrs_ista_pat_plan_len(int64_t nb, int64_t npat);
int64_t lrs_ista_pat_plan(const int32_t *pat, int64_t nb, int64_t npat, int32_t *plan, int64_t cap);
int lrs_ista_pat_preferred(int64_t n, int64_t K, int64_t nb, int64_t npat, int Nit);
size_t lrs_ista_pat_workspace(int64_t n, int64_t K, int64_t npat);
int lrs_ista_pat_prepare(const float *D, int64_t n, int64_t K, const uint8_t *obs_pat, int64_t npat,
                         int64_t n_pad, void *ws, size_t ws_bytes, void *stream);
int lrs_ista_pat_f32(const float *Yb, const uint8_t *obs_pat, int64_t npat, const int32_t *plan,
                     int64_t ntiles, int64_t n, int64_t n_pad, int64_t K, int64_t nb,
                     const float *alpha, const double *thr, int Nit, int prox, float *coefs, float *phi,
                     const lrs_ista_opts *opts, void *ws, size_t ws_bytes, void *stream);
/* NLmeansfilter(g, 3, 3, h) (LRS-PnP(Matlab Code)/NLmeansfilter.m:18-78, the prox of
 * pnp_ista.m:30) of nvec columns of length K, fp64, 'symmetric' padding. */
int lrs_nlm_matlab_col_f32(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K,
                           int64_t nvec, double h, const double *h_per_vec, void *stream);
/* Options of the DIP engine and the conv primitives (NULL = defaults), fixed per call or, for a
 * lrs_dipnet, at creation -- the library keeps no process-wide mode:
 *   precision: arithmetic of the conv GEMMs.  LRS_DIP_SPLIT_BF16 (default): bf16 matrix cores on
 *     operands split into three bf16 terms, six partial products, fp32 accumulation (fp32-GEMM
 *     accuracy); LRS_DIP_F32: v_mfma_f32_16x16x4_f32 (the explicit-im2col kernels; a lrs_dipnet
 *     created with it runs every conv on them).
 *   upsample_dgrad: data gradient of an upsampled stride-1 conv (nearest x2, then 2x2 unpadded or
 *     3x3 pad 1): 0 (default) = correlation over the padded upsampled domain + fold; 1 = a stride-2
 *     conv with the (k+1)x(k+1) effective kernel on the source grid (2.25x fewer products) +
 *     reflection border terms.  lrs_conv2d_workspace must be queried with the same options. */
#define LRS_DIP_F32 0
#define LRS_DIP_SPLIT_BF16 1
typedef struct {
    int32_t precision;
    int32_t upsample_dgrad;
    int32_t reserved[6];
} lrs_dip_opts;

/* ---- SVT low-rank prox ---------------------------------------------------------------------
 * U = SVT(Z, tau) with Z = X + c2 * L2 (c2 = float(1/mu_2); L2 may be NULL), via an fp64 Gram
 * Z^T Z, a one-workgroup symmetric eigensolver and U = Z * V diag(max(1 - tau/s, 0)) V^T.
 * `warm` is a flag word:
 *   default (0): Householder tridiagonalisation + multisection + inverse iteration with a
 *     Davis-Kahan orthogonality certificate, falling back (inside the same workgroup) to the
 *     Jacobi solve when the certificate fails (clustered / repeated eigenvalues);
 *   LRS_SVT_JACOBI: the cyclic Jacobi solver only, warm-started from the previous call's
 *     eigenvectors kept in ws when LRS_SVT_WARM is also set;
 *   LRS_SVT_MULTI_WG (default path only): the same solver with its eigenvalue, inverse-iteration
 *     and back-transformation phases spread over many workgroups (bit-identical result); for a
 *     caller whose eigensolver is on the critical path (a row-slab shard), not beside a
 *     chip-filling sparse-coding kernel.
 * s_out (nullable, device, B doubles) receives the singular values (descending).  B <= 256: up to
 * 198 bands the eigensolver holds the packed fp64 Gram in its CU's LDS, above it (the 224-band
 * cubes) the same one-workgroup chain works on the packed Gram in ws (L2-resident);
 * LRS_E_UNSUPPORTED above 256 (main_LRS_PnP.py:112-124's np.linalg.svd takes any B). */
#define LRS_SVT_WARM 1
#define LRS_SVT_JACOBI 2
#define LRS_SVT_MULTI_WG 4
size_t lrs_svt_workspace(int64_t P, int64_t B);
int lrs_svt_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau,
                float *U, double *s_out, int warm, void *ws, size_t ws_bytes, void *stream);
/* The same call split in two stream-ordered halves so the caller can start the sparse-coding
 * kernel between them: _gram (multi-workgroup Gram, plus the warm-start products for
 * LRS_SVT_JACOBI | LRS_SVT_WARM) and _finish (the one-workgroup eigensolver, then U), which then
 * runs beside the sparse coding. */
int lrs_svt_gram_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, int warm,
                     void *ws, size_t ws_bytes, void *stream);
int lrs_svt_finish_f32(const float *X, const float *L2, float c2, int64_t P, int64_t B, double tau,
                       float *U, double *s_out, int warm, void *ws, size_t ws_bytes, void *stream);
/* Byte offset and leading dimension (Bp = B rounded up to even) of the fp64 Gram (X + c2 L2)^T
 * (X + c2 L2) that lrs_svt_gram_f32 leaves in ws. A caller that holds one row slab of the
 * unfolded cube per rank sums the slabs' Grams in place (all-reduce of Bp*Bp doubles) between
 * _gram and _finish: the Gram is additive over pixel rows (single cube on
 * several GPUs). Not valid with LRS_SVT_JACOBI | LRS_SVT_WARM (its warm-start products are
 * formed from the local Gram inside _gram). Host-only, no device access. */
int lrs_svt_gram_offset(int64_t P, int64_t B, int64_t *offset_bytes, int64_t *ld);

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

/* ==== DIP low-rank prox (the 1-Lipschitz U-Net of main_LRS_PnP_DIP_1-LiP.py) ================
 * Activations are [C][H][W] float32 (batch 1).  Reference interfaces replaced:
 *   lrs_conv2d_*        ReflectionPad2d + Conv2d + nn.Upsample(x2, nearest)
 *                       (models/lipschitz_constraint_layer.py:65-78, my_Lipschitz_Unet.py:71-94)
 *   lrs_bn_act_*        BatchNormSpectralNorm-wrapped BatchNorm2d (train mode) + LeakyReLU(0.2)
 *                       (lipschitz_constraint_layer.py:88-122,154-159, 6-22)
 *   lrs_sigma_max_f32   SpectralNorm._update_u_v: torch.svd(W.view(Co,-1))[0]  (:36-44)
 *   lrs_adam_f32        torch.optim.Adam(lr) step                      (…1-LiP.py:215,237)
 *   lrs_masked_mse_f32  MSELoss(target*mask, out*mask) + its gradient  (…1-LiP.py:216,234)
 *   lrs_es_*            EarlyStop / myMetric variance test             (…1-LiP.py:71-103,244-264)
 *   lrs_dipnet_*        my_Lipschitz_Unet + the get_DIP_out training loop (…1-LiP.py:208-264) */
#define LRS_PAD_ZERO 0
#define LRS_PAD_REFLECT 1
#define LRS_ACT_NONE 0
#define LRS_ACT_LRELU 1   /* LeakyReLU(0.2) */
#define LRS_ACT_SIGMOID 2

/* Output size of the conv unit (upsample, pad, k, stride). */
int lrs_conv2d_out_size(int H, int W, int k, int stride, int pad, int upsample, int *Ho, int *Wo);
/* col workspace (floats) for lrs_conv2d_fwd_f32: Cin*k*k*Ho*Wo (0 when the unit is a plain 1x1). */
int64_t lrs_conv2d_col_size(int Cin, int H, int W, int k, int stride, int pad, int upsample);
/* y[Cout][Ho][Wo] = conv(pad(upsample(x))) + bias.  col receives the im2col matrix (kept for
 * the backward); col == NULL (k <= 3): implicit GEMM, the im2col is gathered inside the
 * split-bf16 kernel and never stored (backward: lrs_conv2d_bwd_x_f32).
 * ws/ws_bytes: split-K partials (lrs_conv2d_workspace). */
size_t lrs_conv2d_workspace(int Cin, int H, int W, int Cout, int k, int stride, int pad, int upsample,
                            const lrs_dip_opts *opts);
int lrs_conv2d_fwd_f32(const float *x, int Cin, int H, int W, const float *w, const float *bias,
                       int Cout, int k, int stride, int pad, int pad_mode, int upsample, float *col,
                       float *y, const lrs_dip_opts *opts, void *ws, size_t ws_bytes, void *stream);
/* gw = (gy col^T) / *w_div (w_div nullable, device scalar: the spectral-norm scale);
 * gx (nullable) = adjoint of the im2col of gy through w.  gbias is produced by lrs_bn_act_bwd.
 * col = the forward's col (or x itself for a plain 1x1 unit). */
int lrs_conv2d_bwd_f32(const float *gy, const float *col, const float *w, const float *w_div, int Cin,
                       int H, int W, int Cout, int k, int stride, int pad, int pad_mode, int upsample,
                       float *gx, float *gw, const lrs_dip_opts *opts, void *ws, size_t ws_bytes,
                       void *stream);
/* The same from the conv input x (k <= 3): gw's col^T is gathered inside the GEMM. */
int lrs_conv2d_bwd_x_f32(const float *gy, const float *x, const float *w, const float *w_div, int Cin,
                         int H, int W, int Cout, int k, int stride, int pad, int pad_mode, int upsample,
                         float *gx, float *gw, const lrs_dip_opts *opts, void *ws, size_t ws_bytes,
                         void *stream);

/* y = act(BN_lip(z)) with batch statistics (gamma == NULL: y = act(z)).  Saves mean / invstd
 * [C]; running stats (nullable) get the momentum update.  ws: lrs_bn_act_workspace bytes,
 * zero-filled before its first use (it is left zeroed for the next call). */
size_t lrs_bn_act_workspace(int C, int64_t P);
int lrs_bn_act_fwd_f32(const float *z, float *y, const float *gamma, const float *beta, float *mean,
                       float *invstd, float *run_mean, float *run_var, int C, int64_t P, int act,
                       float eps, float momentum, void *ws, size_t ws_bytes, void *stream);
int lrs_bn_act_bwd_f32(const float *gy, const float *y, const float *z, const float *gamma,
                       const float *mean, const float *invstd, float *gz, float *ggamma,
                       float *gbeta, float *gbias, int C, int64_t P, int act, void *ws, size_t ws_bytes,
                       void *stream);
/* Conv -> BatchNorm(train) -> act in one launch on a small map (the network engine's forward for the
 * <= 9^2 maps): z = conv(reflect_pad(x)) + bias (bias nullable), y = act(BN_lip(z)), mean / invstd
 * [Cout] saved, running stats (nullable, both or neither) momentum-updated (eps 1e-5, momentum 0.1);
 * lip = 1: BatchNormSpectralNorm's gamma / c, beta / c.  Replaces a Conv2d + BatchNorm2d +
 * LeakyReLU block (lipschitz_constraint_layer.py:65-78,88-101, models/common.py:71-121).
 * LRS_E_UNSUPPORTED where the one-launch kernel does not take the geometry (zero padding, upsample,
 * a source under 2 x 2, > 1024 output pixels, more than two staged input chunks). */
int lrs_conv_bn_small_f32(const float *x, int Cin, int H, int W, const float *w, const float *bias, int Cout,
                          int k, int stride, int pad, int pad_mode, int upsample, const float *gamma,
                          const float *beta, int lip, int act, float *z, float *y, float *mean, float *invstd,
                          float *run_mean, float *run_var, void *stream);

/* sigma_max of n weight matrices W[i] (rows[i] x cols[i], min(rows, cols) <= 128; host arrays
 * of device pointers), exact to fp64 before the float32 rounding; scale = max(1, sigma/ln_lambda)
 * and, when Wn != NULL, Wn[i] = W[i] / scale[i]. */
size_t lrs_sigma_max_workspace(int n);
int lrs_sigma_max_f32(const float *const *W, float *const *Wn, const int *rows, const int *cols, int n,
                      float ln_lambda, float *sigma, float *scale, void *ws, size_t ws_bytes,
                      void *stream);

/* One Adam step over a flat buffer; step (device int) is the 1-based step count. */
int lrs_adam_f32(float *p, const float *g, float *m, float *v, int64_t n, const int *step, float lr,
                 float beta1, float beta2, float eps, void *stream);
/* loss_acc (device double) += sum((target*mask - out*mask)^2); gout (nullable) = dL/dout of the
 * mean.  mask (nullable) is [P], broadcast over the C channels. */
int lrs_masked_mse_f32(const float *out, const float *target, const float *mask, int C, int64_t P,
                       float *gout, double *loss_acc, void *stream);

/* Layout transforms between the unfolded matrix X[p = i + H j][b] and the DIP image img[b][i][j]
 * (…1-LiP.py:404 DIP_input = X + (1/mu_2) lambda_2 as (1,B,H,W); :411 U back to (P,B)). */
int lrs_unfolded_to_image_f32(const float *X, const float *L, float c, int64_t H, int64_t W, int64_t B,
                              float *img, void *stream);
int lrs_image_to_unfolded_f32(const float *img, int64_t H, int64_t W, int64_t B, float *X, void *stream);

/* Early stopping state (device memory).  lrs_es_init fills it; every lrs_es_update_f32 pushes one
 * output into the ring and, once full, applies the variance test.  ring: lrs_es_ring_bytes(size, N)
 * bytes of device memory -- the last `size` outputs as [size][N] floats (slot = epoch % size), then
 * the per-pixel window sums (fp64) and the window's sum of squares that the test slides from step to
 * step. */
typedef struct {
    int32_t count, size, patience, wait, stop, stop_epoch, best_epoch, reserved;
    double best, var_acc, last_var;
} lrs_es_state;
size_t lrs_es_ring_bytes(int size, int64_t N);
int lrs_es_init(lrs_es_state *st, int size, int patience, void *stream);
int lrs_es_update_f32(const float *out, int64_t N, float *ring, lrs_es_state *st, void *stream);

/* ---- Whole network + training step ---------------------------------------------------------
 * A DAG of nodes; tensor 0 is the network input (C x H x W), node i produces tensor i + 1 and
 * may read any earlier tensor.  The 1-Lip U-Net is a chain of CONV nodes; the skip net
 * (models/skip.py) adds BN and CONCAT nodes.  The host object holds shapes and offsets only;
 * parameters, gradients, Adam moments and the workspace are caller-owned device buffers given
 * to lrs_dipnet_bind. */
#define LRS_NODE_CONV 0    /* [upsample x2] -> pad -> conv(k, stride) -> [BN] -> act            */
#define LRS_NODE_BN 1      /* BN -> act on in0                                                  */
#define LRS_NODE_CONCAT 2  /* cat(in0, [upsample x2](in1)) along channels, centre-cropped       */
#define LRS_BN_NONE 0
#define LRS_BN_PLAIN 1     /* nn.BatchNorm2d, train mode (models/common.py:71)                 */
#define LRS_BN_LIP 2       /* BatchNormSpectralNorm-wrapped (lipschitz_constraint_layer.py:88)  */
#define LRS_WINIT_DEFAULT 0   /* nn.Conv2d default init: U(-1/sqrt(fan_in), +)                  */
#define LRS_WINIT_KAIMING 1   /* kaiming_uniform_(a=0, fan_in) (lipschitz_constraint_layer.py:74) */
typedef struct {
    int32_t kind, in0, in1, cout, k, stride, pad, pad_mode, upsample, bn, act, sn, winit;
} lrs_dip_node;
typedef struct lrs_dipnet lrs_dipnet;
int lrs_dipnet_create(const lrs_dip_node *nodes, int n_nodes, int C, int H, int W, const lrs_dip_opts *opts,
                      lrs_dipnet **out);
/* the options the net was created with */
int lrs_dipnet_get_opts(const lrs_dipnet *net, lrs_dip_opts *opts);
void lrs_dipnet_destroy(lrs_dipnet *net);
int64_t lrs_dipnet_num_params(const lrs_dipnet *net);
int64_t lrs_dipnet_num_bnstats(const lrs_dipnet *net);
size_t lrs_dipnet_workspace(const lrs_dipnet *net);
/* offsets (floats) of node i's parameters in the flat buffer; -1 when absent */
int lrs_dipnet_param_offsets(const lrs_dipnet *net, int node, int64_t *w, int64_t *b, int64_t *gamma,
                             int64_t *beta);
/* shape of node i's output (node = -1: the input) */
int lrs_dipnet_node_shape(const lrs_dipnet *net, int node, int *C, int *H, int *W);
int lrs_dipnet_out_shape(const lrs_dipnet *net, int *C, int *H, int *W);
int lrs_dipnet_bind(lrs_dipnet *net, float *params, float *grads, float *adam_m, float *adam_v,
                    float *bnstats, void *ws, size_t ws_bytes);
/* Conv weights per node winit, torch-default biases, gamma = 1, beta = 0, zero Adam state; a
 * counter-based RNG keyed by seed (the reference draws from the unseeded torch RNG). */
int lrs_dipnet_init_params(lrs_dipnet *net, uint64_t seed, void *stream);
/* zero the Adam moments and the step count (a fresh optimizer on the current parameters) */
int lrs_dipnet_reset_optimizer(lrs_dipnet *net, void *stream);
/* forward only (spectral norms included); the output stays in lrs_dipnet_output() */
int lrs_dipnet_forward(lrs_dipnet *net, const float *x, void *stream);
/* backward from gout = dL/d(output) (C x H x W, device) through the activations of the last
 * lrs_dipnet_forward on the same x: every parameter gradient into the bound grads buffer (sigma
 * and the BN scale c are constants, as the reference takes them from .data); no input gradient.
 * Replaces loss.backward() through my_Lipschitz_Unet / skip (…1-LiP.py:237, pro :245). */
int lrs_dipnet_backward(lrs_dipnet *net, const float *x, const float *gout, void *stream);
/* ln_lambda of the spectral normalisation (my_Lipschitz_Unet(..., ln_lambda); default 1) */
int lrs_dipnet_set_ln_lambda(lrs_dipnet *net, float ln_lambda);
const float *lrs_dipnet_output(const lrs_dipnet *net);
const float *lrs_dipnet_grads(const lrs_dipnet *net);
/* diagnostics: node i's buffers in the workspace after a forward / backward (NULL where absent):
 * its output, its pre-BatchNorm z, dL/dz, dL/d(output) */
#define LRS_BUF_OUT 0
#define LRS_BUF_Z 1
#define LRS_BUF_GZ 2
#define LRS_BUF_GRAD 3
const float *lrs_dipnet_node_buffer(const lrs_dipnet *net, int node, int which);
/* nsteps training steps: forward, masked MSE, backward, Adam; es (nullable) gets every step's
 * forward output (ring: es->size * C*H*W floats).  use_graph != 0 captures one step into a
 * hipGraph (on first use, re-captured when any argument changes) and replays it.  The weight
 * gradients run on a second stream the net owns with the calling stream's priority (one such
 * stream per priority seen, kept for the net's lifetime: switching priorities costs nothing). */
int lrs_dipnet_train_steps(lrs_dipnet *net, const float *x, const float *target, const float *mask,
                           float lr, float beta1, float beta2, float eps, lrs_es_state *es,
                           float *ring, int nsteps, int use_graph, void *stream);
/* loss of the last step (synchronises the stream; diagnostics only) */
int lrs_dipnet_last_loss(lrs_dipnet *net, double *loss, void *stream);
/* Stream ordering between two streams of one device: work enqueued on `waiter` after this call runs
 * after the work enqueued on `signaler` before it (an event with a device-scope release: cheaper
 * than a default event when nothing on the host waits on it).  The Python side orders the DIP
 * stream against the caller's this way. */
int lrs_stream_wait(void *waiter, void *signaler);

/* ---- Metrics (not timed) -------------------------------------------------------------------
 * acc (device double) = sum of the SSIM map of pytorch_ssim.ssim(img1, img2) over C x H x W
 * (pytorch_ssim/__init__.py:17-37; called at main_LRS_PnP_DIP_1-LiP.py:480-481); MSSIM =
 * acc / (C*H*W).  Images are [C][H][W] float32. */
int lrs_ssim_f32(const float *img1, const float *img2, int C, int H, int W, double *acc, void *stream);
/* Per-band PSNR 10 log10(255 / sqrt(mse_b)) (100 when mse_b < 1e-10) of X against C, both P x B
 * float32 unfolded (main_LRS_PnP.py:379-384, psnr() :40-46, bach_mpsnr :49-58); psnr: device, B
 * doubles.  fp64 accumulation, fixed-order reduction (deterministic). */
size_t lrs_psnr_workspace(int64_t P, int64_t B);
int lrs_psnr_bands_f32(const float *X, const float *C, int64_t P, int64_t B, double *psnr, void *ws,
                       size_t ws_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LRSPNP_H */
