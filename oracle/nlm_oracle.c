/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * CPU restatement of the plug-and-play denoiser the reference calls inside `ista`:
 *     denoise_nl_means(gradient, h=T, fast_mode=True, patch_size=3, patch_distance=3)
 *   main_LRS_PnP_DIP_1-LiP.py:192-196, main_LRS_PnP_DIP_pro.py:195-199,
 *   main_LRS_PnP.py:143-146 (h = 0.1*T).
 * The arithmetic lives in a third-party dependency that is not vendored in /root/reference:
 *   scikit-image 0.18.3 (conda build py39h51133e4_0),
 *   skimage/restoration/non_local_means.py:136-157 -> _nl_means_denoising.pyx
 *   `_fast_nl_means_denoising_2d` (Darbon et al. integral-image NLM, Froment variant,
 *   Schraudolph fast exp).
 * Restated from the published algorithm; pinned bit-exactly against golden vectors produced by
 * that .so (tests/golden/nlm_golden.npz, generator tests/golden/gen_golden.py).
 *
 * Two entry points:
 *   oracle_nlm_fast2d  — the full 2-D integral-image loop nest (any H x W x C image),
 *                        in skimage's loop and accumulation order.
 *   oracle_nlm_col     — the closed form of the same algorithm for a (K,1) column, which is the
 *                        only shape the reference ever passes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NLM_DISTANCE_CUTOFF 5.0

/* Schraudolph (1999) exp approximation as used by skimage: the high word of an IEEE double is
 * (int32)(1512775.3951951856938 * y) + 1072632447, the low word 0. */
static inline double fast_exp(double y) {
    int32_t hi = (int32_t)(1512775.3951951856938 * y) + 1072632447;
    uint64_t bits = ((uint64_t)(uint32_t)hi) << 32;
    double d;
    memcpy(&d, &bits, sizeof d);
    return d;
}

double oracle_fast_exp(double y) { return fast_exp(y); }

/* numpy.pad(mode='reflect') index map (mirror without repeating the edge sample). */
static int reflect_idx(int i, int n) {
    if (n == 1) return 0;
    int period = 2 * (n - 1);
    i %= period;
    if (i < 0) i += period;
    return i < n ? i : period - i;
}

/* img: H x W x C float32, C-contiguous. out: H x W x C float32. returns 0 on success. */
int oracle_nlm_fast2d(const float *img, int H, int W, int C, int s, int d, double h, double var,
                      float *out) {
    if (s % 2 == 0) s += 1;
    const int offset = s / 2;
    const int pad = offset + d + 1;
    const int nr = H + 2 * pad, nc = W + 2 * pad;
    float *padded = (float *)malloc(sizeof(float) * (size_t)nr * nc * C);
    double *result = (double *)calloc((size_t)nr * nc * C, sizeof(double));
    double *weights = (double *)calloc((size_t)nr * nc, sizeof(double));
    double *integral = (double *)calloc((size_t)nr * nc, sizeof(double));
    if (!padded || !result || !weights || !integral) {
        free(padded); free(result); free(weights); free(integral);
        return -1;
    }
    for (int r = 0; r < nr; ++r)
        for (int c = 0; c < nc; ++c) {
            int sr = reflect_idx(r - pad, H), sc = reflect_idx(c - pad, W);
            for (int ch = 0; ch < C; ++ch)
                padded[((size_t)r * nc + c) * C + ch] = img[((size_t)sr * W + sc) * C + ch];
        }
    const double h2s2 = (double)C * h * h * (double)s * (double)s;
    const double var2 = var * 2.0;
#define P(r, c, ch) ((double)padded[((size_t)(r) * nc + (c)) * C + (ch)])
#define I(r, c) integral[(size_t)(r) * nc + (c)]
    for (int t_row = -d; t_row <= d; ++t_row) {
        int row_start = offset > offset - t_row ? offset : offset - t_row;
        int row_end = (nr - offset) < (nr - offset - t_row) ? (nr - offset) : (nr - offset - t_row);
        for (int t_col = 0; t_col <= d; ++t_col) {
            int col_start = offset > offset - t_col ? offset : offset - t_col;
            int col_end = (nc - offset) < (nc - offset - t_col) ? (nc - offset) : (nc - offset - t_col);
            double alpha = (t_col == 0 && t_row != 0) ? 0.5 : 1.0;
            /* integral image of the squared shifted difference */
            int r0 = 1 > -t_row ? 1 : -t_row, r1 = nr < nr - t_row ? nr : nr - t_row;
            int c0 = 1 > -t_col ? 1 : -t_col, c1 = nc < nc - t_col ? nc : nc - t_col;
            for (int r = r0; r < r1; ++r)
                for (int c = c0; c < c1; ++c) {
                    double dist = 0.0;
                    for (int ch = 0; ch < C; ++ch) {
                        double t = P(r, c, ch) - P(r + t_row, c + t_col, ch);
                        dist += t * t;
                    }
                    dist -= C * var2;
                    I(r, c) = dist + I(r - 1, c) + I(r, c - 1) - I(r - 1, c - 1);
                }
            for (int r = row_start; r < row_end; ++r)
                for (int c = col_start; c < col_end; ++c) {
                    double dist = I(r + offset, c + offset) + I(r - offset, c - offset) -
                                  I(r - offset, c + offset) - I(r + offset, c - offset);
                    dist = (dist > 0.0 ? dist : 0.0) / h2s2;
                    if (dist > NLM_DISTANCE_CUTOFF) continue;
                    double w = alpha * fast_exp(-dist);
                    weights[(size_t)r * nc + c] += w;
                    weights[(size_t)(r + t_row) * nc + (c + t_col)] += w;
                    for (int ch = 0; ch < C; ++ch) {
                        result[((size_t)r * nc + c) * C + ch] += w * P(r + t_row, c + t_col, ch);
                        result[((size_t)(r + t_row) * nc + (c + t_col)) * C + ch] += w * P(r, c, ch);
                    }
                }
        }
    }
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c)
            for (int ch = 0; ch < C; ++ch) {
                size_t pi = ((size_t)(r + pad) * nc + (c + pad));
                out[((size_t)r * W + c) * C + ch] = (float)(result[pi * C + ch] / weights[pi]);
            }
#undef P
#undef I
    free(padded); free(result); free(weights); free(integral);
    return 0;
}

/*
 * Closed form for a (K,1) column, s = 3, d = 3.  With the image one column wide
 * all 11 padded columns are equal, the integral-image window degenerates to rows p..p+1 and the
 * 28 shifts fold into
 *     out[i] = (8 w0 v[p] + 7 sum_t w(p,t) v[p+t]) / (8 w0 + 7 sum_t w(p,t)),   t = +-1,+-2,+-3
 * with distance D(p,t) = [(v[p]-v[p+t])^2 + (v[p+1]-v[p+1+t])^2] * 2/(9 h^2) and
 * w = fast_exp(-D) unless D > 5.  CANONICAL evaluation order, reproduced bit-for-bit by the HIP
 * kernels (csrc/lrs_nlm.h): the Schraudolph scale is folded into the normaliser,
 *     y = S * kneg,  kneg = -1512775.3951951856938 * (2/((h*h)*9)),  skip if y < -1512775.39..*5,
 *     w = double{hi = (int)y + 1072632447, lo = 0},
 * sums in t = -3..3 order, fma for the weighted sums, one double division.
 * Against skimage's integral-image loop it differs only through rounding of D and of the double
 * accumulators (<= 1 ulp of the float32 output, ~1e-5 of elements; tests/test_oracle.py).
 * g: K floats with stride `ldg`; out: K floats with stride `ldo`.
 */
void oracle_nlm_col(const float *g, long K, long ldg, double h, float *out, long ldo) {
    const int d = 3, pad = 5;
    const long n = K + 2 * pad;
    double *v = (double *)malloc(sizeof(double) * (size_t)n);
    for (long i = 0; i < n; ++i) v[i] = (double)g[reflect_idx((int)(i - pad), (int)K) * ldg];
    const double A = 1512775.3951951856938;
    const double kneg = -A * (2.0 / ((h * h) * 9.0));
    const double ycut = -A * 5.0;
    const double c0 = 8.0 * fast_exp(-0.0);
    for (long i = 0; i < K; ++i) {
        long p = i + pad;
        double sw = 0.0, swv = 0.0;
        for (int t = -d; t <= d; ++t) {
            if (t == 0) continue;
            double a = v[p] - v[p + t], b = v[p + 1] - v[p + 1 + t];
            double aa = a * a, bb = b * b;
            double y = (aa + bb) * kneg;
            double w = 0.0;
            if (!(y < ycut)) {
                int32_t hi = (int32_t)y + 1072632447;
                uint64_t bits = ((uint64_t)(uint32_t)hi) << 32;
                memcpy(&w, &bits, sizeof w);
            }
            sw = sw + w;
            swv = fma(w, v[p + t], swv);
        }
        double num = fma(7.0, swv, c0 * v[p]);
        double den = fma(7.0, sw, c0);
        out[i * ldo] = (float)(num / den);
    }
    free(v);
}

/*
 * The MATLAB variant of the PnP prox (LRS-PnP(Matlab Code)/pnp_ista.m:30 calls
 * NLmeansfilter(gradient, 3, 3, 0.1*T)), restated for a (K,1) column in fp64
 * (NLmeansfilter.m:18-78):
 *   input2 = padarray(g, [3 3], 'symmetric')  -> g-hat[j] = g[-j-1] (j < 0), g[2K-1-j] (j >= K);
 *   kernel = make_kernel(3) normalised (sum 1); for a one-column image every column of the 7x7
 *   windows is the same, so d = sum_u krow[u] (g-hat[i+u] - g-hat[r+u])^2 with krow[u] the row
 *   sums of the kernel, (1/3) sum_{d=max(|u|,1)..3} 1/(2d+1);
 *   w = exp(-d / h^2) over r in [i-3, i+3] clipped to [0, K-1], r != i; wmax = max w;
 *   out = (sum w g[r] + wmax g[i]) / (sum w + wmax), or g[i] when that sum is 0.
 * Evaluation order (shared bit for bit with the HIP kernel, -ffp-contract=off): d accumulated over
 * u = -3..3 as d + krow*(diff*diff); neighbours r ascending.  MATLAB's own order of the 7x7 sum
 * (columns first) is not reproduced: there is no MATLAB/Octave here, so this mode is pinned by
 * a literal transcription of NLmeansfilter.m (oracle.py: nlm_matlab_literal), not by MATLAB.
 */
void oracle_nlm_matlab_krow(double krow[7]) {
    for (int u = -3; u <= 3; ++u) {
        const int a = u < 0 ? -u : u;
        double s = 0.0;
        for (int d = (a < 1 ? 1 : a); d <= 3; ++d) s = s + 1.0 / (double)(2 * d + 1);
        krow[u + 3] = s / 3.0;
    }
}

void oracle_nlm_matlab_col(const float *g, long K, long ldg, double h, float *out, long ldo) {
    double krow[7];
    oracle_nlm_matlab_krow(krow);
    const double h2 = h * h;
    double *v = (double *)malloc(sizeof(double) * (size_t)(K + 6));
    for (long j = -3; j < K + 3; ++j) {
        const long s = j < 0 ? -j - 1 : (j >= K ? 2 * K - 1 - j : j);
        v[j + 3] = (double)g[s * ldg];
    }
    for (long i = 0; i < K; ++i) {
        double sw = 0.0, av = 0.0, wmax = 0.0;
        for (int t = -3; t <= 3; ++t) {
            const long r = i + t;
            if (t == 0 || r < 0 || r >= K) continue;
            double d = 0.0;
            for (int u = -3; u <= 3; ++u) {
                const double df = v[i + u + 3] - v[r + u + 3];
                d = d + krow[u + 3] * (df * df);
            }
            const double w = exp(-d / h2);
            if (w > wmax) wmax = w;
            sw = sw + w;
            av = av + w * v[r + 3];
        }
        av = av + wmax * v[i + 3];
        sw = sw + wmax;
        out[i * ldo] = sw > 0.0 ? (float)(av / sw) : g[i * ldg];
    }
    free(v);
}
