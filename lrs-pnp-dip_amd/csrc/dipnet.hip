// DIP low-rank prox: C-ABI of the layer primitives and the sequential-network training engine.
//
// Reference: main_LRS_PnP_DIP_1-LiP.py:208-264 (get_DIP_out: fresh my_Lipschitz_Unet, Adam,
// masked MSE, early stopping) and models/my_Lipschitz_Unet.py:21-148.  The engine launches one
// training step as ~8 kernels per conv unit from C++ (no per-layer Python), and can capture the
// step in a hipGraph and replay it: the Adam step count and the early-stopping state live in
// device memory, so a replayed step is exactly the eager step.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "dip_kernels.h"

using namespace lrs;

namespace {

constexpr int kEw = 256;   // elementwise block size

inline unsigned ew_blocks(int64_t n, int64_t cap = 4096) {
    int64_t b = (n + kEw - 1) / kEw;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

int make_geom(int Cin, int H, int W, int k, int stride, int pad, int pad_mode, int up, ConvGeom &g) {
    if (Cin <= 0 || H <= 0 || W <= 0 || k <= 0 || stride <= 0 || pad < 0) return LRS_E_INVALID;
    if (pad_mode != LRS_PAD_ZERO && pad_mode != LRS_PAD_REFLECT) return LRS_E_INVALID;
    g.Cin = Cin;
    g.Hs = H;
    g.Ws = W;
    g.up = up ? 1 : 0;
    g.Hu = up ? 2 * H : H;
    g.Wu = up ? 2 * W : W;
    g.pad = pad;
    g.pad_mode = pad_mode;
    g.k = k;
    g.stride = stride;
    if (pad_mode == LRS_PAD_REFLECT && (pad >= g.Hu || pad >= g.Wu)) return LRS_E_INVALID;
    const int hp = g.Hu + 2 * pad, wp = g.Wu + 2 * pad;
    if (hp < k || wp < k) return LRS_E_INVALID;
    g.Ho = (hp - k) / stride + 1;
    g.Wo = (wp - k) / stride + 1;
    return LRS_OK;
}

inline bool plain_unit(const ConvGeom &g) { return g.k == 1 && g.stride == 1 && g.pad == 0 && !g.up; }

struct Split {
    int S, kchunk;
    bool big;   // 128x128 tiles (k_gemm) or 64x64 (k_gemm64)
};

// Tile choice and split-K: 128x128 tiles when they alone give >= 128 workgroups, else 64x64;
// then split K until ~512 workgroups (2 per CU), keeping >= 128 of K per split and <= 64 splits.
Split choose_split(int M, int N, int K) {
    const int64_t t128 = (int64_t)((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
    const bool big = t128 >= 128;
    const int64_t tiles = big ? t128 : (int64_t)((M + kBM64 - 1) / kBM64) * ((N + kBN64 - 1) / kBN64);
    int S = 1;
    if (tiles < 256) {
        S = (int)((512 + tiles - 1) / tiles);
        const int smax = (K + 127) / 128;
        if (S > smax) S = smax;
        if (S > 64) S = 64;
        if (S < 1) S = 1;
    }
    int kchunk = (int)round_up((K + S - 1) / S, kBK);
    if (kchunk < kBK) kchunk = kBK;
    S = (K + kchunk - 1) / kchunk;
    if (S < 1) S = 1;
    return {S, kchunk, big};
}

int64_t gemm_part_floats(int M, int N, int K) {
    const Split s = choose_split(M, N, K);
    return s.S > 1 ? (int64_t)s.S * M * N : 0;
}

// C = op(A) op(B) (+ bias) (/ *div); part: split-K scratch (>= gemm_part_floats)
int gemm(int TA, int TB, const float *A, const float *B, float *C, const float *bias, const float *div, int M,
         int N, int K, float *part, int64_t part_cap, hipStream_t st) {
    if (M <= 0 || N <= 0) return LRS_OK;
    const Split s = choose_split(M, N, K);
    GemmArgs g{A, B, C, bias, div, M, N, K, s.kchunk};
    if (s.S > 1) {
        if (!part || part_cap < (int64_t)s.S * M * N) return LRS_E_WORKSPACE;
        g.C = part;
    }
    if (s.big) {
        dim3 grid((N + kBN - 1) / kBN, (M + kBM - 1) / kBM, s.S);
        if (!TA && !TB) hipLaunchKernelGGL((k_gemm<0, 0>), grid, dim3(kGemmThreads), 0, st, g);
        else if (!TA && TB) hipLaunchKernelGGL((k_gemm<0, 1>), grid, dim3(kGemmThreads), 0, st, g);
        else if (TA && !TB) hipLaunchKernelGGL((k_gemm<1, 0>), grid, dim3(kGemmThreads), 0, st, g);
        else hipLaunchKernelGGL((k_gemm<1, 1>), grid, dim3(kGemmThreads), 0, st, g);
    } else {
        dim3 grid((N + kBN64 - 1) / kBN64, (M + kBM64 - 1) / kBM64, s.S);
        if (!TA && !TB) hipLaunchKernelGGL((k_gemm64<0, 0>), grid, dim3(kGemmThreads), 0, st, g);
        else if (!TA && TB) hipLaunchKernelGGL((k_gemm64<0, 1>), grid, dim3(kGemmThreads), 0, st, g);
        else if (TA && !TB) hipLaunchKernelGGL((k_gemm64<1, 0>), grid, dim3(kGemmThreads), 0, st, g);
        else hipLaunchKernelGGL((k_gemm64<1, 1>), grid, dim3(kGemmThreads), 0, st, g);
    }
    if (s.S > 1) {
        const int64_t MN = (int64_t)M * N;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((MN + kEw - 1) / kEw)), dim3(kEw), 0, st, part, s.S, M,
                           N, bias, div, C);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int64_t conv_part_floats(const ConvGeom &g, int Cout) {
    const int P = g.Ho * g.Wo, Kc = g.Cin * g.k * g.k;
    int64_t m = gemm_part_floats(Cout, P, Kc);                       // forward
    const int64_t b = gemm_part_floats(Cout, Kc, P);                 // dW
    const int64_t c = gemm_part_floats(Kc, P, Cout);                 // dcol
    if (b > m) m = b;
    if (c > m) m = c;
    return m;
}

int conv_fwd(const ConvGeom &g, const float *x, const float *w, const float *bias, int Cout, float *col, float *y,
             float *part, int64_t part_cap, hipStream_t st) {
    const int P = g.Ho * g.Wo, Kc = g.Cin * g.k * g.k;
    const float *B = x;
    if (!plain_unit(g)) {
        if (!col) return LRS_E_WORKSPACE;
        const int64_t n = (int64_t)Kc * P;
        hipLaunchKernelGGL(k_im2col, dim3(ew_blocks(n, 1 << 16)), dim3(kEw), 0, st, x, g, col);
        B = col;
    }
    return gemm(0, 0, w, B, y, bias, nullptr, Cout, P, Kc, part, part_cap, st);
}

// gw = gz col^T / div ; gx = col2im(w^T gz) (gx nullable).  dcol: Kc*P floats when !plain.
int conv_bwd(const ConvGeom &g, const float *gz, const float *col, const float *w, const float *div, int Cout,
             float *gx, float *gw, float *dcol, float *part, int64_t part_cap, hipStream_t st) {
    const int P = g.Ho * g.Wo, Kc = g.Cin * g.k * g.k;
    int rc = gemm(0, 1, gz, col, gw, nullptr, div, Cout, Kc, P, part, part_cap, st);
    if (rc || !gx) return rc;
    if (plain_unit(g)) return gemm(1, 0, w, gz, gx, nullptr, nullptr, Kc, P, Cout, part, part_cap, st);
    if (!dcol) return LRS_E_WORKSPACE;
    rc = gemm(1, 0, w, gz, dcol, nullptr, nullptr, Kc, P, Cout, part, part_cap, st);
    if (rc) return rc;
    const int64_t n = (int64_t)g.Cin * g.Hs * g.Ws;
    hipLaunchKernelGGL(k_col2im, dim3(ew_blocks(n, 1 << 16)), dim3(kEw), 0, st, dcol, g, gx);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// workgroups per channel for the BN kernels: ~4096 elements each, at most 64
inline int bn_split(int64_t P) {
    int64_t S = (P + 4095) / 4096;
    if (S < 1) S = 1;
    if (S > 64) S = 64;
    return (int)S;
}

inline int64_t bn_part_doubles(int C, int64_t P) { return (int64_t)C * bn_split(P) * 3; }

int bn_fwd(const float *z, float *y, const float *gamma, const float *beta, float *mean, float *invstd, float *rm,
           float *rv, int C, int64_t P, int act, float eps, float mom, double *part, hipStream_t st) {
    const int S = bn_split(P);
    const int chunk = (int)((P + S - 1) / S);
    BnArgs a{z, y, gamma, beta, mean, invstd, rm, rv, part, C, (int)P, S, chunk, gamma ? 1 : 0, act, eps, mom};
    if (gamma) hipLaunchKernelGGL(k_bn_stats, dim3(S, C), dim3(kBnThreads), 0, st, a);
    hipLaunchKernelGGL(k_bn_apply, dim3(S, C), dim3(kBnThreads), 0, st, a);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int bn_bwd(const float *gy, const float *y, const float *z, const float *gamma, const float *mean,
           const float *invstd, float *gz, float *ggamma, float *gbeta, float *gbias, int C, int64_t P, int act,
           double *part, hipStream_t st) {
    const int S = bn_split(P);
    const int chunk = (int)((P + S - 1) / S);
    BnBwdArgs a{gy, y, z, gamma, mean, invstd, gz, ggamma, gbeta, gbias, part, C, (int)P, S, chunk,
                gamma ? 1 : 0, act};
    if (gamma || gbias) hipLaunchKernelGGL(k_bn_bwd_stats, dim3(S, C), dim3(kBnThreads), 0, st, a);
    hipLaunchKernelGGL(k_bn_bwd_apply, dim3(S, C), dim3(kBnThreads), 0, st, a);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int sn_launch(const SnConv *table_dev, int n, int64_t max_elems, double *gram, float *sigma, float *scale,
              float ln_lambda, bool apply, hipStream_t st, long long *prof = nullptr) {
    const int tiles = (kSnMaxDim + 31) / 32;
    hipLaunchKernelGGL(k_sn_gram, dim3(tiles * tiles, kSnSplit, n), dim3(256), 0, st, table_dev, gram);
    const size_t lds = sizeof(double) * kSnMaxDim * (kSnMaxDim + 1);
    hipError_t e = hipFuncSetAttribute((const void *)k_sn_sigma, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_sn_sigma, dim3(n), dim3(256), lds, st, table_dev, gram, sigma, scale, ln_lambda, prof);
    if (apply) hipLaunchKernelGGL(k_sn_apply, dim3(ew_blocks(max_elems, 256), n), dim3(kEw), 0, st, table_dev, scale);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

__global__ void k_es_init(lrs_es_state *st, int size, int patience) {
    st->count = 0;
    st->size = size;
    st->patience = patience;
    st->wait = 0;
    st->stop = 0;
    st->stop_epoch = -1;
    st->best_epoch = 0;
    st->reserved = 0;
    st->best = INFINITY;
    st->var_acc = 0.0;
    st->last_var = NAN;
}

int es_update(const float *out, int64_t N, float *ring, lrs_es_state *es, hipStream_t st) {
    hipLaunchKernelGGL(k_es_push, dim3(ew_blocks(N, 1024)), dim3(kEw), 0, st, out, N, ring, es);
    hipLaunchKernelGGL(k_es_var, dim3(ew_blocks(N, 1024)), dim3(kEw), 0, st, ring, N, es);
    hipLaunchKernelGGL(k_es_decide, dim3(1), dim3(64), 0, st, N, es);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

inline uint64_t mix64(uint64_t z) {   // splitmix64 finaliser (host + device)
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__global__ void k_init_uniform(float *p, int64_t n, float bound, uint64_t key) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = key + 0x9e3779b97f4a7c15ULL * (uint64_t)(i + 1);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        z ^= z >> 31;
        const float u = (float)(z >> 40) * (1.0f / 16777216.0f);   // [0, 1)
        p[i] = (2.0f * u - 1.0f) * bound;
    }
}

__global__ void k_fill(float *p, int64_t n, float v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// img[b][i][j] = X[(i + H j) B + b] + c * L[...]   (…1-LiP.py:404; L nullable)
__global__ void k_unfolded_to_image(const float *__restrict__ X, const float *__restrict__ L, float c, int64_t H,
                                    int64_t W, int64_t B, float *__restrict__ img) {
    const int64_t n = H * W * B;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = o % W, i = (o / W) % H, b = o / (W * H);
        const int64_t src = (i + H * j) * B + b;
        float v = X[src];
        if (L) v = v + c * L[src];
        img[o] = v;
    }
}

// X[(i + H j) B + b] = img[b][i][j]   (…1-LiP.py:411)
__global__ void k_image_to_unfolded(const float *__restrict__ img, int64_t H, int64_t W, int64_t B,
                                    float *__restrict__ X) {
    const int64_t n = H * W * B;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = o % B, p = o / B;
        const int64_t i = p % H, j = p / H;
        X[o] = img[(b * H + i) * W + j];
    }
}

}  // namespace

// ============================================================================================
// Primitive C ABI
// ============================================================================================
extern "C" int lrs_conv2d_out_size(int H, int W, int k, int stride, int pad, int upsample, int *Ho, int *Wo) {
    ConvGeom g;
    const int rc = make_geom(1, H, W, k, stride, pad, LRS_PAD_ZERO, upsample, g);
    if (rc) return rc;
    if (Ho) *Ho = g.Ho;
    if (Wo) *Wo = g.Wo;
    return LRS_OK;
}

extern "C" int64_t lrs_conv2d_col_size(int Cin, int H, int W, int k, int stride, int pad, int upsample) {
    ConvGeom g;
    if (make_geom(Cin, H, W, k, stride, pad, LRS_PAD_ZERO, upsample, g)) return -1;
    return plain_unit(g) ? 0 : (int64_t)Cin * k * k * g.Ho * g.Wo;
}

extern "C" size_t lrs_conv2d_workspace(int Cin, int H, int W, int Cout, int k, int stride, int pad, int upsample) {
    ConvGeom g;
    if (make_geom(Cin, H, W, k, stride, pad, LRS_PAD_ZERO, upsample, g) || Cout <= 0) return 0;
    const int64_t dcol = plain_unit(g) ? 0 : (int64_t)Cin * k * k * g.Ho * g.Wo;
    return (size_t)(conv_part_floats(g, Cout) + dcol) * sizeof(float) + 256;
}

extern "C" int lrs_conv2d_fwd_f32(const float *x, int Cin, int H, int W, const float *w, const float *bias, int Cout,
                                  int k, int stride, int pad, int pad_mode, int upsample, float *col, float *y,
                                  void *ws, size_t ws_bytes, void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g);
    if (rc) return rc;
    if (!x || !w || !y || Cout <= 0) return LRS_E_INVALID;
    const int64_t part = conv_part_floats(g, Cout);
    if (part > 0 && (!ws || ws_bytes < (size_t)part * sizeof(float))) return LRS_E_WORKSPACE;
    return conv_fwd(g, x, w, bias, Cout, col, y, (float *)ws, part, (hipStream_t)stream);
}

extern "C" int lrs_conv2d_bwd_f32(const float *gy, const float *col, const float *w, const float *w_div, int Cin,
                                  int H, int W, int Cout, int k, int stride, int pad, int pad_mode, int upsample,
                                  float *gx, float *gw, void *ws, size_t ws_bytes, void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g);
    if (rc) return rc;
    if (!gy || !col || !w || !gw || Cout <= 0) return LRS_E_INVALID;
    const int64_t part = conv_part_floats(g, Cout);
    const int64_t dcol = plain_unit(g) ? 0 : (int64_t)Cin * k * k * g.Ho * g.Wo;
    if (ws_bytes < (size_t)(part + dcol) * sizeof(float) || (!ws && part + dcol > 0)) return LRS_E_WORKSPACE;
    float *dc = dcol ? (float *)ws : nullptr;
    float *pt = (float *)ws + dcol;
    return conv_bwd(g, gy, col, w, w_div, Cout, gx, gw, dc, pt, part, (hipStream_t)stream);
}

extern "C" size_t lrs_bn_act_workspace(int C, int64_t P) {
    if (C <= 0 || P <= 0) return 0;
    return (size_t)bn_part_doubles(C, P) * sizeof(double) + 256;
}

static int bn_ws(void *ws, size_t ws_bytes, int C, int64_t P, double **part) {
    if (!ws || ws_bytes < lrs_bn_act_workspace(C, P)) return LRS_E_WORKSPACE;
    *part = (double *)ws;
    return LRS_OK;
}

extern "C" int lrs_bn_act_fwd_f32(const float *z, float *y, const float *gamma, const float *beta, float *mean,
                                  float *invstd, float *run_mean, float *run_var, int C, int64_t P, int act,
                                  float eps, float momentum, void *ws, size_t ws_bytes, void *stream) {
    if (!z || !y || C <= 0 || P <= 0 || P > INT32_MAX) return LRS_E_INVALID;
    if (gamma && (!beta || !mean || !invstd)) return LRS_E_INVALID;
    double *part;
    const int rc = bn_ws(ws, ws_bytes, C, P, &part);
    if (rc) return rc;
    return bn_fwd(z, y, gamma, beta, mean, invstd, run_mean, run_var, C, P, act, eps, momentum, part,
                  (hipStream_t)stream);
}

extern "C" int lrs_bn_act_bwd_f32(const float *gy, const float *y, const float *z, const float *gamma,
                                  const float *mean, const float *invstd, float *gz, float *ggamma, float *gbeta,
                                  float *gbias, int C, int64_t P, int act, void *ws, size_t ws_bytes, void *stream) {
    if (!gy || !y || !gz || C <= 0 || P <= 0 || P > INT32_MAX) return LRS_E_INVALID;
    if (gamma && (!z || !mean || !invstd || !ggamma || !gbeta)) return LRS_E_INVALID;
    double *part;
    const int rc = bn_ws(ws, ws_bytes, C, P, &part);
    if (rc) return rc;
    return bn_bwd(gy, y, z, gamma, mean, invstd, gz, ggamma, gbeta, gbias, C, P, act, part, (hipStream_t)stream);
}

extern "C" size_t lrs_sigma_max_workspace(int n) {
    if (n <= 0) return 0;
    return (size_t)n * kSnSplit * kSnMaxDim * kSnMaxDim * sizeof(double) + (size_t)n * sizeof(SnConv) + 256;
}

extern "C" int lrs_sigma_max_f32(const float *const *W, float *const *Wn, const int *rows, const int *cols, int n,
                                 float ln_lambda, float *sigma, float *scale, void *ws, size_t ws_bytes,
                                 void *stream) {
    if (n <= 0) return LRS_OK;
    if (!W || !rows || !cols || !sigma || !scale || !(ln_lambda > 0.0f)) return LRS_E_INVALID;
    if (!ws || ws_bytes < lrs_sigma_max_workspace(n)) return LRS_E_WORKSPACE;
    std::vector<SnConv> tab(n);
    int64_t maxe = 0;
    for (int i = 0; i < n; ++i) {
        if (!W[i] || rows[i] <= 0 || cols[i] <= 0) return LRS_E_INVALID;
        if ((rows[i] < cols[i] ? rows[i] : cols[i]) > kSnMaxDim) return LRS_E_UNSUPPORTED;
        tab[i] = SnConv{W[i], Wn ? Wn[i] : nullptr, rows[i], cols[i]};
        const int64_t e = (int64_t)rows[i] * cols[i];
        if (e > maxe) maxe = e;
    }
    double *gram = (double *)ws;
    SnConv *tdev = (SnConv *)((char *)ws + (size_t)n * kSnSplit * kSnMaxDim * kSnMaxDim * sizeof(double));
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(tdev, tab.data(), sizeof(SnConv) * n, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return (int)e;
    e = hipStreamSynchronize(st);   // the host table is a local
    if (e != hipSuccess) return (int)e;
    return sn_launch(tdev, n, maxe, gram, sigma, scale, ln_lambda, Wn != nullptr, st);
}

// diagnostics: phase timestamps (wall_clock64 ticks) of the sigma kernel, 8 int64 per matrix:
// [start, Gram loaded, Lanczos done, multisection done, Lanczos steps]
extern "C" int lrs_diag_sigma_phases(const float *const *W, const int *rows, const int *cols, int n, void *ws,
                                     size_t ws_bytes, long long *prof, void *stream) {
    if (n <= 0 || !W || !prof) return LRS_E_INVALID;
    if (!ws || ws_bytes < lrs_sigma_max_workspace(n) + 2 * n * sizeof(float)) return LRS_E_WORKSPACE;
    std::vector<SnConv> tab(n);
    for (int i = 0; i < n; ++i) tab[i] = SnConv{W[i], nullptr, rows[i], cols[i]};
    double *gram = (double *)ws;
    SnConv *tdev = (SnConv *)((char *)ws + (size_t)n * kSnSplit * kSnMaxDim * kSnMaxDim * sizeof(double));
    float *sig = (float *)((char *)ws + lrs_sigma_max_workspace(n));
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(tdev, tab.data(), sizeof(SnConv) * n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    return sn_launch(tdev, n, 0, gram, sig, sig + n, 1.0f, false, st, prof);
}

extern "C" int lrs_adam_f32(float *p, const float *g, float *m, float *v, int64_t n, const int *step, float lr,
                            float beta1, float beta2, float eps, void *stream) {
    if (!p || !g || !m || !v || !step || n < 0) return LRS_E_INVALID;
    if (n == 0) return LRS_OK;
    hipLaunchKernelGGL(k_adam, dim3(ew_blocks(n, 8192)), dim3(kEw), 0, (hipStream_t)stream, p, g, m, v, n, step, lr,
                       beta1, beta2, eps);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_masked_mse_f32(const float *out, const float *target, const float *mask, int C, int64_t P,
                                  float *gout, double *loss_acc, void *stream) {
    if (!out || !target || !loss_acc || C <= 0 || P <= 0) return LRS_E_INVALID;
    hipLaunchKernelGGL(k_masked_mse, dim3(ew_blocks((int64_t)C * P, 2048)), dim3(kEw), 0, (hipStream_t)stream, out,
                       target, mask, C, P, gout, loss_acc);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_unfolded_to_image_f32(const float *X, const float *L, float c, int64_t H, int64_t W, int64_t B,
                                         float *img, void *stream) {
    if (!X || !img || H <= 0 || W <= 0 || B <= 0) return LRS_E_INVALID;
    hipLaunchKernelGGL(k_unfolded_to_image, dim3(ew_blocks(H * W * B, 8192)), dim3(kEw), 0, (hipStream_t)stream, X,
                       L, c, H, W, B, img);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_image_to_unfolded_f32(const float *img, int64_t H, int64_t W, int64_t B, float *X, void *stream) {
    if (!X || !img || H <= 0 || W <= 0 || B <= 0) return LRS_E_INVALID;
    hipLaunchKernelGGL(k_image_to_unfolded, dim3(ew_blocks(H * W * B, 8192)), dim3(kEw), 0, (hipStream_t)stream,
                       img, H, W, B, X);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_es_init(lrs_es_state *st, int size, int patience, void *stream) {
    if (!st || size <= 0 || patience <= 0) return LRS_E_INVALID;
    hipLaunchKernelGGL(k_es_init, dim3(1), dim3(1), 0, (hipStream_t)stream, st, size, patience);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_es_update_f32(const float *out, int64_t N, float *ring, lrs_es_state *st, void *stream) {
    if (!out || !ring || !st || N <= 0) return LRS_E_INVALID;
    return es_update(out, N, ring, st, (hipStream_t)stream);
}

// ============================================================================================
// Sequential network engine
// ============================================================================================
struct lrs_dipnet {
    struct Unit {
        lrs_conv_unit u;
        ConvGeom g;
        int64_t P, Kc;
        int64_t w_off, b_off, gm_off, bt_off, rs_off;   // params / bn running stats
        int64_t act_off, z_off, col_off, mean_off, istd_off, wn_off;   // workspace (floats)
    };
    std::vector<Unit> units;
    int H = 0, W = 0;
    int64_t n_params = 0, n_bnstats = 0;
    // workspace layout (floats unless noted)
    int64_t ws_floats = 0;
    int64_t ga_off = 0, gb_off = 0, dz_off = 0, dcol_off = 0, part_off = 0, part_cap = 0;
    int64_t sigma_off = 0, scale_off = 0, gram_off_bytes = 0, table_off_bytes = 0, misc_off_bytes = 0;
    int64_t bnpart_off_bytes = 0, ticket_off_bytes = 0, ticket_bytes = 0;
    size_t ws_bytes = 0;
    int64_t max_w = 0;
    // bound buffers
    float *params = nullptr, *grads = nullptr, *am = nullptr, *av = nullptr, *bnstats = nullptr;
    char *ws = nullptr;
    // graph cache
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    struct Key {
        const void *x, *t, *m, *es, *ring;
        float lr, b1, b2, eps;
    } key{};
    bool have_key = false;

    float *f(int64_t off) const { return (float *)ws + off; }
    double *gram() const { return (double *)(ws + gram_off_bytes); }
    SnConv *table() const { return (SnConv *)(ws + table_off_bytes); }
    double *loss_acc() const { return (double *)(ws + misc_off_bytes); }
    int *step() const { return (int *)(ws + misc_off_bytes + 8); }
    double *bnpart() const { return (double *)(ws + bnpart_off_bytes); }
    int *ticket() const { return (int *)(ws + ticket_off_bytes); }
};

namespace {

int64_t align64(int64_t n) { return (n + 63) / 64 * 64; }   // floats (256 bytes)

int dipnet_forward(lrs_dipnet *net, const float *x, hipStream_t st) {
    const int n = (int)net->units.size();
    int rc = sn_launch(net->table(), n, net->max_w, net->gram(), net->f(net->sigma_off), net->f(net->scale_off), 1.0f,
                       true, st);
    if (rc) return rc;
    const float *src = x;
    for (int i = 0; i < n; ++i) {
        auto &U = net->units[i];
        const bool bn = U.u.bn != 0;
        float *act = net->f(U.act_off);
        float *z = bn ? net->f(U.z_off) : act;
        rc = conv_fwd(U.g, src, net->f(U.wn_off), net->params + U.b_off, U.u.cout,
                      U.col_off >= 0 ? net->f(U.col_off) : nullptr, z, net->f(net->part_off), net->part_cap, st);
        if (rc) return rc;
        rc = bn_fwd(z, act, bn ? net->params + U.gm_off : nullptr, bn ? net->params + U.bt_off : nullptr,
                    net->f(U.mean_off), net->f(U.istd_off), bn ? net->bnstats + U.rs_off : nullptr,
                    bn ? net->bnstats + U.rs_off + U.u.cout : nullptr, U.u.cout, U.P, U.u.act, 1e-5f, 0.1f,
                    net->bnpart(), st);
        if (rc) return rc;
        src = act;
    }
    return LRS_OK;
}

int dipnet_step(lrs_dipnet *net, const float *x, const float *target, const float *mask, float lr, float b1, float b2,
                float eps, lrs_es_state *es, float *ring, hipStream_t st) {
    int rc = dipnet_forward(net, x, st);
    if (rc) return rc;
    const int n = (int)net->units.size();
    const auto &L = net->units[n - 1];
    const float *out = net->f(L.act_off);
    const int64_t Pout = L.P;
    hipError_t e = hipMemsetAsync(net->loss_acc(), 0, sizeof(double), st);
    if (e != hipSuccess) return (int)e;
    float *g = net->f(net->ga_off), *g2 = net->f(net->gb_off);
    rc = lrs_masked_mse_f32(out, target, mask, L.u.cout, Pout, g, net->loss_acc(), st);
    if (rc) return rc;
    for (int i = n - 1; i >= 0; --i) {
        auto &U = net->units[i];
        const bool bn = U.u.bn != 0;
        float *act = net->f(U.act_off);
        float *z = bn ? net->f(U.z_off) : act;
        float *gz = net->f(net->dz_off);
        rc = bn_bwd(g, act, z, bn ? net->params + U.gm_off : nullptr, net->f(U.mean_off), net->f(U.istd_off), gz,
                    bn ? net->grads + U.gm_off : nullptr, bn ? net->grads + U.bt_off : nullptr, net->grads + U.b_off,
                    U.u.cout, U.P, U.u.act, net->bnpart(), st);
        if (rc) return rc;
        const float *colsrc = U.col_off >= 0 ? net->f(U.col_off) : (i == 0 ? x : net->f(net->units[i - 1].act_off));
        rc = conv_bwd(U.g, gz, colsrc, net->f(U.wn_off), net->f(net->scale_off) + i, U.u.cout, i > 0 ? g2 : nullptr,
                      net->grads + U.w_off, U.col_off >= 0 ? net->f(net->dcol_off) : nullptr, net->f(net->part_off),
                      net->part_cap, st);
        if (rc) return rc;
        float *tmp = g;
        g = g2;
        g2 = tmp;
    }
    hipLaunchKernelGGL(k_counter_inc, dim3(1), dim3(64), 0, st, net->step());
    rc = lrs_adam_f32(net->params, net->grads, net->am, net->av, net->n_params, net->step(), lr, b1, b2, eps, st);
    if (rc) return rc;
    if (es) {
        rc = es_update(out, (int64_t)L.u.cout * Pout, ring, es, st);
        if (rc) return rc;
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

void drop_graph(lrs_dipnet *net) {
    if (net->gexec) (void)hipGraphExecDestroy(net->gexec);
    if (net->graph) (void)hipGraphDestroy(net->graph);
    net->gexec = nullptr;
    net->graph = nullptr;
    net->have_key = false;
}

}  // namespace

extern "C" int lrs_dipnet_create(const lrs_conv_unit *units, int n_units, int H, int W, lrs_dipnet **out) {
    if (!units || n_units <= 0 || H <= 0 || W <= 0 || !out) return LRS_E_INVALID;
    lrs_dipnet *net = new (std::nothrow) lrs_dipnet();
    if (!net) return LRS_E_INVALID;
    net->H = H;
    net->W = W;
    int cin = units[0].cin, h = H, w = W;
    int64_t pofs = 0, rofs = 0, ofs = 0, max_act = (int64_t)cin * H * W, max_dz = 0, max_dcol = 0, part = 0;
    int64_t max_bnpart = 0, max_c = 0;
    for (int i = 0; i < n_units; ++i) {
        lrs_dipnet::Unit U{};
        U.u = units[i];
        if (U.u.cin != cin || U.u.cout <= 0) { delete net; return LRS_E_INVALID; }
        if (U.u.act != LRS_ACT_NONE && U.u.act != LRS_ACT_LRELU && U.u.act != LRS_ACT_SIGMOID) { delete net; return LRS_E_INVALID; }
        int rc = make_geom(cin, h, w, U.u.k, U.u.stride, U.u.pad, U.u.pad_mode, U.u.upsample, U.g);
        if (rc) { delete net; return rc; }
        U.P = (int64_t)U.g.Ho * U.g.Wo;
        U.Kc = (int64_t)cin * U.u.k * U.u.k;
        if ((U.Kc < U.u.cout ? U.Kc : U.u.cout) > kSnMaxDim) { delete net; return LRS_E_UNSUPPORTED; }
        // parameters (flat): W_bar, bias, [gamma_orig, beta_orig]
        U.w_off = pofs; pofs += U.u.cout * U.Kc;
        U.b_off = pofs; pofs += U.u.cout;
        U.gm_off = U.bt_off = U.rs_off = -1;
        if (U.u.bn) {
            U.gm_off = pofs; pofs += U.u.cout;
            U.bt_off = pofs; pofs += U.u.cout;
            U.rs_off = rofs; rofs += 2 * U.u.cout;
        }
        // workspace
        U.act_off = ofs; ofs += align64(U.u.cout * U.P);
        U.z_off = -1;
        if (U.u.bn) { U.z_off = ofs; ofs += align64(U.u.cout * U.P); }
        U.col_off = -1;
        if (!plain_unit(U.g)) {
            U.col_off = ofs; ofs += align64(U.Kc * U.P);
            if (i > 0 && U.Kc * U.P > max_dcol) max_dcol = U.Kc * U.P;
        }
        U.mean_off = ofs; ofs += align64(U.u.cout);
        U.istd_off = ofs; ofs += align64(U.u.cout);
        U.wn_off = ofs; ofs += align64(U.u.cout * U.Kc);
        if (U.u.cout * U.Kc > net->max_w) net->max_w = U.u.cout * U.Kc;
        if (U.u.cout * U.P > max_act) max_act = U.u.cout * U.P;
        if (U.u.cout * U.P > max_dz) max_dz = U.u.cout * U.P;
        if (bn_part_doubles(U.u.cout, U.P) > max_bnpart) max_bnpart = bn_part_doubles(U.u.cout, U.P);
        if (U.u.cout > max_c) max_c = U.u.cout;
        const int64_t pc = conv_part_floats(U.g, U.u.cout);
        if (pc > part) part = pc;
        net->units.push_back(U);
        cin = U.u.cout;
        h = U.g.Ho;
        w = U.g.Wo;
    }
    net->n_params = pofs;
    net->n_bnstats = rofs;
    net->ga_off = ofs; ofs += align64(max_act);
    net->gb_off = ofs; ofs += align64(max_act);
    net->dz_off = ofs; ofs += align64(max_dz);
    net->dcol_off = ofs; ofs += align64(max_dcol);
    net->part_off = ofs; ofs += align64(part);
    net->part_cap = part;
    net->sigma_off = ofs; ofs += align64(n_units);
    net->scale_off = ofs; ofs += align64(n_units);
    net->ws_floats = ofs;
    size_t bytes = (size_t)ofs * sizeof(float);
    net->gram_off_bytes = (int64_t)bytes;
    bytes += (size_t)n_units * kSnSplit * kSnMaxDim * kSnMaxDim * sizeof(double);
    net->bnpart_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up(max_bnpart * (int64_t)sizeof(double), 256);
    net->ticket_off_bytes = (int64_t)bytes;
    net->ticket_bytes = round_up(max_c * (int64_t)sizeof(int), 256);
    bytes += (size_t)net->ticket_bytes;
    net->table_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up((int64_t)(n_units * sizeof(SnConv)), 256);
    net->misc_off_bytes = (int64_t)bytes;
    bytes += 256;
    net->ws_bytes = bytes;
    *out = net;
    return LRS_OK;
}

extern "C" void lrs_dipnet_destroy(lrs_dipnet *net) {
    if (!net) return;
    drop_graph(net);
    delete net;
}

extern "C" int64_t lrs_dipnet_num_params(const lrs_dipnet *net) { return net ? net->n_params : -1; }
extern "C" int64_t lrs_dipnet_num_bnstats(const lrs_dipnet *net) { return net ? net->n_bnstats : -1; }
extern "C" size_t lrs_dipnet_workspace(const lrs_dipnet *net) { return net ? net->ws_bytes : 0; }

extern "C" int lrs_dipnet_param_offsets(const lrs_dipnet *net, int unit, int64_t *w, int64_t *b, int64_t *gamma,
                                        int64_t *beta) {
    if (!net || unit < 0 || unit >= (int)net->units.size()) return LRS_E_INVALID;
    const auto &U = net->units[unit];
    if (w) *w = U.w_off;
    if (b) *b = U.b_off;
    if (gamma) *gamma = U.gm_off;
    if (beta) *beta = U.bt_off;
    return LRS_OK;
}

extern "C" int lrs_dipnet_out_shape(const lrs_dipnet *net, int *C, int *H, int *W) {
    if (!net) return LRS_E_INVALID;
    const auto &L = net->units.back();
    if (C) *C = L.u.cout;
    if (H) *H = L.g.Ho;
    if (W) *W = L.g.Wo;
    return LRS_OK;
}

extern "C" int lrs_dipnet_bind(lrs_dipnet *net, float *params, float *grads, float *adam_m, float *adam_v,
                               float *bnstats, void *ws, size_t ws_bytes) {
    if (!net || !params || !grads || !adam_m || !adam_v || (!bnstats && net->n_bnstats)) return LRS_E_INVALID;
    if (!ws || ws_bytes < net->ws_bytes) return LRS_E_WORKSPACE;
    drop_graph(net);
    net->params = params;
    net->grads = grads;
    net->am = adam_m;
    net->av = adam_v;
    net->bnstats = bnstats;
    net->ws = (char *)ws;
    const int n = (int)net->units.size();
    std::vector<SnConv> tab(n);
    for (int i = 0; i < n; ++i) {
        const auto &U = net->units[i];
        tab[i] = SnConv{params + U.w_off, net->f(U.wn_off), U.u.cout, (int)U.Kc};
    }
    hipError_t e = hipMemcpy(net->table(), tab.data(), sizeof(SnConv) * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) return (int)e;
    e = hipMemset(net->misc_off_bytes + net->ws, 0, 256);
    if (e == hipSuccess) e = hipMemset(net->ticket(), 0, (size_t)net->ticket_bytes);
    return e == hipSuccess ? LRS_OK : (int)e;
}

extern "C" int lrs_dipnet_init_params(lrs_dipnet *net, uint64_t seed, void *stream) {
    if (!net || !net->params) return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    for (size_t i = 0; i < net->units.size(); ++i) {
        const auto &U = net->units[i];
        const float fan_in = (float)U.Kc;
        const float wb = sqrtf(6.0f / fan_in);          // kaiming_uniform_(a=0, mode='fan_in'), gain sqrt(2)
        const float bb = 1.0f / sqrtf(fan_in);          // nn.Conv2d default bias init
        const uint64_t k1 = mix64(seed * 0x100000001b3ULL + 2 * i + 1), k2 = mix64(seed * 0x100000001b3ULL + 2 * i + 2);
        hipLaunchKernelGGL(k_init_uniform, dim3(ew_blocks(U.u.cout * U.Kc)), dim3(kEw), 0, st, net->params + U.w_off,
                           (int64_t)(U.u.cout * U.Kc), wb, k1);
        hipLaunchKernelGGL(k_init_uniform, dim3(1), dim3(kEw), 0, st, net->params + U.b_off, (int64_t)U.u.cout, bb, k2);
        if (U.u.bn) {
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->params + U.gm_off, (int64_t)U.u.cout, 1.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->params + U.bt_off, (int64_t)U.u.cout, 0.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->bnstats + U.rs_off, (int64_t)U.u.cout, 0.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->bnstats + U.rs_off + U.u.cout,
                               (int64_t)U.u.cout, 1.0f);
        }
    }
    hipError_t e = hipMemsetAsync(net->am, 0, sizeof(float) * net->n_params, st);
    if (e == hipSuccess) e = hipMemsetAsync(net->av, 0, sizeof(float) * net->n_params, st);
    if (e == hipSuccess) e = hipMemsetAsync(net->grads, 0, sizeof(float) * net->n_params, st);
    if (e == hipSuccess) e = hipMemsetAsync(net->ws + net->misc_off_bytes, 0, 256, st);
    if (e != hipSuccess) return (int)e;
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_dipnet_reset_optimizer(lrs_dipnet *net, void *stream) {
    if (!net || !net->ws) return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(net->am, 0, sizeof(float) * net->n_params, st);
    if (e == hipSuccess) e = hipMemsetAsync(net->av, 0, sizeof(float) * net->n_params, st);
    if (e == hipSuccess) e = hipMemsetAsync(net->ws + net->misc_off_bytes, 0, 256, st);
    return e == hipSuccess ? LRS_OK : (int)e;
}

extern "C" int lrs_dipnet_forward(lrs_dipnet *net, const float *x, void *stream) {
    if (!net || !net->ws || !x) return LRS_E_INVALID;
    return dipnet_forward(net, x, (hipStream_t)stream);
}

extern "C" const float *lrs_dipnet_output(const lrs_dipnet *net) {
    return (net && net->ws) ? net->f(net->units.back().act_off) : nullptr;
}

extern "C" const float *lrs_dipnet_grads(const lrs_dipnet *net) { return net ? net->grads : nullptr; }

extern "C" int lrs_dipnet_train_steps(lrs_dipnet *net, const float *x, const float *target, const float *mask,
                                      float lr, float beta1, float beta2, float eps, lrs_es_state *es, float *ring,
                                      int nsteps, int use_graph, void *stream) {
    if (!net || !net->ws || !x || !target || nsteps < 0 || (es && !ring)) return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (!use_graph) {
        for (int s = 0; s < nsteps; ++s) {
            const int rc = dipnet_step(net, x, target, mask, lr, beta1, beta2, eps, es, ring, st);
            if (rc) return rc;
        }
        return LRS_OK;
    }
    if (!st) return LRS_E_INVALID;   // capture needs a non-default stream
    const lrs_dipnet::Key k{x, target, mask, es, ring, lr, beta1, beta2, eps};
    if (!net->have_key || memcmp(&k, &net->key, sizeof(k)) != 0) {
        drop_graph(net);
        hipError_t e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
        if (e != hipSuccess) return (int)e;
        const int rc = dipnet_step(net, x, target, mask, lr, beta1, beta2, eps, es, ring, st);
        hipGraph_t g = nullptr;
        e = hipStreamEndCapture(st, &g);
        if (rc) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        if (e != hipSuccess) return (int)e;
        e = hipGraphInstantiate(&net->gexec, g, nullptr, nullptr, 0);
        if (e != hipSuccess) {
            (void)hipGraphDestroy(g);
            return (int)e;
        }
        net->graph = g;
        net->key = k;
        net->have_key = true;
    }
    for (int s = 0; s < nsteps; ++s) {
        const hipError_t e = hipGraphLaunch(net->gexec, st);
        if (e != hipSuccess) return (int)e;
    }
    return LRS_OK;
}

extern "C" int lrs_dipnet_last_loss(lrs_dipnet *net, double *loss, void *stream) {
    if (!net || !net->ws || !loss) return LRS_E_INVALID;
    double acc = 0.0;
    hipError_t e = hipMemcpyAsync(&acc, net->loss_acc(), sizeof(double), hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
    const auto &L = net->units.back();
    *loss = acc / ((double)L.u.cout * (double)L.P);
    return LRS_OK;
}
