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

#include <algorithm>
#include <new>
#include <vector>

#include "dip_kernels.h"
#include "dip_gemm.h"
#include "dip_sm.h"
#include "dip_dir.h"

using namespace lrs;

namespace {

constexpr int kEw = 256;   // elementwise block size
constexpr int64_t kForkBigP = 9604;   // sigma beside the first conv: only where that conv's map is >= 98^2

// A/B tuning knobs.  The environment is read only by the tuning build (make TUNING=1 ->
// liblrspnp_hip_tune.so, -DLRS_TUNING); the product library always takes the default, so a
// variable left set on a production box cannot change its arithmetic path.
inline int64_t tune_knob(const char *name, int64_t dflt) {
#ifdef LRS_TUNING
    const char *e = getenv(name);
    return e ? atoll(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}
inline const char *tune_str(const char *name) {
#ifdef LRS_TUNING
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

inline unsigned ew_blocks(int64_t n, int64_t cap = 4096) {
    int64_t b = (n + kEw - 1) / kEw;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

// the defaults of a NULL lrs_dip_opts
inline lrs_dip_opts dip_opts(const lrs_dip_opts *o) {
    lrs_dip_opts d{};
    d.precision = LRS_DIP_SPLIT_BF16;
    d.upsample_dgrad = 0;
    return o ? *o : d;
}

int make_geom(int Cin, int H, int W, int k, int stride, int pad, int pad_mode, int up, ConvGeom &g,
              const lrs_dip_opts *opts = nullptr) {
    const lrs_dip_opts o = dip_opts(opts);
    if (o.precision != LRS_DIP_F32 && o.precision != LRS_DIP_SPLIT_BF16) return LRS_E_INVALID;
    if (o.upsample_dgrad != 0 && o.upsample_dgrad != 1) return LRS_E_INVALID;
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
    g.prec = o.precision;
    // effective kernel of the upsampled data gradient as a stride-2 conv on the source grid
    g.ke = 0;
    if (o.upsample_dgrad && g.up && g.stride == 1 && g.Hs >= 2 && g.Ws >= 2) {
        if (g.k == 3 && g.pad == 1) g.ke = 4;
        if (g.k == 2 && g.pad == 0) g.ke = 3;
    }
    return LRS_OK;
}

inline bool plain_unit(const ConvGeom &g) { return g.k == 1 && g.stride == 1 && g.pad == 0 && !g.up; }

struct Split {
    int S, kchunk;
    bool big;   // 128x128 tiles (k_gemm) or 64x64 (k_gemm64)
};

// Tile choice and split-K: 128x128 tiles when they alone give >= 64 workgroups, else 64x64;
// then split K until ~512 workgroups (2 per CU), keeping >= 128 of K per split and <= 64 splits.
// (Measured with the f32 kernels: 128-tiles with deeper split-K on the small-N weight-gradient
// GEMMs, or a 1024-WG target, are slower at both the 36x36 and the 196x196 sizes.)
Split choose_split(int M, int N, int K, int precision = LRS_DIP_SPLIT_BF16, bool force_big = false, int target = 512) {
    const int64_t t128 = (int64_t)((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
    // long-K GEMMs (the weight gradients, K = pixels) take 128-tiles with deep split-K on the
    // split-bf16 path when that still gives >= 256 workgroups (measured 25-30 % faster at 196^2 and
    // 512^2; the 1x1 layer's 2-tile gradient is faster on 64-tiles)
    // Very long K with few tiles (a 1x1 conv's weight gradient over 512^2 pixels) splits up to 256
    // ways on the split-bf16 path, keeping >= 16 k-steps per workgroup.
    const bool deep = precision == LRS_DIP_SPLIT_BF16 && K >= 65536;
    const bool big = force_big || t128 >= 64 || (precision == LRS_DIP_SPLIT_BF16 && K >= 8192 && t128 >= 4) || deep;
    const int64_t tiles = big ? t128 : (int64_t)((M + kBM64 - 1) / kBM64) * ((N + kBN64 - 1) / kBN64);
    int S = 1;
    // split-K below this many tiles (LRS_DIP_SPLIT_MIN_TILES, tuning only)
    static const int64_t min_tiles = tune_knob("LRS_DIP_SPLIT_MIN_TILES", 256);
    if (tiles < min_tiles) {
        S = (int)((target + tiles - 1) / tiles);   // ~2 workgroups per CU (256 and 1024 measured slower)
        const int smax = deep ? K / 512 : (K + 127) / 128;
        if (S > smax) S = smax;
        // at most 64 splits otherwise (LRS_DIP_SPLIT_CAP, tuning only; 196^2 step, 2 rounds:
        // 32 -> 1.327 ms, 64 -> 1.265, 128 -> 1.279, 256 -> 1.285; profiles/r04/split_cap/)
        static const int cap = (int)std::max<int64_t>(1, tune_knob("LRS_DIP_SPLIT_CAP", 64));
        if (S > (deep ? 256 : cap)) S = deep ? 256 : cap;
        if (S < 1) S = 1;
    }
    const int bk = (big && precision == LRS_DIP_SPLIT_BF16) ? kBK32 : kBK;
    int kchunk = (int)round_up((K + S - 1) / S, bk);
    if (kchunk < bk) kchunk = bk;
    S = (K + kchunk - 1) / kchunk;
    if (S < 1) S = 1;
    return {S, kchunk, big};
}

// split-K scratch of an implicit-GEMM conv product (always 128-tiles, split-bf16)
int64_t s3_part_floats(int M, int N, int K) {
    const Split s = choose_split(M, N, K, LRS_DIP_SPLIT_BF16, true);
    return s.S > 1 ? (int64_t)s.S * M * N : 0;
}

int64_t gemm_part_floats(int M, int N, int K) {
    // sized for both precisions, so that the precision can change after a workspace was sized
    const Split a = choose_split(M, N, K, LRS_DIP_F32), b = choose_split(M, N, K, LRS_DIP_SPLIT_BF16);
    const int S = std::max(a.S, b.S);
    return S > 1 ? (int64_t)S * M * N : 0;
}

// C = op(A) op(B) (+ bias) (/ *div); part: split-K scratch (>= gemm_part_floats); prec: the
// conv's ConvGeom::prec
int gemm(int prec, int TA, int TB, const float *A, const float *B, float *C, const float *bias, const float *div, int M,
         int N, int K, float *part, int64_t part_cap, hipStream_t st, int accum = 0, int *nsplit_out = nullptr,
         bool force_big = false, int target = 512) {
    if (M <= 0 || N <= 0) return LRS_OK;
    const Split s = choose_split(M, N, K, prec, force_big, target);
    if (nsplit_out) *nsplit_out = s.S;   // > 1: the caller finishes the split-K sum (no reduce here)
    GemmArgs g{A, B, C, bias, div, M, N, K, s.kchunk, accum};
    if (s.S > 1) {
        if (!part || part_cap < (int64_t)s.S * M * N) return LRS_E_WORKSPACE;
        g.C = part;
    }
    if (s.big && prec == LRS_DIP_SPLIT_BF16) {
        dim3 grid((N + kBN - 1) / kBN, (M + kBM - 1) / kBM, s.S);
        const int lda = TA ? M : K, ldb = TB ? K : N;
        if (!TA && !TB)
            hipLaunchKernelGGL((k_gemm_s3<LdDense<true>, LdDense<false>>), grid, dim3(kGemmThreads), 0, st, g,
                               LdDense<true>{A, lda, M}, LdDense<false>{B, ldb, N});
        else if (!TA && TB)
            hipLaunchKernelGGL((k_gemm_s3<LdDense<true>, LdDense<true>>), grid, dim3(kGemmThreads), 0, st, g,
                               LdDense<true>{A, lda, M}, LdDense<true>{B, ldb, N});
        else if (TA && !TB)
            hipLaunchKernelGGL((k_gemm_s3<LdDense<false>, LdDense<false>>), grid, dim3(kGemmThreads), 0, st, g,
                               LdDense<false>{A, lda, M}, LdDense<false>{B, ldb, N});
        else
            hipLaunchKernelGGL((k_gemm_s3<LdDense<false>, LdDense<true>>), grid, dim3(kGemmThreads), 0, st, g,
                               LdDense<false>{A, lda, M}, LdDense<true>{B, ldb, N});
    } else if (s.big) {
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
    if (s.S > 1 && !nsplit_out) {
        const int64_t MN = (int64_t)M * N;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((MN + kEw - 1) / kEw)), dim3(kEw), 0, st, part, s.S, M,
                           N, bias, div, accum, C);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

inline int r16(int x) { return (x + 15) & ~15; }

// Data gradient of an upsampled stride-1 conv (the U-Net's up_1..up_4: nearest x2, then 2 x 2 unpadded
// or reflection-padded 3 x 3) as a stride-2 conv over dL/dz with a (k+1) x (k+1) effective kernel on
// the source grid (conv_bwd): 2.25x fewer products than correlating over the padded upsampled domain
// and folding.  Returns k + 1, or 0 where the identity is not used.
// Off by default: measured in the whole 196^2 training step (bench configs[2], 2 x 2 A/B runs) it is
// ~1 % slower than the padded-domain correlation + fold -- the up_4 data-gradient work it saves ran
// beside that layer's weight gradient anyway, and it adds a split-K reduce and the border launches
// to the critical chain.  lrs_dip_opts::upsample_dgrad = 1 selects it (tests cover both).
// An upsampled, reflection-padded 3 x 3 stride-1 conv runs by output parity class in the network
// engine (dip_gemm.h LdUpFwdTM / LdUpDgradTM, 4/9 of the direct products).  LRS_DIP_UPC=0 keeps the
// direct implicit GEMM over the upsampled grid (A/B only).
inline bool upc_conv(const ConvGeom &g) {
    static const bool on = tune_knob("LRS_DIP_UPC", 1) != 0;
    return on && g.up && g.k == 3 && g.pad == 1 && g.pad_mode == LRS_PAD_REFLECT && g.stride == 1 && g.Hs >= 2 &&
           g.Ws >= 2;
}

// fixed with the geometry (make_geom, lrs_dip_opts::upsample_dgrad): the workspace size, the
// weight-preparation table and the backward all read this one value
inline int up_eff_k(const ConvGeom &g) { return g.ke; }
// ---- small-map convs on k_conv_sm (dip_sm.h) ------------------------------------------------
// A conv runs there when it is not 1x1, k <= 3 and its output map is below implicit_min_pixels()
// (the maps that had the explicit im2col path).  LRS_DIP_SM=0 keeps the explicit path (A/B only).
inline bool sm_enabled() {
    static const bool v = tune_knob("LRS_DIP_SM", 1) != 0;
    return v;
}

// 64 x 64 tiles; split K so that the grid has ~sm_target() workgroups (k per split a multiple of
// 64).  LRS_DIP_SM_WG overrides the target (tuning only).
inline int64_t sm_target() {
    static const int64_t v = std::max<int64_t>(1, tune_knob("LRS_DIP_SM_WG", 640));
    return v;
}
Split sm_split(int M, int N, int K) {
    const int64_t T = (int64_t)((M + 63) / 64) * ((N + 63) / 64), W = sm_target();
    int64_t kc = round_up(std::max<int64_t>(1, ((int64_t)K * T + W - 1) / W), kSmK);
    if (kc > K) kc = round_up(K, kSmK);
    int S = (int)((K + kc - 1) / kc);
    kc = round_up((K + S - 1) / S, kSmK);
    S = (int)((K + kc - 1) / kc);
    return {S, (int)kc, false};
}

int64_t sm_part_floats(int M, int N, int K) {
    const Split s = sm_split(M, N, K);
    return s.S > 1 ? (int64_t)s.S * M * N : 0;
}

// C (+)= A B (+ bias) (/ *div) on k_conv_sm; split-K partials summed by k_gemm_reduce unless
// nsplit_out is given (the caller then finishes the sum, e.g. k_reduce_bn1); one_launch: no split
template <class LB, class LA = SmPre>
int sm_launch(const LA &la, const LB &lb, float *C, const float *bias, int M, int N, int K, int accum, float *part,
              int64_t part_cap, hipStream_t st, int *nsplit_out = nullptr, const float *div = nullptr,
              bool one_launch = false) {
    if (M <= 0 || N <= 0) return LRS_OK;
    Split s = sm_split(M, N, K);
    if (one_launch) s = {1, (int)round_up(K, kSmK), false};
    if (nsplit_out) *nsplit_out = s.S;
    GemmArgs g{nullptr, nullptr, C, bias, div, M, N, K, s.kchunk, accum};
    if (s.S > 1) {
        if (!part || part_cap < (int64_t)s.S * M * N) return LRS_E_WORKSPACE;
        g.C = part;
    }
    hipLaunchKernelGGL((k_conv_sm<LB, LA>), dim3((N + 63) / 64, (M + 63) / 64, s.S), dim3(256), 0, st, g, la, lb);
    if (s.S > 1 && !nsplit_out) {
        const int64_t MN = (int64_t)M * N;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((MN + kEw - 1) / kEw)), dim3(kEw), 0, st, part, s.S, M, N,
                           bias, div, accum, C);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// The weight-gradient gather table of a small-map conv: for tap t and output pixel p, the byte
// offset within a source channel plane of the value col[(c, t)][p] reads (kOob = zero pad); [kk][P]
std::vector<int> sm_wgrad_table(const ConvGeom &g) {
    const int kk = g.k * g.k, P = g.Ho * g.Wo;
    std::vector<int> t((size_t)kk * P, kOob);
    for (int kyx = 0; kyx < kk; ++kyx)
        for (int p = 0; p < P; ++p) {
            const int oy = p / g.Wo, ox = p - oy * g.Wo, ky = kyx / g.k, kx = kyx - ky * g.k;
            const int sy = conv_src(oy * g.stride + ky - g.pad, g.Hu, g.pad_mode, g.up);
            const int sx = conv_src(ox * g.stride + kx - g.pad, g.Wu, g.pad_mode, g.up);
            if (sy >= 0 && sx >= 0) t[(size_t)kyx * P + p] = 4 * (sy * g.Ws + sx);
        }
    return t;
}

// A small-map weight gradient on the side stream runs as one implicit k_conv_sm launch (no
// k_im2col, no split-K, no reduce) up to this many output pixels; above it the explicit col +
// split-K GEMM + reduce is faster (at 36^2: 18^2 maps 34 us one launch vs ~15 us for the three; the
// split-K implicit form 22 vs ~20 us).  196^2 step (13^2 maps, side stream) 1.275 -> 1.263 ms; on the
// single stream of a 36^2 net (no fork) 0.726 -> 0.735 ms, so it is used only where the net forks.
constexpr int kSmWgradOneLaunchP = 200;

// The data-gradient gather table of a small-map conv: for tap (ty, tx) and input pixel q, the
// byte offsets (within a dL/dz plane) of the <= 2 x 2 output pixels that read q through it (the
// products of the per-dimension lists), kOob-padded; [kk][Q] int4.  Empty where sm_adj_dim fails.
std::vector<int> sm_adj_table(const ConvGeom &g);

// The conv's adjoint along one dimension: for tap t and source coordinate q, the output
// coordinates o with src(o, t) = q (reflection / zero pad, stride, x2 upsample), in increasing
// order, at most 2 (-1 = none).  False where some list would need more (the caller then keeps the
// explicit data gradient).
bool sm_adj_dim(int n_src, int n_up, int n_out, int k, int stride, int pad, int mode, int up, short *L) {
    for (int i = 0; i < k * n_src * 2; ++i) L[i] = -1;
    for (int o = 0; o < n_out; ++o)
        for (int t = 0; t < k; ++t) {
            const int q = conv_src(o * stride + t - pad, n_up, mode, up);
            if (q < 0) continue;
            short *e = L + (t * n_src + q) * 2;
            if (e[0] < 0) e[0] = (short)o;
            else if (e[1] < 0) e[1] = (short)o;
            else return false;
        }
    return true;
}

std::vector<int> sm_adj_table(const ConvGeom &g) {
    std::vector<short> Ly((size_t)2 * g.k * g.Hs), Lx((size_t)2 * g.k * g.Ws);
    if (!sm_adj_dim(g.Hs, g.Hu, g.Ho, g.k, g.stride, g.pad, g.pad_mode, g.up, Ly.data()) ||
        !sm_adj_dim(g.Ws, g.Wu, g.Wo, g.k, g.stride, g.pad, g.pad_mode, g.up, Lx.data()))
        return {};
    const int Q = g.Hs * g.Ws;
    std::vector<int> t((size_t)4 * g.k * g.k * Q, kOob);
    for (int ty = 0; ty < g.k; ++ty)
        for (int tx = 0; tx < g.k; ++tx)
            for (int q = 0; q < Q; ++q) {
                const int qy = q / g.Ws, qx = q % g.Ws;
                int *e = t.data() + 4 * ((int64_t)(ty * g.k + tx) * Q + q);
                for (int a = 0; a < 2; ++a)
                    for (int b = 0; b < 2; ++b) {
                        const int oy = Ly[(ty * g.Hs + qy) * 2 + a], ox = Lx[(tx * g.Ws + qx) * 2 + b];
                        if (oy >= 0 && ox >= 0) e[2 * a + b] = 4 * (oy * g.Wo + ox);
                    }
            }
    return t;
}

int64_t conv_part_floats(const ConvGeom &g, int Cout) {
    const int P = g.Ho * g.Wo, kk = g.k * g.k, Kc = g.Cin * kk;
    int64_t m = gemm_part_floats(Cout, P, Kc);                       // forward
    const int64_t b = gemm_part_floats(Cout, Kc, P);                 // dW
    const int64_t c = gemm_part_floats(Kc, P, Cout);                 // dcol
    if (b > m) m = b;
    if (c > m) m = c;
    // implicit forms (tap-major K, channels rounded up to 16)
    m = std::max(m, std::max(s3_part_floats(Cout, P, kk * r16(g.Cin)), s3_part_floats(Cout, Kc, P)));
    const int Qp = (g.Hu + 2 * g.pad) * (g.Wu + 2 * g.pad);
    m = std::max(m, s3_part_floats(g.Cin, Qp, kk * r16(Cout)));
    if (const int ke = up_eff_k(g)) m = std::max(m, s3_part_floats(g.Cin, g.Hs * g.Ws, ke * ke * r16(Cout)));
    m = std::max(m, std::max(sm_part_floats(Cout, P, kk * r16(g.Cin)), sm_part_floats(g.Cin, g.Hs * g.Ws, kk * r16(Cout))));
    m = std::max(m, sm_part_floats(Cout, Kc, P));   // the small-map weight gradient (SmWgrad)
    return m;
}

// split-K scratch of a parity-class conv (network engine only): forward partials over the whole
// output, the data gradient over the extended source grid, the weight gradient [split][cls][Cout][4 Cin]
int64_t upc_part_floats(const ConvGeom &g, int Cout) {
    const int64_t P = (int64_t)g.Ho * g.Wo;
    int64_t m = 0;
    const Split f = choose_split(Cout, 4 * g.Hs * g.Ws, 4 * r16(g.Cin), LRS_DIP_SPLIT_BF16, true);
    if (f.S > 1) m = (int64_t)f.S * Cout * P;
    m = std::max(m, s3_part_floats(g.Cin, (g.Hs + 2) * (g.Ws + 2), 16 * r16(Cout)));
    const Split w = choose_split(Cout, 16 * g.Cin, g.Hs * g.Ws, LRS_DIP_SPLIT_BF16, true);
    return std::max(m, (int64_t)w.S * 16 * Cout * g.Cin);
}

// bf16 elements of a conv's pre-split weight planes: forward operand WF [3][Cout][kk*Cp], then
// the data-gradient operand WD [3][Cin][kk*Cop]
// planes of the parity-class forward (WUF) / data gradient (WUD) when upc, else WF / WD (WE)
inline int64_t wprep_fwd_elems(const ConvGeom &g, int Cout, bool upc = false) {
    return 3 * (int64_t)Cout * (upc ? 16 : g.k * g.k) * r16(g.Cin);
}
inline int64_t wprep_elems(const ConvGeom &g, int Cout, bool upc) {
    return wprep_fwd_elems(g, Cout, true) + 3 * (int64_t)g.Cin * 16 * r16(Cout);
}
inline int64_t wprep_elems(const ConvGeom &g, int Cout) {
    const int ke = up_eff_k(g);
    return wprep_fwd_elems(g, Cout) + 3 * (int64_t)g.Cin * (ke ? ke * ke : g.k * g.k) * r16(Cout);
}

// Implicit-GEMM conv product on the split-bf16 kernel, with the same split-K / reduce tail as
// gemm().
// split-K workgroup target of a forward conv whose partials a fused BN kernel finishes: fewer
// splits than the GEMMs' 512 (the BN kernel, one workgroup per channel, re-reads every partial):
// 196^2 step 1.336 -> 1.312 ms at 384 (A/B on one box: 256 1.317, 320 1.313).  The workspace is
// sized for 512, so a larger LRS_DIP_FWD_SPLIT_WG (tuning only) fails with LRS_E_WORKSPACE.
inline int fwd_split_target() {
    static const int v = (int)std::max<int64_t>(1, tune_knob("LRS_DIP_FWD_SPLIT_WG", 384));
    return v;
}

// Split target of the padded-domain data-gradient GEMMs whose split-K partials k_fold_pad sums
// (every partial is re-read by the fold, as by the forward BN kernels above).
inline int dgrad_split_target() {
    static const int v = (int)std::max<int64_t>(1, std::min<int64_t>(512, tune_knob("LRS_DIP_DGRAD_SPLIT_WG", 512)));
    return v;
}

template <class LA, class LB>
int gemm_s3_conv(const LA &la, const LB &lb, float *C, const float *bias, const float *div, int M, int N, int K,
                 float *part, int64_t part_cap, hipStream_t st, int *nsplit_out = nullptr, int accum = 0,
                 int target = 512) {
    if (M <= 0 || N <= 0) return LRS_OK;
    const Split s = choose_split(M, N, K, LRS_DIP_SPLIT_BF16, true, target);
    if (nsplit_out) *nsplit_out = s.S;
    GemmArgs g{nullptr, nullptr, C, bias, div, M, N, K, s.kchunk, accum};
    if (s.S > 1) {
        if (!part || part_cap < (int64_t)s.S * M * N) return LRS_E_WORKSPACE;
        g.C = part;
    }
    dim3 grid((N + 127) / 128, (M + 127) / 128, s.S);
    hipLaunchKernelGGL((k_gemm_s3<LA, LB>), grid, dim3(kGemmThreads), 0, st, g, la, lb);
    if (s.S > 1 && !nsplit_out) {
        const int64_t MN = (int64_t)M * N;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((MN + kEw - 1) / kEw)), dim3(kEw), 0, st, part, s.S, M, N,
                           bias, div, accum, C);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// Forward of an upsampled 3 x 3 conv by output parity class: one launch, gridDim.z = 4 classes x
// split-K; y (or the split-K partials) over the whole output.  wpre = the WUF planes.
int upc_fwd(const ConvGeom &g, const float *x, const __bf16 *wpre, const float *bias, int Cout, float *y, float *part,
            int64_t part_cap, hipStream_t st, int *nsplit_out) {
    const int Cp = r16(g.Cin), Q = g.Hs * g.Ws, K = 4 * Cp;
    const int64_t P = (int64_t)g.Ho * g.Wo;
    const Split s = choose_split(Cout, 4 * Q, K, LRS_DIP_SPLIT_BF16, true, nsplit_out ? fwd_split_target() : 512);
    if (nsplit_out) *nsplit_out = s.S;
    GemmArgs a{nullptr, nullptr, y, bias, nullptr, Cout, Q, K, s.kchunk, 0, 4, g.Ws, g.Wo, P};
    if (s.S > 1) {
        if (!part || part_cap < (int64_t)s.S * Cout * P) return LRS_E_WORKSPACE;
        a.C = part;
    }
    const dim3 grid((Q + 127) / 128, (Cout + 127) / 128, 4 * s.S);
    hipLaunchKernelGGL((k_gemm_s3<LdPre, LdUpFwdTM>), grid, dim3(kGemmThreads), 0, st, a,
                       LdPre{wpre, (int64_t)4 * Cout * K, K, Cout, (int64_t)Cout * K},
                       LdUpFwdTM{x, g.Cin * Q * 4, g, Cp, nullptr});
    if (s.S > 1 && !nsplit_out)
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((Cout * P + kEw - 1) / kEw)), dim3(kEw), 0, st, part, s.S,
                           Cout, (int)P, bias, nullptr, 0, y);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// Its data gradient: gxe over the source grid extended by one pixel (one GEMM with K = 4 classes x
// 4 effective taps x Cout, into the scratch gxe), then k_fold_pad in kPadClamp mode adds the outside
// ring onto the border pixels (gx += when accum).  wd = the WUD planes.
int upc_dgrad(const ConvGeom &g, const float *gz, const __bf16 *wd, int Cout, float *gx, float *gxe, float *part,
              int64_t part_cap, hipStream_t st, int accum) {
    const int Cop = r16(Cout), K = 16 * Cop, Qe = (g.Hs + 2) * (g.Ws + 2);
    int nsplit = 1;   // split-K partials are summed inside the fold
    int rc = gemm_s3_conv(LdPre{wd, (int64_t)g.Cin * K, K, g.Cin}, LdUpDgradTM{gz, Cout * g.Ho * g.Wo * 4, g, Cout, Cop, nullptr},
                          gxe, nullptr, nullptr, g.Cin, Qe, K, part, part_cap, st, &nsplit, 0,
                          dgrad_split_target());
    if (rc) return rc;
    ConvGeom fg = g;
    fg.up = 0;
    fg.Hu = g.Hs;
    fg.Wu = g.Ws;
    fg.pad = 1;
    fg.pad_mode = kPadClamp;
    const dim3 grid((unsigned)((g.Hs * g.Ws + 255) / 256), (unsigned)std::min(g.Cin, 65535));
    hipLaunchKernelGGL(k_fold_pad, grid, dim3(256), 0, st, nsplit > 1 ? part : gxe, nsplit, (int64_t)g.Cin * Qe, fg, gx,
                       accum);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// Its weight gradient: per class dWE_cls = dL/dz(class pixels) x col_cls^T (one launch, classes and
// split-K over gridDim.z, partials [split][cls][Cout][4 Cin] in part), then k_upc_wgrad_combine sums
// splits and classes into dW (/ *div).
int upc_wgrad(const ConvGeom &g, const float *gz, const float *x, const float *div, int Cout, float *gw, float *part,
              int64_t part_cap, hipStream_t st, int target = 512) {
    const int Q = g.Hs * g.Ws, N = 4 * g.Cin;
    const Split s = choose_split(Cout, 4 * N, Q, LRS_DIP_SPLIT_BF16, true, target);
    if (!part || part_cap < (int64_t)s.S * 4 * Cout * N) return LRS_E_WORKSPACE;
    const GemmArgs a{nullptr, nullptr, part, nullptr, nullptr, Cout, N, Q, s.kchunk, 0, 4, g.Ws, 0, 0};
    const dim3 grid((N + 127) / 128, (Cout + 127) / 128, 4 * s.S);
    hipLaunchKernelGGL((k_gemm_s3<LdGzCls, LdWgradCls>), grid, dim3(kGemmThreads), 0, st, a,
                       LdGzCls{gz, g.Hs, g.Ws, g.Wo, Cout, 0}, LdWgradCls{x, g.Cin * Q * 4, g, nullptr, 0, 0});
    const int64_t n = (int64_t)Cout * g.Cin * 9;
    hipLaunchKernelGGL(k_upc_wgrad_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, s.S, Cout, g.Cin,
                       div, gw);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// implicit GEMM: k <= 3 (LDS tables) and both operand tensors addressable by 32-bit buffer offsets
inline bool conv_implicit_ok(const ConvGeom &g, int Cout) {
    return g.k <= 3 && (int64_t)g.Cin * g.Hs * g.Ws * 4 < kOob && (int64_t)Cout * g.Ho * g.Wo * 4 < kOob;
}

// The engine runs a conv as an implicit GEMM from this many output pixels up; below it the maps
// are small enough that an explicit im2col into a cached col buffer plus the 64-tile GEMMs is
// faster (round 1, at 36x36: 1.23 vs 1.41 ms per U-Net step).  Round 4 re-measured the kernels of
// today: 2048 -> 1024 moves the 36^2 maps (1296 pixels) to the implicit paths, 36^2 step 0.652 ->
// 0.638 ms, and the skip net's 32^2 maps, 512^2 step 9.27 -> 9.23 ms; 512 (the 196^2 net's 25^2 maps
// too) is slower there, 1.244 -> 1.288 ms (profiles/r04/implicit_min_p/).
// LRS_DIP_IMPLICIT_MIN_P overrides (tuning only).
inline int64_t implicit_min_pixels() {
    static const int64_t v = tune_knob("LRS_DIP_IMPLICIT_MIN_P", 1024);
    return v;
}

// split w into the bf16 planes of the forward operand (and of the data-gradient one if wd)
int wprep(const ConvGeom &g, const float *w, int Cout, __bf16 *wf, __bf16 *wd, hipStream_t st) {
    const int kk = g.k * g.k;
    if (wprep_elems(g, Cout) >= INT32_MAX / 3) return LRS_E_UNSUPPORTED;   // k_conv_prep's 32-bit indices
    const int64_t n = wprep_elems(g, Cout) / 3;
    const ConvPrep c{w, nullptr, wf, wd, Cout, g.Cin, kk, r16(g.Cin), r16(Cout), -1, g.k, wd ? up_eff_k(g) : 0};
    hipLaunchKernelGGL(k_conv_prep1, dim3(ew_blocks(n, 2048)), dim3(256), 0, st, c);
    return LRS_OK;
}

// LRS_DIP_PW_NB = the allowed NB digits, e.g. "4" keeps 64-pixel workgroups everywhere (A/B only)
inline bool pw_nb_allowed(int nb) {
    static const char *v = tune_str("LRS_DIP_PW_NB");
    return !v || strchr(v, '0' + nb) != nullptr;
}

// k_pw instantiations: MT row blocks x NB 16-pixel column blocks, and the workgroups per CU their
// registers allow (one wave per SIMD each; gfx950: 512 VGPRs per SIMD lane over the waves, in
// granules of 8; the counts of the current build: 80, 150, 192, 234, 198).  48-pixel workgroups
// (NB = 3) for the LDS-bound K = 198 data gradient measured ~10 us per 196^2 step slower (A/B,
// LRS_DIP_PW_NB) and were dropped.
struct PwKernel {
    int mt, nb, wg_per_cu;
    void (*fn)(PwArgs);
};
static const PwKernel kPwKernels[] = {
    {1, 4, 6, k_pw<1, 4>}, {2, 4, 3, k_pw<2, 4>}, {3, 4, 2, k_pw<3, 4>}, {4, 4, 2, k_pw<4, 4>}, {4, 5, 2, k_pw<4, 5>},
};

// Pointwise conv product on k_pw (A: pre-split planes [3][M][lda], B: [K][N] fp32).
// The pixel width of a workgroup is chosen per launch: the fewest rounds of the CU slots (LDS
// 3 x 16 NB x ldsrow bytes and the registers both limit them) times the per-workgroup work (NB),
// wider on ties.  At 196^2 the 198-row last 1x1 runs on 80 pixels: 481 workgroups, one round of
// 2 per CU instead of 1.2 rounds at 64 (A/B: -10 us per step).
struct PwHead {   // the fused masked-MSE head of a network's last conv (PwArgs::tgt)
    const float *tgt, *msk;
    float *gz;
    double *hpart;
    float norm;
    int *nwg_out;   // the grid the launch used (k_head_reduce's partial count)
};

int pw_launch(const __bf16 *A, int64_t pstride, int lda, int M, const float *B, int K, int64_t N, float *C,
              const float *bias, int accum, hipStream_t st, int act = 0, const PwHead *head = nullptr) {
    if (M <= 0 || N <= 0) return LRS_OK;
    if (M > 256 || lda < K || lda % 16) return LRS_E_UNSUPPORTED;
    const int Kp32 = (int)round_up(lda, 32), ldsrow = pw_ldsrow(Kp32);
    static std::atomic<uint64_t> attr_set[sizeof(kPwKernels) / sizeof(kPwKernels[0])];   // per device
    for (size_t i = 0; i < sizeof(kPwKernels) / sizeof(kPwKernels[0]); ++i)   // up to K = 256: 3 x 80 x 528 B
        if (const int rc = lds_opt_in((const void *)kPwKernels[i].fn, 3 * 80 * pw_ldsrow(256), attr_set[i])) return rc;
    if (Kp32 > 256 || (int64_t)K * N * 4 >= kOob || 3 * pstride * 2 >= kOob) return LRS_E_UNSUPPORTED;
    static const int dbg = (int)tune_knob("LRS_PW_DBG", 0);
    const PwArgs a{A, pstride, lda, B, K, N, C, bias, M, Kp32, ldsrow, accum, dbg, act};
    const int mt = (M + 63) / 64;
    const PwKernel *best = nullptr;
    int64_t best_cost = 0;
    for (const PwKernel &k : kPwKernels) {
        if (k.mt != mt || !pw_nb_allowed(k.nb)) continue;
        const int lds = 3 * 16 * k.nb * ldsrow;
        const int per_cu = std::min(k.wg_per_cu, (160 * 1024) / lds);
        const int64_t wgs = (N + 16 * k.nb - 1) / (16 * k.nb);
        const int64_t rounds = (wgs + 256 * per_cu - 1) / (256 * per_cu);
        const int64_t cost = rounds * k.nb;
        if (!best || cost < best_cost || (cost == best_cost && k.nb > best->nb)) {
            best = &k;
            best_cost = cost;
        }
    }
    if (!best) return LRS_E_UNSUPPORTED;
    const int npx = 16 * best->nb;
    PwArgs ah = a;
    if (head) {
        ah.tgt = head->tgt;
        ah.msk = head->msk;
        ah.gz = head->gz;
        ah.hpart = head->hpart;
        ah.hnorm = head->norm;
        *head->nwg_out = (int)((N + npx - 1) / npx);
    }
    hipLaunchKernelGGL(best->fn, dim3((unsigned)((N + npx - 1) / npx)), dim3(256), 3 * npx * ldsrow, st, ah);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

inline bool pw_ok(const ConvGeom &g, int Cout) { return plain_unit(g) && Cout <= 256 && r16(g.Cin) <= 256 && r16(Cout) <= 256; }

// y = conv(x) + bias.  Explicit (col != NULL): im2col + GEMM.  Implicit (col == NULL, wpre =
// the weight planes from wprep): tap-major implicit GEMM.
// act_pw: activation for the pointwise kernel's epilogue (a 1x1 conv without BN), applied only there.
int conv_fwd(const ConvGeom &g, const float *x, const float *w, const float *bias, int Cout, float *col, float *y,
             float *part, int64_t part_cap, hipStream_t st, const __bf16 *wpre = nullptr, int *nsplit_out = nullptr,
             int act_pw = 0, const PwHead *head = nullptr) {
    const int P = g.Ho * g.Wo, Kc = g.Cin * g.k * g.k;
    if (nsplit_out) *nsplit_out = 1;
    const float *B = x;
    if (plain_unit(g) && wpre)      // 1x1: pointwise kernel on the pre-split weights
        return pw_launch(wpre, (int64_t)Cout * r16(g.Cin), r16(g.Cin), Cout, x, g.Cin, P, y, bias, 0, st, act_pw, head);
    if (head) return LRS_E_UNSUPPORTED;
    if (!plain_unit(g) && !col) {   // implicit im2col
        if (!conv_implicit_ok(g, Cout) || !wpre) return LRS_E_UNSUPPORTED;
        const int kk = g.k * g.k, Cp = r16(g.Cin);
        return gemm_s3_conv(LdPre{wpre, (int64_t)Cout * kk * Cp, kk * Cp, Cout},
                            LdFwdTM{x, g.Cin * g.Hs * g.Ws * 4, g, Cp, nullptr}, y, bias, nullptr, Cout, P, kk * Cp,
                            part, part_cap, st, nsplit_out, 0, nsplit_out ? fwd_split_target() : 512);
    }
    if (!plain_unit(g)) {
        const dim3 grid((unsigned)((P + 255) / 256), (unsigned)std::min(Kc, 65535));
        hipLaunchKernelGGL(k_im2col, grid, dim3(256), 0, st, x, g, col);
        B = col;
    }
    return gemm(g.prec, 0, 0, w, B, y, bias, nullptr, Cout, P, Kc, part, part_cap, st, 0, nsplit_out);
}

// gw = gz col^T / div ; gx = col2im(w^T gz) (gw, gx nullable).  dcol: Kc*P floats when !plain.
// implicit: `col` is the conv input x, col^T is gathered inside the GEMM, and wpre holds the
// weight planes (wprep) for the stride-1 data gradient.
int conv_bwd(const ConvGeom &g, const float *gz, const float *col, const float *w, const float *div, int Cout,
             float *gx, float *gw, float *dcol, float *part, int64_t part_cap, hipStream_t st, int accum_gx = 0,
             bool implicit = false, const __bf16 *wpre = nullptr, int *wsplit_out = nullptr, int wtarget = 512) {
    const int P = g.Ho * g.Wo, kk = g.k * g.k, Kc = g.Cin * kk;
    int rc;
    implicit = implicit && !plain_unit(g);
    rc = LRS_OK;
    if (!gw) {
        // data gradient only (the weight gradient runs elsewhere)
    } else if (implicit) {
        if (!conv_implicit_ok(g, Cout)) return LRS_E_UNSUPPORTED;
        // wsplit_out: the caller finishes the split-K sum (k_adam's AdamPend)
        rc = gemm_s3_conv(LdDense<true>{gz, P, Cout}, LdWgradTM{col, g.Cin * g.Hs * g.Ws * 4, g, nullptr, 0}, gw,
                          nullptr, div, Cout, Kc, P, part, part_cap, st, wsplit_out, 0, wtarget);
    } else {
        // a 1x1 conv's weight gradient (K = all pixels): 128-tiles with deep split-K on the split-bf16
        // kernel (A/B in the 196^2 training step, configs[2]: 5.50 -> 5.65 outer it/s against the f32
        // 64-tile kernel; alone the two are within 12 %, but the f32 kernel's 512 workgroups hold the
        // CUs the concurrent data-gradient chain needs for longer)
        // (wsplit_out: as above, the caller's k_adam finishes the split-K sum)
        rc = gemm(g.prec, 0, 1, gz, col, gw, nullptr, div, Cout, Kc, P, part, part_cap, st, 0, wsplit_out, plain_unit(g),
                  wtarget);
    }
    if (rc || !gx) return rc;
    if (plain_unit(g) && wpre)      // 1x1 data gradient: W^T planes (wprep's WD)
        return pw_launch(wpre + wprep_fwd_elems(g, Cout), (int64_t)g.Cin * r16(Cout), r16(Cout), g.Cin, gz, Cout, P,
                         gx, nullptr, accum_gx, st);
    if (plain_unit(g)) return gemm(g.prec, 1, 0, w, gz, gx, nullptr, nullptr, Kc, P, Cout, part, part_cap, st, accum_gx);
    const int ke = up_eff_k(g);
    const bool refl_border = g.pad_mode == LRS_PAD_REFLECT && g.k == 3;
    const int Lmax = std::max(g.Ws, g.Hs);
    // the border scratch (S and corr) lives in the col-gradient buffer, unused on this path
    const bool border_fits = dcol && (int64_t)4 * (3 * Cout + g.Cin) * Lmax <= (int64_t)g.Cin * g.k * g.k * P;
    if (implicit && wpre && ke && !accum_gx && (!refl_border || border_fits)) {
        // gx = the stride-2 (ke x ke, zero pad 1) conv of dL/dz with the effective weights WE
        // (k_conv_prep), then the reflection terms of the border rows / columns
        const int Cop = r16(Cout), ke2 = ke * ke;
        ConvGeom ge{};
        ge.Cin = Cout; ge.Hs = g.Ho; ge.Ws = g.Wo; ge.up = 0; ge.Hu = g.Ho; ge.Wu = g.Wo;
        ge.pad = 1; ge.pad_mode = LRS_PAD_ZERO; ge.k = ke; ge.stride = 2; ge.Ho = g.Hs; ge.Wo = g.Ws;
        if ((g.Ho + 2 - ke) / 2 + 1 != g.Hs || (g.Wo + 2 - ke) / 2 + 1 != g.Ws) return LRS_E_INVALID;
        rc = gemm_s3_conv(LdPre{wpre + wprep_fwd_elems(g, Cout), (int64_t)g.Cin * ke2 * Cop, ke2 * Cop, g.Cin},
                          LdFwdTM{gz, Cout * P * 4, ge, Cop, nullptr}, gx, nullptr, nullptr, g.Cin, g.Hs * g.Ws,
                          ke2 * Cop, part, part_cap, st);
        if (rc) return rc;
        if (refl_border) {
            float *S = dcol, *corr = dcol + (int64_t)4 * 3 * Cout * Lmax;
            hipLaunchKernelGGL(k_up_border_s, dim3((unsigned)((12 * Lmax + 255) / 256), (unsigned)Cout), dim3(256), 0, st,
                               gz, Cout, g.Hs, g.Ws, Lmax, S);
            hipLaunchKernelGGL(k_up_border_mm, dim3(4, (unsigned)((g.Cin + kUbC - 1) / kUbC), (unsigned)((Lmax + 127) / 128)),
                               dim3(256), 0, st, S, w, g.Cin, Cout, g.Hs, g.Ws, Lmax, corr);
            const int nper = 2 * g.Ws + 2 * (g.Hs - 2);
            hipLaunchKernelGGL(k_up_border_add, dim3((unsigned)((nper + 255) / 256), (unsigned)g.Cin), dim3(256), 0, st,
                               corr, g.Cin, g.Hs, g.Ws, Lmax, gx);
        }
        LRS_CHECK_LAUNCH();
        return LRS_OK;
    }
    if (!dcol) return LRS_E_WORKSPACE;
    const int Qp = (g.Hu + 2 * g.pad) * (g.Wu + 2 * g.pad);
    if (implicit && wpre && g.stride == 1 && (int64_t)g.Cin * Qp <= (int64_t)Kc * P) {
        // gxp = W^T (x) gz over the padded domain (implicit, in the dcol space), then fold the
        // padding / upsample
        const int Cop = r16(Cout);
        const __bf16 *wd = wpre + wprep_fwd_elems(g, Cout);
        int nsplit = 1;   // split-K partials are summed inside the fold
        rc = gemm_s3_conv(LdPre{wd, (int64_t)g.Cin * kk * Cop, kk * Cop, g.Cin},
                          LdDgradTM{gz, Cout * P * 4, g, Cout, Cop, nullptr}, dcol, nullptr, nullptr, g.Cin, Qp,
                          kk * Cop, part, part_cap, st, &nsplit, 0, dgrad_split_target());
        if (rc) return rc;
        if (nsplit == 1 && !g.up && g.Ws % 4 == 0 && g.Cin <= 65535 && ((uintptr_t)gx & 15) == 0) {   // one partial: row quads
            const int q = g.Hs * (g.Ws / 4);
            hipLaunchKernelGGL(k_fold_pad1q, dim3((unsigned)((q + 255) / 256), (unsigned)g.Cin), dim3(256), 0, st, dcol,
                               g, gx, accum_gx);
        } else {
            const dim3 grid((unsigned)((g.Hs * g.Ws + 255) / 256), (unsigned)std::min(g.Cin, 65535));
            hipLaunchKernelGGL(k_fold_pad, grid, dim3(256), 0, st, nsplit > 1 ? part : dcol, nsplit, (int64_t)g.Cin * Qp,
                               g, gx, accum_gx);
        }
        LRS_CHECK_LAUNCH();
        return LRS_OK;
    }
    rc = gemm(g.prec, 1, 0, w, gz, dcol, nullptr, nullptr, Kc, P, Cout, part, part_cap, st);
    if (rc) return rc;
    const dim3 grid((unsigned)((g.Hs * g.Ws + 255) / 256), (unsigned)std::min(g.Cin, 65535));
    if (g.stride == 1) hipLaunchKernelGGL(k_col2im<1>, grid, dim3(256), 0, st, dcol, g, gx, accum_gx);
    else if (g.stride == 2) hipLaunchKernelGGL(k_col2im<2>, grid, dim3(256), 0, st, dcol, g, gx, accum_gx);
    else hipLaunchKernelGGL(k_col2im<0>, grid, dim3(256), 0, st, dcol, g, gx, accum_gx);
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

inline bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// Register-resident one-workgroup-per-channel BN (k_bn_fwd_r / k_bn_bwd_r): float4 quads per
// thread for a channel of P pixels, or 0 where the S-way split / the P <= 4096 kernels are used.
// LRS_DIP_BNREG_MAX_P overrides the upper limit (tuning only; 0 disables).
inline int bn_reg_q(int64_t P, bool vec) {
    static const int64_t maxp = tune_knob("LRS_DIP_BNREG_MAX_P", (int64_t)4 * kBn1Threads * kBnRegMaxQ);
    if (!vec || P <= 4 * kBn1Threads || P > maxp || P > (int64_t)4 * kBn1Threads * kBnRegMaxQ) return 0;
    const int q = (int)((P + 4 * kBn1Threads - 1) / (4 * kBn1Threads));
    static const int qs[] = {2, 3, 4, 6, 8, 10};
    for (int v : qs)
        if (v >= q) return v;
    return 0;
}

// Threads of a one-workgroup-per-channel BatchNorm kernel (k_reduce_bn1, k_reduce_bn_bwd1, k_bn_fwd1,
// k_bn_bwd1): kBn1Small where the channel fits 2 values per thread of it (the 18^2 and smaller maps at
// 36^2, the 13^2 ones at 196^2), else kBn1Threads.  A/B (tuning build, 2 rounds): 36^2 step 0.671 ->
// 0.657 ms with 256 threads up to 1024 pixels, but the 196^2 step 1.274 -> 1.280 (its 25^2 maps then
// hold 3 values per thread).  LRS_DIP_BN1_SMALL = the pixel limit (0: 1024 threads everywhere).
inline int bn1_threads(int64_t P) {
    // (clamped to what a kBn1Small-thread kernel covers: 4 values per thread)
    static const int64_t lim = std::min<int64_t>(tune_knob("LRS_DIP_BN1_SMALL", 2 * kBn1Small), 4 * kBn1Small);
    return P <= lim ? kBn1Small : kBn1Threads;
}

// 98^2 maps' register BN forward on 256-thread workgroups (tuning build only; default off)
inline bool bnr_small_wg() {
    static const bool v = tune_knob("LRS_DIP_BNR_SMALL_WG", 0) != 0;
    return v;
}

#define LRS_BNR_SWITCH(nq, K, ...)                                                                \
    switch (nq) {                                                                                 \
    case 2: hipLaunchKernelGGL(K<2>, __VA_ARGS__); break;                                         \
    case 3: hipLaunchKernelGGL(K<3>, __VA_ARGS__); break;                                         \
    case 4: hipLaunchKernelGGL(K<4>, __VA_ARGS__); break;                                         \
    case 6: hipLaunchKernelGGL(K<6>, __VA_ARGS__); break;                                         \
    case 8: hipLaunchKernelGGL(K<8>, __VA_ARGS__); break;                                         \
    default: hipLaunchKernelGGL(K<10>, __VA_ARGS__); break;                                       \
    }

int bn_fwd(const float *z, float *y, const float *gamma, const float *beta, float *mean, float *invstd, float *rm,
           float *rv, int C, int64_t P, int act, float eps, float mom, double *part, hipStream_t st, int lip = 1) {
    const int S = bn_split(P);
    const int vec = (P % 4 == 0 && al16(z) && al16(y)) ? 1 : 0;
    int chunk = (int)((P + S - 1) / S);
    if (vec) chunk = (chunk + 3) & ~3;
    BnArgs a{z, y, gamma, beta, mean, invstd, rm, rv, part, C, (int)P, S, chunk, gamma ? 1 : 0, act, eps, mom, lip,
             vec};
    if (const int nq = gamma ? bn_reg_q(P, vec) : 0) {
        LRS_BNR_SWITCH(nq, k_bn_fwd_r, dim3(1, C), dim3(kBn1Threads), 0, st, (const float *)nullptr, 0,
                       (const float *)nullptr, a);
    } else if (gamma && S == 1) {
        hipLaunchKernelGGL(k_bn_fwd1, dim3(1, C), dim3(bn1_threads(P)), 0, st, a);
    } else {
        if (gamma) hipLaunchKernelGGL(k_bn_stats, dim3(S, C), dim3(kBnThreads), 0, st, a);
        hipLaunchKernelGGL(k_bn_apply, dim3(S, C), dim3(kBnThreads), 0, st, a);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int bn_bwd(const float *gy, const float *y, const float *z, const float *gamma, const float *mean,
           const float *invstd, float *gz, float *ggamma, float *gbeta, float *gbias, int C, int64_t P, int act,
           double *part, hipStream_t st, int lip = 1, int accum = 0, const float *beta = nullptr) {
    const int S = bn_split(P);
    const int vec = (P % 4 == 0 && al16(gy) && al16(y) && al16(z) && al16(gz)) ? 1 : 0;
    int chunk = (int)((P + S - 1) / S);
    if (vec) chunk = (chunk + 3) & ~3;
    BnBwdArgs a{gy, y, z, gamma, mean, invstd, gz, ggamma, gbeta, gbias, part, C, (int)P, S, chunk,
                gamma ? 1 : 0, act, lip, accum, vec, gamma ? beta : nullptr};
    if (const int nq = gamma ? bn_reg_q(P, vec) : 0) {
        LRS_BNR_SWITCH(nq, k_bn_bwd_r, dim3(1, C), dim3(kBn1Threads), 0, st, a);
    } else if ((gamma || gbias) && S == 1) {
        hipLaunchKernelGGL(k_bn_bwd1, dim3(1, C), dim3(bn1_threads(P)), 0, st, a);
    } else {
        if (gamma || gbias) hipLaunchKernelGGL(k_bn_bwd_stats, dim3(S, C), dim3(kBnThreads), 0, st, a);
        hipLaunchKernelGGL(k_bn_bwd_apply, dim3(S, C), dim3(kBnThreads), 0, st, a);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// The step head of the overlapped sigma (lrs_dipnet::sn_overlap): the spectral-norm Gram partials of
// the n convs (blockIdx.y < n, k_sn_gram's body) and, in the extra row blockIdx.y == n, the first
// conv's forward planes from the raw weights (the head ConvPrep) with the step's loss reset and Adam
// step count: one launch instead of two.
__global__ __launch_bounds__(256) void k_sn_gram_head(const SnConv *convs, double *gram, int n, const ConvPrep *head,
                                                     double *loss_acc, int *step) {
    __shared__ float Ws[128][36];
    if ((int)blockIdx.y >= n) {   // rows n, n + 1, ...: the planes
        const int64_t b = (int64_t)(blockIdx.y - n) * gridDim.x + blockIdx.x;
        if (b == 0 && threadIdx.x == 0) {   // a training step begins
            *loss_acc = 0.0;
            *step += 1;
        }
        conv_prep_body(*head, 1.0f, b * blockDim.x + threadIdx.x, (int64_t)(gridDim.y - n) * gridDim.x * blockDim.x);
        return;
    }
    const SnConv cv = convs[blockIdx.y];
    double *out = gram + (int64_t)blockIdx.y * kSnGramDoubles + (int64_t)kSnMaxDim * kSnMaxDim +
                  (int64_t)blockIdx.x * kSnPairs * 256;
    switch (threadIdx.x >> 6) {
    case 0: sn_gram_body<0>(cv, Ws, out); break;
    case 1: sn_gram_body<1>(cv, Ws, out); break;
    case 2: sn_gram_body<2>(cv, Ws, out); break;
    default: sn_gram_body<3>(cv, Ws, out); break;
    }
}

int sn_launch(const SnConv *table_dev, int n, int64_t max_elems, double *gram, float *sigma, float *scale,
              float ln_lambda, bool apply, hipStream_t st, long long *prof = nullptr) {
    hipLaunchKernelGGL(k_sn_gram, dim3(kSnSplit, n), dim3(256), 0, st, table_dev, gram);
    hipLaunchKernelGGL(k_sn_gram_reduce, dim3(kSnPairs, n), dim3(256), 0, st, table_dev, gram);
    hipLaunchKernelGGL(k_sn_sigma, dim3(n), dim3(256), 0, st, table_dev, gram, sigma, scale, ln_lambda, prof);
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
    const unsigned nblk = ew_blocks(N, kEsMaxBlocks);
#ifdef LRS_TUNING
    static const bool two_pass = tune_knob("LRS_DIP_ES_TWO_PASS", 0) != 0;
    if (two_pass) {
        hipLaunchKernelGGL(k_es_push_r5, dim3(nblk), dim3(kEw), 0, st, out, N, ring, es);
        hipLaunchKernelGGL(k_es_var_r5, dim3(nblk), dim3(kEw), 0, st, (const float *)ring, N, es);
        hipLaunchKernelGGL(k_es_decide, dim3(1), dim3(64), 0, st, (const float *)ring, N, 0, es);
        LRS_CHECK_LAUNCH();
        return LRS_OK;
    }
#endif
    hipLaunchKernelGGL(k_es_step, dim3(nblk), dim3(kEw), 0, st, out, N, ring, es);
    hipLaunchKernelGGL(k_es_decide, dim3(1), dim3(64), 0, st, (const float *)ring, N, (int)nblk, es);
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

// Dense fp32-accurate GEMM for the library's other components (the K > 512 ISTA path, ista.hip):
// C[M][N] = op(A) op(B) with the DIP engine's split-bf16 / f32 kernels, split-K summed in fixed
// order (deterministic).  part: >= dense_gemm_part_floats(M, N, K) floats.
namespace lrs {
int64_t dense_gemm_part_floats(int M, int N, int K) { return gemm_part_floats(M, N, K); }
int dense_gemm(int TA, int TB, const float *A, const float *B, float *C, int M, int N, int K, float *part,
               int64_t part_cap, hipStream_t st) {
    return gemm(LRS_DIP_SPLIT_BF16, TA, TB, A, B, C, nullptr, nullptr, M, N, K, part, part_cap, st);
}
}  // namespace lrs

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

// conv workspace: [dcol: Kc*P floats when not plain][split-K partials][weight planes (bf16)]
struct ConvWs {
    int64_t dcol, part, wpre_floats;
};
inline ConvWs conv_ws(const ConvGeom &g, int Cout) {
    ConvWs w;
    w.dcol = plain_unit(g) ? 0 : (int64_t)g.Cin * g.k * g.k * g.Ho * g.Wo;
    w.part = conv_part_floats(g, Cout);
    w.wpre_floats = (plain_unit(g) && !pw_ok(g, Cout)) ? 0 : (wprep_elems(g, Cout) + 7) / 2;
    return w;
}

extern "C" size_t lrs_conv2d_workspace(int Cin, int H, int W, int Cout, int k, int stride, int pad, int upsample,
                                       const lrs_dip_opts *opts) {
    ConvGeom g;
    if (make_geom(Cin, H, W, k, stride, pad, LRS_PAD_ZERO, upsample, g, opts) || Cout <= 0) return 0;
    const ConvWs w = conv_ws(g, Cout);
    return (size_t)(w.dcol + w.part + w.wpre_floats) * sizeof(float) + 256;
}

extern "C" int lrs_conv2d_fwd_f32(const float *x, int Cin, int H, int W, const float *w, const float *bias, int Cout,
                                  int k, int stride, int pad, int pad_mode, int upsample, float *col, float *y,
                                  const lrs_dip_opts *opts, void *ws, size_t ws_bytes, void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g, opts);
    if (rc) return rc;
    if (!x || !w || !y || Cout <= 0) return LRS_E_INVALID;
    // col == NULL: implicit GEMM, or for a 1x1 conv the pointwise kernel on pre-split weights
    const bool implicit = !col && (!plain_unit(g) || pw_ok(g, Cout));
    if (implicit && !plain_unit(g) && !conv_implicit_ok(g, Cout)) return LRS_E_UNSUPPORTED;
    const ConvWs cw = conv_ws(g, Cout);
    const int64_t need = implicit ? cw.dcol + cw.part + cw.wpre_floats : cw.part;
    if (need > 0 && (!ws || ws_bytes < (size_t)need * sizeof(float))) return LRS_E_WORKSPACE;
    float *pt = implicit ? (float *)ws + cw.dcol : (float *)ws;
    __bf16 *wp = implicit ? (__bf16 *)((float *)ws + cw.dcol + cw.part) : nullptr;
    if (implicit && (rc = wprep(g, w, Cout, wp, nullptr, (hipStream_t)stream))) return rc;
    return conv_fwd(g, x, w, bias, Cout, col, y, pt, cw.part, (hipStream_t)stream, wp);
}

extern "C" int lrs_conv2d_bwd_f32(const float *gy, const float *col, const float *w, const float *w_div, int Cin,
                                  int H, int W, int Cout, int k, int stride, int pad, int pad_mode, int upsample,
                                  float *gx, float *gw, const lrs_dip_opts *opts, void *ws, size_t ws_bytes,
                                  void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g, opts);
    if (rc) return rc;
    if (!gy || !col || !w || !gw || Cout <= 0) return LRS_E_INVALID;
    const ConvWs cw = conv_ws(g, Cout);
    if (ws_bytes < (size_t)(cw.part + cw.dcol) * sizeof(float) || (!ws && cw.part + cw.dcol > 0))
        return LRS_E_WORKSPACE;
    float *dc = cw.dcol ? (float *)ws : nullptr;
    float *pt = (float *)ws + cw.dcol;
    return conv_bwd(g, gy, col, w, w_div, Cout, gx, gw, dc, pt, cw.part, (hipStream_t)stream);
}

extern "C" int lrs_conv2d_bwd_x_f32(const float *gy, const float *x, const float *w, const float *w_div, int Cin,
                                    int H, int W, int Cout, int k, int stride, int pad, int pad_mode, int upsample,
                                    float *gx, float *gw, const lrs_dip_opts *opts, void *ws, size_t ws_bytes,
                                    void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g, opts);
    if (rc) return rc;
    if (!gy || !x || !w || !gw || Cout <= 0) return LRS_E_INVALID;
    if (!conv_implicit_ok(g, Cout)) return LRS_E_UNSUPPORTED;
    const ConvWs cw = conv_ws(g, Cout);
    const int64_t need = cw.dcol + cw.part + cw.wpre_floats;
    if (ws_bytes < (size_t)need * sizeof(float) || (!ws && need > 0)) return LRS_E_WORKSPACE;
    float *dc = cw.dcol ? (float *)ws : nullptr;
    float *pt = (float *)ws + cw.dcol;
    __bf16 *wp = cw.wpre_floats ? (__bf16 *)((float *)ws + cw.dcol + cw.part) : nullptr;
    if (wp && gx && (rc = wprep(g, w, Cout, wp, wp + wprep_fwd_elems(g, Cout), (hipStream_t)stream))) return rc;
    return conv_bwd(g, gy, x, w, w_div, Cout, gx, gw, dc, pt, cw.part, (hipStream_t)stream, 0, true, wp);
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

// The engine's one-launch small-map conv + BatchNorm (k_conv_bn_dir, dip_dir.h) on its own: the same
// launch dipnet_forward makes for a conv with BN on a map of <= dir_max_p() pixels.
extern "C" int lrs_conv_bn_small_f32(const float *x, int Cin, int H, int W, const float *w, const float *bias, int Cout,
                                     int k, int stride, int pad, int pad_mode, int upsample, const float *gamma,
                                     const float *beta, int lip, int act, float *z, float *y, float *mean, float *invstd,
                                     float *run_mean, float *run_var, void *stream) {
    ConvGeom g;
    int rc = make_geom(Cin, H, W, k, stride, pad, pad_mode, upsample, g);
    if (rc) return rc;
    if (!x || !w || !gamma || !beta || !z || !y || !mean || !invstd || Cout <= 0 || Cout > 65535 ||
        (!run_mean) != (!run_var) || (lip != 0 && lip != 1))
        return LRS_E_INVALID;
    if (act != LRS_ACT_NONE && act != LRS_ACT_LRELU && act != LRS_ACT_SIGMOID) return LRS_E_INVALID;
    DirGeom dg;
    if (!dir_geom(g, dg)) return LRS_E_UNSUPPORTED;
    const int P = g.Ho * g.Wo;
    const BnArgs a{z, y, gamma, beta, mean, invstd, run_mean, run_var, nullptr, Cout, P, 1, P, 1, act, 1e-5f, 0.1f, lip, 0};
    const dim3 grid(1, Cout);
    hipStream_t st = (hipStream_t)stream;
#define LRS_DIR1(KS, S)                                                                                        \
    do {                                                                                                        \
        if (dg.vec4) hipLaunchKernelGGL((k_conv_bn_dir<KS, S, true>), grid, dim3(kDirTh), 0, st, x, w, bias, g, dg, a); \
        else hipLaunchKernelGGL((k_conv_bn_dir<KS, S, false>), grid, dim3(kDirTh), 0, st, x, w, bias, g, dg, a);     \
    } while (0)
    if (g.k == 3 && g.stride == 1) LRS_DIR1(3, 1);
    else if (g.k == 3) LRS_DIR1(3, 2);
    else if (g.stride == 1) LRS_DIR1(1, 1);
    else LRS_DIR1(1, 2);
#undef LRS_DIR1
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" size_t lrs_sigma_max_workspace(int n) {
    if (n <= 0) return 0;
    return (size_t)n * kSnGramDoubles * sizeof(double) + (size_t)n * sizeof(SnConv) + 256;
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
    SnConv *tdev = (SnConv *)((char *)ws + (size_t)n * kSnGramDoubles * sizeof(double));
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
    SnConv *tdev = (SnConv *)((char *)ws + (size_t)n * kSnGramDoubles * sizeof(double));
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
    hipLaunchKernelGGL(k_adam, dim3(ew_blocks((n + 3) / 4, 8192)), dim3(kEw), 0, (hipStream_t)stream, p, g, m, v, n, step, lr,
                       beta1, beta2, eps, AdamPend{});
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_masked_mse_f32(const float *out, const float *target, const float *mask, int C, int64_t P,
                                  float *gout, double *loss_acc, void *stream) {
    if (!out || !target || !loss_acc || C <= 0 || P <= 0) return LRS_E_INVALID;
    const int vec = (P % 4 == 0 && al16(out) && al16(target) && (!mask || al16(mask)) && (!gout || al16(gout))) ? 1 : 0;
    int64_t S = (512 + C - 1) / C;   // ~512 workgroups over the C channels (fewer loss atomics)
    S = std::max<int64_t>(1, std::min<int64_t>(S, (P + 1023) / 1024));
    int64_t chunk = (P + S - 1) / S;
    if (vec) chunk = (chunk + 3) & ~(int64_t)3;
    if (chunk > INT32_MAX || C > 65535) return LRS_E_UNSUPPORTED;
    hipLaunchKernelGGL(k_masked_mse, dim3((unsigned)S, (unsigned)C), dim3(256), 0, (hipStream_t)stream, out, target,
                       mask, C, P, (int)chunk, vec, gout, loss_acc);
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

extern "C" size_t lrs_es_ring_bytes(int size, int64_t N) {
    if (size <= 0 || N <= 0) return 0;
    return (size_t)(es_ab_offset_bytes(size, N) + N * 8 + (2 * kEsMaxBlocks + 2) * 8);
}

extern "C" int lrs_es_update_f32(const float *out, int64_t N, float *ring, lrs_es_state *st, void *stream) {
    if (!out || !ring || !st || N <= 0) return LRS_E_INVALID;
    return es_update(out, N, ring, st, (hipStream_t)stream);
}

// ============================================================================================
// Network engine: a DAG of conv / BN / concat nodes (the 1-Lip U-Net is a chain; the skip net
// of models/skip.py has concatenations).  Tensor 0 is the input, node i produces tensor i+1.
// ============================================================================================
struct lrs_dipnet {
    struct Node {
        lrs_dip_node d;
        int C, H, W;                  // output shape
        ConvGeom g{};                 // CONV
        CatGeom cg{};                 // CONCAT
        int64_t P = 0, Kc = 0;
        int64_t w_off = -1, b_off = -1, gm_off = -1, bt_off = -1, rs_off = -1;   // params / bn running stats
        int64_t out_off = 0, z_off = -1, col_off = -1, mean_off = -1, istd_off = -1, wn_off = -1, grad_off = 0;
        int64_t wpre_off = -1;        // implicit convs: bf16 weight planes (wprep)
        int64_t gz_off = -1;          // conv: dL/dz (read by the side-stream weight gradient)
        int sn_index = -1;            // position in the spectral-norm table
        bool sm = false;              // small map: forward / data gradient on k_conv_sm (dip_sm.h)
        bool upc = false;             // upsampled 3 x 3: forward / data gradient by output parity class
        bool sm_dgrad = false;        // ... data gradient through the adjoint table below
        bool fork_pt = true;          // weight-gradient side stream: fork after its BN backward (else its
                                      // weight gradient waits for the next fork point)
        int64_t adj_off = -1;         // the lists in the workspace (shorts, sm_adj_dim)
        std::vector<int> adj;         // host copy (sm_adj_table), uploaded at bind
        int64_t wtab_off = -1;        // small map: the weight gradient's gather table (sm_wgrad_table)
        std::vector<int> wtab;
    };
    std::vector<Node> nodes;
    int C0 = 0, H = 0, W = 0;
    int64_t n_params = 0, n_bnstats = 0;
    int64_t dz_off = 0, dcol_off = 0, part_off = 0, part_cap = 0, sigma_off = 0, scale_off = 0;
    int64_t gram_off_bytes = 0, table_off_bytes = 0, misc_off_bytes = 0, bnpart_off_bytes = 0, prep_off_bytes = 0;
    int n_prep = 0;           // convs in the per-step weight-preparation table (spectral norm and/or planes)
    // sigma overlapped with the first conv (dipnet_step): the side stream runs the spectral-norm
    // chain and the preparation of every conv but the first, whose planes the main stream writes from
    // the raw weights (prep_head table); its BatchNorm kernel divides by the scale (sn_overlap)
    bool sn_overlap = false;
    int n_prep_side = 0;
    int64_t prep_head_off_bytes = 0, prep_side_off_bytes = 0;
    // prep_split: the data-gradient planes (read first in the backward) prepared on the side stream beside
    // the forward; the forward planes and W / scale stay where they were (prep_f: forward / prep_fs: the
    // overlapped side table, without the data-gradient planes; prep_d: the data-gradient planes only)
    bool prep_split = false, wd_pending = false;
    int n_prep_d = 0;
    int64_t prep_f_off_bytes = 0, prep_fs_off_bytes = 0, prep_d_off_bytes = 0;
    hipEvent_t ev_wdgo = nullptr, ev_wd = nullptr;
    hipEvent_t ev_head = nullptr, ev_sigma = nullptr;
    // split_ev: ev_sigma right after the Lanczos (the first BatchNorm needs the scale only) and ev_prep
    // after the other convs' planes (the second conv waits for it); else ev_sigma after both
    hipEvent_t ev_prep = nullptr;
    bool split_ev = false;
    int64_t headcnt_off_bytes = 0;   // per-channel counters of k_mse_head (zeroed at bind, reset by the kernel)
    bool head_fusable = false;       // last node = conv without BN: loss + its activation backward in one kernel
    // ... and when that conv is a 1x1 on k_pw, the loss head runs in the conv's own epilogue (PwHead);
    // its per-workgroup sums go to hpart, reduced by k_head_reduce / k_head_loss on the side stream
    bool head_pw = false;
    int head_nwg = 0;
    int64_t hpart_off_bytes = 0, closs_off_bytes = 0;
    size_t ws_bytes = 0;
    int n_sn = 0;
    int64_t max_w = 0;
    bool implicit = false;   // convs gather im2col inside the split-bf16 GEMM (no col buffers)
    float *params = nullptr, *grads = nullptr, *am = nullptr, *av = nullptr, *bnstats = nullptr;
    char *ws = nullptr;
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    // weight gradients run on a side stream beside the data-gradient chain (fork per conv node
    // after its BN backward, join before Adam)
    hipStream_t side = nullptr;   // the one for the current call's priority (one of sides)
    std::vector<std::pair<int, hipStream_t>> sides;   // (priority, stream): one per priority seen
    std::vector<hipEvent_t> ev_fork;
    hipEvent_t ev_join = nullptr;
    int64_t part2_off = 0;
    int64_t part3_off = -1;   // grouped backward (group_bwd): the main stream's weight-gradient partials
    bool group_bwd = false;   // a conv's data and weight gradients in one launch (k_gemm_s3x2; tuning build)
    // forking pays only when the layers fill the chip (measured: 512^2 skip net 13.0 -> 12.1 ms
    // per step; 196^2 even; 36^2 7-16 % slower from the event overhead)
    bool fork_w = false;
    struct Key {
        const void *x, *t, *m, *es, *ring;
        float lr, b1, b2, eps;
    } key{};
    bool have_key = false;
    lrs_dip_opts opts{};      // fixed at creation (precision, upsampled data-gradient form)
    float ln_lambda = 1.0f;   // W_used = W / max(1, sigma / ln_lambda)   (lipschitz_constraint_layer.py:42-44)

    float *f(int64_t off) const { return (float *)ws + off; }
    double *gram() const { return (double *)(ws + gram_off_bytes); }
    SnConv *table() const { return (SnConv *)(ws + table_off_bytes); }
    ConvPrep *prep() const { return (ConvPrep *)(ws + prep_off_bytes); }
    ConvPrep *prep_head() const { return (ConvPrep *)(ws + prep_head_off_bytes); }
    ConvPrep *prep_side() const { return (ConvPrep *)(ws + prep_side_off_bytes); }
    ConvPrep *prep_f() const { return (ConvPrep *)(ws + prep_f_off_bytes); }
    ConvPrep *prep_fs() const { return (ConvPrep *)(ws + prep_fs_off_bytes); }
    ConvPrep *prep_d() const { return (ConvPrep *)(ws + prep_d_off_bytes); }
    int *headcnt() const { return (int *)(ws + headcnt_off_bytes); }
    double *loss_acc() const { return (double *)(ws + misc_off_bytes); }
    int *step() const { return (int *)(ws + misc_off_bytes + 8); }
    double *bnpart() const { return (double *)(ws + bnpart_off_bytes); }
    double *hpart() const { return (double *)(ws + hpart_off_bytes); }
    double *closs() const { return (double *)(ws + closs_off_bytes); }
    const float *tensor(int t, const float *x) const { return t == 0 ? x : f(nodes[t - 1].out_off); }
    int tC(int t) const { return t == 0 ? C0 : nodes[t - 1].C; }
    int tH(int t) const { return t == 0 ? H : nodes[t - 1].H; }
    int tW(int t) const { return t == 0 ? W : nodes[t - 1].W; }
};

namespace {

int64_t align64(int64_t n) { return (n + 63) / 64 * 64; }   // floats (256 bytes)

// Can node j's BN backward finish a split-K dL/dy itself (k_reduce_bn_bwd1: a conv with BN whose
// channel fits one workgroup)?
bool bn_bwd_fusable(const lrs_dipnet *net, int j) {
    const auto &N = net->nodes[j];
    return N.d.kind == LRS_NODE_CONV && N.d.bn && N.P <= 4 * kBn1Threads && bn_split(N.P) == 1;
}

// workgroups per conv of the per-step weight preparation (LRS_DIP_PREP_WG overrides: tuning only)
inline int prep_blocks() {
    static const int v = (int)std::max<int64_t>(1, tune_knob("LRS_DIP_PREP_WG", 512));
    return v;
}

// the largest small map (output pixels) whose conv + BatchNorm run as one k_conv_bn_dir launch:
// the 9^2 and smaller maps (36^2 step 0.635 -> 0.621 ms; 196^2 within noise; with the 13^2 / 18^2
// maps too both are slower: 196^2 +28 us, 36^2 +3 us; tuning build, 2 interleaved rounds,
// profiles/r05/dir/)
inline int64_t dir_max_p() {
    static const int64_t v = tune_knob("LRS_DIP_DIR_P", 100);
    return v;
}

// raw_first (dipnet_step's overlapped sigma, lrs_dipnet::sn_overlap): the spectral-norm chain and
// the weight preparation were enqueued by the caller (the first conv's planes from the raw weights on
// st, the rest on the side stream, which records ev_sigma); the first conv runs on the raw planes and
// st waits for ev_sigma before its BatchNorm kernel, which divides by the scale.
int dipnet_forward(lrs_dipnet *net, const float *x, hipStream_t st, bool step_begin = false, bool raw_first = false,
                   const PwHead *head = nullptr) {
    int rc;
    if (net->n_sn && !raw_first) {
        rc = sn_launch(net->table(), net->n_sn, net->max_w, net->gram(), net->f(net->sigma_off),
                       net->f(net->scale_off), net->ln_lambda, false, st);
        if (rc) return rc;
    }
    if (net->n_prep && !raw_first) {   // W / scale and the bf16 planes of every conv, one launch
        const bool split = net->prep_split && step_begin && net->side && net->ev_wdgo && net->ev_wd;
        hipLaunchKernelGGL(k_conv_prep, dim3(prep_blocks(), net->n_prep), dim3(256), 0, st, split ? net->prep_f() : net->prep(),
                           net->f(net->scale_off), step_begin ? net->loss_acc() : nullptr, net->step());
        if (split && net->n_prep_d) {   // the data-gradient planes beside the forward (the backward waits)
            hipError_t e = hipEventRecord(net->ev_wdgo, st);
            if (e == hipSuccess) e = hipStreamWaitEvent(net->side, net->ev_wdgo, 0);
            if (e != hipSuccess) return (int)e;
            hipLaunchKernelGGL(k_conv_prep, dim3(prep_blocks(), net->n_prep_d), dim3(256), 0, net->side, net->prep_d(),
                               net->f(net->scale_off), (double *)nullptr, net->step());
            if ((e = hipEventRecord(net->ev_wd, net->side)) != hipSuccess) return (int)e;
            net->wd_pending = true;
        }
        LRS_CHECK_LAUNCH();
    }
    bool prep_waited = !(raw_first && net->split_ev);
    for (size_t i = 0; i < net->nodes.size(); ++i) {
        auto &N = net->nodes[i];
        float *out = net->f(N.out_off);
        const int lip = N.d.bn == 2 ? 1 : 0;
        if (!prep_waited && i > 0) {   // every later node may read the side stream's planes / W / scale
            const hipError_t e = hipStreamWaitEvent(st, net->ev_prep, 0);
            if (e != hipSuccess) return (int)e;
            prep_waited = true;
        }
        if (N.d.kind == LRS_NODE_CONV) {
            const bool bn = N.d.bn != 0;
            float *z = bn ? net->f(N.z_off) : out;
            const float *w = N.sn_index >= 0 ? net->f(N.wn_off) : net->params + N.w_off;
            __bf16 *wp = N.wpre_off >= 0 ? (__bf16 *)net->f(N.wpre_off) : nullptr;
            // a BN channel that fits one workgroup finishes the conv's split-K sum itself (k_reduce_bn1)
            const bool fuse = bn && N.P <= 4 * kBn1Threads && bn_split(N.P) == 1;
            // ... and so does the register-resident per-channel kernel for mid-size maps (k_bn_fwd_r)
            const int nq = bn ? bn_reg_q(N.P, N.P % 4 == 0 && al16(z) && al16(out) && al16(net->f(net->part_off))) : 0;
            // a 1x1 conv without BN applies its activation in the pointwise kernel's epilogue
            const bool act_in_pw = !bn && plain_unit(N.g) && wp;
            DirGeom dg;
            if (bn && N.sm && !N.upc && !(raw_first && i == 0) && N.P <= dir_max_p() && dir_geom(N.g, dg)) {
                // one launch: direct fp32 conv + BatchNorm (+act), one workgroup per output channel
                const BnArgs a{z, out, net->params + N.gm_off, net->params + N.bt_off, net->f(N.mean_off),
                               net->f(N.istd_off), net->bnstats + N.rs_off, net->bnstats + N.rs_off + N.C, nullptr, N.C,
                               (int)N.P, 1, (int)N.P, 1, N.d.act, 1e-5f, 0.1f, lip, 0};
                const float *xin = net->tensor(N.d.in0, x), *bias = net->params + N.b_off;
                const dim3 grid(1, N.C);
#define LRS_DIR(KS, S)                                                                                           \
    do {                                                                                                          \
        if (dg.vec4)                                                                                              \
            hipLaunchKernelGGL((k_conv_bn_dir<KS, S, true>), grid, dim3(kDirTh), 0, st, xin, w, bias, N.g, dg, a);  \
        else                                                                                                      \
            hipLaunchKernelGGL((k_conv_bn_dir<KS, S, false>), grid, dim3(kDirTh), 0, st, xin, w, bias, N.g, dg, a); \
    } while (0)
                if (N.g.k == 3 && N.g.stride == 1) LRS_DIR(3, 1);
                else if (N.g.k == 3) LRS_DIR(3, 2);
                else if (N.g.stride == 1) LRS_DIR(1, 1);
                else LRS_DIR(1, 2);
#undef LRS_DIR
                continue;
            }
            int nsplit = 1;
            if (N.upc) {   // upsampled 3 x 3: by output parity class
                rc = upc_fwd(N.g, net->tensor(N.d.in0, x), wp, net->params + N.b_off, N.C, z, net->f(net->part_off),
                             net->part_cap, st, (fuse || nq) ? &nsplit : nullptr);
            } else if (N.sm) {   // small map: implicit GEMM on k_conv_sm, no col written
                const int kk = N.g.k * N.g.k, Cp = r16(N.g.Cin);
                rc = sm_launch(SmPre{wp, (int64_t)N.C * kk * Cp, kk * Cp, N.C},
                               SmFwd{net->tensor(N.d.in0, x), N.g.Cin * N.g.Hs * N.g.Ws * 4, N.g, Cp, nullptr}, z,
                               net->params + N.b_off, N.C, (int)N.P, kk * Cp, 0, net->f(net->part_off), net->part_cap, st,
                               (fuse || nq) ? &nsplit : nullptr);
            } else {
                rc = conv_fwd(N.g, net->tensor(N.d.in0, x), w, net->params + N.b_off, N.C,
                              N.col_off >= 0 ? net->f(N.col_off) : nullptr, z, net->f(net->part_off), net->part_cap, st,
                              wp, (fuse || nq) ? &nsplit : nullptr, act_in_pw ? N.d.act : 0,
                              (head && i + 1 == net->nodes.size() && act_in_pw) ? head : nullptr);
            }
            if (rc) return rc;
            // the raw-weight first conv: its BatchNorm kernel needs the scale (and the GEMM left nsplit
            // > 1 partials: sn_overlap requires it)
            const float *sdiv = nullptr;
            if (raw_first && i == 0) {
                if (nsplit < 2 || !(nq || fuse)) return LRS_E_INVALID;   // sn_overlap's checks at creation
                const hipError_t e = hipStreamWaitEvent(st, net->ev_sigma, 0);
                if (e != hipSuccess) return (int)e;
                sdiv = net->f(net->scale_off) + N.sn_index;
            }
            if (act_in_pw) {
                rc = LRS_OK;
            } else if (nq) {
                const BnArgs a{z, out, net->params + N.gm_off, net->params + N.bt_off, net->f(N.mean_off),
                               net->f(N.istd_off), net->bnstats + N.rs_off, net->bnstats + N.rs_off + N.C, nullptr, N.C,
                               (int)N.P, 1, (int)N.P, 1, N.d.act, 1e-5f, 0.1f, lip, 1};
                const float *pp = nsplit > 1 ? (const float *)net->f(net->part_off) : nullptr;
                if (bnr_small_wg() && nq == 3 && N.P <= 4 * 256 * 10)
                    hipLaunchKernelGGL((k_bn_fwd_r<10, 256>), dim3(1, N.C), dim3(256), 0, st, pp, nsplit,
                                       (const float *)(net->params + N.b_off), a, sdiv);
                else
                    LRS_BNR_SWITCH(nq, k_bn_fwd_r, dim3(1, N.C), dim3(kBn1Threads), 0, st, pp, nsplit,
                                   (const float *)(net->params + N.b_off), a, sdiv);
                rc = LRS_OK;
            } else if (fuse && nsplit > 1) {
                const BnArgs a{z, out, net->params + N.gm_off, net->params + N.bt_off, net->f(N.mean_off),
                               net->f(N.istd_off), net->bnstats + N.rs_off, net->bnstats + N.rs_off + N.C, nullptr, N.C,
                               (int)N.P, 1, (int)N.P, 1, N.d.act, 1e-5f, 0.1f, lip, 0};
                if (bn1_threads(N.P) == kBn1Small)
                    hipLaunchKernelGGL(k_reduce_bn1<kBn1Small>, dim3(1, N.C), dim3(kBn1Small), 0, st,
                                       (const float *)net->f(net->part_off), nsplit, (const float *)(net->params + N.b_off), a,
                                       sdiv);
                else
                    hipLaunchKernelGGL(k_reduce_bn1<kBn1Threads>, dim3(1, N.C), dim3(kBn1Threads), 0, st,
                                       (const float *)net->f(net->part_off), nsplit, (const float *)(net->params + N.b_off), a,
                                       sdiv);
                rc = LRS_OK;
            } else {
                rc = bn_fwd(z, out, bn ? net->params + N.gm_off : nullptr, bn ? net->params + N.bt_off : nullptr,
                            net->f(N.mean_off), net->f(N.istd_off), bn ? net->bnstats + N.rs_off : nullptr,
                            bn ? net->bnstats + N.rs_off + N.C : nullptr, N.C, N.P, N.d.act, 1e-5f, 0.1f, net->bnpart(), st,
                            lip);
            }
        } else if (N.d.kind == LRS_NODE_BN) {
            rc = bn_fwd(net->tensor(N.d.in0, x), out, net->params + N.gm_off, net->params + N.bt_off,
                        net->f(N.mean_off), net->f(N.istd_off), net->bnstats + N.rs_off, net->bnstats + N.rs_off + N.C,
                        N.C, N.P, N.d.act, 1e-5f, 0.1f, net->bnpart(), st, lip);
        } else {
            const int q = N.cg.H * ((N.cg.W + 3) / 4);
            if (N.cg.Ca + N.cg.Cb > 65535 || !al16(out)) return LRS_E_UNSUPPORTED;
            hipLaunchKernelGGL(k_concat_fwd4, dim3((unsigned)((q + 255) / 256), (unsigned)(N.cg.Ca + N.cg.Cb)), dim3(256),
                               0, st, net->tensor(N.d.in0, x), net->tensor(N.d.in1, x), N.cg, out);
            rc = LRS_OK;
        }
        if (rc) return rc;
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

struct EsJob {   // the early-stopping update of this step's output, run beside the backward (dipnet_step)
    const float *out;
    int64_t N;
    float *ring;
    lrs_es_state *es;
};
int es_update(const float *out, int64_t N, float *ring, lrs_es_state *es, hipStream_t st);
int dipnet_backward(lrs_dipnet *net, const float *x, hipStream_t st, bool head_done = false, AdamPend *pw = nullptr,
                    bool head_reduce = false, const EsJob *esj = nullptr);
int mse_head(lrs_dipnet *net, const float *out, const float *target, const float *mask, hipStream_t st);

// k_mse_head over the last node (conv without BN): gz and the bias gradient of that node, + loss
int mse_head(lrs_dipnet *net, const float *out, const float *target, const float *mask, hipStream_t st) {
    const auto &N = net->nodes.back();
    float *gz = net->f(N.gz_off);
    const int64_t P = N.P;
    const int vec = (P % 4 == 0 && al16(out) && al16(target) && (!mask || al16(mask)) && al16(gz)) ? 1 : 0;
    int64_t S = bn_split(P);   // ~4096 pixels per workgroup
    int64_t chunk = (P + S - 1) / S;
    if (vec) chunk = (chunk + 3) & ~(int64_t)3;
    S = (P + chunk - 1) / chunk;
    // partials: bias [C][S], loss [C][S], channel losses [C]  (bn_part_doubles = 3 C bn_split(P))
    if (chunk > INT32_MAX || P > INT32_MAX || 2 * (int64_t)N.C * S + N.C > bn_part_doubles(N.C, P))
        return LRS_E_UNSUPPORTED;
    hipLaunchKernelGGL(k_mse_head, dim3((unsigned)S, (unsigned)N.C), dim3(256), 0, st, out, target, mask, N.C, P,
                       (int)chunk, vec, N.d.act, gz, net->loss_acc(), net->bnpart(), net->headcnt(),
                       net->grads + N.b_off);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int dipnet_step(lrs_dipnet *net, const float *x, const float *target, const float *mask, float lr, float b1, float b2,
                float eps, lrs_es_state *es, float *ring, hipStream_t st) {
    // the weight-preparation launch at the head of the forward also zeroes the loss accumulator
    // and advances Adam's step counter (read only by this step's k_adam); without one, a tiny launch
    const bool folded = net->n_prep > 0;
    // (the workspace's 16-B alignment completes the conditions lrs_dipnet_create checked: every
    // buffer offset is a multiple of 256 B, so the first conv's BatchNorm kernel then takes the
    // register / fused form the overlap needs, and the forward cannot refuse it mid-step)
    const bool overlap = net->sn_overlap && net->side && net->ev_head && net->ev_sigma && (!net->split_ev || net->ev_prep) &&
                         al16(net->ws);
    if (overlap) {
        // the spectral-norm Grams here (alone they take 19 us at 196^2; on the side stream beside the
        // first conv, 50), then the rest of the chain (Gram reduce, Lanczos) and the preparation of every
        // conv but the first on the side stream beside the first conv, whose planes come from the raw
        // weights here
        // (the Gram reduce too: on the side stream beside the first conv it took 23 us instead of 6)
        // the first conv's planes on 8 grid rows of kSnSplit workgroups (one row: the kernel took 36.7 us,
        // its 16 plane workgroups the longest; 8 rows: 19.2 us, 196^2 step 1.194 -> 1.177 ms, 3 interleaved
        // rounds, profiles/r06/ab/head_plane_rows.txt; LRS_DIP_HEAD_PLANE_ROWS, tuning only)
        static const int prow = (int)std::max<int64_t>(1, std::min<int64_t>(64, tune_knob("LRS_DIP_HEAD_PLANE_ROWS", 8)));
        hipLaunchKernelGGL(k_sn_gram_head, dim3(kSnSplit, net->n_sn + prow), dim3(256), 0, st, net->table(), net->gram(),
                           net->n_sn, (const ConvPrep *)net->prep_head(), net->loss_acc(), net->step());
        hipLaunchKernelGGL(k_sn_gram_reduce, dim3(kSnPairs, net->n_sn), dim3(256), 0, st, net->table(), net->gram());
        hipError_t e = hipEventRecord(net->ev_head, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(net->side, net->ev_head, 0);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_sn_sigma, dim3(net->n_sn), dim3(256), 0, net->side, net->table(), net->gram(),
                           net->f(net->sigma_off), net->f(net->scale_off), net->ln_lambda, (long long *)nullptr);
        if (net->split_ev && (e = hipEventRecord(net->ev_sigma, net->side)) != hipSuccess) return (int)e;
        const bool split = net->prep_split && net->ev_wd;
        if (net->n_prep_side)
            hipLaunchKernelGGL(k_conv_prep, dim3(prep_blocks(), net->n_prep_side), dim3(256), 0, net->side,
                               split ? net->prep_fs() : net->prep_side(), net->f(net->scale_off), (double *)nullptr,
                               net->step());
        e = hipEventRecord(net->split_ev ? net->ev_prep : net->ev_sigma, net->side);
        if (e != hipSuccess) return (int)e;
        if (split && net->n_prep_d) {   // the data-gradient planes after the forward's (the backward waits)
            hipLaunchKernelGGL(k_conv_prep, dim3(prep_blocks(), net->n_prep_d), dim3(256), 0, net->side, net->prep_d(),
                               net->f(net->scale_off), (double *)nullptr, net->step());
            if ((e = hipEventRecord(net->ev_wd, net->side)) != hipSuccess) return (int)e;
            net->wd_pending = true;
        }
        LRS_CHECK_LAUNCH();
    }
    const int n = (int)net->nodes.size();
    const auto &Lst = net->nodes[n - 1];
    // the loss head in the last conv's epilogue (k_pw): gz, and per-workgroup sums for the bias gradient
    // and the loss, reduced in the backward on the side stream (k_mse_head's arithmetic per element)
    const PwHead hd{target, mask, net->f(Lst.gz_off), net->hpart(), (float)(2.0 / ((double)Lst.C * (double)Lst.P)),
                    &net->head_nwg};
    const bool fused_head = net->head_pw && (!mask || al16(mask)) && al16(target);
    int rc = dipnet_forward(net, x, st, folded, overlap, fused_head ? &hd : nullptr);
    if (rc) return rc;
    const float *out = net->f(Lst.out_off);
    if (!folded) hipLaunchKernelGGL(k_step_begin, dim3(1), dim3(64), 0, st, net->loss_acc(), net->step());
    if (fused_head) {
        rc = LRS_OK;
    } else if (net->head_fusable) {
        rc = mse_head(net, out, target, mask, st);
    } else {
        rc = lrs_masked_mse_f32(out, target, mask, Lst.C, Lst.P, net->f(Lst.grad_off), net->loss_acc(), st);
    }
    if (rc) return rc;
    // the input conv's weight-gradient split-K sum is finished inside Adam (one launch less on the
    // step's tail)
    AdamPend pw{};
    // (LRS_DIP_ES_SIDE=0, tuning only: the ES update after Adam on this stream, as until round 6)
    static const bool es_side = tune_knob("LRS_DIP_ES_SIDE", 1) != 0;
    const EsJob esj{out, (int64_t)Lst.C * Lst.P, ring, es};
    const bool es_beside = es && es_side && net->fork_w;
    rc = dipnet_backward(net, x, st, net->head_fusable, &pw, fused_head, es_beside ? &esj : nullptr);
    if (rc) return rc;
    hipLaunchKernelGGL(k_adam, dim3(ew_blocks((net->n_params + 3) / 4, 8192)), dim3(kEw), 0, st, net->params,
                       (const float *)net->grads, net->am, net->av, net->n_params, (const int *)net->step(), lr, b1, b2,
                       eps, pw);
    if (es && !es_beside) {
        rc = es_update(out, (int64_t)Lst.C * Lst.P, ring, es, st);
        if (rc) return rc;
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// Backward from dL/d(output) already in the last node's gradient buffer: every parameter
// gradient into net->grads (the input gets none: the reference's DIP input needs no gradient).
// Weight gradient of conv node i on stream ws: reads dL/dz, the layer input and the scale only.
// scratch: its split-K partials (part2 on the side stream; part on the main one)
// split-K workgroup target of the weight gradients on the side stream (LRS_DIP_WGRAD_SPLIT_WG, tuning
// only): fewer splits write fewer partials and hold fewer CUs beside the data-gradient chain
inline int wgrad_split_target() {
    static const int v = (int)std::max<int64_t>(1, std::min<int64_t>(512, tune_knob("LRS_DIP_WGRAD_SPLIT_WG", 512)));
    return v;
}

int weight_grad(lrs_dipnet *net, int i, const float *x, hipStream_t ws, float *scratch, int *wsplit_out = nullptr) {
    if (wsplit_out) *wsplit_out = 1;
    const int wt = ws == net->side ? wgrad_split_target() : 512;
    auto &N = net->nodes[i];
    const int t = N.d.in0;
    const float *gz = net->f(N.gz_off);
    const float *colsrc = N.col_off >= 0 ? net->f(N.col_off) : net->tensor(t, x);
    const bool sn = N.sn_index >= 0;
    const float *w = sn ? net->f(N.wn_off) : net->params + N.w_off;
    const float *wdiv = sn ? net->f(net->scale_off) + N.sn_index : nullptr;
    if (N.sm && N.wtab_off >= 0) {   // implicit col^T on k_conv_sm (SmWgrad), dW / scale in its epilogue
        const int P = (int)N.P, kk = N.g.k * N.g.k;
        return sm_launch(SmDense{gz, P, N.C},
                         SmWgrad{net->tensor(t, x), N.g.Cin * N.g.Hs * N.g.Ws * 4, (int)N.Kc, kk, P,
                                 N.g.Hs * N.g.Ws * 4, (const int *)net->f(N.wtab_off)},
                         net->grads + N.w_off, nullptr, N.C, (int)N.Kc, P, 0, scratch, net->part_cap, ws, nullptr, wdiv,
                         true);
    }
    if (N.sm) {   // the forward gathered inside k_conv_sm: the col for the weight gradient now
        const int P = N.g.Ho * N.g.Wo;
        const dim3 grid((unsigned)((P + 255) / 256), (unsigned)std::min<int64_t>(N.Kc, 65535));
        hipLaunchKernelGGL(k_im2col, grid, dim3(256), 0, ws, net->tensor(t, x), N.g, net->f(N.col_off));
    }
    if (N.upc)
        return upc_wgrad(N.g, gz, net->tensor(t, x), wdiv, N.C, net->grads + N.w_off, scratch, net->part_cap, ws, wt);
    return conv_bwd(N.g, gz, colsrc, w, wdiv, N.C, nullptr, net->grads + N.w_off, nullptr, scratch, net->part_cap, ws, 0,
                    N.col_off < 0, nullptr, wsplit_out, wt);
}

// Is conv node i a fork point of the weight-gradient side stream (Node::fork_pt, lrs_dipnet_create)?
// LRS_DIP_FORK_SET (tuning only) = the node indices that fork instead, e.g. "13,12,11,10,7,4,1,0".
bool fork_at(const lrs_dipnet *net, int i) {
    static const char *set = tune_str("LRS_DIP_FORK_SET");
    if (!set) return net->nodes[i].fork_pt;
    for (const char *p = set; *p;) {
        char *e = nullptr;
        const long v = strtol(p, &e, 10);
        if (e == p) break;
        if (v == i) return true;
        p = (*e == ',' || *e == '.') ? e + 1 : e;   // '.' too (tools/gpu.sh specs split on ',')
    }
    return false;
}

// A conv's data gradient and weight gradient as ONE launch (k_gemm_s3x2: the data-gradient tiles
// first, then the weight-gradient tiles; both read dL/dz), then the fold of the data gradient and the
// weight gradient's split-K sum, all on stream st: no side-stream fork for this conv.  The stride-1
// implicit convs (LdDgradTM over the padded domain) and the parity-class upsampled ones.  Returns
// LRS_E_UNSUPPORTED for a conv it does not take (the caller keeps the two-stream path).
// Tuning build only (LRS_DIP_GROUP=1): parity-green, but the 196^2 step takes 1.259 ms against 1.189
// with the side stream (profiles/r06/ab/grouped_backward.txt): the weight gradients'
// overlap with the folds and BatchNorm kernels is worth more than the forks it saves.
#ifdef LRS_TUNING
int group_bwd_conv(lrs_dipnet *net, int i, const float *x, float *gx, int accum_gx, hipStream_t st) {
    auto &N = net->nodes[i];
    const ConvGeom &g = N.g;
    if (N.sm || N.col_off >= 0 || plain_unit(g) || N.wpre_off < 0 || !gx) return LRS_E_UNSUPPORTED;
    const float *gz = net->f(N.gz_off), *xin = net->tensor(N.d.in0, x);
    const bool sn = N.sn_index >= 0;
    const float *wdiv = sn ? net->f(net->scale_off) + N.sn_index : nullptr;
    float *gw = net->grads + N.w_off, *part = net->f(net->part_off), *part3 = net->f(net->part3_off);
    float *dcol = net->f(net->dcol_off);
    const int64_t cap = net->part_cap;
    const int P = (int)N.P, Cout = N.C, Cop = r16(Cout);
    if (N.upc) {
        const int K1 = 16 * Cop, Qe = (g.Hs + 2) * (g.Ws + 2), Q = g.Hs * g.Ws, N2 = 4 * g.Cin;
        const Split s1 = choose_split(g.Cin, Qe, K1, LRS_DIP_SPLIT_BF16, true, dgrad_split_target());
        const Split s2 = choose_split(Cout, 4 * N2, Q, LRS_DIP_SPLIT_BF16, true);
        if ((s1.S > 1 && cap < (int64_t)s1.S * g.Cin * Qe) || cap < (int64_t)s2.S * 4 * Cout * N2) return LRS_E_WORKSPACE;
        const GemmArgs a1{nullptr, nullptr, s1.S > 1 ? part : dcol, nullptr, nullptr, g.Cin, Qe, K1, s1.kchunk, 0};
        const GemmArgs a2{nullptr, nullptr, part3, nullptr, nullptr, Cout, N2, Q, s2.kchunk, 0, 4, g.Ws, 0, 0};
        const S3Grid d1{(unsigned)((Qe + 127) / 128), (unsigned)((g.Cin + 127) / 128), (unsigned)s1.S};
        const S3Grid d2{(unsigned)((N2 + 127) / 128), (unsigned)((Cout + 127) / 128), (unsigned)(4 * s2.S)};
        const unsigned nwg = ((d1.x * d1.y * d1.z + 7) & ~7u) + d2.x * d2.y * d2.z;
        const __bf16 *wd = (const __bf16 *)net->f(N.wpre_off) + wprep_fwd_elems(g, Cout, true);
        hipLaunchKernelGGL((k_gemm_s3x2<LdPre, LdUpDgradTM, LdGzCls, LdWgradCls>), dim3(nwg), dim3(kGemmThreads), 0, st, a1,
                           LdPre{wd, (int64_t)g.Cin * K1, K1, g.Cin}, LdUpDgradTM{gz, Cout * g.Ho * g.Wo * 4, g, Cout, Cop, nullptr},
                           d1, a2, LdGzCls{gz, g.Hs, g.Ws, g.Wo, Cout, 0}, LdWgradCls{xin, g.Cin * Q * 4, g, nullptr, 0, 0}, d2);
        ConvGeom fg = g;
        fg.up = 0; fg.Hu = g.Hs; fg.Wu = g.Ws; fg.pad = 1; fg.pad_mode = kPadClamp;
        hipLaunchKernelGGL(k_fold_pad, dim3((unsigned)((Q + 255) / 256), (unsigned)std::min(g.Cin, 65535)), dim3(256), 0, st,
                           s1.S > 1 ? part : dcol, s1.S, (int64_t)g.Cin * Qe, fg, gx, accum_gx);
        const int64_t n = (int64_t)Cout * g.Cin * 9;
        hipLaunchKernelGGL(k_upc_wgrad_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const float *)part3, s2.S,
                           Cout, g.Cin, wdiv, gw);
        LRS_CHECK_LAUNCH();
        return LRS_OK;
    }
    const int kk = g.k * g.k, Qp = (g.Hu + 2 * g.pad) * (g.Wu + 2 * g.pad), Kc = (int)N.Kc;
    if (g.stride != 1 || up_eff_k(g) || (int64_t)g.Cin * Qp > (int64_t)Kc * P || !conv_implicit_ok(g, Cout))
        return LRS_E_UNSUPPORTED;
    const Split s1 = choose_split(g.Cin, Qp, kk * Cop, LRS_DIP_SPLIT_BF16, true, dgrad_split_target());
    const Split s2 = choose_split(Cout, Kc, P, LRS_DIP_SPLIT_BF16, true);
    if ((s1.S > 1 && cap < (int64_t)s1.S * g.Cin * Qp) || (s2.S > 1 && cap < (int64_t)s2.S * Cout * Kc))
        return LRS_E_WORKSPACE;
    const GemmArgs a1{nullptr, nullptr, s1.S > 1 ? part : dcol, nullptr, nullptr, g.Cin, Qp, kk * Cop, s1.kchunk, 0};
    const GemmArgs a2{nullptr, nullptr, s2.S > 1 ? part3 : gw, nullptr, wdiv, Cout, Kc, P, s2.kchunk, 0};
    const S3Grid d1{(unsigned)((Qp + 127) / 128), (unsigned)((g.Cin + 127) / 128), (unsigned)s1.S};
    const S3Grid d2{(unsigned)((Kc + 127) / 128), (unsigned)((Cout + 127) / 128), (unsigned)s2.S};
    const unsigned nwg = ((d1.x * d1.y * d1.z + 7) & ~7u) + d2.x * d2.y * d2.z;
    const __bf16 *wd = (const __bf16 *)net->f(N.wpre_off) + wprep_fwd_elems(g, Cout);
    hipLaunchKernelGGL((k_gemm_s3x2<LdPre, LdDgradTM, LdDense<true>, LdWgradTM>), dim3(nwg), dim3(kGemmThreads), 0, st, a1,
                       LdPre{wd, (int64_t)g.Cin * kk * Cop, kk * Cop, g.Cin}, LdDgradTM{gz, Cout * P * 4, g, Cout, Cop, nullptr},
                       d1, a2, LdDense<true>{gz, P, Cout}, LdWgradTM{xin, g.Cin * g.Hs * g.Ws * 4, g, nullptr, 0}, d2);
    if (s1.S == 1 && !g.up && g.Ws % 4 == 0 && g.Cin <= 65535 && al16(gx)) {
        const int q = g.Hs * (g.Ws / 4);
        hipLaunchKernelGGL(k_fold_pad1q, dim3((unsigned)((q + 255) / 256), (unsigned)g.Cin), dim3(256), 0, st, (const float *)dcol,
                           g, gx, accum_gx);
    } else {
        hipLaunchKernelGGL(k_fold_pad, dim3((unsigned)((g.Hs * g.Ws + 255) / 256), (unsigned)std::min(g.Cin, 65535)), dim3(256), 0,
                           st, (const float *)(s1.S > 1 ? part : dcol), s1.S, (int64_t)g.Cin * Qp, g, gx, accum_gx);
    }
    if (s2.S > 1) {
        const int64_t MN = (int64_t)Cout * Kc;
        hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)((MN + kEw - 1) / kEw)), dim3(kEw), 0, st, (const float *)part3, s2.S,
                           Cout, Kc, (const float *)nullptr, wdiv, 0, gw);
    }
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
#endif

// pw (lrs_dipnet_train_steps): the input conv's weight gradient may leave its split-K partials for
// k_adam to finish (AdamPend; pw->part == nullptr when nothing is pending)
int dipnet_backward(lrs_dipnet *net, const float *x, hipStream_t st, bool head_done, AdamPend *pw, bool head_reduce,
                    const EsJob *esj) {
    int rc;
    const int n = (int)net->nodes.size();
    // the ES update reads only the forward's output and its own ring: on the side stream with the first
    // weight gradients (its ring slot and window sums follow the previous step's there), joined before Adam
    auto es_side = [&](hipStream_t hs) -> int {
        if (!esj) return LRS_OK;
        const int r = es_update(esj->out, esj->N, esj->ring, esj->es, hs);
        esj = nullptr;
        return r;
    };
    // the fused loss head's sums (PwHead): the bias gradient of the last conv (read by Adam only) and the
    // loss, on the side stream with the first weight gradients (or here, without a side stream)
    auto head_sums = [&](hipStream_t hs) {
        if (!head_reduce) return;
        const auto &Lh = net->nodes[n - 1];
        hipLaunchKernelGGL(k_head_reduce, dim3((unsigned)Lh.C), dim3(256), 0, hs, (const double *)net->hpart(), Lh.C,
                           net->head_nwg, net->grads + Lh.b_off, net->closs());
        hipLaunchKernelGGL(k_head_loss, dim3(1), dim3(64), 0, hs, (const double *)net->closs(), Lh.C, net->loss_acc());
        head_reduce = false;
    };
    if (!net->fork_w) head_sums(st);
    if (net->wd_pending) {   // the data-gradient planes prepared on the side stream (prep_split)
        const hipError_t e = hipStreamWaitEvent(st, net->ev_wd, 0);
        if (e != hipSuccess) return (int)e;
        net->wd_pending = false;
    }
    // gradient buffers: the first contribution to a tensor writes, later ones accumulate
    std::vector<char> written(n + 1, 0);
    written[n] = 1;
    // weight gradients queued for the side stream, launched after the fork that follows node j's BN
    // backward (every queued node's dL/dz is complete by then)
    std::vector<int> wq;
    int first_conv = 0;
    while (first_conv < n && net->nodes[first_conv].d.kind != LRS_NODE_CONV) ++first_conv;
    auto flush_w = [&](int j) -> int {
        if (wq.empty()) return LRS_OK;
        hipError_t e = hipEventRecord(net->ev_fork[j], st);
        if (e == hipSuccess) e = hipStreamWaitEvent(net->side, net->ev_fork[j], 0);
        if (e != hipSuccess) return (int)e;
        head_sums(net->side);
        if (const int r = es_side(net->side)) return r;
        for (int q : wq)
            if (const int r = weight_grad(net, q, x, net->side, net->f(net->part2_off))) return r;
        wq.clear();
        return LRS_OK;
    };
    // a small-map data gradient may leave dL/dy of the next node as split-K partials, finished by
    // that node's k_reduce_bn_bwd1 (pend = the partials, pend_S their count)
    const float *pend = nullptr;
    int pend_S = 0;
    for (int i = n - 1; i >= 0; --i) {
        auto &N = net->nodes[i];
        float *gout = net->f(N.grad_off);
        float *outp = net->f(N.out_off);
        const int lip = N.d.bn == 2 ? 1 : 0;
        if (!written[i + 1]) continue;   // output unused by the loss (cannot happen for a valid net)
        if (N.d.kind == LRS_NODE_CONV) {
            const bool bn = N.d.bn != 0;
            float *z = bn ? net->f(N.z_off) : outp;
            float *gz = net->f(N.gz_off);
            if (pend) {
                const BnBwdArgs a{nullptr, outp, z, net->params + N.gm_off, net->f(N.mean_off), net->f(N.istd_off), gz,
                                  net->grads + N.gm_off, net->grads + N.bt_off, net->grads + N.b_off, nullptr, N.C,
                                  (int)N.P, 1, (int)N.P, 1, N.d.act, lip, 0, 0, net->params + N.bt_off};
                if (bn1_threads(N.P) == kBn1Small)
                    hipLaunchKernelGGL(k_reduce_bn_bwd1<kBn1Small>, dim3(1, N.C), dim3(kBn1Small), 0, st, pend, pend_S, a);
                else
                    hipLaunchKernelGGL(k_reduce_bn_bwd1<kBn1Threads>, dim3(1, N.C), dim3(kBn1Threads), 0, st, pend, pend_S, a);
                pend = nullptr;
            } else if (!(head_done && i == n - 1)) {   // else k_mse_head wrote gz and the bias gradient
                rc = bn_bwd(gout, outp, z, bn ? net->params + N.gm_off : nullptr, net->f(N.mean_off),
                            net->f(N.istd_off), gz, bn ? net->grads + N.gm_off : nullptr,
                            bn ? net->grads + N.bt_off : nullptr, net->grads + N.b_off, N.C, N.P, N.d.act,
                            net->bnpart(), st, lip, 0, bn ? net->params + N.bt_off : nullptr);
                if (rc) return rc;
            }
            const int t = N.d.in0;
            const float *colsrc = N.col_off >= 0 ? net->f(N.col_off) : net->tensor(t, x);
            const bool sn = N.sn_index >= 0;
            const float *w = sn ? net->f(N.wn_off) : net->params + N.w_off;
            float *gx = t > 0 ? net->f(net->nodes[t - 1].grad_off) : nullptr;
            const float *wdiv = sn ? net->f(net->scale_off) + N.sn_index : nullptr;
#ifdef LRS_TUNING
            // grouped (tuning build): data and weight gradient in one launch on this stream
            if (net->group_bwd && gx) {
                rc = group_bwd_conv(net, i, x, gx, written[t], st);
                if (rc == LRS_OK) {
                    written[t] = 1;
                    continue;
                }
                if (rc != LRS_E_UNSUPPORTED) return rc;
            }
#endif
            // weight gradient on the side stream (reads gz, the layer input and the scale only); the
            // nodes between two fork points queue theirs until the next one (fork_at)
            if (net->fork_w && !(t == 0 && i == first_conv)) {
                wq.push_back(i);
                if (fork_at(net, i) && (rc = flush_w(i))) return rc;
            } else {
                // no fork: or the first conv on the input, after which the main stream has no work left
                // of its own (a fork there only adds the event latency to the step's tail); it uses the
                // main stream's scratch, free by then, beside whatever the side stream still runs
                if (net->fork_w && (rc = flush_w(i))) return rc;
                int wsplit = 1;
                // (LRS_DIP_DEFER_EXPLICIT=0, tuning only: the explicit (small-map) input conv's sum by
                // k_gemm_reduce instead, as before round 6)
                static const bool defer_explicit = tune_knob("LRS_DIP_DEFER_EXPLICIT", 1) != 0;
                const bool defer = pw && t == 0 && i == first_conv && (defer_explicit || N.col_off < 0);
                if ((rc = weight_grad(net, i, x, st, net->f(net->part_off), defer ? &wsplit : nullptr))) return rc;
                if (defer && wsplit > 1)
                    *pw = AdamPend{net->f(net->part_off), wsplit, N.w_off, (int64_t)N.C * N.Kc,
                                   N.sn_index >= 0 ? net->f(net->scale_off) + N.sn_index : nullptr,
                                   net->grads};
            }
            if (gx && N.upc) {   // by output parity class over the extended source grid, then the clamp fold
                rc = upc_dgrad(N.g, gz, (const __bf16 *)net->f(N.wpre_off) + wprep_fwd_elems(N.g, N.C, true), N.C, gx,
                               net->f(net->dcol_off), net->f(net->part_off), net->part_cap, st, written[t]);
                if (rc) return rc;
            } else if (gx && N.sm_dgrad) {   // gx = the adjoint gather of dL/dz on k_conv_sm, one GEMM
                const auto &g = N.g;
                const int kk = g.k * g.k, Cop = r16(N.C);
                const __bf16 *wd = (const __bf16 *)net->f(N.wpre_off) + wprep_fwd_elems(g, N.C);
                const SmPre la{wd, (int64_t)g.Cin * kk * Cop, kk * Cop, g.Cin};
                const int4 *adj = (const int4 *)net->f(N.adj_off);
                // the next node (t - 1 = i - 1, this tensor's only other writer would come before it)
                // finishes the split-K sum inside its BN backward when that fits one workgroup
                const bool fuse_next = t == i && !written[t] && bn_bwd_fusable(net, t - 1) && !(head_done && t - 1 == n - 1);
                int nsplit = 1;
                rc = sm_launch(la, SmAdj{gz, (int)(N.C * N.P * 4), g, N.C, Cop, adj, nullptr}, gx, nullptr, g.Cin,
                               g.Hs * g.Ws, kk * Cop, written[t], net->f(net->part_off), net->part_cap, st,
                               fuse_next ? &nsplit : nullptr);
                if (rc) return rc;
                if (fuse_next && nsplit > 1) {
                    pend = net->f(net->part_off);
                    pend_S = nsplit;
                }
            } else if (gx) {
                rc = conv_bwd(N.g, gz, colsrc, w, wdiv, N.C, gx, nullptr,
                              !plain_unit(N.g) ? net->f(net->dcol_off) : nullptr, net->f(net->part_off),
                              net->part_cap, st, written[t], N.col_off < 0,
                              N.wpre_off >= 0 ? (const __bf16 *)net->f(N.wpre_off) : nullptr);
                if (rc) return rc;
            }
            if (t > 0) written[t] = 1;
        } else if (N.d.kind == LRS_NODE_BN) {
            const int t = N.d.in0;
            if (t > 0) {
                rc = bn_bwd(gout, outp, net->tensor(t, x), net->params + N.gm_off, net->f(N.mean_off),
                            net->f(N.istd_off), net->f(net->nodes[t - 1].grad_off), net->grads + N.gm_off,
                            net->grads + N.bt_off, nullptr, N.C, N.P, N.d.act, net->bnpart(), st, lip, written[t],
                            net->params + N.bt_off);
                written[t] = 1;
            } else {   // BN straight on the input: parameter grads only
                rc = bn_bwd(gout, outp, net->tensor(t, x), net->params + N.gm_off, net->f(N.mean_off),
                            net->f(N.istd_off), net->f(net->dz_off), net->grads + N.gm_off, net->grads + N.bt_off,
                            nullptr, N.C, N.P, N.d.act, net->bnpart(), st, lip, 0, net->params + N.bt_off);
            }
            if (rc) return rc;
        } else {
            const int ta = N.d.in0, tb = N.d.in1;
            float *ga = ta > 0 ? net->f(net->nodes[ta - 1].grad_off) : nullptr;
            float *gb = tb > 0 ? net->f(net->nodes[tb - 1].grad_off) : nullptr;
            const int64_t na = ga ? (int64_t)N.cg.Ca * N.cg.Ha * N.cg.Wa : 0;
            const int64_t nb = gb ? (int64_t)N.cg.Cb * N.cg.Hb * N.cg.Wb : 0;
            if (na + nb > 0) {
                const int acc_a = ta > 0 ? written[ta] : 0;
                // both inputs may be the same tensor: the b pass must then accumulate onto the a pass
                const int acc_b = tb > 0 ? (written[tb] || (tb == ta)) : 0;
                // a then b (the same order as one launch over both when ta == tb)
                const CatGeom &cg = N.cg;
                if (ga) {
                    if (!al16(ga)) return LRS_E_UNSUPPORTED;
                    const int q = cg.Ha * ((cg.Wa + 3) / 4);
                    hipLaunchKernelGGL(k_concat_bwd4, dim3((unsigned)((q + 255) / 256), (unsigned)cg.Ca), dim3(256), 0,
                                       st, gout, cg, ga, acc_a, 0);
                }
                if (gb) {
                    if (!al16(gb)) return LRS_E_UNSUPPORTED;
                    const int q = cg.Hb * ((cg.Wb + 3) / 4);
                    hipLaunchKernelGGL(k_concat_bwd4, dim3((unsigned)((q + 255) / 256), (unsigned)cg.Cb), dim3(256), 0,
                                       st, gout, cg, gb, (ta == tb && ga) ? 1 : acc_b, 1);
                }
            }
            if (ta > 0) written[ta] = 1;
            if (tb > 0) written[tb] = 1;
        }
    }
    if (net->fork_w) {   // join the side stream before anyone reads the weight gradients
        if ((rc = flush_w(0))) return rc;
        hipError_t e = hipEventRecord(net->ev_join, net->side);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, net->ev_join, 0);
        if (e != hipSuccess) return (int)e;
    }
    head_sums(st);   // (only if no fork took them)
    if ((rc = es_side(st))) return rc;
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

extern "C" int lrs_dipnet_create(const lrs_dip_node *nodes, int n_nodes, int C, int H, int W,
                                 const lrs_dip_opts *opts, lrs_dipnet **out) {
    if (!nodes || n_nodes <= 0 || C <= 0 || H <= 0 || W <= 0 || !out) return LRS_E_INVALID;
    const lrs_dip_opts o = dip_opts(opts);
    if (o.precision != LRS_DIP_F32 && o.precision != LRS_DIP_SPLIT_BF16) return LRS_E_INVALID;
    if (o.upsample_dgrad != 0 && o.upsample_dgrad != 1) return LRS_E_INVALID;
    lrs_dipnet *net = new (std::nothrow) lrs_dipnet();
    if (!net) return LRS_E_INVALID;
    net->C0 = C;
    net->H = H;
    net->W = W;
    auto fail = [&](int rc) { delete net; return rc; };
    net->opts = o;
    net->implicit = o.precision == LRS_DIP_SPLIT_BF16;
    // weight gradients on a side stream at every size: beside the concurrent sparse-coding kernel
    // the second stream keeps the DIP its share of the chip (configs[2] 4.73 -> 5.19 outer it/s,
    // round 1); at 36^2 it was slower in round 1 (1.03 -> 1.19 ms per step) and is faster since the
    // small-map fork points pair up (round 4, interleaved: 0.729 -> 0.676 ms per step)
    net->fork_w = true;
    net->fork_w = tune_knob("LRS_DIP_FORK", net->fork_w ? 1 : 0) != 0;   // tuning build only
    int64_t pofs = 0, rofs = 0, ofs = 0, max_dz = 0, max_dcol = 0, part = 0, max_bnpart = 0;
    int n_sn = 0;
    for (int i = 0; i < n_nodes; ++i) {
        lrs_dipnet::Node N;
        N.d = nodes[i];
        const int t0 = N.d.in0;
        if (t0 < 0 || t0 > i) return fail(LRS_E_INVALID);
        if (N.d.act != LRS_ACT_NONE && N.d.act != LRS_ACT_LRELU && N.d.act != LRS_ACT_SIGMOID) return fail(LRS_E_INVALID);
        if (N.d.bn < 0 || N.d.bn > 2) return fail(LRS_E_INVALID);
        const int ci = net->tC(t0), hi = net->tH(t0), wi = net->tW(t0);
        if (N.d.kind == LRS_NODE_CONV) {
            if (N.d.cout <= 0) return fail(LRS_E_INVALID);
            int rc = make_geom(ci, hi, wi, N.d.k, N.d.stride, N.d.pad, N.d.pad_mode, N.d.upsample, N.g, &o);
            if (rc) return fail(rc);
            N.C = N.d.cout;
            N.H = N.g.Ho;
            N.W = N.g.Wo;
            N.P = (int64_t)N.H * N.W;
            N.Kc = (int64_t)ci * N.d.k * N.d.k;
            N.w_off = pofs; pofs += N.C * N.Kc;
            N.b_off = pofs; pofs += N.C;
            if (N.d.sn) {
                if ((N.Kc < N.C ? N.Kc : N.C) > kSnMaxDim) return fail(LRS_E_UNSUPPORTED);
                N.sn_index = n_sn++;
                N.wn_off = ofs; ofs += align64(N.C * N.Kc);
                if (N.C * N.Kc > net->max_w) net->max_w = N.C * N.Kc;
            }
            if (plain_unit(N.g) && net->implicit && pw_ok(N.g, N.C) && N.P >= implicit_min_pixels() &&
                wprep_elems(N.g, N.C) < INT32_MAX / 3) {
                N.wpre_off = ofs;   // 1x1 on k_pw: its pre-split weight planes
                ofs += align64((wprep_elems(N.g, N.C) + 1) / 2);
            }
            if (!plain_unit(N.g)) {
                if (!(net->implicit && conv_implicit_ok(N.g, N.C) && N.P >= implicit_min_pixels())) {
                    // col: the weight gradient's explicit im2col (written in the backward for a
                    // small-map conv, whose forward gathers it inside k_conv_sm)
                    N.col_off = ofs;
                    ofs += align64(N.Kc * N.P);
                    if (net->implicit && sm_enabled() && N.d.k <= 3 && conv_implicit_ok(N.g, N.C) &&
                        wprep_elems(N.g, N.C) < INT32_MAX / 3) {
                        N.sm = true;
                        N.wpre_off = ofs;
                        ofs += align64((wprep_elems(N.g, N.C) + 1) / 2);
                        if (N.P <= kSmWgradOneLaunchP && net->fork_w) {
                            N.wtab = sm_wgrad_table(N.g);
                            N.wtab_off = ofs;
                            ofs += align64((int64_t)N.wtab.size());
                        }
                        if (t0 > 0) {
                            N.adj = sm_adj_table(N.g);
                            N.sm_dgrad = !N.adj.empty();
                            if (N.sm_dgrad) {
                                N.adj_off = ofs;
                                ofs += align64((int64_t)N.adj.size());
                            }
                        }
                    }
                } else {
                    N.upc = upc_conv(N.g);
                    if ((N.upc ? wprep_elems(N.g, N.C, true) : wprep_elems(N.g, N.C)) >= INT32_MAX / 3)
                        return fail(LRS_E_UNSUPPORTED);   // k_conv_prep's 32-bit plane indices
                    N.wpre_off = ofs;
                    ofs += align64(((N.upc ? wprep_elems(N.g, N.C, true) : wprep_elems(N.g, N.C)) + 1) / 2);
                }
                if (N.Kc * N.P > max_dcol) max_dcol = N.Kc * N.P;
            }
            if (N.d.bn) { N.z_off = ofs; ofs += align64(N.C * N.P); }
            N.gz_off = ofs; ofs += align64(N.C * N.P);
            const int64_t pc = std::max(conv_part_floats(N.g, N.C), N.upc ? upc_part_floats(N.g, N.C) : 0);
            if (pc > part) part = pc;
            if (N.C * N.P > max_dz) max_dz = N.C * N.P;
        } else if (N.d.kind == LRS_NODE_BN) {
            if (!N.d.bn) N.d.bn = 1;
            N.C = ci;
            N.H = hi;
            N.W = wi;
            N.P = (int64_t)hi * wi;
            if (N.C * N.P > max_dz) max_dz = N.C * N.P;
        } else if (N.d.kind == LRS_NODE_CONCAT) {
            const int t1 = N.d.in1;
            if (t1 < 0 || t1 > i) return fail(LRS_E_INVALID);
            auto &cg = N.cg;
            cg.Ca = ci; cg.Ha = hi; cg.Wa = wi;
            cg.Cb = net->tC(t1); cg.Hb = net->tH(t1); cg.Wb = net->tW(t1); cg.upb = N.d.upsample ? 1 : 0;
            const int hb = cg.upb ? 2 * cg.Hb : cg.Hb, wb = cg.upb ? 2 * cg.Wb : cg.Wb;
            cg.H = hi < hb ? hi : hb;
            cg.W = wi < wb ? wi : wb;
            cg.oay = (hi - cg.H) / 2; cg.oax = (wi - cg.W) / 2;
            cg.oby = (hb - cg.H) / 2; cg.obx = (wb - cg.W) / 2;
            N.C = cg.Ca + cg.Cb;
            N.H = cg.H;
            N.W = cg.W;
            N.P = (int64_t)N.H * N.W;
            N.d.bn = 0;
        } else {
            return fail(LRS_E_INVALID);
        }
        // BN partials: every BN and every conv (its bias gradient is reduced the same way)
        if ((N.d.bn || N.d.kind == LRS_NODE_CONV) && bn_part_doubles(N.C, N.P) > max_bnpart)
            max_bnpart = bn_part_doubles(N.C, N.P);
        if (N.d.bn) {
            N.gm_off = pofs; pofs += N.C;
            N.bt_off = pofs; pofs += N.C;
            N.rs_off = rofs; rofs += 2 * N.C;
            N.mean_off = ofs; ofs += align64(N.C);
            N.istd_off = ofs; ofs += align64(N.C);
        } else if (N.d.kind == LRS_NODE_CONV) {
            N.mean_off = ofs; ofs += align64(N.C);   // unused placeholders (the kernels take them)
            N.istd_off = ofs; ofs += align64(N.C);
        }
        N.out_off = ofs; ofs += align64((int64_t)N.C * N.P);
        N.grad_off = ofs; ofs += align64((int64_t)N.C * N.P);
        net->nodes.push_back(N);
    }
    // Fork points: every conv forks its weight gradient to the side stream right after its BatchNorm
    // backward (Node::fork_pt stays true).  Until round 5 a run of small maps forked every second conv
    // (a fork cost the critical stream ~7 us with system-scope events); with the device-scope events
    // (ensure_side) forking at every conv is faster at both sizes: 196^2 1.192 -> 1.189 ms, 36^2 0.584
    // -> 0.580 ms (3 interleaved rounds, profiles/r06/ab/fork_sets.txt).  LRS_DIP_FORK_SET (tuning
    // build) still picks the fork points for A/B.
    net->n_sn = n_sn;
    net->n_params = pofs;
    net->n_bnstats = rofs;
    net->dz_off = ofs; ofs += align64(max_dz);
    net->dcol_off = ofs; ofs += align64(max_dcol);
    net->part_off = ofs; ofs += align64(part);
    net->part2_off = ofs; ofs += align64(part);
#ifdef LRS_TUNING
    net->group_bwd = tune_knob("LRS_DIP_GROUP", 0) != 0;
#endif
    if (net->group_bwd) { net->part3_off = ofs; ofs += align64(part); }
    net->part_cap = part;
    net->sigma_off = ofs; ofs += align64(n_sn > 0 ? n_sn : 1);
    net->scale_off = ofs; ofs += align64(n_sn > 0 ? n_sn : 1);
    size_t bytes = (size_t)ofs * sizeof(float);
    net->gram_off_bytes = (int64_t)bytes;
    bytes += (size_t)n_sn * kSnGramDoubles * sizeof(double);
    net->bnpart_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up((max_bnpart > 0 ? max_bnpart : 1) * (int64_t)sizeof(double), 256);
    net->table_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up((int64_t)((n_sn > 0 ? n_sn : 1) * sizeof(SnConv)), 256);
    for (const auto &N : net->nodes)
        if (N.d.kind == LRS_NODE_CONV && (N.sn_index >= 0 || N.wpre_off >= 0)) ++net->n_prep;
    net->prep_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up((int64_t)((net->n_prep > 0 ? net->n_prep : 1) * sizeof(ConvPrep)), 256);
    // sigma beside the first conv: a spectrally normalised first conv on the network input whose
    // BatchNorm kernel finishes its split-K sum (k_bn_fwd_r or k_reduce_bn1, at least 2 partials), read
    // from weight planes; only where the weight gradients already fork (the side stream exists)
    {
        const auto &N0 = net->nodes[0];
        bool ok = net->fork_w && n_sn > 0 && N0.d.kind == LRS_NODE_CONV && N0.d.in0 == 0 && N0.sn_index >= 0 &&
                  N0.d.bn && N0.wpre_off >= 0 && !plain_unit(N0.g) && !N0.upc;
        if (ok) {
            const bool fuse = N0.P <= 4 * kBn1Threads && bn_split(N0.P) == 1;
            const bool nq = bn_reg_q(N0.P, N0.P % 4 == 0) > 0;
            const int kk = N0.g.k * N0.g.k, K = kk * r16(N0.g.Cin);
            const int S = N0.sm ? sm_split(N0.C, (int)N0.P, K).S
                                : choose_split(N0.C, (int)N0.P, K, LRS_DIP_SPLIT_BF16, true, fwd_split_target()).S;
            // only where the first conv is long enough to hide the side chain (~70 us at 196^2: the Gram
            // reduce, Lanczos and the other convs' planes); at 36^2 the 18^2 first conv takes 7 us and the
            // overlap measured slower (tuning build: 0.647 -> 0.663 ms per step)
            ok = (fuse || nq) && S >= 2 && N0.P >= tune_knob("LRS_DIP_SN_OVERLAP_MINP", kForkBigP);
        }
        net->sn_overlap = ok && tune_knob("LRS_DIP_SN_OVERLAP", 1) != 0;
        // the first BatchNorm waits for the scale only, the second conv for the planes as well: 196^2 step
        // 1.185 -> 1.179 ms (3 interleaved rounds, profiles/r06/ab/split_event_and_es.txt)
        net->split_ev = net->sn_overlap && tune_knob("LRS_DIP_SPLIT_EV", 1) != 0;
    }
    net->n_prep_side = net->n_prep;
    net->prep_head_off_bytes = (int64_t)bytes;
    bytes += 256;   // one ConvPrep
    net->prep_side_off_bytes = (int64_t)bytes;
    bytes += (size_t)round_up((int64_t)((net->n_prep > 0 ? net->n_prep : 1) * sizeof(ConvPrep)), 256);
    {
        const int64_t tb = round_up((int64_t)((net->n_prep > 0 ? net->n_prep : 1) * sizeof(ConvPrep)), 256);
        net->prep_f_off_bytes = (int64_t)bytes;
        bytes += (size_t)tb;
        net->prep_fs_off_bytes = (int64_t)bytes;
        bytes += (size_t)tb;
        net->prep_d_off_bytes = (int64_t)bytes;
        bytes += (size_t)tb;
        // off: 196^2 1.189 -> 1.192 ms, 36^2 0.572 -> 0.576 ms with it (3 interleaved rounds,
        // profiles/r06/ab/prep_split_dropped.txt): the extra event and launch cost more than the half of
        // the preparation it takes off the critical stream (LRS_DIP_PREP_SPLIT=1, tuning only)
        net->prep_split = net->fork_w && net->n_prep > 0 && tune_knob("LRS_DIP_PREP_SPLIT", 0) != 0;
    }
    net->head_fusable = net->nodes.back().d.kind == LRS_NODE_CONV && net->nodes.back().d.bn == 0 &&
                        net->nodes.back().C <= 65535;
    {
        const auto &Lh = net->nodes.back();
        // only on small maps: 36^2 step 0.578 -> 0.571 ms, but 196^2 1.187 -> 1.192 ms (3 interleaved rounds,
        // profiles/r06/ab/fused_head.txt): there the epilogue's extra 60 MB (target in, gz out) lengthens
        // the 481-workgroup conv by more than the separate k_mse_head launch costs
        net->head_pw = net->head_fusable && plain_unit(Lh.g) && Lh.wpre_off >= 0 && tune_knob("LRS_DIP_HEAD_PW", 1) != 0 &&
                       Lh.P <= tune_knob("LRS_DIP_HEAD_PW_MAXP", 4096);
        if (net->head_pw) {
            net->hpart_off_bytes = (int64_t)bytes;   // [2][C][<= ceil(P / 64) workgroups]
            bytes += (size_t)round_up(2 * (int64_t)Lh.C * ((Lh.P + 63) / 64) * 8, 256);
            net->closs_off_bytes = (int64_t)bytes;
            bytes += (size_t)round_up((int64_t)Lh.C * 8, 256);
        }
    }
    net->headcnt_off_bytes = (int64_t)bytes;   // C per-channel counters + the channel counter
    bytes += (size_t)round_up((int64_t)(net->nodes.back().C + 1) * 4, 256);
    net->misc_off_bytes = (int64_t)bytes;
    bytes += 256;
    net->ws_bytes = bytes;
    net->ev_fork.assign(net->nodes.size(), nullptr);   // side stream + events: ensure_side()
    *out = net;
    return LRS_OK;
}

extern "C" void lrs_dipnet_destroy(lrs_dipnet *net) {
    if (!net) return;
    drop_graph(net);
    for (auto &ps : net->sides) (void)hipStreamSynchronize(ps.second);
    for (hipEvent_t ev : net->ev_fork)
        if (ev) (void)hipEventDestroy(ev);
    if (net->ev_join) (void)hipEventDestroy(net->ev_join);
    if (net->ev_head) (void)hipEventDestroy(net->ev_head);
    if (net->ev_sigma) (void)hipEventDestroy(net->ev_sigma);
    if (net->ev_prep) (void)hipEventDestroy(net->ev_prep);
    if (net->ev_wdgo) (void)hipEventDestroy(net->ev_wdgo);
    if (net->ev_wd) (void)hipEventDestroy(net->ev_wd);
    for (auto &ps : net->sides) (void)hipStreamDestroy(ps.second);
    delete net;
}

extern "C" int64_t lrs_dipnet_num_params(const lrs_dipnet *net) { return net ? net->n_params : -1; }
extern "C" int64_t lrs_dipnet_num_bnstats(const lrs_dipnet *net) { return net ? net->n_bnstats : -1; }
extern "C" size_t lrs_dipnet_workspace(const lrs_dipnet *net) { return net ? net->ws_bytes : 0; }

extern "C" int lrs_dipnet_param_offsets(const lrs_dipnet *net, int node, int64_t *w, int64_t *b, int64_t *gamma,
                                        int64_t *beta) {
    if (!net || node < 0 || node >= (int)net->nodes.size()) return LRS_E_INVALID;
    const auto &N = net->nodes[node];
    if (w) *w = N.w_off;
    if (b) *b = N.b_off;
    if (gamma) *gamma = N.gm_off;
    if (beta) *beta = N.bt_off;
    return LRS_OK;
}

extern "C" int lrs_dipnet_node_shape(const lrs_dipnet *net, int node, int *C, int *H, int *W) {
    if (!net || node < -1 || node >= (int)net->nodes.size()) return LRS_E_INVALID;
    const int t = node + 1;
    if (C) *C = net->tC(t);
    if (H) *H = net->tH(t);
    if (W) *W = net->tW(t);
    return LRS_OK;
}

extern "C" int lrs_dipnet_out_shape(const lrs_dipnet *net, int *C, int *H, int *W) {
    if (!net) return LRS_E_INVALID;
    return lrs_dipnet_node_shape(net, (int)net->nodes.size() - 1, C, H, W);
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
    std::vector<SnConv> tab;
    for (const auto &N : net->nodes)
        if (N.sn_index >= 0) tab.push_back(SnConv{params + N.w_off, net->f(N.wn_off), N.C, (int)N.Kc});
    std::vector<ConvPrep> prep;
    for (size_t i = 0; i < net->nodes.size(); ++i) {
        const auto &N = net->nodes[i];
        if (N.d.kind != LRS_NODE_CONV || (N.sn_index < 0 && N.wpre_off < 0)) continue;
        __bf16 *wf = N.wpre_off >= 0 ? (__bf16 *)net->f(N.wpre_off) : nullptr;
        __bf16 *wd = (wf && N.d.in0 > 0) ? wf + wprep_fwd_elems(N.g, N.C, N.upc) : nullptr;
        prep.push_back(ConvPrep{params + N.w_off, N.sn_index >= 0 ? net->f(N.wn_off) : nullptr, wf, wd, N.C, N.g.Cin,
                                N.g.k * N.g.k, r16(N.g.Cin), r16(N.C), N.sn_index, N.g.k,
                                (wd && !N.sm && !N.upc) ? up_eff_k(N.g) : 0, N.upc ? 1 : 0});
    }
    hipError_t e = hipSuccess;
    for (const auto &N : net->nodes) {
        if (e == hipSuccess && N.sm_dgrad)
            e = hipMemcpy(net->f(N.adj_off), N.adj.data(), sizeof(int) * N.adj.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess && N.wtab_off >= 0)
            e = hipMemcpy(net->f(N.wtab_off), N.wtab.data(), sizeof(int) * N.wtab.size(), hipMemcpyHostToDevice);
    }
    if (!tab.empty()) e = hipMemcpy(net->table(), tab.data(), sizeof(SnConv) * tab.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && !prep.empty())
        e = hipMemcpy(net->prep(), prep.data(), sizeof(ConvPrep) * prep.size(), hipMemcpyHostToDevice);
    if (net->sn_overlap && !prep.empty()) {
        // head: the first conv's forward planes from the raw weights (si = -1: no division, no W / s);
        // side: every entry, the first conv's without its planes (the main stream reads them meanwhile)
        ConvPrep head = prep[0], side0 = prep[0];
        head.Wn = nullptr;
        head.wd = nullptr;
        head.si = -1;
        side0.wf = nullptr;
        side0.wd = nullptr;
        std::vector<ConvPrep> side(prep);
        side[0] = side0;
        static_assert(sizeof(ConvPrep) <= 256, "one ConvPrep in the head slot");
        if (e == hipSuccess) e = hipMemcpy(net->prep_head(), &head, sizeof(ConvPrep), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(net->prep_side(), side.data(), sizeof(ConvPrep) * side.size(), hipMemcpyHostToDevice);
    }
    if (net->prep_split && !prep.empty()) {
        std::vector<ConvPrep> pf(prep), pd;
        for (auto &c : pf) c.wd = nullptr;
        for (const auto &c : prep)
            if (c.wd) {
                ConvPrep d = c;
                d.Wn = nullptr;
                d.wf = nullptr;
                pd.push_back(d);
            }
        net->n_prep_d = (int)pd.size();
        if (e == hipSuccess) e = hipMemcpy(net->prep_f(), pf.data(), sizeof(ConvPrep) * pf.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess && !pd.empty())
            e = hipMemcpy(net->prep_d(), pd.data(), sizeof(ConvPrep) * pd.size(), hipMemcpyHostToDevice);
        if (net->sn_overlap) {
            std::vector<ConvPrep> fs(pf);
            fs[0].wf = nullptr;   // (the first conv's forward planes: the head slot, raw weights)
            if (e == hipSuccess) e = hipMemcpy(net->prep_fs(), fs.data(), sizeof(ConvPrep) * fs.size(), hipMemcpyHostToDevice);
        }
    }
    if (e == hipSuccess) e = hipMemset(net->misc_off_bytes + net->ws, 0, 256);
    if (e == hipSuccess) e = hipMemset(net->headcnt(), 0, sizeof(int) * (net->nodes.back().C + 1));
    return e == hipSuccess ? LRS_OK : (int)e;
}

extern "C" int lrs_dipnet_init_params(lrs_dipnet *net, uint64_t seed, void *stream) {
    if (!net || !net->params) return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    for (size_t i = 0; i < net->nodes.size(); ++i) {
        const auto &N = net->nodes[i];
        const uint64_t k1 = mix64(seed * 0x100000001b3ULL + 2 * i + 1), k2 = mix64(seed * 0x100000001b3ULL + 2 * i + 2);
        if (N.d.kind == LRS_NODE_CONV) {
            const float fan_in = (float)N.Kc;
            // kaiming_uniform_(a=0, fan_in) (lipschitz_constraint_layer.py:74) or the nn.Conv2d
            // default kaiming_uniform_(a=sqrt(5)) = U(-1/sqrt(fan_in), +)
            const float wb = N.d.winit == LRS_WINIT_KAIMING ? sqrtf(6.0f / fan_in) : 1.0f / sqrtf(fan_in);
            const float bb = 1.0f / sqrtf(fan_in);
            hipLaunchKernelGGL(k_init_uniform, dim3(ew_blocks(N.C * N.Kc)), dim3(kEw), 0, st, net->params + N.w_off,
                               (int64_t)(N.C * N.Kc), wb, k1);
            hipLaunchKernelGGL(k_init_uniform, dim3(1), dim3(kEw), 0, st, net->params + N.b_off, (int64_t)N.C, bb, k2);
        }
        if (N.d.bn) {
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->params + N.gm_off, (int64_t)N.C, 1.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->params + N.bt_off, (int64_t)N.C, 0.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->bnstats + N.rs_off, (int64_t)N.C, 0.0f);
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kEw), 0, st, net->bnstats + N.rs_off + N.C, (int64_t)N.C, 1.0f);
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

static int ensure_side(lrs_dipnet *net, hipStream_t st);

extern "C" int lrs_dipnet_backward(lrs_dipnet *net, const float *x, const float *gout, void *stream) {
    if (!net || !net->ws || !x || !gout) return LRS_E_INVALID;
    if (const int rs = ensure_side(net, (hipStream_t)stream)) return rs;
    hipStream_t st = (hipStream_t)stream;
    const auto &Lst = net->nodes.back();
    const hipError_t e = hipMemcpyAsync(net->f(Lst.grad_off), gout, sizeof(float) * Lst.C * Lst.P,
                                        hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return (int)e;
    return dipnet_backward(net, x, st);
}

extern "C" int lrs_dipnet_set_ln_lambda(lrs_dipnet *net, float ln_lambda) {
    if (!net || !(ln_lambda > 0.0f)) return LRS_E_INVALID;
    drop_graph(net);
    net->ln_lambda = ln_lambda;
    return LRS_OK;
}

extern "C" const float *lrs_dipnet_output(const lrs_dipnet *net) {
    return (net && net->ws) ? net->f(net->nodes.back().out_off) : nullptr;
}

extern "C" const float *lrs_dipnet_grads(const lrs_dipnet *net) { return net ? net->grads : nullptr; }

// Diagnostics: a node's activation buffers in the bound workspace (node's output, its pre-BN z,
// dL/dz, dL/d(output)); NULL where the node has none.  Valid until the next call on the net.
extern "C" const float *lrs_dipnet_node_buffer(const lrs_dipnet *net, int node, int which) {
    if (!net || !net->ws || node < 0 || node >= (int)net->nodes.size()) return nullptr;
    const auto &N = net->nodes[node];
    int64_t off = -1;
    if (which == LRS_BUF_OUT) off = N.out_off;
    else if (which == LRS_BUF_Z) off = N.z_off;
    else if (which == LRS_BUF_GZ) off = N.gz_off;
    else if (which == LRS_BUF_GRAD) off = N.grad_off;
    return off >= 0 ? net->f(off) : nullptr;
}

// The side streams and the fork/join events are created on the first training call that needs
// them (outside any capture), so that creating a net and querying its layout needs no device.
// The side stream takes the priority of the calling stream, so a caller that trains the net on a
// high-priority stream (LrsPnPConfig.lowrank_priority) gets its weight gradients placed with the
// same priority.  One side stream is kept per priority seen (at most two in practice), so a call
// on a stream of another priority only selects a different one: no host synchronisation and no
// graph drop (a captured graph holds its own nodes, not the stream).
static int ensure_side(lrs_dipnet *net, hipStream_t st) {
    if (!net->fork_w) return LRS_OK;
    int prio = 0;
    hipError_t e = hipStreamGetPriority(st, &prio);
    if (e != hipSuccess) return (int)e;
    for (auto &ps : net->sides)
        if (ps.first == prio) {
            net->side = ps.second;
            return LRS_OK;
        }
    hipStream_t s = nullptr;
#ifdef LRS_TUNING
    // A/B only: the side stream on a subset of the CUs (every k-th CU left to the critical stream)
    static const int cuskip = (int)tune_knob("LRS_DIP_SIDE_CUSKIP", 0);
    if (cuskip > 1) {
        int dev = 0, ncu = 0;
        if ((e = hipGetDevice(&dev)) == hipSuccess)
            e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return (int)e;
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
            if (i % cuskip != cuskip - 1) mask[(size_t)i / 32] |= 1u << (i % 32);
        e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    } else
#endif
        e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio);
    if (e != hipSuccess) return (int)e;
    net->sides.emplace_back(prio, s);
    net->side = s;
    // The fork / join events only order kernels of this device against each other (nothing on the host
    // waits on them), so they are recorded with device-scope fences -- what a kernel boundary inside one
    // stream has -- instead of the default system-scope release, whose cache write-back the critical
    // stream paid at every fork (tools/micro/fork_cost: DESIGN.md §5).  LRS_DIP_SYSFENCE=1 (tuning
    // build only) keeps the default events for A/B.
    static const unsigned evf = hipEventDisableTiming | (tune_knob("LRS_DIP_SYSFENCE", 0) ? 0u : hipEventDisableSystemFence);
    if (!net->ev_join) e = hipEventCreateWithFlags(&net->ev_join, evf);
    if (e == hipSuccess && !net->ev_head) e = hipEventCreateWithFlags(&net->ev_head, evf);
    if (e == hipSuccess && !net->ev_sigma) e = hipEventCreateWithFlags(&net->ev_sigma, evf);
    if (e == hipSuccess && !net->ev_prep) e = hipEventCreateWithFlags(&net->ev_prep, evf);
    if (e == hipSuccess && !net->ev_wdgo) e = hipEventCreateWithFlags(&net->ev_wdgo, evf);
    if (e == hipSuccess && !net->ev_wd) e = hipEventCreateWithFlags(&net->ev_wd, evf);
    for (size_t i = 0; i < net->ev_fork.size() && e == hipSuccess; ++i)
        if (!net->ev_fork[i]) e = hipEventCreateWithFlags(&net->ev_fork[i], evf);
    return (int)e;
}

extern "C" int lrs_dipnet_train_steps(lrs_dipnet *net, const float *x, const float *target, const float *mask,
                                      float lr, float beta1, float beta2, float eps, lrs_es_state *es, float *ring,
                                      int nsteps, int use_graph, void *stream) {
    if (!net || !net->ws || !x || !target || nsteps < 0 || (es && !ring)) return LRS_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (const int rs = ensure_side(net, (hipStream_t)stream)) return rs;
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
    const auto &L = net->nodes.back();
    *loss = acc / ((double)L.C * (double)L.P);
    return LRS_OK;
}

extern "C" int lrs_dipnet_get_opts(const lrs_dipnet *net, lrs_dip_opts *opts) {
    if (!net || !opts) return LRS_E_INVALID;
    *opts = net->opts;
    return LRS_OK;
}
