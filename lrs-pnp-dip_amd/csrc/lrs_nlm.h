// Device-side PnP-NLM prox for a (K,1) coefficient column — the closed form of scikit-image
// 0.18.3 `_fast_nl_means_denoising_2d` at patch_size=3, patch_distance=3 (the call in
// main_LRS_PnP_DIP_1-LiP.py:192-196 / main_LRS_PnP.py:143-146), SURVEY.md Appendix A.1.
//
// Evaluation order is the canonical one of oracle/nlm_oracle.c:oracle_nlm_col, reproduced
// bit-for-bit (the library is built with -ffp-contract=off; the fma() are explicit):
//   kneg = -1512775.3951951856938 * (2 / ((h*h) * 9)),  ycut = -1512775.3951951856938 * 5
//   for t in -3,-2,-1,1,2,3:  S = (v[p]-v[p+t])^2 + (v[p+1]-v[p+1+t])^2 ;  y = S * kneg
//                             w = (y < ycut) ? 0 : double{hi = (int)y + 1072632447, lo = 0}
//                             sw = sw + w ;  swv = fma(w, v[p+t], swv)
//   out = float( fma(7, swv, c0*v[p]) / fma(7, sw, c0) ),   c0 = 8 * fast_exp(0)
// i.e. skimage's `distance > 5 -> skip; fast_exp(-distance)` with the Schraudolph scale folded into
// the distance normaliser (differences are O(1e-16) relative in y, far below the integral-image
// rounding skimage itself carries).  w(p,+t) == w(p+t,-t), so a chunk computes each weight once.
#pragma once
#include <hip/hip_runtime.h>

namespace lrs {

constexpr double kSchraudolphA = 1512775.3951951856938;
constexpr int kSchraudolphB = 1072632447;
constexpr double kNlmYCut = -1512775.3951951856938 * 5.0;

__device__ __forceinline__ double nlm_kneg(double h) { return -kSchraudolphA * (2.0 / ((h * h) * 9.0)); }

// high word of the weight of squared-distance sum S (0 when beyond the cutoff)
__device__ __forceinline__ int nlm_weight_hi(double S, double kneg) {
    const double y = S * kneg;
    const int hi = __double2int_rz(y) + kSchraudolphB;
    return (y < kNlmYCut) ? 0 : hi;
}

__device__ __forceinline__ double hi_to_double(int hi) { return __hiloint2double(hi, 0); }

// c0 = 8 * fast_exp(-0.0): fast_exp(0) has high word 1072632447 = 0x3FEFF07F.
__device__ __forceinline__ double nlm_c0() { return 8.0 * __hiloint2double(kSchraudolphB, 0); }

// One output of the closed form.  w[0..10] holds v-hat[p-3 .. p+7] relative to a chunk; `C` is
// the centre index inside w (3..6).  All values already promoted to double.
template <int C>
__device__ __forceinline__ float nlm_point(const double (&w)[11], double kneg, double c0) {
    double sw = 0.0, swv = 0.0;
#pragma unroll
    for (int t = -3; t <= 3; ++t) {
        if (t == 0) continue;
        const double a = w[C] - w[C + t];
        const double b = w[C + 1] - w[C + 1 + t];
        const double aa = a * a, bb = b * b;
        const double wt = hi_to_double(nlm_weight_hi(aa + bb, kneg));
        sw = sw + wt;
        swv = __fma_rn(wt, w[C + t], swv);
    }
    const double num = __fma_rn(7.0, swv, c0 * w[C]);
    const double den = __fma_rn(7.0, sw, c0);
    return (float)(num / den);
}

// ---- 4-output chunk with the 18 pair weights computed once (shared by the ISTA kernels) ----
template <int DIV>
__device__ __forceinline__ float nlm_div_v(double num, double den) {
    double r = __builtin_amdgcn_rcp(den);
    if (DIV == 0) return (float)(num * r);
    const double e = __fma_rn(-den, r, 1.0);
    r = __fma_rn(r, e, r);
    return (float)(num * r);
}

__device__ __forceinline__ float nlm_div_fast(double num, double den) {
    double r = __builtin_amdgcn_rcp(den);
    const double e = __fma_rn(-den, r, 1.0);
    r = __fma_rn(r, e, r);
    const double q = num * r;
    const double rem = __fma_rn(-den, q, num);
    return (float)__fma_rn(rem, r, q);
}

// W_t[i] = weight(s_t(i) + s_t(i+1)), s_t(k) = (w[k] - w[k+t])^2, for i >= i0 (FULL: all 18)
template <bool FULL>
__device__ __forceinline__ void nlm_weights(const double (&w)[11], double kneg, int (&W1)[7], int (&W2)[7],
                                            int (&W3)[7]) {
    {
        constexpr int i0 = FULL ? 2 : 3;
        double sp = (w[i0] - w[i0 + 1]) * (w[i0] - w[i0 + 1]);
#pragma unroll
        for (int i = i0; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 2], sn = d * d;
            W1[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
    {
        constexpr int i0 = FULL ? 1 : 3;
        double sp = (w[i0] - w[i0 + 2]) * (w[i0] - w[i0 + 2]);
#pragma unroll
        for (int i = i0; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 3], sn = d * d;
            W2[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
    {
        constexpr int i0 = FULL ? 0 : 3;
        double sp = (w[i0] - w[i0 + 3]) * (w[i0] - w[i0 + 3]);
#pragma unroll
        for (int i = i0; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 4], sn = d * d;
            W3[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
}

template <int DIV = 2>
__device__ __forceinline__ void nlm_outputs(const double (&w)[11], const int (&W1)[7], const int (&W2)[7],
                                            const int (&W3)[7], double c0, double seven, float (&out)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int C = 3 + e;
        const double ws[6] = {hi_to_double(W3[C - 3]), hi_to_double(W2[C - 2]), hi_to_double(W1[C - 1]),
                              hi_to_double(W1[C]), hi_to_double(W2[C]), hi_to_double(W3[C])};
        const double vs[6] = {w[C - 3], w[C - 2], w[C - 1], w[C + 1], w[C + 2], w[C + 3]};
        double swv = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) swv = __fma_rn(ws[k], vs[k], swv);   // canonical order
        const double sw = ((ws[0] + ws[5]) + (ws[1] + ws[4])) + (ws[2] + ws[3]);   // exact
        const double num = __fma_rn(seven, swv, c0 * w[C]);
        const double den = __fma_rn(seven, sw, c0);
        out[e] = DIV == 2 ? nlm_div_fast(num, den) : nlm_div_v<DIV>(num, den);
    }
}

}  // namespace lrs
