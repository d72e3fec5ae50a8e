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

}  // namespace lrs
