// Device-side PnP-NLM prox for a (K,1) coefficient column — the closed form of scikit-image
// 0.18.3 `_fast_nl_means_denoising_2d` at patch_size=3, patch_distance=3 (the call in
// main_LRS_PnP_DIP_1-LiP.py:192-196 / main_LRS_PnP.py:143-146), SURVEY.md Appendix A.1.
//
// Evaluation order is the canonical one of oracle/nlm_oracle.c:oracle_nlm_col, reproduced
// bit-for-bit (the library is built with -ffp-contract=off; the two fma() are explicit):
//   inv2 = 2 / ((h*h) * 9)
//   for t in -3,-2,-1,1,2,3:  D = ((v[p]-v[p+t])^2 + (v[p+1]-v[p+1+t])^2) * inv2
//                             if D <= 5: w = fast_exp(-D); sw += w; swv = fma(w, v[p+t], swv)
//   out = float( fma(7, swv, c0*v[p]) / fma(7, sw, c0) ),   c0 = 8 * fast_exp(0)
#pragma once
#include <hip/hip_runtime.h>

namespace lrs {

constexpr double kNlmCutoff = 5.0;

// Schraudolph exp as in skimage: high word (int)(1512775.3951951856938*y) + 1072632447, low 0.
__device__ __forceinline__ double nlm_fast_exp(double y) {
    int hi = __double2int_rz(1512775.3951951856938 * y) + 1072632447;
    return __hiloint2double(hi, 0);
}

// c0 = 8 * fast_exp(-0.0): fast_exp(0) has high word 1072632447 = 0x3FEFF07F.
__device__ __forceinline__ double nlm_c0() { return 8.0 * __hiloint2double(1072632447, 0); }

// One output of the closed form.  w[0..10] holds v-hat[p-3 .. p+7] relative to a chunk; `c` is
// the centre index inside w (3..6).  All values already promoted to double.
template <int C>
__device__ __forceinline__ float nlm_point(const double (&w)[11], double inv2, double c0) {
    double sw = 0.0, swv = 0.0;
#pragma unroll
    for (int t = -3; t <= 3; ++t) {
        if (t == 0) continue;
        double a = w[C] - w[C + t];
        double b = w[C + 1] - w[C + 1 + t];
        double aa = a * a, bb = b * b;
        double D = (aa + bb) * inv2;
        if (!(D > kNlmCutoff)) {
            double wt = nlm_fast_exp(-D);
            sw = sw + wt;
            swv = __fma_rn(wt, w[C + t], swv);
        }
    }
    double num = __fma_rn(7.0, swv, c0 * w[C]);
    double den = __fma_rn(7.0, sw, c0);
    return (float)(num / den);
}

}  // namespace lrs
