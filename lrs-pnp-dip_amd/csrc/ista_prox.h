// The ISTA prox of one gradient row in LDS, shared by the row-split (ista_rs.hip) and per-pattern
// Gram (ista_pat.hip) kernels: the skimage fast NLM chunk, the MATLAB NLmeansfilter point, the
// soft threshold's quotient, and the LDS row swizzle both kernels use.
#pragma once
#include "lrs_common.h"
#include "lrs_nlm.h"

namespace lrs {

// numpy 'reflect' (no edge repeat) of index i into [0, K)
__device__ __forceinline__ int reflect_idx(int i, int K) {
    if (K == 1) return 0;
    const int period = 2 * (K - 1);
    i %= period;
    if (i < 0) i += period;
    return i >= K ? period - i : i;
}

// MATLAB 'symmetric' padding (edge repeated) of index i, |overhang| <= K
__device__ __forceinline__ int symmetric_idx(int i, int K) {
    if (i < 0) return -i - 1;
    if (i >= K) return 2 * K - 1 - i;
    return i;
}

// skimage 0.18.3 fast NLM of atoms a0..a0+3 of one gradient row in LDS
// gradient-row chunk index XOR-swizzled by block: [16 blocks][KP] floats read by the prox
__device__ __forceinline__ int gsw(int b, int a) { return a ^ ((b & 15) << 2); }

// The same chunk with the interior window (a0 - 3 .. a0 + 7 inside [0, K)) read as three aligned
// 16-byte LDS loads (the swizzle keeps 4-float groups contiguous); identical values and outputs.
__device__ __forceinline__ void prox_nlm_chunk_v4(const float *row, int b, int a0, int K, double kneg, double c0,
                                                  double seven, float (&out)[4]) {
    double w[11];
    if (a0 >= 4 && a0 + 8 <= K) {
        float4 v[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) v[u] = *reinterpret_cast<const float4 *>(&row[gsw(b, a0 - 4 + 4 * u)]);
        const float f[12] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                             v[2].x, v[2].y, v[2].z, v[2].w};
#pragma unroll
        for (int k = 0; k < 11; ++k) w[k] = (double)f[k + 1];
    } else {
#pragma unroll
        for (int k = 0; k < 11; ++k) w[k] = (double)row[gsw(b, reflect_idx(a0 - 3 + k, K))];
    }
    int W1[7], W2[7], W3[7];
    nlm_weights<true>(w, kneg, W1, W2, W3);
    nlm_outputs<2>(w, W1, W2, W3, c0, seven, out);
}

__device__ __forceinline__ void prox_nlm_chunk(const float *row, int b, int a0, int K, double kneg, double c0,
                                               double seven, float (&out)[4]) {
    double w[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) w[k] = (double)row[gsw(b, reflect_idx(a0 - 3 + k, K))];
    int W1[7], W2[7], W3[7];
    nlm_weights<true>(w, kneg, W1, W2, W3);
    nlm_outputs<2>(w, W1, W2, W3, c0, seven, out);
}

// NLmeansfilter(g, 3, 3, h) of LRS-PnP(Matlab Code)/NLmeansfilter.m:18-78, one output, fp64, in the
// evaluation order of oracle/nlm_oracle.c:oracle_nlm_matlab_col
__device__ __forceinline__ float prox_nlm_matlab_point(const float *row, int b, int i, int K,
                                                       const double (&krow)[7], double h2) {
    double v[13];   // g-hat[i-6 .. i+6]
#pragma unroll
    for (int k = 0; k < 13; ++k) {
        const int j = i - 6 + k;
        v[k] = (j >= -3 && j < K + 3) ? (double)row[gsw(b, symmetric_idx(j, K))] : 0.0;
    }
    double sw = 0.0, av = 0.0, wmax = 0.0;
#pragma unroll
    for (int t = -3; t <= 3; ++t) {
        const int r = i + t;
        if (t == 0 || r < 0 || r >= K) continue;
        double d = 0.0;
#pragma unroll
        for (int u = -3; u <= 3; ++u) {
            const double df = v[6 + u] - v[6 + t + u];
            d = d + krow[u + 3] * (df * df);
        }
        const double wt = exp(-d / h2);
        if (wt > wmax) wmax = wt;
        sw = sw + wt;
        av = av + wt * v[6 + t];
    }
    av = av + wmax * v[6];
    sw = sw + wmax;
    return sw > 0.0 ? (float)(av / sw) : row[gsw(b, i)];
}

__device__ __forceinline__ void nlm_matlab_krow_d(double (&krow)[7]) {
#pragma unroll
    for (int u = -3; u <= 3; ++u) {
        const int a = u < 0 ? -u : u;
        double s = 0.0;
        for (int d = (a < 1 ? 1 : a); d <= 3; ++d) s = s + 1.0 / (double)(2 * d + 1);
        krow[u + 3] = s / 3.0;
    }
}

// a / b from y = 1/b (correctly rounded reciprocal) and one remainder step: the IEEE quotient
// away from overflow / underflow (…1-LiP.py:190 torch division by alpha)
__device__ __forceinline__ float rs_div(float a, float b, float y) {
    const float q = a * y;
    const float r = __fmaf_rn(-b, q, a);
    return __fmaf_rn(r, y, q);
}

}  // namespace lrs
