// Direct small-map conv + BatchNorm (+activation) in ONE launch (k_conv_bn_dir).
//
// On the small maps of a U-Net (18^2 and below at 36^2, 25^2 and below at 196^2) a conv followed by
// BatchNorm is two dependent launches of latency-bound work (k_conv_sm's split-K partials, then
// k_reduce_bn1's sum + statistics + normalisation), ~12 us per layer.  Here one workgroup owns one
// output channel: the conv in fp32 FMA (no split-K, no partials) from the input copied into LDS as
// is (each thread's tap offsets, reflection resolved, computed once), then k_reduce_bn1's BatchNorm arithmetic on the values in
// registers.  Reference: the Conv2d -> BatchNorm2d -> LeakyReLU blocks of models/skip.py /
// models/unet.py, the same outputs as k_conv_sm + k_reduce_bn1 (z, y, mean, invstd,
// running statistics), fp32 products summed in a fixed order (deterministic).
//
// Work split: output row strips of kDirSW pixels; lanes of a wave = (strip, input-channel group),
// gpw groups per wave, G = 8 gpw groups in all, group g taking the chunk's input channels g, g + G, ...
// Partial sums of the G groups are summed in group order through LDS.
#pragma once

#include "dip_gemm.h"
#include "dip_kernels.h"

namespace lrs {

constexpr int kDirTh = 512, kDirWaves = kDirTh / 64, kDirSW = 6;
constexpr int kDirStage = 64;                    // staged input floats per thread per chunk (16-B pieces)
constexpr int kDirStage1 = 32;                   // ... when staged value by value
constexpr int kDirX = kDirTh * kDirStage;        // LDS floats of one staged chunk
constexpr int kDirW = 4608;                      // LDS floats of the channel's weights (Cin k^2)
constexpr int kDirMaxG = 32;                     // input-channel groups at most (the partial sums' depth)

struct DirGeom {
    int ns, NS;       // strips per output row, strips in all
    int gpw, G;       // input-channel groups per wave, in all
    int CC, nchunk;   // input channels per staged chunk, chunks
    int nq;           // 16-B pieces (vec4) or values staged per thread per chunk
    int vec4;         // Hs Ws % 4 == 0: the chunk copied in 16-B pieces
};

// Host: the launch geometry, false when the conv does not fit the kernel's limits (reflection
// padding, not upsampled, <= 2 staged chunks, <= 64 strips)
inline bool dir_geom(const ConvGeom &g, DirGeom &d) {
    if (g.up || g.pad_mode != LRS_PAD_REFLECT || !((g.k == 3 && g.pad == 1) || (g.k == 1 && g.pad == 0)) ||
        !(g.stride == 1 || g.stride == 2))
        return false;
    const int P = g.Ho * g.Wo, HW = g.Hs * g.Ws;
    if (g.Hs < 2 || g.Ws < 2) return false;   // a reflection needs two rows / columns
    d.ns = (g.Wo + kDirSW - 1) / kDirSW;
    d.NS = g.Ho * d.ns;
    if (P > 2 * kDirTh || d.NS > 64 || g.Cin * g.k * g.k > kDirW) return false;
    d.gpw = std::min(64 / d.NS, kDirMaxG / kDirWaves);
    d.G = kDirWaves * d.gpw;
    if (d.G * P > kDirX) return false;   // the groups' partial sums reuse the staging buffer
    d.vec4 = HW % 4 == 0;
    d.CC = std::min(g.Cin, d.vec4 ? kDirX / HW : kDirTh * kDirStage1 / HW);
    d.nchunk = (g.Cin + d.CC - 1) / d.CC;
    d.nq = d.vec4 ? (d.CC * HW / 4 + kDirTh - 1) / kDirTh : (d.CC * HW + kDirTh - 1) / kDirTh;
    if (d.nq > (d.vec4 ? kDirStage / 4 : kDirStage1)) return false;
    return d.nchunk <= 2 && (int64_t)g.Cin * HW * 4 < kOob;
}

template <int KS, int S, bool V4>
__global__ __launch_bounds__(kDirTh) void k_conv_bn_dir(const float *__restrict__ x, const float *__restrict__ w,
                                                       const float *__restrict__ bias, ConvGeom g, DirGeom d, BnArgs a) {
    __shared__ __attribute__((aligned(16))) float xs[kDirX];
    __shared__ float ws[kDirW];
    __shared__ double red[2 * kDirTh / 64];
    constexpr int KK = KS * KS, NR = (kDirSW - 1) * S + KS;
    const int c = blockIdx.y, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int HW = g.Hs * g.Ws, P = g.Ho * g.Wo;
    // staging: the chunk's channels are one contiguous range of x, copied as is (16-B pieces when
    // the planes allow); all of a thread's loads in flight together, the next chunk's behind the
    // current chunk's products
    const __amdgpu_buffer_rsrc_t rs = s3_rsrc(x, g.Cin * HW * 4);
    float4 v4[V4 ? kDirStage / 4 : 1];
    float v1[V4 ? 1 : kDirStage1];
    auto load = [&](int c0) {   // past Cin: outside the buffer, zeros
        if constexpr (V4) {
#pragma unroll
            for (int q = 0; q < kDirStage / 4; ++q)
                if (q < d.nq)
                    v4[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (t + kDirTh * q) + 4 * c0 * HW, 0, 0));
        } else {
#pragma unroll
            for (int q = 0; q < kDirStage1; ++q)
                if (q < d.nq) v1[q] = s3_bload(rs, 4 * (t + kDirTh * q + c0 * HW), 0);
        }
    };
    auto store = [&]() {
        if constexpr (V4) {
#pragma unroll
            for (int q = 0; q < kDirStage / 4; ++q)
                if (q < d.nq) reinterpret_cast<float4 *>(xs)[t + kDirTh * q] = v4[q];
        } else {
#pragma unroll
            for (int q = 0; q < kDirStage1; ++q)
                if (q < d.nq) xs[t + kDirTh * q] = v1[q];
        }
    };
    load(0);
    // the BatchNorm tail's parameters, fetched now so that their latency hides behind the products
    const float cs = a.lip ? bn_lip_scale_w(a.gamma, a.C) : 1.0f;
    const float bc = bias ? bias[c] : 0.0f, gc = a.gamma[c], btc = a.beta[c];
    const float rm = a.run_mean && t == 0 ? a.run_mean[c] : 0.0f, rv = a.run_mean && t == 0 ? a.run_var[c] : 0.0f;
    for (int i = t; i < g.Cin * KK; i += kDirTh) ws[i] = w[(int64_t)c * g.Cin * KK + i];
    const int sub = lane / d.NS, strip = lane - sub * d.NS, grp = wv * d.gpw + sub;
    const bool active = sub < d.gpw;
    const int oy = strip / d.ns, ox0 = (strip - oy * d.ns) * kDirSW;
    // the strip's taps in a source plane (reflection resolved; columns past the map clamped: they
    // only feed outputs that are not stored)
    int off[KS][NR];
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
        const int sy = conv_src(min(oy * S + ky - g.pad, g.Hs), g.Hs, LRS_PAD_REFLECT, 0);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int sx = conv_src(min(ox0 * S + i - g.pad, g.Ws), g.Ws, LRS_PAD_REFLECT, 0);
            off[ky][i] = sy * g.Ws + sx;
        }
    }
    float acc[kDirSW];
#pragma unroll
    for (int s = 0; s < kDirSW; ++s) acc[s] = 0.0f;
    for (int ch = 0; ch < d.nchunk; ++ch) {
        const int c0 = ch * d.CC;
        if (ch) __syncthreads();   // the previous chunk's reads are done
        store();
        __syncthreads();
        if (ch + 1 < d.nchunk) load(c0 + d.CC);
        const int cc = min(d.CC, g.Cin - c0);
        if (active)
            for (int j = grp; j < cc; j += d.G) {
                const float *xr = xs + j * HW;
                const float *wr = ws + (c0 + j) * KK;
#pragma unroll
                for (int ky = 0; ky < KS; ++ky) {
                    float r[NR];
#pragma unroll
                    for (int i = 0; i < NR; ++i) r[i] = xr[off[ky][i]];
#pragma unroll
                    for (int kx = 0; kx < KS; ++kx) {
                        const float wt = wr[ky * KS + kx];
#pragma unroll
                        for (int s = 0; s < kDirSW; ++s) acc[s] = fmaf(wt, r[s * S + kx], acc[s]);
                    }
                }
            }
    }
    __syncthreads();
    float *pr = xs;   // [G][P] partial sums
    if (active)
#pragma unroll
        for (int s = 0; s < kDirSW; ++s)
            if (ox0 + s < g.Wo) pr[grp * P + oy * g.Wo + ox0 + s] = acc[s];
    __syncthreads();
    const int64_t zoff = (int64_t)c * P;
    auto zsum = [&](int i) {   // the groups in a fixed order, four running sums
        float z0 = 0.0f, z1 = 0.0f, z2 = 0.0f, z3 = 0.0f;
        int k = 0;
        for (; k + 4 <= d.G; k += 4) {
            z0 += pr[k * P + i];
            z1 += pr[(k + 1) * P + i];
            z2 += pr[(k + 2) * P + i];
            z3 += pr[(k + 3) * P + i];
        }
        for (; k < d.G; ++k) z0 += pr[k * P + i];
        float z = (z0 + z1) + (z2 + z3);
        if (bias) z = z + bc;
        return z;
    };
    // k_reduce_bn1's BatchNorm (bn_fwd_finish's arithmetic) from here on
    float zv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + u * kDirTh;
        zv[u] = 0.0f;
        if (i >= P) continue;
        zv[u] = zsum(i);
        const_cast<float *>(a.z)[zoff + i] = zv[u];
    }
    const double K = (double)zsum(0);
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
        if (t + u * kDirTh < P) {
            const double dd = (double)zv[u] - K;
            s1 += dd;
            s2 += dd * dd;
        }
    block_sum2_d(s1, s2, red);
    const double m = s1 / a.P;
    double var = s2 / a.P - m * m;
    if (var < 0.0) var = 0.0;
    const float m32 = (float)(K + m), is32 = (float)(1.0 / sqrt(var + (double)a.eps));
    if (t == 0) {
        a.mean[c] = m32;
        a.invstd[c] = is32;
        if (a.run_mean) {
            const double unb = a.P > 1 ? var * a.P / (a.P - 1) : var;
            a.run_mean[c] = (1.0f - a.momentum) * rm + a.momentum * m32;
            a.run_var[c] = (1.0f - a.momentum) * rv + a.momentum * (float)unb;
        }
    }
    const float gm = gc / cs, bt = btc / cs;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = t + u * kDirTh;
        if (i < P) a.y[zoff + i] = act_fwd((zv[u] - m32) * is32 * gm + bt, a.act);
    }
}

}  // namespace lrs
