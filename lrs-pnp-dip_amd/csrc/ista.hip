// Fused masked ISTA with the PnP-NLM prox over every block of the unfolded cube.
//
// Reference path (shuoli0708/LRS-PnP-DIP): the per-block Python loop of main_LRS_PnP.py:270-303
// (…1-LiP.py:367-392) calling ista() (main_LRS_PnP.py:131-149 / …1-LiP.py:185-198) on the pruned
// dictionary (delete_element, :152-155), then Phi_z[:,jj] = Full_Dictionary @ Coefs.
//
// MI355X design:
//  * blocks are the GEMM N dimension: one wave owns 16 blocks (one v_mfma_f32_16x16x4_f32 column
//    tile), a 512-thread workgroup 128 blocks, 2 waves per SIMD so one wave's fp64 NLM overlaps
//    the other's MFMA;
//  * pruning becomes masking: H^T(y - Hx) == D^T(m .* (y - Dx)) with m the observed-row mask;
//  * both products per inner iteration run on MFMA with the coefficients resident in VGPRs for
//    all Nit iterations: R = m.*(y - D x) (M = rows, K = atoms) then G = D^T R (M = atoms,
//    K = rows).  The accumulator of each product is directly the B operand of the next one
//    (C[4(l>>4)+i][l&15] == B[k=l>>4][l&15] for k-step i), so nothing crosses LDS but D;
//  * D is staged in LDS in two images, [row][atom] for the first product and [atom][row] for
//    the second, both read with ds_read_b128 (4 k-steps per read).  When n <= 64 (bb = 8) the
//    whole dictionary stays resident for the kernel's lifetime; larger n streams 64-row stages;
//  * the NLM prox runs in fp64 on the accumulator layout: a lane holds 4 consecutive atoms per
//    16-atom tile, the 3+4 neighbours it needs come from lanes l-16 / l+16 (ds_bpermute).
#include <algorithm>

#include "lrs_common.h"
#include "lrs_nlm.h"

namespace lrs {

constexpr int kIstaWaves = 8;
constexpr int kIstaThreads = kIstaWaves * kWave;
constexpr int kStageRows = 64;

template <int K>
struct alignas(16) IstaSmem {
    float DA[kStageRows][K + 4];  // [row][atom]; +4 keeps b128 rows aligned, spreads banks
    float DT[K][kStageRows + 4];  // [atom][row]
};

// a / b from the correctly rounded reciprocal y = 1/b with one Markstein correction step:
// q = a*y, r = fma(-b, q, a) (exact), q + r*y.  Equals the IEEE quotient a/b (the reference's
// torch division) away from overflow/underflow, at 3 instructions instead of ~10.
__device__ __forceinline__ float div_by(float a, float b, float y) {
    const float q = a * y;
    const float r = __fmaf_rn(-b, q, a);
    return __fmaf_rn(r, y, q);
}

struct IstaParams {
    const float *Yb;
    const uint8_t *obs;
    const float *D;
    const float *alpha;
    const double *thr;
    float *coefs;
    float *phi;
    int n, n_pad, Nit, prox;
    int64_t nb;
    double seven;   // 7.0, passed in so fma(7, x, c) keeps its addend in place (no per-use copy)
};

template <int K>
__device__ __forceinline__ void stage_dictionary(IstaSmem<K> &S, const float *__restrict__ D, int n,
                                                 int r0) {
    for (int idx = threadIdx.x; idx < kStageRows * K; idx += kIstaThreads) {
        const int r = idx / K, a = idx % K;
        const float v = (r0 + r < n) ? D[(int64_t)(r0 + r) * K + a] : 0.0f;
        S.DA[r][a] = v;
        S.DT[a][r] = v;
    }
}

// acc = (D x) rows [16t, 16t+16) of the staged slab, for this lane's block.
template <int K>
__device__ __forceinline__ floatx4 dict_times_x(const IstaSmem<K> &S, int t, const float (&X)[K / 16][4],
                                                int jl, int g) {
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < K / 16; q += 2) {
        const float4 a = *reinterpret_cast<const float4 *>(&S.DA[16 * t + jl][16 * q + 4 * g]);
        acc0 = mfma16x16x4(a.x, X[q][0], acc0);
        acc0 = mfma16x16x4(a.y, X[q][1], acc0);
        acc0 = mfma16x16x4(a.z, X[q][2], acc0);
        acc0 = mfma16x16x4(a.w, X[q][3], acc0);
        const float4 b = *reinterpret_cast<const float4 *>(&S.DA[16 * t + jl][16 * (q + 1) + 4 * g]);
        acc1 = mfma16x16x4(b.x, X[q + 1][0], acc1);
        acc1 = mfma16x16x4(b.y, X[q + 1][1], acc1);
        acc1 = mfma16x16x4(b.z, X[q + 1][2], acc1);
        acc1 = mfma16x16x4(b.w, X[q + 1][3], acc1);
    }
    return acc0 + acc1;
}

// G[q] += D^T r over rows [16t, 16t+16) of the staged slab.
template <int K>
__device__ __forceinline__ void dict_t_times_r(const IstaSmem<K> &S, int t, const float (&r)[4],
                                               floatx4 (&G)[K / 16], int jl, int g) {
#pragma unroll
    for (int q = 0; q < K / 16; ++q) {
        const float4 a = *reinterpret_cast<const float4 *>(&S.DT[16 * q + jl][16 * t + 4 * g]);
        G[q] = mfma16x16x4(a.x, r[0], G[q]);
        G[q] = mfma16x16x4(a.y, r[1], G[q]);
        G[q] = mfma16x16x4(a.z, r[2], G[q]);
        G[q] = mfma16x16x4(a.w, r[3], G[q]);
    }
}

// The 4 NLM outputs of one chunk; w[0..10] = v-hat[a0-3 .. a0+7] (a0 = first atom of chunk).
// Each symmetric weight w(i,+t) == w(i+t,-t) is computed once: 18 weights for 4 outputs.
__device__ __forceinline__ void nlm_chunk(const double (&w)[11], double kneg, double c0, float (&out)[4]) {
    int W1[7], W2[7], W3[7];      // W_t[i] = hi word of w(a0-3+i, +t), s_t[i] = (w[i] - w[i+t])^2
    {
        double sp = (w[2] - w[3]) * (w[2] - w[3]);
#pragma unroll
        for (int i = 2; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 2], sn = d * d;
            W1[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
    {
        double sp = (w[1] - w[3]) * (w[1] - w[3]);
#pragma unroll
        for (int i = 1; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 3], sn = d * d;
            W2[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
    {
        double sp = (w[0] - w[3]) * (w[0] - w[3]);
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const double d = w[i + 1] - w[i + 4], sn = d * d;
            W3[i] = nlm_weight_hi(sp + sn, kneg);
            sp = sn;
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int C = 3 + e;
        // t = -3,-2,-1,+1,+2,+3 (the canonical order of oracle_nlm_col)
        const double ws[6] = {hi_to_double(W3[C - 3]), hi_to_double(W2[C - 2]), hi_to_double(W1[C - 1]),
                              hi_to_double(W1[C]), hi_to_double(W2[C]), hi_to_double(W3[C])};
        const double vs[6] = {w[C - 3], w[C - 2], w[C - 1], w[C + 1], w[C + 2], w[C + 3]};
        double sw = 0.0, swv = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            sw = sw + ws[k];
            swv = __fma_rn(ws[k], vs[k], swv);
        }
        const double num = __fma_rn(7.0, swv, c0 * w[C]);
        const double den = __fma_rn(7.0, sw, c0);
        out[e] = (float)(num / den);
    }
}

// Neighbour-exchange state for the in-register NLM along the atom axis.  A lane (block l&15,
// group g = l>>4) holds atoms 16q+4g .. 16q+4g+3 of every 16-atom tile q; chunk c-1 lives in
// lane l-16 (same tile, or tile q-1 when g == 0), chunk c+1 in lane l+16 (tile q+1 when g == 3).
struct NlmLanes {
    int g, src_prev, src_next;
    __device__ __forceinline__ explicit NlmLanes(int lane)
        : g(lane >> 4), src_prev((lane + 48) & 63), src_next((lane + 16) & 63) {}
};

// NLM of tile q given this lane's gradient chunk `own`, the shuffled neighbours of tiles q-1/q/q+1
// (Pprev = prev-lane chunk of tile q-1, Pcur = of tile q; Ncur = next-lane chunk of tile q,
// Nnext = of tile q+1), with numpy-style reflection at both ends of the K atoms.
template <int NQ>
__device__ __forceinline__ void nlm_tile(int q, const NlmLanes &L, const float (&own)[4], const float (&Pprev)[3],
                                         const float (&Pcur)[3], const float (&Ncur)[4], const float (&Nnext)[4],
                                         double kneg, double c0, float (&out)[4]) {
    float prv[3], nxt[4];
    if (L.g == 0) {
        if (q == 0) { prv[0] = own[3]; prv[1] = own[2]; prv[2] = own[1]; }   // reflect
        else { prv[0] = Pprev[0]; prv[1] = Pprev[1]; prv[2] = Pprev[2]; }
    } else {
        prv[0] = Pcur[0]; prv[1] = Pcur[1]; prv[2] = Pcur[2];
    }
    if (L.g == 3) {
        if (q == NQ - 1) { nxt[0] = own[2]; nxt[1] = own[1]; nxt[2] = own[0]; nxt[3] = prv[2]; }
        else { nxt[0] = Nnext[0]; nxt[1] = Nnext[1]; nxt[2] = Nnext[2]; nxt[3] = Nnext[3]; }
    } else {
        nxt[0] = Ncur[0]; nxt[1] = Ncur[1]; nxt[2] = Ncur[2]; nxt[3] = Ncur[3];
    }
    const double w[11] = {prv[0], prv[1], prv[2], own[0], own[1], own[2], own[3],
                          nxt[0], nxt[1], nxt[2], nxt[3]};
    nlm_chunk(w, kneg, c0, out);
}

// X <- NLM(G) along the atom axis, for this lane's block (4 atoms per 16-atom tile per lane).
template <int K>
__device__ __forceinline__ void nlm_prox_registers(const floatx4 (&G)[K / 16], float (&X)[K / 16][4],
                                                   double h, int lane) {
    constexpr int NQ = K / 16;
    const NlmLanes L(lane);
    const double kneg = nlm_kneg(h);
    const double c0 = nlm_c0();
    float Pprev[3] = {0.f, 0.f, 0.f}, Pcur[3], Ncur[4], Nnext[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) Ncur[e] = __shfl(G[0][e], L.src_next, 64);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
        for (int e = 0; e < 3; ++e) Pcur[e] = __shfl(G[q][e + 1], L.src_prev, 64);
        if (q + 1 < NQ) {
#pragma unroll
            for (int e = 0; e < 4; ++e) Nnext[e] = __shfl(G[q + 1][e], L.src_next, 64);
        }
        const float own[4] = {G[q][0], G[q][1], G[q][2], G[q][3]};
        float o[4];
        nlm_tile<NQ>(q, L, own, Pprev, Pcur, Ncur, Nnext, kneg, c0, o);
        X[q][0] = o[0]; X[q][1] = o[1]; X[q][2] = o[2]; X[q][3] = o[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) Pprev[e] = Pcur[e];
#pragma unroll
        for (int e = 0; e < 4; ++e) Ncur[e] = Nnext[e];
    }
}

// ------------------------------------------------------------------------------------------------
// Resident kernel (n_pad <= 64, i.e. bb <= 8): dictionary in LDS for the whole launch, y and the
// row mask in VGPRs, and a software pipeline over the 16 atom tiles q of each inner iteration:
//     MFMA : G[q+2] = D^T r (tile q+2)        | VALU : NLM of tile q -> x_new[q]
//     MFMA : R_next += D[:, tile q] x_new[q]  | VALU : g[q+2] = x[q+2] + G[q+2]/alpha
// so the matrix pipe works on the next products while the fp64 NLM of the current tile runs.
// R_next = D x_new is complete when the last tile is done: it is the next iteration's residual
// input and, after the last iteration, Phi = D x.
// ------------------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ floatx4 gemm2_tile(const IstaSmem<K> &S, int q, const float (&r)[4][4], int jl, int g) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 a = *reinterpret_cast<const float4 *>(&S.DT[16 * q + jl][16 * t + 4 * g]);
        acc = mfma16x16x4(a.x, r[t][0], acc);
        acc = mfma16x16x4(a.y, r[t][1], acc);
        acc = mfma16x16x4(a.z, r[t][2], acc);
        acc = mfma16x16x4(a.w, r[t][3], acc);
    }
    return acc;
}

template <int K>
__device__ __forceinline__ void gemm1_tile(const IstaSmem<K> &S, int q, const float (&x)[4], floatx4 (&R)[4], int jl,
                                           int g) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float4 a = *reinterpret_cast<const float4 *>(&S.DA[16 * t + jl][16 * q + 4 * g]);
        R[t] = mfma16x16x4(a.x, x[0], R[t]);
        R[t] = mfma16x16x4(a.y, x[1], R[t]);
        R[t] = mfma16x16x4(a.z, x[2], R[t]);
        R[t] = mfma16x16x4(a.w, x[3], R[t]);
    }
}

// ABLATE (diagnostic builds only, never selected by lrs_ista_f32): 1 = prox replaced by a copy
// (MFMA + data movement only), 2 = products replaced by register moves (NLM + movement only).
template <int K, bool SOFT, int ABLATE = 0>
__global__ __launch_bounds__(kIstaThreads, 2) void k_ista_res(IstaParams p) {
    constexpr int NQ = K / 16;
    __shared__ __attribute__((aligned(16))) IstaSmem<K> S;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int jl = lane & 15, g = lane >> 4;
    const int64_t j = ((int64_t)blockIdx.x * kIstaWaves + wave) * 16 + jl;
    const bool valid = j < p.nb;
    const int NT = p.n_pad / 16;
    const NlmLanes L(lane);

    const float alpha = valid ? p.alpha[j] : 1.0f;
    const double thr = valid ? p.thr[j] : 1.0;
    const double kneg = nlm_kneg(thr);
    const double c0 = nlm_c0();
    const float Tsoft = (float)thr;

    float y[4][4];
    uint32_t mres = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        float4 yv = {0.f, 0.f, 0.f, 0.f};
        uint32_t mv = 0;
        if (valid && t < NT) {
            yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
            mv = *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * t + 4 * g]);
        }
        y[t][0] = yv.x; y[t][1] = yv.y; y[t][2] = yv.z; y[t][3] = yv.w;
#pragma unroll
        for (int i = 0; i < 4; ++i) mres |= (((mv >> (8 * i)) & 0xffu) ? 1u : 0u) << (4 * t + i);
    }
    stage_dictionary<K>(S, p.D, p.n, 0);
    __syncthreads();

    float X[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q) X[q][0] = X[q][1] = X[q][2] = X[q][3] = 0.f;
    floatx4 R[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) R[t] = floatx4{0.f, 0.f, 0.f, 0.f};   // D x for x = 0

    const float ainv = 1.0f / alpha;
    auto gradient = [&](floatx4 &Gq, const float (&xq)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Gq[i] = xq[i] + div_by(Gq[i], alpha, ainv);   // x + (D^T r)/alpha
    };

    for (int it = 0; it < p.Nit; ++it) {
        float r[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) r[t][i] = ((mres >> (4 * t + i)) & 1u) ? (y[t][i] - R[t][i]) : 0.0f;
            R[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        floatx4 G[NQ];
        auto gemm2 = [&](int q) -> floatx4 {
            if (ABLATE == 2) {
                floatx4 v = {r[q & 3][0], r[q & 3][1], r[q & 3][2], r[q & 3][3]};
                return v;
            }
            return gemm2_tile<K>(S, q, r, jl, g);
        };
        G[0] = gemm2(0);
        G[1] = gemm2(1);
        __builtin_amdgcn_sched_barrier(0);
        gradient(G[0], X[0]);
        gradient(G[1], X[1]);
        float Pprev[3] = {0.f, 0.f, 0.f}, Pcur[3], Ncur[4], Nnext[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) Ncur[e] = __shfl(G[0][e], L.src_next, 64);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 2 < NQ) G[q + 2] = gemm2(q + 2);
            const float own[4] = {G[q][0], G[q][1], G[q][2], G[q][3]};
            float o[4];
            if (ABLATE == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = own[i] * 0.5f;
            } else if (SOFT) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float t = fabsf(own[i]) - Tsoft;
                    t = t > 0.f ? t : 0.f;
                    o[i] = own[i] > 0.f ? t : (own[i] < 0.f ? -t : 0.f);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 3; ++e) Pcur[e] = __shfl(G[q][e + 1], L.src_prev, 64);
                if (q + 1 < NQ) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) Nnext[e] = __shfl(G[q + 1][e], L.src_next, 64);
                }
                nlm_tile<NQ>(q, L, own, Pprev, Pcur, Ncur, Nnext, kneg, c0, o);
#pragma unroll
                for (int e = 0; e < 3; ++e) Pprev[e] = Pcur[e];
#pragma unroll
                for (int e = 0; e < 4; ++e) Ncur[e] = Nnext[e];
            }
            X[q][0] = o[0]; X[q][1] = o[1]; X[q][2] = o[2]; X[q][3] = o[3];
            if (ABLATE == 2) {
#pragma unroll
                for (int t = 0; t < 4; ++t) R[t] += floatx4{o[0], o[1], o[2], o[3]};
            } else {
                gemm1_tile<K>(S, q, X[q], R, jl, g);
            }
            if (q + 2 < NQ) gradient(G[q + 2], X[q + 2]);
            // keep each pipeline step's LDS reads and MFMAs inside the step: without this fence
            // the scheduler hoists every tile's ds_reads to the loop top and spills
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    if (valid) {
        if (p.coefs) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                *reinterpret_cast<float4 *>(&p.coefs[j * K + 16 * q + 4 * g]) =
                    make_float4(X[q][0], X[q][1], X[q][2], X[q][3]);
        }
        // Phi_z = Full_Dictionary @ Coefs == R (all rows, missing ones included)
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t < NT)
                *reinterpret_cast<float4 *>(&p.phi[j * p.n_pad + 16 * t + 4 * g]) =
                    make_float4(R[t][0], R[t][1], R[t][2], R[t][3]);
    }
}


// ------------------------------------------------------------------------------------------------
// Split-bf16 resident kernel (n_pad <= 64, K = 256).  The two products per inner iteration run on
// the bf16 matrix cores (v_mfma_f32_16x16x32_bf16, 16x the f32 MFMA rate, and unlike the f32
// MFMA not on the VALU's FMA datapath) with every fp32 operand split exactly into three bf16
// terms, v = v1 + v2 + v3 (8 significand bits each: 24 = fp32); the six products with
// i + j <= 4 are kept (the dropped ones are <= 2^-24 relative), accumulated in fp32, so each
// product has fp32-GEMM accuracy (not the bitwise f32 MFMA result; parity is held to the same
// 1e-5 relative L2 as the rest of the pipeline).
//   * D lives in LDS once, as three bf16 images [row][atom] with 8-byte chunks XOR-swizzled per
//     row; the first product reads its A fragments by rows (ds_read_b64), the second reads the
//     same images transposed (ds_read_b64_tr_b16): 96 KB instead of the f32 kernel's 136 KB;
//   * accumulators feed the next product's B operand directly (C rows 4g..4g+3 of two 16-tiles
//     = the 8 k-values of lane group g), as in the f32 kernel.
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));

template <int K>
struct alignas(16) IstaSmemB3 {
    __bf16 D[3][kStageRows][K];   // split s of D, [row][atom], chunk-swizzled
};

// XOR swizzle of the 8-byte chunk index by row (linear over GF(2) in row & 15): conflict-free for
// the 32-lane halves of both the row reads and the transposed reads (searched exhaustively)
__device__ __forceinline__ int b3_swz(int row) {
    return ((row & 1) ? 26 : 0) ^ ((row & 2) ? 12 : 0) ^ ((row & 4) ? 62 : 0) ^ ((row & 8) ? 3 : 0);
}

template <int K>
__device__ __forceinline__ int b3_off(int row, int chunk) {   // element offset within one image
    return row * K + 4 * (chunk ^ b3_swz(row));
}

__device__ __forceinline__ void split3(float v, __bf16 &a, __bf16 &b, __bf16 &c) {
    a = (__bf16)v;
    const float r1 = v - (float)a;
    b = (__bf16)r1;
    const float r2 = r1 - (float)b;
    c = (__bf16)r2;
}

constexpr int kB3Waves = 4;                       // one wave per SIMD: the whole 512-entry register file
constexpr int kB3Threads = kB3Waves * kWave;

template <int K, int THREADS>
__device__ __forceinline__ void stage_dictionary_b3(IstaSmemB3<K> &S, const float *__restrict__ D, int n) {
    for (int idx = threadIdx.x; idx < kStageRows * K; idx += THREADS) {
        const int r = idx / K, a = idx % K;
        const float v = r < n ? D[(int64_t)r * K + a] : 0.0f;
        __bf16 h, m, l;
        split3(v, h, m, l);
        const int o = b3_off<K>(r, a >> 2) + (a & 3);
        S.D[0][0][o] = h;
        S.D[1][0][o] = m;
        S.D[2][0][o] = l;
    }
}

// 8 bf16 per split from 2 x 4 fp32 (elements 0..3 = u, 4..7 = w)
__device__ __forceinline__ void split_frag(const float (&u)[4], const float (&w)[4], bf16x8 (&f)[3]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        __bf16 a, b, c;
        split3(u[e], a, b, c);
        f[0][e] = a; f[1][e] = b; f[2][e] = c;
        split3(w[e], a, b, c);
        f[0][e + 4] = a; f[1][e + 4] = b; f[2][e + 4] = c;
    }
}

__device__ __forceinline__ floatx4 mfma_bf(const bf16x8 &a, const bf16x8 &b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc += A B with both split three ways, small terms first
__device__ __forceinline__ floatx4 mfma_split6(const bf16x8 (&A)[3], const bf16x8 (&B)[3], floatx4 acc) {
    acc = mfma_bf(A[2], B[0], acc);
    acc = mfma_bf(A[1], B[1], acc);
    acc = mfma_bf(A[0], B[2], acc);
    acc = mfma_bf(A[1], B[0], acc);
    acc = mfma_bf(A[0], B[1], acc);
    acc = mfma_bf(A[0], B[0], acc);
    return acc;
}

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

// G tile q = D^T r: A = D^T rows (atoms 16q..16q+15) by transposed reads, B = r split, per row pair
template <int K>
__device__ __forceinline__ floatx4 b3_gemm2(const IstaSmemB3<K> &S, int q, const bf16x8 (&rf)[2][3], int lane) {
    const int g = lane >> 4, ll = lane & 15, qq = ll >> 2, pp = ll & 3;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
        const int r0 = 32 * pr + 4 * g + qq, r1 = r0 + 16;
        bf16x8 A[3];
#pragma unroll
        for (int sp = 0; sp < 3; ++sp) {
            typedef __attribute__((address_space(3))) short4v lds_s4;
            const short4v a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4 *)(&S.D[sp][0][b3_off<K>(r0, 4 * q + pp)]));
            const short4v a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4 *)(&S.D[sp][0][b3_off<K>(r1, 4 * q + pp)]));
            A[sp] = cat4(__builtin_bit_cast(bf16x4, a0), __builtin_bit_cast(bf16x4, a1));
        }
        acc = mfma_split6(A, rf[pr], acc);
    }
    return acc;
}

// R[t] += D rows (16t..) x (atom tiles 2p, 2p+1): A = D rows by row reads, B = x split
template <int K>
__device__ __forceinline__ void b3_gemm1(const IstaSmemB3<K> &S, int p, const bf16x8 (&xf)[3], floatx4 (&R)[4],
                                         int lane) {
    const int g = lane >> 4, ll = lane & 15;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int row = 16 * t + ll;
        bf16x8 A[3];
#pragma unroll
        for (int sp = 0; sp < 3; ++sp) {
            const bf16x4 a0 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][b3_off<K>(row, 8 * p + g)]);
            const bf16x4 a1 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][b3_off<K>(row, 8 * p + 4 + g)]);
            A[sp] = cat4(a0, a1);
        }
        R[t] = mfma_split6(A, xf, R[t]);
    }
}


// ---- NLM chunk with weight reuse (split-bf16 kernel) ---------------------------------------------
// Chunk c's weights W1[2], W2[1..2], W3[0..2] (pairs starting left of the chunk) equal chunk c-1's
// W1[6], W2[5..6], W3[4..6], so a lane computes 12 of the 18 weights and takes the other 6 (hi
// words) from lane l-16 (chunk c-1).  Weights are bitwise the same as nlm_chunk's.  The weight sums
// are exact in fp64 (<= 6 terms of 21 significant bits within 8 binades), so their order is free;
// num/den uses one Newton step on v_rcp_f64 and a remainder correction (|error| < 1 ulp of fp64
// before the final float rounding, instead of the IEEE division sequence).
template <int ABL>
__device__ __forceinline__ int shf(int v, int src) { return ABL == 1 ? v : __shfl(v, src, 64); }
template <int ABL>
__device__ __forceinline__ float shf(float v, int src) { return ABL == 1 ? v : __shfl(v, src, 64); }

struct Reuse6 {
    int v[6];   // W1[6], W2[5], W2[6], W3[4], W3[5], W3[6] of a chunk
};

// tile q of the NLM with weight reuse (FULL for the first tile, whose g == 0 chunk has a
// reflected window).  `carry`: this lane's trailing weights of tile q-1 on entry, of tile q on
// exit; only the g == 3 lanes' copy is read (by the g == 0 lanes of the next tile).
template <int NQ, bool FULL, int ABL = 0>
__device__ __forceinline__ void nlm_tile_reuse(int q, const NlmLanes &L, const float (&own)[4], const float (&Pprev)[3],
                                               const float (&Pcur)[3], const float (&Ncur)[4], const float (&Nnext)[4],
                                               double kneg, double c0, double seven, Reuse6 &carry,
                                               float (&out)[4]) {
    float prv[3], nxt[4];
    if (L.g == 0) {
        if (q == 0) { prv[0] = own[3]; prv[1] = own[2]; prv[2] = own[1]; }
        else { prv[0] = Pprev[0]; prv[1] = Pprev[1]; prv[2] = Pprev[2]; }
    } else {
        prv[0] = Pcur[0]; prv[1] = Pcur[1]; prv[2] = Pcur[2];
    }
    if (L.g == 3) {
        if (q == NQ - 1) { nxt[0] = own[2]; nxt[1] = own[1]; nxt[2] = own[0]; nxt[3] = prv[2]; }
        else { nxt[0] = Nnext[0]; nxt[1] = Nnext[1]; nxt[2] = Nnext[2]; nxt[3] = Nnext[3]; }
    } else {
        nxt[0] = Ncur[0]; nxt[1] = Ncur[1]; nxt[2] = Ncur[2]; nxt[3] = Ncur[3];
    }
    const double w[11] = {prv[0], prv[1], prv[2], own[0], own[1], own[2], own[3],
                          nxt[0], nxt[1], nxt[2], nxt[3]};
    int W1[7], W2[7], W3[7];
    nlm_weights<FULL>(w, kneg, W1, W2, W3);
    if (!FULL) {
        // chunk c-1 is lane l-16's chunk of this tile (g >= 1) or lane l+48's chunk of tile q-1
        // (g == 0): the g == 3 source serves its tile q-1 weights
        const int mine[6] = {W1[6], W2[5], W2[6], W3[4], W3[5], W3[6]};
        int prev[6];
#pragma unroll
        for (int e = 0; e < 6; ++e) prev[e] = shf<ABL>((L.g == 3) ? carry.v[e] : mine[e], L.src_prev);
        W1[2] = prev[0];
        W2[1] = prev[1]; W2[2] = prev[2];
        W3[0] = prev[3]; W3[1] = prev[4]; W3[2] = prev[5];
    }
    carry.v[0] = W1[6];
    carry.v[1] = W2[5]; carry.v[2] = W2[6];
    carry.v[3] = W3[4]; carry.v[4] = W3[5]; carry.v[5] = W3[6];
    nlm_outputs(w, W1, W2, W3, c0, seven, out);
}

// sched_group_barrier pattern for one pipeline step with NM MFMAs (groups of 6 sharing 6 LDS reads,
// the reads one group ahead) and V VALU instructions after each MFMA
template <int NM, int V>
__device__ __forceinline__ void b3_interleave() {
    constexpr int NG = NM / 6;
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        if (gi + 1 < NG) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
        }
    }
}

template <int K, bool SOFT, int WAVES = kB3Waves, bool SEQ = false, int ABL = 0, int PIPE = 0>
__global__ __launch_bounds__(WAVES * kWave, 1) void k_ista_b3(IstaParams p) {
    static_assert(K == 256, "the chunk swizzle assumes 64 chunks per row");
    constexpr int NQ = K / 16;
    __shared__ __attribute__((aligned(16))) IstaSmemB3<K> S;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int jl = lane & 15, g = lane >> 4;
    const int64_t j = ((int64_t)blockIdx.x * WAVES + wave) * 16 + jl;
    const bool valid = j < p.nb;
    const int NT = p.n_pad / 16;
    const NlmLanes L(lane);

    const float alpha = valid ? p.alpha[j] : 1.0f;
    const double thr = valid ? p.thr[j] : 1.0;
    const double kneg = nlm_kneg(thr);
    const double c0 = nlm_c0();
    const float Tsoft = (float)thr;

    float y[4][4];
    uint32_t mres = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        float4 yv = {0.f, 0.f, 0.f, 0.f};
        uint32_t mv = 0;
        if (valid && t < NT) {
            yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
            mv = *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * t + 4 * g]);
        }
        y[t][0] = yv.x; y[t][1] = yv.y; y[t][2] = yv.z; y[t][3] = yv.w;
#pragma unroll
        for (int i = 0; i < 4; ++i) mres |= (((mv >> (8 * i)) & 0xffu) ? 1u : 0u) << (4 * t + i);
    }
    stage_dictionary_b3<K, WAVES * kWave>(S, p.D, p.n);
    __syncthreads();

    float X[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q) X[q][0] = X[q][1] = X[q][2] = X[q][3] = 0.f;
    floatx4 R[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) R[t] = floatx4{0.f, 0.f, 0.f, 0.f};

    const float ainv = 1.0f / alpha;
    auto gradient = [&](floatx4 &Gq, const float (&xq)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Gq[i] = xq[i] + div_by(Gq[i], alpha, ainv);
    };

    for (int it = 0; it < p.Nit; ++it) {
        float r[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) r[t][i] = ((mres >> (4 * t + i)) & 1u) ? (y[t][i] - R[t][i]) : 0.0f;
            R[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        bf16x8 rf[2][3];
        split_frag(r[0], r[1], rf[0]);
        split_frag(r[2], r[3], rf[1]);
        // pipeline over tile pairs: step p runs the products of tiles 2p+4, 2p+5 and the
        // (independent, so interleavable) NLM of tiles 2p and 2p+1 on one wave's instruction stream
        floatx4 G[NQ];
        auto gemm2q = [&](int q) -> floatx4 {
            if (ABL == 3) return floatx4{r[0][0] + q, r[1][1], r[2][2], r[3][3]};
            return b3_gemm2<K>(S, q, rf, lane);
        };
#pragma unroll
        for (int q = 0; q < 4; ++q) G[q] = gemm2q(q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) gradient(G[q], X[q]);
        float Pprev[3] = {0.f, 0.f, 0.f}, Ncur[4];
        Reuse6 carry{};
#pragma unroll
        for (int e = 0; e < 4; ++e) Ncur[e] = shf<ABL>(G[0][e], L.src_next);
#pragma unroll
        for (int pp = 0; pp < NQ / 2; ++pp) {
            const int qa = 2 * pp, qb = qa + 1;
            if (qa + 4 < NQ) G[qa + 4] = gemm2q(qa + 4);
            if (qb + 4 < NQ) G[qb + 4] = gemm2q(qb + 4);
            if (PIPE && pp > 0) {   // D x of the previous pair beside this pair's NLM
                bf16x8 xf[3];
                split_frag(X[qa - 2], X[qb - 2], xf);
                b3_gemm1<K>(S, pp - 1, xf, R, lane);
            }
            float oa[4], ob[4];
            if (SOFT) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float t = fabsf(G[qa][i]) - Tsoft;
                    t = t > 0.f ? t : 0.f;
                    oa[i] = G[qa][i] > 0.f ? t : (G[qa][i] < 0.f ? -t : 0.f);
                    float u = fabsf(G[qb][i]) - Tsoft;
                    u = u > 0.f ? u : 0.f;
                    ob[i] = G[qb][i] > 0.f ? u : (G[qb][i] < 0.f ? -u : 0.f);
                }
            } else if (ABL == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) { oa[i] = G[qa][i]; ob[i] = G[qb][i]; }
            } else {
                const float owna[4] = {G[qa][0], G[qa][1], G[qa][2], G[qa][3]};
                const float ownb[4] = {G[qb][0], G[qb][1], G[qb][2], G[qb][3]};
                float Pa[3], Pb[3], Nb[4], Nn[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    Pa[e] = shf<ABL>(G[qa][e + 1], L.src_prev);
                    Pb[e] = shf<ABL>(G[qb][e + 1], L.src_prev);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) Nb[e] = shf<ABL>(G[qb][e], L.src_next);
                if (qb + 1 < NQ) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) Nn[e] = shf<ABL>(G[qb + 1][e], L.src_next);
                }
                if (qa == 0) nlm_tile_reuse<NQ, true, ABL>(qa, L, owna, Pprev, Pa, Ncur, Nb, kneg, c0, p.seven, carry, oa);
                else nlm_tile_reuse<NQ, false, ABL>(qa, L, owna, Pprev, Pa, Ncur, Nb, kneg, c0, p.seven, carry, oa);
                if (SEQ) __builtin_amdgcn_sched_barrier(0);
                nlm_tile_reuse<NQ, false, ABL>(qb, L, ownb, Pa, Pb, Nb, Nn, kneg, c0, p.seven, carry, ob);
#pragma unroll
                for (int e = 0; e < 3; ++e) Pprev[e] = Pb[e];
#pragma unroll
                for (int e = 0; e < 4; ++e) Ncur[e] = Nn[e];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) { X[qa][i] = oa[i]; X[qb][i] = ob[i]; }
            if (!PIPE) {
                bf16x8 xf[3];
                split_frag(X[qa], X[qb], xf);
                if (ABL == 3) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) R[t][t] += X[qa][t] * X[qb][3 - t];
                } else {
                    b3_gemm1<K>(S, pp, xf, R, lane);
                }
            }
            if (qa + 4 < NQ) gradient(G[qa + 4], X[qa + 4]);
            if (qb + 4 < NQ) gradient(G[qb + 4], X[qb + 4]);
            if (PIPE == 2) {
                if (pp > 0 && qa + 4 < NQ) b3_interleave<48, 12>();
                else b3_interleave<24, 24>();
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (PIPE) {
            bf16x8 xf[3];
            split_frag(X[NQ - 2], X[NQ - 1], xf);
            b3_gemm1<K>(S, NQ / 2 - 1, xf, R, lane);
        }
    }

    if (valid) {
        if (p.coefs) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                *reinterpret_cast<float4 *>(&p.coefs[j * K + 16 * q + 4 * g]) =
                    make_float4(X[q][0], X[q][1], X[q][2], X[q][3]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t < NT)
                *reinterpret_cast<float4 *>(&p.phi[j * p.n_pad + 16 * t + 4 * g]) =
                    make_float4(R[t][0], R[t][1], R[t][2], R[t][3]);
    }
}

// ---- split-bf16 kernel, lane-contiguous atom layout ----------------------------------------------
// The atom order inside the MFMA tiles is free (it is the A operand's row choice), so tile q row
// 4g+i holds atom 64g + 4q + i: lane group g owns the 64 consecutive atoms 64g .. 64g+63 across its
// 16 tiles.  The NLM neighbours of a chunk are then the lane's own previous / next tile, except at
// the group edges (tile 0's left and tile 15's right neighbours: 7 shuffles per iteration instead
// of ~200), and the 6 reused weights of each chunk are the lane's own previous chunk's.
// LDS image: split s of D at [row][atom], 4-atom chunk c stored at pi(c) ^ (row & 15) with
// pi(c) = c ^ 8 (c >= 32): conflict-free for both the gemm2 transposed reads (chunks 16p + q)
// and the gemm1 row reads (chunks 16g + 2p, +1) — exhaustively checked per 32-lane half.
template <int K>
__device__ __forceinline__ int ln_off(int row, int chunk) {
    const int pc = chunk ^ (((chunk >> 5) & 1) << 3);
    return row * K + 4 * (pc ^ (row & 15));
}

template <int K, int THREADS>
__device__ __forceinline__ void stage_dictionary_ln(IstaSmemB3<K> &S, const float *__restrict__ D, int n) {
    for (int idx = threadIdx.x; idx < kStageRows * K; idx += THREADS) {
        const int r = idx / K, a = idx % K;
        const float v = r < n ? D[(int64_t)r * K + a] : 0.0f;
        __bf16 h, m, l;
        split3(v, h, m, l);
        const int o = ln_off<K>(r, a >> 2) + (a & 3);
        S.D[0][0][o] = h;
        S.D[1][0][o] = m;
        S.D[2][0][o] = l;
    }
}

// G tile q = D^T r with tile row 4g+i = atom 64g + 4q + i
template <int K>
__device__ __forceinline__ floatx4 ln_gemm2(const IstaSmemB3<K> &S, int q, const bf16x8 (&rf)[2][3], int lane) {
    const int g = lane >> 4, ll = lane & 15, qq = ll >> 2, pp = ll & 3;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
        const int r0 = 32 * pr + 4 * g + qq, r1 = r0 + 16;
        bf16x8 A[3];
#pragma unroll
        for (int sp = 0; sp < 3; ++sp) {
            typedef __attribute__((address_space(3))) short4v lds_s4;
            const short4v a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4 *)(&S.D[sp][0][ln_off<K>(r0, 16 * pp + q)]));
            const short4v a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s4 *)(&S.D[sp][0][ln_off<K>(r1, 16 * pp + q)]));
            A[sp] = cat4(__builtin_bit_cast(bf16x4, a0), __builtin_bit_cast(bf16x4, a1));
        }
        acc = mfma_split6(A, rf[pr], acc);
    }
    return acc;
}

// R[t] += D rows (16t..) x the lane's atoms 64g + 8p .. 64g + 8p + 7 (tiles 2p, 2p+1)
template <int K>
__device__ __forceinline__ void ln_gemm1(const IstaSmemB3<K> &S, int p, const bf16x8 (&xf)[3], floatx4 (&R)[4],
                                         int lane) {
    const int g = lane >> 4, ll = lane & 15;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int row = 16 * t + ll;
        bf16x8 A[3];
#pragma unroll
        for (int sp = 0; sp < 3; ++sp) {
            const bf16x4 a0 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][ln_off<K>(row, 16 * g + 2 * p)]);
            const bf16x4 a1 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][ln_off<K>(row, 16 * g + 2 * p + 1)]);
            A[sp] = cat4(a0, a1);
        }
        R[t] = mfma_split6(A, xf, R[t]);
    }
}

// NLM of one 4-atom chunk from its 3 left / 4 right neighbours; `carry` = the previous chunk's
// trailing weights on entry (unused when FULL), this chunk's on exit
template <bool FULL>
__device__ __forceinline__ void nlm_chunk_ln(const float (&prv)[3], const floatx4 &own, const float (&nxt)[4],
                                             double kneg, double c0, double seven, int (&carry)[6],
                                             float (&out)[4]) {
    const double w[11] = {prv[0], prv[1], prv[2], own[0], own[1], own[2], own[3],
                          nxt[0], nxt[1], nxt[2], nxt[3]};
    int W1[7], W2[7], W3[7];
    nlm_weights<FULL>(w, kneg, W1, W2, W3);
    if (!FULL) {
        W1[2] = carry[0];
        W2[1] = carry[1]; W2[2] = carry[2];
        W3[0] = carry[3]; W3[1] = carry[4]; W3[2] = carry[5];
    }
    carry[0] = W1[6];
    carry[1] = W2[5]; carry[2] = W2[6];
    carry[3] = W3[4]; carry[4] = W3[5]; carry[5] = W3[6];
    nlm_outputs(w, W1, W2, W3, c0, seven, out);
}

// ---- explicitly scheduled lane-layout kernel -------------------------------------------------------
// Per iteration: prologue (residual, tiles 0..3 and the edge copy of tile 15), then 8 steps of 4
// slots.  Slot k of step p runs one NLM phase (weights / outputs of chunk 2p, then of 2p+1) beside
// the MFMAs of up to two 6-MFMA units (a gemm2 tile half or a gemm1 row tile) whose LDS operands
// the previous slot loaded, and loads the next slot's operands.
struct Frag3 {
    bf16x8 a[3];
};

// Tile-major image (LAY 1): chunk c = 16 p' + q' of row r at element q' * 1024 + r * 16 + 4 (p' ^ s(r)),
// s(r) = 2 ((r >> 3) & 1).  Every read of a tile / row tile is a lane-constant base plus an
// immediate (no per-read address VALU), and both read kinds are conflict-free per 32-lane half.
__device__ __forceinline__ int tm_off(int row, int chunk) {
    return (chunk & 15) * 1024 + row * 16 + 4 * ((chunk >> 4) ^ (((row >> 3) & 1) << 1));
}

template <int K, int THREADS>
__device__ __forceinline__ void stage_dictionary_tm(IstaSmemB3<K> &S, const float *__restrict__ D, int n) {
    for (int idx = threadIdx.x; idx < kStageRows * K; idx += THREADS) {
        const int r = idx / K, a = idx % K;
        const float v = r < n ? D[(int64_t)r * K + a] : 0.0f;
        __bf16 h, m, l;
        split3(v, h, m, l);
        const int o = tm_off(r, a >> 2) + (a & 3);
        S.D[0][0][o] = h;
        S.D[1][0][o] = m;
        S.D[2][0][o] = l;
    }
}

struct TmLane {
    int tr, g1;   // lane-constant element offsets of the transposed and the row reads
    __device__ __forceinline__ explicit TmLane(int lane) {
        const int g = lane >> 4, ll = lane & 15, qq = ll >> 2, pp = ll & 3, rt = 4 * g + qq;
        tr = rt * 16 + 4 * (pp ^ (((rt >> 3) & 1) << 1));
        g1 = ll * 16 + 4 * (g ^ (((ll >> 3) & 1) << 1));
    }
};

template <int K>
__device__ __forceinline__ void tm_load_g2(const IstaSmemB3<K> &S, int q, int pr, const TmLane &A, Frag3 &F) {
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
        typedef __attribute__((address_space(3))) short4v lds_s4;
        const __bf16 *b = &S.D[sp][0][0] + A.tr + q * 1024 + pr * 512;
        const short4v a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)b);
        const short4v a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(b + 256));
        F.a[sp] = cat4(__builtin_bit_cast(bf16x4, a0), __builtin_bit_cast(bf16x4, a1));
    }
}

template <int K>
__device__ __forceinline__ void tm_load_g1(const IstaSmemB3<K> &S, int t, int p, const TmLane &A, Frag3 &F) {
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
        const __bf16 *b = &S.D[sp][0][0] + A.g1 + 2 * p * 1024 + t * 256;
        const bf16x4 a0 = *reinterpret_cast<const bf16x4 *>(b);
        const bf16x4 a1 = *reinterpret_cast<const bf16x4 *>(b + 1024);
        F.a[sp] = cat4(a0, a1);
    }
}

template <int K>
__device__ __forceinline__ void ln_load_g2(const IstaSmemB3<K> &S, int q, int pr, int lane, Frag3 &F) {
    const int g = lane >> 4, ll = lane & 15, qq = ll >> 2, pp = ll & 3;
    const int r0 = 32 * pr + 4 * g + qq, r1 = r0 + 16;
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
        typedef __attribute__((address_space(3))) short4v lds_s4;
        const short4v a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(&S.D[sp][0][ln_off<K>(r0, 16 * pp + q)]));
        const short4v a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4 *)(&S.D[sp][0][ln_off<K>(r1, 16 * pp + q)]));
        F.a[sp] = cat4(__builtin_bit_cast(bf16x4, a0), __builtin_bit_cast(bf16x4, a1));
    }
}

template <int K>
__device__ __forceinline__ void ln_load_g1(const IstaSmemB3<K> &S, int t, int p, int lane, Frag3 &F) {
    const int g = lane >> 4, ll = lane & 15, row = 16 * t + ll;
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
        const bf16x4 a0 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][ln_off<K>(row, 16 * g + 2 * p)]);
        const bf16x4 a1 = *reinterpret_cast<const bf16x4 *>(&S.D[sp][0][ln_off<K>(row, 16 * g + 2 * p + 1)]);
        F.a[sp] = cat4(a0, a1);
    }
}

// unit u (0/1) of slot k of step pp: kind 0 none, 1 gemm2 (tile a, half b), 2 gemm1 (row tile a, pair b)
struct LnUnit {
    int kind, a, b;
};
__device__ constexpr LnUnit ln_unit(int pp, int k, int u) {
    if (pp < 0 || pp > 7) return {0, 0, 0};
    if (pp == 0) return u == 0 ? LnUnit{1, 4 + (k >> 1), k & 1} : LnUnit{0, 0, 0};
    if (pp >= 6) return u == 0 ? LnUnit{2, k, pp - 1} : LnUnit{0, 0, 0};
    const int idx = 2 * k + u;      // 0..3 gemm2 halves of tiles 2pp+4, 2pp+5; 4..7 gemm1 row tiles
    if (idx < 4) return {1, 2 * pp + 4 + (idx >> 1), idx & 1};
    return {2, idx - 4, pp - 1};
}

template <int K, int LAY>
__device__ __forceinline__ void ln_load_unit(const IstaSmemB3<K> &S, LnUnit U, int lane, const TmLane &A, Frag3 &F) {
    if (LAY == 1) {
        if (U.kind == 1) tm_load_g2<K>(S, U.a, U.b, A, F);
        else if (U.kind == 2) tm_load_g1<K>(S, U.a, U.b, A, F);
    } else {
        if (U.kind == 1) ln_load_g2<K>(S, U.a, U.b, lane, F);
        else if (U.kind == 2) ln_load_g1<K>(S, U.a, U.b, lane, F);
    }
}

// whole-tile products through the unit loaders (prologue / epilogue)
template <int K, int LAY>
__device__ __forceinline__ floatx4 lay_gemm2(const IstaSmemB3<K> &S, int q, const bf16x8 (&rf)[2][3], int lane,
                                             const TmLane &A) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
        Frag3 F;
        ln_load_unit<K, LAY>(S, LnUnit{1, q, pr}, lane, A, F);
        acc = mfma_split6(F.a, rf[pr], acc);
    }
    return acc;
}

template <int K, int LAY>
__device__ __forceinline__ void lay_gemm1(const IstaSmemB3<K> &S, int p, const bf16x8 (&xf)[3], floatx4 (&R)[4],
                                          int lane, const TmLane &A) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        Frag3 F;
        ln_load_unit<K, LAY>(S, LnUnit{2, t, p}, lane, A, F);
        R[t] = mfma_split6(F.a, xf, R[t]);
    }
}

template <int K, bool GB, int LAY = 0, bool FOLD = false, int DIV = 2>
__global__ __launch_bounds__(kB3Threads, 1) void k_ista_ln2(IstaParams p) {
    static_assert(K == 256, "the lane layout assumes 4 groups of 64 atoms");
    constexpr int NQ = K / 16;
    __shared__ __attribute__((aligned(16))) IstaSmemB3<K> S;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int jl = lane & 15, g = lane >> 4;
    const int64_t j = ((int64_t)blockIdx.x * kB3Waves + wave) * 16 + jl;
    const bool valid = j < p.nb;
    const int NT = p.n_pad / 16;
    const int src_prev = (lane + 48) & 63, src_next = (lane + 16) & 63;
    const TmLane AL(lane);

    const float alpha = valid ? p.alpha[j] : 1.0f;
    const double thr = valid ? p.thr[j] : 1.0;
    const double kneg = nlm_kneg(thr);
    const double c0 = nlm_c0();

    float y[4][4];
    uint32_t mres = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        float4 yv = {0.f, 0.f, 0.f, 0.f};
        uint32_t mv = 0;
        if (valid && t < NT) {
            yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
            mv = *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * t + 4 * g]);
        }
        y[t][0] = yv.x; y[t][1] = yv.y; y[t][2] = yv.z; y[t][3] = yv.w;
#pragma unroll
        for (int i = 0; i < 4; ++i) mres |= (((mv >> (8 * i)) & 0xffu) ? 1u : 0u) << (4 * t + i);
    }
    if (LAY == 1) stage_dictionary_tm<K, kB3Threads>(S, p.D, p.n);
    else stage_dictionary_ln<K, kB3Threads>(S, p.D, p.n);
    __syncthreads();

    float X[NQ][4];   // X[q][i] = coefficient of atom 64g + 4q + i
#pragma unroll
    for (int q = 0; q < NQ; ++q) X[q][0] = X[q][1] = X[q][2] = X[q][3] = 0.f;
    floatx4 R[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) R[t] = floatx4{0.f, 0.f, 0.f, 0.f};

    const float ainv = 1.0f / alpha;
    auto gradient = [&](floatx4 &Gq, const float (&xq)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) Gq[i] = FOLD ? xq[i] + Gq[i] : xq[i] + div_by(Gq[i], alpha, ainv);
    };

    for (int it = 0; it < p.Nit; ++it) {
        float r[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                r[t][i] = ((mres >> (4 * t + i)) & 1u) ? (y[t][i] - R[t][i]) : 0.0f;
                if (FOLD) r[t][i] = div_by(r[t][i], alpha, ainv);   // D^T (r / alpha)
            }
            R[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        bf16x8 rf[2][3];
        split_frag(r[0], r[1], rf[0]);
        split_frag(r[2], r[3], rf[1]);
        floatx4 G[NQ];
        float edge_prev[3], edge_next[4];
        {
            floatx4 G15 = lay_gemm2<K, LAY>(S, NQ - 1, rf, lane, AL);
#pragma unroll
            for (int q = 0; q < 4; ++q) G[q] = lay_gemm2<K, LAY>(S, q, rf, lane, AL);
            gradient(G15, X[NQ - 1]);
#pragma unroll
            for (int q = 0; q < 4; ++q) gradient(G[q], X[q]);
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                const float v = __shfl(G15[e + 1], src_prev, 64);
                edge_prev[e] = (g == 0) ? G[0][3 - e] : v;      // reflect: atoms -3,-2,-1 -> 3,2,1
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) edge_next[e] = __shfl(G[0][e], src_next, 64);
        }
        Frag3 F[2][2];
        ln_load_unit<K, LAY>(S, ln_unit(0, 0, 0), lane, AL, F[0][0]);
        ln_load_unit<K, LAY>(S, ln_unit(0, 0, 1), lane, AL, F[0][1]);
        __builtin_amdgcn_sched_barrier(0);

        int carry[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int pp = 0; pp < NQ / 2; ++pp) {
            const int qa = 2 * pp, qb = qa + 1;
            // tiles whose products were issued in the previous step get their gradient step
            if (pp >= 1 && pp <= 6) {
                gradient(G[qa + 2], X[qa + 2]);
                gradient(G[qb + 2], X[qb + 2]);
            }
            bf16x8 xf[3];
            if (pp >= 1) split_frag(X[qa - 2], X[qb - 2], xf);
            double w[11];
            int W1[7], W2[7], W3[7];
            float out[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * pp + k, cur = s & 1, nxt = cur ^ 1;
                // MFMAs of this slot's units
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const LnUnit U = ln_unit(pp, k, u);
                    if (U.kind == 1) G[U.a] = mfma_split6(F[cur][u].a, rf[U.b], U.b == 0 ? floatx4{0.f, 0.f, 0.f, 0.f} : G[U.a]);
                    else if (U.kind == 2) R[U.a] = mfma_split6(F[cur][u].a, xf, R[U.a]);
                }
                // operands of the next slot
                const int pn = (k == 3) ? pp + 1 : pp, kn = (k + 1) & 3;
#pragma unroll
                for (int u = 0; u < 2; ++u) ln_load_unit<K, LAY>(S, ln_unit(pn, kn, u), lane, AL, F[nxt][u]);
                // NLM phase
                const int q = (k < 2) ? qa : qb;
                if (k == 0 || k == 2) {
                    float prv[3], nx[4];
                    if (q == 0) {
#pragma unroll
                        for (int e = 0; e < 3; ++e) prv[e] = edge_prev[e];
                    } else {
#pragma unroll
                        for (int e = 0; e < 3; ++e) prv[e] = G[q - 1][e + 1];
                    }
                    if (q == NQ - 1) {    // reflect: atoms 256..259 -> 254, 253, 252, 251
                        const float rfl[4] = {G[q][2], G[q][1], G[q][0], G[q - 1][3]};
#pragma unroll
                        for (int e = 0; e < 4; ++e) nx[e] = (g == 3) ? rfl[e] : edge_next[e];
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) nx[e] = G[q + 1][e];
                    }
                    const double wv[11] = {prv[0], prv[1], prv[2], G[q][0], G[q][1], G[q][2], G[q][3],
                                           nx[0], nx[1], nx[2], nx[3]};
#pragma unroll
                    for (int e = 0; e < 11; ++e) w[e] = wv[e];
                    if (q == 0) {
                        nlm_weights<true>(w, kneg, W1, W2, W3);
                    } else {
                        nlm_weights<false>(w, kneg, W1, W2, W3);
                        W1[2] = carry[0];
                        W2[1] = carry[1]; W2[2] = carry[2];
                        W3[0] = carry[3]; W3[1] = carry[4]; W3[2] = carry[5];
                    }
                    carry[0] = W1[6];
                    carry[1] = W2[5]; carry[2] = W2[6];
                    carry[3] = W3[4]; carry[4] = W3[5]; carry[5] = W3[6];
                } else {
                    nlm_outputs<DIV>(w, W1, W2, W3, c0, p.seven, out);
#pragma unroll
                    for (int i = 0; i < 4; ++i) X[q][i] = out[i];
                }
                if (GB) {
#pragma unroll
                    for (int u = 0; u < 6 * ((ln_unit(pp, k, 0).kind ? 1 : 0) + (ln_unit(pp, k, 1).kind ? 1 : 0)); ++u) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        {
            bf16x8 xf[3];
            split_frag(X[NQ - 2], X[NQ - 1], xf);
            lay_gemm1<K, LAY>(S, NQ / 2 - 1, xf, R, lane, AL);
        }
    }

    if (valid) {
        if (p.coefs) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                *reinterpret_cast<float4 *>(&p.coefs[j * K + 64 * g + 4 * q]) =
                    make_float4(X[q][0], X[q][1], X[q][2], X[q][3]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t < NT)
                *reinterpret_cast<float4 *>(&p.phi[j * p.n_pad + 16 * t + 4 * g]) =
                    make_float4(R[t][0], R[t][1], R[t][2], R[t][3]);
    }
}

// A second instantiation of k_ista_ln2 (the DIV = 0 quotient, never launched) beside the product's
// <256, false, 1, true, 1>: with it the product kernel compiles to exactly round 1's code (30 AGPRs,
// 104 v_accvgpr moves); compiled alone, the same source gets 82 AGPRs and 241 moves, and configs[1]
// loses 2.8 % (k_ista_ln2 7.88 vs 7.59 ms per launch; profiles/r04/ab_pnp).  Every helper is
// __forceinline__, so this is not inlining: the device IR of the product kernel differs in what the
// middle end leaves to the backend (with the second instantiation a dozen [4 x float] / <4 x float>
// allocas survive to AMDGPUPromoteAlloca; alone, SROA splits them earlier), and the register
// allocation of this VGPR-saturated kernel follows.  amdgpu_waves_per_eu, amdgpu_num_vgpr and
// amdgpu_flat_work_group_size on the kernel leave 82.  tests/test_codegen.py reads the built
// library's kernel metadata and fails above 32 AGPRs (or on any spill), so a compiler update or an
// edit here that loses the allocation is caught on the CPU.
template __global__ void k_ista_ln2<256, false, 1, true, 0>(IstaParams);

// Standalone NLM over nvec columns of length K (any K >= 1): one workgroup per column, the
// column reflect-padded in LDS, one thread per output.  Used by lrs_nlm_col_f32 (the
// denoise_nl_means drop-in) — the fused ISTA kernel above does not call it.
__global__ __launch_bounds__(256) void k_nlm_col(const float *__restrict__ g, int64_t ldg,
                                                 float *__restrict__ out, int64_t ldo, int K,
                                                 double h, const double *__restrict__ hv) {
    extern __shared__ float col[];  // K + 10
    const int64_t v = blockIdx.x;
    const float *gv = g + v * ldg;
    const int n = K + 10;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int s = i - 5;
        if (K > 1) {
            const int period = 2 * (K - 1);
            s %= period;
            if (s < 0) s += period;
            if (s >= K) s = period - s;
        } else {
            s = 0;
        }
        col[i] = gv[s];
    }
    __syncthreads();
    const double hh = hv ? hv[v] : h;
    const double kneg = nlm_kneg(hh);
    const double c0 = nlm_c0();
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
        double w[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) w[k] = (double)col[i + 5 - 3 + k];
        out[v * ldo + i] = nlm_point<3>(w, kneg, c0);
    }
}

// k_nlm_col's dynamic LDS is (K + 10) floats: above 64 KiB (K > 16374) the launch must be opted into
// more (gfx950: 160 KiB per workgroup).  Set once per device.
static int nlm_col_lds(int64_t K) {
    const size_t bytes = (size_t)(K + 10) * sizeof(float);
    static std::atomic<uint64_t> opted{0};
    if (bytes > 65536) return lds_opt_in((const void *)k_nlm_col, 160 * 1024, opted);
    return LRS_OK;
}

}  // namespace lrs

using namespace lrs;

// k_ista_ln2's quotient: 2 = one Newton step on v_rcp_f64 plus a remainder correction, 1 = the Newton
// step alone.  Both are < 1 ulp of fp64 before the float rounding; the register allocation of this
// VGPR-saturated kernel is what differs.
#ifndef LRS_LN2_DIV
#define LRS_LN2_DIV 1
#endif

// row-split kernel (csrc/ista_rs.hip): any n, K <= 512, every prox
namespace lrs {
size_t ista_rs_workspace(int64_t n, int64_t K);
int ista_rs_launch(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad, int64_t K, int64_t nb,
                   const float *alpha, const double *thr, int Nit, int prox, float *coefs, float *phi, void *ws,
                   size_t ws_bytes, int64_t max_wg, hipStream_t st, const float *x0);
int nlm_matlab_col_launch(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K, int64_t nvec, double h,
                          const double *h_per_vec, hipStream_t st);
int64_t dense_gemm_part_floats(int M, int N, int K);
int dense_gemm(int TA, int TB, const float *A, const float *B, float *C, int M, int N, int K, float *part,
               int64_t part_cap, hipStream_t st);

// ---- generic path (any K; the only one for K > 512): the iteration as dense GEMMs ----------------
// Per chunk of up to kGenChunk blocks, every inner iteration is
//   R = X D^T            (chunk x n, dense GEMM)       r = obs .* (Yb - R)
//   G = r D              (chunk x K, dense GEMM)       g = X + G / alpha        X = prox(g)
// and finally Phi = X D^T, the reference's per-block loop (main_LRS_PnP.py:270-303, ista() :131-149)
// for all blocks of the chunk at once.  The products are fp32-accurate (split-bf16 or f32 MFMA),
// the prox is the same kernel as lrs_nlm_col_f32 / lrs_nlm_matlab_col_f32.
constexpr int64_t kGenChunk = 4096;

__global__ void k_gen_resid(float *__restrict__ R, const float *__restrict__ Yb, const uint8_t *__restrict__ obs,
                            int64_t rows, int n, int n_pad) {
    const int64_t total = rows * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = i / n;
        const int r = (int)(i - j * n);
        R[i] = obs[j * n_pad + r] ? Yb[j * n_pad + r] - R[i] : 0.0f;
    }
}

// g = x + G / alpha (in place in G); the quotient as the oracle / reference ((H^T r) / alpha)
__global__ void k_gen_grad(float *__restrict__ G, const float *__restrict__ X, const float *__restrict__ alpha,
                           int64_t rows, int K) {
    const int64_t total = rows * K;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = i / K;
        G[i] = X[i] + G[i] / alpha[j];
    }
}

__global__ void k_gen_soft(const float *__restrict__ G, float *__restrict__ X, const double *__restrict__ thr,
                           int64_t rows, int K) {
    const int64_t total = rows * K;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const float T = (float)thr[i / K], gv = G[i];
        float t = fabsf(gv) - T;
        t = t > 0.f ? t : 0.f;
        X[i] = gv > 0.f ? t : (gv < 0.f ? -t : 0.f);
    }
}

__global__ void k_gen_phi(const float *__restrict__ R, float *__restrict__ phi, int64_t rows, int n, int n_pad) {
    const int64_t total = rows * n_pad;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = i / n_pad;
        const int r = (int)(i - j * n_pad);
        phi[i] = r < n ? R[j * n + r] : 0.0f;
    }
}

inline unsigned gen_blocks(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 8192); }

// split-K scratch for any chunk of <= kGenChunk blocks: the split count grows as the tile count falls,
// so the need peaks at the top of each 64-row band, not at the full chunk
int64_t ista_generic_part_floats(int64_t n, int64_t K) {
    int64_t m = 0;
    for (int64_t rows = 64; rows <= kGenChunk; rows += 64)
        m = std::max(m, std::max(dense_gemm_part_floats((int)rows, (int)n, (int)K),
                                 dense_gemm_part_floats((int)rows, (int)K, (int)n)));
    return m;
}

size_t ista_generic_workspace(int64_t n, int64_t K) {
    const int64_t c = kGenChunk;
    return (size_t)(2 * c * K + c * n + ista_generic_part_floats(n, K)) * sizeof(float) + 256;
}

int ista_generic(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad, int64_t K, int64_t nb,
                 const float *alpha, const double *thr, int Nit, int prox, float *coefs, float *phi, void *ws,
                 size_t ws_bytes, hipStream_t st) {
    if (!ws || ws_bytes < ista_generic_workspace(n, K)) return LRS_E_WORKSPACE;
    if (n > INT32_MAX / 2 || K > 16384) return LRS_E_UNSUPPORTED;
    const int64_t c = kGenChunk;
    float *X = (float *)ws, *G = X + c * K, *R = G + c * K, *part = R + c * n;
    const int64_t part_cap = ista_generic_part_floats(n, K);
    for (int64_t j0 = 0; j0 < nb; j0 += c) {
        const int rows = (int)std::min(c, nb - j0);
        hipError_t e = hipMemsetAsync(X, 0, sizeof(float) * rows * K, st);
        if (e != hipSuccess) return (int)e;
        for (int it = 0; it < Nit; ++it) {
            int rc = dense_gemm(0, 1, X, D, R, rows, (int)n, (int)K, part, part_cap, st);   // R = X D^T
            if (rc) return rc;
            hipLaunchKernelGGL(k_gen_resid, dim3(gen_blocks(rows * n)), dim3(256), 0, st, R, Yb + j0 * n_pad,
                               obs + j0 * n_pad, (int64_t)rows, (int)n, (int)n_pad);
            rc = dense_gemm(0, 0, R, D, G, rows, (int)K, (int)n, part, part_cap, st);          // G = r D
            if (rc) return rc;
            hipLaunchKernelGGL(k_gen_grad, dim3(gen_blocks(rows * K)), dim3(256), 0, st, G, X, alpha + j0,
                               (int64_t)rows, (int)K);
            if (prox == LRS_PROX_SOFT) {
                hipLaunchKernelGGL(k_gen_soft, dim3(gen_blocks(rows * K)), dim3(256), 0, st, G, X, thr + j0,
                                   (int64_t)rows, (int)K);
            } else if (prox == LRS_PROX_NLM_MATLAB) {
                rc = nlm_matlab_col_launch(G, K, X, K, K, rows, 0.0, thr + j0, st);
                if (rc) return rc;
            } else {
                rc = nlm_col_lds(K);
                if (rc) return rc;
                hipLaunchKernelGGL(k_nlm_col, dim3((unsigned)rows), dim3(256), (size_t)(K + 10) * sizeof(float), st, G,
                                   K, X, K, (int)K, 0.0, thr + j0);
            }
            LRS_CHECK_LAUNCH();
        }
        int rc = dense_gemm(0, 1, X, D, R, rows, (int)n, (int)K, part, part_cap, st);          // Phi = X D^T
        if (rc) return rc;
        hipLaunchKernelGGL(k_gen_phi, dim3(gen_blocks(rows * n_pad)), dim3(256), 0, st, R, phi + j0 * n_pad,
                           (int64_t)rows, (int)n, (int)n_pad);
        if (coefs) {
            e = hipMemcpyAsync(coefs + j0 * K, X, sizeof(float) * rows * K, hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return (int)e;
        }
        LRS_CHECK_LAUNCH();
    }
    return LRS_OK;
}
}  // namespace lrs

// The resident kernels (dictionary in LDS) serve n_pad <= 64 with K = 256 and the skimage / soft
// prox; everything else runs the row-split kernel, which needs the fragment-ordered dictionary.
static bool ista_resident(int64_t n_pad, int64_t K, int prox) {
    return n_pad <= kStageRows && K == 256 && prox != LRS_PROX_NLM_MATLAB;
}

// the dense-GEMM path: K > 512, or asked for (lrs_ista_opts.algorithm)
static bool ista_use_generic(int64_t K, const lrs_ista_opts *opts) {
    return K > 512 || (opts && opts->algorithm == LRS_ISTA_ALGO_GENERIC);
}

extern "C" size_t lrs_ista_workspace(int64_t n, int64_t K, int prox, const lrs_ista_opts *opts) {
    if (n <= 0 || K <= 0) return 0;
    if (ista_use_generic(K, opts)) return ista_generic_workspace(n, K);
    if (ista_resident(round_up(n, 16), K, prox)) return 0;
    return ista_rs_workspace(n, K);
}

extern "C" int lrs_ista_f32(const float *Yb, const uint8_t *obs, const float *D, int64_t n,
                            int64_t n_pad, int64_t K, int64_t nb, const float *alpha, const double *thr,
                            int Nit, int prox, float *coefs, float *phi, const lrs_ista_opts *opts, void *ws,
                            size_t ws_bytes, void *stream) {
    if (!Yb || !obs || !D || !alpha || !thr || !phi || n <= 0 || nb < 0 || Nit < 0 || K <= 0) return LRS_E_INVALID;
    const int precision = opts ? opts->precision : LRS_ISTA_SPLIT_BF16;   // per call (no process state)
    if (precision != LRS_ISTA_F32 && precision != LRS_ISTA_SPLIT_BF16) return LRS_E_INVALID;
    const int64_t max_wg = opts ? opts->max_workgroups : 0;
    if (max_wg < 0) return LRS_E_INVALID;
    if (opts && opts->algorithm != LRS_ISTA_ALGO_AUTO && opts->algorithm != LRS_ISTA_ALGO_GENERIC) return LRS_E_INVALID;
    if (opts && opts->warm_start != 0 && opts->warm_start != 1) return LRS_E_INVALID;
    if (n_pad % 16 != 0 || n_pad < n) return LRS_E_INVALID;
    if (prox != LRS_PROX_NLM && prox != LRS_PROX_SOFT && prox != LRS_PROX_NLM_MATLAB) return LRS_E_INVALID;
    if (n_pad > (int64_t)1 << 20 || nb > ((int64_t)1 << 40)) return LRS_E_INVALID;
    if (nb == 0) return LRS_OK;
    hipStream_t st = (hipStream_t)stream;
    // warm start exists only on the row-split kernel: refuse it before any dispatch (the generic path
    // would otherwise restart from zero on every slice)
    const bool warm = opts && opts->warm_start;
    if (warm && (!coefs || ista_use_generic(K, opts) || ista_resident(n_pad, K, prox))) return LRS_E_UNSUPPORTED;
    if (ista_use_generic(K, opts))
        return ista_generic(Yb, obs, D, n, n_pad, K, nb, alpha, thr, Nit, prox, coefs, phi, ws, ws_bytes, st);
    if (!ista_resident(n_pad, K, prox))
        return ista_rs_launch(Yb, obs, D, n, n_pad, K, nb, alpha, thr, Nit, prox, coefs, phi, ws, ws_bytes, max_wg, st,
                              warm ? coefs : nullptr);
    IstaParams p{Yb, obs, D, alpha, thr, coefs, phi, (int)n, (int)n_pad, Nit, prox, nb, 7.0};
    const int64_t blocks_per_wg = (int64_t)kIstaWaves * 16;
    dim3 grid((unsigned)((nb + blocks_per_wg - 1) / blocks_per_wg));
    const bool split = precision == LRS_ISTA_SPLIT_BF16;
    const dim3 grid_b3((unsigned)((nb + kB3Waves * 16 - 1) / (kB3Waves * 16)));
    if (split && prox == LRS_PROX_SOFT)
        hipLaunchKernelGGL((k_ista_b3<256, true>), grid_b3, dim3(kB3Threads), 0, st, p);
    else if (split)
        hipLaunchKernelGGL((k_ista_ln2<256, false, 1, true, LRS_LN2_DIV>), grid_b3, dim3(kB3Threads), 0, st, p);
    else if (prox == LRS_PROX_SOFT)
        hipLaunchKernelGGL((k_ista_res<256, true>), grid, dim3(kIstaThreads), 0, st, p);
    else
        hipLaunchKernelGGL((k_ista_res<256, false>), grid, dim3(kIstaThreads), 0, st, p);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_nlm_col_f32(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K,
                               int64_t nvec, double h, const double *h_per_vec, int patch_size,
                               int patch_distance, void *stream) {
    if (!g || !out || K <= 0 || nvec < 0 || ldg < K || ldo < K) return LRS_E_INVALID;
    if (patch_size != 3 || patch_distance != 3) return LRS_E_UNSUPPORTED;
    if (K > 16384) return LRS_E_UNSUPPORTED;
    if (nvec == 0) return LRS_OK;
    const int rc = nlm_col_lds(K);
    if (rc) return rc;
    hipLaunchKernelGGL(k_nlm_col, dim3((unsigned)nvec), dim3(256), (size_t)(K + 10) * sizeof(float),
                       (hipStream_t)stream, g, ldg, out, ldo, (int)K, h, h_per_vec);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

extern "C" int lrs_nlm_matlab_col_f32(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K,
                                      int64_t nvec, double h, const double *h_per_vec, void *stream) {
    if (!g || !out || K <= 0 || nvec < 0 || ldg < K || ldo < K) return LRS_E_INVALID;
    if (K > 16384) return LRS_E_UNSUPPORTED;
    if (nvec == 0) return LRS_OK;
    return nlm_matlab_col_launch(g, ldg, out, ldo, K, nvec, h, h_per_vec, (hipStream_t)stream);
}
