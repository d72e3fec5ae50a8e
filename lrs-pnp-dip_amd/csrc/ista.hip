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
__device__ __forceinline__ void nlm_chunk(const double (&w)[11], double inv2, double c0, float (&out)[4]) {
    double s1[10], s2[9], s3[8];
#pragma unroll
    for (int i = 0; i < 10; ++i) { double d = w[i] - w[i + 1]; s1[i] = d * d; }
#pragma unroll
    for (int i = 0; i < 9; ++i) { double d = w[i] - w[i + 2]; s2[i] = d * d; }
#pragma unroll
    for (int i = 0; i < 8; ++i) { double d = w[i] - w[i + 3]; s3[i] = d * d; }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int C = 3 + e;
        // t = -3,-2,-1,+1,+2,+3 (the canonical order of oracle_nlm_col)
        const double Dm3 = (s3[C - 3] + s3[C - 2]) * inv2;
        const double Dm2 = (s2[C - 2] + s2[C - 1]) * inv2;
        const double Dm1 = (s1[C - 1] + s1[C]) * inv2;
        const double Dp1 = (s1[C] + s1[C + 1]) * inv2;
        const double Dp2 = (s2[C] + s2[C + 1]) * inv2;
        const double Dp3 = (s3[C] + s3[C + 1]) * inv2;
        const double Ds[6] = {Dm3, Dm2, Dm1, Dp1, Dp2, Dp3};
        const double Vs[6] = {w[C - 3], w[C - 2], w[C - 1], w[C + 1], w[C + 2], w[C + 3]};
        double sw = 0.0, swv = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double wt = (Ds[k] > kNlmCutoff) ? 0.0 : nlm_fast_exp(-Ds[k]);
            sw = sw + wt;
            swv = __fma_rn(wt, Vs[k], swv);
        }
        const double num = __fma_rn(7.0, swv, c0 * w[C]);
        const double den = __fma_rn(7.0, sw, c0);
        out[e] = (float)(num / den);
    }
}

// X <- NLM(G) along the atom axis, for this lane's block (4 atoms per 16-atom tile per lane).
template <int K>
__device__ __forceinline__ void nlm_prox_registers(const floatx4 (&G)[K / 16], float (&X)[K / 16][4],
                                                   double h, int lane) {
    constexpr int NQ = K / 16;
    const int g = lane >> 4;
    const int src_prev = (lane + 48) & 63;  // lane - 16: chunk c-1 (same q) or c-1 of q-1 (g == 0)
    const int src_next = (lane + 16) & 63;  // lane + 16: chunk c+1 (same q) or c+1 of q+1 (g == 3)
    const double inv2 = 2.0 / ((h * h) * 9.0);
    const double c0 = nlm_c0();
    float Pprev[3], Pcur[3], Ncur[4], Nnext[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) Ncur[e] = __shfl(G[0][e], src_next, 64);
#pragma unroll
    for (int e = 0; e < 3; ++e) { Pprev[e] = 0.f; Pcur[e] = 0.f; }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
        for (int e = 0; e < 3; ++e) Pcur[e] = __shfl(G[q][e + 1], src_prev, 64);
        if (q + 1 < NQ) {
#pragma unroll
            for (int e = 0; e < 4; ++e) Nnext[e] = __shfl(G[q + 1][e], src_next, 64);
        }
        float own[4] = {G[q][0], G[q][1], G[q][2], G[q][3]};
        float prv[3], nxt[4];
        if (g == 0) {
            if (q == 0) { prv[0] = own[3]; prv[1] = own[2]; prv[2] = own[1]; }   // reflect
            else { prv[0] = Pprev[0]; prv[1] = Pprev[1]; prv[2] = Pprev[2]; }
        } else {
            prv[0] = Pcur[0]; prv[1] = Pcur[1]; prv[2] = Pcur[2];
        }
        if (g == 3) {
            if (q == NQ - 1) { nxt[0] = own[2]; nxt[1] = own[1]; nxt[2] = own[0]; nxt[3] = prv[2]; }
            else { nxt[0] = Nnext[0]; nxt[1] = Nnext[1]; nxt[2] = Nnext[2]; nxt[3] = Nnext[3]; }
        } else {
            nxt[0] = Ncur[0]; nxt[1] = Ncur[1]; nxt[2] = Ncur[2]; nxt[3] = Ncur[3];
        }
        const double w[11] = {prv[0], prv[1], prv[2], own[0], own[1], own[2], own[3],
                              nxt[0], nxt[1], nxt[2], nxt[3]};
        float o[4];
        nlm_chunk(w, inv2, c0, o);
        X[q][0] = o[0]; X[q][1] = o[1]; X[q][2] = o[2]; X[q][3] = o[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) Pprev[e] = Pcur[e];
#pragma unroll
        for (int e = 0; e < 4; ++e) Ncur[e] = Nnext[e];
    }
}

template <int K, bool RESIDENT>
__global__ __launch_bounds__(kIstaThreads, 2) void k_ista(IstaParams p) {
    constexpr int NQ = K / 16;
    __shared__ __attribute__((aligned(16))) IstaSmem<K> S;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int jl = lane & 15, g = lane >> 4;
    const int64_t j = ((int64_t)blockIdx.x * kIstaWaves + wave) * 16 + jl;
    const bool valid = j < p.nb;
    const int NT = p.n_pad / 16;
    const int nstage = (p.n_pad + kStageRows - 1) / kStageRows;

    const float alpha = valid ? p.alpha[j] : 1.0f;
    const double thr = valid ? p.thr[j] : 1.0;

    float X[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q) X[q][0] = X[q][1] = X[q][2] = X[q][3] = 0.f;

    // Resident mode (n_pad <= 64): y and the row mask live in registers for all iterations.
    float yres[4][4];
    uint32_t mres = 0;
    if (RESIDENT) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            float4 yv = {0.f, 0.f, 0.f, 0.f};
            uint32_t mv = 0;
            if (valid && t < NT) {
                yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
                mv = *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * t + 4 * g]);
            }
            yres[t][0] = yv.x; yres[t][1] = yv.y; yres[t][2] = yv.z; yres[t][3] = yv.w;
#pragma unroll
            for (int i = 0; i < 4; ++i) mres |= (((mv >> (8 * i)) & 0xffu) ? 1u : 0u) << (4 * t + i);
        }
        stage_dictionary<K>(S, p.D, p.n, 0);
        __syncthreads();
    }

    for (int it = 0; it < p.Nit; ++it) {
        floatx4 G[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) G[q] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < nstage; ++s) {
            if (!RESIDENT) {
                __syncthreads();
                stage_dictionary<K>(S, p.D, p.n, s * kStageRows);
                __syncthreads();
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int T = s * 4 + t;
                if (T >= NT) break;
                const floatx4 acc = dict_times_x<K>(S, t, X, jl, g);
                float y[4];
                uint32_t m4;
                if (RESIDENT) {
                    y[0] = yres[t][0]; y[1] = yres[t][1]; y[2] = yres[t][2]; y[3] = yres[t][3];
                    m4 = (mres >> (4 * t)) & 0xfu;
                } else {
                    float4 yv = {0.f, 0.f, 0.f, 0.f};
                    uint32_t mv = 0;
                    if (valid) {
                        yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * T + 4 * g]);
                        mv = *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * T + 4 * g]);
                    }
                    y[0] = yv.x; y[1] = yv.y; y[2] = yv.z; y[3] = yv.w;
                    m4 = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) m4 |= (((mv >> (8 * i)) & 0xffu) ? 1u : 0u) << i;
                }
                float r[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) r[i] = ((m4 >> i) & 1u) ? (y[i] - acc[i]) : 0.0f;
                dict_t_times_r<K>(S, t, r, G, jl, g);
            }
        }
        // gradient = x + (D^T r) / alpha   (…1-LiP.py:190: torch.mm(...) / alpha, then x +)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
#pragma unroll
            for (int i = 0; i < 4; ++i) G[q][i] = X[q][i] + G[q][i] / alpha;
        }
        if (p.prox == LRS_PROX_SOFT) {
            const float T = (float)thr;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float gv = G[q][i];
                    float t = fabsf(gv) - T;
                    t = t > 0.f ? t : 0.f;
                    X[q][i] = gv > 0.f ? t : (gv < 0.f ? -t : 0.f);
                }
            }
        } else {
            nlm_prox_registers<K>(G, X, thr, lane);
        }
    }

    if (valid && p.coefs) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            *reinterpret_cast<float4 *>(&p.coefs[j * K + 16 * q + 4 * g]) =
                make_float4(X[q][0], X[q][1], X[q][2], X[q][3]);
    }
    // Phi_z = Full_Dictionary @ Coefs (all rows, missing ones included: the inpainting step)
    for (int s = 0; s < nstage; ++s) {
        if (!RESIDENT) {
            __syncthreads();
            stage_dictionary<K>(S, p.D, p.n, s * kStageRows);
            __syncthreads();
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int T = s * 4 + t;
            if (T >= NT) break;
            const floatx4 acc = dict_times_x<K>(S, t, X, jl, g);
            if (valid)
                *reinterpret_cast<float4 *>(&p.phi[j * p.n_pad + 16 * T + 4 * g]) =
                    make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    }
}

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
    const double inv2 = 2.0 / ((hh * hh) * 9.0);
    const double c0 = nlm_c0();
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
        double w[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) w[k] = (double)col[i + 5 - 3 + k];
        out[v * ldo + i] = nlm_point<3>(w, inv2, c0);
    }
}

}  // namespace lrs

using namespace lrs;

extern "C" int lrs_ista_f32(const float *Yb, const uint8_t *obs, const float *D, int64_t n,
                            int64_t n_pad, int64_t K, int64_t nb, const float *alpha, const double *thr,
                            int Nit, int prox, float *coefs, float *phi, void *stream) {
    if (!Yb || !obs || !D || !alpha || !thr || !phi || n <= 0 || nb < 0 || Nit < 0) return LRS_E_INVALID;
    if (n_pad % 16 != 0 || n_pad < n) return LRS_E_INVALID;
    if (prox != LRS_PROX_NLM && prox != LRS_PROX_SOFT) return LRS_E_INVALID;
    if (K != 256) return LRS_E_UNSUPPORTED;
    if (nb == 0) return LRS_OK;
    if (n_pad > (int64_t)1 << 20 || nb > ((int64_t)1 << 40)) return LRS_E_INVALID;
    IstaParams p{Yb, obs, D, alpha, thr, coefs, phi, (int)n, (int)n_pad, Nit, prox, nb};
    const int64_t blocks_per_wg = (int64_t)kIstaWaves * 16;
    dim3 grid((unsigned)((nb + blocks_per_wg - 1) / blocks_per_wg));
    hipStream_t st = (hipStream_t)stream;
    if (n_pad <= kStageRows)
        hipLaunchKernelGGL((k_ista<256, true>), grid, dim3(kIstaThreads), 0, st, p);
    else
        hipLaunchKernelGGL((k_ista<256, false>), grid, dim3(kIstaThreads), 0, st, p);
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
    hipLaunchKernelGGL(k_nlm_col, dim3((unsigned)nvec), dim3(256), (size_t)(K + 10) * sizeof(float),
                       (hipStream_t)stream, g, ldg, out, ldo, (int)K, h, h_per_vec);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}
