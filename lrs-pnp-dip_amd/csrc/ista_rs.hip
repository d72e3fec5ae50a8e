// Row-split fused masked ISTA for any block length n and K <= 512 atoms (bb = 36: n = 1296).
//
// Reference path (shuoli0708/LRS-PnP-DIP): the per-block loop of main_LRS_PnP_DIP_1-LiP.py:367-392
// (main_LRS_PnP.py:270-303) calling ista() (…1-LiP.py:185-198 / main_LRS_PnP.py:131-149) on the
// pruned dictionary (delete_element, :201-204), then Phi_z[:,jj] = Full_Dictionary @ Coefs.
//
// Why a second kernel: with n = 1296 the dictionary (n x K fp32 = 1.3 MB at K = 256) cannot stay
// in LDS, and a block's per-iteration work (4 n K FLOP) is 20x the bb = 8 case.  One wave per 16
// blocks over all rows gives only nb/16 waves (401 for the 196x196x198 cube: 39 % of the 1024
// SIMDs), so here the ROWS of a 16-block column tile are split over the S waves of a workgroup:
//
//   wave w, row tiles t in [t0(w), t1(w)):   R_t = D_t x            (16 rows x 16 blocks, MFMA)
//                                             r_t = m .* (y_t - R_t)
//                                             G_w += D_t^T r_t       (K atoms x 16 blocks, MFMA)
//   G = sum_w G_w  (LDS, fixed wave order), gradient g = x + G / alpha, prox(g) -> x  (LDS rows)
//
// Masking instead of pruning: H^T (y - H x) == D^T (m .* (y - D x)), m = observed-row mask.
// Every wave keeps all K coefficients of its 16 blocks in VGPRs (the B operand of R_t); the S
// partial G are reduced by the wave owning each 16-atom tile, which also runs that tile's prox and
// publishes x through LDS.  Four barriers per inner iteration; everything else is wave-local.
//
// The dictionary is read straight from L2 (no LDS staging: each wave reads rows no other wave of
// the workgroup reads) in two images prepared once per call in MFMA fragment order, so every
// load is one 1-KiB coalesced wave instruction:
//   DAf[t][q][lane] = D[16t + (lane&15)][16q + 4(lane>>4) + 0..3]     (A operand of R_t)
//   DTf[t][q][lane] = D[16t + 4(lane>>4) + 0..3][16q + (lane&15)]     (A operand of G_q)
// Products use v_mfma_f32_16x16x4_f32 (exact f32 products; f32 accumulation in MFMA order).
// A ring of 8 float4 keeps the next 8 dictionary fragments in flight across the product and
// row-tile boundaries.
#include "lrs_common.h"
#include "lrs_nlm.h"

namespace lrs {

struct IstaRsParams {
    const float *Yb;       // [nb][n_pad]
    const uint8_t *obs;    // [nb][n_pad]
    const float4 *DAf;     // [NT][NQ][64]
    const float4 *DTf;     // [NT][NQ][64]
    const float *alpha;    // [nb]
    const double *thr;     // [nb]
    float *coefs;          // [nb][K] or null
    float *phi;            // [nb][n_pad]
    int n_pad, K, Nit, prox;
    int64_t nb;
    double seven;
};

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
__device__ __forceinline__ void prox_nlm_chunk(const float *row, int a0, int K, double kneg, double c0, double seven,
                                               float (&out)[4]) {
    double w[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) w[k] = (double)row[reflect_idx(a0 - 3 + k, K)];
    int W1[7], W2[7], W3[7];
    nlm_weights<true>(w, kneg, W1, W2, W3);
    nlm_outputs<2>(w, W1, W2, W3, c0, seven, out);
}

// NLmeansfilter(g, 3, 3, h) of LRS-PnP(Matlab Code)/NLmeansfilter.m:18-78, one output, fp64, in the
// evaluation order of oracle/nlm_oracle.c:oracle_nlm_matlab_col
__device__ __forceinline__ float prox_nlm_matlab_point(const float *row, int i, int K, const double (&krow)[7],
                                                       double h2) {
    double v[13];   // g-hat[i-6 .. i+6]
#pragma unroll
    for (int k = 0; k < 13; ++k) {
        const int j = i - 6 + k;
        v[k] = (j >= -3 && j < K + 3) ? (double)row[symmetric_idx(j, K)] : 0.0;
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
    return sw > 0.0 ? (float)(av / sw) : row[i];
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

// LDS bytes of one workgroup: max(S-1, 1) partial G images of the C*NQ atom tiles (the last one
// doubles as the published x) + the gradient rows
__host__ __device__ constexpr int rs_gstride(int NQ) { return NQ * 16 + 8; }
__host__ __device__ constexpr size_t rs_lds_bytes(int NQ, int C, int S) {
    return (size_t)(S > 1 ? S - 1 : 1) * C * NQ * 1024 + (size_t)C * 16 * rs_gstride(NQ) * 4;
}

template <int NQ, int C, int MINW>
__global__ __launch_bounds__(256, MINW) void k_ista_rs(IstaRsParams p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NTILE = C * NQ;
    constexpr int KS = rs_gstride(NQ);
    constexpr int RING = 8;
    const int lane = threadIdx.x & 63, S = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row range in SGPRs
    const int jl = lane & 15, g = lane >> 4;
    floatx4 *part = reinterpret_cast<floatx4 *>(smem);                 // [NTILE][S-1][64]
    float *gbuf = smem + (size_t)NTILE * (S > 1 ? S - 1 : 1) * 256;  // [C*16][KS]
    floatx4 *xbuf = part;                                              // [NTILE][64], aliases part
    const int NT = p.n_pad >> 4;
    const int t0 = (NT * w) / S, t1 = (NT * (w + 1)) / S;
    const int K = p.K;

    int64_t jc[C];
    bool valid[C];
    float al[C], ral[C];
    double th[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        jc[c] = ((int64_t)blockIdx.x * C + c) * 16 + jl;
        valid[c] = jc[c] < p.nb;
        al[c] = valid[c] ? p.alpha[jc[c]] : 1.0f;
        ral[c] = 1.0f / al[c];
        th[c] = valid[c] ? p.thr[jc[c]] : 1.0;
    }
    const double c0 = nlm_c0();
    double krow[7];
    nlm_matlab_krow_d(krow);

    float X[C][NQ][4];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < NQ; ++q) X[c][q][0] = X[c][q][1] = X[c][q][2] = X[c][q][3] = 0.f;

    // fragment k of row tile t: k < NQ -> DAf q = k, else DTf q = k - NQ.  Buffer loads: the lane's
    // 16-byte offset is the only VGPR, the wave-uniform fragment offset goes in soffset.
    const int img_bytes = NT * NQ * 1024;
    const __amdgpu_buffer_rsrc_t rDA = __builtin_amdgcn_make_buffer_rsrc((void *)p.DAf, 0, img_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rDT = __builtin_amdgcn_make_buffer_rsrc((void *)p.DTf, 0, img_bytes, 0x00020000);
    const int voff = lane * 16;
    auto frag = [&](int t, int k) -> float4 {
        const auto v = k < NQ ? __builtin_amdgcn_raw_buffer_load_b128(rDA, voff, (t * NQ + k) * 1024, 0)
                              : __builtin_amdgcn_raw_buffer_load_b128(rDT, voff, (t * NQ + k - NQ) * 1024, 0);
        return __builtin_bit_cast(float4, v);
    };

    for (int it = 0; it < p.Nit; ++it) {
        floatx4 G[C][NQ];
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int q = 0; q < NQ; ++q) G[c][q] = floatx4{0.f, 0.f, 0.f, 0.f};

        float4 ring[RING];
        if (t0 < t1) {
#pragma unroll
            for (int k = 0; k < RING; ++k) ring[k] = frag(t0, k);
        }
        for (int t = t0; t < t1; ++t) {
            // observations of this row tile (consumed after product A)
            float4 yv[C];
            uint32_t mv[C];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                yv[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                mv[c] = 0;
                if (valid[c]) {
                    yv[c] = *reinterpret_cast<const float4 *>(&p.Yb[jc[c] * p.n_pad + 16 * t + 4 * g]);
                    mv[c] = *reinterpret_cast<const uint32_t *>(&p.obs[jc[c] * p.n_pad + 16 * t + 4 * g]);
                }
            }
            floatx4 RA[C], RB[C];
#pragma unroll
            for (int c = 0; c < C; ++c) RA[c] = RB[c] = floatx4{0.f, 0.f, 0.f, 0.f};
            float r[C][4];
            float4 pend = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 2 * NQ; ++k) {
                const float4 a = ring[k % RING];
                const int kk = k + RING;
                if (kk < 2 * NQ) ring[k % RING] = frag(t, kk);
                else if (t + 1 < t1) ring[k % RING] = frag(t + 1, kk - 2 * NQ);
                if (k < NQ) {
                    // R_t += D[rows of t][atoms 16q..] x[16q..]; even / odd q on two accumulators
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        floatx4 &acc = (k & 1) ? RB[c] : RA[c];
                        acc = mfma16x16x4(a.x, X[c][k][0], acc);
                        acc = mfma16x16x4(a.y, X[c][k][1], acc);
                        acc = mfma16x16x4(a.z, X[c][k][2], acc);
                        acc = mfma16x16x4(a.w, X[c][k][3], acc);
                    }
                    if (k == NQ - 1) {
#pragma unroll
                        for (int c = 0; c < C; ++c) {
                            const floatx4 R = RA[c] + RB[c];
                            const float y4[4] = {yv[c].x, yv[c].y, yv[c].z, yv[c].w};
#pragma unroll
                            for (int e = 0; e < 4; ++e) r[c][e] = ((mv[c] >> (8 * e)) & 0xffu) ? (y4[e] - R[e]) : 0.0f;
                        }
                    }
                } else {
                    // G_q += D^T[atoms 16q..][rows of t] r_t; q pairs interleaved (MFMA latency)
                    const int q = k - NQ;
                    if ((q & 1) == 0) {
                        pend = a;
                    } else {
#pragma unroll
                        for (int s = 0; s < 4; ++s) {
                            const float a0 = s == 0 ? pend.x : s == 1 ? pend.y : s == 2 ? pend.z : pend.w;
                            const float a1 = s == 0 ? a.x : s == 1 ? a.y : s == 2 ? a.z : a.w;
#pragma unroll
                            for (int c = 0; c < C; ++c) {
                                G[c][q - 1] = mfma16x16x4(a0, r[c][s], G[c][q - 1]);
                                G[c][q] = mfma16x16x4(a1, r[c][s], G[c][q]);
                            }
                        }
                    }
                }
            }
        }

        // ---- reduce the S partial gradients (fixed wave order) and form g = x + G / alpha -------
        if (S > 1) {
#pragma unroll
            for (int T = 0; T < NTILE; ++T) {
                const int o = T % S;
                if (w != o) part[((size_t)T * (S - 1) + (w - (w > o))) * 64 + lane] = G[T / NQ][T % NQ];
            }
            __syncthreads();
        }
#pragma unroll
        for (int T = 0; T < NTILE; ++T) {
            const int c = T / NQ, q = T % NQ;
            if (w == T % S) {
                floatx4 s = floatx4{0.f, 0.f, 0.f, 0.f};
                for (int k = 0; k < S; ++k) {
                    if (k == w) {
                        s += G[c][q];
                    } else {
                        s += part[((size_t)T * (S - 1) + (k - (k > w))) * 64 + lane];
                    }
                }
                float4 gr;
                gr.x = X[c][q][0] + rs_div(s[0], al[c], ral[c]);
                gr.y = X[c][q][1] + rs_div(s[1], al[c], ral[c]);
                gr.z = X[c][q][2] + rs_div(s[2], al[c], ral[c]);
                gr.w = X[c][q][3] + rs_div(s[3], al[c], ral[c]);
                *reinterpret_cast<float4 *>(&gbuf[(c * 16 + jl) * KS + 16 * q + 4 * g]) = gr;
            }
        }
        __syncthreads();

        // ---- prox of the owned atom tiles (runtime loop: one inlined prox body), x through LDS ----
        for (int T = w; T < NTILE; T += S) {
            const int c = T / NQ, q = T - c * NQ;
            const double thc = (C == 1 || c == 0) ? th[0] : th[C - 1];
            const float *row = gbuf + (c * 16 + jl) * KS;
            const int a0 = 16 * q + 4 * g;
            float o[4];
            if (p.prox == LRS_PROX_SOFT) {
                const float Tt = (float)thc;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float gv = row[a0 + e];
                    float tv = fabsf(gv) - Tt;
                    tv = tv > 0.f ? tv : 0.f;
                    o[e] = gv > 0.f ? tv : (gv < 0.f ? -tv : 0.f);
                }
            } else if (p.prox == LRS_PROX_NLM_MATLAB) {
                const double h2 = thc * thc;
                for (int e = 0; e < 4; ++e) o[e] = a0 + e < K ? prox_nlm_matlab_point(row, a0 + e, K, krow, h2) : 0.f;
            } else {
                prox_nlm_chunk(row, a0, K, nlm_kneg(thc), c0, p.seven, o);
            }
            xbuf[(size_t)T * 64 + lane] = floatx4{a0 < K ? o[0] : 0.f, a0 + 1 < K ? o[1] : 0.f, a0 + 2 < K ? o[2] : 0.f,
                                                  a0 + 3 < K ? o[3] : 0.f};
        }
        __syncthreads();
#pragma unroll
        for (int T = 0; T < NTILE; ++T) {
            const floatx4 v = xbuf[(size_t)T * 64 + lane];
            X[T / NQ][T % NQ][0] = v[0]; X[T / NQ][T % NQ][1] = v[1];
            X[T / NQ][T % NQ][2] = v[2]; X[T / NQ][T % NQ][3] = v[3];
        }
        __syncthreads();   // the next iteration's partials overwrite xbuf
    }

    // ---- outputs: coefficients (owned tiles) and Phi = D x over this wave's row tiles ----------
    if (p.coefs) {
#pragma unroll
        for (int T = 0; T < NTILE; ++T) {
            const int c = T / NQ, q = T % NQ;
            if (w == T % S && valid[c]) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int a = 16 * q + 4 * g + e;
                    if (a < K) p.coefs[jc[c] * K + a] = X[c][q][e];
                }
            }
        }
    }
    for (int t = t0; t < t1; ++t) {
        floatx4 RA[C], RB[C];
#pragma unroll
        for (int c = 0; c < C; ++c) RA[c] = RB[c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float4 a = p.DAf[((size_t)t * NQ + q) * 64 + lane];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                floatx4 &acc = (q & 1) ? RB[c] : RA[c];
                acc = mfma16x16x4(a.x, X[c][q][0], acc);
                acc = mfma16x16x4(a.y, X[c][q][1], acc);
                acc = mfma16x16x4(a.z, X[c][q][2], acc);
                acc = mfma16x16x4(a.w, X[c][q][3], acc);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (!valid[c]) continue;
            const floatx4 R = RA[c] + RB[c];
            *reinterpret_cast<float4 *>(&p.phi[jc[c] * p.n_pad + 16 * t + 4 * g]) = make_float4(R[0], R[1], R[2], R[3]);
        }
    }
}

// Fragment-ordered dictionary images (zero past n rows / K atoms).  One thread per float4.
__global__ __launch_bounds__(256) void k_ista_rs_prep(const float *__restrict__ D, int n, int K, int NT, int NQ,
                                                      float4 *__restrict__ DAf, float4 *__restrict__ DTf) {
    const int64_t total = (int64_t)NT * NQ * 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        const int64_t tq = i >> 6;
        const int q = (int)(tq % NQ), t = (int)(tq / NQ);
        const int jl = lane & 15, g = lane >> 4;
        float a[4], b[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int ra = 16 * t + jl, ca = 16 * q + 4 * g + s;
            a[s] = (ra < n && ca < K) ? D[(int64_t)ra * K + ca] : 0.f;
            const int rb = 16 * t + 4 * g + s, cb = 16 * q + jl;
            b[s] = (rb < n && cb < K) ? D[(int64_t)rb * K + cb] : 0.f;
        }
        DAf[i] = make_float4(a[0], a[1], a[2], a[3]);
        DTf[i] = make_float4(b[0], b[1], b[2], b[3]);
    }
}

// NLmeansfilter(g, 3, 3, h) of one column per workgroup (the MATLAB-variant prox drop-in)
__global__ __launch_bounds__(256) void k_nlm_matlab_col(const float *__restrict__ g, int64_t ldg,
                                                        float *__restrict__ out, int64_t ldo, int K, double h,
                                                        const double *__restrict__ hv) {
    extern __shared__ float col[];
    const int64_t v = blockIdx.x;
    for (int i = threadIdx.x; i < K; i += blockDim.x) col[i] = g[v * ldg + i];
    __syncthreads();
    const double hh = hv ? hv[v] : h;
    double krow[7];
    nlm_matlab_krow_d(krow);
    for (int i = threadIdx.x; i < K; i += blockDim.x) out[v * ldo + i] = prox_nlm_matlab_point(col, i, K, krow, hh * hh);
}

// ---- launcher ---------------------------------------------------------------------------------

static int g_cu_count = 0;

static int cu_count() {
    if (g_cu_count == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                      hipSuccess || n <= 0)
            n = 256;
        g_cu_count = n;
    }
    return g_cu_count;
}

static int rs_nq(int64_t K) { return K <= 64 ? 4 : K <= 128 ? 8 : K <= 256 ? 16 : 32; }

size_t ista_rs_workspace(int64_t n, int64_t K) {
    const int64_t n_pad = round_up(n, 16);
    return (size_t)2 * n_pad * rs_nq(K) * 16 * sizeof(float);
}

// Waves per workgroup S: the per-SIMD makespan ceil(tiles S / SIMDs) / S, smallest S on ties;
// capped by the rows (one row tile per wave at least) and by LDS (two workgroups per CU).
static int rs_pick_waves(int64_t tiles, int NT, int NQ, int C, int minw) {
    const int64_t simds = (int64_t)cu_count() * 4 * (minw >= 2 ? 2 : 1);
    int best = 1;
    double best_t = 1e30;
    for (int S = 1; S <= 4 && S <= NT; ++S) {
        if (rs_lds_bytes(NQ, C, S) > (minw >= 2 ? 81920u : 163840u)) break;
        const double t = (double)((tiles * S + simds - 1) / simds) / S;
        if (t < best_t * 0.999) {
            best_t = t;
            best = S;
        }
    }
    return best;
}

template <int NQ, int C, int MINW>
static int launch_rs(const IstaRsParams &p, int NT, hipStream_t st) {
    const int64_t cols = 16 * C;
    const int64_t tiles = (p.nb + cols - 1) / cols;
    const int S = rs_pick_waves(tiles, NT, NQ, C, MINW);
    const size_t lds = rs_lds_bytes(NQ, C, S);
    static bool lds_opt_in = false;   // dynamic LDS beyond 64 KiB
    if (!lds_opt_in) {
        const hipError_t e = hipFuncSetAttribute((const void *)k_ista_rs<NQ, C, MINW>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return (int)e;
        lds_opt_in = true;
    }
    hipLaunchKernelGGL((k_ista_rs<NQ, C, MINW>), dim3((unsigned)tiles), dim3(64 * S), lds, st, p);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int ista_rs_launch(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad, int64_t K, int64_t nb,
                   const float *alpha, const double *thr, int Nit, int prox, float *coefs, float *phi, void *ws,
                   size_t ws_bytes, int cols_per_wave, hipStream_t st) {
    if (K < 1 || K > 512) return LRS_E_UNSUPPORTED;
    const int NQ = rs_nq(K);
    const int NT = (int)(n_pad / 16);
    if (!ws || ws_bytes < ista_rs_workspace(n, K)) return LRS_E_WORKSPACE;
    float4 *DAf = reinterpret_cast<float4 *>(ws);
    float4 *DTf = DAf + (size_t)NT * NQ * 64;
    {
        const int64_t total = (int64_t)NT * NQ * 64;
        const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
        hipLaunchKernelGGL(k_ista_rs_prep, dim3(blocks), dim3(256), 0, st, D, (int)n, (int)K, NT, NQ, DAf, DTf);
        LRS_CHECK_LAUNCH();
    }
    IstaRsParams p{Yb, obs, DAf, DTf, alpha, thr, coefs, phi, (int)n_pad, (int)K, Nit, prox, nb, 7.0};
    switch (NQ) {
    case 4: return launch_rs<4, 1, 2>(p, NT, st);
    case 8: return launch_rs<8, 1, 2>(p, NT, st);
    case 16: return cols_per_wave == 2 ? launch_rs<16, 2, 1>(p, NT, st) : launch_rs<16, 1, 2>(p, NT, st);
    default: return launch_rs<32, 1, 1>(p, NT, st);
    }
}

int nlm_matlab_col_launch(const float *g, int64_t ldg, float *out, int64_t ldo, int64_t K, int64_t nvec, double h,
                          const double *h_per_vec, hipStream_t st) {
    hipLaunchKernelGGL(k_nlm_matlab_col, dim3((unsigned)nvec), dim3(256), (size_t)K * sizeof(float), st, g, ldg, out,
                       ldo, (int)K, h, h_per_vec);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

}  // namespace lrs
