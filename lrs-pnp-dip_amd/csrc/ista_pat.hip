// Masked ISTA on per-pattern Grams: the row-split kernel's iteration for blocks that share
// observation patterns (any n, K <= 512, every prox).
//
// Reference path (shuoli0708/LRS-PnP-DIP): ista() (main_LRS_PnP.py:131-149, …1-LiP.py:185-198) on
// the dictionary pruned to a block's observed rows (delete_element, :201-204), once per block
// (main_LRS_PnP.py:270-303, …1-LiP.py:367-392).  Its gradient is
//     H^T (y - H x) = D^T (m .* y) - D^T diag(m) D x = b - Q_m x        (m = the observed-row mask)
// and the masks of a hyperspectral cube repeat: the bands of a block share their pixels' mask,
// and a tiled mask repeats along the pixel rows (the bench's 196 x 196 x 198 cube: 27 patterns for
// 6,408 blocks).  So Q_p is formed once per pattern (lrs_ista_pat_prepare, once per D and set of
// patterns), b once per block and call, and every inner iteration costs 2 K^2 FLOP per block
// instead of 4 n K (n = 1296, K = 256: 10x fewer):
//   k_pat_gram : Q_p = D^T diag(m_p) D for every pattern, fp64 sums on v_mfma_f64_16x16x4 (exact
//                products of float32 values), rounded to float32 and stored as MFMA A-fragment
//                images QAf[p][q][kq][lane] = Q[16 q + (lane & 15)][16 kq + 4 (lane >> 4) + 0..3];
//   k_ista_pat : one workgroup per tile of <= 16 blocks of ONE pattern (lrs_ista_pat_plan groups
//                them).  Wave w owns the atom tiles q = w, w + S, ...: b_q = D_q^T (m .* y) once, then
//                per iteration acc_q = Q_p[q, :] x (x from LDS, Q fragments from L2 through a
//                register ring), g = x + (b_q - acc_q) / alpha into LDS, barrier, the prox of its
//                tiles back into x, barrier.  No cross-wave reduction: each wave sums all K atoms of
//                its rows.  Finally Phi = D x over row tiles split across the waves.
// Products are v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation), the prox is the
// row-split kernel's (ista_prox.h), so the result differs from lrs_ista_f32's by rounding only
// (tests/test_gpu_kernels.py: both against the oracle at 1e-5).
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ista_prox.h"

namespace lrs {

// row-split kernel's dictionary images (ista_rs.hip)
int ista_rs_images(const float *D, int64_t n, int64_t K, int NT, int NQ, float4 *DAf, float4 *DTf, hipStream_t st);

typedef double pg_d4 __attribute__((ext_vector_type(4)));

static int pat_nq(int64_t K) { return K <= 64 ? 4 : K <= 128 ? 8 : K <= 256 ? 16 : 32; }

// ---- Q_p = D^T diag(m_p) D ----------------------------------------------------------------------
// grid (upper 64 x 64 block pairs (bi <= bj) of the KP x KP Gram, npat), 256 threads: wave w forms
// the 16 rows of atom tile 4 bi + w against the 64 columns of block bj (4 f64 accumulators), the
// inner sum over the n dictionary rows 4 at a time in row order.  The sum of exact products is the
// same for (a, c) and (c, a), so the mirror tile is written from the same values.
__global__ __launch_bounds__(256) void k_pat_gram(const float *__restrict__ D, int n, int K, int NQ,
                                                  const uint8_t *__restrict__ obs_pat, int n_pad,
                                                  float *__restrict__ QAf) {
    const int NB = NQ >> 2;
    int bi = 0, rem = blockIdx.x;
    while (rem >= NB - bi) { rem -= NB - bi; ++bi; }
    const int bj = bi + rem;
    const int p = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, kk = lane >> 4;
    const int qt = 4 * bi + w;
    const int a = 16 * qt + i;
    const uint8_t *m = obs_pat + (int64_t)p * n_pad;
    pg_d4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = pg_d4{0.0, 0.0, 0.0, 0.0};
    // the next 16 rows' operands are loaded while this step's 16 MFMAs run
    double av[4], bv[4][4];
    auto load = [&](int r0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int r = r0 + 4 * s + kk;
            const bool ok = r < n;
            av[s] = (ok && a < K && m[r]) ? (double)D[(int64_t)r * K + a] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = 16 * (4 * bj + u) + i;
                bv[s][u] = (ok && c < K) ? (double)D[(int64_t)r * K + c] : 0.0;
            }
        }
    };
    load(0);
    for (int r0 = 0; r0 < n; r0 += 16) {
        double ca[4], cb[4][4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            ca[s] = av[s];
#pragma unroll
            for (int u = 0; u < 4; ++u) cb[s][u] = bv[s][u];
        }
        if (r0 + 16 < n) load(r0 + 16);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[s], cb[s][u], acc[u], 0, 0, 0);
    }
    // C/D layout of the f64 MFMA: column lane & 15, row (lane >> 4) + 4 r
    float *Qp = QAf + (int64_t)p * NQ * NQ * 256;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int kt = 4 * bj + u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ii = kk + 4 * r, jj = i;   // (row 16 qt + ii, column 16 kt + jj)
            const float v = (float)acc[u][r];
            Qp[((int64_t)(qt * NQ + kt) * 64 + ii + 16 * (jj >> 2)) * 4 + (jj & 3)] = v;
            if (bi != bj) Qp[((int64_t)(kt * NQ + qt) * 64 + jj + 16 * (ii >> 2)) * 4 + (ii & 3)] = v;
        }
    }
}

struct IstaPatParams {
    const float *Yb;          // [nb][n_pad]
    const uint8_t *obs_pat;   // [npat][n_pad]
    const int32_t *plan;      // lrs_ista_pat_plan: order [nb], then tiles [ntiles][2]
    const float4 *DAf;        // [NT][NQ][64]
    const float4 *DTf;        // [NT][NQ][64]
    const float4 *QAf;        // [npat][NQ][NQ][64]
    const float *alpha;       // [nb]
    const double *thr;        // [nb]
    float *coefs;             // [nb][K] or null
    float *phi;               // [nb][n_pad]
    const float *x0;          // [nb][K] start coefficients (warm start; may alias coefs) or null = 0
    int n_pad, K, Nit, prox;
    int64_t nb, ntiles, npat;
    double seven;
};

// LDS: x [NQ][64] floatx4 (the B operand of every product, rewritten by the prox), then the
// gradient rows [16 blocks][KP] read by the prox (chunk index XOR-swizzled by block)
__host__ __device__ constexpr size_t pat_lds_bytes(int NQ) { return (size_t)NQ * 2048; }

// WPE: waves per SIMD the registers are bounded for (2: one 512-thread workgroup per CU; 4: two)
template <int NQ, int S, int WPE = 2>
__global__ __launch_bounds__(64 * S, WPE) void k_ista_pat(IstaPatParams p) {
    static_assert(NQ % S == 0, "atom tiles split evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int KP = NQ * 16;
    constexpr int NOWN = NQ / S;                  // atom tiles per wave
    constexpr int NFRAG = NQ * NOWN;              // Q fragments per wave and iteration
    constexpr int RMAX = WPE > 2 ? 4 : 8;
    constexpr int RING = NFRAG < RMAX ? NFRAG : RMAX;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int jl = lane & 15, g = lane >> 4;
    floatx4 *xbuf = reinterpret_cast<floatx4 *>(smem);
    float *gbuf = reinterpret_cast<float *>(xbuf + NQ * 64);
    const int NT = p.n_pad >> 4;
    const int t0 = (NT * w) / S, t1 = (NT * (w + 1)) / S;
    const int K = p.K;
    const int32_t *order = p.plan;
    const int32_t *tiles = p.plan + p.nb;
    const int voff = lane * 16;
    const int img_bytes = NT * NQ * 1024;
    const __amdgpu_buffer_rsrc_t rDA = __builtin_amdgcn_make_buffer_rsrc((void *)p.DAf, 0, img_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rDT = __builtin_amdgcn_make_buffer_rsrc((void *)p.DTf, 0, img_bytes, 0x00020000);
    auto gq = [&](const floatx4 &G, float4 a, const float (&r)[4]) -> floatx4 {
        floatx4 acc = G;
        acc = mfma16x16x4(a.x, r[0], acc);
        acc = mfma16x16x4(a.y, r[1], acc);
        acc = mfma16x16x4(a.z, r[2], acc);
        acc = mfma16x16x4(a.w, r[3], acc);
        return acc;
    };

    // XCD-aware tile order: workgroup b runs on XCD b % 8 (round-robin dispatch), so with one
    // workgroup per tile XCD x takes the x-th contiguous eighth of the (pattern-major) tile list and
    // its L2 holds only those patterns' Q images (all 27 of the bench cube: 6.9 MB > 4 MB per XCD)
    int64_t first = blockIdx.x;
    if (gridDim.x == p.ntiles) {
        const int64_t q = p.ntiles >> 3, r = p.ntiles & 7, x = blockIdx.x & 7, i = blockIdx.x >> 3;
        first = x * q + std::min<int64_t>(x, r) + i;
    }
    for (int64_t tile = first; tile < p.ntiles; tile += gridDim.x) {
        if (tile != first) __syncthreads();   // the previous tile's last reads of xbuf / gbuf are done
        // tile descriptor (clamped: a malformed plan cannot address outside the arrays; a start
        // outside [0, nb) makes the tile empty)
        const int64_t start = tiles[2 * tile];
        const int pc = tiles[2 * tile + 1];
        const int pat = (int)std::min<int64_t>(std::max(pc >> 5, 0), p.npat - 1);
        const int cnt = (start >= 0 && start < p.nb) ? std::min(pc & 31, 16) : 0;
        const int64_t jo = start + jl;
        int64_t j = (jl < cnt && jo < p.nb) ? order[jo] : -1;
        const bool valid = j >= 0 && j < p.nb;
        if (!valid) j = 0;
        const float al = valid ? p.alpha[j] : 1.0f;
        const float ral = 1.0f / al;
        const double th = valid ? p.thr[j] : 1.0;
        const double c0 = nlm_c0();
        double krow[7];
        nlm_matlab_krow_d(krow);

        for (int i = threadIdx.x; i < NQ * 64; i += 64 * S) {
            floatx4 v = {0.f, 0.f, 0.f, 0.f};
            const int b = i & 15;
            if (p.x0 && b < cnt && start + b < p.nb) {
                const int64_t jb = order[start + b];
                const int a0 = 16 * (i >> 6) + 4 * ((i & 63) >> 4);
                if (jb >= 0 && jb < p.nb)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (a0 + e < K) v[e] = p.x0[jb * K + a0 + e];
            }
            xbuf[i] = v;
        }

        // ---- b_q = D_q^T (m .* y) of the owned atom tiles, all row tiles ----------------------------
        const uint8_t *mrow = p.obs_pat + (int64_t)pat * p.n_pad;
        floatx4 bown[NOWN];
#pragma unroll
        for (int o = 0; o < NOWN; ++o) bown[o] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < NT; ++t) {
            const uint32_t mv = *reinterpret_cast<const uint32_t *>(mrow + 16 * t + 4 * g);
            float4 yv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (valid) yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
            const float r[4] = {(mv & 0xffu) ? yv.x : 0.f, (mv & 0xff00u) ? yv.y : 0.f, (mv & 0xff0000u) ? yv.z : 0.f,
                                (mv & 0xff000000u) ? yv.w : 0.f};
#pragma unroll
            for (int o = 0; o < NOWN; ++o) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rDT, voff, (t * NQ + w + S * o) * 1024, 0);
                bown[o] = gq(bown[o], __builtin_bit_cast(float4, v), r);
            }
        }

        // Q fragments of this wave in iteration order k = kq NOWN + o (the same sequence every
        // iteration, so the ring runs on across iterations)
        const __amdgpu_buffer_rsrc_t rQ = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.QAf + (int64_t)pat * NQ * NQ * 64), 0, NQ * NQ * 1024, 0x00020000);
        auto qfrag = [&](int k) -> float4 {
            const int kq = k / NOWN, o = k - kq * NOWN;
            return __builtin_bit_cast(float4,
                                      __builtin_amdgcn_raw_buffer_load_b128(rQ, voff, ((w + S * o) * NQ + kq) * 1024, 0));
        };
        float4 ring[RING];
#pragma unroll
        for (int k = 0; k < RING; ++k) ring[k] = qfrag(k);
        __syncthreads();   // x0 in LDS

        for (int it = 0; it < p.Nit; ++it) {
            floatx4 acc[NOWN];
#pragma unroll
            for (int o = 0; o < NOWN; ++o) acc[o] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kq = 0; kq < NQ; ++kq) {
                const floatx4 xv = xbuf[kq * 64 + lane];
#pragma unroll
                for (int o = 0; o < NOWN; ++o) {
                    const int k = kq * NOWN + o;
                    const float4 a = ring[k % RING];
                    ring[k % RING] = qfrag((k + RING) % NFRAG);
                    acc[o] = mfma16x16x4(a.x, xv[0], acc[o]);
                    acc[o] = mfma16x16x4(a.y, xv[1], acc[o]);
                    acc[o] = mfma16x16x4(a.z, xv[2], acc[o]);
                    acc[o] = mfma16x16x4(a.w, xv[3], acc[o]);
                }
            }
            // g = x + (b - Q x) / alpha of the owned tiles -> gbuf
#pragma unroll
            for (int o = 0; o < NOWN; ++o) {
                const int q = w + S * o;
                const floatx4 xo = xbuf[q * 64 + lane];
                float4 gr;
                gr.x = xo[0] + rs_div(bown[o][0] - acc[o][0], al, ral);
                gr.y = xo[1] + rs_div(bown[o][1] - acc[o][1], al, ral);
                gr.z = xo[2] + rs_div(bown[o][2] - acc[o][2], al, ral);
                gr.w = xo[3] + rs_div(bown[o][3] - acc[o][3], al, ral);
                *reinterpret_cast<float4 *>(&gbuf[jl * KP + gsw(jl, 16 * q + 4 * g)]) = gr;
            }
            __syncthreads();   // every wave's products have read x; the gradient rows are complete

            // ---- prox of the owned atom tiles (runtime loop: one inlined prox body) -> xbuf -------------
            for (int q = w; q < NQ; q += S) {
                const float *row = gbuf + jl * KP;
                const int a0 = 16 * q + 4 * g;
                float o[4];
                if (p.prox == LRS_PROX_SOFT) {
                    const float Tt = (float)th;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float gv = row[gsw(jl, a0 + e)];
                        float tv = fabsf(gv) - Tt;
                        tv = tv > 0.f ? tv : 0.f;
                        o[e] = gv > 0.f ? tv : (gv < 0.f ? -tv : 0.f);
                    }
                } else if (p.prox == LRS_PROX_NLM_MATLAB) {
                    const double h2 = th * th;
                    for (int e = 0; e < 4; ++e)
                        o[e] = a0 + e < K ? prox_nlm_matlab_point(row, jl, a0 + e, K, krow, h2) : 0.f;
                } else {
                    prox_nlm_chunk_v4(row, jl, a0, K, nlm_kneg(th), c0, p.seven, o);
                }
                xbuf[q * 64 + lane] = floatx4{a0 < K ? o[0] : 0.f, a0 + 1 < K ? o[1] : 0.f, a0 + 2 < K ? o[2] : 0.f,
                                              a0 + 3 < K ? o[3] : 0.f};
            }
            __syncthreads();
        }

        // ---- outputs: coefficients (owned tiles) and Phi = D x over this wave's row tiles ----------
        if (p.coefs && valid) {
            for (int q = w; q < NQ; q += S) {
                const floatx4 xv = xbuf[q * 64 + lane];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int a = 16 * q + 4 * g + e;
                    if (a < K) p.coefs[j * K + a] = xv[e];
                }
            }
        }
        for (int t = t0; t < t1; ++t) {
            floatx4 RA = {0.f, 0.f, 0.f, 0.f}, RB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const float4 a =
                    __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rDA, voff, (t * NQ + q) * 1024, 0));
                const floatx4 xv = xbuf[q * 64 + lane];
                floatx4 &acc = (q & 1) ? RB : RA;
                acc = mfma16x16x4(a.x, xv[0], acc);
                acc = mfma16x16x4(a.y, xv[1], acc);
                acc = mfma16x16x4(a.z, xv[2], acc);
                acc = mfma16x16x4(a.w, xv[3], acc);
            }
            if (valid) {
                const floatx4 R = RA + RB;
                *reinterpret_cast<float4 *>(&p.phi[j * p.n_pad + 16 * t + 4 * g]) = make_float4(R[0], R[1], R[2], R[3]);
            }
        }
    }   // tile
}

// ---- host side --------------------------------------------------------------------------------

// n_pad: the images' row count (the kernels index them with NT = n_pad / 16)
static int64_t pat_images_floats(int64_t n_pad, int64_t K, int64_t npat) {
    const int64_t NT = round_up(n_pad, 16) / 16, NQ = pat_nq(K);
    return 2 * NT * NQ * 64 * 4 + npat * NQ * NQ * 256;
}

size_t ista_pat_workspace(int64_t n, int64_t K, int64_t npat) {
    if (n <= 0 || K <= 0 || K > 512 || npat <= 0) return 0;
    return (size_t)pat_images_floats(n, K, npat) * sizeof(float);
}

// Waves per workgroup: 8 for K > 128 (configs[2] sparse coding alone: 2.00 ms vs 2.10 ms with 4;
// profiles/r04/ista_pat/), 4 below (one or two atom tiles per wave).
#ifdef LRS_TUNING
static int pat_waves_knob() {
    const char *e = getenv("LRS_ISTA_PAT_WAVES");
    return e ? atoi(e) : 0;
}
static int pat_wpe_knob() {   // LRS_ISTA_PAT_WPE=4: the 128-register form (two workgroups per CU)
    const char *e = getenv("LRS_ISTA_PAT_WPE");
    return e ? atoi(e) : 0;
}
#endif

template <int NQ, int S, int WPE = 2>
static int launch_pat_k(const IstaPatParams &p, int64_t max_wg, hipStream_t st) {
    static std::atomic<uint64_t> opted{0};   // per device
    if (const int rc = lds_opt_in((const void *)k_ista_pat<NQ, S, WPE>, 160 * 1024, opted)) return rc;
    int64_t grid = p.ntiles;
    if (max_wg > 0 && grid > max_wg) grid = max_wg;
    hipLaunchKernelGGL((k_ista_pat<NQ, S, WPE>), dim3((unsigned)grid), dim3(64 * S), pat_lds_bytes(NQ), st, p);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

// The dictionary images (DAf, DTf) and every pattern's Gram image (QAf) into ws: once per D and
// set of patterns (the solver prepares at construction: both are fixed for a whole solve).
int ista_pat_prepare(const float *D, int64_t n, int64_t K, const uint8_t *obs_pat, int64_t npat, int64_t n_pad,
                     void *ws, size_t ws_bytes, hipStream_t st) {
    if (K < 1 || K > 512) return LRS_E_UNSUPPORTED;
    // sized from n_pad, which sets the images' row count (lrs_ista_pat_workspace(n) covers the
    // n_pad = round_up(n, 16) every caller of the solver uses; a larger n_pad needs its own size)
    if (!ws || ws_bytes < (size_t)pat_images_floats(n_pad, K, npat) * sizeof(float)) return LRS_E_WORKSPACE;
    const int NQ = pat_nq(K);
    const int NT = (int)(n_pad / 16);
    if ((int64_t)NT * NQ * 1024 >= ((int64_t)1 << 31)) return LRS_E_UNSUPPORTED;   // 32-bit buffer offsets
    if (n > INT32_MAX / 2 || npat > 65535) return LRS_E_UNSUPPORTED;
    float4 *DAf = reinterpret_cast<float4 *>(ws);
    float4 *DTf = DAf + (size_t)NT * NQ * 64;
    float4 *QAf = DTf + (size_t)NT * NQ * 64;
    const int rc = ista_rs_images(D, n, K, NT, NQ, DAf, DTf, st);
    if (rc) return rc;
    const int NB = NQ / 4;
    hipLaunchKernelGGL(k_pat_gram, dim3((unsigned)(NB * (NB + 1) / 2), (unsigned)npat), dim3(256), 0, st, D, (int)n,
                       (int)K, NQ, obs_pat, (int)n_pad, reinterpret_cast<float *>(QAf));
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int ista_pat_launch(const float *Yb, const uint8_t *obs_pat, int64_t npat, const int32_t *plan, int64_t ntiles,
                    int64_t n, int64_t n_pad, int64_t K, int64_t nb, const float *alpha, const double *thr, int Nit,
                    int prox, float *coefs, float *phi, void *ws, size_t ws_bytes, int64_t max_wg, hipStream_t st,
                    const float *x0) {
    if (K < 1 || K > 512) return LRS_E_UNSUPPORTED;
    if (!ws || ws_bytes < (size_t)pat_images_floats(n_pad, K, npat) * sizeof(float)) return LRS_E_WORKSPACE;
    const int NQ = pat_nq(K);
    const int NT = (int)(n_pad / 16);
    if ((int64_t)NT * NQ * 1024 >= ((int64_t)1 << 31)) return LRS_E_UNSUPPORTED;
    if (n > INT32_MAX / 2 || npat > 65535) return LRS_E_UNSUPPORTED;
    const float4 *DAf = reinterpret_cast<const float4 *>(ws);
    const float4 *DTf = DAf + (size_t)NT * NQ * 64;
    const float4 *QAf = DTf + (size_t)NT * NQ * 64;
    if (ntiles == 0) return LRS_OK;
    IstaPatParams p{Yb, obs_pat, plan, DAf, DTf, QAf, alpha, thr, coefs, phi, x0, (int)n_pad, (int)K, Nit, prox,
                    nb, ntiles, npat, 7.0};
    int waves = NQ >= 16 ? 8 : 4;
#ifdef LRS_TUNING
    if (const int kw = pat_waves_knob()) waves = kw;
#endif
    switch (NQ) {
    case 4: return launch_pat_k<4, 4>(p, max_wg, st);
    case 8: return launch_pat_k<8, 4>(p, max_wg, st);
    case 16:
        // 8 waves, registers unbounded (192, one workgroup per CU).  The 128-register bound (two
        // workgroups per CU; LRS_ISTA_PAT_WPE=4, tuning build) is bit-identical and a little faster
        // (configs[3]'s sparse coding 11.3 -> 10.6 ms, configs[2]'s beside the DIP 1.745 -> 1.683 ms;
        // the configs[2] bench 7.87 either way, profiles/r04/ista_pat_wpe/), but spills 37 registers
        // (152 B of scratch per lane, 29 with a 2-deep ring): the PMC pass then measured 1.26 GB of
        // fabric traffic per configs[2] launch instead of 122 MB (profiles/r04/ista_pat_spill/).
#ifdef LRS_TUNING
        if (waves == 8 && pat_wpe_knob() == 4) return launch_pat_k<16, 8, 4>(p, max_wg, st);
#endif
        return waves == 8 ? launch_pat_k<16, 8>(p, max_wg, st) : launch_pat_k<16, 4>(p, max_wg, st);
    default: return launch_pat_k<32, 8>(p, max_wg, st);
    }
}

}  // namespace lrs

// ---- C ABI --------------------------------------------------------------------------------------
extern "C" int64_t lrs_ista_pat_plan_len(int64_t nb, int64_t npat) {
    if (nb < 0 || npat < 1) return LRS_E_INVALID;
    return nb + 2 * ((nb + 15) / 16 + npat);
}

extern "C" int64_t lrs_ista_pat_plan(const int32_t *pat, int64_t nb, int64_t npat, int32_t *plan, int64_t cap) {
    if ((!pat && nb > 0) || !plan || nb < 0 || npat < 1 || npat > 65535 || nb > INT32_MAX) return LRS_E_INVALID;
    if (cap < lrs_ista_pat_plan_len(nb, npat)) return LRS_E_INVALID;
    std::vector<int64_t> count((size_t)npat + 1, 0);
    for (int64_t j = 0; j < nb; ++j) {
        if (pat[j] < 0 || pat[j] >= npat) return LRS_E_INVALID;
        ++count[(size_t)pat[j] + 1];
    }
    for (int64_t q = 0; q < npat; ++q) count[(size_t)q + 1] += count[(size_t)q];
    std::vector<int64_t> pos(count.begin(), count.end() - 1);
    for (int64_t j = 0; j < nb; ++j) plan[pos[(size_t)pat[j]]++] = (int32_t)j;   // stable: ascending j per pattern
    int64_t nt = 0;
    for (int64_t q = 0; q < npat; ++q)
        for (int64_t s = count[(size_t)q]; s < count[(size_t)q + 1]; s += 16) {
            const int64_t c = std::min<int64_t>(16, count[(size_t)q + 1] - s);
            plan[nb + 2 * nt] = (int32_t)s;
            plan[nb + 2 * nt + 1] = (int32_t)(q * 32 + c);
            ++nt;
        }
    return nt;
}

extern "C" int lrs_ista_pat_preferred(int64_t n, int64_t K, int64_t nb, int64_t npat, int Nit) {
    if (n <= 0 || K <= 0 || K > 512 || nb <= 0 || npat < 1 || Nit < 1) return 0;
    // matrix-core work per call (f64 Gram at half the f32 rate) against the row-split kernel's;
    // the prox is the same in both.  Half the row-split work at most: the Q stream and the tile
    // raggedness of many small patterns are not free.
    const double nd = (double)n, Kd = (double)K;
    const double pat = 2.0 * (2.0 * (double)npat * nd * Kd * Kd) + (double)nb * (4.0 * nd * Kd + (double)Nit * 2.0 * Kd * Kd);
    const double rs = (double)nb * (double)Nit * 4.0 * nd * Kd;
    return pat < 0.5 * rs ? 1 : 0;
}

extern "C" size_t lrs_ista_pat_workspace(int64_t n, int64_t K, int64_t npat) { return lrs::ista_pat_workspace(n, K, npat); }

extern "C" int lrs_ista_pat_prepare(const float *D, int64_t n, int64_t K, const uint8_t *obs_pat, int64_t npat,
                                    int64_t n_pad, void *ws, size_t ws_bytes, void *stream) {
    if (!D || !obs_pat || n <= 0 || K <= 0 || npat < 1) return LRS_E_INVALID;
    if (n_pad % 16 != 0 || n_pad < n || n_pad > (int64_t)1 << 20) return LRS_E_INVALID;
    return lrs::ista_pat_prepare(D, n, K, obs_pat, npat, n_pad, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int lrs_ista_pat_f32(const float *Yb, const uint8_t *obs_pat, int64_t npat, const int32_t *plan, int64_t ntiles,
                                int64_t n, int64_t n_pad, int64_t K, int64_t nb, const float *alpha, const double *thr,
                                int Nit, int prox, float *coefs, float *phi, const lrs_ista_opts *opts, void *ws,
                                size_t ws_bytes, void *stream) {
    if (!Yb || !obs_pat || !plan || !alpha || !thr || !phi || n <= 0 || nb < 0 || Nit < 0 || K <= 0 || npat < 1 ||
        ntiles < 0)
        return LRS_E_INVALID;
    if (n_pad % 16 != 0 || n_pad < n || n_pad > (int64_t)1 << 20 || nb > INT32_MAX) return LRS_E_INVALID;
    if (prox != LRS_PROX_NLM && prox != LRS_PROX_SOFT && prox != LRS_PROX_NLM_MATLAB) return LRS_E_INVALID;
    if (ntiles > (nb + 15) / 16 + npat) return LRS_E_INVALID;
    const int64_t max_wg = opts ? opts->max_workgroups : 0;
    if (max_wg < 0) return LRS_E_INVALID;
    if (opts && opts->precision != LRS_ISTA_F32 && opts->precision != LRS_ISTA_SPLIT_BF16) return LRS_E_INVALID;
    if (opts && opts->algorithm != LRS_ISTA_ALGO_AUTO) return LRS_E_INVALID;
    if (opts && opts->warm_start != 0 && opts->warm_start != 1) return LRS_E_INVALID;
    const bool warm = opts && opts->warm_start;
    if (warm && !coefs) return LRS_E_UNSUPPORTED;
    if (K > 512) return LRS_E_UNSUPPORTED;
    if (nb == 0) return LRS_OK;
    return lrs::ista_pat_launch(Yb, obs_pat, npat, plan, ntiles, n, n_pad, K, nb, alpha, thr, Nit, prox, coefs, phi, ws,
                                ws_bytes, max_wg, (hipStream_t)stream, warm ? coefs : nullptr);
}
