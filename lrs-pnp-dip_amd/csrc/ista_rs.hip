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
#include <stdlib.h>

#include <algorithm>

#include "ista_prox.h"

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
    const float *x0;       // [nb][K] start coefficients (lrs_ista_opts.warm_start; may alias coefs) or null = 0
};

// LDS of one workgroup (floatx4 = 16 B units of [tile][lane]):
//   part  [NQ atom tiles][S-1 partial G images][64]     (S = 1: none)
//   xbuf  [NQ][64]            the coefficients x: B operand of every R_t, rewritten by the prox
//   gbuf  [16 blocks][NQ*16]  the gradient rows read by the prox (chunk index XOR-swizzled by block)
__host__ __device__ constexpr size_t rs_lds_bytes(int NQ, int S) { return (size_t)(S + 1) * NQ * 1024; }

// The observation term is split off the residual: D^T (m .* (y - D x)) = b - D^T (m .* D x) with
// b = D^T (m .* y) formed once per launch (each owner keeps its atom tiles of b in VGPRs), so the
// inner iterations never re-read y: per row tile they need D (L2), x (LDS) and 4 mask bits (VGPR).
template <int NQ, int MINW, int S>
__global__ __launch_bounds__(256, MINW) void k_ista_rs(IstaRsParams p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int KP = NQ * 16;
    constexpr int RING = 8;
    constexpr int NOWN = (NQ + S - 1) / S;       // atom tiles owned per wave (at most)
    constexpr int NMW = 4;                       // mask words: 8 row tiles each, in VGPRs
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row range in SGPRs
    const int jl = lane & 15, g = lane >> 4;
    floatx4 *part = reinterpret_cast<floatx4 *>(smem);                         // [NQ][S-1][64]
    floatx4 *xbuf = part + (size_t)(S - 1) * NQ * 64;                          // [NQ][64]
    float *gbuf = reinterpret_cast<float *>(xbuf + NQ * 64);                   // [16][KP]
    const int NT = p.n_pad >> 4;
    const int t0 = (NT * w) / S, t1 = (NT * (w + 1)) / S;
    const int K = p.K;
    const int64_t ntiles = (p.nb + 15) / 16;

    // persistent over column tiles when the grid is bounded (lrs_ista_opts.max_workgroups): each
    // tile is independent, so the results do not depend on the grid
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    if (tile != blockIdx.x) __syncthreads();   // the previous tile's last reads of xbuf / gbuf are done
    const int64_t j = tile * 16 + jl;
    const bool valid = j < p.nb;
    const float al = valid ? p.alpha[j] : 1.0f;
    const float ral = 1.0f / al;
    const double th = valid ? p.thr[j] : 1.0;
    const double c0 = nlm_c0();
    double krow[7];
    nlm_matlab_krow_d(krow);

    // x0 = 0, or the coefficients a previous launch left (warm start: the iteration continues exactly;
    // each workgroup reads and later writes only its own blocks' rows, so x0 may alias coefs)
    for (int i = threadIdx.x; i < NQ * 64; i += 64 * S) {
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        const int64_t jb = tile * 16 + (i & 15);
        const int a0 = 16 * (i >> 6) + 4 * ((i & 63) >> 4);
        if (p.x0 && jb < p.nb)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (a0 + e < K) v[e] = p.x0[jb * K + a0 + e];
        xbuf[i] = v;
    }

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
    auto mask4 = [&](int t) -> uint32_t {          // observed-row bits of rows 16t + 4g .. +3
        const uint32_t mv = valid ? *reinterpret_cast<const uint32_t *>(&p.obs[j * p.n_pad + 16 * t + 4 * g]) : 0u;
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) bits |= (((mv >> (8 * e)) & 0xffu) ? 1u : 0u) << e;
        return bits;
    };
    auto gq = [&](const floatx4 &G, float4 a, const float (&r)[4]) -> floatx4 {
        floatx4 acc = G;
        acc = mfma16x16x4(a.x, r[0], acc);
        acc = mfma16x16x4(a.y, r[1], acc);
        acc = mfma16x16x4(a.z, r[2], acc);
        acc = mfma16x16x4(a.w, r[3], acc);
        return acc;
    };

    // mask bits of this wave's row tiles (tile i: word i / 8, bits 4 (i % 8) .. +3); tiles beyond
    // 8 NMW per wave re-read theirs
    uint32_t ms[NMW];
#pragma unroll
    for (int v = 0; v < NMW; ++v) {
        ms[v] = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (8 * v + u < t1 - t0) ms[v] |= mask4(t0 + 8 * v + u) << (4 * u);
    }
    auto mbits = [&](int i) -> uint32_t {
        if (i >= 8 * NMW) return mask4(t0 + i);
        const uint32_t word = i < 8 ? ms[0] : i < 16 ? ms[1] : i < 24 ? ms[2] : ms[3];
        return (word >> (4 * (i & 7))) & 0xfu;
    };

    // ---- b = D^T (m .* y): partial over this wave's rows, reduced into the owners' VGPRs ----------
    floatx4 G[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) G[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int t = t0; t < t1; ++t) {
        const uint32_t m4 = mbits(t - t0);
        float4 yv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (valid) yv = *reinterpret_cast<const float4 *>(&p.Yb[j * p.n_pad + 16 * t + 4 * g]);
        const float r[4] = {(m4 & 1u) ? yv.x : 0.f, (m4 & 2u) ? yv.y : 0.f, (m4 & 4u) ? yv.z : 0.f,
                            (m4 & 8u) ? yv.w : 0.f};
#pragma unroll
        for (int q = 0; q < NQ; ++q) G[q] = gq(G[q], frag(t, NQ + q), r);
    }
    auto publish = [&]() {          // partials of the tiles this wave does not own
        if (S > 1) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int o = q % S;
                if (w != o) part[((size_t)q * (S - 1) + (w - (w > o))) * 64 + lane] = G[q];
            }
        }
        __syncthreads();
    };
    auto reduced = [&](int q, floatx4 acc) -> floatx4 {   // acc + sum over waves, fixed wave order
#pragma unroll
        for (int k = 0; k < S; ++k) {
            if (k == w) acc += G[q];
            else acc += part[((size_t)q * (S - 1) + (k - (k > w))) * 64 + lane];
        }
        return acc;
    };
    floatx4 bown[NOWN];
    publish();
#pragma unroll
    for (int q = 0; q < NQ; ++q)
        if (w == q % S) bown[q / S] = reduced(q, floatx4{0.f, 0.f, 0.f, 0.f});
    __syncthreads();

    // one row tile: R_t = D_t x (x from LDS), r_t = -m .* R_t, G += D_t^T r_t
    auto row_tile = [&](int t, float4 (&ring)[RING], uint32_t m4) {
        asm volatile("" ::: "memory");   // x is re-read from LDS per tile, not hoisted into 4 NQ VGPRs
        floatx4 RA = {0.f, 0.f, 0.f, 0.f}, RB = {0.f, 0.f, 0.f, 0.f};
        float r[4];
        float4 pend = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 2 * NQ; ++k) {
            const float4 a = ring[k % RING];
            const int kk = k + RING;
            if (kk < 2 * NQ) ring[k % RING] = frag(t, kk);
            else if (t + 1 < t1) ring[k % RING] = frag(t + 1, kk - 2 * NQ);
            if (k < NQ) {
                const floatx4 xv = xbuf[k * 64 + lane];
                floatx4 &acc = (k & 1) ? RB : RA;      // even / odd q on two accumulators (MFMA latency)
                acc = mfma16x16x4(a.x, xv[0], acc);
                acc = mfma16x16x4(a.y, xv[1], acc);
                acc = mfma16x16x4(a.z, xv[2], acc);
                acc = mfma16x16x4(a.w, xv[3], acc);
                if (k == NQ - 1) {
                    const floatx4 R = RA + RB;
#pragma unroll
                    for (int e = 0; e < 4; ++e) r[e] = ((m4 >> e) & 1u) ? -R[e] : 0.0f;
                }
            } else {
                const int q = k - NQ;             // q pairs interleaved (MFMA latency)
                if ((q & 1) == 0) {
                    pend = a;
                } else {
                    G[q - 1] = mfma16x16x4(pend.x, r[0], G[q - 1]);
                    G[q] = mfma16x16x4(a.x, r[0], G[q]);
                    G[q - 1] = mfma16x16x4(pend.y, r[1], G[q - 1]);
                    G[q] = mfma16x16x4(a.y, r[1], G[q]);
                    G[q - 1] = mfma16x16x4(pend.z, r[2], G[q - 1]);
                    G[q] = mfma16x16x4(a.z, r[2], G[q]);
                    G[q - 1] = mfma16x16x4(pend.w, r[3], G[q - 1]);
                    G[q] = mfma16x16x4(a.w, r[3], G[q]);
                }
            }
        }
    };

    for (int it = 0; it < p.Nit; ++it) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) G[q] = floatx4{0.f, 0.f, 0.f, 0.f};
        float4 ring[RING];
#pragma unroll
        for (int k = 0; k < RING; ++k) ring[k] = frag(t0, k);
        for (int t = t0; t < t1; ++t) row_tile(t, ring, mbits(t - t0));

        // ---- owner: G = b + sum_w G_w, g = x + G / alpha -> gbuf ----------------------------------
        publish();
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (w == q % S) {
                const floatx4 sum = reduced(q, bown[q / S]);
                const floatx4 xo = xbuf[q * 64 + lane];
                float4 gr;
                gr.x = xo[0] + rs_div(sum[0], al, ral);
                gr.y = xo[1] + rs_div(sum[1], al, ral);
                gr.z = xo[2] + rs_div(sum[2], al, ral);
                gr.w = xo[3] + rs_div(sum[3], al, ral);
                *reinterpret_cast<float4 *>(&gbuf[jl * KP + gsw(jl, 16 * q + 4 * g)]) = gr;
            }
        }
        __syncthreads();

        // ---- prox of the owned atom tiles (runtime loop: one inlined prox body) -> xbuf ----------
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
                prox_nlm_chunk(row, jl, a0, K, nlm_kneg(th), c0, p.seven, o);
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
            const float4 a = frag(t, q);
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
    for (int i = threadIdx.x; i < K; i += blockDim.x) out[v * ldo + i] = prox_nlm_matlab_point(col, 0, i, K, krow, hh * hh);
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
// capped by the rows (one row tile per wave at least) and by LDS (two workgroups per CU at MINW 2);
// S = 1 only when there is a single row tile (its owner would hold all of b in VGPRs).
static int rs_pick_waves(int64_t tiles, int NT, int NQ, int minw) {
    const int64_t simds = (int64_t)cu_count() * 4 * (minw >= 2 ? 2 : 1);
    int best = NT > 1 ? 2 : 1;
    double best_t = 1e30;
    for (int S = (NT > 1 ? 2 : 1); S <= 4 && S <= NT; ++S) {
        if (rs_lds_bytes(NQ, S) > (minw >= 2 ? 81920u : 163840u)) break;
        const double t = (double)((tiles * S + simds - 1) / simds) / S;
        if (t < best_t * 0.999) {
            best_t = t;
            best = S;
        }
    }
    return best;
}

template <int NQ, int MINW, int S>
static int launch_rs_k(const IstaRsParams &p, int64_t max_wg, hipStream_t st) {
    int64_t tiles = (p.nb + 15) / 16;
    if (max_wg > 0 && tiles > max_wg) tiles = max_wg;
    static std::atomic<uint64_t> opted{0};   // dynamic LDS beyond 64 KiB, per device
    if (const int rc = lds_opt_in((const void *)k_ista_rs<NQ, MINW, S>, 160 * 1024, opted)) return rc;
    size_t lds = rs_lds_bytes(NQ, S);
#ifdef LRS_TUNING
    // A/B only: LRS_ISTA_RS_LDS = dynamic LDS per workgroup (bytes, >= the kernel's), e.g. 98304 holds
    // the sparse coding to one workgroup per CU beside the DIP
    if (const char *e = getenv("LRS_ISTA_RS_LDS")) lds = std::max<size_t>(lds, (size_t)atoll(e));
#endif
    hipLaunchKernelGGL((k_ista_rs<NQ, MINW, S>), dim3((unsigned)tiles), dim3(64 * S), lds, st, p);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

template <int NQ, int MINW>
static int launch_rs(const IstaRsParams &p, int NT, int64_t max_wg, hipStream_t st) {
    const int64_t tiles = (p.nb + 15) / 16;
    switch (rs_pick_waves(tiles, NT, NQ, MINW)) {
    case 1: return launch_rs_k<NQ, MINW, 1>(p, max_wg, st);
    case 2: return launch_rs_k<NQ, MINW, 2>(p, max_wg, st);
    case 3: return launch_rs_k<NQ, MINW, 3>(p, max_wg, st);
    default: return launch_rs_k<NQ, MINW, 4>(p, max_wg, st);
    }
}

// the two fragment-ordered dictionary images (also used by the per-pattern Gram kernel, ista_pat.hip)
int ista_rs_images(const float *D, int64_t n, int64_t K, int NT, int NQ, float4 *DAf, float4 *DTf, hipStream_t st) {
    const int64_t total = (int64_t)NT * NQ * 64;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_ista_rs_prep, dim3(blocks), dim3(256), 0, st, D, (int)n, (int)K, NT, NQ, DAf, DTf);
    LRS_CHECK_LAUNCH();
    return LRS_OK;
}

int ista_rs_launch(const float *Yb, const uint8_t *obs, const float *D, int64_t n, int64_t n_pad, int64_t K, int64_t nb,
                   const float *alpha, const double *thr, int Nit, int prox, float *coefs, float *phi, void *ws,
                   size_t ws_bytes, int64_t max_wg, hipStream_t st, const float *x0) {
    if (K < 1 || K > 512) return LRS_E_UNSUPPORTED;
    const int NQ = rs_nq(K);
    const int NT = (int)(n_pad / 16);
    // the dictionary images are addressed by 32-bit buffer offsets (t * NQ + k) * 1024
    if ((int64_t)NT * NQ * 1024 >= ((int64_t)1 << 31)) return LRS_E_UNSUPPORTED;
    // the images have NT = n_pad / 16 row tiles: size the check from n_pad (ista_rs_workspace(n)
    // covers n_pad = round_up(n, 16); a larger n_pad needs lrs_ista_workspace(n_pad, ...))
    if (!ws || ws_bytes < ista_rs_workspace(n_pad, K)) return LRS_E_WORKSPACE;
    float4 *DAf = reinterpret_cast<float4 *>(ws);
    float4 *DTf = DAf + (size_t)NT * NQ * 64;
    {
        const int64_t total = (int64_t)NT * NQ * 64;
        const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
        hipLaunchKernelGGL(k_ista_rs_prep, dim3(blocks), dim3(256), 0, st, D, (int)n, (int)K, NT, NQ, DAf, DTf);
        LRS_CHECK_LAUNCH();
    }
    IstaRsParams p{Yb, obs, DAf, DTf, alpha, thr, coefs, phi, (int)n_pad, (int)K, Nit, prox, nb, 7.0, x0};
    switch (NQ) {
    case 4: return launch_rs<4, 2>(p, NT, max_wg, st);
    case 8: return launch_rs<8, 2>(p, NT, max_wg, st);
    case 16: return launch_rs<16, 2>(p, NT, max_wg, st);
    default: return launch_rs<32, 1>(p, NT, max_wg, st);
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
