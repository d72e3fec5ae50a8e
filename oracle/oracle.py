"""ORACLE — TEST INFRASTRUCTURE ONLY (parity checker, never the product path).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.  It restates the reference's hot path on the CPU:

* ``block_grid``        get_image_block corner logic      main_LRS_PnP.py:73-107
* ``ista_alpha_h``      alpha / T / h of the two ``ista`` variants
                        main_LRS_PnP.py:134-146 (alpha=||H||_2^2, h=0.1T)
                        main_LRS_PnP_DIP_1-LiP.py:187-196 (alpha=4||H||_F^2, h=T)
* ``svt``               SVT / Shrinkage_Operator           main_LRS_PnP.py:112-124
* ``psnr_bands``        per-band PSNR, MPSNR               main_LRS_PnP.py:379-384
* ``LrsPnpOracle``      one outer ADMM iteration of main_LRS_PnP.py:250-362
* C restatements (``liblrs_oracle.so``, built from ``nlm_oracle.c`` + ``lrs_oracle.c``):
  NLM (skimage 0.18.3 ``_fast_nl_means_denoising_2d``), block ISTA, col2im + X/dual update.

Scalar types follow numpy >= 2 (NEP 50) promotion, the environment the golden fixtures were
generated in (tests/golden/gen_golden.py): alpha, T and h are float32.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblrs_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the C restatement (gcc, -ffp-contract=off, OpenMP)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        f32 = np.ctypeslib.ndpointer(np.float32, flags="C")
        f64 = np.ctypeslib.ndpointer(np.float64, flags="C")
        u8 = np.ctypeslib.ndpointer(np.uint8, flags="C")
        i64 = np.ctypeslib.ndpointer(np.int64, flags="C")
        c_long, c_int, c_double, c_float = ctypes.c_long, ctypes.c_int, ctypes.c_double, ctypes.c_float
        L.oracle_fast_exp.restype = c_double
        L.oracle_fast_exp.argtypes = [c_double]
        L.oracle_nlm_fast2d.restype = c_int
        L.oracle_nlm_fast2d.argtypes = [f32, c_int, c_int, c_int, c_int, c_int, c_double, c_double, f32]
        L.oracle_nlm_col.restype = None
        L.oracle_nlm_col.argtypes = [f32, c_long, c_long, c_double, f32, c_long]
        L.oracle_nlm_matlab_col.restype = None
        L.oracle_nlm_matlab_col.argtypes = [f32, c_long, c_long, c_double, f32, c_long]
        L.oracle_ista_block.restype = None
        L.oracle_ista_block.argtypes = [f32, u8, f32, c_long, c_long, c_float, c_double, c_int, c_int,
                                        f32, ctypes.c_void_p]
        L.oracle_ista_batch.restype = None
        L.oracle_ista_batch.argtypes = [f32, u8, f32, c_long, c_long, c_long, f32, f64, c_int, c_int,
                                        f32, ctypes.c_void_p]
        L.oracle_admm_update.restype = None
        L.oracle_admm_update.argtypes = [c_long, c_long, c_long, c_long, i64, i64, f32, f32, f32, f32,
                                         f32, f32, c_float, c_float, c_float, f32, f32, f32,
                                         ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_im2col.restype = None
        L.oracle_im2col.argtypes = [c_long, c_long, c_long, c_long, i64, i64, f32, f32]
        _lib = L
    return _lib


PROX_NLM, PROX_SOFT, PROX_NLM_MATLAB = 0, 1, 2


# --------------------------------------------------------------------------------------------
# NLM
# --------------------------------------------------------------------------------------------
def nlm_fast2d(img: np.ndarray, h: float, patch_size: int = 3, patch_distance: int = 3) -> np.ndarray:
    """skimage 0.18.3 denoise_nl_means(img, h, fast_mode=True, ...) for a 2-D float32 image."""
    a = np.ascontiguousarray(img, dtype=np.float32)
    if a.ndim == 2:
        a3 = a[..., None]
    else:
        a3 = a
    out = np.empty_like(a3)
    rc = lib().oracle_nlm_fast2d(np.ascontiguousarray(a3), a3.shape[0], a3.shape[1], a3.shape[2],
                                 patch_size, patch_distance, float(h), 0.0, out)
    assert rc == 0
    return np.squeeze(out)


def nlm_col(g: np.ndarray, h: float) -> np.ndarray:
    """Closed form of nlm_fast2d for a (K,1) column."""
    g = np.ascontiguousarray(g, dtype=np.float32).reshape(-1)
    out = np.empty_like(g)
    lib().oracle_nlm_col(g, g.size, 1, float(h), out, 1)
    return out


def nlm_matlab_col(g: np.ndarray, h: float) -> np.ndarray:
    """NLmeansfilter(g, 3, 3, h) for a (K,1) column, closed form in C (nlm_oracle.c)."""
    g = np.ascontiguousarray(g, dtype=np.float32).reshape(-1)
    out = np.empty_like(g)
    lib().oracle_nlm_matlab_col(g, g.size, 1, float(h), out, 1)
    return out


def nlm_matlab_literal(image: np.ndarray, t: int, f: int, h: float) -> np.ndarray:
    """Literal transcription of LRS-PnP(Matlab Code)/NLmeansfilter.m:1-91 (any m x n image,
    fp64, MATLAB's 1-based loops shifted by one, padarray 'symmetric', make_kernel, the
    sum(sum(.)) of column sums).  Slow: the pin of nlm_matlab_col on small inputs."""
    inp = np.asarray(image, dtype=np.float64)
    m, n = inp.shape
    input2 = np.pad(inp, f, mode="symmetric")                      # padarray(input,[f f],'symmetric')
    kernel = np.zeros((2 * f + 1, 2 * f + 1))                     # make_kernel(f)  :80-91
    for d in range(1, f + 1):
        value = 1.0 / (2 * d + 1) ** 2
        for i in range(-d, d + 1):
            for j in range(-d, d + 1):
                kernel[f - i, f - j] = kernel[f - i, f - j] + value
    kernel = kernel / f
    kernel = kernel / kernel.sum(axis=0).sum()                    # kernel / sum(sum(kernel))
    h = h * h
    out = np.zeros((m, n))
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            i1, j1 = i + f, j + f
            W1 = input2[i1 - f - 1:i1 + f, j1 - f - 1:j1 + f]
            wmax = average = sweight = 0.0
            for r in range(max(i1 - t, f + 1), min(i1 + t, m + f) + 1):
                for s_ in range(max(j1 - t, f + 1), min(j1 + t, n + f) + 1):
                    if r == i1 and s_ == j1:
                        continue
                    W2 = input2[r - f - 1:r + f, s_ - f - 1:s_ + f]
                    d = (kernel * (W1 - W2) * (W1 - W2)).sum(axis=0).sum()
                    w = np.exp(-d / h)
                    if w > wmax:
                        wmax = w
                    sweight = sweight + w
                    average = average + w * input2[r - 1, s_ - 1]
            average = average + wmax * input2[i1 - 1, j1 - 1]
            sweight = sweight + wmax
            out[i - 1, j - 1] = average / sweight if sweight > 0 else inp[i - 1, j - 1]
    return out


# --------------------------------------------------------------------------------------------
# Block grid (get_image_block)
# --------------------------------------------------------------------------------------------
def block_grid(P: int, B: int, bb: int, sliding: int):
    """Corner rows/cols of get_image_block (main_LRS_PnP.py:76-99), in the reference's order.

    idx_Mat[0:row+1:s, 0:col+1:s] = 1 plus the appended last row/column when P or B is not a
    multiple of bb; corners enumerated with np.argwhere on the F-flattened indicator.
    """
    nr, nc = P - bb + 1, B - bb + 1
    ind = np.zeros((nr, nc), dtype=bool)
    ind[0:nr + 1:sliding, 0:nc + 1:sliding] = True
    if B % bb != 0:
        ind[0:nr + 1:sliding, nc - 1] = True
    if P % bb != 0:
        ind[nr - 1, 0:nc + 1:sliding] = True
    if P % bb != 0 and B % bb != 0:
        ind[nr - 1, nc - 1] = True
    idx = np.argwhere(ind.flatten(order="F"))
    r, c = np.unravel_index(idx, ind.shape, order="F")
    return r.flatten().astype(np.int64), c.flatten().astype(np.int64)


def im2col(X: np.ndarray, bb: int, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.float32)
    out = np.empty((rows.size, bb * bb), np.float32)
    lib().oracle_im2col(X.shape[0], X.shape[1], bb, rows.size, rows, cols, X, out)
    return out


# --------------------------------------------------------------------------------------------
# ISTA step size / threshold (numpy, exactly the reference expressions)
# --------------------------------------------------------------------------------------------
def ista_alpha_h(H: np.ndarray, lambda_ista: float, variant: str):
    """Return (alpha, thr) as the reference computes them for pruned dictionary H.

    variant 'spec2' : main_LRS_PnP.py:134-146     alpha = ||H||_2^2, NLM h = 0.1*T
    variant 'fro4'  : …1-LiP.py:187-196            alpha = 2(tr(H^T H)+tr(H^T H)), h = T
    variant 'soft'  : ista.m:15-23                 alpha = ||H||_2^2, soft threshold T
    variant 'matlab': pnp_ista.m:16,30             alpha = max eig(H^T H), NLmeansfilter h = 0.1*T
    """
    H = np.asarray(H, dtype=np.float32)
    if H.shape[0] == 0:
        # no observed row: the reference divides by alpha = 0 (undefined); lrspnp's convention
        return np.float32(1.0), 1.0
    if variant in ("spec2", "soft", "matlab"):
        alpha = np.linalg.norm(H, 2) ** 2
    elif variant == "fro4":
        G = H.T @ H
        alpha = 2 * (np.trace(G) + np.trace(G))
    else:
        raise ValueError(variant)
    alpha = np.float32(alpha)
    T = np.float32(lambda_ista) / (np.float32(2) * alpha)
    if variant in ("spec2", "matlab"):      # pnp_ista.m:30 NLmeansfilter(., 3, 3, T*0.1)
        thr = T * np.float32(0.1)
    else:
        thr = T
    return np.float32(alpha), float(np.float32(thr))


def ista_block(y, obs, D, alpha, thr, Nit, prox=PROX_NLM):
    D = np.ascontiguousarray(D, dtype=np.float32)
    n, K = D.shape
    x = np.empty(K, np.float32)
    phi = np.empty(n, np.float32)
    lib().oracle_ista_block(np.ascontiguousarray(y, dtype=np.float32).reshape(-1),
                            np.ascontiguousarray(obs, dtype=np.uint8).reshape(-1), D, n, K,
                            float(alpha), float(thr), int(Nit), int(prox), x,
                            phi.ctypes.data_as(ctypes.c_void_p))
    return x, phi


def ista_batch(Yb, OBS, D, alpha, thr, Nit, prox=PROX_NLM):
    D = np.ascontiguousarray(D, dtype=np.float32)
    n, K = D.shape
    nb = Yb.shape[0]
    X = np.empty((nb, K), np.float32)
    PHI = np.empty((nb, n), np.float32)
    lib().oracle_ista_batch(np.ascontiguousarray(Yb, dtype=np.float32),
                            np.ascontiguousarray(OBS, dtype=np.uint8), D, n, K, nb,
                            np.ascontiguousarray(alpha, dtype=np.float32),
                            np.ascontiguousarray(thr, dtype=np.float64), int(Nit), int(prox), X,
                            PHI.ctypes.data_as(ctypes.c_void_p))
    return X, PHI


# --------------------------------------------------------------------------------------------
# SVT (numpy float32 LAPACK, the reference's own call)
# --------------------------------------------------------------------------------------------
def svt(X: np.ndarray, tau: float) -> np.ndarray:
    """SVT(X, tau) of main_LRS_PnP.py:118-124 (Shrinkage_Operator on diag(S), :112-116)."""
    U, S, V = np.linalg.svd(np.asarray(X, dtype=np.float32), full_matrices=False)
    Sd = np.diag(S)
    sh = np.sign(Sd) * np.maximum(np.abs(Sd) - tau, 0)
    return np.matmul(np.matmul(U, sh), V).astype(np.float32)


# --------------------------------------------------------------------------------------------
# Metrics (main_LRS_PnP.py:379-384; the reference's 10*log10(255/RMSE))
# --------------------------------------------------------------------------------------------
def psnr_bands(X: np.ndarray, clean_bhw: np.ndarray) -> np.ndarray:
    """Per-band PSNR of X (P x B, row p = i + H*j) against clean (B, H, W)."""
    B, H, W = clean_bhw.shape
    img = np.asarray(X, np.float64).reshape(W, H, B).transpose(2, 1, 0)  # [b, i, j]
    mse = ((img - clean_bhw.astype(np.float64)) ** 2).mean(axis=(1, 2))
    return 10.0 * np.log10(255.0 / np.sqrt(mse))


# --------------------------------------------------------------------------------------------
# One outer iteration of main_LRS_PnP.py (no DIP, SVT low-rank prox)
# --------------------------------------------------------------------------------------------
class LrsPnpOracle:
    """CPU restatement of the main_LRS_PnP.py outer loop (:244-362).

    Y: observed P x B (zeros at missing entries), M: mask P x B, D: n x K dictionary.
    """

    def __init__(self, Y, M, D, bb=36, sliding=36, gamma=0.5, mu1=0.15, mu2=0.15 * 6,
                 lambda_ista=0.1, Nit=80, variant="spec2", lowrank="svt"):
        self.Y = np.ascontiguousarray(Y, np.float32)
        self.M = np.ascontiguousarray(M, np.float32)
        self.D = np.ascontiguousarray(D, np.float32)
        self.P, self.B = self.Y.shape
        self.bb, self.sliding = bb, sliding
        self.gamma, self.mu1, self.mu2 = gamma, mu1, mu2
        self.Nit, self.variant = Nit, variant
        self.lowrank = lowrank
        self.prox = {"soft": PROX_SOFT, "matlab": PROX_NLM_MATLAB}.get(variant, PROX_NLM)
        self.rows, self.cols = block_grid(self.P, self.B, bb, sliding)
        self.nb = self.rows.size
        blocks_copy = im2col(self.Y, bb, self.rows, self.cols)       # :244
        self.obs = (blocks_copy != 0).astype(np.uint8)                # :278 missing = ==0
        self.alpha = np.empty(self.nb, np.float32)
        self.thr = np.empty(self.nb, np.float64)
        cache = {}
        for j in range(self.nb):
            key = self.obs[j].tobytes()
            if key not in cache:
                H = self.D[self.obs[j].astype(bool)]
                cache[key] = ista_alpha_h(H, lambda_ista, variant)
            self.alpha[j], self.thr[j] = cache[key]
        self.X = self.Y.copy()
        self.L1 = np.zeros_like(self.Y)
        self.L2 = np.zeros_like(self.Y)

    def step(self):
        f32 = np.float32
        mu1, mu2 = f32(self.mu1), f32(self.mu2)
        Xsc = self.X + self.L1 / mu1                                   # :259
        blocks = im2col(Xsc, self.bb, self.rows, self.cols)
        _, PHI = ista_batch(blocks, self.obs, self.D, self.alpha, self.thr, self.Nit, self.prox)
        Xlr = self.X + f32(1 / self.mu2) * self.L2                     # :315
        # low-rank prox: the SVT (:315), or a callable standing for the DIP mains' get_DIP_out on
        # (X + L2/mu2) (main_LRS_PnP_DIP_1-LiP.py:399-411; tests/golden/gen_dip196_traj.py)
        U = self.lowrank(Xlr) if callable(self.lowrank) else svt(Xlr, 1 / self.mu2)
        Xn, L1n, L2n = (np.empty_like(self.X) for _ in range(3))
        IM = np.empty_like(self.X)
        lib().oracle_admm_update(self.P, self.B, self.bb, self.nb, self.rows, self.cols,
                                 np.ascontiguousarray(PHI), self.Y, self.M, U, self.L1, self.L2,
                                 float(f32(self.gamma)), float(mu1), float(mu2), Xn, L1n, L2n,
                                 IM.ctypes.data_as(ctypes.c_void_p), None)
        self.U, self.IM, self.PHI = U, IM, PHI
        self.X, self.L1, self.L2 = Xn, L1n, L2n
        return Xn
