"""Tensor-level wrappers over the C ABI (include/lrspnp.h).

torch is only plumbing here: device memory, the current HIP stream, dtype/shape checks.  Every
arithmetic step runs in liblrspnp_hip.so; nothing falls back to torch/numpy compute.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as _libmod
from ._lib import (ALPHA_FRO4, ALPHA_SOFT, ALPHA_SPEC2, PROX_NLM, PROX_NLM_MATLAB, PROX_SOFT, LrsError, check,
                   device_lib, lib)

__all__ = ["nlm_col", "block_grid", "cover_ranges", "im2col", "ista_alpha", "ista", "svt_workspace",
           "ista_workspace", "ista_pat_plan", "ista_pat_preferred", "ista_pat_workspace", "ista_pat_prepare", "ista_pat", "nlm_matlab_col", "svt", "svt_gram", "svt_gram_view", "svt_finish", "admm_update", "unfolded_to_image", "image_to_unfolded", "ALPHA_SPEC2", "ALPHA_FRO4", "ALPHA_SOFT", "PROX_NLM", "PROX_SOFT",
           "PROX_NLM_MATLAB"]


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _s(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dev(t, dtype, name):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise LrsError(f"{name} must be a CUDA(ROCm) tensor")
    if t.dtype != dtype:
        raise LrsError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise LrsError(f"{name} must be contiguous")
    return t


# ---------------------------------------------------------------------------------------------
def nlm_col(g: torch.Tensor, h, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """NLM prox of every row of g (nvec, K): skimage denoise_nl_means(g_v[:,None], h, fast_mode=True,
    patch_size=3, patch_distance=3) per vector.  h: float or a float64 device tensor (nvec,)."""
    L = device_lib()
    g = _dev(g, torch.float32, "g")
    if g.dim() == 1:
        g2 = g.view(1, -1)
    else:
        g2 = g
    nvec, K = g2.shape
    o = torch.empty_like(g2) if out is None else _dev(out, torch.float32, "out").view(nvec, K)
    hv = None
    hs = 0.0
    if isinstance(h, torch.Tensor):
        hv = _dev(h, torch.float64, "h")
    else:
        hs = float(h)
    check(L.lrs_nlm_col_f32(_p(g2), K, _p(o), K, K, nvec, hs, _p(hv), 3, 3, _s(stream)), "lrs_nlm_col_f32")
    return o.view_as(g)


def block_grid(P: int, B: int, bb: int, sliding: int):
    """get_image_block corners (host int32 arrays), in the reference's order."""
    L = lib()
    nb = L.lrs_block_count(P, B, bb, sliding)
    if nb < 0:
        check(int(nb), "lrs_block_count")
    rows = np.empty(nb, np.int32)
    cols = np.empty(nb, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    check(L.lrs_block_grid(P, B, bb, sliding, rows.ctypes.data_as(i32p), cols.ctypes.data_as(i32p), nb),
          "lrs_block_grid")
    return rows, cols


def cover_ranges(extent: int, bb: int, starts: np.ndarray):
    L = lib()
    starts = np.ascontiguousarray(starts, np.int32)
    lo = np.empty(extent, np.int32)
    hi = np.empty(extent, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    check(L.lrs_cover_ranges(extent, bb, starts.ctypes.data_as(i32p), starts.size, lo.ctypes.data_as(i32p),
                             hi.ctypes.data_as(i32p)), "lrs_cover_ranges")
    return lo, hi


def im2col(X, Lm, mu: float, bb: int, rows_d, cols_d, n_pad: int, Yb=None, obs=None, want_obs=False,
           stream=None):
    """Yb[j] = block j of (X + Lm/mu) flattened F-order (get_image_block), zero-padded to n_pad."""
    L = device_lib()
    X = _dev(X, torch.float32, "X")
    if Lm is not None:
        _dev(Lm, torch.float32, "L")
    P, B = X.shape
    nb = rows_d.numel()
    if Yb is None:
        Yb = torch.empty((nb, n_pad), dtype=torch.float32, device=X.device)
    if want_obs and obs is None:
        obs = torch.empty((nb, n_pad), dtype=torch.uint8, device=X.device)
    check(L.lrs_im2col_f32(_p(X), _p(Lm), float(mu), P, B, bb, _p(rows_d), _p(cols_d), nb, n_pad, _p(Yb),
                           _p(obs) if want_obs else None, _s(stream)), "lrs_im2col_f32")
    return (Yb, obs) if want_obs else Yb


def ista_alpha(D, obs_pat, n: int, mode: int, lambda_ista: float, stream=None):
    L = device_lib()
    D = _dev(D, torch.float32, "D")
    obs_pat = _dev(obs_pat, torch.uint8, "obs_pat")
    nD, K = D.shape
    npat, n_pad = obs_pat.shape
    alpha = torch.empty(npat, dtype=torch.float32, device=D.device)
    thr = torch.empty(npat, dtype=torch.float64, device=D.device)
    wsb = L.lrs_ista_alpha_workspace(n, K, npat)
    ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=D.device)
    check(L.lrs_ista_alpha_f32(_p(D), n, K, _p(obs_pat), npat, n_pad, mode, float(lambda_ista), _p(alpha),
                               _p(thr), _p(ws), ws.numel(), _s(stream)), "lrs_ista_alpha_f32")
    return alpha, thr


def ista_workspace(n: int, K: int, prox: int, device, algorithm: int = 0) -> torch.Tensor | None:
    """Device workspace of lrs_ista_f32 (the row-split kernel's fragment-ordered dictionary images,
    or the generic path's chunk buffers for K > 512); None when the dictionary-resident kernels serve
    (n <= 64, K = 256, skimage / soft prox)."""
    opts = ctypes.byref(_libmod.ista_opts(algorithm=int(algorithm))) if algorithm else None
    nbytes = int(lib().lrs_ista_workspace(int(n), int(K), int(prox), opts))
    return torch.empty(nbytes, dtype=torch.uint8, device=device) if nbytes else None


def ista(Yb, obs, D, n: int, alpha, thr, Nit: int, prox: int = PROX_NLM, phi=None, coefs=None,
         want_coefs=False, ws=None, stream=None, precision: int | None = None, max_workgroups: int = 0,
         algorithm: int = 0, warm_start: bool = False):
    """Masked ISTA + prox over all blocks; returns phi (nb, n_pad) [, coefs (nb, K)].  `ws`: an
    ista_workspace() buffer (allocated here when None and needed).  precision / max_workgroups /
    algorithm / warm_start: this call's lrs_ista_opts (None / 0 = the library defaults; algorithm 1 =
    the generic dense-GEMM path that K > 512 always takes; warm_start: continue from `coefs`, which
    must be given, and write the result back to it)."""
    L = device_lib()
    _dev(Yb, torch.float32, "Yb")
    _dev(obs, torch.uint8, "obs")
    _dev(D, torch.float32, "D")
    _dev(alpha, torch.float32, "alpha")
    _dev(thr, torch.float64, "thr")
    nb, n_pad = Yb.shape
    K = D.shape[1]
    if phi is None:
        phi = torch.empty((nb, n_pad), dtype=torch.float32, device=Yb.device)
    if warm_start:
        if coefs is None:
            raise LrsError("ista(warm_start=True) continues from `coefs`: pass it")
        want_coefs = True
    if want_coefs and coefs is None:
        coefs = torch.empty((nb, K), dtype=torch.float32, device=Yb.device)
    if ws is None:
        ws = ista_workspace(n, K, prox, Yb.device, algorithm)
    opts = None
    if precision is not None or max_workgroups or algorithm or warm_start:
        opts = ctypes.byref(_libmod.ista_opts(_libmod.ISTA_SPLIT_BF16 if precision is None else int(precision),
                                              int(max_workgroups), int(algorithm), 1 if warm_start else 0))
    check(L.lrs_ista_f32(_p(Yb), _p(obs), _p(D), n, n_pad, K, nb, _p(alpha), _p(thr), int(Nit), int(prox),
                         _p(coefs) if want_coefs else None, _p(phi), opts, _p(ws), 0 if ws is None else ws.numel(),
                         _s(stream)), "lrs_ista_f32")
    return (phi, coefs) if want_coefs else phi


def ista_pat_plan(pat, npat: int):
    """Blocks grouped by observation pattern (lrs_ista_pat_plan, host): returns (plan int32 numpy
    array, ntiles).  pat: block j's pattern index in [0, npat) (host int32 array)."""
    L = lib()
    pat = np.ascontiguousarray(np.asarray(pat), dtype=np.int32)
    nb = pat.size
    cap = int(L.lrs_ista_pat_plan_len(nb, int(npat)))
    if cap < 0:
        check(cap, "lrs_ista_pat_plan_len")
    plan = np.zeros(cap, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    nt = int(L.lrs_ista_pat_plan(pat.ctypes.data_as(i32p), nb, int(npat), plan.ctypes.data_as(i32p), cap))
    if nt < 0:
        check(nt, "lrs_ista_pat_plan")
    return plan, nt


def ista_pat_preferred(n: int, K: int, nb: int, npat: int, Nit: int) -> bool:
    """Whether the per-pattern Gram path does less matrix-core work than the row-split kernel."""
    return bool(lib().lrs_ista_pat_preferred(int(n), int(K), int(nb), int(npat), int(Nit)))


def ista_pat_workspace(n: int, K: int, npat: int, device) -> torch.Tensor:
    return torch.empty(max(int(lib().lrs_ista_pat_workspace(int(n), int(K), int(npat))), 1), dtype=torch.uint8,
                       device=device)


def ista_pat_prepare(D, obs_pat, n: int, ws=None, stream=None) -> torch.Tensor:
    """The dictionary images and every pattern's masked Gram Q_p = D^T diag(m_p) D in `ws`
    (lrs_ista_pat_prepare; allocated here when None); returns ws, which ista_pat() then reads."""
    L = device_lib()
    _dev(D, torch.float32, "D")
    _dev(obs_pat, torch.uint8, "obs_pat")
    K = D.shape[1]
    npat, n_pad = obs_pat.shape
    if ws is None:
        ws = ista_pat_workspace(n, K, npat, D.device)
    check(L.lrs_ista_pat_prepare(_p(D), n, K, _p(obs_pat), npat, n_pad, _p(ws), ws.numel(), _s(stream)),
          "lrs_ista_pat_prepare")
    return ws


def ista_pat(Yb, obs_pat, plan, ntiles: int, K: int, n: int, alpha, thr, Nit: int, ws, prox: int = PROX_NLM,
             phi=None, coefs=None, want_coefs=False, stream=None, max_workgroups: int = 0, warm_start: bool = False):
    """Masked ISTA + prox on per-pattern Grams (lrs_ista_pat_f32) for blocks that share observation
    patterns, on the images ista_pat_prepare() left in `ws`.  obs_pat (npat, n_pad) u8 and plan
    (ista_pat_plan's, as an int32 device tensor) on the device; the rest as ista().  Returns
    phi [, coefs]."""
    L = device_lib()
    _dev(Yb, torch.float32, "Yb")
    _dev(obs_pat, torch.uint8, "obs_pat")
    _dev(plan, torch.int32, "plan")
    _dev(alpha, torch.float32, "alpha")
    _dev(thr, torch.float64, "thr")
    _dev(ws, torch.uint8, "ws")
    nb, n_pad = Yb.shape
    npat = obs_pat.shape[0]
    if phi is None:
        phi = torch.empty((nb, n_pad), dtype=torch.float32, device=Yb.device)
    if warm_start:
        if coefs is None:
            raise LrsError("ista_pat(warm_start=True) continues from `coefs`: pass it")
        want_coefs = True
    if want_coefs and coefs is None:
        coefs = torch.empty((nb, K), dtype=torch.float32, device=Yb.device)
    opts = None
    if max_workgroups or warm_start:
        opts = ctypes.byref(_libmod.ista_opts(_libmod.ISTA_SPLIT_BF16, int(max_workgroups), 0, 1 if warm_start else 0))
    check(L.lrs_ista_pat_f32(_p(Yb), _p(obs_pat), npat, _p(plan), int(ntiles), n, n_pad, int(K), nb, _p(alpha),
                             _p(thr), int(Nit), int(prox), _p(coefs) if want_coefs else None, _p(phi), opts, _p(ws),
                             ws.numel(), _s(stream)), "lrs_ista_pat_f32")
    return (phi, coefs) if want_coefs else phi


def nlm_matlab_col(g: torch.Tensor, h, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """NLmeansfilter(g_v, 3, 3, h) (LRS-PnP(Matlab Code)/NLmeansfilter.m) of every row of g (nvec, K)."""
    L = device_lib()
    g = _dev(g, torch.float32, "g")
    g2 = g.view(1, -1) if g.dim() == 1 else g
    nvec, K = g2.shape
    o = torch.empty_like(g2) if out is None else _dev(out, torch.float32, "out").view(nvec, K)
    hv, hs = (_dev(h, torch.float64, "h"), 0.0) if isinstance(h, torch.Tensor) else (None, float(h))
    check(L.lrs_nlm_matlab_col_f32(_p(g2), K, _p(o), K, K, nvec, hs, _p(hv), _s(stream)), "lrs_nlm_matlab_col_f32")
    return o.view_as(g)


def svt_workspace(P: int, B: int, device) -> torch.Tensor:
    n = int(lib().lrs_svt_workspace(P, B))
    return torch.zeros(n, dtype=torch.uint8, device=device)


SVT_WARM, SVT_JACOBI, SVT_MULTI_WG = 1, 2, 4   # include/lrspnp.h flag word of the svt calls


def _svt_flags(warm, method, multi_wg=False):
    if method not in ("tri", "jacobi"):
        raise LrsError(f"unknown SVT eigensolver {method!r} (tri | jacobi)")
    return (SVT_WARM if warm else 0) | (SVT_JACOBI if method == "jacobi" else 0) | (SVT_MULTI_WG if multi_wg else 0)


def svt(X, L2, c2: float, tau: float, ws, U=None, s_out=None, warm=False, stream=None, method="tri",
        multi_wg=False):
    """U = SVT(X + c2*L2, tau) (main_LRS_PnP.py:118-124).  method 'tri': tridiagonal eigensolver
    with a certified Jacobi fallback (default); 'jacobi': Jacobi only (warm-startable).  multi_wg:
    the tridiagonal solver's eigenvalue / eigenvector / back-transformation phases over many
    workgroups (LRS_SVT_MULTI_WG, bit-identical)."""
    L = device_lib()
    _dev(X, torch.float32, "X")
    if L2 is not None:
        _dev(L2, torch.float32, "L2")
    P, B = X.shape
    if U is None:
        U = torch.empty_like(X)
    check(L.lrs_svt_f32(_p(X), _p(L2), float(c2), P, B, float(tau), _p(U), _p(s_out),
                        _svt_flags(warm, method, multi_wg), _p(ws), ws.numel(), _s(stream)), "lrs_svt_f32")
    return U


def svt_gram(X, L2, c2: float, ws, warm=False, stream=None, method="tri"):
    """First half of svt(): fp64 Gram (+ the Jacobi warm-start product), multi-workgroup."""
    L = device_lib()
    P, B = X.shape
    check(L.lrs_svt_gram_f32(_p(X), _p(L2), float(c2), P, B, _svt_flags(warm, method), _p(ws), ws.numel(),
                             _s(stream)), "lrs_svt_gram_f32")


def svt_gram_view(ws, P: int, B: int) -> torch.Tensor:
    """The fp64 Gram (Bp x Bp, Bp = B rounded up to even) that svt_gram() leaves in `ws`, as a
    tensor view: a slab-sharded caller all-reduces it in place before svt_finish()."""
    off, ld = ctypes.c_int64(), ctypes.c_int64()
    check(lib().lrs_svt_gram_offset(P, B, ctypes.byref(off), ctypes.byref(ld)), "lrs_svt_gram_offset")
    n = ld.value * ld.value
    return ws[off.value: off.value + 8 * n].view(torch.float64).view(ld.value, ld.value)


def svt_finish(X, L2, c2: float, tau: float, ws, U, s_out=None, warm=False, stream=None, method="tri",
               multi_wg=False):
    """Second half of svt(): the eigensolver (one workgroup, or multi_wg), E, then U = Z - Z E."""
    L = device_lib()
    P, B = X.shape
    check(L.lrs_svt_finish_f32(_p(X), _p(L2), float(c2), P, B, float(tau), _p(U), _p(s_out),
                               _svt_flags(warm, method, multi_wg), _p(ws), ws.numel(), _s(stream)),
          "lrs_svt_finish_f32")
    return U


def svt_state(ws, P: int, B: int):
    """(V valid, V buffer, Jacobi rounds, sweeps, path, -, -, -) of the last SVT call, path 1 =
    tridiagonal, 2 = Jacobi fallback, 3 = Jacobi (diagnostics; syncs)."""
    out = (ctypes.c_int * 32)()
    check(device_lib().lrs_diag_svt_state(_p(ws), P, B, ctypes.cast(out, ctypes.c_void_p)), "lrs_diag_svt_state")
    return list(out)


def svt_phase_us(ws, P: int, B: int):
    """Phase durations (us) of the last tridiagonal-path solve: load+tridiagonalise, eigenvalues,
    inverse iteration, back-transformation, certificate/orthogonalisation, fallback+E (syncs)."""
    st = np.array(svt_state(ws, P, B), dtype=np.int32)
    t = st[16:32].view(np.uint64).astype(np.float64)
    return [(t[k + 1] - t[k]) / 100.0 for k in range(6)]


def admm_update(X, L1, L2, Y, M, U, phi, bb, grid, gamma, mu1, mu2, norms=None, imout=None, stream=None):
    """In-place col2im + X update + dual updates (main_LRS_PnP.py:324-362)."""
    L = device_lib()
    P, B = X.shape
    n_pad = phi.shape[1]
    check(L.lrs_admm_update_f32(_p(X), _p(L1), _p(L2), _p(Y), _p(M), _p(U), _p(phi), P, B, bb, n_pad,
                                _p(grid["rstarts"]), _p(grid["cstarts"]), grid["nbr"], _p(grid["rlo"]),
                                _p(grid["rhi"]), _p(grid["clo"]), _p(grid["chi"]), float(gamma), float(mu1),
                                float(mu2), _p(norms), _p(imout), _s(stream)), "lrs_admm_update_f32")


def unfolded_to_image(X, L, c: float, H: int, W: int, out=None, stream=None):
    """img[b][i][j] = X[i + H j][b] + c * L[...]   (…1-LiP.py:404 DIP_input layout)."""
    Ld = device_lib()
    _dev(X, torch.float32, "X")
    P, B = X.shape
    if P != H * W:
        raise LrsError(f"P = {P} != H*W = {H * W}")
    out = out if out is not None else torch.empty((B, H, W), dtype=torch.float32, device=X.device)
    check(Ld.lrs_unfolded_to_image_f32(_p(X), _p(L), ctypes.c_float(c), H, W, B, _p(out), _s(stream)),
          "lrs_unfolded_to_image_f32")
    return out


def image_to_unfolded(img, H: int, W: int, out=None, stream=None):
    """X[i + H j][b] = img[b][i][j]   (…1-LiP.py:411 U layout)."""
    Ld = device_lib()
    _dev(img, torch.float32, "img")
    B = img.numel() // (H * W)
    out = out if out is not None else torch.empty((H * W, B), dtype=torch.float32, device=img.device)
    check(Ld.lrs_image_to_unfolded_f32(_p(img), H, W, B, _p(out), _s(stream)), "lrs_image_to_unfolded_f32")
    return out
