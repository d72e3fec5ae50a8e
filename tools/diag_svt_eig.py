"""Diagnostic: phase-by-phase check of the one-workgroup tridiagonal eigensolver against numpy
(eigenvalues of T vs eig(G), residual of W on T, orthogonality and residual of V on G)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np
import torch

from lrspnp import _lib, ops

L = _lib.device_lib()
f = L.lrs_diag_svt_eig
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
for (P, B, rank, noise) in [(1296, 128, 8, 0.12), (4000, 198, 8, 0.02), (777, 45, 5, 0.05)]:
    rng = np.random.default_rng(P + B)
    X = (rng.random((P, rank)) @ rng.random((rank, B)) * 0.3 + noise * rng.standard_normal((P, B))).astype(np.float32)
    Xd = torch.from_numpy(X).cuda()
    ws = ops.svt_workspace(P, B, "cuda")
    ops.svt_gram(Xd, None, 1.0, ws)
    Bp = B + (B & 1)
    out = np.zeros(3 * Bp + 3 * Bp * Bp)
    path = f(ctypes.c_void_p(ws.data_ptr()), P, B, out.ctypes.data_as(ctypes.c_void_p),
             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    d, e, lam = out[:Bp], out[Bp:2 * Bp], out[2 * Bp:3 * Bp]
    m = Bp * Bp
    W = out[3 * Bp:3 * Bp + m].reshape(Bp, Bp)
    V = out[3 * Bp + m:3 * Bp + 2 * m].reshape(Bp, Bp)
    S = out[3 * Bp + 2 * m:].reshape(Bp, Bp)
    G = np.zeros((Bp, Bp))
    G[:B, :B] = X.astype(np.float64).T @ X.astype(np.float64)
    T = np.diag(d) + np.diag(e[:-1], 1) + np.diag(e[:-1], -1)
    ev_G = np.linalg.eigvalsh(G)
    ev_T = np.linalg.eigvalsh(T)
    tn = np.abs(ev_G).max()
    print(f"P={P} B={B}: path {path}")
    print(f"  eig(T) vs eig(G): {np.abs(ev_T - ev_G).max() / tn:.2e} (rel to ||G||)")
    print(f"  lam vs eig(T):    {np.abs(np.sort(lam) - ev_T).max() / tn:.2e}, sorted {np.all(np.diff(lam) >= 0)}")
    rW = np.linalg.norm(T @ W - W * lam[None, :], axis=0) / tn
    print(f"  ||T w - lam w||/||T|| max {rW.max():.2e}, |W^T W - I| max {np.abs(W.T @ W - np.eye(Bp)).max():.2e}")
    rV = np.linalg.norm(G @ V - V * lam[None, :], axis=0) / tn
    print(f"  ||G v - lam v||/||G|| max {rV.max():.2e}, |V^T V - I| max {np.abs(V.T @ V - np.eye(Bp)).max():.2e}, "
          f"S vs V^T V {np.abs(S - V.T @ V).max():.2e}")
