"""Drop-in replacements for the names the reference scripts resolve on the hot path.

A maintainer swaps the reference's imports / module-level defs for these:

    from lrspnp.compat import denoise_nl_means          # for skimage.restoration's
    from lrspnp.compat import get_image_block, delete_element, SVT
    from lrspnp.compat import ista_lip as ista          # main_LRS_PnP_DIP_{1-LiP,pro}.py:185-198
    from lrspnp.compat import ista_main as ista         # main_LRS_PnP.py:131-149

Same argument meaning, return types and shapes as the reference (CPU torch tensors / numpy
arrays in, same out), computed by liblrspnp_hip.so on the current ROCm device.  There is no CPU
fallback: every function raises LrsError when the HIP library or a gfx950 device is missing.

These are per-call (per-block) entry points for compatibility; the batched driver
(`lrspnp.LrsPnP`) is the fast path and does not call them.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from ._lib import LrsError

_DEV = "cuda"


def _as_f32_cpu(a) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        return a.detach().to("cpu", torch.float32).numpy()
    return np.asarray(a, dtype=np.float32)


# ----------------------------------------------------------------------------------------------
def denoise_nl_means(image, h=0.1, fast_mode=True, patch_size=7, patch_distance=11, multichannel=False,
                     sigma=0.0, preserve_range=None):
    """skimage.restoration.denoise_nl_means for what the reference passes: a (K,1) (or (K,)) float
    column, fast_mode=True, patch_size=3, patch_distance=3, sigma=0 (main_LRS_PnP.py:143-146,
    …1-LiP.py:192-196).  Returns float32 ndarray of shape (K,) like skimage's np.squeeze."""
    if not fast_mode or patch_size != 3 or patch_distance != 3 or sigma != 0.0:
        raise NotImplementedError("lrspnp implements the reference's call: fast_mode=True, patch_size=3, "
                                  "patch_distance=3, sigma=0")
    a = _as_f32_cpu(image)
    if a.ndim == 2 and a.shape[1] == 1:
        a = a[:, 0]
    if a.ndim != 1:
        raise NotImplementedError("lrspnp.compat.denoise_nl_means handles (K,1) columns")
    g = torch.from_numpy(np.ascontiguousarray(a)).to(_DEV)
    return ops.nlm_col(g, float(h)).cpu().numpy()


# ----------------------------------------------------------------------------------------------
def get_image_block(input_img, block_size, slidingDis):
    """get_image_block (main_LRS_PnP.py:73-107): (blocks [bb^2 x nb] CPU tensor, x_index, y_index,
    idx_Mat).  The gather runs on the GPU (lrs_im2col_f32)."""
    X = input_img if isinstance(input_img, torch.Tensor) else torch.as_tensor(np.asarray(input_img))
    P, B = X.shape
    bb = int(block_size)
    rows, cols = ops.block_grid(P, B, bb, int(slidingDis))
    Xd = X.detach().to(_DEV, torch.float32).contiguous()
    n = bb * bb
    n_pad = -(-n // 16) * 16
    Yb = ops.im2col(Xd, None, 1.0, bb, torch.from_numpy(rows).to(_DEV), torch.from_numpy(cols).to(_DEV), n_pad)
    blocks = Yb[:, :n].t().contiguous().cpu()
    idx_Mat = torch.zeros(P - bb + 1, B - bb + 1)
    idx_Mat[torch.from_numpy(rows.astype(np.int64)), torch.from_numpy(cols.astype(np.int64))] = 1
    return blocks, rows.astype(np.int64), cols.astype(np.int64), idx_Mat


def delete_element(tensor, indices):
    """delete_element (main_LRS_PnP.py:152-155): drop the listed rows (host-side bookkeeping)."""
    keep = torch.ones(tensor.size(0), dtype=torch.bool)
    keep[torch.as_tensor(np.asarray(indices, dtype=np.int64))] = False
    return tensor[keep].reshape(-1, tensor.size(1))


# ----------------------------------------------------------------------------------------------
def _ista(y, H, lambda_ista, Nit, mode, prox):
    Hn = _as_f32_cpu(H)
    m, K = Hn.shape
    if K > 4096:       # the alpha kernel's LDS bound; K > 512 runs the generic dense-GEMM ISTA path
        raise LrsError(f"lrspnp's ISTA takes K <= 4096 atoms, got {K}")
    yn = _as_f32_cpu(y).reshape(-1)
    if yn.size != m:
        raise ValueError(f"y has {yn.size} rows, H has {m}")
    m_pad = max(16, -(-m // 16) * 16)
    D = torch.from_numpy(np.ascontiguousarray(Hn)).to(_DEV)
    obs = np.zeros((1, m_pad), np.uint8)
    obs[0, :m] = 1
    Yb = np.zeros((1, m_pad), np.float32)
    Yb[0, :m] = yn
    obs_d = torch.from_numpy(obs).to(_DEV)
    alpha, thr = ops.ista_alpha(D, obs_d, m, mode, lambda_ista)
    phi, coefs = ops.ista(torch.from_numpy(Yb).to(_DEV), obs_d, D, m, alpha, thr, int(Nit), prox, want_coefs=True)
    return coefs.view(-1, 1).cpu()


def ista_main(y, H, lambda_ista, alpha, Nit):
    """ista() of main_LRS_PnP.py:131-149: alpha = ||H||_2^2, NLM h = 0.1*T (the `alpha` argument is
    ignored, as in the reference).  Returns the K x 1 coefficient tensor (CPU)."""
    return _ista(y, H, lambda_ista, Nit, ops.ALPHA_SPEC2, ops.PROX_NLM)


def ista_lip(y, H, lambda_ista, alpha, Nit):
    """ista() of main_LRS_PnP_DIP_1-LiP.py:185-198 / …pro.py:188-201: alpha = 4||H||_F^2, h = T."""
    return _ista(y, H, lambda_ista, Nit, ops.ALPHA_FRO4, ops.PROX_NLM)


def pnp_ista(y, H, lambda_ista, alpha, Nit, noise_sigma=None):
    """pnp_ista.m (LRS-PnP Matlab Code/pnp_ista.m:1-32): alpha = max eig(H^T H) (= ||H||_2^2, the
    value main_LRS_PnP.m passes), T = lambda/(2 alpha), x = NLmeansfilter(gradient, 3, 3, 0.1 T)
    (NLmeansfilter.m).  The returned J (objective) of the MATLAB function is not computed."""
    return _ista(y, H, lambda_ista, Nit, ops.ALPHA_SPEC2, ops.PROX_NLM_MATLAB)


def ista_soft(y, H, lambda_ista, alpha, Nit):
    """ista.m (LRS-PnP Matlab Code/ista.m:1-24): alpha = norm(H)^2, soft threshold T."""
    return _ista(y, H, lambda_ista, Nit, ops.ALPHA_SOFT, ops.PROX_SOFT)


ista = ista_lip


# ----------------------------------------------------------------------------------------------
def SVT(X, tau):
    """SVT (main_LRS_PnP.py:118-124): U S' V with S' = max(S - tau, 0).  Returns a CPU tensor."""
    Xd = (X if isinstance(X, torch.Tensor) else torch.as_tensor(np.asarray(X))).detach().to(_DEV, torch.float32)
    Xd = Xd.contiguous()
    P, B = Xd.shape
    ws = ops.svt_workspace(P, B, Xd.device)
    return ops.svt(Xd, None, 0.0, float(np.float32(tau)), ws).cpu()   # numpy applies tau in float32
