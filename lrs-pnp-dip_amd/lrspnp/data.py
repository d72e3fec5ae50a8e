"""Input data: committed fixtures of the reference's data/*.mat, seeded synthetic dictionaries and
seeded synthetic hyperspectral cubes.

Layout conventions: a cube is held as img[b, i, j] (bands, rows, cols); the
solver works on the unfolded matrix X[p, b] with p = i + H*j (MATLAB column-major pixel order),
obtained by img.transpose(2, 1, 0).reshape(H*W, B) (main_LRS_PnP.py:209).
"""
from __future__ import annotations

import os

import numpy as np

FIXTURE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "tests", "golden")


def synthetic_dictionary(n: int, K: int, seed: int = 0) -> np.ndarray:
    """Seeded stand-in for the missing data/trained_dictionary.mat (.MISSING_LARGE_BLOBS:3).

    iid N(0,1) entries, columns L2-normalised (columnNormalise.m semantics), float32, n x K.
    """
    rng = np.random.default_rng(seed)
    D = rng.standard_normal((n, K))
    D /= np.sqrt((D * D).sum(axis=0, keepdims=True))
    return np.ascontiguousarray(D.astype(np.float32))


def unfold(img_bhw: np.ndarray) -> np.ndarray:
    """(B, H, W) cube -> X (H*W, B) with row p = i + H*j (main_LRS_PnP.py:209)."""
    B, H, W = img_bhw.shape
    return np.ascontiguousarray(np.asarray(img_bhw, np.float32).transpose(2, 1, 0).reshape(H * W, B))


def fold(X: np.ndarray, H: int, W: int) -> np.ndarray:
    """Inverse of unfold: X (H*W, B) -> (B, H, W)."""
    B = X.shape[1]
    return np.ascontiguousarray(np.asarray(X).reshape(W, H, B).transpose(2, 1, 0))


def mask_matrix(msk_hw: np.ndarray, B: int) -> np.ndarray:
    """M (H*W, B): the reference's mask replication (main_LRS_PnP.py:188-192).

    single_mask = msk.transpose((0,1,3,2)) flattened C-order and copied into every band column,
    i.e. row p = a*W + b holds msk[b, a]; with p = i + H*j that is msk[i, j] (square images).
    """
    m = np.asarray(msk_hw, np.float32)
    flat = m.T.reshape(-1)
    return np.ascontiguousarray(np.repeat(flat[:, None], B, axis=1))


def load_fixture(name: str) -> dict:
    path = os.path.join(FIXTURE_DIR, name)
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def synthetic_cube(H: int, W: int, B: int, seed: int = 0, rank: int = 8, noise_sigma: float = 0.12,
                   base_mask: np.ndarray | None = None):
    """Seeded synthetic low-rank HSI cube (SURVEY.md §8d "Synthetic inputs").

    clean = A S^T with `rank` endmembers: S[b,k] = 0.3 + 0.25 sin(2 pi f_k b / B + phi_k), A smooth
    non-negative abundances summing to 1, scaled to [0, 0.65]; noisy = clean + N(0, sigma^2);
    mask = `base_mask` (the 36x36 low_rank_sparsity_mask when given) tiled over H x W;
    observation = mask * noisy.  Returns (noisy_obs_bhw, clean_bhw, mask_hw) float32.
    """
    rng = np.random.default_rng(seed)
    b = np.arange(B)[:, None]
    f = rng.uniform(0.5, 3.0, rank)[None, :]
    ph = rng.uniform(0, 2 * np.pi, rank)[None, :]
    S = 0.3 + 0.25 * np.sin(2 * np.pi * f * b / B + ph)                 # B x r
    yy, xx = np.meshgrid(np.arange(H) / H, np.arange(W) / W, indexing="ij")
    A = np.empty((rank, H, W))
    for k in range(rank):
        cy, cx = rng.uniform(0, 1, 2)
        sy, sx = rng.uniform(0.15, 0.6, 2)
        A[k] = np.exp(-((yy - cy) ** 2) / (2 * sy * sy) - ((xx - cx) ** 2) / (2 * sx * sx))
    A /= A.sum(axis=0, keepdims=True)
    clean = np.einsum("br,rhw->bhw", S, A)
    clean *= 0.65 / clean.max()
    noisy = clean + rng.standard_normal(clean.shape) * noise_sigma
    if base_mask is None:
        mask = (rng.uniform(size=(H, W)) > 0.051).astype(np.float32)
    else:
        bm = np.asarray(base_mask, np.float32)
        reps = (-(-H // bm.shape[0]), -(-W // bm.shape[1]))
        mask = np.tile(bm, reps)[:H, :W]
    obs = (noisy * mask[None]).astype(np.float32)
    return obs, clean.astype(np.float32), mask.astype(np.float32)
