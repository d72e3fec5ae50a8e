"""Quality metrics of the reference (not timed): per-band PSNR with its 10*log10(255/RMSE)
definition and the band mean (main_LRS_PnP.py:40-58, :379-384)."""
from __future__ import annotations

import torch


def fold(X: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """X (H*W, B), row p = i + H*j  ->  (B, H, W)."""
    B = X.shape[1]
    return X.reshape(W, H, B).permute(2, 1, 0)


def psnr_bands(X: torch.Tensor, clean_bhw: torch.Tensor) -> torch.Tensor:
    B, H, W = clean_bhw.shape
    img = fold(X, H, W).double()
    mse = ((img - clean_bhw.double()) ** 2).mean(dim=(1, 2))
    return 10.0 * torch.log10(255.0 / torch.sqrt(mse))


def mpsnr(X: torch.Tensor, clean_bhw: torch.Tensor) -> float:
    return float(psnr_bands(X, clean_bhw).mean())
