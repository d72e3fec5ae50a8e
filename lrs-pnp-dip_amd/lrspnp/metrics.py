"""Quality metrics of the reference (not timed), on the device: per-band PSNR with its
10*log10(255/RMSE) definition and the band mean (main_LRS_PnP.py:40-58, :379-384) on the HIP kernel
lrs_psnr_bands_f32, and MSSIM (pytorch_ssim.ssim, main_LRS_PnP_DIP_1-LiP.py:480-481) on lrs_ssim_f32.
Nothing leaves the GPU but the final scalar."""
from __future__ import annotations

import torch


def fold(X: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """X (H*W, B), row p = i + H*j  ->  (B, H, W)."""
    B = X.shape[1]
    return X.reshape(W, H, B).permute(2, 1, 0)


def psnr_bands(X: torch.Tensor, clean_bhw: torch.Tensor) -> torch.Tensor:
    """Per-band PSNR (device float64 [B]) of the unfolded X (P x B) against clean (B, H, W)."""
    import ctypes

    from . import ops
    from ._lib import check, device_lib
    B, H, W = clean_bhw.shape
    C = ops.image_to_unfolded(clean_bhw.contiguous().float(), H, W)
    Xc = X.contiguous().float()
    L = device_lib()
    P = H * W
    ws = torch.empty(int(L.lrs_psnr_workspace(P, B)), dtype=torch.uint8, device=X.device)
    out = torch.empty(B, dtype=torch.float64, device=X.device)
    vp = ctypes.c_void_p
    check(L.lrs_psnr_bands_f32(vp(Xc.data_ptr()), vp(C.data_ptr()), P, B, vp(out.data_ptr()), vp(ws.data_ptr()),
                               ws.numel(), vp(torch.cuda.current_stream().cuda_stream)), "lrs_psnr_bands_f32")
    return out


def mpsnr(X: torch.Tensor, clean_bhw: torch.Tensor) -> float:
    return float(psnr_bands(X, clean_bhw).mean())


def mssim(img1: torch.Tensor, img2: torch.Tensor) -> float:
    """pytorch_ssim.ssim(img1, img2) for (B, H, W) (or (1, B, H, W)) float32 device images."""
    import ctypes

    from ._lib import check, device_lib
    a = img1.reshape(-1, *img1.shape[-2:]).contiguous().float()
    b = img2.reshape(-1, *img2.shape[-2:]).contiguous().float()
    C, H, W = a.shape
    acc = torch.zeros(1, dtype=torch.float64, device=a.device)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    check(device_lib().lrs_ssim_f32(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), C, H, W,
                                    ctypes.c_void_p(acc.data_ptr()), s), "lrs_ssim_f32")
    return float(acc) / (C * H * W)
