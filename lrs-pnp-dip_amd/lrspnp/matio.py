"""Data formats of the reference (SURVEY.md §5 checkpoint/IO, §8f item 2).

The reference loads its cubes and masks inline:

* MAT v5 files (``noisy.mat``, the ``*_mask.mat`` files, ``trained_dictionary.mat``) with
  ``scipy.io.loadmat`` (main_LRS_PnP.py:159,183);
* MAT v7.3 files (``clean*.mat``, ``noisy_img2..5.mat``: HDF5, gzip, 36x36x11 chunks) with
  ``h5py.File(path)[key]`` (main_LRS_PnP.py:170,177), whose arrays come out in HDF5 (C) order,
  (36, 36, 128, 1) for a cube, which the script turns into (1, 128, 36, 36) with
  ``.transpose((-1, 2, 1, 0))`` (:174,181).

h5py is not part of the runtime image, so v7.3 files are read through a one-off conversion to
``.npz`` (``tools/convert_mat73.py``, run wherever h5py exists) that stores every dataset exactly
as ``h5py`` returns it.  ``load_mat`` serves v5 files, converted ``.npz`` files and — when h5py is
importable — v7.3 files directly, always in the orientation the reference's own loader sees.

``write_spectrum`` writes the per-iteration recovered spectrum the way the reference's
results/spectrum/<method>/<iter>.npy files hold it (one float vector of B values per outer
iteration: the spectrum of one pixel).
"""
from __future__ import annotations

import os

import numpy as np

_HDF5_MAGIC = b"\x89HDF\r\n\x1a\n"


def mat_version(path: str) -> str:
    """'v5' (scipy.io.loadmat), 'v7.3' (HDF5, user block of 512 bytes) or 'npz'."""
    with open(path, "rb") as f:
        head = f.read(520)
    if head[:4] == b"PK\x03\x04":
        return "npz"
    if head[:8] == _HDF5_MAGIC or head[512:520] == _HDF5_MAGIC:
        return "v7.3"
    return "v5"


def _load_h5(path: str) -> dict:
    import h5py  # optional: absent from the runtime image
    out = {}
    with h5py.File(path, "r") as f:
        for k in f.keys():
            if isinstance(f[k], h5py.Dataset):
                out[k] = np.asarray(f[k])
    return out


def _load_npz(path: str) -> dict:
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_mat(path: str) -> dict:
    """Variables of a reference data file as {name: ndarray}.

    v5 via scipy.io.loadmat (MATLAB orientation, header entries dropped); v7.3 via h5py when it
    is importable, else the ``<path>.npz`` (or ``<stem>.npz``) written by tools/convert_mat73.py,
    both in h5py orientation — what the reference's ``h5py.File(path)[key]`` returns.
    """
    kind = mat_version(path)
    if kind == "npz":
        return _load_npz(path)
    if kind == "v5":
        import scipy.io
        d = scipy.io.loadmat(path)
        return {k: v for k, v in d.items() if not k.startswith("__")}
    try:
        return _load_h5(path)
    except ImportError:
        pass
    for cand in (path + ".npz", os.path.splitext(path)[0] + ".npz"):
        if os.path.exists(cand):
            return _load_npz(cand)
    raise RuntimeError(f"{path} is a MAT v7.3 (HDF5) file and h5py is not importable: convert it once with "
                       "tools/convert_mat73.py under a Python that has h5py and keep the .npz beside it")


def cube_from_h5(arr: np.ndarray) -> np.ndarray:
    """h5py-orientation cube (H', W', B, 1) -> (B, H, W) float32: the reference's
    ``.transpose((-1, 2, 1, 0))`` (main_LRS_PnP.py:174) without the leading batch axis."""
    a = np.asarray(arr, np.float32)
    if a.ndim == 3:
        a = a[..., None]
    return np.ascontiguousarray(a.transpose(3, 2, 1, 0)[0])


def write_spectrum(root: str, method: str, iteration: int, X: np.ndarray, pixel: int) -> str:
    """<root>/spectrum/<method>/<iteration>.npy: the B-band spectrum of unfolded row `pixel`."""
    d = os.path.join(root, "spectrum", method)
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{iteration}.npy")
    np.save(path, np.ascontiguousarray(np.asarray(X, np.float32)[pixel]))
    return path
