"""Data formats (lrspnp.matio): MAT v5 via scipy, converted MAT v7.3 (.npz in
h5py orientation), the reference's cube orientation, the spectrum writer.  CPU only.

Pinned once against the reference's own files (in the build container): tools/convert_mat73.py on
data/low_rank_sparsity_noisy_img5.mat followed by matio.cube_from_h5 reproduces the committed
fixture tests/golden/data_img5.npz['noisy_img5'][0] bit for bit, and matio.load_mat on
data/fourth_mask.mat gives msk (1, 1, 36, 36) u8 whose [0, 0] is fixture['fourth_mask'].
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))

from lrspnp import matio  # noqa: E402
from lrspnp.data import load_fixture, unfold  # noqa: E402


def test_v5_roundtrip(tmp_path):
    scipy_io = pytest.importorskip("scipy.io")
    msk = (np.arange(36 * 36).reshape(1, 1, 36, 36) % 7 != 0).astype(np.uint8)
    p = str(tmp_path / "mask.mat")
    scipy_io.savemat(p, {"msk": msk})
    assert matio.mat_version(p) == "v5"
    d = matio.load_mat(p)
    assert list(d) == ["msk"]
    np.testing.assert_array_equal(d["msk"], msk)


def test_v73_header_and_npz_sidecar(tmp_path):
    # a MAT v7.3 file is HDF5 behind a 512-byte user block
    p = str(tmp_path / "cube.mat")
    with open(p, "wb") as f:
        f.write(b"MATLAB 7.3 MAT-file".ljust(512, b" ") + b"\x89HDF\r\n\x1a\n" + bytes(64))
    assert matio.mat_version(p) == "v7.3"
    h5 = np.random.default_rng(0).random((36, 36, 128, 1)).astype(np.float32)
    np.savez(p + ".npz", masked_image=h5)
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py importable: the stub file would be read by h5py")
    except ImportError:
        pass
    d = matio.load_mat(p)
    np.testing.assert_array_equal(d["masked_image"], h5)


def test_v73_without_converter_raises(tmp_path):
    p = str(tmp_path / "cube.mat")
    with open(p, "wb") as f:
        f.write(bytes(512) + b"\x89HDF\r\n\x1a\n")
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py importable")
    except ImportError:
        pass
    with pytest.raises(RuntimeError, match="convert_mat73"):
        matio.load_mat(p)


def test_cube_orientation_matches_reference_transpose():
    """cube_from_h5 is the reference's .transpose((-1, 2, 1, 0)) (main_LRS_PnP.py:174) and feeds
    the unfolding of :209 (lrspnp.data.unfold)."""
    fx = load_fixture("data_img5.npz")["noisy_img5"]          # (1, 128, 36, 36)
    h5 = np.ascontiguousarray(fx.transpose(3, 2, 1, 0))       # what h5py returns: (36, 36, 128, 1)
    cube = matio.cube_from_h5(h5)
    np.testing.assert_array_equal(cube, fx[0])
    Y = unfold(cube)
    # main_LRS_PnP.py:209: noisy.view(128, 36, 36).transpose(2, 1, 0).reshape(1296, 128)
    np.testing.assert_array_equal(Y, fx[0].transpose(2, 1, 0).reshape(36 * 36, 128))


def test_write_spectrum(tmp_path):
    X = np.random.default_rng(1).random((1296, 128)).astype(np.float32)
    p = matio.write_spectrum(str(tmp_path), "LRS-PnP", 3, X, pixel=100)
    assert p.endswith(os.path.join("spectrum", "LRS-PnP", "3.npy"))
    np.testing.assert_array_equal(np.load(p), X[100])
