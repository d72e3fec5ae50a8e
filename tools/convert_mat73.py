"""Convert a MAT v7.3 (HDF5) reference data file to .npz, every dataset stored exactly as
h5py returns it (the orientation the reference's h5py.File(path)[key] sees,
main_LRS_PnP.py:170-181).  Run once under a Python that has h5py (in the build container:
/opt/conda/bin/python3.9); lrspnp.matio.load_mat then reads the .npz beside the .mat.

    /opt/conda/bin/python3.9 tools/convert_mat73.py data/low_rank_sparsity_noisy_img5.mat [out.npz]
"""
import sys

import h5py
import numpy as np


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else src + ".npz"
    arrays = {}
    with h5py.File(src, "r") as f:
        for k in f.keys():
            if isinstance(f[k], h5py.Dataset):
                arrays[k] = np.asarray(f[k])
    np.savez_compressed(dst, **arrays)
    print(dst, {k: (v.shape, str(v.dtype)) for k, v in arrays.items()})


if __name__ == "__main__":
    main()
