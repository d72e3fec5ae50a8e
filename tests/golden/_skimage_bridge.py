"""Fixture-generation helper, run ONLY in the build container under /opt/conda/bin/python3.9.

That interpreter carries the third-party arithmetic the reference depends on and which is not
vendored in /root/reference: scikit-image 0.18.3 (the NLM denoiser the reference calls inside
`ista`) and h5py 3.3.0 (MAT v7.3 input files).  System python (torch) drives the reference code
and talks to this process over stdin/stdout:

  request  : b'N' + <int32 H, W, patch, dist> + <float64 h> + H*W float32   -> H*W float32
             b'M' + <int32 len> + utf-8 path + <int32 len> + utf-8 key    -> npy bytes (v7.3 read)
             b'Q'                                                            -> exit
"""
import io
import struct
import sys
import warnings

warnings.filterwarnings("ignore")

import numpy as np  # noqa: E402


def main():
    from skimage.restoration import denoise_nl_means

    rd, wr = sys.stdin.buffer, sys.stdout.buffer
    while True:
        op = rd.read(1)
        if not op or op == b"Q":
            return
        if op == b"N":
            H, W, s, d = struct.unpack("<4i", rd.read(16))
            (h,) = struct.unpack("<d", rd.read(8))
            a = np.frombuffer(rd.read(4 * H * W), dtype=np.float32).reshape(H, W)
            out = denoise_nl_means(a, h=h, fast_mode=True, patch_size=s, patch_distance=d)
            out = np.ascontiguousarray(out, dtype=np.float32)
            wr.write(out.tobytes())
            wr.flush()
        elif op == b"M":
            import h5py

            (n,) = struct.unpack("<i", rd.read(4))
            path = rd.read(n).decode()
            (n,) = struct.unpack("<i", rd.read(4))
            key = rd.read(n).decode()
            with h5py.File(path, "r") as f:
                arr = np.array(f[key])
            buf = io.BytesIO()
            np.save(buf, arr, allow_pickle=False)
            b = buf.getvalue()
            wr.write(struct.pack("<q", len(b)))
            wr.write(b)
            wr.flush()
        else:
            raise SystemExit("bad op %r" % op)


if __name__ == "__main__":
    main()
