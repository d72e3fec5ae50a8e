"""The C-ABI library (no GPU needed): builds, loads, exports every symbol include/lrspnp.h declares,
and its host-side entry points (block grid, cover ranges) agree with the oracle."""
import ctypes
import os
import re

import numpy as np

from lrspnp import _lib
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "lrspnp.h")).read()
    return sorted(set(re.findall(r"\b(lrs_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), n
    assert _lib.lib().lrs_version().startswith(b"lrspnp-hip")


def test_no_process_wide_mode():
    """reentrant, no global mutable state.  Every mode is a per-call option
    (lrs_ista_opts, lrs_dip_opts) or fixed per handle; the only setter takes a lrs_dipnet; the
    product library reads no environment variable (A/B knobs exist only in the tuning build)."""
    src = open(os.path.join(REPO, "include", "lrspnp.h")).read()
    setters = re.findall(r"int\s+(lrs_[a-z0-9_]*set_[a-z0-9_]*)\s*\(([^)]*)\)", src)
    assert setters, "expected the per-handle lrs_dipnet_set_ln_lambda"
    for name, args in setters:
        assert args.strip().startswith("lrs_dipnet *net"), name
    L = ctypes.CDLL(_lib.LIB_PATH)
    for gone in ("lrs_dip_set_precision", "lrs_dip_get_precision", "lrs_dip_set_upsample_dgrad",
                 "lrs_ista_set_precision", "lrs_ista_get_precision", "lrs_ista_set_rs_cols"):
        assert not hasattr(L, gone), gone
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    und = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert not re.search(r"\bgetenv\b", und), "the product library must not read the environment"


def test_block_grid_matches_oracle():
    from lrspnp import ops
    for (P, B, bb, s) in [(1296, 128, 36, 36), (40000, 198, 8, 8), (262144, 224, 36, 36), (103, 29, 7, 7),
                          (100, 40, 10, 5), (64, 64, 8, 3)]:
        r, c = ops.block_grid(P, B, bb, s)
        ro, co = O.block_grid(P, B, bb, s)
        assert np.array_equal(r, ro) and np.array_equal(c, co), (P, B, bb, s)


def test_cover_ranges():
    from lrspnp import ops
    for (P, bb, s) in [(1296, 36, 36), (103, 7, 7), (100, 10, 5), (64, 8, 3)]:
        r, _ = O.block_grid(P, bb, bb, s)  # B = bb: one block column
        starts = np.unique(r).astype(np.int32)
        lo, hi = ops.cover_ranges(P, bb, starts)
        for x in range(P):
            cov = [i for i, st in enumerate(starts) if st <= x < st + bb]
            assert cov == list(range(lo[x], hi[x] + 1)), (P, bb, s, x)


def test_invalid_arguments_rejected():
    L = _lib.lib()
    off, ld = ctypes.c_int64(), ctypes.c_int64()
    assert L.lrs_svt_gram_offset(4000, 198, ctypes.byref(off), ctypes.byref(ld)) == 0 and ld.value == 198
    # B <= 256: up to 198 bands the eigensolver's packed triangle is in LDS, above it in the workspace
    assert L.lrs_svt_gram_offset(4000, 199, ctypes.byref(off), ctypes.byref(ld)) == 0 and ld.value == 200
    assert L.lrs_svt_gram_offset(4000, 224, ctypes.byref(off), ctypes.byref(ld)) == 0 and ld.value == 224
    assert L.lrs_svt_gram_offset(4000, 256, ctypes.byref(off), ctypes.byref(ld)) == 0
    assert L.lrs_svt_gram_offset(4000, 257, ctypes.byref(off), ctypes.byref(ld)) == -2
    assert L.lrs_block_count(10, 10, 20, 20) < 0
    assert L.lrs_ista_f32(None, None, None, 64, 64, 256, 10, None, None, 10, 0, None, None, None, None, 0,
                          None) == -1
    assert L.lrs_nlm_col_f32(None, 0, None, 0, 0, 0, 0.0, None, 3, 3, None) == -1


def test_ista_pattern_plan():
    """lrs_ista_pat_plan (host): the blocks grouped by observation pattern, ascending within one,
    in tiles of at most 16 blocks of a single pattern; malformed pattern indices refused."""
    from lrspnp import ops
    rng = np.random.default_rng(5)
    for nb, npat in [(1, 1), (16, 1), (17, 1), (100, 7), (6408, 27), (513, 300)]:
        pat = rng.integers(0, npat, nb).astype(np.int32)
        plan, nt = ops.ista_pat_plan(pat, npat)
        order, tiles = plan[:nb], plan[nb:nb + 2 * nt].reshape(nt, 2)
        assert sorted(order.tolist()) == list(range(nb))
        seen = []
        for start, pc in tiles:
            p, c = pc >> 5, pc & 31
            assert 1 <= c <= 16
            blk = order[start:start + c]
            assert np.all(pat[blk] == p) and np.all(np.diff(blk) > 0)
            seen.extend(blk.tolist())
        assert sorted(seen) == list(range(nb))
        counts = np.bincount(pat, minlength=npat)
        assert nt == int(np.sum((counts + 15) // 16))
    L = _lib.lib()
    bad = np.array([0, 3], np.int32)
    out = np.zeros(64, np.int32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    assert L.lrs_ista_pat_plan(bad.ctypes.data_as(i32p), 2, 3, out.ctypes.data_as(i32p), 64) < 0
    assert L.lrs_ista_pat_plan(bad.ctypes.data_as(i32p), 2, 4, out.ctypes.data_as(i32p), 1) < 0


def test_ista_pattern_cost_model():
    """The per-pattern Gram path is chosen for the DIP mains' blocks (n = 1296, K = 256, 27 patterns
    for 6,408 blocks on the bench cube) and not when every block has its own pattern, nor for
    bb = 8 blocks (n = 64 < K / 2)."""
    from lrspnp import ops
    assert ops.ista_pat_preferred(1296, 256, 6408, 27, 100)
    assert ops.ista_pat_preferred(1296, 256, 50974, 24, 100)
    assert not ops.ista_pat_preferred(1296, 256, 6408, 6408, 100)
    assert not ops.ista_pat_preferred(64, 256, 125000, 40, 80)
    assert not ops.ista_pat_preferred(1296, 768, 6408, 27, 100)   # K > 512: the generic path


def test_workspace_sized_from_n_pad():
    """the sparse-coding images have n_pad / 16 row tiles, so a caller passing
    n_pad > round_up(n, 16) with the workspace sized for n is refused before anything is launched
    (host-side check: these calls never reach the device)."""
    L = _lib.lib()
    n, K, npat, nb = 1296, 256, 3, 48
    n_pad = (n + 15) // 16 * 16 + 16
    fake = ctypes.c_void_p(4096)   # never dereferenced: the size check comes first
    ws = L.lrs_ista_pat_workspace(n, K, npat)
    assert ws > 0
    assert L.lrs_ista_pat_prepare(fake, n, K, fake, npat, n_pad, fake, ws, None) == -3
    assert L.lrs_ista_pat_f32(fake, fake, npat, fake, 3, n, n_pad, K, nb, fake, fake, 10, 0, fake, fake, None,
                              fake, ws, None) == -3
    wr = L.lrs_ista_workspace(n, K, 0, None)
    assert wr > 0
    assert L.lrs_ista_f32(fake, fake, fake, n, n_pad, K, nb, fake, fake, 10, 0, fake, fake, None, fake, wr,
                          None) == -3
    # sized from n_pad instead, the same calls pass the check (then need a device: not called here)
    assert L.lrs_ista_pat_workspace(n_pad, K, npat) > ws and L.lrs_ista_workspace(n_pad, K, 0, None) > wr


def test_es_ring_bytes():
    """lrs_es_ring_bytes: the ring [size][N] floats (16-B aligned), then the fp64 window sums A [N], the
    workgroup partials (2 x kEsMaxBlocks doubles) and the window's sum of squares (+ one spare double);
    0 for a bad size."""
    L = _lib.lib()
    for size, N in [(30, 128 * 36 * 36), (30, 198 * 196 * 196), (7, 13)]:
        ring = (size * N * 4 + 15) // 16 * 16
        assert L.lrs_es_ring_bytes(size, N) == ring + N * 8 + (2 * 1024 + 2) * 8
    assert L.lrs_es_ring_bytes(0, 10) == 0 and L.lrs_es_ring_bytes(30, 0) == 0
