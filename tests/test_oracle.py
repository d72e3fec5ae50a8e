"""The oracle pinned against the reference's own outputs (tests/golden/*, gen_golden.py).

* NLM: the 2-D integral-image restatement is bit-exact against scikit-image 0.18.3; the (K,1)
  closed form agrees bit-exactly except for rare 1-ulp cases (integral-image rounding).
* ISTA: oracle block ISTA vs the reference `ista` on real blocks, both variants.
* ADMM: two outer iterations of main_LRS_PnP.py reproduced to 1e-6 rel L2, MPSNR to 2 dp.
"""
import numpy as np
import pytest

from oracle import oracle as O
from lrspnp.data import synthetic_dictionary, unfold, mask_matrix


def _split(flat, sizes):
    out, o = [], 0
    for s in sizes:
        out.append(flat[o:o + s]); o += s
    return out


def test_fast_exp_known_values():
    assert O.lib().oracle_fast_exp(0.0) == pytest.approx(0.9710078, abs=1e-6)
    # Schraudolph: high word (int)(1512775.39.. * y) + 1072632447, truncation toward zero
    assert O.lib().oracle_fast_exp(-1.0) == pytest.approx(np.exp(-1.0), rel=0.07)


def test_nlm_2d_restatement_bit_exact(golden):
    z = golden("nlm_golden.npz")
    cols = _split(z["col_in"], z["col_K"])
    outs = _split(z["col_out"], z["col_K"])
    for g, h, ref in zip(cols, z["col_h"], outs):
        got = O.nlm_fast2d(g[:, None], h).reshape(-1)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (g.size, h)
    sizes = [int(a * b) for a, b, _ in z["img_shape_h"]]
    for (H, W, h), a, ref in zip(z["img_shape_h"], _split(z["img_in"], sizes), _split(z["img_out"], sizes)):
        got = O.nlm_fast2d(a.reshape(int(H), int(W)), h).reshape(-1)
        assert np.array_equal(got, ref)


def test_nlm_closed_form_vs_skimage(golden):
    z = golden("nlm_golden.npz")
    tot = bad = 0
    for g, h, ref in zip(_split(z["col_in"], z["col_K"]), z["col_h"], _split(z["col_out"], z["col_K"])):
        got = O.nlm_col(g, h)
        d = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert d.max() <= 1
        tot += g.size; bad += int((d != 0).sum())
    assert bad <= max(1, tot // 10000)
    for v in ("spec2", "fro4"):
        ista = golden("ista_golden.npz")
        for a, h, o in zip(ista[v + "_nlm_in"], ista[v + "_nlm_h"], ista[v + "_nlm_out"]):
            assert np.array_equal(O.nlm_col(a, h), o)


@pytest.mark.parametrize("variant", ["spec2", "fro4"])
def test_ista_block_vs_reference(golden, variant):
    z = golden("ista_golden.npz")
    D = synthetic_dictionary(1296, 256, 0)
    import hashlib
    assert hashlib.sha256(D.tobytes()).digest() == z["D_sha256"].tobytes()
    for i in range(z[variant + "_y"].shape[0]):
        y, ob = z[variant + "_y"][i], z[variant + "_obs"][i]
        a, t = O.ista_alpha_h(D[ob.astype(bool)], 0.1, variant)
        x, phi = O.ista_block(y, ob, D, a, t, int(z[variant + "_Nit"]))
        ref = z[variant + "_coefs"][i]
        assert np.linalg.norm(x - ref) / np.linalg.norm(ref) < 1e-6
        assert np.linalg.norm(phi - z[variant + "_phi"][i]) / np.linalg.norm(z[variant + "_phi"][i]) < 1e-6


def test_block_grid_counts():
    # SURVEY.md §8 block-count table
    for (P, B, bb, nb) in [(1296, 128, 36, 144), (40000, 198, 8, 125000), (40000, 198, 36, 6672),
                           (38416, 198, 36, 6408), (262144, 224, 36, 50974), (262144, 224, 8, 917504)]:
        r, c = O.block_grid(P, B, bb, bb)
        assert r.size == nb
    r, c = O.block_grid(1296, 128, 36, 36)
    assert list(c[:36]) == [0] * 36 and c[-1] == 92 and r[1] == 36   # F-order, appended column


def test_lrs_pnp_two_iterations_vs_reference(golden):
    d = golden("data_img5.npz")
    g = golden("lrs_pnp_2iter.npz")
    D = synthetic_dictionary(1296, 256, 0)
    Y = unfold(d["noisy_img5"][0])
    M = mask_matrix(d["fourth_mask"], 128)
    o = O.LrsPnpOracle(Y, M, D, bb=36, sliding=36, Nit=80, variant="spec2")
    rel = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
    o.step()
    assert rel(o.X, g["it1_X"]) < 1e-6 and rel(o.L1, g["it1_L1"]) < 1e-6 and rel(o.L2, g["it1_L2"]) < 2e-6
    assert rel(o.PHI, g["it1_PHI"]) < 1e-6
    p1 = O.psnr_bands(o.X, d["clean_img5"][0]).mean()
    o.step()
    assert rel(o.X, g["it2_X"]) < 1e-6
    p2 = O.psnr_bands(o.X, d["clean_img5"][0]).mean()
    assert round(p1, 2) == round(float(g["mpsnr"][0]), 2) and round(p2, 2) == round(float(g["mpsnr"][1]), 2)


def test_nlm_matlab_closed_form_vs_literal():
    """The MATLAB-variant prox (pnp_ista.m:30 -> NLmeansfilter.m): the oracle's C closed form for a
    (K,1) column against a literal, loop-for-loop transcription of NLmeansfilter.m (padarray
    'symmetric', make_kernel, sum(sum(.))).  No MATLAB/Octave here: this pins the restatement to
    the reference file's own algorithm, not to MATLAB's arithmetic."""
    rng = np.random.default_rng(0)
    for K, h in [(16, 0.05), (40, 0.01), (64, 0.2), (9, 1.0), (256, 0.02)]:
        g = (rng.standard_normal(K) * 0.1).astype(np.float32)
        closed = O.nlm_matlab_col(g, h)
        literal = O.nlm_matlab_literal(g.reshape(-1, 1).astype(np.float64), 3, 3, h).reshape(-1)
        np.testing.assert_allclose(closed, literal.astype(np.float32), rtol=2e-7, atol=1e-9)
        assert np.abs(closed - g).max() > 0      # the filter is not the identity at these h


def test_config0_oracle_vs_reference_first_iterations(golden):
    """BASELINE configs[0] as written (tests/golden/gen_golden.py cfg0: the reference's
    main_LRS_PnP.py run for 50 outer iterations on low_rank_sparsity_noisy.mat + fourth_mask.mat):
    the oracle's first two iterates (X to 1e-6 relative) and MPSNR of three iterations to 4 dp.
    (The GPU solver runs all 50 against the same golden in test_gpu_solver.py.)"""
    d = golden("data_img5.npz")
    g = golden("lrs_pnp_cfg0_50iter.npz")
    Y = unfold(d["noisy"][0])
    M = mask_matrix(d["fourth_mask"], 128)
    o = O.LrsPnpOracle(Y, M, synthetic_dictionary(1296, 256, 0), bb=36, sliding=36, Nit=80, variant="spec2")
    clean = d["clean"][0]
    for it in range(3):
        o.step()
        if it < 2:
            ref = g["X1"] if it == 0 else g["X2"]
            assert np.linalg.norm(o.X - ref) / np.linalg.norm(ref) < 1e-6
        assert abs(O.psnr_bands(o.X, clean).mean() - g["mpsnr"][it]) < 1e-4
