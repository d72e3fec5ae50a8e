"""Drop-in compat functions (reference names) and edge cases, on the GPU.

Tolerances: NLM <= 1 ulp vs skimage (bit-exact vs the oracle's closed form); ISTA / SVT / whole
outer iterations 1e-5 relative L2 vs the oracle or the reference's own outputs.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def compat():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lrspnp import compat as c
    return c


def test_compat_denoise_nl_means(compat, golden):
    z = golden("ista_golden.npz")
    for v in ("spec2", "fro4"):
        for a, h, o in zip(z[v + "_nlm_in"], z[v + "_nlm_h"], z[v + "_nlm_out"]):
            got = compat.denoise_nl_means(torch.from_numpy(a).view(-1, 1), h=h, fast_mode=True, patch_size=3,
                                          patch_distance=3)
            assert got.shape == o.shape and got.dtype == np.float32
            assert np.max(np.abs(got.view(np.int32).astype(np.int64) - o.view(np.int32))) <= 1
    with pytest.raises(NotImplementedError):
        compat.denoise_nl_means(np.zeros((8, 1), np.float32), h=0.1, patch_size=5, patch_distance=3)


def test_compat_ista_vs_reference(compat, golden):
    from lrspnp.data import synthetic_dictionary
    z = golden("ista_golden.npz")
    D = torch.from_numpy(synthetic_dictionary(1296, 256, 0))
    for v, fn in (("spec2", compat.ista_main), ("fro4", compat.ista_lip)):
        for i in range(z[v + "_y"].shape[0]):
            y = torch.from_numpy(z[v + "_y"][i]).view(-1, 1)
            miss = np.where(z[v + "_obs"][i] == 0)[0]
            yy = compat.delete_element(y, miss)
            H = compat.delete_element(D, miss)
            x = fn(yy, H, 0.1, 0, int(z[v + "_Nit"]))
            assert x.shape == (256, 1)
            assert rel(x.numpy().ravel(), z[v + "_coefs"][i]) < 1e-5


def test_compat_get_image_block_and_svt(compat):
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.standard_normal((103, 29)).astype(np.float32))
    blocks, r, c, idx = compat.get_image_block(X, 7, 7)
    ro, co = O.block_grid(103, 29, 7, 7)
    assert np.array_equal(r, ro) and np.array_equal(c, co)
    assert np.array_equal(blocks.numpy(), O.im2col(X.numpy(), 7, ro, co).T)
    assert int(idx.sum()) == r.size
    Z = (rng.random((400, 6)) @ rng.random((6, 50)) + 0.05 * rng.standard_normal((400, 50))).astype(np.float32)
    U = compat.SVT(torch.from_numpy(Z), 1 / 0.9)
    assert rel(U.numpy(), O.svt(Z, 1 / 0.9)) < 1e-5


@pytest.mark.parametrize("H,W,B,bb,sliding,variant", [
    (30, 20, 37, 8, 8, "spec2"),      # appended block row and column, odd B (padded Gram)
    (24, 24, 40, 5, 5, "fro4"),       # n = 25 -> n_pad = 32 (resident kernel, padded rows)
    (26, 18, 30, 12, 12, "spec2"),    # n = 144 -> streaming kernel, partial stage
    (20, 20, 24, 8, 4, "soft"),       # overlapping blocks (sliding < bb): up to 4 covers per axis
])
def test_solver_edge_shapes_vs_oracle(H, W, B, bb, sliding, variant):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    obs, clean, mask = synthetic_cube(H, W, B, seed=7)
    Y, M = unfold(obs), mask_matrix(mask, B)
    D = synthetic_dictionary(bb * bb, 256, 1)
    cfg = LrsPnPConfig(bb=bb, sliding=sliding, Nit=15, variant=variant)
    s = LrsPnP(Y, M, D, cfg)
    o = O.LrsPnpOracle(Y, M, D, bb=bb, sliding=sliding, Nit=15, variant=variant)
    for _ in range(2):
        s.step()
        o.step()
    torch.cuda.synchronize()
    assert rel(s.X.cpu().numpy(), o.X) < 1e-5
    assert rel(s.L1.cpu().numpy(), o.L1) < 1e-5
    assert rel(s.L2.cpu().numpy(), o.L2) < 1e-5


def test_fully_missing_block_gives_zero_code():
    """A block whose observed values are all zero: the reference divides by alpha = 0 (undefined);
    lrspnp defines alpha := 1 so the code stays 0 and Phi = 0 (documented in DESIGN.md)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lrspnp import ops
    from lrspnp.data import synthetic_dictionary
    D = torch.from_numpy(synthetic_dictionary(64, 256, 0)).cuda()
    nb = 130                                  # one partial workgroup
    rng = np.random.default_rng(1)
    Yb = (rng.standard_normal((nb, 64)) * 0.2).astype(np.float32)
    obs = np.ones((nb, 64), np.uint8)
    obs[5] = 0
    Yb[5] = 0
    obs_d = torch.from_numpy(obs).cuda()
    alpha, thr = ops.ista_alpha(D, obs_d, 64, ops.ALPHA_SPEC2, 0.1)
    assert alpha[5].item() == 1.0 and np.isfinite(alpha.cpu().numpy()).all()
    phi, coefs = ops.ista(torch.from_numpy(Yb).cuda(), obs_d, D, 64, alpha, thr, 10, ops.PROX_NLM, want_coefs=True)
    assert torch.all(coefs[5] == 0) and torch.all(phi[5] == 0)
    assert torch.isfinite(phi).all()
