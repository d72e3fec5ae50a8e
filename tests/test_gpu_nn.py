"""GPU: the nn.Module drop-ins (lrspnp.nn.my_Lipschitz_Unet / skip) driven exactly as get_DIP_out
drives the reference modules (main_LRS_PnP_DIP_1-LiP.py:214-238, main_LRS_PnP_DIP_pro.py:215-246):
torch.optim.Adam(net.parameters()), out = net(x), MSELoss on the masked images, loss.backward(),
opt.step().  Pinned to the reference modules' own outputs (tests/golden/dip_golden.npz,
skip_golden.npz: the reference nets run on the same seeded parameters) at the existing step-0
tolerances: output 1e-5, loss 1e-6, gradients 1e-4 of the fp64 restatement (U-Net).
"""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import dip_ref  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


def _inputs(seed):
    from gen_dip_golden import problem
    x, t, m = (torch.from_numpy(a) for a in problem(seed))
    return x[None].cuda(), t[None].cuda(), m.reshape(1, 1, *m.shape).cuda()


def test_lipschitz_unet_module_step_vs_reference(gpu, golden):
    from gen_dip_golden import flat_params
    from lrspnp.dip import lipschitz_unet_units
    from lrspnp.nn import my_Lipschitz_Unet
    gold = golden("dip_golden.npz")
    seed = int(gold["seed"])
    units = lipschitz_unet_units(128, 128, 128)
    flat = torch.from_numpy(flat_params(units, seed))
    net = my_Lipschitz_Unet(num_input_channels=128, num_output_channels=128, ln_lambda=1, pad="reflection").cuda()
    net.load_flat(flat)
    params = list(net.parameters())
    assert sum(p.numel() for p in params) == flat.numel()
    opt_z = torch.optim.Adam(net.parameters(), 0.1)
    mse = torch.nn.MSELoss()
    x, t, mask_bkg = _inputs(seed)
    opt_z.zero_grad()
    out = net(x)
    assert out.shape == (1, 128, 36, 36)
    sub = int(gold["sub"])
    assert rel(out.detach().reshape(-1)[::sub], torch.from_numpy(gold["out_sub"][0])) < 1e-5
    loss = mse(t * mask_bkg, out * mask_bkg)
    assert abs(float(loss.detach()) - gold["loss"][0]) < 1e-6 * gold["loss"][0]
    loss.backward()
    # gradients against the fp64 restatement from the same state
    p64 = flat.double().clone().requires_grad_(True)
    dip_ref.loss_fn(dip_ref.forward(p64, units, x[0].cpu().double()), t[0].cpu().double(),
                    mask_bkg.reshape(-1).cpu().double()).backward()
    g_r = p64.grad
    offs, _ = dip_ref.param_offsets(units, 128)
    gflat = torch.cat([p.grad.reshape(-1).cpu() for p in params])
    for i, u in enumerate(units):
        Wg, bg, gg, beg = dip_ref.views(gflat.double(), units, i, offs)
        Wr, br, gr, ber = dip_ref.views(g_r, units, i, offs)
        assert rel(Wg, Wr) < 1e-4, i
        if gg is not None:
            assert rel(gg, gr) < 1e-4 and rel(beg, ber) < 1e-4, i
    # torch's Adam moved the engine's own buffer: -lr * g / (|g| + eps) on the first step
    before = torch.cat([p.detach().reshape(-1).cpu() for p in params]).clone()
    opt_z.step()
    after = net._flat.cpu()
    expect = before.double() - 0.1 * gflat.double() / (gflat.double().abs() + 1e-8)
    assert float(((after.double() - expect).abs() > 1e-6).float().mean()) < 1e-4
    # the next forward reads the updated parameters
    out2 = net(x)
    assert torch.isfinite(out2).all() and rel(out2.detach(), out.detach()) > 1e-3


def test_lipschitz_unet_module_other_sizes(gpu):
    """One module, two image sizes (engines built lazily on the shared parameter buffer); the
    backward of an older forward raises."""
    from lrspnp._lib import LrsError
    from lrspnp.nn import my_Lipschitz_Unet
    net = my_Lipschitz_Unet(198, 198, 1)
    opt = torch.optim.Adam(net.parameters(), 0.1)
    for hw in (36, 52):
        x = torch.rand(1, 198, hw, hw, device="cuda")
        out = net(x)
        assert out.shape == (1, 198, hw, hw)
        opt.zero_grad()
        out.square().mean().backward()
        opt.step()
    o1 = net(x)
    net(x)
    with pytest.raises(LrsError):
        o1.sum().backward()


def test_skip_module_step_vs_reference(gpu, golden):
    from gen_dip_golden import flat_params
    from lrspnp.dip import skip_nodes
    from lrspnp.nn import skip
    gold = golden("skip_golden.npz")
    seed = int(gold["seed"])
    net = skip(128, 128, num_channels_down=[128] * 5, num_channels_up=[128] * 5, num_channels_skip=[128] * 5,
               filter_size_up=3, filter_size_down=3, upsample_mode="nearest", filter_skip_size=1,
               need_sigmoid=True, need_bias=True, pad="reflection", act_fun="LeakyReLU").cuda()
    net.load_flat(torch.from_numpy(flat_params(skip_nodes(128, 128), seed)))
    opt_z = torch.optim.Adam(net.parameters(), 0.1)
    mse = torch.nn.MSELoss()
    x, t, mask_bkg = _inputs(seed)
    out = net(x)
    sub = int(gold["sub"])
    assert rel(out.detach().reshape(-1)[::sub], torch.from_numpy(gold["out_sub"][0])) < 1e-5
    loss = mse(t * mask_bkg, out * mask_bkg)
    assert abs(float(loss.detach()) - gold["loss"][0]) < 1e-6 * gold["loss"][0]
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in net.parameters())
    opt_z.step()
    assert torch.isfinite(net(x)).all()
