"""nn.Module drop-ins for the reference's DIP networks, on the HIP engine.

    from lrspnp.nn import my_Lipschitz_Unet, skip       # models/my_Lipschitz_Unet.py:21, models/skip.py:5

    net = my_Lipschitz_Unet(num_input_channels=128, num_output_channels=128, ln_lambda=1,
                            pad='reflection').cuda()
    opt_z = torch.optim.Adam(net.parameters(), 0.1)     # …1-LiP.py:214-215, unchanged
    out = net(DIP_input)                                # (1, C, H, W) -> (1, C_out, H, W)
    loss = mse(DIP_target * mask_bkg, out * mask_bkg)
    loss.backward()                                     # parameter .grad from lrs_dipnet_backward
    opt_z.step()

The module's parameters are torch Parameters that alias one flat device buffer the engine reads
(conv weight_bar / bias, BN weight_orig / bias_orig, in node order), so torch's own optimizer
updates exactly what the next forward uses.  Forward and backward are single C-ABI calls
(lrs_dipnet_forward / lrs_dipnet_backward: sigma_max of every spectrally normalised conv, the BN
scale c = max(max|gamma|, 1), all layers); autograd sees the network as one Function.
Semantics kept from the reference: BatchNorm in training mode always (the scripts never call
.eval()), sigma and c treated as constants in the gradient (.data in
lipschitz_constraint_layer.py:41,96), no gradient with respect to the network input (the DIP
input is a fixed tensor).  The backward uses the activations of the module's most recent forward,
as in the reference loop (out = net(x); loss.backward()); calling it for an older forward raises.

There is no CPU path: constructing a module needs the HIP library and a gfx950 device.
"""
from __future__ import annotations

import torch

from ._lib import LrsError
from .dip import NODE_CONV, DipNet, lipschitz_unet_nodes, skip_nodes


class _DipFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        eng = module._engine_for(x.shape[-2], x.shape[-1])
        x3 = x.detach().reshape(x.shape[-3:]).to(torch.float32).contiguous()
        out = eng.forward(x3).clone()
        module._fwd_id += 1
        ctx.module, ctx.fwd_id, ctx.eng = module, module._fwd_id, eng
        ctx.save_for_backward(x3)
        return out.unsqueeze(0) if x.dim() == 4 else out

    @staticmethod
    def backward(ctx, gout):
        module, eng = ctx.module, ctx.eng
        if ctx.fwd_id != module._fwd_id:
            raise LrsError("lrspnp.nn: backward of an older forward (the engine keeps the last forward's "
                           "activations only)")
        (x3,) = ctx.saved_tensors
        eng.backward(x3, gout.reshape(eng.out_shape).to(torch.float32).contiguous())
        g = eng.grads
        grads = tuple(g[a:b].view(shape).clone() for (a, b, shape) in module._slices)
        return (None, None) + grads


class DipModule(torch.nn.Module):
    """A DIP network (lrspnp.dip node list) as an nn.Module with engine-backed forward/backward."""

    def __init__(self, nodes, in_channels: int, nominal_hw=(32, 32), seed: int = 0, ln_lambda: float = 1.0,
                 device="cuda"):
        super().__init__()
        self._nodes = list(nodes)
        self._c_in = int(in_channels)
        self._ln_lambda = float(ln_lambda)
        self._device = torch.device(device)
        # the parameter layout does not depend on H x W: a nominal-size engine defines it and
        # initialises the flat buffer; engines for real sizes are built lazily and bind that buffer
        base = DipNet(self._nodes, self._c_in, nominal_hw[0], nominal_hw[1], device=self._device)
        base.init_params(seed)
        torch.cuda.current_stream().wait_stream(base.stream)
        self._flat = base.params
        self._bnstats = base.bnstats
        self._engines = {tuple(nominal_hw): base}
        base.set_ln_lambda(self._ln_lambda)
        self._fwd_id = 0
        self._slices = []
        plist = []
        for i, nd in enumerate(self._nodes):
            w, b, g, be = base.param_views(i, self._flat)
            for kind, t in (("weight", w), ("bias", b), ("bn_weight", g), ("bn_bias", be)):
                if t is None:
                    continue
                a = t.storage_offset() - self._flat.storage_offset()
                self._slices.append((a, a + t.numel(), tuple(t.shape)))
                p = torch.nn.Parameter(t)          # aliases the flat buffer (same storage)
                self.register_parameter(f"n{i}_{kind}", p)
                plist.append(p)
        self._plist = plist

    # -- engines -----------------------------------------------------------------------------------
    def _engine_for(self, H: int, W: int) -> DipNet:
        key = (int(H), int(W))
        eng = self._engines.get(key)
        if eng is None:
            eng = DipNet(self._nodes, self._c_in, key[0], key[1], device=self._device, params=self._flat,
                         bnstats=self._bnstats)
            eng.set_ln_lambda(self._ln_lambda)
            self._engines[key] = eng
        return eng

    def forward(self, x):
        if x.dim() not in (3, 4) or (x.dim() == 4 and x.shape[0] != 1):
            raise LrsError("lrspnp.nn: input must be (1, C, H, W) or (C, H, W) (the reference's batch of one)")
        if x.shape[-3] != self._c_in:
            raise LrsError(f"lrspnp.nn: expected {self._c_in} input channels, got {x.shape[-3]}")
        if not x.is_cuda:
            raise LrsError("lrspnp.nn: input must be on the ROCm device (.cuda())")
        return _DipFunction.apply(x, self, *self._plist)

    # -- torch.nn.Module plumbing --------------------------------------------------------------------
    def cuda(self, device=None):
        return self          # already resident; keeps the parameters aliased to the engine buffer

    def to(self, *args, **kwargs):
        dev = kwargs.get("device", args[0] if args else None)
        if dev is not None and torch.device(dev).type != "cuda":
            raise LrsError("lrspnp.nn modules live on the ROCm device only")
        return self

    def _apply(self, fn, recurse=True):
        return self          # no re-allocation (float casts / moves would break the aliasing)

    def load_reference_state_dict(self, sd):
        """A my_Lipschitz_Unet state_dict of the reference module (weight_bar / bias / weight_orig /
        bias_orig names)."""
        self._engines[next(iter(self._engines))].load_reference_state_dict(sd)

    def load_flat(self, flat):
        """All parameters at once, in the engine's node order (tests / restarts)."""
        with torch.no_grad():
            self._flat.copy_(torch.as_tensor(flat, dtype=torch.float32).reshape(-1))

    def conv_weight_count(self) -> int:
        return sum(1 for nd in self._nodes if nd.kind == NODE_CONV)


def my_Lipschitz_Unet(num_input_channels=128, num_output_channels=128, ln_lambda=1, pad="reflection", seed=0):
    """models/my_Lipschitz_Unet.py:21-148: 14 spectrally normalised conv units (hidden 128), 1-Lipschitz
    BatchNorm, LeakyReLU(0.2); Kaiming-uniform weights (the engine's seeded RNG: the reference draws
    from the unseeded torch RNG).  The reference hard-codes 128 channels; other counts generalise the
    first and last conv."""
    if pad not in ("reflection", "zero"):
        raise LrsError(f"pad {pad!r}: reflection | zero")
    nodes = lipschitz_unet_nodes(int(num_input_channels), int(num_output_channels), 128, pad)
    return DipModule(nodes, int(num_input_channels), nominal_hw=(36, 36), seed=seed, ln_lambda=float(ln_lambda))


def skip(num_input_channels=2, num_output_channels=3, num_channels_down=(16, 32, 64, 128, 128),
         num_channels_up=(16, 32, 64, 128, 128), num_channels_skip=(4, 4, 4, 4, 4), filter_size_down=3,
         filter_size_up=3, filter_skip_size=1, need_sigmoid=True, need_bias=True, pad="zero",
         upsample_mode="nearest", downsample_mode="stride", act_fun="LeakyReLU", need1x1_up=True, seed=0):
    """models/skip.py:5-99 (called at main_LRS_PnP_DIP_pro.py:215-221): encoder-decoder with
    Concat skips, plain BatchNorm, LeakyReLU, optional Sigmoid head; the options the reference's
    scripts use (nearest upsampling, stride downsampling, LeakyReLU, biases) are supported."""
    if upsample_mode != "nearest" or downsample_mode != "stride" or act_fun != "LeakyReLU" or not need_bias:
        raise LrsError("lrspnp.nn.skip supports upsample_mode='nearest', downsample_mode='stride', "
                       "act_fun='LeakyReLU', need_bias=True (the reference's call)")
    if not (len(num_channels_down) == len(num_channels_up) == len(num_channels_skip)):
        raise LrsError("num_channels_down / _up / _skip must have the same length (skip.py:22)")
    if pad not in ("reflection", "zero"):
        raise LrsError(f"pad {pad!r}: reflection | zero")
    nodes = skip_nodes(int(num_input_channels), int(num_output_channels), tuple(num_channels_down),
                       tuple(num_channels_up), tuple(num_channels_skip), int(filter_size_down), int(filter_size_up),
                       int(filter_skip_size), pad, bool(need_sigmoid), bool(need1x1_up))
    n = len(num_channels_down)
    side = 2 ** (n + 1)          # the deepest map stays >= 2 (reflection pad 1)
    return DipModule(nodes, int(num_input_channels), nominal_hw=(side, side), seed=seed)
