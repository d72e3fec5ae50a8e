"""DIP low-rank prox: the 1-Lipschitz U-Net and its training loop on the HIP engine.

Reference (shuoli0708/LRS-PnP-DIP):
  models/my_Lipschitz_Unet.py:21-148           my_Lipschitz_Unet (conv / bn / act stack)
  models/lipschitz_constraint_layer.py:36-44   SpectralNorm (exact sigma_max, W_bar / max(1, sigma))
  lipschitz_constraint_layer.py:65-78          conv(): ReflectionPad2d((k-1)//2) + Conv2d(pad 0),
                                               kaiming_uniform_(a=0, fan_in)
  lipschitz_constraint_layer.py:88-122         BatchNormSpectralNorm (gamma/c, beta/c)
  main_LRS_PnP_DIP_1-LiP.py:71-103             EarlyStop, myMetric
  main_LRS_PnP_DIP_1-LiP.py:208-264            get_DIP_out: fresh net, Adam(lr), masked MSE, ES
  main_LRS_PnP_DIP_1-LiP.py:404-411            DIP_input / U layout transforms

Every layer runs in liblrspnp_hip.so (lrs_dipnet_*): explicit im2col + MFMA GEMMs, fused
BN + LeakyReLU, an exact fp64 sigma_max per conv, Adam, the masked MSE and the early-stopping
test, all on device; one training step is optionally a single hipGraph launch.  There is no
PyTorch compute here: torch only allocates the device buffers.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

PAD_ZERO, PAD_REFLECT = 0, 1
ACT_NONE, ACT_LRELU, ACT_SIGMOID = 0, 1, 2


class ConvUnit(ctypes.Structure):
    """lrs_conv_unit: [upsample x2] -> pad -> conv(k, stride) -> [BN_lip] -> act."""
    _fields_ = [(n, ctypes.c_int32) for n in
                ("cin", "cout", "k", "stride", "pad", "pad_mode", "upsample", "bn", "act")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class EsState(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int32), ("size", ctypes.c_int32), ("patience", ctypes.c_int32),
                ("wait", ctypes.c_int32), ("stop", ctypes.c_int32), ("stop_epoch", ctypes.c_int32),
                ("best_epoch", ctypes.c_int32), ("reserved", ctypes.c_int32), ("best", ctypes.c_double),
                ("var_acc", ctypes.c_double), ("last_var", ctypes.c_double)]


def lipschitz_unet_units(c_in: int = 128, c_out: int = 128, hidden: int = 128,
                         pad: str = "reflection") -> list[ConvUnit]:
    """The 14 conv units of my_Lipschitz_Unet (my_Lipschitz_Unet.py:31-103).

    The reference hard-codes 128 everywhere; c_in / c_out generalise the first / last conv to
    other band counts (hidden stays 128), as SURVEY.md §8 a8 sizes the 196x196x198 config."""
    pm = PAD_REFLECT if pad == "reflection" else PAD_ZERO

    def u(cin, cout, k, stride=1, up=0, bn=1, act=ACT_LRELU):
        return ConvUnit(cin, cout, k, stride, (k - 1) // 2, pm, up, bn, act)

    h = hidden
    units = [u(c_in, h, 3, 2), u(h, h, 3)]                      # d_1  (:31-39)
    for _ in range(3):                                          # d_2..d_4 (:40-66)
        units += [u(h, h, 3, 2), u(h, h, 3)]
    units += [u(h, h, 2, up=1), u(h, h, 2, up=1)]               # up_1, up_2 (:71-82)
    units += [u(h, h, 3, up=1), u(h, h, 3, up=1)]               # up_3, up_4 (:83-94)
    units += [u(h, h, 1), u(h, c_out, 1, bn=0)]                 # last (:96-103)
    return units


# reference state_dict prefixes of each unit's conv / bn (named_parameters of my_Lipschitz_Unet)
UNET_REF_NAMES = (
    [("d_%d.0.1.module" % i, "d_%d.1" % i) if j == 0 else ("d_%d.3.1.module" % i, "d_%d.4" % i)
     for i in range(1, 5) for j in range(2)]
    + [("up_%d.1.1.module" % i, "up_%d.2" % i) for i in range(1, 5)]
    + [("last.0.1.module", "last.1"), ("last.3.1.module", None)]
)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _check(rc, what):
    if rc != 0:
        raise _lib.LrsError(f"{what} failed: {_lib.LRS_E.get(rc, rc)}")


class DipNet:
    """A sequential conv net on the HIP engine (lrs_dipnet_*), with flat parameter buffers."""

    def __init__(self, units: list[ConvUnit], H: int, W: int, device="cuda"):
        import torch

        self.L = _lib.device_lib()
        self.units = list(units)
        arr = (ConvUnit * len(units))(*units)
        h = ctypes.c_void_p()
        _check(self.L.lrs_dipnet_create(arr, len(units), H, W, ctypes.byref(h)), "lrs_dipnet_create")
        self.h = h
        self.H, self.W = H, W
        self.n_params = int(self.L.lrs_dipnet_num_params(h))
        nbs = int(self.L.lrs_dipnet_num_bnstats(h))
        ws = int(self.L.lrs_dipnet_workspace(h))
        f32 = dict(dtype=torch.float32, device=device)
        self.params = torch.zeros(self.n_params, **f32)
        self.grads = torch.zeros(self.n_params, **f32)
        self.exp_avg = torch.zeros(self.n_params, **f32)
        self.exp_avg_sq = torch.zeros(self.n_params, **f32)
        self.bnstats = torch.zeros(max(nbs, 1), **f32)
        self.ws = torch.zeros(ws, dtype=torch.uint8, device=device)
        _check(self.L.lrs_dipnet_bind(h, _ptr(self.params), _ptr(self.grads), _ptr(self.exp_avg),
                                      _ptr(self.exp_avg_sq), _ptr(self.bnstats), _ptr(self.ws), ws),
               "lrs_dipnet_bind")
        c, ho, wo = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.lrs_dipnet_out_shape(h, ctypes.byref(c), ctypes.byref(ho), ctypes.byref(wo))
        self.out_shape = (c.value, ho.value, wo.value)
        self.in_shape = (units[0].cin, H, W)
        self.offsets = []
        for i in range(len(units)):
            o = [ctypes.c_int64() for _ in range(4)]
            self.L.lrs_dipnet_param_offsets(h, i, *[ctypes.byref(x) for x in o])
            self.offsets.append(tuple(x.value for x in o))
        self.stream = torch.cuda.Stream(device=device)
        self._es = None

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.L.lrs_dipnet_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # ---- parameters ---------------------------------------------------------------------------
    def init_params(self, seed: int):
        """Fresh parameters and optimizer state, enqueued on the engine stream."""
        _check(self.L.lrs_dipnet_init_params(self.h, ctypes.c_uint64(seed & (2**64 - 1)),
                                             ctypes.c_void_p(self.stream.cuda_stream)), "init_params")

    def param_views(self, i: int, flat=None):
        """(weight [cout,cin,k,k], bias, gamma|None, beta|None) views into `flat` (default params)."""
        flat = self.params if flat is None else flat
        u = self.units[i]
        w, b, g, be = self.offsets[i]
        kk = u.cin * u.k * u.k
        out = [flat[w:w + u.cout * kk].view(u.cout, u.cin, u.k, u.k), flat[b:b + u.cout]]
        out += [flat[g:g + u.cout] if g >= 0 else None, flat[be:be + u.cout] if be >= 0 else None]
        return tuple(out)

    def load_reference_state_dict(self, sd, names=UNET_REF_NAMES):
        """Copy a my_Lipschitz_Unet state_dict (weight_bar / bias / weight_orig / bias_orig)."""
        import torch
        with torch.no_grad():
            for i, (cp, bp) in enumerate(names):
                w, b, g, be = self.param_views(i)
                w.copy_(torch.as_tensor(sd[cp + ".weight_bar"]).view_as(w))
                b.copy_(torch.as_tensor(sd[cp + ".bias"]))
                if bp is not None:
                    g.copy_(torch.as_tensor(sd[bp + ".weight_orig"]))
                    be.copy_(torch.as_tensor(sd[bp + ".bias_orig"]))
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            self.grads.zero_()
        torch.cuda.synchronize()
        self.reset_optimizer()

    def reset_optimizer(self):
        """Zero the Adam moments and the step count (a fresh torch.optim.Adam)."""
        _check(self.L.lrs_dipnet_reset_optimizer(self.h, ctypes.c_void_p(self.stream.cuda_stream)),
               "lrs_dipnet_reset_optimizer")
        self.stream.synchronize()

    # ---- compute ------------------------------------------------------------------------------
    def forward(self, x):
        """Network output (C, H, W) for input x (C_in, H, W) — a view of the engine's buffer."""
        import torch
        x = x.contiguous()
        assert tuple(x.shape[-3:]) == self.in_shape and x.dtype == torch.float32 and x.is_cuda
        self.stream.wait_stream(torch.cuda.current_stream())
        _check(self.L.lrs_dipnet_forward(self.h, _ptr(x), ctypes.c_void_p(self.stream.cuda_stream)),
               "lrs_dipnet_forward")
        torch.cuda.current_stream().wait_stream(self.stream)
        return self.output()

    def output(self):
        import torch
        n = int(np.prod(self.out_shape))
        p = self.L.lrs_dipnet_output(self.h)
        buf = self.ws
        off = p - buf.data_ptr()
        assert 0 <= off and off + 4 * n <= buf.numel()
        return buf[off:off + 4 * n].view(torch.float32).view(*self.out_shape)

    def train_steps(self, x, target, mask, nsteps: int, lr: float = 0.1, betas=(0.9, 0.999),
                    eps: float = 1e-8, es=None, use_graph: bool = True):
        """nsteps of: forward, masked MSE, backward, Adam (and the ES update when es is given)."""
        import torch
        self.stream.wait_stream(torch.cuda.current_stream())
        rc = self.L.lrs_dipnet_train_steps(
            self.h, _ptr(x), _ptr(target), _ptr(mask), ctypes.c_float(lr), ctypes.c_float(betas[0]),
            ctypes.c_float(betas[1]), ctypes.c_float(eps), _ptr(es.state) if es else None,
            _ptr(es.ring) if es else None, int(nsteps), 1 if use_graph else 0,
            ctypes.c_void_p(self.stream.cuda_stream))
        _check(rc, "lrs_dipnet_train_steps")
        torch.cuda.current_stream().wait_stream(self.stream)

    def last_loss(self) -> float:
        v = ctypes.c_double()
        _check(self.L.lrs_dipnet_last_loss(self.h, ctypes.byref(v), ctypes.c_void_p(self.stream.cuda_stream)),
               "lrs_dipnet_last_loss")
        return v.value


class EarlyStopper:
    """Device-side EarlyStop (main_LRS_PnP_DIP_1-LiP.py:71-99): ring of the last `size` outputs."""

    def __init__(self, n_elems: int, size: int = 30, patience: int = 60, device="cuda"):
        import torch
        self.size, self.patience, self.n = size, patience, n_elems
        nbytes = ctypes.sizeof(EsState)
        self.state = torch.zeros((nbytes + 7) // 8, dtype=torch.float64, device=device)
        self.ring = torch.zeros(size * n_elems, dtype=torch.float32, device=device)
        self._host = None
        L = _lib.device_lib()
        _check(L.lrs_es_init(_ptr(self.state), size, patience, None), "lrs_es_init")

    def read(self, stream=None) -> EsState:
        """Copy the state to the host after the work queued on `stream` (default: current)."""
        import torch
        s = stream or torch.cuda.current_stream()
        if self._host is None:
            self._host = torch.empty(self.state.numel(), dtype=torch.float64, pin_memory=True)
        with torch.cuda.stream(s):
            self._host.copy_(self.state, non_blocking=True)
        s.synchronize()
        return EsState.from_buffer_copy(self._host.numpy().tobytes()[:ctypes.sizeof(EsState)])

    def slot_of(self, epoch: int):
        return self.ring.view(self.size, self.n)[epoch % self.size]


@dataclass
class DipConfig:
    """get_DIP_out settings (main_LRS_PnP_DIP_1-LiP.py:208-225, :345-346)."""
    num_iter: int = 5000
    learning_rate: float = 0.1
    es_size: int = 30
    patience: int = 60
    poll_every: int = 10          # host polls the device ES flag every this many steps (< es_size)
    use_graph: bool = False       # replay one captured hipGraph per step (measured slower than
                                  # direct launches on ROCm 7.2 for this ~110-kernel step)
    hidden: int = 128
    early_stop: bool = True       # False: exactly num_iter steps (the timed-benchmark mode, §8d)


class LipschitzDip:
    """get_DIP_out on the HIP engine; one network object reused across outer iterations
    (re-initialised each call, as the reference builds a fresh net per call)."""

    def __init__(self, bands: int, H: int, W: int, cfg: DipConfig | None = None, device="cuda"):
        self.cfg = cfg or DipConfig()
        self.net = DipNet(lipschitz_unet_units(bands, bands, self.cfg.hidden), H, W, device=device)
        if self.net.out_shape != (bands, H, W):
            raise ValueError(f"my_Lipschitz_Unet maps {H}x{W} to {self.net.out_shape[1:]}; the reference "
                             "architecture needs sizes it reproduces (e.g. 36, 196)")
        self.es = EarlyStopper(bands * H * W, self.cfg.es_size, self.cfg.patience, device=device)
        self.calls = 0
        self.last_steps = 0
        self.last_stop_epoch = None

    def run(self, target, dip_input, mask, seed: int | None = None, num_iter: int | None = None,
            early_stop: bool = True):
        """Train a freshly initialised net on (dip_input -> target under mask) and return the output
        at the early-stopping epoch (or after num_iter steps with early_stop=False).

        The result is a view of an engine buffer, valid until the next call; it is ordered after
        the caller's current stream (the caller's stream waits for the DIP stream on return)."""
        import torch
        cfg = self.cfg
        n_iter = cfg.num_iter if num_iter is None else num_iter
        net = self.net
        net.stream.wait_stream(torch.cuda.current_stream())
        net.init_params(self.calls if seed is None else seed)
        self.calls += 1
        if not early_stop:
            net.train_steps(dip_input, target, mask, n_iter, cfg.learning_rate, use_graph=cfg.use_graph)
            self.last_steps, self.last_stop_epoch = n_iter, None
            return net.output()                    # the last step's forward output (`out`)
        L = _lib.device_lib()
        _check(L.lrs_es_init(_ptr(self.es.state), cfg.es_size, cfg.patience, ctypes.c_void_p(net.stream.cuda_stream)),
               "lrs_es_init")
        done = 0
        st = None
        while done < n_iter:
            k = min(cfg.poll_every, n_iter - done)
            net.train_steps(dip_input, target, mask, k, cfg.learning_rate, es=self.es, use_graph=cfg.use_graph)
            done += k
            st = self.es.read(net.stream)
            if st.stop:
                break
        torch.cuda.current_stream().wait_stream(net.stream)
        self.last_steps = done
        if st is not None and st.stop:
            self.last_stop_epoch = st.stop_epoch
            return self.es.slot_of(st.stop_epoch).view(net.out_shape)
        # the reference returns None here (its loop ends without returning); use the last output
        self.last_stop_epoch = None
        return self.es.slot_of(st.count - 1).view(net.out_shape)


def dip_input_from_unfolded(Z, H: int, W: int):
    """(P, B) unfolded matrix (p = i + H j) -> (B, H, W) image (…1-LiP.py:404)."""
    B = Z.shape[1]
    return Z.t().reshape(B, W, H).transpose(1, 2).contiguous()


def unfolded_from_image(img):
    """(B, H, W) image -> (P, B) unfolded matrix with p = i + H j (…1-LiP.py:411)."""
    B, H, W = img.shape
    return img.transpose(1, 2).reshape(B, H * W).t().contiguous()


def sigma_max(weights, ln_lambda: float = 1.0):
    """sigma_max of each [rows, ...] weight tensor (lrs_sigma_max_f32); returns (sigma, scale)."""
    import torch
    L = _lib.device_lib()
    n = len(weights)
    mats = [w.contiguous().view(w.shape[0], -1) for w in weights]
    W = (ctypes.c_void_p * n)(*[m.data_ptr() for m in mats])
    rows = (ctypes.c_int * n)(*[m.shape[0] for m in mats])
    cols = (ctypes.c_int * n)(*[m.shape[1] for m in mats])
    sig = torch.empty(n, dtype=torch.float32, device=mats[0].device)
    sc = torch.empty_like(sig)
    nb = int(L.lrs_sigma_max_workspace(n))
    ws = torch.empty(nb, dtype=torch.uint8, device=mats[0].device)
    s = torch.cuda.current_stream().cuda_stream
    _check(L.lrs_sigma_max_f32(W, None, rows, cols, n, ctypes.c_float(ln_lambda), _ptr(sig), _ptr(sc),
                               _ptr(ws), nb, ctypes.c_void_p(s)), "lrs_sigma_max_f32")
    return sig, sc


def out_size(H, W, k, stride, pad, up):
    ho, wo = ctypes.c_int(), ctypes.c_int()
    _check(_lib.lib().lrs_conv2d_out_size(H, W, k, stride, pad, up, ctypes.byref(ho), ctypes.byref(wo)),
           "lrs_conv2d_out_size")
    return ho.value, wo.value


def unet_size_ok(H: int, W: int) -> bool:
    """True when my_Lipschitz_Unet maps H x W back to H x W."""
    h, w = H, W
    for u in lipschitz_unet_units(1, 1, 1):
        h, w = out_size(h, w, u.k, u.stride, u.pad, u.upsample)
    return (h, w) == (H, W)


__all__ = ["ConvUnit", "DipNet", "EarlyStopper", "DipConfig", "LipschitzDip", "lipschitz_unet_units",
           "UNET_REF_NAMES", "dip_input_from_unfolded", "unfolded_from_image", "sigma_max", "unet_size_ok"]
