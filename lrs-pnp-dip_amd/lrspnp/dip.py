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
NODE_CONV, NODE_BN, NODE_CONCAT = 0, 1, 2
BN_NONE, BN_PLAIN, BN_LIP = 0, 1, 2
WINIT_DEFAULT, WINIT_KAIMING = 0, 1


class DipNode(ctypes.Structure):
    """lrs_dip_node: one node of the network DAG (include/lrspnp.h).  Tensor 0 is the input and
    node i produces tensor i + 1."""
    _fields_ = [(n, ctypes.c_int32) for n in
                ("kind", "in0", "in1", "cout", "k", "stride", "pad", "pad_mode", "upsample", "bn", "act", "sn",
                 "winit")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


def conv_node(src, cin_unused, cout, k, stride=1, up=0, bn=BN_LIP, act=ACT_LRELU, pad_mode=PAD_REFLECT, sn=1,
              winit=WINIT_KAIMING):
    return DipNode(NODE_CONV, src, 0, cout, k, stride, (k - 1) // 2, pad_mode, up, bn, act, sn, winit)


class EsState(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int32), ("size", ctypes.c_int32), ("patience", ctypes.c_int32),
                ("wait", ctypes.c_int32), ("stop", ctypes.c_int32), ("stop_epoch", ctypes.c_int32),
                ("best_epoch", ctypes.c_int32), ("reserved", ctypes.c_int32), ("best", ctypes.c_double),
                ("var_acc", ctypes.c_double), ("last_var", ctypes.c_double)]


def lipschitz_unet_nodes(c_in: int = 128, c_out: int = 128, hidden: int = 128,
                         pad: str = "reflection") -> list[DipNode]:
    """The 14 conv units of my_Lipschitz_Unet (my_Lipschitz_Unet.py:31-103) as a chain.

    The reference hard-codes 128 everywhere; c_in / c_out generalise the first / last conv to
    other band counts (hidden stays 128), as SURVEY.md §8 a8 sizes the 196x196x198 config."""
    pm = PAD_REFLECT if pad == "reflection" else PAD_ZERO
    nodes = []

    def u(cout, k, stride=1, up=0, bn=BN_LIP):
        nodes.append(conv_node(len(nodes), 0, cout, k, stride, up, bn, ACT_LRELU, pm))

    h = hidden
    u(h, 3, 2); u(h, 3)                                          # d_1  (:31-39)
    for _ in range(3):                                          # d_2..d_4 (:40-66)
        u(h, 3, 2); u(h, 3)
    u(h, 2, up=1); u(h, 2, up=1)                                # up_1, up_2 (:71-82)
    u(h, 3, up=1); u(h, 3, up=1)                                # up_3, up_4 (:83-94)
    u(h, 1); u(c_out, 1, bn=BN_NONE)                            # last (:96-103)
    return nodes


# backwards-compatible name
lipschitz_unet_units = lipschitz_unet_nodes


def skip_nodes(c_in: int = 128, c_out: int = 128, down=(128,) * 5, up=(128,) * 5, skip=(128,) * 5,
               filter_down: int = 3, filter_up: int = 3, filter_skip: int = 1, pad: str = "reflection",
               need_sigmoid: bool = True, need1x1_up: bool = True) -> list[DipNode]:
    """models/skip.py:5-99 (the DIP net of main_LRS_PnP_DIP_pro.py:215-221) as a DAG.

    Per scale i with input x:  out_i = act(BN(conv1x1(act(BN(conv3x3(BN(cat(skip_i(x),
    up2(deeper_i(x)))))))))) where skip_i = act(BN(conv1x1 x)), deeper_i = act(BN(conv3x3(
    act(BN(conv3x3 stride 2 (x)))))) followed by scale i+1 (not at the deepest); the final 1x1
    conv + Sigmoid.  Plain BatchNorm2d, nn.Conv2d default init, no spectral norm."""
    pm = PAD_REFLECT if pad == "reflection" else PAD_ZERO
    nodes: list[DipNode] = []

    def add(nd):
        nodes.append(nd)
        return len(nodes)          # tensor id of its output

    def conv(src, cout, k, stride=1, bn=BN_PLAIN, act=ACT_LRELU):
        return add(DipNode(NODE_CONV, src, 0, cout, k, stride, (k - 1) // 2, pm, 0, bn, act, 0, WINIT_DEFAULT))

    def level(i, x):
        s = conv(x, skip[i], filter_skip) if skip[i] else None                  # skip.py:57-60
        d = conv(x, down[i], filter_down, 2)                                   # :63-65
        d = conv(d, down[i], filter_down)                                      # :67-69
        if i < len(down) - 1:
            d = level(i + 1, d)                                                # deeper_main (:71-78)
        if s is not None:
            c = add(DipNode(NODE_CONCAT, s, d, 0, 0, 0, 0, 0, 1, 0, ACT_NONE, 0, 0))   # Concat + Upsample
        else:
            raise NotImplementedError("num_channels_skip = 0 (no Concat) is not used by the reference")
        c = add(DipNode(NODE_BN, c, 0, 0, 0, 0, 0, 0, 0, BN_PLAIN, ACT_NONE, 0, 0))      # bn(skip + k) (:55)
        c = conv(c, up[i], filter_up)                                           # :82-84
        if need1x1_up:
            c = conv(c, up[i], 1)                                               # :87-90
        return c

    top = level(0, 0)
    conv(top, c_out, 1, bn=BN_NONE, act=ACT_SIGMOID if need_sigmoid else ACT_NONE)   # :95-97
    return nodes


# reference state_dict prefixes of each conv node of my_Lipschitz_Unet (named_parameters)
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


# Orders the DIP stream against the caller's with a device-scope event (lrs_stream_wait) instead of
# torch's wait_stream (an event with the default system-scope release); False: torch's (A/B only).
DEVICE_SCOPE_WAITS = True


def stream_wait(waiter, signaler):
    """waiter's later work runs after signaler's work so far (two streams of one device)."""
    if not DEVICE_SCOPE_WAITS:
        waiter.wait_stream(signaler)
        return
    _check(_lib.device_lib().lrs_stream_wait(ctypes.c_void_p(waiter.cuda_stream), ctypes.c_void_p(signaler.cuda_stream)),
           "lrs_stream_wait")


class DipNet:
    """A sequential conv net on the HIP engine (lrs_dipnet_*), with flat parameter buffers."""

    def __init__(self, nodes: list[DipNode], C: int, H: int, W: int, device="cuda", params=None, bnstats=None,
                 precision: int = _lib.DIP_SPLIT_BF16, upsample_dgrad: int = 0, stream_priority: int = 0):
        """params / bnstats (optional): existing flat device buffers to bind (shared with another
        engine of the same nodes at another H x W: the parameter layout does not depend on it).
        precision / upsample_dgrad: this net's lrs_dip_opts, fixed at creation.
        stream_priority: priority of the net's stream (torch.cuda.Stream; the engine's weight-gradient
        side stream takes the same)."""
        import torch

        self.L = _lib.device_lib()
        self.units = self.nodes = list(nodes)
        arr = (DipNode * len(nodes))(*nodes)
        h = ctypes.c_void_p()
        self.opts = _lib.dip_opts(precision, upsample_dgrad)
        _check(self.L.lrs_dipnet_create(arr, len(nodes), C, H, W, ctypes.byref(self.opts), ctypes.byref(h)),
               "lrs_dipnet_create")
        self.h = h
        self.H, self.W = H, W
        self.n_params = int(self.L.lrs_dipnet_num_params(h))
        nbs = int(self.L.lrs_dipnet_num_bnstats(h))
        ws = int(self.L.lrs_dipnet_workspace(h))
        f32 = dict(dtype=torch.float32, device=device)
        if params is not None and (params.numel() != self.n_params or params.dtype != torch.float32 or not params.is_cuda):
            raise _lib.LrsError(f"shared params must be {self.n_params} float32 on the device")
        self.params = params if params is not None else torch.zeros(self.n_params, **f32)
        self.grads = torch.zeros(self.n_params, **f32)
        self.exp_avg = torch.zeros(self.n_params, **f32)
        self.exp_avg_sq = torch.zeros(self.n_params, **f32)
        self.bnstats = bnstats if bnstats is not None else torch.zeros(max(nbs, 1), **f32)
        self.ws = torch.zeros(ws, dtype=torch.uint8, device=device)
        _check(self.L.lrs_dipnet_bind(h, _ptr(self.params), _ptr(self.grads), _ptr(self.exp_avg),
                                      _ptr(self.exp_avg_sq), _ptr(self.bnstats), _ptr(self.ws), ws),
               "lrs_dipnet_bind")
        c, ho, wo = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.lrs_dipnet_out_shape(h, ctypes.byref(c), ctypes.byref(ho), ctypes.byref(wo))
        self.out_shape = (c.value, ho.value, wo.value)
        self.in_shape = (C, H, W)
        self.shapes = []
        for i in range(len(nodes)):
            cc, hh, ww = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            self.L.lrs_dipnet_node_shape(h, i, ctypes.byref(cc), ctypes.byref(hh), ctypes.byref(ww))
            self.shapes.append((cc.value, hh.value, ww.value))
        self.offsets = []
        for i in range(len(nodes)):
            o = [ctypes.c_int64() for _ in range(4)]
            self.L.lrs_dipnet_param_offsets(h, i, *[ctypes.byref(x) for x in o])
            self.offsets.append(tuple(x.value for x in o))
        self.stream = torch.cuda.Stream(device=device, priority=int(stream_priority))
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
        """(weight [cout,cin,k,k] | None, bias | None, gamma | None, beta | None) of node i, as views
        into `flat` (default: the parameters)."""
        flat = self.params if flat is None else flat
        nd = self.nodes[i]
        w, b, g, be = self.offsets[i]
        C = self.shapes[i][0]
        out = [None, None]
        if nd.kind == NODE_CONV:
            cin = self.in_shape[0] if nd.in0 == 0 else self.shapes[nd.in0 - 1][0]
            out = [flat[w:w + C * cin * nd.k * nd.k].view(C, cin, nd.k, nd.k), flat[b:b + C]]
        out += [flat[g:g + C] if g >= 0 else None, flat[be:be + C] if be >= 0 else None]
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

    def backward(self, x, gout):
        """Parameter gradients (into self.grads) of the last forward(x) for dL/dout = gout."""
        import torch
        x, gout = x.contiguous(), gout.contiguous()
        assert tuple(gout.shape[-3:]) == self.out_shape and gout.dtype == torch.float32 and gout.is_cuda
        self.stream.wait_stream(torch.cuda.current_stream())
        _check(self.L.lrs_dipnet_backward(self.h, _ptr(x), _ptr(gout), ctypes.c_void_p(self.stream.cuda_stream)),
               "lrs_dipnet_backward")
        torch.cuda.current_stream().wait_stream(self.stream)

    def set_ln_lambda(self, ln_lambda: float):
        _check(self.L.lrs_dipnet_set_ln_lambda(self.h, ctypes.c_float(ln_lambda)), "lrs_dipnet_set_ln_lambda")

    def output(self):
        import torch
        n = int(np.prod(self.out_shape))
        p = self.L.lrs_dipnet_output(self.h)
        buf = self.ws
        off = p - buf.data_ptr()
        assert 0 <= off and off + 4 * n <= buf.numel()
        return buf[off:off + 4 * n].view(torch.float32).view(*self.out_shape)

    def train_steps(self, x, target, mask, nsteps: int, lr: float = 0.1, betas=(0.9, 0.999),
                    eps: float = 1e-8, es=None, use_graph: bool = False):
        """nsteps of: forward, masked MSE, backward, Adam (and the ES update when es is given).
        use_graph: replay one captured hipGraph per step instead of the eager launches (bit-identical,
        measured slower: DESIGN.md §5 -- off by default, as in DipConfig)."""
        import torch
        stream_wait(self.stream, torch.cuda.current_stream())
        rc = self.L.lrs_dipnet_train_steps(
            self.h, _ptr(x), _ptr(target), _ptr(mask), ctypes.c_float(lr), ctypes.c_float(betas[0]),
            ctypes.c_float(betas[1]), ctypes.c_float(eps), _ptr(es.state) if es else None,
            _ptr(es.ring) if es else None, int(nsteps), 1 if use_graph else 0,
            ctypes.c_void_p(self.stream.cuda_stream))
        _check(rc, "lrs_dipnet_train_steps")
        stream_wait(torch.cuda.current_stream(), self.stream)

    def node_buffer(self, node: int, which: int = 0):
        """A copy of node `node`'s workspace buffer (0 output, 1 pre-BN z, 2 dL/dz, 3 dL/d(output);
        None where absent), shaped (C, H, W) -- diagnostics."""
        import torch
        ptr = int(self.L.lrs_dipnet_node_buffer(self.h, int(node), int(which)))
        if not ptr:
            return None
        c, h, w = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.lrs_dipnet_node_shape(self.h, int(node), ctypes.byref(c), ctypes.byref(h), ctypes.byref(w))
        n = c.value * h.value * w.value
        base = self.ws.data_ptr()
        off = (ptr - base) // 4
        assert 0 <= off and (ptr - base) % 4 == 0 and off + n <= self.ws.numel() // 4
        torch.cuda.synchronize()
        return self.ws.view(torch.float32)[off:off + n].clone().view(c.value, h.value, w.value)

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
        L = _lib.device_lib()
        # the ring [size][N] floats, then the sliding window sums (lrs_es_ring_bytes)
        self.ring = torch.zeros((L.lrs_es_ring_bytes(size, n_elems) + 3) // 4, dtype=torch.float32, device=device)
        self._host = None
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
        return self.ring[:self.size * self.n].view(self.size, self.n)[epoch % self.size]


@dataclass
class DipConfig:
    """get_DIP_out settings (main_LRS_PnP_DIP_1-LiP.py:208-225, :345-346)."""
    num_iter: int = 5000
    learning_rate: float = 0.1
    es_size: int = 30
    patience: int = 60
    # host polls of the device ES state: None = after exactly the steps until the earliest epoch at
    # which the rule could stop (es_size - count + patience while filling, else patience - wait): a
    # stop always falls on a batch's last step, so no step runs past it and polls are few; an int =
    # every this many steps (< es_size, so the stop epoch's ring slot survives the overshoot)
    poll_every: int | None = None
    use_graph: bool = False       # replay one captured hipGraph per step (measured slower than
                                  # direct launches on ROCm 7.2 for this ~110-kernel step)
    hidden: int = 128
    net: str = "unet1lip"         # 'unet1lip' (…1-LiP.py:214) or 'skip' (…pro.py:215-221)
    early_stop: bool = True       # False: exactly num_iter steps (the timed-benchmark mode, §8d)


class DipProx:
    """get_DIP_out on the HIP engine (…1-LiP.py:208-264 with my_Lipschitz_Unet, …pro.py:211-272
    with skip()); one network object reused across outer iterations (re-initialised each call,
    as the reference builds a fresh net per call)."""

    def __init__(self, bands: int, H: int, W: int, cfg: DipConfig | None = None, device="cuda",
                 stream_priority: int = 0):
        self.cfg = cfg or DipConfig()
        nodes = (skip_nodes(bands, bands) if self.cfg.net == "skip"
                 else lipschitz_unet_nodes(bands, bands, self.cfg.hidden))
        self.net = DipNet(nodes, bands, H, W, device=device, stream_priority=stream_priority)
        if self.net.out_shape != (bands, H, W):
            raise ValueError(f"the DIP net maps {H}x{W} to {self.net.out_shape[1:]}; the reference "
                             "architecture needs sizes it reproduces (e.g. 36, 196 for the U-Net)")
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
        stream_wait(net.stream, torch.cuda.current_stream())
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
            k = min(cfg.poll_every or self.steps_to_possible_stop(st), n_iter - done)
            net.train_steps(dip_input, target, mask, k, cfg.learning_rate, es=self.es, use_graph=cfg.use_graph)
            done += k
            st = self.es.read(net.stream)
            if st.stop:
                break
        stream_wait(torch.cuda.current_stream(), net.stream)
        self.last_steps = done
        if st is not None and st.stop:
            self.last_stop_epoch = st.stop_epoch
            return self.es.slot_of(st.stop_epoch).view(net.out_shape)
        # the reference returns None here (its loop ends without returning); use the last output
        self.last_stop_epoch = None
        return self.es.slot_of(st.count - 1).view(net.out_shape)


    def steps_to_possible_stop(self, st) -> int:
        """Training steps until the earliest epoch at which EarlyStop could stop, from the state after
        the last poll (None: before the first step).  While the window fills no test runs; the first
        test always improves on best = inf (wait = 0); after it, wait grows by at most one per step and
        the rule stops when it reaches patience (…1-LiP.py:71-99)."""
        size, patience = self.cfg.es_size, self.cfg.patience
        count = 0 if st is None else st.count
        if count < size:
            return size - count + patience
        return max(1, patience - st.wait)


LipschitzDip = DipProx   # the 1-Lip name used by the first callers


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
    for u in lipschitz_unet_nodes(1, 1, 1):
        h, w = out_size(h, w, u.k, u.stride, u.pad, u.upsample)
    return (h, w) == (H, W)


__all__ = ["DipNode", "DipNet", "EarlyStopper", "DipConfig", "DipProx", "LipschitzDip", "lipschitz_unet_nodes",
           "lipschitz_unet_units", "skip_nodes",
           "UNET_REF_NAMES", "dip_input_from_unfolded", "unfolded_from_image", "sigma_max", "unet_size_ok"]
