"""ctypes binding of liblrspnp_hip.so (include/lrspnp.h).

The product path has no CPU fallback: if the library is missing, fails to load, or the device is
not gfx950, every op raises ``LrsError`` instead of computing anything elsewhere.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LRSPNP_LIB: another build of the same library (A/B timing of kernel variants, tools/ab_*.sh)
LIB_PATH = os.environ.get("LRSPNP_LIB") or os.path.join(_HERE, "liblrspnp_hip.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

LRS_OK = 0
LRS_E = {-1: "LRS_E_INVALID", -2: "LRS_E_UNSUPPORTED", -3: "LRS_E_WORKSPACE", -4: "LRS_E_NODEVICE"}

ALPHA_SPEC2, ALPHA_FRO4, ALPHA_SOFT = 0, 1, 2
PROX_NLM, PROX_SOFT, PROX_NLM_MATLAB = 0, 1, 2


class LrsError(RuntimeError):
    pass


# per-call / per-handle options (include/lrspnp.h); the library keeps no process-wide mode
ISTA_F32, ISTA_SPLIT_BF16 = 0, 1
DIP_F32, DIP_SPLIT_BF16 = 0, 1


ISTA_ALGO_AUTO, ISTA_ALGO_GENERIC = 0, 1


class IstaOpts(ctypes.Structure):
    _fields_ = [("precision", ctypes.c_int32), ("max_workgroups", ctypes.c_int32), ("algorithm", ctypes.c_int32),
                ("warm_start", ctypes.c_int32), ("reserved", ctypes.c_int32 * 4)]


class DipOpts(ctypes.Structure):
    _fields_ = [("precision", ctypes.c_int32), ("upsample_dgrad", ctypes.c_int32), ("reserved", ctypes.c_int32 * 6)]


def ista_opts(precision: int = ISTA_SPLIT_BF16, max_workgroups: int = 0, algorithm: int = ISTA_ALGO_AUTO,
              warm_start: int = 0) -> IstaOpts:
    return IstaOpts(precision=precision, max_workgroups=max_workgroups, algorithm=algorithm, warm_start=warm_start)


def dip_opts(precision: int = DIP_SPLIT_BF16, upsample_dgrad: int = 0) -> DipOpts:
    return DipOpts(precision=precision, upsample_dgrad=upsample_dgrad)


_lib = None
_device_checked = False


def build(force: bool = False) -> str:
    """Compile csrc/ for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    import subprocess

    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(["make", "-s", "-j8", "-C", CSRC])
    return LIB_PATH


def _declare(L):
    c = ctypes
    vp, i64, i32, f32, f64, sz = c.c_void_p, c.c_int64, c.c_int, c.c_float, c.c_double, c.c_size_t
    i32p = c.POINTER(c.c_int32)
    dop = c.POINTER(DipOpts)
    sig = {
        "lrs_version": (c.c_char_p, []),
        "lrs_check_device": (i32, []),
        "lrs_nlm_col_f32": (i32, [vp, i64, vp, i64, i64, i64, f64, vp, i32, i32, vp]),
        "lrs_block_count": (i64, [i64, i64, i64, i64]),
        "lrs_block_grid": (i32, [i64, i64, i64, i64, i32p, i32p, i64]),
        "lrs_cover_ranges": (i32, [i64, i64, i32p, i64, i32p, i32p]),
        "lrs_im2col_f32": (i32, [vp, vp, f32, i64, i64, i64, vp, vp, i64, i64, vp, vp, vp]),
        "lrs_ista_alpha_workspace": (sz, [i64, i64, i64]),
        "lrs_ista_alpha_f32": (i32, [vp, i64, i64, vp, i64, i64, i32, f32, vp, vp, vp, sz, vp]),
        "lrs_ista_workspace": (sz, [i64, i64, i32, c.POINTER(IstaOpts)]),
        "lrs_ista_f32": (i32, [vp, vp, vp, i64, i64, i64, i64, vp, vp, i32, i32, vp, vp, c.POINTER(IstaOpts), vp,
                               sz, vp]),
        "lrs_nlm_matlab_col_f32": (i32, [vp, i64, vp, i64, i64, i64, f64, vp, vp]),
        "lrs_ista_pat_plan_len": (i64, [i64, i64]),
        "lrs_ista_pat_plan": (i64, [i32p, i64, i64, i32p, i64]),
        "lrs_ista_pat_preferred": (i32, [i64, i64, i64, i64, i32]),
        "lrs_ista_pat_workspace": (sz, [i64, i64, i64]),
        "lrs_ista_pat_prepare": (i32, [vp, i64, i64, vp, i64, i64, vp, sz, vp]),
        "lrs_ista_pat_f32": (i32, [vp, vp, i64, vp, i64, i64, i64, i64, i64, vp, vp, i32, i32, vp, vp,
                                   c.POINTER(IstaOpts), vp, sz, vp]),
        "lrs_ssim_f32": (i32, [vp, vp, i32, i32, i32, vp, vp]),
        "lrs_psnr_workspace": (sz, [i64, i64]),
        "lrs_psnr_bands_f32": (i32, [vp, vp, i64, i64, vp, vp, sz, vp]),
        "lrs_svt_workspace": (sz, [i64, i64]),
        "lrs_svt_f32": (i32, [vp, vp, f32, i64, i64, f64, vp, vp, i32, vp, sz, vp]),
        "lrs_svt_gram_f32": (i32, [vp, vp, f32, i64, i64, i32, vp, sz, vp]),
        "lrs_svt_finish_f32": (i32, [vp, vp, f32, i64, i64, f64, vp, vp, i32, vp, sz, vp]),
        "lrs_svt_gram_offset": (i32, [i64, i64, vp, vp]),
        "lrs_diag_svt_state": (i32, [vp, i64, i64, vp]),
        "lrs_admm_update_f32": (i32, [vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, vp, i64, vp, vp,
                                      vp, vp, f32, f32, f32, vp, vp, vp]),
        # DIP low-rank prox
        "lrs_conv2d_out_size": (i32, [i32, i32, i32, i32, i32, i32, c.POINTER(c.c_int), c.POINTER(c.c_int)]),
        "lrs_conv2d_col_size": (i64, [i32, i32, i32, i32, i32, i32, i32]),
        "lrs_conv2d_workspace": (sz, [i32, i32, i32, i32, i32, i32, i32, i32, dop]),
        "lrs_conv2d_fwd_f32": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, dop, vp, sz,
                                     vp]),
        "lrs_conv2d_bwd_f32": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, dop, vp,
                                     sz, vp]),
        "lrs_conv2d_bwd_x_f32": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, dop, vp,
                                       sz, vp]),
        "lrs_bn_act_workspace": (sz, [i32, i64]),
        "lrs_bn_act_fwd_f32": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, f32, f32, vp, sz, vp]),
        "lrs_bn_act_bwd_f32": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, vp, sz, vp]),
        "lrs_conv_bn_small_f32": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, i32,
                                        vp, vp, vp, vp, vp, vp, vp]),
        "lrs_sigma_max_workspace": (sz, [i32]),
        "lrs_sigma_max_f32": (i32, [c.POINTER(vp), c.POINTER(vp), c.POINTER(c.c_int), c.POINTER(c.c_int), i32,
                                    f32, vp, vp, vp, sz, vp]),
        "lrs_diag_sigma_phases": (i32, [c.POINTER(vp), c.POINTER(c.c_int), c.POINTER(c.c_int), i32, vp, sz, vp, vp]),
        "lrs_adam_f32": (i32, [vp, vp, vp, vp, i64, vp, f32, f32, f32, f32, vp]),
        "lrs_masked_mse_f32": (i32, [vp, vp, vp, i32, i64, vp, vp, vp]),
        "lrs_unfolded_to_image_f32": (i32, [vp, vp, f32, i64, i64, i64, vp, vp]),
        "lrs_image_to_unfolded_f32": (i32, [vp, i64, i64, i64, vp, vp]),
        "lrs_es_ring_bytes": (sz, [i32, i64]),
        "lrs_es_init": (i32, [vp, i32, i32, vp]),
        "lrs_es_update_f32": (i32, [vp, i64, vp, vp, vp]),
        "lrs_dipnet_create": (i32, [vp, i32, i32, i32, i32, dop, c.POINTER(vp)]),
        "lrs_dipnet_get_opts": (i32, [vp, dop]),
        "lrs_dipnet_node_shape": (i32, [vp, i32, c.POINTER(c.c_int), c.POINTER(c.c_int), c.POINTER(c.c_int)]),
        "lrs_dipnet_destroy": (None, [vp]),
        "lrs_dipnet_num_params": (i64, [vp]),
        "lrs_dipnet_num_bnstats": (i64, [vp]),
        "lrs_dipnet_workspace": (sz, [vp]),
        "lrs_dipnet_param_offsets": (i32, [vp, i32, c.POINTER(i64), c.POINTER(i64), c.POINTER(i64),
                                           c.POINTER(i64)]),
        "lrs_dipnet_out_shape": (i32, [vp, c.POINTER(c.c_int), c.POINTER(c.c_int), c.POINTER(c.c_int)]),
        "lrs_dipnet_bind": (i32, [vp, vp, vp, vp, vp, vp, vp, sz]),
        "lrs_dipnet_init_params": (i32, [vp, c.c_uint64, vp]),
        "lrs_dipnet_reset_optimizer": (i32, [vp, vp]),
        "lrs_dipnet_forward": (i32, [vp, vp, vp]),
        "lrs_dipnet_backward": (i32, [vp, vp, vp, vp]),
        "lrs_dipnet_set_ln_lambda": (i32, [vp, f32]),
        "lrs_dipnet_output": (c.c_size_t, [vp]),
        "lrs_dipnet_grads": (c.c_size_t, [vp]),
        "lrs_dipnet_node_buffer": (c.c_size_t, [vp, i32, i32]),
        "lrs_dipnet_train_steps": (i32, [vp, vp, vp, vp, f32, f32, f32, f32, vp, vp, i32, i32, vp]),
        "lrs_dipnet_last_loss": (i32, [vp, c.POINTER(f64), vp]),
        "lrs_stream_wait": (i32, [vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """The loaded library (host-side entry points usable without a GPU)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LrsError(f"{LIB_PATH} not built: run __graft_entry__.build() (make -C {CSRC})")
        try:
            _lib = _declare(ctypes.CDLL(LIB_PATH))
        except OSError as e:  # pragma: no cover - environment problem
            raise LrsError(f"cannot load {LIB_PATH}: {e}") from e
    return _lib


def device_lib():
    """The library, after checking that the current device is a gfx950 (MI355X)."""
    global _device_checked
    L = lib()
    if not _device_checked:
        import torch

        if not torch.cuda.is_available():
            raise LrsError("no ROCm GPU visible: lrspnp has no CPU fallback")
        rc = L.lrs_check_device()
        if rc != LRS_OK:
            raise LrsError(f"lrs_check_device: {LRS_E.get(rc, rc)} (need gfx950)")
        _device_checked = True
    return L


def check(rc: int, what: str) -> None:
    if rc != LRS_OK:
        raise LrsError(f"{what} failed: {LRS_E.get(rc, f'hipError {rc}')}")
