"""lrspnp — MI355X-native LRS-PnP inner loop (shuoli0708/LRS-PnP-DIP hot path).

Hot path (sparse-coding prox with the PnP-NLM denoiser, SVT low-rank prox, ADMM update) runs in
liblrspnp_hip.so (csrc/, gfx950).  `LrsPnP` is the batched driver; `compat` re-exports the
reference's own function names for drop-in use.
"""
from ._lib import LrsError, build, lib  # noqa: F401
from .solver import LrsPnP, LrsPnPConfig  # noqa: F401

__version__ = "0.1.0"
