"""Import shims: run the reference scripts unchanged with the hot-path names resolved to lrspnp.

    python -m lrspnp.shim /path/to/main_LRS_PnP_DIP_1-LiP.py [script args]

or, inside a process, ``lrspnp.shim.install()`` before the script's imports run.  A meta-path
finder placed first on sys.meta_path answers exactly these imports:

    from skimage.restoration import denoise_nl_means           -> lrspnp.compat.denoise_nl_means
    from models.my_Lipschitz_Unet import my_Lipschitz_Unet      -> lrspnp.nn.my_Lipschitz_Unet
    from models.skip import skip                                -> lrspnp.nn.skip

Everything else (the reference's own models package for models.unet / models.resnet, utils,
include, pytorch_ssim, the data files) resolves as it would without the shim.  The shim changes
where these three names come from, nothing in the scripts.
"""
from __future__ import annotations

import importlib.abc
import importlib.util
import os
import runpy
import sys

_TARGETS = {
    "skimage": None,                                  # a package holding only .restoration
    "skimage.restoration": ("lrspnp.compat", ["denoise_nl_means"]),
    "models.my_Lipschitz_Unet": ("lrspnp.nn", ["my_Lipschitz_Unet"]),
    "models.skip": ("lrspnp.nn", ["skip"]),
}


class _Loader(importlib.abc.Loader):
    def __init__(self, name):
        self.name = name

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        tgt = _TARGETS[self.name]
        if tgt is None:
            module.__path__ = []                      # package: submodules come from this finder
            module.__lrspnp_shim__ = "package"
            return
        src = importlib.import_module(tgt[0])
        for attr in tgt[1]:
            setattr(module, attr, getattr(src, attr))
        module.__lrspnp_shim__ = tgt[0]


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if fullname not in _TARGETS:
            return None
        return importlib.util.spec_from_loader(fullname, _Loader(fullname), is_package=_TARGETS[fullname] is None)


_FINDER = _Finder()


def install() -> None:
    """Put the finder first on sys.meta_path (idempotent) and drop already-imported targets."""
    if _FINDER not in sys.meta_path:
        sys.meta_path.insert(0, _FINDER)
    for name in _TARGETS:
        mod = sys.modules.get(name)
        if mod is not None and not hasattr(mod, "__lrspnp_shim__"):
            del sys.modules[name]


def uninstall() -> None:
    if _FINDER in sys.meta_path:
        sys.meta_path.remove(_FINDER)
    for name in _TARGETS:
        if hasattr(sys.modules.get(name), "__lrspnp_shim__"):
            del sys.modules[name]


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        sys.exit("usage: python -m lrspnp.shim SCRIPT.py [args...]")
    script = os.path.abspath(argv[0])
    install()
    sys.argv = [script] + argv[1:]
    sys.path.insert(0, os.path.dirname(script))
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
