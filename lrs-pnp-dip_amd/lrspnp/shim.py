"""Import shims: run the reference scripts unchanged with the hot-path names resolved to lrspnp.

    python -m lrspnp.shim /path/to/main_LRS_PnP_DIP_1-LiP.py [script args]

or, inside a process, ``lrspnp.shim.install()`` before the script's imports run.  A meta-path
finder placed first on sys.meta_path answers exactly these imports:

    from skimage.restoration import denoise_nl_means           -> lrspnp.compat.denoise_nl_means
                                                                   (on the real skimage.restoration
                                                                   when scikit-image is installed)
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
    "skimage.restoration": ("lrspnp.compat", ["denoise_nl_means"]),
    "models.my_Lipschitz_Unet": ("lrspnp.nn", ["my_Lipschitz_Unet"]),
    "models.skip": ("lrspnp.nn", ["skip"]),
}
# Only skimage.restoration.denoise_nl_means is replaced: when scikit-image is installed, the real
# skimage.restoration loads and that one name is overridden on it (estimate_sigma,
# denoise_tv_chambolle, skimage.metrics, skimage.io ... stay the real ones); without it, an empty
# `skimage` package is provided so that the import resolves.
_STUB_PARENT = "skimage"


def _override(module, name):
    tgt = _TARGETS[name]
    src = importlib.import_module(tgt[0])
    for attr in tgt[1]:
        setattr(module, attr, getattr(src, attr))
    module.__lrspnp_shim__ = tgt[0]


class _Loader(importlib.abc.Loader):
    """A target with no real module (or the stub parent package)."""

    def __init__(self, name):
        self.name = name

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        if self.name == _STUB_PARENT:
            module.__path__ = []                      # package: .restoration comes from this finder
            module.__lrspnp_shim__ = "package"
            return
        _override(module, self.name)


class _OverrideLoader(importlib.abc.Loader):
    """The real module, then the hot-path names replaced on it."""

    def __init__(self, real, name):
        self.real, self.name = real, name

    def create_module(self, spec):
        return self.real.create_module(spec)

    def exec_module(self, module):
        self.real.exec_module(module)
        _override(module, self.name)


def _real_spec(fullname, path):
    import importlib.machinery
    try:
        return importlib.machinery.PathFinder.find_spec(fullname, path)
    except (ImportError, ValueError):
        return None


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if fullname == _STUB_PARENT:
            if _real_spec(fullname, path) is not None:
                return None                           # the real scikit-image package
            return importlib.util.spec_from_loader(fullname, _Loader(fullname), is_package=True)
        if fullname not in _TARGETS:
            return None
        real = _real_spec(fullname, path) if fullname == "skimage.restoration" else None
        if real is not None and real.loader is not None:
            real.loader = _OverrideLoader(real.loader, fullname)
            return real
        return importlib.util.spec_from_loader(fullname, _Loader(fullname))


_FINDER = _Finder()


def install() -> None:
    """Put the finder first on sys.meta_path (idempotent).  An already-imported real
    skimage.restoration gets the override in place; other already-imported targets are dropped so
    that the next import goes through the finder."""
    if _FINDER not in sys.meta_path:
        sys.meta_path.insert(0, _FINDER)
    for name in _TARGETS:
        mod = sys.modules.get(name)
        if mod is None or hasattr(mod, "__lrspnp_shim__"):
            continue
        if name == "skimage.restoration":
            _override(mod, name)
        else:
            del sys.modules[name]


def uninstall() -> None:
    if _FINDER in sys.meta_path:
        sys.meta_path.remove(_FINDER)
    for name in list(_TARGETS) + [_STUB_PARENT]:
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
