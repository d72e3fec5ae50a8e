"""lrspnp.shim: the reference scripts' hot-path imports resolve to lrspnp (CPU: name resolution only;
the modules themselves need the GPU, tests/test_gpu_nn.py)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shim_resolves_reference_imports(tmp_path):
    # a stand-in "reference" tree: its own models package (with a skip.py that must NOT be used)
    (tmp_path / "models").mkdir()
    (tmp_path / "models" / "__init__.py").write_text("from .skip import skip\nfrom .unet import UNet\n")
    (tmp_path / "models" / "skip.py").write_text("def skip(*a, **k):\n    raise RuntimeError('reference skip')\n")
    (tmp_path / "models" / "unet.py").write_text("class UNet:\n    pass\n")
    (tmp_path / "script.py").write_text(
        "import sys\n"
        "from skimage.restoration import denoise_nl_means\n"
        "from models.my_Lipschitz_Unet import my_Lipschitz_Unet\n"
        "from models.skip import skip\n"
        "from models.unet import UNet\n"
        "import models\n"
        "print(denoise_nl_means.__module__, my_Lipschitz_Unet.__module__, skip.__module__, models.skip is skip,\n"
        "      UNet.__module__, sys.argv[1:])\n")
    env = dict(os.environ, PYTHONPATH=os.path.join(REPO, "lrs-pnp-dip_amd"))
    p = subprocess.run([sys.executable, "-m", "lrspnp.shim", str(tmp_path / "script.py"), "a1"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["lrspnp.compat", "lrspnp.nn", "lrspnp.nn", "True", "models.unet", "['a1']"]


def test_shim_keeps_real_skimage_submodules(tmp_path):
    """With a scikit-image installed, only skimage.restoration.denoise_nl_means is replaced: the real
    package, its other restoration functions and its other submodules stay importable."""
    sk = tmp_path / "site" / "skimage"
    (sk / "restoration").mkdir(parents=True)
    (sk / "metrics").mkdir()
    (sk / "__init__.py").write_text("REAL = True\n")
    (sk / "restoration" / "__init__.py").write_text(
        "def denoise_nl_means(*a, **k):\n    raise RuntimeError('real nlm')\n"
        "def estimate_sigma(x):\n    return 'real-sigma'\n")
    (sk / "metrics" / "__init__.py").write_text("def peak_signal_noise_ratio():\n    return 'real-psnr'\n")
    (tmp_path / "script.py").write_text(
        "import skimage\n"
        "from skimage.restoration import denoise_nl_means, estimate_sigma\n"
        "from skimage.metrics import peak_signal_noise_ratio\n"
        "print(skimage.REAL, denoise_nl_means.__module__, estimate_sigma(0), peak_signal_noise_ratio())\n")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(REPO, "lrs-pnp-dip_amd"), str(tmp_path / "site")]))
    p = subprocess.run([sys.executable, "-m", "lrspnp.shim", str(tmp_path / "script.py")], capture_output=True,
                       text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["True", "lrspnp.compat", "real-sigma", "real-psnr"]
