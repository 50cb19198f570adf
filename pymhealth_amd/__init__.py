"""pymhealth_amd — MI355X-native sliding-window feature engine.

A drop-in for the windowed-feature hot path of pymhealth (``mhealth.util.windows.
rolling_apply`` + the per-window features of ``mhealth.generic`` / ``mhealth.heart``):
Python host code on PyTorch-ROCm tensors calling hand-written HIP kernels (gfx950)
through the C-ABI of include/mhfeat.h (``libmhfeat.so``). No CPU fallback.

``install_mhealth_alias()`` makes ``import mhealth.util.windows`` (and the other
reference module paths, plus ``mhealth.features`` / ``mhealth.processing``) resolve to
this package.
"""
import sys

__version__ = "0.1.0"

from . import features, processing  # noqa: E402,F401
from .util import windows  # noqa: E402,F401
from . import fft, generic, heart, inertial, util  # noqa: E402,F401

_ALIASES = ("util", "util.windows", "generic", "generic.stats", "generic.timedom",
            "generic.information", "generic.rqa", "generic.frequency", "generic.frequency.density",
            "generic.filters", "heart", "heart.hrv", "heart.qrs", "inertial",
            "inertial.accelerometer", "features", "processing", "fft")


def install_mhealth_alias():
    """Register this package under the reference's import name ``mhealth``."""
    sys.modules["mhealth"] = sys.modules[__name__]
    for name in _ALIASES:
        sys.modules["mhealth." + name] = sys.modules[__name__ + "." + name]
    return sys.modules["mhealth"]
