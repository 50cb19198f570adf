"""Drop-in for ``mhealth.generic.information`` (src/mhealth/generic/information.py).

``entropy`` of the reference (information.py:10-20) is applied to a window's PSD;
the window-level form is ``spectral_entropy(fs)``."""
from ..features import spectral_entropy  # noqa: F401

__all__ = ["spectral_entropy"]
