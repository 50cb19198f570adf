"""Drop-in for ``mhealth.generic.frequency.density`` (density.py:9-32).

``peak_frequency(psd, freqs, lower=None, upper=None)`` keeps the reference's signature on
a PSD the caller computed (pymhealth_amd.spectrum: one lane per psd row, float32/float64);
the window-level dominant frequency of each window's on-chip periodogram is
``features.dominant_frequency(fs, lower, upper)``.
"""
import numpy as np

from ...features import dominant_frequency  # noqa: F401
from ...spectrum import peak_frequency  # noqa: F401


def first_index(arr, x):
    """density.first_index (density.py:9-14): the first i with x <= arr[i], else len(arr)."""
    hit = np.nonzero(x <= np.asarray(arr))[0]
    return int(hit[0]) if hit.size else len(arr)


__all__ = ["first_index", "peak_frequency", "dominant_frequency"]
