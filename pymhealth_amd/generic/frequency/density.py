"""Drop-in for ``mhealth.generic.frequency.density`` (density.py:9-32): the dominant
(peak) frequency of a window's PSD as a WindowFeature factory."""
from ...features import dominant_frequency  # noqa: F401


def peak_frequency(fs, lower=None, upper=None):
    """Window-level ``density.peak_frequency``: first argmax of psd(x) over
    [first f >= lower, first f >= upper)."""
    return dominant_frequency(fs, lower, upper)


__all__ = ["peak_frequency", "dominant_frequency"]
