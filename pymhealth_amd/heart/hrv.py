"""Drop-in for the spectral band-power features of ``mhealth.heart.hrv``
(src/mhealth/heart/hrv.py:173-198) at window level: ``power_band(fs, lower, upper)``
and ``relative_power_band(fs, lower, upper)`` return WindowFeatures computing the
reference function on the window's periodogram."""
from ..features import band_power, relative_band_power, rms  # noqa: F401


def power_band(fs, lower=None, upper=None):
    return band_power(fs, lower, upper)


def relative_power_band(fs, lower=None, upper=None):
    return relative_band_power(fs, lower, upper)


__all__ = ["power_band", "relative_power_band", "rms"]
