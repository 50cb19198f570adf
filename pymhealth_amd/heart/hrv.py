"""Drop-in for ``mhealth.heart.hrv`` (src/mhealth/heart/hrv.py).

Every per-window metric is a WindowFeature computed by the MI355X engine: call it on a
whole RR series (one window), pass it to ``rolling_apply`` (fixed-length windows of
beats) or to ``nonuniform_rolling_apply`` (windows of a fixed duration on the beat time
axis), alone or fused with other features in one list:

* time domain: ``sdnn`` (hrv.py:49-62), ``pnn50`` / ``pnnx`` (hrv.py:111-135),
  ``rmssd`` (hrv.py:138-146), ``ssd`` (hrv.py:149-157), ``sdsd`` (hrv.py:160-169);
* Poincare / Lorenz: ``csi_sd1``, ``csi_sd2``, ``lorenz_csi``, ``lorenz_cvi``,
  ``lorenz_mcsi`` (hrv.py:207-266), with the ``factor`` argument;
* frequency domain, with the reference's signatures on a PSD the caller computed:
  ``power_band(psd, freqs, lower, upper)``, ``relative_power_band`` and
  ``peak_frequency`` (hrv.py:173-198; pymhealth_amd.spectrum, one lane per psd row).
  The window-level forms (periodogram of each window on chip) are
  ``features.band_power(fs, lo, hi)`` / ``features.relative_band_power``.

``sdann`` / ``sdnni`` (hrv.py:65-108) do not run in the reference: numba cannot type the
module-level ``nonuniform_rolling_apply`` closures they call (TypingError "Untyped
global name '_window_mean'", recorded by tests/golden/make_golden.py). Here they do
what their docstrings say — the std / mean over 5-minute segments of the per-segment
mean / std — with the reference's building blocks (pinned individually): the segment
values come from ``nonuniform_rolling_apply`` and the final ``.std()`` / ``.mean()``
are numba's array_std / array_mean of that float32 array, computed on the GPU.
"""
import numpy as np

from ..feature import td_factor  # noqa: F401
from ..features import (band_power, csi_sd1, csi_sd2, lorenz_csi, lorenz_cvi,  # noqa: F401
                        lorenz_mcsi, mean32, pnn50, pnnx, relative_band_power, rms, rmssd,
                        sdnn, sdsd, ssd, std32)
from ..spectrum import power_band, relative_power_band  # noqa: F401
from ..spectrum import hrv_peak_frequency as peak_frequency  # noqa: F401
from ..util.windows import nonuniform_rolling_apply


def nni_to_ms(nni, current_unit="ns"):
    """hrv.nni_to_ms (hrv.py:38-40)."""
    return td_factor(current_unit) * nni.astype(float) / 1e6


def nni_cumulative(nni):
    """hrv.nni_cumulative (hrv.py:43-45)."""
    return np.cumsum(nni)


def _segment_index(nni, index, unit, what):
    if index is None:
        if unit is None:
            raise ValueError("index or unit must be specified" if what == "sdann"
                             else "index or interval_unit must be specified")
        index = nni_cumulative(np.asarray(nni)) * td_factor(unit)
    index = np.asarray(index)
    if index.dtype.kind == "M":
        index = index.astype("datetime64[ns]").view(np.int64)
    return index.astype(np.int64)


def sdann(nni, index=None, interval=60 * 5, unit=None):
    """Std of the per-segment mean NN interval over segments of ``interval`` seconds
    (hrv.py:65-85): index in ns (or cumulative nni in ``unit``)."""
    index = _segment_index(nni, index, unit, "sdann")
    interval = interval * 1e9
    seg = nonuniform_rolling_apply(np.mean)(index, nni, interval, interval)
    return std32(seg)


def sdnni(nni, index=None, interval=60 * 5, unit=None):
    """Mean of the per-segment std of NN intervals over segments of ``interval``
    seconds (hrv.py:88-108)."""
    index = _segment_index(nni, index, unit, "sdnni")
    interval = interval * 1e9
    seg = nonuniform_rolling_apply(np.std)(index, nni, interval, interval)
    return mean32(seg)


__all__ = ["sdnn", "sdann", "sdnni", "pnn50", "pnnx", "rmssd", "ssd", "sdsd", "csi_sd1",
           "csi_sd2", "lorenz_csi", "lorenz_cvi", "lorenz_mcsi", "power_band",
           "relative_power_band", "peak_frequency", "band_power", "relative_band_power", "rms",
           "td_factor", "nni_to_ms", "nni_cumulative"]
