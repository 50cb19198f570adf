"""The reference's PSD-level feature functions, on spectra the caller computed.

In the reference these take ONE 1-D array and are called by user code on a PSD it
computed itself:

    hrv.power_band(psd, freqs, lower=None, upper=None)          heart/hrv.py:173-179
    hrv.relative_power_band(psd, freqs, lower=None, upper=None) heart/hrv.py:192-198
    hrv.peak_frequency(psd, freqs, lower=None, upper=None)      heart/hrv.py:182-189
    density.peak_frequency(psd, freqs, lower=None, upper=None)  generic/frequency/density.py:17-32
    information.entropy(x)                                      generic/information.py:10-20

Here each keeps that signature and runs ``mhf_psd_features`` (include/mhfeat.h): one
lane per row, numba's sequential reductions in the row's dtype (float32 / float64), so a
1-D call returns the reference's float bit for bit (entropy: last-bit libm log). A 2-D
``(rows, bins)`` psd is evaluated row by row in one launch and returns one value per row
(numpy in, numpy out; a CUDA tensor in, a CUDA tensor out). Where the reference raises
(0/0 relative power, arg max of an empty range) the value is NaN. A bound given as NaN
is read as None.
"""
import ctypes
import math

import numpy as np

from . import _lib


def _as_device(a, name):
    import torch
    if isinstance(a, torch.Tensor):
        t = a
    else:
        arr = np.asarray(a)
        if arr.dtype.kind in "iub":
            arr = arr.astype(np.float64)      # numba: int / int sum -> float64 quotients
        t = torch.from_numpy(np.ascontiguousarray(arr))
    if t.dtype not in (torch.float32, torch.float64):
        if t.dtype.is_floating_point or t.dtype.is_complex:
            raise TypeError("%s must be float32 or float64 (got %s)" % (name, t.dtype))
        t = t.to(torch.float64)
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to("cuda")
    return t


def psd_features(psd, freqs, ops, lower=None, upper=None, stream=None):
    """``mhf_psd_features``: the PSD-level functions ``ops`` (``_lib.MHF_PSD_*`` ids) of
    every row of ``psd`` ((bins,) or (rows, bins), float32/float64, numpy or CUDA tensor)
    against ``freqs`` ((bins,), may be None for entropy only). Returns a
    (len(ops), rows) float64 CUDA tensor."""
    import torch
    p = _as_device(psd, "psd")
    if p.dim() == 1:
        p = p.unsqueeze(0)
    if p.dim() != 2:
        raise ValueError("psd must be 1-D (bins,) or 2-D (rows, bins)")
    if p.stride(1) != 1:
        p = p.contiguous()
    rows, bins = p.shape
    f = None
    if freqs is not None:
        f = _as_device(freqs, "freqs").to(p.device).contiguous()
        if f.dim() != 1:
            raise ValueError("freqs must be 1-D")
        if f.shape[0] != bins:
            # numba: psd[mask] with a mask of another length is an IndexError
            raise IndexError("freqs has %d values for %d psd bins" % (f.shape[0], bins))
    ids = np.ascontiguousarray(np.asarray(list(ops), dtype=np.int32))
    out = torch.empty((len(ids), rows), dtype=torch.float64, device=p.device)
    if rows == 0:
        return out
    if stream is None:
        stream = torch.cuda.current_stream(p.device).cuda_stream
    nan = math.nan
    with torch.cuda.device(p.device):
        rc = _lib.lib().mhf_psd_features(
            ctypes.c_void_p(p.data_ptr()),
            _lib.MHF_DTYPE_F64 if p.dtype == torch.float64 else _lib.MHF_DTYPE_F32,
            rows, bins, p.stride(0) if rows > 1 else bins,
            None if f is None else ctypes.c_void_p(f.data_ptr()),
            _lib.MHF_DTYPE_F64 if f is None or f.dtype == torch.float64 else _lib.MHF_DTYPE_F32,
            ids.ctypes.data, len(ids), nan if lower is None else float(lower),
            nan if upper is None else float(upper), ctypes.c_void_p(out.data_ptr()), rows,
            _lib.cstream(stream, p, f, out))
    _lib.check(rc)
    return out


_WINDOW_FORMS = {
    _lib.MHF_PSD_POWER_BAND: "features.band_power(fs, lower, upper)",
    _lib.MHF_PSD_REL_POWER_BAND: "features.relative_band_power(fs, lower, upper)",
    _lib.MHF_PSD_PEAK_FREQUENCY: "features.dominant_frequency(fs, lower, upper)",
    _lib.MHF_PSD_PEAK_FREQUENCY_HRV: "features.dominant_frequency(fs, lower, upper)",
}


def _call(op, psd, freqs, lower, upper):
    import torch
    is_torch = isinstance(psd, torch.Tensor)
    nd = psd.dim() if is_torch else np.ndim(psd)
    if nd == 0 and op in _WINDOW_FORMS:
        # round-1 callers built window features as power_band(fs, lo, hi); the reference
        # signature takes a PSD array (hrv.py:173-198)
        raise TypeError("%s takes a PSD array (psd, freqs, lower, upper) as in the reference; "
                        "the per-window feature for rolling_apply is %s"
                        % ({v: k for k, v in (("power_band", _lib.MHF_PSD_POWER_BAND),
                                                ("relative_power_band", _lib.MHF_PSD_REL_POWER_BAND),
                                                ("peak_frequency", _lib.MHF_PSD_PEAK_FREQUENCY),
                                                ("peak_frequency", _lib.MHF_PSD_PEAK_FREQUENCY_HRV))}[op],
                           _WINDOW_FORMS[op]))
    r = psd_features(psd, freqs, [op], lower, upper)[0]
    if nd == 1:
        return float(r[0].item())
    return r if is_torch else r.cpu().numpy()


def power_band(psd, freqs, lower=None, upper=None):
    """hrv.power_band (heart/hrv.py:173-179): sum |psd| over lower <= freqs <= upper
    (both inclusive; None = np.min / np.max(freqs))."""
    return _call(_lib.MHF_PSD_POWER_BAND, psd, freqs, lower, upper)


def relative_power_band(psd, freqs, lower=None, upper=None):
    """hrv.relative_power_band (heart/hrv.py:192-198): power_band / sum |psd| (NaN where
    the reference raises ZeroDivisionError)."""
    return _call(_lib.MHF_PSD_REL_POWER_BAND, psd, freqs, lower, upper)


def hrv_peak_frequency(psd, freqs, lower=None, upper=None):
    """hrv.peak_frequency (heart/hrv.py:182-189) as the reference computes it:
    freqs[argmax(psd[mask])] — the arg max of the MASKED psd indexes the unmasked freqs
    (so for lower > min(freqs) it is not the peak's frequency; density.peak_frequency
    is). NaN where the reference raises (empty mask)."""
    return _call(_lib.MHF_PSD_PEAK_FREQUENCY_HRV, psd, freqs, lower, upper)


def peak_frequency(psd, freqs, lower=None, upper=None):
    """density.peak_frequency (generic/frequency/density.py:17-32): freqs of the first
    arg max of psd[first_index(freqs, lower) : first_index(freqs, upper)] (None = 0 /
    len(psd)); NaN where the reference raises (empty range)."""
    return _call(_lib.MHF_PSD_PEAK_FREQUENCY, psd, freqs, lower, upper)


def entropy_of(x):
    """information.entropy (generic/information.py:10-20) of a whole array (or of each
    row of a 2-D one): p = x / sum(x) + 1e-30, -sum(p ln p), in x's dtype."""
    return _call(_lib.MHF_PSD_ENTROPY, x, None, None, None)


__all__ = ["psd_features", "power_band", "relative_power_band", "hrv_peak_frequency",
           "peak_frequency", "entropy_of"]
