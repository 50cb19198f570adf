"""Drop-in for ``mhealth.heart.qrs`` peak functions (src/mhealth/heart/qrs.py:200-220):
the peak-count window feature (``len(nb_find_peaks(x))``) and the array forms
``find_peaks`` / ``nb_find_peaks`` — the ascending indices of strict local maxima, found by
one stream-compaction launch sequence (``mhf_find_peaks``). The Pan-Tompkins /
Hamilton-Tompkins detectors (qrs.py:12-197) are sequential state machines, out of scope
(DESIGN.md §8)."""
import numpy as np

from ..features import peak_count  # noqa: F401


def _peaks(x):
    import torch
    from ..engine import find_peaks as fp
    out = fp(x)
    return out if isinstance(x, torch.Tensor) else out.cpu().numpy()


def find_peaks(x, comp=np.greater):
    """Indices i of x with comp(x[i], x[i-1]) and comp(x[i], x[i+1]) (qrs.py:200-212);
    the default comparison (np.greater) only."""
    if comp is not np.greater:
        raise TypeError("find_peaks: only comp=np.greater has an MI355X kernel")
    return _peaks(x)


def nb_find_peaks(x):
    """Indices of strict local maxima (qrs.py:215-220)."""
    return _peaks(x)


__all__ = ["peak_count", "find_peaks", "nb_find_peaks"]
