"""Drop-in for ``mhealth.heart.qrs`` peak functions (src/mhealth/heart/qrs.py:200-220):
the peak-count window feature (``len(nb_find_peaks(x))``) and the array forms
``find_peaks`` / ``nb_find_peaks`` — the ascending indices of strict local maxima, found by
one stream-compaction launch sequence (``mhf_find_peaks``). The Pan-Tompkins /
Hamilton-Tompkins detectors (qrs.py:12-197) are sequential state machines, out of scope
(DESIGN.md §8)."""
import operator

import numpy as np

from .. import _lib
from ..features import peak_count  # noqa: F401


def _peaks(x, comp=_lib.MHF_CMP_GREATER):
    import torch
    from ..engine import find_peaks as fp
    out = fp(x, comp)
    return out if isinstance(x, torch.Tensor) else out.cpu().numpy()


_COMPARISONS = {np.greater: _lib.MHF_CMP_GREATER, np.greater_equal: _lib.MHF_CMP_GREATER_EQUAL,
                np.less: _lib.MHF_CMP_LESS, np.less_equal: _lib.MHF_CMP_LESS_EQUAL,
                operator.gt: _lib.MHF_CMP_GREATER, operator.ge: _lib.MHF_CMP_GREATER_EQUAL,
                operator.lt: _lib.MHF_CMP_LESS, operator.le: _lib.MHF_CMP_LESS_EQUAL}


def find_peaks(x, comp=np.greater):
    """Indices i of x with comp(x[i], x[i-1]) and comp(x[i], x[i+1]) (qrs.py:200-212),
    ascending int64; comp one of np.greater (default: strict maxima), np.greater_equal,
    np.less (minima), np.less_equal, or their ``operator`` forms."""
    try:
        code = _COMPARISONS[comp]
    except (KeyError, TypeError):
        raise TypeError("find_peaks: comp must be np.greater, np.greater_equal, np.less or "
                        "np.less_equal (got %r)" % (comp,)) from None
    return _peaks(x, code)


def nb_find_peaks(x):
    """Indices of strict local maxima (qrs.py:215-220)."""
    return _peaks(x)


__all__ = ["peak_count", "find_peaks", "nb_find_peaks"]
