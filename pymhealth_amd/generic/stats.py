"""Drop-in for ``mhealth.generic.stats`` (src/mhealth/generic/stats.py): the per-window
statistical moments, as MI355X WindowFeatures. ``mean/var/std`` stay numpy's own
functions, exactly as the reference aliases them (stats.py:156-163), so passing them to
``rolling_apply`` selects the reference's parfor numerics."""
import numpy as np

from ..features import (coeff_var, drange, interquartile_range, kurtosis,  # noqa: F401
                        kurtosis_excess, mode, skewness)



def minmax(x):
    """Minimum and maximum of an array looping once (stats.py:12-32): ``(min, max)`` of
    ``x.ravel()`` in x's dtype, with the reference's sequential rule (start from x[0],
    replace only on a strict < / >: a NaN x[0] is both answers, later NaN never win,
    the first of equal values stays). One device reduction (``mhf_minmax``); Python
    scalars, as numba boxes them."""
    from ..engine import minmax as dev_minmax
    r = dev_minmax(x)
    if not isinstance(r, np.ndarray):
        r = r.cpu().numpy()
    return (r[0].item(), r[1].item())


absolute = np.absolute
mean = np.mean
median = np.median
std = np.std
var = np.var
dmin = np.min
dmax = np.max
percentile = np.percentile

__all__ = ["minmax", "skewness", "kurtosis", "kurtosis_excess", "drange", "coeff_var", "mean", "std",
           "var", "median", "percentile", "interquartile_range", "mode", "dmin", "dmax",
           "absolute"]
