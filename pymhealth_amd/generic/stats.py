"""Drop-in for ``mhealth.generic.stats`` (src/mhealth/generic/stats.py): the per-window
statistical moments, as MI355X WindowFeatures. ``mean/var/std`` stay numpy's own
functions, exactly as the reference aliases them (stats.py:156-163), so passing them to
``rolling_apply`` selects the reference's parfor numerics."""
import numpy as np

from ..features import (coeff_var, drange, interquartile_range, kurtosis,  # noqa: F401
                        kurtosis_excess, mode, skewness)

absolute = np.absolute
mean = np.mean
median = np.median
std = np.std
var = np.var
dmin = np.min
dmax = np.max
percentile = np.percentile

__all__ = ["skewness", "kurtosis", "kurtosis_excess", "drange", "coeff_var", "mean", "std",
           "var", "median", "percentile", "interquartile_range", "mode", "dmin", "dmax",
           "absolute"]
