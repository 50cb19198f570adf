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
    scalars, as numba boxes them.

    The kernel takes float32 / float64 / int32 / int64; the other dtypes go through a type
    that holds every value exactly and come back in their own dtype: bool, int8 / int16 and
    uint8 / 16 / 32 as int64, float16 as float32, uint64 as int64 with the top bit flipped
    (x ^ 2^63 keeps the order). numpy arrays and torch tensors alike."""
    import torch
    from ..engine import minmax as dev_minmax
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    back = None
    if t.dtype == torch.uint64:
        t = t.view(torch.int64) ^ _U64_FLIP
        back = "u64"
    elif t.dtype in (torch.bool, torch.int8, torch.int16, torch.uint8, torch.uint16, torch.uint32):
        back = t.dtype
        t = t.to(torch.int64)
    elif t.dtype in (torch.float16, torch.bfloat16):
        back = t.dtype
        t = t.to(torch.float32)
    r = dev_minmax(t).cpu()
    if back == "u64":
        r = (r ^ _U64_FLIP).view(torch.uint64)
    elif back is not None:
        r = r.to(back)
    return (r[0].item(), r[1].item())


_U64_FLIP = -(1 << 63)   # x ^ 2^63 maps uint64 order onto int64 order


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
