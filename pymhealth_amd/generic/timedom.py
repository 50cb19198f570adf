"""Drop-in for ``mhealth.generic.timedom`` (src/mhealth/generic/timedom.py):
time-domain per-window features as MI355X WindowFeatures.

``zero_crossing_count(x, th=0)`` keeps the threshold argument; for rolling_apply bind
it with ``functools.partial(zero_crossing_count, th=...)`` (rolling_apply passes one
argument, as in the reference)."""
import numpy as np

from ..features import (hjorth_activity, hjorth_complexity, hjorth_mobility,  # noqa: F401
                        line_length, zero_crossing_count)


def _host(t, like):
    import torch
    return t if isinstance(like, torch.Tensor) else t.cpu().numpy()


def gradient(x):
    """Derivative of the input (timedom.py:11-31): out[0] = x[1] - x[0], out[-1] =
    x[-1] - x[-2], out[i] = (x[i+1] - x[i-1]) / 2 (difference in x's dtype, halved in
    float64); float64 array. One elementwise kernel (``mhf_gradient``)."""
    from ..engine import gradient as grad
    return _host(grad(x), x)


def zero_crossings(x, th=0):
    """Whether a zero crossing follows each sample (timedom.py:34-48): samples with
    |x| <= th count as 0, pos = x > 0, out = pos[:-1] ^ pos[1:]; bool array of n - 1.
    One elementwise kernel (``mhf_zero_crossings``)."""
    from ..engine import zero_crossings as zc
    return _host(zc(x, th), x)


__all__ = ["gradient", "zero_crossings", "zero_crossing_count", "line_length",
           "hjorth_activity", "hjorth_mobility", "hjorth_complexity"]
