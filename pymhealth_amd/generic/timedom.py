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


def _var(a):
    """numba's serial np.var of a whole array in its own dtype (array_var: float32 for a
    float32 array, float64 otherwise) — one window of the engine's var32 feature."""
    import torch
    from .. import _lib
    from ..engine import window_features
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(a)))
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to("cuda")
    t = t.reshape(-1)
    n = t.shape[0]
    if n < 1:
        raise ValueError("variance of an empty array")
    v = float(window_features(t, n, n, [_lib.MHF_VAR32])[0, 0, 0].item())
    return np.float32(v) if t.dtype == torch.float32 else np.float64(v)


def hjorth_mobility_derivative(x, deriv):
    """sqrt(var(deriv) / var(x)) with a precomputed first derivative (timedom.py:115-131):
    each np.var in its array's dtype on the device, the quotient and sqrt in numba's type
    promotion (float32 / float32 stays float32)."""
    return float(np.sqrt(_var(deriv) / _var(x)))


def hjorth_complexity_derivatives(x, deriv1, deriv2):
    """hjorth_mobility_derivative(deriv1, deriv2) / hjorth_mobility_derivative(x, deriv1)
    (timedom.py:151-170)."""
    vx, v1, v2 = _var(x), _var(deriv1), _var(deriv2)
    return float(np.sqrt(v2 / v1) / np.sqrt(v1 / vx))


def hjorth_parameters(x):
    """(activity, mobility, complexity) of a signal (timedom.py:173-193): np.var(x),
    hjorth_mobility(x), hjorth_complexity(x) — the same arithmetic as the reference's
    shared-gradient form — from ONE window of the engine (var32, Hjorth mobility and
    complexity in one launch)."""
    from .. import _lib
    from ..engine import to_device, window_features
    t = to_device(x, allow_f64=True)
    if t.dim() != 1:
        raise ValueError("hjorth_parameters: x must be 1-D")
    n = t.shape[0]
    if n < 2:
        raise ValueError("hjorth_parameters needs at least 2 samples (np.gradient)")
    v = window_features(t, n, n, [_lib.MHF_VAR32, _lib.MHF_HJORTH_MOBILITY,
                                  _lib.MHF_HJORTH_COMPLEXITY])[0, :, 0].cpu().tolist()
    return (v[0], v[1], v[2])


__all__ = ["gradient", "zero_crossings", "zero_crossing_count", "line_length",
           "hjorth_activity", "hjorth_mobility", "hjorth_complexity",
           "hjorth_mobility_derivative", "hjorth_complexity_derivatives", "hjorth_parameters"]
