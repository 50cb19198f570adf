"""Drop-in for ``mhealth.inertial.accelerometer`` preprocessing (§8f N2):
``linear_filter`` / ``gravity_filter`` (accelerometer.py:77-183) filter every axis of an
(N, C) record in ONE ``mhf_filtfilt`` call (the reference loops over columns), and
``magnitude`` (accelerometer.py:198-225) is one elementwise kernel over the AoS record.
float32 samples; filtered outputs are float64 like the reference's ``np.zeros(acc.shape)``.
``roll`` / ``pitch`` (accelerometer.py:13-75) and ``magnitude_dot`` (:236-259) are
elementwise / reduction kernels (``mhf_orientation``, ``mhf_magnitude_dot``) taking arrays
or scalars, float32 or float64, and the DataFrame forms of the reference.
"""
import numpy as np

from ..generic.filters import design, filtfilt_device


def linear_filter(acc, freq, cutoff=0.5, order=5):
    """Non-gravitational acceleration: high-pass (scalar cutoff) or band-pass ((lo, hi))
    Butterworth, zero phase, per axis (accelerometer.py:78-124)."""
    ftype = "highpass" if np.shape(cutoff) == () else "bandpass"
    b, a, zi = design(cutoff, freq, order, ftype)
    return filtfilt_device(acc, b, a, zi)


def gravity_filter(acc, freq, cutoff=0.5, order=5):
    """Gravitational acceleration: low-pass Butterworth, zero phase, per axis
    (accelerometer.py:142-183)."""
    b, a, zi = design(cutoff, freq, order, "lowpass")
    return filtfilt_device(acc, b, a, zi)


def magnitude(x, y=None, z=None):
    """sqrt(x**2 + y**2 + z**2) per sample, fp32 (accelerometer.py:198-225). Takes the
    three axes, or one (N, 3) array / CUDA tensor."""
    import torch
    from ..engine import magnitude as mag, to_device
    if y is None and z is None:
        xyz = x
    elif isinstance(x, torch.Tensor):
        xyz = torch.stack([x, y, z], dim=1)
    else:
        xyz = np.stack([np.asarray(x), np.asarray(y), np.asarray(z)], axis=1)
    is_torch = isinstance(xyz, torch.Tensor)
    t = to_device(xyz if is_torch else np.asarray(xyz))
    out = mag(t)
    return out if is_torch else out.cpu().numpy()


def _host_out(t, like_torch, scalar):
    if like_torch:
        return t
    v = t.cpu().numpy()
    return float(v[0]) if scalar else v


def _is_df(v):
    return type(v).__name__ == "DataFrame"


def _angles(which, args):
    import torch
    like_torch = any(isinstance(a, torch.Tensor) for a in args)
    scalar = all(np.ndim(a) == 0 for a in args if not isinstance(a, torch.Tensor)) and not like_torch
    from ..engine import orientation
    from .. import _lib
    out = orientation(_lib.MHF_ROLL if which == "roll" else _lib.MHF_PITCH,
                      *([None] + list(args) if which == "roll" else args))
    return _host_out(out, like_torch, scalar)


def roll(y, z=None, ycol="y", zcol="z"):
    """Angular roll from gravitational acceleration, degrees: arctan2(y, z) * 180 / pi
    (accelerometer.py:13-26); a DataFrame returns a pd.Series named 'roll' (:29-42)."""
    if _is_df(y):
        import pandas as pd
        return pd.Series(roll(y[ycol].values, y[zcol].values), name="roll")
    return _angles("roll", (y, z))


def pitch(x, y=None, z=None, xcol="x", ycol="y", zcol="z"):
    """Angular pitch, degrees: arctan2(-x, sqrt(y*y + z*z)) * 180 / pi
    (accelerometer.py:45-58); a DataFrame returns a pd.Series named 'pitch' (:61-75)."""
    if _is_df(x):
        import pandas as pd
        return pd.Series(pitch(x[xcol].values, x[ycol].values, x[zcol].values), name="pitch")
    return _angles("pitch", (x, y, z))


def magnitude_dot(x, y=None, z=None, xcol="x", ycol="y", zcol="z"):
    """sqrt(x.x + y.y + z.z) of three acceleration arrays, one float
    (accelerometer.py:236-259; DataFrame form :262-265)."""
    import torch
    from ..engine import magnitude_dot as mdot
    if _is_df(x):
        return magnitude_dot(x[xcol].values, x[ycol].values, x[zcol].values)
    out = mdot(x, y, z)
    return out if isinstance(x, torch.Tensor) else float(out.cpu().numpy()[0])


__all__ = ["linear_filter", "gravity_filter", "magnitude", "roll", "pitch", "magnitude_dot"]
