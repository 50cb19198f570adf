"""Drop-in for ``mhealth.inertial.accelerometer`` preprocessing (§8f N2):
``linear_filter`` / ``gravity_filter`` (accelerometer.py:77-183) filter every axis of an
(N, C) record in ONE ``mhf_filtfilt`` call (the reference loops over columns), and
``magnitude`` (accelerometer.py:198-225) is one elementwise kernel over the AoS record.
float32 samples; filtered outputs are float64 like the reference's ``np.zeros(acc.shape)``.
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


__all__ = ["linear_filter", "gravity_filter", "magnitude"]
