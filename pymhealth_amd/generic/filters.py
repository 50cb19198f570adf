"""Drop-in for ``mhealth.generic.filters`` (src/mhealth/generic/filters.py): the
Butterworth zero-phase filter. The filter is DESIGNED on the host exactly as the
reference does (``scipy.signal.butter``; ``lfilter_zi`` for the initial state) and
APPLIED on the GPU (``mhf_filtfilt``: both passes, all channels in one call)."""
import numpy as np


def design(cutoff, freq, order=5, ftype="highpass"):
    """(b, a, zi) of the reference's butterworth (filters.py:31-35)."""
    from scipy import signal
    nyq = 0.5 * freq
    if np.size(cutoff) == 1:
        Wn = cutoff / nyq
    else:
        Wn = [c / nyq for c in cutoff]
    b, a = signal.butter(order, Wn, ftype)
    return b, a, signal.lfilter_zi(b, a)


def filtfilt_device(arr, b, a, zi):
    """filtfilt of a float32 1-D/2-D array or CUDA tensor; numpy in -> float64 numpy out,
    tensor in -> float64 tensor out."""
    import torch
    from ..engine import filtfilt, to_device
    is_torch = isinstance(arr, torch.Tensor)
    t = to_device(arr if is_torch else np.asarray(arr))
    y = filtfilt(t, b, a, zi)
    return y if is_torch else y.cpu().numpy()


def butterworth(arr, cutoff, freq, order=5, ftype="highpass"):
    """Zero-phase Butterworth filter of ``arr`` (filters.py:8-35): scipy.signal.filtfilt
    of the ``order``-th order ``ftype`` filter with critical frequency ``cutoff`` (Hz; a
    (low, high) pair for 'bandpass') at sampling frequency ``freq``. float32 input,
    float64 output (the reference's filtfilt result)."""
    b, a, zi = design(cutoff, freq, order, ftype)
    return filtfilt_device(arr, b, a, zi)


__all__ = ["butterworth", "design"]
