"""Drop-in for ``mhealth.fft`` (src/mhealth/fft/__init__.py, _fft.py:18-58): ``fft`` /
``ifft`` of complex128 data on the MI355X (``mhf_fft``, pymhealth_amd/csrc/fft.hip).

The reference's ``fft(a)`` is FFTW's unnormalised forward DFT of ``a.astype(complex128)``
(a cffi call, ``fftw_fft(n, in, out, FFTW_FORWARD)``, _fftw_binder.py:11-17) and
``ifft(a)`` the backward one divided by ``a.shape[0]``; without the compiled binder it
falls back to ``numpy.fft.fft`` / ``ifft`` — the same transforms. Here both run as fp64
device FFTs (radix-2 in LDS / global passes for powers of two, Bluestein otherwise).

numpy input returns a complex128 numpy array, a torch tensor returns a complex128 tensor
on its own device (a CPU tensor is transformed on the GPU and handed back on the CPU).
1-D arrays as in the reference; a 2-D array is transformed row by row along its last axis (numpy's convention; the reference's FFTW call is 1-D only). The
reference's ``@overload(np.fft.fft)`` (_fft.py:51-58) only makes ``np.fft.fft`` callable
inside numba-compiled code; there is no numba here, so it has no counterpart.
"""
import numpy as np

from . import _lib

FFTW_FORWARD = -1
FFTW_BACKWARD = 1


def _call(a, direction, inverse):
    import torch
    from .engine import fft as dev_fft
    is_torch = isinstance(a, torch.Tensor)
    if not is_torch:
        a = np.asarray(a)
    n = a.shape[-1] if a.ndim else 0
    out = dev_fft(a, direction, (1.0 / n) if (inverse and n) else 1.0)
    if is_torch:
        return out if out.device == a.device else out.to(a.device)
    return out.cpu().numpy()


def fft(a):
    """Unnormalised forward DFT, X_k = sum_j a_j exp(-2 pi i jk / n) (_fft.py:18-28)."""
    return _call(a, _lib.MHF_FFT_FORWARD, False)


def ifft(a):
    """Inverse DFT: the unnormalised backward transform divided by n (_fft.py:31-48)."""
    return _call(a, _lib.MHF_FFT_BACKWARD, True)


__all__ = ["fft", "ifft"]
