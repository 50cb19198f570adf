"""Drop-in for ``mhealth.generic.information`` (src/mhealth/generic/information.py).

``entropy(x)`` (information.py:10-20) keeps both of the reference's uses: called on an
array (a PSD or any counts / probabilities, float32 / float64, 1-D or row-wise 2-D) it
runs ``mhf_psd_features``; passed to ``rolling_apply`` it is the per-window feature
``MHF_ENTROPY`` of the window's own samples (generic kernel, one fused launch). The
entropy of each window's on-chip periodogram is ``spectral_entropy(fs)``. ``sampen``
(information.py:23-113) is the per-window sample entropy (pairwise kernel); bind
``mm`` / ``r`` / ``sd`` with ``functools.partial(sampen, mm=3, r=0.15)``.
"""
from ..features import entropy, sampen, spectral_entropy  # noqa: F401

__all__ = ["entropy", "sampen", "spectral_entropy"]
