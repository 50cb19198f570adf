"""Drop-in for the peak-count feature of ``mhealth.heart.qrs``
(``len(nb_find_peaks(x))``, src/mhealth/heart/qrs.py:215-220)."""
from ..features import peak_count  # noqa: F401

__all__ = ["peak_count"]
