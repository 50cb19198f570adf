"""Drop-in for ``mhealth.generic``."""
from . import filters, frequency, information, stats, timedom  # noqa: F401
