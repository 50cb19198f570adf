"""Drop-in for ``mhealth.generic``."""
from . import filters, frequency, information, rqa, stats, timedom  # noqa: F401
