"""Drop-in for ``mhealth.generic``."""
from . import frequency, information, stats, timedom  # noqa: F401
