"""Drop-in for ``mhealth.heart`` (window features only)."""
from . import hrv, qrs  # noqa: F401
