"""Drop-in for ``mhealth.util`` (windowing)."""
from . import windows  # noqa: F401
