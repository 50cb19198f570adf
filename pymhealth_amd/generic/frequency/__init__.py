from . import density  # noqa: F401
