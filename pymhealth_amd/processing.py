"""``mhealth.processing`` — windowing entry points (the north star's namespace; in the
reference they live in ``mhealth.util.windows``)."""
from .util.windows import array_shape, rolling_apply, view  # noqa: F401

__all__ = ["rolling_apply", "view", "array_shape"]
