"""Drop-in for ``mhealth.inertial`` (accelerometer preprocessing, §8f N2)."""
from . import accelerometer  # noqa: F401
