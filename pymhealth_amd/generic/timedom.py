"""Drop-in for ``mhealth.generic.timedom`` (src/mhealth/generic/timedom.py):
time-domain per-window features as MI355X WindowFeatures.

``zero_crossing_count(x, th=0)`` keeps the threshold argument; for rolling_apply bind
it with ``functools.partial(zero_crossing_count, th=...)`` (rolling_apply passes one
argument, as in the reference)."""
from ..features import (hjorth_activity, hjorth_complexity, hjorth_mobility,  # noqa: F401
                        line_length, zero_crossing_count)

__all__ = ["zero_crossing_count", "line_length", "hjorth_activity", "hjorth_mobility",
           "hjorth_complexity"]
