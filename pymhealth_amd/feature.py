"""Per-window feature objects: what ``rolling_apply`` receives as ``func``.

In the reference a feature is any numba-jittable callable ``f(window) -> scalar``
keyed by identity (``rolling_apply``'s ``lru_cache``, windows.py:55). Here each
supported callable resolves to a :class:`WindowFeature` — an ``mhf_feature`` id of
include/mhfeat.h plus its parameters — which the fused HIP kernel computes. The
numpy reductions the reference users pass directly (``np.mean``, ``np.var``,
``np.std``; aliased as ``stats.mean/var/std``, stats.py:156-163) resolve to the ids
that reproduce numba's parfor row semantics (row 0 serial, rows >= 1 swapped).

A WindowFeature is also callable on one window, like the reference functions
(``stats.skewness(x)``); that call runs the same kernel on a single window.
"""
import functools
import math

import numpy as np

from . import _lib


class WindowFeature:
    """One per-window feature: an engine id + parameters.

    ``params`` keys: ``zc_threshold`` (zero crossings), ``fs``, ``band`` (lo, hi),
    ``dom`` (lo, hi) for spectral features.
    """

    def __init__(self, name, fid, ref, doc="", **params):
        self.name = name
        self.fid = int(fid)
        self.params = dict(params)
        self.__wrapped_ref__ = ref
        self.__doc__ = "%s [MI355X kernel; reference: %s]\n\n%s" % (name, ref, doc)

    @property
    def __name__(self):
        return self.name

    def with_params(self, **params):
        p = dict(self.params)
        p.update(params)
        return WindowFeature(self.name, self.fid, self.__wrapped_ref__, "", **p)

    @property
    def spectral(self):
        return self.fid in _lib.SPECTRAL_IDS

    def __call__(self, x, *args, **kwargs):
        """Evaluate on ONE window (the whole of ``x``), on the GPU."""
        f = self
        if args or kwargs:
            f = bind_args(self, args, kwargs)
        from .engine import to_device, window_features
        t = to_device(x)
        if t.dim() != 1:
            raise ValueError("%s(x): x must be 1-D" % self.name)
        n = t.shape[0]
        if n < 1:
            raise ValueError("%s of an empty window" % self.name)
        kw = engine_kwargs([f])
        # a lone window is row 0 of the reference's loop (serial numerics)
        v = window_features(t, n, n, [f.fid], **kw)
        return float(v[0, 0, 0].item())

    def __repr__(self):
        extra = "" if not self.params else " %s" % self.params
        return "<WindowFeature %s%s>" % (self.name, extra)


_BAND_IDS = (_lib.MHF_BAND_POWER, _lib.MHF_REL_BAND_POWER)


def _norm(v):
    return None if v is None else float(v)


def _constraints(f):
    """Engine parameters a feature pins (a launch has one value of each)."""
    c = {}
    p = f.params
    if f.fid == _lib.MHF_ZERO_CROSSINGS:
        c["zc_threshold"] = float(p.get("zc_threshold", 0.0))
    if f.fid == _lib.MHF_PNNX:
        c["pnn_threshold"] = float(p.get("pnn_threshold", 50.0))
    if f.fid in _lib.CSI_IDS:
        c["csi_factor"] = float(p.get("csi_factor", _lib.CSI_FACTOR))
    if f.fid == _lib.MHF_PERCENTILE:
        if p.get("percentile_q") is None:
            raise ValueError("percentile needs q (features.percentile(q))")
        c["percentile_q"] = float(p["percentile_q"])
    if f.fid == _lib.MHF_SAMPEN:
        c["sampen"] = (int(p.get("sampen_m", 2)), float(p.get("sampen_r", 0.2)),
                       _norm(p.get("sampen_sd")))
    if f.fid in _lib.RQA_IDS:
        c["rqa_radius"] = float(p.get("rqa_radius", 0.0))
        if f.fid == _lib.MHF_RQA_ENT:
            c["rqa_minlen"] = int(p.get("rqa_minlen", 2))
    if f.spectral:
        if p.get("fs") is None:
            raise ValueError("%s needs fs (sampling frequency)" % f.name)
        c["fs"] = float(p["fs"])
        if f.fid in _BAND_IDS:
            c["band"] = tuple(_norm(v) for v in p.get("band", (None, None)))
        if f.fid == _lib.MHF_DOMINANT_FREQ:
            c["dom"] = tuple(_norm(v) for v in p.get("dom", (None, None)))
    return c


def plan_groups(feats):
    """Partition features into launches: as few as the parameters allow (one for any
    feature list whose zc threshold, fs, band and dominant-frequency range agree).
    Returns [(indices, engine_kwargs)]."""
    groups = []  # [indices, constraints]
    for j, f in enumerate(feats):
        c = _constraints(f)
        for g in groups:
            if all(g[1].get(k, v) == v for k, v in c.items()):
                g[0].append(j)
                g[1].update(c)
                break
        else:
            groups.append([[j], dict(c)])
    out = []
    for idx, c in groups:
        kw = {"zc_threshold": c.get("zc_threshold", 0.0)}
        for k in ("pnn_threshold", "csi_factor", "percentile_q", "rqa_radius", "rqa_minlen"):
            if k in c:
                kw[k] = c[k]
        if "sampen" in c:
            kw["sampen_m"], kw["sampen_r"], kw["sampen_sd"] = c["sampen"]
        if "fs" in c:
            kw["fs"] = c["fs"]
            kw["band"] = c.get("band", (None, None))
            kw["dom"] = c.get("dom", (None, None))
        out.append((idx, kw))
    return out


def engine_kwargs(feats):
    """Engine parameters of a feature list that fits one launch."""
    groups = plan_groups(feats)
    if len(groups) != 1:
        raise ValueError("features need %d launches (conflicting parameters)" % len(groups))
    return groups[0][1]


def bind_args(feat, args, kwargs):
    """Extra positional/keyword args the reference functions accept
    (``zero_crossing_count(x, th)``, timedom.py:53)."""
    if feat.fid == _lib.MHF_ZERO_CROSSINGS:
        th = kwargs.pop("th", args[0] if args else feat.params.get("zc_threshold", 0.0))
        if kwargs or len(args) > 1:
            raise TypeError("zero_crossing_count(x, th=0) takes one threshold")
        return feat.with_params(zc_threshold=float(th))
    if feat.fid == _lib.MHF_PNNX:
        # pnn50(nni, unit='ms') / pnnx(nni, unit='ms', x=50.) (hrv.py:111-135)
        names = ("unit",) if feat.name == "pnn50" else ("unit", "x")
        if len(args) > len(names) or set(kwargs) - set(names):
            raise TypeError("%s(nni, %s)" % (feat.name, ", ".join(names)))
        vals = dict(zip(names, args))
        vals.update(kwargs)
        unit = vals.get("unit", feat.params.get("unit", "ms"))
        x = float(vals.get("x", feat.params.get("x", 50.0)))
        return feat.with_params(unit=unit, x=x, pnn_threshold=x * 1e6 / td_factor(unit))
    if feat.fid in _lib.CSI_IDS:
        # csi_sd1(rri, factor=1/np.sqrt(2)) and the lorenz_* family (hrv.py:207-266)
        if len(args) > 1 or set(kwargs) - {"factor"}:
            raise TypeError("%s(rri, factor=1/sqrt(2))" % feat.name)
        fac = kwargs.get("factor", args[0] if args else feat.params.get("csi_factor",
                                                                        _lib.CSI_FACTOR))
        return feat.with_params(csi_factor=float(fac))
    if feat.fid == _lib.MHF_SAMPEN:
        # sampen(x, mm=2, r=0.2, sd=None) (information.py:23-24)
        names = ("mm", "r", "sd")
        if len(args) > 3 or set(kwargs) - set(names):
            raise TypeError("sampen(x, mm=2, r=0.2, sd=None)")
        vals = dict(zip(names, args))
        vals.update(kwargs)
        mm = vals.get("mm", feat.params.get("sampen_m", 2))
        if int(mm) != mm or mm < 0:
            raise ValueError("sampen: mm must be a non-negative integer")
        return feat.with_params(sampen_m=int(mm), sampen_r=float(vals.get("r", feat.params.get(
            "sampen_r", 0.2))), sampen_sd=_norm(vals.get("sd", feat.params.get("sampen_sd"))))
    if feat.fid == _lib.MHF_PERCENTILE:
        # np.percentile(a, q)
        if len(args) > 1 or set(kwargs) - {"q"}:
            raise TypeError("percentile(x, q) takes one scalar q")
        q = kwargs.get("q", args[0] if args else feat.params.get("percentile_q"))
        return feat.with_params(percentile_q=_percentile_q(q))
    if args or kwargs:
        raise TypeError("%s takes only the window" % feat.name)
    return feat


def _percentile_q(q):
    q = np.asarray(q, dtype=np.float64)
    if q.ndim != 0:
        raise TypeError("percentile: one scalar q per feature (bind each q separately)")
    q = float(q)
    if not (0.0 <= q <= 100.0):
        raise ValueError("Percentiles must be in the range [0, 100]")
    return q


def td_factor(unit):
    """hrv.td_factor (hrv.py:25-35): nanoseconds per unit."""
    table = {"ns": 1.0, "us": 1e3, "ms": 1e6, "s": 1e9}
    if unit not in table:
        raise ValueError('Unknown unit. Must be: "ns", "us", "ms", or "s"')
    return table[unit]


# numpy reductions passed directly to rolling_apply (parfor-swapped in rows >= 1)
_DIRECT = {}


def _direct(fn, fid, name):
    _DIRECT[fn] = WindowFeature(name, fid, "numpy.%s passed to rolling_apply" % name)


_direct(np.mean, _lib.MHF_MEAN, "mean")
_direct(np.var, _lib.MHF_VAR, "var")
_direct(np.std, _lib.MHF_STD, "std")
_direct(np.min, _lib.MHF_MIN, "min")     # stats.dmin (stats.py:161)
_direct(np.max, _lib.MHF_MAX, "max")     # stats.dmax (stats.py:162)
_direct(np.median, _lib.MHF_MEDIAN, "median")   # stats.median (stats.py:158)
PERCENTILE = WindowFeature("percentile", _lib.MHF_PERCENTILE,
                           "numpy.percentile (stats.percentile, stats.py:163)",
                           "q-th percentile, numba's linear interpolation between order "
                           "statistics (any NaN -> NaN).")
if np.amin is not np.min:
    _direct(np.amin, _lib.MHF_MIN, "min")
if np.amax is not np.max:
    _direct(np.amax, _lib.MHF_MAX, "max")


def resolve(func):
    """Map a reference-style feature callable to a WindowFeature, or raise.

    Unsupported callables raise TypeError: arbitrary Python code has no MI355X kernel
    and this package never evaluates windows on the CPU.
    """
    if isinstance(func, WindowFeature):
        return func
    try:
        if func in _DIRECT:
            return _DIRECT[func]
    except TypeError:
        pass
    if isinstance(func, functools.partial) and isinstance(func.func, WindowFeature):
        return bind_args(func.func, func.args, dict(func.keywords))
    if isinstance(func, functools.partial) and func.func is np.percentile:
        # functools.partial(np.percentile, q=90): the reference needs a jittable wrapper
        # (lambda w: np.percentile(w, 90)); the bound partial is its drop-in
        q = func.keywords.get("q", func.args[0] if func.args else None)
        if q is None or len(func.args) > 1 or set(func.keywords) - {"q"}:
            raise TypeError("functools.partial(np.percentile, q=...) binds exactly q")
        return PERCENTILE.with_params(percentile_q=_percentile_q(q))
    if func is np.percentile:
        raise TypeError("rolling_apply(np.percentile) needs q: pass "
                        "functools.partial(np.percentile, q=...) or features.percentile(q)")
    raise TypeError(
        "rolling_apply: no MI355X kernel for %r. Supported: np.mean, np.var, np.std, np.min, "
        "np.max, np.median and the "
        "WindowFeature objects of pymhealth_amd.features (stats.skewness, stats.kurtosis, "
        "timedom.zero_crossing_count, features.rms, features.band_power(fs, lo, hi), ...)."
        % (func,))


def nan_to_none(v):
    return None if v is None or (isinstance(v, float) and math.isnan(v)) else v
