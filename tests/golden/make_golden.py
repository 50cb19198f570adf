#!/usr/bin/env python3
"""Generate the golden parity fixtures from the REFERENCE itself (pymhealth @ 2025-03-07).

Test infrastructure only. This script is the provenance of every ``tests/golden/*.npz``
fixture: it imports the reference's own ``mhealth`` package from ``/root/reference/src``
under numba 0.54.1 (``/opt/conda/bin/python3.9`` in the build container) and records
inputs + the reference's outputs. It never runs on the GPU box and nothing in the
product imports it.

Run (build container only)::

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src \
        /opt/conda/bin/python3.9 tests/golden/make_golden.py tests/golden

numba 0.54.1 refuses to import next to numpy 1.26 (version gate, ABI-incompatible
``_internal`` ufunc extension, removed ``np.MachAr``); the in-memory shim below fixes
that without touching anything on disk. ``vectorize``/``guvectorize``
stay unusable, which only affects ``mhealth.location`` (off the hot path).

What is pinned (reference file:line):
  * ``rolling_apply`` semantics: nw formula, float64 output, row 0 serial / rows>=1
    prange (``src/mhealth/util/windows.py:54-95``), list dispatch (``:98-107``).
  * per-window features H4-H10/H15: ``np.mean/np.var/np.std`` passed
    directly, ``stats.skewness/kurtosis/kurtosis_excess/drange``
    (``generic/stats.py:12-45,97-139``), ``timedom.zero_crossing_count/line_length``
    (``generic/timedom.py:34-78``), RMS in the ``hrv.rmssd`` form
    (``heart/hrv.py:138-146`` without ``np.diff``), peak count ``len(qrs.nb_find_peaks)``
    (``heart/qrs.py:215-220``), ``np.var`` inside a function (``timedom.hjorth_activity``,
    ``generic/timedom.py:81-94``).
  * spectral features H12-H14 on fp64 periodogram rows (numpy.fft is the reference's own
    fallback FFT, ``src/mhealth/fft/__init__.py:3-7``): ``hrv.power_band``,
    ``hrv.relative_power_band`` (``heart/hrv.py:173-198``), ``information.entropy``
    (``generic/information.py:10-20``), ``density.peak_frequency``
    (``generic/frequency/density.py:9-32``).
"""
import hashlib
import os
import sys
import types

import numpy as np

# ---------------------------------------------------------------- numba shim (in memory)
_m = types.ModuleType("numba.np.ufunc._internal")
_m.PyUFunc_None, _m.PyUFunc_Zero, _m.PyUFunc_One, _m.PyUFunc_ReorderableNone = -1, 0, 1, -2


class _DUFunc:  # placeholder type; DUFunc is never instantiated on the hot path
    pass


def _fromfunc(*a, **k):
    raise RuntimeError("numba ufunc builder unavailable under the shim")


_m._DUFunc, _m.fromfunc = _DUFunc, _fromfunc
sys.modules["numba.np.ufunc._internal"] = _m
np.MachAr = type("MachAr", (), {})
_real_version, np.__version__ = np.__version__, "1.20.3"
import numba  # noqa: E402
np.__version__ = _real_version

from numba import njit  # noqa: E402
from mhealth.util.windows import (get_indices, indices_rolling_apply,  # noqa: E402
                                  nonuniform_rolling_apply, rolling_apply)
from mhealth.generic import stats, timedom, information, rqa  # noqa: E402
from mhealth.generic.frequency import density  # noqa: E402
from mhealth.heart import hrv, qrs  # noqa: E402


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ------------------------------------------------------------------- window features
# name -> callable handed to the reference's rolling_apply exactly as a user would.
def _rms(w):
    return np.sqrt(np.mean(np.square(w)))


def _peaks(w):
    return len(qrs.nb_find_peaks(w))


def _zc_th(w):
    return timedom.zero_crossing_count(w, 0.05)


def _var_in_fn(w):
    return timedom.hjorth_activity(w)


def _std_in_fn(w):
    return np.std(w)


def _mean_in_fn(w):
    return np.mean(w)


FEATURES = {
    "mean": np.mean,
    "var": np.var,
    "std": np.std,
    "skewness": stats.skewness.py_func,       # @jit features need .py_func
    "kurtosis": stats.kurtosis.py_func,
    "kurtosis_excess": stats.kurtosis_excess,
    "drange": stats.drange,
    "zero_crossing_count": timedom.zero_crossing_count.py_func,
    "zero_crossing_count_th0.05": _zc_th,
    "line_length": timedom.line_length.py_func,
    "rms": _rms,
    "peak_count": _peaks,
    "hjorth_activity": _var_in_fn,
    "std_in_fn": _std_in_fn,
    "mean_in_fn": _mean_in_fn,
}


def _edge_signal(W, nwin, rng):
    """Hand-built windows that exercise every corner the reference has."""
    rows = []
    rows.append(np.zeros(W))                                  # all zero
    rows.append(np.full(W, 3.25))                             # constant -> skew/kurt 0
    rows.append(np.full(W, -0.0))                             # negative zero
    r = rng.standard_normal(W); r[W // 3] = np.nan; rows.append(r)          # NaN
    r = rng.standard_normal(W); r[::7] = 0.0; rows.append(r)  # exact zeros (zc threshold)
    r = np.repeat(rng.standard_normal(W // 4 + 1), 4)[:W]; rows.append(r)  # plateaus
    r = np.tile([0.0, 1.0, 0.0, -1.0], W // 4 + 1)[:W]; rows.append(r)     # alternating
    r = np.tile([1.0, 1.0, 2.0, 2.0, 1.0], W // 5 + 1)[:W]; rows.append(r)  # flat-top peaks
    r = rng.standard_normal(W) * 1e-20; rows.append(r)        # tiny (subnormal cubes)
    r = rng.standard_normal(W) * 1e15 + 1e17; rows.append(r)  # huge offset
    r = 9.81 + 0.01 * rng.standard_normal(W); rows.append(r)  # gravity offset
    r = np.full(W, 0.05); r[::2] = -0.05; rows.append(r)      # exactly at +-threshold
    r = rng.standard_normal(W); r[5] = np.inf; rows.append(r)  # inf
    while len(rows) < nwin:
        rows.append(rng.standard_normal(W) * rng.uniform(0.1, 10) + rng.uniform(-5, 5))
    return np.concatenate(rows[:nwin]).astype(np.float32)


def _per_window(f, x, W, S):
    """Evaluate window by window when the reference raises somewhere in the prange.

    Each window is placed in row 1 of a two-window array so it is evaluated by the
    prange body exactly as in the full call (row 0 is serial, ``windows.py:87``)."""
    nw = max(0, 1 + (len(x) - W) // S)
    out = np.zeros(nw)
    raises = np.zeros(nw, np.bool_)
    g = rolling_apply(f, W, W)
    benign = np.linspace(-1.0, 1.0, W).astype(x.dtype)   # raises in no feature
    for i in range(nw):
        w = x[i * S:i * S + W]
        try:
            if i == 0:
                out[i] = g(np.concatenate([w, benign]))[0]
            else:
                out[i] = g(np.concatenate([benign, w]))[1]
        except (ZeroDivisionError, SystemError):
            out[i] = np.nan
            raises[i] = True
    return out, raises


def _moment_case(name, x, W, S, out, feats=FEATURES, probe=False):
    """Run every feature through the reference's rolling_apply.

    numba scalar division raises ZeroDivisionError where IEEE gives inf/nan (a
    feature compiled with the 'python' error model, e.g. ``kurtosis`` called from
    ``kurtosis_excess`` on a window whose variance squares to 0). Inside the prange
    such an exception either propagates (SystemError) or is silently dropped, leaving
    the rest of that thread's chunk as the zeros ``np.zeros`` put there
    (``windows.py:89``). ``probe=True`` evaluates window by window so those rows are
    flagged in ``raises_<feature>`` (NaN in the fixture) instead of pinned to garbage.
    """
    rec = {"x": x, "wsize": np.int64(W), "wstep": np.int64(S)}
    for fname, f in feats.items():
        try:
            full = rolling_apply(f, W, S)(x)
        except (ZeroDivisionError, SystemError):
            full = None
        if probe or full is None:
            per, raises = _per_window(f, x, W, S)
            if raises.any() or full is None:
                rec["out_" + fname], rec["raises_" + fname] = per, raises
                continue
        rec["out_" + fname] = full
    out[name] = rec


def _accel(n, fs, rng):
    t = np.arange(n) / fs
    e = rng.standard_normal((n, 3))
    ax = 0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * e[:, 0]
    ay = 0.2 * np.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * e[:, 1]
    az = 1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2) + 0.05 * e[:, 2]
    return np.stack([ax, ay, az], axis=1).astype(np.float32)


# --------------------------------------------------------------------- spectral oracle
@njit
def _power_band_rows(psd, freqs, lo, hi):
    out = np.zeros(psd.shape[0])
    for i in range(psd.shape[0]):
        out[i] = hrv.power_band(psd[i], freqs, lo, hi)
    return out


@njit
def _entropy_rows(psd):
    out = np.zeros(psd.shape[0])
    for i in range(psd.shape[0]):
        out[i] = information.entropy(psd[i])
    return out


@njit
def _peak_frequency_rows(psd, freqs, lo, hi):
    out = np.zeros(psd.shape[0])
    for i in range(psd.shape[0]):
        out[i] = density.peak_frequency(psd[i], freqs, lo, hi)
    return out


@njit
def _relative_power_band_one(p, freqs, lo, hi):
    return hrv.relative_power_band(p, freqs, lo, hi)


def _spectral_rows(psd, freqs, bp_lo, bp_hi, df_lo, df_hi):
    """Reference features per psd row. A row on which the reference RAISES
    (numba scalar 0/0 -> ZeroDivisionError in relative_power_band on an all-zero psd)
    is recorded as NaN and flagged in ``raises_relative_band_power``."""
    n = psd.shape[0]
    out = np.zeros((n, 4))
    raises = np.zeros(n, np.bool_)
    out[:, 0] = _power_band_rows(psd, freqs, bp_lo, bp_hi)
    for i in range(n):
        try:
            out[i, 1] = _relative_power_band_one(psd[i], freqs, bp_lo, bp_hi)
        except ZeroDivisionError:
            out[i, 1] = np.nan
            raises[i] = True
    out[:, 2] = _entropy_rows(psd)
    out[:, 3] = _peak_frequency_rows(psd, freqs, df_lo, df_hi)
    return out, raises


def periodogram_rows(win, fs):
    """fp64 one-sided periodogram (boxcar, no detrend, density) of each row."""
    W = win.shape[1]
    X = np.fft.rfft(win.astype(np.float64), axis=1)
    psd = (X.real ** 2 + X.imag ** 2) / (fs * W)
    if W % 2:
        psd[:, 1:] *= 2
    else:
        psd[:, 1:-1] *= 2
    return psd


def _spectral_case(name, x, W, S, fs, bp, df, out):
    nw = max(0, 1 + (len(x) - W) // S)
    idx = np.arange(nw)[:, None] * S + np.arange(W)[None, :]
    win = x[idx]
    psd = periodogram_rows(win, fs)
    freqs = np.fft.rfftfreq(W, 1.0 / fs)
    res, raises = _spectral_rows(psd, freqs, bp[0], bp[1], df[0], df[1])
    out[name] = {"x": x, "wsize": np.int64(W), "wstep": np.int64(S), "fs": np.float64(fs),
                 "band": np.array(bp, np.float64), "dom_range": np.array(df, np.float64),
                 "freqs": freqs, "out_band_power": res[:, 0],
                 "out_relative_band_power": res[:, 1], "out_spectral_entropy": res[:, 2],
                 "out_dominant_frequency": res[:, 3],
                 "raises_relative_band_power": raises}


# ------------------------------------------------------- time-indexed (nonuniform) windows
# §8f N1: nonuniform_rolling_apply / get_indices / indices_rolling_apply
# (src/mhealth/util/windows.py:122-249). The feature callables run inside the reference's
# serial @jit loop, so they must be jittable: np.mean/var/std and the @jit features.
NU_FEATURES = {
    "mean": np.mean, "var": np.var, "std": np.std, "skewness": stats.skewness,
    "kurtosis": stats.kurtosis, "zero_crossing_count": timedom.zero_crossing_count,
    "line_length": timedom.line_length,
}


def _nu_case(name, index, x, wsize, wstep, min_len, out, index_ns=None, feats=None):
    rec = {"x": x, "index": np.asarray(index_ns if index_ns is not None else index),
           "min_window_len": np.int64(min_len),
           "indices": get_indices(index, wsize, wstep).astype(np.int64)}
    if isinstance(wsize, np.timedelta64):
        rec["wsize_ns"] = np.int64(wsize.astype("timedelta64[ns]").astype(np.int64))
        rec["wstep_ns"] = np.int64(wstep.astype("timedelta64[ns]").astype(np.int64))
    else:
        rec["wsize"] = np.asarray(wsize)
        rec["wstep"] = np.asarray(wstep)
    for fname, f in (feats or NU_FEATURES).items():
        try:
            rec["out_" + fname] = nonuniform_rolling_apply(f, min_len)(index, x, wsize, wstep)
        except ZeroDivisionError:
            rec["raises_" + fname] = np.bool_(True)
    lst = nonuniform_rolling_apply([np.mean, np.std], min_len)(index, x, wsize, wstep)
    rec["list_mean"], rec["list_std"] = lst
    out[name] = rec


def nonuniform_cases(rng):
    cases = {}
    # integer ns-like index with random gaps, int window/step (short windows -> NaN)
    idx = np.cumsum(rng.integers(1, 20, 3000)).astype(np.int64)
    x = (rng.standard_normal(3000) * 2 + 0.5).astype(np.float32)
    _nu_case("nu_int", idx, x, 60, 40, 3, cases)
    _nu_case("nu_int_min1", idx, x, 25, 25, 1, cases)
    # datetime64[ns] index (RR-interval style timestamps), timedelta64 window and step
    t0 = np.datetime64("2025-03-07T08:00:00", "ns")
    gaps = rng.integers(400, 1300, 2000).astype("timedelta64[ms]")
    didx = t0 + np.cumsum(gaps).astype("timedelta64[ns]")
    rr = (800 + 60 * rng.standard_normal(2000)).astype(np.float32)
    _nu_case("nu_datetime", didx, rr, np.timedelta64(30, "s"), np.timedelta64(15, "s"), 5,
             cases, index_ns=didx.astype(np.int64))
    # float window/step on an int64 ns index (hrv.sdann / sdnni pass interval * 1e9)
    nidx = np.cumsum(rng.integers(600_000_000, 1_100_000_000, 1500)).astype(np.int64)
    rr2 = (900 + 50 * rng.standard_normal(1500)).astype(np.float32)
    _nu_case("nu_float_step", nidx, rr2, 60 * 1e9, 60 * 1e9, 1, cases)
    # a gap with no samples: empty windows (min_len 1 -> NaN)
    gidx = np.concatenate([np.arange(0, 500), np.arange(2000, 2600)]).astype(np.int64)
    gx = rng.standard_normal(gidx.size).astype(np.float32)
    _nu_case("nu_gap", gidx, gx, 100, 50, 1, cases)
    return cases


def nonuniform64_cases(rng):
    """nonuniform_rolling_apply on float64 records (RR intervals as pandas gives them): the
    moment / time-domain set, order statistics (median, IQR, mode) and rmssd, float64 out
    (np.zeros(n, arr.dtype)); ties and a gap (empty windows) included."""
    feats = dict(NU_FEATURES)
    feats.update({"median": np.median, "interquartile_range": stats.interquartile_range,
                  "mode": stats.mode, "rmssd": hrv.rmssd})
    # (the jitted functions: a plain Python function would drop the reference's @jit
    # windows_loop into object mode, i.e. numpy's pairwise sums instead of numba's)
    cases = {}
    t0 = np.datetime64("2025-03-07T08:00:00", "ns")
    gaps = rng.integers(400, 1300, 2000).astype("timedelta64[ms]")
    didx = t0 + np.cumsum(gaps).astype("timedelta64[ns]")
    rr = 800 + 60 * rng.standard_normal(2000)
    rr[::5] = np.round(rr[::5] / 8) * 8                                 # ties
    _nu_case("nu64_datetime", didx, rr, np.timedelta64(30, "s"), np.timedelta64(15, "s"), 5,
             cases, index_ns=didx.astype(np.int64), feats=feats)
    gidx = np.concatenate([np.arange(0, 500), np.arange(2000, 2600)]).astype(np.int64)
    gx = np.round(rng.standard_normal(gidx.size) * 4) / 4
    _nu_case("nu64_gap", gidx, gx, 100, 50, 1, cases, feats=feats)
    return cases


# ----------------------------------------------------- §8f N3 / N4 per-window features
# N3: coeff_var (generic/stats.py:142-153), Hjorth mobility / complexity
# (generic/timedom.py:97-169); N4: HRV time-domain metrics of an RR series
# (heart/hrv.py:111-266) applied to windows (rolling_apply / nonuniform_rolling_apply)
# and to whole records.
def _pnnx20(w):
    return hrv.pnnx(w, 'ms', 20.0)


def _csi_sd1_half(w):
    return hrv.csi_sd1(w, 0.5)


N3_FEATURES = {
    "coeff_var": stats.coeff_var.py_func,
    "hjorth_mobility": timedom.hjorth_mobility.py_func,
    "hjorth_complexity": timedom.hjorth_complexity.py_func,
}
N4_FEATURES = {
    "rmssd": hrv.rmssd.py_func, "sdsd": hrv.sdsd.py_func, "ssd": hrv.ssd.py_func,
    "pnn50": hrv.pnn50.py_func, "pnnx20": _pnnx20, "csi_sd1": hrv.csi_sd1.py_func,
    "csi_sd1_half": _csi_sd1_half, "csi_sd2": hrv.csi_sd2.py_func,
    "lorenz_csi": hrv.lorenz_csi.py_func, "lorenz_cvi": hrv.lorenz_cvi.py_func,
    "lorenz_mcsi": hrv.lorenz_mcsi.py_func, "sdnn": hrv.sdnn,
}


def _rolling_case(x, W, S, feats):
    rec = {"x": x, "wsize": np.int64(W), "wstep": np.int64(S)}
    for name, f in feats.items():
        try:
            rec["out_" + name] = rolling_apply(f, W, S)(x)
        except ZeroDivisionError:
            rec["raises_" + name] = np.bool_(True)
    return rec


def n3n4_cases(rng):
    cases = {}
    n = 127 * 64 + 128
    t = np.arange(n) / 50.0
    acc = (0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * rng.standard_normal(n)
           + 0.02).astype(np.float32)
    cases["n3_hjorth_w128"] = _rolling_case(acc, 128, 64, N3_FEATURES)
    cases["n3_hjorth_w100"] = _rolling_case(acc[:100 * 90], 100, 100, N3_FEATURES)
    rr = (800 + 40 * np.sin(np.arange(6000) / 30.0)
          + 25 * rng.standard_normal(6000)).astype(np.float32)
    cases["n4_hrv_w64"] = _rolling_case(rr, 64, 16, N4_FEATURES)
    cases["n4_hrv_w300"] = _rolling_case(rr, 300, 300, N4_FEATURES)
    # whole-record calls of the jit functions themselves
    whole = {"x": rr[:2000], "x3": acc[:1000]}
    for name, f in N4_FEATURES.items():
        g = getattr(hrv, name, None)
        whole["val_" + name] = np.float64(g(rr[:2000]) if g is not None else f(rr[:2000]))
    for name in N3_FEATURES:
        mod = stats if name == "coeff_var" else timedom
        whole["val_" + name] = np.float64(getattr(mod, name)(acc[:1000]))
    cases["n4_whole"] = whole
    # RR series on its own time axis: 60-s windows every 30 s (nonuniform_rolling_apply)
    t0 = np.datetime64("2025-03-07T08:00:00", "ns")
    idx = t0 + np.cumsum(rr.astype(np.int64)).astype("timedelta64[ms]").astype("timedelta64[ns]")
    ws, st = np.timedelta64(60, "s"), np.timedelta64(30, "s")
    nu = {"x": rr, "index": idx.astype(np.int64), "wsize_ns": np.int64(60_000_000_000),
          "wstep_ns": np.int64(30_000_000_000), "min_window_len": np.int64(3),
          "indices": get_indices(idx, ws, st).astype(np.int64)}
    for name in ("rmssd", "sdsd", "pnn50", "csi_sd1", "csi_sd2", "lorenz_mcsi"):
        nu["out_" + name] = nonuniform_rolling_apply(getattr(hrv, name), 3)(idx, rr, ws, st)
    cases["nu_hrv"] = nu
    for name in ("sdnni", "sdann"):
        try:
            getattr(hrv, name)(rr.astype(np.float64), idx.astype(np.int64), 60.0)
            print(name, "ran")
        except Exception as e:  # noqa: BLE001 — record how the reference fails
            print(name, "fails in the reference:", type(e).__name__, str(e)[:300])
    return cases


# ------------------------------------------------------------ §8f N2 preprocessing
# generic/filters.py:8-35 butterworth (scipy.signal.butter + filtfilt),
# inertial/accelerometer.py:77-225 linear_filter / gravity_filter / magnitude.
def n2_cases(rng):
    from scipy import signal
    from mhealth.generic.filters import butterworth
    from mhealth.inertial import accelerometer as accm
    n = 6000
    t = np.arange(n) / 50.0
    acc = np.stack([0.3 * np.sin(2 * np.pi * 1.7 * t), 0.2 * np.sin(2 * np.pi * 0.4 * t + 1),
                    1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2)], axis=1)
    acc = (acc + 0.05 * rng.standard_normal((n, 3))).astype(np.float32)
    rec = {"x": acc, "fs": np.float64(50.0)}
    designs = {"hp": (0.5, "highpass"), "lp": (0.5, "lowpass"), "bp": ((0.5, 10.0), "bandpass"),
               "lp8": (3.0, "lowpass")}
    for name, (cut, ftype) in designs.items():
        order = 8 if name == "lp8" else 5
        nyq = 25.0
        wn = cut / nyq if np.size(cut) == 1 else [c / nyq for c in cut]
        b, a = signal.butter(order, wn, ftype)
        rec["b_" + name], rec["a_" + name] = b, a
        rec["zi_" + name] = signal.lfilter_zi(b, a)
        rec["out_" + name] = butterworth(acc[:, 0], cut, 50.0, order, ftype)
    rec["linear"] = accm.linear_filter(acc, 50.0)
    rec["linear_bp"] = accm.linear_filter(acc, 50.0, (0.5, 10.0))
    rec["gravity"] = accm.gravity_filter(acc, 50.0)
    rec["magnitude"] = accm.magnitude(acc[:, 0], acc[:, 1], acc[:, 2])
    return {"n2_filters": rec}


# ------------------------------------------------------------ np.min / np.max (stats.dmin/dmax)
# generic/stats.py:161-162 alias np.min / np.max. Row 0 of rolling_apply runs numba's serial
# array_min/max (numba/np/arraymath.py:471-630: a NaN returns at once); rows >= 1 run
# min/max_parallel_impl (numba/parfors/parfor.py:124-168: from +-inf, builtin min/max,
# which skips NaN). Edge windows put NaN / -0.0 / inf / all-NaN rows at row 0 and later.
def minmax_cases(rng):
    cases = {}
    for W in (128, 100):
        x = _edge_signal(W, 24, rng).astype(np.float64)
        allnan = np.full(W, np.nan); allnan[0] = np.nan
        x = np.concatenate([x[W * 3:W * 4], x, allnan,
                            np.where(np.arange(W) % 2 == 0, -0.0, 0.0),
                            np.where(np.arange(W) % 2 == 0, 0.0, -0.0)]).astype(np.float32)
        cases["minmax_w%d" % W] = _rolling_case(x, W, W, {"min": np.min, "max": np.max,
                                                          "median": np.median})
    x = rng.standard_normal(64 * 40).astype(np.float32)
    x[0] = np.nan                                            # NaN in row 0 and row 1
    cases["minmax_w64_s32"] = _rolling_case(x, 64, 32, {"min": np.min, "max": np.max,
                                                        "median": np.median})
    # np.median (stats.median): odd window, repeated values, NaN rows (numba's quickselect
    # puts a NaN wherever its < comparisons leave it)
    x = np.round(rng.standard_normal(75 * 60) * 3).astype(np.float32)
    x[75 * 4 + 10] = np.nan
    x[75 * 9:75 * 10] = np.nan
    x[75 * 20 + 3] = np.inf
    cases["median_w75_s50"] = _rolling_case(x, 75, 50, {"median": np.median})
    return cases


# --------------------------------------------- PSD-level functions on caller-computed psd
# The reference's hrv.power_band / relative_power_band / peak_frequency (heart/hrv.py:173-198),
# density.peak_frequency (generic/frequency/density.py:9-32) and information.entropy
# (generic/information.py:10-20) called on ONE psd row each, exactly as a user calls them,
# for float64 and float32 rows / freqs and several bound patterns (None = np.min/np.max or
# 0/len). A row on which the reference raises (0/0, argmax of an empty slice) is NaN and
# flagged in raises_<key>.
@njit
def _one_power_band(p, f, lo, hi):
    return hrv.power_band(p, f, lo, hi)


@njit
def _one_rel_power_band(p, f, lo, hi):
    return hrv.relative_power_band(p, f, lo, hi)


@njit
def _one_hrv_peak(p, f, lo, hi):
    return hrv.peak_frequency(p, f, lo, hi)


@njit
def _one_density_peak(p, f, lo, hi):
    return density.peak_frequency(p, f, lo, hi)


@njit
def _one_entropy(p):
    return information.entropy(p)


PSD_BOUNDS = {"none": (None, None), "band": (0.5, 4.0), "empty": (4.0, 0.5),
              "lo_only": (2.0, None), "hi_only": (None, 3.0), "wide": (-1.0, 1e9),
              "edge": (0.25, 8.0)}


def psd_cases(rng):
    W, fs = 256, 64.0
    n = 120
    t = np.arange(W) / fs
    f0 = rng.uniform(0.3, 10.0, n)
    sig = (np.sin(2 * np.pi * f0[:, None] * t) + 0.4 * rng.standard_normal((n, W))
           + rng.uniform(-1, 1, (n, 1)))
    psd = periodogram_rows(sig, fs)
    psd[3] = 0.0                                         # all zero: 0/0, entropy NaN
    psd[4, 40] = np.nan                                  # NaN: arg max stops there
    psd[5] = 1.0                                         # flat: first index wins
    psd[6, 10] = psd[6, 70] = psd[6].max() * 2           # exact tie
    psd[7] = -psd[7]                                     # negative values (|.| sums)
    psd[8, 0] = np.inf
    psd[9] = 1e-300                                      # tiny
    freqs = np.fft.rfftfreq(W, 1.0 / fs)
    cases = {}
    for tag, pdt, fdt in (("f64", np.float64, np.float64), ("f32", np.float32, np.float32),
                          ("f32f64", np.float32, np.float64)):
        P, F = psd.astype(pdt), freqs.astype(fdt)
        rec = {"psd": P, "freqs": F}
        for bname, (lo, hi) in PSD_BOUNDS.items():
            rec["bounds_" + bname] = np.array([np.nan if lo is None else lo,
                                               np.nan if hi is None else hi])
            for key, fn in (("power_band", _one_power_band),
                            ("relative_power_band", _one_rel_power_band),
                            ("hrv_peak_frequency", _one_hrv_peak),
                            ("density_peak_frequency", _one_density_peak)):
                vals = np.zeros(n)
                raises = np.zeros(n, np.bool_)
                for i in range(n):
                    try:
                        vals[i] = fn(P[i], F, lo, hi)
                    except (ZeroDivisionError, ValueError):
                        vals[i], raises[i] = np.nan, True
                rec["out_%s_%s" % (key, bname)] = vals
                rec["raises_%s_%s" % (key, bname)] = raises
        rec["out_entropy"] = np.array([_one_entropy(P[i]) for i in range(n)])
        cases["psd_rows_" + tag] = rec
    # information.entropy on raw sample windows through rolling_apply (a legal reference call)
    x = np.abs(rng.standard_normal(64 * 50)).astype(np.float32)
    x[64 * 3:64 * 4] = 0.0
    x[64 * 5 + 7] = -1.0
    x[64 * 6 + 2] = np.nan
    cases["entropy_w64"] = _rolling_case(x, 64, 64, {"entropy": information.entropy.py_func})
    return cases


# --------------------------------------------- §8f N3: sort-based and O(W^2) features
# stats.interquartile_range (generic/stats.py:48-59: np.percentile(x, [75, 25]) -> numba
# _collect_percentiles, numba/np/arraymath.py:1402-1515), stats.mode (stats.py:62-94: the
# @overload jit version, mode_impl, is what rolling_apply compiles), np.percentile at
# several q through jittable wrappers, information.sampen (information.py:23-113).
def _p0(w):
    return np.percentile(w, 0.0)


def _p12(w):
    return np.percentile(w, 12.5)


def _p33(w):
    return np.percentile(w, 33.0)


def _p50(w):
    return np.percentile(w, 50.0)


def _p90(w):
    return np.percentile(w, 90.0)


def _p100(w):
    return np.percentile(w, 100.0)


def _sampen_m3(w):
    return information.sampen(w, 3, 0.15)


def _sampen_sd(w):
    return information.sampen(w, 2, 0.2, 0.5)


SORT_FEATURES = {"interquartile_range": stats.interquartile_range, "mode": stats.mode,
                 "percentile_0": _p0, "percentile_12.5": _p12, "percentile_33": _p33,
                 "percentile_50": _p50, "percentile_90": _p90, "percentile_100": _p100}
SAMPEN_FEATURES = {"sampen": information.sampen.py_func, "sampen_m3_r0.15": _sampen_m3,
                   "sampen_sd0.5": _sampen_sd}


def _sort_signal(W, nwin, rng):
    rows = [np.zeros(W), np.where(np.arange(W) % 3 == 0, -0.0, 0.0),
            np.where(np.arange(W) % 2 == 0, 0.0, -0.0)]
    r = np.round(rng.standard_normal(W) * 2); r[W // 2] = np.nan; rows.append(r)
    r = np.round(rng.standard_normal(W) * 2); r[W // 3] = np.inf; rows.append(r)
    r = np.round(rng.standard_normal(W) * 2); r[W // 4] = -np.inf; r[-1] = np.inf; rows.append(r)
    r = np.round(rng.standard_normal(W) * 2); r[W // 5] = np.inf; r[W // 2] = np.inf; rows.append(r)
    r = np.full(W, np.nan); rows.append(r)
    rows.append(np.full(W, 7.0))
    rows.append(np.repeat(np.arange(W // 2 + 1, dtype=np.float64), 2)[:W][::-1].copy())
    r = np.round(rng.standard_normal(W)); r[r == 0] = -0.0; rows.append(r)
    while len(rows) < nwin:
        k = len(rows) % 3
        if k == 0:
            rows.append(np.round(rng.standard_normal(W) * rng.uniform(0.5, 6)))
        elif k == 1:
            rows.append(rng.standard_normal(W) * rng.uniform(0.1, 10) + rng.uniform(-5, 5))
        else:
            rows.append(np.round(rng.standard_normal(W) * 3) * 0.25)
    return np.concatenate(rows[:nwin]).astype(np.float32)


def n3_sort_cases(rng):
    cases = {}
    for W, S, nwin in ((64, 64, 60), (100, 37, 60), (256, 256, 40), (7, 3, 200),
                       (1, 1, 30), (2, 1, 40)):
        x = _sort_signal(W, nwin * W // S + 1, rng)[:(nwin - 1) * S + W]
        cases["n3_sort_w%d_s%d" % (W, S)] = _rolling_case(x, W, S, SORT_FEATURES)
    for W, S in ((64, 64), (128, 97), (300, 300)):
        x = (np.sin(np.arange(W * 24) * 0.21) + 0.5 * rng.standard_normal(W * 24)).astype(np.float32)
        x[W * 2:W * 3] = 1.5                                      # constant: no matches -> inf
        x[W * 4:W * 5] = np.round(x[W * 4:W * 5] * 2) / 2         # many exact ties
        cases["n3_sampen_w%d_s%d" % (W, S)] = _rolling_case(x, W, S, SAMPEN_FEATURES)
    return cases


# --------------------------------------------- §8f N3: recurrence quantification (rqa.py)
# Window features through the reference's rolling_apply, each a jittable composition of
# rqa.rq(x, radius) (rqa.py:9-28) with recurrence_rate / determinism / laminarity /
# length_entropy (rqa.py:49-187); plus the matrix-level functions on one record.
def _rqa_rr(w):
    return rqa.recurrence_rate(rqa.rq(w, 0.3))


def _rqa_det(w):
    return rqa.determinism(rqa.rq(w, 0.3))


def _rqa_lam(w):
    return rqa.laminarity(rqa.rq(w, 0.3))


def _rqa_ent(w):
    return rqa.length_entropy(rqa.rq(w, 0.3), 2)


def _rqa_ent3(w):
    return rqa.length_entropy(rqa.rq(w, 0.3), 3)


def _rqa_det0(w):
    return rqa.determinism(rqa.rq(w))


def _rqa_rr0(w):
    return rqa.recurrence_rate(rqa.rq(w))


RQA_FEATURES = {"rqa_recurrence_rate": _rqa_rr, "rqa_determinism": _rqa_det,
                "rqa_laminarity": _rqa_lam, "rqa_length_entropy": _rqa_ent,
                "rqa_length_entropy_min3": _rqa_ent3, "rqa_determinism_r0": _rqa_det0,
                "rqa_recurrence_rate_r0": _rqa_rr0}


def rqa_cases(rng):
    cases = {}
    for W, S in ((64, 64), (100, 37), (33, 33)):
        nw = 40
        x = (np.sin(np.arange((nw - 1) * S + W) * 0.3) + 0.3 * rng.standard_normal(
            (nw - 1) * S + W))
        x = (np.round(x * 8) / 8).astype(np.float32)          # exact ties for radius 0
        x[S * 3:S * 3 + W] = 0.5                                # constant window
        x[S * 5 + 4] = np.nan
        cases["n3_rqa_w%d_s%d" % (W, S)] = _rolling_case(x, W, S, RQA_FEATURES)
    xr = (np.round(np.sin(np.arange(80) * 0.4) * 6) / 6).astype(np.float32)
    r = rqa.rq(xr, 0.2)
    cases["n3_rqa_matrix"] = {
        "x": xr, "rq": r, "rq0": rqa.rq(xr), "recurrence_rate": np.float64(rqa.recurrence_rate(r)),
        "determinism": np.float64(rqa.determinism(r)), "laminarity": np.float64(rqa.laminarity(r)),
        "diagonal_lengths": rqa.diagonal_lengths(r, 2), "vertical_lengths": rqa.vertical_lengths(r, 2),
        "diagonal_lengths3": rqa.diagonal_lengths(r, 3),
        "length_entropy": np.float64(rqa.length_entropy(r, 2))}
    return cases


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(20250307)
    cases = {}

    # cfg1 exactly (10k x 128, N(0,1), seed 0): input regenerated from the seed, sha pinned.
    x1 = np.random.default_rng(0).standard_normal(10_000 * 128).astype(np.float32)
    rec = {"x_sha256": np.array(_sha(x1)), "x_seed": np.int64(0), "n": np.int64(x1.size),
           "wsize": np.int64(128), "wstep": np.int64(128)}
    for fname in ("mean", "var", "skewness", "kurtosis"):
        rec["out_" + fname] = rolling_apply(FEATURES[fname], 128, 128)(x1)
    lst = rolling_apply([FEATURES[f] for f in ("mean", "var", "skewness", "kurtosis")],
                        128, 128)(x1)
    for f, v in zip(("mean", "var", "skewness", "kurtosis"), lst):
        rec["list_" + f] = v
    cases["cfg1"] = rec

    # cfg2 regime: 3-axis accel at 50 Hz, 1 g offset on z, W=S=256; per-axis columns are
    # strided views of the (N,3) AoS array exactly as a reference user would pass them.
    acc = _accel(256 * 384, 50.0, rng)
    for k, ax in enumerate("xyz"):
        _moment_case("accel_" + ax, np.ascontiguousarray(acc[:, k]), 256, 256, cases)
    cases["accel_aos"] = {"x": acc}
    # column view semantics: rolling_apply on acc[:, 2] (non-contiguous) == contiguous
    cases["accel_z_strided"] = {"out_skewness": rolling_apply(
        FEATURES["skewness"], 256, 256)(acc[:, 2])}

    # edge windows at W=128 and W=256 (S=W), plus N(0,1) at W=256 with overlap.
    _moment_case("edge_128", _edge_signal(128, 48, rng), 128, 128, cases, probe=True)
    _moment_case("edge_256", _edge_signal(256, 40, rng), 256, 256, cases, probe=True)
    _moment_case("randn_256_s64", rng.standard_normal(256 * 64).astype(np.float32),
                 256, 64, cases)
    # W=1024 on a 9.81-offset signal (worst skew regime), stride 128 (cfg5 geometry)
    _moment_case("grav_1024_s128", (9.81 + 0.3 * rng.standard_normal(1024 * 24)).astype(
        np.float32), 1024, 128, cases)
    # non-power-of-two window and ragged tail
    _moment_case("ragged_100_s37", (rng.standard_normal(5000) * 2 + 0.7).astype(np.float32),
                 100, 37, cases)
    # tiny / degenerate sizes: N == W (one window), N < W (zero windows), W=3
    _moment_case("one_window", rng.standard_normal(64).astype(np.float32), 64, 64, cases)
    _moment_case("w3_s1", rng.standard_normal(50).astype(np.float32), 3, 1, cases)
    small = rng.standard_normal(10).astype(np.float32)
    cases["empty"] = {"x": small, "wsize": np.int64(16), "wstep": np.int64(16),
                      "out_mean": rolling_apply(np.mean, 16, 16)(small)}

    # spectral cases
    fs3 = 64.0
    f0 = rng.uniform(0.8, 3.0, 96)
    t = np.arange(256) / fs3
    ppg = (np.sin(2 * np.pi * f0[:, None] * t) + 0.5 * np.sin(4 * np.pi * f0[:, None] * t + 1)
           + 0.3 * rng.standard_normal((96, 256))).astype(np.float32).ravel()
    ppg[256 * 5:256 * 6] = 0.0            # all-zero window -> NaN entropy / rel power
    ppg[256 * 6:256 * 7] = 2.5            # constant window -> DC only
    _spectral_case("ppg_256", ppg, 256, 256, fs3, (0.5, 4.0), (0.5, 8.0), cases)
    _spectral_case("accel_256", np.ascontiguousarray(acc[:256 * 96, 2]), 256, 256, 50.0,
                   (0.5, 4.0), (0.5, 8.0), cases)
    n5 = 1024 + 127 * 128
    t5 = np.arange(n5) / 256.0
    ecg = np.zeros(n5)
    for c in np.cumsum(rng.uniform(0.35, 1.2, 80)):
        ecg += np.exp(-0.5 * ((t5 - c) / 0.012) ** 2)
    ecg += 0.2 * np.sin(2 * np.pi * 0.3 * t5) + 0.02 * rng.standard_normal(n5)
    _spectral_case("ecg_1024_s128", ecg.astype(np.float32), 1024, 128, 256.0,
                   (0.5, 40.0), (0.5, 40.0), cases)
    _spectral_case("odd_99_s50", rng.standard_normal(99 * 40).astype(np.float32), 99, 50,
                   10.0, (0.7, 3.3), (1.0, 4.0), cases)
    _spectral_case("randn_128_fullband", rng.standard_normal(128 * 64).astype(np.float32),
                   128, 128, 32.0, (0.0, 16.0), (0.0, 1e9), cases)

    cases.update(nonuniform_cases(np.random.default_rng(20250308)))
    cases.update(n3n4_cases(np.random.default_rng(20250309)))
    cases.update(n2_cases(np.random.default_rng(20250310)))
    write(outdir, cases)


# ------------------------------------------------------------------- 2-D (N, c) input
# rolling_apply on a 2-D array: window i is the (W, c) block arr[i*S : i*S + W]
# (windows.py:68-91). Features numba evaluates on such a block (the others raise).
def _p25(w):
    return np.percentile(w, 25.0)


BLOCK_FEATURES = {k: FEATURES[k] for k in (
    "mean", "var", "std", "skewness", "kurtosis", "kurtosis_excess", "drange", "line_length",
    "rms", "hjorth_activity", "std_in_fn", "mean_in_fn")}
BLOCK_FEATURES.update({"coeff_var": stats.coeff_var.py_func, "min": np.min, "max": np.max,
                       "median": np.median, "p25": _p25,
                       "interquartile_range": stats.interquartile_range})


def block2d_cases(rng):
    """2-D records: 3-axis accel (edge rows mixed in), a 2-column record with a
    non-power-of-two row count per window, and a 1-column 2-D record."""
    cases = {}
    acc = _accel(64 * 40, 50.0, rng)
    edge = _edge_signal(64, 13, rng).reshape(-1, 4)[:, :3]       # NaN / inf / 0 / +-0 rows
    acc[:edge.shape[0]] = edge[:min(edge.shape[0], acc.shape[0])]
    for name, x, W, S in (("block_accel_64_s32", acc, 64, 32),
                          ("block_accel_100_s37", acc, 100, 37),
                          ("block_c2_50", (rng.standard_normal((2000, 2)) * 3 + 1).astype(np.float32),
                           50, 50),
                          ("block_c1_64_s16", rng.standard_normal((900, 1)).astype(np.float32),
                           64, 16)):
        rec = {"x": x, "wsize": np.int64(W), "wstep": np.int64(S)}
        for fname, f in BLOCK_FEATURES.items():
            rec["out_" + fname] = rolling_apply(f, W, S)(x)
        cases[name] = rec
    return cases


# ---------------------------------------------------------------------- float64 input
def f64_cases(rng):
    """rolling_apply on float64 arrays (numba types every reduction from the input dtype:
    fp64 sums, fp64 deviations): the moment / time-domain set on edge and offset windows,
    the N3 lane features and the N4 HRV family on an RR series, np.min / np.max, and a
    2-D float64 record."""
    cases = {}
    feats = dict(FEATURES)
    feats.update({"coeff_var": stats.coeff_var.py_func, "min": np.min, "max": np.max,
                  "entropy": information.entropy.py_func})
    feats.update(N3_FEATURES)
    _moment_case("f64_edge_128", _edge_signal(128, 48, rng).astype(np.float64), 128, 128,
                 cases, feats=feats, probe=True)
    # windows where the jitted function itself raises ZeroDivisionError (0/0 in a scalar
    # division, e.g. Hjorth of a constant window): inside the prange numba drops the
    # exception and leaves np.zeros' 0.0, so the serial call is the only way to flag them
    rec, x = cases["f64_edge_128"], cases["f64_edge_128"]["x"]
    for name, g in (("hjorth_mobility", timedom.hjorth_mobility),
                    ("hjorth_complexity", timedom.hjorth_complexity),
                    ("coeff_var", stats.coeff_var)):
        raises = np.zeros(rec["out_" + name].shape[0], np.bool_)
        for i in range(raises.shape[0]):
            try:
                g(x[i * 128:(i + 1) * 128])
            except ZeroDivisionError:
                raises[i] = True
        if raises.any():
            rec["raises_" + name] = raises | rec.get("raises_" + name, False)
    _moment_case("f64_grav_256_s64", (9.81 + 0.3 * rng.standard_normal(256 * 40)), 256, 64,
                 cases, feats=feats)
    _moment_case("f64_ragged_100_s37", rng.standard_normal(5000) * 2 + 0.7, 100, 37, cases,
                 feats=feats)
    rr = 800 + 40 * np.sin(np.arange(6000) / 30.0) + 25 * rng.standard_normal(6000)
    cases["f64_hrv_w64"] = _rolling_case(rr, 64, 16, N4_FEATURES)
    x2 = rng.standard_normal((2000, 3)) + np.array([0.0, 0.0, 9.81])
    rec = {"x": x2, "wsize": np.int64(50), "wstep": np.int64(25)}
    for fname, f in BLOCK_FEATURES.items():
        if fname not in ("median", "p25", "interquartile_range"):
            rec["out_" + fname] = rolling_apply(f, 50, 25)(x2)
    cases["f64_block_c3_50"] = rec
    return cases


def f64_sort_cases(rng):
    """float64 records through the order statistics (np.median, np.percentile at several q,
    stats.interquartile_range, stats.mode): the _sort_signal rows (zeros of both signs,
    NaN, +-inf, ties) in float64, every third window perturbed below float32 resolution
    (values equal as float32 but ordered as float64), windows up to 1500 samples."""
    cases = {}
    feats = dict(SORT_FEATURES)
    feats["median"] = np.median
    for W, S, nwin in ((64, 64, 60), (100, 37, 60), (256, 256, 40), (7, 3, 200), (1, 1, 30),
                       (2, 1, 40), (1024, 512, 8), (1500, 1500, 4)):
        x = _sort_signal(W, nwin * W // S + 1, rng)[:(nwin - 1) * S + W].astype(np.float64)
        for k in range(0, nwin, 3):
            seg = x[k * S:k * S + W]
            fin = np.isfinite(seg) & (seg != 0)
            seg[fin] = seg[fin] * (1.0 + rng.integers(-4, 5, fin.sum()) * 2.0 ** -40)
        cases["f64_sort_w%d_s%d" % (W, S)] = _rolling_case(x, W, S, feats)
    return cases


def f64_pairwise_cases(rng):
    """information.sampen and the RQA window functions on float64 records (fp64
    differences, fp64 np.std): differences below float32 resolution near the threshold,
    exact ties for radius 0, a constant window and a NaN."""
    cases = {}
    for W, S in ((64, 64), (100, 37)):
        n = 24 * S + W
        x = np.sin(np.arange(n) * 0.21) + 0.5 * rng.standard_normal(n)
        x[W * 2:W * 3] = 1.5
        x[W * 4:W * 5] = np.round(x[W * 4:W * 5] * 2) / 2
        x[W * 6:W * 7] = np.round(x[W * 6:W * 7] * 8) / 8 * (1.0 + 2.0 ** -36)
        cases["f64_sampen_w%d_s%d" % (W, S)] = _rolling_case(x, W, S, SAMPEN_FEATURES)
        nw = 30
        xr = np.round((np.sin(np.arange((nw - 1) * S + W) * 0.3)
                       + 0.3 * rng.standard_normal((nw - 1) * S + W)) * 8) / 8
        xr[S * 3:S * 3 + W] = 0.5
        xr[S * 5 + 4] = np.nan
        xr[S * 7:S * 7 + W] += rng.integers(-2, 3, W) * 2.0 ** -40
        cases["f64_rqa_w%d_s%d" % (W, S)] = _rolling_case(xr, W, S, RQA_FEATURES)
    return cases


# ------------------------------------------------------------------ per-sample helpers
def elementwise_cases(rng):
    """accelerometer.roll / pitch / magnitude_dot (accelerometer.py:13-75, 236-259) and
    timedom.gradient / zero_crossings (timedom.py:11-48) on float32 and float64 axes with
    zeros, signed zeros, NaN, inf and tiny / huge values mixed in."""
    from mhealth.inertial import accelerometer as acc
    cases = {}
    n = 4000
    for dt in (np.float32, np.float64):
        x, y, z = (rng.standard_normal((3, n)) * rng.uniform(0.1, 3.0, (3, 1))).astype(dt)
        special = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e-30, -1e-30, 1e30, 0.05,
                            -0.05], dt)
        for k, a in enumerate((x, y, z)):
            a[:len(special)] = np.roll(special, k)
            a[20:40:2] = 0.0
        rec = {"x": x, "y": y, "z": z, "out_roll": acc.roll(y, z), "out_pitch": acc.pitch(x, y, z),
               "out_magnitude_dot": np.float64(acc.magnitude_dot(x[40:], y[40:], z[40:])),
               "out_gradient": timedom.gradient(x)}
        for th in (0.0, 0.05):
            rec["out_zero_crossings_th%g" % th] = timedom.zero_crossings(x, th)
        # qrs.find_peaks / nb_find_peaks on a record with plateaus, NaN and +-inf
        pk = np.round(x * 4) / 4
        pk[100:110] = 1.0
        rec["x_peaks"] = pk
        rec["out_find_peaks"] = qrs.find_peaks(pk)
        rec["out_nb_find_peaks"] = qrs.nb_find_peaks(pk)
        cases["elementwise_%s" % np.dtype(dt).name] = rec
    return cases


# ------------------------------------------------------------------ drop-in surface
def _user_first_last(w):
    return w[0] * 2.0 + w[-1]


def _user_max_minus_mean(w):
    return np.max(w) - np.mean(w)


FFT_SIZES = (1, 2, 3, 7, 64, 100, 256, 1000, 4096, 6000, 8192, 10007)


def fft_inputs():
    """The fft fixture inputs, regenerated from seeds by the tests (complex and real)."""
    out = {}
    for n in FFT_SIZES:
        r = np.random.default_rng(1000 + n)
        out["c%d" % n] = r.standard_normal(n) + 1j * r.standard_normal(n)
        out["r%d" % n] = r.standard_normal(n).astype(np.float32)
    return out


def surface_cases(rng):
    """Module functions around the window path that users call directly:
    stats.minmax (stats.py:12-32), timedom.hjorth_mobility_derivative /
    hjorth_complexity_derivatives / hjorth_parameters (timedom.py:115-193),
    qrs.find_peaks(x, comp) for every comparison (qrs.py:200-212), mhealth.fft.fft / ifft
    (here the reference's own numpy fallback, fft/__init__.py:3-7: FFTW is not built), and
    rolling_apply of user callables the engine has no kernel for (windows.py:93)."""
    import mhealth.fft as mfft
    cases = {}
    # minmax: NaN in the middle, signed zeros tied at the minimum, NaN first, ints, 2-D
    a = (rng.standard_normal(5000) * 3).astype(np.float32)
    a[[10, 700, 2500]] = np.nan
    a[a.argmin()] = 0.0
    lo = np.float32(-0.0)
    b = a.copy()
    b[100], b[200] = lo, np.float32(-50.0)
    b[300] = np.float32(-50.0)
    c = a.copy()
    c[0] = np.nan
    d = rng.standard_normal(3001) * 1e5
    d[[5, 17]] = [np.inf, -np.inf]
    e = rng.integers(-10**12, 10**12, 4097)
    f = (rng.standard_normal((40, 3)) + 1).astype(np.float32)
    z = np.array([0.0, -0.0, 0.0, -0.0], np.float32)
    rec = {}
    for k, v in (("a", a), ("b", b), ("c", c), ("d", d), ("e", e), ("f", f), ("z", z),
                 ("z2", -z)):
        mn, mx = stats.minmax(v)
        rec["x_" + k] = v
        rec["out_" + k] = np.array([mn, mx], dtype=v.dtype)
    cases["surface_minmax"] = rec
    # Hjorth variants on float32 / float64 signals and user-supplied derivatives
    rec = {}
    for dt in (np.float32, np.float64):
        t = np.arange(3000)
        x = (np.sin(t * 0.05) + 0.3 * np.sin(t * 0.31) + 0.1 * rng.standard_normal(3000)).astype(dt)
        d1 = timedom.gradient(x)
        d2 = timedom.gradient(d1)
        dd = np.diff(x)                                   # a derivative in x's own dtype
        nm = np.dtype(dt).name
        rec["x_" + nm] = x
        rec["dd_" + nm] = dd
        rec["params_" + nm] = np.array(timedom.hjorth_parameters(x), np.float64)
        rec["mob_d_" + nm] = np.float64(timedom.hjorth_mobility_derivative(x, d1))
        rec["mob_dd_" + nm] = np.float64(timedom.hjorth_mobility_derivative(x, dd))
        rec["cmp_d_" + nm] = np.float64(timedom.hjorth_complexity_derivatives(x, d1, d2))
        rec["cmp_dd_" + nm] = np.float64(timedom.hjorth_complexity_derivatives(x, dd, np.diff(dd)))
    cases["surface_hjorth"] = rec
    # find_peaks with every comparison on plateaus, NaN and +-inf
    rec = {}
    for dt in (np.float32, np.float64):
        x = np.round(rng.standard_normal(6000) * 3).astype(dt) / 2
        x[50:60] = 1.0
        x[[200, 201, 900]] = [np.nan, np.inf, -np.inf]
        nm = np.dtype(dt).name
        rec["x_" + nm] = x
        for cname, comp in (("greater", np.greater), ("greater_equal", np.greater_equal),
                            ("less", np.less), ("less_equal", np.less_equal)):
            rec["out_%s_%s" % (cname, nm)] = qrs.find_peaks(x, comp)
    cases["surface_find_peaks"] = rec
    # fft / ifft
    rec = {}
    for key, v in fft_inputs().items():
        rec["fft_" + key] = mfft.fft(v)
        if key[0] == "c":
            rec["ifft_" + key] = mfft.ifft(v)
    cases["surface_fft"] = rec
    # rolling_apply of user callables (no engine kernel): the reference JIT-compiles them
    x = (rng.standard_normal(64 * 50) + 0.5).astype(np.float32)
    cases["surface_user_callables"] = {
        "x": x, "wsize": np.int64(64), "wstep": np.int64(32),
        "out_first_last": rolling_apply(_user_first_last, 64, 32)(x),
        "out_max_minus_mean": rolling_apply(_user_max_minus_mean, 64, 32)(x)}
    return cases


# ------------------------------------------------------ float64 records: spectral features
def f64_spectral_cases(rng):
    """Spectral features of FLOAT64 records: the reference transforms a.astype(complex128)
    (fft/_fft.py:18-28; numpy's fp64 pocketfft is its fallback, fft/__init__.py:3-7) and runs
    hrv.power_band / relative_power_band (heart/hrv.py:173-198), information.entropy
    (generic/information.py:10-20) and density.peak_frequency (generic/frequency/density.py:
    9-32) on that spectrum. Cases: PPG at full float64 precision (an all-zero, a constant and
    a NaN window), a large offset with an AC part below float32 resolution (its float32
    rounding loses the spectrum), ECG at cfg5 geometry, a non-power-of-two window, and W=2."""
    cases = {}
    fs = 64.0
    f0 = rng.uniform(0.8, 3.0, 48)
    t = np.arange(256) / fs
    ppg = (np.sin(2 * np.pi * f0[:, None] * t) + 0.5 * np.sin(4 * np.pi * f0[:, None] * t + 1)
           + 0.3 * rng.standard_normal((48, 256))).ravel()
    ppg[256 * 5:256 * 6] = 0.0
    ppg[256 * 6:256 * 7] = 2.5
    ppg[256 * 9 + 17] = np.nan
    _spectral_case("f64spec_ppg_256", ppg, 256, 256, fs, (0.5, 4.0), (0.5, 8.0), cases)
    n = 128 * 40
    ta = np.arange(n) / 50.0
    off = (1.0e4 + 2e-3 * np.sin(2 * np.pi * 1.3 * ta) + 1e-3 * np.sin(2 * np.pi * 6.1 * ta)
           + 2e-4 * rng.standard_normal(n))
    _spectral_case("f64spec_offset_128", off, 128, 128, 50.0, (0.5, 4.0), (0.5, 8.0), cases)
    n5 = 1024 + 31 * 128
    t5 = np.arange(n5) / 256.0
    ecg = np.zeros(n5)
    for c in np.cumsum(rng.uniform(0.35, 1.2, 30)):
        ecg += np.exp(-0.5 * ((t5 - c) / 0.012) ** 2)
    ecg += 9.81 + 0.2 * np.sin(2 * np.pi * 0.3 * t5) + 0.02 * rng.standard_normal(n5)
    _spectral_case("f64spec_ecg_1024_s128", ecg, 1024, 128, 256.0, (0.5, 40.0), (0.5, 40.0),
                   cases)
    _spectral_case("f64spec_odd_100_s37", rng.standard_normal(100 * 30) * 3 + 1.0, 100, 37,
                   10.0, (0.7, 3.3), (1.0, 4.0), cases)
    _spectral_case("f64spec_w2", rng.standard_normal(64), 2, 1, 4.0, (None, None),
                   (None, None), cases)
    return cases


# ------------------------------------- time-indexed windows with user callables (N1 surface)
@njit
def _nu_user_range(w):
    return w.max() - w.min()


@njit
def _nu_user_first_last(w):
    return w[0] * 2.0 + w[-1]


def nu_user_cases(rng):
    """nonuniform_rolling_apply / indices_rolling_apply with user functions the engine has no
    kernel for (windows.py:134-157 JIT-compiles any func): jitted user code alone and next to
    np.mean in a list, float32 and float64 records, short windows NaN (min_window_len 3)."""
    cases = {}
    idx = np.cumsum(rng.integers(1, 20, 3000)).astype(np.int64)
    idx[1500:] += 400                                   # a gap: empty / short windows -> NaN
    for dt in (np.float32, np.float64):
        x = (rng.standard_normal(3000) * 2 + 0.5).astype(dt)
        rec = {"x": x, "index": idx, "wsize": np.int64(60), "wstep": np.int64(40),
               "min_window_len": np.int64(3), "indices": get_indices(idx, 60, 40).astype(np.int64)}
        rec["out_range"] = nonuniform_rolling_apply(_nu_user_range, 3)(idx, x, 60, 40)
        rec["out_first_last"] = nonuniform_rolling_apply(_nu_user_first_last, 3)(idx, x, 60, 40)
        lst = nonuniform_rolling_apply([np.mean, _nu_user_range], 3)(idx, x, 60, 40)
        rec["list_mean"], rec["list_range"] = lst
        rec["irap_range"] = indices_rolling_apply(_nu_user_range, 3)(rec["indices"], x)
        cases["nu_user_%s" % np.dtype(dt).name] = rec
    return cases


def write(outdir, cases):
    for name, rec in cases.items():
        np.savez_compressed(os.path.join(outdir, name + ".npz"), **rec)
        print(name, {k: getattr(v, "shape", None) for k, v in rec.items()})


if __name__ == "__main__":
    # `make_golden.py DIR nonuniform` writes only the time-indexed window fixtures
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.abspath(__file__))
    if len(sys.argv) > 2 and sys.argv[2] == "nonuniform":
        write(out_dir, nonuniform_cases(np.random.default_rng(20250308)))
    elif len(sys.argv) > 2 and sys.argv[2] == "n2":
        write(out_dir, n2_cases(np.random.default_rng(20250310)))
    elif len(sys.argv) > 2 and sys.argv[2] == "minmax":
        write(out_dir, minmax_cases(np.random.default_rng(20250311)))
    elif len(sys.argv) > 2 and sys.argv[2] == "n3n4":
        write(out_dir, n3n4_cases(np.random.default_rng(20250309)))
    elif len(sys.argv) > 2 and sys.argv[2] == "psd":
        write(out_dir, psd_cases(np.random.default_rng(20250312)))
    elif len(sys.argv) > 2 and sys.argv[2] == "rqa":
        write(out_dir, rqa_cases(np.random.default_rng(20250314)))
    elif len(sys.argv) > 2 and sys.argv[2] == "f64":
        write(out_dir, f64_cases(np.random.default_rng(20250317)))
    elif len(sys.argv) > 2 and sys.argv[2] == "f64pair":
        write(out_dir, f64_pairwise_cases(np.random.default_rng(20250320)))
    elif len(sys.argv) > 2 and sys.argv[2] == "nu64":
        write(out_dir, nonuniform64_cases(np.random.default_rng(20250319)))
    elif len(sys.argv) > 2 and sys.argv[2] == "f64sort":
        write(out_dir, f64_sort_cases(np.random.default_rng(20250318)))
    elif len(sys.argv) > 2 and sys.argv[2] == "elementwise":
        write(out_dir, elementwise_cases(np.random.default_rng(20250316)))
    elif len(sys.argv) > 2 and sys.argv[2] == "block2d":
        write(out_dir, block2d_cases(np.random.default_rng(20250315)))
    elif len(sys.argv) > 2 and sys.argv[2] == "surface":
        write(out_dir, surface_cases(np.random.default_rng(20250321)))
    elif len(sys.argv) > 2 and sys.argv[2] == "f64spec":
        write(out_dir, f64_spectral_cases(np.random.default_rng(20250401)))
    elif len(sys.argv) > 2 and sys.argv[2] == "nuuser":
        write(out_dir, nu_user_cases(np.random.default_rng(20250402)))
    elif len(sys.argv) > 2 and sys.argv[2] == "n3sort":
        write(out_dir, n3_sort_cases(np.random.default_rng(20250313)))
    else:
        main(out_dir)
