"""ctypes wrapper around oracle/_build/libmhf_oracle.so (test infrastructure only).

Same argument meaning as the product C-ABI ``mhf_window_features`` (include/mhfeat.h)
but on host numpy arrays, OpenMP over windows.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmhf_oracle.so")

# ids of include/mhfeat.h `mhf_feature`
FEATURE_IDS = {
    "mean": 0, "mean32": 1, "var": 2, "var32": 3, "std": 4, "std32": 5, "skewness": 6,
    "kurtosis": 7, "kurtosis_excess": 8, "rms": 9, "zero_crossings": 10, "peak_count": 11,
    "drange": 12, "line_length": 13, "band_power": 14, "relative_band_power": 15,
    "spectral_entropy": 16, "dominant_frequency": 17, "coeff_var": 18,
    "hjorth_mobility": 19, "hjorth_complexity": 20, "rmssd": 21, "sdsd": 22, "ssd": 23,
    "pnnx": 24, "csi_sd1": 25, "csi_sd2": 26, "lorenz_csi": 27, "lorenz_cvi": 28,
    "lorenz_mcsi": 29, "min": 30, "max": 31, "median": 32, "entropy": 33,
    "interquartile_range": 34, "mode": 35, "percentile": 36, "sampen": 37,
    "rqa_recurrence_rate": 38, "rqa_determinism": 39, "rqa_laminarity": 40,
    "rqa_length_entropy": 41,
}
# include/mhfeat.h `mhf_psd_op`
PSD_OPS = {"power_band": 0, "relative_power_band": 1, "density_peak_frequency": 2,
           "hrv_peak_frequency": 3, "entropy": 4}
CSI_FACTOR = 0.70710678118654746   # 1 / np.sqrt(2), hrv.py:208


class Params(ctypes.Structure):
    _fields_ = [("fs", ctypes.c_double), ("band_lo", ctypes.c_double),
                ("band_hi", ctypes.c_double), ("dom_lo", ctypes.c_double),
                ("dom_hi", ctypes.c_double), ("zc_threshold", ctypes.c_double),
                ("pnn_threshold", ctypes.c_double), ("csi_factor", ctypes.c_double),
                ("percentile_q", ctypes.c_double), ("sampen_m", ctypes.c_double),
                ("sampen_r", ctypes.c_double), ("sampen_sd", ctypes.c_double),
                ("rqa_radius", ctypes.c_double), ("rqa_minlen", ctypes.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.mhf_oracle_window_features.restype = ctypes.c_int
        lib.mhf_oracle_window_features.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(Params), ctypes.c_int32,
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
        lib.mhf_oracle_window_features_ex.restype = ctypes.c_int
        lib.mhf_oracle_window_features_ex.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(Params), ctypes.c_int32,
            ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
        lib.mhf_oracle_num_windows.restype = ctypes.c_int64
        lib.mhf_oracle_num_windows.argtypes = [ctypes.c_int64] * 3
        lib.mhf_oracle_zc_threshold32.restype = ctypes.c_float
        lib.mhf_oracle_zc_threshold32.argtypes = [ctypes.c_double]
        lib.mhf_oracle_indexed_features.restype = ctypes.c_int
        lib.mhf_oracle_indexed_features.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(Params), ctypes.c_int32,
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
        lib.mhf_oracle_indexed_features64.restype = ctypes.c_int
        lib.mhf_oracle_indexed_features64.argtypes = lib.mhf_oracle_indexed_features.argtypes[:-1]
        lib.mhf_oracle_filtfilt.restype = ctypes.c_int
        lib.mhf_oracle_filtfilt.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
            ctypes.c_void_p]
        lib.mhf_oracle_magnitude.restype = None
        lib.mhf_oracle_magnitude.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_void_p]
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.mhf_oracle_window_features64.restype = ctypes.c_int
        lib.mhf_oracle_window_features64.argtypes = [
            vp, i64, i32, i64, i64, i64, i64, i64, i64, vp, i32, ctypes.POINTER(Params), i32,
            i32, vp, i64]
        for sfx in ("32", "64"):
            getattr(lib, "mhf_oracle_orientation" + sfx).restype = None
            getattr(lib, "mhf_oracle_orientation" + sfx).argtypes = [i32, vp, vp, vp, i64, vp]
            getattr(lib, "mhf_oracle_gradient" + sfx).restype = None
            getattr(lib, "mhf_oracle_gradient" + sfx).argtypes = [vp, i64, vp]
            getattr(lib, "mhf_oracle_zero_crossings" + sfx).restype = None
            getattr(lib, "mhf_oracle_zero_crossings" + sfx).argtypes = [vp, i64, ctypes.c_double,
                                                                        vp]
            getattr(lib, "mhf_oracle_find_peaks" + sfx).restype = i64
            getattr(lib, "mhf_oracle_find_peaks" + sfx).argtypes = [vp, i64, vp]
            getattr(lib, "mhf_oracle_magnitude_dot" + sfx).restype = ctypes.c_double
            getattr(lib, "mhf_oracle_magnitude_dot" + sfx).argtypes = [vp, vp, vp, i64]
        lib.mhf_oracle_psd_features.restype = ctypes.c_int
        lib.mhf_oracle_psd_features.argtypes = [
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_double,
            ctypes.c_double, ctypes.c_void_p, ctypes.c_int64]
        lib.mhf_oracle_periodogram.restype = ctypes.c_int
        lib.mhf_oracle_periodogram.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                               ctypes.c_double, ctypes.c_void_p]
        lib.mhf_oracle_periodogram64.restype = ctypes.c_int
        lib.mhf_oracle_periodogram64.argtypes = lib.mhf_oracle_periodogram.argtypes
        _lib = lib
    return _lib


def _none(v):
    return math.nan if v is None else float(v)


def make_params(fs=None, band=(None, None), dom=(None, None), zc_threshold=0.0,
                pnn_threshold=50.0, csi_factor=CSI_FACTOR, percentile_q=50.0, sampen_m=2,
                sampen_r=0.2, sampen_sd=None, rqa_radius=0.0, rqa_minlen=2):
    return Params(_none(fs) if fs is not None else 0.0, _none(band[0]), _none(band[1]),
                  _none(dom[0]), _none(dom[1]), float(zc_threshold), float(pnn_threshold),
                  float(csi_factor), float(percentile_q), float(sampen_m), float(sampen_r),
                  _none(sampen_sd), float(rqa_radius), float(rqa_minlen))


def num_windows(n, w, s):
    return load().mhf_oracle_num_windows(n, w, s)


def zc_threshold32(th):
    return load().mhf_oracle_zc_threshold32(th)


def _window_features64(lib, x, wsize, wstep, features, block, p, out_dtype):
    """float64 samples: the lane features (mhf_oracle_window_features64)."""
    ids = np.asarray([FEATURE_IDS[f] if isinstance(f, str) else int(f) for f in features],
                     np.int32)
    if block:
        x = np.ascontiguousarray(x)
        c = x.shape[1]
        flat, N, C, cs, ss, W, S, numerics = x.reshape(-1), x.shape[0] * c, 1, 0, 1, \
            wsize * c, wstep * c, c << 8
        nw = max(0, num_windows(x.shape[0], wsize, wstep))
    else:
        flat = x
        if x.ndim == 1:
            C, cs, ss = 1, 0, x.strides[0] // 8
        else:
            C, cs, ss = x.shape[1], x.strides[1] // 8, x.strides[0] // 8
        N, W, S, numerics = x.shape[0], wsize, wstep, 0
        nw = max(0, num_windows(N, wsize, wstep))
    out = np.zeros((C, len(ids), nw), dtype=out_dtype)
    if nw == 0:
        return out
    rc = lib.mhf_oracle_window_features64(flat.ctypes.data, N, C, cs, ss, W, S, 0, nw,
                                          ids.ctypes.data, len(ids), ctypes.byref(p), numerics,
                                          1 if out_dtype == np.float32 else 0, out.ctypes.data,
                                          nw)
    if rc != 0:
        raise ValueError("oracle rejected arguments (code %d)" % rc)
    return out


def window_features(x, wsize, wstep, features, *, fs=None, band=(None, None),
                    dom=(None, None), zc_threshold=0.0, first_window=0, n_windows=None,
                    out_dtype=np.float64, threads=0, base_window=0, pnn_threshold=50.0,
                    csi_factor=CSI_FACTOR, percentile_q=50.0, sampen_m=2, sampen_r=0.2,
                    sampen_sd=None, rqa_radius=0.0, rqa_minlen=2, block=False):
    """Features of every window of every column of ``x``.

    ``x``: (N,) or (N, C) float32 (any strides). Returns (C, F, nw) (C=1 for 1-D input).
    ``base_window``: x[0] is the first sample of that global window (a shard).
    ``block=True``: x is ONE 2-D (N, c) record and window i is the (wsize, c) block
    x[i*wstep : i*wstep + wsize] (the reference's rolling_apply on a 2-D array;
    MHF_NUMERICS_BLOCK). Returns (1, F, nw).
    """
    lib = load()
    if np.asarray(x).dtype == np.float64:
        return _window_features64(lib, np.asarray(x), wsize, wstep, features, block,
                                  make_params(fs, band, dom, zc_threshold, pnn_threshold,
                                              csi_factor, percentile_q, sampen_m, sampen_r,
                                              sampen_sd, rqa_radius, rqa_minlen), out_dtype)
    if block:
        x = np.ascontiguousarray(np.asarray(x))
        if x.ndim != 2 or x.dtype != np.float32:
            raise TypeError("block=True takes a 2-D float32 (N, c) record")
        c = x.shape[1]
        flat = x.reshape(-1)
        N = x.shape[0]
        nw = max(0, num_windows(N, wsize, wstep))
        ids = np.asarray([FEATURE_IDS[f] if isinstance(f, str) else int(f) for f in features],
                         np.int32)
        out = np.zeros((1, len(ids), nw), dtype=out_dtype)
        if nw == 0:
            return out
        p = make_params(fs, band, dom, zc_threshold, pnn_threshold, csi_factor, percentile_q,
                        sampen_m, sampen_r, sampen_sd, rqa_radius, rqa_minlen)
        numerics = c << 8
        rc = lib.mhf_oracle_window_features_ex(
            flat.ctypes.data, N * c, 1, 0, 1, wsize * c, wstep * c, 0, nw, ids.ctypes.data,
            len(ids), ctypes.byref(p), numerics, 1 if out_dtype == np.float32 else 0,
            out.ctypes.data, nw, threads)
        if rc != 0:
            raise ValueError("oracle rejected arguments (code %d)" % rc)
        return out
    if hasattr(x, "cpu"):
        x = x.cpu().numpy()
    x = np.asarray(x)
    if base_window:
        pad_shape = (base_window * wstep,) + tuple(x.shape[1:])
        x = np.concatenate([np.zeros(pad_shape, np.float32), x])
    if x.dtype != np.float32:
        raise TypeError("oracle takes float32 samples")
    if x.ndim == 1:
        x2, C, cs, ss = x, 1, 0, x.strides[0] // 4
    else:
        x2, C, cs, ss = x, x.shape[1], x.strides[1] // 4, x.strides[0] // 4
    N = x.shape[0]
    nw_all = max(0, num_windows(N, wsize, wstep))
    if n_windows is None:
        n_windows = nw_all - first_window
    ids = np.asarray([FEATURE_IDS[f] if isinstance(f, str) else int(f) for f in features],
                     np.int32)
    out = np.zeros((C, len(ids), max(n_windows, 0)), dtype=out_dtype)
    if n_windows <= 0:
        return out
    p = make_params(fs, band, dom, zc_threshold, pnn_threshold, csi_factor, percentile_q,
                    sampen_m, sampen_r, sampen_sd, rqa_radius, rqa_minlen)
    rc = lib.mhf_oracle_window_features(
        x2.ctypes.data, N, C, cs, ss, wsize, wstep, first_window, n_windows,
        ids.ctypes.data, len(ids), ctypes.byref(p),
        1 if out_dtype == np.float32 else 0, out.ctypes.data, n_windows, threads)
    if rc != 0:
        raise ValueError("oracle rejected arguments (code %d)" % rc)
    return out


def get_indices(index, wsize, wstep):
    """The reference's get_indices (src/mhealth/util/windows.py:162-178), restated with
    numpy (it is plain numpy when called from Python): arange starts, starts + wsize,
    searchsorted(side='left'), shape (2, n)."""
    starts = np.arange(index[0], index[-1], wstep)
    ends = starts + wsize
    return np.searchsorted(index, np.concatenate((starts, ends))).reshape((2, len(starts)))


def indexed_features(x, indices, features, *, min_len=1, zc_threshold=0.0,
                     out_dtype=np.float32, threads=0, pnn_threshold=50.0, csi_factor=CSI_FACTOR,
                     percentile_q=50.0, sampen_m=2, sampen_r=0.2, sampen_sd=None,
                     rqa_radius=0.0, rqa_minlen=2):
    """indices_rolling_apply (windows.py:134-157) of every column of ``x`` over the
    (2, nw) start/end ``indices``. Returns (C, F, nw)."""
    lib = load()
    x = np.asarray(x)
    if x.dtype not in (np.float32, np.float64):
        raise TypeError("oracle takes float32 or float64 samples")
    isz = x.dtype.itemsize
    if x.ndim == 1:
        C, cs, ss = 1, 0, x.strides[0] // isz
    else:
        C, cs, ss = x.shape[1], x.strides[1] // isz, x.strides[0] // isz
    ind = np.ascontiguousarray(np.asarray(indices, np.int64))
    starts, ends = np.ascontiguousarray(ind[0]), np.ascontiguousarray(ind[1])
    nw = starts.shape[0]
    ids = np.asarray([FEATURE_IDS[f] if isinstance(f, str) else int(f) for f in features],
                     np.int32)
    out = np.zeros((C, len(ids), nw), dtype=out_dtype)
    if nw == 0:
        return out
    p = make_params(None, (None, None), (None, None), zc_threshold, pnn_threshold, csi_factor,
                    percentile_q, sampen_m, sampen_r, sampen_sd, rqa_radius, rqa_minlen)
    if x.dtype == np.float64:
        # float64 record (windows.py:151 np.zeros(n, arr.dtype)): fp64 models, serial
        rc = lib.mhf_oracle_indexed_features64(
            x.ctypes.data, x.shape[0], C, cs, ss, starts.ctypes.data, ends.ctypes.data, nw,
            int(min_len), ids.ctypes.data, len(ids), ctypes.byref(p),
            1 if out_dtype == np.float32 else 0, out.ctypes.data, nw)
    else:
        rc = lib.mhf_oracle_indexed_features(
            x.ctypes.data, x.shape[0], C, cs, ss, starts.ctypes.data, ends.ctypes.data, nw,
            int(min_len), ids.ctypes.data, len(ids), ctypes.byref(p),
            1 if out_dtype == np.float32 else 0, out.ctypes.data, nw, threads)
    if rc != 0:
        raise ValueError("oracle rejected arguments (code %d)" % rc)
    return out


def psd_features(psd, freqs, ops, lower=None, upper=None):
    """The reference's PSD-level functions on every row of a (rows, bins) float32/float64
    array (mhf_psd_features semantics). Returns (len(ops), rows) float64."""
    psd = np.asarray(psd)
    P = np.ascontiguousarray(psd.reshape(1, -1) if psd.ndim == 1 else psd)
    if P.dtype not in (np.float32, np.float64):
        raise TypeError("psd must be float32 or float64")
    F = None if freqs is None else np.ascontiguousarray(np.asarray(freqs))
    ids = np.asarray([PSD_OPS[o] if isinstance(o, str) else int(o) for o in ops], np.int32)
    out = np.zeros((len(ids), P.shape[0]))
    rc = load().mhf_oracle_psd_features(
        P.ctypes.data, 1 if P.dtype == np.float64 else 0, P.shape[0], P.shape[1], P.shape[1],
        None if F is None else F.ctypes.data,
        1 if F is None or F.dtype == np.float64 else 0, ids.ctypes.data, len(ids),
        _none(lower), _none(upper), out.ctypes.data, P.shape[0])
    if rc != 0:
        raise ValueError("oracle rejected arguments (code %d)" % rc)
    return out


def periodogram(win, fs):
    """fp64 one-sided periodogram rows of (R, W) float32 or float64 windows (OpenMP)."""
    win = np.asarray(win)
    f64 = win.dtype == np.float64
    win = np.ascontiguousarray(win, np.float64 if f64 else np.float32)
    R, W = win.shape
    out = np.zeros((R, W // 2 + 1))
    if R:
        fn = load().mhf_oracle_periodogram64 if f64 else load().mhf_oracle_periodogram
        fn(win.ctypes.data, R, W, fs, out.ctypes.data)
    return out


def filtfilt(b, a, x, zi=None):
    """scipy.signal.filtfilt(b, a, x) restated in C (mhf_oracle_filtfilt) for float32 x of
    shape (n,) or (n, C); returns float64 of the same shape. ``zi``: lfilter_zi(b, a)
    (None: solved by the oracle's own elimination)."""
    lib = load()
    x = np.asarray(x)
    if x.dtype != np.float32:
        raise TypeError("oracle takes float32 samples")
    C = 1 if x.ndim == 1 else x.shape[1]
    cs = 0 if x.ndim == 1 else x.strides[1] // 4
    b = np.ascontiguousarray(np.atleast_1d(b), np.float64)
    a = np.ascontiguousarray(np.atleast_1d(a), np.float64)
    out = np.zeros((x.shape[0], C), np.float64)
    zp = None
    if zi is not None:
        zi = np.ascontiguousarray(zi, np.float64)
        zp = zi.ctypes.data
    rc = lib.mhf_oracle_filtfilt(x.ctypes.data, x.shape[0], C, cs, x.strides[0] // 4,
                                 b.ctypes.data, len(b), a.ctypes.data, len(a), zp,
                                 out.ctypes.data)
    if rc != 0:
        raise ValueError("oracle rejected arguments (code %d)" % rc)
    return out.reshape(x.shape)


def magnitude(xyz):
    """sqrt(x**2 + y**2 + z**2) of an (n, 3) float32 array, fp32 (accelerometer.py:198-225)."""
    lib = load()
    xyz = np.asarray(xyz)
    out = np.zeros(xyz.shape[0], np.float32)
    lib.mhf_oracle_magnitude(xyz.ctypes.data, xyz.shape[0], xyz.strides[0] // 4,
                             xyz.strides[1] // 4, out.ctypes.data)
    return out


# ---------------------------------------------------------------- per-sample helpers
def _same_dtype(*arrs):
    arrs = [np.ascontiguousarray(np.asarray(a)) for a in arrs]
    dt = np.float64 if any(a.dtype == np.float64 for a in arrs) else np.float32
    return [a.astype(dt, copy=False).reshape(-1) for a in arrs], ("64" if dt == np.float64 else "32")


def roll(y, z):
    """accelerometer.roll (accelerometer.py:13-26): float64 degrees."""
    (y, z), sfx = _same_dtype(y, z)
    out = np.zeros(y.shape[0])
    getattr(load(), "mhf_oracle_orientation" + sfx)(0, y.ctypes.data, y.ctypes.data,
                                                    z.ctypes.data, y.shape[0], out.ctypes.data)
    return out


def pitch(x, y, z):
    """accelerometer.pitch (accelerometer.py:45-58): float64 degrees."""
    (x, y, z), sfx = _same_dtype(x, y, z)
    out = np.zeros(x.shape[0])
    getattr(load(), "mhf_oracle_orientation" + sfx)(1, x.ctypes.data, y.ctypes.data,
                                                    z.ctypes.data, x.shape[0], out.ctypes.data)
    return out


def gradient(x):
    """timedom.gradient (timedom.py:11-31): float64."""
    (x,), sfx = _same_dtype(x)
    out = np.zeros(x.shape[0])
    getattr(load(), "mhf_oracle_gradient" + sfx)(x.ctypes.data, x.shape[0], out.ctypes.data)
    return out


def zero_crossings(x, th=0.0):
    """timedom.zero_crossings (timedom.py:34-48): bool, n - 1."""
    (x,), sfx = _same_dtype(x)
    out = np.zeros(max(x.shape[0] - 1, 0), np.uint8)
    getattr(load(), "mhf_oracle_zero_crossings" + sfx)(x.ctypes.data, x.shape[0], float(th),
                                                       out.ctypes.data)
    return out.astype(bool)


def magnitude_dot(x, y, z):
    """accelerometer.magnitude_dot (accelerometer.py:236-259): one float."""
    (x, y, z), sfx = _same_dtype(x, y, z)
    return getattr(load(), "mhf_oracle_magnitude_dot" + sfx)(x.ctypes.data, y.ctypes.data,
                                                             z.ctypes.data, x.shape[0])


def find_peaks(x):
    """qrs.nb_find_peaks (qrs.py:215-220): int64 indices of strict local maxima."""
    (x,), sfx = _same_dtype(x)
    out = np.zeros(max(x.shape[0], 1), np.int64)
    k = getattr(load(), "mhf_oracle_find_peaks" + sfx)(x.ctypes.data, x.shape[0], out.ctypes.data)
    return out[:k]
