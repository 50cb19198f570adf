"""Device-side entry point: fused sliding-window features of torch CUDA tensors.

``window_features`` is the one call everything else in the package (the
``rolling_apply`` drop-in, the single-window feature calls, the multi-GPU sharder,
the bench) goes through. It hands the tensor's device pointer, strides and the
current HIP stream to ``mhf_window_features`` (include/mhfeat.h) — zero copies,
stream-ordered, asynchronous.
"""
import ctypes

import numpy as np
import torch

from . import _lib

# Rows >= 1 of np.var / np.std on the register-tile path: False (default) derives them from
# the fp32-deviation sum, within 3.6e-7 relative of numba's var_parallel_impl;
# True replays its fp64 chain bit for bit (MHF_NUMERICS_EXACT_VAR, +4 VALU per sample).
# A per-call ``exact_var`` argument overrides it.
EXACT_VAR = False


def num_windows(n_samples, wsize, wstep):
    """``max(0, 1 + (n - wsize) // wstep)`` — loop_wrapper's ``nw`` (windows.py:86)."""
    if wsize is None or wstep is None or int(wsize) < 1 or int(wstep) < 1:
        raise ValueError("wsize and wstep must be integers >= 1")
    return max(0, 1 + (int(n_samples) - int(wsize)) // int(wstep))


def _require_device(x, allow_f64=False):
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
        raise TypeError("window_features takes a torch CUDA tensor (got %r)" % type(x))
    if x.dtype != torch.float32 and not (allow_f64 and x.dtype == torch.float64):
        raise TypeError("samples must be float32 (got %s)" % x.dtype)


def window_features(x, wsize, wstep, feature_ids, *, fs=None, band=(None, None),
                    dom=(None, None), zc_threshold=0.0, first_window=0, n_windows=None,
                    base_window=0, out_dtype=torch.float64, out=None, stream=None,
                    pnn_threshold=50.0, csi_factor=_lib.CSI_FACTOR, percentile_q=50.0,
                    sampen_m=2, sampen_r=0.2, sampen_sd=None, rqa_radius=0.0, rqa_minlen=2,
                    block=0, exact_var=None):
    """Features of windows of every channel of ``x``.

    x:            torch.float32 (or float64) CUDA tensor, (N,) or (N, C), any strides (AoS
                  (N,3) ok). float64: every feature in fp64 (numba's fp64 models for the
                  lane features, an fp64 transform for the spectral ones).
    feature_ids:  sequence of ``mhf_feature`` ids (``_lib.MHF_*``).
    first_window, n_windows: GLOBAL window range to compute.
    base_window:  x[0] is the first sample of global window ``base_window`` (a shard of a
                  longer record); window indices stay global so window 0 keeps the
                  reference's row-0 numerics. Default 0: x is the whole record.
    Returns a (C, F, n_windows) tensor of ``out_dtype`` (float64 like the reference's
    ``np.zeros((nw,))``, windows.py:89, or float32), or fills ``out``.
    block:        c >= 1: ``x`` is a 2-D (rows, c) record passed FLAT (1-D, rows * c
                  samples) and wsize / wstep count flat samples (rows * c); each window is
                  the reference's (wsize / c, c) block (``MHF_NUMERICS_BLOCK``).
    exact_var:    bit-exact rows >= 1 of np.var / np.std on the register tiles
                  (``MHF_NUMERICS_EXACT_VAR``); None = the module default ``EXACT_VAR``.
    """
    _require_device(x, allow_f64=True)
    block = int(block) if block else 0
    if block > 0 and x.dim() != 1:
        raise ValueError("block > 0 takes the 2-D record flattened to 1-D")
    if x.dim() == 1:
        n, C, cs, ss = x.shape[0], 1, 0, x.stride(0)
    elif x.dim() == 2:
        n, C, cs, ss = x.shape[0], x.shape[1], x.stride(1), x.stride(0)
    else:
        raise ValueError("x must be 1-D (N,) or 2-D (N, C)")
    ids = np.ascontiguousarray(np.asarray(list(feature_ids), dtype=np.int32))
    F = len(ids)
    base_window = int(base_window)
    if base_window < 0:
        raise ValueError("base_window must be >= 0")
    base_off = base_window * int(wstep)          # samples before x[0] in the record
    n += base_off
    nw_all = num_windows(n, wsize, wstep)
    first_window = int(first_window)
    if first_window < base_window:
        raise ValueError("first_window precedes the shard (base_window)")
    if n_windows is None:
        n_windows = nw_all - first_window
    n_windows = int(n_windows)
    if out_dtype not in (torch.float64, torch.float32):
        raise TypeError("out_dtype must be torch.float64 or torch.float32")
    if out is None:
        out = torch.empty((C, F, max(n_windows, 0)), dtype=out_dtype, device=x.device)
    else:
        if out.shape != (C, F, n_windows) or out.dtype != out_dtype or not out.is_contiguous():
            raise ValueError("out must be a contiguous (C, F, n_windows) %s tensor" % out_dtype)
    if n_windows == 0 or F == 0:
        return out
    p = _lib.make_params(fs, band, dom, zc_threshold, pnn_threshold, csi_factor, percentile_q,
                         sampen_m, sampen_r, sampen_sd, rqa_radius, rqa_minlen)
    if stream is None:
        stream = torch.cuda.current_stream(x.device).cuda_stream
    L = _lib.lib()
    if x.dtype == torch.float64:
        # float64 record: every feature in fp64 (mhf_window_features_f64) — the lane
        # features in numba's fp64 models, order statistics / sampen / RQA on the float64
        # values, spectral features from an fp64 transform (spectral64.hip), as the
        # reference transforms a.astype(complex128) (fft/_fft.py:18-28)
        with torch.cuda.device(x.device):
            rc = L.mhf_window_features_f64(
                ctypes.c_void_p(x.data_ptr() - 8 * base_off * ss), n, C, cs, ss, int(wsize),
                int(wstep), first_window, n_windows, ids.ctypes.data, F, ctypes.byref(p),
                _lib.MHF_NUMERICS_REFERENCE | (block << 8),
                _lib.MHF_OUT_F32 if out_dtype == torch.float32 else _lib.MHF_OUT_F64,
                ctypes.c_void_p(out.data_ptr()), n_windows, _lib.cstream(stream, x, out))
        _lib.check(rc)
        return out
    with torch.cuda.device(x.device):
        rc = L.mhf_window_features(
            ctypes.c_void_p(x.data_ptr() - 4 * base_off * ss), n, C, cs, ss, int(wsize),
            int(wstep), first_window,
            n_windows, ids.ctypes.data, F, ctypes.byref(p),
            _lib.MHF_NUMERICS_REFERENCE | (block << 8) |
            (_lib.MHF_NUMERICS_EXACT_VAR if (EXACT_VAR if exact_var is None else exact_var) else 0),
            _lib.MHF_OUT_F32 if out_dtype == torch.float32 else _lib.MHF_OUT_F64,
            ctypes.c_void_p(out.data_ptr()), n_windows, _lib.cstream(stream, x, out))
    _lib.check(rc)
    return out


def indexed_window_features(x, indices, feature_ids, *, min_len=1, zc_threshold=0.0,
                            out_dtype=torch.float32, out=None, stream=None,
                            pnn_threshold=50.0, csi_factor=_lib.CSI_FACTOR, percentile_q=50.0,
                            sampen_m=2, sampen_r=0.2, sampen_sd=None, rqa_radius=0.0,
                            rqa_minlen=2):
    """Features of windows with known sample ranges (indices_rolling_apply's loop,
    windows.py:132-157): window i of every channel of ``x`` is ``x[indices[0, i]:indices[1, i]]``.

    x:        torch.float32 or float64 CUDA tensor, (N,) or (N, C), any strides (float64:
              ``mhf_indexed_window_features_f64``, the lane features and order statistics).
    indices:  (2, n) int64 CUDA tensor of start / end sample indices (``get_indices``).
    Every window gets the reference's serial numerics (its loop is a plain @jit loop);
    a window with ``end - start < min_len`` (or empty) is NaN in every feature.
    Returns a (C, F, n) tensor of ``out_dtype`` (the reference's ``np.zeros(n, arr.dtype)``,
    windows.py:151: the record's dtype), or fills ``out``.
    """
    _require_device(x, allow_f64=True)
    f64 = x.dtype == torch.float64
    if x.dim() == 1:
        n, C, cs, ss = x.shape[0], 1, 0, x.stride(0)
    elif x.dim() == 2:
        n, C, cs, ss = x.shape[0], x.shape[1], x.stride(1), x.stride(0)
    else:
        raise ValueError("x must be 1-D (N,) or 2-D (N, C)")
    if (not isinstance(indices, torch.Tensor) or indices.device != x.device
            or indices.dtype != torch.int64 or indices.dim() != 2 or indices.shape[0] != 2):
        raise TypeError("indices must be a (2, n) int64 tensor on the device of x")
    if indices.stride(1) != 1:
        indices = indices.contiguous()
    ids = np.ascontiguousarray(np.asarray(list(feature_ids), dtype=np.int32))
    F, nw = len(ids), indices.shape[1]
    if out_dtype not in (torch.float64, torch.float32):
        raise TypeError("out_dtype must be torch.float64 or torch.float32")
    if out is None:
        out = torch.empty((C, F, nw), dtype=out_dtype, device=x.device)
    elif out.shape != (C, F, nw) or out.dtype != out_dtype or not out.is_contiguous():
        raise ValueError("out must be a contiguous (C, F, n) %s tensor" % out_dtype)
    if nw == 0 or F == 0:
        return out
    # window lengths are only known on the device: the library sizes the order-statistic /
    # sampen / RQA launches from the longest kept (clamped) window itself, sorts order
    # statistics of windows beyond the LDS capacity in the caller's workspace, and refuses
    # sampen / RQA windows beyond theirs (MHF_EUNSUPPORTED -> NotImplementedError). The
    # workspace is sized for the longest window the indices can describe: min(n, max(end -
    # start)) (one reduction, read back only when such features are asked for)
    L = _lib.lib()
    dt = _lib.MHF_DTYPE_F64 if f64 else _lib.MHF_DTYPE_F32
    if stream is None:
        stream = torch.cuda.current_stream(x.device).cuda_stream
    # only order statistics of windows past the LDS capacity need scratch beyond the fixed
    # slot: no clamped window is longer than the record, so when a record-long window would
    # need none, the device reduction + readback of the longest window is skipped
    need = L.mhf_indexed_workspace(0, C, dt, ids.ctypes.data, F)
    if need > 0 and L.mhf_indexed_workspace(n, C, dt, ids.ctypes.data, F) > need:
        longest = max(0, min(n, int((indices[1] - indices[0]).max().item())))
        need = L.mhf_indexed_workspace(longest, C, dt, ids.ctypes.data, F)
    ws, wsp, wsn = _lib.workspace(need, x.device, stream)
    p = _lib.make_params(zc_threshold=zc_threshold, pnn_threshold=pnn_threshold,
                         csi_factor=csi_factor, percentile_q=percentile_q, sampen_m=sampen_m,
                         sampen_r=sampen_r, sampen_sd=sampen_sd, rqa_radius=rqa_radius,
                         rqa_minlen=rqa_minlen)
    entry = L.mhf_indexed_window_features_f64 if f64 else L.mhf_indexed_window_features
    with torch.cuda.device(x.device):
        rc = entry(
            ctypes.c_void_p(x.data_ptr()), n, C, cs, ss, ctypes.c_void_p(indices[0].data_ptr()),
            ctypes.c_void_p(indices[1].data_ptr()), nw, int(min_len), ids.ctypes.data, F,
            ctypes.byref(p),
            _lib.MHF_OUT_F32 if out_dtype == torch.float32 else _lib.MHF_OUT_F64,
            ctypes.c_void_p(out.data_ptr()), nw, wsp, wsn, _lib.cstream(stream, x, indices, out))
    _lib.check(rc)
    del ws
    return out


def window_bounds(index, n_windows, mode, t0, wstep, wsize, stream=None):
    """``mhf_window_bounds``: (2, n_windows) int64 start/end indices of windows
    ``[t0 + i*wstep, t0 + i*wstep + wsize)`` in the sorted int64 CUDA tensor ``index``.
    ``mode``: ``MHF_BOUNDS_FLOAT_*`` bits (which bounds numpy computes in float64)."""
    if (not isinstance(index, torch.Tensor) or index.device.type != "cuda"
            or index.dtype != torch.int64 or index.dim() != 1):
        raise TypeError("index must be a 1-D int64 CUDA tensor")
    index = index.contiguous()
    out = torch.empty((2, int(n_windows)), dtype=torch.int64, device=index.device)
    if n_windows == 0:
        return out
    fi = (lambda v: 0) if mode & _lib.MHF_BOUNDS_FLOAT_STARTS else int
    if stream is None:
        stream = torch.cuda.current_stream(index.device).cuda_stream
    with torch.cuda.device(index.device):
        rc = _lib.lib().mhf_window_bounds(
            ctypes.c_void_p(index.data_ptr()), index.shape[0], int(n_windows), int(mode),
            fi(t0), fi(wstep), 0 if mode & _lib.MHF_BOUNDS_FLOAT_ENDS else int(wsize),
            float(t0), float(wstep), float(wsize), ctypes.c_void_p(out[0].data_ptr()),
            ctypes.c_void_p(out[1].data_ptr()), _lib.cstream(stream, index, out))
    _lib.check(rc)
    return out


def filtfilt(x, b, a, zi=None, *, out_dtype=torch.float64, out=None, stream=None):
    """``scipy.signal.filtfilt(b, a, x)`` (padtype 'odd', method 'pad') of every channel
    of ``x`` (float32 CUDA tensor, (N,) or (N, C), any strides) — ``mhf_filtfilt``.
    ``zi``: ``lfilter_zi(b, a)`` (None: solved on the device). Returns a tensor of x's
    shape in ``out_dtype`` (float64: the reference's ``np.zeros(acc.shape)``)."""
    _require_device(x)
    if x.dim() == 1:
        n, C, cs, ss = x.shape[0], 1, 0, x.stride(0)
    elif x.dim() == 2:
        n, C, cs, ss = x.shape[0], x.shape[1], x.stride(1), x.stride(0)
    else:
        raise ValueError("x must be 1-D (N,) or 2-D (N, C)")
    b = np.ascontiguousarray(np.atleast_1d(np.asarray(b, dtype=np.float64)))
    a = np.ascontiguousarray(np.atleast_1d(np.asarray(a, dtype=np.float64)))
    zp = None
    if zi is not None:
        zi = np.ascontiguousarray(np.asarray(zi, dtype=np.float64).ravel())
        if zi.size != max(len(a), len(b)) - 1:
            raise ValueError("zi must have max(len(a), len(b)) - 1 values")
        zp = zi.ctypes.data
    if out_dtype not in (torch.float64, torch.float32):
        raise TypeError("out_dtype must be torch.float64 or torch.float32")
    if out is None:
        out = torch.empty(tuple(x.shape), dtype=out_dtype, device=x.device)
    elif out.shape != x.shape or out.dtype != out_dtype:
        raise ValueError("out must be a %s tensor of x's shape" % out_dtype)
    ocs, oss = (0, out.stride(0)) if out.dim() == 1 else (out.stride(1), out.stride(0))
    if stream is None:
        stream = torch.cuda.current_stream(x.device).cuda_stream
    L = _lib.lib()
    ws, wsp, wsn = _lib.workspace(L.mhf_filtfilt_workspace(n, C, len(b), len(a)), x.device, stream)
    with torch.cuda.device(x.device):
        rc = L.mhf_filtfilt(
            ctypes.c_void_p(x.data_ptr()), n, C, cs, ss, b.ctypes.data, len(b), a.ctypes.data,
            len(a), zp, _lib.MHF_OUT_F32 if out_dtype == torch.float32 else _lib.MHF_OUT_F64,
            ctypes.c_void_p(out.data_ptr()), ocs, oss, wsp, wsn, _lib.cstream(stream, x, out))
    _lib.check(rc)
    del ws
    return out


def magnitude(xyz, *, out=None, stream=None):
    """sqrt(x^2 + y^2 + z^2) of an (N, 3) float32 CUDA tensor (``mhf_magnitude``)."""
    _require_device(xyz)
    if xyz.dim() != 2 or xyz.shape[1] != 3:
        raise ValueError("magnitude takes an (N, 3) tensor")
    if out is None:
        out = torch.empty(xyz.shape[0], dtype=torch.float32, device=xyz.device)
    if stream is None:
        stream = torch.cuda.current_stream(xyz.device).cuda_stream
    with torch.cuda.device(xyz.device):
        rc = _lib.lib().mhf_magnitude(ctypes.c_void_p(xyz.data_ptr()), xyz.shape[0],
                                      xyz.stride(0), xyz.stride(1),
                                      ctypes.c_void_p(out.data_ptr()), _lib.cstream(stream, xyz, out))
    _lib.check(rc)
    return out


# ---------------------------------------------------------- per-sample helpers (elementwise.hip)
def _elem_device(*arrs):
    """numpy / torch inputs -> 1-D CUDA tensors of one float dtype (float32 or float64, the
    reference's numba typing follows it), plus the MHF dtype code."""
    ts = []
    for a in arrs:
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(np.asarray(a)))
        if t.dtype not in (torch.float32, torch.float64):
            t = t.to(torch.float64)            # ints / Python floats: numba computes in fp64
        if t.device.type != "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                                   "is False); there is no CPU path")
            t = t.to("cuda")
        ts.append(t.reshape(-1).contiguous())
    dt = torch.float64 if any(t.dtype == torch.float64 for t in ts) else torch.float32
    ts = [t.to(dt) for t in ts]
    n = ts[0].shape[0]
    if any(t.shape[0] != n for t in ts):
        raise ValueError("arrays must have the same length")
    return ts, (_lib.MHF_DTYPE_F64 if dt == torch.float64 else _lib.MHF_DTYPE_F32)


def orientation(which, x, y, z, *, stream=None):
    """accelerometer roll (which = MHF_ROLL, x unused) / pitch in degrees, float64
    (``mhf_orientation``)."""
    ts, dt = _elem_device(*([y, z] if which == _lib.MHF_ROLL else [x, y, z]))
    yz = ts if which == _lib.MHF_ROLL else ts[1:]
    xp = ts[0] if which == _lib.MHF_PITCH else yz[0]
    out = torch.empty(yz[0].shape[0], dtype=torch.float64, device=yz[0].device)
    stream = torch.cuda.current_stream(out.device).cuda_stream if stream is None else stream
    with torch.cuda.device(out.device):
        rc = _lib.lib().mhf_orientation(which, ctypes.c_void_p(xp.data_ptr()),
                                        ctypes.c_void_p(yz[0].data_ptr()),
                                        ctypes.c_void_p(yz[1].data_ptr()), out.shape[0], 1, dt,
                                        ctypes.c_void_p(out.data_ptr()), _lib.cstream(stream, *ts, out))
    _lib.check(rc)
    return out


def gradient(x, *, stream=None):
    """timedom.gradient: float64 (``mhf_gradient``)."""
    (t,), dt = _elem_device(x)
    out = torch.empty(t.shape[0], dtype=torch.float64, device=t.device)
    stream = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
    with torch.cuda.device(t.device):
        rc = _lib.lib().mhf_gradient(ctypes.c_void_p(t.data_ptr()), t.shape[0], 1, dt,
                                     ctypes.c_void_p(out.data_ptr()), _lib.cstream(stream, t, out))
    _lib.check(rc)
    return out


def zero_crossings(x, th=0.0, *, stream=None):
    """timedom.zero_crossings: bool, length n - 1 (``mhf_zero_crossings``)."""
    (t,), dt = _elem_device(x)
    n = t.shape[0]
    out = torch.empty(max(n - 1, 0), dtype=torch.uint8, device=t.device)
    stream = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
    with torch.cuda.device(t.device):
        rc = _lib.lib().mhf_zero_crossings(ctypes.c_void_p(t.data_ptr()), n, 1, dt, float(th),
                                           ctypes.c_void_p(out.data_ptr() if n > 1 else 0),
                                           _lib.cstream(stream, t, out))
    _lib.check(rc)
    _lib.join(stream)
    return out.to(torch.bool)


def magnitude_dot(x, y, z, *, stream=None):
    """accelerometer.magnitude_dot: one value of the input dtype, on the device
    (``mhf_magnitude_dot``)."""
    ts, dt = _elem_device(x, y, z)
    out = torch.empty(1, dtype=ts[0].dtype, device=ts[0].device)
    stream = torch.cuda.current_stream(out.device).cuda_stream if stream is None else stream
    L = _lib.lib()
    ws, wsp, wsn = _lib.workspace(L.mhf_magnitude_dot_workspace(ts[0].shape[0]), out.device, stream)
    with torch.cuda.device(out.device):
        rc = L.mhf_magnitude_dot(*(ctypes.c_void_p(t.data_ptr()) for t in ts),
                                 ts[0].shape[0], 1, dt, ctypes.c_void_p(out.data_ptr()), wsp, wsn,
                                 _lib.cstream(stream, *ts, out))
    _lib.check(rc)
    del ws
    return out


def find_peaks(x, comp=_lib.MHF_CMP_GREATER, *, stream=None):
    """Indices i with comp(x[i], x[i-1]) and comp(x[i], x[i+1]), int64 ascending
    (``mhf_find_peaks_cmp``; comp an ``MHF_CMP_*`` code, default strict maxima)."""
    (t,), dt = _elem_device(x)
    n = t.shape[0]
    L = _lib.lib()
    stream = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
    ws = torch.empty(max(L.mhf_find_peaks_workspace(n) // 8, 1), dtype=torch.int64, device=t.device)
    if int(stream) != torch.cuda.current_stream(t.device).cuda_stream:
        ws.record_stream(torch.cuda.ExternalStream(int(stream), device=t.device))
    room = (n - 1) // 2 if comp in (_lib.MHF_CMP_GREATER, _lib.MHF_CMP_LESS) else n - 2
    out = torch.empty(max(room, 1), dtype=torch.int64, device=t.device)
    with torch.cuda.device(t.device):
        rc = L.mhf_find_peaks_cmp(ctypes.c_void_p(t.data_ptr()), n, 1, dt, int(comp),
                                  ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                  _lib.cstream(stream, t, out, ws))
    _lib.check(rc)
    _lib.join(stream)                      # the count is read on the current stream
    count = int(ws[(n + 1023) // 1024].item())
    return out[:count]


_MINMAX_DTYPES = {torch.float32: _lib.MHF_DTYPE_F32, torch.float64: _lib.MHF_DTYPE_F64,
                  torch.int32: _lib.MHF_DTYPE_I32, torch.int64: _lib.MHF_DTYPE_I64}


def minmax(x, *, stream=None):
    """stats.minmax kernel: (min, max) of x.ravel() as a 2-element device tensor of x's
    dtype (``mhf_minmax``). Takes float32 / float64 / int32 / int64 arrays or tensors (one
    return type: always a device tensor); every other dtype — bool, 8 / 16-bit integers,
    unsigned integers, float16 — is mapped onto these by ``generic.stats.minmax``, which
    returns the reference's Python scalars."""
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if t.dtype not in _MINMAX_DTYPES:
        raise TypeError("engine.minmax takes float32 / float64 / int32 / int64 (got %s); "
                        "generic.stats.minmax maps the other dtypes" % t.dtype)
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to("cuda")
    t = t.reshape(-1)
    if t.shape[0] == 0:
        raise ValueError("minmax of an empty array")
    out = torch.empty(2, dtype=t.dtype, device=t.device)
    stream = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
    L = _lib.lib()
    ws, wsp, wsn = _lib.workspace(L.mhf_minmax_workspace(t.shape[0], _MINMAX_DTYPES[t.dtype]),
                                  t.device, stream)
    with torch.cuda.device(t.device):
        rc = L.mhf_minmax(ctypes.c_void_p(t.data_ptr()), t.shape[0], t.stride(0),
                          _MINMAX_DTYPES[t.dtype], ctypes.c_void_p(out.data_ptr()), wsp, wsn,
                          _lib.cstream(stream, t, out))
    _lib.check(rc)
    del ws
    return out


def fft(a, direction=_lib.MHF_FFT_FORWARD, scale=1.0, *, stream=None):
    """Complex128 FFT of the last axis of ``a`` (every row of a 2-D array), ``mhf_fft``:
    unnormalised for direction MHF_FFT_FORWARD (-1) / MHF_FFT_BACKWARD (+1), times
    ``scale``. Returns a complex128 CUDA tensor of a's shape."""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(a)))
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to("cuda")
    if t.dim() == 0 or t.dim() > 2:
        raise ValueError("fft takes a 1-D array (or a 2-D batch of rows)")
    t = t.to(torch.complex128).contiguous()
    n = t.shape[-1]
    batch = 1 if t.dim() == 1 else t.shape[0]
    out = torch.empty_like(t)
    if n == 0 or batch == 0:
        if n == 0:
            raise ValueError("Invalid number of FFT data points (0) specified.")
        return out
    stream = torch.cuda.current_stream(t.device).cuda_stream if stream is None else stream
    L = _lib.lib()
    ws, wsp, wsn = _lib.workspace(L.mhf_fft_workspace(n, batch), t.device, stream)
    with torch.cuda.device(t.device):
        rc = L.mhf_fft(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                       n, batch, int(direction), float(scale), wsp, wsn, _lib.cstream(stream, t, out))
    _lib.check(rc)
    del ws
    return out


def plan_name(x_shape_strides, wsize, wstep, feature_ids, out_dtype=torch.float64):
    """Kernel variant the engine would launch (for tests / profiling)."""
    C, cs, ss = x_shape_strides
    ids = np.ascontiguousarray(np.asarray(list(feature_ids), dtype=np.int32))
    name = _lib.lib().mhf_plan_name(C, cs, ss, int(wsize), int(wstep), ids.ctypes.data,
                                    len(ids), _lib.MHF_OUT_F32 if out_dtype == torch.float32
                                    else _lib.MHF_OUT_F64)
    return None if name is None else name.decode()


def algorithmic_bytes(n_samples, channels, wsize, wstep, n_windows, n_features,
                      out_dtype=torch.float64, sample_bytes=4):
    """``mhf_algorithmic_bytes`` (float32 samples); ``sample_bytes=8`` counts the input
    term of a float64 record twice."""
    b = _lib.lib().mhf_algorithmic_bytes(
        n_samples, channels, wsize, wstep, n_windows, n_features,
        _lib.MHF_OUT_F32 if out_dtype == torch.float32 else _lib.MHF_OUT_F64)
    if sample_bytes == 8 and n_windows > 0:
        samples = n_windows * wsize if wstep >= wsize else (n_windows - 1) * wstep + wsize
        b += 4 * channels * samples
    return b


def plan_name_indexed(x_shape_strides, feature_ids, dtype=torch.float32):
    """Kernel variants ``mhf_indexed_window_features(_f64)`` would launch (tests / profiling)."""
    C, cs, ss = x_shape_strides
    ids = np.ascontiguousarray(np.asarray(list(feature_ids), dtype=np.int32))
    name = _lib.lib().mhf_plan_name_indexed(
        C, cs, ss, ids.ctypes.data, len(ids),
        _lib.MHF_DTYPE_F64 if dtype == torch.float64 else _lib.MHF_DTYPE_F32)
    return None if name is None else name.decode()


def plan_name_f64(x_shape_strides, wsize, wstep, feature_ids, out_dtype=torch.float64):
    """Kernel variant ``mhf_window_features_f64`` would launch (tests / profiling)."""
    C, cs, ss = x_shape_strides
    ids = np.ascontiguousarray(np.asarray(list(feature_ids), dtype=np.int32))
    name = _lib.lib().mhf_plan_name_f64(C, cs, ss, int(wsize), int(wstep), ids.ctypes.data,
                                        len(ids), _lib.MHF_OUT_F32 if out_dtype == torch.float32
                                        else _lib.MHF_OUT_F64)
    return None if name is None else name.decode()


def to_device(arr, device=None, allow_f64=False):
    """numpy / torch input -> float32 CUDA tensor (H2D copy for host input); float64 kept
    as float64 when ``allow_f64`` (window_features' fp64 lane path)."""
    if isinstance(arr, torch.Tensor):
        t = arr
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(arr)))
    if t.dtype != torch.float32 and not (allow_f64 and t.dtype == torch.float64):
        raise TypeError("the MI355X engine takes float32 samples here (got %s); cast "
                        "explicitly" % t.dtype)
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to(device or "cuda", non_blocking=False)
    return t
