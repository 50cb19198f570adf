"""Rolling window operations — drop-in for ``mhealth.util.windows``
(src/mhealth/util/windows.py).

``rolling_apply(func, wsize, wstep)`` keeps the reference's signature, its
``singledispatch`` on the type of ``func`` (callable / list / tuple / dict,
windows.py:54,98-119) and its ``lru_cache(256)`` on ``(func, wsize, wstep)``
(windows.py:55). The returned callable ``loop_wrapper(arr, wsize=wsize, wstep=wstep)``
computes ``nw = max(0, 1 + (len(arr) - wsize) // wstep)`` windows (windows.py:86) and
returns float64 values (``np.zeros((nw, *shape))``, windows.py:89), with the
reference's row-0 (serial) vs rows >= 1 (prange) numerics, by one launch of the fused
HIP kernel of libmhfeat.so. A list of features is ONE launch (the reference makes one
pass per feature, windows.py:104-105).

Input: a 1-D numpy array (copied to the GPU, result returned as numpy) or a 1-D torch
CUDA tensor (zero-copy, result returned as a CUDA tensor), float32 samples (the
engine's arithmetic type) or float64 (numba's fp64 models for the lane features:
``mhf_window_features_f64``); or a 2-D (N, c) array, whose windows are the reference's
(wsize, c) blocks (see ``_run``). Differences from the reference, all where the reference
fails: ``wsize=None`` raises TypeError (numba cannot compile it); the dict form returns
a real ``dict`` (the reference returns ``{zip(names, vals)}``, a set holding one zip
object, windows.py:116).

User callables (a lambda, a user's own @jit function: anything that is not one of the
engine's features, ``resolve`` rejects it) have no kernel: the reference JIT-compiles them
(windows.py:93); here they are evaluated window by window on the host over the same
windows, ``out[i] = func(window_i)`` into ``np.zeros((nw, *shape))``, with a
one-time warning. That path runs only the user's own code — every feature the engine
knows (``np.mean``, ``stats.skewness``, ...) always takes the HIP kernels, in the same
call.
"""
import warnings
from functools import lru_cache, singledispatch
from typing import Callable, Dict, List, Optional

import numpy as np
from numpy.lib.stride_tricks import as_strided

from ..feature import WindowFeature, plan_groups, resolve


def view(x: np.ndarray, w: int, s: int) -> np.ndarray:
    """Strided window view of array (windows.py:20-33): shape (((N-w)//s)+1, w)."""
    stride = x.strides[0]
    N = x.shape[0]
    return as_strided(x, (((N - w) // s) + 1, w), (s * stride, stride))


def array_shape(x):
    """Shape of the given array; a scalar has shape () (windows.py:36-51)."""
    return getattr(x, "shape", tuple())


def _check_sizes(wsize, wstep):
    if wsize is None:
        raise TypeError("rolling_apply: wsize must be given (the reference cannot compile "
                        "wsize=None either)")
    if int(wsize) < 1 or int(wstep) < 1:
        raise ValueError("rolling_apply: wsize and wstep must be >= 1")


# features the reference evaluates on a 2-D (rows, c) window block (MHF_NUMERICS_BLOCK,
# include/mhfeat.h); the others fail there under numba (TypingError / TypeError)
_BLOCK_FEATURES = {"mean", "mean32", "var", "var32", "std", "std32", "skewness", "kurtosis",
                   "kurtosis_excess", "rms", "drange", "line_length", "coeff_var", "min", "max",
                   "median", "percentile", "interquartile_range", "hjorth_activity"}


class UserCallable:
    """A ``func`` with no MI355X kernel: the user's own per-window code."""

    def __init__(self, func):
        self.func = func
        self.name = getattr(func, "__name__", repr(func))

    def __repr__(self):
        return "<UserCallable %s>" % self.name


_warned = set()


def _resolve(func):
    """``resolve`` for rolling_apply: an engine feature, or a UserCallable for a plain
    callable the engine has no kernel for (misuses of known functions still raise)."""
    import functools
    try:
        return resolve(func)
    except TypeError:
        known = (func is np.percentile or isinstance(func, WindowFeature) or
                 (isinstance(func, functools.partial) and
                  (func.func is np.percentile or isinstance(func.func, WindowFeature))))
        if known or not callable(func):
            raise
        return UserCallable(func)


def _warn_user(u):
    key = id(u.func)
    if key not in _warned:
        _warned.add(key)
        warnings.warn("rolling_apply: %r has no MI355X kernel; it is evaluated window by "
                      "window on the host (the engine's own features run on the GPU)"
                      % (u.func,), RuntimeWarning, stacklevel=4)


def _host_array(arr):
    import torch
    if isinstance(arr, torch.Tensor):
        return arr.detach().cpu().numpy()
    return np.asarray(arr)


def _run_user(u, arr, wsize, wstep):
    """``loop_wrapper`` for a user callable (windows.py:75-91): nw windows
    ``arr[i*wstep : i*wstep + wsize]`` (1-D slices or 2-D blocks), row 0 sizes
    ``np.zeros((nw, *shape))`` (float64), ``out[i] = func(window)``."""
    _warn_user(u)
    x = _host_array(arr)
    W, S = int(wsize), int(wstep)
    nw = max(0, 1 + (x.shape[0] - W) // S)
    if nw == 0:
        return np.zeros((0,))
    first = u.func(x[:W])
    out = np.zeros((nw,) + tuple(array_shape(first)))
    out[0] = first
    for i in range(1, nw):
        out[i] = u.func(x[i * S:i * S + W])
    return out


def _run(feats, arr, wsize, wstep):
    """Engine features in fused launches, user callables window by window (_run_user)."""
    user = [j for j, f in enumerate(feats) if isinstance(f, UserCallable)]
    if not user:
        return _run_native(feats, arr, wsize, wstep)
    _check_sizes(wsize, wstep)
    native = [j for j in range(len(feats)) if j not in user]
    res = [None] * len(feats)
    if native:
        for j, r in zip(native, _run_native([feats[j] for j in native], arr, wsize, wstep)):
            res[j] = r
    import torch
    for j in user:
        r = _run_user(feats[j], arr, wsize, wstep)
        res[j] = torch.from_numpy(r).to(arr.device) if isinstance(arr, torch.Tensor) else r
    return res


def _run_native(feats, arr, wsize, wstep):
    """One fused launch per parameter group; returns list of per-feature results.

    A 2-D (N, c) array is the reference's 2-D case (windows.py:68-91): window i is the
    (wsize, c) block arr[i*wstep : i*wstep + wsize], reduced by numba element by element in
    C order — so the record is passed flat with wsize * c / wstep * c and the block
    numerics (skewness / kurtosis divide by the ROW count, line_length differences run
    along the rows)."""
    import torch
    from ..engine import to_device, window_features
    _check_sizes(wsize, wstep)
    is_torch = isinstance(arr, torch.Tensor)
    if not is_torch:
        arr = np.asarray(arr)
    block, arr_2d = 1, arr.ndim == 2
    if arr_2d:
        block = int(arr.shape[1])
        bad = [f.name for f in feats if f.name not in _BLOCK_FEATURES]
        if bad:
            raise TypeError("rolling_apply: %s not defined on 2-D windows (the reference "
                            "fails on (rows, c) blocks); 2-D input takes %s"
                            % (", ".join(bad), ", ".join(sorted(_BLOCK_FEATURES))))
        arr = arr.contiguous().reshape(-1) if is_torch else np.ascontiguousarray(arr).reshape(-1)
    elif arr.ndim != 1:
        raise ValueError("rolling_apply: arr must be 1-D or 2-D")
    t = to_device(arr, allow_f64=True)
    c = block if arr_2d else 1
    res = [None] * len(feats)
    for idx, kw in plan_groups(feats):
        if arr_2d:
            kw = dict(kw, block=block)
        out = window_features(t, int(wsize) * c, int(wstep) * c, [feats[j].fid for j in idx],
                              **kw)
        for k, j in enumerate(idx):
            res[j] = out[0, k]
    if not is_torch:
        host = [r.cpu().numpy() for r in res]
        return host
    return res


@singledispatch
@lru_cache(256)
def rolling_apply(func: Callable, wsize: Optional[int] = None,
                  wstep: int = 1) -> Callable:
    """Create a Callable to apply the given function to windows along an array.

    Params:
        func (Callable): Function to apply to each window
        wsize (int): Window size.
        wstep (int): Step size between start of windows.
    Returns:
        Callable: function which will apply func to windows in an array
    """
    feat = _resolve(func)

    def loop_wrapper(arr, wsize=wsize, wstep=wstep):
        return _run([feat], arr, wsize, wstep)[0]

    loop_wrapper.__doc__ = ("Apply the function {} to windows in a given array (one fused "
                            "MI355X launch).".format(feat.name))
    return loop_wrapper


@rolling_apply.register(list)
@rolling_apply.register(tuple)
def _rolling_apply_coll(funcs: List[Callable], wsize: Optional[int] = None,
                        wstep: int = 1) -> Callable:
    feats = [_resolve(f) for f in funcs]

    def multi_funcs_rolling_apply(arr, wsize=wsize, wstep=wstep):
        return _run(feats, arr, wsize, wstep)
    return multi_funcs_rolling_apply


@rolling_apply.register(dict)
def _rolling_apply_dict(funcs: Dict[str, Callable], wsize: Optional[int] = None,
                        wstep: int = 1) -> Callable:
    names = list(funcs)
    multi = _rolling_apply_coll([funcs[k] for k in names], wsize, wstep)

    def dict_funcs_rolling_apply(arr, wsize=wsize, wstep=wstep):
        return dict(zip(names, multi(arr, wsize, wstep)))
    return dict_funcs_rolling_apply


# ---------------------------------------------------------------- time-indexed windows
# nonuniform_rolling_apply / indices_rolling_apply / get_indices (windows.py:122-249):
# windows of a fixed DURATION over a sorted (datetime64 or integer) index, so each holds a
# different number of samples. Two launches: mhf_window_bounds (one binary search per
# bound) and mhf_indexed_window_features (every feature of every window in one pass).


def _is_int(v):
    return isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_))


def _is_float(v):
    return isinstance(v, (float, np.floating))


def _arange_len(span, step):
    """len(np.arange(a, b, step)) for span = b - a: numpy's ceil(span / step) with the
    true division in float64 (PyArray_ArangeObj)."""
    return max(0, int(np.ceil(np.float64(span) / np.float64(step))))


def _bounds_plan(index, wsize, wstep):
    """Reduce (index, wsize, wstep) to int64 ticks and numpy's arithmetic per bound.

    Returns (index_int64 (numpy or CUDA tensor), n_windows, mode, t0, wstep, wsize), with
    t0/wstep/wsize as Python ints for integer bounds and floats for float ones.
    """
    import torch
    from .. import _lib
    if isinstance(index, torch.Tensor):
        if index.dtype != torch.int64 or index.dim() != 1:
            raise TypeError("get_indices: a tensor index must be 1-D int64 ticks")
        if index.shape[0] == 0:
            raise IndexError("get_indices: empty index (the reference fails on index[0])")
        ends = index[[0, -1]].cpu().numpy()
        idx, first, last = index, int(ends[0]), int(ends[1])
    else:
        index = np.asarray(index)
        if index.ndim != 1:
            raise ValueError("get_indices: index must be 1-D")
        if index.shape[0] == 0:
            raise IndexError("get_indices: empty index (the reference fails on index[0])")
        if index.dtype.kind == "M":
            if not (isinstance(wsize, np.timedelta64) and isinstance(wstep, np.timedelta64)):
                raise TypeError("get_indices: a datetime64 index takes np.timedelta64 "
                                "wsize and wstep")
            # searchsorted compares in the finest unit of index, wstep and wsize
            unit = (index[:1] + wstep + wsize).dtype
            idx = index.astype(unit).view(np.int64)
            td = np.dtype(unit.str.replace("M8", "m8"))
            wstep = int(np.asarray(wstep).astype(td).view(np.int64))
            wsize = int(np.asarray(wsize).astype(td).view(np.int64))
        elif index.dtype.kind in "iu":
            idx = index.astype(np.int64, copy=False)
        else:
            raise TypeError("get_indices: index must be datetime64 or integer ticks "
                            "(got %s)" % index.dtype)
        first, last = int(idx[0]), int(idx[-1])
    for name, v in (("wsize", wsize), ("wstep", wstep)):
        if not (_is_int(v) or _is_float(v)):
            raise TypeError("get_indices: %s must be a number or np.timedelta64 for a "
                            "datetime64 index (got %r)" % (name, v))
    if not wstep > 0:
        raise ValueError("get_indices: wstep must be > 0")
    mode = 0
    if _is_float(wstep):
        mode = _lib.MHF_BOUNDS_FLOAT_STARTS | _lib.MHF_BOUNDS_FLOAT_ENDS
        wstep, wsize, t0 = float(wstep), float(wsize), float(first)
    else:
        wstep, t0 = int(wstep), first
        if _is_float(wsize):
            mode = _lib.MHF_BOUNDS_FLOAT_ENDS
            wsize = float(wsize)
        else:
            wsize = int(wsize)
    nw = _arange_len(np.int64(last) - np.int64(first), wstep)
    return idx, nw, mode, t0, wstep, wsize


def get_indices(index, wsize, wstep):
    """Start ([0, :]) and end ([1, :]) sample indices of windows of duration ``wsize``
    every ``wstep`` over the sorted ``index`` (windows.py:162-178): window starts are
    ``np.arange(index[0], index[-1], wstep)`` and both bounds are
    ``np.searchsorted(index, ., 'left')`` — computed on the GPU.

    index: datetime64 numpy array (with np.timedelta64 wsize / wstep), integer ticks
    (numpy, or a 1-D int64 CUDA tensor) with int or float wsize / wstep. Returns an
    int64 (2, n) numpy array, or a CUDA tensor for a tensor index.
    """
    import torch
    from ..engine import window_bounds
    idx, nw, mode, t0, wstep, wsize = _bounds_plan(index, wsize, wstep)
    host = not isinstance(idx, torch.Tensor)
    if host:
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        idx = torch.from_numpy(np.ascontiguousarray(idx)).to("cuda")
    out = window_bounds(idx, nw, mode, t0, wstep, wsize)
    return out.cpu().numpy() if host else out


def _run_indexed_user(u, ind, x, min_window_len):
    """``windows_loop`` for a user callable (windows.py:146-157): ``out = np.zeros(n,
    arr.dtype)``; ``out[i] = func(arr[si:ei])`` where ``ei - si >= min_window_len``, else
    NaN (Python slice clipping, as numba slices)."""
    _warn_user(u)
    n = ind.shape[1]
    out = np.zeros(n, x.dtype)
    for i in range(n):
        si, ei = int(ind[0, i]), int(ind[1, i])
        if ei - si >= min_window_len:
            out[i] = u.func(x[si:ei])
        else:
            out[i] = np.nan
    return out


def _run_indexed(feats, indices, arr, min_window_len):
    """Engine features: one fused launch per parameter group over the known windows; user
    callables window by window on the host (_run_indexed_user). Per-feature results."""
    import torch
    from ..engine import indexed_window_features, to_device
    is_torch = isinstance(arr, torch.Tensor)
    if not is_torch:
        arr = np.asarray(arr)
    if arr.ndim != 1:
        raise ValueError("indices_rolling_apply: arr must be 1-D")
    user = [j for j, f in enumerate(feats) if isinstance(f, UserCallable)]
    native = [j for j in range(len(feats)) if j not in user]
    res = [None] * len(feats)
    if user:
        xh = _host_array(arr)
        ih = _host_array(indices)
        if ih.ndim != 2 or ih.shape[0] != 2:
            raise ValueError("indices must have shape (2, n)")
        for j in user:
            r = _run_indexed_user(feats[j], ih, xh, int(min_window_len))
            res[j] = torch.from_numpy(r).to(arr.device) if is_torch else r
    if not native:
        return res
    t = to_device(arr, allow_f64=True)
    if isinstance(indices, torch.Tensor):
        ind = indices.to(device=t.device, dtype=torch.int64)
    else:
        ind = np.asarray(indices)
        if ind.ndim != 2 or ind.shape[0] != 2:
            raise ValueError("indices must have shape (2, n)")
        ind = torch.from_numpy(np.ascontiguousarray(ind, dtype=np.int64)).to(t.device)
    nfeats = [feats[j] for j in native]
    for idx, kw in plan_groups(nfeats):
        if "fs" in kw:
            raise TypeError("indices_rolling_apply: spectral features need equal-length "
                            "windows (use rolling_apply)")
        # np.zeros(n, arr.dtype) (windows.py:151): float32 or float64 like the record
        out = indexed_window_features(t, ind, [nfeats[j].fid for j in idx],
                                      min_len=int(min_window_len), out_dtype=t.dtype, **kw)
        for k, j in enumerate(idx):
            res[native[j]] = out[0, k] if is_torch else out[0, k].cpu().numpy()
    return res


@lru_cache(256)
def indices_rolling_apply(func: Callable, min_window_len: int = 1) -> Callable:
    """Create a Callable applying ``func`` to windows with known indices
    (windows.py:122-159). The callable is ``windows_loop(indices, arr,
    min_window_len=min_window_len)``: ``out[i] = func(arr[indices[0, i]:indices[1, i]])``,
    NaN where the window holds fewer than ``min_window_len`` samples; float32 output
    (``np.zeros(n, arr.dtype)``). Every window gets the reference's serial numerics. A user
    callable with no kernel runs window by window on the host (the reference JIT-compiles
    any ``func``, windows.py:134-157)."""
    feat = _resolve(func)

    def windows_loop(indices, arr, min_window_len=min_window_len):
        return _run_indexed([feat], indices, arr, min_window_len)[0]

    windows_loop.__doc__ = ("Apply the '{}' function to windows with known indices (one "
                            "MI355X launch).".format(feat.name))
    return windows_loop


@singledispatch
def nonuniform_rolling_apply(func: Callable, min_window_len: int = 1) -> Callable:
    """Moving-window aggregation over a non-uniform (e.g. datetime) index
    (windows.py:181-216). Returns ``moving_window(index, arr, wsize, wstep,
    min_window_len=min_window_len)``: ``get_indices`` then ``indices_rolling_apply``."""
    f = indices_rolling_apply(func, min_window_len)

    def moving_window(index, arr, wsize, wstep, min_window_len=min_window_len):
        return f(get_indices(index, wsize, wstep), arr, min_window_len)

    moving_window.__doc__ = ("Aggregate windows with the '{}' function."
                             .format(_resolve(func).name))
    return moving_window


@nonuniform_rolling_apply.register(list)
@nonuniform_rolling_apply.register(tuple)
def _nu_rolling_apply_coll(funcs: List[Callable], min_window_len: int = 1) -> Callable:
    """List form (windows.py:219-231): one result per function, ONE fused launch for the
    engine's features (user callables beside it on the host)."""
    feats = [_resolve(f) for f in funcs]

    def moving_window(index, arr, wsize, wstep):
        return _run_indexed(feats, get_indices(index, wsize, wstep), arr, min_window_len)
    return moving_window


@nonuniform_rolling_apply.register(dict)
def _nu_rolling_apply_dict(funcs: Dict[str, Callable], min_window_len: int = 1) -> Callable:
    """Dict form (windows.py:234-249): ``{name: result}``."""
    names = list(funcs)
    multi = _nu_rolling_apply_coll([funcs[k] for k in names], min_window_len)

    def moving_window(index, arr, wsize, wstep):
        return dict(zip(names, multi(index, arr, wsize, wstep)))
    return moving_window


__all__ = ["view", "array_shape", "rolling_apply", "get_indices", "indices_rolling_apply",
           "nonuniform_rolling_apply"]
