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
CUDA tensor (zero-copy, result returned as a CUDA tensor). float32 samples (the
engine's arithmetic type). Differences from the reference, all where the reference
fails: ``wsize=None`` raises TypeError (numba cannot compile it); the dict form returns
a real ``dict`` (the reference returns ``{zip(names, vals)}``, a set holding one zip
object, windows.py:116); callables without an MI355X kernel raise TypeError instead of
being JIT-compiled.
"""
from functools import lru_cache, singledispatch
from typing import Callable, Dict, List, Optional

import numpy as np
from numpy.lib.stride_tricks import as_strided

from ..feature import plan_groups, resolve


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


def _run(feats, arr, wsize, wstep):
    """One fused launch per parameter group; returns list of per-feature results."""
    import torch
    from ..engine import to_device, window_features
    _check_sizes(wsize, wstep)
    is_torch = isinstance(arr, torch.Tensor)
    if not is_torch:
        arr = np.asarray(arr)
    if arr.ndim != 1:
        raise ValueError("rolling_apply: arr must be 1-D; for (N, C) data pass columns "
                         "(arr[:, k]) or use pymhealth_amd.features.extract for per-channel "
                         "features in one pass")
    t = to_device(arr)
    res = [None] * len(feats)
    for idx, kw in plan_groups(feats):
        out = window_features(t, int(wsize), int(wstep), [feats[j].fid for j in idx], **kw)
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
    feat = resolve(func)

    def loop_wrapper(arr, wsize=wsize, wstep=wstep):
        return _run([feat], arr, wsize, wstep)[0]

    loop_wrapper.__doc__ = ("Apply the function {} to windows in a given array (one fused "
                            "MI355X launch).".format(feat.name))
    return loop_wrapper


@rolling_apply.register(list)
@rolling_apply.register(tuple)
def _rolling_apply_coll(funcs: List[Callable], wsize: Optional[int] = None,
                        wstep: int = 1) -> Callable:
    feats = [resolve(f) for f in funcs]

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


__all__ = ["view", "array_shape", "rolling_apply"]
