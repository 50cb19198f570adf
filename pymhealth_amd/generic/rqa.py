"""Drop-in for ``mhealth.generic.rqa`` (src/mhealth/generic/rqa.py): recurrence
quantification.

Two forms, as with the spectral functions:

* per-window features for ``rolling_apply`` — the reference composes them by hand,
  ``rolling_apply(lambda w: rqa.determinism(rqa.rq(w, 0.3)), W, S)``; here that is
  ``features.rqa_determinism(0.3)`` (likewise ``rqa_recurrence_rate``,
  ``rqa_laminarity``, ``rqa_length_entropy(radius, minlen)``), one pairwise HIP kernel
  (order.hip ``rqa_kernel``) that never builds the W x W matrix;
* the matrix-level functions below on one recurrence matrix, with the reference's
  signatures: ``rq(x, radius)`` builds it on the GPU (fp32 differences compared with
  the float64 radius, rqa.py:9-28), and ``recurrence_rate`` / ``determinism`` /
  ``laminarity`` / ``diagonal_lengths`` / ``vertical_lengths`` / ``length_entropy``
  evaluate the reference's loops (rqa.py:49-187) as device tensor ops on it. numpy in,
  numpy out; CUDA tensors stay on the device. ``rq2`` (scipy pdist, not jittable in the
  reference) is not provided.
"""
import numpy as np

from ..features import (rqa_determinism, rqa_laminarity, rqa_length_entropy,  # noqa: F401
                        rqa_recurrence_rate)


def _dev(a, dtype=None):
    import torch
    if isinstance(a, torch.Tensor):
        t = a
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(a)))
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("pymhealth_amd needs an MI355X GPU (torch.cuda.is_available() "
                               "is False); there is no CPU path")
        t = t.to("cuda")
    return t if dtype is None else t.to(dtype)


def _out(t, like):
    import torch
    return t if isinstance(like, torch.Tensor) else t.cpu().numpy()


def rq(x, radius=0.0):
    """Recurrence matrix (rqa.py:9-28): r[i, j] = |x_i - x_j| <= radius."""
    import torch
    t = _dev(x)
    if t.dtype not in (torch.float32, torch.float64):
        t = t.to(torch.float64)
    d = (t[:, None] - t[None, :]).abs()       # in x's dtype, as numba computes it
    return _out(d.to(torch.float64) <= float(radius), x)


def recurrence_rate(r):
    """np.sum(r) / (n m) (rqa.py:49-60)."""
    t = _dev(r).bool()
    return float(t.sum().item()) / float(t.shape[0] * t.shape[1])


def _shift(t, di, dj):
    """t[i + di, j + dj] with out-of-range entries False."""
    import torch
    out = torch.zeros_like(t)
    n, m = t.shape
    i0, i1 = max(0, -di), min(n, n - di)
    j0, j1 = max(0, -dj), min(m, m - dj)
    if i1 > i0 and j1 > j0:
        out[i0:i1, j0:j1] = t[i0 + di:i1 + di, j0 + dj:j1 + dj]
    return out


def determinism(r):
    """Points with a recurrent diagonal neighbour, / n m (rqa.py:63-88; the reference's edge
    cases are exactly 'out-of-range neighbours are not recurrent')."""
    t = _dev(r).bool()
    out = t & (_shift(t, -1, -1) | _shift(t, 1, 1))
    return float(out.sum().item()) / float(t.shape[0] * t.shape[1])


def laminarity(r):
    """Points with a recurrent horizontal neighbour, / n m (rqa.py:91-111)."""
    t = _dev(r).bool()
    out = t & (_shift(t, 0, -1) | _shift(t, 0, 1))
    return float(out.sum().item()) / float(t.shape[0] * t.shape[1])


def _lengths(t, diagonal):
    """The reference's line-length matrix (rqa.py:114-153) before `out += 1`: the length
    (in steps) of each line stored at its last point, every other entry 0."""
    import torch
    n, m = t.shape
    out = torch.zeros((n, m), dtype=torch.int32, device=t.device)
    ti = t.to(torch.int32)
    for i in range(1, n):
        if diagonal:
            step = (out[i - 1, :-1] + 1) * (ti[i, 1:] & ti[i - 1, :-1])
            out[i, 1:] = step
            out[i - 1, :-1] = torch.where(step > 0, torch.zeros_like(step), out[i - 1, :-1])
        else:
            step = (out[i - 1, :] + 1) * (ti[i - 1, :] & ti[i, :])
            out[i, :] = step
            out[i - 1, :] = torch.where(step >= 1, torch.zeros_like(step), out[i - 1, :])
    return out


def diagonal_lengths(r, minlen=2):
    """Lengths of diagonal lines (rqa.py:114-133), in the reference's row-major order."""
    t = _dev(r).bool()
    v = (_lengths(t, True) + 1).reshape(-1)
    return _out(v[v >= minlen], r)


def vertical_lengths(r, minlen=2):
    """Lengths of vertical lines (rqa.py:136-153), in the reference's row-major order."""
    t = _dev(r).bool()
    v = (_lengths(t, False) + 1).reshape(-1)
    return _out(v[v >= minlen], r)


def length_entropy(r, minlen=2):
    """Entropy of the diagonal line-length distribution (rqa.py:156-187): counts of lengths
    minlen .. N-1 (a length-N line falls past the reference's N-element count array and is
    dropped), then information.entropy of the counts."""
    import torch
    t = _dev(r).bool()
    N = t.shape[0]
    v = (_lengths(t, True) + 1).reshape(-1).to(torch.int64)
    v = v[(v >= minlen) & (v < N)]
    counts = torch.bincount(v, minlength=N)[minlen:N].to(torch.float64)
    p = counts / counts.sum()
    p = p + 1e-30
    terms = (p * torch.log(p)).cpu().numpy()
    e = 0.0
    for term in terms:          # numba's np.sum: sequential, in bin order
        e = e + float(term)
    return -e


__all__ = ["rq", "recurrence_rate", "determinism", "laminarity", "diagonal_lengths",
           "vertical_lengths", "length_entropy", "rqa_recurrence_rate", "rqa_determinism",
           "rqa_laminarity", "rqa_length_entropy"]
