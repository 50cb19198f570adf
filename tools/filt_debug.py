"""Diagnostic (GPU): run mhf_filtfilt through the C-ABI with a caller workspace and compare
the forward pass it leaves there (the LDS-streamed path keeps it reversed AoS, yr) and the
output against a sequential fp64 filtfilt, reporting where they differ (chunk, block)."""
import ctypes
import os
import sys

import numpy as np
import torch
from scipy import signal

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pymhealth_amd import _lib  # noqa: E402


def main():
    n, C = int(sys.argv[1]) if len(sys.argv) > 1 else 70001, 1
    rng = np.random.default_rng(41)
    x = (np.cumsum(rng.standard_normal(n)) * 0.01 + rng.standard_normal(n)).astype(np.float32)
    b, a = signal.butter(5, 0.5 / 25.0, "highpass")
    zi = signal.lfilter_zi(b, a)
    taps = max(len(a), len(b))
    padlen = 3 * taps
    L = n + 2 * padlen
    x64 = x.astype(np.float64)
    xe = np.concatenate([2 * x64[0] - x64[padlen:0:-1], x64, 2 * x64[-1] - x64[-2:-padlen - 2:-1]]).astype(np.float64)
    yf, _ = signal.lfilter(b, a, xe.astype(np.float64), zi=zi * float(xe[0]))
    yb, _ = signal.lfilter(b, a, yf[::-1], zi=zi * yf[-1])
    ref = yb[::-1][padlen:-padlen]
    print("scipy check", np.abs(signal.filtfilt(b, a, x.astype(np.float64)) - ref).max())
    if not torch.cuda.is_available():
        print("reference ok (no GPU)")
        return
    L_ = _lib.lib()
    t = torch.from_numpy(x).cuda()
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    need = L_.mhf_filtfilt_workspace(n, C, len(b), len(a))
    ws = torch.zeros(need // 8, dtype=torch.float64, device="cuda")
    bb = np.ascontiguousarray(b, np.float64)
    aa = np.ascontiguousarray(a, np.float64)
    zz = np.ascontiguousarray(zi, np.float64)
    rc = L_.mhf_filtfilt(ctypes.c_void_p(t.data_ptr()), n, C, 0, 1, bb.ctypes.data, len(b),
                         aa.ctypes.data, len(a), zz.ctypes.data, _lib.MHF_OUT_F64, ctypes.c_void_p(out.data_ptr()),
                         0, 1, ctypes.c_void_p(ws.data_ptr()), need, None)
    torch.cuda.synchronize()
    _lib.check(rc)
    yr = ws.cpu().numpy()[:L]
    fwd = yr[::-1]                     # tile path: yr[L-1-j] = y_fwd[j]
    scale = max(1.0, np.abs(yf).max())
    err = np.abs(fwd - yf) / scale
    bad = np.nonzero(~(err <= 1e-8))[0]
    print("forward: max err %.3g, bad %d of %d" % (np.nanmax(err), bad.size, L))
    if bad.size:
        print("first bad j", bad[:20], "last", bad[-5:])
        print("got", fwd[bad[:5]], "want", yf[bad[:5]])
    o = out.cpu().numpy()
    e2 = np.abs(o - ref) / max(1.0, np.abs(ref).max())
    bad2 = np.nonzero(~(e2 <= 1e-8))[0]
    print("output: max err %.3g, bad %d of %d" % (np.nanmax(e2), bad2.size, n))
    if bad2.size:
        print("first bad t", bad2[:20], "last", bad2[-5:])


if __name__ == "__main__":
    main()
