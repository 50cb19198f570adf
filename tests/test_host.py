"""CPU-only tests: C-ABI library loads and exports every declared symbol, host-side
argument validation, windowing arithmetic and drop-in dispatch (no GPU compute)."""
import ctypes
import functools
import os
import re

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    import __graft_entry__
    __graft_entry__.build()
    from pymhealth_amd import _lib
    return _lib.lib()


def test_exports_every_header_symbol(L):
    hdr = open(os.path.join(ROOT, "include", "mhfeat.h")).read()
    decls = set(re.findall(r"^\s*MHF_API\s+(?:const\s+)?\w+\*?\s+\*?(mhf_\w+)\(", hdr, re.M))
    assert decls == {"mhf_num_windows", "mhf_window_features", "mhf_window_features_f64",
                     "mhf_algorithmic_bytes",
                     "mhf_plan_name", "mhf_plan_name_f64", "mhf_last_error", "mhf_version",
                     "mhf_indexed_window_features", "mhf_indexed_window_features_f64",
                     "mhf_window_bounds", "mhf_filtfilt",
                     "mhf_magnitude", "mhf_psd_features", "mhf_orientation", "mhf_gradient",
                     "mhf_zero_crossings", "mhf_magnitude_dot", "mhf_find_peaks_workspace",
                     "mhf_find_peaks", "mhf_find_peaks_cmp", "mhf_minmax", "mhf_fft",
                     "mhf_indexed_workspace", "mhf_filtfilt_workspace",
                     "mhf_magnitude_dot_workspace", "mhf_minmax_workspace", "mhf_fft_workspace",
                     "mhf_plan_name_indexed"}
    for name in decls:
        assert hasattr(L, name), name
    from pymhealth_amd import _lib
    assert set(_lib.EXPORTS) == decls
    assert L.mhf_version() == _lib.MHF_ABI_VERSION
    # nothing else leaks out of the shared object
    import subprocess
    lines = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                           text=True).stdout.splitlines()
    funcs = {ln.split()[-1] for ln in lines if len(ln.split()) == 3 and ln.split()[1] == "T"}
    assert funcs == decls, funcs ^ decls   # (HIP kernel handles are data symbols, 'V')


def test_header_enum_matches_python(L):
    from pymhealth_amd import _lib
    import oracle
    hdr = open(os.path.join(ROOT, "include", "mhfeat.h")).read()
    enum = dict((k, int(v)) for k, v in re.findall(r"(MHF_[A-Z0-9_]+) = (\d+),", hdr))
    for k, v in enum.items():
        assert getattr(_lib, k) == v, k
    assert sorted(oracle.FEATURE_IDS.values()) == list(range(_lib.MHF_NUM_FEATURES))


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 10**6), st.integers(1, 5000), st.integers(1, 5000))
def test_num_windows_property(L, n, w, s):
    from pymhealth_amd.engine import num_windows
    ref = max(0, 1 + (n - w) // s)
    assert L.mhf_num_windows(n, w, s) == ref == num_windows(n, w, s)


def test_num_windows_bad_args(L):
    assert L.mhf_num_windows(10, 0, 1) == -1
    assert L.mhf_num_windows(10, 1, 0) == -1


def _call(L, **kw):
    from pymhealth_amd import _lib
    a = dict(x=1, n=1000, C=1, cs=0, ss=1, W=100, S=100, first=0, nw=10,
             feats=[_lib.MHF_MEAN], params=_lib.make_params(), numerics=0, dtype=0, out=1,
             ld=10)
    a.update(kw)
    ids = np.asarray(a["feats"], np.int32)
    return L.mhf_window_features(
        ctypes.c_void_p(a["x"]), a["n"], a["C"], a["cs"], a["ss"], a["W"], a["S"], a["first"],
        a["nw"], ids.ctypes.data, len(ids), ctypes.byref(a["params"]), a["numerics"],
        a["dtype"], ctypes.c_void_p(a["out"]), a["ld"], None)


def test_argument_validation_without_gpu(L):
    """Every invalid request is rejected on the host before any device call."""
    from pymhealth_amd import _lib
    bad = [dict(W=0), dict(S=0), dict(C=0), dict(ss=0), dict(feats=[99]), dict(feats=[]),
           dict(dtype=5), dict(first=5, nw=10), dict(ld=5), dict(numerics=3),
           dict(feats=[_lib.MHF_BAND_POWER]),  # no fs
           dict(x=0), dict(nw=-1)]
    for b in bad:
        rc = _call(L, **b)
        assert rc == -1, (b, rc)
        assert L.mhf_last_error()
    big = _lib.make_params(fs=10.0)
    assert _call(L, feats=[_lib.MHF_BAND_POWER], W=8192, S=8192, n=8192 * 2, nw=2,
                 params=big) == -2
    assert _call(L, nw=0) == 0          # nothing to do: no device call


def test_block_numerics_validation_without_gpu(L):
    """MHF_NUMERICS_BLOCK(c) (2-D records): one flat channel, wsize / wstep multiples of c,
    only the features the reference evaluates on (rows, c) blocks; checked on the host."""
    from pymhealth_amd import _lib
    blk3 = 3 << 8
    assert _call(L, numerics=blk3, C=3, cs=1, ss=3, W=99, S=99, n=999) == -1   # not flat
    assert _call(L, numerics=blk3, W=100, S=99, n=999) == -1                   # W % 3
    assert _call(L, numerics=blk3, W=99, S=100, n=999) == -1                   # S % 3
    assert _call(L, numerics=blk3, W=99, S=99, n=1000) == -1                   # N % 3
    assert _call(L, numerics=-256) == -1
    for f in (_lib.MHF_ZERO_CROSSINGS, _lib.MHF_PEAK_COUNT, _lib.MHF_HJORTH_MOBILITY,
              _lib.MHF_RMSSD, _lib.MHF_ENTROPY, _lib.MHF_MODE):
        assert _call(L, numerics=blk3, W=99, S=99, n=999, feats=[f]) == -2, f
    assert _call(L, numerics=blk3, W=99, S=99, n=999, nw=0) == 0


def test_f64_entry_validation_without_gpu(L):
    """mhf_window_features_f64: lane, spectral and order-statistic features, same argument
    checks, on the host."""
    from pymhealth_amd import _lib
    ids = np.asarray([_lib.MHF_MEAN], np.int32)
    p = _lib.make_params(fs=10.0)

    def call(feats, numerics=0, W=100, S=100, nw=10, n=1000, x=1):
        f = np.asarray(feats, np.int32)
        return L.mhf_window_features_f64(ctypes.c_void_p(x), n, 1, 0, 1, W, S, 0, nw,
                                         f.ctypes.data, len(f), ctypes.byref(p), numerics, 0,
                                         ctypes.c_void_p(1), nw, None)
    # spectral features of a float64 record: the fp64 transform (spectral64.hip)
    assert call([_lib.MHF_BAND_POWER], nw=0) == 0
    assert call([_lib.MHF_BAND_POWER], W=5000, S=5000, n=50000) == -2
    assert call([_lib.MHF_BAND_POWER], numerics=2 << 8, W=100, S=100, n=1000) == -2
    p.fs = 0.0
    assert call([_lib.MHF_DOMINANT_FREQ]) == -1
    p.fs = 10.0
    # float64 sampen / RQA: fp64 samples in LDS (8192 / 5460 samples per window)
    assert call([_lib.MHF_SAMPEN], W=9000, S=9000, n=90000) == -2
    assert call([_lib.MHF_RQA_RR], W=6000, S=6000, n=60000) == -2
    assert call([_lib.MHF_SAMPEN, _lib.MHF_RQA_RR], nw=0) == 0
    # float64 order statistics: 64-bit keys, windows up to 8192 samples x channels
    assert call([_lib.MHF_MEDIAN], W=9000, S=9000, n=90000) == -2
    assert call([_lib.MHF_MEDIAN], nw=0) == 0
    p.percentile_q = 101.0
    assert call([_lib.MHF_PERCENTILE]) == -1
    p.percentile_q = 50.0
    assert call([_lib.MHF_MEAN], W=0) == -1
    assert call([_lib.MHF_MEAN], numerics=3 << 8, W=99, S=99, n=999, nw=0) == 0
    assert call([_lib.MHF_ZERO_CROSSINGS], numerics=3 << 8, W=99, S=99, n=999) == -2
    assert call([_lib.MHF_MEAN], nw=0) == 0
    del ids


def test_caller_workspaces_without_gpu(L):
    """ABI 7: the library allocates nothing. Every entry point with device scratch takes a
    caller-owned workspace sized by its mhf_*_workspace query (the reference's
    FFI is caller-owned buffers, fft/_fftw_binder.py:11-17), and an undersized one fails
    with MHF_EINVAL, naming the bytes needed, before any device call (so on the host)."""
    from pymhealth_amd import _lib
    vp = ctypes.c_void_p
    # queries: exact sizes
    assert L.mhf_filtfilt_workspace(1000, 3, 6, 6) == 8 * 3 * (1000 + 2 * 18)
    assert L.mhf_filtfilt_workspace(0, 3, 6, 6) == -1
    assert L.mhf_magnitude_dot_workspace(10_000) == 3 * 40 * 8
    assert L.mhf_magnitude_dot_workspace(10 ** 9) == 3 * 1024 * 8
    assert L.mhf_minmax_workspace(1000, _lib.MHF_DTYPE_F32) > 0
    assert L.mhf_minmax_workspace(1000, 9) == -1
    assert L.mhf_fft_workspace(4096, 2) >= 2048 * 16
    assert L.mhf_fft_workspace(8192, 3) >= 3 * 8192 * 16     # global passes: a work copy
    assert L.mhf_fft_workspace(1000, 1) > 2048 * 16           # Bluestein: M = 2048 rows
    assert L.mhf_fft_workspace(7, 0) == 0
    mom = np.asarray([_lib.MHF_MEAN, _lib.MHF_SKEWNESS], np.int32)
    med = np.asarray([_lib.MHF_MEAN, _lib.MHF_MEDIAN], np.int32)
    assert L.mhf_indexed_workspace(100000, 1, _lib.MHF_DTYPE_F32, mom.ctypes.data, 2) == 0
    small = L.mhf_indexed_workspace(100, 1, _lib.MHF_DTYPE_F32, med.ctypes.data, 2)
    big = L.mhf_indexed_workspace(100000, 1, _lib.MHF_DTYPE_F32, med.ctypes.data, 2)
    assert small == 256 and big == 256 + 256 * 131072 * 4
    assert L.mhf_indexed_workspace(100000, 1, _lib.MHF_DTYPE_F64, med.ctypes.data, 2) == \
        256 + 256 * 131072 * 8
    # undersized workspaces: MHF_EINVAL before any launch
    b = np.asarray([0.2, 0.3], np.float64)
    a = np.asarray([1.0, -0.5], np.float64)
    rc = L.mhf_filtfilt(vp(16), 1000, 1, 0, 1, b.ctypes.data, 2, a.ctypes.data, 2, None, 0,
                        vp(16), 0, 1, vp(16), L.mhf_filtfilt_workspace(1000, 1, 2, 2) - 8, None)
    assert rc == -1 and b"filtfilt workspace too small" in L.mhf_last_error()
    assert L.mhf_filtfilt(vp(16), 1000, 1, 0, 1, b.ctypes.data, 2, a.ctypes.data, 2, None, 0,
                          vp(16), 0, 1, None, 10 ** 9, None) == -1
    rc = L.mhf_magnitude_dot(vp(16), vp(16), vp(16), 10_000, 1, _lib.MHF_DTYPE_F32, vp(16),
                             vp(16), 100, None)
    assert rc == -1 and b"960 bytes needed" in L.mhf_last_error()
    rc = L.mhf_minmax(vp(16), 1000, 1, _lib.MHF_DTYPE_F64, vp(16), vp(16), 8, None)
    assert rc == -1 and b"minmax workspace too small" in L.mhf_last_error()
    rc = L.mhf_fft(vp(16), vp(16), 1000, 1, -1, 1.0, vp(16), 1024, None)
    assert rc == -1 and b"fft workspace too small" in L.mhf_last_error()
    for entry in (L.mhf_indexed_window_features, L.mhf_indexed_window_features_f64):
        for ws, nb in ((None, 0), (vp(16), 8)):
            rc = entry(vp(16), 100, 1, 0, 1, vp(16), vp(16), 4, 1, med.ctypes.data, 2,
                       ctypes.byref(_lib.make_params()), 0, vp(16), 4, ws, nb, None)
            assert rc == -1 and b"workspace" in L.mhf_last_error()


def test_rolling_apply_2d_rejects_row_indexing_features():
    """On a 2-D record the reference fails for zero crossings / peaks / Hjorth mobility
    (numba TypingError); the drop-in refuses them before any device call."""
    import pymhealth_amd.features as F
    from pymhealth_amd.util.windows import rolling_apply
    x = np.zeros((100, 3), np.float32)
    for f in (F.zero_crossing_count, F.peak_count, F.hjorth_mobility):
        with pytest.raises(TypeError, match="2-D"):
            rolling_apply(f, 10, 10)(x)
    with pytest.raises(TypeError, match="2-D"):
        rolling_apply([np.mean, F.peak_count], 10, 10)(x)


def test_plan_names(L):
    from pymhealth_amd import _lib
    ids = np.asarray([_lib.MHF_MEAN, _lib.MHF_BAND_POWER], np.int32)
    assert L.mhf_plan_name(1, 0, 1, 100, 100, ids.ctypes.data, 2, 0).decode()
    assert L.mhf_plan_name(0, 0, 1, 100, 100, ids.ctypes.data, 2, 0) is None


def test_register_tile_plans(monkeypatch):
    """Which kernel a request takes (host-side planning, no GPU): W in {128, 256} at a 16-B
    stride -> the fixed tile; any other W <= 288 at any step -> the register tile of
    tile_idx.hip.h (tile_fix); indexed windows -> tile_idx, unless a feature needs the lane
    walk; longer W, strided channels and float64 records keep their kernels. The diagnostic
    opt-outs MHF_NO_TILE_FIX / MHF_NO_TILE_IDX (read at every call) restore the span kernel
    and the lane walk — only while MHF_DIAGNOSTICS=1 is set too."""
    import torch
    from pymhealth_amd.engine import plan_name, plan_name_indexed
    for v in ("MHF_NO_TILE_FIX", "MHF_NO_TILE_IDX", "MHF_DIAGNOSTICS", "MHF_FORCE_GENERIC"):
        monkeypatch.delenv(v, raising=False)
    f = bench_ids(["mean", "var", "skewness", "kurtosis"])
    fi = bench_ids(["mean", "var", "skewness", "kurtosis", "zero_crossings"])
    shapes = [(250, 125, 1), (288, 1, 3), (100, 300, 1), (1, 1, 3), (256, 101, 1)]
    assert plan_name((1, 0, 1), 256, 256, f) == "tile_w256_c1"
    assert plan_name((3, 1, 3), 256, 128, f) == "tile_w256_c3"
    for W, S, C in shapes:
        assert plan_name((C, 1 if C > 1 else 0, C), W, S, f) == "tile_fix", (W, S, C)
    assert plan_name((1, 0, 1), 289, 100, f) == "span"
    assert plan_name((1, 0, 1), 1024, 128, f) == "span"
    assert plan_name((1, 0, 1), 250, 125, bench_ids(["mean", "hjorth_mobility"])) == "span"
    assert plan_name((1, 0, 2), 250, 125, f) == "span"           # strided: not AoS
    assert plan_name_indexed((3, 1, 3), fi) == "tile_idx"
    assert plan_name_indexed((1, 0, 1), fi) == "tile_idx"
    assert plan_name_indexed((3, 1, 3), bench_ids(["mean", "rmssd"])) == "moments_indexed"
    assert plan_name_indexed((3, 1, 3), bench_ids(["mean", "median"])) == "tile_idx+order/pairwise"
    assert plan_name_indexed((3, 1, 3), fi, dtype=torch.float64) == "moments_indexed_f64"
    # a stray switch alone changes nothing: the library honours its diagnostic switches
    # only while MHF_DIAGNOSTICS=1 is set too (engine_common.h diag_env)
    monkeypatch.setenv("MHF_NO_TILE_FIX", "1")
    monkeypatch.setenv("MHF_NO_TILE_IDX", "1")
    monkeypatch.setenv("MHF_FORCE_GENERIC", "1")
    for W, S, C in shapes:
        assert plan_name((C, 1 if C > 1 else 0, C), W, S, f) == "tile_fix", (W, S, C)
    assert plan_name((1, 0, 1), 256, 256, f) == "tile_w256_c1"
    assert plan_name_indexed((3, 1, 3), fi) == "tile_idx"
    monkeypatch.delenv("MHF_FORCE_GENERIC")
    monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
    for W, S, C in shapes:
        assert plan_name((C, 1 if C > 1 else 0, C), W, S, f) == "span", (W, S, C)
    assert plan_name_indexed((3, 1, 3), fi) == "moments_indexed"


def bench_ids(names):
    from pymhealth_amd import _lib
    return [getattr(_lib, "MHF_" + n.upper()) if hasattr(_lib, "MHF_" + n.upper())
            else _lib.FEATURE_IDS[n] for n in names]


def test_algorithmic_bytes(L):
    # 3 channels x (256 samples x 4 B + 5 features x 8 B) per window
    assert L.mhf_algorithmic_bytes(0, 3, 256, 256, 1000, 5, 0) == 1000 * 3 * (1024 + 40)
    # overlapping windows: distinct samples read once
    assert L.mhf_algorithmic_bytes(0, 1, 1024, 128, 10, 2, 1) == (9 * 128 + 1024) * 4 + 80


def test_resolve_and_groups():
    import pymhealth_amd.features as F
    from pymhealth_amd import _lib
    from pymhealth_amd.feature import plan_groups, resolve
    assert resolve(np.mean).fid == _lib.MHF_MEAN
    assert resolve(np.var).fid == _lib.MHF_VAR
    assert resolve(np.std).fid == _lib.MHF_STD
    z = resolve(functools.partial(F.zero_crossing_count, th=0.25))
    assert z.fid == _lib.MHF_ZERO_CROSSINGS and z.params["zc_threshold"] == 0.25
    with pytest.raises(TypeError):
        resolve(lambda w: 0)
    with pytest.raises(TypeError):
        resolve(np.percentile)
    fs = 50.0
    g = plan_groups([resolve(f) for f in (
        F.mean, F.band_power(fs, 0.5, 4), F.relative_band_power(fs, 0.5, 4),
        F.dominant_frequency(fs, 0.5, 8), F.spectral_entropy(fs), F.band_power(fs, 4, 8))])
    assert [i for i, _ in g] == [[0, 1, 2, 3, 4], [5]]
    with pytest.raises(ValueError):
        plan_groups([resolve(F.band_power(None))])


def test_user_callable_resolution_and_host_loop():
    """rolling_apply of a callable the engine has no kernel for (windows.py:93 JIT-compiles
    any callable): resolved to a UserCallable, evaluated window by window over the same
    windows into float64 rows, one warning per callable; known functions never take that
    path, misuses of them still raise. The user-only call needs no GPU (no engine feature
    in the list)."""
    import warnings
    import golden_cases as gc
    import pymhealth_amd.features as F
    from pymhealth_amd.util.windows import UserCallable, _resolve, rolling_apply
    for f in (np.mean, np.var, np.median, F.skewness, functools.partial(np.percentile, q=5)):
        assert not isinstance(_resolve(f), UserCallable)
    with pytest.raises(TypeError):
        _resolve(np.percentile)
    with pytest.raises(TypeError):
        _resolve(functools.partial(F.zero_crossing_count, bogus=1))
    with pytest.raises(TypeError):
        _resolve(3.0)
    d = gc.load("surface_user_callables")

    def first_last(w):
        return w[0] * 2.0 + w[-1]

    assert isinstance(_resolve(first_last), UserCallable)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        got = rolling_apply(first_last, int(d["wsize"]), int(d["wstep"]))(d["x"])
        rolling_apply(first_last, int(d["wsize"]), int(d["wstep"]))(d["x"])
    assert sum("no MI355X kernel" in str(w.message) for w in rec) == 1
    # numba types w[0] * 2.0 of a float32 window in float64, numpy 2 (NEP 50) in float32:
    # user code evaluated by numpy matches the reference to float32 rounding, not bit for bit
    assert got.dtype == np.float64
    np.testing.assert_allclose(got, d["out_first_last"], rtol=1e-6, atol=1e-7)
    # vector-valued user function: np.zeros((nw, *shape)) (windows.py:88-89)
    out = rolling_apply(lambda w: w[:2], 4, 4)(np.arange(10, dtype=np.float32))
    assert out.shape == (2, 2) and (out == [[0, 1], [4, 5]]).all()
    assert rolling_apply(lambda w: 1.0, 16, 16)(np.ones(8)).shape == (0,)


@pytest.mark.parametrize("case", ["nu_user_float32", "nu_user_float64"])
def test_indexed_user_callable_host_loop(case):
    """indices_rolling_apply of a user callable (windows.py:134-157 JIT-compiles any func):
    the host loop over the fixture's own (2, n) indices, out dtype = the record's
    (np.zeros(n, arr.dtype)), NaN below min_window_len — against the reference's output on
    the same windows. Needs no GPU (no engine feature in the call)."""
    import warnings
    import golden_cases as gc
    from pymhealth_amd.util.windows import indices_rolling_apply
    d = gc.load(case)
    ml = int(d["min_window_len"])

    def rng_(w):
        return w.max() - w.min()

    def first_last(w):
        return w[0] * 2.0 + w[-1]

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        got = indices_rolling_apply(rng_, ml)(d["indices"], d["x"])
        fl = indices_rolling_apply(first_last, ml)(d["indices"], d["x"])
    assert got.dtype == d["x"].dtype and got.shape == d["irap_range"].shape
    # max - min is one rounding in either typing: bit for bit (NaN where the window is short)
    assert gc.same(got, d["irap_range"]).all()
    assert np.isnan(got).sum() > 0
    # w[0] * 2.0 + w[-1]: numba widens to float64, numpy keeps float32 (NEP 50)
    np.testing.assert_allclose(fl, d["out_first_last"], rtol=1e-6, atol=1e-7, equal_nan=True)


def test_drop_in_surface_argument_checks():
    """Host-side checks of the module functions added for the drop-in surface (no GPU
    compute): find_peaks comparison ufuncs, old-style power_band calls, fft namespace."""
    import pymhealth_amd
    from pymhealth_amd import _lib
    pymhealth_amd.install_mhealth_alias()
    import mhealth.fft as mfft
    from mhealth.generic import stats, timedom
    from mhealth.heart import hrv, qrs
    assert callable(mfft.fft) and callable(mfft.ifft)
    assert callable(stats.minmax) and callable(timedom.hjorth_parameters)
    assert callable(timedom.hjorth_mobility_derivative)
    assert callable(timedom.hjorth_complexity_derivatives)
    assert qrs._COMPARISONS[np.greater_equal] == _lib.MHF_CMP_GREATER_EQUAL
    with pytest.raises(TypeError, match="comp must be"):
        qrs.find_peaks(np.ones(5), np.equal)
    with pytest.raises(TypeError, match="features.band_power"):
        hrv.power_band(50.0, 0.5, 4.0)


def test_mhealth_alias_and_reference_module_paths():
    import pymhealth_amd
    pymhealth_amd.install_mhealth_alias()
    from mhealth.util.windows import rolling_apply, view, array_shape  # noqa: F401
    from mhealth.generic import stats, timedom  # noqa: F401
    from mhealth.generic.frequency import density  # noqa: F401
    from mhealth.heart import hrv, qrs  # noqa: F401
    import mhealth.features  # noqa: F401
    import mhealth.processing  # noqa: F401
    assert stats.mean is np.mean and stats.var is np.var and stats.std is np.std
    assert rolling_apply(stats.skewness, 4, 4) is rolling_apply(stats.skewness, 4, 4)
    x = np.arange(10.0)
    v = view(x, 4, 3)
    assert v.shape == (3, 4) and (v[1] == x[3:7]).all()
    assert array_shape(1.0) == () and array_shape(np.zeros((2, 3))) == (2, 3)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import pymhealth_amd.features as F
    with pytest.raises(RuntimeError, match="no CPU path"):
        F.skewness(np.ones(8, np.float32))
    with pytest.raises(RuntimeError):
        pymhealth_amd_ra = __import__("pymhealth_amd").util.windows.rolling_apply
        pymhealth_amd_ra(np.mean, 4, 4)(np.ones(8, np.float32))


# ------------------------------------------- nonuniform windows: host-side bounds planning
def _golden_nonuniform():
    import golden_cases as gc
    return [(c, gc.load(c)) for c in gc.nonuniform_cases()]


def test_bounds_plan_matches_reference_window_count():
    import golden_cases as gc
    from pymhealth_amd import _lib
    from pymhealth_amd.util.windows import _bounds_plan
    for case, d in _golden_nonuniform():
        idx, nw, mode, t0, wstep, wsize = _bounds_plan(*gc.nonuniform_args(d))
        assert nw == d["indices"].shape[1], case
        float_step = case == "nu_float_step"
        assert bool(mode & _lib.MHF_BOUNDS_FLOAT_STARTS) == float_step
        assert idx.dtype == np.int64 and t0 == idx[0]


def test_bounds_plan_units_and_modes():
    from pymhealth_amd import _lib
    from pymhealth_amd.util.windows import _bounds_plan
    idx = (np.datetime64("2024-01-01T00:00:00", "s")
           + np.arange(0, 100, 3).astype("timedelta64[s]"))
    # finest unit of (index, wstep, wsize) wins: ms here
    i64, nw, mode, t0, step, size = _bounds_plan(idx, np.timedelta64(2500, "ms"),
                                                 np.timedelta64(7, "s"))
    assert mode == 0 and step == 7000 and size == 2500 and i64[1] - i64[0] == 3000
    assert nw == len(np.arange(idx[0], idx[-1], np.timedelta64(7, "s")))
    ints = np.arange(0, 1000, 7, dtype=np.int64)
    assert _bounds_plan(ints, 10.5, 4)[2] == _lib.MHF_BOUNDS_FLOAT_ENDS
    assert _bounds_plan(ints, 10, 4.5)[2] == (_lib.MHF_BOUNDS_FLOAT_STARTS
                                              | _lib.MHF_BOUNDS_FLOAT_ENDS)
    for step in (4, 4.5, 0.3, 1e3):
        assert _bounds_plan(ints, 10, step)[1] == len(np.arange(ints[0], ints[-1], step))
    with pytest.raises(TypeError):
        _bounds_plan(ints.astype(np.float64), 10, 4)
    with pytest.raises(TypeError):
        _bounds_plan(idx, 10, 4)
    with pytest.raises(IndexError):
        _bounds_plan(np.zeros(0, np.int64), 10, 4)
    with pytest.raises(ValueError):
        _bounds_plan(ints, 10, 0)


def test_butterworth_design_matches_reference():
    """Filter design stays on the host, as in the reference (filters.py:31-34)."""
    import golden_cases as gc
    from pymhealth_amd.generic.filters import design
    d = gc.load("n2_filters")
    for k, (cut, ftype, order) in {"hp": (0.5, "highpass", 5), "lp": (0.5, "lowpass", 5),
                                   "bp": ((0.5, 10.0), "bandpass", 5),
                                   "lp8": (3.0, "lowpass", 8)}.items():
        b, a, zi = design(cut, 50.0, order, ftype)
        np.testing.assert_allclose(b, d["b_" + k], rtol=1e-12, atol=1e-18)
        np.testing.assert_allclose(a, d["a_" + k], rtol=1e-12, atol=0)
        np.testing.assert_allclose(zi, d["zi_" + k], rtol=1e-7, atol=1e-9)


def _c_decls(text):
    """{name: (return type, [parameter types])} and the mhf_params fields of C text
    (comments, parameter names and MHF_API stripped; whitespace normalised)."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    types = {"const", "int", "int32_t", "int64_t", "uint64_t", "double", "float", "void",
             "char", "mhf_params"}

    def norm(p):
        p = re.sub(r"\s*\*\s*", "* ", p.strip()).split()
        if len(p) > 1 and p[-1] not in types and not p[-1].endswith("*"):
            p = p[:-1]
        return " ".join(p).replace("* ", "*").strip()

    decls = {}
    for ret, name, params in re.findall(
            r"(?:MHF_API\s+)?((?:const\s+)?\w+\s*\*?)\s*(mhf_\w+)\s*\(([^)]*)\)\s*;", text):
        ps = [norm(p) for p in params.split(",")]
        decls[name] = (norm(ret + " x"), [] if ps == ["void"] else ps)
    st = re.search(r"typedef struct(?: mhf_params)?\s*\{(.*?)\}\s*mhf_params;", text, re.S)
    fields = []
    for line in st.group(1).split(";"):
        toks = line.replace(",", " , ").split()
        if not toks:
            continue
        ty = toks[0]
        fields += [(ty, t) for t in toks[1:] if t != ","]
    return decls, fields


def test_integration_cdef_matches_header():
    """INTEGRATION.md's cffi cdef declares exactly the header's struct fields and
    prototypes (cffi is not importable here: compared textually)."""
    hdr_decls, hdr_fields = _c_decls(open(os.path.join(ROOT, "include", "mhfeat.h")).read())
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    cdef = re.search(r'ffi\.cdef\("""(.*?)"""\)', doc, re.S).group(1)
    doc_decls, doc_fields = _c_decls(cdef)
    assert doc_fields == hdr_fields
    assert len(hdr_fields) == 14 and hdr_fields[7] == ("double", "csi_factor")
    assert doc_decls == hdr_decls, {k for k in set(doc_decls) | set(hdr_decls)
                                    if doc_decls.get(k) != hdr_decls.get(k)}
    from pymhealth_amd import _lib
    assert set(hdr_decls) == set(_lib.EXPORTS)
    assert "mhf_version() == %d" % _lib.MHF_ABI_VERSION in doc


def _sampen_walk_counts(x, mm, t32):
    """sampen_kernel's match-word walk (order.hip sampen_words) restated in Python: lane l
    takes the snake diagonals d1 = 64q + l + 1 and d2 = 64q + 128 - l of each round pair;
    each diagonal's positions go 32 at a time into words (bit 31 - k: position p0 + k
    matches), positions past the diagonal's end are 0, and with the previous word shifted
    in (alignbit) A += popc(w & w>>1 & .. & w>>mm), B += popc(w & .. & w>>(mB-1)) without
    the diagonal's last position (j = n - 1)."""
    n = len(x)
    nd, mB = n - 1, max(mm, 1)
    M = 0xffffffff
    A = B = 0

    def alignbit(hi, lo, sh):
        return (((hi << 32) | lo) >> sh) & M
    for lane in range(64):
        q = 0
        while q * 64 < nd:
            d1, d2 = 64 * q + lane + 1, 64 * q + 128 - lane
            len1 = n - d1 if d1 <= nd else 0
            len2 = n - d2 if d2 <= nd else 0
            for d, ln in ((d1, len1), (d2, len2)):
                prev = 0
                for p0 in range(0, max(len1, len2), 32):
                    w = 0
                    for k in range(32):
                        i = p0 + k
                        c = i < ln and abs(np.float32(x[i + d]) - np.float32(x[i])) < t32
                        w = ((w << 1) | int(c)) & M
                    r = ln - p0
                    last = ~(1 << (32 - r)) & M if 1 <= r <= 32 else M
                    a = b = w
                    for sh in range(1, mm + 1):
                        sv = alignbit(prev, w, sh)
                        a &= sv
                        if sh < mB:
                            b &= sv
                    A += bin(a).count("1")
                    B += bin(b & last).count("1")
                    prev = w
            q += 2
    return A, B


def _pos_bits(lo, ln, p0):
    """order.hip pos_bits: the bits of positions [lo, lo + ln) in the word of p0 .. p0+31."""
    M = ((((1 << ln) - 1) if ln < 32 else (1 << 64) - 1) << 32) & ((1 << 64) - 1)
    sh = min(max(lo - p0 + ln, 0), 64)
    return 0 if sh >= 64 else (M >> sh) & 0xffffffff


def _sampen_cyclic_counts(x, mm, t32):
    """sampen_kernel's cyclic-diagonal walk (order.hip sampen_cyclic) restated in Python:
    stream e of lane l (e = s0 + l, s0 + 64 + l) pairs (i, (i + d) mod n), d = e + 1, over a
    doubled copy of the window — diagonal d then diagonal n - d, boundary b = n - d; the
    stream's words as in the straight walk, with A's chains cleared over [b, b + mm), B's
    over [b, b + mB - 1) and at both diagonals' last positions b - 1 and L - 1."""
    n = len(x)
    mB = max(mm, 1)
    M = 0xffffffff
    xx = np.concatenate([x, x, np.zeros(192, np.float32)])
    ncyc = (n - 1) >> 1
    nstr = ncyc + (1 if n % 2 == 0 else 0)
    A = B = 0

    def alignbit(hi, lo, sh):
        return (((hi << 32) | lo) >> sh) & M
    for s0 in range(0, nstr, 128):
        for lane in range(64):
            streams = []
            for e in (s0 + lane, s0 + 64 + lane):
                ln = n if e < ncyc else ((n >> 1) if e < nstr else 0)
                streams.append((e + 1 if ln > 0 else 1, ln))
            lmax = max(ln for _, ln in streams)
            for d, ln in streams:
                b = n - d
                kb = ((b - 1) >> 5) << 5
                two = b < ln
                cA = (_pos_bits(b, mm, kb) if two else 0, _pos_bits(b, mm, kb + 32) if two else 0)
                cB = ((_pos_bits(b, mB - 1, kb) if two else 0) | _pos_bits(b - 1, 1, kb),
                      _pos_bits(b, mB - 1, kb + 32) if two else 0)
                prev = 0
                for p0 in range(0, lmax, 32):
                    w = 0
                    for k in range(32):
                        c = abs(np.float32(xx[p0 + k + d]) - np.float32(xx[p0 + k])) < t32
                        w = ((w << 1) | int(c)) & M
                    r = ln - p0
                    keep = M if r >= 32 else (0 if r <= 0 else (M << (32 - r)) & M)
                    lastb = (1 << (32 - r)) if 1 <= r <= 32 else 0
                    w &= keep
                    a = bb = w
                    for sh in range(1, mm + 1):
                        sv = alignbit(prev, w, sh)
                        a &= sv
                        if sh < mB:
                            bb &= sv
                    ma = cA[0] if p0 == kb else (cA[1] if p0 == kb + 32 else 0)
                    mb = (cB[0] if p0 == kb else (cB[1] if p0 == kb + 32 else 0)) | lastb
                    A += bin(a & ~ma & M).count("1")
                    B += bin(bb & ~mb & M).count("1")
                    prev = w
    return A, B


def test_sampen_kernel_walk_counts_match_reference_loop():
    """The counts of both sample-entropy walks (straight and cyclic diagonals) equal the
    reference's pair loop
    (information.py:23-113: per diagonal run length L of |x[j] - x[i]| < r, a[m] for
    L >= m + 1, b[m] for L >= m with j <= n - 2): windows shorter and longer than one
    round of 64 diagonals, ties at r, m = 1 .. 3."""
    rng = np.random.default_rng(4)
    for n in (2, 3, 33, 40, 64, 65, 129, 200):
        for mm in (0, 1, 2, 3, 5):
            x = (np.round(rng.standard_normal(n) * 4) / 4).astype(np.float32)
            r = 0.25                        # a multiple of the grid: ties |d| == r
            A, B = _sampen_walk_counts(x, mm, np.float32(r))
            Ac, Bc = _sampen_cyclic_counts(x, mm, np.float32(r))
            a = b = 0
            for d in range(1, n):
                L = 0
                for i in range(n - d):
                    j = i + d
                    L = L + 1 if float(abs(np.float32(x[j]) - np.float32(x[i]))) < r else 0
                    a += L >= mm + 1
                    b += (L >= mm) and L > 0 and j <= n - 2
            assert A == a and (mm == 0 or B == b), (n, mm)
            assert Ac == a and (mm == 0 or Bc == b), ("cyclic", n, mm)



def _select_rank(keys, k):
    """order.hip select_rank_u32 restated: the largest P with #{keys < P} <= k, bit by bit
    from the top, two steps per exit test; once [P, top) holds one key (hi - lo == 1) the
    answer is the smallest key >= P."""
    P, lo, hi = 0, 0, len(keys)
    for b in range(31, 0, -2):
        for bb in (b, b - 1):
            T = P | (1 << bb)
            cnt = int((keys < T).sum())
            if cnt <= k:
                P, lo = T, cnt
            else:
                hi = cnt
        if hi - lo == 1:
            return int(keys[keys >= P].min())
    return P


def test_rank_selection_matches_sorting():
    """The bit-serial rank search of the order kernel's selection path returns the k-th
    smallest key for every rank, on distinct keys, heavy ties and the padding keys (all
    ones) of short windows — the value the sorting path reads off the sorted keys."""
    rng = np.random.default_rng(12)
    for it in range(600):
        n = int(rng.integers(1, 257))
        kind = it % 3
        if kind == 0:
            x = rng.integers(0, 2 ** 32, size=256, dtype=np.uint64)
        elif kind == 1:
            x = rng.integers(0, 5, size=256, dtype=np.uint64) * 12345
        else:
            x = np.sort(rng.integers(0, 2 ** 32, size=256, dtype=np.uint64))
        x[n:] = 2 ** 32 - 1
        srt = np.sort(x)
        for k in {0, n // 2, n - 1, int(rng.integers(0, n))}:
            assert _select_rank(x, k) == srt[k], (it, n, k)


def _select_pair(keys, k):
    """order.hip select_two_u32 restated: ranks k and k + 1 from one search (early exit:
    the smallest keys >= P and >= top; a full search: P, then P again or the smallest key
    above it)."""
    P, lo, hi = 0, 0, len(keys)
    for b in range(31, 0, -2):
        for bb in (b, b - 1):
            T = P | (1 << bb)
            cnt = int((keys < T).sum())
            if cnt <= k:
                P, lo = T, cnt
            else:
                hi = cnt
        if hi - lo == 1:
            top = P + (1 << (b - 1))
            assert top < 2 ** 32
            return int(keys[keys >= P].min()), int(keys[keys >= top].min())
    if hi > k + 1:
        return P, P
    return P, int(keys[keys > P].min())


def _select_multi(keys, k, two):
    """order.hip select_multi_u32 restated for one of its interleaved searches: the search
    starts below the common prefix of the minimum and maximum key, a step at bit 0 is a
    no-op, the loop ends (two steps per test) once the range holds one key or the bits are
    used up; then rank k = the smallest key >= P, rank k + 1 = the same key when more than
    k + 1 keys lie below top, else the smallest key >= top."""
    mn, mx = int(keys.min()), int(keys.max())
    d = mn ^ mx
    hb = (1 << (d.bit_length() - 1)) if d else 0
    P = mn & ~((hb << 1) - 1) & 0xFFFFFFFF if hb else mn
    lo, hi, bit = 0, len(keys), hb
    for _ in range(16):
        for _ in range(2):
            T = P | bit
            cnt = int((keys < T).sum())
            if cnt <= k:
                P, lo = T, cnt
            else:
                hi = cnt
            bit >>= 1
        if not (bit and hi - lo - 1):
            break
    k0 = int(keys[keys >= P].min())
    if not two or hi > k + 1:
        return k0, k0
    top = P + ((bit << 1) if bit else 1)
    assert top < 2 ** 32
    return k0, int(keys[keys >= top].min())


def _key_value(kv):
    u = (kv & 0x7FFFFFFF) if kv & 0x80000000 else (~kv) & 0xFFFFFFFF
    return np.array([u], dtype=np.uint32).view(np.float32)[0]


def _float_key(f):
    b = int(np.array([f], dtype=np.float32).view(np.uint32)[0])
    return (b ^ 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)


def _select_range(keys, k, two, ninterp=3):
    """order.hip select_range_u32 restated: the range [P, Q] from the minimum and maximum
    key, MHF_SEL_NINTERP = 3 thresholds interpolated in value space (clamped into (P, Q]), then halving;
    rank k = the smallest key >= P, rank k + 1 = the same value when hi > k + 1, else the
    smallest key > Q. The interpolation is float32 here and an approximate reciprocal on
    the device: any threshold in (P, Q] gives the same ranks."""
    P, Q, lo, hi = int(keys.min()), int(keys.max()), 0, len(keys)

    def step(T):
        nonlocal P, Q, lo, hi
        cnt = int((keys < T).sum())
        if cnt <= k:
            P, lo = T, cnt
        else:
            Q, hi = T - 1, cnt
    with np.errstate(all="ignore"):
        for _ in range(ninterp):
            if hi - lo <= 1 or Q <= P:
                break
            a, b = _key_value(P), _key_value(Q)
            fr = np.float32((k - lo) + 0.5) / np.float32(hi - lo)
            T = _float_key(np.float32(a + (b - a) * fr))
            step(min(max(T, P + 1), Q))
    while hi - lo > 1 and Q > P:
        step(P + ((Q - P) >> 1) + 1)
    k0 = int(keys[keys >= P].min())
    if not two or hi > k + 1:
        return k0, k0
    return k0, int(keys[keys > Q].min())


def test_range_rank_selection_matches_sorting():
    """The selection kernel's range search (value-interpolated then halved thresholds)
    returns ranks k and k + 1 of the sorted keys: ties, constant windows, shared prefixes,
    NaN-key padding, signed values."""
    rng = np.random.default_rng(19)
    for it in range(800):
        n = int(rng.integers(2, 257))
        kind = it % 6
        if kind == 0:
            x = rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64)
        elif kind == 1:
            x = rng.integers(0, 4, size=256, dtype=np.uint64) * 777
        elif kind == 2:
            x = np.full(256, int(rng.integers(0, 2 ** 32 - 1)), dtype=np.uint64)
        elif kind == 3:
            x = 0xBF000000 + rng.integers(0, 2 ** 22, size=256, dtype=np.uint64)
        elif kind == 4:   # float keys of a signed sinusoid plus noise
            f = (0.3 * np.sin(np.arange(256) * 0.2 + it) + 0.05 * rng.standard_normal(256)).astype(np.float32)
            x = np.array([_float_key(v) for v in f], dtype=np.uint64)
        else:
            x = np.sort(rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64))
        if it % 2:
            x[n:] = 2 ** 32 - 1
        else:
            n = 256
        srt = np.sort(x)
        for k in {0, n // 2 - 1, (n - 1) // 2, n - 2, int(rng.integers(0, n - 1))}:
            assert _select_range(x, k, True) == (srt[k], srt[k + 1]), (it, n, k)
            assert _select_range(x, k, False)[0] == srt[k], (it, n, k)


def test_interleaved_rank_selection_matches_sorting():
    """The order kernel's interleaved search of the vector path (np.median alone: the
    channels' searches in step, each from its keys' common prefix) returns ranks k and
    k + 1 of the sorted keys: ties, constant windows, shared prefixes, padding."""
    rng = np.random.default_rng(17)
    for it in range(800):
        n = int(rng.integers(2, 257))
        kind = it % 5
        if kind == 0:
            x = rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64)
        elif kind == 1:
            x = rng.integers(0, 4, size=256, dtype=np.uint64) * 777
        elif kind == 2:
            x = np.full(256, int(rng.integers(0, 2 ** 32 - 1)), dtype=np.uint64)
        elif kind == 3:   # a shared top byte (z axes near 1 g)
            x = 0xBF000000 + rng.integers(0, 2 ** 22, size=256, dtype=np.uint64)
        else:
            x = np.sort(rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64))
        if it % 2:
            x[n:] = 2 ** 32 - 1
        else:
            n = 256
        srt = np.sort(x)
        for k in {0, n // 2 - 1, (n - 1) // 2, n - 2, int(rng.integers(0, n - 1))}:
            assert _select_multi(x, k, True) == (srt[k], srt[k + 1]), (it, n, k)
            assert _select_multi(x, k, False)[0] == srt[k], (it, n, k)


def test_rank_pair_selection_matches_sorting():
    """The order kernel's two-rank search (median of even windows, percentile
    interpolation) returns ranks k and k + 1 of the sorted keys, ties included."""
    rng = np.random.default_rng(13)
    for it in range(600):
        n = int(rng.integers(2, 257))
        kind = it % 3
        if kind == 0:
            x = rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64)
        elif kind == 1:
            x = rng.integers(0, 4, size=256, dtype=np.uint64) * 777
        else:
            x = np.sort(rng.integers(0, 2 ** 32 - 1, size=256, dtype=np.uint64))
        x[n:] = 2 ** 32 - 1
        srt = np.sort(x)
        for k in {0, n // 2 - 1 if n > 1 else 0, n - 2, int(rng.integers(0, n - 1))}:
            assert _select_pair(x, k) == (srt[k], srt[k + 1]), (it, n, k)


def _run_host_program(name):
    import subprocess
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host")
    subprocess.run(["make", "-s", "-C", here, "_build/" + name], check=True, timeout=300)
    r = subprocess.run([os.path.join(here, "_build", name)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_dma_address_maps_under_asan():
    """The register tiles' LDS-DMA address maps (pymhealth_amd/csrc/dma_map.h, the kernels'
    own expressions), emulated lane by lane on the host under AddressSanitizer + UBSan
    (tests/host/dma_map_emul.cpp): every 16-B piece of every chunk of every tile lies inside
    the record, and every lane the tile path keeps reads exactly its own window's samples —
    for time-indexed windows (short / empty / long / negative / past-the-end), fixed windows
    of any length <= 288 at any step, and the W = 128 / 256 tile, with records placed at
    device addresses whose low 32-bit word is >= 2^31 or that cross a 2^32 boundary (round
    5's GPU fault: a sign-extended readfirstlane word)."""
    out = _run_host_program("dma_map_emul")
    assert "DMA MAPS OK" in out, out


def test_oracle_under_asan():
    """The CPU oracle (test infrastructure) under AddressSanitizer + UBSan
    (tests/host/oracle_asan.c): every feature id over exact-size records of the GPU tests'
    shapes, time-indexed windows, 2-D blocks, float64 records, periodogram rows."""
    out = _run_host_program("oracle_asan")
    assert "ORACLE ASAN OK" in out, out


def test_prof_summary_refuses_clock_when_runs_disagree():
    """tools/prof_summary.py derives the effective clock from a PMC run's GRBM_GUI_ACTIVE and
    the trace run's duration; a clock the part cannot run (the two runs timed different
    things) is reported as not derived rather than as a number."""
    import importlib.util
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("prof_summary",
                                                  os.path.join(here, "tools", "prof_summary.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    ok = ps.clock_line(8 * 2.1e9 * 6.5e-3, 6.5e6)         # 2.1 GHz over 6.5 ms
    assert ok.startswith("effective clock (") and "2.10 GHz" in ok
    bad = ps.clock_line(8 * 2.1e9 * 6.5e-3, 2.0e6)        # busy cycles of 6.5 ms over 2 ms
    assert "NOT derived" in bad and "6.83 GHz" in bad
    low = ps.clock_line(8 * 0.3e9 * 1e-3, 1e6)
    assert "NOT derived" in low
