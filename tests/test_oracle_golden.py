"""The CPU oracle against the reference's own outputs (tests/golden, made by running
pymhealth under numba 0.54.1: make_golden.py). CPU only."""
import numpy as np
import pytest

import golden_cases as gc


@pytest.mark.parametrize("case,key,feat,kw", gc.moment_cases())
def test_moment_feature_bit_exact(oracle_lib, case, key, feat, kw):
    d = gc.load(case)
    x, W, S = d["x"], int(d["wsize"]), int(d["wstep"])
    got = oracle_lib.window_features(x, W, S, [feat], **kw)[0, 0]
    ref = d["out_" + key]
    assert got.shape == ref.shape
    eq = gc.same(got, ref, d.get("raises_" + key))
    assert eq.all(), (np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


@pytest.mark.parametrize("case,key,feat,kw", gc.block_cases())
def test_block2d_feature_bit_exact(oracle_lib, case, key, feat, kw):
    """2-D (N, c) records: window i is the (wsize, c) block (MHF_NUMERICS_BLOCK)."""
    d = gc.load(case)
    x, W, S = d["x"], int(d["wsize"]), int(d["wstep"])
    got = oracle_lib.window_features(x, W, S, [feat], block=True, **kw)[0, 0]
    ref = d["out_" + key]
    assert got.shape == ref.shape
    eq = gc.same(got, ref)
    assert eq.all(), (np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


@pytest.mark.parametrize("case,key,feat,kw", gc.f64_cases())
def test_f64_feature_bit_exact(oracle_lib, case, key, feat, kw):
    """float64 input: numba's fp64 models (every reduction typed from the input)."""
    d = gc.load(case)
    x, W, S = d["x"], int(d["wsize"]), int(d["wstep"])
    assert x.dtype == np.float64
    kw = dict(kw, zc_threshold=gc.ZC_THRESHOLD.get(key, 0.0))
    got = oracle_lib.window_features(x, W, S, [feat], block=x.ndim == 2, **kw)[0, 0]
    ref = d["out_" + key]
    assert got.shape == ref.shape
    if key in gc.LIBM_KEYS:
        np.testing.assert_allclose(got, ref, rtol=gc.LIBM_KEYS[key], atol=0, equal_nan=True)
        return
    eq = gc.same(got, ref, d.get("raises_" + key))
    assert eq.all(), (np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


@pytest.mark.parametrize("case", gc.psd_cases())
def test_psd_level_functions_bit_exact(oracle_lib, case):
    """hrv.power_band / relative_power_band / peak_frequency, density.peak_frequency and
    information.entropy on the reference's own psd rows, every bound pattern."""
    d = gc.load(case)
    for b in gc.PSD_BOUNDS:
        lo, hi = gc.psd_bounds(d, b)
        got = oracle_lib.psd_features(d["psd"], d["freqs"], gc.PSD_FUNCS, lo, hi)
        for j, k in enumerate(gc.PSD_FUNCS):
            ref = d["out_%s_%s" % (k, b)]
            eq = gc.same(got[j], ref, d["raises_%s_%s" % (k, b)])
            assert eq.all(), (b, k, np.nonzero(~eq)[0][:8])
    ent = oracle_lib.psd_features(d["psd"], None, ["entropy"])[0]
    assert gc.same(ent, d["out_entropy"]).all()


def test_cfg1_list_dispatch(oracle_lib):
    d = gc.load("cfg1")
    feats = ["mean", "var", "skewness", "kurtosis"]
    got = oracle_lib.window_features(d["x"], 128, 128, feats)[0]
    for j, f in enumerate(feats):
        assert gc.same(got[j], d["list_" + f]).all()
        assert gc.same(got[j], d["out_" + f]).all()


def test_strided_column_equals_contiguous(oracle_lib):
    aos = gc.load("accel_aos")["x"]
    ref = gc.load("accel_z_strided")["out_skewness"]
    got = oracle_lib.window_features(aos[:, 2], 256, 256, ["skewness"])[0, 0]
    assert gc.same(got, ref).all()
    allc = oracle_lib.window_features(aos, 256, 256, ["skewness"])
    assert gc.same(allc[2, 0], ref).all()


@pytest.mark.parametrize("case", gc.spectral_cases())
def test_spectral_oracle(oracle_lib, case):
    d = gc.load(case)
    got = oracle_lib.window_features(
        d["x"], int(d["wsize"]), int(d["wstep"]), gc.SPECTRAL_FEATURES, fs=float(d["fs"]),
        band=tuple(d["band"]), dom=tuple(d["dom_range"]))[0]
    for j, f in enumerate(gc.SPECTRAL_FEATURES):
        ref = d["out_" + f]
        if f == "relative_band_power":
            ref = np.where(d["raises_relative_band_power"], np.nan, ref)
        np.testing.assert_allclose(got[j], ref, rtol=1e-12, atol=0, equal_nan=True,
                                   err_msg=f)


def test_periodogram_matches_numpy(oracle_lib):
    rng = np.random.default_rng(1)
    for W in (8, 99, 128, 1024):
        win = rng.standard_normal((5, W)).astype(np.float32)
        X = np.fft.rfft(win.astype(np.float64), axis=1)
        ref = (X.real ** 2 + X.imag ** 2) / (10.0 * W)
        if W % 2:
            ref[:, 1:] *= 2
        else:
            ref[:, 1:-1] *= 2
        np.testing.assert_allclose(oracle_lib.periodogram(win, 10.0), ref, rtol=1e-11,
                                   atol=1e-14)


def test_empty_and_num_windows(oracle_lib):
    d = gc.load("empty")
    assert d["out_mean"].shape == (0,)
    assert oracle_lib.num_windows(10, 16, 16) == 0
    got = oracle_lib.window_features(d["x"], 16, 16, ["mean"])
    assert got.shape == (1, 1, 0)
    for n, w, s in [(1000, 256, 100), (256, 256, 1), (255, 256, 1), (0, 1, 1), (5, 3, 1)]:
        assert oracle_lib.num_windows(n, w, s) == max(0, 1 + (n - w) // s)


def test_zc_threshold_rounding(oracle_lib):
    # x > th in fp64 for every fp32 x  <=>  x > t32
    for th in (0.05, 0.1, 1e-8, 0.0, -1.0, 3.0, 1e39):
        t32 = np.float32(oracle_lib.zc_threshold32(th))
        cand = np.array([t32, np.nextafter(t32, np.float32(np.inf)),
                         np.nextafter(t32, np.float32(-np.inf))], np.float32)
        for c in cand:
            assert (float(c) > max(th, 0.0)) == (c > t32)


# ------------------------------------------------ time-indexed (nonuniform) windows (§8f N1)
@pytest.mark.parametrize("case", gc.nonuniform_cases())
def test_nonuniform_get_indices_oracle(oracle_lib, case):
    d = gc.load(case)
    got = oracle_lib.get_indices(*gc.nonuniform_args(d))
    np.testing.assert_array_equal(got, d["indices"])


@pytest.mark.parametrize("case,key,feat", gc.nonuniform_feature_cases())
def test_nonuniform_features_oracle_bit_exact(oracle_lib, case, key, feat):
    d = gc.load(case)
    got = oracle_lib.indexed_features(d["x"], d["indices"], [feat],
                                      min_len=int(d["min_window_len"]), out_dtype=d["x"].dtype,
                                      **gc.FEATURE_KWARGS.get(key, {}))[0, 0]
    ref = d["out_" + key]
    assert got.dtype == ref.dtype == d["x"].dtype      # np.zeros(n, arr.dtype)
    eq = gc.same(got, ref, d.get("raises_" + key))
    assert eq.all(), (np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


def test_nonuniform_list_form_oracle(oracle_lib):
    for case in gc.nonuniform_cases():
        d = gc.load(case)
        if "list_mean" not in d:
            continue
        got = oracle_lib.indexed_features(d["x"], d["indices"], ["mean", "std"],
                                          min_len=int(d["min_window_len"]),
                                          out_dtype=d["x"].dtype)[0]
        assert gc.same(got[0], d["list_mean"]).all() and gc.same(got[1], d["list_std"]).all()


def test_indexed_oracle_python_slice_semantics(oracle_lib):
    """arr[si:ei] with negative / out-of-range / reversed bounds, as the reference's loop
    slices (windows.py:152-156); empty slices are NaN."""
    x = np.arange(10, dtype=np.float32)
    ind = np.array([[-4, 8, 3, 5, -20, 2], [-1, 50, 3, 2, 3, 7]], np.int64)
    got = oracle_lib.indexed_features(x, ind, ["mean"], min_len=0)[0, 0]
    ref = [np.mean(x[s:e]) if len(x[s:e]) else np.nan for s, e in ind.T]
    np.testing.assert_array_equal(got, np.asarray(ref, np.float32))
    got1 = oracle_lib.indexed_features(x, ind, ["mean"], min_len=2)[0, 0]
    assert np.isnan(got1[[2, 3]]).all() and got1[0] == np.float32(np.mean(x[-4:-1]))


# ------------------------------------------------------- §8f N3 / N4 whole-record calls
def test_whole_record_hrv_and_hjorth_oracle(oracle_lib):
    """The reference's jit functions called on a whole array == one window."""
    d = gc.load("n4_whole")
    for k in d:
        if not k.startswith("val_"):
            continue
        key = k[4:]
        x = d["x3"] if key in ("coeff_var", "hjorth_mobility", "hjorth_complexity") else d["x"]
        got = oracle_lib.window_features(x, len(x), len(x), [gc.MOMENT_FEATURES[key]],
                                         **gc.FEATURE_KWARGS.get(key, {}))[0, 0, 0]
        assert got == d[k], (key, got, float(d[k]))


# ------------------------------------------------------------ §8f N2 preprocessing
def test_filtfilt_oracle_bit_exact_vs_reference():
    """The C restatement of scipy.signal.filtfilt (with the reference's own lfilter_zi)
    reproduces the reference's butterworth / linear_filter / gravity_filter bit for bit."""
    import oracle
    d = gc.load("n2_filters")
    x = d["x"]
    for k in ("hp", "lp", "bp", "lp8"):
        got = oracle.filtfilt(d["b_" + k], d["a_" + k], x[:, 0], zi=d["zi_" + k])
        assert (got == d["out_" + k]).all(), k
    for key, k in (("linear", "hp"), ("linear_bp", "bp"), ("gravity", "lp")):
        got = oracle.filtfilt(d["b_" + k], d["a_" + k], x, zi=d["zi_" + k])
        assert got.shape == x.shape and (got == d[key]).all(), key
    assert (oracle.magnitude(x) == d["magnitude"]).all()


@pytest.mark.parametrize("case", ["minmax_w128", "minmax_w100", "minmax_w64_s32",
                                  "median_w75_s50"])
def test_minmax_oracle_bits(oracle_lib, case):
    """np.min / np.max (stats.dmin / dmax): bit patterns incl. the sign of zero, NaN at
    row 0 only, +-inf for all-NaN rows >= 1 (numba array_min vs min_parallel_impl)."""
    d = gc.load(case)
    W, S = int(d["wsize"]), int(d["wstep"])
    keys = [k for k in ("out_min", "out_max", "out_median") if k in d]
    got = oracle_lib.window_features(d["x"], W, S, [k[4:] for k in keys])[0]
    for j, k in enumerate(keys):
        ref = d[k]
        assert (np.isnan(got[j]) == np.isnan(ref)).all(), k
        fin = ~np.isnan(ref)
        assert (got[j][fin].view(np.int64) == ref[fin].view(np.int64)).all(), k


@pytest.mark.parametrize("case", ["elementwise_float32", "elementwise_float64"])
def test_elementwise_helpers_vs_reference(oracle_lib, case):
    """accelerometer.roll / pitch / magnitude_dot and timedom.gradient / zero_crossings:
    the C restatement (glibc atan2f / atan2 as numba's float ufuncs call them) against the
    reference's outputs; magnitude_dot by tolerance (BLAS dot order)."""
    d = gc.load(case)
    x, y, z = d["x"], d["y"], d["z"]
    assert gc.same(oracle_lib.roll(y, z), d["out_roll"]).all()
    assert gc.same(oracle_lib.pitch(x, y, z), d["out_pitch"]).all()
    assert gc.same(oracle_lib.gradient(x), d["out_gradient"]).all()
    for th in (0.0, 0.05):
        assert (oracle_lib.zero_crossings(x, th) == d["out_zero_crossings_th%g" % th]).all()
    tol = 1e-6 if x.dtype == np.float32 else 1e-14
    np.testing.assert_allclose(oracle_lib.magnitude_dot(x[40:], y[40:], z[40:]),
                               d["out_magnitude_dot"], rtol=tol)
    pk = oracle_lib.find_peaks(d["x_peaks"])
    assert np.array_equal(pk, d["out_find_peaks"]) and np.array_equal(pk, d["out_nb_find_peaks"])


def test_f64_spectral_needs_the_fp64_transform(oracle_lib):
    """f64spec_offset_128: a 1e4 offset with an AC part near float32 resolution. The
    reference's float64 path (fft/_fft.py:18-28, a.astype(complex128)) is reproduced by the
    fp64 oracle; the same record rounded to float32 is not (its band power is off by far more
    than the spectral bar) — so float64 records must not take the float32 path."""
    d = gc.load("f64spec_offset_128")
    kw = dict(fs=float(d["fs"]), band=tuple(d["band"]), dom=tuple(d["dom_range"]))
    W, S = int(d["wsize"]), int(d["wstep"])
    f64 = oracle_lib.window_features(d["x"], W, S, ["band_power"], **kw)[0, 0]
    f32 = oracle_lib.window_features(d["x"].astype(np.float32), W, S, ["band_power"], **kw)[0, 0]
    np.testing.assert_allclose(f64, d["out_band_power"], rtol=1e-12)
    assert np.max(np.abs(f32 / d["out_band_power"] - 1.0)) > 1e-2
