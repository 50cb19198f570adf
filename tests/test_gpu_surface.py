"""GPU parity of the module functions around the window path that reference users call
directly (VERDICT r02 "fill the drop-in surface"), against fixtures made by running the
reference itself (tests/golden/make_golden.py surface_cases):

  stats.minmax                       generic/stats.py:12-32         bit-exact (+-0 too)
  timedom.hjorth_mobility_derivative generic/timedom.py:115-131     bit-exact
  timedom.hjorth_complexity_derivatives  timedom.py:151-170         bit-exact
  timedom.hjorth_parameters          generic/timedom.py:173-193     bit-exact
  qrs.find_peaks(x, comp)            heart/qrs.py:200-212           exact indices
  mhealth.fft.fft / ifft             fft/_fft.py:18-48 (numpy fallback, fft/__init__.py:3-7)
                                     max |err| <= 1e-12 x max |X| (fp64 FFT vs pocketfft)
  rolling_apply(user callable)       util/windows.py:93             within 1e-6 relative:
        user code is evaluated by numpy on the host, the reference compiles it with numba —
        numpy 2's promotion (NEP 50: float32 * Python float stays float32) and pairwise sums
        differ from numba's typing (float64) and sequential sums in the low bits (parity
        unpinned below that)
"""
import warnings

import numpy as np
import pytest

import golden_cases as gc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

FFT_TOL = 1e-12


@pytest.fixture(scope="module")
def mh():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    import pymhealth_amd
    from pymhealth_amd import _lib
    _lib.lib()
    return pymhealth_amd.install_mhealth_alias()


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return bool(((a == b) & (np.signbit(a) == np.signbit(b)) | (np.isnan(a) & np.isnan(b))).all())
    return bool((a == b).all())


def test_minmax_vs_reference(mh):
    from mhealth.generic import stats
    d = gc.load("surface_minmax")
    for k in ("a", "b", "c", "d", "e", "f", "z", "z2"):
        x, ref = d["x_" + k], d["out_" + k]
        got = np.array(stats.minmax(x), dtype=ref.dtype)
        assert _bits_equal(got, ref), (k, got, ref)
        # a torch CUDA tensor gives the same
        got_t = np.array(stats.minmax(torch.from_numpy(np.ascontiguousarray(x)).cuda()), dtype=ref.dtype)
        assert _bits_equal(got_t, ref), (k, "torch")
    with pytest.raises(ValueError):
        stats.minmax(np.zeros(0, np.float32))


def test_minmax_large_multiblock(mh):
    """A record spanning every block of the reduction: the first occurrence of a value
    repeated far apart wins, the answer equals numpy's min / max."""
    from mhealth.generic import stats
    rng = np.random.default_rng(3)
    x = rng.standard_normal(5_000_001).astype(np.float32)
    x[123] = np.nan
    mn, mx = stats.minmax(x)
    assert mn == np.nanmin(x) and mx == np.nanmax(x)
    x[:] = 1.0
    x[4_000_000] = -0.0
    x[17] = 0.0
    mn, mx = stats.minmax(x)
    assert mn == 0.0 and not np.signbit(mn) and mx == 1.0


def test_hjorth_variants_vs_reference(mh):
    from mhealth.generic import timedom
    d = gc.load("surface_hjorth")
    for nm in ("float32", "float64"):
        x, dd = d["x_" + nm], d["dd_" + nm]
        d1 = timedom.gradient(x)
        d2 = timedom.gradient(d1)
        got = np.array(timedom.hjorth_parameters(x), np.float64)
        assert _bits_equal(got, d["params_" + nm]), (nm, got, d["params_" + nm])
        assert _bits_equal(timedom.hjorth_mobility_derivative(x, d1), d["mob_d_" + nm]), nm
        assert _bits_equal(timedom.hjorth_mobility_derivative(x, dd), d["mob_dd_" + nm]), nm
        assert _bits_equal(timedom.hjorth_complexity_derivatives(x, d1, d2), d["cmp_d_" + nm]), nm
        assert _bits_equal(timedom.hjorth_complexity_derivatives(x, dd, np.diff(dd)),
                           d["cmp_dd_" + nm]), nm


def test_find_peaks_comparisons_vs_reference(mh):
    import operator
    from mhealth.heart import qrs
    d = gc.load("surface_find_peaks")
    for nm in ("float32", "float64"):
        x = d["x_" + nm]
        for cname, comp, op in (("greater", np.greater, operator.gt),
                                ("greater_equal", np.greater_equal, operator.ge),
                                ("less", np.less, operator.lt),
                                ("less_equal", np.less_equal, operator.le)):
            ref = d["out_%s_%s" % (cname, nm)]
            got = qrs.find_peaks(x, comp)
            assert got.dtype == np.int64 and np.array_equal(got, ref), (cname, nm)
            assert np.array_equal(qrs.find_peaks(x, op), ref)
    with pytest.raises(TypeError):
        qrs.find_peaks(d["x_float32"], np.equal)
    assert np.array_equal(qrs.find_peaks(d["x_float32"]), d["out_greater_float32"])


def _fft_inputs():
    out = {}
    for n in (1, 2, 3, 7, 64, 100, 256, 1000, 4096, 6000, 8192, 10007):
        r = np.random.default_rng(1000 + n)
        out["c%d" % n] = r.standard_normal(n) + 1j * r.standard_normal(n)
        out["r%d" % n] = r.standard_normal(n).astype(np.float32)
    return out


def _fft_close(got, ref):
    err = np.abs(got - ref).max() if ref.size else 0.0
    return err <= FFT_TOL * max(np.abs(ref).max(), 1e-300)


def test_fft_ifft_vs_reference(mh):
    import mhealth.fft as mfft
    d = gc.load("surface_fft")
    for key, v in _fft_inputs().items():
        got = mfft.fft(v)
        assert got.dtype == np.complex128 and got.shape == v.shape
        assert _fft_close(got, d["fft_" + key]), key
        if "ifft_" + key in d:
            got = mfft.ifft(v)
            assert _fft_close(got, d["ifft_" + key]), ("ifft", key)
            # round trip
            assert _fft_close(mfft.ifft(mfft.fft(v)), v), ("round trip", key)


@pytest.mark.parametrize("n", [128, 1024, 4096, 32768, 1 << 20, 3000, 65537])
def test_fft_batched_rows_vs_numpy(mh, n):
    """Row batches through every path (LDS, global passes, Bluestein), torch in / out."""
    import mhealth.fft as mfft
    rng = np.random.default_rng(n)
    rows = max(1, min(64, (1 << 22) // n))
    a = rng.standard_normal((rows, n)) + 1j * rng.standard_normal((rows, n))
    t = torch.from_numpy(a).cuda()
    got = mfft.fft(t)
    assert isinstance(got, torch.Tensor) and got.is_cuda and got.dtype == torch.complex128
    ref = np.fft.fft(a, axis=-1)
    assert _fft_close(got.cpu().numpy(), ref)
    back = mfft.ifft(got).cpu().numpy()
    assert _fft_close(back, a)


def test_user_callables_through_rolling_apply(mh):
    from mhealth.util.windows import rolling_apply
    from mhealth.generic import stats
    d = gc.load("surface_user_callables")
    x, W, S = d["x"], int(d["wsize"]), int(d["wstep"])

    def first_last(w):
        return w[0] * 2.0 + w[-1]

    def max_minus_mean(w):
        return np.max(w) - np.mean(w)

    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        got = rolling_apply(first_last, W, S)(x)
        got2 = rolling_apply(first_last, W, S)(x)
    assert sum("no MI355X kernel" in str(w.message) for w in rec) == 1
    # numba types w[0] * 2.0 of a float32 window in float64, numpy 2 (NEP 50) in float32:
    # user code evaluated by numpy matches the reference to float32 rounding, not bit for bit
    assert got.dtype == np.float64
    np.testing.assert_allclose(got, d["out_first_last"], rtol=1e-6, atol=1e-7)
    assert np.array_equal(got2, got)
    got = rolling_apply(max_minus_mean, W, S)(x)
    np.testing.assert_allclose(got, d["out_max_minus_mean"], rtol=1e-6, atol=1e-7)
    # mixed with engine features in one list: the engine ones still run on the GPU
    res = rolling_apply([np.mean, first_last, stats.skewness], W, S)(x)
    np.testing.assert_allclose(res[1], d["out_first_last"], rtol=1e-6, atol=1e-7)
    from pymhealth_amd.engine import window_features
    dev = window_features(torch.from_numpy(x).cuda(), W, S, [0, 6]).cpu().numpy()
    assert np.array_equal(res[0], dev[0, 0]) and np.array_equal(res[2], dev[0, 1])


@pytest.mark.parametrize("case", ["nu_user_float32", "nu_user_float64"])
def test_nonuniform_user_callables_with_engine_features(mh, case):
    """nonuniform_rolling_apply([np.mean, user_fn], min_window_len)(index, arr, wsize, wstep)
    with the reference's argument list (windows.py:219-231): np.mean on the GPU (fused
    indexed launch) bit-exact, the jitted user function on the host over the same GPU-found
    windows (windows.py:146-157: np.zeros(n, arr.dtype), NaN below min_window_len)."""
    from mhealth.util.windows import nonuniform_rolling_apply
    d = gc.load(case)
    ml, W, S = int(d["min_window_len"]), int(d["wsize"]), int(d["wstep"])

    def rng_(w):
        return w.max() - w.min()

    def first_last(w):
        return w[0] * 2.0 + w[-1]

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        m, r = nonuniform_rolling_apply([np.mean, rng_], ml)(d["index"], d["x"], W, S)
        single = nonuniform_rolling_apply(rng_, ml)(d["index"], d["x"], W, S)
        fl = nonuniform_rolling_apply(first_last, ml)(d["index"], d["x"], W, S)
        both = nonuniform_rolling_apply({"m": np.mean, "r": rng_}, ml)(d["index"], d["x"], W, S)
    assert m.dtype == r.dtype == d["x"].dtype
    assert gc.same(m, d["list_mean"]).all()
    assert gc.same(r, d["list_range"]).all() and gc.same(single, d["out_range"]).all()
    assert np.isnan(r).any()
    np.testing.assert_allclose(fl, d["out_first_last"], rtol=1e-6, atol=1e-7, equal_nan=True)
    assert gc.same(both["m"], d["list_mean"]).all() and gc.same(both["r"], d["list_range"]).all()


def test_minmax_every_numpy_dtype_keeps_its_type(mh):
    """stats.minmax (stats.py:12-32) on dtypes without a kernel type of their own: bool,
    int8 / int16, uint8 / 16 / 32 / 64 (uint64 beyond 2^63 included) and float16 go through
    an exact wider type and come back as values of the input dtype, like the reference's
    (min, max) of x itself."""
    from mhealth.generic import stats
    rng = np.random.default_rng(11)
    cases = [rng.integers(0, 2, 3001).astype(np.bool_),
             rng.integers(-128, 128, 5000).astype(np.int8),
             rng.integers(-30000, 30000, 5000).astype(np.int16),
             rng.integers(0, 256, 5000).astype(np.uint8),
             rng.integers(0, 65536, 5000).astype(np.uint16),
             rng.integers(0, 2 ** 32, 5000, dtype=np.uint64).astype(np.uint32),
             rng.integers(0, 2 ** 63, 5000, dtype=np.uint64) * np.uint64(2) + np.uint64(1),
             (rng.standard_normal(5000) * 100).astype(np.float16)]
    for x in cases:
        lo, hi = stats.minmax(x)
        assert type(lo) is type(x[0].item()) and type(hi) is type(x[0].item()), x.dtype
        assert lo == x.min().item() and hi == x.max().item(), x.dtype
    lo, hi = stats.minmax(np.array([np.uint64(2 ** 64 - 1), np.uint64(3)]))
    assert (lo, hi) == (3, 2 ** 64 - 1)


def test_fft_cpu_tensor_comes_back_on_the_cpu(mh):
    """mhealth.fft on a CPU torch tensor: transformed on the GPU, returned on the CPU (the
    input's device), equal to numpy's fp64 FFT."""
    import mhealth.fft as mfft
    a = torch.from_numpy(np.random.default_rng(3).standard_normal(1000))
    out = mfft.fft(a)
    assert out.device.type == "cpu" and out.dtype == torch.complex128
    assert _fft_close(out.numpy(), np.fft.fft(a.numpy()))
    back = mfft.ifft(out)
    assert back.device.type == "cpu"
    assert _fft_close(back.numpy(), a.numpy())
