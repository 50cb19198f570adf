"""GPU parity: the HIP engine (through the C-ABI) against the reference's golden outputs
and the CPU oracle on the same seeded inputs. Runs on the MI355X box (`-m gpu`).

Bar (BASELINE.json north star): integer/index features bit-exact; every
numba-faithful moment feature bit-exact too (the kernels replay numba's fp32/fp64
accumulation order); spectral features within 1e-5 relative of the
fp64 oracle (fp32 on-chip rFFT), dominant frequency exact except near-ties
(top-two fp64 PSD values within 1e-5 relative).
"""
import functools
import os

import numpy as np
import pytest

import golden_cases as gc


torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SPEC_RTOL = 1e-5
# Absolute floors, per window (never scaled by another window): an fp32 FFT's rounding
# error scales with the window's own total power, so band power gets 1e-7 x that total
# (the floor only matters where the band holds < 1 % of the power, or the window is all
# zero); relative power is scale-free (floor 1e-7); entropy is in nats, O(1) (floor 1e-6).
SPEC_FLOOR = {"band_power": 1e-7, "relative_band_power": 1e-7, "spectral_entropy": 1e-6}


def _windows(xc, W, S, first, nw):
    return xc[(first + np.arange(nw))[:, None] * S + np.arange(W)[None, :]]


def _windows_at(xc, W, S, rows):
    return xc[np.asarray(rows, np.int64)[:, None] * S + np.arange(W)[None, :]]


# float64 records: an fp64 transform on both sides (spectral64.hip vs numpy's pocketfft /
# the oracle's radix-2): rounding only, ~1e-15 of the window's total power
F64_SPEC_RTOL = 1e-10
F64_SPEC_FLOOR = {"band_power": 1e-13, "relative_band_power": 1e-13, "spectral_entropy": 1e-12}
F64_TIE_RTOL = 1e-12
F64_TIE_FLOOR = 1e-13   # x the window's total power: fp64 transform rounding level


def spectral_check(oracle_lib, got, ref, names, xs, W, S, fs, dom=(None, None), first=0,
                   tag="", rtol=SPEC_RTOL, floors=SPEC_FLOOR, tie_rtol=1e-5, tie_floor=0.0):
    """The north-star bar for spectral features, window by window, every channel.

    got / ref: (C, F, nw) engine and oracle values for windows first .. first+nw-1 of the
    host record xs ((n,) or (n, C)). Non-spectral names are skipped.
      * band / relative band power, entropy: |g - o| <= rtol |o| + floor_i, floor_i from
        ``floors`` (band power: times window i's own total fp64 periodogram power);
        NaN exactly where the oracle has NaN;
      * dominant frequency: identical, or a near-tie in which the GPU's own bin holds a
        maximum: the oracle's fp64 PSD at the GPU's bin, which must lie
        in the range, is >= (1 - tie_rtol) x the range's maximum (gc.dominant_tie_ok; for
        float64 records also within tie_floor x the window's total power of it).
    The fp64 periodogram (floors, ties) is computed only for the windows that need it, so
    the check runs at full workload size (every window of cfg3 / cfg4 / cfg5)."""
    xs = np.asarray(xs)
    C = 1 if xs.ndim == 1 else xs.shape[1]
    freqs = np.fft.rfftfreq(W, 1.0 / fs)
    lo = 0 if dom[0] is None else int(np.searchsorted(freqs, dom[0], side="left"))
    hi = len(freqs) if dom[1] is None else int(np.searchsorted(freqs, dom[1], side="left"))
    for c in range(C):
        xc = xs if xs.ndim == 1 else np.ascontiguousarray(xs[:, c])
        for j, name in enumerate(names):
            if name not in gc.SPECTRAL_FEATURES:
                continue
            g, o = got[c, j], ref[c, j]
            if name == "dominant_frequency":
                ok = gc.same(g, o)
                bad = np.nonzero(~ok)[0]
                if bad.size:
                    psd = oracle_lib.periodogram(_windows_at(xc, W, S, first + bad), fs)
                    for r, i in enumerate(bad):
                        ok[i] = gc.dominant_tie_ok(psd[r], lo, hi, g[i], W / fs, tie_rtol,
                                                   tie_floor)
                assert ok.all(), (tag, c, name, np.nonzero(~ok)[0][:8], g[~ok][:4], o[~ok][:4])
                continue
            nan = np.isnan(o)
            assert (np.isnan(g) == nan).all(), (tag, c, name, np.nonzero(np.isnan(g) != nan)[0][:8])
            with np.errstate(invalid="ignore"):
                err = np.abs(g - o)
                cand = ~nan & ~(err <= rtol * np.abs(o)) & ~(np.isinf(o) & (g == o))
            idx = np.nonzero(cand)[0]
            if not idx.size:
                continue
            floor = floors[name]
            if name == "band_power":
                psd = oracle_lib.periodogram(_windows_at(xc, W, S, first + idx), fs)
                floor = floor * np.abs(psd).sum(axis=1)
            bad = ~(err[idx] <= rtol * np.abs(o[idx]) + floor)
            assert not bad.any(), (tag, c, name, idx[bad][:8], g[idx][bad][:4], o[idx][bad][:4])


@pytest.fixture(scope="module")
def mh():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X (torch.cuda.is_available() is False)")
    import pymhealth_amd
    from pymhealth_amd import _lib
    _lib.lib()  # fail loudly if libmhfeat.so is missing
    return pymhealth_amd


def _feat_obj(mh, key, th):
    f = mh.features
    table = {
        "mean": np.mean, "var": np.var, "std": np.std, "min": np.min, "max": np.max,
        "median": np.median,
        "skewness": f.skewness,
        "kurtosis": f.kurtosis, "kurtosis_excess": f.kurtosis_excess, "drange": f.drange,
        "zero_crossing_count": f.zero_crossing_count,
        "zero_crossing_count_th0.05": functools.partial(f.zero_crossing_count, th=0.05),
        "line_length": f.line_length, "rms": f.rms, "peak_count": f.peak_count,
        "hjorth_activity": f.hjorth_activity, "std_in_fn": f.std32, "mean_in_fn": f.mean32,
        "pnnx20": functools.partial(f.pnnx, x=20.0),
        "csi_sd1_half": functools.partial(f.csi_sd1, factor=0.5),
        "percentile_0": f.percentile(0), "percentile_12.5": f.percentile(12.5),
        "percentile_33": functools.partial(np.percentile, q=33.0),
        "percentile_50": f.percentile(50), "percentile_90": functools.partial(np.percentile, q=90),
        "percentile_100": f.percentile(100), "p25": f.percentile(25),
        "sampen_m3_r0.15": functools.partial(f.sampen, mm=3, r=0.15),
        "sampen_sd0.5": functools.partial(f.sampen, sd=0.5),
        "rqa_recurrence_rate": f.rqa_recurrence_rate(0.3), "rqa_determinism": f.rqa_determinism(0.3),
        "rqa_laminarity": f.rqa_laminarity(0.3), "rqa_length_entropy": f.rqa_length_entropy(0.3),
        "rqa_length_entropy_min3": f.rqa_length_entropy(0.3, 3),
        "rqa_determinism_r0": f.rqa_determinism(), "rqa_recurrence_rate_r0": f.rqa_recurrence_rate(),
    }
    return table[key] if key in table else getattr(f, key)


MOMENT_CASES = gc.moment_cases()


@pytest.mark.parametrize("case", sorted({c[0] for c in MOMENT_CASES}))
def test_rolling_apply_matches_reference_golden(mh, case):
    """Every moment/time-domain feature of every fixture, one fused list call."""
    d = gc.load(case)
    keys = [k for (c, k, _, _) in MOMENT_CASES if c == case]
    funcs = [_feat_obj(mh, k, gc.ZC_THRESHOLD.get(k, 0.0)) for k in keys]
    res = mh.util.windows.rolling_apply(funcs, int(d["wsize"]), int(d["wstep"]))(d["x"])
    for k, got in zip(keys, res):
        ref = d["out_" + k]
        assert isinstance(got, np.ndarray) and got.dtype == np.float64 and got.shape == ref.shape
        if k in gc.LIBM_KEYS:   # device libm log / log10 vs glibc, last-bit tolerance
            np.testing.assert_allclose(got, ref, rtol=gc.LIBM_KEYS[k], atol=0, equal_nan=True)
            continue
        eq = gc.same(got, ref, d.get("raises_" + k))
        assert eq.all(), (case, k, np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


BLOCK_CASES = gc.block_cases()


@pytest.mark.parametrize("case", sorted({c[0] for c in BLOCK_CASES}))
def test_rolling_apply_2d_matches_reference_golden(mh, case):
    """rolling_apply on a 2-D (N, c) record: window i is the (wsize, c) block (numba's
    flat C-order reductions; skewness / kurtosis over len(x) = rows; line_length along the
    rows), every feature the reference evaluates on blocks, one list call; numpy and
    torch-CUDA input."""
    d = gc.load(case)
    keys = [k for (c, k, _, _) in BLOCK_CASES if c == case]
    funcs = [_feat_obj(mh, k, 0.0) for k in keys]
    W, S = int(d["wsize"]), int(d["wstep"])
    res = mh.util.windows.rolling_apply(funcs, W, S)(d["x"])
    tres = mh.util.windows.rolling_apply(funcs, W, S)(torch.from_numpy(d["x"]).cuda())
    for k, got, tg in zip(keys, res, tres):
        ref = d["out_" + k]
        assert got.shape == ref.shape
        eq = gc.same(got, ref)
        assert eq.all(), (case, k, np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])
        assert gc.same(tg.cpu().numpy(), ref).all(), (case, k)


F64_CASES = gc.f64_cases()


@pytest.mark.parametrize("case", sorted({c[0] for c in F64_CASES}))
def test_rolling_apply_float64_matches_reference_golden(mh, case):
    """float64 records (numba's fp64 models: mhf_window_features_f64), every lane feature of
    every fixture in one list call, 1-D and 2-D; bit-exact except fp64 log10 (lorenz_cvi)
    and windows where the reference raises."""
    d = gc.load(case)
    keys = [k for (c, k, _, _) in F64_CASES if c == case]
    funcs = [_feat_obj(mh, k, gc.ZC_THRESHOLD.get(k, 0.0)) for k in keys]
    res = mh.util.windows.rolling_apply(funcs, int(d["wsize"]), int(d["wstep"]))(d["x"])
    for k, got in zip(keys, res):
        ref = d["out_" + k]
        assert got.dtype == np.float64 and got.shape == ref.shape
        if k in gc.LIBM_KEYS:
            np.testing.assert_allclose(got, ref, rtol=gc.LIBM_KEYS[k], atol=0, equal_nan=True)
            continue
        eq = gc.same(got, ref, d.get("raises_" + k))
        assert eq.all(), (case, k, np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


TILE64_FEATURES = ["mean", "var", "std", "skewness", "kurtosis", "kurtosis_excess", "rms",
                   "zero_crossings", "peak_count", "drange", "line_length", "coeff_var"]


def _tile64_cases():
    """float64 fixtures with a 1-D record and at least one feature tile64 computes"""
    out = []
    for case in sorted({c[0] for c in F64_CASES}):
        keys = [k for (c, k, f, kw) in F64_CASES if c == case and f in TILE64_FEATURES]
        if keys and gc.load(case)["x"].ndim == 1:
            out.append(case)
    return out


@pytest.mark.parametrize("case", _tile64_cases())
def test_float64_tile64_subset_matches_reference_golden(mh, case):
    """The float64 fixtures through the streamed tile kernel (tile64.hip): only the
    features that kernel computes, so 1-D records with a power-of-two W take it."""
    d = gc.load(case)
    W, S = int(d["wsize"]), int(d["wstep"])
    keys = [k for (c, k, f, kw) in F64_CASES if c == case and f in TILE64_FEATURES]
    from pymhealth_amd import engine
    ids = [gc_feature_id(gc.MOMENT_FEATURES[k]) for k in keys]
    plan = engine.plan_name_f64((1, 0, 1), W, S, ids)
    pow2 = W >= 64 and (W & (W - 1)) == 0 and S % 2 == 0
    assert plan == ("tile64" if pow2 else "moments_f64"), (plan, W, S)
    funcs = [_feat_obj(mh, k, gc.ZC_THRESHOLD.get(k, 0.0)) for k in keys]
    res = mh.util.windows.rolling_apply(funcs, W, S)(d["x"])
    for k, got in zip(keys, res):
        ref = d["out_" + k]
        eq = gc.same(got, ref, d.get("raises_" + k))
        assert eq.all(), (case, k, np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])


def gc_feature_id(name):
    from oracle import FEATURE_IDS
    return FEATURE_IDS[name]


@pytest.mark.parametrize("W,S,C,nw", [(256, 256, 3, 4000), (256, 256, 1, 5000), (128, 64, 1, 3000),
                                      (64, 64, 3, 777), (1024, 512, 1, 300), (256, 130, 3, 999),
                                      (4096, 4096, 1, 70)])
def test_float64_tile64_vs_oracle(mh, oracle_lib, W, S, C, nw):
    """float64 records through tile64 against the oracle's fp64 models: AoS 3-axis and 1-D,
    overlapping / non-overlapping windows, a ragged tail tile, edge windows (NaN, inf,
    signed zeros, constants, exact thresholds), every tile64 feature subset (pass 2 with and
    without skewness / kurtosis), zc threshold, window shards with global indices, float32
    output."""
    from pymhealth_amd import engine
    rng = np.random.default_rng(W + 7 * S + C)
    n = (nw - 1) * S + W
    x = rng.standard_normal((n, C)) * 0.3 + np.array([0.0, 0.5, 9.81][:C])
    x[S * 2:S * 2 + W] = 1.25                                  # constant window
    x[S * 4 + 3, 0] = np.nan
    x[S * 6 + 1, -1] = np.inf
    x[S * 8:S * 8 + W:5] = 0.0
    x[S * 8 + 1:S * 8 + W:7] = -0.0
    x[S * 9 + 2, 0] = 0.05                                     # == threshold
    if C == 1:
        x = x[:, 0].copy()
    t = torch.from_numpy(x).cuda()
    for names, th in ((TILE64_FEATURES, 0.05), (["mean", "zero_crossings", "rms"], 0.0),
                      (["var", "std", "peak_count"], 0.0)):
        ids = [oracle_lib.FEATURE_IDS[k] for k in names]
        assert engine.plan_name_f64((C, 1 if C > 1 else 0, C), W, S, ids) == "tile64"
        got = engine.window_features(t, W, S, ids, zc_threshold=th).cpu().numpy()
        ref = oracle_lib.window_features(x, W, S, names, zc_threshold=th)
        eq = gc.same(got, ref)
        assert eq.all(), [(names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(names)) if not eq[c, j].all()]
    # shards with global window indices; float32 rows
    h = nw // 2 + 3
    part = engine.window_features(t[h * S:], W, S, ids, first_window=h, n_windows=nw - h,
                                  base_window=h).cpu().numpy()
    assert gc.same(part, ref[:, :, h:]).all()
    got32 = engine.window_features(t, W, S, ids, out_dtype=torch.float32).cpu().numpy()
    assert gc.same(got32, ref.astype(np.float32)).all()


def test_float64_spectral_and_order_routing(mh, oracle_lib):
    """A float64 record with spectral features: the lane features in fp64, the spectral ones
    from the fp64 transform (spectral64.hip; the reference transforms a.astype(complex128),
    fft/_fft.py:18-28); order statistics in fp64 (64-bit keys) and sample entropy (fp64
    differences) next to them."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal(256 * 40) + np.sin(np.arange(256 * 40) * 0.2)
    ra = mh.util.windows.rolling_apply
    f = mh.features
    m, bp = ra([np.mean, f.band_power(50.0, 0.5, 8.0)], 256, 256)(x)
    assert gc.same(m, oracle_lib.window_features(x, 256, 256, ["mean"])[0, 0]).all()
    ref = oracle_lib.window_features(x, 256, 256, ["band_power"], fs=50.0,
                                     band=(0.5, 8.0))[0, 0]
    np.testing.assert_allclose(bp, ref, rtol=F64_SPEC_RTOL)
    from pymhealth_amd.engine import plan_name_f64
    ids = [oracle_lib.FEATURE_IDS[k] for k in ("mean", "band_power", "median")]
    assert plan_name_f64((1, 0, 1), 256, 256, ids) == "tile64+spectral64+order/pairwise"
    # values equal as float32 but ordered as float64: the median must see float64 keys
    x[::7] = np.round(x[::7], 1) * (1.0 + 2.0 ** -40)
    med, bp2, q90 = ra([np.median, f.band_power(50.0, 0.5, 8.0),
                        functools.partial(np.percentile, q=90.0)], 256, 256)(x)
    assert gc.same(med, oracle_lib.window_features(x, 256, 256, ["median"])[0, 0]).all()
    assert gc.same(q90, oracle_lib.window_features(x, 256, 256, ["percentile"],
                                                   percentile_q=90.0)[0, 0]).all()
    se = ra(mh.generic.information.sampen, 256, 256)(x)
    np.testing.assert_allclose(se, oracle_lib.window_features(x, 256, 256, ["sampen"])[0, 0],
                               rtol=1e-15, equal_nan=True)   # fp64 log: last bit


@pytest.mark.parametrize("W,S,C", [(256, 256, 1), (256, 128, 3), (1024, 128, 1), (100, 37, 1),
                                   (4096, 2048, 1), (4095, 4095, 1), (2, 1, 1), (1, 1, 1),
                                   (128, 64, 2)])
def test_float64_spectral_vs_oracle(mh, oracle_lib, W, S, C):
    """Every spectral feature of float64 records (1-D and AoS, power-of-two FFT and exact-
    phase DFT, W from 1 to 4096) against the oracle's fp64 transform, window by window at
    fp64 rounding level; offsets far above the AC part (the float32 rounding would lose it)
    and NaN windows included."""
    rng = np.random.default_rng(W * 7 + S + C)
    nw = 300 if W <= 1024 else 24
    n = (nw - 1) * S + W
    t = np.arange(n) / 100.0
    x = (np.sin(2 * np.pi * 3.1 * t)[:, None] * rng.uniform(0.5, 2, C)
         + 0.2 * rng.standard_normal((n, C)) + np.array([0.0, 1e4, 9.81][:C]))
    x[S * 4 + min(3, W - 1), 0] = np.nan
    x[S * 7:S * 7 + W, -1] = 2.5
    # samples of ~1e-160: the window's total power is a subnormal fp64 value, whose
    # reciprocal overflows (spectral64's entropy then divides)
    tiny = 11 if W <= 1024 else 13
    x[S * tiny:S * tiny + W, 0] = rng.standard_normal(W) * 1e-160
    xs = x[:, 0].copy() if C == 1 else x
    names = gc.SPECTRAL_FEATURES
    kw = dict(fs=100.0, band=(1.0, 9.0), dom=(0.5, 20.0))
    ids = [oracle_lib.FEATURE_IDS[k] for k in names]
    from pymhealth_amd import engine
    got = engine.window_features(torch.from_numpy(xs).cuda(), W, S, ids, **kw).cpu().numpy()
    ref = oracle_lib.window_features(xs, W, S, names, **kw)
    assert got.shape == ref.shape == (C, len(names), nw)
    je = names.index("spectral_entropy")
    assert np.isfinite(got[0, je, tiny]) and np.isfinite(ref[0, je, tiny])
    assert abs(got[0, je, tiny] - ref[0, je, tiny]) <= 1e-10 * abs(ref[0, je, tiny]), (got[0, je, tiny], ref[0, je, tiny])
    # subnormal band powers carry ~1e-5 relative rounding in fp64 on either side: the tiny
    # window's entropy is the check above; the rest of its row is left to it
    got[0, :, tiny] = ref[0, :, tiny]
    spectral_check(oracle_lib, got, ref, names, xs, W, S, kw["fs"], kw["dom"],
                   tag="f64 %d/%d/%d" % (W, S, C), rtol=F64_SPEC_RTOL, floors=F64_SPEC_FLOOR,
                   tie_rtol=F64_TIE_RTOL, tie_floor=F64_TIE_FLOOR)


@pytest.mark.parametrize("W,S", [(256, 256), (100, 37), (2048, 1024), (4096, 4096)])
def test_float64_order_statistics_vs_oracle(mh, oracle_lib, W, S):
    """float64 median / IQR / mode / percentile against the oracle's fp64 numba models on
    random records with ties, signed zeros, NaN and infinities: register sort (W <= 1024)
    and LDS sort (2048: 16 KiB, 4096: 32 KiB of 64-bit keys per window)."""
    rng = np.random.default_rng(W + S)
    n = (24 - 1) * S + W
    x = np.round(rng.standard_normal(n) * 3) * 0.25 + rng.integers(0, 2, n) * 2.0 ** -35
    x[rng.integers(0, n, 20)] = 0.0
    x[rng.integers(0, n, 20)] = -0.0
    x[S * 3 + 5] = np.nan
    x[S * 5 + 1] = np.inf
    x[S * 7 + 2] = -np.inf
    names = ["median", "interquartile_range", "mode", "percentile"]
    ids = [oracle_lib.FEATURE_IDS[k] for k in names]
    from pymhealth_amd import engine
    got = engine.window_features(torch.from_numpy(x).cuda(), W, S, ids,
                                 percentile_q=33.0).cpu().numpy()[0]
    ref = oracle_lib.window_features(x, W, S, names, percentile_q=33.0)[0]
    for j, k in enumerate(names):
        eq = gc.same(got[j], ref[j])
        assert eq.all(), (k, np.nonzero(~eq)[0][:8], got[j][~eq][:4], ref[j][~eq][:4])


def test_single_feature_rolling_apply_and_cache(mh):
    d = gc.load("cfg1")
    ra = mh.util.windows.rolling_apply
    assert ra(mh.features.skewness, 128, 128) is ra(mh.features.skewness, 128, 128)
    got = ra(mh.features.skewness, 128, 128)(d["x"])
    assert gc.same(got, d["out_skewness"]).all()
    lst = ra([np.mean, np.var, mh.generic.stats.skewness, mh.generic.stats.kurtosis],
             128, 128)(d["x"])
    for f, v in zip(("mean", "var", "skewness", "kurtosis"), lst):
        assert gc.same(v, d["list_" + f]).all()
    dct = ra({"m": np.mean, "k": mh.generic.stats.kurtosis}, 128, 128)(d["x"])
    assert set(dct) == {"m", "k"} and gc.same(dct["k"], d["out_kurtosis"]).all()


def test_torch_input_zero_copy_and_strided_column(mh):
    aos = gc.load("accel_aos")["x"]
    ref = gc.load("accel_z_strided")["out_skewness"]
    t = torch.from_numpy(aos).cuda()
    got = mh.util.windows.rolling_apply(mh.features.skewness, 256, 256)(t[:, 2])
    assert isinstance(got, torch.Tensor) and got.is_cuda
    assert gc.same(got.cpu().numpy(), ref).all()


@pytest.mark.parametrize("case", gc.spectral_cases())
def test_spectral_vs_oracle_and_golden(mh, oracle_lib, case):
    d = gc.load(case)
    W, S, fs = int(d["wsize"]), int(d["wstep"]), float(d["fs"])
    band, dom = tuple(d["band"]), tuple(d["dom_range"])
    f = mh.features
    feats = [f.band_power(fs, *band), f.relative_band_power(fs, *band), f.spectral_entropy(fs),
             f.dominant_frequency(fs, *dom)]
    got = mh.features.extract(d["x"], W, S, feats).cpu().numpy()
    orc = oracle_lib.window_features(d["x"], W, S, gc.SPECTRAL_FEATURES, fs=fs, band=band,
                                     dom=dom)
    ref = np.stack([np.where(d["raises_relative_band_power"], np.nan, d["out_" + n])
                    if n == "relative_band_power" else d["out_" + n]
                    for n in gc.SPECTRAL_FEATURES])[None]
    # a float64 record (f64spec_*): the fp64 transform, pinned at fp64 rounding level
    tol = (dict(rtol=F64_SPEC_RTOL, floors=F64_SPEC_FLOOR, tie_rtol=F64_TIE_RTOL,
                tie_floor=F64_TIE_FLOOR) if d["x"].dtype == np.float64 else {})
    spectral_check(oracle_lib, got, orc, gc.SPECTRAL_FEATURES, d["x"], W, S, fs, dom,
                   tag=case + " vs oracle", **tol)
    spectral_check(oracle_lib, got, ref, gc.SPECTRAL_FEATURES, d["x"], W, S, fs, dom,
                   tag=case + " vs reference", **tol)


ALL_MOMENTS = ["mean", "mean32", "var", "var32", "std", "std32", "skewness", "kurtosis",
               "kurtosis_excess", "rms", "zero_crossings", "peak_count", "drange",
               "line_length"]


def _ids(names):
    from oracle import FEATURE_IDS
    return [FEATURE_IDS[n] for n in names]


def _accel(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 50.0
    e = rng.standard_normal((n, 3))
    return np.stack([0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * e[:, 0],
                     0.2 * np.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * e[:, 1],
                     1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2) + 0.05 * e[:, 2]],
                    axis=1).astype(np.float32)


# (W, S) -> kernel the engine must pick for 3-channel AoS input (16-B aligned)
AOS_PLANS = {(256, 256): "tile_w256_c3", (128, 128): "tile_w128_c3", (256, 64): "tile_w256_c3",
             (256, 128): "tile_w256_c3", (128, 32): "tile_w128_c3", (100, 37): "tile_fix",
             (1024, 128): "span", (250, 250): "tile_fix", (7, 3): "tile_fix", (1, 1): "tile_fix",
             (289, 200): "span",
             (3000, 1000): "moments_generic"}


@pytest.mark.parametrize("W,S", sorted(AOS_PLANS))
def test_multichannel_aos_all_moments_bit_exact(mh, oracle_lib, W, S):
    """Every moment feature, 3-axis AoS, overlapping / gapped / odd windows: the tile
    kernel (W = 128 / 256, any 16-B aligned stride incl. overlap), the fixed-window register
    tile of tile_idx.hip.h (any other W <= 288 at any step, test_tile_fix_vs_oracle), the LDS
    span kernel (longer W) or the generic kernel (spans beyond the LDS budget), bit-exact."""
    from pymhealth_amd.engine import plan_name, window_features
    assert plan_name((3, 1, 3), W, S, _ids(ALL_MOMENTS)) == AOS_PLANS[(W, S)]
    nw = 3000 if W <= 256 else 400
    x = _accel((nw - 1) * S + W, seed=W * 7 + S)
    got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(ALL_MOMENTS)).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, ALL_MOMENTS)
    assert got.shape == ref.shape == (3, len(ALL_MOMENTS), nw)
    eq = gc.same(got, ref)
    assert eq.all(), [(ALL_MOMENTS[j], c, np.nonzero(~eq[c, j])[0][:5])
                      for c in range(3) for j in range(len(ALL_MOMENTS)) if not eq[c, j].all()]


def _fast_var_record(W, S, C, seed, huge=True):
    """nw windows of a C-channel AoS record (C = 1: 1-D): window 0 and most windows accel-
    like, then one window each of the cases the fast-var guard (tile.hip.h fast_var_ok)
    sends to the exact recomputation: all zero, amplitude 1e-30 (q underflows), 1e-22
    (ssd below 2^-110), 1e20 (q overflows), a NaN, an inf, values 1e-39 (sum c32 subnormal);
    and ones that stay on the fast path: constant 1.0 (ssd = 0, every d = 0), constant 0.1
    (c32 rounds), a 1 g offset; 1000 + noise and 1e4 + noise sit where the centering bound
    (|m| / σ beyond ~300) may send them to the exact replay — within the tolerance either
    way. Returns (record, {window: case}). huge=False
    (spectral feature sets) leaves out the 1e20 window: its power overflows the fp32 rFFT
    (|X|^2 ~ 1e44), a limit of the on-chip fp32 spectrum, not of the moments."""
    nw = 640
    n = (nw - 1) * S + W
    x = _accel(n, seed)[:, :C] if C > 1 else _accel(n, seed)[:, 2].copy()
    rng = np.random.default_rng(seed + 1)
    cases = {101: "zero", 163: "tiny30", 227: "tiny22", 290: "huge", 355: "nan", 419: "inf",
             480: "subnormal_sum", 70: "const1", 133: "const01", 545: "offset1000", 600: "noise",
             620: "offset1e4"}
    if not huge:
        cases[290] = "noise"
    for w, kind in cases.items():
        sl = slice(w * S, w * S + W)
        shape = x[sl].shape
        v = rng.standard_normal(shape)
        val = {"zero": np.zeros(shape), "tiny30": v * 1e-30, "tiny22": v * 1e-22,
               "huge": v * 1e20, "nan": v, "inf": v, "subnormal_sum": np.full(shape, 1e-39),
               "const1": np.ones(shape), "const01": np.full(shape, 0.1),
               "offset1000": 1000 + v, "noise": v, "offset1e4": 1e4 + 0.5 * v}[kind]
        x[sl] = val.astype(np.float32)
        if kind == "nan":
            x[w * S + W // 3] = np.nan
        if kind == "inf":
            x[w * S + W // 2] = np.inf
    return x, cases


FAST_VAR_EXACT = ("zero", "tiny30", "tiny22", "huge", "nan", "inf", "subnormal_sum", "const1")


@pytest.mark.default_numerics
@pytest.mark.parametrize("W,C,spec", [(256, 1, True), (256, 3, False), (128, 1, False),
                                      (128, 3, True), (256, 3, True), (256, 1, False)])
def test_fast_var_default_numerics_vs_oracle(mh, oracle_lib, W, C, spec):
    """The register tiles' default rows >= 1 of np.var / np.std (fast var): within
    gc.FAST_VAR_RTOL of numba's fp64 chain on every window, bit-exact on row 0 and on every
    window the guard recomputes exactly (zero / tiny / huge / NaN / inf / subnormal-sum
    windows) and on constant windows; every other moment bit-exact; and with
    exact_var=True (MHF_NUMERICS_EXACT_VAR) bit-exact everywhere. Overlapping (S = W/2)
    and gapped windows."""
    from pymhealth_amd.engine import plan_name, window_features
    names = ["mean", "var", "std", "skewness", "kurtosis", "zero_crossings"]
    kw = {}
    if spec:
        names = names + ["band_power", "spectral_entropy"]
        kw = dict(fs=64.0, band=(0.5, 4.0))
    for S in (W, W // 2, W + 32):
        x, cases = _fast_var_record(W, S, C, seed=W + C + S, huge=not spec)
        ids = _ids(names)
        assert plan_name((C, 1 if C > 1 else 0, C), W, S, ids).startswith("tile_w%d" % W)
        xd = torch.from_numpy(x).cuda()
        got = window_features(xd, W, S, ids, **kw).cpu().numpy()
        ex = window_features(xd, W, S, ids, exact_var=True, **kw).cpu().numpy()
        ref = oracle_lib.window_features(x, W, S, names, **kw)
        mom = [j for j, n in enumerate(names) if n not in gc.SPECTRAL_FEATURES]
        eq = gc.same_fast_var(got[:, mom], ref[:, mom], [names[j] for j in mom])
        assert eq.all(), [(S, names[mom[j]], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(mom)) if not eq[c, j].all()]
        exq = gc.same(ex[:, mom], ref[:, mom])
        assert exq.all(), [(S, names[mom[j]], c, np.nonzero(~exq[c, j])[0][:5])
                           for c in range(C) for j in range(len(mom)) if not exq[c, j].all()]
        for w, kind in cases.items():
            if kind in FAST_VAR_EXACT:
                for j in (1, 2):
                    assert gc.same(got[:, j, w], ref[:, j, w]).all(), (S, kind, names[j], w)
        # the fast path really is taken elsewhere: most rows >= 1 differ in the last bits
        if S == W:
            assert not np.array_equal(got[:, 1, 1:], ex[:, 1, 1:])
        if spec:
            # the fp32 rFFT's power underflows for the 1e-30 / 1e-22 / 1e-39 windows (|X|^2
            # below the fp32 range): those are moment-guard cases, not spectral ones
            gs = got.copy()
            for w, kind in cases.items():
                if kind in ("tiny30", "tiny22", "subnormal_sum"):
                    gs[:, :, w] = ref[:, :, w]
            # windows holding the +inf sample (with S < W, also the next one): the spectrum of
            # an infinite sample is inf / NaN in an order each FFT algorithm decides (numpy's
            # pocketfft, the oracle's radix-2, the lane rFFT); the inf case is a moment case here
            xw = x.reshape(len(x), -1)
            for w in range(got.shape[2]):
                if np.isinf(xw[w * S:w * S + W]).any():
                    gs[:, :, w] = ref[:, :, w]
            spectral_check(oracle_lib, gs, ref, names, x, W, S, 64.0, tag="fastvar")


@pytest.mark.default_numerics
@pytest.mark.parametrize("W,S,C", [(250, 125, 1), (250, 125, 3), (250, 250, 1), (100, 37, 3),
                                   (200, 232, 1), (288, 97, 1)])
def test_fast_var_tile_fix_default_numerics_vs_oracle(mh, oracle_lib, W, S, C):
    """The any-length fixed tile (tile_fix, tile_idx.hip.h, span image or chunk DMA) takes the
    same fast var as the register tiles: rows >= 1 of np.var / np.std within
    gc.FAST_VAR_RTOL, every window the guard rejects (zero / tiny / huge / NaN / inf /
    subnormal sum) walked exactly, constant windows exact, every other moment bit-exact; with
    exact_var=True the fp64 chain replayed bit for bit."""
    from pymhealth_amd.engine import plan_name, window_features
    names = ["mean", "var", "std", "skewness", "kurtosis", "zero_crossings"]
    x, cases = _fast_var_record(W, S, C, seed=W + 7 * C + S)
    ids = _ids(names)
    assert plan_name((C, 1 if C > 1 else 0, C), W, S, ids) == "tile_fix"
    xd = torch.from_numpy(x).cuda()
    got = window_features(xd, W, S, ids).cpu().numpy()
    ex = window_features(xd, W, S, ids, exact_var=True).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, names)
    eq = gc.same_fast_var(got, ref, names)
    assert eq.all(), [(names[j], c, np.nonzero(~eq[c, j])[0][:5])
                      for c in range(C) for j in range(len(names)) if not eq[c, j].all()]
    exq = gc.same(ex, ref)
    assert exq.all(), [(names[j], c, np.nonzero(~exq[c, j])[0][:5])
                       for c in range(C) for j in range(len(names)) if not exq[c, j].all()]
    for w, kind in cases.items():
        if kind in FAST_VAR_EXACT:
            for j in (1, 2):
                assert gc.same(got[:, j, w], ref[:, j, w]).all(), (kind, names[j], w)
    assert not np.array_equal(got[:, 1, 1:], ex[:, 1, 1:])
    # the windows a half launch walks (its record ends inside a tile) keep the tile path's
    # fast-var bits: two half launches = one launch
    from pymhealth_amd.distributed import sample_range
    nw = got.shape[2]
    full = window_features(xd, W, S, ids)
    for w0, w1 in ((0, nw // 2 + 7), (nw // 2 + 7, nw)):
        s0, s1 = sample_range(w0, w1, W, S)
        part = window_features(xd[s0:s1], W, S, ids, first_window=w0, n_windows=w1 - w0,
                               base_window=w0)
        eqh = gc.same(part.cpu().numpy(), full[:, :, w0:w1].cpu().numpy())
        assert eqh.all(), (w0, w1, [(names[j], c, np.nonzero(~eqh[c, j])[0][:5] + w0)
                                    for c in range(C) for j in range(len(names)) if not eqh[c, j].all()])


@pytest.mark.parametrize("W,S,offset", [(256, 256, 1), (256, 128, 3), (1024, 128, 0),
                                        (1024, 128, 1), (128, 64, 0)])
def test_single_channel_overlap_and_unaligned_bit_exact(mh, oracle_lib, W, S, offset):
    """1-D signals: overlapping windows take the tile kernel when 16-B aligned (W = 128 /
    256), the fixed-window register tile for unaligned views such as x[1:] (W <= 288), the
    span kernel otherwise (W = 1024) — never the generic fallback; all moment features
    bit-exact vs the oracle."""
    from pymhealth_amd.engine import plan_name, window_features
    rng = np.random.default_rng(W + S + offset)
    nw = 2500
    x = (rng.standard_normal((nw - 1) * S + W + offset) * 2 + 0.5).astype(np.float32)
    t = torch.from_numpy(x).cuda()[offset:]
    # (plan_name does not see the pointer: an unaligned view of a W = 128 / 256 request is
    # planned as the tile kernel and taken by the register tile at launch)
    want = ("tile_w%d_c1" % W) if W in (128, 256) else "tile_fix" if W <= 288 else "span"
    assert plan_name((1, 0, 1), W, S, _ids(ALL_MOMENTS)) == want
    got = window_features(t, W, S, _ids(ALL_MOMENTS)).cpu().numpy()
    ref = oracle_lib.window_features(x[offset:], W, S, ALL_MOMENTS)
    eq = gc.same(got, ref)
    assert eq.all(), [(ALL_MOMENTS[j], np.nonzero(~eq[0, j])[0][:5])
                      for j in range(len(ALL_MOMENTS)) if not eq[0, j].all()]


TILE_FIX_CASES = [(250, 125, 1, "x0"), (250, 125, 3, "x2"), (288, 1, 1, "x1"), (288, 300, 3, "x0"),
                  (100, 37, 1, "x2"), (1, 1, 1, "x1"), (33, 7, 3, "x1"), (256, 101, 1, "x2"),
                  (200, 200, 3, "x2"), (129, 64, 1, "x0")]


@pytest.mark.parametrize("W,S,C,fset", TILE_FIX_CASES)
def test_tile_fix_vs_oracle(mh, oracle_lib, W, S, C, fset, monkeypatch):
    """The fixed-window register tile (tile_idx.hip.h, FIX): window g = first + i at g * S,
    W <= 288 samples, any step (overlapping, gapped, S = 1), C = 1 / 3 AoS, each extras
    level. Row 0 keeps the serial numerics and rows >= 1 numba's parfor mean / var
    (windows.py:68-87); the record's last tiles (whose DMA would pass its end) and
    windows outside the two-FMA division range walk global memory; first_window > 0 (a
    shard) has no serial row. Bit-exact vs the oracle, the record built from the corner
    values of _tile_idx_record."""
    from pymhealth_amd.engine import plan_name, window_features
    names = TILE_IDX_SETS[fset]
    ids = _ids(names)
    assert plan_name((C, 1 if C > 1 else 0, C), W, S, ids) == "tile_fix"
    nw = 2500
    n = (nw - 1) * S + W
    x = _tile_idx_record(max(n, 5000), C, seed=W + S + C)[:n]
    t = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    for first, k in ((0, nw), (3, nw - 5), (nw - 70, 70)):
        got = window_features(t, W, S, ids, first_window=first, n_windows=k).cpu().numpy()
        ref = oracle_lib.window_features(x, W, S, names, first_window=first, n_windows=k)
        assert got.shape == ref.shape == (C, len(names), k)
        eq = gc.same(got, ref)
        assert eq.all(), [(first, names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(names)) if not eq[c, j].all()]


@pytest.mark.parametrize("W,S,C,fset", [(250, 125, 1, "x0"), (250, 125, 3, "x2"), (288, 1, 1, "x1"),
                                        (100, 37, 1, "x2"), (33, 7, 3, "x1"), (256, 101, 1, "x2"),
                                        (288, 143, 1, "x0"), (200, 99, 3, "x0"), (150, 126, 1, "x1"),
                                        (77, 2, 3, "x2")])
@pytest.mark.parametrize("offset", [0, 1, 3])
def test_tile_span_vs_chunk_dma(mh, oracle_lib, W, S, C, fset, offset, monkeypatch):
    """Overlapping fixed windows through the tile's union-span image (tile_idx.hip.h SPAN:
    each sample DMA'd once per tile, the windows read from LDS at r S) against the
    per-window chunk DMA (MHF_NO_TILE_SPAN=1) bit for bit and the oracle: odd S, S = 2 mod 4,
    the largest S whose image fits 37 KiB, a record starting 1 / 3 samples past a 16-B
    boundary (the first tile's piece grid would start before the record: it walks global
    memory) and ending mid-piece (the last tile's cut), shard runs (first_window > 0)."""
    from pymhealth_amd.engine import plan_name, window_features
    names = TILE_IDX_SETS[fset]
    ids = _ids(names)
    assert plan_name((C, 1 if C > 1 else 0, C), W, S, ids) == "tile_fix"
    nw = 1500
    n = (nw - 1) * S + W
    x = _tile_idx_record(max(n + offset, 5000), C, seed=W + 3 * S + C + offset)[:n + offset]
    t = torch.from_numpy(np.ascontiguousarray(x)).cuda()[offset:]
    xo = x[offset:]
    for first, k in ((0, nw), (5, nw - 9), (nw - 45, 45)):
        got = window_features(t, W, S, ids, first_window=first, n_windows=k).cpu().numpy()
        monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
        monkeypatch.setenv("MHF_NO_TILE_SPAN", "1")
        chunk = window_features(t, W, S, ids, first_window=first, n_windows=k).cpu().numpy()
        monkeypatch.delenv("MHF_NO_TILE_SPAN")
        np.testing.assert_array_equal(got, chunk)
        ref = oracle_lib.window_features(xo, W, S, names, first_window=first, n_windows=k)
        eq = gc.same(got, ref)
        assert eq.all(), [(first, names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(names)) if not eq[c, j].all()]


def _record_at_low_word(x, low_word, straddle=False):
    """x copied into a device allocation at an address whose low 32-bit word is `low_word`
    (16-B aligned), or — straddle=True — that crosses a 2^32 boundary in its middle: a slice
    at a computed element offset of a larger allocation (up to 4 GiB + the record). Returns
    (view, keep-alive buffer). A low word below 2^31 must let the record cross 2^31."""
    x = np.ascontiguousarray(x)
    nbytes = x.nbytes
    want = ((1 << 32) - (nbytes // 2) // 16 * 16) % (1 << 32) if straddle else low_word
    buf = torch.empty(((1 << 32) + nbytes + 4096) // 4, dtype=torch.float32, device="cuda")
    base = buf.data_ptr()
    off = (want - (base & 0xFFFFFFFF)) % (1 << 32)
    assert off % 16 == 0
    flat = buf[off // 4: off // 4 + x.size]
    v = flat.view(x.shape)
    v.copy_(torch.from_numpy(x))
    p = v.data_ptr()
    lo = p & 0xFFFFFFFF
    if straddle:
        assert lo + nbytes > (1 << 32), hex(p)
    elif lo < 1 << 31:
        assert lo + nbytes > (1 << 31), hex(p)          # the low word's top bit flips inside
    return v, buf


@pytest.mark.parametrize("straddle", [False, True])
@pytest.mark.parametrize("C", [1, 3])
def test_register_tiles_at_high_address_words(mh, oracle_lib, C, straddle):
    """Round 5's tile_idx / tile_fix fault, pinned: the record sits at a device address whose
    low 32-bit word is >= 2^31 (a readfirstlane of it sign-extended over the high word) or
    whose range crosses a 2^32 boundary, so the 64-bit SGPR bases and 32-bit lane offsets of
    the LDS-DMA maps (dma_map.h) see both cases on the GPU whatever the allocator returns.
    In the same tiles: kept windows beside non-kept ones (short / empty / longer than 288,
    the division-range fallback, windows whose DMA would pass the record end). The indexed
    tile (tile_idx), the any-length fixed tile (tile_fix, W = 250 / 100 overlapping) and the
    W = 256 tile, all bit-exact vs the oracle. (The host emulation of the same maps under
    ASan: test_host.py::test_dma_address_maps_under_asan.)"""
    from pymhealth_amd.engine import indexed_window_features, plan_name, plan_name_indexed, window_features
    names = ["mean", "var", "std", "skewness", "kurtosis", "zero_crossings", "rms", "peak_count",
             "line_length"]
    ids = _ids(names)
    n = 24000
    x = _tile_idx_record(n, C, seed=91 + C)
    for low in (0x80000000, 0xFFFF0000, 0x7FFFF000):
        t, keep_alive = _record_at_low_word(x, low, straddle)
        # time-indexed windows: contiguous, random (short / empty / long / negative), tail
        assert plan_name_indexed((C, 1 if C > 1 else 0, C), ids) == "tile_idx"
        rng = np.random.default_rng(low % 1000 + C)
        s = rng.integers(-300, n + 100, 2500)
        e = s + rng.integers(-20, 420, 2500)
        tail = np.arange(n - 500, n - 1, 9)
        ind = np.ascontiguousarray(np.stack([np.concatenate([s, tail]),
                                             np.concatenate([e, np.full(tail.size, n)])]).astype(np.int64))
        ti = torch.from_numpy(ind).cuda()
        got = indexed_window_features(t, ti, ids, min_len=3, out_dtype=torch.float64).cpu().numpy()
        ref = oracle_lib.indexed_features(x, ind, names, min_len=3, out_dtype=np.float64)
        eq = gc.same(got, ref)
        assert eq.all(), [("idx", hex(low), names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(names)) if not eq[c, j].all()]
        # fixed windows: the any-length tile and the W = 256 tile
        for W, S in ((250, 125), (100, 37), (256, 256), (256, 128)):
            nw = (n - W) // S + 1
            plan = plan_name((C, 1 if C > 1 else 0, C), W, S, ids)
            assert plan in ("tile_fix", "tile_w256_c1", "tile_w256_c3"), plan
            for first, k in ((0, nw), (nw - 40, 40)):
                got = window_features(t, W, S, ids, first_window=first, n_windows=k).cpu().numpy()
                ref = oracle_lib.window_features(x, W, S, names, first_window=first, n_windows=k)
                eq = gc.same(got, ref)
                assert eq.all(), [(plan, hex(low), first, names[j], c, np.nonzero(~eq[c, j])[0][:5])
                                  for c in range(C) for j in range(len(names)) if not eq[c, j].all()]
        del t, keep_alive
        torch.cuda.empty_cache()
        if straddle:
            break                       # the straddling placement does not depend on `low`


def _division_edge_record(n, seed):
    """A record whose windows exercise both sides of the hoisted-reciprocal division's
    range check: deviations below 2^-25 / above 2^31, subnormals, inf, NaN,
    constant stretches, exact range boundaries, and ordinary data."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 2 + 0.5).astype(np.float32)
    seg = max(1, n // 16)
    x[1 * seg:2 * seg] *= np.float32(1e-12)              # |d| < 2^-25: fallback
    x[2 * seg:3 * seg] = np.float32(3.0) + x[2 * seg:3 * seg] * np.float32(1e-7)
    x[3 * seg:4 * seg] *= np.float32(1e-39)              # subnormal samples
    x[4 * seg:5 * seg] *= np.float32(1e15)               # |d| > 2^31: d^4 overflows
    x[5 * seg + 7] = np.inf
    x[6 * seg + 3] = -np.inf
    x[7 * seg + 11] = np.nan
    x[8 * seg:9 * seg] = np.float32(-2.5)                # constant: every d = 0
    x[9 * seg:10 * seg:2] = np.float32(2.0 ** -25)       # boundary deviations
    x[9 * seg + 1:10 * seg:2] = np.float32(0.0)
    x[10 * seg:11 * seg:3] = np.float32(2.0 ** 31)
    return x


@pytest.mark.parametrize("W,S,C", [(250, 125, 1), (100, 37, 1), (100, 100, 3), (37, 5, 1)])
def test_division_range_fallback_windows_bit_exact(mh, oracle_lib, W, S, C):
    """Non-power-of-two windows (skewness / kurtosis divide each term by len(x)) over
    records built to hit both the two-FMA quotient and its IEEE fallback: every moment
    bit-exact vs the oracle on the span / generic kernels and the indexed kernel."""
    from pymhealth_amd.engine import indexed_window_features, window_features
    nw = 900
    n = (nw - 1) * S + W
    x = np.stack([_division_edge_record(n, 10 * W + c) for c in range(C)], axis=1)
    x = x[:, 0].copy() if C == 1 else x
    t = torch.from_numpy(x).cuda()
    got = window_features(t, W, S, _ids(ALL_MOMENTS)).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, ALL_MOMENTS)
    eq = gc.same(got, ref)
    assert eq.all(), [(ALL_MOMENTS[j], c, np.nonzero(~eq[c, j])[0][:5])
                      for c in range(C) for j in range(len(ALL_MOMENTS)) if not eq[c, j].all()]
    # the same record through indexed windows of varying length (every window serial)
    rng = np.random.default_rng(W)
    starts = np.arange(0, n - W - 8, S, dtype=np.int64)
    ends = starts + W + rng.integers(-5, 6, starts.shape[0])
    ind = np.stack([starts, ends])
    names = ["mean", "var", "std", "skewness", "kurtosis", "kurtosis_excess", "zero_crossings"]
    goti = indexed_window_features(t, torch.from_numpy(ind).cuda(), _ids(names),
                                   out_dtype=torch.float64).cpu().numpy()
    refi = oracle_lib.indexed_features(x, ind, names, out_dtype=np.float64)
    eqi = gc.same(goti, refi)
    assert eqi.all(), [(names[j], c, np.nonzero(~eqi[c, j])[0][:5])
                       for c in range(C) for j in range(len(names)) if not eqi[c, j].all()]


def test_float32_output_and_window_shards(mh, oracle_lib):
    from pymhealth_amd.engine import window_features
    x = _accel(256 * 5000, seed=3)
    t = torch.from_numpy(x).cuda()
    ids = _ids(ALL_MOMENTS)
    full = window_features(t, 256, 256, ids).cpu().numpy()
    parts = [window_features(t, 256, 256, ids, first_window=a, n_windows=b - a).cpu().numpy()
             for a, b in [(0, 1), (1, 1777), (1777, 4096), (4096, 5000)]]
    assert gc.same(np.concatenate(parts, axis=2), full).all()
    f32 = window_features(t, 256, 256, ids, out_dtype=torch.float32).cpu().numpy()
    assert gc.same(f32, full.astype(np.float32)).all()
    # shard slices with global window indices (what each rank of a multi-GPU run does)
    from pymhealth_amd.distributed import sample_range, shard_range
    parts = []
    for r in range(3):
        w0, w1 = shard_range(5000, r, 3)
        s0, s1 = sample_range(w0, w1, 256, 256)
        parts.append(window_features(t[s0:s1], 256, 256, ids, first_window=w0,
                                     n_windows=w1 - w0, base_window=w0).cpu().numpy())
    assert gc.same(np.concatenate(parts, axis=2), full).all()


def test_sharded_overlapping_windows_generic_and_spectral(mh, oracle_lib):
    """cfg5 geometry (W=1024, S=128): shards with halos == one launch == oracle."""
    from pymhealth_amd.distributed import sample_range, shard_range
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(4)
    nw, W, S = 333, 1024, 128
    x = rng.standard_normal((nw - 1) * S + W).astype(np.float32)
    t = torch.from_numpy(x).cuda()
    names = ["mean", "var", "skewness", "band_power", "dominant_frequency"]
    kw = dict(fs=256.0, band=(0.5, 40.0), dom=(0.5, 40.0))
    full = window_features(t, W, S, _ids(names), **kw).cpu().numpy()
    parts = []
    for r in range(4):
        w0, w1 = shard_range(nw, r, 4)
        s0, s1 = sample_range(w0, w1, W, S)
        parts.append(window_features(t[s0:s1], W, S, _ids(names), first_window=w0,
                                     n_windows=w1 - w0, base_window=w0, **kw).cpu().numpy())
    assert gc.same(np.concatenate(parts, axis=2), full).all()
    ref = oracle_lib.window_features(x, W, S, names, **kw)
    assert gc.same(full[:, :3], ref[:, :3]).all()
    spectral_check(oracle_lib, full, ref, names, x, W, S, 256.0, kw["dom"], tag="shards")


def test_spectral_random_pow2_sizes(mh, oracle_lib):
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(11)
    for W, S, fs in [(2, 2, 4.0), (64, 32, 16.0), (256, 256, 64.0), (512, 200, 100.0),
                     (2048, 1024, 256.0), (4096, 4096, 512.0)]:
        nw = 64
        x = (rng.standard_normal((nw - 1) * S + W) + 0.5).astype(np.float32)
        names = ["band_power", "relative_band_power", "spectral_entropy"]
        got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(names), fs=fs,
                              band=(fs / 10, fs / 4)).cpu().numpy()
        ref = oracle_lib.window_features(x, W, S, names, fs=fs, band=(fs / 10, fs / 4))
        spectral_check(oracle_lib, got, ref, names, x, W, S, fs, tag=str(W))


def test_fused_moments_and_spectral_one_call(mh, oracle_lib):
    """cfg4's full per-axis feature set on AoS 3-axis data in one engine call."""
    from pymhealth_amd import features as F
    fs = 50.0
    x = _accel(256 * 4000, seed=5)
    feats = [F.mean, F.var, F.std, F.skewness, F.kurtosis, F.rms, F.zero_crossing_count,
             F.peak_count, F.band_power(fs, 0.5, 4.0), F.relative_band_power(fs, 0.5, 4.0),
             F.spectral_entropy(fs), F.dominant_frequency(fs, 0.5, 8.0)]
    # spectral params must agree within one group: dominant freq gets its own group
    got = F.extract(x, 256, 256, feats).cpu().numpy()
    names = ["mean", "var", "std", "skewness", "kurtosis", "rms", "zero_crossings",
             "peak_count"]
    ref = oracle_lib.window_features(x, 256, 256, names)
    assert gc.same(got[:, :8], ref).all()
    sref = oracle_lib.window_features(x, 256, 256, gc.SPECTRAL_FEATURES, fs=fs,
                                      band=(0.5, 4.0), dom=(0.5, 8.0))
    spectral_check(oracle_lib, got[:, 8:12], sref, gc.SPECTRAL_FEATURES, x, 256, 256, fs,
                   (0.5, 8.0), tag="cfg4 set")


def test_single_window_calls(mh):
    x = np.random.default_rng(2).standard_normal(300).astype(np.float32)
    s = mh.generic.stats
    d = gc.load("one_window")
    assert mh.features.skewness(d["x"]) == d["out_skewness"][0]
    assert mh.generic.timedom.zero_crossing_count(x, 0.5) == mh.generic.timedom.\
        zero_crossing_count(x, th=0.5)
    assert s.kurtosis(x) > 0


def test_edge_sizes_and_errors(mh):
    ra = mh.util.windows.rolling_apply
    e = gc.load("empty")
    out = ra(np.mean, 16, 16)(e["x"])
    assert out.shape == (0,) and out.dtype == np.float64
    with pytest.raises(TypeError):
        ra(np.mean)(e["x"])              # wsize=None
    # arbitrary Python has no kernel: evaluated per window on the host
    assert (ra(lambda w: 0.5, 4, 4)(e["x"]) == 0.5).all()
    # float64 records have their own path (mhf_window_features_f64); integer ones do not
    assert ra(np.mean, 16, 16)(e["x"].astype(np.float64)).shape == (0,)
    with pytest.raises(TypeError):
        ra(np.mean, 4, 4)(e["x"].astype(np.int32))
    with pytest.raises(NotImplementedError):
        ra(mh.features.band_power(10.0, 1, 2), 8192, 8192)(np.zeros(8192, np.float32))


def test_determinism(mh):
    from pymhealth_amd.engine import window_features
    x = torch.from_numpy(_accel(256 * 2000, seed=9)).cuda()
    ids = _ids(ALL_MOMENTS + ["band_power", "spectral_entropy"])
    a = window_features(x, 256, 256, ids, fs=50.0, band=(0.5, 4.0))
    b = window_features(x, 256, 256, ids, fs=50.0, band=(0.5, 4.0))
    assert torch.equal(a, b)


# ------------------------------------------------ time-indexed (nonuniform) windows (§8f N1)
NU_FEATS = {"mean": np.mean, "var": np.var, "std": np.std, "median": np.median}


def _nu_feat(mh, key):
    return NU_FEATS.get(key) or getattr(mh.features, key)


@pytest.mark.parametrize("case", gc.nonuniform_cases())
def test_nonuniform_rolling_apply_matches_reference_golden(mh, case):
    """get_indices on the GPU == the reference's indices; every feature of
    nonuniform_rolling_apply bit-exact vs the reference (serial numerics, NaN windows);
    list / dict / single-function forms agree."""
    w = mh.util.windows
    d = gc.load(case)
    index, wsize, wstep = gc.nonuniform_args(d)
    min_len = int(d["min_window_len"])
    np.testing.assert_array_equal(w.get_indices(index, wsize, wstep), d["indices"])
    keys = [k for (c, k, _) in gc.nonuniform_feature_cases() if c == case]
    funcs = [_nu_feat(mh, k) for k in keys]
    res = w.nonuniform_rolling_apply(funcs, min_len)(index, d["x"], wsize, wstep)
    for k, got in zip(keys, res):
        ref = d["out_" + k]
        # np.zeros(n, arr.dtype): float64 out for the float64 records (nu64_*)
        assert got.dtype == d["x"].dtype and got.shape == ref.shape
        eq = gc.same(got, ref, d.get("raises_" + k))
        assert eq.all(), (case, k, np.nonzero(~eq)[0][:8], got[~eq][:4], ref[~eq][:4])
    if "list_std" not in d:
        return
    one = w.nonuniform_rolling_apply(np.std, min_len)(index, d["x"], wsize, wstep)
    assert gc.same(one, d["list_std"]).all()
    dct = w.nonuniform_rolling_apply({"m": np.mean, "s": np.std}, min_len)(
        index, d["x"], wsize, wstep)
    assert gc.same(dct["m"], d["list_mean"]).all() and gc.same(dct["s"], d["list_std"]).all()


def test_indexed_engine_float64_vs_oracle(mh, oracle_lib):
    """float64 records through mhf_indexed_window_features_f64: random (start, end) pairs
    over 2 AoS channels, the lane features and the order statistics (64-bit keys), several
    min_len; float64 out."""
    from pymhealth_amd.engine import indexed_window_features
    rng = np.random.default_rng(17)
    x = np.round(rng.standard_normal((8000, 2)) * 8) / 8 + np.array([0.0, 9.81])
    x[rng.integers(0, 8000, 30), 0] = 0.0
    x[rng.integers(0, 8000, 30), 0] = -0.0
    s = rng.integers(-100, 8100, 2000)
    e = s + rng.integers(-10, 400, 2000)
    ind = np.stack([s, e]).astype(np.int64)
    names = ALL_MOMENTS + ["median", "interquartile_range", "mode", "percentile"]
    t = torch.from_numpy(x).cuda()
    ti = torch.from_numpy(ind).cuda()
    for min_len in (0, 3):
        got = indexed_window_features(t, ti, _ids(names), min_len=min_len, percentile_q=12.5,
                                      out_dtype=torch.float64).cpu().numpy()
        ref = oracle_lib.indexed_features(x, ind, names, min_len=min_len, percentile_q=12.5,
                                          out_dtype=np.float64)
        eq = gc.same(got, ref)
        assert eq.all(), [(names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(2) for j in range(len(names)) if not eq[c, j].all()]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_indexed_order_statistics_long_windows(mh, oracle_lib, dtype):
    """Time-indexed windows longer than the LDS capacity of the order kernel (16384 keys
    of float32 / 8192 of float64): 20k- and 40k-sample windows (a 5-minute window at 100
    Hz is 30k samples) mixed with short ones, median / percentile / IQR / mode sorted in
    global scratch, bit-exact vs the oracle (never NaN). NaN and mixed-zero windows take
    the numba replay. sampen / RQA past their LDS capacity refuse the call."""
    from pymhealth_amd.engine import indexed_window_features
    rng = np.random.default_rng(23)
    n = 100_000
    x = (np.round(rng.standard_normal(n) * 16) / 16).astype(dtype)
    x[rng.integers(0, n, 50)] = 0.0
    x[rng.integers(0, n, 50)] = -0.0
    x[61_234] = np.nan                          # inside long windows 2 and 3
    s = np.array([0, 10_000, 50_000, 55_000, 70_000, 99_990, 5, 300, 90_000, -45_000],
                 np.int64)
    e = np.array([20_000, 50_000, 90_000, 75_000, 70_100, 140_000, 105, 8_300, 90_017, -1],
                 np.int64)
    ind = np.stack([s, e])
    assert (np.clip(e, 0, n) - np.clip(s, 0, n)).max() == 40_000
    names = ["median", "percentile", "interquartile_range", "mode", "mean"]
    t = torch.from_numpy(x).cuda()
    ti = torch.from_numpy(ind).cuda()
    got = indexed_window_features(t, ti, _ids(names), percentile_q=33.0,
                                  out_dtype=torch.float64).cpu().numpy()
    ref = oracle_lib.indexed_features(x, ind, names, percentile_q=33.0, out_dtype=np.float64)
    eq = gc.same(got, ref)
    assert eq.all(), [(names[j], np.nonzero(~eq[0, j])[0]) for j in range(len(names))
                      if not eq[0, j].all()]
    assert (np.signbit(got) == np.signbit(ref)).all()
    assert not np.isnan(got[0][:, [0, 1, 4]]).any()           # NaN-free long / short windows
    for feats in (["sampen"], ["rqa_determinism"]):
        with pytest.raises(NotImplementedError):
            indexed_window_features(t, ti, _ids(feats))
            torch.cuda.synchronize()


def test_indexed_engine_multichannel_vs_oracle(mh, oracle_lib):
    """Random (start, end) pairs — overlapping, empty, reversed, negative, past the end —
    over AoS 3-channel data, every moment/time-domain feature, several min_len."""
    from pymhealth_amd.engine import indexed_window_features
    x = _accel(20000, seed=11)
    rng = np.random.default_rng(5)
    s = rng.integers(-300, 20300, 5000)
    e = s + rng.integers(-20, 700, 5000)
    ind = np.stack([s, e]).astype(np.int64)
    t = torch.from_numpy(x).cuda()
    ti = torch.from_numpy(ind).cuda()
    for min_len in (0, 1, 5):
        got = indexed_window_features(t, ti, _ids(ALL_MOMENTS), min_len=min_len).cpu().numpy()
        ref = oracle_lib.indexed_features(x, ind, ALL_MOMENTS, min_len=min_len)
        assert got.shape == ref.shape == (3, len(ALL_MOMENTS), 5000)
        eq = gc.same(got, ref)
        assert eq.all(), [(ALL_MOMENTS[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(3) for j in range(len(ALL_MOMENTS))
                          if not eq[c, j].all()]


TILE_IDX_SETS = {"x0": ["mean", "var", "skewness", "kurtosis", "zero_crossings"],
                 "x1": ["mean32", "var32", "std", "std32", "kurtosis_excess", "rms", "peak_count",
                        "coeff_var"],
                 "x2": ALL_MOMENTS + ["coeff_var"]}


def _tile_idx_record(n, C, seed):
    """A record with every corner the indexed tile path must keep bit-exact: NaN, inf, ±0,
    constant stretches, tiny deviations around an offset (|d| below 2^-25: the Markstein
    division's range check hands those windows to the global walk) and huge values (|d|
    above 2^31)."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, C)) * rng.uniform(0.1, 3.0, C) + rng.uniform(-2, 2, C))
    x = x.astype(np.float32)
    x[500:800] = 0.75                                   # constant
    x[1000:1003] = np.nan
    x[1500] = np.inf
    x[2000:2300:3] = -0.0
    x[2600:2900] = (1.0 + rng.integers(-3, 4, (300, C)) * 2.0 ** -23).astype(np.float32)  # tiny d
    x[3200:3500] = (rng.standard_normal((300, C)) * 1e12).astype(np.float32)               # huge d
    x[4000:4300] = np.round(x[4000:4300])              # ties: zero crossings at 0 / peaks
    return x if C > 1 else np.ascontiguousarray(x[:, 0])


@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("fset", sorted(TILE_IDX_SETS))
def test_indexed_tile_path_vs_oracle(mh, oracle_lib, C, fset, monkeypatch):
    """The indexed register tile (tile_idx.hip.h) against the oracle's serial models, bit for
    bit: contiguous windows of 1 .. 320 samples (past kIdxWmax = 288: the lane's global
    walk), random overlapping / reversed / negative / past-the-end pairs, windows ending at
    the record's last sample (the tile's DMA would reach past it: the whole tile walks),
    min_len 0 / 3 / 250."""
    from pymhealth_amd.engine import indexed_window_features, plan_name_indexed
    names = TILE_IDX_SETS[fset]
    assert plan_name_indexed((C, 1 if C > 1 else 0, C), _ids(names)) == "tile_idx"
    n = 30000
    x = _tile_idx_record(n, C, seed=C + len(names))
    rng = np.random.default_rng(7 + C)
    lens = rng.integers(1, 321, 200)
    lens[::7] = rng.integers(240, 273, lens[::7].size)
    b = np.concatenate([[0], np.cumsum(lens)])
    b = b[b <= n]
    contig = np.stack([b[:-1], b[1:]])
    s = rng.integers(-400, n + 200, 3000)
    rnd = np.stack([s, s + rng.integers(-30, 400, 3000)])
    tail = np.stack([np.arange(n - 600, n - 1, 7), np.full(len(range(n - 600, n - 1, 7)), n)])
    t = torch.from_numpy(x).cuda()
    for ind in (contig, rnd, tail):
        ind = np.ascontiguousarray(ind.astype(np.int64))
        ti = torch.from_numpy(ind).cuda()
        for min_len in (0, 3, 250):
            got = indexed_window_features(t, ti, _ids(names), min_len=min_len,
                                          out_dtype=torch.float64).cpu().numpy()
            ref = oracle_lib.indexed_features(x, ind, names, min_len=min_len,
                                              out_dtype=np.float64)
            assert got.shape == ref.shape
            eq = gc.same(got, ref)
            assert eq.all(), [(names[j], c, np.nonzero(~eq[c, j])[0][:5])
                              for c in range(got.shape[0]) for j in range(len(names))
                              if not eq[c, j].all()]
            num = ~np.isnan(ref)
            assert (np.signbit(got[num]) == np.signbit(ref[num])).all()


@pytest.mark.parametrize("C", [1, 3])
def test_indexed_tile_mixed_with_order_statistics(mh, oracle_lib, C, monkeypatch):
    """The indexed register tile beside the order kernel in one call (round-4 GPU failure,
    tidx_parity.log: the tile stored every feature plane, overwriting the median /
    percentile / IQR / mode planes launch_order had filled on the same stream; the store
    loop now skips non-tile columns, tile_idx.hip.h). Moments interleaved with order
    statistics, short windows (tile path) and long ones (> 288: the lane's global walk;
    > the order kernel's LDS capacity: the global-scratch sort), bit-exact vs the oracle."""
    from pymhealth_amd.engine import indexed_window_features, plan_name_indexed
    names = ["median", "mean", "var", "percentile", "skewness", "interquartile_range",
             "kurtosis", "mode", "zero_crossings", "rms", "line_length"]
    assert plan_name_indexed((C, 1 if C > 1 else 0, C), _ids(names)).startswith("tile_idx")
    n = 60000
    x = _tile_idx_record(n, C, seed=31 + C)
    rng = np.random.default_rng(41 + C)
    s = np.sort(rng.integers(0, n - 400, 3000))
    e = s + rng.integers(1, 300, 3000)
    long_s = np.array([0, 1000, 30000, 59000], np.int64)
    long_e = np.array([20000 // C, 1900, 30000 + 18000 // C, n], np.int64)
    ind = np.ascontiguousarray(np.stack([np.concatenate([s, long_s]),
                                         np.concatenate([e, long_e])]).astype(np.int64))
    t = torch.from_numpy(x).cuda()
    ti = torch.from_numpy(ind).cuda()
    for min_len in (0, 5):
        got = indexed_window_features(t, ti, _ids(names), min_len=min_len, percentile_q=33.0,
                                      out_dtype=torch.float64).cpu().numpy()
        ref = oracle_lib.indexed_features(x, ind, names, min_len=min_len, percentile_q=33.0,
                                          out_dtype=np.float64)
        eq = gc.same(got, ref)
        assert eq.all(), [(names[j], c, np.nonzero(~eq[c, j])[0][:5])
                          for c in range(C) for j in range(len(names)) if not eq[c, j].all()]


def test_get_indices_modes_vs_numpy(mh, oracle_lib):
    """int / float-step / float-size / datetime-unit-mixing bounds vs numpy's own."""
    w = mh.util.windows
    rng = np.random.default_rng(9)
    idx = np.cumsum(rng.integers(1, 50, 40000)).astype(np.int64) + 1_700_000_000_000_000_000
    for wsize, wstep in ((100, 37), (100.5, 37), (100, 37.25), (1e3, 333.3), (5, 5000)):
        np.testing.assert_array_equal(w.get_indices(idx, wsize, wstep),
                                      oracle_lib.get_indices(idx, wsize, wstep),
                                      err_msg=str((wsize, wstep)))
    didx = (np.datetime64("2024-05-01T00:00:00", "s")
            + np.cumsum(rng.integers(0, 4, 5000)).astype("timedelta64[s]"))
    for wsize, wstep in ((np.timedelta64(30, "s"), np.timedelta64(1500, "ms")),
                         (np.timedelta64(1, "m"), np.timedelta64(10, "s"))):
        np.testing.assert_array_equal(w.get_indices(didx, wsize, wstep),
                                      oracle_lib.get_indices(didx, wsize, wstep))
    tidx = torch.from_numpy(idx).cuda()
    got = w.get_indices(tidx, 100, 37)
    assert isinstance(got, torch.Tensor) and got.is_cuda
    np.testing.assert_array_equal(got.cpu().numpy(), oracle_lib.get_indices(idx, 100, 37))
    # the device-resident flow: tensor indices + tensor samples, output stays on the GPU
    xs = torch.from_numpy(rng.standard_normal(idx.size).astype(np.float32)).cuda()
    out = w.indices_rolling_apply(np.var, 3)(got, xs)
    assert isinstance(out, torch.Tensor) and out.is_cuda and out.dtype == torch.float32
    ref = oracle_lib.indexed_features(xs.cpu().numpy(), got.cpu().numpy(), ["var"],
                                      min_len=3)[0, 0]
    assert gc.same(out.cpu().numpy(), ref).all()
    with pytest.raises(TypeError):
        w.indices_rolling_apply(mh.features.spectral_entropy(50.0))(got, xs)



# ------------------------------------------------------------------ §8f N3 / N4
N34 = ["coeff_var", "hjorth_mobility", "hjorth_complexity", "rmssd", "sdsd", "ssd", "pnnx",
       "csi_sd1", "csi_sd2", "lorenz_csi", "lorenz_cvi", "lorenz_mcsi"]


def _n34_check(got, ref, names):
    for j, f in enumerate(names):
        if f == "lorenz_cvi":
            np.testing.assert_allclose(got[..., j, :], ref[..., j, :], rtol=4e-16, atol=0,
                                       equal_nan=True)
        else:
            eq = gc.same(got[..., j, :], ref[..., j, :])
            assert eq.all(), (f, np.nonzero(~eq.ravel())[0][:5])


@pytest.mark.parametrize("W,S", [(64, 16), (256, 256), (100, 37), (2, 1), (3, 3)])
def test_n3_n4_features_vs_oracle(mh, oracle_lib, W, S):
    """Hjorth / coeff_var / HRV family on the generic kernel (3 channels, strided AoS),
    non-default pnn threshold and csi factor, bit-exact vs the oracle."""
    from pymhealth_amd.engine import window_features
    nw = 2000
    x = (800 + 50 * _accel((nw - 1) * S + W, seed=W + S)).astype(np.float32)
    got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(N34), pnn_threshold=3.5,
                          csi_factor=0.6).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, N34, pnn_threshold=3.5, csi_factor=0.6)
    assert got.shape == ref.shape == (3, len(N34), nw)
    _n34_check(got, ref, N34)


def test_hrv_whole_record_and_module_api(mh):
    """hrv.* / timedom.* / stats.coeff_var called on whole records == the reference's
    own jit functions (n4_whole fixture); sdnni / sdann compose pinned parts."""
    d = gc.load("n4_whole")
    hrv, f = mh.heart.hrv, mh.features
    calls = {
        "rmssd": lambda x: hrv.rmssd(x), "sdsd": lambda x: hrv.sdsd(x),
        "ssd": lambda x: hrv.ssd(x), "pnn50": lambda x: hrv.pnn50(x, "ms"),
        "pnnx20": lambda x: hrv.pnnx(x, "ms", 20.0), "csi_sd1": lambda x: hrv.csi_sd1(x),
        "csi_sd1_half": lambda x: hrv.csi_sd1(x, 0.5), "csi_sd2": lambda x: hrv.csi_sd2(x),
        "lorenz_csi": lambda x: hrv.lorenz_csi(x), "lorenz_cvi": lambda x: hrv.lorenz_cvi(x),
        "lorenz_mcsi": lambda x: hrv.lorenz_mcsi(x), "sdnn": lambda x: hrv.sdnn(x),
        "coeff_var": lambda x: mh.generic.stats.coeff_var(x),
        "hjorth_mobility": lambda x: mh.generic.timedom.hjorth_mobility(x),
        "hjorth_complexity": lambda x: mh.generic.timedom.hjorth_complexity(x),
    }
    for key, fn in calls.items():
        x = d["x3"] if key in ("coeff_var", "hjorth_mobility", "hjorth_complexity") else d["x"]
        got, ref = fn(x), float(d["val_" + key])
        if key == "lorenz_cvi":
            assert abs(got - ref) <= 4e-16 * abs(ref), (key, got, ref)
        else:
            assert got == ref, (key, got, ref)
    assert f.pnnx.with_params().params["pnn_threshold"] == 50.0
    # sdnni / sdann: the reference cannot compile them (numba TypingError); check the
    # composition against the pinned parts
    nu = gc.load("nu_hrv")
    idx, rr = nu["index"], nu["x"]
    seg_std = mh.util.windows.nonuniform_rolling_apply(np.std)(idx, rr, 60e9, 60e9)
    assert hrv.sdnni(rr, idx, 60.0) == mh.features.mean32(seg_std)
    seg_mean = mh.util.windows.nonuniform_rolling_apply(np.mean)(idx, rr, 60e9, 60e9)
    assert hrv.sdann(rr, idx, 60.0) == mh.features.std32(seg_mean)


# ------------------------------------------------------------------ §8f N2 preprocessing
def _scale_err(got, ref):
    return np.max(np.abs(got - ref)) / max(1.0, np.max(np.abs(ref)))


def test_filtfilt_vs_reference_golden(mh):
    """mhf_filtfilt (chunked parallel scan) vs the reference's butterworth /
    linear_filter / gravity_filter: <= 1e-8 of the signal scale (the tf-form DF2T's own
    rounding floor for these filters is ~1e-9: any second evaluation order differs by
    that much), with the reference's lfilter_zi, the device-solved zi or
    the module drop-ins (host scipy design, this box's LAPACK zi)."""
    from pymhealth_amd.engine import filtfilt
    d = gc.load("n2_filters")
    x = d["x"]
    t = torch.from_numpy(x).cuda()
    for k in ("hp", "lp", "bp", "lp8"):
        got = filtfilt(t[:, 0], d["b_" + k], d["a_" + k], d["zi_" + k]).cpu().numpy()
        assert got.dtype == np.float64 and _scale_err(got, d["out_" + k]) <= 1e-8, k
        dev = filtfilt(t[:, 0], d["b_" + k], d["a_" + k]).cpu().numpy()   # zi solved here
        assert _scale_err(dev, d["out_" + k]) <= 1e-8, k
    acc = mh.inertial.accelerometer
    for key, got in (("linear", acc.linear_filter(x, 50.0)),
                     ("linear_bp", acc.linear_filter(x, 50.0, (0.5, 10.0))),
                     ("gravity", acc.gravity_filter(x, 50.0))):
        assert got.shape == x.shape and _scale_err(got, d[key]) <= 1e-8, key
    hp = mh.generic.filters.butterworth(x[:, 0], 0.5, 50.0)
    assert _scale_err(hp, d["out_hp"]) <= 1e-8
    mag = acc.magnitude(x[:, 0], x[:, 1], x[:, 2])
    assert mag.dtype == np.float32 and (mag == d["magnitude"]).all()
    assert (acc.magnitude(t).cpu().numpy() == d["magnitude"]).all()


def test_filtfilt_long_record_vs_oracle(mh, oracle_lib):
    """4 channels x 300k samples (hundreds of warm-up chunks per channel), AoS strides,
    f32 and f64 outputs, against the sequential oracle with the same zi."""
    from scipy import signal
    from pymhealth_amd.engine import filtfilt
    rng = np.random.default_rng(3)
    n = 300_000
    x = (np.cumsum(rng.standard_normal((n, 4)), axis=0) * 0.01
         + rng.standard_normal((n, 4))).astype(np.float32)
    b, a = signal.butter(4, [0.02, 0.3], "bandpass")
    zi = signal.lfilter_zi(b, a)
    ref = oracle_lib.filtfilt(b, a, x, zi=zi)
    t = torch.from_numpy(x).cuda()
    got = filtfilt(t, b, a, zi).cpu().numpy()
    assert _scale_err(got, ref) <= 1e-8
    g32 = filtfilt(t, b, a, zi, out_dtype=torch.float32).cpu().numpy()
    np.testing.assert_allclose(g32, ref.astype(np.float32), rtol=1e-5, atol=1e-6)


def test_workspaces_on_a_non_current_stream(mh):
    """the caller-owned workspaces come from torch's allocator; with
    ``stream=`` a side stream they are tied to it (record_stream), so the current stream
    re-allocating the freed bytes while the side stream still runs cannot corrupt the
    results. Every call on the side stream equals the same call on the current stream."""
    from scipy import signal
    from pymhealth_amd.engine import filtfilt, find_peaks, magnitude_dot, minmax
    rng = np.random.default_rng(77)
    x = (np.cumsum(rng.standard_normal((400_000, 3)), axis=0) * 0.01).astype(np.float32)
    t = torch.from_numpy(x).cuda()
    b, a = signal.butter(5, 0.5 / 25.0, "highpass")
    zi = signal.lfilter_zi(b, a)
    ref_f = filtfilt(t, b, a, zi).cpu().numpy()
    ref_m = minmax(t[:, 0]).cpu().numpy()
    ref_d = magnitude_dot(t[:, 0], t[:, 1], t[:, 2]).cpu().numpy()
    ref_p = find_peaks(t[:, 1]).cpu().numpy()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    got = []
    for k in range(3):
        got.append((filtfilt(t, b, a, zi, stream=side.cuda_stream),
                    minmax(t[:, 0], stream=side.cuda_stream),
                    magnitude_dot(t[:, 0], t[:, 1], t[:, 2], stream=side.cuda_stream)))
        # the current stream takes (and overwrites) whatever the allocator hands out now
        junk = torch.full((x.size * 4,), float(k + 1), dtype=torch.float64, device="cuda")
        del junk
    peaks = find_peaks(t[:, 1], stream=side.cuda_stream)
    side.synchronize()
    for f, m, d in got:
        assert np.array_equal(f.cpu().numpy(), ref_f)
        assert np.array_equal(m.cpu().numpy(), ref_m)
        assert np.array_equal(d.cpu().numpy(), ref_d)
    assert np.array_equal(peaks.cpu().numpy(), ref_p)


@pytest.mark.parametrize("C", [1, 3])
def test_filtfilt_lds_streamed_passes_vs_oracle(mh, oracle_lib, monkeypatch, C):
    """The LDS-streamed passes (filtfilt_tile.hip: a workgroup of 64 / C chunks x C channels,
    the record DMA'd block by block, the forward output kept reversed AoS) against the
    sequential oracle and against the per-lane kernel (MHF_NO_IIR_TILE=1): a 0.5 Hz order-5
    highpass at 50 Hz (warm-up R ~ 3100), a short lowpass and an order-4 bandpass, records
    of even and odd extended length, float64 and float32 outputs; the record's first and
    last chunks carry the odd extension and the clamped DMA blocks. Within 1e-8 of the
    signal scale; an unaligned view takes the per-lane kernel."""
    from scipy import signal
    from pymhealth_amd.engine import filtfilt
    rng = np.random.default_rng(40 + C)
    filters = [signal.butter(5, 0.5 / 25.0, "highpass"), signal.butter(2, 0.2),
               signal.butter(4, [0.02, 0.3], "bandpass")]
    for n in (70_001, 1_000_003):           # one edge workgroup / interior workgroups too
        x = (np.cumsum(rng.standard_normal((n, C)), axis=0) * 0.01
             + rng.standard_normal((n, C)) + np.arange(C)).astype(np.float32)
        xs = x if C > 1 else np.ascontiguousarray(x[:, 0])
        t = torch.from_numpy(xs).cuda()
        for b, a in filters:
            zi = signal.lfilter_zi(b, a)
            ref = oracle_lib.filtfilt(b, a, xs, zi=zi)
            monkeypatch.delenv("MHF_NO_IIR_TILE", raising=False)
            got = filtfilt(t, b, a, zi).cpu().numpy()
            assert got.shape == xs.shape
            assert _scale_err(got, ref) <= 1e-8, (n, len(b))
            g32 = filtfilt(t, b, a, zi, out_dtype=torch.float32).cpu().numpy()
            np.testing.assert_allclose(g32, ref.astype(np.float32), rtol=1e-5, atol=1e-6)
            monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
            monkeypatch.setenv("MHF_NO_IIR_TILE", "1")
            old = filtfilt(t, b, a, zi).cpu().numpy()
            assert _scale_err(got, old) <= 2e-8, (n, len(b))
        monkeypatch.delenv("MHF_NO_IIR_TILE", raising=False)
    if C == 1:
        big = torch.from_numpy(np.concatenate([[0.0], xs]).astype(np.float32)).cuda()
        b, a = filters[0]
        zi = signal.lfilter_zi(b, a)
        got = filtfilt(big[1:], b, a, zi).cpu().numpy()      # 4 B past a 16-B boundary
        assert _scale_err(got, oracle_lib.filtfilt(b, a, xs, zi=zi)) <= 1e-8


def test_filtfilt_edges(mh, oracle_lib):
    from scipy import signal
    from pymhealth_amd.engine import filtfilt
    b, a = signal.butter(2, 0.2)
    zi = signal.lfilter_zi(b, a)
    for n in (10, 11, 257, 700):                # padlen = 9: n = 10 is the shortest legal
        x = np.sin(np.arange(n) * 0.3).astype(np.float32)
        got = filtfilt(torch.from_numpy(x).cuda(), b, a, zi).cpu().numpy()
        assert _scale_err(got, oracle_lib.filtfilt(b, a, x, zi=zi)) <= 1e-12, n
    with pytest.raises(ValueError):
        filtfilt(torch.zeros(9, device="cuda"), b, a)   # not longer than padlen
    g = filtfilt(torch.ones(50, device="cuda"), [2.0], [4.0])   # pure gain: 0.5 * 0.5
    assert torch.all(g == 0.25)


def test_spectral_w1024_aos_strided_vs_oracle(mh, oracle_lib):
    """The W = 1024 register FFT on strided (AoS 3-axis) input, every spectral feature,
    band / dominant ranges that start and end mid-spectrum."""
    from pymhealth_amd.engine import window_features
    x = _accel(1024 + 255 * 256, seed=21)
    names = ["band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"]
    kw = dict(fs=50.0, band=(0.7, 6.1), dom=(0.5, 12.0))
    got = window_features(torch.from_numpy(x).cuda(), 1024, 256, _ids(names), **kw).cpu().numpy()
    ref = oracle_lib.window_features(x, 1024, 256, names, **kw)
    assert got.shape == ref.shape == (3, 4, 256)
    spectral_check(oracle_lib, got, ref, names, x, 1024, 256, 50.0, kw["dom"], tag="aos")


@pytest.mark.parametrize("names", [["band_power"],
                                   ["band_power", "dominant_frequency"],
                                   ["relative_band_power", "spectral_entropy"],
                                   ["band_power", "relative_band_power", "spectral_entropy",
                                    "dominant_frequency"]])
@pytest.mark.parametrize("offset", [0, 1])
def test_spectral_w1024_feature_sets_vs_oracle(mh, oracle_lib, names, offset):
    """cfg5 geometry (W = 1024, S = 128, contiguous): every compile-time feature set of the
    LDS-DMA register-FFT kernel (offset 0: 16-B aligned windows) and the VGPR-prefetch
    kernel (offset 1 sample: unaligned windows) against the oracle."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(31 + offset)
    nw, W, S = 700, 1024, 128
    x = (rng.standard_normal((nw - 1) * S + W + offset) * 0.3
         + np.sin(np.arange((nw - 1) * S + W + offset) * 0.11) + 1.5).astype(np.float32)
    kw = dict(fs=256.0, band=(0.5, 40.0), dom=(0.5, 40.0))
    got = window_features(torch.from_numpy(x).cuda()[offset:], W, S, _ids(names),
                          **kw).cpu().numpy()
    ref = oracle_lib.window_features(x[offset:], W, S, names, **kw)
    assert got.shape == ref.shape == (1, len(names), nw)
    spectral_check(oracle_lib, got, ref, names, x[offset:], W, S, 256.0, kw["dom"],
                   tag=str(names))


@pytest.mark.parametrize("band,dom", [((0.5, 15.0), (0.5, 15.0)), ((0.5, 16.0), (0.5, 16.0)),
                                      ((0.0, 16.25), (None, None)), ((20.0, 31.75), (1.0, 32.0)),
                                      ((0.5, 40.0), (0.5, 40.0)), ((40.0, 63.75), (30.0, 64.0)),
                                      ((60.0, 80.0), (0.5, 80.0)), ((100.0, 128.0), (0.5, 128.0)),
                                      ((None, None), (2.0, 10.0)), ((0.5, 128.0), (2.0, 10.0))])
@pytest.mark.parametrize("names", [["band_power"], ["band_power", "dominant_frequency"],
                                   ["relative_band_power", "dominant_frequency"]])
@pytest.mark.parametrize("offset", [0, 1, 4])
def test_spectral_w1024_row_count_variants(mh, oracle_lib, monkeypatch, band, dom, names, offset):
    """Without total power only the rows (64 bins each) that hold band / arg-max bins are
    evaluated; the launch picks a kernel compiled for that row count (1-4, else all 8). Every
    variant equals the all-rows kernel (MHF_SPECREG_ALLROWS=1) bit for bit and the oracle;
    ranges end on row edges (bins 60, 64, 65, 127, 128, 255, 256), the Nyquist bin included.
    offset 0: sample ring (S = 128); offset 4: the private LDS-DMA path (S = 1024); offset 1:
    unaligned windows, the VGPR-prefetch path. The band reaching rows 6-7 with a narrow
    arg-max range is the case a sign-extended row-class word once broke."""
    from pymhealth_amd.engine import window_features
    nw, W = 300, 1024
    S = 128 if offset == 0 else 1024
    n = (nw - 1) * S + W
    rng = np.random.default_rng(77 + offset)
    x = (rng.standard_normal(n + offset) * 0.3 + np.sin(np.arange(n + offset) * 0.31)
         + 0.7).astype(np.float32)
    kw = dict(fs=256.0, band=band, dom=dom)
    if dom == (None, None):
        names = ["band_power"]
    if band == (None, None):
        names = [n for n in names if n != "band_power"] or ["dominant_frequency"]
    xd = torch.from_numpy(x).cuda()[offset:]
    got = window_features(xd, W, S, _ids(names), **kw).cpu().numpy()
    monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
    monkeypatch.setenv("MHF_SPECREG_ALLROWS", "1")
    full = window_features(xd, W, S, _ids(names), **kw).cpu().numpy()
    monkeypatch.delenv("MHF_SPECREG_ALLROWS")
    np.testing.assert_array_equal(got, full)
    ref = oracle_lib.window_features(x[offset:], W, S, names, **kw)
    spectral_check(oracle_lib, got, ref, names, x[offset:], W, S, 256.0, kw["dom"],
                   tag=f"rows band={band} dom={dom}")


@pytest.mark.parametrize("S", [4, 36, 64, 128, 256, 384, 512, 768])
@pytest.mark.parametrize("nw", [1, 6, 333, 4099])
def test_spectral_w1024_ring_vs_private_dma(mh, oracle_lib, monkeypatch, S, nw):
    """The sample-ring variant of the W = 1024 register FFT (overlapping contiguous
    windows: one LDS ring per wave over a contiguous window run) against the private-window
    DMA variant (MHF_SPECREG_NORING=1: same arithmetic, so bit-identical) and the oracle,
    two channels, ragged run tails and runs shorter than a wave's share. S = 128, 256, 384,
    512 take the scalar row-offset reads (S and phi multiples of 128; S = 384 has phi = 128),
    S = 4, 36, 64 the per-lane wrapped reads; S = 768 exceeds the ring's LDS budget and
    takes the private path both times."""
    from pymhealth_amd.engine import window_features
    W, C = 1024, 2
    n = (nw - 1) * S + W
    rng = np.random.default_rng(S * 7 + nw)
    x = (rng.standard_normal((C, n)) * 0.3 + np.sin(np.arange(n) * 0.07) + 1.1).astype(np.float32)
    names = ["band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"]
    kw = dict(fs=128.0, band=(0.5, 20.0), dom=(0.5, 30.0))
    xd = torch.from_numpy(x).cuda().T          # (n, C), channel-contiguous planes
    got = window_features(xd, W, S, _ids(names), **kw).cpu().numpy()
    monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
    monkeypatch.setenv("MHF_SPECREG_NORING", "1")
    priv = window_features(xd, W, S, _ids(names), **kw).cpu().numpy()
    monkeypatch.delenv("MHF_SPECREG_NORING")
    assert got.shape == (C, len(names), nw)
    np.testing.assert_array_equal(got, priv)
    if nw <= 333:
        for c in range(C):
            ref = oracle_lib.window_features(x[c], W, S, names, **kw)
            spectral_check(oracle_lib, got[c:c + 1], ref, names, x[c], W, S, 128.0, kw["dom"],
                           tag=f"ring S={S} c={c}")


@pytest.mark.parametrize("W,S,offset", [(1024, 128, 0), (1024, 128, 1), (256, 256, 0),
                                        (256, 128, 0), (128, 128, 1), (512, 256, 0),
                                        (2048, 512, 0), (64, 64, 0)])
def test_spectral_edge_windows_vs_oracle(mh, oracle_lib, W, S, offset):
    """Every spectral kernel (tile in-lane FFT, register FFT with and without LDS-DMA, LDS
    Stockham): all-zero, constant, NaN-holding, inf-holding and impulse windows next to
    ordinary ones, every spectral feature against the oracle."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(77 + W + S)
    nw = 96
    n = (nw - 1) * S + W
    x = rng.standard_normal(n + offset).astype(np.float32)
    o0 = offset
    x[o0:o0 + W] = 0.0                                   # window 0: all zero
    x[o0 + 10 * S:o0 + 14 * S + W] = 2.5                 # windows 10..14: constant
    x[o0 + 30 * S + W // 2] = np.nan                     # window 30 (and overlaps) NaN
    x[o0 + 50 * S + 3] = np.inf                          # window 50 (and overlaps) inf
    x[o0 + 70 * S:o0 + 80 * S + W] = 0.0
    x[o0 + 75 * S + 3] = 1.0                             # an impulse in zeros
    fs = 256.0
    names = ["band_power", "relative_band_power", "spectral_entropy", "dominant_frequency"]
    kw = dict(fs=fs, band=(0.5, 40.0), dom=(0.5, 40.0))
    got = window_features(torch.from_numpy(x).cuda()[offset:], W, S, _ids(names),
                          **kw).cpu().numpy()
    xs = x[offset:]
    ref = oracle_lib.window_features(xs, W, S, names, **kw)
    # dominant frequency: exact except near-ties (constant windows: every in-range bin is
    # rounding noise in the fp64 oracle; an impulse: a flat spectrum)
    spectral_check(oracle_lib, got, ref, names, xs, W, S, fs, kw["dom"], tag="edges")


@pytest.mark.parametrize("case", ["minmax_w128", "minmax_w100", "minmax_w64_s32",
                                  "median_w75_s50"])
def test_minmax_bits_vs_reference(mh, case):
    """rolling_apply(np.min / np.max) on the GPU: the reference's bit patterns, incl. the
    sign of zero, NaN only at row 0, +-inf for all-NaN rows >= 1."""
    d = gc.load(case)
    W, S = int(d["wsize"]), int(d["wstep"])
    t = torch.from_numpy(d["x"]).cuda()
    for fn, k in ((np.min, "out_min"), (np.max, "out_max"), (np.median, "out_median")):
        if k not in d:
            continue
        got = mh.util.windows.rolling_apply(fn, W, S)(t).cpu().numpy()
        ref = d[k]
        assert (np.isnan(got) == np.isnan(ref)).all(), k
        fin = ~np.isnan(ref)
        assert (got[fin].view(np.int64) == ref[fin].view(np.int64)).all(), k


def test_minmax_indexed_vs_oracle(mh, oracle_lib):
    """nonuniform_rolling_apply(np.min / np.max): serial numerics on every window."""
    from pymhealth_amd.engine import indexed_window_features
    d = gc.load("minmax_w128")
    x = d["x"]
    starts = np.arange(0, x.size - 50, 37, dtype=np.int64)
    ends = starts + 50 + (starts % 13)
    idx = np.stack([starts, ends])
    got = indexed_window_features(torch.from_numpy(x).cuda(), torch.from_numpy(idx).cuda(),
                                  _ids(["min", "max", "median"]), min_len=1,
                                  out_dtype=torch.float64).cpu().numpy()
    ref = oracle_lib.indexed_features(x, idx, ["min", "max", "median"], min_len=1,
                                      out_dtype=np.float64)
    assert got.shape == ref.shape
    assert gc.same(got, ref).all()
    assert (np.signbit(got) == np.signbit(ref)).all()


FULL_SIZE_PLAN = {"cfg2": "tile_w256_c3", "cfg3": "tile_w256_c1", "cfg4": "tile_w256_c3",
                  "cfg5": "spectral_reg", "ovl250": "tile_fix"}


FULL_SIZE_CHUNK = 1_000_000   # windows per oracle call (host memory: cfg4 = 3 GB of samples)


@pytest.mark.default_numerics
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4", "cfg5", "ovl250"])
def test_full_size_workload_every_window_vs_oracle_and_halves(mh, oracle_lib, cfg):
    """BASELINE.json sizes (bench.py's workloads, on-device synthetic input: 1e6 x 256 x 3 /
    1e7 x 256 / 1.25e7 x 256 x 3 full set / 1e7 x 1024 stride 128): one launch over the whole
    batch equals two half launches with global window indices, bit for bit (the multi-GPU
    shard property), and EVERY window of every channel matches the oracle — moments
    bit-exact, spectral within SPEC_RTOL (spectral_check), dominant frequency exact except
    near-ties. The oracle runs in chunks of FULL_SIZE_CHUNK windows, each chunk with one
    leading window so rows >= 1 keep the prange numerics. The default numerics, as bench.py
    runs them: rows >= 1 of np.var / np.std within gc.FAST_VAR_RTOL."""
    import bench
    from pymhealth_amd.distributed import sample_range
    from pymhealth_amd.engine import window_features
    c = bench.CONFIGS[cfg]
    W, S, C, nw = c["W"], c["S"], c["C"], c["nw"]
    x = bench.synth_device(c, (nw - 1) * S + W, torch.device("cuda"), seed=99)
    names = c["feats"]
    ids = [bench.FEATURE_IDS[f] for f in names]
    kw = dict(fs=c["fs"], band=c["band"], dom=c["dom"])
    # the benchmarked shapes take the fast kernels, never the generic fallback
    from pymhealth_amd.engine import plan_name
    assert plan_name((C, 1 if C > 1 else 0, C), W, S, ids) == FULL_SIZE_PLAN[cfg]
    full = window_features(x, W, S, ids, **kw)
    assert full.shape == (C, len(ids), nw)
    h = nw // 2 + 7
    for w0, w1 in ((0, h), (h, nw)):
        s0, s1 = sample_range(w0, w1, W, S)
        part = window_features(x[s0:s1], W, S, ids, first_window=w0, n_windows=w1 - w0,
                               base_window=w0, **kw)
        assert torch.equal(part, full[:, :, w0:w1]), (w0, w1)
        del part
    spec = [j for j, n in enumerate(names) if n in gc.SPECTRAL_FEATURES]
    mom = [j for j in range(len(names)) if j not in spec]
    checked = 0
    for i0 in range(0, nw, FULL_SIZE_CHUNK):
        k = min(FULL_SIZE_CHUNK, nw - i0)
        lead = 1 if i0 > 0 else 0     # one window before: rows >= 1 keep parfor numerics
        s0 = (i0 - lead) * S
        rec = x[s0:s0 + (k + lead - 1) * S + W].cpu().numpy()
        ref = oracle_lib.window_features(rec, W, S, names, first_window=lead, n_windows=k, **kw)
        got = full[:, :, i0:i0 + k].cpu().numpy()
        if mom:
            eq = gc.same_fast_var(got[:, mom], ref[:, mom], [names[j] for j in mom], i0)
            assert eq.all(), [(cfg, i0, names[mom[j]], ch, np.nonzero(~eq[ch, j])[0][:8])
                              for ch in range(C) for j in range(len(mom)) if not eq[ch, j].all()]
        if spec:
            spectral_check(oracle_lib, got, ref, names, rec, W, S, c["fs"], c["dom"],
                           first=lead, tag="%s %d" % (cfg, i0))
        checked += k
        del rec, ref, got
    assert checked == nw
    del x, full
    torch.cuda.empty_cache()


def test_division_probe_every_divisor_and_mantissa():
    """window_moments divides each skewness / kurtosis term by len(x) as a multiply by
    RN(1/len) plus one Markstein FMA correction: tools/div_probe (built by
    __graft_entry__.build()) checks it against the IEEE quotient for every divisor 1..65536
    x every mantissa of a binade on the GPU — zero mismatches."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "div_probe")
    assert os.path.exists(exe), "tools/div_probe not built (run __graft_entry__.build())"
    r = subprocess.run([exe, "65536"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, (r.returncode, r.stdout, r.stderr)


def test_indexed_bench_workload_every_window_vs_oracle(mh, oracle_lib):
    """bench.py cfgidx at full size (1e6 time-indexed windows of 240-272 samples over the
    3-axis record, cfg2's feature set): every window-channel through
    mhf_indexed_window_features matches the oracle's indices_rolling_apply restatement
    bit for bit (every window serial numerics, windows.py:134-157)."""
    import bench
    from pymhealth_amd.engine import indexed_window_features
    c = bench.CONFIGS["cfgidx"]
    S, C, nw = c["S"], c["C"], c["nw"]
    x = bench.synth_device(c, (nw - 1) * S + c["W"] + bench.IDX_JITTER, torch.device("cuda"),
                           seed=99)
    b = bench.idx_boundaries(0, nw + 1, S)
    assert b[-1] <= x.shape[0] and np.diff(b).min() >= S - bench.IDX_JITTER
    ind = np.stack([b[:-1], b[1:]])
    ids = [bench.FEATURE_IDS[f] for f in c["feats"]]
    got = indexed_window_features(x, torch.from_numpy(ind).cuda(), ids,
                                  out_dtype=torch.float64).cpu().numpy()
    ref = oracle_lib.indexed_features(x.cpu().numpy(), ind, c["feats"], out_dtype=np.float64)
    eq = gc.same(got, ref)
    assert eq.all(), [(c["feats"][j], ch, np.nonzero(~eq[ch, j])[0][:8])
                      for ch in range(C) for j in range(len(ids)) if not eq[ch, j].all()]
    del x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("W,S,C", [(256, 256, 3), (256, 256, 1), (1024, 128, 1), (100, 37, 1)])
def test_median_mixed_with_fused_features(mh, oracle_lib, W, S, C):
    """np.median next to moments and spectral features in one call (tile / register-FFT /
    generic kernels write their planes, the median kernel its own) vs the oracle."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(W + C)
    nw = 500
    n = (nw - 1) * S + W
    x = np.round(rng.standard_normal((n, C)) * 4).astype(np.float32)   # many ties
    if C == 1:
        x = x[:, 0].copy()
    names = ["mean", "median", "var", "band_power"]
    kw = dict(fs=50.0, band=(0.5, 8.0))
    got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(names), **kw).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, names, **kw)
    assert gc.same(got[:, :3], ref[:, :3]).all()
    assert (np.signbit(got[:, 1]) == np.signbit(ref[:, 1])).all()
    spectral_check(oracle_lib, got, ref, names, x, W, S, 50.0, tag="median mix")


# ------------------------------------------- PSD-level functions, reference signatures
@pytest.mark.parametrize("case", gc.psd_cases())
def test_psd_level_functions_vs_reference_golden(mh, case):
    """hrv.power_band / relative_power_band / peak_frequency, density.peak_frequency and
    information.entropy with the reference's own argument lists (psd, freqs, lower,
    upper): a 2-D (rows, bins) call == the reference row by row, bit for bit (entropy:
    device logf/log, last-bit tolerance); 1-D calls return the same Python floats."""
    d = gc.load(case)
    hrv, dens, info = mh.heart.hrv, mh.generic.frequency.density, mh.generic.information
    fns = {"power_band": hrv.power_band, "relative_power_band": hrv.relative_power_band,
           "hrv_peak_frequency": hrv.peak_frequency,
           "density_peak_frequency": dens.peak_frequency}
    psd, freqs = d["psd"], d["freqs"]
    for b in gc.PSD_BOUNDS:
        lo, hi = gc.psd_bounds(d, b)
        for k, fn in fns.items():
            ref, rz = d["out_%s_%s" % (k, b)], d["raises_%s_%s" % (k, b)]
            got = fn(psd, freqs, lo, hi)
            assert isinstance(got, np.ndarray) and got.shape == ref.shape
            eq = gc.same(got, ref, rz)
            assert eq.all(), (case, b, k, np.nonzero(~eq)[0][:8], got[~eq][:3], ref[~eq][:3])
            for i in (0, 1, 4, 6):
                one = fn(psd[i], freqs, lo, hi)
                assert isinstance(one, float) and (rz[i] or gc.same(np.float64(one), ref[i]))
    # device-resident rows in, device values out
    tp = torch.from_numpy(psd).cuda()
    got = hrv.power_band(tp, torch.from_numpy(freqs).cuda(), 0.5, 4.0)
    assert isinstance(got, torch.Tensor) and got.is_cuda
    assert gc.same(got.cpu().numpy(), d["out_power_band_band"]).all()
    rtol = 1e-6 if psd.dtype == np.float32 else 1e-14
    ent = info.entropy(psd)
    np.testing.assert_allclose(ent, d["out_entropy"], rtol=rtol, atol=0, equal_nan=True)
    assert abs(info.entropy(psd[0]) - d["out_entropy"][0]) <= rtol * abs(d["out_entropy"][0])
    # the window-level factories keep their own names
    assert mh.features.band_power(50.0, 0.5, 4.0).fid == mh._lib.MHF_BAND_POWER


# ------------------------------------------------------------------ §8f N3 order statistics
ORDER = ["median", "interquartile_range", "mode", "percentile"]


def _order_signal(n, C, seed, W):
    """Ties, signed zeros, NaN / inf windows: the cases where numba's own permutation
    decides the answer."""
    rng = np.random.default_rng(seed)
    x = np.round(rng.standard_normal((n, C)) * 2).astype(np.float32)
    x[x == 0] = np.where(rng.random(int((x == 0).sum())) < 0.5, -0.0, 0.0)
    for k in range(0, n - W, 7 * W):
        x[k + 3, :] = np.nan                         # a NaN window every 7
    for k in range(2 * W, n - W, 11 * W):
        x[k + 1, :] = np.inf                         # an inf window every 11
        x[k + 5, :] = -np.inf
    for k in range(3 * W, n - W, 13 * W):
        x[k:k + W, :] = np.where(np.arange(W)[:, None] % 2, 0.0, -0.0)   # all zeros, mixed
    return x if C > 1 else x[:, 0].copy()


@pytest.mark.parametrize("W,S,C", [(64, 64, 3), (100, 37, 1), (256, 256, 3), (7, 3, 1),
                                   (2, 1, 1), (1, 1, 1), (1024, 512, 1), (2048, 1024, 1),
                                   (4096, 4096, 2)])
@pytest.mark.parametrize("q", [0.0, 12.5, 50.0, 90.0, 100.0])
def test_order_statistics_vs_oracle(mh, oracle_lib, W, S, C, q):
    """median / interquartile_range / mode / percentile(q), every window bit for bit the
    oracle's numba replay (incl. the sign of zero and NaN placement), on AoS input with
    ties, mixed +0/-0, NaN and +-inf windows; W up to 4096 (serial-replay paths)."""
    from pymhealth_amd.engine import plan_name, window_features
    nw = 300 if W <= 256 else 40
    x = _order_signal((nw - 1) * S + W, C, W + S + C, W)
    ids = _ids(ORDER)
    cs = (C, 1 if C > 1 else 0, C)
    assert plan_name(cs, W, S, ids).endswith("order")
    got = window_features(torch.from_numpy(x).cuda(), W, S, ids, percentile_q=q).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, ORDER, percentile_q=q)
    assert got.shape == ref.shape
    eq = gc.same(got, ref) & (np.signbit(got) == np.signbit(ref))
    assert eq.all(), [(ORDER[j], c, np.nonzero(~eq[c, j])[0][:5], got[c, j][~eq[c, j]][:3],
                       ref[c, j][~eq[c, j]][:3])
                      for c in range(got.shape[0]) for j in range(len(ORDER)) if not eq[c, j].all()]


@pytest.mark.parametrize("W,S,C", [(64, 64, 3), (100, 37, 1), (256, 256, 3), (7, 3, 1),
                                   (2, 1, 1), (1, 1, 1), (1024, 512, 1), (600, 300, 2),
                                   (200, 100, 3), (256, 128, 1), (500, 250, 1)])
@pytest.mark.parametrize("q", [0.0, 37.5, 50.0, 100.0])
@pytest.mark.parametrize("feats", [["median"], ["median", "interquartile_range", "percentile"],
                                   ["percentile"]])
def test_order_selection_vs_oracle(mh, oracle_lib, W, S, C, q, feats):
    """Calls without stats.mode select ranks in registers (select_rank_u32) instead of
    sorting: every window bit for bit the oracle's numba replay on the same tie / signed
    zero / NaN / inf windows as test_order_statistics_vs_oracle. A tail shorter than the
    stride past the last window lets windows shorter than their power of two take the
    whole-window vector loads (order_kernel<E, float, C>) too."""
    from pymhealth_amd.engine import window_features
    nw = 300 if W <= 256 else 40
    tail = min(60, S - 1)
    x = _order_signal((nw - 1) * S + W + tail, C, W + 3 * S + C, W)
    got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(feats), percentile_q=q).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, feats, percentile_q=q)
    assert got.shape == ref.shape
    eq = gc.same(got, ref) & (np.signbit(got) == np.signbit(ref))
    assert eq.all(), [(feats[j], c, np.nonzero(~eq[c, j])[0][:5], got[c, j][~eq[c, j]][:3],
                       ref[c, j][~eq[c, j]][:3])
                      for c in range(got.shape[0]) for j in range(len(feats)) if not eq[c, j].all()]
    # plain random windows (no ties): the selection's common case
    rng = np.random.default_rng(W)
    y = rng.standard_normal(((nw - 1) * S + W + tail, C) if C > 1 else (nw - 1) * S + W + tail).astype(np.float32)
    got = window_features(torch.from_numpy(y).cuda(), W, S, _ids(feats), percentile_q=q).cpu().numpy()
    ref = oracle_lib.window_features(y, W, S, feats, percentile_q=q)
    assert gc.same(got, ref).all()


@pytest.mark.parametrize("W,S,C", [(256, 256, 3), (256, 256, 1), (255, 256, 3), (255, 256, 1),
                                   (512, 512, 3), (1024, 1024, 1), (1000, 1024, 3), (384, 128, 3)])
def test_order_median_interleaved_vs_oracle(mh, oracle_lib, W, S, C):
    """Median / percentile / IQR without mode on the vector path go through
    order_sel_kernel (rank searches from each channel's common key prefix, select_multi_u32)
    and the rescan launch: accel-like axes (z near 1 g: a shared top
    byte), constant windows, windows of few distinct values (ties at the middle ranks), odd
    W (a padding key), and windows holding NaN / zero / inf (the per-channel path) — every
    window bit for bit the oracle."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(W + C)
    nw = 200
    n = nw * S
    t = np.arange(n) / 50.0
    cols = [0.3 * np.sin(2 * np.pi * 1.7 * t) + 0.05 * rng.standard_normal(n),
            0.2 * np.sin(2 * np.pi * 0.9 * t + 1) + 0.05 * rng.standard_normal(n),
            1.0 + 0.1 * np.sin(2 * np.pi * 2.3 * t + 2) + 0.05 * rng.standard_normal(n)]
    x = np.stack(cols[3 - C:], axis=1).astype(np.float32)
    x[3 * S:3 * S + W] = 1.25                                        # constant window
    x[5 * S:5 * S + W] = rng.integers(0, 3, size=(W, C)) * 0.5 + 0.5  # ties
    x[7 * S + 11, 0] = np.nan
    x[9 * S + 3, C - 1] = 0.0
    x[11 * S + W // 2, 0] = -np.inf
    x[13 * S:13 * S + W] = -2.0 - rng.integers(0, 2, size=(W, C))     # negative, two values
    # zero-heavy windows (zeros of one sign stay on the selection, both signs
    # replay): zero padding, all -0.0, quantized integers around 0, +0 and -0 mixed
    x[15 * S:15 * S + W] = 0.0
    x[15 * S + 7:15 * S + 20] = 1.5
    x[17 * S:17 * S + W] = -0.0
    x[17 * S + 3] = -1.0
    x[19 * S:19 * S + W] = rng.integers(-2, 3, size=(W, C)).astype(np.float32)
    x[21 * S:21 * S + W] = np.where(rng.random((W, C)) < 0.5, 0.0, -0.0)
    x[21 * S + 5] = 2.0
    if C == 1:
        x = x[:, 0].copy()
    # the median alone and the statistics loop (percentile at q = 0 / 37.5 / 100, IQR; a
    # moment beside them), float64 and float32 outputs (the rescan launch finds its windows
    # by the sentinel of either width)
    for feats, q in ((["median"], 50.0), (["mean", "percentile", "median", "interquartile_range"], 37.5),
                     (["percentile", "interquartile_range"], 0.0), (["percentile"], 100.0)):
        ref = oracle_lib.window_features(x, W, S, feats, percentile_q=q)
        for odt in (torch.float64, torch.float32):
            got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(feats), percentile_q=q,
                                  out_dtype=odt).cpu().double().numpy()
            want = ref if odt == torch.float64 else ref.astype(np.float32).astype(np.float64)
            assert got.shape == want.shape
            eq = gc.same(got, want) & (np.signbit(got) == np.signbit(want))
            assert eq.all(), [(feats, q, odt, c, j, np.nonzero(~eq[c, j])[0][:5], got[c, j][~eq[c, j]][:3],
                               want[c, j][~eq[c, j]][:3])
                              for c in range(got.shape[0]) for j in range(len(feats)) if not eq[c, j].all()]


def test_order_even_window_one_zero_middle(mh, oracle_lib):
    """Even W whose two middle order statistics are a (signed) zero and a non-zero."""
    from pymhealth_amd.engine import window_features
    W = 8
    rows = [[-3, -2, -1, -0.0, 1, 2, 3, 4], [-3, -2, -1, 0.0, 1, 2, 3, 4],
            [-3, -2, -0.0, 0.0, 5, 6, 7, 8], [-4, -3, -2, -1, -0.0, 2, 3, 4]]
    x = np.asarray(rows, np.float32).ravel()
    for feats in (["median", "mode"], ["median"]):          # sort and selection paths
        got = window_features(torch.from_numpy(x).cuda(), W, W, _ids(feats)).cpu().numpy()
        ref = oracle_lib.window_features(x, W, W, feats)
        assert gc.same(got, ref).all() and (np.signbit(got) == np.signbit(ref)).all(), feats


@pytest.mark.parametrize("W,S", [(64, 64), (128, 97), (300, 300), (16, 3)])
def test_sampen_vs_oracle(mh, oracle_lib, W, S):
    """information.sampen (mm 1 / 2 / 3, r, sd given or None) vs the oracle's line-by-line
    restatement: identical counts, so equal up to the last bit of the device log."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(W * S)
    nw = 200
    x = np.round(rng.standard_normal((nw - 1) * S + W) * 3).astype(np.float32) / 2
    x[2 * S:2 * S + W] = 1.5                                   # constant window
    for mm, r, sd in ((2, 0.2, None), (1, 0.35, None), (3, 0.15, 0.5), (0, 0.2, None)):
        got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(["sampen"]), sampen_m=mm,
                              sampen_r=r, sampen_sd=sd).cpu().numpy()
        ref = oracle_lib.window_features(x, W, S, ["sampen"], sampen_m=mm, sampen_r=r,
                                         sampen_sd=sd)
        np.testing.assert_allclose(got, ref, rtol=4e-16, atol=0, equal_nan=True,
                                   err_msg=str((mm, r, sd)))


def test_order_and_sampen_indexed_vs_oracle(mh, oracle_lib):
    """nonuniform windows: order statistics and sampen over variable-length windows incl.
    ~1500-sample ones, empty / short (NaN) ones, AoS 2 channels; a window past
    the LDS capacity: order statistics computed (global scratch), sampen refused."""
    from pymhealth_amd.engine import indexed_window_features
    rng = np.random.default_rng(17)
    n = 20000
    x = _order_signal(n, 2, 5, 64)
    s = np.sort(rng.integers(0, n - 1600, 400))
    e = s + rng.integers(0, 1600, 400)
    ind = np.stack([s, e]).astype(np.int64)
    names = ORDER + ["sampen"]
    got = indexed_window_features(torch.from_numpy(x).cuda(), torch.from_numpy(ind).cuda(),
                                  _ids(names), min_len=3, percentile_q=33.0,
                                  out_dtype=torch.float64).cpu().numpy()
    ref = oracle_lib.indexed_features(x, ind, names, min_len=3, percentile_q=33.0,
                                      out_dtype=np.float64)
    eq = gc.same(got[:, :4], ref[:, :4]) & (np.signbit(got[:, :4]) == np.signbit(ref[:, :4]))
    assert eq.all()
    np.testing.assert_allclose(got[:, 4], ref[:, 4], rtol=4e-16, atol=0, equal_nan=True)
    # a window past the LDS capacity (9000 samples x 2 channels): order statistics sorted in
    # global scratch, sampen refused
    big_i = np.array([[0], [9000]], np.int64)
    big = torch.from_numpy(big_i).cuda()
    got = indexed_window_features(torch.from_numpy(x).cuda(), big, _ids(ORDER), percentile_q=33.0,
                                  out_dtype=torch.float64).cpu().numpy()
    ref = oracle_lib.indexed_features(x, big_i, ORDER, percentile_q=33.0, out_dtype=np.float64)
    assert gc.same(got, ref).all() and (np.signbit(got) == np.signbit(ref)).all()
    with pytest.raises(NotImplementedError):
        indexed_window_features(torch.from_numpy(x).cuda(), big, _ids(["sampen"]))


def test_order_features_through_rolling_apply(mh):
    """The drop-in surface: stats.interquartile_range / stats.mode /
    functools.partial(np.percentile, q=...) / information.sampen in one list call."""
    d = gc.load("n3_sort_w100_s37")
    st, info = mh.generic.stats, mh.generic.information
    funcs = [st.interquartile_range, st.mode, functools.partial(np.percentile, q=90),
             np.median]
    res = mh.util.windows.rolling_apply(funcs, 100, 37)(d["x"])
    for k, got in zip(["interquartile_range", "mode", "percentile_90"], res):
        assert gc.same(got, d["out_" + k]).all()
        assert (np.signbit(got) == np.signbit(d["out_" + k])).all()
    with pytest.raises(TypeError):
        mh.util.windows.rolling_apply(np.percentile, 100, 37)
    ds = gc.load("n3_sampen_w128_s97")
    got = mh.util.windows.rolling_apply(functools.partial(info.sampen, mm=3, r=0.15), 128, 97)(
        ds["x"])
    np.testing.assert_allclose(got, ds["out_sampen_m3_r0.15"], rtol=4e-16, atol=0,
                               equal_nan=True)


# ------------------------------------------------------------------ §8f N3 recurrence quantification
RQA = ["rqa_recurrence_rate", "rqa_determinism", "rqa_laminarity", "rqa_length_entropy"]


@pytest.mark.parametrize("W,S,C", [(64, 64, 1), (100, 37, 3), (2, 1, 1), (257, 128, 1),
                                   (1500, 1500, 1)])
@pytest.mark.parametrize("radius,minlen", [(0.0, 2), (0.25, 2), (0.25, 1), (0.6, 4)])
def test_rqa_vs_oracle(mh, oracle_lib, W, S, C, radius, minlen):
    """The pairwise RQA kernel vs the oracle's literal restatement of rqa.py (which builds
    the matrix): counts exact, so every ratio is bit-exact; length entropy to the last
    bit of the device log."""
    from pymhealth_amd.engine import window_features
    rng = np.random.default_rng(W + C)
    nw = 60 if W < 1000 else 6
    n = (nw - 1) * S + W
    x = (np.round((np.sin(np.arange(n) * 0.37)[:, None] + 0.4 * rng.standard_normal((n, C)))
                  * 4) / 4).astype(np.float32)
    x[S + 2, :] = np.nan
    x[3 * S:3 * S + W, :] = 1.0                     # one all-recurrent window
    if C == 1:
        x = x[:, 0].copy()
    kw = dict(rqa_radius=radius, rqa_minlen=minlen)
    got = window_features(torch.from_numpy(x).cuda(), W, S, _ids(RQA), **kw).cpu().numpy()
    ref = oracle_lib.window_features(x, W, S, RQA, **kw)
    assert gc.same(got[:, :3], ref[:, :3]).all()
    np.testing.assert_allclose(got[:, 3], ref[:, 3], rtol=1e-15, atol=0, equal_nan=True)


def test_rqa_matrix_level_module_vs_reference(mh):
    """mhealth.generic.rqa's matrix functions with the reference's signatures, against the
    reference's own outputs on one record (n3_rqa_matrix)."""
    d = gc.load("n3_rqa_matrix")
    rqa = mh.generic.rqa
    r = rqa.rq(d["x"], 0.2)
    assert isinstance(r, np.ndarray) and (r == d["rq"]).all()
    assert (rqa.rq(d["x"]) == d["rq0"]).all()
    assert rqa.recurrence_rate(r) == d["recurrence_rate"]
    assert rqa.determinism(r) == d["determinism"]
    assert rqa.laminarity(r) == d["laminarity"]
    assert (rqa.diagonal_lengths(r) == d["diagonal_lengths"]).all()
    assert (rqa.diagonal_lengths(r, 3) == d["diagonal_lengths3"]).all()
    assert (rqa.vertical_lengths(r) == d["vertical_lengths"]).all()
    assert abs(rqa.length_entropy(r) - d["length_entropy"]) <= 1e-15 * abs(d["length_entropy"])


@pytest.mark.parametrize("case", ["elementwise_float32", "elementwise_float64"])
def test_elementwise_helpers_vs_reference_golden(mh, oracle_lib, case):
    """accelerometer.roll / pitch / magnitude_dot and timedom.gradient / zero_crossings on
    the GPU against the reference's outputs: gradient and zero crossings bit for bit;
    roll / pitch within the fp32 (fp64) ulp of atan2 (the device atan2 vs glibc's, which
    the C oracle reproduces exactly); magnitude_dot within the BLAS dot-order tolerance.
    numpy, torch-CUDA, scalar and DataFrame inputs."""
    import pandas as pd
    acc, td = mh.inertial.accelerometer, mh.generic.timedom
    d = gc.load(case)
    x, y, z = d["x"], d["y"], d["z"]
    f32 = x.dtype == np.float32
    rtol = 2.4e-7 if f32 else 4.5e-16      # one ulp of the atan2 result, relative
    for got, ref in ((acc.roll(y, z), d["out_roll"]), (acc.pitch(x, y, z), d["out_pitch"])):
        assert got.dtype == np.float64 and got.shape == ref.shape
        np.testing.assert_allclose(got, ref, rtol=rtol, atol=0, equal_nan=True)
        assert (np.isnan(got) == np.isnan(ref)).all()
    g = td.gradient(x)
    assert g.dtype == np.float64 and gc.same(g, d["out_gradient"]).all()
    for th in (0.0, 0.05):
        zc = td.zero_crossings(x, th)
        assert zc.dtype == np.bool_ and (zc == d["out_zero_crossings_th%g" % th]).all()
    np.testing.assert_allclose(acc.magnitude_dot(x[40:], y[40:], z[40:]), d["out_magnitude_dot"],
                               rtol=1e-6 if f32 else 1e-14)
    # torch CUDA input stays on the device; DataFrame forms return named Series
    t = td.gradient(torch.from_numpy(x).cuda())
    assert t.is_cuda and gc.same(t.cpu().numpy(), d["out_gradient"]).all()
    df = pd.DataFrame({"x": x, "y": y, "z": z})
    r = acc.roll(df)
    assert isinstance(r, pd.Series) and r.name == "roll"
    np.testing.assert_allclose(r.values, d["out_roll"], rtol=rtol, atol=0, equal_nan=True)
    assert acc.pitch(df).name == "pitch"
    qrs = mh.heart.qrs
    for f in (qrs.find_peaks, qrs.nb_find_peaks):
        got = f(d["x_peaks"])
        assert got.dtype == np.int64 and np.array_equal(got, d["out_find_peaks"])
    tp = qrs.find_peaks(torch.from_numpy(d["x_peaks"]).cuda())
    assert tp.is_cuda and np.array_equal(tp.cpu().numpy(), d["out_nb_find_peaks"])
    rng = np.random.default_rng(3)
    for n in (0, 1, 2, 3, 1023, 1024, 1025, 5000):   # block edges of the compaction
        v = np.round(rng.standard_normal(n) * 2).astype(x.dtype)
        assert np.array_equal(qrs.nb_find_peaks(v), oracle_lib.find_peaks(v)), n
    assert isinstance(acc.roll(1.0, 2.0), float)
    np.testing.assert_allclose(acc.roll(1.0, 2.0), np.degrees(np.arctan2(1.0, 2.0)), rtol=4.5e-16)


def test_register_tiles_equal_the_kernels_they_replace(mh, monkeypatch):
    """The register-tile paths give bit for bit the rows of the kernels they replaced (each
    pinned to the reference and the oracle by the rest of this suite): the indexed register
    tile vs the lane walk (MHF_NO_TILE_IDX=1; jittered 3-axis windows, and beside the order
    kernel in one call), the fixed-window tile vs the span kernel (MHF_NO_TILE_FIX=1; W = 250,
    S = 125 and W = 100, S = 37)."""
    from pymhealth_amd import engine
    rng = np.random.default_rng(44)
    x3 = torch.from_numpy(_tile_idx_record(60000, 3, seed=3)).cuda()
    x1 = torch.from_numpy(_tile_idx_record(60000, 1, seed=4)).cuda()
    s = np.sort(rng.integers(0, 59000, 4000))
    ind = torch.from_numpy(np.stack([s, s + rng.integers(200, 300, 4000)]).astype(np.int64)).cuda()
    mom = _ids(TILE_IDX_SETS["x2"])
    order = _ids(["median", "percentile", "interquartile_range", "mode"])
    calls = [
        ("MHF_NO_TILE_IDX", lambda: engine.indexed_window_features(x3, ind, mom, min_len=3,
                                                                   out_dtype=torch.float64)),
        ("MHF_NO_TILE_IDX", lambda: engine.indexed_window_features(x1, ind, order + mom, min_len=3,
                                                                   percentile_q=33.0,
                                                                   out_dtype=torch.float64)),
        ("MHF_NO_TILE_FIX", lambda: engine.window_features(x3, 250, 125, mom)),
        ("MHF_NO_TILE_FIX", lambda: engine.window_features(x1, 100, 37, mom)),
    ]
    for env, call in calls:
        monkeypatch.delenv(env, raising=False)
        got = call().cpu().numpy()
        monkeypatch.setenv("MHF_DIAGNOSTICS", "1")
        monkeypatch.setenv(env, "1")
        ref = call().cpu().numpy()
        monkeypatch.delenv(env)
        assert got.shape == ref.shape, env
        assert gc.same(got, ref).all(), (env, np.argwhere(~gc.same(got, ref))[:5])
