"""Loader for the reference-generated fixtures in tests/golden (see make_golden.py)."""
import glob
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# fixture key -> oracle / engine feature name
MOMENT_FEATURES = {
    "mean": "mean", "var": "var", "std": "std", "skewness": "skewness",
    "kurtosis": "kurtosis", "kurtosis_excess": "kurtosis_excess", "drange": "drange",
    "zero_crossing_count": "zero_crossings", "zero_crossing_count_th0.05": "zero_crossings",
    "line_length": "line_length", "rms": "rms", "peak_count": "peak_count",
    "hjorth_activity": "var32", "std_in_fn": "std32", "mean_in_fn": "mean32",
    # §8f N3 / N4 (make_golden.py n3n4_cases)
    "coeff_var": "coeff_var", "hjorth_mobility": "hjorth_mobility",
    "hjorth_complexity": "hjorth_complexity", "rmssd": "rmssd", "sdsd": "sdsd", "ssd": "ssd",
    "pnn50": "pnnx", "pnnx20": "pnnx", "csi_sd1": "csi_sd1", "csi_sd1_half": "csi_sd1",
    "csi_sd2": "csi_sd2", "lorenz_csi": "lorenz_csi", "lorenz_cvi": "lorenz_cvi",
    "lorenz_mcsi": "lorenz_mcsi", "sdnn": "std32",
    # np.min / np.max passed directly (make_golden.py minmax_cases)
    "min": "min", "max": "max", "median": "median",
    # information.entropy on the window's samples (make_golden.py psd_cases)
    "entropy": "entropy",
    # §8f N3 order statistics and sample entropy (make_golden.py n3_sort_cases)
    "interquartile_range": "interquartile_range", "mode": "mode",
    "percentile_0": "percentile", "percentile_12.5": "percentile", "percentile_33": "percentile",
    "percentile_50": "percentile", "percentile_90": "percentile", "percentile_100": "percentile",
    "sampen": "sampen", "sampen_m3_r0.15": "sampen", "sampen_sd0.5": "sampen",
    # recurrence quantification (make_golden.py rqa_cases)
    "rqa_recurrence_rate": "rqa_recurrence_rate", "rqa_determinism": "rqa_determinism",
    "rqa_laminarity": "rqa_laminarity", "rqa_length_entropy": "rqa_length_entropy",
    "rqa_length_entropy_min3": "rqa_length_entropy", "rqa_determinism_r0": "rqa_determinism",
    "rqa_recurrence_rate_r0": "rqa_recurrence_rate",
    # 2-D (N, c) records (make_golden.py block2d_cases)
    "p25": "percentile",
}
ZC_THRESHOLD = {"zero_crossing_count_th0.05": 0.05}
# engine / oracle keyword parameters a fixture key was made with
FEATURE_KWARGS = {
    "zero_crossing_count_th0.05": {"zc_threshold": 0.05},
    "percentile_0": {"percentile_q": 0.0}, "percentile_12.5": {"percentile_q": 12.5},
    "percentile_33": {"percentile_q": 33.0}, "percentile_50": {"percentile_q": 50.0},
    "percentile_90": {"percentile_q": 90.0}, "percentile_100": {"percentile_q": 100.0},
    "sampen_m3_r0.15": {"sampen_m": 3, "sampen_r": 0.15}, "sampen_sd0.5": {"sampen_sd": 0.5},
    "rqa_recurrence_rate": {"rqa_radius": 0.3}, "rqa_determinism": {"rqa_radius": 0.3},
    "rqa_laminarity": {"rqa_radius": 0.3}, "rqa_length_entropy": {"rqa_radius": 0.3},
    "rqa_length_entropy_min3": {"rqa_radius": 0.3, "rqa_minlen": 3},
    "pnnx20": {"pnn_threshold": 20.0},
    "csi_sd1_half": {"csi_factor": 0.5},
    "p25": {"percentile_q": 25.0},
}
# fixture keys whose reference value goes through a libm transcendental in fp64
# (np.log10): the device's log10 may differ from glibc's in the last bit
LIBM_KEYS = {"lorenz_cvi": 4e-16, "entropy": 1e-6, "sampen": 4e-16, "sampen_m3_r0.15": 4e-16,
             "sampen_sd0.5": 4e-16, "rqa_length_entropy": 1e-15,
             "rqa_length_entropy_min3": 1e-15}
PSD_FUNCS = ["power_band", "relative_power_band", "hrv_peak_frequency",
             "density_peak_frequency"]
PSD_BOUNDS = ["none", "band", "empty", "lo_only", "hi_only", "wide", "edge"]
SPECTRAL_FEATURES = ["band_power", "relative_band_power", "spectral_entropy",
                     "dominant_frequency"]


def load(name):
    d = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    if "x" not in d and "x_seed" in d:
        x = np.random.default_rng(int(d["x_seed"])).standard_normal(int(d["n"])).astype(
            np.float32)
        if hashlib.sha256(x.tobytes()).hexdigest() != str(d["x_sha256"]):
            raise RuntimeError("regenerated input of %s does not match its sha256" % name)
        d["x"] = x
    return d


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def moment_cases():
    """(case, fixture_key, engine_feature, zc_threshold) for every moment fixture."""
    out = []
    for n in names():
        d = np.load(os.path.join(GOLDEN, n + ".npz"))
        if ("fs" in d.files or "wsize" not in d.files or "indices" in d.files
                or n == "n3_rqa_matrix" or n.startswith("block_") or n.startswith("f64_")
                or n.startswith("surface_")):
            continue
        for k in d.files:
            if k.startswith("out_"):
                f = k[4:]
                out.append((n, f, MOMENT_FEATURES[f], FEATURE_KWARGS.get(f, {})))
    return out


def block_cases():
    """(case, fixture_key, engine_feature, kwargs) for the 2-D record fixtures: window i is
    the (wsize, c) block x[i*wstep : i*wstep + wsize] (make_golden.py block2d_cases)."""
    out = []
    for n in names():
        if n.startswith("block_"):
            d = np.load(os.path.join(GOLDEN, n + ".npz"))
            out += [(n, k[4:], MOMENT_FEATURES[k[4:]], FEATURE_KWARGS.get(k[4:], {}))
                    for k in d.files if k.startswith("out_")]
    return out


def f64_cases():
    """(case, fixture_key, engine_feature, kwargs) for the float64-input fixtures
    (make_golden.py f64_cases); 2-D records among them have a 2-D x."""
    out = []
    for n in names():
        if n.startswith("f64_"):
            d = np.load(os.path.join(GOLDEN, n + ".npz"))
            out += [(n, k[4:], MOMENT_FEATURES[k[4:]], FEATURE_KWARGS.get(k[4:], {}))
                    for k in d.files if k.startswith("out_")]
    return out


def nonuniform_cases():
    """Time-indexed window fixtures of engine features (nonuniform_rolling_apply,
    make_golden.py); the user-callable ones (nu_user_*) are nu_user_cases()."""
    return [n for n in names() if "indices" in np.load(os.path.join(GOLDEN, n + ".npz")).files
            and not n.startswith("nu_user_")]


def nu_user_cases():
    """nonuniform_rolling_apply with jitted user functions (make_golden.py nu_user_cases)."""
    return [n for n in names() if n.startswith("nu_user_")]


def nonuniform_feature_cases():
    out = []
    for n in nonuniform_cases():
        d = np.load(os.path.join(GOLDEN, n + ".npz"))
        out += [(n, k[4:], MOMENT_FEATURES[k[4:]]) for k in d.files if k.startswith("out_")]
    return out


def nonuniform_args(d):
    """(index, wsize, wstep) as the reference received them."""
    if "wsize_ns" in d:
        return (d["index"].view("M8[ns]"), np.timedelta64(int(d["wsize_ns"]), "ns"),
                np.timedelta64(int(d["wstep_ns"]), "ns"))
    return d["index"], d["wsize"][()], d["wstep"][()]


def psd_cases():
    """PSD-level function fixtures (make_golden.py psd_cases): psd_rows_f64/f32/f32f64."""
    return [n for n in names() if n.startswith("psd_rows_")]


def psd_bounds(d, b):
    lo, hi = d["bounds_" + b]
    return (None if np.isnan(lo) else float(lo)), (None if np.isnan(hi) else float(hi))


def spectral_cases():
    out = []
    for n in names():
        f = np.load(os.path.join(GOLDEN, n + ".npz")).files
        if "fs" in f and "wsize" in f:
            out.append(n)
    return out


def same(got, ref, mask=None):
    """Bit-exact equality with NaN == NaN; rows in `mask` (reference raised) ignored."""
    eq = (got == ref) | (np.isnan(got) & np.isnan(ref))
    if mask is not None:
        eq |= mask
    return eq


# Rows >= 1 of np.var / np.std on the register tiles in the default numerics (fast var,
# include/mhfeat.h MHF_NUMERICS_EXACT_VAR): var_par from the fp32-deviation sum, within
# (1 + 2^-24)^3 - 1 + 2 * 255 * 2^-53 of numba's fp64 chain; std: half that.
FAST_VAR_RTOL = {"var": 3.6e-7, "std": 1.8e-7}   # rounding 1.79e-7 + centering 1.8e-7


def same_fast_var(got, ref, names, first_window=0):
    """`same` for (..., F, nw) planes, except that rows >= 1 (global index) of the var / std
    planes may differ from the reference by FAST_VAR_RTOL relative (row 0 is array_var's
    serial fp32 result: bit-exact)."""
    eq = same(got, ref)
    for j, n in enumerate(names):
        if n not in FAST_VAR_RTOL:
            continue
        g, o = got[..., j, :], ref[..., j, :]
        with np.errstate(invalid="ignore"):
            ok = np.abs(g - o) <= FAST_VAR_RTOL[n] * np.abs(o)
        ok |= same(g, o)
        if first_window == 0:
            ok[..., 0] = same(g[..., 0], o[..., 0])
        eq[..., j, :] = ok
    return eq


def dominant_tie_ok(psd_row, lo_bin, hi_bin, got_freq, bins_per_hz, rtol=1e-5, floor=0.0):
    """A dominant-frequency answer that differs from the oracle's is acceptable only if it
    names an in-range bin whose fp64 PSD value ties the range's maximum: psd[bin] >=
    (1 - rtol) * max(psd[lo_bin:hi_bin]) - floor * sum|psd| (``floor``: the rounding level
    of the transform relative to the window's total power — a window whose in-range bins
    are all at that level, e.g. a constant window's AC bins, ties everywhere).
    ``bins_per_hz`` = W / fs (bin k sits at k fs / W)."""
    if not np.isfinite(got_freq):
        return False
    k = got_freq * bins_per_hz
    kb = int(round(k))
    if abs(k - kb) > 1e-6 * max(1.0, abs(k)) or not (lo_bin <= kb < hi_bin):
        return False
    seg = psd_row[lo_bin:hi_bin]
    top = seg.max()
    return bool(psd_row[kb] >= (1.0 - rtol) * top - floor * np.abs(psd_row).sum())
