"""``mhealth.features`` — the per-window feature catalogue of the MI355X engine.

The north star names a ``mhealth.features.*`` namespace; in the reference these
functions live in ``mhealth.generic.stats`` / ``generic.timedom`` /
``generic.information`` / ``generic.frequency.density`` / ``heart.hrv`` / ``heart.qrs``
(the ``features`` name appears only in stale docs, docs/intro.rst:26-29). Every object
here is a :class:`~pymhealth_amd.feature.WindowFeature`: pass it to
``rolling_apply`` (one fused HIP launch for a whole list) or call it on one window.

Spectral features take the sampling frequency and band edges as parameters; psd(x)
is the one-sided periodogram |X_k|^2/(fs W) (bins 1..ceil(W/2)-1 doubled) of an
on-chip fp32 rFFT, freqs = numpy.fft.rfftfreq(W, 1/fs).
"""
from . import _lib
from .feature import WindowFeature


class _ArrayEntropy(WindowFeature):
    """information.entropy: a window feature in rolling_apply, and on a whole array
    (float32 / float64, any length, rows of a 2-D array) a call of mhf_psd_features."""

    def __call__(self, x):
        from .spectrum import entropy_of
        return entropy_of(x)

    def with_params(self, **params):
        return self

mean = WindowFeature("mean", _lib.MHF_MEAN, "numpy.mean (stats.mean, stats.py:157)")
var = WindowFeature("var", _lib.MHF_VAR, "numpy.var (stats.var, stats.py:160)")
std = WindowFeature("std", _lib.MHF_STD, "numpy.std (stats.std, stats.py:159)")
skewness = WindowFeature("skewness", _lib.MHF_SKEWNESS, "stats.skewness (stats.py:97-110)",
                         "Skewness (third moment) of a distribution; 0 if std == 0.")
kurtosis = WindowFeature("kurtosis", _lib.MHF_KURTOSIS, "stats.kurtosis (stats.py:113-126)",
                         "Kurtosis B2 = mu_4 / mu_2^2; 0 if var == 0.")
kurtosis_excess = WindowFeature("kurtosis_excess", _lib.MHF_KURTOSIS_EXCESS,
                                "stats.kurtosis_excess (stats.py:129-139)", "kurtosis - 3.")
drange = WindowFeature("drange", _lib.MHF_DRANGE, "stats.drange (stats.py:35-45)",
                       "max(x) - min(x).")
rms = WindowFeature("rms", _lib.MHF_RMS, "sqrt(mean(square(x))) — hrv.rmssd form "
                    "(hrv.py:138-146) without np.diff", "Root mean square.")
zero_crossing_count = WindowFeature(
    "zero_crossing_count", _lib.MHF_ZERO_CROSSINGS, "timedom.zero_crossing_count "
    "(timedom.py:53-64)", "Number of sign changes; |x| <= th counts as 0.", zc_threshold=0.0)
peak_count = WindowFeature("peak_count", _lib.MHF_PEAK_COUNT,
                           "len(qrs.nb_find_peaks(x)) (qrs.py:215-220)",
                           "Strict local maxima x[i-1] < x[i] > x[i+1].")
line_length = WindowFeature("line_length", _lib.MHF_LINE_LENGTH,
                            "timedom.line_length (timedom.py:67-78)", "sum(|diff(x)|).")
hjorth_activity = WindowFeature("hjorth_activity", _lib.MHF_VAR32,
                                "timedom.hjorth_activity (timedom.py:81-94)",
                                "Variance (numba array_var, fp32) on every row.")
var32 = hjorth_activity
std32 = WindowFeature("std32", _lib.MHF_STD32, "np.std called inside a feature function")
mean32 = WindowFeature("mean32", _lib.MHF_MEAN32, "np.mean called inside a feature function")

# ---- §8f N3: more per-window features (lane-per-window generic kernel)
coeff_var = WindowFeature("coeff_var", _lib.MHF_COEFF_VAR, "stats.coeff_var (stats.py:142-153)",
                          "np.std(x) / np.mean(x) (fp32 quotient).")
hjorth_mobility = WindowFeature(
    "hjorth_mobility", _lib.MHF_HJORTH_MOBILITY, "timedom.hjorth_mobility (timedom.py:97-112)",
    "sqrt(var(gradient(x)) / var(x)); gradient in fp64 (timedom.py:11-31).")
hjorth_complexity = WindowFeature(
    "hjorth_complexity", _lib.MHF_HJORTH_COMPLEXITY,
    "timedom.hjorth_complexity (timedom.py:133-148)",
    "mobility(gradient(x)) / mobility(x).")

# ---- §8f N3 order statistics and sample entropy (order_kernel / sampen_kernel)
interquartile_range = WindowFeature(
    "interquartile_range", _lib.MHF_IQR, "stats.interquartile_range (stats.py:48-59)",
    "75th - 25th percentile (np.percentile(x, [75, 25]), numba's selection).")
mode = WindowFeature("mode", _lib.MHF_MODE, "stats.mode (stats.py:62-94, the jit overload)",
                     "Most frequent value of the sorted window as the reference's jit mode "
                     "counts it (first run one short, ties to the smaller value).")
sampen = WindowFeature("sampen", _lib.MHF_SAMPEN, "information.sampen (information.py:23-113)",
                       "Sample entropy -log(A / B); sampen(x, mm=2, r=0.2, sd=None), bind "
                       "mm / r / sd with functools.partial.", sampen_m=2, sampen_r=0.2,
                       sampen_sd=None)


def rqa_recurrence_rate(radius=0.0):
    """rqa.recurrence_rate(rqa.rq(x, radius)) of every window (rqa.py:9-60), without building
    the W x W matrix."""
    return WindowFeature("rqa_recurrence_rate", _lib.MHF_RQA_RR,
                         "rqa.recurrence_rate(rqa.rq(x, radius)) (rqa.py:9-60)",
                         rqa_radius=float(radius))


def rqa_determinism(radius=0.0):
    """rqa.determinism(rqa.rq(x, radius)) (rqa.py:63-88): points on diagonal lines of >= 2."""
    return WindowFeature("rqa_determinism", _lib.MHF_RQA_DET,
                         "rqa.determinism(rqa.rq(x, radius)) (rqa.py:63-88)",
                         rqa_radius=float(radius))


def rqa_laminarity(radius=0.0):
    """rqa.laminarity(rqa.rq(x, radius)) (rqa.py:91-111): points on horizontal lines of >= 2."""
    return WindowFeature("rqa_laminarity", _lib.MHF_RQA_LAM,
                         "rqa.laminarity(rqa.rq(x, radius)) (rqa.py:91-111)",
                         rqa_radius=float(radius))


def rqa_length_entropy(radius=0.0, minlen=2):
    """rqa.length_entropy(rqa.rq(x, radius), minlen) (rqa.py:156-187): entropy of the
    diagonal line-length histogram (lines of the whole window dropped, as the reference's
    _dlen_counts writes them past its array)."""
    if int(minlen) != minlen or minlen < 1:
        raise ValueError("minlen must be an integer >= 1")
    return WindowFeature("rqa_length_entropy", _lib.MHF_RQA_ENT,
                         "rqa.length_entropy(rqa.rq(x, radius), minlen) (rqa.py:156-187)",
                         rqa_radius=float(radius), rqa_minlen=int(minlen))


def percentile(q):
    """np.percentile(x, q) of every window (stats.percentile = np.percentile, stats.py:163):
    numba's _collect_percentiles — any NaN gives NaN, q = 0 / 100 the min / max with its
    infinity rules, otherwise lower (1 - m) + upper m between order statistics."""
    from .feature import PERCENTILE, _percentile_q
    return PERCENTILE.with_params(percentile_q=_percentile_q(q))


entropy = _ArrayEntropy("entropy", _lib.MHF_ENTROPY, "information.entropy (information.py:10-20)",
                        "Shannon entropy (nats) of x / sum(x) + 1e-30.")

# ---- §8f N4: HRV time-domain metrics of a window of RR intervals (d = np.diff(window))
rmssd = WindowFeature("rmssd", _lib.MHF_RMSSD, "hrv.rmssd (hrv.py:138-146)",
                      "sqrt(mean(square(diff(nni)))).")
sdsd = WindowFeature("sdsd", _lib.MHF_SDSD, "hrv.sdsd (hrv.py:160-169)", "std(diff(nni)).")
ssd = WindowFeature("ssd", _lib.MHF_SSD, "hrv.ssd (hrv.py:149-157)", "sum(diff(nni)).")
sdnn = WindowFeature("sdnn", _lib.MHF_STD32, "hrv.sdnn (hrv.py:49-62)", "std(nni).")
pnn50 = WindowFeature("pnn50", _lib.MHF_PNNX, "hrv.pnn50 (hrv.py:111-121)",
                      "Proportion of |diff(nni)| > 50 ms (nni(x, unit='ms')).",
                      unit="ms", x=50.0, pnn_threshold=50.0)
pnnx = WindowFeature("pnnx", _lib.MHF_PNNX, "hrv.pnnx (hrv.py:124-135)",
                     "Proportion of |diff(nni)| > x ms (nni(x, unit='ms', x=50.)).",
                     unit="ms", x=50.0, pnn_threshold=50.0)
csi_sd1 = WindowFeature("csi_sd1", _lib.MHF_CSI_SD1, "hrv.csi_sd1 (hrv.py:207-217)",
                        "factor * std(diff(rri)).", csi_factor=_lib.CSI_FACTOR)
csi_sd2 = WindowFeature("csi_sd2", _lib.MHF_CSI_SD2, "hrv.csi_sd2 (hrv.py:220-231)",
                        "factor * std(rri[1:] + rri[:-1]).", csi_factor=_lib.CSI_FACTOR)
lorenz_csi = WindowFeature("lorenz_csi", _lib.MHF_LORENZ_CSI, "hrv.lorenz_csi (hrv.py:234-243)",
                           "csi_sd1 / csi_sd2.", csi_factor=_lib.CSI_FACTOR)
lorenz_cvi = WindowFeature("lorenz_cvi", _lib.MHF_LORENZ_CVI, "hrv.lorenz_cvi (hrv.py:246-250)",
                           "log10(csi_sd1 * csi_sd2).", csi_factor=_lib.CSI_FACTOR)
lorenz_mcsi = WindowFeature("lorenz_mcsi", _lib.MHF_LORENZ_MCSI,
                            "hrv.lorenz_mcsi (hrv.py:253-266)", "csi_sd1**2 / csi_sd2.",
                            csi_factor=_lib.CSI_FACTOR)


def band_power(fs, lower=None, upper=None):
    """hrv.power_band(psd(x), freqs, lower, upper) (hrv.py:173-179): sum of |psd| over
    lower <= f <= upper (inclusive); None = min/max(freqs)."""
    return WindowFeature("band_power", _lib.MHF_BAND_POWER, "hrv.power_band (hrv.py:173-179)",
                         fs=fs, band=(lower, upper))


def relative_band_power(fs, lower=None, upper=None):
    """hrv.relative_power_band (hrv.py:192-198): band power / total power. A window of
    zero total power gives NaN (the reference raises ZeroDivisionError)."""
    return WindowFeature("relative_band_power", _lib.MHF_REL_BAND_POWER,
                         "hrv.relative_power_band (hrv.py:192-198)", fs=fs, band=(lower, upper))


def spectral_entropy(fs):
    """information.entropy(psd(x)) (information.py:10-20): p = psd/sum(psd) + 1e-30,
    -sum(p ln p), nats."""
    return WindowFeature("spectral_entropy", _lib.MHF_SPECTRAL_ENTROPY,
                         "information.entropy (information.py:10-20)", fs=fs)


def dominant_frequency(fs, lower=None, upper=None):
    """density.peak_frequency(psd(x), freqs, lower, upper) (density.py:17-32): the freq
    of the first maximum of psd over [first f >= lower, first f >= upper). An empty
    range gives NaN (the reference raises ValueError)."""
    return WindowFeature("dominant_frequency", _lib.MHF_DOMINANT_FREQ,
                         "density.peak_frequency (density.py:17-32)", fs=fs,
                         dom=(lower, upper))


__all__ = ["mean", "var", "std", "skewness", "kurtosis", "kurtosis_excess", "drange", "rms",
           "zero_crossing_count", "peak_count", "line_length", "hjorth_activity", "var32",
           "std32", "mean32", "band_power", "relative_band_power", "spectral_entropy",
           "dominant_frequency", "extract", "entropy", "interquartile_range", "mode",
           "percentile", "sampen", "rqa_recurrence_rate", "rqa_determinism",
           "rqa_laminarity", "rqa_length_entropy", "coeff_var", "hjorth_mobility", "hjorth_complexity",
           "rmssd", "sdsd", "ssd", "sdnn", "pnn50", "pnnx", "csi_sd1", "csi_sd2", "lorenz_csi",
           "lorenz_cvi", "lorenz_mcsi"]


def extract(x, wsize, wstep, feats, *, out_dtype=None, first_window=0, n_windows=None):
    """Fused multi-feature, multi-channel extraction: the engine's native call.

    x: (N,) or (N, C) float32 or float64 (torch CUDA tensor: zero-copy; numpy: copied to
    the GPU); a float64 record gets every feature in fp64 (``mhf_window_features_f64``).
    Returns a (C, F, nw) torch CUDA tensor (float64 unless out_dtype=torch.float32).
    Features with different parameters (zc thresholds, spectral bands) are run as
    separate fused groups.
    """
    import torch
    from .engine import num_windows, to_device, window_features
    from .feature import plan_groups, resolve
    t = to_device(x, allow_f64=True)
    fl = [resolve(f) for f in feats]
    out_dtype = out_dtype or torch.float64
    groups = plan_groups(fl)
    C = 1 if t.dim() == 1 else t.shape[1]
    nw = num_windows(t.shape[0], wsize, wstep) - first_window if n_windows is None else n_windows
    if len(groups) == 1:
        return window_features(t, wsize, wstep, [f.fid for f in fl], out_dtype=out_dtype,
                               first_window=first_window, n_windows=nw, **groups[0][1])
    out = torch.empty((C, len(fl), max(nw, 0)), dtype=out_dtype, device=t.device)
    for idx, kw in groups:
        r = window_features(t, wsize, wstep, [fl[j].fid for j in idx], out_dtype=out_dtype,
                            first_window=first_window, n_windows=nw, **kw)
        out[:, idx, :] = r
    return out
