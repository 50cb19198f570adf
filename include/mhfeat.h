/*
 * mhfeat.h — C-ABI of the MI355X sliding-window feature engine (libmhfeat.so).
 *
 * This is the drop-in boundary for pymhealth's windowed-feature hot path.
 * The reference has no native library for this path: its "operator API" is the
 * numba higher-order function
 *
 *     rolling_apply(func, wsize, wstep)(arr)            src/mhealth/util/windows.py:54-95
 *
 * whose compiled prange loop (windows.py:68-72) calls one per-window feature
 * function per pass (list dispatch windows.py:98-107 = one pass per feature).
 * mhf_window_features() replaces that compiled loop for every feature in one
 * fused launch. Its only FFI is the cffi FFTW binder
 *
 *     void fftw_fft(int N, fftw_complex* in, fftw_complex* out, int direction)
 *                                                        src/mhealth/fft/_fftw_binder.py:11-17
 *
 * which the spectral features of this engine replace with an on-chip rFFT inside
 * the fused kernel (no separate FFT call, no plan).
 *
 * Conventions (all entry points):
 *   - plain C types only; no torch / HIP C++ types in any signature;
 *   - caller owns every buffer, scratch included: nothing is allocated inside. Entry
 *     points that need device scratch take a caller-owned `workspace` (device memory,
 *     256-B aligned) of `workspace_bytes`, sized by the matching mhf_*_workspace() query
 *     (the reference's FFI is caller-owned buffers too,
 *     src/mhealth/fft/_fftw_binder.py:11-17); a workspace that is too small fails the call
 *     with MHF_EINVAL before any launch. The workspace must stay untouched until the
 *     stream reaches the end of the call;
 *   - GPU entry points are stream-ordered and asynchronous (no implicit sync),
 *     `hip_stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - return 0 on success, a negative MHF_E* code on error; the message of the
 *     last error on the calling thread is available from mhf_last_error().
 */
#ifndef MHFEAT_H
#define MHFEAT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHF_ABI_VERSION 7

/* The library is built with -fvisibility=hidden; only these entry points are exported. */
#if defined(__GNUC__) || defined(__clang__)
#define MHF_API __attribute__((visibility("default")))
#else
#define MHF_API
#endif

/* Error codes. */
#define MHF_OK 0
#define MHF_EINVAL (-1)      /* bad argument (sizes, strides, feature ids, dtype) */
#define MHF_EUNSUPPORTED (-2) /* valid request the engine has no kernel for        */
#define MHF_EDEVICE (-3)     /* HIP runtime error (launch failure, no device)      */

/* Per-window features. Each id names one reference callable and its exact
 * numerics. Values are written as float64 (the
 * reference's `np.zeros((nw, *shape))`, windows.py:89) or float32 on request. */
typedef enum mhf_feature {
    MHF_MEAN = 0,             /* np.mean passed to rolling_apply (stats.mean, stats.py:157): row 0 =
                                 numba array_mean (fp32), rows>=1 = parfor mean_parallel_impl
                                 (fp32 sum, fp64 quotient)                                         */
    MHF_MEAN32 = 1,           /* np.mean inside a feature function: fp32 on every row              */
    MHF_VAR = 2,              /* np.var passed directly: row 0 = numba array_var (fp32 result),
                                 rows>=1 = parfor var_parallel_impl (fp64 two-pass; the register
                                 tiles: within 3.6e-7, bit-exact with MHF_NUMERICS_EXACT_VAR) */
    MHF_VAR32 = 3,            /* np.var inside a feature: timedom.hjorth_activity (timedom.py:81) */
    MHF_STD = 4,              /* np.std passed directly: row 0 fp32, rows>=1 sqrt(fp64 var)        */
    MHF_STD32 = 5,            /* np.std inside a feature                                          */
    MHF_SKEWNESS = 6,         /* stats.skewness (stats.py:97-110)                                 */
    MHF_KURTOSIS = 7,         /* stats.kurtosis (stats.py:113-126)                                */
    MHF_KURTOSIS_EXCESS = 8,  /* stats.kurtosis_excess (stats.py:129-139)                         */
    MHF_RMS = 9,              /* sqrt(mean(square(x))): hrv.rmssd form (hrv.py:138-146)           */
    MHF_ZERO_CROSSINGS = 10,  /* timedom.zero_crossing_count(x, th) (timedom.py:34-64)            */
    MHF_PEAK_COUNT = 11,      /* len(qrs.nb_find_peaks(x)) (qrs.py:215-220)                       */
    MHF_DRANGE = 12,          /* stats.drange (stats.py:12-45)                                    */
    MHF_LINE_LENGTH = 13,     /* timedom.line_length (timedom.py:67-78)                           */
    MHF_BAND_POWER = 14,      /* hrv.power_band(psd(x), freqs, lo, hi) (hrv.py:173-179)           */
    MHF_REL_BAND_POWER = 15,  /* hrv.relative_power_band (hrv.py:192-198)                         */
    MHF_SPECTRAL_ENTROPY = 16,/* information.entropy(psd(x)) (information.py:10-20)               */
    MHF_DOMINANT_FREQ = 17,   /* density.peak_frequency(psd(x), freqs, lo, hi) (density.py:17-32) */
    /* §8f N3: more per-window features (generic kernel; serial numerics on every row) */
    MHF_COEFF_VAR = 18,       /* stats.coeff_var = std32 / mean32 (stats.py:142-153)             */
    MHF_HJORTH_MOBILITY = 19, /* timedom.hjorth_mobility (timedom.py:97-112): sqrt(var(g)/var(x)),
                                 g = gradient(x) (timedom.py:11-31) in fp64                       */
    MHF_HJORTH_COMPLEXITY = 20,/* timedom.hjorth_complexity (timedom.py:133-148)                  */
    /* §8f N4: HRV time-domain metrics of an RR-interval window (heart/hrv.py:111-266);
     * d = np.diff(window), n = W - 1 */
    MHF_RMSSD = 21,           /* hrv.rmssd: sqrt(mean(square(d))) (hrv.py:138-146)                */
    MHF_SDSD = 22,            /* hrv.sdsd: std(d) (hrv.py:160-169)                                */
    MHF_SSD = 23,             /* hrv.ssd: sum(d) (hrv.py:149-157)                                 */
    MHF_PNNX = 24,            /* hrv.pnn50 / pnnx: #(|d| > pnn_threshold) / n (hrv.py:111-135)   */
    MHF_CSI_SD1 = 25,         /* hrv.csi_sd1: csi_factor * std(d) (hrv.py:207-217)                */
    MHF_CSI_SD2 = 26,         /* hrv.csi_sd2: csi_factor * std(x[1:] + x[:-1]) (hrv.py:220-231)   */
    MHF_LORENZ_CSI = 27,      /* hrv.lorenz_csi: sd1 / sd2 (hrv.py:234-243)                       */
    MHF_LORENZ_CVI = 28,      /* hrv.lorenz_cvi: log10(sd1 * sd2) (hrv.py:246-250)                */
    MHF_LORENZ_MCSI = 29,     /* hrv.lorenz_mcsi: sd1**2 / sd2 (hrv.py:253-266)                   */
    /* np.min / np.max passed directly (stats.dmin / stats.dmax, stats.py:161-162): row 0 =
     * numba array_min/max (a NaN is returned at once), rows >= 1 = parfor
     * min/max_parallel_impl (from +-inf with builtin min/max: NaN skipped) */
    MHF_MIN = 30,
    MHF_MAX = 31,
    /* np.median passed directly (stats.median, stats.py:158): numba's median_impl
     * (numba/np/arraymath.py:1371-1398): quickselect on a copy (median-of-three pivot,
     * `<` comparisons, :1283-1346); even W: f64(f32(a + b)) / 2. Fixed windows of up to
     * 16384 / channels samples (keys in LDS); indexed windows past that are sorted in the
     * caller's workspace (mhf_indexed_window_features) */
    MHF_MEDIAN = 32,
    /* information.entropy(x) passed to rolling_apply (information.py:10-20) on the window's
     * own samples: p = x / sum(x) + 1e-30, -sum(p ln p), fp32 (logf: device libm) */
    MHF_ENTROPY = 33,
    /* §8f N3 order statistics (order_kernel; windows up to 16384 samples x channels):
     * stats.interquartile_range = np.percentile(x, [75, 25]) difference (stats.py:48-59),
     * stats.mode's jit version (stats.py:73-94: sort, first run counted one short, ties to
     * the earlier run), np.percentile(x, q) with q = mhf_params.percentile_q (numba
     * _collect_percentiles: NaN -> NaN, linear interpolation in float64) */
    MHF_IQR = 34,
    MHF_MODE = 35,
    MHF_PERCENTILE = 36,
    /* information.sampen(x, mm, r, sd) (information.py:23-113): m = mhf_params.sampen_m,
     * r = sampen_r, sd = sampen_sd (NaN = None: the window's own np.std) */
    MHF_SAMPEN = 37,
    /* §8f N3 recurrence quantification of the window's recurrence matrix
     * r = rqa.rq(x, radius) (rqa.py:9-28: |x_i - x_j| <= radius, fp32 differences), radius =
     * mhf_params.rqa_radius: rqa.recurrence_rate(r), rqa.determinism(r), rqa.laminarity(r),
     * rqa.length_entropy(r, minlen) with minlen = mhf_params.rqa_minlen (rqa.py:49-187;
     * lines of the full window length are dropped from the histogram, as the reference's
     * _dlen_counts writes them past its array) */
    MHF_RQA_RR = 38,
    MHF_RQA_DET = 39,
    MHF_RQA_LAM = 40,
    MHF_RQA_ENT = 41,
    MHF_NUM_FEATURES = 42
} mhf_feature;

/* Feature parameters (one set per call).
 * psd(x) is the one-sided periodogram |X_k|^2/(fs*W), bins 1..ceil(W/2)-1 doubled
 * (== scipy.signal.periodogram(x, fs, 'boxcar', detrend=False)); freqs are
 * numpy.fft.rfftfreq(W, 1/fs). A bound given as NaN means "None" in the reference
 * (power_band: min/max(freqs); peak_frequency: 0 / len(psd)). */
typedef struct mhf_params {
    double fs;              /* sampling frequency, Hz (> 0 when a spectral feature is asked) */
    double band_lo;         /* power_band / relative_power_band: lo <= f <= hi (inclusive)  */
    double band_hi;
    double dom_lo;          /* peak_frequency: first bin with lo <= f ..                    */
    double dom_hi;          /* .. up to (excluding) the first bin with hi <= f              */
    double zc_threshold;    /* zero_crossing_count th (default 0)                           */
    double pnn_threshold;   /* MHF_PNNX: x * 1e6 / td_factor(unit) (pnn50: 50 for 'ms')     */
    double csi_factor;      /* MHF_CSI_* / MHF_LORENZ_*: the factor argument (1/sqrt(2))    */
    double percentile_q;    /* MHF_PERCENTILE: q in [0, 100]                                */
    double sampen_m;        /* MHF_SAMPEN: template length mm (integer >= 1; default 2)     */
    double sampen_r;        /* MHF_SAMPEN: tolerance r as a fraction of sd (default 0.2)    */
    double sampen_sd;       /* MHF_SAMPEN: sd, NaN = None (the window's np.std)             */
    double rqa_radius;      /* MHF_RQA_*: rq radius (default 0)                             */
    double rqa_minlen;      /* MHF_RQA_ENT: length_entropy minlen (integer >= 1; default 2) */
} mhf_params;

#define MHF_OUT_F64 0
#define MHF_OUT_F32 1

/* Numerics selector: the numba-faithful mode, optionally for 2-D input.
 *
 * MHF_NUMERICS_BLOCK(c), c >= 1: the record is a C-order 2-D (N, c) array passed flat
 * (channels = 1, N * c samples) and every window is the (wsize / c, c) block
 * arr[i*wstep : i*wstep + wsize] of loop_wrapper applied to it (windows.py:68-91; wsize
 * and wstep here are the flat counts, rows * c). numba reduces such a block element by
 * element in C order, so np.mean / np.var / np.std / np.min / np.max / np.median /
 * np.percentile, drange, rms, coeff_var are the 1-D features of the flat block; the two
 * that index rows differ: skewness / kurtosis divide each term by len(x) = the number of
 * ROWS (stats.py:107,123) and line_length sums |np.diff| along the last axis, i.e. within
 * rows (timedom.py:78; 0 for c = 1). Features that fail on 2-D blocks in the reference (zero
 * crossings, peaks, spectral, Hjorth mobility/complexity, HRV, entropy, mode, sampen,
 * RQA) are rejected with MHF_EUNSUPPORTED.
 *
 * Rows >= 1 of np.var / np.std (numba's var_parallel_impl, an fp64 two-pass about the fp64
 * mean): by default the register-tile kernels (W in {128, 256}, and
 * the fixed-window tile of any W <= 288) derive them from the fp32-deviation sum they already keep for np.var's row 0 / skewness
 * / kurtosis, within 3.6e-7 relative of the reference (proof: DESIGN.md §2; windows whose
 * sums leave the fp32 normal range, or whose offset-to-spread ratio the bound does not
 * cover, are recomputed exactly). OR-ing MHF_NUMERICS_EXACT_VAR
 * into `numerics` replays the reference's fp64 chain bit for bit there as well (+4 VALU
 * per sample). Every other feature, and every other kernel, is unaffected by the flag. */
#define MHF_NUMERICS_REFERENCE 0
#define MHF_NUMERICS_EXACT_VAR 1
#define MHF_NUMERICS_BLOCK(c) ((int32_t)(c) << 8)

/* Number of windows: max(0, 1 + (n_samples - wsize) // wstep) with floor
 * division, exactly loop_wrapper's `nw` (windows.py:86). Returns -1 on bad args. */
MHF_API int64_t mhf_num_windows(int64_t n_samples, int64_t wsize, int64_t wstep);

/* Fused sliding-window features on the GPU.
 *
 *   x             device pointer, float32 samples. Sample t of channel c is
 *                 x[c * ch_stride + t * sample_stride] (AoS (N,3): ch_stride=1,
 *                 sample_stride=3; a contiguous 1-D signal: channels=1, sample_stride=1).
 *   n_samples     samples per channel.
 *   wsize, wstep  window length and step (both >= 1).
 *   first_window  global index of the first window to compute (window i covers
 *                 samples [i*wstep, i*wstep + wsize)). Global window 0 gets the
 *                 reference's serial row-0 numerics (windows.py:87) — this keeps a
 *                 sharded run bit-identical to a single-device run.
 *   n_windows     windows to compute; first_window + n_windows <= mhf_num_windows().
 *   features      host array of n_features mhf_feature ids (any order, repeats ok).
 *   out           device pointer. Value of feature j of channel c for window
 *                 first_window+i is written at out[(c * n_features + j) * out_ld + i],
 *                 float64 (MHF_OUT_F64) or float32 (MHF_OUT_F32). out_ld >= n_windows.
 *   numerics      MHF_NUMERICS_REFERENCE, or MHF_NUMERICS_BLOCK(c) for 2-D input; either
 *                 OR MHF_NUMERICS_EXACT_VAR (bit-exact rows >= 1 of np.var / np.std).
 *   hip_stream    hipStream_t (void*), NULL = null stream.
 */
MHF_API int mhf_window_features(const float* x, int64_t n_samples, int32_t channels,
                        int64_t ch_stride, int64_t sample_stride,
                        int64_t wsize, int64_t wstep,
                        int64_t first_window, int64_t n_windows,
                        const int32_t* features, int32_t n_features,
                        const mhf_params* params, int32_t numerics,
                        int32_t out_dtype, void* out, int64_t out_ld,
                        void* hip_stream);

/* The same for float64 samples (a float64 numpy / pandas record): numba types every
 * reduction from the input dtype, so each feature is the reference function in fp64
 * (sequential fp64 sums; row 0 and the prange rows agree). Lane features (moments, time
 * domain, Hjorth, HRV, min/max, entropy; MHF_NUMERICS_BLOCK allowed) and the order
 * statistics (median, percentile, IQR, mode: numba's selections and sort on the float64
 * values, windows up to 8192 samples x channels), sample entropy and RQA (fp64
 * differences), and the spectral features from an fp64 transform of the float64 window
 * (the reference transforms a.astype(complex128), fft/_fft.py:18-28: radix-2 FFT for a
 * power-of-two W, an exact-phase DFT otherwise; fp64 periodogram, sums, log, arg max). */
MHF_API int mhf_window_features_f64(const double* x, int64_t n_samples, int32_t channels,
                                    int64_t ch_stride, int64_t sample_stride,
                                    int64_t wsize, int64_t wstep,
                                    int64_t first_window, int64_t n_windows,
                                    const int32_t* features, int32_t n_features,
                                    const mhf_params* params, int32_t numerics,
                                    int32_t out_dtype, void* out, int64_t out_ld,
                                    void* hip_stream);

/* Bytes of HBM the call reads and writes by algorithm (input read once per
 * distinct sample + the output rows), for roofline accounting. */
MHF_API int64_t mhf_algorithmic_bytes(int64_t n_samples, int32_t channels, int64_t wsize,
                              int64_t wstep, int64_t n_windows, int32_t n_features,
                              int32_t out_dtype);

/* Name of the kernel variant mhf_window_features() would launch for these
 * arguments (for profiling / tests), or NULL if the request is invalid. */
MHF_API const char* mhf_plan_name(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                          int64_t wsize, int64_t wstep, const int32_t* features,
                          int32_t n_features, int32_t out_dtype);
/* The same for mhf_window_features_f64 (a 16-B aligned record assumed). */
MHF_API const char* mhf_plan_name_f64(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                                      int64_t wsize, int64_t wstep, const int32_t* features,
                                      int32_t n_features, int32_t out_dtype);

/* Indexed (variable-length) windows on the GPU: window i covers samples
 * [starts[i], ends[i]) of every channel (device int64 arrays, e.g. from
 * mhf_window_bounds). Replaces the compiled loop of indices_rolling_apply /
 * nonuniform_rolling_apply (src/mhealth/util/windows.py:122-159, 181-249): a serial
 * @jit loop, so EVERY window gets the serial numerics (np.mean / np.var / np.std as
 * numba's array_mean / array_var / array_std, i.e. MHF_MEAN == MHF_MEAN32 here), and a
 * window with ends[i] - starts[i] < min_len, or empty, is NaN for every feature
 * (the reference raises ZeroDivisionError on an empty window with min_len <= 0).
 * Moment, time-domain and order-statistic features (spectral ids: MHF_EUNSUPPORTED).
 * Output layout as mhf_window_features; stream-ordered, asynchronous — except that when
 * order statistics, sampen or RQA are requested the call reads the longest kept window
 * length back to the host once (the launch shapes of those kernels depend on it; the
 * value passes through the first 8 bytes of the workspace): order statistics of windows
 * longer than the LDS capacity (16384 / channels keys) are sorted in the workspace (up to
 * 2^20 samples per window, as many windows at a time as it holds); sampen / RQA windows
 * past their LDS capacity fail the call with MHF_EUNSUPPORTED (no window is ever written
 * as NaN for being long). workspace: mhf_indexed_workspace(max_window_len, ...) bytes,
 * max_window_len >= the longest window (0 bytes are enough for a call without order
 * statistics / sampen / RQA). */
MHF_API int mhf_indexed_window_features(const float* x, int64_t n_samples, int32_t channels,
                                int64_t ch_stride, int64_t sample_stride,
                                const int64_t* starts, const int64_t* ends,
                                int64_t n_windows, int64_t min_len,
                                const int32_t* features, int32_t n_features,
                                const mhf_params* params, int32_t out_dtype, void* out,
                                int64_t out_ld, void* workspace, int64_t workspace_bytes,
                                void* hip_stream);
/* Name of the kernel variants an indexed call would launch ("tile_idx": the register tile,
 * the default for float32 AoS / 1-D records and the two-pass features; "moments_indexed":
 * the lane walk, for the other features (or with MHF_NO_TILE_IDX=1 and
 * MHF_DIAGNOSTICS=1); "moments_indexed_f64"; "+order/pairwise"), or NULL
 * if invalid. dtype: MHF_DTYPE_F32 / F64 samples (a 4-B aligned record assumed). */
MHF_API const char* mhf_plan_name_indexed(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                                          const int32_t* features, int32_t n_features,
                                          int32_t dtype);
/* Workspace of an indexed call whose windows hold at most max_window_len samples, for
 * `dtype` (MHF_DTYPE_F32 / F64) samples and these features: the 8-B max-length slot when
 * order statistics / sampen / RQA are requested, plus room to sort up to 256 windows past
 * the LDS capacity at once when max_window_len exceeds it (fewer fit a smaller workspace,
 * at least one must). 0 when no feature needs scratch. -1 on bad arguments. */
MHF_API int64_t mhf_indexed_workspace(int64_t max_window_len, int32_t channels, int32_t dtype,
                                      const int32_t* features, int32_t n_features);

/* The same for float64 samples (numba types the serial @jit function per dtype): the lane
 * features in fp64 and the order statistics on 64-bit keys (8192 / channels keys in LDS,
 * longer windows in global scratch, as above), sample entropy and RQA; spectral ids return
 * MHF_EUNSUPPORTED. Replaces indices_rolling_apply on a float64 record
 * (src/mhealth/util/windows.py:134-157, out dtype = the record's). */
MHF_API int mhf_indexed_window_features_f64(const double* x, int64_t n_samples, int32_t channels,
                                            int64_t ch_stride, int64_t sample_stride,
                                            const int64_t* starts, const int64_t* ends,
                                            int64_t n_windows, int64_t min_len,
                                            const int32_t* features, int32_t n_features,
                                            const mhf_params* params, int32_t out_dtype,
                                            void* out, int64_t out_ld, void* workspace,
                                            int64_t workspace_bytes, void* hip_stream);

/* mhf_window_bounds `mode` bits: which of numpy's bounds are float64. */
enum {
    MHF_BOUNDS_FLOAT_STARTS = 1,  /* wstep is a float: np.arange yields float64 starts   */
    MHF_BOUNDS_FLOAT_ENDS = 2     /* starts or wsize is a float: ends = starts + wsize is
                                     f64, and so (np.concatenate) are both searched keys */
};

/* get_indices (src/mhealth/util/windows.py:162-178) on the GPU: window i starts at
 * t0 + i*wstep and ends wsize later; starts[i] / ends[i] = np.searchsorted(index, ., 'left')
 * over the sorted device int64 `index` (datetime64 / int64 ticks) of length n. Integer
 * bounds are exact int64 arithmetic; float bounds reproduce numpy's arange
 * (t0 + i*((t0 + wstep) - t0)) and its float64 comparison against the int64 index.
 * Integer fields (t0_i, wstep_i, wsize_i) are read for integer bounds, float fields for
 * float ones (mode FLOAT_STARTS requires FLOAT_ENDS). n_windows =
 * len(np.arange(index[0], index[-1], wstep)) is computed by the caller. */
MHF_API int mhf_window_bounds(const int64_t* index, int64_t n, int64_t n_windows,
                              int32_t mode, int64_t t0_i, int64_t wstep_i, int64_t wsize_i,
                              double t0_f, double wstep_f, double wsize_f,
                              int64_t* starts, int64_t* ends, void* hip_stream);

/* scipy.signal.filtfilt(b, a, x) of every channel (src/mhealth/generic/filters.py:8-35,
 * `butterworth`; the per-axis loops of inertial/accelerometer.py:78-183): padtype 'odd',
 * padlen = 3 * max(na, nb), initial conditions lfilter_zi(b, a) scaled by the first
 * input of each pass, DF2T lfilter in fp64 (forward, then backward). x is float32
 * (x[t * sample_stride + c * ch_stride], n_samples > padlen), out float64 / float32 at
 * out[t * out_sample_stride + c * out_ch_stride]. Up to 17 taps (Butterworth bandpass
 * order 8). zi: lfilter_zi(b, a) (max(na, nb) - 1 values) or NULL to solve it on the
 * device; that system is ill-conditioned for low cutoffs (cond ~1e8 at 0.02 x Nyquist),
 * so pass the caller's own zi to reproduce its filtfilt to rounding. Stream-ordered;
 * workspace: mhf_filtfilt_workspace(n_samples, channels, nb, na) bytes (the fp64 forward
 * pass, 8 * channels * (n_samples + 2 padlen)). */
MHF_API int mhf_filtfilt(const float* x, int64_t n_samples, int32_t channels, int64_t ch_stride,
                         int64_t sample_stride, const double* b, int32_t nb, const double* a,
                         int32_t na, const double* zi, int32_t out_dtype, void* out,
                         int64_t out_ch_stride, int64_t out_sample_stride, void* workspace,
                         int64_t workspace_bytes, void* hip_stream);
MHF_API int64_t mhf_filtfilt_workspace(int64_t n_samples, int32_t channels, int32_t nb, int32_t na);

/* sqrt(x^2 + y^2 + z^2) per sample of an AoS (n, 3) float32 record
 * (inertial/accelerometer.py:198-225, `magnitude` on float32 arrays: fp32 squares, fp32
 * sums left to right, fp32 sqrt). out: n float32. */
MHF_API int mhf_magnitude(const float* x, int64_t n_samples, int64_t sample_stride,
                          int64_t ch_stride, float* out, void* hip_stream);

/* ---- per-sample helpers of the drop-in modules -----------------------------------------
 * x / y / z: device arrays of n samples (element stride `stride`), dtype MHF_DTYPE_F32 or
 * MHF_DTYPE_F64 (numba types each expression from the input dtype; restated per kernel in
 * pymhealth_amd/csrc/elementwise.hip). Stream-ordered on hip_stream. */
#define MHF_ROLL 0
#define MHF_PITCH 1
/* accelerometer.roll(y, z) = arctan2(y, z) * 180 / pi and pitch(x, y, z) =
 * arctan2(-x, sqrt(y*y + z*z)) * 180 / pi (inertial/accelerometer.py:13-75; x unused for
 * MHF_ROLL). float32 input: the fp32 arctan2 widened to float64 before the scaling, as
 * numba computes it. out: n float64. */
MHF_API int mhf_orientation(int32_t which, const void* x, const void* y, const void* z,
                            int64_t n, int64_t stride, int32_t dtype, double* out,
                            void* hip_stream);
/* timedom.gradient(x) (generic/timedom.py:11-31): out n float64 (n >= 2). */
MHF_API int mhf_gradient(const void* x, int64_t n, int64_t stride, int32_t dtype, double* out,
                         void* hip_stream);
/* timedom.zero_crossings(x, th) (generic/timedom.py:34-48): out[i] = pos(x[i]) xor
 * pos(x[i+1]), i < n - 1, pos(v) = v > 0 unless |v| <= th. out: n - 1 bytes (0 / 1). */
MHF_API int mhf_zero_crossings(const void* x, int64_t n, int64_t stride, int32_t dtype,
                               double th, uint8_t* out, void* hip_stream);
/* accelerometer.magnitude_dot(x, y, z) = sqrt(x.x + y.y + z.z) (accelerometer.py:236-259):
 * one value of the input dtype at device pointer out. Each dot is an fp64 sum over per-block
 * partials (in the workspace: mhf_magnitude_dot_workspace(n) bytes = 3 x min(1024,
 * ceil(n / 256)) doubles), combined in block order (deterministic), rounded to the input
 * dtype as BLAS returns it. */
MHF_API int mhf_magnitude_dot(const void* x, const void* y, const void* z, int64_t n,
                              int64_t stride, int32_t dtype, void* out, void* workspace,
                              int64_t workspace_bytes, void* hip_stream);
MHF_API int64_t mhf_magnitude_dot_workspace(int64_t n);

/* qrs.find_peaks(x) / nb_find_peaks(x) (heart/qrs.py:200-220): the ascending indices i of
 * strict local maxima, x[i] > x[i-1] and x[i] > x[i+1], 1 <= i <= n-2. out: room for
 * (n - 1) / 2 int64 indices; workspace: mhf_find_peaks_workspace(n) bytes of device memory,
 * whose int64 at index ceil(n / 1024) holds the number of peaks when the stream reaches
 * the end of the call. */
MHF_API int64_t mhf_find_peaks_workspace(int64_t n);
MHF_API int mhf_find_peaks(const void* x, int64_t n, int64_t stride, int32_t dtype, int64_t* out,
                           int64_t* workspace, void* hip_stream);
/* qrs.find_peaks(x, comp) with the comparison ufunc `comp` (qrs.py:200-212: i with
 * comp(x[i], x[i-1]) and comp(x[i], x[i+1])): np.greater / greater_equal / less /
 * less_equal. Same out / workspace contract as mhf_find_peaks (which is comp = np.greater);
 * out needs room for n - 2 indices for the non-strict comparisons. */
#define MHF_CMP_GREATER 0
#define MHF_CMP_GREATER_EQUAL 1
#define MHF_CMP_LESS 2
#define MHF_CMP_LESS_EQUAL 3
MHF_API int mhf_find_peaks_cmp(const void* x, int64_t n, int64_t stride, int32_t dtype, int32_t comp,
                               int64_t* out, int64_t* workspace, void* hip_stream);

/* ---- PSD-level feature functions on caller-computed spectra --------------------------
 * The reference applies these to ONE 1-D psd (or any array, for entropy) that the user
 * computed; mhf_psd_features() evaluates them on every row of a
 * (rows, bins) device array, with numba's sequential reductions in the array's dtype
 * (float32 or float64), so the sums are the reference's bit for bit (entropy: last-bit
 * libm log differences). Values are written as float64 at out[j * out_ld + row]. */
typedef enum mhf_psd_op {
    MHF_PSD_POWER_BAND = 0,         /* hrv.power_band(psd, freqs, lower, upper): sum |psd| over
                                       lower <= freqs <= upper (hrv.py:173-179)               */
    MHF_PSD_REL_POWER_BAND = 1,     /* hrv.relative_power_band: power_band / sum |psd|
                                       (hrv.py:192-198); 0/0 gives NaN (reference raises)   */
    MHF_PSD_PEAK_FREQUENCY = 2,     /* density.peak_frequency(psd, freqs, lower, upper): freqs of
                                       the first arg max of psd[first_index(freqs, lower) :
                                       first_index(freqs, upper)] (density.py:9-32)           */
    MHF_PSD_PEAK_FREQUENCY_HRV = 3, /* hrv.peak_frequency (hrv.py:182-189) as written: the
                                       arg max of the masked psd indexes the unmasked freqs */
    MHF_PSD_ENTROPY = 4,            /* information.entropy(x): p = x / sum(x) + 1e-30,
                                       -sum(p ln p) (information.py:10-20)                    */
    MHF_PSD_NUM_OPS = 5
} mhf_psd_op;

#define MHF_DTYPE_F32 0
#define MHF_DTYPE_F64 1
#define MHF_DTYPE_I32 2   /* mhf_minmax only */
#define MHF_DTYPE_I64 3   /* mhf_minmax only */

/* stats.minmax(x) (generic/stats.py:12-32) of the n elements x[i * stride] (x.ravel()):
 * out[0] = minimum, out[1] = maximum, in the input dtype (F32 / F64 / I32 / I64), at device
 * pointer out. The reference's sequential rule: start from x[0], replace only on a strict
 * < / > — so a NaN x[0] is both answers, later NaN never win, and among equal values
 * (+0 / -0) the first occurrence stays. n >= 1. Per-block partials in the workspace:
 * mhf_minmax_workspace(n, dtype) bytes (min(1024, ceil(n / 256)) entries). */
MHF_API int mhf_minmax(const void* x, int64_t n, int64_t stride, int32_t dtype, void* out,
                       void* workspace, int64_t workspace_bytes, void* hip_stream);
MHF_API int64_t mhf_minmax_workspace(int64_t n, int32_t dtype);

/* Complex FFT of `batch` contiguous rows of n complex128 values (interleaved re, im):
 * replaces the reference's FFTW binding
 *     void fftw_fft(int N, fftw_complex* in, fftw_complex* out, int direction)
 *                                            src/mhealth/fft/_fftw_binder.py:11-17
 * with direction MHF_FFT_FORWARD (-1, FFTW_FORWARD: X_k = sum x_j exp(-2 pi i jk / n)) or
 * MHF_FFT_BACKWARD (+1, unnormalised), every output value multiplied by `scale` (1 for
 * mhealth.fft.fft, 1 / n for ifft, fft/_fft.py:18-48). Any n >= 1: powers of two by
 * radix-2 passes (in LDS up to 4096 points, one block per row; global passes beyond),
 * other n by Bluestein's chirp-z transform over a power of two >= 2n - 1. fp64 throughout,
 * twiddles from sincospi. in and out may be the same buffer. Work buffers (twiddles,
 * the global passes' copy, Bluestein's padded rows) live in the workspace:
 * mhf_fft_workspace(n, batch) bytes. */
#define MHF_FFT_FORWARD (-1)
#define MHF_FFT_BACKWARD 1
MHF_API int mhf_fft(const double* in, double* out, int64_t n, int64_t batch, int32_t direction,
                    double scale, void* workspace, int64_t workspace_bytes, void* hip_stream);
MHF_API int64_t mhf_fft_workspace(int64_t n, int64_t batch);

/* PSD-level features of every row of `psd` (device, rows x bins, element (r, k) at
 * psd[r * row_stride + k], dtype MHF_DTYPE_F32 / F64) against the device array `freqs`
 * (bins values, its own dtype; may be NULL when only MHF_PSD_ENTROPY is asked).
 * lower / upper: NaN means None (band functions: np.min / np.max(freqs); density
 * peak frequency: 0 / len(psd)). An empty arg-max range gives NaN (the reference raises
 * ValueError). ops: n_ops (<= 20) mhf_psd_op ids; out: device float64, out_ld >= rows.
 * Stream-ordered, asynchronous. */
MHF_API int mhf_psd_features(const void* psd, int32_t psd_dtype, int64_t rows, int64_t bins,
                             int64_t row_stride, const void* freqs, int32_t freqs_dtype,
                             const int32_t* ops, int32_t n_ops, double lower, double upper,
                             double* out, int64_t out_ld, void* hip_stream);

MHF_API const char* mhf_last_error(void);
MHF_API int mhf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MHFEAT_H */
