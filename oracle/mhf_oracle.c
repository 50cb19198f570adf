/*
 * mhf_oracle.c — CPU restatement of pymhealth's windowed-feature hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity oracle (and the bench's
 * `cpu_baseline` leg, kind "port"). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load it; the product (pymhealth_amd, libmhfeat.so)
 * never links or calls it.
 *
 * Pinned against the reference's own outputs: the tests/golden/ fixtures (.npz) were made by
 * running /root/reference/src/mhealth under numba 0.54.1 (tests/golden/make_golden.py),
 * and tests/test_oracle_golden.py checks this file against every one of them.
 *
 * Each model restates a reference function and the numba 0.54.1 lowering that
 * sets its arithmetic:
 *   loop / nw / row-0 rule ... src/mhealth/util/windows.py:68-91
 *   mean ..................... numba/np/arraymath.py:405-418 (array_mean)
 *   var (row 0, in features).. numba/np/arraymath.py:423-438 (array_var)
 *   var (rows >= 1, direct) .. numba/parfors/parfor.py:314-340 (var_parallel_impl)
 *   std ...................... numba/np/arraymath.py:441-447, parfor.py:342-345
 *   skewness / kurtosis ...... src/mhealth/generic/stats.py:97-139
 *   drange ................... src/mhealth/generic/stats.py:12-45
 *   np.min / np.max .......... numba/np/arraymath.py:471-630, parfor.py:124-168
 *                              (stats.dmin / dmax, src/mhealth/generic/stats.py:161-162)
 *   np.median ................ numba/np/arraymath.py:1283-1398 (quickselect; stats.median)
 *   np.percentile / IQR ...... numba/np/arraymath.py:1402-1515 (stats.py:48-59,163)
 *   stats.mode ............... src/mhealth/generic/stats.py:73-94 + numba/misc/quicksort.py
 *   information.sampen ....... src/mhealth/generic/information.py:23-113
 *   rqa features ............. src/mhealth/generic/rqa.py:9-187
 *   zero_crossing_count ...... src/mhealth/generic/timedom.py:34-64
 *   line_length .............. src/mhealth/generic/timedom.py:67-78
 *   rms ...................... src/mhealth/heart/hrv.py:138-146 (without np.diff)
 *   peak count ............... src/mhealth/heart/qrs.py:215-220
 *   power_band / relative .... src/mhealth/heart/hrv.py:173-198
 *   entropy .................. src/mhealth/generic/information.py:10-20
 *   peak_frequency ........... src/mhealth/generic/frequency/density.py:9-32
 *   coeff_var ................ src/mhealth/generic/stats.py:142-153
 *   hjorth mobility/complexity src/mhealth/generic/timedom.py:11-31 (gradient), 97-169
 *   rmssd/sdsd/ssd/pnnx/csi .. src/mhealth/heart/hrv.py:111-266
 * The FFT has no runnable reference here (FFTW binder unbuildable, numpy.fft
 * fallback, src/mhealth/fft/__init__.py:3-7); this oracle uses an fp64 FFT, checked
 * against numpy.fft (pocketfft, fp64) rows in the fixtures.
 *
 * Build: `make -C oracle` (gcc, -ffp-contract=off so fp32 steps round exactly as
 * numba's do; OpenMP over windows).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/mhfeat.h"

/* ------------------------------------------------------------------ helpers */
static int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}

int64_t mhf_oracle_num_windows(int64_t n, int64_t w, int64_t s) {
    if (w < 1 || s < 1 || n < 0) return -1;
    int64_t nw = 1 + floordiv(n - w, s);
    return nw > 0 ? nw : 0;
}

/* x > max(th, 0) evaluated in fp64 (numba compares the f32 sample against the f64
 * threshold, timedom.py:46-48) == x > t32 with t32 = th rounded toward -inf. */
float mhf_oracle_zc_threshold32(double th) {
    double t = th > 0.0 ? th : 0.0;
    float t32 = (float)t;
    if ((double)t32 > t) t32 = nextafterf(t32, -INFINITY);
    return t32;
}

/* numpy.fft.rfftfreq(W, 1/fs): val = 1.0/(n*d); arange(N) * val */
static double bin_freq(int64_t k, int64_t W, double fs) {
    double d = 1.0 / fs;
    double val = 1.0 / ((double)W * d);
    return (double)k * val;
}

/* -------------------------------------------------------------- fp64 r-DFT */
static void fft64_pow2(double* re, double* im, int64_t n) {
    /* iterative radix-2 DIT, bit reversal first */
    for (int64_t i = 1, j = 0; i < n; i++) {
        int64_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    for (int64_t len = 2; len <= n; len <<= 1) {
        int64_t h = len >> 1;
        for (int64_t k = 0; k < h; k++) {
            double ang = -2.0 * M_PI * (double)k / (double)len;
            double wr = cos(ang), wi = sin(ang);
            for (int64_t i = k; i < n; i += len) {
                double ur = re[i], ui = im[i];
                double vr = re[i + h] * wr - im[i + h] * wi;
                double vi = re[i + h] * wi + im[i + h] * wr;
                re[i] = ur + vr; im[i] = ui + vi;
                re[i + h] = ur - vr; im[i + h] = ui - vi;
            }
        }
    }
}

/* one-sided periodogram of one window (density scaling, boxcar) */
/* w: the window's samples as float64 (a float32 window widened exactly, or a float64
 * record's own values: the reference transforms a.astype(complex128), fft/_fft.py:18-28) */
static void periodogram64(const double* w, int64_t W, double fs, double* psd,
                          double* re, double* im) {
    int64_t nb = W / 2 + 1;
    if ((W & (W - 1)) == 0) {
        for (int64_t i = 0; i < W; i++) { re[i] = w[i]; im[i] = 0.0; }
        fft64_pow2(re, im, W);
    } else {
        for (int64_t k = 0; k < nb; k++) {
            double sr = 0.0, si = 0.0;
            for (int64_t t = 0; t < W; t++) {
                int64_t m = (k * t) % W;
                double ang = -2.0 * M_PI * (double)m / (double)W;
                sr += w[t] * cos(ang);
                si += w[t] * sin(ang);
            }
            re[k] = sr; im[k] = si;
        }
    }
    double scale = 1.0 / (fs * (double)W);
    for (int64_t k = 0; k < nb; k++) {
        double p = (re[k] * re[k] + im[k] * im[k]) * scale;
        int dbl = (W % 2) ? (k >= 1) : (k >= 1 && k < nb - 1);
        psd[k] = dbl ? 2.0 * p : p;
    }
}

/* ------------------------------------------------------------ the features */
typedef struct {
    double mean, mean32, var, std, var32, std32, skew, kurt, kurt_ex, rms, zc, peaks, drange, ll;
    double bp, rbp, ent, dom;
    double cv, hj_mob, hj_cmp;
    double rmssd, sdsd, ssd, pnnx, sd1, sd2, lcsi, lcvi, lmcsi;
    double vmin, vmax, median, entx, iqr, mode, pct, sampen, rqa_rr, rqa_det, rqa_lam, rqa_ent;
} win_out;

#define OT float
#define OS(n) n
#include "order_models.inc"
#undef OT
#undef OS
#define OT double
#define OS(n) n##64
#include "order_models.inc"
#undef OT
#undef OS

/* information.sampen(x, mm, r, sd) (src/mhealth/generic/information.py:23-113), restated
 * line by line (run / run1 / a / b arrays as the reference keeps them). sd NaN = None: the
 * window's own np.std (numba array_std, fp32). */
static double nb_sampen(const float* x, int64_t n, int64_t mm, double r, double sd) {
    int64_t n1 = n - 1;
    mm += 1;
    int64_t mm_dbld = 2 * mm;
    if (isnan(sd)) {
        float s = 0.0f;
        for (int64_t t = 0; t < n; t++) s = s + x[t];
        float m32 = (float)((double)s / (double)n);
        double ssd = 0.0;
        for (int64_t t = 0; t < n; t++) { float d = x[t] - m32; ssd = ssd + (double)(d * d); }
        float var32 = (float)(ssd / (double)n);
        sd = (double)(float)sqrt((double)var32);
    }
    r = r * sd;
    double* run = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double* run1 = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double* a = (double*)calloc((size_t)mm, sizeof(double));
    double* b = (double*)calloc((size_t)mm, sizeof(double));
    for (int64_t i = 0; i < n1; i++) {
        int64_t nj = n1 - i;
        for (int64_t jj = 0; jj < nj; jj++) {
            int64_t j = jj + i + 1;
            if ((double)fabsf(x[j] - x[i]) < r) {
                run[jj] = run1[jj] + 1;
                double m1 = (double)mm < run[jj] ? (double)mm : run[jj];
                for (int64_t m = 0; m < (int64_t)m1; m++) {
                    a[m] += 1;
                    if (j < n1) b[m] += 1;
                }
            } else {
                run[jj] = 0;
            }
        }
        for (int64_t j = 0; j < mm_dbld && j < n; j++) run1[j] = run[j];
        if (nj > mm_dbld - 1)
            for (int64_t j = mm_dbld; j < nj; j++) run1[j] = run[j];
    }
    for (int64_t m = mm - 1; m > 0; m--) b[m] = b[m - 1];
    b[0] = (double)n * (double)n1 / 2.0;
    double res = -log(a[mm - 1] / b[mm - 1]);
    free(run); free(run1); free(a); free(b);
    return res;
}

/* Recurrence quantification (src/mhealth/generic/rqa.py), restated literally on the
 * window's recurrence matrix r = rq(x, radius) (rqa.py:9-28): r[i][j] = |x_i - x_j| <= radius
 * with the fp32 difference compared in float64. */
static unsigned char* rqa_matrix(const float* x, int64_t n, double radius) {
    unsigned char* r = (unsigned char*)malloc((size_t)(n * n));
    for (int64_t i = 0; i < n; i++)
        for (int64_t j = 0; j < n; j++) r[i * n + j] = (double)fabsf(x[i] - x[j]) <= radius;
    return r;
}
/* recurrence_rate (rqa.py:49-60): np.sum(r) / (n * n) */
/* float64 records: the same walk with fp64 differences; sd = np.std of the float64 window
 * (numba array_std: fp64 mean, fp64 sum of squared deviations, sqrt) */
static double nb_sampen64(const double* x, int64_t n, int64_t mm, double r, double sd) {
    int64_t n1 = n - 1;
    mm += 1;
    int64_t mm_dbld = 2 * mm;
    if (isnan(sd)) {
        double s = 0.0;
        for (int64_t t = 0; t < n; t++) s = s + x[t];
        const double m = s / (double)n;
        double ssd = 0.0;
        for (int64_t t = 0; t < n; t++) { double d = x[t] - m; ssd = ssd + d * d; }
        sd = sqrt(ssd / (double)n);
    }
    r = r * sd;
    double* run = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double* run1 = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double* a = (double*)calloc((size_t)mm, sizeof(double));
    double* b = (double*)calloc((size_t)mm, sizeof(double));
    for (int64_t i = 0; i < n1; i++) {
        int64_t nj = n1 - i;
        for (int64_t jj = 0; jj < nj; jj++) {
            int64_t j = jj + i + 1;
            if (fabs(x[j] - x[i]) < r) {
                run[jj] = run1[jj] + 1;
                double m1 = (double)mm < run[jj] ? (double)mm : run[jj];
                for (int64_t m = 0; m < (int64_t)m1; m++) {
                    a[m] += 1;
                    if (j < n1) b[m] += 1;
                }
            } else {
                run[jj] = 0;
            }
        }
        for (int64_t j = 0; j < mm_dbld && j < n; j++) run1[j] = run[j];
        if (nj > mm_dbld - 1)
            for (int64_t j = mm_dbld; j < nj; j++) run1[j] = run[j];
    }
    for (int64_t m = mm - 1; m > 0; m--) b[m] = b[m - 1];
    b[0] = (double)n * (double)n1 / 2.0;
    double res = -log(a[mm - 1] / b[mm - 1]);
    free(run); free(run1); free(a); free(b);
    return res;
}
static unsigned char* rqa_matrix64(const double* x, int64_t n, double radius) {
    unsigned char* r = (unsigned char*)malloc((size_t)(n * n > 0 ? n * n : 1));
    for (int64_t i = 0; i < n; i++)
        for (int64_t j = 0; j < n; j++) r[i * n + j] = fabs(x[i] - x[j]) <= radius;
    return r;
}

static double rqa_rr(const unsigned char* r, int64_t n) {
    int64_t s = 0;
    for (int64_t k = 0; k < n * n; k++) s += r[k];
    return (double)s / (double)(n * n);
}
#define R_(i, j) r[(i) * n + (j)]
/* determinism (rqa.py:63-88) */
static double rqa_det(const unsigned char* r, int64_t n) {
    unsigned char* o = (unsigned char*)calloc((size_t)(n * n), 1);
    for (int64_t i = 1; i < n - 1; i++) {
        for (int64_t j = 1; j < n - 1; j++) o[i * n + j] = (R_(i, j) & R_(i - 1, j - 1)) | (R_(i, j) & R_(i + 1, j + 1));
        o[i * n + 0] = R_(i, 0) & R_(i + 1, 1);
        o[i * n + n - 1] = R_(i, n - 1) & R_(i - 1, n - 2);
    }
    for (int64_t j = 1; j < n - 1; j++) {
        o[0 * n + j] = R_(0, j) & R_(1, j + 1);
        o[(n - 1) * n + j] = R_(n - 1, j) & R_(n - 2, j - 1);
    }
    o[0] = R_(0, 0) & R_(1, 1);
    o[(n - 1) * n + n - 1] = R_(n - 1, n - 1) & R_(n - 2, n - 2);
    int64_t s = 0;
    for (int64_t k = 0; k < n * n; k++) s += o[k];
    free(o);
    return (double)s / (double)(n * n);
}
/* laminarity (rqa.py:91-111) */
static double rqa_lam(const unsigned char* r, int64_t n) {
    int64_t s = 0;
    for (int64_t i = 0; i < n; i++) {
        s += R_(i, 0) & R_(i, 1);
        s += R_(i, n - 1) & R_(i, n - 2);
        for (int64_t j = 1; j < n - 1; j++) s += (R_(i, j) & R_(i, j + 1)) | (R_(i, j) & R_(i, j - 1));
    }
    return (double)s / (double)(n * n);
}
/* length_entropy (rqa.py:156-187): diagonal_lengths (rqa.py:114-133) -> _dlen_counts ->
 * information.entropy. _dlen_counts' out[v] += 1 for v == N lands past its N-element array
 * (numba does not bounds-check); that count is lost, as here. */
static double rqa_ent(const unsigned char* r, int64_t n, int64_t minlen) {
    int32_t* o = (int32_t*)calloc((size_t)(n * n), sizeof(int32_t));
    for (int64_t i = 1; i < n; i++)
        for (int64_t j = 1; j < n; j++) {
            o[i * n + j] = (o[(i - 1) * n + j - 1] + 1) * (R_(i, j) & R_(i - 1, j - 1));
            if (o[i * n + j]) o[(i - 1) * n + j - 1] = 0;
        }
    int64_t* cnt = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t k = 0; k < n * n; k++) {
        int64_t v = (int64_t)o[k] + 1;
        if (v >= minlen) cnt[v] += 1;          /* cnt[n]: the out-of-bounds slot, dropped */
    }
    free(o);
    int64_t tot = 0;
    for (int64_t v = minlen; v < n; v++) tot += cnt[v];
    double e = 0.0;
    for (int64_t v = minlen; v < n; v++) {
        double q = (double)cnt[v] / (double)tot;
        q = q + 1e-30;
        e = e + q * log(q);
    }
    free(cnt);
    return -e;
}
#undef R_

#define BIT(f) ((uint64_t)1 << (f))
#define SPECTRAL_MASK (BIT(MHF_BAND_POWER) | BIT(MHF_REL_BAND_POWER) | \
                       BIT(MHF_SPECTRAL_ENTROPY) | BIT(MHF_DOMINANT_FREQ))
#define HJORTH_MASK (BIT(MHF_HJORTH_MOBILITY) | BIT(MHF_HJORTH_COMPLEXITY))
#define HRV_MASK (BIT(MHF_RMSSD) | BIT(MHF_SDSD) | BIT(MHF_SSD) | BIT(MHF_PNNX) | \
                  BIT(MHF_CSI_SD1) | BIT(MHF_CSI_SD2) | BIT(MHF_LORENZ_CSI) | \
                  BIT(MHF_LORENZ_CVI) | BIT(MHF_LORENZ_MCSI))

/* blk >= 1: the window is a C-order (W / blk, blk) block of a 2-D record (MHF_NUMERICS_BLOCK,
 * include/mhfeat.h): len(x) = W / blk rows in skewness / kurtosis (stats.py:107,123),
 * np.diff along the last axis in line_length (timedom.py:78); the rest reduce the block
 * element by element in C order, i.e. exactly as the flat window. */
static void moments(const float* w, int64_t W, int row0, float t32, win_out* o, int32_t blk) {
    /* mean: c (fp32) += x; c / size in fp64, cast to the fp32 return type */
    float c = 0.0f;
    for (int64_t i = 0; i < W; i++) c = c + w[i];
    float m32 = (float)((double)c / (double)W);
    double m64 = (double)c / (double)W; /* mean_parallel_impl: no cast back to fp32 */
    o->mean32 = (double)m32;
    o->mean = row0 ? (double)m32 : m64;

    /* array_var: ssd (fp64) += f32((x-m)*(x-m)); ssd / size -> fp32 */
    double ssd = 0.0;
    for (int64_t i = 0; i < W; i++) {
        float d = w[i] - m32;
        float q = d * d;
        ssd = ssd + (double)q;
    }
    float var32 = (float)(ssd / (double)W);
    float std32 = (float)sqrt((double)var32); /* var()**0.5 lowers to sqrt */
    o->var32 = (double)var32;
    o->std32 = (double)std32;

    /* var_parallel_impl: its in_arr.mean() is mean_parallel_impl too (fp64 mean of
     * the fp32 sum); fp64 deviations, fp64 result */
    double ssdp = 0.0;
    for (int64_t i = 0; i < W; i++) {
        double d = (double)w[i] - m64;
        ssdp = ssdp + d * d;
    }
    double varp = ssdp / (double)W;
    o->var = row0 ? (double)var32 : varp;
    o->std = row0 ? (double)std32 : sqrt(varp);

    /* skewness: np.sum(((x - mean)**3) / len(x)) / sd**3 */
    float Wf = (float)(blk > 0 ? W / blk : W);
    if (std32 == 0.0f) {
        o->skew = 0.0;
    } else {
        float s3 = 0.0f;
        for (int64_t i = 0; i < W; i++) {
            float d = w[i] - m32;
            float d3 = d * (d * d);
            s3 = s3 + d3 / Wf;
        }
        float sd3 = std32 * (std32 * std32);
        o->skew = (double)(s3 / sd3);
    }
    /* kurtosis: np.sum(((x - mean)**4) / len(x)) / v**2 */
    float kurt;
    if (var32 == 0.0f) {
        kurt = 0.0f;
    } else {
        float s4 = 0.0f;
        for (int64_t i = 0; i < W; i++) {
            float d = w[i] - m32;
            float q = d * d;
            float d4 = q * q;
            s4 = s4 + d4 / Wf;
        }
        kurt = s4 / (var32 * var32);
    }
    o->kurt = (double)kurt;
    o->kurt_ex = (double)kurt - 3.0;

    /* rms = sqrt(mean(square(x))) */
    float a = 0.0f;
    for (int64_t i = 0; i < W; i++) a = a + w[i] * w[i];
    float ma = (float)((double)a / (double)W);
    o->rms = (double)sqrtf(ma);

    /* zero crossings: pos = x > max(th,0); count pos[i] != pos[i+1] */
    int64_t zc = 0;
    for (int64_t i = 0; i + 1 < W; i++) zc += ((w[i] > t32) != (w[i + 1] > t32));
    o->zc = (double)zc;

    /* peaks: strict local maxima on [1, W-2] */
    int64_t pk = 0;
    for (int64_t i = 1; i + 1 < W; i++) pk += (w[i] > w[i - 1] && w[i] > w[i + 1]);
    o->peaks = (double)pk;

    /* drange = max - min (minmax loop; NaN only sticks at x[0]) */
    float mn = w[0], mx = w[0];
    for (int64_t i = 1; i < W; i++) {
        if (w[i] < mn) mn = w[i];
        if (w[i] > mx) mx = w[i];
    }
    o->drange = (double)(mx - mn);

    /* np.min / np.max passed directly. Row 0: numba array_min/max
     * (numba/np/arraymath.py:516-532, 599-615): start at x[0]; a NaN (x[0] or later) is
     * returned at once. Rows >= 1: the parfor swap min/max_parallel_impl
     * (numba/parfors/parfor.py:124-168): start at +-inf, val = min(val, x) with Python's
     * rule (x < val ? x : val), so NaN is skipped and an all-NaN window gives +-inf. */
    if (row0) {
        float a = w[0], b = w[0];
        int nan_hit = isnan(w[0]);
        for (int64_t i = 1; i < W && !nan_hit; i++) {
            if (isnan(w[i])) { a = b = w[i]; nan_hit = 1; break; }
            if (w[i] < a) a = w[i];
            if (w[i] > b) b = w[i];
        }
        o->vmin = (double)a;
        o->vmax = (double)b;
    } else {
        float a = INFINITY, b = -INFINITY;
        for (int64_t i = 0; i < W; i++) {
            a = (w[i] < a) ? w[i] : a;
            b = (w[i] > b) ? w[i] : b;
        }
        o->vmin = (double)a;
        o->vmax = (double)b;
    }

    /* line length: sum(|diff(x)|) */
    float ll = 0.0f;
    for (int64_t i = 1; i < W; i++)
        if (blk == 0 || i % blk != 0) ll = ll + fabsf(w[i] - w[i - 1]);
    o->ll = (double)ll;
}

/* gradient(x) (timedom.py:11-31): out = np.zeros(len(x)) is fp64; out[0] = x[1]-x[0],
 * out[-1] = x[-1]-x[-2], out[i] = (x[i+1]-x[i-1])/2 (the fp32 difference, halved in fp64) */
static void gradient32(const float* x, int64_t W, double* g) {
    g[0] = (double)(x[1] - x[0]);
    g[W - 1] = (double)(x[W - 1] - x[W - 2]);
    for (int64_t i = 1; i < W - 1; i++) g[i] = (double)(x[i + 1] - x[i - 1]) / 2.0;
}
static void gradient64(const double* x, int64_t W, double* g) {
    g[0] = x[1] - x[0];
    g[W - 1] = x[W - 1] - x[W - 2];
    for (int64_t i = 1; i < W - 1; i++) g[i] = (x[i + 1] - x[i - 1]) / 2.0;
}
/* numba array_var of an fp64 array: sequential mean, sequential sum of squares, / n */
static double var64(const double* a, int64_t n) {
    double c = 0.0;
    for (int64_t i = 0; i < n; i++) c = c + a[i];
    double m = c / (double)n;
    double ssd = 0.0;
    for (int64_t i = 0; i < n; i++) {
        double v = a[i] - m;
        ssd = ssd + v * v;
    }
    return ssd / (double)n;
}
/* numba array_std of an fp32 array of n (SURVEY Appendix A with n for W) */
static float std32_of(const float* a, int64_t n) {
    float c = 0.0f;
    for (int64_t i = 0; i < n; i++) c = c + a[i];
    float m = (float)((double)c / (double)n);
    double ssd = 0.0;
    for (int64_t i = 0; i < n; i++) {
        float d = a[i] - m;
        ssd = ssd + (double)(d * d);
    }
    float var = (float)(ssd / (double)n);
    return (float)sqrt((double)var);
}

/* §8f N3 / N4 features of one window (they run inside @jit functions: serial numerics on
 * every row). `scratch` holds >= 2W doubles + 2W floats. */
static void extras(const float* w, int64_t W, uint64_t mask, const mhf_params* p,
                   double* scratch, win_out* o) {
    if (mask & BIT(MHF_MEDIAN)) o->median = W > 0 ? nb_median(w, W) : NAN;
    if (mask & BIT(MHF_PERCENTILE)) {
        double q = p ? p->percentile_q : 50.0;
        nb_percentiles(w, W, &q, 1, &o->pct);
    }
    if (mask & BIT(MHF_IQR)) {
        /* stats.interquartile_range (stats.py:48-59): a, b = np.percentile(x, [75, 25]) */
        const double qs[2] = {75.0, 25.0};
        double v[2];
        nb_percentiles(w, W, qs, 2, v);
        o->iqr = v[0] - v[1];
    }
    if (mask & BIT(MHF_MODE)) o->mode = W > 0 ? nb_mode(w, W) : NAN;
    if (mask & BIT(MHF_SAMPEN))
        o->sampen = W > 0 ? nb_sampen(w, W, p ? (int64_t)p->sampen_m : 2,
                                      p ? p->sampen_r : 0.2, p ? p->sampen_sd : NAN) : NAN;
    if (mask & (BIT(MHF_RQA_RR) | BIT(MHF_RQA_DET) | BIT(MHF_RQA_LAM) | BIT(MHF_RQA_ENT))) {
        double radius = p ? p->rqa_radius : 0.0;
        unsigned char* rm = rqa_matrix(w, W, radius);
        if (mask & BIT(MHF_RQA_RR)) o->rqa_rr = rqa_rr(rm, W);
        if (mask & BIT(MHF_RQA_DET)) o->rqa_det = W >= 2 ? rqa_det(rm, W) : NAN;
        if (mask & BIT(MHF_RQA_LAM)) o->rqa_lam = W >= 2 ? rqa_lam(rm, W) : NAN;
        if (mask & BIT(MHF_RQA_ENT)) o->rqa_ent = rqa_ent(rm, W, p ? (int64_t)p->rqa_minlen : 2);
        free(rm);
    }
    if (mask & BIT(MHF_ENTROPY)) {
        /* information.entropy (information.py:10-20) of a float32 window: x / np.sum(x)
         * (fp32 sequential sum, fp32 quotients), x += 1e-30 (fp32), -np.sum(x * np.log(x)) */
        float s = 0.0f, e = 0.0f;
        for (int64_t t = 0; t < W; t++) s = s + w[t];
        for (int64_t t = 0; t < W; t++) {
            float q = w[t] / s;
            q = q + (float)1e-30;
            e = e + q * logf(q);
        }
        o->entx = (double)(-e);
    }
    /* coeff_var = np.std(x) / np.mean(x): fp32 / fp32 */
    o->cv = (double)((float)o->std32 / (float)o->mean32);
    if (mask & HJORTH_MASK) {
        if (W < 2) {
            o->hj_mob = o->hj_cmp = NAN;
        } else {
            double* g = scratch;
            double* g2 = scratch + W;
            gradient32(w, W, g);
            double vg = var64(g, W);
            o->hj_mob = sqrt(vg / (double)(float)o->var32);
            gradient64(g, W, g2);
            o->hj_cmp = sqrt(var64(g2, W) / vg) / o->hj_mob;
        }
    }
    if (mask & HRV_MASK) {
        int64_t n = W - 1;
        if (n < 1) {
            o->rmssd = o->sdsd = o->ssd = o->pnnx = o->sd1 = o->sd2 = NAN;
            o->lcsi = o->lcvi = o->lmcsi = NAN;
            return;
        }
        float* d = (float*)(scratch + 2 * W);
        float* u = d + W;
        for (int64_t i = 0; i < n; i++) {
            d[i] = w[i + 1] - w[i];   /* np.diff */
            u[i] = w[i + 1] + w[i];   /* rri[1:] + rri[:-1] */
        }
        double th = p ? p->pnn_threshold : 50.0;
        double fac = p ? p->csi_factor : 0.70710678118654746;
        /* rmssd = np.sqrt(np.mean(np.square(d))): fp32 sum of fp32 squares */
        float sq = 0.0f, sd = 0.0f;
        int64_t cnt = 0;
        for (int64_t i = 0; i < n; i++) {
            sq = sq + d[i] * d[i];
            sd = sd + d[i];
            cnt += (double)fabsf(d[i]) > th;
        }
        o->rmssd = (double)sqrtf((float)((double)sq / (double)n));
        o->ssd = (double)sd;
        o->pnnx = (double)cnt / (double)n;
        float s1 = std32_of(d, n), s2 = std32_of(u, n);
        o->sdsd = (double)s1;
        o->sd1 = fac * (double)s1;
        o->sd2 = fac * (double)s2;
        o->lcsi = o->sd1 / o->sd2;
        o->lcvi = log10(o->sd1 * o->sd2);
        o->lmcsi = (o->sd1 * o->sd1) / o->sd2;
    }
}

static void spectral_d(const double* w, int64_t W, const mhf_params* p, double* psd,
                       double* re, double* im, win_out* o) {
    int64_t nb = W / 2 + 1;
    periodogram64(w, W, p->fs, psd, re, im);
    /* power_band: sum |psd[lo <= f <= hi]|; None -> min/max(freqs) */
    double lo = isnan(p->band_lo) ? bin_freq(0, W, p->fs) : p->band_lo;
    double hi = isnan(p->band_hi) ? bin_freq(nb - 1, W, p->fs) : p->band_hi;
    double bp = 0.0, tot = 0.0;
    for (int64_t k = 0; k < nb; k++) {
        double f = bin_freq(k, W, p->fs);
        if (f >= lo && f <= hi) bp = bp + fabs(psd[k]);
    }
    for (int64_t k = 0; k < nb; k++) tot = tot + fabs(psd[k]);
    o->bp = bp;
    o->rbp = bp / tot; /* reference raises ZeroDivisionError on 0/0; IEEE NaN here */
    /* entropy: p = psd / sum(psd); p += 1e-30; -sum(p log p) */
    double s = 0.0;
    for (int64_t k = 0; k < nb; k++) s = s + psd[k];
    double e = 0.0;
    for (int64_t k = 0; k < nb; k++) {
        double q = psd[k] / s + 1e-30;
        e = e + q * log(q);
    }
    o->ent = -e;
    /* peak_frequency: lidx = first lo <= f; uidx = first hi <= f; first argmax */
    int64_t lidx = 0, uidx = nb;
    if (!isnan(p->dom_lo)) {
        lidx = nb;
        for (int64_t k = 0; k < nb; k++) if (p->dom_lo <= bin_freq(k, W, p->fs)) { lidx = k; break; }
    }
    if (!isnan(p->dom_hi)) {
        uidx = nb;
        for (int64_t k = 0; k < nb; k++) if (p->dom_hi <= bin_freq(k, W, p->fs)) { uidx = k; break; }
    }
    if (uidx <= lidx) {
        o->dom = NAN; /* reference raises ValueError (argmax of an empty slice) */
    } else {
        int64_t best = lidx;
        double bv = psd[lidx];
        if (!isnan(bv)) {
            for (int64_t k = lidx + 1; k < uidx; k++) {
                if (isnan(psd[k])) { best = k; break; } /* numpy argmax: first NaN wins */
                if (psd[k] > bv) { bv = psd[k]; best = k; }
            }
        }
        o->dom = bin_freq(best, W, p->fs);
    }
}

/* float32 window: widened to float64 (exact, wd: W doubles), then the fp64 transform */
static void spectral(const float* w, int64_t W, const mhf_params* p, double* psd,
                     double* re, double* im, double* wd, win_out* o) {
    for (int64_t t = 0; t < W; t++) wd[t] = (double)w[t];
    spectral_d(wd, W, p, psd, re, im, o);
}

static double pick(const win_out* o, int32_t f) {
    switch (f) {
    case MHF_MEAN: return o->mean;
    case MHF_MEAN32: return o->mean32;
    case MHF_VAR: return o->var;
    case MHF_STD: return o->std;
    case MHF_VAR32: return o->var32;
    case MHF_STD32: return o->std32;
    case MHF_SKEWNESS: return o->skew;
    case MHF_KURTOSIS: return o->kurt;
    case MHF_KURTOSIS_EXCESS: return o->kurt_ex;
    case MHF_RMS: return o->rms;
    case MHF_ZERO_CROSSINGS: return o->zc;
    case MHF_PEAK_COUNT: return o->peaks;
    case MHF_DRANGE: return o->drange;
    case MHF_LINE_LENGTH: return o->ll;
    case MHF_BAND_POWER: return o->bp;
    case MHF_REL_BAND_POWER: return o->rbp;
    case MHF_SPECTRAL_ENTROPY: return o->ent;
    case MHF_DOMINANT_FREQ: return o->dom;
    case MHF_COEFF_VAR: return o->cv;
    case MHF_HJORTH_MOBILITY: return o->hj_mob;
    case MHF_HJORTH_COMPLEXITY: return o->hj_cmp;
    case MHF_RMSSD: return o->rmssd;
    case MHF_SDSD: return o->sdsd;
    case MHF_SSD: return o->ssd;
    case MHF_PNNX: return o->pnnx;
    case MHF_CSI_SD1: return o->sd1;
    case MHF_CSI_SD2: return o->sd2;
    case MHF_LORENZ_CSI: return o->lcsi;
    case MHF_LORENZ_CVI: return o->lcvi;
    case MHF_LORENZ_MCSI: return o->lmcsi;
    case MHF_MIN: return o->vmin;
    case MHF_MAX: return o->vmax;
    case MHF_MEDIAN: return o->median;
    case MHF_ENTROPY: return o->entx;
    case MHF_IQR: return o->iqr;
    case MHF_MODE: return o->mode;
    case MHF_PERCENTILE: return o->pct;
    case MHF_SAMPEN: return o->sampen;
    case MHF_RQA_RR: return o->rqa_rr;
    case MHF_RQA_DET: return o->rqa_det;
    case MHF_RQA_LAM: return o->rqa_lam;
    case MHF_RQA_ENT: return o->rqa_ent;
    default: return NAN;
    }
}

/* Same argument meaning as mhf_window_features() (include/mhfeat.h), host
 * pointers, n_threads OpenMP threads (<=0: runtime default). */
int mhf_oracle_window_features_ex(const float* x, int64_t n_samples, int32_t channels,
                                  int64_t ch_stride, int64_t sample_stride,
                                  int64_t wsize, int64_t wstep,
                                  int64_t first_window, int64_t n_windows,
                                  const int32_t* features, int32_t n_features,
                                  const mhf_params* p, int32_t numerics, int32_t out_dtype,
                                  void* out, int64_t out_ld, int32_t n_threads);
int mhf_oracle_window_features(const float* x, int64_t n_samples, int32_t channels,
                               int64_t ch_stride, int64_t sample_stride,
                               int64_t wsize, int64_t wstep,
                               int64_t first_window, int64_t n_windows,
                               const int32_t* features, int32_t n_features,
                               const mhf_params* p, int32_t out_dtype, void* out,
                               int64_t out_ld, int32_t n_threads) {
    return mhf_oracle_window_features_ex(x, n_samples, channels, ch_stride, sample_stride, wsize,
                                         wstep, first_window, n_windows, features, n_features, p,
                                         MHF_NUMERICS_REFERENCE, out_dtype, out, out_ld, n_threads);
}

/* numerics: MHF_NUMERICS_REFERENCE or MHF_NUMERICS_BLOCK(c) (2-D record passed flat) */
int mhf_oracle_window_features_ex(const float* x, int64_t n_samples, int32_t channels,
                                  int64_t ch_stride, int64_t sample_stride,
                                  int64_t wsize, int64_t wstep,
                                  int64_t first_window, int64_t n_windows,
                                  const int32_t* features, int32_t n_features,
                                  const mhf_params* p, int32_t numerics, int32_t out_dtype,
                                  void* out, int64_t out_ld, int32_t n_threads) {
    const int32_t blk = numerics >> 8;
    if ((numerics & 0xff) != 0 || blk < 0) return MHF_EINVAL;
    if (blk > 0 && (channels != 1 || wsize % blk != 0 || wstep % blk != 0)) return MHF_EINVAL;
    int64_t nw_all = mhf_oracle_num_windows(n_samples, wsize, wstep);
    if (nw_all < 0 || channels < 1 || n_features < 1 || first_window < 0 || n_windows < 0 ||
        first_window + n_windows > nw_all || out_ld < n_windows)
        return MHF_EINVAL;
    int need_spec = 0;
    uint64_t mask = 0;
    for (int32_t j = 0; j < n_features; j++) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return MHF_EINVAL;
        mask |= BIT(features[j]);
    }
    need_spec = (mask & SPECTRAL_MASK) != 0;
    if (need_spec && !(p && p->fs > 0.0)) return MHF_EINVAL;
    float t32 = mhf_oracle_zc_threshold32(p ? p->zc_threshold : 0.0);
    int64_t total = n_windows * (int64_t)channels;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
#pragma omp parallel
    {
        float* w = (float*)malloc(sizeof(float) * (size_t)wsize);
        double* psd = (double*)malloc(sizeof(double) * (size_t)(wsize / 2 + 1));
        double* re = (double*)malloc(sizeof(double) * (size_t)wsize);
        double* im = (double*)malloc(sizeof(double) * (size_t)wsize);
        double* wd = (double*)malloc(sizeof(double) * (size_t)wsize);
        double* xs = (double*)malloc(sizeof(double) * 3 * (size_t)wsize);
#pragma omp for schedule(static)
        for (int64_t u = 0; u < total; u++) {
            int64_t c = u / n_windows, i = u % n_windows;
            int64_t g = first_window + i;
            const float* base = x + c * ch_stride + g * wstep * sample_stride;
            for (int64_t t = 0; t < wsize; t++) w[t] = base[t * sample_stride];
            win_out o;
            memset(&o, 0, sizeof(o));
            moments(w, wsize, g == 0, t32, &o, blk);
            extras(w, wsize, mask, p, xs, &o);
            if (need_spec) spectral(w, wsize, p, psd, re, im, wd, &o);
            for (int32_t j = 0; j < n_features; j++) {
                int64_t at = (c * n_features + j) * out_ld + i;
                double v = pick(&o, features[j]);
                if (out_dtype == MHF_OUT_F32) ((float*)out)[at] = (float)v;
                else ((double*)out)[at] = v;
            }
        }
        free(w); free(psd); free(re); free(im); free(wd); free(xs);
    }
    return MHF_OK;
}

/* Indexed windows (src/mhealth/util/windows.py:134-157, indices_rolling_apply): window i
 * = arr[starts[i]:ends[i]] (Python slice clipping), serial numerics for every window
 * (a serial @jit loop: np.mean/var/std are numba's array_mean/var/std, the row-0 rule),
 * NaN when ends[i] - starts[i] < min_len or the slice is empty. Moments only. */
int mhf_oracle_indexed_features(const float* x, int64_t n_samples, int32_t channels,
                                int64_t ch_stride, int64_t sample_stride, const int64_t* starts,
                                const int64_t* ends, int64_t n_windows, int64_t min_len,
                                const int32_t* features, int32_t n_features,
                                const mhf_params* p, int32_t out_dtype, void* out,
                                int64_t out_ld, int32_t n_threads) {
    if (channels < 1 || n_features < 1 || n_windows < 0 || out_ld < n_windows) return MHF_EINVAL;
    uint64_t mask = 0;
    for (int32_t j = 0; j < n_features; j++) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return MHF_EINVAL;
        mask |= BIT(features[j]);
    }
    if (mask & SPECTRAL_MASK) return MHF_EINVAL;
    float t32 = mhf_oracle_zc_threshold32(p ? p->zc_threshold : 0.0);
    int64_t total = n_windows * (int64_t)channels;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
#pragma omp parallel
    {
        int64_t cap = 16;
        float* w = (float*)malloc(sizeof(float) * (size_t)cap);
        double* xs = (double*)malloc(sizeof(double) * 3 * (size_t)cap);
#pragma omp for schedule(dynamic, 64)
        for (int64_t u = 0; u < total; u++) {
            int64_t c = u / n_windows, i = u % n_windows;
            int64_t si = starts[i], ei = ends[i];
            /* arr[si:ei]: Python slice bounds (negative counts from the end, then clip) */
            int64_t s0 = si < 0 ? si + n_samples : si, e0 = ei < 0 ? ei + n_samples : ei;
            s0 = s0 < 0 ? 0 : (s0 > n_samples ? n_samples : s0);
            e0 = e0 < 0 ? 0 : (e0 > n_samples ? n_samples : e0);
            int64_t W = e0 > s0 ? e0 - s0 : 0;
            int keep = (ei - si >= min_len) && W > 0;
            win_out o;
            memset(&o, 0, sizeof(o));
            if (keep) {
                if (W > cap) {
                    cap = W;
                    w = (float*)realloc(w, sizeof(float) * (size_t)cap);
                    xs = (double*)realloc(xs, sizeof(double) * 3 * (size_t)cap);
                }
                const float* base = x + c * ch_stride + s0 * sample_stride;
                for (int64_t t = 0; t < W; t++) w[t] = base[t * sample_stride];
                moments(w, W, 1, t32, &o, 0);
                extras(w, W, mask, p, xs, &o);
            }
            for (int32_t j = 0; j < n_features; j++) {
                int64_t at = (c * n_features + j) * out_ld + i;
                double v = keep ? pick(&o, features[j]) : NAN;
                if (out_dtype == MHF_OUT_F32) ((float*)out)[at] = (float)v;
                else ((double*)out)[at] = v;
            }
        }
        free(w);
        free(xs);
    }
    return MHF_OK;
}

/* PSD-level functions on caller-computed rows (mhf_psd_features, include/mhfeat.h):
 * hrv.power_band / relative_power_band / peak_frequency (src/mhealth/heart/hrv.py:173-198),
 * density.peak_frequency (src/mhealth/generic/frequency/density.py:9-32), information.entropy
 * (src/mhealth/generic/information.py:10-20), numba's sequential sums in the row dtype,
 * argmax = first NaN else first strict max (numba/np/arraymath.py:735-753). */
#define PSD_ROWS_BODY(TP, TF, ABS, LOG)                                                       \
    const TP* P = (const TP*)psd;                                                           \
    const TF* F = (const TF*)freqs;                                                         \
    double lo = lower, hi = upper;                                                          \
    if ((isnan(lower) || isnan(upper)) && F && bins > 0) {                                  \
        TF a = F[0], b = F[0];                                                              \
        for (int64_t i = 0; i < bins; i++) {                                                \
            if (F[i] != F[i]) { a = b = F[i]; break; }                                      \
            if (F[i] < a) a = F[i];                                                         \
            if (F[i] > b) b = F[i];                                                         \
        }                                                                                   \
        if (isnan(lower)) lo = (double)a;                                                   \
        if (isnan(upper)) hi = (double)b;                                                   \
    }                                                                                       \
    int64_t li = 0, ui = bins;                                                              \
    if (F && !isnan(lower)) { li = bins; for (int64_t i = 0; i < bins; i++) if (lower <= (double)F[i]) { li = i; break; } } \
    if (F && !isnan(upper)) { ui = bins; for (int64_t i = 0; i < bins; i++) if (upper <= (double)F[i]) { ui = i; break; } } \
    for (int64_t r = 0; r < rows; r++) {                                                    \
        const TP* x = P + r * row_stride;                                                   \
        TP bp = 0, tot = 0, s = 0, e = 0, dv = 0, hv = 0;                                   \
        int64_t dk = -1, hk = -1, hm = 0;                                                   \
        int dn = 0, hn = 0;                                                                 \
        for (int64_t k = 0; k < bins; k++) {                                                \
            TP v = x[k];                                                                    \
            tot = tot + ABS(v);                                                             \
            s = s + v;                                                                      \
            int in = F ? ((double)F[k] >= lo && (double)F[k] <= hi) : 0;                    \
            if (in) bp = bp + ABS(v);                                                       \
            if (k >= li && k < ui && !dn) {                                                 \
                if (v != v) { dn = 1; dk = k; } else if (dk < 0 || v > dv) { dv = v; dk = k; } \
            }                                                                               \
            if (in) {                                                                       \
                if (!hn) { if (v != v) { hn = 1; hk = hm; } else if (hk < 0 || v > hv) { hv = v; hk = hm; } } \
                hm++;                                                                       \
            }                                                                               \
        }                                                                                   \
        for (int64_t k = 0; k < bins; k++) {                                                \
            TP q = x[k] / s;                                                                \
            q = q + (TP)1e-30;                                                              \
            e = e + q * LOG(q);                                                             \
        }                                                                                   \
        for (int j = 0; j < n_ops; j++) {                                                   \
            double v;                                                                       \
            switch (ops[j]) {                                                               \
            case MHF_PSD_POWER_BAND: v = (double)bp; break;                                 \
            case MHF_PSD_REL_POWER_BAND: v = (double)(bp / tot); break;                     \
            case MHF_PSD_PEAK_FREQUENCY: v = dk < 0 ? NAN : (double)F[dk]; break;           \
            case MHF_PSD_PEAK_FREQUENCY_HRV: v = hk < 0 ? NAN : (double)F[hk]; break;       \
            case MHF_PSD_ENTROPY: v = (double)(-e); break;                                  \
            default: v = NAN;                                                               \
            }                                                                               \
            out[j * out_ld + r] = v;                                                        \
        }                                                                                   \
    }

int mhf_oracle_psd_features(const void* psd, int32_t psd_dtype, int64_t rows, int64_t bins,
                            int64_t row_stride, const void* freqs, int32_t freqs_dtype,
                            const int32_t* ops, int32_t n_ops, double lower, double upper,
                            double* out, int64_t out_ld) {
    if (psd_dtype == MHF_DTYPE_F64 && freqs_dtype == MHF_DTYPE_F64) { PSD_ROWS_BODY(double, double, fabs, log) }
    else if (psd_dtype == MHF_DTYPE_F64) { PSD_ROWS_BODY(double, float, fabs, log) }
    else if (freqs_dtype == MHF_DTYPE_F64) { PSD_ROWS_BODY(float, double, fabsf, logf) }
    else { PSD_ROWS_BODY(float, float, fabsf, logf) }
    return MHF_OK;
}

/* Raw fp64 periodogram rows (for tests of the spectral oracle itself). */
int mhf_oracle_periodogram(const float* win, int64_t n_rows, int64_t W, double fs,
                           double* psd_out) {
#pragma omp parallel
    {
        double* re = (double*)malloc(sizeof(double) * (size_t)W);
        double* im = (double*)malloc(sizeof(double) * (size_t)W);
        double* wd = (double*)malloc(sizeof(double) * (size_t)W);
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n_rows; r++) {
            for (int64_t t = 0; t < W; t++) wd[t] = (double)win[r * W + t];
            periodogram64(wd, W, fs, psd_out + r * (W / 2 + 1), re, im);
        }
        free(re); free(im); free(wd);
    }
    return 0;
}

/* The same for float64 rows. */
int mhf_oracle_periodogram64(const double* win, int64_t n_rows, int64_t W, double fs,
                             double* psd_out) {
#pragma omp parallel
    {
        double* re = (double*)malloc(sizeof(double) * (size_t)W);
        double* im = (double*)malloc(sizeof(double) * (size_t)W);
#pragma omp for schedule(static)
        for (int64_t r = 0; r < n_rows; r++)
            periodogram64(win + r * W, W, fs, psd_out + r * (W / 2 + 1), re, im);
        free(re); free(im);
    }
    return 0;
}


/* ---------------------------------------------------------------- §8f N2: filtfilt
 * scipy.signal.filtfilt(b, a, x) as the reference calls it (generic/filters.py:8-35):
 * padtype 'odd' (scipy/signal/_arraytools.py odd_ext, evaluated on the fp32 array),
 * padlen = 3 * max(len(a), len(b)), zi = lfilter_zi(b, a) (scipy/signal/_signaltools.py:
 * solve (I - companion(a).T) zi = b[1:] - a[1:] b0) scaled by the first input of each
 * pass, and lfilter's direct form II transposed in fp64 (scipy/signal/_lfilter.c), one
 * sequential pass forward and one backward. out[t * C + c] (fp64). */
static void oracle_lfilter_zi(const double* b, const double* a, int n, double* zi) {
    double m[32][33];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) m[i][j] = (i == j) ? 1.0 : 0.0;
        m[i][0] += a[i + 1];
        if (i + 1 < n) m[i][i + 1] -= 1.0;
        m[i][n] = b[i + 1] - a[i + 1] * b[0];
    }
    for (int col = 0; col < n; col++) {
        int p = col;
        for (int i = col + 1; i < n; i++) if (fabs(m[i][col]) > fabs(m[p][col])) p = i;
        if (p != col)
            for (int j = 0; j <= n; j++) { double t = m[col][j]; m[col][j] = m[p][j]; m[p][j] = t; }
        for (int i = col + 1; i < n; i++) {
            double f = m[i][col] / m[col][col];
            for (int j = col; j <= n; j++) m[i][j] -= f * m[col][j];
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = m[i][n];
        for (int j = i + 1; j < n; j++) s -= m[i][j] * zi[j];
        zi[i] = s / m[i][i];
    }
}

static void oracle_df2t(const double* b, const double* a, int ns, const double* in,
                        double* outp, int64_t len, double* z) {
    for (int64_t k = 0; k < len; k++) {
        double xn = in[k], yn;
        if (ns > 0) {
            yn = z[0] + b[0] * xn;
            for (int i = 0; i < ns - 1; i++) z[i] = (z[i + 1] + xn * b[i + 1]) - yn * a[i + 1];
            z[ns - 1] = xn * b[ns] - yn * a[ns];
        } else {
            yn = xn * b[0];
        }
        outp[k] = yn;
    }
}

int mhf_oracle_filtfilt(const float* x, int64_t n, int32_t channels, int64_t ch_stride,
                        int64_t sample_stride, const double* b_in, int32_t nb,
                        const double* a_in, int32_t na, const double* zi_in, double* out) {
    int taps = nb > na ? nb : na;
    if (taps > 32 || nb < 1 || na < 1 || a_in[0] == 0.0) return MHF_EINVAL;
    int64_t padlen = 3 * (int64_t)taps;
    if (n <= padlen) return MHF_EINVAL;
    double b[32] = {0}, a[32] = {0};
    for (int i = 0; i < nb; i++) b[i] = b_in[i];
    for (int i = 0; i < na; i++) a[i] = a_in[i];
    if (a[0] != 1.0) {
        double a0 = a[0];
        for (int i = 0; i < taps; i++) { b[i] /= a0; a[i] /= a0; }
    }
    int ns = taps - 1;
    double zi[32];
    if (zi_in) for (int i = 0; i < ns; i++) zi[i] = zi_in[i];
    else oracle_lfilter_zi(b, a, ns, zi);
    int64_t L = n + 2 * padlen;
    double* ext = (double*)malloc(sizeof(double) * (size_t)L);
    double* y = (double*)malloc(sizeof(double) * (size_t)L);
    double* r = (double*)malloc(sizeof(double) * (size_t)L);
    for (int32_t c = 0; c < channels; c++) {
        const float* xc = x + c * ch_stride;
        float x0 = xc[0], xl = xc[(n - 1) * sample_stride];
        for (int64_t j = 0; j < padlen; j++)
            ext[j] = (double)(2.0f * x0 - xc[(padlen - j) * sample_stride]);
        for (int64_t t = 0; t < n; t++) ext[padlen + t] = (double)xc[t * sample_stride];
        for (int64_t j = 0; j < padlen; j++)
            ext[padlen + n + j] = (double)(2.0f * xl - xc[(n - 2 - j) * sample_stride]);
        double z[32];
        for (int i = 0; i < ns; i++) z[i] = zi[i] * ext[0];
        oracle_df2t(b, a, ns, ext, y, L, z);
        for (int64_t j = 0; j < L; j++) r[j] = y[L - 1 - j];
        for (int i = 0; i < ns; i++) z[i] = zi[i] * r[0];
        oracle_df2t(b, a, ns, r, y, L, z);
        for (int64_t t = 0; t < n; t++) out[t * channels + c] = y[L - 1 - (padlen + t)];
    }
    free(ext); free(y); free(r);
    return MHF_OK;
}

/* magnitude(x, y, z) of fp32 arrays (inertial/accelerometer.py:198-225) */
void mhf_oracle_magnitude(const float* x, int64_t n, int64_t ss, int64_t cs, float* out) {
    for (int64_t t = 0; t < n; t++) {
        const float* p = x + t * ss;
        out[t] = sqrtf((p[0] * p[0] + p[cs] * p[cs]) + p[2 * cs] * p[2 * cs]);
    }
}

/* ---- per-sample helpers (inertial/accelerometer.py:13-75, 236-259; generic/timedom.py:11-48).
 * float32 input: numba's float32 ufuncs are the libm float functions (atan2f, sqrtf), so
 * this restatement (glibc) reproduces the reference bit for bit; the products by 180 and
 * the division by pi run in float64 (array(float32) * int64 -> float64 in numba). */
void mhf_oracle_orientation32(int32_t which, const float* x, const float* y, const float* z,
                              int64_t n, double* out) {
    for (int64_t i = 0; i < n; i++) {
        float a = which == 0 ? atan2f(y[i], z[i]) : atan2f(-x[i], sqrtf(y[i] * y[i] + z[i] * z[i]));
        out[i] = (double)a * 180.0 / M_PI;
    }
}
void mhf_oracle_orientation64(int32_t which, const double* x, const double* y, const double* z,
                              int64_t n, double* out) {
    for (int64_t i = 0; i < n; i++) {
        double a = which == 0 ? atan2(y[i], z[i]) : atan2(-x[i], sqrt(y[i] * y[i] + z[i] * z[i]));
        out[i] = a * 180.0 / M_PI;
    }
}
/* gradient: np.zeros(len(x)) float64; edges x[1]-x[0], x[-1]-x[-2]; interior
 * (x[i+1]-x[i-1]) / 2 with the difference in x's dtype */
void mhf_oracle_gradient32(const float* x, int64_t n, double* out) { gradient32(x, n, out); }
void mhf_oracle_gradient64(const double* x, int64_t n, double* out) { gradient64(x, n, out); }
/* zero_crossings: |x| <= th -> 0 (compared in float64), pos = x > 0, pos[:-1] ^ pos[1:] */
void mhf_oracle_zero_crossings32(const float* x, int64_t n, double th, uint8_t* out) {
    for (int64_t i = 0; i + 1 < n; i++) {
        int a = !(fabs((double)x[i]) <= th) && x[i] > 0.0f;
        int b = !(fabs((double)x[i + 1]) <= th) && x[i + 1] > 0.0f;
        out[i] = (uint8_t)(a != b);
    }
}
void mhf_oracle_zero_crossings64(const double* x, int64_t n, double th, uint8_t* out) {
    for (int64_t i = 0; i + 1 < n; i++) {
        int a = !(fabs(x[i]) <= th) && x[i] > 0.0;
        int b = !(fabs(x[i + 1]) <= th) && x[i + 1] > 0.0;
        out[i] = (uint8_t)(a != b);
    }
}
/* magnitude_dot: sqrt(dot(x,x) + dot(y,y) + dot(z,z)); BLAS sdot / ddot sum in blocks of
 * unspecified order — restated as sequential dtype sums (parity by tolerance) */
double mhf_oracle_magnitude_dot32(const float* x, const float* y, const float* z, int64_t n) {
    float d[3] = {0.0f, 0.0f, 0.0f};
    const float* a[3] = {x, y, z};
    for (int k = 0; k < 3; k++)
        for (int64_t i = 0; i < n; i++) d[k] = d[k] + a[k][i] * a[k][i];
    return (double)sqrtf((d[0] + d[1]) + d[2]);
}
double mhf_oracle_magnitude_dot64(const double* x, const double* y, const double* z, int64_t n) {
    double d[3] = {0.0, 0.0, 0.0};
    const double* a[3] = {x, y, z};
    for (int k = 0; k < 3; k++)
        for (int64_t i = 0; i < n; i++) d[k] = d[k] + a[k][i] * a[k][i];
    return sqrt((d[0] + d[1]) + d[2]);
}

/* ---- float64 input (numba types every reduction from the input dtype) -------------------
 * The lane features of an fp64 window, restated from the same reference functions as the
 * fp32 models above with every intermediate in fp64: np.mean = sequential fp64 sum / n
 * (row 0 and the parfor rows agree), np.var = fp64 sum of (x - m)^2 / n, np.std = its
 * sqrt, skewness / kurtosis with per-element division by len(x) (rows for a 2-D block),
 * gradient / diff in fp64. */
static double std64_of(const double* a, int64_t n) { return sqrt(var64(a, n)); }

static void window64(const double* w, int64_t W, int row0, double th, int32_t blk,
                     uint64_t mask, const mhf_params* p, double* scratch, win_out* o) {
    double c = 0.0;
    for (int64_t i = 0; i < W; i++) c = c + w[i];
    const double m = c / (double)W;
    o->mean = o->mean32 = m;
    double ssd = 0.0;
    for (int64_t i = 0; i < W; i++) ssd = ssd + (w[i] - m) * (w[i] - m);
    const double var = ssd / (double)W, sd = sqrt(var);
    o->var = o->var32 = var;
    o->std = o->std32 = sd;
    const double rows = (double)(blk > 0 ? W / blk : W);
    if (sd == 0.0) {
        o->skew = 0.0;
    } else {
        double s3 = 0.0;
        for (int64_t i = 0; i < W; i++) {
            double d = w[i] - m;
            s3 = s3 + (d * (d * d)) / rows;
        }
        o->skew = s3 / (sd * (sd * sd));
    }
    if (var == 0.0) {
        o->kurt = 0.0;
    } else {
        double s4 = 0.0;
        for (int64_t i = 0; i < W; i++) {
            double d = w[i] - m, q = d * d;
            s4 = s4 + (q * q) / rows;
        }
        o->kurt = s4 / (var * var);
    }
    o->kurt_ex = o->kurt - 3.0;
    double a = 0.0;
    for (int64_t i = 0; i < W; i++) a = a + w[i] * w[i];
    o->rms = sqrt(a / (double)W);
    int64_t zc = 0, pk = 0;
    for (int64_t i = 0; i + 1 < W; i++) {
        int pa = !(fabs(w[i]) <= th) && w[i] > 0.0, pb = !(fabs(w[i + 1]) <= th) && w[i + 1] > 0.0;
        zc += pa != pb;
    }
    for (int64_t i = 1; i + 1 < W; i++) pk += (w[i] > w[i - 1] && w[i] > w[i + 1]);
    o->zc = (double)zc;
    o->peaks = (double)pk;
    double mn = w[0], mx = w[0];
    for (int64_t i = 1; i < W; i++) {
        if (w[i] < mn) mn = w[i];
        if (w[i] > mx) mx = w[i];
    }
    o->drange = mx - mn;
    if (row0) {
        double lo = w[0], hi = w[0];
        for (int64_t i = 1; i < W && !isnan(lo); i++) {
            if (isnan(w[i])) { lo = hi = w[i]; break; }
            if (w[i] < lo) lo = w[i];
            if (w[i] > hi) hi = w[i];
        }
        o->vmin = lo;
        o->vmax = hi;
    } else {
        double lo = INFINITY, hi = -INFINITY;
        for (int64_t i = 0; i < W; i++) {
            lo = (w[i] < lo) ? w[i] : lo;
            hi = (w[i] > hi) ? w[i] : hi;
        }
        o->vmin = lo;
        o->vmax = hi;
    }
    double ll = 0.0;
    for (int64_t i = 1; i < W; i++)
        if (blk == 0 || i % blk != 0) ll = ll + fabs(w[i] - w[i - 1]);
    o->ll = ll;
    o->cv = sd / m;
    /* order statistics of a float64 window: the same numba models in float64
     * (order_models.inc with OT = double) */
    if (mask & BIT(MHF_MEDIAN)) o->median = W > 0 ? nb_median64(w, W) : NAN;
    if (mask & BIT(MHF_PERCENTILE)) {
        double q = p ? p->percentile_q : 50.0;
        nb_percentiles64(w, W, &q, 1, &o->pct);
    }
    if (mask & BIT(MHF_IQR)) {
        const double qs[2] = {75.0, 25.0};
        double v[2];
        nb_percentiles64(w, W, qs, 2, v);
        o->iqr = v[0] - v[1];
    }
    if (mask & BIT(MHF_MODE)) o->mode = W > 0 ? nb_mode64(w, W) : NAN;
    if (mask & BIT(MHF_SAMPEN))
        o->sampen = W > 0 ? nb_sampen64(w, W, p ? (int64_t)p->sampen_m : 2,
                                        p ? p->sampen_r : 0.2, p ? p->sampen_sd : NAN) : NAN;
    if (mask & (BIT(MHF_RQA_RR) | BIT(MHF_RQA_DET) | BIT(MHF_RQA_LAM) | BIT(MHF_RQA_ENT))) {
        double radius = p ? p->rqa_radius : 0.0;
        unsigned char* rm = rqa_matrix64(w, W, radius);
        if (mask & BIT(MHF_RQA_RR)) o->rqa_rr = rqa_rr(rm, W);
        if (mask & BIT(MHF_RQA_DET)) o->rqa_det = W >= 2 ? rqa_det(rm, W) : NAN;
        if (mask & BIT(MHF_RQA_LAM)) o->rqa_lam = W >= 2 ? rqa_lam(rm, W) : NAN;
        if (mask & BIT(MHF_RQA_ENT)) o->rqa_ent = rqa_ent(rm, W, p ? (int64_t)p->rqa_minlen : 2);
        free(rm);
    }
    if (mask & BIT(MHF_ENTROPY)) {
        double s = 0.0, e = 0.0;
        for (int64_t t = 0; t < W; t++) s = s + w[t];
        for (int64_t t = 0; t < W; t++) {
            double q = w[t] / s + 1e-30;
            e = e + q * log(q);
        }
        o->entx = -e;
    }
    if (mask & HJORTH_MASK) {
        if (W < 2) {
            o->hj_mob = o->hj_cmp = NAN;
        } else {
            double* g = scratch;
            double* g2 = scratch + W;
            gradient64(w, W, g);
            double vg = var64(g, W);
            o->hj_mob = sqrt(vg / var);
            gradient64(g, W, g2);
            o->hj_cmp = sqrt(var64(g2, W) / vg) / o->hj_mob;
        }
    }
    if (mask & HRV_MASK) {
        int64_t n = W - 1;
        if (n < 1) {
            o->rmssd = o->sdsd = o->ssd = o->pnnx = o->sd1 = o->sd2 = NAN;
            o->lcsi = o->lcvi = o->lmcsi = NAN;
            return;
        }
        double* d = scratch + 2 * W;
        double* u = d + W;
        double sq = 0.0, sdd = 0.0;
        int64_t cnt = 0;
        double pth = p ? p->pnn_threshold : 50.0, fac = p ? p->csi_factor : 0.70710678118654746;
        for (int64_t i = 0; i < n; i++) {
            d[i] = w[i + 1] - w[i];
            u[i] = w[i + 1] + w[i];
            sq = sq + d[i] * d[i];
            sdd = sdd + d[i];
            cnt += fabs(d[i]) > pth;
        }
        o->rmssd = sqrt(sq / (double)n);
        o->ssd = sdd;
        o->pnnx = (double)cnt / (double)n;
        o->sdsd = std64_of(d, n);
        o->sd1 = fac * o->sdsd;
        o->sd2 = fac * std64_of(u, n);
        o->lcsi = o->sd1 / o->sd2;
        o->lcvi = log10(o->sd1 * o->sd2);
        o->lmcsi = (o->sd1 * o->sd1) / o->sd2;
    }
}

/* mhf_window_features_f64 (include/mhfeat.h): float64 samples, the lane features and the
 * order statistics */
int mhf_oracle_window_features64(const double* x, int64_t n_samples, int32_t channels,
                                 int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                                 int64_t wstep, int64_t first_window, int64_t n_windows,
                                 const int32_t* features, int32_t n_features,
                                 const mhf_params* p, int32_t numerics, int32_t out_dtype,
                                 void* out, int64_t out_ld) {
    const int32_t blk = numerics >> 8;
    if ((numerics & 0xff) != 0 || blk < 0) return MHF_EINVAL;
    if (blk > 0 && (channels != 1 || wsize % blk != 0 || wstep % blk != 0)) return MHF_EINVAL;
    int64_t nw_all = mhf_oracle_num_windows(n_samples, wsize, wstep);
    if (nw_all < 0 || channels < 1 || n_features < 1 || first_window < 0 || n_windows < 0 ||
        first_window + n_windows > nw_all || out_ld < n_windows)
        return MHF_EINVAL;
    uint64_t mask = 0;
    for (int32_t j = 0; j < n_features; j++) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return MHF_EINVAL;
        mask |= BIT(features[j]);
    }
    const int need_spec = (mask & SPECTRAL_MASK) != 0;
    if (need_spec && (blk > 0 || !(p && p->fs > 0.0))) return MHF_EINVAL;
    double th = p ? p->zc_threshold : 0.0;
    const size_t wn = (size_t)(wsize > 0 ? wsize : 1);
    const int64_t total = n_windows * (int64_t)channels;
#pragma omp parallel
    {
        double* w = (double*)malloc(sizeof(double) * wn);
        double* scratch = (double*)malloc(sizeof(double) * 4 * wn);
        double* psd = (double*)malloc(sizeof(double) * (wn / 2 + 1));
        double* re = (double*)malloc(sizeof(double) * wn);
        double* im = (double*)malloc(sizeof(double) * wn);
#pragma omp for schedule(static)
        for (int64_t u = 0; u < total; u++) {
            int64_t c = u / n_windows, i = u % n_windows;
            int64_t g = first_window + i;
            const double* base = x + c * ch_stride + g * wstep * sample_stride;
            for (int64_t t = 0; t < wsize; t++) w[t] = base[t * sample_stride];
            win_out o;
            memset(&o, 0, sizeof(o));
            window64(w, wsize, g == 0, th, blk, mask, p, scratch, &o);
            /* spectral features of a float64 window: the fp64 transform of its own values */
            if (need_spec) spectral_d(w, wsize, p, psd, re, im, &o);
            for (int32_t j = 0; j < n_features; j++) {
                int64_t at = (c * n_features + j) * out_ld + i;
                double v = pick(&o, features[j]);
                if (out_dtype == MHF_OUT_F32) ((float*)out)[at] = (float)v;
                else ((double*)out)[at] = v;
            }
        }
        free(w); free(scratch); free(psd); free(re); free(im);
    }
    return MHF_OK;
}
/* indices_rolling_apply (windows.py:134-157) on a float64 record: window i = x[si:ei]
 * (Python slice clipping), the fp64 lane models and order statistics of window64; NaN
 * for windows shorter than min_len. Serial (test sizes). */
int mhf_oracle_indexed_features64(const double* x, int64_t n_samples, int32_t channels,
                                  int64_t ch_stride, int64_t sample_stride, const int64_t* starts,
                                  const int64_t* ends, int64_t n_windows, int64_t min_len,
                                  const int32_t* features, int32_t n_features,
                                  const mhf_params* p, int32_t out_dtype, void* out,
                                  int64_t out_ld) {
    if (channels < 1 || n_features < 1 || n_windows < 0 || out_ld < n_windows) return MHF_EINVAL;
    uint64_t mask = 0;
    for (int32_t j = 0; j < n_features; j++) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return MHF_EINVAL;
        mask |= BIT(features[j]);
    }
    if (mask & SPECTRAL_MASK) return MHF_EINVAL;
    const double th = p ? p->zc_threshold : 0.0;
    int64_t longest = 1;
    for (int64_t i = 0; i < n_windows; i++)
        if (ends[i] - starts[i] > longest) longest = ends[i] - starts[i];
    if (longest > n_samples) longest = n_samples > 0 ? n_samples : 1;
    double* w = (double*)malloc(sizeof(double) * (size_t)longest);
    double* scratch = (double*)malloc(sizeof(double) * 4 * (size_t)longest);
    for (int64_t c = 0; c < channels; c++) {
        for (int64_t i = 0; i < n_windows; i++) {
            const int64_t si = starts[i], ei = ends[i];
            int64_t s0 = si < 0 ? si + n_samples : si, e0 = ei < 0 ? ei + n_samples : ei;
            s0 = s0 < 0 ? 0 : (s0 > n_samples ? n_samples : s0);
            e0 = e0 < 0 ? 0 : (e0 > n_samples ? n_samples : e0);
            const int64_t W = e0 > s0 ? e0 - s0 : 0;
            const int keep = (ei - si >= min_len) && W > 0;
            win_out o;
            memset(&o, 0, sizeof(o));
            if (keep) {
                for (int64_t t = 0; t < W; t++) w[t] = x[c * ch_stride + (s0 + t) * sample_stride];
                window64(w, W, 1, th, 0, mask, p, scratch, &o);
            }
            for (int32_t j = 0; j < n_features; j++) {
                const int64_t at = (c * n_features + j) * out_ld + i;
                const double v = keep ? pick(&o, features[j]) : NAN;
                if (out_dtype == MHF_OUT_F32) ((float*)out)[at] = (float)v;
                else ((double*)out)[at] = v;
            }
        }
    }
    free(w); free(scratch);
    return MHF_OK;
}

/* qrs.nb_find_peaks (heart/qrs.py:215-220): i in [1, n-2] with x[i] > x[i-1] and x[i] > x[i+1] */
int64_t mhf_oracle_find_peaks32(const float* x, int64_t n, int64_t* out) {
    int64_t k = 0;
    for (int64_t i = 1; i + 1 < n; i++)
        if (x[i] > x[i - 1] && x[i] > x[i + 1]) out[k++] = i;
    return k;
}
int64_t mhf_oracle_find_peaks64(const double* x, int64_t n, int64_t* out) {
    int64_t k = 0;
    for (int64_t i = 1; i + 1 < n; i++)
        if (x[i] > x[i - 1] && x[i] > x[i + 1]) out[k++] = i;
    return k;
}
