/* oracle_asan.c — drives the CPU oracle (oracle/mhf_oracle.c, test infrastructure) under
 * AddressSanitizer + UBSan (tests/host/Makefile): every feature id, fixed windows of the
 * shapes the GPU tests use (W = 1 .. 1024, overlapping / gapped steps, 1-D and 3-axis AoS
 * records, 2-D block numerics), time-indexed windows (short / empty / long / negative),
 * float64 records, and the periodogram / filter helpers, on records allocated to their exact
 * size so any read past a window or the record end is reported. Run by
 * tests/test_host.py::test_oracle_under_asan. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mhfeat.h"

int mhf_oracle_window_features_ex(const float* x, int64_t n_samples, int32_t channels,
                                  int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                                  int64_t wstep, int64_t first_window, int64_t n_windows,
                                  const int32_t* features, int32_t n_features, const mhf_params* p,
                                  int32_t numerics, int32_t out_dtype, void* out, int64_t out_ld,
                                  int32_t n_threads);
int mhf_oracle_indexed_features(const float* x, int64_t n_samples, int32_t channels,
                                int64_t ch_stride, int64_t sample_stride, const int64_t* starts,
                                const int64_t* ends, int64_t n_windows, int64_t min_len,
                                const int32_t* features, int32_t n_features, const mhf_params* p,
                                int32_t out_dtype, void* out, int64_t out_ld, int32_t n_threads);
int mhf_oracle_window_features64(const double* x, int64_t n_samples, int32_t channels,
                                 int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                                 int64_t wstep, int64_t first_window, int64_t n_windows,
                                 const int32_t* features, int32_t n_features, const mhf_params* p,
                                 int32_t numerics, int32_t out_dtype, void* out, int64_t out_ld,
                                 int32_t n_threads);
int mhf_oracle_periodogram(const float* win, int64_t n_rows, int64_t W, double fs, double* out);
int64_t mhf_oracle_num_windows(int64_t n, int64_t w, int64_t s);

static uint64_t g_rng = 88172645463325252ull;
static double urand(void) {
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) / 9007199254740992.0;
}

static mhf_params params(void) {
    mhf_params p;
    memset(&p, 0, sizeof p);
    p.fs = 64.0; p.band_lo = 0.5; p.band_hi = 4.0; p.dom_lo = 0.5; p.dom_hi = 8.0;
    p.zc_threshold = 0.0; p.pnn_threshold = 50.0; p.csi_factor = 0.7071067811865476;
    p.percentile_q = 33.0; p.sampen_m = 2.0; p.sampen_r = 0.2; p.sampen_sd = NAN;
    p.rqa_radius = 0.3; p.rqa_minlen = 2.0;
    return p;
}

int main(void) {
    int fails = 0, calls = 0;
    mhf_params p = params();
    int32_t all[MHF_NUM_FEATURES];
    for (int f = 0; f < MHF_NUM_FEATURES; ++f) all[f] = f;
    const int64_t shapes[][2] = {{1, 1}, {7, 3}, {128, 128}, {250, 125}, {256, 256}, {256, 64},
                                 {100, 137}, {1024, 128}, {289, 200}};
    for (size_t si = 0; si < sizeof shapes / sizeof shapes[0]; ++si) {
        const int64_t W = shapes[si][0], S = shapes[si][1];
        for (int C = 1; C <= 3; C += 2) {
            const int64_t nw = W >= 1024 ? 9 : 40;
            const int64_t n = (nw - 1) * S + W;
            float* x = (float*)malloc(sizeof(float) * (size_t)(n * C));   /* exact size */
            for (int64_t i = 0; i < n * C; ++i) x[i] = (float)(urand() * 2.0 - 1.0 + (i % 3 == 2 ? 1.0 : 0.0));
            double* out = (double*)malloc(sizeof(double) * (size_t)(C * MHF_NUM_FEATURES * nw));
            /* spectral ids need W <= 4096 (all here); sort / sampen / rqa need short W */
            int32_t ids[MHF_NUM_FEATURES];
            int nf = 0;
            for (int f = 0; f < MHF_NUM_FEATURES; ++f) {
                if (W > 512 && (f == MHF_SAMPEN || f == MHF_RQA_RR || f == MHF_RQA_DET ||
                                f == MHF_RQA_LAM || f == MHF_RQA_ENT)) continue;
                ids[nf++] = all[f];
            }
            const int rc = mhf_oracle_window_features_ex(x, n, C, C > 1 ? 1 : 0, C, W, S, 0, nw, ids, nf, &p,
                                                         MHF_NUMERICS_REFERENCE, MHF_OUT_F64, out, nw, 1);
            ++calls;
            if (rc != 0) { fprintf(stderr, "window_features W=%lld S=%lld C=%d rc=%d\n", (long long)W, (long long)S, C, rc); ++fails; }
            /* time-indexed windows over the same record */
            int64_t st[64], en[64];
            for (int i = 0; i < 64; ++i) {
                const int64_t s = (int64_t)(urand() * (double)(n - 1));
                int64_t len = (int64_t)(urand() * 300.0);
                if (i % 9 == 0) len = 0;
                st[i] = (i % 7 == 0) ? s - n : s;
                en[i] = st[i] + len;
                if (i % 11 == 0) en[i] = n + 50;          /* clipped at the record end */
            }
            double* out2 = (double*)malloc(sizeof(double) * (size_t)(C * 14 * 64));
            const int32_t mids[14] = {MHF_MEAN, MHF_VAR, MHF_STD, MHF_SKEWNESS, MHF_KURTOSIS, MHF_RMS,
                                      MHF_ZERO_CROSSINGS, MHF_PEAK_COUNT, MHF_DRANGE, MHF_LINE_LENGTH,
                                      MHF_MEDIAN, MHF_PERCENTILE, MHF_IQR, MHF_MODE};
            const int rc2 = mhf_oracle_indexed_features(x, n, C, C > 1 ? 1 : 0, C, st, en, 64, 1, mids, 14, &p,
                                                        MHF_OUT_F64, out2, 64, 1);
            ++calls;
            if (rc2 != 0) { fprintf(stderr, "indexed rc=%d\n", rc2); ++fails; }
            free(out2);
            free(out);
            free(x);
        }
    }
    /* 2-D block numerics: a (rows, 3) record passed flat */
    {
        const int64_t rows = 400, c = 3;
        float* x = (float*)malloc(sizeof(float) * (size_t)(rows * c));
        for (int64_t i = 0; i < rows * c; ++i) x[i] = (float)urand();
        const int32_t ids[6] = {MHF_MEAN, MHF_VAR, MHF_SKEWNESS, MHF_KURTOSIS, MHF_LINE_LENGTH, MHF_MEDIAN};
        double out[6 * 20];
        const int rc = mhf_oracle_window_features_ex(x, rows * c, 1, 0, 1, 60, 60, 0, 20, ids, 6, &p,
                                                     MHF_NUMERICS_BLOCK(3), MHF_OUT_F64, out, 20, 1);
        ++calls;
        if (rc != 0) { fprintf(stderr, "block rc=%d\n", rc); ++fails; }
        free(x);
    }
    /* float64 record */
    {
        const int64_t W = 256, S = 128, nw = 30, n = (nw - 1) * S + W;
        double* x = (double*)malloc(sizeof(double) * (size_t)n);
        for (int64_t i = 0; i < n; ++i) x[i] = urand();
        const int32_t ids[8] = {MHF_MEAN, MHF_VAR, MHF_SKEWNESS, MHF_BAND_POWER, MHF_SPECTRAL_ENTROPY,
                                MHF_DOMINANT_FREQ, MHF_MEDIAN, MHF_SAMPEN};
        double* out = (double*)malloc(sizeof(double) * 8 * nw);
        const int rc = mhf_oracle_window_features64(x, n, 1, 0, 1, W, S, 0, nw, ids, 8, &p,
                                                    MHF_NUMERICS_REFERENCE, MHF_OUT_F64, out, nw, 1);
        ++calls;
        if (rc != 0) { fprintf(stderr, "f64 rc=%d\n", rc); ++fails; }
        free(out);
        free(x);
    }
    /* periodogram rows */
    {
        const int64_t W = 250, rows = 5;
        float* w = (float*)malloc(sizeof(float) * (size_t)(W * rows));
        for (int64_t i = 0; i < W * rows; ++i) w[i] = (float)urand();
        double* psd = (double*)malloc(sizeof(double) * (size_t)((W / 2 + 1) * rows));
        mhf_oracle_periodogram(w, rows, W, 50.0, psd);
        ++calls;
        free(psd);
        free(w);
    }
    if (fails) { fprintf(stderr, "%d of %d oracle calls failed\n", fails, calls); return 1; }
    printf("ORACLE ASAN OK: %d calls\n", calls);
    return 0;
}
