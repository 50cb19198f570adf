// psd_rows.hip — the reference's PSD-level feature functions on rows of a caller-computed
// spectrum (mhf_psd_features, include/mhfeat.h):
//
//   hrv.power_band(psd, freqs, lower, upper)          src/mhealth/heart/hrv.py:173-179
//   hrv.relative_power_band(psd, freqs, lower, upper) hrv.py:192-198
//   hrv.peak_frequency(psd, freqs, lower, upper)      hrv.py:182-189 (as written: the arg max
//                                                     of the masked psd indexes the UNmasked
//                                                     freqs)
//   density.peak_frequency(psd, freqs, lower, upper)  src/mhealth/generic/frequency/density.py:17-32
//   information.entropy(x)                            src/mhealth/generic/information.py:10-20
//
// numba evaluates each on one 1-D array with sequential reductions in the array's dtype
// (numba/np/arraymath.py:165-176 array_sum: `c += v` from 0 of the return type; argmax
// :735-753: first NaN, else first strict maximum). Here one LANE owns one row and walks it
// in that order, so float32 / float64 rows give numba's own sums bit for bit; the only
// non-bit-exact step is entropy's log (device libm vs glibc, last bit). Rows are staged
// through LDS in 64-row x 32-bin tiles read with whole-line coalesced loads (a lane-per-row
// walk straight from HBM would touch 64 lines per load instruction).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/mhfeat.h"
#include "engine_common.h"

namespace mhf {
namespace {

constexpr int kRows = 64;   // rows per wave (one lane each)
constexpr int kCB = 32;     // bins per LDS tile

struct PsdArgs {
    const void* psd;
    const void* freqs;
    int64_t rows, bins, row_stride;
    double lower, upper;        // NaN = None
    int32_t n_ops;
    int32_t ops[MHF_PSD_NUM_OPS * 4];
    double* out;
    int64_t out_ld;
};

__device__ __forceinline__ float absv(float v) { return fabsf(v); }
__device__ __forceinline__ double absv(double v) { return fabs(v); }
__device__ __forceinline__ float logv(float v) { return logf(v); }
__device__ __forceinline__ double logv(double v) { return log(v); }

// np.min / np.max of a float array in numba (arraymath.py array_min/max): a NaN is
// returned as soon as it is met, else the running min / max
template <typename TF>
__device__ void freq_minmax(const TF* f, int64_t n, double& mn, double& mx) {
    mn = NAN;
    mx = NAN;
    if (n < 1) return;
    TF a = f[0], b = f[0];
    for (int64_t i = 0; i < n; ++i) {
        const TF v = f[i];
        if (v != v) { a = v; b = v; break; }
        if (v < a) a = v;
        if (v > b) b = v;
    }
    mn = static_cast<double>(a);
    mx = static_cast<double>(b);
}

template <typename TP, typename TF>
__global__ void __launch_bounds__(kRows) psd_rows_kernel(PsdArgs a) {
    __shared__ TP tile[kRows][kCB + 1];
    __shared__ double ftile[kCB];
    __shared__ double bounds[4];
    const int lane = threadIdx.x;
    const TP* psd = static_cast<const TP*>(a.psd);
    const TF* freqs = static_cast<const TF*>(a.freqs);
    bool want_band = false, want_tot = false, want_sum = false, want_dens = false,
         want_hrv = false;
    for (int j = 0; j < a.n_ops; ++j) {
        const int op = a.ops[j];
        want_band |= op == MHF_PSD_POWER_BAND || op == MHF_PSD_REL_POWER_BAND;
        want_tot |= op == MHF_PSD_REL_POWER_BAND;
        want_sum |= op == MHF_PSD_ENTROPY;
        want_dens |= op == MHF_PSD_PEAK_FREQUENCY;
        want_hrv |= op == MHF_PSD_PEAK_FREQUENCY_HRV;
    }
    const bool need_f = want_band || want_dens || want_hrv;
    // band bounds: None -> np.min / np.max(freqs) (hrv.py:174-177); density.peak_frequency
    // bounds: first_index(freqs, bound) (density.py:9-14), None -> 0 / len(psd)
    if (lane == 0 && need_f) {
        double mn = NAN, mx = NAN;
        if ((want_band || want_hrv) && (std::isnan(a.lower) || std::isnan(a.upper)))
            freq_minmax(freqs, a.bins, mn, mx);
        bounds[0] = std::isnan(a.lower) ? mn : a.lower;
        bounds[1] = std::isnan(a.upper) ? mx : a.upper;
        int64_t li = 0, ui = a.bins;
        if (!std::isnan(a.lower)) {
            li = a.bins;
            for (int64_t i = 0; i < a.bins; ++i)
                if (a.lower <= static_cast<double>(freqs[i])) { li = i; break; }
        }
        if (!std::isnan(a.upper)) {
            ui = a.bins;
            for (int64_t i = 0; i < a.bins; ++i)
                if (a.upper <= static_cast<double>(freqs[i])) { ui = i; break; }
        }
        bounds[2] = static_cast<double>(li);
        bounds[3] = static_cast<double>(ui);
    }
    __syncthreads();
    const double lo = bounds[0], hi = bounds[1];
    const int64_t lidx = need_f ? static_cast<int64_t>(bounds[2]) : 0;
    const int64_t uidx = need_f ? static_cast<int64_t>(bounds[3]) : a.bins;

    for (int64_t r0 = static_cast<int64_t>(blockIdx.x) * kRows; r0 < a.rows;
         r0 += static_cast<int64_t>(gridDim.x) * kRows) {
        const int64_t row = r0 + lane;
        const bool ok = row < a.rows;
        TP bp = TP(0), tot = TP(0), s = TP(0);
        TP dv = TP(0), hv = TP(0);
        int64_t dk = -1, hk = -1, hm = 0;     // arg max (density: bin; hrv: masked index)
        bool dnan = false, hnan = false;
        // tile walk; `second` = entropy's pass over q = x / sum(x) + 1e-30
        for (int pass = 0; pass < (want_sum ? 2 : 1); ++pass) {
            TP e = TP(0);
            for (int64_t b0 = 0; b0 < a.bins; b0 += kCB) {
                const int nb = static_cast<int>(a.bins - b0 < kCB ? a.bins - b0 : kCB);
                __syncthreads();
                // coalesced: each half wave reads kCB consecutive bins of one row
                for (int k = 0; k < kRows * kCB / 64; ++k) {
                    const int e_ = k * 64 + lane, rr = e_ / kCB, cc = e_ % kCB;
                    const int64_t grow = r0 + rr;
                    if (grow < a.rows && cc < nb) tile[rr][cc] = psd[grow * a.row_stride + b0 + cc];
                }
                if (need_f && pass == 0 && lane < nb) ftile[lane] = static_cast<double>(freqs[b0 + lane]);
                __syncthreads();
                if (!ok) continue;
                if (pass == 0) {
                    for (int c = 0; c < nb; ++c) {
                        const TP v = tile[lane][c];
                        const int64_t b = b0 + c;
                        if (want_tot) tot = tot + absv(v);
                        if (want_sum) s = s + v;
                        bool inband = false;
                        if (want_band || want_hrv) {
                            const double f = ftile[c];
                            inband = (f >= lo) && (f <= hi);
                        }
                        if (want_band && inband) bp = bp + absv(v);
                        if (want_dens && b >= lidx && b < uidx && !dnan) {
                            if (v != v) { dnan = true; dk = b; }
                            else if (dk < 0 || v > dv) { dv = v; dk = b; }
                        }
                        if (want_hrv && inband) {
                            if (!hnan) {
                                if (v != v) { hnan = true; hk = hm; }
                                else if (hk < 0 || v > hv) { hv = v; hk = hm; }
                            }
                            ++hm;
                        }
                    }
                } else {
                    for (int c = 0; c < nb; ++c) {
                        // x = x / np.sum(x); x += 1e-30; e = sum(x * log(x))
                        TP q = tile[lane][c] / s;
                        q = q + static_cast<TP>(1e-30);
                        e = e + q * logv(q);
                    }
                }
            }
            if (pass == 1 && ok) {
                for (int j = 0; j < a.n_ops; ++j)
                    if (a.ops[j] == MHF_PSD_ENTROPY) a.out[j * a.out_ld + row] = static_cast<double>(-e);
            }
        }
        if (!ok) continue;
        for (int j = 0; j < a.n_ops; ++j) {
            double v;
            switch (a.ops[j]) {
            case MHF_PSD_POWER_BAND: v = static_cast<double>(bp); break;
            case MHF_PSD_REL_POWER_BAND: v = static_cast<double>(bp / tot); break;
            case MHF_PSD_PEAK_FREQUENCY:
                v = dk < 0 ? static_cast<double>(NAN) : static_cast<double>(freqs[dk]);
                break;
            case MHF_PSD_PEAK_FREQUENCY_HRV:
                v = hk < 0 ? static_cast<double>(NAN) : static_cast<double>(freqs[hk]);
                break;
            default: continue;
            }
            a.out[j * a.out_ld + row] = v;
        }
    }
}

}  // namespace

int launch_psd_rows(const void* psd, int32_t psd_dtype, int64_t rows, int64_t bins,
                    int64_t row_stride, const void* freqs, int32_t freqs_dtype,
                    const int32_t* ops, int32_t n_ops, double lower, double upper, double* out,
                    int64_t out_ld, hipStream_t stream) {
    PsdArgs a{};
    a.psd = psd; a.freqs = freqs; a.rows = rows; a.bins = bins; a.row_stride = row_stride;
    a.lower = lower; a.upper = upper; a.n_ops = n_ops;
    for (int j = 0; j < n_ops; ++j) a.ops[j] = ops[j];
    a.out = out; a.out_ld = out_ld;
    int64_t blocks = (rows + kRows - 1) / kRows;
    if (blocks > 8192) blocks = 8192;
    const dim3 grid(static_cast<unsigned>(blocks)), block(kRows);
    const bool p64 = psd_dtype == MHF_DTYPE_F64, f64 = freqs_dtype == MHF_DTYPE_F64;
    if (p64 && f64) hipLaunchKernelGGL((psd_rows_kernel<double, double>), grid, block, 0, stream, a);
    else if (p64) hipLaunchKernelGGL((psd_rows_kernel<double, float>), grid, block, 0, stream, a);
    else if (f64) hipLaunchKernelGGL((psd_rows_kernel<float, double>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((psd_rows_kernel<float, float>), grid, block, 0, stream, a);
    return MHF_OK;
}

}  // namespace mhf
