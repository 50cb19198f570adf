// engine_common.h — types and device helpers shared by every translation unit of
// libmhfeat.so (generic kernels + C-ABI in mhfeat.hip, tile kernels in tile_w*_c*.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "../../include/mhfeat.h"

namespace mhf {

constexpr int kMaxFeatures = 64;

// Diagnostic switches (A/B timing, and the tests that check a register-tile path bit for
// bit against the kernel it replaced; the list with their effects: INTEGRATION.md
// "Diagnostic switches"). Honoured only while MHF_DIAGNOSTICS=1 is set as well, so a stray
// variable alone never changes which kernel runs; read at every call. Host side only.
inline const char* diag_env(const char* name) {
    const char* d = getenv("MHF_DIAGNOSTICS");
    return (d && d[0] == '1' && d[1] == 0) ? getenv(name) : nullptr;
}
// a path is skipped when its switch is "1" (and MHF_DIAGNOSTICS=1)
inline bool disabled(const char* name) {
    const char* e = diag_env(name);
    return e && e[0] == '1';
}
constexpr int64_t kMaxSpectralW = 4096;

// feature bits
typedef uint64_t fmask_t;   // one bit per mhf_feature id
constexpr fmask_t bit(int f) { return fmask_t(1) << f; }
constexpr fmask_t kPass2Bits = bit(MHF_VAR) | bit(MHF_VAR32) | bit(MHF_STD) | bit(MHF_STD32) |
                                bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) | bit(MHF_KURTOSIS_EXCESS);
constexpr fmask_t kSpectralBits = bit(MHF_BAND_POWER) | bit(MHF_REL_BAND_POWER) |
                                   bit(MHF_SPECTRAL_ENTROPY) | bit(MHF_DOMINANT_FREQ);
// order statistics: their own kernel (order.hip), after the moment / spectral ones
constexpr fmask_t kOrderBits = bit(MHF_MEDIAN) | bit(MHF_IQR) | bit(MHF_MODE) | bit(MHF_PERCENTILE);
// sample entropy and recurrence quantification: their own pairwise kernels (order.hip)
constexpr fmask_t kSampenBits = bit(MHF_SAMPEN);
constexpr fmask_t kRqaBits = bit(MHF_RQA_RR) | bit(MHF_RQA_DET) | bit(MHF_RQA_LAM) | bit(MHF_RQA_ENT);
constexpr fmask_t kMomentBits = ((fmask_t(1) << MHF_NUM_FEATURES) - 1) & ~kSpectralBits &
                                ~kOrderBits & ~kSampenBits & ~kRqaBits;
// features defined on 2-D (rows, c) blocks (MHF_NUMERICS_BLOCK, include/mhfeat.h)
constexpr fmask_t kBlockBits = bit(MHF_MEAN) | bit(MHF_MEAN32) | bit(MHF_VAR) | bit(MHF_VAR32) |
                               bit(MHF_STD) | bit(MHF_STD32) | bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) |
                               bit(MHF_KURTOSIS_EXCESS) | bit(MHF_RMS) | bit(MHF_DRANGE) |
                               bit(MHF_LINE_LENGTH) | bit(MHF_COEFF_VAR) | bit(MHF_MIN) | bit(MHF_MAX) |
                               bit(MHF_MEDIAN) | bit(MHF_PERCENTILE) | bit(MHF_IQR);
// §8f N3 / N4 features: lane-per-window generic kernel only (the tile kernels keep the
// headline feature set; these run inside @jit functions, serial numerics on every row)
constexpr fmask_t kHjorthBits = bit(MHF_HJORTH_MOBILITY) | bit(MHF_HJORTH_COMPLEXITY);
constexpr fmask_t kHrvBits = bit(MHF_RMSSD) | bit(MHF_SDSD) | bit(MHF_SSD) | bit(MHF_PNNX) |
                              bit(MHF_CSI_SD1) | bit(MHF_CSI_SD2) | bit(MHF_LORENZ_CSI) |
                              bit(MHF_LORENZ_CVI) | bit(MHF_LORENZ_MCSI);
constexpr fmask_t kGenericOnlyBits = bit(MHF_COEFF_VAR) | kHjorthBits | kHrvBits | bit(MHF_MIN) |
                                     bit(MHF_MAX) | bit(MHF_ENTROPY);
static_assert(MHF_NUM_FEATURES < 64, "feature masks are 64-bit");
// float64 records: the features of the streamed tile kernel (tile64.hip)
constexpr fmask_t kTile64Bits = bit(MHF_MEAN) | bit(MHF_MEAN32) | bit(MHF_VAR) | bit(MHF_VAR32) |
                                bit(MHF_STD) | bit(MHF_STD32) | bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) |
                                bit(MHF_KURTOSIS_EXCESS) | bit(MHF_RMS) | bit(MHF_ZERO_CROSSINGS) |
                                bit(MHF_PEAK_COUNT) | bit(MHF_DRANGE) | bit(MHF_LINE_LENGTH) |
                                bit(MHF_COEFF_VAR);

// sets the message mhf_last_error() returns (mhfeat.hip); returns `code`
int set_error(int code, const char* msg);

// PSD-level features of caller-computed spectra (psd_rows.hip)
int launch_psd_rows(const void* psd, int32_t psd_dtype, int64_t rows, int64_t bins,
                    int64_t row_stride, const void* freqs, int32_t freqs_dtype,
                    const int32_t* ops, int32_t n_ops, double lower, double upper, double* out,
                    int64_t out_ld, hipStream_t stream);

// per-call parameters of the N4 features
struct ExtraParams {
    double pnn_th, csi_factor;
    int32_t blk;    // MHF_NUMERICS_BLOCK columns of a 2-D record (0: a 1-D record)
};

struct FeatList {
    int32_t n;
    int32_t id[kMaxFeatures];
};

// order statistics (order.hip): fixed windows (starts == nullptr) or indexed windows
constexpr int64_t kOrderLdsBytes = 64 * 1024;    // keys of one window, all channels
constexpr int64_t kMaxOrderSamples = kOrderLdsBytes / 4;   // W * channels
struct OrderLaunch {
    const float* x;
    const double* xd;                    // float64 record (launch_order only; x unused then)
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t channels;
    const int64_t* starts;
    const int64_t* ends;
    int64_t n_samples, min_len, max_w;   // max_w: LDS capacity for indexed windows
    int32_t skip_long;                   // indexed: leave windows > max_w to launch_order_long
    double q;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
};
int launch_order(const OrderLaunch& L, hipStream_t stream);
// indexed windows longer than the LDS capacity: keys sorted in the caller's workspace
// (`keys`, `key_bytes`: as many waves as it holds, each C * pow2ceil(max_len) keys)
constexpr int64_t kMaxLongOrderSamples = int64_t(1) << 20;   // per channel
constexpr int64_t kLongScratchBytes = int64_t(1) << 30;      // default workspace bound
int launch_order_long(const OrderLaunch& L, int64_t max_len, void* keys, int64_t key_bytes,
                      hipStream_t stream);
int launch_sampen(const OrderLaunch& L, int32_t mm, double r, double sd, hipStream_t stream);
int launch_rqa(const OrderLaunch& L, double radius, int32_t minlen, hipStream_t stream);

// ------------------------------------------------------------------ store
__device__ __forceinline__ void store_out(void* out, int out_f32, int64_t at, double v) {
    if (out_f32) static_cast<float*>(out)[at] = static_cast<float>(v);
    else static_cast<double*>(out)[at] = v;
}

// ======================================================================
// Moments: generic lane-per-window kernel (any W, S, strides). One thread owns one
// (channel, window) and walks its W samples twice in the reference's order.
// ======================================================================
struct MomArgs {
    const float* x;
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t channels;
    fmask_t mask;
    float t32;      // zero-crossing threshold, rounded so x > t32 <=> (double)x > max(th,0)
    float invW;     // 1/W (exact when W is a power of two)
    int32_t pow2;   // W is a power of two: q / W == q * invW bit for bit
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    ExtraParams xp;
};

struct WinVals {
    double mean, mean32, var, var32, std_, std32, skew, kurt, kurt_ex, rms, zc, peaks, drange,
        ll;
    double bp, rbp, ent, dom;   // spectral (fused tile kernel only)
    double cv, hj_mob, hj_cmp;  // §8f N3 (generic kernel only)
    double rmssd, sdsd, ssd, pnnx, sd1, sd2, lcsi, lcvi, lmcsi;   // §8f N4
    double vmin, vmax;          // np.min / np.max passed directly
    double entx;                // information.entropy of the window's samples
};

__device__ __forceinline__ float div_w(float q, float Wf, float invW, int pow2) {
    return pow2 ? q * invW : q / Wf;
}

__device__ __forceinline__ double pick_moment(const WinVals& v, int f) {
    switch (f) {
    case MHF_MEAN: return v.mean;
    case MHF_MEAN32: return v.mean32;
    case MHF_VAR: return v.var;
    case MHF_VAR32: return v.var32;
    case MHF_STD: return v.std_;
    case MHF_STD32: return v.std32;
    case MHF_SKEWNESS: return v.skew;
    case MHF_KURTOSIS: return v.kurt;
    case MHF_KURTOSIS_EXCESS: return v.kurt_ex;
    case MHF_RMS: return v.rms;
    case MHF_ZERO_CROSSINGS: return v.zc;
    case MHF_PEAK_COUNT: return v.peaks;
    case MHF_DRANGE: return v.drange;
    case MHF_LINE_LENGTH: return v.ll;
    case MHF_BAND_POWER: return v.bp;
    case MHF_REL_BAND_POWER: return v.rbp;
    case MHF_SPECTRAL_ENTROPY: return v.ent;
    case MHF_DOMINANT_FREQ: return v.dom;
    case MHF_COEFF_VAR: return v.cv;
    case MHF_HJORTH_MOBILITY: return v.hj_mob;
    case MHF_HJORTH_COMPLEXITY: return v.hj_cmp;
    case MHF_RMSSD: return v.rmssd;
    case MHF_SDSD: return v.sdsd;
    case MHF_SSD: return v.ssd;
    case MHF_PNNX: return v.pnnx;
    case MHF_CSI_SD1: return v.sd1;
    case MHF_CSI_SD2: return v.sd2;
    case MHF_LORENZ_CSI: return v.lcsi;
    case MHF_LORENZ_CVI: return v.lcvi;
    case MHF_LORENZ_MCSI: return v.lmcsi;
    case MHF_MIN: return v.vmin;
    case MHF_MAX: return v.vmax;
    case MHF_ENTROPY: return v.entx;
    default: return 0.0;
    }
}

}  // namespace mhf
