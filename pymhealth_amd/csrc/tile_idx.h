// tile_idx.h — launch interface of the indexed register-tile kernel (tile_idx.hip.h): time-
// indexed windows (mhf_indexed_window_features) and, as launch_tile_fix, fixed windows of
// any length up to kIdxWmax and any step (the non-power-of-two / overlapping shapes the
// fixed tile kernel, tile.hip.h, does not take).
#pragma once
#include "engine_common.h"

namespace mhf {

// features of the indexed tile path: numba's serial models of the two passes (the rest —
// Hjorth, HRV, min / max, entropy of x — stay with the lane-walk kernel)
constexpr fmask_t kTileIdxBits = bit(MHF_MEAN) | bit(MHF_MEAN32) | bit(MHF_VAR) | bit(MHF_VAR32) |
                                 bit(MHF_STD) | bit(MHF_STD32) | bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) |
                                 bit(MHF_KURTOSIS_EXCESS) | bit(MHF_RMS) | bit(MHF_ZERO_CROSSINGS) |
                                 bit(MHF_PEAK_COUNT) | bit(MHF_DRANGE) | bit(MHF_LINE_LENGTH) |
                                 bit(MHF_COEFF_VAR);

struct IdxTileArgs {
    const float* x;                    // AoS record: sample t of channel c at x[t * C + c]
    int64_t n_samples;
    const int64_t* starts;             // indexed windows (launch_tile_idx)
    const int64_t* ends;
    int64_t wsize, wstep, first;       // fixed windows (launch_tile_fix): g = first + i
    int64_t nwin, min_len;
    int32_t channels;                  // 1 or 3
    fmask_t mask;
    float t32;
    ExtraParams xp;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    int32_t exact_var;                 // fixed windows: MHF_NUMERICS_EXACT_VAR (tile.hip.h fast_var_ok)
};

bool tile_idx_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, fmask_t mask,
                 const float* x);
int launch_tile_idx(const IdxTileArgs& a, hipStream_t stream);
constexpr int64_t kTileFixWmax = 288;  // = kIdxWmax
bool tile_fix_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                 fmask_t mask);
int launch_tile_fix(const IdxTileArgs& a, hipStream_t stream);

}  // namespace mhf
