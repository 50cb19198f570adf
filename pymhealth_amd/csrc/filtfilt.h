// filtfilt.h — launch interface of the LDS-streamed filtfilt passes (filtfilt_tile.hip).
#pragma once
#include "engine_common.h"

namespace mhf {

constexpr int kIirMaxTaps = 17;   // = filtfilt.hip kMaxTaps

struct IirTileArgs {
    // coefficients normalised by a[0], zero-padded to ns + 1 taps
    double b[kIirMaxTaps], a[kIirMaxTaps];
    double zi[kIirMaxTaps];                  // lfilter_zi(b, a)
    int32_t ns;                              // state size = taps - 1
    int32_t channels;                        // 1 or 3
    const float* x;                          // AoS record x[t * C + c], 16-B aligned
    int64_t n, padlen, L;                    // L = n + 2 padlen
    int64_t M, K;                            // chunk length (multiple of 32), chunks
    int64_t E0, E1;                          // block-grid lead before a chunk, passes 0 / 1
    double* yr;                              // forward output reversed, AoS: (L, C)
    void* out;                               // out[t * C + c]
    int32_t out_f32;
};

int launch_filtfilt_tile(const IirTileArgs& a, hipStream_t s);

}  // namespace mhf
