// spectral64.h — launch interface of the float64 spectral kernel (spectral64.hip).
#pragma once
#include "engine_common.h"

namespace mhf {

struct Spec64Args {
    const double* x;
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t pow2;               // set by launch_spectral64
    int32_t band_lo, band_hi;   // inclusive bin range (band_lo > band_hi: empty)
    int32_t dom_lo, dom_hi;     // [dom_lo, dom_hi)
    int32_t want_ent;
    double scale;               // 1 / (fs * W)
    double freq_step;           // freqs[k] = k * freq_step (numpy.fft.rfftfreq)
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
};

int launch_spectral64(const Spec64Args& a, int channels, hipStream_t stream);

}  // namespace mhf
