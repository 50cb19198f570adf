// spectral_wave.h — launch interface of the wave-per-window spectral kernel (spectral_wave.hip).
#pragma once
#include "engine_common.h"

namespace mhf {

struct SpecWaveArgs {
    const float* x;
    int64_t ch_stride, sample_stride, wstep, first, nwin;
    int32_t band_lo, band_hi;   // inclusive bin range (band_lo > band_hi: empty)
    int32_t dom_lo, dom_hi;     // [dom_lo, dom_hi)
    int32_t want_ent;
    float scale;                // 1 / (fs * W)
    double freq_step;           // freqs[k] = k * freq_step (numpy.fft.rfftfreq)
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
};

bool spectral_wave_ok(int64_t wsize);
// W = 1024: register-resident FFT (spectral_reg.hip)
bool spectral_reg_ok(int64_t wsize);
int launch_spectral_reg(const SpecWaveArgs& a, int channels, hipStream_t stream);
int launch_spectral_wave(const SpecWaveArgs& a, int64_t wsize, int channels, hipStream_t stream);

}  // namespace mhf
