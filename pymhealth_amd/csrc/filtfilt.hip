// filtfilt.hip — §8f N2: zero-phase IIR filtering (scipy.signal.filtfilt, the
// reference's generic/filters.py:8-35 `butterworth` and the per-axis loops of
// inertial/accelerometer.py:78-183) on the GPU, all channels of a record at once.
//
// filtfilt(b, a, x) with padtype='odd', padlen = 3 * max(len(a), len(b)), method='pad':
//   ext = [2x0 - x[padlen..1], x, 2x_{n-1} - x[n-2..n-1-padlen]]   (fp32, like numpy on x)
//   y   = lfilter(b, a, ext, zi = lfilter_zi(b, a) * ext[0])        (fp64, DF2T)
//   y   = lfilter(b, a, y[::-1], zi = lfilter_zi(b, a) * y[-1])[::-1][padlen:-padlen]
//
// An IIR filter is a sequential recurrence; it is also stable, so the effect of its
// state fades: after R samples the zero-input response of any state is below 1e-16 of
// it (R found on the host by running the recurrence from the unit states; fp64's own
// resolution — round 5 lowered it from 1e-21: 1e8 x 3-axis highpass R 3093 -> 2465, the
// chunked result vs the sequential one 1.96e-10 -> 2.06e-10 of the signal scale in a host
// emulation, the evaluation-order difference below dominating either way). One lane
// therefore owns a chunk of M samples and starts R samples before it from a zero state
// (or from the true initial state lfilter_zi * x0 when that reaches back to sample 0):
// by the chunk start its state equals the single-pass state up to rounding, and the
// chunks run independently (no carry, no scan). A carried scan (z_{k+1} = T^M z_k + zs_k)
// was tried first and is numerically useless for low-cutoff transfer-function filters:
// T^M of the companion matrix loses everything to cancellation (2e-2 errors at 0.02 x
// Nyquist). The tf-form DF2T that scipy evaluates is itself ill-conditioned (zero-input
// transients of 1e5-5e5 x the state for 0.5 Hz at 50 Hz): two evaluation orders of the
// same recurrence differ by ~1e-9 of the signal scale, which is the parity tolerance
// (tests; bit-exact only when every chunk reaches back to sample 0).
#include <cstdio>
#include <cstdlib>

#include "engine_common.h"
#include "filtfilt.h"

namespace mhf {

constexpr int kMaxTaps = kIirMaxTaps;        // Butterworth bandpass up to order 8
constexpr int64_t kIirLanes = 32768;         // half a wave per SIMD (see iir_chunk_kernel)
// filtfilt_tile.hip workgroups: 2 per CU (measured, 1e8 x 3-axis: 256 / 384 / 512 / 768 /
// 1024 / 1536 groups 2.44 / 2.58 / 2.25 / 2.34 / 2.68 / 2.94 ms — whole workgroups per CU,
// and longer chunks re-read less warm-up)
constexpr int64_t kIirTileGroups = 512;
constexpr int kMaxState = kMaxTaps - 1;

struct IirArgs {
    // coefficients normalised by a[0] and zero-padded to ns + 1 taps
    double b[kMaxTaps], a[kMaxTaps];
    double zi[kMaxTaps];                     // lfilter_zi(b, a)
    int32_t ns;                              // state size = taps - 1
    int32_t channels;
    const float* x;                          // the record: x[t * ss + c * cs]
    int64_t n, cs, ss, padlen, L;            // L = n + 2 padlen
    int64_t M, K, R;                         // chunk length, chunks per channel, warm-up
    double* yf;                              // forward output, (C, L)
    void* out;                               // (n) samples per channel at out[t*oss + c*ocs]
    int64_t ocs, oss;
    int32_t out_f32;
};

// scipy lfilter, direct form II transposed (scipy/signal/_lfilter: y = Z0 + b0 x;
// Z_i = Z_{i+1} + x b_{i+1} - y a_{i+1}; Z_last = x b_last - y a_last), fp64
template <int NS>
__device__ __forceinline__ double df2t_step(const IirArgs& a, double (&z)[NS > 0 ? NS : 1],
                                            double x) {
    if constexpr (NS == 0) {
        return x * a.b[0];
    } else {
        const double y = z[0] + a.b[0] * x;
#pragma unroll
        for (int i = 0; i < NS - 1; ++i) z[i] = (z[i + 1] + x * a.b[i + 1]) - y * a.a[i + 1];
        z[NS - 1] = x * a.b[NS] - y * a.a[NS];
        return y;
    }
}

// input of pass P at position j: pass 0 = the odd extension of x (fp32 arithmetic, as
// numpy computes it on the fp32 array), pass 1 = the forward output reversed
template <int P>
__device__ __forceinline__ double pass_input(const IirArgs& a, int c, int64_t j) {
    if constexpr (P == 0) {
        const float* xc = a.x + c * a.cs;
        if (j < a.padlen) return static_cast<double>(2.0f * xc[0] - xc[(a.padlen - j) * a.ss]);
        const int64_t t = j - a.padlen;
        if (t < a.n) return static_cast<double>(xc[t * a.ss]);
        const int64_t r = t - a.n;
        return static_cast<double>(2.0f * xc[(a.n - 1) * a.ss] - xc[(a.n - 2 - r) * a.ss]);
    } else {
        return a.yf[static_cast<int64_t>(c) * a.L + (a.L - 1 - j)];
    }
}

// one lane per (channel, chunk): warm up over the R samples before the chunk, then
// filter and store the chunk. Pass 0 writes the forward output (fp64, (C, L)); pass 1
// filters it reversed and stores out[t] for t = (L - 1 - j) - padlen.
//
// The recurrence is a dependent fp64 chain per lane, but its inputs are not: they are
// loaded kIirBatch at a time before the batch is filtered (measured: DESIGN §5.8; a ring of 4
// batches loaded ahead measured slower, 6.49 vs 6.24 ms, round 5). Few lanes matter more
// than many here: every chunk also re-filters R
// warm-up samples (R = 3093 for a 0.5 Hz highpass at 50 Hz at the round-4 threshold, 2465 at 1e-16), so the launch uses
// ~kIirLanes lanes (half a wave per SIMD) and hides latency inside each lane instead.
constexpr int kIirBatch = 8;
template <int NS, int P>
__global__ void __launch_bounds__(64) iir_chunk_kernel(IirArgs a) {
    const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (u >= a.K * a.channels) return;
    const int c = static_cast<int>(u / a.K);
    const int64_t k = u - static_cast<int64_t>(c) * a.K;
    const int64_t j0 = k * a.M;
    const int64_t j1 = (j0 + a.M < a.L) ? j0 + a.M : a.L;
    double z[NS > 0 ? NS : 1] = {};
    int64_t s = j0 - a.R;
    if (s <= 0) {
        s = 0;
        const double x0 = pass_input<P>(a, c, 0);
#pragma unroll
        for (int i = 0; i < NS; ++i) z[i] = a.zi[i] * x0;
    }
    auto emit = [&](int64_t jj, double y) {
        if (jj < j0) return;                       // warm-up: the state only
        if constexpr (P == 0) {
            a.yf[static_cast<int64_t>(c) * a.L + jj] = y;
        } else {
            const int64_t t = a.L - 1 - jj - a.padlen;
            if (t >= 0 && t < a.n) store_out(a.out, a.out_f32, t * a.oss + c * a.ocs, y);
        }
    };
    constexpr int B = kIirBatch;
    int64_t j = s;
    for (; j + B <= j1; j += B) {
        double xin[B];
#pragma unroll
        for (int q = 0; q < B; ++q) xin[q] = pass_input<P>(a, c, j + q);
#pragma unroll
        for (int q = 0; q < B; ++q) emit(j + q, df2t_step<NS>(a, z, xin[q]));
    }
    for (; j < j1; ++j) emit(j, df2t_step<NS>(a, z, pass_input<P>(a, c, j)));
}

template <int NS>
void launch_filtfilt_ns(const IirArgs& a, hipStream_t s) {
    const int64_t units = a.K * a.channels;
    const dim3 g(static_cast<unsigned>((units + 63) / 64)), blk(64);
    hipLaunchKernelGGL((iir_chunk_kernel<NS, 0>), g, blk, 0, s, a);
    hipLaunchKernelGGL((iir_chunk_kernel<NS, 1>), g, blk, 0, s, a);
}

int launch_filtfilt(const IirArgs& a, hipStream_t s) {
    switch (a.ns) {
#define MHF_NS(N) case N: launch_filtfilt_ns<N>(a, s); break;
        MHF_NS(0) MHF_NS(1) MHF_NS(2) MHF_NS(3) MHF_NS(4) MHF_NS(5) MHF_NS(6) MHF_NS(7)
        MHF_NS(8) MHF_NS(9) MHF_NS(10) MHF_NS(11) MHF_NS(12) MHF_NS(13) MHF_NS(14)
        MHF_NS(15) MHF_NS(16)
#undef MHF_NS
    default: return MHF_EUNSUPPORTED;
    }
    return MHF_OK;
}

// ---- host side: lfilter_zi and the warm-up length
// lfilter_zi (scipy.signal.lfilter_zi): solve (I - companion(a)^T) zi = b[1:] - a[1:] b0
// (Gaussian elimination with partial pivoting; numpy's LAPACK solve rounds differently
// and the system is ill-conditioned for low cutoffs: pass the caller's zi for parity)
void host_lfilter_zi(const double* b, const double* a, int n, double* zi) {
    double m[kMaxState][kMaxState + 1];
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) m[i][j] = (i == j ? 1.0 : 0.0);
        m[i][0] += a[i + 1];
        if (i + 1 < n) m[i][i + 1] -= 1.0;
        m[i][n] = b[i + 1] - a[i + 1] * b[0];
    }
    for (int col = 0; col < n; ++col) {
        int p = col;
        for (int i = col + 1; i < n; ++i) if (fabs(m[i][col]) > fabs(m[p][col])) p = i;
        if (p != col)
            for (int j = 0; j <= n; ++j) { const double t = m[col][j]; m[col][j] = m[p][j]; m[p][j] = t; }
        for (int i = col + 1; i < n; ++i) {
            const double f = m[i][col] / m[col][col];
            for (int j = col; j <= n; ++j) m[i][j] -= f * m[col][j];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = m[i][n];
        for (int j = i + 1; j < n; ++j) s -= m[i][j] * zi[j];
        zi[i] = s / m[i][i];
    }
}

// samples until the zero-input response of every unit state is below 1e-16 (or limit)
int64_t host_warmup(const double* a, int n, int64_t limit) {
    if (n == 0) return 0;
    double v[kMaxState][kMaxState];
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) v[j][i] = (i == j) ? 1.0 : 0.0;
    for (int64_t r = 1; r <= limit; ++r) {
        double mx = 0.0;
        for (int j = 0; j < n; ++j) {
            const double y = v[j][0];
            for (int i = 0; i < n - 1; ++i) v[j][i] = v[j][i + 1] - y * a[i + 1];
            v[j][n - 1] = -y * a[n];
            for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(v[j][i]));
        }
        if (!(mx >= 1e-16)) return r;     // NaN (unstable / overflow) also ends the search
    }
    return limit;
}

}  // namespace mhf

// ====================================================================== C-ABI
namespace {
int ffail(int code, const char* msg) { return mhf::set_error(code, msg); }
}  // namespace

extern "C" {

int64_t mhf_filtfilt_workspace(int64_t n_samples, int32_t channels, int32_t nb, int32_t na) {
    if (n_samples < 1 || channels < 1 || nb < 1 || na < 1) return -1;
    const int64_t taps = nb > na ? nb : na;
    return 8 * static_cast<int64_t>(channels) * (n_samples + 2 * 3 * taps);
}

int mhf_filtfilt(const float* x, int64_t n_samples, int32_t channels, int64_t ch_stride,
                 int64_t sample_stride, const double* b, int32_t nb, const double* a,
                 int32_t na, const double* zi, int32_t out_dtype, void* out,
                 int64_t out_ch_stride, int64_t out_sample_stride, void* workspace,
                 int64_t workspace_bytes, void* hip_stream) {
    using namespace mhf;
    set_error(MHF_OK, "");
    if (!x || !out || !b || !a) return ffail(MHF_EINVAL, "null x, out, b or a");
    if (channels < 1 || n_samples < 1 || sample_stride < 1 || ch_stride < 0)
        return ffail(MHF_EINVAL, "channels, n_samples, sample_stride must be >= 1");
    if (nb < 1 || na < 1) return ffail(MHF_EINVAL, "b and a need at least one coefficient");
    if (a[0] == 0.0) return ffail(MHF_EINVAL, "a[0] must be nonzero");
    const int taps = nb > na ? nb : na;
    if (taps > kMaxTaps) return ffail(MHF_EUNSUPPORTED, "filters up to 17 taps");
    if (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32)
        return ffail(MHF_EINVAL, "out_dtype must be MHF_OUT_F64 or MHF_OUT_F32");
    IirArgs p{};
    for (int i = 0; i < kMaxTaps; ++i) {
        p.b[i] = i < nb ? b[i] : 0.0;
        p.a[i] = i < na ? a[i] : 0.0;
    }
    if (a[0] != 1.0) {
        const double a0 = a[0];
        for (int i = 0; i < kMaxTaps; ++i) { p.b[i] /= a0; p.a[i] /= a0; }
    }
    p.ns = taps - 1;
    if (zi) for (int i = 0; i < p.ns; ++i) p.zi[i] = zi[i];
    else host_lfilter_zi(p.b, p.a, p.ns, p.zi);
    p.channels = channels;
    p.x = x; p.n = n_samples; p.cs = ch_stride; p.ss = sample_stride;
    p.padlen = 3 * static_cast<int64_t>(taps);
    if (n_samples <= p.padlen)
        return ffail(MHF_EINVAL, "the length of the input must be greater than padlen "
                                 "(3 * max(len(a), len(b)))");
    p.L = n_samples + 2 * p.padlen;
    // warm-up search capped (2^21 steps x ns^2 on the host); a filter whose transient
    // outlives the cap gets the full reach (every chunk starts at sample 0: exact, K <= 3)
    const int64_t lim = p.L < (int64_t(1) << 21) ? p.L : (int64_t(1) << 21);
    p.R = host_warmup(p.a, p.ns, lim);
    if (p.R >= lim) p.R = p.L;
    // chunks: ~kIirLanes lanes over all channels (the warm-up of R samples per chunk is
    // the price of more lanes: 1e8 x 3-axis, R = 3093, 32k / 64k / 128k / 256k lanes ran
    // 5.35 / 7.3 / 11.2 / 14.3 ms with 8-sample batches; round 3's 8k lanes and per-sample
    // loads 34 ms), at least 256 samples, and no shorter than R / 2 (the warm-up then costs
    // at most 2x the chunk's own work).
    const char* lenv = diag_env("MHF_IIR_LANES");          // diagnostics: lanes target
    const int64_t lanes = (lenv && atoll(lenv) > 0) ? atoll(lenv) : kIirLanes;
    const int64_t want = (p.L * channels + lanes - 1) / lanes;
    p.M = want > 256 ? want : 256;
    if (p.M < p.R / 2) p.M = p.R / 2;
    if (p.M > p.L) p.M = p.L;
    p.K = (p.L + p.M - 1) / p.M;
    p.out = out; p.ocs = out_ch_stride; p.oss = out_sample_stride;
    p.out_f32 = out_dtype == MHF_OUT_F32;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const int64_t ybytes = mhf_filtfilt_workspace(n_samples, channels, nb, na);
    if (!workspace || workspace_bytes < ybytes) {
        char msg[160];
        snprintf(msg, sizeof(msg), "filtfilt workspace too small: %lld bytes needed "
                 "(mhf_filtfilt_workspace), %lld given", (long long)ybytes, (long long)workspace_bytes);
        return ffail(MHF_EINVAL, msg);
    }
    p.yf = static_cast<double*>(workspace);
    // the LDS-streamed passes (filtfilt_tile.hip) for AoS records of 1 or 3 channels with AoS
    // outputs; any other layout (and MHF_NO_IIR_TILE=1, diagnostic) the per-lane kernel
    const int64_t ob = out_dtype == MHF_OUT_F32 ? 4 : 8;
    const bool aos_in = (channels == 1 || ch_stride == 1) && sample_stride == channels;
    const bool aos_out = (channels == 1 || out_ch_stride == 1) && out_sample_stride == channels;
    if (aos_in && aos_out && (channels == 1 || channels == 3) &&
        reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % ob == 0 &&
        reinterpret_cast<uintptr_t>(workspace) % 16 == 0 && n_samples >= 64 && p.R < p.L &&
        !disabled("MHF_NO_IIR_TILE")) {
        IirTileArgs t{};
        for (int i = 0; i < kMaxTaps; ++i) { t.b[i] = p.b[i]; t.a[i] = p.a[i]; t.zi[i] = p.zi[i]; }
        t.ns = p.ns; t.channels = channels; t.x = x; t.n = n_samples; t.padlen = p.padlen;
        t.L = p.L; t.yr = p.yf; t.out = out; t.out_f32 = p.out_f32;
        auto ceil32 = [](int64_t v) { return (v + 31) / 32 * 32; };
        t.E0 = ceil32(p.R + p.padlen);     // pass-0 blocks start on x samples = 0 mod 32
        t.E1 = ceil32(p.R);
        // ~kIirTileGroups workgroups of U = 64 / C chunks (2 per CU), chunks
        // no shorter than the warm-up (which then costs at most as much as the chunk)
        const int64_t U = 64 / channels;
        const int64_t want = (p.L + kIirTileGroups * U - 1) / (kIirTileGroups * U);
        t.M = ceil32(want > p.R ? want : p.R);
        if (t.M < 64) t.M = 64;
        t.K = (p.L + t.M - 1) / t.M;
        if (static_cast<int64_t>(U) * t.M * channels * 8 < (int64_t(1) << 31)) {   // 32-bit DMA offsets
            const int rc = launch_filtfilt_tile(t, s);
            const hipError_t e = hipGetLastError();
            if (rc != MHF_OK) return ffail(rc, "unsupported filter size");
            if (e != hipSuccess) return ffail(MHF_EDEVICE, hipGetErrorString(e));
            return MHF_OK;
        }
    }
    int rc = launch_filtfilt(p, s);
    const hipError_t e = hipGetLastError();
    if (rc != MHF_OK) return ffail(rc, "unsupported filter size");
    if (e != hipSuccess) return ffail(MHF_EDEVICE, hipGetErrorString(e));
    return MHF_OK;
}

}  // extern "C"

// ---- accelerometer magnitude (inertial/accelerometer.py:198-225): elementwise, fp32
namespace mhf {
__global__ void __launch_bounds__(256) magnitude_kernel(const float* __restrict__ x, int64_t n,
                                                        int64_t ss, int64_t cs,
                                                        float* __restrict__ out) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const float* p = x + t * ss;
    const float vx = p[0], vy = p[cs], vz = p[2 * cs];
    out[t] = sqrtf((vx * vx + vy * vy) + vz * vz);
}
}  // namespace mhf

extern "C" int mhf_magnitude(const float* x, int64_t n_samples, int64_t sample_stride,
                             int64_t ch_stride, float* out, void* hip_stream) {
    using namespace mhf;
    set_error(MHF_OK, "");
    if (!x || !out) return set_error(MHF_EINVAL, "null x or out");
    if (n_samples < 0 || sample_stride < 1 || ch_stride < 0)
        return set_error(MHF_EINVAL, "n_samples >= 0, sample_stride >= 1, ch_stride >= 0");
    if (n_samples == 0) return MHF_OK;
    hipLaunchKernelGGL(magnitude_kernel, dim3(static_cast<unsigned>((n_samples + 255) / 256)),
                       dim3(256), 0, static_cast<hipStream_t>(hip_stream), x, n_samples,
                       sample_stride, ch_stride, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(MHF_EDEVICE, hipGetErrorString(e));
    return MHF_OK;
}
