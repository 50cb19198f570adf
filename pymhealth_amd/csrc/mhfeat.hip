// mhfeat.hip — MI355X (gfx950) sliding-window feature engine + its C-ABI (include/mhfeat.h).
//
// Replaces the compiled per-window loop of pymhealth's rolling_apply
// (src/mhealth/util/windows.py:68-91) for the feature functions listed in
// include/mhfeat.h, and the FFTW binder (src/mhealth/fft/_fftw_binder.py:11-17) that
// its spectral features would need, with fused HIP kernels:
//
//   * moments kernels (lane-per-window): every numba-faithful fp32/fp64 sequential
//     accumulation of SURVEY.md Appendix A runs in ONE lane in the reference's order,
//     so results are bit-identical to numba (no tree reductions for these features).
//   * spectral kernel (wave-per-window): real FFT of W samples as a W/2-point complex
//     Stockham FFT in LDS, periodogram, then band power / relative band power /
//     spectral entropy / dominant frequency with wave-shuffle reductions (1e-5 class).
//
// Numerics: compiled with -ffp-contract=off (no FMA contraction, every fp32 step is a
// separately rounded IEEE op as in numba) and default IEEE div/sqrt and f32 denormals.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../../include/mhfeat.h"
#include "engine_common.h"
#include "tile.hip.h"
#include "spectral_wave.h"
#include "spectral64.h"
#include "window_moments.h"
#include "tile_idx.h"

using namespace mhf;

namespace {

thread_local char g_err[512] = "";

ExtraParams extra_params(const mhf_params* p) {
    ExtraParams x;
    x.pnn_th = p ? p->pnn_threshold : 50.0;
    x.csi_factor = p ? p->csi_factor : 0.70710678118654746;   // 1 / np.sqrt(2)
    x.blk = 0;
    return x;
}

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

// ---- float64 input (mhf_window_features_f64). numba types every reduction from the input
// dtype, so a float64 window's features are the same reference functions with every
// intermediate in fp64: np.mean = sequential fp64 sum / n (row 0 and the parfor rows
// agree), np.var = sequential fp64 sum of (x - m)^2 / n, np.std its sqrt, skewness /
// kurtosis with per-element division by len(x) (rows for a 2-D block), gradient / diff
// in fp64. Lane per (window, channel), straight from global memory; pinned by
// tests/golden/f64_*.npz (oracle: mhf_oracle_window_features64).
struct MomArgs64 {
    const double* x;
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t channels;
    fmask_t mask;
    double th;      // zero-crossing threshold (|x| <= th counts as 0)
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    ExtraParams xp;
};

__device__ double var64_strided(const double* p, int64_t ss, int64_t n, int order) {
    // np.var of gradient(x) (order 1) or gradient(gradient(x)) (order 2), fp64
    auto g1 = [&](int64_t t) -> double {
        if (t == 0) return p[ss] - p[0];
        if (t == n - 1) return p[(n - 1) * ss] - p[(n - 2) * ss];
        return (p[(t + 1) * ss] - p[(t - 1) * ss]) / 2.0;
    };
    auto g = [&](int64_t t) -> double {
        if (order == 1) return g1(t);
        if (t == 0) return g1(1) - g1(0);
        if (t == n - 1) return g1(n - 1) - g1(n - 2);
        return (g1(t + 1) - g1(t - 1)) / 2.0;
    };
    double s = 0.0;
    for (int64_t t = 0; t < n; ++t) s = s + g(t);
    const double m = s / static_cast<double>(n);
    double ssd = 0.0;
    for (int64_t t = 0; t < n; ++t) {
        const double d = g(t) - m;
        ssd = ssd + d * d;
    }
    return ssd / static_cast<double>(n);
}

__device__ WinVals window_moments64(const double* p, int64_t ss, int64_t W, bool serial, fmask_t m,
                                    double th, const ExtraParams& xp) {
    WinVals r{};
    double c = 0.0, a = 0.0, ll = 0.0;
    double mn = p[0], mx = p[0];
    double pmin = INFINITY, pmax = -INFINITY, first_nan = 0.0;
    bool any_nan = false;
    int zc = 0, pk = 0;
    bool prevpos = !(fabs(p[0]) <= th) && p[0] > 0.0;
    for (int64_t t = 0; t < W; ++t) {
        const double v = p[t * ss];
        c = c + v;
        a = a + v * v;
        pmin = v < pmin ? v : pmin;
        pmax = v > pmax ? v : pmax;
        if (v != v && !any_nan) { any_nan = true; first_nan = v; }
        if (t > 0) {
            const double u = p[(t - 1) * ss];
            if (xp.blk == 0 || t % xp.blk != 0) ll = ll + fabs(v - u);
            const bool pos = !(fabs(v) <= th) && v > 0.0;
            zc += pos != prevpos;
            prevpos = pos;
            mn = v < mn ? v : mn;
            mx = v > mx ? v : mx;
            if (t + 1 < W) {
                const double w1 = p[(t + 1) * ss];
                pk += (v > u && v > w1);
            }
        }
    }
    const double Wd = static_cast<double>(W);
    const double mean = c / Wd;
    r.mean = r.mean32 = mean;
    r.rms = sqrt(a / Wd);
    r.zc = zc;
    r.peaks = pk;
    r.drange = mx - mn;
    r.ll = ll;
    r.vmin = (serial && any_nan) ? first_nan : pmin;
    r.vmax = (serial && any_nan) ? first_nan : pmax;
    double ssd = 0.0;
    for (int64_t t = 0; t < W; ++t) {
        const double d = p[t * ss] - mean;
        ssd = ssd + d * d;
    }
    const double var = ssd / Wd, sd = sqrt(var);
    r.var = r.var32 = var;
    r.std_ = r.std32 = sd;
    r.cv = sd / mean;
    if (m & (bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) | bit(MHF_KURTOSIS_EXCESS))) {
        const double rows = static_cast<double>(xp.blk > 0 ? W / xp.blk : W);
        double s3 = 0.0, s4 = 0.0;
        for (int64_t t = 0; t < W; ++t) {
            const double d = p[t * ss] - mean, q = d * d;
            s3 = s3 + (d * q) / rows;
            s4 = s4 + (q * q) / rows;
        }
        r.skew = sd == 0.0 ? 0.0 : s3 / (sd * (sd * sd));
        r.kurt = var == 0.0 ? 0.0 : s4 / (var * var);
        r.kurt_ex = r.kurt - 3.0;
    }
    if (m & kHjorthBits) {
        if (W < 2) {
            r.hj_mob = r.hj_cmp = NAN;
        } else {
            const double vg = var64_strided(p, ss, W, 1);
            r.hj_mob = sqrt(vg / var);
            if (m & bit(MHF_HJORTH_COMPLEXITY)) r.hj_cmp = sqrt(var64_strided(p, ss, W, 2) / vg) / r.hj_mob;
        }
    }
    if (m & kHrvBits) {
        const int64_t n = W - 1;
        if (n < 1) {
            r.rmssd = r.sdsd = r.ssd = r.pnnx = r.sd1 = r.sd2 = r.lcsi = r.lcvi = r.lmcsi = NAN;
        } else {
            const double nd = static_cast<double>(n);
            double sq = 0.0, sdd = 0.0, su = 0.0;
            int64_t cnt = 0;
            for (int64_t i = 1; i < W; ++i) {
                const double d = p[i * ss] - p[(i - 1) * ss];
                sq = sq + d * d;
                sdd = sdd + d;
                su = su + (p[i * ss] + p[(i - 1) * ss]);
                cnt += fabs(d) > xp.pnn_th;
            }
            const double md = sdd / nd, mu = su / nd;
            double vd = 0.0, vu = 0.0;
            for (int64_t i = 1; i < W; ++i) {
                const double e = (p[i * ss] - p[(i - 1) * ss]) - md;
                const double f = (p[i * ss] + p[(i - 1) * ss]) - mu;
                vd = vd + e * e;
                vu = vu + f * f;
            }
            r.rmssd = sqrt(sq / nd);
            r.ssd = sdd;
            r.pnnx = static_cast<double>(cnt) / nd;
            r.sdsd = sqrt(vd / nd);
            r.sd1 = xp.csi_factor * r.sdsd;
            r.sd2 = xp.csi_factor * sqrt(vu / nd);
            r.lcsi = r.sd1 / r.sd2;
            r.lcvi = log10(r.sd1 * r.sd2);
            r.lmcsi = (r.sd1 * r.sd1) / r.sd2;
        }
    }
    if (m & bit(MHF_ENTROPY)) {
        double s = 0.0, e = 0.0;
        for (int64_t t = 0; t < W; ++t) s = s + p[t * ss];
        for (int64_t t = 0; t < W; ++t) {
            const double q = p[t * ss] / s + 1e-30;
            e = e + q * log(q);
        }
        r.entx = -e;
    }
    return r;
}

// Dynamic LDS (unused) of the lane-walk kernels (generic, float64, indexed): it caps the
// resident 256-thread blocks per CU so the windows in flight keep their lines in L1 / L2
// between consecutive samples. 40 KiB = 4 blocks = 4 waves per SIMD (cfgidx A/B: 1.99 ms
// against 2.22 uncapped, 2.29 at 2 waves per SIMD); MHF_IDX_SHM (KiB) overrides it for
// timing diagnostics.
inline bool needs_ext(fmask_t mask, int32_t blk) {
    return (mask & (kHjorthBits | kHrvBits | bit(MHF_ENTROPY))) != 0 ||
           (blk > 0 && (mask & bit(MHF_LINE_LENGTH)) != 0);
}
inline size_t lane_walk_shm(int default_kib = 40) {
    const char* e = diag_env("MHF_IDX_SHM");
    return static_cast<size_t>(e ? atoi(e) : default_kib) * 1024;
}

__global__ void __launch_bounds__(256) moments_f64_kernel(MomArgs64 a) {
    // lane per (window, channel), a window's channels side by side (moments_indexed_kernel)
    const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t i = u / a.channels;
    const int c = static_cast<int>(u - i * a.channels);
    if (i >= a.nwin) return;
    const int64_t g = a.first + i;
    const double* p = a.x + c * a.ch_stride + g * a.wstep * a.sample_stride;
    const WinVals r = window_moments64(p, a.sample_stride, a.wsize, g == 0, a.mask, a.th, a.xp);
    for (int j = 0; j < a.feats.n; ++j)
        if (bit(a.feats.id[j]) & kMomentBits)   // order-statistic columns: order_kernel
            store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i,
                      pick_moment(r, a.feats.id[j]));
}

template <bool EXT>
__global__ void __launch_bounds__(256) moments_generic_kernel(MomArgs a) {
    // lane per (window, channel), a window's channels side by side (moments_indexed_kernel)
    const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t i = u / a.channels;
    const int c = static_cast<int>(u - i * a.channels);
    if (i >= a.nwin) return;
    const int64_t g = a.first + i;
    const float* p = a.x + c * a.ch_stride + g * a.wstep * a.sample_stride;
    const WinVals r = window_moments<EXT>(GlobAcc{p, a.sample_stride, a.wsize}, a.wsize, g == 0, a.mask, a.t32, a.xp);
    for (int j = 0; j < a.feats.n; ++j) {
        const int f = a.feats.id[j];
        if (bit(f) & kMomentBits)
            store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i,
                      pick_moment(r, f));
    }
}

// ======================================================================
// Span kernel (any W, S, strides, alignment): lane per (window, channel) like the generic
// kernel, but the block's U consecutive windows are first staged in LDS with coalesced
// loads — the union span [g0*S, (g0+U-1)*S + W) once, overlapping windows sharing it
//  — and every pass of window_moments reads LDS instead of issuing one
// uncoalesced global load per sample per pass. Layout: one plane per channel (pitch Q
// floats), rows of R = min(S, W) samples (pitch P floats, odd: the lanes of a b32 read
// hit distinct banks), row k = samples [(g0 + k) * S, (g0 + k) * S + R).
// ======================================================================
struct SpanArgs {
    MomArgs m;
    int32_t U, R, P, Q, nrows;
    uint32_t M;                  // ceil(2^32 / R) (SpanAcc, span staging)
    uint32_t MC;                 // ceil(2^32 / C) (span staging)
    uint32_t MRC;                // ceil(2^32 / (R * C)) (span staging)
    int32_t vec4;                // staging by 16-B loads: one contiguous channel, R = S, S and
                                 // W multiples of 4, 16-B aligned span starts
};
constexpr int kLoadBatch = 16;

constexpr int kSpanLdsBytes = 40 * 1024;   // 4 one-wave blocks per CU (one per SIMD)

template <bool EXT>
__global__ void __launch_bounds__(64) span_kernel(SpanArgs a) {
    extern __shared__ __attribute__((aligned(16))) float span_lds[];
    const MomArgs& m = a.m;
    const int lane = threadIdx.x;
    const int C = m.channels;
    const int r = lane / C, c = lane - (lane / C) * C;
    const int64_t S = m.wstep, W = m.wsize;
    const int64_t nblk = (m.nwin + a.U - 1) / a.U;
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const int64_t i0 = b * a.U;
        const int64_t g0 = m.first + i0;
        const int Ub = static_cast<int>(m.nwin - i0 < a.U ? m.nwin - i0 : a.U);
        const int64_t s0 = g0 * S;
        const int64_t send = (g0 + Ub - 1) * S + W;          // last sample + 1 of the span
        __syncthreads();                                      // previous block's reads done
        // stage the span: rows of R samples (row k starts at sample (g0 + k) * S), flat over
        // their (row, sample, channel) elements in memory order, kLoadBatch independent
        // loads per lane in flight before their LDS stores
        const int64_t nel = static_cast<int64_t>(a.nrows) * a.R * C;
        const uint32_t RC = static_cast<uint32_t>(a.R * C);
        if (a.vec4) {
            // rows of R = S samples are consecutive in memory: the span is one contiguous
            // run, read 16 B per lane, kLoadBatch loads in flight (4x the bytes of the
            // scalar loop below); every 4-sample group stays inside one row (R % 4 == 0)
            const float4* src = reinterpret_cast<const float4*>(m.x + s0);
            const int64_t n4 = (send - s0) / 4;
            for (int64_t e0 = 0; e0 < n4; e0 += 64 * kLoadBatch) {
                float4 v[kLoadBatch];
#pragma unroll
                for (int u = 0; u < kLoadBatch; ++u) {
                    const int64_t e = e0 + u * 64 + lane;
                    v[u] = e < n4 ? src[e] : float4{0.0f, 0.0f, 0.0f, 0.0f};
                }
#pragma unroll
                for (int u = 0; u < kLoadBatch; ++u) {
                    const uint32_t e = static_cast<uint32_t>(e0 + u * 64 + lane) * 4u;
                    if (e < static_cast<uint32_t>(4 * n4)) {
                        const uint32_t k = __umulhi(e, a.M);
                        const uint32_t at = k * a.P + (e - k * static_cast<uint32_t>(a.R));
                        span_lds[at] = v[u].x;
                        span_lds[at + 1] = v[u].y;
                        span_lds[at + 2] = v[u].z;
                        span_lds[at + 3] = v[u].w;
                    }
                }
            }
        } else
        for (int64_t e0 = 0; e0 < nel; e0 += 64 * kLoadBatch) {
            float v[kLoadBatch];
            uint32_t at[kLoadBatch];
#pragma unroll
            for (int u = 0; u < kLoadBatch; ++u) {
                const uint32_t e = static_cast<uint32_t>(e0 + u * 64 + lane);
                const uint32_t k = RC == 1 ? e : __umulhi(e, a.MRC);
                const uint32_t rem = e - k * RC;
                const uint32_t tt = C == 1 ? rem : __umulhi(rem, a.MC);
                const uint32_t cc = rem - tt * C;
                const int64_t smp = s0 + static_cast<int64_t>(k) * S + tt;
                const bool ok = e < nel && smp < send;
                at[u] = ok ? cc * a.Q + k * a.P + tt : 0xffffffffu;
                v[u] = ok ? m.x[cc * m.ch_stride + smp * m.sample_stride] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < kLoadBatch; ++u)
                if (at[u] != 0xffffffffu) span_lds[at[u]] = v[u];
        }
        __syncthreads();
        if (r < Ub) {
            const int64_t i = i0 + r;
            SpanAcc acc;
            acc.base = (lds_cfloat_t*)(span_lds + c * a.Q + r * a.P);
            acc.R = a.R;
            acc.P = a.P;
            acc.M = a.M;
            const WinVals v = window_moments<EXT>(acc, W, m.first + i == 0, m.mask, m.t32, m.xp);
            for (int j = 0; j < m.feats.n; ++j) {
                const int f = m.feats.id[j];
                if (bit(f) & kMomentBits)
                    store_out(m.out, m.out_f32, (static_cast<int64_t>(c) * m.feats.n + j) * m.out_ld + i,
                              pick_moment(v, f));
            }
        }
    }
}

// Span geometry for (C, W, S): windows per block U (as many as fit kSpanLdsBytes, at most
// 64 / C) and the LDS pitches. Returns false when fewer than kMinSpanUnits lanes would
// work (very long windows): the generic kernel then.
constexpr int kMinSpanUnits = 16;
bool span_plan(int32_t C, int64_t W, int64_t S, SpanArgs* a) {
    if (C < 1 || C > 64 || W > 65535) return false;
    const int64_t R = S < W ? S : W;
    if (R > 65535) return false;
    const int64_t P = R | 1;                                  // odd pitch
    const int64_t rows_w = (W + R - 1) / R;                  // rows one window spans
    int64_t U = 64 / C;
    auto bytes = [&](int64_t u, int64_t q) { return 4 * (C * q); };
    auto plane = [&](int64_t u) { return (u - 1 + rows_w) * P; };
    while (U > 0 && bytes(U, plane(U) + 32) > kSpanLdsBytes) --U;
    if (U * C < kMinSpanUnits && U < 64 / C) return false;
    if (U < 1) return false;
    // plane pitch: the offset (0..31) that spreads the lanes (3r + c ...) of each 32-lane
    // group over the most banks
    const int64_t base = plane(U);
    int64_t bestQ = base, best = 1 << 30;
    for (int64_t d = 0; d < (C > 1 ? 32 : 1); ++d) {
        const int64_t Q = base + d;
        int worst = 0;
        for (int g = 0; g < 2; ++g) {
            int cnt[32] = {0};
            for (int l = 32 * g; l < 32 * g + 32 && l < U * C; ++l) {
                const int64_t addr = (l % C) * Q + (l / C) * P;
                const int bk = static_cast<int>(addr % 32);
                if (++cnt[bk] > worst) worst = cnt[bk];
            }
        }
        if (worst < best) { best = worst; bestQ = Q; }
    }
    a->U = static_cast<int32_t>(U);
    a->R = static_cast<int32_t>(R);
    a->P = static_cast<int32_t>(P);
    a->Q = static_cast<int32_t>(bestQ);
    a->nrows = static_cast<int32_t>(U - 1 + rows_w);
    a->M = R == 1 ? 0u : static_cast<uint32_t>(((uint64_t(1) << 32) + R - 1) / R);
    a->MC = C == 1 ? 0u : static_cast<uint32_t>(((uint64_t(1) << 32) + C - 1) / C);
    a->MRC = R * C == 1 ? 0u : static_cast<uint32_t>(((uint64_t(1) << 32) + R * C - 1) / (R * C));
    return true;
}


// ======================================================================
// Indexed windows: window i = samples [starts[i], ends[i]) of every channel, lengths
// vary; the reference's indices_rolling_apply loop (src/mhealth/util/windows.py:134-157)
// is a serial @jit loop, so every window gets the serial numerics, and a window shorter
// than min_len (or empty) is NaN for every feature.
// ======================================================================
struct IdxArgs {
    const float* x;
    int64_t n_samples, ch_stride, sample_stride, nwin, min_len;
    const int64_t* starts;
    const int64_t* ends;
    int32_t channels;
    fmask_t mask;
    float t32;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    ExtraParams xp;
};

// Lane per (window, channel), the C channel lanes of a window side by side (AoS records:
// one pass over a window's lines serves all its channels at once, instead of C blocks
// re-reading them at different times); the launch caps the waves per CU with dynamic LDS
// so the windows in flight keep their lines in L1 / L2 between consecutive samples.
template <bool EXT>
__global__ void __launch_bounds__(256) moments_indexed_kernel(IdxArgs a) {
    const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int C = a.channels;
    const int64_t i = u / C;
    const int c = static_cast<int>(u - i * C);
    if (i >= a.nwin) return;
    const int64_t si = a.starts[i], ei = a.ends[i];
    // arr[si:ei]: Python slice bounds (negative counts from the end, then clip to [0, n])
    const int64_t n = a.n_samples;
    int64_t s0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
    s0 = s0 < 0 ? 0 : (s0 > n ? n : s0);
    e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
    const int64_t W = e0 > s0 ? e0 - s0 : 0;
    const bool keep = (ei - si >= a.min_len) && W > 0;
    WinVals r;
    if (keep)
        r = window_moments<EXT>(GlobAcc{a.x + c * a.ch_stride + s0 * a.sample_stride, a.sample_stride, W},
                           W, true, a.mask, a.t32, a.xp);
    for (int j = 0; j < a.feats.n; ++j) {
        const int f = a.feats.id[j];
        if (!(bit(f) & kMomentBits)) continue;     // order statistics: order_kernel
        store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i,
                  keep ? pick_moment(r, f) : static_cast<double>(NAN));
    }
}

// float64 records (mhf_indexed_window_features_f64): the same slices through the fp64
// lane models (window_moments64; numba types the serial @jit function per dtype)
struct IdxArgs64 {
    const double* x;
    int64_t n_samples, ch_stride, sample_stride, nwin, min_len;
    const int64_t* starts;
    const int64_t* ends;
    int32_t channels;
    fmask_t mask;
    double th;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    ExtraParams xp;
};

__global__ void __launch_bounds__(256) moments_indexed_f64_kernel(IdxArgs64 a) {
    const int64_t u = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t i = u / a.channels;
    const int c = static_cast<int>(u - i * a.channels);
    if (i >= a.nwin) return;
    const int64_t si = a.starts[i], ei = a.ends[i];
    const int64_t n = a.n_samples;
    int64_t s0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
    s0 = s0 < 0 ? 0 : (s0 > n ? n : s0);
    e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
    const int64_t W = e0 > s0 ? e0 - s0 : 0;
    const bool keep = (ei - si >= a.min_len) && W > 0;
    WinVals r{};
    if (keep)
        r = window_moments64(a.x + c * a.ch_stride + s0 * a.sample_stride, a.sample_stride, W, true,
                             a.mask, a.th, a.xp);
    for (int j = 0; j < a.feats.n; ++j) {
        const int f = a.feats.id[j];
        if (!(bit(f) & kMomentBits)) continue;     // order statistics: order_kernel
        store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i,
                  keep ? pick_moment(r, f) : static_cast<double>(NAN));
    }
}

// Longest kept window of an indexed launch (clamped slice length of every window with
// end - start >= min_len): sizes the order-statistic / sampen / RQA launches, which stage a
// whole window on chip. One atomic max per wave.
__global__ void __launch_bounds__(256) indexed_max_len_kernel(const int64_t* starts, const int64_t* ends,
                                                              int64_t nwin, int64_t n, int64_t min_len,
                                                              unsigned long long* out) {
    unsigned long long m = 0;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nwin;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t si = starts[i], ei = ends[i];
        int64_t s0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
        s0 = s0 < 0 ? 0 : (s0 > n ? n : s0);
        e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
        const int64_t W = e0 > s0 ? e0 - s0 : 0;
        if (ei - si >= min_len && static_cast<unsigned long long>(W) > m) m = W;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(m, o, 64);
        m = w > m ? w : m;
    }
    if ((threadIdx.x & 63) == 0 && m > 0) atomicMax(out, m);
}

// get_indices (windows.py:162-178): window i starts at t0 + i * step and ends wsize
// later; starts/ends = np.searchsorted(index, ., side='left') over the sorted index.
// numpy picks the arithmetic per bound: starts = np.arange(index[0], index[-1], wstep) is
// int64 for an integer step and float64 otherwise (then start_i = t0 + i * delta with
// delta = (t0 + step) - t0, arange's fill rule); ends = starts + wsize is float64 when
// either operand is, and then so is np.concatenate((starts, ends)): every bound is
// compared in float64, with the int64 index element converted as numpy does.
struct BoundsArgs {
    const int64_t* index;
    int64_t n, nwin;
    int32_t mode;
    int64_t t0_i, step_i, wsize_i;
    double t0_f, delta_f, wsize_f;
    int64_t* starts;
    int64_t* ends;
};

__device__ __forceinline__ int64_t lower_bound_i(const int64_t* idx, int64_t n, int64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (idx[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t lower_bound_f(const int64_t* idx, int64_t n, double v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (static_cast<double>(idx[mid]) < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(256) window_bounds_kernel(BoundsArgs a) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.nwin) return;
    if (a.mode & MHF_BOUNDS_FLOAT_STARTS) {
        const double s = a.t0_f + static_cast<double>(i) * a.delta_f;
        a.starts[i] = lower_bound_f(a.index, a.n, s);
        a.ends[i] = lower_bound_f(a.index, a.n, s + a.wsize_f);
    } else {
        const int64_t s = a.t0_i + i * a.step_i;
        if (a.mode & MHF_BOUNDS_FLOAT_ENDS) {
            // np.concatenate((starts, ends)) is float64: the int starts are compared as
            // float64 too
            const double sf = static_cast<double>(s);
            a.starts[i] = lower_bound_f(a.index, a.n, sf);
            a.ends[i] = lower_bound_f(a.index, a.n, sf + a.wsize_f);
        } else {
            a.starts[i] = lower_bound_i(a.index, a.n, s);
            a.ends[i] = lower_bound_i(a.index, a.n, s + a.wsize_i);
        }
    }
}

// ======================================================================
// Spectral: one wavefront per window. rFFT(W) = W/2-point complex Stockham radix-2
// FFT in LDS + the real-input post-processing, periodogram, band sums, entropy and
// first-argmax dominant frequency.
// ======================================================================
struct SpecArgs {
    const float* x;
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t pow2;
    int32_t band_lo, band_hi;   // inclusive bin range (band_lo > band_hi: empty)
    int32_t dom_lo, dom_hi;     // [dom_lo, dom_hi)
    float scale;                // 1 / (fs * W)
    double freq_step;           // freqs[k] = k * freq_step (numpy.fft.rfftfreq)
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// first-argmax with numpy semantics: the first NaN wins, else the first max
__device__ __forceinline__ void argmax_merge(float& bv, int& bk, float ov, int ok) {
    const bool onan = ok >= 0 && (ov != ov);
    const bool bnan = bk >= 0 && (bv != bv);
    bool take;
    if (ok < 0) take = false;
    else if (bk < 0) take = true;
    else if (bnan || onan) take = onan && (!bnan || ok < bk);
    else take = (ov > bv) || (ov == bv && ok < bk);
    if (take) { bv = ov; bk = ok; }
}

// windows (waves) per block: 4 up to W = 1024, fewer above so the block fits the LDS
inline int spec_waves(int64_t W) { return W <= 1024 ? 4 : (W <= 2048 ? 2 : 1); }

__global__ void __launch_bounds__(256) spectral_kernel(SpecArgs a) {
    const int kSpecWaves = blockDim.x >> 6;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int W = static_cast<int>(a.wsize);
    const int N = W / 2;                    // complex FFT length (pow2 path)
    const int nb = W / 2 + 1;
    float2* tw = reinterpret_cast<float2*>(smem);                      // W entries
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* wbase = smem + 2 * W + wid * (2 * W + 2 * nb + 2);
    float2* buf0 = reinterpret_cast<float2*>(wbase);                   // W floats
    float2* buf1 = reinterpret_cast<float2*>(wbase + W);               // W floats
    float* psd = wbase + 2 * W;                                        // nb floats (+pad)
    const int c = blockIdx.y;

    // twiddles T[m] = exp(-2 pi i m / W), m in [0, W), computed once per block in fp64
    for (int m = threadIdx.x; m < W; m += blockDim.x) {
        double s, co;
        sincospi(-2.0 * static_cast<double>(m) / static_cast<double>(W), &s, &co);
        tw[m] = make_float2(static_cast<float>(co), static_cast<float>(s));
    }
    __syncthreads();

    for (int64_t base = static_cast<int64_t>(blockIdx.x) * kSpecWaves; base < a.nwin;
         base += static_cast<int64_t>(gridDim.x) * kSpecWaves) {
        const int64_t i = base + wid;
        const bool valid = i < a.nwin;
        const int64_t g = a.first + (valid ? i : 0);
        const float* p = a.x + c * a.ch_stride + g * a.wstep * a.sample_stride;
        float* b0f = reinterpret_cast<float*>(buf0);
        // load, then remove the window mean (any estimate): the fp32 FFT error then scales
        // with the AC energy, not the DC energy; the DC bin is restored as W*mean + sum(d)
        float lsum = 0.0f;
        if (valid)
            for (int t = lane; t < W; t += 64) {
                const float v = p[static_cast<int64_t>(t) * a.sample_stride];
                b0f[t] = v;
                lsum += v;
            }
        const float wmean = wave_sum(lsum) / static_cast<float>(W);
        if (valid)
            for (int t = lane; t < W; t += 64) b0f[t] -= wmean;
        const float dc = static_cast<float>(W) * wmean;
        __syncthreads();

        if (a.pow2) {
            // Stockham radix-2 over N complex points z_n = x_2n + i x_2n+1
            float2* src = buf0;
            float2* dst = buf1;
            for (int Ns = 1; Ns < N; Ns <<= 1) {
                for (int j = lane; j < N / 2; j += 64) {
                    const int k = j & (Ns - 1);
                    const float2 u = src[j];
                    const float2 v0 = src[j + N / 2];
                    const float2 w = tw[k * (N / Ns)];    // exp(-2 pi i k / (2 Ns))
                    const float2 v = make_float2(v0.x * w.x - v0.y * w.y, v0.x * w.y + v0.y * w.x);
                    const int d = (j - k) * 2 + k;
                    dst[d] = make_float2(u.x + v.x, u.y + v.y);
                    dst[d + Ns] = make_float2(u.x - v.x, u.y - v.y);
                }
                __syncthreads();
                float2* t = src; src = dst; dst = t;
            }
            // real-input post-processing: X_k = E_k + T[k] O_k
            for (int k = lane; k < nb; k += 64) {
                const float2 zk = src[k & (N - 1)];
                const float2 zn = src[(N - k) & (N - 1)];
                const float er = 0.5f * (zk.x + zn.x), ei = 0.5f * (zk.y - zn.y);
                const float orr = 0.5f * (zk.y + zn.y), oi = -0.5f * (zk.x - zn.x);
                const float2 w = (k < N) ? tw[k] : make_float2(-1.0f, 0.0f);
                const float xr = er + (orr * w.x - oi * w.y) + (k == 0 ? dc : 0.0f);
                const float xi = ei + (orr * w.y + oi * w.x);
                float pw = (xr * xr + xi * xi) * a.scale;
                if (k >= 1 && k < N) pw *= 2.0f;
                psd[k] = pw;
            }
        } else {
            // direct DFT with exact integer phase reduction (non power-of-two W)
            for (int k = lane; k < nb; k += 64) {
                float sr = 0.0f, si = 0.0f;
                int ph = 0;
                for (int t = 0; t < W; ++t) {
                    const float2 w = tw[ph];
                    const float xv = b0f[t];
                    sr += xv * w.x;
                    si += xv * w.y;
                    ph += k;
                    if (ph >= W) ph -= W;
                }
                if (k == 0) sr += dc;
                float pw = (sr * sr + si * si) * a.scale;
                const bool dbl = (W & 1) ? (k >= 1) : (k >= 1 && k < nb - 1);
                if (dbl) pw *= 2.0f;
                psd[k] = pw;
            }
        }
        __syncthreads();

        // band / total sums, first-argmax
        float bp = 0.0f, tot = 0.0f;
        float bv = 0.0f;
        int bk = -1;
        for (int k = lane; k < nb; k += 64) {
            const float v = psd[k];
            const float av = fabsf(v);
            tot += av;
            if (k >= a.band_lo && k <= a.band_hi) bp += av;
            if (k >= a.dom_lo && k < a.dom_hi) argmax_merge(bv, bk, v, k);
        }
        bp = wave_sum(bp);
        tot = wave_sum(tot);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int ok = __shfl_xor(bk, o, 64);
            argmax_merge(bv, bk, ov, ok);
        }
        // entropy: p = psd / sum(psd) + 1e-30; -sum(p log p)
        float ent = 0.0f;
        const float ssum = tot;  // psd >= 0, so sum(psd) == sum(|psd|) (NaN propagates)
        for (int k = lane; k < nb; k += 64) {
            const float q = psd[k] / ssum + 1e-30f;
            ent += q * logf(q);
        }
        ent = -wave_sum(ent);

        if (valid && lane == 0) {
            for (int j = 0; j < a.feats.n; ++j) {
                const int f = a.feats.id[j];
                double v;
                if (f == MHF_BAND_POWER) v = bp;
                else if (f == MHF_REL_BAND_POWER) v = bp / tot;
                else if (f == MHF_SPECTRAL_ENTROPY) v = ent;
                else if (f == MHF_DOMINANT_FREQ) v = (bk < 0) ? NAN : static_cast<double>(bk) * a.freq_step;
                else continue;
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i, v);
            }
        }
        __syncthreads();
    }
}

}  // namespace

namespace {

// ------------------------------------------------------------------ host helpers
int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}

// spectral bin ranges over numpy.fft.rfftfreq(W, 1/fs), evaluated exactly as numpy does:
// power_band keeps lo <= f <= hi (hrv.py:173-179), peak_frequency [first_index(lo),
// first_index(hi)) (density.py:9-32); NaN bounds are the reference's None
void spectral_bins(const mhf_params* params, int64_t wsize, int32_t* blo, int32_t* bhi,
                   int32_t* dlo, int32_t* dhi, double* step_out) {
    const int64_t nb = wsize / 2 + 1;
    const double d = 1.0 / params->fs;
    const double step = 1.0 / (static_cast<double>(wsize) * d);
    const double lo = std::isnan(params->band_lo) ? 0.0 * step : params->band_lo;
    const double hi = std::isnan(params->band_hi) ? static_cast<double>(nb - 1) * step : params->band_hi;
    *blo = static_cast<int32_t>(nb);
    for (int64_t k = 0; k < nb; ++k) if (static_cast<double>(k) * step >= lo) { *blo = (int32_t)k; break; }
    *bhi = -1;
    for (int64_t k = nb - 1; k >= 0; --k) if (static_cast<double>(k) * step <= hi) { *bhi = (int32_t)k; break; }
    *dlo = 0;
    if (!std::isnan(params->dom_lo)) {
        *dlo = static_cast<int32_t>(nb);
        for (int64_t k = 0; k < nb; ++k) if (params->dom_lo <= static_cast<double>(k) * step) { *dlo = (int32_t)k; break; }
    }
    *dhi = static_cast<int32_t>(nb);
    if (!std::isnan(params->dom_hi)) {
        for (int64_t k = 0; k < nb; ++k) if (params->dom_hi <= static_cast<double>(k) * step) { *dhi = (int32_t)k; break; }
    }
    *step_out = step;
}

float zc_threshold32(double th) {
    const double t = th > 0.0 ? th : 0.0;
    float t32 = static_cast<float>(t);
    if (static_cast<double>(t32) > t) t32 = nextafterf(t32, -INFINITY);
    return t32;
}

struct Plan {
    fmask_t mask = 0;
    bool moments = false, spectral = false, sort = false;
    bool sampen = false;
    bool rqa = false;
    bool fast = false;  // specialised fused register kernel (tile.hip.h)
    bool span = false;  // moments through the LDS span kernel (else the generic kernel)
    bool tilefix = false;  // moments through the fixed-window register tile (tile_idx.hip.h)
                           // when x is 4-B aligned (else span / generic)
    SpanArgs sa{};
    const char* name = nullptr;
};

thread_local char g_plan_name[96];

void name_plan(Plan* pl, int64_t wsize, int32_t channels) {
    const char* parts[3] = {nullptr, nullptr, nullptr};
    if (pl->fast) parts[0] = fast_plan_name(wsize, channels);
    else if (pl->moments) parts[0] = pl->tilefix ? "tile_fix" : pl->span ? "span" : "moments_generic";
    if (!pl->fast && pl->spectral) {
        const bool wave = spectral_wave_ok(wsize);
        parts[1] = (wave && spectral_reg_ok(wsize)) ? "spectral_reg" : wave ? "spectral_wave" : "spectral";
    }
    static const char* kPairNames[8] = {nullptr, "order", "sampen", "order+sampen", "rqa",
                                        "order+rqa", "sampen+rqa", "order+sampen+rqa"};
    parts[2] = kPairNames[(pl->sort ? 1 : 0) | (pl->sampen ? 2 : 0) | (pl->rqa ? 4 : 0)];
    char* o = g_plan_name;
    o[0] = 0;
    for (const char* part : parts) {
        if (!part) continue;
        if (o[0]) strncat(o, "+", sizeof(g_plan_name) - strlen(o) - 1);
        strncat(o, part, sizeof(g_plan_name) - strlen(o) - 1);
    }
    pl->name = o;
}

// windows of up to 288 samples at any step (non-power-of-two W, overlapping windows): the
// register tile of the indexed path, each window read once (ovl250: 6.54 -> 3.74 ms against
// the span kernel, round 5); MHF_NO_TILE_FIX=1 takes the span kernel (diagnostic)
bool tile_fix_plan(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                   fmask_t mask) {
    return !disabled("MHF_NO_TILE_FIX") && (mask & kMomentBits) &&
           tile_fix_ok(channels, ch_stride, sample_stride, wsize, mask & kMomentBits);
}

int make_plan(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
              int64_t wstep, const int32_t* features, int32_t n_features, int32_t out_dtype,
              Plan* pl) {
    if (channels < 1) return fail(MHF_EINVAL, "channels must be >= 1 (got %d)", channels);
    if (wsize < 1 || wstep < 1) return fail(MHF_EINVAL, "wsize and wstep must be >= 1");
    if (sample_stride < 1 || ch_stride < 0)
        return fail(MHF_EINVAL, "sample_stride must be >= 1 and ch_stride >= 0");
    if (n_features < 1 || n_features > kMaxFeatures || !features)
        return fail(MHF_EINVAL, "n_features must be in [1, %d]", kMaxFeatures);
    if (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32)
        return fail(MHF_EINVAL, "out_dtype must be MHF_OUT_F64 or MHF_OUT_F32");
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES)
            return fail(MHF_EINVAL, "unknown feature id %d", features[j]);
        pl->mask |= bit(features[j]);
    }
    pl->moments = (pl->mask & kMomentBits) != 0;
    pl->spectral = (pl->mask & kSpectralBits) != 0;
    pl->sort = (pl->mask & kOrderBits) != 0;
    pl->sampen = (pl->mask & kSampenBits) != 0;
    pl->rqa = (pl->mask & kRqaBits) != 0;
    if (pl->rqa && 2 * wsize + 2 > kMaxOrderSamples)
        return fail(MHF_EUNSUPPORTED, "recurrence quantification takes windows of up to %lld samples",
                    (long long)(kMaxOrderSamples / 2 - 1));
    if (pl->sampen && wsize > kMaxOrderSamples)
        return fail(MHF_EUNSUPPORTED, "sampen takes windows of up to %lld samples",
                    (long long)kMaxOrderSamples);
    if (pl->sort) {
        int64_t cap = 64;
        while (cap < wsize) cap <<= 1;
        if (cap * channels > kMaxOrderSamples)
            return fail(MHF_EUNSUPPORTED, "order statistics (median / percentile / "
                        "interquartile_range / mode) take windows of up to %lld samples x "
                        "channels after rounding up to a power of two (got %lld x %d)",
                        (long long)kMaxOrderSamples, (long long)wsize, channels);
    }
    if (pl->spectral && wsize > kMaxSpectralW)
        return fail(MHF_EUNSUPPORTED, "spectral features need wsize <= %lld", (long long)kMaxSpectralW);
    pl->fast = (pl->moments || pl->spectral) &&
               fast_plan_ok(channels, ch_stride, sample_stride, wsize, wstep, pl->mask);
    // diagnostics only: MHF_FORCE_GENERIC=1 (with MHF_DIAGNOSTICS=1) routes every request to
    // the generic kernels
    const bool force_generic = disabled("MHF_FORCE_GENERIC");
    if (force_generic) pl->fast = false;
    pl->span = !force_generic && pl->moments && span_plan(channels, wsize, wstep, &pl->sa);
    pl->tilefix = !force_generic && !pl->fast &&
                  tile_fix_plan(channels, ch_stride, sample_stride, wsize, pl->mask);
    name_plan(pl, wsize, channels);
    return MHF_OK;
}

// order statistics and sample entropy: their own launches after the moment / spectral
// ones (same output planes, other columns)
int order_launches(const Plan& pl, const OrderLaunch& L, const mhf_params* params,
                   hipStream_t stream) {
    if (pl.sort) {
        const double q = L.q;
        if (!(q >= 0.0 && q <= 100.0))
            return fail(MHF_EINVAL, "percentile_q must be in [0, 100] (numba raises ValueError)");
        if (launch_order(L, stream) != MHF_OK)
            return fail(MHF_EUNSUPPORTED, "order statistics: window too long for LDS");
    }
    if (pl.sampen) {
        const double mmd = params ? params->sampen_m : 2.0;
        const int32_t mm = static_cast<int32_t>(mmd);
        if (!(mmd >= 0.0) || static_cast<double>(mm) != mmd || mm > 65535)
            return fail(MHF_EINVAL, "sampen_m must be a non-negative integer");
        const double r = params ? params->sampen_r : 0.2;
        const double sd = params ? params->sampen_sd : static_cast<double>(NAN);
        if (launch_sampen(L, mm, r, sd, stream) != MHF_OK)
            return fail(MHF_EUNSUPPORTED, "sampen: window too long for LDS");
    }
    if (pl.rqa) {
        const double radius = params ? params->rqa_radius : 0.0;
        const double mld = params ? params->rqa_minlen : 2.0;
        const int32_t minlen = static_cast<int32_t>(mld);
        if (!(mld >= 1.0) || static_cast<double>(minlen) != mld)
            return fail(MHF_EINVAL, "rqa_minlen must be an integer >= 1");
        OrderLaunch Lr = L;
        if (Lr.starts) Lr.max_w = Lr.xd ? (kOrderLdsBytes / 4 - 2) / 3 : kMaxOrderSamples / 2 - 1;
        if (launch_rqa(Lr, radius, minlen, stream) != MHF_OK)
            return fail(MHF_EUNSUPPORTED, "rqa: window too long for LDS");
    }
    return MHF_OK;
}

}  // namespace

int mhf::set_error(int code, const char* msg) { return fail(code, "%s", msg); }

// ====================================================================== C-ABI
extern "C" {

int mhf_version(void) { return MHF_ABI_VERSION; }

const char* mhf_last_error(void) { return g_err; }

int64_t mhf_num_windows(int64_t n, int64_t w, int64_t s) {
    if (w < 1 || s < 1 || n < 0) return -1;
    const int64_t nw = 1 + floordiv(n - w, s);
    return nw > 0 ? nw : 0;
}

int64_t mhf_algorithmic_bytes(int64_t n_samples, int32_t channels, int64_t wsize, int64_t wstep,
                              int64_t n_windows, int32_t n_features, int32_t out_dtype) {
    (void)n_samples;
    if (n_windows <= 0) return 0;
    const int64_t samples = (wstep >= wsize) ? n_windows * wsize : (n_windows - 1) * wstep + wsize;
    const int64_t ob = (out_dtype == MHF_OUT_F32) ? 4 : 8;
    return static_cast<int64_t>(channels) * (samples * 4 + n_windows * n_features * ob);
}

const char* mhf_plan_name_f64(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                              int64_t wsize, int64_t wstep, const int32_t* features,
                              int32_t n_features, int32_t out_dtype) {
    if (channels < 1 || wsize < 1 || wstep < 1 || n_features < 1 || n_features > kMaxFeatures ||
        !features || (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32))
        return nullptr;
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return nullptr;
        mask |= bit(features[j]);
    }
    // alignment is the caller's to keep (a 16-B aligned record assumed here)
    const double* aligned = reinterpret_cast<const double*>(uintptr_t(256));
    const char* parts[3] = {
        !(mask & kMomentBits) ? nullptr
        : tile64_plan_ok(channels, ch_stride, sample_stride, wsize, wstep, mask, 0, aligned)
            ? "tile64" : "moments_f64",
        (mask & kSpectralBits) ? "spectral64" : nullptr,
        (mask & (kOrderBits | kSampenBits | kRqaBits)) ? "order/pairwise" : nullptr};
    char* o = g_plan_name;
    o[0] = 0;
    for (const char* part : parts) {
        if (!part) continue;
        if (o[0]) strncat(o, "+", sizeof(g_plan_name) - strlen(o) - 1);
        strncat(o, part, sizeof(g_plan_name) - strlen(o) - 1);
    }
    return g_plan_name;
}

const char* mhf_plan_name(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                          int64_t wsize, int64_t wstep, const int32_t* features,
                          int32_t n_features, int32_t out_dtype) {
    Plan pl;
    if (make_plan(channels, ch_stride, sample_stride, wsize, wstep, features, n_features,
                  out_dtype, &pl) != MHF_OK)
        return nullptr;
    return pl.name;
}

int mhf_window_features(const float* x, int64_t n_samples, int32_t channels, int64_t ch_stride,
                        int64_t sample_stride, int64_t wsize, int64_t wstep, int64_t first_window,
                        int64_t n_windows, const int32_t* features, int32_t n_features,
                        const mhf_params* params, int32_t numerics, int32_t out_dtype, void* out,
                        int64_t out_ld, void* hip_stream) {
    g_err[0] = 0;
    Plan pl;
    int rc = make_plan(channels, ch_stride, sample_stride, wsize, wstep, features, n_features,
                       out_dtype, &pl);
    if (rc != MHF_OK) return rc;
    if (pl.fast && reinterpret_cast<uintptr_t>(x) % 16 != 0) {  // DMA needs 16-B
        pl.fast = false;
        pl.tilefix = tile_fix_plan(channels, ch_stride, sample_stride, wsize, pl.mask);
    }
    const int32_t blk = numerics >> 8;
    if ((numerics & 0xff & ~MHF_NUMERICS_EXACT_VAR) != MHF_NUMERICS_REFERENCE || blk < 0)
        return fail(MHF_EINVAL, "unknown numerics mode %d", numerics);
    const bool exact_var = (numerics & MHF_NUMERICS_EXACT_VAR) != 0;
    if (blk > 0) {
        if (channels != 1 || wsize % blk != 0 || wstep % blk != 0 || n_samples % blk != 0)
            return fail(MHF_EINVAL, "MHF_NUMERICS_BLOCK(%d): one flat channel, n_samples, wsize "
                        "and wstep multiples of %d", blk, blk);
        if (pl.mask & ~kBlockBits)
            return fail(MHF_EUNSUPPORTED, "feature not defined on 2-D windows (the reference "
                        "fails on (rows, %d) blocks)", blk);
        if (pl.fast || pl.span || pl.tilefix) {   // tile / span plans assume the 1-D record
            pl.fast = false;
            pl.span = false;
            pl.tilefix = false;
            pl.moments = (pl.mask & kMomentBits) != 0;
        }
    }
    const int64_t nw_all = mhf_num_windows(n_samples, wsize, wstep);
    if (nw_all < 0) return fail(MHF_EINVAL, "n_samples must be >= 0");
    if (first_window < 0 || n_windows < 0 || first_window + n_windows > nw_all)
        return fail(MHF_EINVAL, "window range [%lld, %lld) outside [0, %lld)", (long long)first_window,
                    (long long)(first_window + n_windows), (long long)nw_all);
    if (out_ld < n_windows) return fail(MHF_EINVAL, "out_ld < n_windows");
    if (n_windows == 0) return MHF_OK;
    if (!x || !out) return fail(MHF_EINVAL, "null x or out");
    if (pl.spectral && !(params && params->fs > 0.0))
        return fail(MHF_EINVAL, "spectral features need params->fs > 0");
    hipStream_t stream = static_cast<hipStream_t>(hip_stream);

    FeatList fl;
    fl.n = n_features;
    for (int j = 0; j < n_features; ++j) fl.id[j] = features[j];
    const double th = params ? params->zc_threshold : 0.0;
    const float t32 = zc_threshold32(th);
    const bool pow2 = (wsize & (wsize - 1)) == 0;
    const bool fft_pow2 = pow2 && wsize >= 2;   // W = 1 goes through the direct DFT

    int32_t blo = 0, bhi = -1, dlo = 0, dhi = 0;
    double step = 0.0;
    if (pl.spectral) spectral_bins(params, wsize, &blo, &bhi, &dlo, &dhi, &step);

    if (pl.fast) {
        FastArgs fa;
        fa = FastArgs{};
        fa.x = x; fa.ch_stride = ch_stride; fa.sample_stride = sample_stride; fa.wstep = wstep;
        fa.first = first_window; fa.nwin = n_windows; fa.channels = channels;
        fa.mask = pl.mask; fa.t32 = t32; fa.feats = fl; fa.out = out; fa.out_ld = out_ld;
        fa.out_f32 = out_dtype == MHF_OUT_F32;
        fa.band_lo = blo; fa.band_hi = bhi; fa.dom_lo = dlo; fa.dom_hi = dhi;
        fa.scale = pl.spectral ? static_cast<float>(1.0 / (params->fs * static_cast<double>(wsize))) : 0.0f;
        fa.freq_step = step;
        fa.exact_var = exact_var;
        if (pl.spectral) {
            // bin weights of the in-lane spectral code (spectral_lane.hip.inc): pair k
            // holds bins (k, N-k), pair 0 = (0, N), pair N/2 = (N/2, none)
            const int64_t N = wsize / 2;
            for (int64_t k = 0; k <= N / 2; ++k) {
                const int64_t b0 = k, b1 = (k == 0) ? N : (2 * k == N ? -1 : N - k);
                fa.spec.bw[2 * k] = (b0 >= blo && b0 <= bhi) ? 1.0f : 0.0f;
                fa.spec.bw[2 * k + 1] = (b1 >= 0 && b1 >= blo && b1 <= bhi) ? 1.0f : 0.0f;
            }
            for (int64_t b = 0; b <= N; ++b) {
                fa.spec.dw[2 * b] = (b >= dlo && b < dhi) ? 1.0f : -1.0f;
                fa.spec.dw[2 * b + 1] = 0.0f;
            }
        }
        rc = launch_fast(fa, wsize, stream);
        if (rc != MHF_OK) return rc;
    } else {
        if (pl.moments) {
            MomArgs a{};
            a.x = x; a.ch_stride = ch_stride; a.sample_stride = sample_stride; a.wsize = wsize;
            a.wstep = wstep; a.first = first_window; a.nwin = n_windows; a.channels = channels;
            a.mask = pl.mask; a.t32 = t32; a.invW = 1.0f / static_cast<float>(wsize);
            a.pow2 = pow2; a.feats = fl; a.out = out; a.out_ld = out_ld;
            a.out_f32 = out_dtype == MHF_OUT_F32;
            a.xp = extra_params(params);
            a.xp.blk = blk;
            if (pl.tilefix && reinterpret_cast<uintptr_t>(x) % 4 == 0) {
                IdxTileArgs t{};
                t.x = x; t.n_samples = n_samples; t.wsize = wsize; t.wstep = wstep;
                t.first = first_window; t.nwin = n_windows; t.min_len = 0;
                t.channels = channels; t.mask = pl.mask & kMomentBits; t.t32 = t32;
                t.xp = a.xp; t.feats = fl; t.out = out; t.out_ld = out_ld; t.out_f32 = a.out_f32;
                t.exact_var = exact_var;
                const int trc = launch_tile_fix(t, stream);
                if (trc != MHF_OK) return fail(trc, "tile_fix launch refused its arguments");
            } else if (pl.span) {
                SpanArgs sa = pl.sa;
                sa.m = a;
                sa.vec4 = channels == 1 && sample_stride == 1 && sa.R == wstep && wstep % 4 == 0 &&
                          wsize % 4 == 0 &&
                          reinterpret_cast<uintptr_t>(x + first_window * wstep) % 16 == 0;
                const int64_t nblk = (n_windows + sa.U - 1) / sa.U;
                const unsigned blocks = static_cast<unsigned>(nblk < 2048 ? nblk : 2048);
                const size_t lds = sizeof(float) * static_cast<size_t>(channels) * sa.Q;
                if (needs_ext(a.mask, a.xp.blk)) hipLaunchKernelGGL(span_kernel<true>, dim3(blocks), dim3(64), lds, stream, sa);
                else hipLaunchKernelGGL(span_kernel<false>, dim3(blocks), dim3(64), lds, stream, sa);
            } else {
                a.channels = channels;
                dim3 grid(static_cast<unsigned>((n_windows * channels + 255) / 256));
                // fixed windows: 3 waves per SIMD (53 KiB) measured best (forced-generic cfg2
                // 0.50 -> 0.44 ms at 8 loads per batch), the indexed kernel 4 (40 KiB)
                if (needs_ext(a.mask, a.xp.blk)) hipLaunchKernelGGL(moments_generic_kernel<true>, grid, dim3(256), lane_walk_shm(53), stream, a);
                else hipLaunchKernelGGL(moments_generic_kernel<false>, grid, dim3(256), lane_walk_shm(53), stream, a);
            }
        }
        if (pl.spectral && spectral_wave_ok(wsize)) {
            SpecWaveArgs s{};
            s.x = x; s.ch_stride = ch_stride; s.sample_stride = sample_stride; s.wstep = wstep;
            s.first = first_window; s.nwin = n_windows;
            s.band_lo = blo; s.band_hi = bhi; s.dom_lo = dlo; s.dom_hi = dhi;
            s.want_ent = (pl.mask & bit(MHF_SPECTRAL_ENTROPY)) != 0;
            s.scale = static_cast<float>(1.0 / (params->fs * static_cast<double>(wsize)));
            s.freq_step = step; s.feats = fl; s.out = out; s.out_ld = out_ld;
            s.out_f32 = out_dtype == MHF_OUT_F32;
            rc = launch_spectral_wave(s, wsize, channels, stream);
            if (rc != MHF_OK) return fail(rc, "spectral_wave launch refused");
        } else if (pl.spectral) {
            SpecArgs s{};
            s.x = x; s.ch_stride = ch_stride; s.sample_stride = sample_stride; s.wsize = wsize;
            s.wstep = wstep; s.first = first_window; s.nwin = n_windows; s.pow2 = fft_pow2;
            s.band_lo = blo; s.band_hi = bhi; s.dom_lo = dlo; s.dom_hi = dhi;
            s.scale = static_cast<float>(1.0 / (params->fs * static_cast<double>(wsize)));
            s.freq_step = step; s.feats = fl; s.out = out; s.out_ld = out_ld;
            s.out_f32 = out_dtype == MHF_OUT_F32;
            const int64_t nb = wsize / 2 + 1;
            const int wpb = spec_waves(wsize);
            const size_t lds = sizeof(float) * (2 * wsize + wpb * (2 * wsize + 2 * nb + 2));
            int64_t blocks = (n_windows + wpb - 1) / wpb;
            if (blocks > 8192) blocks = 8192;
            dim3 grid(static_cast<unsigned>(blocks), static_cast<unsigned>(channels));
            hipLaunchKernelGGL(spectral_kernel, grid, dim3(64 * wpb), lds, stream, s);
        }
    }
    if (pl.sort || pl.sampen || pl.rqa) {
        OrderLaunch L{};
        L.x = x; L.ch_stride = ch_stride; L.sample_stride = sample_stride; L.wsize = wsize;
        L.wstep = wstep; L.first = first_window; L.nwin = n_windows; L.channels = channels;
        L.n_samples = n_samples;
        L.q = params ? params->percentile_q : 50.0;
        L.feats = fl; L.out = out; L.out_ld = out_ld; L.out_f32 = out_dtype == MHF_OUT_F32;
        rc = order_launches(pl, L, params, stream);
        if (rc != MHF_OK) return rc;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "HIP launch failed: %s", hipGetErrorString(e));
    return MHF_OK;
}

int mhf_window_features_f64(const double* x, int64_t n_samples, int32_t channels, int64_t ch_stride,
                            int64_t sample_stride, int64_t wsize, int64_t wstep, int64_t first_window,
                            int64_t n_windows, const int32_t* features, int32_t n_features,
                            const mhf_params* params, int32_t numerics, int32_t out_dtype, void* out,
                            int64_t out_ld, void* hip_stream) {
    g_err[0] = 0;
    if (channels < 1) return fail(MHF_EINVAL, "channels must be >= 1 (got %d)", channels);
    if (wsize < 1 || wstep < 1) return fail(MHF_EINVAL, "wsize and wstep must be >= 1");
    if (sample_stride < 1 || ch_stride < 0)
        return fail(MHF_EINVAL, "sample_stride must be >= 1 and ch_stride >= 0");
    if (n_features < 1 || n_features > kMaxFeatures || !features)
        return fail(MHF_EINVAL, "n_features must be in [1, %d]", kMaxFeatures);
    if (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32)
        return fail(MHF_EINVAL, "out_dtype must be MHF_OUT_F64 or MHF_OUT_F32");
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES)
            return fail(MHF_EINVAL, "unknown feature id %d", features[j]);
        mask |= bit(features[j]);
    }
    if ((mask & kSpectralBits) && wsize > kMaxSpectralW)
        return fail(MHF_EUNSUPPORTED, "spectral features need wsize <= %lld", (long long)kMaxSpectralW);
    if ((mask & kSampenBits) && wsize * 8 > kOrderLdsBytes)
        return fail(MHF_EUNSUPPORTED, "float64 sampen takes windows of up to %lld samples",
                    (long long)(kOrderLdsBytes / 8));
    if ((mask & kRqaBits) && (3 * wsize + 2) * 4 > kOrderLdsBytes)
        return fail(MHF_EUNSUPPORTED, "float64 recurrence quantification takes windows of up to "
                    "%lld samples", (long long)((kOrderLdsBytes / 4 - 2) / 3));
    if (mask & kOrderBits) {
        const double q = params ? params->percentile_q : 50.0;
        if ((mask & bit(MHF_PERCENTILE)) && !(q >= 0.0 && q <= 100.0))
            return fail(MHF_EINVAL, "percentile_q must be in [0, 100] (numba raises ValueError)");
        int64_t cap = 64;
        while (cap < wsize) cap <<= 1;
        if (cap * channels * 8 > kOrderLdsBytes)
            return fail(MHF_EUNSUPPORTED, "float64 order statistics take windows of up to %lld "
                        "samples x channels after rounding up to a power of two (got %lld x %d)",
                        (long long)(kOrderLdsBytes / 8), (long long)wsize, channels);
    }
    const int32_t blk = numerics >> 8;
    if ((numerics & 0xff & ~MHF_NUMERICS_EXACT_VAR) != MHF_NUMERICS_REFERENCE || blk < 0)
        return fail(MHF_EINVAL, "unknown numerics mode %d", numerics);   // fp64 kernels: always exact
    if (blk > 0) {
        if (channels != 1 || wsize % blk != 0 || wstep % blk != 0 || n_samples % blk != 0)
            return fail(MHF_EINVAL, "MHF_NUMERICS_BLOCK(%d): one flat channel, n_samples, wsize "
                        "and wstep multiples of %d", blk, blk);
        if (mask & ~kBlockBits)
            return fail(MHF_EUNSUPPORTED, "feature not defined on 2-D windows");
    }
    const int64_t nw_all = mhf_num_windows(n_samples, wsize, wstep);
    if (nw_all < 0) return fail(MHF_EINVAL, "n_samples must be >= 0");
    if (first_window < 0 || n_windows < 0 || first_window + n_windows > nw_all)
        return fail(MHF_EINVAL, "window range [%lld, %lld) outside [0, %lld)", (long long)first_window,
                    (long long)(first_window + n_windows), (long long)nw_all);
    if (out_ld < n_windows) return fail(MHF_EINVAL, "out_ld < n_windows");
    if ((mask & kSpectralBits) && !(params && params->fs > 0.0))
        return fail(MHF_EINVAL, "spectral features need params->fs > 0");
    if (n_windows == 0) return MHF_OK;
    if (!x || !out) return fail(MHF_EINVAL, "null x or out");
    MomArgs64 a{};
    a.x = x; a.ch_stride = ch_stride; a.sample_stride = sample_stride; a.wsize = wsize;
    a.wstep = wstep; a.first = first_window; a.nwin = n_windows; a.mask = mask;
    a.th = params ? params->zc_threshold : 0.0;
    for (int j = 0; j < n_features; ++j) a.feats.id[j] = features[j];
    a.feats.n = n_features;
    a.out = out; a.out_ld = out_ld; a.out_f32 = out_dtype == MHF_OUT_F32;
    a.xp = extra_params(params);
    a.xp.blk = blk;
    if (mask & kMomentBits) {
        // diagnostics only: MHF_NO_TILE64=1 keeps the lane-per-window global-memory kernel
        static const bool no_tile64 = [] {
            const char* e = diag_env("MHF_NO_TILE64");
            return e && e[0] == '1';
        }();
        if (!no_tile64 && tile64_plan_ok(channels, ch_stride, sample_stride, wsize, wstep, mask, blk, x)) {
            // contiguous / AoS records, power-of-two W: the streamed LDS-DMA tile kernel
            Tile64Args t{};
            t.x = x; t.wsize = wsize; t.wstep = wstep; t.first = first_window; t.nwin = n_windows;
            t.channels = channels; t.mask = mask; t.th = a.th; t.feats = a.feats;
            t.out = out; t.out_ld = out_ld; t.out_f32 = a.out_f32;
            const int rc = launch_tile64(t, static_cast<hipStream_t>(hip_stream));
            if (rc != MHF_OK) return fail(rc, "tile64 launch refused its arguments");
        } else {
            a.channels = channels;
            dim3 grid(static_cast<unsigned>((n_windows * channels + 255) / 256));
            hipLaunchKernelGGL(moments_f64_kernel, grid, dim3(256), lane_walk_shm(),
                               static_cast<hipStream_t>(hip_stream), a);
        }
    }
    if (mask & kSpectralBits) {
        // the fp64 transform of the float64 window (fft/_fft.py:18-28 transforms
        // a.astype(complex128)), spectral64.hip
        Spec64Args s{};
        s.x = x; s.ch_stride = ch_stride; s.sample_stride = sample_stride; s.wsize = wsize;
        s.wstep = wstep; s.first = first_window; s.nwin = n_windows;
        double step = 0.0;
        spectral_bins(params, wsize, &s.band_lo, &s.band_hi, &s.dom_lo, &s.dom_hi, &step);
        s.freq_step = step;
        s.want_ent = (mask & bit(MHF_SPECTRAL_ENTROPY)) != 0;
        s.scale = 1.0 / (params->fs * static_cast<double>(wsize));
        s.feats = a.feats; s.out = out; s.out_ld = out_ld; s.out_f32 = a.out_f32;
        const int src = launch_spectral64(s, channels, static_cast<hipStream_t>(hip_stream));
        if (src != MHF_OK) return fail(src, "spectral64 launch refused its arguments");
    }
    if (mask & (kOrderBits | kSampenBits | kRqaBits)) {
        // order statistics (order_kernel<E, double>: 64-bit keys), sample entropy and RQA
        // (fp64 differences) of the float64 windows
        OrderLaunch L{};
        L.xd = x; L.ch_stride = ch_stride; L.sample_stride = sample_stride; L.wsize = wsize;
        L.wstep = wstep; L.first = first_window; L.nwin = n_windows; L.channels = channels;
        L.q = params ? params->percentile_q : 50.0;
        L.feats = a.feats; L.out = out; L.out_ld = out_ld; L.out_f32 = out_dtype == MHF_OUT_F32;
        Plan pl;
        pl.sort = (mask & kOrderBits) != 0;
        pl.sampen = (mask & kSampenBits) != 0;
        pl.rqa = (mask & kRqaBits) != 0;
        const int orc = order_launches(pl, L, params, static_cast<hipStream_t>(hip_stream));
        if (orc != MHF_OK) return orc;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "%s", hipGetErrorString(e));
    return MHF_OK;
}

}  // extern "C"

namespace {
// The caller's workspace of an indexed call (include/mhfeat.h): bytes [0, 256) hold the
// longest-window slot, the rest the keys of order statistics on windows past the LDS
// capacity (launch_order_long), kIdxKeyWaves windows at a time by default.
constexpr int64_t kIdxSlotBytes = 256;
constexpr int64_t kIdxKeyWaves = 256;
// LDS capacity of the indexed order-statistic launch (keys of one window, all channels)
int64_t indexed_lds_cap(int32_t channels, bool f64) {
    int64_t w = 1;
    while (w * 2 * channels * (f64 ? 8 : 4) <= kOrderLdsBytes) w *= 2;
    return w;
}
int64_t long_keys_per_wave(int64_t max_len, int32_t channels, bool f64) {
    int64_t cap = 1;
    while (cap < max_len) cap <<= 1;
    return static_cast<int64_t>(channels) * cap * (f64 ? 8 : 4);
}

// Longest kept window of an indexed call, read back to the host through the workspace
// slot: the one synchronisation of the indexed entry points, taken only when order
// statistics / sampen / RQA are asked for (their launch shape depends on it). Returns -1
// on a device error.
int64_t indexed_max_len(const int64_t* starts, const int64_t* ends, int64_t nwin, int64_t n,
                        int64_t min_len, unsigned long long* slot, hipStream_t stream) {
    unsigned long long h = 0;
    if (hipMemsetAsync(slot, 0, sizeof(*slot), stream) != hipSuccess) return -1;
    int64_t blocks = (nwin + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(indexed_max_len_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       stream, starts, ends, nwin, n, min_len, slot);
    if (hipMemcpyAsync(&h, slot, sizeof(h), hipMemcpyDeviceToHost, stream) != hipSuccess) return -1;
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    return static_cast<int64_t>(h);
}

// The order-statistic / sampen / RQA launches of an indexed call (both sample types):
// windows up to the LDS capacity L.max_w in the LDS kernels; longer order-statistic
// windows through launch_order_long (keys in global scratch); sampen / RQA windows past
// their LDS capacity are refused (MHF_EUNSUPPORTED), never written as NaN.
int indexed_order_launches(OrderLaunch& L, fmask_t mask, const mhf_params* params,
                           void* workspace, int64_t workspace_bytes, hipStream_t stream) {
    if (!workspace || workspace_bytes < kIdxSlotBytes)
        return fail(MHF_EINVAL, "indexed order statistics / sampen / RQA need a workspace of at "
                    "least %lld bytes (mhf_indexed_workspace), %lld given", (long long)kIdxSlotBytes,
                    (long long)workspace_bytes);
    const int64_t longest = indexed_max_len(L.starts, L.ends, L.nwin, L.n_samples, L.min_len,
                                            static_cast<unsigned long long*>(workspace), stream);
    if (longest < 0) return fail(MHF_EDEVICE, "indexed window lengths: %s", hipGetErrorString(hipGetLastError()));
    const bool f64 = L.xd != nullptr;
    if ((mask & kSampenBits) && longest > L.max_w)
        return fail(MHF_EUNSUPPORTED, "sampen takes indexed windows of up to %lld samples (longest "
                    "here: %lld)", (long long)L.max_w, (long long)longest);
    if (mask & kRqaBits) {
        const int64_t cap = f64 ? (kOrderLdsBytes / 4 - 2) / 3 : kMaxOrderSamples / 2 - 1;
        if (longest > cap)
            return fail(MHF_EUNSUPPORTED, "recurrence quantification takes windows of up to %lld "
                        "samples (longest here: %lld)", (long long)cap, (long long)longest);
    }
    if ((mask & kOrderBits) && longest > kMaxLongOrderSamples)
        return fail(MHF_EUNSUPPORTED, "order statistics take indexed windows of up to %lld samples "
                    "(longest here: %lld)", (long long)kMaxLongOrderSamples, (long long)longest);
    const bool long_order = (mask & kOrderBits) && longest > L.max_w;
    const int64_t per_wave = long_keys_per_wave(longest, L.channels, f64);
    const int64_t key_bytes = workspace_bytes - kIdxSlotBytes;
    if (long_order && key_bytes < per_wave)
        return fail(MHF_EINVAL, "indexed order statistics: the longest window (%lld samples) needs a "
                    "workspace of at least %lld bytes (mhf_indexed_workspace), %lld given",
                    (long long)longest, (long long)(kIdxSlotBytes + per_wave), (long long)workspace_bytes);
    L.skip_long = long_order ? 1 : 0;
    Plan pl;
    pl.sort = (mask & kOrderBits) != 0;
    pl.sampen = (mask & kSampenBits) != 0;
    pl.rqa = (mask & kRqaBits) != 0;
    int rc = order_launches(pl, L, params, stream);
    if (rc != MHF_OK) return rc;
    if (long_order) {
        rc = launch_order_long(L, longest, static_cast<char*>(workspace) + kIdxSlotBytes, key_bytes,
                               stream);
        if (rc != MHF_OK) return fail(rc, "order statistics of long indexed windows: launch failed");
    }
    return MHF_OK;
}

// the indexed tile path takes the call's moment features (cfgidx: 1.92 -> 1.21 ms against the
// lane walk, round 5); MHF_NO_TILE_IDX=1 takes the lane-walk kernel (diagnostic)
bool use_tile_idx(int32_t channels, int64_t ch_stride, int64_t sample_stride, fmask_t mask,
                  const float* x) {
    return !disabled("MHF_NO_TILE_IDX") &&
           tile_idx_ok(channels, ch_stride, sample_stride, mask & kMomentBits, x);
}
}  // namespace

extern "C" {

const char* mhf_plan_name_indexed(int32_t channels, int64_t ch_stride, int64_t sample_stride,
                                  const int32_t* features, int32_t n_features, int32_t dtype) {
    if (channels < 1 || n_features < 1 || n_features > kMaxFeatures || !features ||
        (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64))
        return nullptr;
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return nullptr;
        mask |= bit(features[j]);
    }
    if (mask & kSpectralBits) return nullptr;
    const float* aligned = reinterpret_cast<const float*>(uintptr_t(256));
    const char* parts[2] = {
        !(mask & kMomentBits) ? nullptr
        : dtype == MHF_DTYPE_F64 ? "moments_indexed_f64"
        : use_tile_idx(channels, ch_stride, sample_stride, mask, aligned) ? "tile_idx" : "moments_indexed",
        (mask & (kOrderBits | kSampenBits | kRqaBits)) ? "order/pairwise" : nullptr};
    char* o = g_plan_name;
    o[0] = 0;
    for (const char* part : parts) {
        if (!part) continue;
        if (o[0]) strncat(o, "+", sizeof(g_plan_name) - strlen(o) - 1);
        strncat(o, part, sizeof(g_plan_name) - strlen(o) - 1);
    }
    return g_plan_name;
}

int64_t mhf_indexed_workspace(int64_t max_window_len, int32_t channels, int32_t dtype,
                              const int32_t* features, int32_t n_features) {
    if (max_window_len < 0 || channels < 1 || (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) ||
        n_features < 1 || n_features > kMaxFeatures || !features)
        return -1;
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES) return -1;
        mask |= bit(features[j]);
    }
    if (!(mask & (kOrderBits | kSampenBits | kRqaBits))) return 0;
    const bool f64 = dtype == MHF_DTYPE_F64;
    int64_t bytes = kIdxSlotBytes;
    if ((mask & kOrderBits) && max_window_len > indexed_lds_cap(channels, f64)) {
        const int64_t pw = long_keys_per_wave(max_window_len, channels, f64);
        int64_t waves = kLongScratchBytes / pw;
        if (waves > kIdxKeyWaves) waves = kIdxKeyWaves;
        if (waves < 1) waves = 1;
        bytes += pw * waves;
    }
    return bytes;
}

int mhf_indexed_window_features(const float* x, int64_t n_samples, int32_t channels,
                                int64_t ch_stride, int64_t sample_stride, const int64_t* starts,
                                const int64_t* ends, int64_t n_windows, int64_t min_len,
                                const int32_t* features, int32_t n_features,
                                const mhf_params* params, int32_t out_dtype, void* out,
                                int64_t out_ld, void* workspace, int64_t workspace_bytes,
                                void* hip_stream) {
    g_err[0] = 0;
    if (channels < 1) return fail(MHF_EINVAL, "channels must be >= 1 (got %d)", channels);
    if (n_samples < 0 || sample_stride < 1 || ch_stride < 0)
        return fail(MHF_EINVAL, "n_samples must be >= 0, sample_stride >= 1, ch_stride >= 0");
    if (n_features < 1 || n_features > kMaxFeatures || !features)
        return fail(MHF_EINVAL, "n_features must be in [1, %d]", kMaxFeatures);
    if (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32)
        return fail(MHF_EINVAL, "out_dtype must be MHF_OUT_F64 or MHF_OUT_F32");
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES)
            return fail(MHF_EINVAL, "unknown feature id %d", features[j]);
        mask |= bit(features[j]);
    }
    if (mask & kSpectralBits)
        return fail(MHF_EUNSUPPORTED, "indexed (variable-length) windows take moment and "
                                      "time-domain features only");
    if (n_windows < 0) return fail(MHF_EINVAL, "n_windows must be >= 0");
    if (out_ld < n_windows) return fail(MHF_EINVAL, "out_ld < n_windows");
    if (n_windows == 0) return MHF_OK;
    if (!x || !out || !starts || !ends) return fail(MHF_EINVAL, "null x, out, starts or ends");
    IdxArgs a{};
    a.x = x; a.n_samples = n_samples; a.ch_stride = ch_stride; a.sample_stride = sample_stride;
    a.nwin = n_windows; a.min_len = min_len; a.starts = starts; a.ends = ends; a.mask = mask;
    a.t32 = zc_threshold32(params ? params->zc_threshold : 0.0);
    for (int j = 0; j < n_features; ++j) a.feats.id[j] = features[j];
    a.feats.n = n_features;
    a.out = out; a.out_ld = out_ld; a.out_f32 = out_dtype == MHF_OUT_F32;
    a.xp = extra_params(params);
    a.channels = channels;
    // order statistics / sampen / RQA first: their workspace checks and the one length
    // readback come before any launch of this call (include/mhfeat.h)
    if (mask & (kOrderBits | kSampenBits | kRqaBits)) {
        // LDS kernels sized for windows of up to kMaxOrderSamples / channels samples;
        // longer ones: indexed_order_launches
        OrderLaunch L{};
        L.x = x; L.ch_stride = ch_stride; L.sample_stride = sample_stride; L.nwin = n_windows;
        L.channels = channels; L.starts = starts; L.ends = ends; L.n_samples = n_samples;
        L.min_len = min_len;
        L.max_w = indexed_lds_cap(channels, false);
        L.q = params ? params->percentile_q : 50.0;
        L.feats = a.feats; L.out = out; L.out_ld = out_ld; L.out_f32 = out_dtype == MHF_OUT_F32;
        const int rc = indexed_order_launches(L, mask, params, workspace, workspace_bytes,
                                              static_cast<hipStream_t>(hip_stream));
        if (rc != MHF_OK) return rc;
    }
    if ((mask & kMomentBits) && use_tile_idx(channels, ch_stride, sample_stride, mask, x)) {
        // the register tile (tile_idx.hip.h): each window read once, both passes on chip
        IdxTileArgs t{};
        t.x = x; t.n_samples = n_samples; t.starts = starts; t.ends = ends; t.nwin = n_windows;
        t.min_len = min_len; t.channels = channels; t.mask = mask & kMomentBits; t.t32 = a.t32;
        t.xp = a.xp; t.feats = a.feats; t.out = out; t.out_ld = out_ld; t.out_f32 = a.out_f32;
        const int trc = launch_tile_idx(t, static_cast<hipStream_t>(hip_stream));
        if (trc != MHF_OK) return fail(trc, "tile_idx launch refused its arguments");
    } else if (mask & kMomentBits) {
        const int64_t units = n_windows * channels;
        dim3 grid(static_cast<unsigned>((units + 255) / 256));
        if (needs_ext(mask, a.xp.blk))
            hipLaunchKernelGGL(moments_indexed_kernel<true>, grid, dim3(256), lane_walk_shm(),
                               static_cast<hipStream_t>(hip_stream), a);
        else
            hipLaunchKernelGGL(moments_indexed_kernel<false>, grid, dim3(256), lane_walk_shm(),
                               static_cast<hipStream_t>(hip_stream), a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "HIP launch failed: %s", hipGetErrorString(e));
    return MHF_OK;
}

int mhf_indexed_window_features_f64(const double* x, int64_t n_samples, int32_t channels,
                                    int64_t ch_stride, int64_t sample_stride, const int64_t* starts,
                                    const int64_t* ends, int64_t n_windows, int64_t min_len,
                                    const int32_t* features, int32_t n_features,
                                    const mhf_params* params, int32_t out_dtype, void* out,
                                    int64_t out_ld, void* workspace, int64_t workspace_bytes,
                                    void* hip_stream) {
    g_err[0] = 0;
    if (channels < 1) return fail(MHF_EINVAL, "channels must be >= 1 (got %d)", channels);
    if (n_samples < 0 || sample_stride < 1 || ch_stride < 0)
        return fail(MHF_EINVAL, "n_samples must be >= 0, sample_stride >= 1, ch_stride >= 0");
    if (n_features < 1 || n_features > kMaxFeatures || !features)
        return fail(MHF_EINVAL, "n_features must be in [1, %d]", kMaxFeatures);
    if (out_dtype != MHF_OUT_F64 && out_dtype != MHF_OUT_F32)
        return fail(MHF_EINVAL, "out_dtype must be MHF_OUT_F64 or MHF_OUT_F32");
    fmask_t mask = 0;
    for (int j = 0; j < n_features; ++j) {
        if (features[j] < 0 || features[j] >= MHF_NUM_FEATURES)
            return fail(MHF_EINVAL, "unknown feature id %d", features[j]);
        mask |= bit(features[j]);
    }
    if (mask & kSpectralBits)
        return fail(MHF_EUNSUPPORTED, "indexed (variable-length) windows take moment and "
                                      "time-domain features only");
    const double q = params ? params->percentile_q : 50.0;
    if ((mask & bit(MHF_PERCENTILE)) && !(q >= 0.0 && q <= 100.0))
        return fail(MHF_EINVAL, "percentile_q must be in [0, 100] (numba raises ValueError)");
    if (n_windows < 0) return fail(MHF_EINVAL, "n_windows must be >= 0");
    if (out_ld < n_windows) return fail(MHF_EINVAL, "out_ld < n_windows");
    if (n_windows == 0) return MHF_OK;
    if (!x || !out || !starts || !ends) return fail(MHF_EINVAL, "null x, out, starts or ends");
    const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
    IdxArgs64 a{};
    a.x = x; a.n_samples = n_samples; a.ch_stride = ch_stride; a.sample_stride = sample_stride;
    a.nwin = n_windows; a.min_len = min_len; a.starts = starts; a.ends = ends; a.mask = mask;
    a.th = params ? params->zc_threshold : 0.0;
    for (int j = 0; j < n_features; ++j) a.feats.id[j] = features[j];
    a.feats.n = n_features;
    a.out = out; a.out_ld = out_ld; a.out_f32 = out_dtype == MHF_OUT_F32;
    a.xp = extra_params(params);
    if (mask & (kOrderBits | kSampenBits | kRqaBits)) {
        // 64-bit keys / fp64 samples: LDS holds windows of up to kOrderLdsBytes / 8 /
        // channels samples; longer ones: indexed_order_launches (first: its workspace checks
        // and the length readback precede any launch of this call)
        OrderLaunch L{};
        L.xd = x; L.ch_stride = ch_stride; L.sample_stride = sample_stride; L.nwin = n_windows;
        L.channels = channels; L.starts = starts; L.ends = ends; L.n_samples = n_samples;
        L.min_len = min_len;
        L.max_w = indexed_lds_cap(channels, true);
        L.q = q;
        L.feats = a.feats; L.out = out; L.out_ld = out_ld; L.out_f32 = out_dtype == MHF_OUT_F32;
        const int orc = indexed_order_launches(L, mask, params, workspace, workspace_bytes, stream);
        if (orc != MHF_OK) return orc;
    }
    if (mask & kMomentBits) {
        a.channels = channels;
        dim3 grid(static_cast<unsigned>((n_windows * channels + 255) / 256));
        hipLaunchKernelGGL(moments_indexed_f64_kernel, grid, dim3(256), lane_walk_shm(), stream, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "HIP launch failed: %s", hipGetErrorString(e));
    return MHF_OK;
}

int mhf_window_bounds(const int64_t* index, int64_t n, int64_t n_windows, int32_t mode,
                      int64_t t0_i, int64_t step_i, int64_t wsize_i, double t0_f, double step_f,
                      double wsize_f, int64_t* starts, int64_t* ends, void* hip_stream) {
    g_err[0] = 0;
    if (n < 0 || n_windows < 0) return fail(MHF_EINVAL, "n and n_windows must be >= 0");
    if (n_windows == 0) return MHF_OK;
    if (!index || !starts || !ends) return fail(MHF_EINVAL, "null index, starts or ends");
    if (mode & ~(MHF_BOUNDS_FLOAT_STARTS | MHF_BOUNDS_FLOAT_ENDS))
        return fail(MHF_EINVAL, "unknown bounds mode %d", mode);
    const bool fs = mode & MHF_BOUNDS_FLOAT_STARTS;
    if (fs && !(mode & MHF_BOUNDS_FLOAT_ENDS))
        return fail(MHF_EINVAL, "float starts imply float ends (numpy promotion)");
    if (!fs && step_i <= 0) return fail(MHF_EINVAL, "wstep must be > 0");
    if (fs && !(step_f > 0.0)) return fail(MHF_EINVAL, "wstep must be > 0");
    BoundsArgs a{};
    a.index = index; a.n = n; a.nwin = n_windows; a.mode = mode;
    a.t0_i = t0_i; a.step_i = step_i; a.wsize_i = wsize_i;
    a.t0_f = t0_f;
    a.delta_f = (t0_f + step_f) - t0_f;   // numpy arange fills start + i * (x[1] - x[0])
    a.wsize_f = wsize_f;
    a.starts = starts; a.ends = ends;
    hipLaunchKernelGGL(window_bounds_kernel, dim3(static_cast<unsigned>((n_windows + 255) / 256)),
                       dim3(256), 0, static_cast<hipStream_t>(hip_stream), a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "HIP launch failed: %s", hipGetErrorString(e));
    return MHF_OK;
}

int mhf_psd_features(const void* psd, int32_t psd_dtype, int64_t rows, int64_t bins,
                     int64_t row_stride, const void* freqs, int32_t freqs_dtype,
                     const int32_t* ops, int32_t n_ops, double lower, double upper,
                     double* out, int64_t out_ld, void* hip_stream) {
    g_err[0] = 0;
    if (psd_dtype != MHF_DTYPE_F32 && psd_dtype != MHF_DTYPE_F64)
        return fail(MHF_EINVAL, "psd_dtype must be MHF_DTYPE_F32 or MHF_DTYPE_F64");
    if (freqs_dtype != MHF_DTYPE_F32 && freqs_dtype != MHF_DTYPE_F64)
        return fail(MHF_EINVAL, "freqs_dtype must be MHF_DTYPE_F32 or MHF_DTYPE_F64");
    if (rows < 0 || bins < 0) return fail(MHF_EINVAL, "rows and bins must be >= 0");
    if (n_ops < 1 || n_ops > 4 * MHF_PSD_NUM_OPS || !ops)
        return fail(MHF_EINVAL, "n_ops must be in [1, %d]", 4 * MHF_PSD_NUM_OPS);
    bool need_f = false;
    for (int j = 0; j < n_ops; ++j) {
        if (ops[j] < 0 || ops[j] >= MHF_PSD_NUM_OPS) return fail(MHF_EINVAL, "unknown psd op %d", ops[j]);
        need_f |= ops[j] != MHF_PSD_ENTROPY;
    }
    if (rows > 1 && row_stride < bins) return fail(MHF_EINVAL, "row_stride < bins");
    if (out_ld < rows) return fail(MHF_EINVAL, "out_ld < rows");
    if (rows == 0) return MHF_OK;
    if (!psd || !out || (need_f && !freqs)) return fail(MHF_EINVAL, "null psd, freqs or out");
    launch_psd_rows(psd, psd_dtype, rows, bins, row_stride, freqs, freqs_dtype, ops, n_ops,
                    lower, upper, out, out_ld, static_cast<hipStream_t>(hip_stream));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MHF_EDEVICE, "HIP launch failed: %s", hipGetErrorString(e));
    return MHF_OK;
}

}  // extern "C"
