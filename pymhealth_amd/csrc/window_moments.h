// window_moments.h — the lane-walk model of one (window, channel): numba's sequential
// fp32 / fp64 reductions in the reference's order over any sample
// accessor. Shared by the generic / span / indexed kernels (mhfeat.hip) and the indexed
// tile kernel's fallback lanes (tile_idx.hip).
#pragma once
#include "engine_common.h"

#include <type_traits>

namespace mhf {
namespace {

// Sample accessors of one (window, channel): p(t) = sample t. GlobAcc reads HBM through
// the caller's strides (generic / indexed kernels); the span kernel's accessors read the
// LDS-staged span (span.hip.h).
// Both also hand out contiguous segments (seg(k): samples [k*R, k*R + R)), which the two
// main passes walk with a plain pointer: no per-sample index arithmetic.
struct GSeg {
    const float* __restrict__ q;
    int64_t ss;
    __device__ __forceinline__ float operator[](int64_t tt) const { return q[tt * ss]; }
};
struct GlobAcc {
    const float* __restrict__ p;
    int64_t ss;
    int64_t R;      // one segment: the whole window
    __device__ __forceinline__ float operator()(int64_t t) const { return p[t * ss]; }
    __device__ __forceinline__ GSeg seg(int64_t) const { return GSeg{p, ss}; }
};
typedef __attribute__((address_space(3))) const float lds_cfloat_t;
struct LSeg {
    lds_cfloat_t* q;
    __device__ __forceinline__ float operator[](int64_t tt) const { return q[tt]; }
};
// LDS span image (span_kernel): samples in rows of R = min(S, W), row pitch P floats;
// window r's sample t sits in row r + t / R, column t % R. t / R by a multiply-high
// (M = ceil(2^32 / R): exact for t, R < 2^16).
struct SpanAcc {
    lds_cfloat_t* base;       // row 0 of this lane's window
    int32_t R, P;
    uint32_t M;
    __device__ __forceinline__ float operator()(int64_t t) const {
        const uint32_t tu = static_cast<uint32_t>(t);
        const uint32_t q = R == 1 ? tu : __umulhi(tu, M);
        return base[q * static_cast<uint32_t>(P) + (tu - q * static_cast<uint32_t>(R))];
    }
    __device__ __forceinline__ LSeg seg(int64_t k) const { return LSeg{base + k * P}; }
};

// Moments of one (window, channel) of W samples p(0 .. W-1), in the reference's order.
// `serial`: the window is evaluated by numba's serial array_mean / array_var / array_std
// (row 0 of rolling_apply, windows.py:87; every window of indices_rolling_apply,
// windows.py:134-157) instead of the prange's parfor mean/var (rows >= 1).
// ---- §8f N3: Hjorth parameters. gradient(x) (timedom.py:11-31) of the fp32 window is an
// fp64 array (np.zeros(len(x))): g_0 = x1 - x0, g_{W-1} = x_{W-1} - x_{W-2}, else
// (x_{t+1} - x_{t-1}) / 2 (fp32 difference, exact halving in fp64); gradient(g) the same in
// fp64. np.var of an fp64 array is numba's array_var: fp64 sequential mean, then the fp64
// sequential sum of squared deviations, / W.
template <class Acc>
__device__ __forceinline__ double grad1(const Acc& p, int64_t W, int64_t t) {
    if (t == 0) return static_cast<double>(p(1) - p(0));
    if (t == W - 1) return static_cast<double>(p(W - 1) - p(W - 2));
    return static_cast<double>(p(t + 1) - p(t - 1)) / 2.0;
}
template <class Acc>
__device__ __forceinline__ double grad2(const Acc& p, int64_t W, int64_t t) {
    if (t == 0) return grad1(p, W, 1) - grad1(p, W, 0);
    if (t == W - 1) return grad1(p, W, W - 1) - grad1(p, W, W - 2);
    return (grad1(p, W, t + 1) - grad1(p, W, t - 1)) / 2.0;
}
template <int ORDER, class Acc>
__device__ double var64_grad(const Acc& p, int64_t W) {
    double s = 0.0;
    for (int64_t t = 0; t < W; ++t) s = s + (ORDER == 1 ? grad1(p, W, t) : grad2(p, W, t));
    const double m = s / static_cast<double>(W);
    double ssd = 0.0;
    for (int64_t t = 0; t < W; ++t) {
        const double d = (ORDER == 1 ? grad1(p, W, t) : grad2(p, W, t)) - m;
        ssd = ssd + d * d;
    }
    return ssd / static_cast<double>(W);
}

// ---- §8f N4: HRV metrics of an RR window (heart/hrv.py:111-266). d = np.diff(x) and
// u = x[1:] + x[:-1] are fp32 arrays of n = W - 1; np.mean / np.std of them are numba's
// fp32 array_mean / array_std (SURVEY Appendix A with n for W), np.sum an fp32 sequential
// sum, the pnn count compares |d| (promoted) against the fp64 threshold, and the csi
// family multiplies the fp32 std by the fp64 factor.
template <class Acc>
__device__ void hrv_window(const Acc& p, int64_t W, const ExtraParams& xp,
                           WinVals& r) {
    const int64_t n = W - 1;
    if (n < 1) {
        r.rmssd = r.sdsd = r.ssd = r.pnnx = r.sd1 = r.sd2 = r.lcsi = r.lcvi = r.lmcsi = NAN;
        return;
    }
    float sd = 0.0f, sq = 0.0f, su = 0.0f;
    int64_t cnt = 0;
    float prev = p(0);
    for (int64_t i = 1; i < W; ++i) {
        const float v = p(i);
        const float d = v - prev;
        sd = sd + d;
        sq = sq + d * d;
        su = su + (v + prev);
        cnt += static_cast<double>(fabsf(d)) > xp.pnn_th;
        prev = v;
    }
    const double nd = static_cast<double>(n);
    const float md = static_cast<float>(static_cast<double>(sd) / nd);
    const float mu = static_cast<float>(static_cast<double>(su) / nd);
    double vd = 0.0, vu = 0.0;
    prev = p(0);
    for (int64_t i = 1; i < W; ++i) {
        const float v = p(i);
        const float e = (v - prev) - md;
        const float f = (v + prev) - mu;
        vd = vd + static_cast<double>(e * e);
        vu = vu + static_cast<double>(f * f);
        prev = v;
    }
    const float std_d = static_cast<float>(sqrt(static_cast<double>(static_cast<float>(vd / nd))));
    const float std_u = static_cast<float>(sqrt(static_cast<double>(static_cast<float>(vu / nd))));
    r.rmssd = sqrtf(static_cast<float>(static_cast<double>(sq) / nd));
    r.sdsd = std_d;
    r.ssd = sd;
    r.pnnx = static_cast<double>(cnt) / nd;
    r.sd1 = xp.csi_factor * static_cast<double>(std_d);
    r.sd2 = xp.csi_factor * static_cast<double>(std_u);
    r.lcsi = r.sd1 / r.sd2;
    r.lcvi = log10(r.sd1 * r.sd2);
    r.lmcsi = (r.sd1 * r.sd1) / r.sd2;
}

// Walk samples [t0, W) of a window in order, segment by segment, calling f(t, x_t). Each
// segment is read kWalk samples at a time into registers before any of them is used, so
// the loads of a chunk (LDS for the span kernel, HBM/L1 for the generic one) are in
// flight together instead of one dependent load per sample.
constexpr int kWalk = 8;
// global-memory walks (generic / indexed kernels) keep 16 loads in flight per lane: their
// samples come from L2 / MALL, latency-bound (cfgidx 2.09 -> 1.94 ms once window_moments is
// inlined; with the 178-VGPR call it was slower, 2.42; MHF_GLOB_WALK overrides for A/B)
#ifndef MHF_GLOB_WALK
#define MHF_GLOB_WALK 16
#endif
#ifndef MHF_LDS_WALK
#define MHF_LDS_WALK kWalk
#endif
template <class Acc> struct WalkBatch { static constexpr int value = MHF_LDS_WALK; };
template <> struct WalkBatch<GlobAcc> { static constexpr int value = MHF_GLOB_WALK; };
template <class Acc, class F>
__device__ __forceinline__ void walk(const Acc& p, int64_t W, int64_t t0, F&& f) {
    constexpr int kB = WalkBatch<Acc>::value;
    for (int64_t k0 = 0, ks = 0; k0 < W; k0 += p.R, ++ks) {
        if (k0 + p.R <= t0) continue;
        const auto sg = p.seg(ks);
        const int64_t n = W - k0 < p.R ? W - k0 : p.R;
        int64_t tt = t0 > k0 ? t0 - k0 : 0;
        for (; tt + kB <= n; tt += kB) {
            float v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) v[u] = sg[tt + u];
#pragma unroll
            for (int u = 0; u < kB; ++u) f(v[u]);
        }
        for (; tt < n; ++tt) f(sg[tt]);
    }
}

// The two main passes, specialised on the requested feature groups so the per-sample
// loop carries no feature branches: XL = pass-1 extras level (1: zero crossings; 2: also
// rms / line length / np.min / np.max / peaks / drange), P2 = any pass-2 feature, PAR = the fp64 var_parallel_impl chain (rows >= 1 of a direct np.var /
// np.std), S34 = skewness / kurtosis sums.
// rows: len(x) of the window — W for a 1-D record, W / c for a 2-D (rows, c) block
// (skewness / kurtosis divide each term by it, stats.py:107,123)
template <int XL, bool P2, bool PAR, bool S34, class Acc>
__device__ __forceinline__ WinVals window_moments_t(const Acc& p, int64_t W, int64_t rows, bool serial,
                                                    float t32, WinVals& r) {
    // XL: pass-1 extras level — 0 none, 1 zero crossings only, 2 every extra
    constexpr bool XT = XL >= 2;
    constexpr bool ZC = XL >= 1;
    const float Wf = static_cast<float>(rows);
    const int pow2 = rows > 0 && (rows & (rows - 1)) == 0;
    const float invW = 1.0f / Wf;

    // ---- pass 1: fp32 sum (numba array_mean), rms sum, zc, peaks, drange, line length,
    // np.min / np.max. Samples 0 and 1 are peeled so the loop has no t > 0 / t > 1 tests.
    float c32 = 0.0f, a32 = 0.0f, ll = 0.0f;
    float mn = 0.0f, mx = 0.0f;
    float prev2 = 0.0f, prev1 = 0.0f;
    bool prevpos = false;
    int zc = 0, pk = 0;
    // np.min / np.max: rows >= 1 from +-inf, v < acc (builtin min: NaN skipped); row 0
    // returns the first NaN (numba array_min/max); otherwise both agree
    float pmin = INFINITY, pmax = -INFINITY, first_nan = 0.0f;
    bool any_nan = false;
    auto mm = [&](float v) {
        if (XT) {
            pmin = v < pmin ? v : pmin;
            pmax = v > pmax ? v : pmax;
            if (v != v && !any_nan) { any_nan = true; first_nan = v; }
        }
    };
    if (W > 0) {
        const float v = p(0);
        c32 = c32 + v;
        mm(v);
        if (XT) a32 = a32 + v * v;
        mn = v;
        mx = v;
        prevpos = v > t32;
        prev1 = v;
    }
    auto step1 = [&](float v) {      // t >= 1
        c32 = c32 + v;
        mm(v);
        if (XT) {
            a32 = a32 + v * v;
            ll = ll + fabsf(v - prev1);
        }
        if (ZC) {
            const bool pos = v > t32;
            zc += (pos != prevpos);
            prevpos = pos;
        }
        if (XT) {
            mn = v < mn ? v : mn;
            mx = v > mx ? v : mx;
        }
    };
    if (W > 1) {
        const float v = p(1);
        step1(v);
        prev2 = prev1;
        prev1 = v;
    }
    walk(p, W, 2, [&](float v) {
        step1(v);
        if (XT) pk += (prev1 > prev2 && prev1 > v);
        prev2 = prev1;
        prev1 = v;
    });
    const float m32 = static_cast<float>(static_cast<double>(c32) / static_cast<double>(W));
    const double m64 = static_cast<double>(c32) / static_cast<double>(W);
    r.mean32 = m32;
    r.mean = serial ? static_cast<double>(m32) : m64;
    r.rms = sqrtf(static_cast<float>(static_cast<double>(a32) / static_cast<double>(W)));
    r.zc = zc;
    r.peaks = pk;
    r.drange = static_cast<double>(mx - mn);
    r.ll = ll;
    r.vmin = (serial && any_nan) ? static_cast<double>(first_nan) : static_cast<double>(pmin);
    r.vmax = (serial && any_nan) ? static_cast<double>(first_nan) : static_cast<double>(pmax);

    // ---- pass 2: deviations from the fp32 mean (array_var / skewness / kurtosis) and
    // from the fp64 mean (var_parallel_impl for rows >= 1 of a direct np.var)
    r.var = r.var32 = r.std_ = r.std32 = r.skew = r.kurt = r.kurt_ex = 0.0;
    if (P2) {
        double ssd = 0.0, ssdp = 0.0;
        float s3 = 0.0f, s4 = 0.0f;
        const bool par = PAR && !serial;
        // the power-of-two test outside the sample loop: a per-sample select made every
        // sample pay for both the multiply and the IEEE division sequence.
        // Other lengths: the reference divides every term by len(x) (stats.py:107,123). The
        // quotient is formed as a multiply by invW = RN(1/rows) plus one Markstein
        // correction, q = RN(q0 + RN(a - q0 rows) invW) (two FMAs), which equals the IEEE
        // RN(a / rows) bit for bit for every rows <= 65536 and 2^-100 <= |a| <= FLT_MAX
        // (tools/div_probe.hip: every divisor x every mantissa of a binade; scaling a by a
        // power of two scales every intermediate exactly inside that range), and for a = 0
        // or NaN. The terms a = d^3, d^4 stay inside it while each nonzero |d| is in
        // [2^-25, 2^31]: the pass tracks the extremes of |d| and a lane outside them (or
        // with rows > 65536) redoes its s3 / s4 sums with the IEEE division.
        uint32_t dmin1 = 0xffffffffu;     // min over d != 0 of bits(|d|) - 1 (0 -> wraps high)
        float dmax = 0.0f;
        auto pass2 = [&](auto POW2) {
            walk(p, W, 0, [&](float v) {
                const float d = v - m32;
                const float q = d * d;
                ssd = ssd + static_cast<double>(q);
                if (PAR) {
                    const double dd = static_cast<double>(v) - m64;
                    ssdp = ssdp + dd * dd;
                }
                if (S34) {
                    if constexpr (decltype(POW2)::value) {
                        s3 = s3 + (d * q) * invW;
                        s4 = s4 + (q * q) * invW;
                    } else {
                        const float a3 = d * q, a4 = q * q;
                        const float q3 = a3 * invW, q4 = a4 * invW;
                        s3 = s3 + fmaf(fmaf(-q3, Wf, a3), invW, q3);
                        s4 = s4 + fmaf(fmaf(-q4, Wf, a4), invW, q4);
                        const uint32_t db = __float_as_uint(d) & 0x7fffffffu;
                        dmin1 = min(dmin1, db - 1u);
                        dmax = fmaxf(dmax, __uint_as_float(db));
                    }
                }
            });
        };
        if (S34 && pow2) pass2(std::true_type{});
        else pass2(std::false_type{});
        if (S34 && !pow2) {
            const uint32_t mnz = dmin1 + 1u;          // smallest nonzero |d| (0: none)
            const bool exact = rows <= 65536 && !(dmax > 0x1p31f) &&
                               (mnz == 0u || mnz >= 0x33000000u /* 2^-25 */);
            if (!exact) {
                s3 = 0.0f;
                s4 = 0.0f;
                walk(p, W, 0, [&](float v) {
                    const float d = v - m32;
                    const float q = d * d;
                    s3 = s3 + (d * q) / Wf;
                    s4 = s4 + (q * q) / Wf;
                });
            }
        }
        const float var32 = static_cast<float>(ssd / static_cast<double>(W));
        const float std32 = static_cast<float>(sqrt(static_cast<double>(var32)));
        const double varp = ssdp / static_cast<double>(W);
        r.var32 = var32;
        r.std32 = std32;
        r.var = par ? varp : static_cast<double>(var32);
        r.std_ = par ? sqrt(varp) : static_cast<double>(std32);
        r.skew = (std32 == 0.0f) ? 0.0 : static_cast<double>(s3 / (std32 * (std32 * std32)));
        const float kurt = (var32 == 0.0f) ? 0.0f : s4 / (var32 * var32);
        r.kurt = kurt;
        r.kurt_ex = static_cast<double>(kurt) - 3.0;
        r.cv = static_cast<double>(std32 / m32);   // np.std(x) / np.mean(x), fp32 quotient
    }
    return r;
}

// window_moments inlined into every kernel (the generic / indexed kernels otherwise call it
// as a function: 178 VGPRs and 304 B of scratch per lane for the call frame, against 61 and
// 24 inlined); MHF_WM_FORCE_INLINE=0 restores the call for A/B
#ifndef MHF_WM_FORCE_INLINE
#define MHF_WM_FORCE_INLINE 1
#endif
#if MHF_WM_FORCE_INLINE
#define MHF_WM_INLINE __attribute__((always_inline))
#else
#define MHF_WM_INLINE
#endif
// EXT: the features beyond the two passes (2-D block line length, Hjorth, HRV, entropy
// of x) are compiled in; the kernels launch an EXT = false instance for the plain moment
// sets, which keeps those paths' registers (206 VGPRs and scratch spills in the span
// kernel) out of the moment loops
template <bool EXT = true, class Acc>
__device__ MHF_WM_INLINE WinVals window_moments(const Acc& p, int64_t W, bool serial,
                                  fmask_t m, float t32, const ExtraParams& xp) {
    WinVals r;
    // pass-1 extras level: 2 when any of rms / line length / min / max / peaks / drange is
    // requested, 1 for zero crossings alone (the moments + zero-crossing sets: ~10 fewer
    // instructions per sample), 0 for none
    const int xl = (m & (bit(MHF_RMS) | bit(MHF_LINE_LENGTH) | bit(MHF_MIN) | bit(MHF_MAX) |
                         bit(MHF_PEAK_COUNT) | bit(MHF_DRANGE))) ? 2
                   : (m & bit(MHF_ZERO_CROSSINGS)) ? 1 : 0;
    const bool p2 = (m & (kPass2Bits | bit(MHF_COEFF_VAR) | kHjorthBits)) != 0;
    const bool par = !serial && (m & (bit(MHF_VAR) | bit(MHF_STD)));
    const bool s34 = (m & (bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) | bit(MHF_KURTOSIS_EXCESS))) != 0;
    const int64_t rows = xp.blk > 0 ? W / xp.blk : W;
#define MHF_WM(X, P, Q, S) window_moments_t<X, P, Q, S>(p, W, rows, serial, t32, r)
    if (!p2) {
        if (xl == 2) MHF_WM(2, false, false, false);
        else if (xl == 1) MHF_WM(1, false, false, false);
        else MHF_WM(0, false, false, false);
    } else if (xl == 2) {
        if (par) { if (s34) MHF_WM(2, true, true, true); else MHF_WM(2, true, true, false); }
        else { if (s34) MHF_WM(2, true, false, true); else MHF_WM(2, true, false, false); }
    } else if (xl == 1) {
        if (par) { if (s34) MHF_WM(1, true, true, true); else MHF_WM(1, true, true, false); }
        else { if (s34) MHF_WM(1, true, false, true); else MHF_WM(1, true, false, false); }
    } else {
        if (par) { if (s34) MHF_WM(0, true, true, true); else MHF_WM(0, true, true, false); }
        else { if (s34) MHF_WM(0, true, false, true); else MHF_WM(0, true, false, false); }
    }
#undef MHF_WM
    if constexpr (!EXT) return r;
    if (xp.blk > 0 && (m & bit(MHF_LINE_LENGTH))) {
        // np.sum(np.abs(np.diff(block))): diffs along the last axis (within rows), summed
        // flat in C order, fp32
        float ll = 0.0f;
        for (int64_t t = 1; t < W; ++t)
            if (t % xp.blk != 0) ll = ll + fabsf(p(t) - p(t - 1));
        r.ll = ll;
    }
    if (m & kHjorthBits) {
        if (W < 2) {
            r.hj_mob = r.hj_cmp = NAN;
        } else {
            const double vg = var64_grad<1>(p, W);
            r.hj_mob = sqrt(vg / static_cast<double>(static_cast<float>(r.var32)));
            if (m & bit(MHF_HJORTH_COMPLEXITY))
                r.hj_cmp = sqrt(var64_grad<2>(p, W) / vg) / r.hj_mob;
        }
    }
    if (m & kHrvBits) hrv_window(p, W, xp, r);
    if (m & bit(MHF_ENTROPY)) {
        // information.entropy (information.py:10-20) of the fp32 window: x / np.sum(x),
        // x += 1e-30, -np.sum(x * np.log(x)), every step fp32 and sequential
        float s = 0.0f, e = 0.0f;
        for (int64_t t = 0; t < W; ++t) s = s + p(t);
        for (int64_t t = 0; t < W; ++t) {
            float q = p(t) / s;
            q = q + 1e-30f;
            e = e + q * logf(q);
        }
        r.entx = -e;
    }
    return r;
}


}  // namespace
}  // namespace mhf
