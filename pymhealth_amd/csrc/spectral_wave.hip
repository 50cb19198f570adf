// spectral_wave.hip — spectral features of long windows (W = 256 … 4096, power of two):
// one wavefront per window, Stockham radix-8/4/2 FFT with the butterflies in registers
// and one LDS round trip per stage.
//
// rFFT(W) = N = W/2 point complex FFT of z_n = x_2n + i x_2n+1; a stage of radix R does
// N/R butterflies spread over the 64 lanes (N/(64R) per lane), each reading R values at
// stride N/R, twiddling, an R-point DFT in registers, and writing in Stockham (autosort)
// order, so the result is in natural order after the last stage. Twiddles come from a
// per-block LDS table T[k] = exp(-2 pi i k / W), k < N (fp64-computed once per block).
// The window mean is removed before the FFT (fp32 error then scales with the AC energy)
// and the DC bin restored as W*mean + sum(x - mean). Features as in spectral_lane.hip.inc.
//
// Work assignment: a block (4 waves) takes a CONTIGUOUS run of windows, so overlapping
// windows (stride S < W, cfg5: 8x overlap) re-read each other's samples from the same
// CU's L1/L2 instead of from HBM.
#include "engine_common.h"
#include "spectral_wave.h"

namespace mhf {
namespace {

constexpr float kSqrtHalf = 0.70710678118654752440f;

struct cf {
    float x, y;
};
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf w) {
    return {fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x)};
}
__device__ __forceinline__ cf mul_mi(cf a) { return {a.y, -a.x}; }           // * (-i)
__device__ __forceinline__ cf mul_w8(cf a) {                                  // * exp(-i pi/4)
    return {(a.x + a.y) * kSqrtHalf, (a.y - a.x) * kSqrtHalf};
}
__device__ __forceinline__ cf mul_w8_3(cf a) {                                // * exp(-3i pi/4)
    return {(a.y - a.x) * kSqrtHalf, -(a.x + a.y) * kSqrtHalf};
}

template <int R>
__device__ __forceinline__ void dft(cf (&v)[R]);

template <>
__device__ __forceinline__ void dft<2>(cf (&v)[2]) {
    const cf a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}

template <>
__device__ __forceinline__ void dft<4>(cf (&v)[4]) {
    const cf s0 = cadd(v[0], v[2]), d0 = csub(v[0], v[2]);
    const cf s1 = cadd(v[1], v[3]), d1 = mul_mi(csub(v[1], v[3]));
    v[0] = cadd(s0, s1);
    v[2] = csub(s0, s1);
    v[1] = cadd(d0, d1);
    v[3] = csub(d0, d1);
}

template <>
__device__ __forceinline__ void dft<8>(cf (&v)[8]) {
    // radix-2 split into two 4-point DFTs of the even / odd elements
    cf e[4] = {v[0], v[2], v[4], v[6]};
    cf o[4] = {v[1], v[3], v[5], v[7]};
    dft<4>(e);
    dft<4>(o);
    const cf t1 = mul_w8(o[1]), t2 = mul_mi(o[2]), t3 = mul_w8_3(o[3]);
    v[0] = cadd(e[0], o[0]);
    v[4] = csub(e[0], o[0]);
    v[1] = cadd(e[1], t1);
    v[5] = csub(e[1], t1);
    v[2] = cadd(e[2], t2);
    v[6] = csub(e[2], t2);
    v[3] = cadd(e[3], t3);
    v[7] = csub(e[3], t3);
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// first-argmax merge with numpy's rule: first NaN wins, else first maximum
__device__ __forceinline__ void amax_merge(float& bv, int& bk, float ov, int ok) {
    const bool onan = ok >= 0 && (ov != ov);
    const bool bnan = bk >= 0 && (bv != bv);
    bool take;
    if (ok < 0) take = false;
    else if (bk < 0) take = true;
    else if (bnan || onan) take = onan && (!bnan || ok < bk);
    else take = (ov > bv) || (ov == bv && ok < bk);
    if (take) { bv = ov; bk = ok; }
}

// wave-local LDS ordering: the lanes of ONE wave exchange data through LDS between
// stages; LDS executes a wave's instructions in order, so a fence that stops the
// compiler from moving LDS accesses across this point is all that is needed.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One Stockham stage of radix R: Ns = product of the radices before it.
template <int N, int R, int Ns>
__device__ __forceinline__ void stage(const cf* __restrict__ src, cf* __restrict__ dst,
                                      const cf* __restrict__ tw, int lane, float dcr) {
    constexpr int NB = N / R;              // butterflies
    constexpr int PER = NB / 64;           // per lane
    static_assert(NB % 64 == 0, "a stage must give every lane a butterfly");
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int j = lane + 64 * b;
        cf v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = src[j + r * NB];
        if constexpr (Ns == 1) {
            // first stage: remove the window mean here (dcr = mean, both parts)
#pragma unroll
            for (int r = 0; r < R; ++r) { v[r].x -= dcr; v[r].y -= dcr; }
        } else {
            const int k = j % Ns;
            // W_{Ns R}^{r k} = exp(-2 pi i r k / (Ns R)) = T[2 r k N / (Ns R)] (T has W = 2N steps)
#pragma unroll
            for (int r = 1; r < R; ++r) {
                const int idx = (2 * r * k * (N / (Ns * R))) & (2 * N - 1);
                cf w = tw[idx & (N - 1)];
                if (idx >= N) { w.x = -w.x; w.y = -w.y; }   // exp(-i pi) factor
                v[r] = cmul(v[r], w);
            }
        }
        dft<R>(v);
        const int k = j % Ns;
        const int base = (j / Ns) * Ns * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) dst[base + r * Ns] = v[r];
    }
}

template <int N>
struct StagePlan;
// radices per N (every stage must have >= 64 butterflies)
template <> struct StagePlan<128> { static constexpr int r[7] = {2, 2, 2, 2, 2, 2, 2}; static constexpr int n = 7; };
template <> struct StagePlan<256> { static constexpr int r[4] = {4, 4, 4, 4}; static constexpr int n = 4; };
template <> struct StagePlan<512> { static constexpr int r[3] = {8, 8, 8}; static constexpr int n = 3; };  // NOLINT
template <> struct StagePlan<1024> { static constexpr int r[4] = {8, 8, 4, 4}; static constexpr int n = 4; };
template <> struct StagePlan<2048> { static constexpr int r[4] = {8, 8, 8, 4}; static constexpr int n = 4; };

template <int N, int S, int Ns>
__device__ __forceinline__ cf* run_stages(cf* a, cf* b, const cf* tw, int lane, float mean) {
    if constexpr (S == StagePlan<N>::n) {
        return a;
    } else {
        constexpr int R = StagePlan<N>::r[S];
        stage<N, R, Ns>(a, b, tw, lane, mean);
        wave_lds_sync();
        return run_stages<N, S + 1, Ns * R>(b, a, tw, lane, mean);
    }
}

template <int N>
__global__ void __launch_bounds__(256) spectral_wave_kernel(SpecWaveArgs a) {
    constexpr int W = 2 * N;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    cf* tw = reinterpret_cast<cf*>(smem_raw);                     // N entries
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    cf* buf_a = tw + N + wid * (2 * N);
    cf* buf_b = buf_a + N;
    const int c = blockIdx.y;

    for (int m = threadIdx.x; m < N; m += blockDim.x) {
        double s, co;
        sincospi(-2.0 * static_cast<double>(m) / static_cast<double>(W), &s, &co);
        tw[m] = {static_cast<float>(co), static_cast<float>(s)};
    }
    __syncthreads();

    // contiguous run of windows per block; waves take consecutive windows of it
    const int64_t per_block = (a.nwin + gridDim.x - 1) / gridDim.x;
    const int64_t w_begin = static_cast<int64_t>(blockIdx.x) * per_block;
    const int64_t w_end = w_begin + per_block < a.nwin ? w_begin + per_block : a.nwin;
    for (int64_t i = w_begin + wid; i < w_end; i += 4) {
        const int64_t g = a.first + i;
        const float* p = a.x + c * a.ch_stride + g * a.wstep * a.sample_stride;
        // load z_n = (x_2n, x_2n+1) into buf_a; lane sums for the mean
        float lsum = 0.0f;
        if (a.sample_stride == 1) {
#pragma unroll
            for (int q = 0; q < W / 128; ++q) {
                const int n = lane + 64 * q;
                const float2 v = *reinterpret_cast<const float2*>(p + 2 * n);
                buf_a[n] = {v.x, v.y};
                lsum += v.x + v.y;
            }
        } else {
            for (int n = lane; n < N; n += 64) {
                const float v0 = p[static_cast<int64_t>(2 * n) * a.sample_stride];
                const float v1 = p[static_cast<int64_t>(2 * n + 1) * a.sample_stride];
                buf_a[n] = {v0, v1};
                lsum += v0 + v1;
            }
        }
        const float mean = wsum(lsum) / static_cast<float>(W);
        wave_lds_sync();
        const cf* Z = run_stages<N, 0, 1>(buf_a, buf_b, tw, lane, mean);

        // real-input post-processing, periodogram, band / total sums, argmax
        float bp = 0.0f, tot = 0.0f, pmax = 0.0f;
        float bv = 0.0f;
        int bk = -1;
        float lent_psd[(N + 1 + 63) / 64];
        const float dcw = static_cast<float>(W) * mean;
#pragma unroll
        for (int q = 0; q < (N + 1 + 63) / 64; ++q) {
            const int k = lane + 64 * q;
            float pw = 0.0f;
            if (k <= N) {
                const cf zk = Z[k & (N - 1)], zn = Z[(N - k) & (N - 1)];
                const float er = zk.x + zn.x, ei = zk.y - zn.y;     // 2 E_k
                const float orr = zk.y + zn.y, oi = zn.x - zk.x;    // 2 O_k
                float xr, xi;
                if (k == 0) {
                    xr = fmaf(2.0f, dcw, er + orr); xi = ei + oi;
                } else if (k == N) {
                    xr = er - orr; xi = ei - oi;
                } else {
                    const cf t = tw[k];
                    xr = er + fmaf(orr, t.x, -oi * t.y);
                    xi = ei + fmaf(orr, t.y, oi * t.x);
                }
                pw = fmaf(xr, xr, xi * xi) * (0.25f * a.scale);
                if (k != 0 && k != N) pw = pw + pw;
                tot += pw;
                pmax = fmaxf(pmax, pw);
                if (k >= a.band_lo && k <= a.band_hi) bp += pw;
                if (k >= a.dom_lo && k < a.dom_hi) amax_merge(bv, bk, pw, k);
            }
            lent_psd[q] = pw;
        }
        bp = wsum(bp);
        tot = wsum(tot);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            pmax = fmaxf(pmax, __shfl_xor(pmax, o, 64));
            const float ov = __shfl_xor(bv, o, 64);
            const int ok = __shfl_xor(bk, o, 64);
            amax_merge(bv, bk, ov, ok);
        }
        float ent = 0.0f;
        if (a.want_ent) {
            // -sum(q ln q), q = psd/sum + 1e-30 (information.py:10-20); the largest bin
            // uses log1p(-(sum - max)/sum) with sum - max from an fp64 total
            double tot64 = 0.0;
            float e = 0.0f;
            const float inv = 1.0f / tot;
#pragma unroll
            for (int q = 0; q < (N + 1 + 63) / 64; ++q) {
                const int k = lane + 64 * q;
                if (k <= N) {
                    tot64 += static_cast<double>(lent_psd[q]);
                    const float qq = fmaf(lent_psd[q], inv, 1e-30f);
                    e = fmaf(qq, __logf(qq), e);
                }
            }
            e = wsum(e);
            double t64 = tot64;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) t64 += __shfl_xor(t64, o, 64);
            const float qmax = fmaf(pmax, inv, 1e-30f);
            const float lacc = log1pf(-static_cast<float>((t64 - pmax) / t64));
            e = fmaf(qmax, lacc - __logf(qmax), e);
            ent = -e;
        }
        if (lane == 0) {
            for (int jf = 0; jf < a.feats.n; ++jf) {
                const int f = a.feats.id[jf];
                double v;
                if (f == MHF_BAND_POWER) v = bp;
                else if (f == MHF_REL_BAND_POWER) v = bp / tot;
                else if (f == MHF_SPECTRAL_ENTROPY) v = ent;
                else if (f == MHF_DOMINANT_FREQ) v = (bk < 0) ? NAN : static_cast<double>(bk) * a.freq_step;
                else continue;
                store_out(a.out, a.out_f32,
                          (static_cast<int64_t>(c) * a.feats.n + jf) * a.out_ld + i, v);
            }
        }
        wave_lds_sync();   // buffers are reused by the next window
    }
}

template <int N>
int launch_n(const SpecWaveArgs& a, int channels, hipStream_t stream) {
    const size_t lds = sizeof(cf) * (static_cast<size_t>(N) + 4 * 2 * N);
    // one round of resident blocks (LDS-limited per CU), each a contiguous window run
    const int64_t per_cu = (160 * 1024) / static_cast<int64_t>(lds);
    int64_t blocks = (a.nwin + 15) / 16;
    const int64_t cap = 256 * (per_cu > 8 ? 8 : (per_cu < 1 ? 1 : per_cu)) / (channels > 0 ? channels : 1);
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(spectral_wave_kernel<N>, dim3(static_cast<unsigned>(blocks),
                       static_cast<unsigned>(channels)), dim3(256), lds, stream, a);
    return MHF_OK;
}

}  // namespace

bool spectral_wave_ok(int64_t wsize) {
    return wsize == 256 || wsize == 512 || wsize == 1024 || wsize == 2048 || wsize == 4096;
}

int launch_spectral_wave(const SpecWaveArgs& a, int64_t wsize, int channels, hipStream_t stream) {
    switch (wsize) {
    case 256: return launch_n<128>(a, channels, stream);
    case 512: return launch_n<256>(a, channels, stream);
    case 1024: return launch_spectral_reg(a, channels, stream);   // spectral_reg.hip
    case 2048: return launch_n<1024>(a, channels, stream);
    case 4096: return launch_n<2048>(a, channels, stream);
    default: return MHF_EUNSUPPORTED;
    }
}

}  // namespace mhf
