// spectral64.hip — spectral features of a float64 record, computed in float64.
//
// The reference transforms a.astype(complex128) (FFTW double, or its numpy fp64 fallback:
// src/mhealth/fft/_fft.py:18-28, fft/__init__.py:3-7) and runs the post-FFT functions on
// that spectrum (heart/hrv.py:173-198, generic/information.py:10-20,
// generic/frequency/density.py:9-32). A float64 window therefore gets an fp64 transform
// here too — never the float32 rounding of the record.
//
// One wavefront per (window, channel): the window's samples in LDS, then
//   * W a power of two >= 2: N = W/2 point complex Stockham radix-2 FFT of
//     z_n = x_2n + i x_2n+1 (twiddles T[m] = exp(-2 pi i m / W), m < N, from sincospi),
//     then the real-input split X_k = E_k + T[k] O_k;
//   * any other W: direct DFT with the phase k*t reduced exactly mod W in integers.
// The window mean is removed before the transform (rounding then scales with the AC
// energy) and the DC bin restored as W * mean + sum(x - mean). Periodogram, band / total
// sums, first arg max (numpy: the first NaN wins, else the first maximum) and
// -sum(q ln q), q = psd / sum(psd) + 1e-30, all in fp64.
//
// Roofline: HBM (8 B per sample, read once per window — overlapping windows re-read from
// L2) for small W; fp64 VALU (W log2 W butterflies) beyond. Not on the headline metric.
#include <type_traits>

#include "engine_common.h"
#include "spectral64.h"

namespace mhf {
namespace {

// The value of lane l ^ M (butterfly partner) without LDS: DPP quad permutations (M = 1,
// 2), row rotations (4: by 4 or 12 chosen by lane bit 2 — both moves made, a DPP move
// under a partial EXEC reads disabled lanes; 8: by 8), and for M = 16 / 32 the pair
// {own, partner} of a v_permlane16/32_swap of the value with itself (which of the two
// is which depends on the row, so the reductions below combine both: sums add them,
// the arg max takes both as candidates). ds_bpermute-based __shfl_xor paid an LDS round
// trip per step, five reductions x six steps per window.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, false));
}
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
    if constexpr (M == 1) return dpp32<0xB1>(v);
    else if constexpr (M == 2) return dpp32<0x4E>(v);
    else if constexpr (M == 8) return dpp32<0x128>(v);
    else {
        static_assert(M == 4, "DPP partner");
        const uint32_t down = dpp32<0x124>(v), up = dpp32<0x12C>(v);
        return (__lane_id() & 4) ? down : up;
    }
}
template <int M>
__device__ __forceinline__ void swap_pair(uint32_t v, uint32_t& x0, uint32_t& x1) {
    const auto pr = M == 16 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                            : __builtin_amdgcn_permlane32_swap(v, v, false, false);
    x0 = static_cast<uint32_t>(pr[0]);
    x1 = static_cast<uint32_t>(pr[1]);
}
__device__ __forceinline__ double mk64(uint32_t lo, uint32_t hi) {
    return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}
__device__ __forceinline__ uint32_t lo32(double v) {
    return static_cast<uint32_t>(static_cast<uint64_t>(__double_as_longlong(v)));
}
__device__ __forceinline__ uint32_t hi32(double v) {
    return static_cast<uint32_t>(static_cast<uint64_t>(__double_as_longlong(v)) >> 32);
}
template <int M>
__device__ __forceinline__ double xor_add64(double v) {
    if constexpr (M <= 8) {
        return v + mk64(xor_lane<M>(lo32(v)), xor_lane<M>(hi32(v)));
    } else {
        uint32_t l0, l1, h0, h1;
        swap_pair<M>(lo32(v), l0, l1);
        swap_pair<M>(hi32(v), h0, h1);
        return mk64(l0, h0) + mk64(l1, h1);
    }
}
template <int M>
__device__ __forceinline__ double xor_max64(double v) {
    if constexpr (M <= 8) {
        return fmax(v, mk64(xor_lane<M>(lo32(v)), xor_lane<M>(hi32(v))));
    } else {
        uint32_t l0, l1, h0, h1;
        swap_pair<M>(lo32(v), l0, l1);
        swap_pair<M>(hi32(v), h0, h1);
        return fmax(mk64(l0, h0), mk64(l1, h1));
    }
}
template <int M>
__device__ __forceinline__ int xor_min32(int v) {
    if constexpr (M <= 8) {
        return min(v, static_cast<int>(xor_lane<M>(static_cast<uint32_t>(v))));
    } else {
        uint32_t x0, x1;
        swap_pair<M>(static_cast<uint32_t>(v), x0, x1);
        return min(static_cast<int>(x0), static_cast<int>(x1));
    }
}
// max of non-NaN doubles / min of ints over the wave, every lane
__device__ __forceinline__ double wmax64(double v) {
    v = xor_max64<1>(v);
    v = xor_max64<2>(v);
    v = xor_max64<4>(v);
    v = xor_max64<8>(v);
    v = xor_max64<16>(v);
    return xor_max64<32>(v);
}
__device__ __forceinline__ int wmin_i32(int v) {
    v = xor_min32<1>(v);
    v = xor_min32<2>(v);
    v = xor_min32<4>(v);
    v = xor_min32<8>(v);
    v = xor_min32<16>(v);
    return xor_min32<32>(v);
}
// fp64 sum over the wave, every lane (the order differs from numpy's pairwise sum: the
// fp64 features are pinned at 1e-10 relative, §5.14)
__device__ __forceinline__ double wsum64(double v) {
    v = xor_add64<1>(v);
    v = xor_add64<2>(v);
    v = xor_add64<4>(v);
    v = xor_add64<8>(v);
    v = xor_add64<16>(v);
    v = xor_add64<32>(v);
    return v;
}

// the lanes of one wave exchange data through LDS; a wave's LDS instructions execute in
// order, so a compiler fence + wave barrier orders them
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// WT > 0: the window length fixed at compile time (W = 128 / 256 / 512, the common
// powers of two): the stage and bin loops unroll with constant bounds and indices (their
// loop control was most of the kernel's 548 scalar instructions per window)
template <int WT>
__global__ void __launch_bounds__(256) spectral64_kernel(Spec64Args a) {
    extern __shared__ __attribute__((aligned(16))) double sm64[];
    const int W = WT > 0 ? WT : static_cast<int>(a.wsize);
    const int N = W / 2;
    const int nb = W / 2 + 1;
    const bool fft = a.pow2 != 0;
    const int wpb = blockDim.x >> 6;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tw_n = fft ? N : W;                       // complex twiddles in the table
    double2* tw = reinterpret_cast<double2*>(sm64);
    double* wbase = sm64 + 2 * tw_n + static_cast<int64_t>(wid) * (fft ? 2 * W : W + nb);
    const int c = blockIdx.y;

    for (int m = threadIdx.x; m < tw_n; m += blockDim.x) {
        double s, co;
        sincospi(-2.0 * static_cast<double>(m) / static_cast<double>(W), &s, &co);
        tw[m] = make_double2(co, s);
    }
    __syncthreads();

    const int64_t stride = static_cast<int64_t>(gridDim.x) * wpb;
    // W <= 512 (<= 8 samples per lane): the next window's samples load into registers while
    // this one is transformed, and a window's outputs (one store instruction, lane j feature
    // j) leave one iteration later, after those loads — one wave per window spends its time
    // in LDS round trips and wave barriers, and the HBM latency of each window's load sat in
    // front of every transform (stores and loads share vmcnt: a store at the end of an
    // iteration would hold the next iteration's wait for the prefetched samples)
    const bool pf = W <= 8 * 64;
    auto win_ptr = [&](int64_t ii) { return a.x + c * a.ch_stride + (a.first + ii) * a.wstep * a.sample_stride; };
    double nx[8];
    auto load_win = [&](int64_t ii) __attribute__((always_inline)) {
        const double* q = win_ptr(ii);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int t = lane + 64 * k;
            nx[k] = t < W ? q[static_cast<int64_t>(t) * a.sample_stride] : 0.0;
        }
    };
    const int64_t i0 = static_cast<int64_t>(blockIdx.x) * wpb + wid;
    if (pf && i0 < a.nwin) load_win(i0);
    double o_val = 0.0;
    int64_t o_row = -1;
    for (int64_t i = i0; i < a.nwin; i += stride) {
        double* xs = wbase;                              // W doubles (pow2: = N complex)
        double lsum = 0.0;
        if (pf) {
            // this window's samples (loaded an iteration ago) into LDS, then the next
            // window's loads and this wave's previous outputs
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int t = lane + 64 * k;
                if (t < W) {
                    xs[t] = nx[k];
                    lsum += nx[k];
                }
            }
            if (i + stride < a.nwin) load_win(i + stride);
            if (o_row >= 0) store_out(a.out, a.out_f32, o_row, o_val);
            o_row = -1;
        } else {
            const double* p = win_ptr(i);
            for (int t = lane; t < W; t += 64) {
                const double v = p[static_cast<int64_t>(t) * a.sample_stride];
                xs[t] = v;
                lsum += v;
            }
        }
        const double wmean = wsum64(lsum) / static_cast<double>(W);
        wave_sync();
        for (int t = lane; t < W; t += 64) xs[t] -= wmean;
        const double dc = static_cast<double>(W) * wmean;
        wave_sync();

        double* psd;
        if (fft) {
            double2* src = reinterpret_cast<double2*>(xs);
            double2* dst = reinterpret_cast<double2*>(xs + W);
            for (int Ns = 1; Ns < N; Ns <<= 1) {
                for (int jj = 0; jj < (N / 2 + 63) / 64; ++jj) {   // (uniform trip count)
                    const int j = lane + 64 * jj;
                    if (j >= N / 2) break;
                    const int k = j & (Ns - 1);
                    const double2 u = src[j];
                    const double2 v0 = src[j + N / 2];
                    const double2 w = tw[k * (N / Ns)];     // exp(-2 pi i k / (2 Ns))
                    const double2 v = make_double2(fma(v0.x, w.x, -v0.y * w.y),
                                                   fma(v0.x, w.y, v0.y * w.x));
                    const int d = (j - k) * 2 + k;
                    dst[d] = make_double2(u.x + v.x, u.y + v.y);
                    dst[d + Ns] = make_double2(u.x - v.x, u.y - v.y);
                }
                wave_sync();
                double2* t = src; src = dst; dst = t;
            }
            // the other buffer (N complex = W doubles >= nb) takes the periodogram
            psd = reinterpret_cast<double*>(dst);
            for (int kk = 0; kk < (nb + 63) / 64; ++kk) {
                const int k = lane + 64 * kk;
                if (k >= nb) break;
                const double2 zk = src[k & (N - 1)];
                const double2 zn = src[(N - k) & (N - 1)];
                const double er = 0.5 * (zk.x + zn.x), ei = 0.5 * (zk.y - zn.y);
                const double orr = 0.5 * (zk.y + zn.y), oi = -0.5 * (zk.x - zn.x);
                const double2 w = (k < N) ? tw[k] : make_double2(-1.0, 0.0);
                const double xr = er + fma(orr, w.x, -oi * w.y) + (k == 0 ? dc : 0.0);
                const double xi = ei + fma(orr, w.y, oi * w.x);
                double pw = fma(xr, xr, xi * xi) * a.scale;
                if (k >= 1 && k < N) pw *= 2.0;
                psd[k] = pw;
            }
        } else {
            psd = xs + W;
            for (int k = lane; k < nb; k += 64) {
                double sr = 0.0, si = 0.0;
                int ph = 0;
                for (int t = 0; t < W; ++t) {
                    const double2 w = tw[ph];
                    const double xv = xs[t];
                    sr = fma(xv, w.x, sr);
                    si = fma(xv, w.y, si);
                    ph += k;
                    if (ph >= W) ph -= W;
                }
                if (k == 0) sr += dc;
                double pw = fma(sr, sr, si * si) * a.scale;
                const bool dbl = (W & 1) ? (k >= 1) : (k >= 1 && k < nb - 1);
                if (dbl) pw *= 2.0;
                psd[k] = pw;
            }
        }
        wave_sync();

        // band / total sums, and numpy's argmax over [dom_lo, dom_hi): the first NaN if
        // there is one, else the first maximum — per lane (its bins in increasing order:
        // a strict > keeps the first), then over the wave: a NaN ballot and an index
        // minimum, or the value maximum and the smallest index holding it (DPP / permlane
        // butterflies; round 5 — the pairwise (value, index) arg max of every step was a
        // dozen compares and branches, eight times per window)
        double bp = 0.0, tot = 0.0, lmax = -INFINITY;
        int lidx = 0x7fffffff, nidx = 0x7fffffff;
        for (int kk = 0; kk < (nb + 63) / 64; ++kk) {
            const int k = lane + 64 * kk;
            if (k >= nb) break;
            const double v = psd[k];
            const double av = fabs(v);
            tot += av;
            if (k >= a.band_lo && k <= a.band_hi) bp += av;
            if (k >= a.dom_lo && k < a.dom_hi) {
                if (v != v) nidx = min(nidx, k);
                else if (v > lmax || lidx == 0x7fffffff) {
                    lmax = v;
                    lidx = k;
                }
            }
        }
        bp = wsum64(bp);
        tot = wsum64(tot);
        int bk;
        if (__ballot(nidx != 0x7fffffff) != 0) {
            bk = wmin_i32(nidx);
        } else {
            const double m = wmax64(lidx != 0x7fffffff ? lmax : -INFINITY);
            bk = wmin_i32(lidx != 0x7fffffff && lmax == m ? lidx : 0x7fffffff);
            if (bk == 0x7fffffff) bk = -1;                    // an empty range
        }
        double ent = 0.0;
        if (a.want_ent) {
            const double rtot = 1.0 / tot;
            // a subnormal total (a window of ~1e-160 samples): 1 / tot overflows where the
            // reference's psd / tot is finite — divide then (tot is wave-uniform: no divergence)
            const bool by_div = !(rtot < INFINITY) && tot != 0.0;
            for (int kk = 0; kk < (nb + 63) / 64; ++kk) {
                const int k = lane + 64 * kk;
                if (k >= nb) break;
                const double q = by_div ? psd[k] / tot + 1e-30
                                        : fma(psd[k], rtot, 1e-30);   // psd / sum (a reciprocal: 1e-16)
                ent = fma(q, log(q), ent);
            }
            ent = -wsum64(ent);
        }
        // (bp, tot, ent, bk are wave-uniform after the reductions)
        auto fval = [&](int f, bool& ok) -> double {
            ok = true;
            if (f == MHF_BAND_POWER) return bp;
            if (f == MHF_REL_BAND_POWER) return bp / tot;
            if (f == MHF_SPECTRAL_ENTROPY) return ent;
            if (f == MHF_DOMINANT_FREQ) return (bk < 0) ? NAN : static_cast<double>(bk) * a.freq_step;
            ok = false;
            return 0.0;
        };
        if (pf && a.feats.n <= 64) {
            if (lane < a.feats.n) {
                bool ok;
                const double v = fval(a.feats.id[lane], ok);
                if (ok) {
                    o_val = v;
                    o_row = (static_cast<int64_t>(c) * a.feats.n + lane) * a.out_ld + i;
                }
            }
        } else if (lane == 0) {
            for (int j = 0; j < a.feats.n; ++j) {
                bool ok;
                const double v = fval(a.feats.id[j], ok);
                if (!ok) continue;
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i, v);
            }
        }
        wave_sync();   // the buffers are reused by this wave's next window
    }
    if (o_row >= 0) store_out(a.out, a.out_f32, o_row, o_val);
}

}  // namespace

int launch_spectral64(const Spec64Args& a0, int channels, hipStream_t stream) {
    Spec64Args a = a0;
    const int64_t W = a.wsize;
    if (W < 1 || W > kMaxSpectralW || channels < 1) return MHF_EINVAL;
    a.pow2 = (W >= 2 && (W & (W - 1)) == 0) ? 1 : 0;
    const int64_t nb = W / 2 + 1;
    const int64_t table = a.pow2 ? W : 2 * W;                 // doubles
    const int64_t per_wave = a.pow2 ? 2 * W : W + nb;        // doubles
    const int64_t budget = (64 * 1024) / 8;                   // 64 KiB per block: >= 2 blocks / CU
    int64_t wpb = (budget - table) / per_wave;
    if (wpb > 4) wpb = 4;
    if (wpb < 1) wpb = 1;
    const size_t lds = sizeof(double) * static_cast<size_t>(table + wpb * per_wave);
    if (lds > 160 * 1024) return MHF_EUNSUPPORTED;
    int64_t blocks = (a.nwin + wpb - 1) / wpb;
    const int64_t cap = 2048 / channels > 0 ? 2048 / channels : 1;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const dim3 grid(static_cast<unsigned>(blocks), static_cast<unsigned>(channels)),
        block(static_cast<unsigned>(64 * wpb));
    if (W == 256) hipLaunchKernelGGL(spectral64_kernel<256>, grid, block, lds, stream, a);
    else if (W == 128) hipLaunchKernelGGL(spectral64_kernel<128>, grid, block, lds, stream, a);
    else if (W == 512) hipLaunchKernelGGL(spectral64_kernel<512>, grid, block, lds, stream, a);
    else hipLaunchKernelGGL(spectral64_kernel<0>, grid, block, lds, stream, a);
    return MHF_OK;
}

}  // namespace mhf
