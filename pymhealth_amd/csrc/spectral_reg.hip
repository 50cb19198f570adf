// spectral_reg.hip — spectral features of W = 1024 windows (cfg5: ECG, stride 128) with
// the FFT held in registers: one wavefront per window, 8 complex points per lane, three
// radix-8 passes, two LDS transposes (bank-conflict-free for the ds_read2/write2_b64 the
// compiler forms) and one lane permute for the real-FFT bin pairs; twiddles from three
// fp64-accurate per-lane bases.
//
// Why: the LDS Stockham kernel (spectral_wave.hip) makes every radix pass an LDS round
// trip with scattered writes and LDS twiddle reads (cfg5: 16.3 ms). Here a window costs
// 432 VALU, 36 LDS and 47 SALU instructions (PMC); cfg5 runs in 9.8-10.0 ms at 3 waves per
// SIMD (LDS-DMA variant, 168 VGPRs; rocprof: 44 % issue-active, 28 % parked at waitcnt).
//
// rFFT(1024) = 512-point complex FFT of z_n = (x_2n - m) + i (x_2n+1 - m). With
// n = l + 64 r (lane l, register r) and K = k + 8 c + 64 d:
//   pass 1 (in lane l):        y_k(l) = w512^(l k) * DFT8_r(z_{l+64r})_k
//   transpose 1 -> lane (k,b): u_a = y_k(8a + b)
//   pass 2:                    v_c = w64^(b c) * DFT8_a(u)_c
//   transpose 2 -> lane (k,c): v(b) for b = 0..7
//   pass 3:                    Z[k + 8c + 64d] = DFT8_b(v)_d
//   each lane then fetches the partners Z[512 - K] of its 8 bins from one partner lane
//   (16 ds_bpermute) and evaluates its own bins.
// Post-processing, features and scaling as in spectral_lane.hip.inc / spectral_wave.hip.
#include "engine_common.h"
#include "spectral_wave.h"

namespace mhf {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kN = 512;          // complex FFT length (W = 1024)
constexpr int kW = 2 * kN;
constexpr int kT1 = 72;          // transpose-1 row stride (cf): reads hit 64 distinct banks
constexpr int kT2 = 65;          // transpose-2 row stride (cf)
constexpr int kBufCf = 8 * kT1;  // per-wave LDS buffer (cf), reused by the 3 transposes
constexpr float kS2 = 0.70710678118654752440f;
// w16^d = exp(-2 pi i d / 16)
__constant__ float kC16[8] = {1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                              0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f};
__constant__ float kS16[8] = {0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                              -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};

__device__ __forceinline__ f2 cmul(f2 a, f2 w) {
    // (a.x w.x - a.y w.y, a.x w.y + a.y w.x)
    return __builtin_elementwise_fma(f2{a.x, a.x}, w, f2{a.y, a.y} * f2{-w.y, w.x});
}
__device__ __forceinline__ f2 mul_mi(f2 a) { return f2{a.y, -a.x}; }   // * (-i)

// in-register 8-point DFT (forward, e^{-2 pi i / 8} kernel), natural order in and out
__device__ __forceinline__ void dft8(f2 (&v)[8]) {
    const f2 a0 = v[0] + v[4], a1 = v[0] - v[4];
    const f2 a2 = v[2] + v[6], a3 = mul_mi(v[2] - v[6]);
    const f2 b0 = v[1] + v[5], b1 = v[1] - v[5];
    const f2 b2 = v[3] + v[7], b3 = mul_mi(v[3] - v[7]);
    const f2 e0 = a0 + a2, e2 = a0 - a2, e1 = a1 + a3, e3 = a1 - a3;   // DFT4 of evens
    const f2 o0 = b0 + b2, o2 = b0 - b2, o1 = b1 + b3, o3 = b1 - b3;   // DFT4 of odds
    const f2 t1 = f2{o1.x + o1.y, o1.y - o1.x} * kS2;                   // o1 * w8
    const f2 t2 = mul_mi(o2);                                           // o2 * w8^2
    const f2 t3 = f2{o3.y - o3.x, -(o3.x + o3.y)} * kS2;                // o3 * w8^3
    v[0] = e0 + o0; v[4] = e0 - o0;
    v[1] = e1 + t1; v[5] = e1 - t1;
    v[2] = e2 + t2; v[6] = e2 - t2;
    v[3] = e3 + t3; v[7] = e3 - t3;
}

__device__ __forceinline__ f2 twiddle(int num, int den) {   // exp(-2 pi i num / den), fp64
    double s, c;
    sincospi(-2.0 * static_cast<double>(num) / static_cast<double>(den), &s, &c);
    return f2{static_cast<float>(c), static_cast<float>(s)};
}

// Wave reductions without LDS round trips: DPP within each 16-lane row (quad_perm
// [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8 leave the row total in every lane), then
// the four row totals through v_readlane (uniform result).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xb1>(v);
    v += dpp_f<0x4e>(v);
    v += dpp_f<0x124>(v);
    v += dpp_f<0x128>(v);
    return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                                          static_cast<uint32_t>(lo));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<int>(b), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), l);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}
// max of two arg-max keys (never NaN as doubles: the hi word is a float's bits, a float NaN
// 0x7fc00000 reads as a finite double); a plain v_max_f64 — fmax() would first quiet both
// operands (two more v_max_f64 each) because bit-cast values are not known canonical
__device__ __forceinline__ double kmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double wave_max_key(double v) {
    v = kmax(v, dpp_d<0xb1>(v));
    v = kmax(v, dpp_d<0x4e>(v));
    v = kmax(v, dpp_d<0x124>(v));
    v = kmax(v, dpp_d<0x128>(v));
    return kmax(kmax(readlane_d(v, 0), readlane_d(v, 16)), kmax(readlane_d(v, 32), readlane_d(v, 48)));
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// B_i = (lane p's A_i), p = idx / 4, for four complex values: 8 ds_bpermute_b32, waited
__device__ __forceinline__ void permute4(int idx, f2 a0, f2 a1, f2 a2, f2 a3, f2& b0, f2& b1,
                                         f2& b2, f2& b3) {
    float r0, r1, r2, r3, r4, r5, r6, r7;
    asm volatile(
        "ds_bpermute_b32 %0, %8, %9\n\t"
        "ds_bpermute_b32 %1, %8, %10\n\t"
        "ds_bpermute_b32 %2, %8, %11\n\t"
        "ds_bpermute_b32 %3, %8, %12\n\t"
        "ds_bpermute_b32 %4, %8, %13\n\t"
        "ds_bpermute_b32 %5, %8, %14\n\t"
        "ds_bpermute_b32 %6, %8, %15\n\t"
        "ds_bpermute_b32 %7, %8, %16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
        : "v"(idx), "v"(a0.x), "v"(a0.y), "v"(a1.x), "v"(a1.y), "v"(a2.x), "v"(a2.y), "v"(a3.x),
          "v"(a3.y)
        : "memory");
    b0 = f2{r0, r1}; b1 = f2{r2, r3}; b2 = f2{r4, r5}; b3 = f2{r6, r7};
}

// the arg-max key of bin k with weighted power pw (w = +1 inside [dom_lo, dom_hi), -1
// outside): hi word = bits of pw, lo word = 0xffff - k; for pw >= 0 the f64 order is
// (power, then smaller k); a NaN's bits read as a large key (first NaN wins, numpy);
// outside bins are negative keys
__device__ __forceinline__ double amax_key(float pw, int k) {
    return __builtin_bit_cast(double, (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, pw)) << 32) |
                                          static_cast<uint64_t>(0xffffu - static_cast<uint32_t>(k)));
}

// DMA: the next window's samples are prefetched by LDS-DMA (global_load_lds_dwordx4, nothing
// held in VGPRs) into the wave's 4-KiB window buffer instead of into 16 VGPRs, which brings
// the kernel under 168 VGPRs: 3 waves per SIMD (contiguous, 16-B aligned windows only).
// FS >= 0: the requested feature set fixed at compile time (bit 0 dominant frequency, bit 1
// total power), so the per-bin loop carries no uniform branches; FS = -1: from the args.
// bit 0: dominant frequency wanted; bit 1: total power (relative band power, entropy)
__host__ __device__ inline int spec_reg_fs(const SpecWaveArgs& a) {
    bool tot = a.want_ent != 0;
    for (int jf = 0; jf < a.feats.n; ++jf) tot |= a.feats.id[jf] == MHF_REL_BAND_POWER;
    return (a.dom_lo < a.dom_hi ? 1 : 0) | (tot ? 2 : 0);
}

template <bool CONTIG, bool DMA, int FS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DMA ? 3 : 2, DMA ? 3 : 2)))
spectral_reg_kernel(SpecWaveArgs a) {
    __shared__ __attribute__((aligned(16))) f2 lds[4][kBufCf];
    __shared__ __attribute__((aligned(16))) float winbuf[DMA ? 4 : 1][DMA ? kW : 4];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f2* T = lds[wid];
    const int c = blockIdx.y;
    const int kk = lane >> 3, bb = lane & 7;   // lane = 8 k + b after transpose 1, 8 k + c after 2

    // per-lane twiddle bases (fp64-accurate): pass 1 w512^lane, pass 2 w64^b, and the
    // bin twiddle w1024^(k + 8c) of this lane's bins K = k + 8c + 64d (times w16^d)
    const f2 base1 = twiddle(lane, kN), base2 = twiddle(bb, 64), basep = twiddle(kk + 8 * bb, kW);
    // the partner of bin K is 512 - K: lane 71 - lane (lanes 8..63), 8 - lane (1..7), register
    // 7 - d; lane 0 holds its own partners (K = 64 d <-> 64 (8 - d))
    const int partner = (lane >= 8 ? 71 - lane : (lane == 0 ? 0 : 8 - lane)) * 4;
    const bool want_dom = FS >= 0 ? (FS & 1) != 0 : spec_reg_fs(a) & 1;
    const bool want_tot = FS >= 0 ? (FS & 2) != 0 : (spec_reg_fs(a) & 2) != 0;
    // band / arg-max membership of this lane's 8 bins K = k + 8c + 64d, as bit masks
    uint32_t bandm = 0, domm = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const int K = kk + 8 * bb + 64 * d;
        bandm |= static_cast<uint32_t>(K >= a.band_lo && K <= a.band_hi) << d;
        domm |= static_cast<uint32_t>(K >= a.dom_lo && K < a.dom_hi) << d;
    }

    const int64_t per_block = (a.nwin + gridDim.x - 1) / gridDim.x;
    const int64_t w_begin = static_cast<int64_t>(blockIdx.x) * per_block;
    const int64_t w_end = w_begin + per_block < a.nwin ? w_begin + per_block : a.nwin;
    // samples of window i: z_n, n = lane + 64 r (coalesced float2 loads for stride 1)
    auto load = [&](int64_t i, f2 (&v)[8]) {
        const int64_t g = a.first + i;
        const float* p = a.x + c * a.ch_stride + g * a.wstep * a.sample_stride;
        if constexpr (CONTIG) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const float2 t = *reinterpret_cast<const float2*>(p + 2 * (lane + 64 * r));
                v[r] = f2{t.x, t.y};
            }
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int64_t n = lane + 64 * r;
                v[r] = f2{p[2 * n * a.sample_stride], p[(2 * n + 1) * a.sample_stride]};
            }
        }
    };
    // LDS-DMA of window i into this wave's buffer: 4 x 1 KiB, lane l's 16 B of piece j at
    // byte 1024 j + 16 l (the instruction's wave-uniform base + lane x 16)
    auto dma = [&](int64_t i) {
        const float* p = a.x + c * a.ch_stride + (a.first + i) * a.wstep;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds(
                const_cast<float*>(p + 256 * j + 4 * lane),
                (__attribute__((address_space(3))) void*)(&winbuf[wid][256 * j]), 16, 0, 0);
    };
    f2 nxt[DMA ? 1 : 8];
    if (w_begin + wid < w_end) {
        if constexpr (DMA) dma(w_begin + wid);
        else load(w_begin + wid, nxt);
    }
    for (int64_t i = w_begin + wid; i < w_end; i += 4) {
        f2 v[8];
        if constexpr (DMA) {
            // window i has landed (the only vector-memory ops in flight are its DMA and
            // the previous window's lane-0 stores); read it, then refill the buffer with
            // window i + 4 once the reads have returned
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = *reinterpret_cast<const f2*>(&winbuf[wid][2 * (lane + 64 * r)]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (i + 4 < w_end) dma(i + 4);
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = nxt[r];
            if (i + 4 < w_end) load(i + 4, nxt);   // in flight during this window's FFT
        }
        float lsum = 0.0f;
#pragma unroll
        for (int r = 0; r < 8; ++r) lsum += v[r].x + v[r].y;
        const float mean = wave_sum(lsum) / static_cast<float>(kW);
        const f2 M2 = {mean, mean};
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = v[r] - M2;

        // pass 1 + transpose 1 (T[k][l], row stride kT1)
        dft8(v);
        {
            f2 t = base1;
#pragma unroll
            for (int k = 1; k < 8; ++k) {
                v[k] = cmul(v[k], t);
                if (k < 7) t = cmul(t, base1);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) T[k * kT1 + lane] = v[k];
        wave_lds_sync();
#pragma unroll
        for (int a8 = 0; a8 < 8; ++a8) v[a8] = T[kk * kT1 + 8 * a8 + bb];
        wave_lds_sync();

        // pass 2 + transpose 2 (T[c][8k + b], row stride kT2)
        dft8(v);
        {
            f2 t = base2;
#pragma unroll
            for (int cc = 1; cc < 8; ++cc) {
                v[cc] = cmul(v[cc], t);
                if (cc < 7) t = cmul(t, base2);
            }
        }
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) T[cc * kT2 + 8 * kk + bb] = v[cc];
        wave_lds_sync();
        // lane = 8 k + c now: read v(b) = T[c][8k + b]
#pragma unroll
        for (int b8 = 0; b8 < 8; ++b8) v[b8] = T[bb * kT2 + 8 * kk + b8];
        wave_lds_sync();

        // pass 3: Z[k + 8c + 64d] = v[d]; the partners Z[512 - K] by one permute per float
        dft8(v);
        // (inline asm: LLVM merged the .y permute of each pair into the .x one)
        f2 B[8];
        permute4(partner, v[7], v[6], v[5], v[4], B[0], B[1], B[2], B[3]);
        permute4(partner, v[3], v[2], v[1], v[0], B[4], B[5], B[6], B[7]);
        if (lane == 0) {
#pragma unroll
            for (int d = 0; d < 8; ++d) B[d] = v[(8 - d) & 7];
        }

        // bin K of this lane: 2E = A + conj B, 2O = -i (A - conj B), 2X_K = 2E + w^K 2O
        // (spectral_lane.hip.inc); K = 0 gives bins 0 (DC restored) and 512. Powers in
        // units of 2 / scale (one-sided |2X|^2 / 2): the psd scale is applied once to the
        // band sum (ratios, entropy and the arg max do not depend on it)
        float pw[8], pny = 0.0f;
        float bp = 0.0f, tot = 0.0f;
        double key = -2.0;
        const float dcw = static_cast<float>(kW) * mean;
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const int K = kk + 8 * bb + 64 * d;
            const f2 A = v[d], Bd = B[d];
            const f2 w16 = f2{kC16[d], kS16[d]};
            const f2 tw = cmul(basep, w16);
            const f2 E2 = f2{A.x + Bd.x, A.y - Bd.y};
            const f2 O2 = f2{A.y + Bd.y, Bd.x - A.x};
            const f2 Tt = cmul(O2, tw);
            const float re = E2.x + Tt.x, im = E2.y + Tt.y;
            pw[d] = fmaf(re, re, im * im);
            if (d == 0 && lane == 0) {
                const float x0 = 2.0f * (A.x + A.y) + 2.0f * dcw, xn = 2.0f * (A.x - A.y);
                pw[0] = (x0 * x0) * 0.5f;   // DC and Nyquist are not doubled
                pny = (xn * xn) * 0.5f;
            }
            if (bandm & (1u << d)) bp += pw[d];
            if (want_tot) tot += pw[d];
            if (want_dom) key = kmax(key, amax_key((domm & (1u << d)) ? pw[d] : -1.0f, K));
        }
        if (lane == 0) {                       // the Nyquist bin 512
            if (kN >= a.band_lo && kN <= a.band_hi) bp += pny;
            tot += pny;
            if (want_dom) key = kmax(key, amax_key((kN >= a.dom_lo && kN < a.dom_hi) ? pny : -1.0f, kN));
        }
        bp = wave_sum(bp);
        if (want_tot) tot = wave_sum(tot);
        int bk = -1;
        if (want_dom) {
            const double kmax = wave_max_key(key);
            const uint64_t kb = __builtin_bit_cast(uint64_t, kmax);
            bk = (static_cast<int64_t>(kb) < 0) ? -1 : static_cast<int>(0xffffu - (kb & 0xffffu));
            // a NaN / inf sample makes the (wave-uniform) mean non-finite and every bin NaN,
            // whose sign the FFT's negations scatter (a negative NaN's key loses): numpy's
            // argmax over an all-NaN range is its first bin (as spectral_lane.hip.inc does)
            if (!(fabsf(mean) <= 3.402823466e38f)) bk = a.dom_lo;
        }
        float ent = 0.0f;
        if (a.want_ent) {
            // -sum(q ln q), q = psd/sum + 1e-30 (information.py:10-20); the largest bin's
            // ln q as log1p(-(sum - max)/sum) from an fp64 total
            double t64 = 0.0;
            float pmax = 0.0f, e = 0.0f;
            const float inv = 1.0f / tot;
#pragma unroll
            for (int d = 0; d < 9; ++d) {
                if (d == 8 && lane != 0) continue;
                const float pv = d < 8 ? pw[d] : pny;
                t64 += static_cast<double>(pv);
                pmax = fmaxf(pmax, pv);
                const float qq = fmaf(pv, inv, 1e-30f);
                e = fmaf(qq, __logf(qq), e);
            }
            e = wave_sum(e);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                t64 += __shfl_xor(t64, o, 64);
                pmax = fmaxf(pmax, __shfl_xor(pmax, o, 64));
            }
            const float qmax = fmaf(pmax, inv, 1e-30f);
            const float lacc = log1pf(-static_cast<float>((t64 - pmax) / t64));
            e = fmaf(qmax, lacc - __logf(qmax), e);
            ent = -e;
        }
        if (lane == 0) {
            for (int jf = 0; jf < a.feats.n; ++jf) {
                const int f = a.feats.id[jf];
                double val;
                if (f == MHF_BAND_POWER) val = bp * (0.5f * a.scale);
                else if (f == MHF_REL_BAND_POWER) val = bp / tot;
                else if (f == MHF_SPECTRAL_ENTROPY) val = ent;
                else if (f == MHF_DOMINANT_FREQ) val = (bk < 0) ? NAN : static_cast<double>(bk) * a.freq_step;
                else continue;
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + jf) * a.out_ld + i, val);
            }
        }
    }
}

// diagnostic switches (A/B on the box without a rebuild)
int getenv_int(const char* name) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : 0;
}

}  // namespace

bool spectral_reg_ok(int64_t wsize) { return wsize == kW; }

int launch_spectral_reg(const SpecWaveArgs& a, int channels, hipStream_t stream) {
    // persistent: one resident round (176 VGPRs: 2 waves per SIMD = 2 blocks of 4 waves
    // per CU), each block a contiguous window run (overlapping windows share L1/L2 lines)
    // DMA variant: contiguous samples, every window start 16-B aligned
    bool dma = a.sample_stride == 1 && a.wstep % 4 == 0 && getenv_int("MHF_SPECREG_NODMA") == 0;
    for (int c = 0; c < channels && dma; ++c)
        dma = reinterpret_cast<uintptr_t>(a.x + c * a.ch_stride + a.first * a.wstep) % 16 == 0;
    int64_t blocks = (a.nwin + 15) / 16;
    const int64_t cap = 256 * (dma ? 3 : 2) / (channels > 0 ? channels : 1);
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const dim3 grid(static_cast<unsigned>(blocks), static_cast<unsigned>(channels));
    if (dma) {
        switch (spec_reg_fs(a)) {
        case 0: hipLaunchKernelGGL((spectral_reg_kernel<true, true, 0>), grid, dim3(256), 0, stream, a); break;
        case 1: hipLaunchKernelGGL((spectral_reg_kernel<true, true, 1>), grid, dim3(256), 0, stream, a); break;
        case 2: hipLaunchKernelGGL((spectral_reg_kernel<true, true, 2>), grid, dim3(256), 0, stream, a); break;
        default: hipLaunchKernelGGL((spectral_reg_kernel<true, true, 3>), grid, dim3(256), 0, stream, a); break;
        }
    } else if (a.sample_stride == 1) {
        hipLaunchKernelGGL((spectral_reg_kernel<true, false, -1>), grid, dim3(256), 0, stream, a);
    } else {
        hipLaunchKernelGGL((spectral_reg_kernel<false, false, -1>), grid, dim3(256), 0, stream, a);
    }
    return MHF_OK;
}

}  // namespace mhf
