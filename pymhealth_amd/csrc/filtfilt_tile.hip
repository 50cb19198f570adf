// filtfilt_tile.hip — the two passes of filtfilt (filtfilt.hip) with the record streamed
// through LDS: the chunked-recurrence design of iir_chunk_kernel (one lane per chunk of M
// positions, warmed up over the R positions before it) with its memory traffic made
// coalesced (generic/filters.py:28-35, inertial/accelerometer.py:78-183).
//
// iir_chunk_kernel gave each lane its own chunk and let it load and store its own samples:
// every wave instruction touched 64 rows far apart (pass 0 read 3.25 x its input, pass 1
// wrote 3.0 x its output, issue-active 0.17: 6.1 ms for 1e8 x 3-axis). Here a wave owns U =
// 64 / C consecutive chunks and ALL their channels — lane = (chunk r, channel c), the
// channels of a chunk side by side — and walks them in lock step, 32 positions (a "block")
// at a time:
//   * the block's input rows (U rows of 32 x C samples, contiguous in memory) are DMA'd
//     (global_load_lds_dwordx4, SGPR base + per-lane 32-bit offsets, whole 16-B pieces)
//     into a ring of LDS slots several blocks ahead, so HBM latency hides behind the
//     recurrence of the blocks before it — the tile kernel's geometry for pass 0 (fp32 x,
//     tile.hip.h) and the same with 8-byte samples for pass 1 (the fp64 forward output);
//   * each lane reads its own (chunk, channel) samples from the slot (ds_read2 / b128),
//     runs the DF2T recurrence in fp64 (fused multiply-adds: 2 dependent FMAs per step)
//     and stores its outputs, the C channels of a position side by side (AoS rows).
// The forward output is kept reversed and AoS — yr[(L - 1 - j) C + c] = y_fwd[j, c] — so
// pass 1 streams it forwards exactly like pass 0 streams x.
//
// Edges: pass 0 reads x at positions t = j - padlen. Blocks of the first / last chunks that
// reach outside x (the odd extension, and the alignment slack of the block grid) are DMA'd
// from a clamped in-range block and their extension samples written into the lane's LDS row
// from x (2 x0 - x[-t], 2 x[n-1] - x[2n-2-t], fp32 like numpy); positions before a lane's
// start or past its end are masked. Chunks whose warm-up would reach before the record
// start there from lfilter_zi x the first input, as in iir_chunk_kernel.
#define MHF_TILE_IMPL
#include "tile.hip.h"
#include "filtfilt.h"

namespace mhf {
namespace {

constexpr int kFB = 32;                      // positions per block (= kChunk)
static_assert(kFB == kChunk, "pass-0 blocks use the tile chunk geometry");

// geometry of one pass: ES = bytes per sample (4: x, 8: yr)
template <int C, int ES>
struct FGeom {
    static constexpr int U = 64 / C;                         // chunks per wave
    static constexpr int kPieces = kFB * C * ES / 16;        // 16-B pieces per row
    static constexpr int kRowSlots = kPieces + 1;            // + one pad slot (banks)
    static constexpr int kNI = (U * kRowSlots + 63) / 64;    // DMA instructions per block
    static constexpr int kSlotBytes = kNI * 1024;
    static constexpr int kRingN = ES == 4 ? 4 : 3;           // ring slots
};

// DMA of one block: kNI global_load_lds_dwordx4 in groups of up to 5 sharing one M0 (each
// statement opens with s_nop 4: VALU-written SGPR base -> VMEM, tile.hip.h dma_chunk)
// (instruction offsets -2 .. +2 KiB around it); off[i] carries kBias - (that offset)
template <int G, int NI>
__device__ __forceinline__ void dma_group(uint64_t base, uint32_t slot, const uint32_t (&o)[NI]) {
    constexpr int i0 = 5 * G, n = NI - i0 < 5 ? NI - i0 : 5;
    const uint32_t m0 = slot + static_cast<uint32_t>((i0 + 2) * 1024);
    if constexpr (n == 5)
        asm volatile("s_nop 4\n\t"
                     "global_load_lds_dwordx4 %1, %6 offset:-2048\n\t"
                     "global_load_lds_dwordx4 %2, %6 offset:-1024\n\t"
                     "global_load_lds_dwordx4 %3, %6\n\t"
                     "global_load_lds_dwordx4 %4, %6 offset:1024\n\t"
                     "global_load_lds_dwordx4 %5, %6 offset:2048"
                     :
                     : "{m0}"(m0), "v"(o[i0]), "v"(o[i0 + 1]), "v"(o[i0 + 2]), "v"(o[i0 + 3]),
                       "v"(o[i0 + 4]), "s"(base)
                     : "memory");
    else if constexpr (n == 4)
        asm volatile("s_nop 4\n\t"
                     "global_load_lds_dwordx4 %1, %5 offset:-2048\n\t"
                     "global_load_lds_dwordx4 %2, %5 offset:-1024\n\t"
                     "global_load_lds_dwordx4 %3, %5\n\t"
                     "global_load_lds_dwordx4 %4, %5 offset:1024"
                     :
                     : "{m0}"(m0), "v"(o[i0]), "v"(o[i0 + 1]), "v"(o[i0 + 2]), "v"(o[i0 + 3]), "s"(base)
                     : "memory");
    else if constexpr (n == 3)
        asm volatile("s_nop 4\n\t"
                     "global_load_lds_dwordx4 %1, %4 offset:-2048\n\t"
                     "global_load_lds_dwordx4 %2, %4 offset:-1024\n\t"
                     "global_load_lds_dwordx4 %3, %4"
                     :
                     : "{m0}"(m0), "v"(o[i0]), "v"(o[i0 + 1]), "v"(o[i0 + 2]), "s"(base)
                     : "memory");
    else if constexpr (n == 2)
        asm volatile("s_nop 4\n\t"
                     "global_load_lds_dwordx4 %1, %3 offset:-2048\n\t"
                     "global_load_lds_dwordx4 %2, %3 offset:-1024"
                     :
                     : "{m0}"(m0), "v"(o[i0]), "v"(o[i0 + 1]), "s"(base)
                     : "memory");
    else
        asm volatile("s_nop 4\n\t"
                     "global_load_lds_dwordx4 %1, %2 offset:-2048"
                     :
                     : "{m0}"(m0), "v"(o[i0]), "s"(base)
                     : "memory");
    if constexpr (i0 + 5 < NI) dma_group<G + 1, NI>(base, slot, o);
}
__host__ __device__ constexpr int fdma_inst_off(int i) { return (i % 5 - 2) * 1024; }

// A lane's 32 fp64 samples of the block from its row (row base `addr`, LDS bytes), in order
typedef double d2 __attribute__((ext_vector_type(2)));
template <int C>
__device__ __forceinline__ void lds_read_row64(uint32_t addr, double (&v)[kFB]);
template <>
__device__ __forceinline__ void lds_read_row64<1>(uint32_t addr, double (&v)[kFB]) {
    d2 o[16];
    asm volatile(
        "ds_read_b128 %0, %16\n\t"
        "ds_read_b128 %1, %16 offset:16\n\t"
        "ds_read_b128 %2, %16 offset:32\n\t"
        "ds_read_b128 %3, %16 offset:48\n\t"
        "ds_read_b128 %4, %16 offset:64\n\t"
        "ds_read_b128 %5, %16 offset:80\n\t"
        "ds_read_b128 %6, %16 offset:96\n\t"
        "ds_read_b128 %7, %16 offset:112\n\t"
        "ds_read_b128 %8, %16 offset:128\n\t"
        "ds_read_b128 %9, %16 offset:144\n\t"
        "ds_read_b128 %10, %16 offset:160\n\t"
        "ds_read_b128 %11, %16 offset:176\n\t"
        "ds_read_b128 %12, %16 offset:192\n\t"
        "ds_read_b128 %13, %16 offset:208\n\t"
        "ds_read_b128 %14, %16 offset:224\n\t"
        "ds_read_b128 %15, %16 offset:240\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]),
          "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]),
          "=&v"(o[14]), "=&v"(o[15])
        : "v"(addr)
        : "memory");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[2 * i] = o[i].x;
        v[2 * i + 1] = o[i].y;
    }
}
template <>
__device__ __forceinline__ void lds_read_row64<3>(uint32_t addr, double (&v)[kFB]) {
    // sample p of the lane's channel at byte 24 p (+ the lane base: row + 8 c): two samples
    // per ds_read2_b64 (offsets in 8-B units, 3 apart)
    d2 o[16];
    asm volatile(
        "ds_read2_b64 %0, %16 offset1:3\n\t"
        "ds_read2_b64 %1, %16 offset0:6 offset1:9\n\t"
        "ds_read2_b64 %2, %16 offset0:12 offset1:15\n\t"
        "ds_read2_b64 %3, %16 offset0:18 offset1:21\n\t"
        "ds_read2_b64 %4, %16 offset0:24 offset1:27\n\t"
        "ds_read2_b64 %5, %16 offset0:30 offset1:33\n\t"
        "ds_read2_b64 %6, %16 offset0:36 offset1:39\n\t"
        "ds_read2_b64 %7, %16 offset0:42 offset1:45\n\t"
        "ds_read2_b64 %8, %16 offset0:48 offset1:51\n\t"
        "ds_read2_b64 %9, %16 offset0:54 offset1:57\n\t"
        "ds_read2_b64 %10, %16 offset0:60 offset1:63\n\t"
        "ds_read2_b64 %11, %16 offset0:66 offset1:69\n\t"
        "ds_read2_b64 %12, %16 offset0:72 offset1:75\n\t"
        "ds_read2_b64 %13, %16 offset0:78 offset1:81\n\t"
        "ds_read2_b64 %14, %16 offset0:84 offset1:87\n\t"
        "ds_read2_b64 %15, %16 offset0:90 offset1:93\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]),
          "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]),
          "=&v"(o[14]), "=&v"(o[15])
        : "v"(addr)
        : "memory");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[2 * i] = o[i].x;
        v[2 * i + 1] = o[i].y;
    }
}

// scipy lfilter DF2T step in fp64 with fused multiply-adds: y = z0 + b0 x,
// z_i = z_{i+1} + b_{i+1} x - a_{i+1} y (the b x + z part is off the y -> z chain)
template <int NS>
__device__ __forceinline__ double df2t_fma(const IirTileArgs& a, double (&z)[NS > 0 ? NS : 1], double x) {
    if constexpr (NS == 0) {
        return x * a.b[0];
    } else {
        const double y = __builtin_fma(a.b[0], x, z[0]);
#pragma unroll
        for (int i = 0; i < NS - 1; ++i) z[i] = __builtin_fma(-a.a[i + 1], y, __builtin_fma(a.b[i + 1], x, z[i + 1]));
        z[NS - 1] = __builtin_fma(-a.a[NS], y, a.b[NS] * x);
        return y;
    }
}

// the odd extension value at x sample t (t < 0 or t >= n), fp32 like numpy on the array
__device__ __forceinline__ float ext_value(const float* xc, int64_t ss, int64_t n, int64_t t) {
    if (t < 0) return 2.0f * xc[0] - xc[(-t) * ss];
    return 2.0f * xc[(n - 1) * ss] - xc[(2 * n - 2 - t) * ss];
}

// Two waves per workgroup: wave 1 is the DMA producer, wave 0 runs the recurrence. On
// gfx9 stores count in vmcnt with the loads, so a wave that both streams its input by DMA
// and stores its outputs cannot wait for "block b has landed" without also waiting for
// every store issued after that block's DMA (the ring would drain to one block ahead).
// Split, each wave's vmcnt holds one kind of operation: the producer waits for block b,
// fills in the extension samples, meets the consumer at an s_barrier and refills the slot
// the consumer finished with; the consumer reads block b after the same barrier.
template <int NS, int C, int P>
__global__ void __launch_bounds__(128) iir_tile_kernel(IirTileArgs a) {
    constexpr int ES = P == 0 ? 4 : 8;
    using G = FGeom<C, ES>;
    constexpr int U = G::U, NI = G::kNI, RN = G::kRingN, NP = G::kPieces, RS = G::kRowSlots;
    constexpr uint32_t kSlot = G::kSlotBytes;
    __shared__ __attribute__((aligned(16))) float4 ring[RN][NI * 64];
    const uint32_t ring_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)&ring[0][0]));

    const bool producer = threadIdx.x >= 64;
    const int lane = threadIdx.x & 63;
    const int r = lane / C, c = lane - (lane / C) * C;
    const int64_t k0 = static_cast<int64_t>(blockIdx.x) * U;  // first chunk of this workgroup
    const int64_t nk = a.K - k0 < U ? a.K - k0 : U;          // its chunks
    const bool unit = r < nk;
    const int64_t k = k0 + (unit ? r : nk - 1);
    const int64_t M = a.M, E = P == 0 ? a.E0 : a.E1;
    const int64_t NB = (E + M) / kFB;                        // blocks per chunk
    // pass-P position u: P0 the x sample t = j - padlen (x holds [0, n)), P1 the yr row j'
    // (yr holds [0, L)). Chunk k's blocks start at u = kM - E (a multiple of 32).
    const int64_t shift = P == 0 ? a.padlen : 0;
    const int64_t nvalid = P == 0 ? a.n : a.L;
    const int64_t ublk0 = k * M - E;
    const int64_t u_first = -shift;                          // the sequence's first position
    const int64_t cend0 = (k + 1) * M < a.L ? (k + 1) * M : a.L;
    // outputs: P0 every position of the chunk (yr holds all L of them); P1 those that map
    // to out rows t = L - 1 - padlen - j' in [0, n)
    const int64_t ebeg = P == 0 ? k * M - shift : (k * M > a.padlen ? k * M : a.padlen);
    const int64_t eend = P == 0 ? cend0 - shift : (cend0 < a.L - a.padlen ? cend0 : a.L - a.padlen);
    const int64_t ustart = ublk0 > u_first ? ublk0 : u_first;
    const bool init = ublk0 <= u_first;                      // starts at the sequence start
    const int64_t wave_u0 = k0 * M - E;                      // chunk k0's block 0
    const int64_t wave_uend = (k0 + nk - 1) * M - E + NB * kFB;
    const bool edge = wave_u0 < 0 || wave_uend > nvalid;     // some row leaves the array
    const uint32_t row_addr = ring_addr + static_cast<uint32_t>((unit ? r : 0) * RS * 16) +
                              static_cast<uint32_t>(c * ES);

    if (producer) {
        const char* in = P == 0 ? reinterpret_cast<const char*>(a.x) : reinterpret_cast<const char*>(a.yr);
        // per-lane DMA offsets: slot j = 64 i + lane holds piece kk of row rr
        uint32_t off[NI], poff[NI];
        int32_t row_u[NI];                                   // rr's block-0 u - wave_u0
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            int j = i * 64 + lane;
            if (j > U * RS - 1) j = U * RS - 1;
            int rr = j / RS;
            int kk = j - rr * RS;
            if (kk == NP) kk = NP - 1;                       // the pad slot repeats a piece
            if (rr > nk - 1) rr = static_cast<int>(nk - 1);
            row_u[i] = static_cast<int32_t>(rr * M);
            poff[i] = static_cast<uint32_t>(16 * kk) + kBias - static_cast<uint32_t>(fdma_inst_off(i));
            off[i] = static_cast<uint32_t>(static_cast<int64_t>(rr) * M * C * ES) + poff[i];
        }
        auto issue = [&](int64_t b) {
            const uint32_t slot = ring_addr + static_cast<uint32_t>(b % RN) * kSlot;
            if (!edge) {
                const uint64_t base = reinterpret_cast<uint64_t>(in) +
                                      static_cast<uint64_t>((wave_u0 + b * kFB) * C * ES) - kBias;
                dma_group<0, NI>(base, slot, off);
            } else {
                // every row's block clamped into [0, nvalid - 32] (rows leaving the array read
                // the nearest in-range block; the producer writes the extension samples, the
                // consumer masks the rest); the base is row 0's clamped block, the smallest,
                // so the 32-bit lane offsets stay non-negative
                auto clampu = [&](int64_t u) { return u < 0 ? int64_t(0) : (u > nvalid - kFB ? nvalid - kFB : u); };
                const int64_t ubase = clampu(wave_u0 + b * kFB);
                const uint64_t base = reinterpret_cast<uint64_t>(in) + static_cast<uint64_t>(ubase * C * ES) - kBias;
                uint32_t o2[NI];
#pragma unroll
                for (int i = 0; i < NI; ++i)
                    o2[i] = static_cast<uint32_t>((clampu(wave_u0 + row_u[i] + b * kFB) - ubase) * C * ES) + poff[i];
                dma_group<0, NI>(base, slot, o2);
            }
        };
        const float* xc = a.x + c;
#pragma unroll
        for (int s = 0; s < RN - 1; ++s)
            if (s < NB) issue(s);
        for (int64_t b = 0; b < NB; ++b) {
            // block b has landed once at most min(RN - 2, NB - 1 - b) newer blocks are out
            const int64_t newer = NB - 1 - b < RN - 2 ? NB - 1 - b : RN - 2;
            if (newer >= 2) wait_vmcnt<2 * NI>();
            else if (newer == 1) wait_vmcnt<NI>();
            else wait_vmcnt<0>();
            // a block that leaves the array was DMA'd from the clamped block: rewrite the
            // lane's row where it matters. Blocks start at multiples of 32, so at the start
            // they are wholly outside (pass 0: the odd extension); the one straddling the end
            // also holds in-range samples, shifted by the clamp, rewritten from memory.
            const int64_t ub = ublk0 + b * kFB;
            if (edge && unit && (ub < 0 || ub + kFB > nvalid)) {
                const uint32_t saddr = row_addr + static_cast<uint32_t>(b % RN) * kSlot;
                for (int p = 0; p < kFB; ++p) {
                    const int64_t t = ub + p;
                    if constexpr (P == 0) {
                        if (t >= -a.padlen && t < a.n + a.padlen) {
                            const float v = t < 0 || t >= a.n ? ext_value(xc, C, a.n, t) : xc[t * C];
                            *reinterpret_cast<__attribute__((address_space(3))) float*>(
                                static_cast<uintptr_t>(saddr + static_cast<uint32_t>(p * C * 4))) = v;
                        }
                    } else {
                        if (t >= 0 && t < a.L)
                            *reinterpret_cast<__attribute__((address_space(3))) double*>(
                                static_cast<uintptr_t>(saddr + static_cast<uint32_t>(p * C * 8))) = a.yr[t * C + c];
                    }
                }
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();                    // block b ready; b - 1 consumed
            if (b + RN - 1 < NB) issue(b + RN - 1);          // into block b - 1's slot
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }

    // ---- consumer: the recurrence, one lane per (chunk, channel)
    double z[NS > 0 ? NS : 1];
#pragma unroll
    for (int i = 0; i < (NS > 0 ? NS : 1); ++i) z[i] = 0.0;
    for (int64_t b = 0; b < NB; ++b) {
        __builtin_amdgcn_s_barrier();
        const uint32_t saddr = row_addr + static_cast<uint32_t>(b % RN) * kSlot;
        double xin[kFB];
        if constexpr (P == 0) {
            f2 v2[kFB / 2];
            lds_read_chunk<C>(saddr, v2);
#pragma unroll
            for (int q = 0; q < kFB / 2; ++q) {
                xin[2 * q] = static_cast<double>(v2[q].x);
                xin[2 * q + 1] = static_cast<double>(v2[q].y);
            }
        } else {
            lds_read_row64<C>(saddr, xin);
        }
        if (!unit) continue;
        const int64_t ub = ublk0 + b * kFB;                  // this lane's first position
        const bool full = ub >= ustart && ub + kFB <= eend && !(init && ub <= u_first && u_first < ub + kFB);
        const bool emit_all = ub >= ebeg && ub + kFB <= eend;
        const bool emit_none = ub + kFB <= ebeg;
        if (full && (emit_all || emit_none)) {
            if (emit_none) {
#pragma unroll
                for (int p = 0; p < kFB; ++p) (void)df2t_fma<NS>(a, z, xin[p]);
            } else if constexpr (P == 0) {
                // yr row of position u: L - 1 - (u + padlen), C doubles per row
                double* yp = a.yr + (a.L - 1 - a.padlen - ub) * C + c;
#pragma unroll
                for (int p = 0; p < kFB; ++p) yp[-p * C] = df2t_fma<NS>(a, z, xin[p]);
            } else {
                // out row t = L - 1 - padlen - u, in [0, n) for every u of an output block
                const int64_t t0 = a.L - 1 - a.padlen - ub;
                if (a.out_f32) {
                    float* op = static_cast<float*>(a.out) + t0 * C + c;
#pragma unroll
                    for (int p = 0; p < kFB; ++p) op[-p * C] = static_cast<float>(df2t_fma<NS>(a, z, xin[p]));
                } else {
                    double* op = static_cast<double*>(a.out) + t0 * C + c;
#pragma unroll
                    for (int p = 0; p < kFB; ++p) op[-p * C] = df2t_fma<NS>(a, z, xin[p]);
                }
            }
        } else {
            // a lane's first / last blocks: per-position start, init and output masks
            for (int p = 0; p < kFB; ++p) {
                const int64_t u = ub + p;
                if (u < ustart || u >= eend) continue;
                if (init && u == u_first) {
#pragma unroll
                    for (int i = 0; i < NS; ++i) z[i] = a.zi[i] * xin[p];
                }
                const double y = df2t_fma<NS>(a, z, xin[p]);
                if (u < ebeg) continue;
                if constexpr (P == 0) {
                    a.yr[(a.L - 1 - a.padlen - u) * C + c] = y;
                } else {
                    store_out(a.out, a.out_f32, (a.L - 1 - a.padlen - u) * C + c, y);
                }
            }
        }
    }
}

template <int NS, int C>
void launch_tile_ns(const IirTileArgs& a, hipStream_t s) {
    constexpr int U = 64 / C;
    const dim3 g(static_cast<unsigned>((a.K + U - 1) / U)), blk(128);
    hipLaunchKernelGGL((iir_tile_kernel<NS, C, 0>), g, blk, 0, s, a);
    hipLaunchKernelGGL((iir_tile_kernel<NS, C, 1>), g, blk, 0, s, a);
}

template <int C>
int launch_tile_c(const IirTileArgs& a, hipStream_t s) {
    switch (a.ns) {
#define MHF_NS(N) case N: launch_tile_ns<N, C>(a, s); break;
        MHF_NS(0) MHF_NS(1) MHF_NS(2) MHF_NS(3) MHF_NS(4) MHF_NS(5) MHF_NS(6) MHF_NS(7)
        MHF_NS(8) MHF_NS(9) MHF_NS(10) MHF_NS(11) MHF_NS(12) MHF_NS(13) MHF_NS(14)
        MHF_NS(15) MHF_NS(16)
#undef MHF_NS
    default: return MHF_EUNSUPPORTED;
    }
    return MHF_OK;
}

}  // namespace

int launch_filtfilt_tile(const IirTileArgs& a, hipStream_t s) {
    if (a.channels == 3) return launch_tile_c<3>(a, s);
    if (a.channels == 1) return launch_tile_c<1>(a, s);
    return MHF_EUNSUPPORTED;
}

}  // namespace mhf
