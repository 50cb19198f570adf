// tile_idx.hip.h — time-indexed windows (indices_rolling_apply / nonuniform_rolling_apply,
// src/mhealth/util/windows.py:134-157) through a register tile: each window is read from
// HBM once and kept on chip between the two passes.
//
// The reference's loop is a serial @jit loop over (start, end) pairs (windows.py:146-157):
// every window gets numba's serial models (np.mean = array_mean in fp32, np.var =
// array_var, ...), lengths vary window by window, and a window shorter than
// min_window_len is NaN. The lane-walk kernel (moments_indexed_kernel, mhfeat.hip) reads
// each window twice from global memory, and between its two passes a CU has ~1 MB of
// other windows in flight: pass 2 misses L2 (round 3: FETCH 2.03x the input, issue-active
// 0.11, 1.92 ms for 1e6 windows x 3 axes).
//
// Here, as in the fixed-window tile kernel (tile.hip.h), a lane owns one (window, channel)
// and a wave a tile of U = 64 / C consecutive windows; the windows' samples stream by
// LDS-DMA (global_load_lds_dwordx4, per-lane 32-bit offsets from a uniform SGPR base) in
// 32-sample chunks into a 4-slot ring and from there into registers (pass 1), and pass 2
// runs from registers. What differs:
//   * window starts are arbitrary: each window's DMA pieces start at its first byte
//     rounded down to 16 B (one more 16-B piece per chunk: the chunk image's pad slot),
//     and the lane's LDS reads start that many dwords in (ds_read2_b32 at any dword);
//   * lengths vary (at most kIdxWmax = 288 samples in the tile path): samples past a
//     window's end are zeroed as they are read, and the chunks past the tile's shortest
//     window take a predicated pass (t < W) — a ±0 term leaves a sum that started at +0
//     unchanged, so the kept sums are the reference's sequential sums bit for bit;
//   * len(x) is the window's own length: the skewness / kurtosis terms are divided by it
//     with the hoisted-reciprocal + Markstein correction of window_moments (mhfeat.hip,
//     exact for len <= 65536 while every nonzero |d| lies in [2^-25, 2^31]);
//   * any window the tile path cannot take — longer than kIdxWmax, outside that division
//     range, or in a tile whose DMA would reach past the record — is computed by its lane
//     with window_moments from global memory (the lane-walk kernel's own code), so every
//     window of every call is covered by this one launch.
#pragma once
#define MHF_TILE_IMPL
#ifndef MHF_TILE_FIX_EXTRA_NA
#define MHF_TILE_FIX_EXTRA_NA 96
#endif
#include "tile.hip.h"
#include "tile_idx.h"
#include "window_moments.h"

namespace mhf {
namespace {

constexpr int kIdxWmax = 288;                    // samples per window in the tile path
constexpr int kIdxNch = kIdxWmax / kChunk;       // 9 chunks
constexpr int kIdxNA = 96;                       // samples [NV, Wmax) parked in AGPRs
constexpr int kIdxNV = kIdxWmax - kIdxNA;        // 192 in VGPR pairs
// the fixed-window form with pass-1 extras carries more live state (the parfor chain, the
// extras' running values): it parks 96 more samples in AGPRs (192 of 288), which keeps it
// clear of scratch (+32 / +64 left 208 / 128 B per lane of spills) at one accvgpr read per
// sample more in pass 2
template <int X, bool FIX>
constexpr int idx_na() { return (FIX && X >= 1) ? kIdxNA + MHF_TILE_FIX_EXTRA_NA : kIdxNA; }
static_assert(kIdxNch >= kRing && kIdxWmax % kChunk == 0, "tile geometry");

// 32 samples of this lane's (window, channel) at any dword (ds_read2_b32 pairs: the C = 1
// image is no longer 16-B aligned per lane once windows start anywhere)
template <int C>
__device__ __forceinline__ void lds_read_chunk_any(uint32_t addr, f2 (&v)[16]);
template <>
__device__ __forceinline__ void lds_read_chunk_any<3>(uint32_t addr, f2 (&v)[16]) {
    lds_read_chunk<3>(addr, v);   // sample s of the lane's channel at dword 3s (+ the lane base)
}
template <>
__device__ __forceinline__ void lds_read_chunk_any<1>(uint32_t addr, f2 (&v)[16]) {
    asm volatile(
        "ds_read2_b32 %0, %16 offset1:1\n\t"
        "ds_read2_b32 %1, %16 offset0:2 offset1:3\n\t"
        "ds_read2_b32 %2, %16 offset0:4 offset1:5\n\t"
        "ds_read2_b32 %3, %16 offset0:6 offset1:7\n\t"
        "ds_read2_b32 %4, %16 offset0:8 offset1:9\n\t"
        "ds_read2_b32 %5, %16 offset0:10 offset1:11\n\t"
        "ds_read2_b32 %6, %16 offset0:12 offset1:13\n\t"
        "ds_read2_b32 %7, %16 offset0:14 offset1:15\n\t"
        "ds_read2_b32 %8, %16 offset0:16 offset1:17\n\t"
        "ds_read2_b32 %9, %16 offset0:18 offset1:19\n\t"
        "ds_read2_b32 %10, %16 offset0:20 offset1:21\n\t"
        "ds_read2_b32 %11, %16 offset0:22 offset1:23\n\t"
        "ds_read2_b32 %12, %16 offset0:24 offset1:25\n\t"
        "ds_read2_b32 %13, %16 offset0:26 offset1:27\n\t"
        "ds_read2_b32 %14, %16 offset0:28 offset1:29\n\t"
        "ds_read2_b32 %15, %16 offset0:30 offset1:31\n\t"
        MHF_LDS_WAIT
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
          "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]),
          "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15])
        : "v"(addr)
        : "memory");
}

// Full-wave reductions through DPP: row_ror 1 / 2 / 4 / 8 leave every lane of a row of 16
// with the row's value, row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry them up,
// lane 63 holds the wave's (read as a scalar). The __shfl_xor butterflies they replace were
// 6 (12 for 64-bit) dependent ds_bpermute round trips each, four reductions per tile
// (round 6: ~4k cycles of a time-indexed tile's setup). Lanes a row_bcast does not write
// keep their own value (old = v).
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), CTRL, RM,
                                                             0xf, false));
}
template <int CTRL, int RM, bool MAX>
__device__ __forceinline__ uint64_t dpp_step_u64(uint64_t v) {
    const uint64_t w = static_cast<uint64_t>(dpp_u32<CTRL, RM>(static_cast<uint32_t>(v))) |
                       (static_cast<uint64_t>(dpp_u32<CTRL, RM>(static_cast<uint32_t>(v >> 32))) << 32);
    return MAX ? (w > v ? w : v) : (w < v ? w : v);
}
template <bool MAX>
__device__ __forceinline__ uint64_t wave_reduce_u64(uint64_t v) {
    v = dpp_step_u64<0x121, 0xf, MAX>(v);   // row_ror:1
    v = dpp_step_u64<0x122, 0xf, MAX>(v);   // row_ror:2
    v = dpp_step_u64<0x124, 0xf, MAX>(v);   // row_ror:4
    v = dpp_step_u64<0x128, 0xf, MAX>(v);   // row_ror:8
    v = dpp_step_u64<0x142, 0xa, MAX>(v);   // row_bcast:15
    v = dpp_step_u64<0x143, 0xc, MAX>(v);   // row_bcast:31
    return static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63))) |
           (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), 63))) << 32);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) { return wave_reduce_u64<false>(v); }
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) { return wave_reduce_u64<true>(v); }
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_min_i32(int v) {
    const int w = static_cast<int>(dpp_u32<CTRL, RM>(static_cast<uint32_t>(v)));
    return w < v ? w : v;
}
__device__ __forceinline__ int wave_min_i32(int v) {
    v = dpp_min_i32<0x121, 0xf>(v);
    v = dpp_min_i32<0x122, 0xf>(v);
    v = dpp_min_i32<0x124, 0xf>(v);
    v = dpp_min_i32<0x128, 0xf>(v);
    v = dpp_min_i32<0x142, 0xa>(v);
    v = dpp_min_i32<0x143, 0xc>(v);
    return __builtin_amdgcn_readlane(v, 63);
}

// SPAN (fixed windows overlapping, S < W): the LDS image of the tile's union span, one DMA
// pass per tile (dma::span_geom, dma::kSpanBytes per wave)
using dma::kSpanBytes;

// the tile's span image: piece p = 64 k + lane of DMA instruction k, 16 B from g.gbase + 16 p
// into span byte 16 p (nt: each byte of the span is read by this wave only, once)
__device__ __forceinline__ void issue_span(const dma::SpanGeom& g, uint32_t span_addr, int lane) {
    const uint32_t voff = 16u * static_cast<uint32_t>(lane);
    const int ni = static_cast<int>((g.nbytes + 1023u) >> 10);
    for (int k = 0; k < ni; ++k) {
        if (voff < g.nbytes - 1024u * static_cast<uint32_t>(k)) {
            // M0 (SALU) -> LDS-DMA needs 1 wait state, a VALU-written SGPR base -> VMEM 5
            // (dma_chunk, tile.hip.h): s_nop 4 covers both
            asm volatile("s_nop 4\n\tglobal_load_lds_dwordx4 %1, %2" MHF_DMA_POLICY
                         :
                         : "{m0}"(span_addr + 1024u * static_cast<uint32_t>(k)), "v"(voff),
                           "s"(g.gbase + 1024u * static_cast<uint64_t>(k))
                         : "memory");
        }
    }
}
template <int C, int X, bool FIX, bool SPAN = false, bool PAR = false>
__global__ void __launch_bounds__(64, 1) tile_idx_kernel(IdxTileArgs a) {
    static_assert(!SPAN || FIX, "the span image is for fixed windows");
    static_assert(!PAR || FIX, "the parfor chain is for fixed windows");
    using G = TileGeom<C>;
    constexpr int U = G::U;
    constexpr int KD = kDma;
    constexpr int NCH = kIdxNch;
    constexpr int NA = idx_na<X, FIX>(), NV = kIdxWmax - NA;
    constexpr int64_t CH = kChunk * C * 4;        // bytes of one chunk of one window
    static_assert(dma::kSpanRead == kIdxWmax, "span reads = the tile's window registers");
    __shared__ __attribute__((aligned(16))) float4 ring[SPAN ? kSpanBytes / 16 : kRing * KD * 64];

    const int lane = threadIdx.x;
    const int r = lane / C, c = lane - (lane / C) * C;
    const bool unit = r < U;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    const uint32_t ring_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)&ring[0]));
    // the span geometry of tile tl (uniform)
    auto span_of = [&](int64_t tl) {
        const int64_t i0 = tl * U;
        const int64_t ntw = a.nwin - i0 < U ? a.nwin - i0 : U;
        return dma::span_geom(reinterpret_cast<uintptr_t>(a.x), a.n_samples, C, a.first + i0, ntw,
                              a.wstep, a.wsize, kSpanBytes);
    };
    if constexpr (SPAN) {
        if (static_cast<int64_t>(blockIdx.x) < ntiles) issue_span(span_of(blockIdx.x), ring_addr, lane);
    }
    constexpr uint32_t kSlotBytes = KD * 1024;
    const int64_t F = a.feats.n;
    const bool need_p2 = (a.mask & (kPass2Bits | bit(MHF_COEFF_VAR))) != 0;
    // fixed windows: rows >= 1 of a direct np.var / np.std are numba's parfor chain (fp64
    // deviations from the fp64 mean, var_parallel_impl; tile.hip.h): replayed (PAR, on
    // MHF_NUMERICS_EXACT_VAR) or by default taken from pass 2's ssd within the fast-var
    // bound, a lane that fails fast_var_ok walking the exact models instead
    const bool want_var = FIX && (a.mask & (bit(MHF_VAR) | bit(MHF_STD))) != 0;
    const bool want_par = PAR && want_var;
    const bool want_zc = (a.mask & bit(MHF_ZERO_CROSSINGS)) != 0;
    const uintptr_t xb = reinterpret_cast<uintptr_t>(a.x);

    f2 R[NV / 2];
    float RA[NA];

    // time-indexed windows: the (start, end) pair of the lane's window in the next tile is
    // loaded one tile ahead (its global-load latency used to open every tile's setup)
    int64_t nsi = 0, nei = 0;
    if constexpr (!FIX) {
        const int64_t i0 = static_cast<int64_t>(blockIdx.x) * U + r;
        if (unit && i0 < a.nwin) { nsi = a.starts[i0]; nei = a.ends[i0]; }
    }
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        // ---- this lane's window: Python slice bounds of arr[si:ei] (windows.py:150-154)
        const int64_t i = tile * U + r;
        const bool valid = unit && i < a.nwin;
        int64_t s0 = 0, W64 = 0, g = 0;
        bool keep = false;
        const int64_t csi = nsi, cei = nei;
        if constexpr (!FIX) {
            const int64_t in = (tile + gridDim.x) * U + r;
            if (unit && in < a.nwin) { nsi = a.starts[in]; nei = a.ends[in]; }
        }
        if (FIX && valid) {
            // rolling_apply's window g = first + i: x[g * wstep : g * wstep + wsize]
            // (windows.py:68-72), every one inside the record
            g = a.first + i;
            s0 = g * a.wstep;
            W64 = a.wsize;
            keep = true;
        } else if (valid) {
            const int64_t si = csi, ei = cei, n = a.n_samples;
            int64_t b0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
            b0 = b0 < 0 ? 0 : (b0 > n ? n : b0);
            e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
            s0 = b0;
            W64 = e0 > b0 ? e0 - b0 : 0;
            keep = (ei - si >= a.min_len) && W64 > 0;
        }
        dma::SpanGeom sg{};
        if constexpr (SPAN) {
            sg = span_of(tile);
#ifndef MHF_DIAG_NO_SPANWAIT
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tile's span image is in
#endif
        }
        // ---- the tile path: every kept window's 9 chunks inside the record (DMA bounds:
        // the last piece ends before sample s0 + kIdxWmax + 4), offsets within 2^31
        const uint64_t bstart = xb + static_cast<uint64_t>(s0) * C * 4;
        const uint64_t base_lane = dma::idx_piece_base(bstart);    // 16-B aligned piece grid
        // (a record not 16-B aligned: window 0's first piece would start before it)
        const bool dma_ok = !keep || (s0 + kIdxWmax + 4 <= a.n_samples && base_lane >= xb);
        const uint64_t bmin = SPAN ? 0 : wave_min_u64(keep ? base_lane : ~uint64_t(0));
        const uint64_t bmax = SPAN ? 0 : wave_max_u64(keep ? base_lane : 0);
        const bool any_keep = __ballot(keep) != 0;
        const bool tile_ok = SPAN ? any_keep && sg.ok
                                  : any_keep && __ballot(!dma_ok) == 0 && bmax - bmin < (uint64_t(1) << 30);
        // lanes the tile path leaves to the global-memory walk (longer than the tile)
        bool slow = keep && (!tile_ok || W64 > kIdxWmax);
        const int W = static_cast<int>(tile_ok && keep && !slow ? W64 : 0);
        WinVals v{};
        if (tile_ok) {
            // shortest window of the tile path: chunks wholly below it need no predicate
            const int wmin = wave_min_i32(keep && !slow ? W : kIdxWmax);
            // longest: chunks wholly past it are skipped (their DMA still runs, as the ring's
            // wait counts are static)
            const int wmax = -wave_min_i32(keep && !slow ? -W : 0);
            // per-slot DMA offsets: slot j = 64 q + lane of instruction q holds piece k of
            // tile-window rr; a window that is not kept borrows the first kept one's pieces
            // (the first kept window's base by readlane, outside any branch: round 5's first
            // GPU runs faulted because `krr ? brr : __shfl(...)` evaluated the second shuffle
            // only in the lanes of non-kept windows, and a ds_bpermute under a partial EXEC
            // reads the disabled source lanes as 0 — a base of 0, an offset 4 GiB wide)
            // (SPAN: none of the ring's per-slot offsets — the span image is in LDS already)
            const int first_keep = SPAN ? 0 : __builtin_ctzll(__ballot(keep)) / C;
            const uint64_t bfk =
                dma::sgpr_pair(__builtin_amdgcn_readlane(static_cast<int>(dma::lo_word(base_lane)), first_keep * C),
                               __builtin_amdgcn_readlane(static_cast<int>(dma::hi_word(base_lane)), first_keep * C));
            // lim[q]: the slot's piece is past its window's last byte in chunks jj with
            // jj * CH >= lim[q] (non-kept windows: never); those pieces are fetched from the
            // previous chunk's slot address instead — bytes the previous DMA just read, so
            // the window's DMA no longer reaches into the next window's lines (HBM read was
            // 1.28 x the covered input, profiles/r05b_cfgidx_summary.md). The LDS slot then
            // holds other samples, past the window's end, which pass 1 zeroes as it reads.
            const int wbytes = keep ? static_cast<int>(static_cast<uint32_t>(bstart - base_lane) +
                                                       (W64 < 4096 ? W64 : 4096) * C * 4)
                                    : 0x7fffffff;
            uint32_t off[kDma];
            int32_t lim[kDma];
#pragma unroll
            for (int q = 0; q < (SPAN ? 0 : kDma); ++q) {
                int j = q * 64 + lane;
                if (j > U * G::kWinSlots - 1) j = U * G::kWinSlots - 1;
                int rr = j / G::kWinSlots;
                const int k = j - rr * G::kWinSlots;
                const int src = rr * C;                           // lane of window rr
                const uint64_t brr = __shfl(base_lane, src, 64);
                const bool krr = __shfl(static_cast<int>(keep), src, 64) != 0;
                const int wrr = __shfl(wbytes, src, 64);
                const uint64_t b = krr ? brr : bfk;
                off[q] = dma::idx_lane_off(b, bmin, k, q);
                lim[q] = dma::idx_lane_lim(krr, wrr, k);
            }
            // (readfirstlane returns int: the low word goes through uint32_t, or a low word
            // >= 2^31 sign-extends over the high word — the address fault of the first GPU
            // run of this kernel, round 5)
            const uint64_t sbase = dma::sgpr_pair(__builtin_amdgcn_readfirstlane(dma::lo_word(bmin - kBias)),
                                                  __builtin_amdgcn_readfirstlane(dma::hi_word(bmin - kBias)));
            // this lane's reads: window r's image starts at dword r * kWinSlots * 4 (+ c), and
            // its first sample (bstart - base_lane) bytes into it
            const uint32_t mis = static_cast<uint32_t>(bstart - base_lane);
            uint32_t lane_addr = ring_addr + static_cast<uint32_t>((unit ? r : 0) * G::kWinSlots * 16) + mis;
            if constexpr (C > 1) lane_addr += static_cast<uint32_t>(c * 4);
            // SPAN: window r's samples from span byte mis0 + (r S C + c) 4, chunk j 128 C
            // bytes further (lanes past the tile's last window read what lies there: unused)
            if constexpr (SPAN)
                lane_addr = ring_addr + dma::span_lane_byte(sg.mis0, unit ? r : 0, a.wstep, C, c, 0);
            // chunk jj of every window; chunks that reach past the tile's shortest window
            // (uniform) redirect the pieces past each window's end (lim). Chunk 0 never does:
            // its previous-chunk address could precede the record. Time-indexed windows
            // only: past a fixed window's end are the next windows' samples when they
            // overlap, a prefetch (ovl250 measured 3.64 -> 3.93 ms with the redirect)
            auto issue = [&](auto JJ, uint32_t slot) {
                constexpr int jj = decltype(JJ)::value;
                if (!FIX && jj > 0 && (jj + 1) * kChunk > wmin) {
                    uint32_t o2[kDma];
#pragma unroll
                    for (int q = 0; q < kDma; ++q)
                        o2[q] = dma::idx_redirect(off[q], jj * CH, lim[q], CH);
                    dma_chunk(sbase + static_cast<uint64_t>(jj * CH), slot, o2);
                } else {
                    dma_chunk(sbase + static_cast<uint64_t>(jj * CH), slot, off);
                }
            };
            if constexpr (!SPAN) static_for<0, kRing>([&](auto J) { issue(J, ring_addr + J.value * kSlotBytes); });

            // ---- pass 1 (reference order): fp32 sum, zero crossings, extras; the window
            // lands in R / RA with the samples past its end zeroed
            float c32 = 0.0f, a32 = 0.0f, ll = 0.0f, mn = 0.0f, mx = 0.0f, p1 = 0.0f, p2 = 0.0f;
            int zc = 0, pk = 0;
            bool prevpos = false;
            static_for<0, NCH>([&](auto JJ) {
                constexpr int j = decltype(JJ)::value;
                constexpr int last = (j + kRing - 1 < NCH - 1) ? j + kRing - 1 : NCH - 1;
                if constexpr (!SPAN) wait_vmcnt<(last - j) * KD>();
                // (chunks past every window of the tile are still read here — a skipped read
                // left the extras-level kernels 128-256 B per lane of spills — and skipped
                // by pass 2)
                f2 v2[kChunk / 2];
                if constexpr (SPAN) {
                    lds_read_chunk_any<C>(lane_addr + static_cast<uint32_t>(j * CH), v2);
                } else {
                    lds_read_chunk_any<C>(lane_addr + (j % kRing) * kSlotBytes, v2);
                    // slot j % kRing is free again: refill with chunk j + kRing
                    if constexpr (j + kRing < NCH)
                        issue(std::integral_constant<int, j + kRing>{}, ring_addr + (j % kRing) * kSlotBytes);
                }
                const bool tail = (j + 1) * kChunk > wmin;        // uniform
                auto body = [&](auto TAILT) {
                    constexpr bool TAIL = decltype(TAILT)::value;
                    static_for<0, kChunk / 2>([&](auto Q) {
                        constexpr int q = decltype(Q)::value;
                        constexpr int t0 = j * kChunk + 2 * q;
                        f2 pv = v2[q];
                        if constexpr (TAIL) {
                            pv.x = (t0 < W) ? pv.x : 0.0f;
                            pv.y = (t0 + 1 < W) ? pv.y : 0.0f;
                        }
                        if constexpr (t0 < NV) {
                            R[t0 / 2] = pv;
                        } else {
                            asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t0 - NV]) : "v"(pv.x));
                            asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t0 + 1 - NV]) : "v"(pv.y));
                        }
                        static_for<0, 2>([&](auto H) {
                            constexpr int t = t0 + decltype(H)::value;
                            const float x = decltype(H)::value ? pv.y : pv.x;
                            const bool in = !TAIL || t < W;
                            c32 = c32 + x;                 // a zeroed sample adds +0: no change
                            if (want_zc) {
                                const bool pos = x > a.t32;
                                if constexpr (t > 0) zc += (in && pos != prevpos) ? 1 : 0;
                                prevpos = pos;
                                asm volatile("" : "+v"(zc));
                            }
                            if constexpr (X >= 1) {
                                a32 = a32 + x * x;
                                if constexpr (t > 1) pk += (in && p1 > p2 && p1 > x) ? 1 : 0;
                                asm volatile("" : "+v"(pk));
                            }
                            if constexpr (X >= 2) {
                                if constexpr (t == 0) {
                                    mn = x; mx = x;
                                } else if (in) {
                                    mn = (x < mn) ? x : mn;
                                    mx = (x > mx) ? x : mx;
                                    ll = ll + fabsf(x - p1);
                                }
                            }
                            if constexpr (X >= 1) {
                                p2 = p1;
                                p1 = x;
                            }
                        });
                    });
                };
                if (tail) body(std::true_type{});
                else body(std::false_type{});
            });

            // SPAN: pass 1 has read the image (each chunk read waits for its data), so the
            // next tile's span DMA runs under this tile's pass 2
            if constexpr (SPAN) {
                if (tile + gridDim.x < ntiles) issue_span(span_of(tile + gridDim.x), ring_addr, lane);
            }
            // ---- pass 2 from registers: deviations from the fp32 mean (array_var,
            // skewness, kurtosis); each term / len(x) as a multiply by y = RN(1 / W) plus
            // one Markstein correction (window_moments, mhfeat.hip), with the |d| range
            // that makes it exact tracked per lane
            const float Wf = static_cast<float>(W > 0 ? W : 1);
            const float invW = 1.0f / Wf;
            const float m32 = static_cast<float>(static_cast<double>(c32) / static_cast<double>(W > 0 ? W : 1));
            const double m64 = static_cast<double>(c32) / static_cast<double>(W > 0 ? W : 1);
            double ssd = 0.0, ssdp = 0.0;
            float s3 = 0.0f, s4 = 0.0f, dmax = 0.0f;
            uint32_t dmin2 = 0xfffffffeu, dmin1 = 0xffffffffu;
            if (need_p2) {
                const f2 M2 = {m32, m32}, IW2 = {invW, invW}, WF2 = {Wf, Wf};
                static_for<0, NCH>([&](auto JJ) {
                    constexpr int j = decltype(JJ)::value;
                    const bool tail = (j + 1) * kChunk > wmin;
                    if (j > 0 && j * kChunk >= wmax) return;       // past every window
                    auto body = [&](auto TAILT) {
                        constexpr bool TAIL = decltype(TAILT)::value;
                        static_for<0, kChunk / 2>([&](auto Q) {
                            constexpr int t0 = j * kChunk + 2 * decltype(Q)::value;
                            f2 X2;
                            if constexpr (t0 < NV) {
                                X2 = R[t0 / 2];
                            } else {
                                asm("v_accvgpr_read_b32 %0, %1" : "=v"(X2.x) : "a"(RA[t0 - NV]));
                                asm("v_accvgpr_read_b32 %0, %1" : "=v"(X2.y) : "a"(RA[t0 + 1 - NV]));
                            }
                            f2 D = X2 - M2;
                            if constexpr (TAIL) {                  // d = ±0 past the end
                                D.x = (t0 < W) ? D.x : 0.0f;
                                D.y = (t0 + 1 < W) ? D.y : 0.0f;
                            }
                            const f2 Q2 = D * D;
                            const f2 A3 = D * Q2, A4 = Q2 * Q2;
                            const f2 Q3 = A3 * IW2, Q4 = A4 * IW2;
                            const f2 T3 = __builtin_elementwise_fma(__builtin_elementwise_fma(-Q3, WF2, A3), IW2, Q3);
                            const f2 T4 = __builtin_elementwise_fma(__builtin_elementwise_fma(-Q4, WF2, A4), IW2, Q4);
                            ssd = ssd + static_cast<double>(Q2.x);
                            s3 = s3 + T3.x;
                            s4 = s4 + T4.x;
                            ssd = ssd + static_cast<double>(Q2.y);
                            s3 = s3 + T3.y;
                            s4 = s4 + T4.y;
                            if constexpr (PAR) {
                                if (want_par) {
                                    double dx = static_cast<double>(X2.x) - m64;
                                    double dy = static_cast<double>(X2.y) - m64;
                                    if constexpr (TAIL) {
                                        dx = (t0 < W) ? dx : 0.0;
                                        dy = (t0 + 1 < W) ? dy : 0.0;
                                    }
                                    ssdp = ssdp + dx * dx;
                                    ssdp = ssdp + dy * dy;
                                }
                            }
                            asm volatile("" : "+v"(ssd), "+v"(s3), "+v"(s4), "+v"(ssdp));
                            // |d| bits x 2 - 2 (the shift drops the sign, a zero wraps to
                            // the top): one v_lshl_add each, then a v_min3_u32; the |d| max
                            // as a v_max3_f32 with abs modifiers (was 8 VALU per pair). The
                            // fixed-window kernel keeps the masked form: measured faster
                            // there (ovl250 3.66-3.69 vs 3.88-3.95 ms; cfgidx 1.15 vs 1.17-1.19)
                            if constexpr (!FIX) {
                                const uint32_t ux = __float_as_uint(D.x) * 2u - 2u;
                                const uint32_t uy = __float_as_uint(D.y) * 2u - 2u;
                                dmin2 = min(dmin2, min(ux, uy));
                                dmax = fmaxf(dmax, fmaxf(fabsf(D.x), fabsf(D.y)));
                            } else {
                                const uint32_t bx = __float_as_uint(D.x) & 0x7fffffffu;
                                const uint32_t by = __float_as_uint(D.y) & 0x7fffffffu;
                                dmin1 = min(dmin1, min(bx - 1u, by - 1u));
                                dmax = fmaxf(dmax, fmaxf(__uint_as_float(bx), __uint_as_float(by)));
                            }
                        });
                    };
                    if (tail) body(std::true_type{});
                    else body(std::false_type{});
                });
                // smallest nonzero |d| (bits; x 2 in the indexed form), 0 if every d is 0
                const uint32_t mnz = FIX ? dmin1 + 1u : (dmin2 + 2u) >> 1;
                const bool exact = W <= 65536 && !(dmax > 0x1p31f) &&
                                   (mnz == 0u || mnz >= 0x33000000u /* 2^-25 */);
                if (!exact) slow = slow || keep;                      // IEEE division: the walk
                if constexpr (FIX && !PAR) {
                    if (want_var && keep && g != 0 && !fast_var_ok(ssd, c32, m32, m64, W)) slow = true;
                }
            }
            const float var32 = static_cast<float>(ssd / static_cast<double>(W > 0 ? W : 1));
            const float std32 = static_cast<float>(sqrt(static_cast<double>(var32)));
            const bool par = FIX && g != 0;                   // prange rows (windows.py:68-72)
            const double varp = (PAR ? ssdp : ssd) / static_cast<double>(W > 0 ? W : 1);
            v.mean32 = m32;
            v.mean = par ? m64 : static_cast<double>(m32);
            v.var32 = var32;
            v.var = par ? varp : static_cast<double>(var32);
            v.std32 = std32;
            v.std_ = par ? sqrt(varp) : static_cast<double>(std32);
            v.skew = (std32 == 0.0f) ? 0.0 : static_cast<double>(s3 / (std32 * (std32 * std32)));
            const float kurt = (var32 == 0.0f) ? 0.0f : s4 / (var32 * var32);
            v.kurt = kurt;
            v.kurt_ex = static_cast<double>(kurt) - 3.0;
            v.rms = sqrtf(static_cast<float>(static_cast<double>(a32) / static_cast<double>(W > 0 ? W : 1)));
            v.zc = zc;
            v.peaks = pk;
            v.drange = static_cast<double>(mx - mn);
            v.ll = ll;
            v.cv = static_cast<double>(std32 / m32);
        }
        // SPAN: a tile the image does not serve (its lanes walk global memory) still starts
        // the next tile's span DMA
        if constexpr (SPAN) {
            if (!tile_ok && tile + gridDim.x < ntiles) issue_span(span_of(tile + gridDim.x), ring_addr, lane);
        }
        // ---- the lanes the tile path left: numba's serial models straight from global
        // memory (moments_indexed_kernel's code), one lane per (window, channel)
        if (slow) {
            const float* p = a.x + c + s0 * C;
            v = window_moments<false>(GlobAcc{p, C, W64}, W64, !FIX || g == 0, a.mask, a.t32, a.xp);
            // default numerics: rows >= 1 of np.var / np.std by the tile path's rule (ssd / W
            // where fast_var_ok holds), so a window gets the same bits whichever path took it
            // (a tile at the record's end walks: one launch = two half launches, bit for bit)
            if constexpr (FIX && !PAR) {
                if (want_var && keep && g != 0) {
                    float c32w = 0.0f;
                    double ssdw = 0.0;
                    for (int64_t t = 0; t < W64; ++t) c32w = c32w + p[t * C];
                    for (int64_t t = 0; t < W64; ++t) {
                        const float d = p[t * C] - v.mean32;
                        const float q = d * d;
                        ssdw = ssdw + static_cast<double>(q);
                    }
                    if (fast_var_ok(ssdw, c32w, v.mean32, v.mean, static_cast<int>(W64))) {
                        v.var = ssdw / static_cast<double>(W64);
                        v.std_ = sqrt(v.var);
                    }
                }
            }
        }
#ifdef MHF_DIAG_NO_STORE
        if (valid && a.first < 0) {   // timing diagnostic only (results garbage): price the stores
#else
        if (valid) {
#endif
            for (int jf = 0; jf < F; ++jf) {
                const int f = a.feats.id[jf];
                if (!(bit(f) & kTileIdxBits)) continue;         // order-statistic columns
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * F + jf) * a.out_ld + i,
                          keep ? pick_moment(v, f) : static_cast<double>(NAN));
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// the span image (SPAN) for overlapping fixed windows whose tile span fits kSpanBytes and whose
// span reads stay <= 2-way bank-conflicted (odd S, or S = 2 mod 4, for C = 1); MHF_NO_TILE_SPAN
// (diagnostic) keeps the per-window chunk DMA
template <int C>
bool tile_span_plan(const IdxTileArgs& a) {
    constexpr int64_t U = 64 / C;
    return a.wstep < a.wsize && 16 + ((U - 1) * a.wstep + dma::kSpanRead) * C * 4 <= kSpanBytes &&
           dma::span_bank_ways(a.wstep, C) <= 2 && !disabled("MHF_NO_TILE_SPAN");
}

template <int C, bool FIX>
int launch_tile_idx_c(const IdxTileArgs& a, hipStream_t stream) {
    const int64_t U = 64 / C;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    const int64_t blocks = ntiles < 1024 ? ntiles : 1024;   // 256 CUs x 4 waves, persistent
    const fmask_t xl1 = bit(MHF_RMS) | bit(MHF_PEAK_COUNT), xl2 = bit(MHF_DRANGE) | bit(MHF_LINE_LENGTH);
    const int x = (a.mask & xl2) ? 2 : ((a.mask & xl1) ? 1 : 0);
    const dim3 grid(static_cast<unsigned>(blocks)), block(64);
    if constexpr (FIX) {
        const bool par = a.exact_var && (a.mask & (bit(MHF_VAR) | bit(MHF_STD))) != 0;
#define MHF_TF(X, SP, P) hipLaunchKernelGGL((tile_idx_kernel<C, X, true, SP, P>), grid, block, 0, stream, a)
#define MHF_TFX(SP, P) do { if (x == 2) MHF_TF(2, SP, P); else if (x == 1) MHF_TF(1, SP, P); else MHF_TF(0, SP, P); } while (0)
        if (tile_span_plan<C>(a)) {
            if (par) MHF_TFX(true, true);
            else MHF_TFX(true, false);
        } else {
            if (par) MHF_TFX(false, true);
            else MHF_TFX(false, false);
        }
#undef MHF_TFX
#undef MHF_TF
        return MHF_OK;
    }
    if (x == 2) hipLaunchKernelGGL((tile_idx_kernel<C, 2, FIX>), grid, block, 0, stream, a);
    else if (x == 1) hipLaunchKernelGGL((tile_idx_kernel<C, 1, FIX>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((tile_idx_kernel<C, 0, FIX>), grid, block, 0, stream, a);
    return MHF_OK;
}

}  // namespace mhf
