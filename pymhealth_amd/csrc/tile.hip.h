// tile.hip.h — the fused tile kernel: register-resident windows fed by LDS-DMA.
//
// Why this shape: numba's per-window reductions are sequential
// fp32/fp64 accumulations, so one LANE must own one window and walk
// its samples in order; two passes (mean, then deviations) need the whole window on
// chip. A lane keeps its window in registers (W = 128 / 256 floats: VGPRs, plus AGPRs
// for the last 64 samples of W = 256), so a wave holds 64 (window, channel) units and
// runs at one wave per SIMD. At one wave per SIMD every instruction costs one issue
// slot of ~5 cycles (tools/valu_probe.hip: v_add_f32 4.7, v_pk_*_f32 / f64 5.4, an
// interleaved SALU op +4.1), so the kernel is written for the fewest instructions per
// sample: packed fp32 (v_pk_*) for the independent per-sample products of pass 2, the
// AoS channel split done by the LDS read (ds_read2_b32), DMA addresses from a
// uniform SGPR base plus 32-bit lane offsets.
//
// HBM is streamed by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) into a per-wave
// ring of 16-sample chunks, kept RING-1 chunks ahead — across tile boundaries too, so the
// second pass and the stores of one tile overlap the loads of the next.
//
// Data layout: x is AoS float32, sample t of channel c of the signal at x[t*C + c]
// (C = 1: a contiguous 1-D signal). Window w covers samples [w*S, w*S + W).
// Lane l owns unit (window r = l / C of the tile, channel c = l % C); a tile is
// U = 64 / C windows. LDS image of one chunk (16 samples of U windows, all channels,
// 16-byte pieces):
//   C = 1: piece k (k < 4) of tile-window r at slot k*64 + r: the owning lane reads
//          consecutive slots with ds_read_b128 (conflict-free);
//   C = 3: the 12 pieces of tile-window r at slots 13r .. 13r+11 (slot 13r+12 pads the
//          window stride to 52 dwords: <= 2-way bank conflicts), so sample s of channel
//          c sits at dword 52r + 3s + c and a lane reads its own channel with
//          ds_read2_b32 (two samples per instruction, no select).
#pragma once

#include "engine_common.h"
#include "dma_map.h"

#include <cstddef>

namespace mhf {

// Kernel-argument tables of the in-lane spectral features (host-built per call, read
// through scalar loads). Bins come in pairs (k, N-k), k = 0..N/2: pair 0 = (DC, Nyquist),
// pair N/2 = (N/2, unused). bw: band weights (0/1) per pair lane; dw[2k] = +1 inside the
// dominant-frequency range [dom_lo, dom_hi) and -1 outside, bin k = 0..N (dw[2k+1] unused).
constexpr int kMaxLanePairs = 65;   // W = 256: N/2 + 1
constexpr int kMaxLaneBins = 129;   // W/2 + 1
struct SpecTables {
    float bw[2 * kMaxLanePairs];
    float dw[2 * kMaxLaneBins];
};

struct FastArgs {
    const float* x;
    int64_t ch_stride, sample_stride, wstep, first, nwin;
    int32_t channels;
    fmask_t mask;
    float t32;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    int32_t band_lo, band_hi, dom_lo, dom_hi;
    float scale;
    double freq_step;
    int32_t exact_var;   // MHF_NUMERICS_EXACT_VAR: replay var_parallel_impl's fp64 chain
    SpecTables spec;     // band / dominant-frequency bin weights (spectral_lane.hip.inc)
};

inline bool fast_plan_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                         int64_t wstep, fmask_t mask) {
    if (mask & kGenericOnlyBits) return false;
    if (!(wsize == 128 || wsize == 256)) return false;
    if (!(channels == 1 || channels == 3)) return false;
    if (sample_stride != channels) return false;
    if (channels > 1 && ch_stride != 1) return false;
    // overlapping windows (wstep < wsize) are fine: every window's chunks are DMA'd on
    // their own; the shared samples of neighbouring windows are L2 hits of lines the
    // same or the previous DMA instruction fetched, so HBM still sees each byte once
    if ((wstep * channels) % 4 != 0) return false;    // 16-B aligned window starts
    // per-lane DMA offsets are 32-bit: a tile (64 windows) must span < 2 GiB
    if (wstep * channels * 4 * 64 >= (int64_t(1) << 31)) return false;
    return true;
}

inline const char* fast_plan_name(int64_t wsize, int32_t channels) {
    if (wsize == 256) return channels == 1 ? "tile_w256_c1" : "tile_w256_c3";
    return channels == 1 ? "tile_w128_c1" : "tile_w128_c3";
}

// one translation unit per (W, C, spectral): tile_w<W>_c<C>_s<0|1>.hip (parallel builds)
int launch_tile_w256_c1_s0(const FastArgs& a, hipStream_t stream);
int launch_tile_w256_c1_s1(const FastArgs& a, hipStream_t stream);
int launch_tile_w256_c3_s0(const FastArgs& a, hipStream_t stream);
int launch_tile_w256_c3_s1(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c1_s0(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c1_s1(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c3_s0(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c3_s1(const FastArgs& a, hipStream_t stream);

// float64 records (tile64.hip): each tile streamed twice through the LDS-DMA ring
struct Tile64Args {
    const double* x;
    int64_t wsize, wstep, first, nwin;
    int32_t channels;
    fmask_t mask;
    double th;          // zero-crossing threshold, compared with |x| in fp64
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
};
bool tile64_plan_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                    int64_t wstep, fmask_t mask, int32_t blk, const double* x);
int launch_tile64(const Tile64Args& a, hipStream_t stream);

inline int launch_fast(const FastArgs& a, int64_t wsize, hipStream_t stream) {
    // every field the kernel dereferences must have been filled in (FastArgs is zero-
    // initialised by the caller): refuse rather than launch with a wild stride
    if (!a.x || !a.out || a.wstep < 1 || a.nwin < 1 || a.first < 0 || a.out_ld < a.nwin ||
        a.feats.n < 1 || a.sample_stride != a.channels ||
        a.wstep * a.channels * 4 * 64 >= (int64_t(1) << 31))
        return MHF_EINVAL;
    const bool spec = (a.mask & kSpectralBits) != 0;
    if (wsize == 256) {
        if (a.channels == 1) return spec ? launch_tile_w256_c1_s1(a, stream) : launch_tile_w256_c1_s0(a, stream);
        return spec ? launch_tile_w256_c3_s1(a, stream) : launch_tile_w256_c3_s0(a, stream);
    }
    if (a.channels == 1) return spec ? launch_tile_w128_c1_s1(a, stream) : launch_tile_w128_c1_s0(a, stream);
    return spec ? launch_tile_w128_c3_s1(a, stream) : launch_tile_w128_c3_s0(a, stream);
}

}  // namespace mhf

#ifdef MHF_TILE_IMPL
#include "spectral_lane.hip.inc"

namespace mhf {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kChunk = dma::kChunk;   // samples per chunk: 128 B (C = 1) / 384 B (C = 3) per window,
                               // whole 128-B lines (16-sample chunks = half or 1.5 lines
                               // made every line two requests: C = 1 streamed at 4.75 TB/s)
#ifndef MHF_RING
#define MHF_RING 4
#endif
constexpr int kRing = MHF_RING;  // chunk slots per wave (4 x 9 KiB; diagnostic override -DMHF_RING)
constexpr int kDma = dma::kDma;   // DMA instructions (1 KiB = 64 lanes x 16 B) per chunk
// refill granularity: after every kGroup consumed chunks the kGroup freed slots are refilled
// back to back, so a window's consecutive chunks reach HBM together (DRAM row locality)
#ifndef MHF_DMA_GROUP
#define MHF_DMA_GROUP 1
#endif
constexpr int kGroup = MHF_DMA_GROUP;
static_assert(kRing % kGroup == 0, "DMA refill groups must tile the ring");

constexpr fmask_t kExtraBits = bit(MHF_RMS) | bit(MHF_PEAK_COUNT) | bit(MHF_DRANGE) |
                                bit(MHF_LINE_LENGTH);
// pass-1 extras level X of a kernel variant: 0 none, 1 RMS + peak count (the "full feature
// set" of BASELINE cfg4), 2 every extra (+ min/max for drange, line length)
constexpr fmask_t kExtra1Bits = bit(MHF_RMS) | bit(MHF_PEAK_COUNT);
inline int extra_level(fmask_t mask) {
    if (mask & (bit(MHF_DRANGE) | bit(MHF_LINE_LENGTH))) return 2;
    return (mask & kExtra1Bits) ? 1 : 0;
}
constexpr fmask_t kParBits = bit(MHF_VAR) | bit(MHF_STD);
#ifndef MHF_KEEP_D
#define MHF_KEEP_D 1
#endif
constexpr bool kKeepD = MHF_KEEP_D;   // pass 2 leaves D = x - m in R for the FFT
// -DMHF_PHASE_MARKS (analysis builds only, tools/phase_mix.py): a comment line in the
// listing at each phase boundary of the tile loop, to count the ISA per phase
#ifdef MHF_PHASE_MARKS
#define MHF_PHASE(name) asm volatile(";@mhf-phase " name)
#else
#define MHF_PHASE(name) ((void)0)
#endif

// Rows >= 1 of np.var / np.std (numba's var_parallel_impl: ssdp = Σseq64 (f64(x) - m)^2,
// SURVEY App. A). The exact replay costs 4 VALU per sample (cvt, sub, mul, add in fp64);
// by default the tile kernels take var_par = ssd / W instead, where ssd = Σseq64 f64(q),
// q = f32(d^2), d = f32(x - m) is the array_var sum pass 2 computes anyway. Each term's
// relative error is at most (1 + u)^3 - 1 (u = 2^-24: rounding of d and of q), all terms
// are non-negative and both fp64 sums are within 255 * 2^-53 of exact, so
// ssd stays within 1.79e-7 of ssd' = Σ (x - m32)^2 — provided no d or q left
// the fp32 normal range in a way that matters: a lane whose ssd is below 2^-110,
// non-finite, or whose fp32 sum c32 is a non-zero value below 2^-100 recomputes ssdp
// exactly from global memory (tile_exact_ssdp). ssd == 0 with |m| >= 2^-40 means every
// x == m (a non-zero x - m is then >= 2^-64, its square a non-zero fp32): ssdp == 0 exactly.
// Centering: ssd is about m32, the reference's chain about m64 = f64(c32) / W. With
// δ = m64 - m32 (exact in fp64) and μ the exact mean, Σ (x - m64)^2 = ssd' - 2 δ Σ (x - m32)
// + W δ^2 and |Σ (x - m32)| = W |μ - m32| <= W (E + |δ|), where E = |Σ x - c32| / W <=
// W u Σ|x| / W (the sequential fp32 sum's bound, u = 2^-24) <= W u (|m32| + sqrt(2 ssd / W))
// (Σ|x| <= W |m32| + sqrt(W ssd'), ssd' <= 2 ssd). The lane keeps ssd only if that
// centering term W |δ| (2 E + 3 |δ|) is <= 1.8e-7 ssd: |ssd - ssdp| <= 3.6e-7 ssdp. It
// holds for moderate offsets (|m| / σ up to ~300 at W = 256: accelerometers, the bench's
// signals); larger offsets take the exact replay.
__device__ __forceinline__ bool fast_var_ok(double ssd, float c32, float m32, double m64, int W) {
    if (ssd >= 0x1p-110 && ssd <= 1.7976931348623157e308) {
        if (c32 != 0.0f && fabsf(c32) < 0x1p-100f) return false;
        const double dl = fabs(m64 - static_cast<double>(m32));
        const double E = W * 0x1p-24 * (fabs(static_cast<double>(m32)) + sqrt(2.0 * ssd / W));
        return W * dl * (2.0 * E + 3.0 * dl) <= 1.8e-7 * ssd;
    }
    return ssd == 0.0 && fabsf(m32) >= 0x1p-40f;
}
// the exact fp64 chain of var_parallel_impl over window g's samples, from global memory
template <int W, int C>
__device__ __forceinline__ double tile_exact_ssdp(const float* x, int64_t g, int64_t S, int c, double m64) {
    const float* p = x + g * S * C + c;
    double s = 0.0;
#pragma unroll 16
    for (int t = 0; t < W; ++t) {
        const double dd = static_cast<double>(p[t * C]) - m64;
        s = s + dd * dd;
    }
    return s;
}

// Chunk image in LDS, window-major (dma_map.h dma::Geom): the kPieces 16-B pieces of
// tile-window r at slots r*kWinSlots .. + kPieces - 1, one pad slot after each window (bank
// spread), 64*kDma slots in all; slot j is filled by lane j % 64 of DMA instruction j / 64.
template <int C>
using TileGeom = dma::Geom<C>;

// Timing diagnostics only (results are garbage): -DMHF_DIAG_NO_VMWAIT drops the ring's
// DMA waits, -DMHF_DIAG_NO_LDSWAIT the LDS read waits, to price each kind of wait.
#ifndef MHF_LDS_WAIT
#ifdef MHF_DIAG_NO_LDSWAIT
#define MHF_LDS_WAIT "s_nop 0"
#else
#define MHF_LDS_WAIT "s_waitcnt lgkmcnt(0)"
#endif
#endif
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
#ifndef MHF_DIAG_NO_VMWAIT
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#endif
}

// Read the 32 samples of this lane's (window, channel) from ring slot `addr` into
// v[0..15] (pairs (s, s+1)) and wait for them, in one asm statement so the compiler
// neither inserts a vmcnt(0) nor touches the registers early.
template <int C>
__device__ __forceinline__ void lds_read_chunk(uint32_t addr, f2 (&v)[16]);

template <>
__device__ __forceinline__ void lds_read_chunk<1>(uint32_t addr, f2 (&v)[16]) {
    // window r at dword 36r: 16 lanes of a ds_read_b128 group hit 16 distinct 4-bank
    // groups (36r mod 64), conflict-free
    float4 o[8];
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:16\n\t"
        "ds_read_b128 %2, %8 offset:32\n\t"
        "ds_read_b128 %3, %8 offset:48\n\t"
        "ds_read_b128 %4, %8 offset:64\n\t"
        "ds_read_b128 %5, %8 offset:80\n\t"
        "ds_read_b128 %6, %8 offset:96\n\t"
        "ds_read_b128 %7, %8 offset:112\n\t"
        MHF_LDS_WAIT
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]),
          "=&v"(o[6]), "=&v"(o[7])
        : "v"(addr)
        : "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[2 * i] = f2{o[i].x, o[i].y};
        v[2 * i + 1] = f2{o[i].z, o[i].w};
    }
}

template <>
__device__ __forceinline__ void lds_read_chunk<3>(uint32_t addr, f2 (&v)[16]) {
    // sample s of this lane's channel at dword 3s (lane base holds 100r + c)
    asm volatile(
        "ds_read2_b32 %0, %16 offset1:3\n\t"
        "ds_read2_b32 %1, %16 offset0:6 offset1:9\n\t"
        "ds_read2_b32 %2, %16 offset0:12 offset1:15\n\t"
        "ds_read2_b32 %3, %16 offset0:18 offset1:21\n\t"
        "ds_read2_b32 %4, %16 offset0:24 offset1:27\n\t"
        "ds_read2_b32 %5, %16 offset0:30 offset1:33\n\t"
        "ds_read2_b32 %6, %16 offset0:36 offset1:39\n\t"
        "ds_read2_b32 %7, %16 offset0:42 offset1:45\n\t"
        "ds_read2_b32 %8, %16 offset0:48 offset1:51\n\t"
        "ds_read2_b32 %9, %16 offset0:54 offset1:57\n\t"
        "ds_read2_b32 %10, %16 offset0:60 offset1:63\n\t"
        "ds_read2_b32 %11, %16 offset0:66 offset1:69\n\t"
        "ds_read2_b32 %12, %16 offset0:72 offset1:75\n\t"
        "ds_read2_b32 %13, %16 offset0:78 offset1:81\n\t"
        "ds_read2_b32 %14, %16 offset0:84 offset1:87\n\t"
        "ds_read2_b32 %15, %16 offset0:90 offset1:93\n\t"
        MHF_LDS_WAIT
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
          "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]),
          "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15])
        : "v"(addr)
        : "memory");
}

// Per-lane DMA source offsets. DMA instruction i of a chunk fetches, for every lane, the
// 16-B piece the chunk image puts in slot 64i + lane. The 9 instructions of a chunk run
// in two groups with one M0 each (the instruction offset, added to both the LDS and the
// global address, is 13-bit signed): i = 0..4 at M0 = slot + 2 KiB, offsets -2..+2 KiB;
// i = 5..8 at M0 = slot + 6 KiB, offsets -1..+2 KiB. The lane offset carries the opposite
// of the instruction offset, the SGPR base a -kBias so it stays non-negative.
// Windows past the last one (tail tile) are clamped to it.
constexpr uint32_t kBias = dma::kBias;
__host__ __device__ constexpr int dma_inst_off(int i) { return dma::inst_off(i); }

template <int C>
struct TileSrc {
    uint32_t off[kDma];
};

template <int C>
__device__ __forceinline__ TileSrc<C> tile_src(int64_t rmax, int64_t S, int lane) {
    using G = TileGeom<C>;
    TileSrc<C> ts;
#pragma unroll
    for (int i = 0; i < kDma; ++i) {
        int r, k;
        G::piece(i * 64 + lane, r, k);
        const int64_t rr = r < rmax ? r : rmax;
        ts.off[i] = dma::fix_lane_off(rr, S, C, k, i);
    }
    return ts;
}

// SGPR base (byte address) of chunk 0 of the tile starting at window g0, minus kBias
__device__ __forceinline__ uint64_t tile_base(const float* x, int64_t g0, int64_t S, int C) {
    return dma::fix_tile_base(reinterpret_cast<uint64_t>(x), g0, S, C);
}

// Cache policy of the input stream: nt (streaming) — every input byte is read exactly once.
// Measured against the default policy (tools/ab_bench.sh): cfg2 0.666 -> 0.619 ms, cfg3
// 2.83 -> 2.80, cfg4 17.6 -> 15.65; pass-1-only floors cfg2 0.552 -> 0.511, cfg3 1.79 ->
// 1.53-1.67. Diagnostic override: -DMHF_DMA_POLICY='""'.
#ifndef MHF_DMA_POLICY
#define MHF_DMA_POLICY " nt"
#endif

// One chunk = 9 LDS-DMA instructions into ring slot `slot` (LDS byte address). Inline asm:
// M0 set by the compiler ("{m0}" operand), saddr form (SGPR base + 32-bit lane offset).
// The hazards around the statement are ours to pad (the compiler does not look inside
// asm): SALU writes M0 -> LDS-DMA (1 wait state) and — tile_idx's base comes from
// v_readfirstlane — VALU writes SGPR -> VMEM reads it as its base (5 wait states): s_nop 4.
// (With s_nop 0 the tile_idx kernel read a stale base whenever LLVM placed the
// readfirstlane right before the statement: round 6's tile_fix fault)
__device__ __forceinline__ void dma_chunk(uint64_t base, uint32_t slot, const uint32_t (&o)[kDma]) {
#ifdef MHF_DIAG_NO_DMA
    // timing diagnostic only (results garbage): no HBM traffic at all — the kernel's pure
    // instruction time at one wave per SIMD (the compute floor of the bit-exact design)
    (void)base; (void)slot; (void)o;
    return;
#endif
    asm volatile(
        "s_nop 4\n\t"
        "global_load_lds_dwordx4 %1, %6 offset:-2048" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %2, %6 offset:-1024" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %3, %6" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %4, %6 offset:1024" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %5, %6 offset:2048" MHF_DMA_POLICY
        :
        : "{m0}"(slot + 2048u), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "s"(base)
        : "memory");
    asm volatile(
        "s_nop 4\n\t"
        "global_load_lds_dwordx4 %1, %5 offset:-1024" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %2, %5" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %3, %5 offset:1024" MHF_DMA_POLICY "\n\t"
        "global_load_lds_dwordx4 %4, %5 offset:2048" MHF_DMA_POLICY
        :
        : "{m0}"(slot + 6144u), "v"(o[5]), "v"(o[6]), "v"(o[7]), "v"(o[8]), "s"(base)
        : "memory");
}

template <int C, int J>
__device__ __forceinline__ void issue_chunk(uint64_t base, const TileSrc<C>& ts, uint32_t slot_addr) {
    dma_chunk(base + static_cast<uint64_t>(J * kChunk * C * 4), slot_addr, ts.off);
}

// pass-1 state of one (window, channel): fp32 sum and the one-pass features
struct P1State {
    float c32, a32, ll, mn, mx, p1, p2;
    int zc, pk;
    bool prevpos;
};

// pass-2 state: deviation sums, plus the software-pipelined products of the next pair
struct P2State {
    double ssd, ssdp, m64;
    float s3, s4, m32;
    f2 Xc, Dc, Qc, A3c, A4c;
};

template <int W, int C, int X, bool PAR, bool SPEC>
__global__ void __launch_bounds__(64, 1) tile_kernel(FastArgs a) {
    using G = TileGeom<C>;
    constexpr int U = G::U;
    constexpr int KD = kDma;
    constexpr int NCH = W / kChunk;
    __shared__ __attribute__((aligned(16))) float4 ring[kRing][KD * 64];

    const int lane = threadIdx.x;
    const int r = lane / C, c = lane - (lane / C) * C;
    const bool unit_ok = r < U;
    const int64_t S = a.wstep;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    const int64_t gmax = a.first + a.nwin - 1;
    const float invW = 1.0f / static_cast<float>(W);
    const f2 IW2 = {invW, invW};
    const int64_t F = a.feats.n;
    const bool need_p2 = (a.mask & kPass2Bits) != 0;
    // zero crossings cost 3 issue slots per sample (v_cmp, s_xor, v_addc): pass 1 has a
    // variant without them, chosen per chunk by this uniform flag
    const bool want_zc = (a.mask & bit(MHF_ZERO_CROSSINGS)) != 0;
    const bool want_par = (a.mask & kParBits) != 0;

    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    static_assert(NCH >= kRing, "window shorter than the DMA ring");
    static_assert(NCH % kRing == 0, "ring slots must be static per chunk");
    // LDS byte address of the ring and of this lane's reads inside a ring slot
    const uint32_t ring_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)&ring[0][0]));
    constexpr uint32_t kSlotBytes = KD * 1024;
    uint32_t lane_addr;
    if constexpr (C == 1) lane_addr = ring_addr + static_cast<uint32_t>((unit_ok ? r : 0) * G::kWinSlots * 16);
    else lane_addr = ring_addr + static_cast<uint32_t>(((unit_ok ? r : 0) * G::kWinSlots * 4 + c) * 4);

    // the window: samples [0, NV) in VGPR pairs, [NV, W) parked in AGPRs (VALU cannot
    // read AGPRs: one v_accvgpr_write / _read per parked sample)
    constexpr int NA = (W > 128) ? 64 : 0;
    constexpr int NV = W - NA;
    // W = 256 spectral kernels: split FFT (spectral_lane.hip.inc lane_spectrum_split);
    // -DMHF_NO_SPLIT_FFT: the whole-window lane_spectrum (A/B diagnostic)
#ifdef MHF_NO_SPLIT_FFT
    constexpr bool kSplitFFT = false;
#else
    constexpr bool kSplitFFT = SPEC && W == 256 && kKeepD;
#endif
    f2 R[NV / 2];
    float RA[NA > 0 ? NA : 1];

    // DMA streams: tile t1 is the one pass 1 consumes, t2 the one after it (prefetched
    // into ring slots freed by t1's last chunks)
    int64_t t1 = tile;
    // One set of per-lane DMA offsets is live at a time (9 VGPRs): pass 1 of t1 refills
    // with t1's own chunks for j < NCH - kRing, then switches `src` over to t2.
    uint64_t base1 = tile_base(a.x, a.first + t1 * U, S, C);
    TileSrc<C> src = tile_src<C>(gmax - (a.first + t1 * U), S, lane);
    int64_t t2 = t1 + gridDim.x;
    uint64_t base2 = 0;
    if (t2 < ntiles) base2 = tile_base(a.x, a.first + t2 * U, S, C);
    // prologue: chunks 0 .. kRing-1 of the first tile into slots 0 .. kRing-1
    static_for<0, kRing>([&](auto J) {
        issue_chunk<C, J.value>(base1, src, ring_addr + J.value * kSlotBytes);
    });

    // ---- pass 1 over chunk j of tile t1 (reference order): fp32 sum, zero crossings,
    // extras; the samples land in R / RA. Waits for the chunk, then refills its ring slot
    // with chunk j + kRing of t1 or chunk j + kRing - NCH of t2.
    auto pass1_chunk = [&](auto JJ, P1State& st, bool have2, auto ZCT) {
        constexpr int j = decltype(JJ)::value;
        constexpr bool ZC = decltype(ZCT)::value;
        // chunks issued after chunk j so far (groups of kGroup, see below): the last one
        // is chunk `last` of this tile's numbering (>= NCH: the next tile's)
        constexpr int last = ((j + kRing - kGroup) / kGroup) * kGroup + kGroup - 1;
        if (have2 || last < NCH) {
            wait_vmcnt<(last - j) * KD>();
        } else {
            wait_vmcnt<((last < NCH ? last : NCH - 1) - j) * KD>();
        }
        // inline-asm LDS reads: a compiler-visible ds_read after an LDS-DMA gets an
        // s_waitcnt vmcnt(0) in front of it, which would drain the whole ring
        f2 v2[kChunk / 2];
        lds_read_chunk<C>(lane_addr + (j % kRing) * kSlotBytes, v2);
        static_for<0, kChunk / 2>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr int t0 = j * kChunk + 2 * q;
            if constexpr (t0 < NV) {
                R[t0 / 2] = v2[q];
            } else {
                asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t0 - NV]) : "v"(v2[q].x));
                asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t0 + 1 - NV]) : "v"(v2[q].y));
            }
            static_for<0, 2>([&](auto H) {
                constexpr int t = t0 + decltype(H)::value;
                const float v = decltype(H)::value ? v2[q].y : v2[q].x;
                st.c32 = st.c32 + v;
                if constexpr (ZC) {
                    const bool pos = v > a.t32;
                    if constexpr (t > 0) st.zc += (pos != st.prevpos);
                    st.prevpos = pos;
                    // keep the integer count sequential: LLVM would otherwise reassociate
                    // the adds into a tree and keep every per-sample bool alive. (Only
                    // integer chains are pinned: the hazard recognizer pads a read of an
                    // asm output right after the asm with s_nop; fp chains never reorder.)
                    asm volatile("" : "+v"(st.zc));
                }
                if constexpr (X >= 1) {
                    st.a32 = st.a32 + v * v;
                    if constexpr (t > 1) st.pk += (st.p1 > st.p2 && st.p1 > v);
                    asm volatile("" : "+v"(st.pk));
                }
                if constexpr (X >= 2) {
                    if constexpr (t == 0) {
                        st.mn = v; st.mx = v;
                    } else {
                        st.mn = (v < st.mn) ? v : st.mn;
                        st.mx = (v > st.mx) ? v : st.mx;
                        st.ll = st.ll + fabsf(v - st.p1);
                    }
                }
                if constexpr (X >= 1) {
                    st.p2 = st.p1;
                    st.p1 = v;
                }
            });
        });
        // slot j % kRing is free again (its reads completed inside lds_read_chunk); the
        // refills go out kGroup at a time, after the last chunk of each group of slots
        if constexpr ((j + 1) % kGroup == 0) {
            static_for<0, kGroup>([&](auto I) {
                constexpr int jj = j + 1 - kGroup + decltype(I)::value;   // slot of chunk jj
                constexpr int jn = jj + kRing;
                if constexpr (jn < NCH) {
                    issue_chunk<C, jn>(base1, src, ring_addr + (jj % kRing) * kSlotBytes);
                } else {
                    if constexpr (jn == NCH) {   // t1's DMAs are all issued: offsets of t2 from here
                        if (have2) src = tile_src<C>(gmax - (a.first + t2 * U), S, lane);
                    }
                    if (have2) issue_chunk<C, jn - NCH>(base2, src, ring_addr + (jj % kRing) * kSlotBytes);
                }
            });
        }
    };

    auto load_pair = [&](auto T) -> f2 {
        constexpr int t = decltype(T)::value;
        if constexpr (t < NV) {
            return R[t / 2];
        } else {
            float xa, xb;
            asm("v_accvgpr_read_b32 %0, %1" : "=v"(xa) : "a"(RA[t - NV]));
            asm("v_accvgpr_read_b32 %0, %1" : "=v"(xb) : "a"(RA[t + 1 - NV]));
            return f2{xa, xb};
        }
    };
    // ---- pass 2 over samples [T0, T1) from registers: deviations from the fp32 mean
    // (array_var, skewness, kurtosis) and, for rows >= 1 of a direct np.var/np.std, from
    // the fp64 mean. Two samples per step: the independent products are packed
    // (v_pk_*_f32), the accumulations stay sequential scalar chains in the reference's
    // order; software-pipelined by one pair (the products of pair t+2 are issued before
    // the accumulations of pair t: no accumulation reads a v_pk result the instruction
    // before, which gfx950 would pad with s_nop).
    auto pass2_begin = [&](P2State& p, float c32) {
        p.m32 = static_cast<float>(static_cast<double>(c32) / static_cast<double>(W));
        p.m64 = static_cast<double>(c32) / static_cast<double>(W);
        p.ssd = 0.0; p.ssdp = 0.0; p.s3 = 0.0f; p.s4 = 0.0f;
        const f2 M2 = {p.m32, p.m32};
        p.Xc = load_pair(IntC<0>{});
        const f2 D = p.Xc - M2;
        p.Dc = D;
        p.Qc = D * D;
        p.A3c = (D * p.Qc) * IW2;
        p.A4c = (p.Qc * p.Qc) * IW2;
    };
    auto no_hook = [](auto, f2) {};
    // hook(IntC<t>, D): called for pair t after its accumulations, with D = x - m of the pair
    auto pass2_range = [&](P2State& p, auto T0, auto T1, auto&& hook) {
        const f2 M2 = {p.m32, p.m32};
        static_for<0, (decltype(T1)::value - decltype(T0)::value) / 2>([&](auto K) {
            constexpr int t = decltype(T0)::value + 2 * decltype(K)::value;
            f2 Xn = p.Xc, Dn = p.Dc, Qn = p.Qc, A3n = p.A3c, A4n = p.A4c;
            if constexpr (t + 2 < W) {
                Xn = load_pair(IntC<t + 2>{});
                Dn = Xn - M2;
                Qn = Dn * Dn;
                A3n = (Dn * Qn) * IW2;
                A4n = (Qn * Qn) * IW2;
            }
            // spectral kernels keep D = x - m (the FFT input) in place of x
            if constexpr (kKeepD && SPEC && t < NV) R[t / 2] = p.Dc;
            p.ssd = p.ssd + static_cast<double>(p.Qc.x);
            p.s3 = p.s3 + p.A3c.x;
            p.s4 = p.s4 + p.A4c.x;
            if constexpr (PAR) {
                const double dd = static_cast<double>(p.Xc.x) - p.m64;
                p.ssdp = p.ssdp + dd * dd;
            }
            p.ssd = p.ssd + static_cast<double>(p.Qc.y);
            p.s3 = p.s3 + p.A3c.y;
            p.s4 = p.s4 + p.A4c.y;
            if constexpr (PAR) {
                const double dd = static_cast<double>(p.Xc.y) - p.m64;
                p.ssdp = p.ssdp + dd * dd;
            }
            // advance all accumulation chains in lockstep: LLVM otherwise runs each chain
            // over the whole window in turn and keeps every D and Q alive in between
            asm volatile("" : "+v"(p.ssd), "+v"(p.s3), "+v"(p.s4), "+v"(p.ssdp));
            hook(IntC<t>{}, p.Dc);
            p.Xc = Xn; p.Dc = Dn; p.Qc = Qn; p.A3c = A3n; p.A4c = A4n;
        });
    };

    auto finish = [&](int64_t tl, const P1State& s1, const P2State& p, double spec_bp,
                      double spec_rbp, double spec_ent, double spec_dom) {
        const int64_t g = a.first + tl * U + r;
        const float var32 = static_cast<float>(p.ssd / static_cast<double>(W));
        const float std32 = static_cast<float>(sqrt(static_cast<double>(var32)));
        double varp;
        if constexpr (PAR) {
            varp = p.ssdp / static_cast<double>(W);
        } else {
            double ssdp = p.ssd;
            if (want_par && unit_ok && g > 0 && g <= gmax && !fast_var_ok(p.ssd, s1.c32, p.m32, p.m64, W))
                ssdp = tile_exact_ssdp<W, C>(a.x, g, S, c, p.m64);
            varp = ssdp / static_cast<double>(W);
        }
        const float kurt = (var32 == 0.0f) ? 0.0f : p.s4 / (var32 * var32);
        WinVals v;
        v.mean32 = p.m32;
        v.mean = (g == 0) ? static_cast<double>(p.m32) : p.m64;
        v.var32 = var32;
        v.std32 = std32;
        v.var = (g == 0) ? static_cast<double>(var32) : varp;
        v.std_ = (g == 0) ? static_cast<double>(std32) : sqrt(varp);
        v.skew = (std32 == 0.0f) ? 0.0 : static_cast<double>(p.s3 / (std32 * (std32 * std32)));
        v.kurt = kurt;
        v.kurt_ex = static_cast<double>(kurt) - 3.0;
        v.rms = sqrtf(static_cast<float>(static_cast<double>(s1.a32) / static_cast<double>(W)));
        v.zc = s1.zc;
        v.peaks = s1.pk;
        v.drange = static_cast<double>(s1.mx - s1.mn);
        v.ll = s1.ll;
        v.bp = spec_bp;
        v.rbp = spec_rbp;
        v.ent = spec_ent;
        v.dom = spec_dom;
#ifdef MHF_DIAG_NO_STORE
        // timing diagnostic only (results garbage): price the output stores
        if (g < 0) {
#else
        if (unit_ok && g <= gmax) {
#endif
            const int64_t i = g - a.first;
            for (int jf = 0; jf < F; ++jf) {
                // int32 ids: a scalar kernarg load (an int8 id became a per-lane global
                // load + vmcnt(0), which drained the DMA ring at every store)
                const int f = a.feats.id[jf];
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * F + jf) * a.out_ld + i,
                          pick_moment(v, f));
            }
        }
    };

    // ---- main loop. Iteration k: pass 2 (+ spectral, + results) of the tile pass 1
    // filled into registers in iteration k-1 ("prev"), and pass 1 of the next tile
    // ("cur"); one extra iteration drains the last tile. One copy of each pass in code.
    P1State s1 = {};
    bool have_prev = false;
    int64_t prev = -1, cur = t1;
    for (;;) {
        const bool have_cur = cur < ntiles;
        if (!have_prev && !have_cur) break;
        const bool have2 = t2 < ntiles;
        P2State p;
        P1State s1n = {};
        if (have_prev) pass2_begin(p, s1.c32);
        if constexpr (SPEC) {
            // spectral: the FFT needs the whole window after pass 2, so the next tile's
            // pass 1 runs after it (its first kRing chunks are already in flight)
            if (have_prev) {
                // the weight tables, addressed inside the kernarg segment (FastArgs is the
                // kernel's only argument, at offset 0)
                const char* ks = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
                const float* bw = reinterpret_cast<const float*>(ks + offsetof(FastArgs, spec) + offsetof(SpecTables, bw));
                const float* dw = reinterpret_cast<const float*>(ks + offsetof(FastArgs, spec) + offsetof(SpecTables, dw));
                const bool want_ent = (a.mask & bit(MHF_SPECTRAL_ENTROPY)) != 0;
                const bool want_dom = (a.mask & bit(MHF_DOMINANT_FREQ)) != 0;
                SpecOut so;
                if constexpr (kSplitFFT) {
                    // W = 256: the split FFT, sub-FFT 3 parked in the AGPRs of the window's last
                    // quarter (lane_spectrum_split)
                    SpecK k = spec_consts<W>(bw, dw);
                    split_begin<W>(k);
                    constexpr int Z4 = W / 8;          // z index of the second quarter
                    auto stage1 = [&R, &RA, &k](auto J, f2 D) {
                        constexpr int j = decltype(J)::value;
                        split_stage1<W, j>(R[j], R[j + Z4], R[j + 2 * Z4], D, k);
                        asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[2 * j]) : "v"(D.x));
                        asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[2 * j + 1]) : "v"(D.y));
                    };
                    // D = x - m into R and, for the last quarter, back into its AGPRs by pass 2
                    // (kKeepD), which runs here even when no moment feature is requested: a
                    // second branch computing D alone (or running stage 1 itself) made LLVM
                    // keep both branches' inputs alive — 100+ scratch spills. Stage 1 after pass
                    // 2: fused into its last quarter, R + the pass-2 state + the butterflies
                    // exceeded the VGPRs.
                    auto park_d = [&RA](auto T, f2 D) {
                        constexpr int t = decltype(T)::value;
                        if constexpr (t >= NV) {
                            asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t - NV]) : "v"(D.x));
                            asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t + 1 - NV]) : "v"(D.y));
                        }
                    };
                    MHF_PHASE("pass2");
                    pass2_range(p, IntC<0>{}, IntC<NV>{}, no_hook);
                    MHF_PHASE("pass2-last-quarter+fft-stage1");
                    pass2_range(p, IntC<NV>{}, IntC<W>{}, [&](auto T, f2 D) {
                        stage1(IntC<(decltype(T)::value - NV) / 2>{}, D);
                    });
                    MHF_PHASE("fft+features");
                    so = lane_spectrum_split<W>(R, RA, static_cast<float>(W) * p.m32, a.scale,
                                                want_ent, want_dom, a.dom_lo, a.dom_hi, k);
                } else {
                if (need_p2) pass2_range(p, IntC<0>{}, IntC<W>{}, no_hook);
                f2 z[W / 2];
                const f2 M2 = {p.m32, p.m32};
                // mean removed: pass 2 already left D = x - m in the VGPR part of the window
                if (kKeepD && need_p2) {
                    static_for<0, W / 2>([&](auto K) {
                        constexpr int k = decltype(K)::value;
                        if constexpr (2 * k < NV) z[k] = R[k];
                        else z[k] = load_pair(IntC<2 * k>{}) - M2;
                    });
                } else {
                    static_for<0, W / 2>([&](auto K) {
                        z[decltype(K)::value] = load_pair(IntC<2 * decltype(K)::value>{}) - M2;
                    });
                }
                so = lane_spectrum<W>(z, static_cast<float>(W) * p.m32, a.scale, bw, dw,
                                      want_ent, want_dom, a.dom_lo, a.dom_hi);
                }
                // keep the moment results (WinVals: 18 doubles) from being computed before
                // the FFT and held across it: their inputs pass through this asm after it
                asm volatile("" : "+v"(p.ssd), "+v"(p.ssdp), "+v"(p.s3), "+v"(p.s4), "+v"(p.m32),
                             "+v"(p.m64), "+v"(s1.a32), "+v"(s1.ll), "+v"(s1.mn), "+v"(s1.mx),
                             "+v"(s1.zc), "+v"(s1.pk));
                MHF_PHASE("finish+stores");
                finish(prev, s1, p, so.bp, so.bp / so.tot, so.ent,
                       (so.bk < 0) ? static_cast<double>(NAN) : static_cast<double>(so.bk) * a.freq_step);
            }
            if (have_cur) {
                // the split FFT needs every VGPR it can get: the 9 DMA offsets of this tile are
                // formed again here instead of being carried across pass 2 and the FFT
                if constexpr (kSplitFFT) src = tile_src<C>(gmax - (a.first + cur * U), S, lane);
                MHF_PHASE("pass1");
                static_for<0, NCH>([&](auto JJ) {
                    if (want_zc) pass1_chunk(JJ, s1n, have2, IntC<1>{});
                    else pass1_chunk(JJ, s1n, have2, IntC<0>{});
                });
            } else {
                // the loop ends after this iteration: give R / RA defined values on this
                // path, or the phi at the loop head keeps the old window alive across the
                // FFT (a 256-register live range -> scratch spills)
                static_for<0, NV / 2>([&](auto K) { R[K.value] = f2{0.0f, 0.0f}; });
                if constexpr (NA > 0) static_for<0, NA>([&](auto K) { RA[K.value] = 0.0f; });
            }
        } else {
            // moments: pass 2 of prev interleaved chunk by chunk with pass 1 of cur —
            // pass 1 refills exactly the registers pass 2 has just released, and the DMA
            // ring keeps streaming while pass 2 runs
            static_for<0, NCH>([&](auto JJ) {
                constexpr int j = decltype(JJ)::value;
                if (have_prev && need_p2) pass2_range(p, IntC<j * kChunk>{}, IntC<(j + 1) * kChunk>{}, no_hook);
                if (have_cur) {
                    if (want_zc) pass1_chunk(JJ, s1n, have2, IntC<1>{});
                    else pass1_chunk(JJ, s1n, have2, IntC<0>{});
                }
            });
            if (have_prev) finish(prev, s1, p, 0.0, 0.0, 0.0, 0.0);
        }
        // advance: cur becomes prev; the DMA streams move on by one tile
        MHF_PHASE("advance");
        have_prev = have_cur;
        prev = cur;
        s1 = s1n;
        cur = t2;
        base1 = base2;
        t2 = cur + gridDim.x;
        if (t2 < ntiles) base2 = tile_base(a.x, a.first + t2 * U, S, C);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int W, int C, bool SPEC>
int launch_tile(const FastArgs& a, hipStream_t stream) {
    const int64_t U = TileGeom<C>::U;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    int64_t blocks = ntiles < 1024 ? ntiles : 1024;   // 256 CUs x 4 waves, persistent
    const int x = extra_level(a.mask);
    // PAR: the exact fp64 replay of var_parallel_impl, only on request (MHF_NUMERICS_EXACT_VAR);
    // otherwise rows >= 1 of np.var / np.std come from ssd (fast_var_ok above)
    const bool par = (a.mask & kParBits) != 0 && a.exact_var;
    dim3 grid(static_cast<unsigned>(blocks)), block(64);
#define MHF_TL(X, P) hipLaunchKernelGGL((tile_kernel<W, C, X, P, SPEC>), grid, block, 0, stream, a)
    if (x == 2) { if (par) MHF_TL(2, true); else MHF_TL(2, false); }
    else if (x == 1) { if (par) MHF_TL(1, true); else MHF_TL(1, false); }
    else { if (par) MHF_TL(0, true); else MHF_TL(0, false); }
#undef MHF_TL
    return MHF_OK;
}

}  // namespace mhf

// one translation unit per (W, C, spectral) so the unrolled variants build in parallel
#define MHF_DEFINE_TILE_LAUNCH(W, C, S)                                                  \
    int mhf::launch_tile_w##W##_c##C##_s##S(const FastArgs& a, hipStream_t stream) {    \
        return launch_tile<W, C, S != 0>(a, stream);                                     \
    }
#endif  // MHF_TILE_IMPL
