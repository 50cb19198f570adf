// kernels_fast.hip.inc — the fused tile kernel: register-resident windows fed by LDS-DMA.
//
// Why this shape: numba's per-window reductions are sequential
// fp32/fp64 accumulations, so one LANE must own one window and walk
// its samples in order; two passes (mean, then deviations) need the whole window on
// chip. A lane keeps its window in W VGPRs (W = 128 / 256), so a wave holds 64
// (window, channel) units and runs at one wave per SIMD (4 waves per CU, ~300 VGPRs).
// HBM is streamed by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) into a per-wave
// ring of 16-sample chunks, kept RING-1 chunks ahead — across tile boundaries too, so the
// second pass and the stores of one tile overlap the loads of the next.
//
// Data layout: x is AoS float32, sample t of channel c of the signal at x[t*C + c]
// (C = 1: a contiguous 1-D signal). Window w covers samples [w*S, w*S + W).
// Lane l owns unit (window r = l / C of the tile, channel c = l % C); a tile is
// U = 64 / C windows. LDS image of one chunk (16 samples of U windows, all channels):
// 16-byte piece k (k < 4C) of tile-window r sits at slot k*U + r, so the owning lanes
// read consecutive slots (conflict-free ds_read_b128); lanes of one window broadcast.
#pragma once

#include "engine_common.h"

namespace mhf {

struct FastArgs {
    const float* x;
    int64_t ch_stride, sample_stride, wstep, first, nwin;
    int32_t channels;
    uint32_t mask;
    float t32;
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    int32_t band_lo, band_hi, dom_lo, dom_hi;
    float scale;
    double freq_step;
};

inline bool fast_plan_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                         int64_t wstep, uint32_t mask) {
    (void)mask;
    if (!(wsize == 128 || wsize == 256)) return false;
    if (!(channels == 1 || channels == 3)) return false;
    if (sample_stride != channels) return false;
    if (channels > 1 && ch_stride != 1) return false;
    if (wstep < wsize) return false;                   // disjoint windows only
    if ((wstep * channels) % 4 != 0) return false;    // 16-B aligned window starts
    return true;
}

inline const char* fast_plan_name(int64_t wsize, int32_t channels) {
    if (wsize == 256) return channels == 1 ? "tile_w256_c1" : "tile_w256_c3";
    return channels == 1 ? "tile_w128_c1" : "tile_w128_c3";
}

// one translation unit per (W, C): tile_w<W>_c<C>.hip (parallel builds)
int launch_tile_w256_c1(const FastArgs& a, hipStream_t stream);
int launch_tile_w256_c3(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c1(const FastArgs& a, hipStream_t stream);
int launch_tile_w128_c3(const FastArgs& a, hipStream_t stream);

inline int launch_fast(const FastArgs& a, int64_t wsize, hipStream_t stream) {
    // every field the kernel dereferences must have been filled in (FastArgs is zero-
    // initialised by the caller): refuse rather than launch with a wild stride
    if (!a.x || !a.out || a.wstep < wsize || a.nwin < 1 || a.first < 0 || a.out_ld < a.nwin ||
        a.feats.n < 1 || a.sample_stride != a.channels)
        return MHF_EINVAL;
    if (wsize == 256)
        return a.channels == 1 ? launch_tile_w256_c1(a, stream) : launch_tile_w256_c3(a, stream);
    return a.channels == 1 ? launch_tile_w128_c1(a, stream) : launch_tile_w128_c3(a, stream);
}

}  // namespace mhf

#ifdef MHF_TILE_IMPL
#include "spectral_lane.hip.inc"

namespace mhf {


typedef __attribute__((address_space(3))) void lds_void_t;



constexpr int kChunk = 16;     // samples per chunk
constexpr int kRing = 8;       // chunk slots per wave
constexpr int kDmaPerChunk = 4; // 64 lanes x 16 B x 4 = 4 KiB >= U * 4C * 16 B

constexpr uint32_t kExtraBits = bit(MHF_RMS) | bit(MHF_PEAK_COUNT) | bit(MHF_DRANGE) |
                                bit(MHF_LINE_LENGTH);
constexpr uint32_t kParBits = bit(MHF_VAR) | bit(MHF_STD);

template <int C>
struct TileGeom {
    static constexpr int U = 64 / C;              // windows per tile
    static constexpr int kPieces = 4 * C;         // 16-B pieces per window per chunk
    static constexpr int kUsed = U * kPieces;     // <= 256 slots used per chunk
};

// s_waitcnt vmcnt(n) for n known after unrolling (the switch folds to one instruction)
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
#define MHF_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MHF_VM(0) MHF_VM(4) MHF_VM(8) MHF_VM(12) MHF_VM(16) MHF_VM(20) MHF_VM(24) MHF_VM(28)
    MHF_VM(32) MHF_VM(36) MHF_VM(40) MHF_VM(44) MHF_VM(48) MHF_VM(52) MHF_VM(56) MHF_VM(60)
#undef MHF_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// Read the 4C pieces of one chunk that this lane's window needs (piece k at byte
// k*U*16 of the slot, lane part folded into `addr`) and wait for them, in one asm
// statement so the compiler neither inserts a vmcnt(0) nor touches the registers early.
template <int C, int U>
__device__ __forceinline__ void lds_read_chunk(uint32_t addr, float4 (&o)[4 * C]);

template <>
__device__ __forceinline__ void lds_read_chunk<1, 64>(uint32_t addr, float4 (&o)[4]) {
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %4 offset:1024\n\t"
        "ds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3])
        : "v"(addr)
        : "memory");
}

template <>
__device__ __forceinline__ void lds_read_chunk<3, 21>(uint32_t addr, float4 (&o)[12]) {
    asm volatile(
        "ds_read_b128 %0, %12\n\t"
        "ds_read_b128 %1, %12 offset:336\n\t"
        "ds_read_b128 %2, %12 offset:672\n\t"
        "ds_read_b128 %3, %12 offset:1008\n\t"
        "ds_read_b128 %4, %12 offset:1344\n\t"
        "ds_read_b128 %5, %12 offset:1680\n\t"
        "ds_read_b128 %6, %12 offset:2016\n\t"
        "ds_read_b128 %7, %12 offset:2352\n\t"
        "ds_read_b128 %8, %12 offset:2688\n\t"
        "ds_read_b128 %9, %12 offset:3024\n\t"
        "ds_read_b128 %10, %12 offset:3360\n\t"
        "ds_read_b128 %11, %12 offset:3696\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]),
          "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11])
        : "v"(addr)
        : "memory");
}

// Per-lane source of each of the 4 DMA instructions of chunk 0 of a tile; chunk j adds
// j*kChunk*C floats to it. (Not via the instruction's immediate offset: on an LDS-DMA
// that offset is added to the LDS destination as well.)
template <int C>
struct TileSrc {
    const float* p[kDmaPerChunk];
};

template <int C>
__device__ __forceinline__ TileSrc<C> tile_src(const float* __restrict__ x, int64_t g0,
                                               int64_t gmax, int64_t S, int lane) {
    using G = TileGeom<C>;
    TileSrc<C> ts;
#pragma unroll
    for (int i = 0; i < kDmaPerChunk; ++i) {
        int q = i * 64 + lane;
        if (q >= G::kUsed) q = G::kUsed - 1;      // spare lanes re-load a valid piece
        const int k = q / G::U, r = q - k * G::U;
        int64_t w = g0 + r;
        if (w > gmax) w = gmax;                    // tail tile: clamp to a real window
        ts.p[i] = x + w * S * C + 4 * k;
    }
    return ts;
}

template <int C, int J>
__device__ __forceinline__ void issue_chunk(const TileSrc<C>& ts, float4* slot) {
#pragma unroll
    for (int i = 0; i < kDmaPerChunk; ++i)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(ts.p[i] + J * kChunk * C),
                                         (lds_void_t*)(slot + i * 64), 16, 0, 0);
}

template <int W, int C, bool EXTRA, bool PAR, bool SPEC>
__global__ void __launch_bounds__(64, 1) tile_kernel(FastArgs a) {
    using G = TileGeom<C>;
    constexpr int U = G::U;
    constexpr int NCH = W / kChunk;
    __shared__ __attribute__((aligned(16))) float4 ring[kRing][kDmaPerChunk * 64];

    const int lane = threadIdx.x;
    const int r = lane / C, c = lane - (lane / C) * C;
    const bool unit_ok = r < U;
    const int64_t S = a.wstep;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    const int64_t gmax = a.first + a.nwin - 1;
    const float invW = 1.0f / static_cast<float>(W);
    const int64_t F = a.feats.n;
    // per-lane channel selects (C-way), computed once
    bool is_c[C > 1 ? C : 1];
#pragma unroll
    for (int cc = 0; cc < (C > 1 ? C : 1); ++cc) is_c[cc] = (c == cc);

    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    // prologue: chunks 0 .. kRing-1 of the first tile into slots 0 .. kRing-1
    static_assert(NCH >= kRing, "window shorter than the DMA ring");
    TileSrc<C> src_next = tile_src<C>(a.x, a.first + tile * U, gmax, S, lane);
    static_for<0, kRing>([&](auto J) { issue_chunk<C, J.value>(src_next, ring[J.value]); });

    static_assert(NCH % kRing == 0, "ring slots must be static per chunk");
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t g0 = a.first + tile * U;
        const int64_t next_tile = tile + gridDim.x;
        const bool have_next = next_tile < ntiles;
        const TileSrc<C> src_cur = src_next;
        if (have_next) src_next = tile_src<C>(a.x, a.first + next_tile * U, gmax, S, lane);

        // the window: samples [0, W-NA) in VGPRs, [W-NA, W) parked in AGPRs (VALU
        // cannot read AGPRs: one v_accvgpr_write / _read per parked sample)
        constexpr int NA = (W > 128) ? 64 : 0;
        constexpr int NV = W - NA;
        float R[NV];
        float RA[NA > 0 ? NA : 1];
        float c32 = 0.0f, a32 = 0.0f, ll = 0.0f, mn = 0.0f, mx = 0.0f;
        float p1 = 0.0f, p2 = 0.0f;
        bool prevpos = false;
        int zc = 0, pk = 0;

        const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)&ring[0][0])) +
                                  static_cast<uint32_t>((unit_ok ? r : 0) * 16);
        static_for<0, NCH>([&](auto JJ) {
            constexpr int j = JJ.value;
            // wait for chunk j: everything but the DMAs of the kRing-1 chunks issued after
            // it (fewer once the wave's last tile drains the ring)
            if (have_next || j + kRing - 1 < NCH) {
                wait_vmcnt((kRing - 1) * kDmaPerChunk);
            } else {
                wait_vmcnt((NCH - 1 - j) * kDmaPerChunk);
            }
            // inline-asm LDS reads: a compiler-visible ds_read after an LDS-DMA gets an
            // s_waitcnt vmcnt(0) in front of it, which would drain the whole ring
            float4 pc4[4 * C];
            lds_read_chunk<C, U>(lds_base + static_cast<uint32_t>((j % kRing) * kDmaPerChunk * 64 * 16), pc4);
#pragma unroll
            for (int q4 = 0; q4 < kChunk / 4; ++q4) {
                // the 4 samples 4*q4 .. 4*q4+3 of every channel = pieces q4*C .. q4*C+C-1
                float f[4 * C];
#pragma unroll
                for (int pc = 0; pc < C; ++pc) {
                    const float4 v = pc4[q4 * C + pc];
                    f[4 * pc + 0] = v.x; f[4 * pc + 1] = v.y;
                    f[4 * pc + 2] = v.z; f[4 * pc + 3] = v.w;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = f[i * C];
#pragma unroll
                    for (int cc = 1; cc < C; ++cc) v = is_c[cc] ? f[i * C + cc] : v;
                    const int t = j * kChunk + q4 * 4 + i;
                    if (t < NV) R[t < NV ? t : 0] = v;
                    else asm("v_accvgpr_write_b32 %0, %1" : "=a"(RA[t >= NV ? t - NV : 0]) : "v"(v));
                    // ---- pass 1 (reference order): fp32 sum, zero crossings, extras
                    c32 = c32 + v;
                    const bool pos = v > a.t32;
                    if (t > 0) zc += (pos != prevpos);
                    prevpos = pos;
                    // keep the integer counts sequential: LLVM would otherwise reassociate
                    // the 255 adds into a tree and keep every per-sample bool alive
                    asm volatile("" : "+v"(zc), "+v"(c32));
                    if constexpr (EXTRA) {
                        a32 = a32 + v * v;
                        if (t == 0) {
                            mn = v; mx = v;
                        } else {
                            mn = (v < mn) ? v : mn;
                            mx = (v > mx) ? v : mx;
                            ll = ll + fabsf(v - p1);
                        }
                        if (t > 1) pk += (p1 > p2 && p1 > v);
                        asm volatile("" : "+v"(pk), "+v"(a32), "+v"(ll), "+v"(mn), "+v"(mx));
                        p2 = p1;
                        p1 = v;
                    }
                }
            }
            // slot j % kRing is free again (its reads completed inside lds_read_chunk):
            // refill it with chunk j + kRing (this tile or the next)
            constexpr int jn = j + kRing;
            if constexpr (jn < NCH) {
                issue_chunk<C, jn>(src_cur, ring[j % kRing]);
            } else {
                if (have_next) issue_chunk<C, jn - NCH>(src_next, ring[j % kRing]);
            }
        });

        // ---- pass 2 from registers: deviations from the fp32 mean (array_var, skewness,
        // kurtosis) and, for rows >= 1 of a direct np.var/np.std, from the fp64 mean.
        const float m32 = static_cast<float>(static_cast<double>(c32) / static_cast<double>(W));
        const double m64 = static_cast<double>(c32) / static_cast<double>(W);
        double ssd = 0.0, ssdp = 0.0;
        float s3 = 0.0f, s4 = 0.0f;
#pragma unroll
        for (int t = 0; t < W; ++t) {
            float xt;
            if (t < NV) xt = R[t < NV ? t : 0];
            else asm("v_accvgpr_read_b32 %0, %1" : "=v"(xt) : "a"(RA[t >= NV ? t - NV : 0]));
            const float d = xt - m32;
            const float q = d * d;
            ssd = ssd + static_cast<double>(q);
            s3 = s3 + (d * q) * invW;
            s4 = s4 + (q * q) * invW;
            if constexpr (PAR) {
                const double dd = static_cast<double>(xt) - m64;
                ssdp = ssdp + dd * dd;
            }
            // advance all accumulation chains in lockstep, one sample at a time: LLVM
            // otherwise runs each chain over the whole window in turn and keeps every
            // d and q alive in between (2W extra registers)
            asm volatile("" : "+v"(ssd), "+v"(s3), "+v"(s4), "+v"(ssdp));
        }
        // ---- spectral features while the window is still on chip (before the moment
        // results are materialised, to keep the FFT's 256 live values the peak)
        double spec_bp = 0.0, spec_rbp = 0.0, spec_ent = 0.0, spec_dom = 0.0;
        if constexpr (SPEC) {
            // the window is still on chip: real FFT + spectral features in this lane
            float zr[W / 2], zi[W / 2];
            const float m32s = static_cast<float>(static_cast<double>(c32) / static_cast<double>(W));
#pragma unroll
            for (int t = 0; t < W; ++t) {
                float xt;
                if (t < NV) xt = R[t < NV ? t : 0];
                else asm("v_accvgpr_read_b32 %0, %1" : "=v"(xt) : "a"(RA[t >= NV ? t - NV : 0]));
                const float dt = xt - m32s;           // mean removed (see lane_spectrum)
                if (t & 1) zi[t >> 1] = dt;
                else zr[t >> 1] = dt;
            }
            const SpecOut so = lane_spectrum<W>(zr, zi, static_cast<float>(W) * m32s, a.scale,
                                                a.band_lo, a.band_hi, a.dom_lo,
                                                a.dom_hi, (a.mask & bit(MHF_SPECTRAL_ENTROPY)) != 0,
                                                (a.mask & bit(MHF_DOMINANT_FREQ)) != 0);
            spec_bp = so.bp;
            spec_rbp = so.bp / so.tot;
            spec_ent = so.ent;
            spec_dom = (so.bk < 0) ? static_cast<double>(NAN) : static_cast<double>(so.bk) * a.freq_step;
        }
        const int64_t g = g0 + r;
        const float var32 = static_cast<float>(ssd / static_cast<double>(W));
        const float std32 = static_cast<float>(sqrt(static_cast<double>(var32)));
        const double varp = ssdp / static_cast<double>(W);
        const float kurt = (var32 == 0.0f) ? 0.0f : s4 / (var32 * var32);
        WinVals v;
        v.mean32 = m32;
        v.mean = (g == 0) ? static_cast<double>(m32) : m64;
        v.var32 = var32;
        v.std32 = std32;
        v.var = (g == 0) ? static_cast<double>(var32) : varp;
        v.std_ = (g == 0) ? static_cast<double>(std32) : sqrt(varp);
        v.skew = (std32 == 0.0f) ? 0.0 : static_cast<double>(s3 / (std32 * (std32 * std32)));
        v.kurt = kurt;
        v.kurt_ex = static_cast<double>(kurt) - 3.0;
        v.rms = sqrtf(static_cast<float>(static_cast<double>(a32) / static_cast<double>(W)));
        v.zc = zc;
        v.peaks = pk;
        v.drange = static_cast<double>(mx - mn);
        v.ll = ll;
        v.bp = spec_bp;
        v.rbp = spec_rbp;
        v.ent = spec_ent;
        v.dom = spec_dom;
        if (unit_ok && g <= gmax) {
            const int64_t i = g - a.first;
            for (int jf = 0; jf < F; ++jf) {
                // int32 ids: a scalar kernarg load (an int8 id became a per-lane global
                // load + vmcnt(0), which drained the DMA ring at every store)
                const int f = a.feats.id[jf];
                store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * F + jf) * a.out_ld + i,
                          pick_moment(v, f));
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int W, int C, bool SPEC>
int launch_tile(const FastArgs& a, hipStream_t stream) {
    const int64_t U = 64 / C;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    int64_t blocks = ntiles < 1024 ? ntiles : 1024;   // 256 CUs x 4 waves, persistent
    const bool extra = (a.mask & kExtraBits) != 0;
    const bool par = (a.mask & kParBits) != 0;
    dim3 grid(static_cast<unsigned>(blocks)), block(64);
    if (extra && par) hipLaunchKernelGGL((tile_kernel<W, C, true, true, SPEC>), grid, block, 0, stream, a);
    else if (extra) hipLaunchKernelGGL((tile_kernel<W, C, true, false, SPEC>), grid, block, 0, stream, a);
    else if (par) hipLaunchKernelGGL((tile_kernel<W, C, false, true, SPEC>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((tile_kernel<W, C, false, false, SPEC>), grid, block, 0, stream, a);
    return MHF_OK;
}

template <int W, int C>
int launch_tile_spec(const FastArgs& a, hipStream_t stream) {
    return (a.mask & kSpectralBits) ? launch_tile<W, C, true>(a, stream)
                                    : launch_tile<W, C, false>(a, stream);
}


}  // namespace mhf

#define MHF_DEFINE_TILE_LAUNCH(W, C)                                                   \
    int mhf::launch_tile_w##W##_c##C(const FastArgs& a, hipStream_t stream) {          \
        return launch_tile_spec<W, C>(a, stream);                                      \
    }
#endif  // MHF_TILE_IMPL
