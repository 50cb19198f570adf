// tile64.hip — float64 records (mhf_window_features_f64): the streamed tile kernel.
//
// numba types every reduction of a float64 window in fp64 (SURVEY App. A restated for
// float64, mhfeat.hip window_moments64; pinned by tests/golden/f64_*.npz): sequential fp64
// sums, np.mean = c / W, np.var = sum (x - m)^2 / W (row 0 and the parfor rows agree),
// skewness / kurtosis with per-element division by len(x), RMS sqrt(a / W), zero crossings
// with |x| <= th compared in fp64, strict peaks, minmax-style drange, line length.
//
// Why a different shape from the float32 tile kernel (tile.hip.h): a float64 window of 256
// samples is 512 registers per lane, the whole register file, so the window cannot stay
// on chip between the two passes. One lane per (window, channel), 64 / C windows per
// tile; pass 1 (sums, crossings, peaks, extremes) streams the tile through the LDS-DMA
// ring and parks its first chunks in registers — 8 chunks in AGPRs (v_accvgpr_write: 256
// AGPRs), 3 more in VGPRs — so pass 2 (deviations from the fp64 mean) re-streams only the
// rest: W <= 176 samples never re-read, W = 256 re-reads 5 of 16 chunks (the re-read is
// served by the memory-side cache; what it costs is fabric bandwidth: measured, the
// kernel moves ~5.8 TB/s of total traffic whatever its HBM share). One flat job stream
// per wave (tile q, pass-1 chunk j / pass-2 chunk KEEP + j), RING-1 chunks ahead across
// pass and tile boundaries.
// Chunks are 16 doubles (128 B = one line per window and channel), so the LDS image and
// the DMA geometry are the float32 kernel's (TileGeom<C>, 9 DMA instructions per chunk).
// W is a runtime power of two (>= 16 * RING); the chunk loop is not unrolled over W
// (the parked chunks are addressed through uniform branches on the chunk index).
#define MHF_TILE_IMPL
#include "tile.hip.h"

namespace mhf {
namespace {

constexpr int kC64 = 16;        // doubles per chunk per (window, channel)
constexpr int kRing64 = 4;      // ring slots (4 x 9 KiB per wave)
constexpr int kKeepChunks = 8;  // chunks held in AGPRs between the passes (8 x 32 = 256)
constexpr int kKeepVChunks = 3; // and after them in VGPRs (3 x 32)

template <int C>
__device__ __forceinline__ void lds_read_chunk64(uint32_t addr, double (&v)[kC64]);

template <>
__device__ __forceinline__ void lds_read_chunk64<1>(uint32_t addr, double (&v)[kC64]) {
    // window r at dword 36r (8 pieces + a pad piece): conflict-free ds_read_b128
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
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]),
          "=&v"(o[6]), "=&v"(o[7])
        : "v"(addr)
        : "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[2 * i] = __builtin_bit_cast(double, f2{o[i].x, o[i].y});
        v[2 * i + 1] = __builtin_bit_cast(double, f2{o[i].z, o[i].w});
    }
}

template <>
__device__ __forceinline__ void lds_read_chunk64<3>(uint32_t addr, double (&v)[kC64]) {
    // sample s of this lane's channel at byte 24 s (lane base: window 400 r + channel 8 c)
    float4 o[8];
    asm volatile(
        "ds_read2_b64 %0, %8 offset1:3\n\t"
        "ds_read2_b64 %1, %8 offset0:6 offset1:9\n\t"
        "ds_read2_b64 %2, %8 offset0:12 offset1:15\n\t"
        "ds_read2_b64 %3, %8 offset0:18 offset1:21\n\t"
        "ds_read2_b64 %4, %8 offset0:24 offset1:27\n\t"
        "ds_read2_b64 %5, %8 offset0:30 offset1:33\n\t"
        "ds_read2_b64 %6, %8 offset0:36 offset1:39\n\t"
        "ds_read2_b64 %7, %8 offset0:42 offset1:45\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]),
          "=&v"(o[6]), "=&v"(o[7])
        : "v"(addr)
        : "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[2 * i] = __builtin_bit_cast(double, f2{o[i].x, o[i].y});
        v[2 * i + 1] = __builtin_bit_cast(double, f2{o[i].z, o[i].w});
    }
}

// per-lane DMA byte offsets of a tile (pieces as TileGeom<C>, windows past rmax clamped)
template <int C>
__device__ __forceinline__ void tile64_src(int64_t rmax, int64_t S, int lane, uint32_t (&off)[kDma]) {
    using G = TileGeom<C>;
#pragma unroll
    for (int i = 0; i < kDma; ++i) {
        int r, k;
        G::piece(i * 64 + lane, r, k);
        const int64_t rr = r < rmax ? r : rmax;
        off[i] = static_cast<uint32_t>(rr * S * C * 8 + 16 * k + kBias - dma_inst_off(i));
    }
}

struct P1_64 {
    double c, a, mn, mx, ll, p1, p2;
    int zc, pk;
    bool prevpos;
};

template <int C>
__global__ void __launch_bounds__(64, 1) tile64_kernel(Tile64Args a) {
    using G = TileGeom<C>;
    constexpr int U = G::U;
    constexpr int KD = kDma;
    constexpr int RING = kRing64;
    __shared__ __attribute__((aligned(16))) float4 ring[RING][KD * 64];
    constexpr uint32_t kSlotBytes = KD * 1024;
    constexpr uint32_t kChunkBytes = kC64 * C * 8;

    const int lane = threadIdx.x;
    const int r = lane / C, c = lane - (lane / C) * C;
    const bool unit_ok = r < U;
    const int64_t S = a.wstep;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    if (blockIdx.x >= ntiles) return;
    const int64_t myT = (ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x;
    const int NCH = static_cast<int>(a.wsize / kC64);
    const bool p2 = (a.mask & kPass2Bits) != 0 || (a.mask & bit(MHF_COEFF_VAR)) != 0;
    const bool sk = (a.mask & (bit(MHF_SKEWNESS) | bit(MHF_KURTOSIS) | bit(MHF_KURTOSIS_EXCESS))) != 0;
    const bool want_zc = (a.mask & bit(MHF_ZERO_CROSSINGS)) != 0;
    const bool want_a = (a.mask & bit(MHF_RMS)) != 0;
    const bool want_pk = (a.mask & bit(MHF_PEAK_COUNT)) != 0;
    const bool want_x2 = (a.mask & (bit(MHF_DRANGE) | bit(MHF_LINE_LENGTH))) != 0;
    // the first KEEP chunks of each window stay in AGPRs from pass 1 to pass 2 (parked by
    // v_accvgpr_write: VALU cannot read AGPRs), so pass 2 re-streams only the rest
    constexpr int KA = kKeepChunks, KV = kKeepVChunks;
    const int KEEP = p2 ? (NCH < KA + KV ? NCH : KA + KV) : 0;
    const int JPT = p2 ? 2 * NCH - KEEP : NCH;    // jobs per tile
    const int64_t total = myT * JPT;
    const int64_t gmax = a.first + a.nwin - 1;
    const double invW = 1.0 / static_cast<double>(a.wsize);   // W is a power of two: exact
    const double th = a.th;

    const uint32_t ring_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)&ring[0][0]));
    uint32_t lane_addr;
    if constexpr (C == 1) lane_addr = ring_addr + static_cast<uint32_t>((unit_ok ? r : 0) * G::kWinSlots * 16);
    else lane_addr = ring_addr + static_cast<uint32_t>((unit_ok ? r : 0) * G::kWinSlots * 16 + 8 * c);

    // ---- DMA issue cursor: tile q_i, job j_i within the tile
    int64_t q_i = 0;
    int j_i = 0;
    uint32_t off[kDma];
    uint64_t base_i = 0;
    auto set_issue_tile = [&](int64_t q) {
        const int64_t t = blockIdx.x + q * gridDim.x;
        const int64_t g0 = a.first + t * U;
        base_i = reinterpret_cast<uint64_t>(a.x + g0 * S * C) - kBias;
        tile64_src<C>(gmax - g0, S, lane, off);
    };
    auto issue_next = [&](int slot) {
        const int jc = j_i < NCH ? j_i : KEEP + (j_i - NCH);
        dma_chunk(base_i + static_cast<uint64_t>(jc) * kChunkBytes, ring_addr + slot * kSlotBytes, off);
        if (++j_i == JPT) {
            j_i = 0;
            if (++q_i < myT) set_issue_tile(q_i);
        }
    };
    set_issue_tile(0);
    for (int k = 0; k < RING && k < total; ++k) issue_next(k);

    P1_64 s1{};
    double mean = 0.0, ssd = 0.0, s3 = 0.0, s4 = 0.0;
    float ka[KA][2 * kC64];          // AGPR-parked chunks, 32-bit halves
    double kv[KV][kC64];             // VGPR-held chunks KA .. KA + KV - 1
    // pass 2 over one chunk, deviations from the fp64 mean (a macro: the same code as a
    // lambda with the sums captured by reference took 82 more VGPRs)
#define MHF_T64_PASS2(V)                                         \
    _Pragma("unroll") for (int s = 0; s < kC64; ++s) {           \
        const double d = (V)[s] - mean, q = d * d;               \
        ssd = ssd + q;                                           \
        if (sk) {                                                \
            s3 = s3 + (d * q) * invW;                            \
            s4 = s4 + (q * q) * invW;                            \
        }                                                        \
    }
    int64_t q_p = 0;
    int j_p = 0;
    for (int64_t k = 0; k < total; ++k) {
        const int slot = static_cast<int>(k & (RING - 1));
        if (k + RING - 1 < total) wait_vmcnt<(RING - 1) * KD>();
        else wait_vmcnt<0>();
        double v[kC64];
        lds_read_chunk64<C>(lane_addr + slot * kSlotBytes, v);
        if (k + RING < total) issue_next(slot);

        if (j_p < NCH) {
            // ---- pass 1 over chunk j_p
            int s0 = 0;
            if (j_p == 0) {
                const double x0 = v[0];
                s1 = P1_64{};
                s1.c = 0.0 + x0;            // numba starts the sum at 0.0 (-0.0 -> +0.0)
                s1.a = x0 * x0;
                s1.mn = x0;
                s1.mx = x0;
                s1.p1 = x0;
                s1.prevpos = !(fabs(x0) <= th) && x0 > 0.0;
                s0 = 1;
            }
#pragma unroll
            for (int s = 0; s < kC64; ++s) {
                if (s < s0) continue;
                const double x = v[s];
                s1.c = s1.c + x;
                if (want_a) s1.a = s1.a + x * x;
                if (want_zc) {
                    const bool pos = !(fabs(x) <= th) && x > 0.0;
                    s1.zc += pos != s1.prevpos;
                    s1.prevpos = pos;
                }
                if (want_pk && (j_p > 0 || s >= 2)) s1.pk += (s1.p1 > s1.p2 && s1.p1 > x);
                if (want_x2) {
                    s1.ll = s1.ll + fabs(x - s1.p1);
                    s1.mn = x < s1.mn ? x : s1.mn;
                    s1.mx = x > s1.mx ? x : s1.mx;
                }
                s1.p2 = s1.p1;
                s1.p1 = x;
            }
            if (j_p < KEEP) {
                // park the chunk (a uniform switch: every AGPR index is static)
#pragma unroll
                for (int i = 0; i < KA; ++i) {
                    if (j_p == i) {
#pragma unroll
                        for (int s = 0; s < kC64; ++s) {
                            const f2 h = __builtin_bit_cast(f2, v[s]);
                            asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(ka[i][2 * s]) : "v"(h.x));
                            asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(ka[i][2 * s + 1]) : "v"(h.y));
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < KV; ++i) {
                    if (j_p == KA + i) {
#pragma unroll
                        for (int s = 0; s < kC64; ++s) kv[i][s] = v[s];
                    }
                }
            }
            if (j_p == NCH - 1) {
                mean = s1.c * invW;
                ssd = 0.0; s3 = 0.0; s4 = 0.0;
                // ---- pass 2 over the parked chunks 0 .. KEEP-1 (no memory traffic)
#pragma unroll
                for (int i = 0; i < KA; ++i) {
                    if (i < KEEP) {
                        double u[kC64];
#pragma unroll
                        for (int s = 0; s < kC64; ++s) {
                            float lo, hi;
                            asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(lo) : "a"(ka[i][2 * s]));
                            asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(hi) : "a"(ka[i][2 * s + 1]));
                            u[s] = __builtin_bit_cast(double, f2{lo, hi});
                        }
                        MHF_T64_PASS2(u);
                    }
                }
#pragma unroll
                for (int i = 0; i < KV; ++i) {
                    if (KA + i < KEEP) {
                        MHF_T64_PASS2(kv[i]);
                    }
                }
            }
        } else {
            // ---- pass 2 over chunk KEEP + j_p - NCH: deviations from the fp64 mean
            MHF_T64_PASS2(v);
        }
        if (++j_p == JPT) {
            // ---- tile q_p done: results of (window r, channel c)
            const int64_t g = a.first + (blockIdx.x + q_p * gridDim.x) * U + r;
            WinVals w{};
            const double var = ssd * invW, sd = sqrt(var);
            w.mean = w.mean32 = mean;
            w.var = w.var32 = var;
            w.std_ = w.std32 = sd;
            w.skew = sd == 0.0 ? 0.0 : s3 / (sd * (sd * sd));
            w.kurt = var == 0.0 ? 0.0 : s4 / (var * var);
            w.kurt_ex = w.kurt - 3.0;
            w.rms = sqrt(s1.a * invW);
            w.zc = s1.zc;
            w.peaks = s1.pk;
            w.drange = s1.mx - s1.mn;
            w.ll = s1.ll;
            w.cv = sd / mean;
            if (unit_ok && g <= gmax) {
                const int64_t i = g - a.first;
                for (int jf = 0; jf < a.feats.n; ++jf) {
                    const int f = a.feats.id[jf];
                    if (bit(f) & kTile64Bits)
                        store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + jf) * a.out_ld + i,
                                  pick_moment(w, f));
                }
            }
            j_p = 0;
            ++q_p;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef MHF_T64_PASS2
}

}  // namespace

bool tile64_plan_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                    int64_t wstep, fmask_t mask, int32_t blk, const double* x) {
    if (blk != 0) return false;
    if ((mask & kMomentBits & ~kTile64Bits) != 0 || (mask & kTile64Bits) == 0) return false;
    if (!(channels == 1 || channels == 3)) return false;
    if (sample_stride != channels || (channels > 1 && ch_stride != 1)) return false;
    if (wsize < kC64 * kRing64 || wsize > 65536 || (wsize & (wsize - 1)) != 0) return false;
    if ((wstep * channels) % 2 != 0) return false;                 // 16-B aligned window starts
    if (reinterpret_cast<uintptr_t>(x) % 16 != 0) return false;
    if (wstep * channels * 8 * 64 >= (int64_t(1) << 31)) return false;   // 32-bit DMA offsets
    return true;
}

int launch_tile64(const Tile64Args& a, hipStream_t stream) {
    if (!a.x || !a.out || a.wstep < 1 || a.nwin < 1 || a.first < 0 || a.out_ld < a.nwin ||
        a.feats.n < 1 || a.wsize < kC64 * kRing64 || (a.wsize & (a.wsize - 1)) != 0 ||
        !(a.channels == 1 || a.channels == 3) ||
        a.wstep * a.channels * 8 * 64 >= (int64_t(1) << 31))
        return MHF_EINVAL;
    const int64_t U = 64 / a.channels;
    const int64_t ntiles = (a.nwin + U - 1) / U;
    const int64_t blocks = ntiles < 1024 ? ntiles : 1024;     // 256 CUs x 4 waves, persistent
    if (a.channels == 1)
        hipLaunchKernelGGL(tile64_kernel<1>, dim3(static_cast<unsigned>(blocks)), dim3(64), 0, stream, a);
    else
        hipLaunchKernelGGL(tile64_kernel<3>, dim3(static_cast<unsigned>(blocks)), dim3(64), 0, stream, a);
    return MHF_OK;
}

}  // namespace mhf
