// dma_map.h — the address arithmetic of the register tiles' LDS-DMA streams, shared by the
// kernels (tile.hip.h: fixed windows, W in {128, 256}; tile_idx.hip.h: time-indexed windows
// and fixed windows of any length <= 288) and by their host emulation
// (tests/host/dma_map_emul.cpp, built with -fsanitize=address,undefined by
// tests/host/Makefile), so the emulation checks the kernels' own expressions.
//
// One chunk of a tile = kDma LDS-DMA instructions (global_load_lds_dwordx4, saddr form): lane
// l of instruction q fetches the 16 bytes at
//     SGPR base + zero-extended 32-bit lane offset + signed 13-bit instruction offset
// into LDS slot j = 64 q + l of the chunk image (M0 + the same instruction offset + 16 l).
// The instruction offsets run -2..+2 KiB (q < 5) and -1..+2 KiB (q >= 5); the lane offsets
// carry the opposite of it plus kBias, and the SGPR base carries -kBias, so every lane
// offset stays a non-negative 32-bit value.
//
// Round 5's first GPU run of tile_idx faulted twice here: a readfirstlane result (int) of a
// low address word >= 2^31 was sign-extended over the high word (sgpr_pair below now
// takes both words through uint32_t), and a ds_bpermute under partial EXEC read disabled
// lanes as 0 (the kernel now broadcasts the borrowed base with readlane outside any branch).
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define MHF_HD __host__ __device__ __forceinline__
#else
#define MHF_HD inline
#endif

namespace mhf {
namespace dma {

constexpr uint32_t kBias = 4096;
constexpr int kDma = 9;           // instructions (64 lanes x 16 B) per chunk image
constexpr int kChunk = 32;        // samples per chunk and window

MHF_HD constexpr int inst_off(int q) { return (q < 5 ? q - 2 : q - 6) * 1024; }

// an SGPR pair from the two readfirstlane results (int) of an address's words: each word
// goes through uint32_t (a low word >= 2^31 must not sign-extend over the high one)
MHF_HD constexpr uint64_t sgpr_pair(int lo, int hi) {
    return static_cast<uint64_t>(static_cast<uint32_t>(lo)) |
           (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32);
}
MHF_HD constexpr uint32_t lo_word(uint64_t v) { return static_cast<uint32_t>(v); }
MHF_HD constexpr uint32_t hi_word(uint64_t v) { return static_cast<uint32_t>(v >> 32); }

// the global address lane `lane_off` of instruction q reaches from SGPR base `sbase`
MHF_HD constexpr uint64_t piece_addr(uint64_t sbase, uint32_t lane_off, int q) {
    return sbase + static_cast<uint64_t>(lane_off) + static_cast<uint64_t>(static_cast<int64_t>(inst_off(q)));
}
// the LDS byte (relative to the chunk slot) lane l of instruction q writes
MHF_HD constexpr uint32_t lds_slot_byte(int q, int lane) { return static_cast<uint32_t>((64 * q + lane) * 16); }

// Chunk image of a tile of U = 64 / C windows: the kPieces 16-B pieces of tile-window r at
// slots r * kWinSlots .. + kPieces - 1, one pad slot after each window (bank spread); slot
// j -> (r, k); pad and spare slots re-load a real piece (an L2 hit on a line the same
// instruction fetches)
template <int C>
struct Geom {
    static constexpr int U = 64 / C;
    static constexpr int kPieces = kChunk * C * 4 / 16;   // 8 (C = 1) / 24 (C = 3)
    static constexpr int kWinSlots = kPieces + 1;         // window stride: 36 / 100 dwords
    static_assert(U * kWinSlots <= 64 * kDma, "chunk image exceeds the DMA slots");
    MHF_HD static void piece(int j, int& r, int& k) {
        if (j > U * kWinSlots - 1) j = U * kWinSlots - 1;
        r = j / kWinSlots;
        k = j - r * kWinSlots;
        if (k == kPieces) k = kPieces - 1;
    }
};

// ---- fixed windows, W in {128, 256}, 16-B aligned starts (tile.hip.h)
// lane offset of instruction q for tile-window rr (clamped to the last window by the caller)
// and piece k; the tile's SGPR base (window g0's first byte minus kBias)
MHF_HD constexpr uint32_t fix_lane_off(int64_t rr, int64_t S, int C, int k, int q) {
    return static_cast<uint32_t>(static_cast<int64_t>((rr * S * C + 4 * k) * 4) + kBias - inst_off(q));
}
MHF_HD constexpr uint64_t fix_tile_base(uint64_t x, int64_t g0, int64_t S, int C) {
    return x + static_cast<uint64_t>(g0 * S * C) * 4u - kBias;
}

// ---- time-indexed windows / any-length fixed windows (tile_idx.hip.h)
// a window's 16-B piece grid starts at its first byte rounded down to 16 B
MHF_HD constexpr uint64_t idx_piece_base(uint64_t bstart) { return bstart & ~uint64_t(15); }
// lane offset of instruction q for piece k of the window whose grid starts at b, the tile's
// lowest grid start bmin (SGPR base = bmin - kBias; the tile needs bmax - bmin < 2^30)
MHF_HD constexpr uint32_t idx_lane_off(uint64_t b, uint64_t bmin, int k, int q) {
    return static_cast<uint32_t>(b - bmin) + static_cast<uint32_t>(16 * k) + kBias -
           static_cast<uint32_t>(inst_off(q));
}
// chunk offset (bytes) from which slot q's piece lies past its window's last byte
// (wbytes: the window's bytes from its grid start; windows the tile does not keep: never)
MHF_HD constexpr int32_t idx_lane_lim(bool kept, int32_t wbytes, int k) {
    return kept ? wbytes - 16 * k : 0x7fffffff;
}
// the lane offset chunk jj uses: pieces past the window's end re-read the previous chunk's
// address (bytes the previous DMA just fetched) instead of the next window's lines
MHF_HD constexpr uint32_t idx_redirect(uint32_t off, int64_t chunk_byte, int32_t lim, int64_t CH) {
    return chunk_byte < lim ? off : off - static_cast<uint32_t>(CH);
}

// ---- overlapping fixed windows, staged as the tile's union span (tile_idx.hip.h, SPAN)
// The ntw windows g0 .. g0 + ntw - 1 of a tile (S < W) cover samples [g0 S, (g0 + ntw - 1) S
// + W); the span image is the 16-B piece grid from g0 S's first byte (gbase, mis0 bytes
// before it) through the bytes pass 1 reads (every window's kSpanRead samples: 9 chunks,
// past a window's end the next windows' samples, zeroed as read), cut at the last whole
// 16-B piece of the record. Piece p (lane p % 64 of instruction p / 64) fetches the 16 bytes
// at gbase + 16 p into span byte 16 p; lane (r, c) reads sample t of its window at span byte
// mis0 + ((r S + t) C + c) 4. ok = false (the tile's lanes take the global-memory walk) when
// the grid would start before the record, the cut would drop a window sample, or the image
// would exceed cap bytes.
constexpr int64_t kSpanRead = 288;   // samples pass 1 reads per window (kIdxWmax)
// the image's LDS per wave: 37 KiB keeps 4 waves per CU (148 of 160 KiB)
constexpr int kSpanBytes = 37 * 1024;
struct SpanGeom {
    uint64_t gbase;
    uint32_t mis0, nbytes;
    bool ok;
};
MHF_HD constexpr SpanGeom span_geom(uint64_t xb, int64_t n_samples, int C, int64_t g0, int64_t ntw,
                                    int64_t S, int64_t W, int64_t cap) {
    const uint64_t gs = xb + static_cast<uint64_t>(g0 * S * C) * 4u;
    const uint64_t gbase = gs & ~uint64_t(15);
    const uint64_t need = (gs + static_cast<uint64_t>(((ntw - 1) * S + kSpanRead) * C) * 4u + 15u) & ~uint64_t(15);
    const uint64_t xe = (xb + static_cast<uint64_t>(n_samples * C) * 4u) & ~uint64_t(15);
    const uint64_t end = need < xe ? need : xe;
    const uint64_t wend = gs + static_cast<uint64_t>(((ntw - 1) * S + W) * C) * 4u;
    const bool ok = ntw >= 1 && gbase >= xb && end >= wend && end - gbase <= static_cast<uint64_t>(cap);
    return SpanGeom{gbase, static_cast<uint32_t>(gs - gbase), ok ? static_cast<uint32_t>(end - gbase) : 0u, ok};
}
// LDS byte of sample t of lane (r, c)'s window in the span image
MHF_HD constexpr uint32_t span_lane_byte(uint32_t mis0, int64_t r, int64_t S, int C, int c, int64_t t) {
    return mis0 + static_cast<uint32_t>(((r * S + t) * C + c) * 4);
}
// worst bank multiplicity of the span reads (ds_read2_b32: banks (a / 4) mod 32 per 32-lane
// group) for window stride S: the host takes the span path only when it is small
inline int span_bank_ways(int64_t S, int C) {
    int worst = 1;
    const int U = 64 / C;
    for (int g = 0; g < 2; ++g) {
        int cnt[32] = {0};
        for (int l = 32 * g; l < 32 * g + 32; ++l) {
            const int r = l / C, c = l - (l / C) * C;
            if (r >= U) continue;
            const int b = static_cast<int>(((static_cast<int64_t>(r) * S * C + c) % 32 + 32) % 32);
            if (++cnt[b] > worst) worst = cnt[b];
        }
    }
    return worst;
}

}  // namespace dma
}  // namespace mhf
