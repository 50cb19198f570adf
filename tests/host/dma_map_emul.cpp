// dma_map_emul.cpp — host emulation of the register tiles' LDS-DMA address maps (test
// infrastructure; built with -fsanitize=address,undefined by tests/host/Makefile and run by
// tests/test_host.py::test_dma_address_maps_under_asan).
//
// For every tile of a launch it replays, with the kernels' own address arithmetic
// (pymhealth_amd/csrc/dma_map.h), what the 64 lanes of a wave compute: the per-lane window
// bounds, the wave reductions (min / max / ballot / readfirstlane / readlane), each DMA
// piece's global address and LDS slot, and then each lane's LDS reads. It checks that
//   * every 16-B piece lies inside the record [x, x + n * C * 4) (the bytes are copied
//     from a host buffer of exactly that size through the translated address, so ASan
//     sees any byte outside it);
//   * every lane the tile path keeps reads exactly its own window's samples (chunk by
//     chunk, for the samples before its end), and its LDS reads stay inside the slot.
// Records are placed at device addresses whose low 32-bit word is >= 2^31 and at
// addresses whose range crosses a 2^32 boundary — the two cases behind round 5's GPU fault
// (a sign-extended readfirstlane word; see dma_map.h).
//
// Kernels emulated: tile_kernel's stream (tile.hip.h, fixed windows W in {128, 256}) and
// tile_idx_kernel's (tile_idx.hip.h: time-indexed windows, fixed windows of any length
// <= 288 at any step, FIX, and overlapping ones read from the tile's union span, SPAN).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../pymhealth_amd/csrc/dma_map.h"

using namespace mhf;

static int g_fail = 0;
#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            if (g_fail < 20) {                                             \
                fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);       \
                fprintf(stderr, __VA_ARGS__);                              \
                fprintf(stderr, "\n");                                     \
            }                                                              \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

// a device record: `xb` the fake device address of sample 0, `host` n * C words
struct Record {
    uint64_t xb;
    int64_t n;
    int C;
    std::vector<uint32_t> host;    // word w holds w + 1 (every sample distinct)
    Record(uint64_t xb_, int64_t n_, int C_) : xb(xb_), n(n_), C(C_), host(n_ * C_) {
        for (size_t w = 0; w < host.size(); ++w) host[w] = static_cast<uint32_t>(w + 1);
    }
    // 16 bytes at device address a into dst, through the host buffer (ASan-visible)
    bool fetch16(uint64_t a, uint8_t* dst) const {
        const uint64_t bytes = static_cast<uint64_t>(n) * C * 4, end = xb + bytes;
        const bool in = a >= xb && a - xb <= bytes - 16;     // (no wrap-around at 2^64)
        CHECK(in, "piece [%#llx, +16) outside the record [%#llx, %#llx)", (unsigned long long)a,
              (unsigned long long)xb, (unsigned long long)end);
        if (!in) return false;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(host.data()) + (a - xb);
        memcpy(dst, src, 16);
        return true;
    }
};

// readfirstlane / readlane return int, as __builtin_amdgcn_readfirstlane does
static int rfl(uint32_t v) { return static_cast<int>(v); }

constexpr uint32_t kSlotBytes = dma::kDma * 1024;

// ---- tile.hip.h: fixed windows W in {128, 256}, 16-B aligned window starts -------------
template <int C>
static void emulate_fixed_tile(const Record& rec, int64_t W, int64_t S, int64_t first, int64_t nwin) {
    using G = dma::Geom<C>;
    const int U = G::U;
    const int64_t gmax = first + nwin - 1;
    const int64_t ntiles = (nwin + U - 1) / U;
    std::vector<uint8_t> lds(kSlotBytes);
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t g0 = first + t * U;
        const int64_t rmax = gmax - g0;
        const uint64_t base = dma::fix_tile_base(rec.xb, g0, S, C);
        for (int J = 0; J < W / dma::kChunk; ++J) {
            std::fill(lds.begin(), lds.end(), 0xAB);
            const uint64_t cb = base + static_cast<uint64_t>(J) * dma::kChunk * C * 4;
            for (int q = 0; q < dma::kDma; ++q)
                for (int lane = 0; lane < 64; ++lane) {
                    int r, k;
                    G::piece(q * 64 + lane, r, k);
                    const int64_t rr = r < rmax ? r : rmax;
                    const uint32_t off = dma::fix_lane_off(rr, S, C, k, q);
                    rec.fetch16(dma::piece_addr(cb, off, q), &lds[dma::lds_slot_byte(q, lane)]);
                }
            // lane reads: C = 1 window r at dword 36 r (8 x ds_read_b128); C = 3 window r,
            // channel c at dword 100 r + c + 3 s
            for (int lane = 0; lane < 64; ++lane) {
                const int r = lane / C, c = lane % C;
                if (r >= U || g0 + r > gmax) continue;
                const uint32_t la = static_cast<uint32_t>((r * G::kWinSlots * 4 + (C == 1 ? 0 : c)) * 4);
                for (int s = 0; s < dma::kChunk; ++s) {
                    const uint32_t at = la + static_cast<uint32_t>(4 * C * s);
                    CHECK(at + 4 <= kSlotBytes, "fixed C=%d read past the slot", C);
                    uint32_t v;
                    memcpy(&v, &lds[at], 4);
                    const int64_t smp = (g0 + r) * S + J * dma::kChunk + s;
                    const uint32_t want = static_cast<uint32_t>(smp * C + c + 1);
                    CHECK(v == want, "fixed C=%d tile %lld window %d chunk %d sample %d: got %u want %u",
                          C, (long long)t, r, J, s, v, want);
                }
            }
        }
    }
}

// ---- tile_idx.hip.h: time-indexed windows (FIX = false) or fixed windows of any length
template <int C>
static void emulate_idx_tile(const Record& rec, bool FIX, const std::vector<int64_t>& starts,
                             const std::vector<int64_t>& ends, int64_t min_len, int64_t wsize,
                             int64_t wstep, int64_t first, int64_t nwin, int64_t* kept_tiles) {
    using G = dma::Geom<C>;
    constexpr int U = G::U;
    constexpr int kWmax = 288, NCH = kWmax / dma::kChunk;
    const int64_t CH = dma::kChunk * C * 4;
    const int64_t ntiles = (nwin + U - 1) / U;
    std::vector<uint8_t> lds(kSlotBytes);
    for (int64_t tile = 0; tile < ntiles; ++tile) {
        int64_t s0[64], W64[64];
        bool keep[64], valid[64], dma_ok[64];
        uint64_t bstart[64], base_lane[64];
        for (int lane = 0; lane < 64; ++lane) {
            const int r = lane / C;
            const int64_t i = tile * U + r;
            valid[lane] = r < U && i < nwin;
            s0[lane] = 0; W64[lane] = 0; keep[lane] = false;
            if (FIX && valid[lane]) {
                const int64_t g = first + i;
                s0[lane] = g * wstep;
                W64[lane] = wsize;
                keep[lane] = true;
            } else if (valid[lane]) {
                const int64_t si = starts[i], ei = ends[i], n = rec.n;
                int64_t b0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
                b0 = b0 < 0 ? 0 : (b0 > n ? n : b0);
                e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
                s0[lane] = b0;
                W64[lane] = e0 > b0 ? e0 - b0 : 0;
                keep[lane] = (ei - si >= min_len) && W64[lane] > 0;
            }
            bstart[lane] = rec.xb + static_cast<uint64_t>(s0[lane]) * C * 4;
            base_lane[lane] = dma::idx_piece_base(bstart[lane]);
            dma_ok[lane] = !keep[lane] || (s0[lane] + kWmax + 4 <= rec.n && base_lane[lane] >= rec.xb);
        }
        uint64_t bmin = ~uint64_t(0), bmax = 0;
        bool any_keep = false, all_ok = true;
        for (int lane = 0; lane < 64; ++lane) {
            if (keep[lane]) {
                bmin = base_lane[lane] < bmin ? base_lane[lane] : bmin;
                bmax = base_lane[lane] > bmax ? base_lane[lane] : bmax;
                any_keep = true;
            }
            all_ok = all_ok && dma_ok[lane];
        }
        const bool tile_ok = any_keep && all_ok && bmax - bmin < (uint64_t(1) << 30);
        bool slow[64];
        int W[64];
        for (int lane = 0; lane < 64; ++lane) {
            slow[lane] = keep[lane] && (!tile_ok || W64[lane] > kWmax);
            W[lane] = static_cast<int>(tile_ok && keep[lane] && !slow[lane] ? W64[lane] : 0);
            // the global-memory walk of a slow lane reads samples [s0, s0 + W64)
            if (slow[lane]) CHECK(s0[lane] + W64[lane] <= rec.n, "slow walk past the record");
        }
        if (!tile_ok) continue;
        ++*kept_tiles;
        int wmin = kWmax;
        int first_keep = -1;
        for (int lane = 0; lane < 64; ++lane) {
            if (keep[lane] && !slow[lane]) wmin = W[lane] < wmin ? W[lane] : wmin;
            if (keep[lane] && first_keep < 0) first_keep = lane / C;
        }
        const uint64_t bfk = dma::sgpr_pair(rfl(dma::lo_word(base_lane[first_keep * C])),
                                            rfl(dma::hi_word(base_lane[first_keep * C])));
        int32_t wbytes[64];
        for (int lane = 0; lane < 64; ++lane)
            wbytes[lane] = keep[lane] ? static_cast<int>(static_cast<uint32_t>(bstart[lane] - base_lane[lane]) +
                                                         (W64[lane] < 4096 ? W64[lane] : 4096) * C * 4)
                                      : 0x7fffffff;
        uint32_t off[dma::kDma][64];
        int32_t lim[dma::kDma][64];
        for (int q = 0; q < dma::kDma; ++q)
            for (int lane = 0; lane < 64; ++lane) {
                int j = q * 64 + lane;
                if (j > U * G::kWinSlots - 1) j = U * G::kWinSlots - 1;
                const int rr = j / G::kWinSlots;
                const int k = j - rr * G::kWinSlots;
                const int src = rr * C;
                const uint64_t b = keep[src] ? base_lane[src] : bfk;
                off[q][lane] = dma::idx_lane_off(b, bmin, k, q);
                lim[q][lane] = dma::idx_lane_lim(keep[src], wbytes[src], k);
            }
        const uint64_t sbase = dma::sgpr_pair(rfl(dma::lo_word(bmin - dma::kBias)),
                                              rfl(dma::hi_word(bmin - dma::kBias)));
        CHECK(sbase == bmin - dma::kBias, "SGPR base %#llx != %#llx", (unsigned long long)sbase,
              (unsigned long long)(bmin - dma::kBias));
        for (int jj = 0; jj < NCH; ++jj) {
            std::fill(lds.begin(), lds.end(), 0xAB);
            const bool redirect = !FIX && jj > 0 && (jj + 1) * dma::kChunk > wmin;
            for (int q = 0; q < dma::kDma; ++q)
                for (int lane = 0; lane < 64; ++lane) {
                    const uint32_t o = redirect ? dma::idx_redirect(off[q][lane], jj * CH, lim[q][lane], CH)
                                                : off[q][lane];
                    rec.fetch16(dma::piece_addr(sbase + static_cast<uint64_t>(jj * CH), o, q),
                                &lds[dma::lds_slot_byte(q, lane)]);
                }
            for (int lane = 0; lane < 64; ++lane) {
                const int r = lane / C, c = lane % C;
                if (!keep[lane] || slow[lane]) continue;
                const uint32_t mis = static_cast<uint32_t>(bstart[lane] - base_lane[lane]);
                const uint32_t la = static_cast<uint32_t>(r * G::kWinSlots * 16) + mis +
                                    static_cast<uint32_t>(C > 1 ? c * 4 : 0);
                for (int s = 0; s < dma::kChunk; ++s) {
                    const int t = jj * dma::kChunk + s;
                    const uint32_t at = la + static_cast<uint32_t>(4 * C * s);
                    CHECK(at + 4 <= kSlotBytes, "idx C=%d read past the slot", C);
                    if (t >= W[lane]) continue;              // zeroed by pass 1
                    uint32_t v;
                    memcpy(&v, &lds[at], 4);
                    const uint32_t want = static_cast<uint32_t>((s0[lane] + t) * C + c + 1);
                    CHECK(v == want, "idx C=%d FIX=%d tile %lld lane %d sample %d: got %u want %u", C, FIX,
                          (long long)tile, lane, t, v, want);
                }
            }
        }
    }
}

// ---- tile_idx.hip.h, SPAN: overlapping fixed windows read from the tile's union span image
// (the host plan's conditions: S < W, the image within kSpanBytes for every tile)
template <int C>
static void emulate_span_tile(const Record& rec, int64_t W, int64_t S, int64_t first, int64_t nwin,
                              int64_t* span_tiles) {
    constexpr int U = 64 / C;
    if (!(S < W && 16 + ((U - 1) * S + dma::kSpanRead) * C * 4 <= dma::kSpanBytes)) return;
    const int64_t ntiles = (nwin + U - 1) / U;
    std::vector<uint8_t> lds(dma::kSpanBytes);
    for (int64_t tile = 0; tile < ntiles; ++tile) {
        const int64_t i0 = tile * U;
        const int64_t ntw = nwin - i0 < U ? nwin - i0 : U;
        const dma::SpanGeom g = dma::span_geom(rec.xb, rec.n, C, first + i0, ntw, S, W, dma::kSpanBytes);
        if (!g.ok) {            // the tile's lanes walk global memory: inside the record
            for (int64_t r = 0; r < ntw; ++r)
                CHECK((first + i0 + r) * S + W <= rec.n, "span: slow walk past the record");
            continue;
        }
        ++*span_tiles;
        CHECK(g.nbytes <= static_cast<uint32_t>(dma::kSpanBytes), "span image %u B over the cap", g.nbytes);
        std::fill(lds.begin(), lds.end(), 0xAB);
        const int ni = static_cast<int>((g.nbytes + 1023u) >> 10);
        for (int k = 0; k < ni; ++k)
            for (int lane = 0; lane < 64; ++lane) {
                const uint32_t voff = 16u * static_cast<uint32_t>(lane);
                if (!(voff < g.nbytes - 1024u * static_cast<uint32_t>(k))) continue;   // the kernel's predicate
                const uint32_t at = 1024u * static_cast<uint32_t>(k) + voff;
                CHECK(at + 16 <= static_cast<uint32_t>(dma::kSpanBytes), "span DMA past the LDS image");
                if (at + 16 > static_cast<uint32_t>(dma::kSpanBytes)) continue;
                rec.fetch16(g.gbase + 1024u * static_cast<uint64_t>(k) + voff, &lds[at]);
            }
        // every unit lane reads 9 chunks (kSpanRead samples) from its window's span byte;
        // kept windows' samples before their end must be their own
        for (int lane = 0; lane < U * C; ++lane) {
            const int r = lane / C, c = lane % C;
            for (int64_t t = 0; t < dma::kSpanRead; ++t) {
                const uint32_t at = dma::span_lane_byte(g.mis0, r, S, C, c, t);
                CHECK(at + 4 <= static_cast<uint32_t>(dma::kSpanBytes), "span C=%d read past the image", C);
                if (r >= ntw || t >= W || at + 4 > static_cast<uint32_t>(dma::kSpanBytes)) continue;
                uint32_t v;
                memcpy(&v, &lds[at], 4);
                const uint32_t want = static_cast<uint32_t>(((first + i0 + r) * S + t) * C + c + 1);
                CHECK(v == want, "span C=%d W=%lld S=%lld tile %lld window %d sample %lld: got %u want %u", C,
                      (long long)W, (long long)S, (long long)tile, r, (long long)t, v, want);
            }
        }
    }
}

int main() {
    std::mt19937_64 rng(12345);
    // device addresses: low word >= 2^31; the record crossing a 2^32 boundary; low word
    // just below 2^31 (the sign flips inside the record); a record near 0 (bases underflow?)
    const uint64_t bases[] = {0x7f3a80000000ull, 0x7f3affffe000ull, 0x7f3a7ffff000ull,
                              0x00000fff0000ull, 0x7f3bfffff000ull};
    int64_t idx_tiles = 0, fix_tiles = 0, span_tiles = 0;
    for (uint64_t b0 : bases) {
        for (int mis4 = 0; mis4 < 4; ++mis4) {             // 4-B aligned records (tile_idx)
            const uint64_t xb = b0 + 4u * mis4;
            for (int C : {1, 3}) {
                const int64_t n = 40000 + (rng() % 5000);
                Record rec(xb, n, C);
                // time-indexed windows: mixed lengths, short / empty / long / negative /
                // past-the-end windows, unsorted
                const int64_t nw = 700;
                std::vector<int64_t> st(nw), en(nw);
                for (int64_t i = 0; i < nw; ++i) {
                    const int64_t s = static_cast<int64_t>(rng() % (n - 10));
                    int64_t len = 1 + static_cast<int64_t>(rng() % 300);
                    const int kind = static_cast<int>(rng() % 16);
                    if (kind == 0) len = 289 + static_cast<int64_t>(rng() % 400);   // longer than the tile
                    if (kind == 1) len = 0;                                         // empty
                    st[i] = s;
                    en[i] = s + len;
                    if (kind == 2) { st[i] = s - n; en[i] = s + len - n; }         // negative indices
                    if (kind == 3) { st[i] = n - 1 - static_cast<int64_t>(rng() % 200); en[i] = st[i] + len; }
                    if (kind == 4) en[i] = st[i] - 3;                               // reversed: empty
                }
                if (C == 1) emulate_idx_tile<1>(rec, false, st, en, 2, 0, 0, 0, nw, &idx_tiles);
                else emulate_idx_tile<3>(rec, false, st, en, 2, 0, 0, 0, nw, &idx_tiles);
                // sorted, dense windows (the bench's cfgidx shape): most tiles take the tile path
                for (int64_t i = 0; i < nw; ++i) {
                    st[i] = i * 50 + static_cast<int64_t>(rng() % 7);
                    en[i] = st[i] + 240 + static_cast<int64_t>(rng() % 40);
                }
                if (C == 1) emulate_idx_tile<1>(rec, false, st, en, 1, 0, 0, 0, nw, &idx_tiles);
                else emulate_idx_tile<3>(rec, false, st, en, 1, 0, 0, 0, nw, &idx_tiles);
                // fixed windows of any length <= 288 at any step (tile_fix), incl. the last
                // windows of the record
                for (int64_t W : {7, 100, 250, 288}) {
                    for (int64_t S : {1, 3, 37, 125, 250, 300}) {
                        const int64_t nwf = 1 + (n - W) / S;
                        const int64_t f0 = nwf > 300 ? nwf - 300 : 0;
                        if (C == 1) emulate_idx_tile<1>(rec, true, st, en, 0, W, S, f0, nwf - f0, &fix_tiles);
                        else emulate_idx_tile<3>(rec, true, st, en, 0, W, S, f0, nwf - f0, &fix_tiles);
                    }
                    // the span image (S < W): the record's last windows, a run from window 0,
                    // a run ending mid-record
                    for (int64_t S : {1, 3, 37, 63, 99, 125, 126, 143}) {
                        const int64_t nwf = 1 + (n - W) / S;
                        const int64_t f0 = nwf > 300 ? nwf - 300 : 0;
                        const int64_t m = nwf < 200 ? nwf : 200;
                        if (C == 1) {
                            emulate_span_tile<1>(rec, W, S, f0, nwf - f0, &span_tiles);
                            emulate_span_tile<1>(rec, W, S, 0, m, &span_tiles);
                            emulate_span_tile<1>(rec, W, S, nwf / 2, m / 2, &span_tiles);
                        } else {
                            emulate_span_tile<3>(rec, W, S, f0, nwf - f0, &span_tiles);
                            emulate_span_tile<3>(rec, W, S, 0, m, &span_tiles);
                            emulate_span_tile<3>(rec, W, S, nwf / 2, m / 2, &span_tiles);
                        }
                    }
                }
            }
        }
        // tile.hip.h: 16-B aligned record, window starts 16-B aligned ((S * C) % 4 == 0)
        for (int C : {1, 3}) {
            const int64_t n = 30000 + 4 * (rng() % 1000);
            Record rec(b0, n, C);
            for (int64_t W : {128, 256})
                for (int64_t S : {W, W / 2, W + 32, int64_t(64), int64_t(4), int64_t(1024)}) {
                    if ((S * C) % 4) continue;
                    const int64_t nw = 1 + (n - W) / S;
                    if (C == 1) { emulate_fixed_tile<1>(rec, W, S, 0, nw); emulate_fixed_tile<1>(rec, W, S, nw / 3, nw - nw / 3); }
                    else { emulate_fixed_tile<3>(rec, W, S, 0, nw); emulate_fixed_tile<3>(rec, W, S, nw / 3, nw - nw / 3); }
                }
        }
    }
    // the sign-extension case on its own: a low word >= 2^31 through sgpr_pair
    const uint64_t hi = 0x7f3a8000ab10ull;
    CHECK(dma::sgpr_pair(rfl(dma::lo_word(hi)), rfl(dma::hi_word(hi))) == hi, "sgpr_pair sign-extends");
    CHECK(idx_tiles > 100 && fix_tiles > 100 && span_tiles > 100,
          "too few tiles took the tile path: %lld / %lld / %lld", (long long)idx_tiles,
          (long long)fix_tiles, (long long)span_tiles);
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("DMA MAPS OK: %lld indexed tiles, %lld fixed-window (any length) tiles, %lld span-image "
           "tiles emulated\n", (long long)idx_tiles, (long long)fix_tiles, (long long)span_tiles);
    return 0;
}
