// spectral_reg.hip — spectral features of W = 1024 windows (cfg5: ECG, stride 128) with
// the FFT held in registers: one wavefront per window, 8 complex points per lane, three
// radix-8 passes, two LDS transposes (bank-conflict-free for the ds_read2/write2_b64 the
// compiler forms) and one lane permute for the real-FFT bin pairs; per-lane twiddle
// tables (fp64-accurate) held in VGPRs.
//
// Why: the LDS Stockham kernel (spectral_wave.hip) makes every radix pass an LDS round
// trip with scattered writes and LDS twiddle reads (cfg5: 16.3 ms). Here a window costs
// ~270 VALU, ~100 SALU and 36 LDS instructions (PMC, profiles/r02g_cfg5_summary.md); cfg5
// runs in 7.7 ms, reading each input sample from HBM once (FETCH = 1.00 x the distinct
// input: per-wave sample ring, MODE 2 below).
//
// rFFT(1024) = 512-point complex FFT of z_n = x_2n + i x_2n+1 (uncentred, see
// fft_windows). With n = l + 64 r (lane l, register r) and K = k + 8 c + 64 d:
//   pass 1 (in lane l):        y_k(l) = w512^(l k) * DFT8_r(z_{l+64r})_k
//   transpose 1 -> lane (k,b): u_a = y_k(8a + b)
//   pass 2:                    v_c = w64^(b c) * DFT8_a(u)_c
//   transpose 2 -> lane k + 8c: v(b) for b = 0..7
//   pass 3:                    Z[k + 8c + 64d] = DFT8_b(v)_d (lane K mod 64, register K / 64)
//   each lane then fetches the partners Z[512 - K] of its 8 bins from one partner lane
//   (16 ds_bpermute) and evaluates its own bins.
// Post-processing, features and scaling as in spectral_lane.hip.inc / spectral_wave.hip.
#include "engine_common.h"
#include "spectral_wave.h"
#include <type_traits>

namespace mhf {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kN = 512;          // complex FFT length (W = 1024)
constexpr int kW = 2 * kN;
constexpr int kT1 = 72;          // transpose-1 row stride (cf): reads hit 64 distinct banks
// transpose 2: element (k, b, c) — pass 2's output c of lane 8 k + b — at cf 8 c + 66 b + k,
// so that lane k + 8 c (bin K = k + 8 c + 64 d in register d: lane order = bin order within
// a row) reads its v(b) at cf lane + 66 b; conflict-free for the ds_write_b64 (16-lane
// groups) and the ds_read_b64 / ds_read2_b64 (32- / 16-lane groups) of both sides (an
// exhaustive search over c P + b R + k Q; the old lane 8 k + c order needed a bit-transposed
// ballot to find the first arg-max bin: 14 SALU per window)
constexpr int kT2c = 8, kT2b = 66;
constexpr int kBufCf = 8 * kT1;  // per-wave LDS buffer (cf), reused by the 3 transposes
constexpr float kS2 = 0.70710678118654752440f;
// w16^d = exp(-2 pi i d / 16)
__constant__ float kC16[8] = {1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                              0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f};
__constant__ float kS16[8] = {0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
                              -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};

__device__ __forceinline__ f2 cmul(f2 a, f2 w) {
    // (a.x w.x - a.y w.y, a.x w.y + a.y w.x) = fma(a.xx, w, (-a.y w.y, a.y w.x)): two VOP3P
    // instructions, the swap and sign in the operand selects (LLVM spent a v_xor + v_mov
    // building (-w.y, w.x) whenever w was not loop-invariant)
    f2 p, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]" : "=v"(p) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(w), "v"(p));
    return r;
}
// (a.x + b.x, a.y - b.y) = a + conj b, one v_pk_add_f32
__device__ __forceinline__ f2 add_conj(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (a.y + b.y, b.x - a.x) = -i (a - conj b), one v_pk_add_f32
__device__ __forceinline__ f2 odd_pair(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// a + (-i) b = (a.x + b.y, a.y - b.x) and a - (-i) b = (a.x - b.y, a.y + b.x): one
// v_pk_add_f32 each, the swap and sign in the operand selects (LLVM materialised -i b as
// a v_mov + v_xor pair before every such add)
__device__ __forceinline__ f2 add_mi(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 sub_mi(f2 a, f2 b) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (o.x + o.y, o.y - o.x) = o (1 - i) and (o.y - o.x, -o.x - o.y) = o (-1 - i)
__device__ __forceinline__ f2 mul_1mi(f2 o) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(o));
    return r;
}
__device__ __forceinline__ f2 mul_m1mi(f2 o) {
    f2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(r) : "v"(o));
    return r;
}

// in-register 8-point DFT (forward, e^{-2 pi i / 8} kernel), natural order in and out:
// 24 v_pk instructions (w8 = (1 - i) / sqrt 2, w8^3 = (-1 - i) / sqrt 2 as one swap-add
// and a fused multiply-add into the output)
__device__ __forceinline__ void dft8(f2 (&v)[8]) {
    const f2 a0 = v[0] + v[4], a1 = v[0] - v[4], a2 = v[2] + v[6], d26 = v[2] - v[6];
    const f2 b0 = v[1] + v[5], b1 = v[1] - v[5], b2 = v[3] + v[7], d37 = v[3] - v[7];
    const f2 e0 = a0 + a2, e2 = a0 - a2, e1 = add_mi(a1, d26), e3 = sub_mi(a1, d26);   // DFT4 evens
    const f2 o0 = b0 + b2, o2 = b0 - b2, o1 = add_mi(b1, d37), o3 = sub_mi(b1, d37);   // DFT4 odds
    const f2 u1 = mul_1mi(o1), u3 = mul_m1mi(o3);
    const f2 s2 = {kS2, kS2};
    v[0] = e0 + o0; v[4] = e0 - o0;
    v[1] = __builtin_elementwise_fma(u1, s2, e1); v[5] = __builtin_elementwise_fma(u1, -s2, e1);
    v[2] = add_mi(e2, o2); v[6] = sub_mi(e2, o2);
    v[3] = __builtin_elementwise_fma(u3, s2, e3); v[7] = __builtin_elementwise_fma(u3, -s2, e3);
}

__device__ __forceinline__ f2 twiddle(int num, int den) {   // exp(-2 pi i num / den), fp64
    double s, c;
    sincospi(-2.0 * static_cast<double>(num) / static_cast<double>(den), &s, &c);
    return f2{static_cast<float>(c), static_cast<float>(s)};
}

// Wave reductions without LDS round trips: DPP within each 16-lane row (quad_perm
// [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8 leave the row total in every lane), then
// row_bcast:15 (rows 1, 3 add row 0, 2's total) and row_bcast:31 (row 3 adds row 1's):
// lane 63 holds (r3 + r2) + (r1 + r0), one v_readlane makes it uniform.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// DPP move into the rows of ROWS only (the other rows' lanes are left undefined: the
// reductions below never read them)
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_rows(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// one reduction step as a single DPP-modified VALU op: v = op(dpp(v), v) in the rows of
// RMASK (the others keep v); the s_nop 1 covers the VALU-write -> DPP-read hazard (2 wait
// states). LLVM does not fold its v_mov_b32_dpp into the add / max here, which costs a
// second VALU op per step. op is commutative (fp32 add, v_max_f32 of non-NaN values), so
// the results equal the mov + op form bit for bit.
#define MHF_DPP_STEP(OP, CTRL, RMASK) \
    "s_nop 1\n\t" OP "_dpp %0, %0, %0 " CTRL " row_mask:" RMASK " bank_mask:0xf\n\t"
// (one asm statement for the six steps: as six, LLVM pads each boundary with an s_nop of
// its own on top of the step's)
#define MHF_DPP_REDUCE(OP)                                       \
    asm(MHF_DPP_STEP(OP, "quad_perm:[1,0,3,2]", "0xf")           \
        MHF_DPP_STEP(OP, "quad_perm:[2,3,0,1]", "0xf")           \
        MHF_DPP_STEP(OP, "row_ror:4", "0xf")                     \
        MHF_DPP_STEP(OP, "row_ror:8", "0xf")                     \
        MHF_DPP_STEP(OP, "row_bcast:15", "0xa")                  \
        MHF_DPP_STEP(OP, "row_bcast:31", "0xc")                  \
        "s_nop 1" : "+v"(v))
__device__ __forceinline__ float wave_sum(float v) {
    MHF_DPP_REDUCE("v_add_f32");
    return readlane_f(v, 63);
}
// max of non-NaN floats over the wave (lane 63's value, as wave_sum); v_max_f32 in asm:
// fmaxf would first canonicalise both operands (LLVM cannot tell the powers are canonical)
__device__ __forceinline__ float max_f32(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float wave_max_f32(float v) {
    MHF_DPP_REDUCE("v_max_f32");
    return readlane_f(v, 63);
}
// smallest bin of a row among the lanes set in m (m != 0): lane = K mod 64 (transpose 2)
__device__ __forceinline__ int min_lanep(uint64_t m) { return __builtin_ctzll(m); }

template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = dpp_rows<CTRL, ROWS>(static_cast<int>(b));
    const int hi = dpp_rows<CTRL, ROWS>(static_cast<int>(b >> 32));
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
// (lane 63's result reads only rows the row_bcast steps write)
__device__ __forceinline__ double wave_max_key(double v) {
    v = kmax(v, dpp_d<0xb1>(v));
    v = kmax(v, dpp_d<0x4e>(v));
    v = kmax(v, dpp_d<0x124>(v));
    v = kmax(v, dpp_d<0x128>(v));
    v = kmax(v, dpp_d<0x142, 0xa>(v));
    v = kmax(v, dpp_d<0x143, 0xc>(v));
    return readlane_d(v, 63);
}

// Partner fetch: r = lane p's values of the 8 complex A_i (p = idx / 4) by 16
// ds_bpermute_b32, issued without a wait (inline asm: LLVM merged the .y permute of each
// pair into the .x one); lgkm_wait_tie then waits once for every window's permutes and
// carries their results through "+v", so nothing reads them before the s_waitcnt.
__device__ __forceinline__ void bperm_issue(int idx, const f2 (&A)[8], float (&r)[16]) {
    asm volatile(
        "ds_bpermute_b32 %0, %16, %17\n\t"
        "ds_bpermute_b32 %1, %16, %18\n\t"
        "ds_bpermute_b32 %2, %16, %19\n\t"
        "ds_bpermute_b32 %3, %16, %20\n\t"
        "ds_bpermute_b32 %4, %16, %21\n\t"
        "ds_bpermute_b32 %5, %16, %22\n\t"
        "ds_bpermute_b32 %6, %16, %23\n\t"
        "ds_bpermute_b32 %7, %16, %24\n\t"
        "ds_bpermute_b32 %8, %16, %25\n\t"
        "ds_bpermute_b32 %9, %16, %26\n\t"
        "ds_bpermute_b32 %10, %16, %27\n\t"
        "ds_bpermute_b32 %11, %16, %28\n\t"
        "ds_bpermute_b32 %12, %16, %29\n\t"
        "ds_bpermute_b32 %13, %16, %30\n\t"
        "ds_bpermute_b32 %14, %16, %31\n\t"
        "ds_bpermute_b32 %15, %16, %32"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
          "=&v"(r[7]), "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]),
          "=&v"(r[14]), "=&v"(r[15])
        : "v"(idx), "v"(A[0].x), "v"(A[0].y), "v"(A[1].x), "v"(A[1].y), "v"(A[2].x), "v"(A[2].y),
          "v"(A[3].x), "v"(A[3].y), "v"(A[4].x), "v"(A[4].y), "v"(A[5].x), "v"(A[5].y), "v"(A[6].x),
          "v"(A[6].y), "v"(A[7].x), "v"(A[7].y)
        : "memory");
}
// the first NB of the 8 pairs only (one ds_bpermute_b32 per float, issued back to back; the
// volatile asm statements keep their order), and the matching wait
template <int NB>
__device__ __forceinline__ void bperm_issue_n(int idx, const f2 (&A)[8], float (&r)[16]) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(r[2 * i]) : "v"(idx), "v"(A[i].x) : "memory");
        asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(r[2 * i + 1]) : "v"(idx), "v"(A[i].y) : "memory");
    }
}
template <int NB>
__device__ __forceinline__ void lgkm_wait_tie_n(float (&r)[16]) {
    if constexpr (NB == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]) : : "memory");
    else if constexpr (NB == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : : "memory");
    else if constexpr (NB == 3)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5])
                     :
                     : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),
                       "+v"(r[7])
                     :
                     : "memory");
}
// two windows' partial partner fetches (NR <= 4), one wait
template <int NR>
__device__ __forceinline__ void lgkm_wait_tie_n2(float (&r0)[16], float (&r1)[16]) {
    if constexpr (NR == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r0[0]), "+v"(r0[1]), "+v"(r1[0]), "+v"(r1[1]) : : "memory");
    else if constexpr (NR == 2)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(r0[0]), "+v"(r0[1]), "+v"(r0[2]), "+v"(r0[3]), "+v"(r1[0]), "+v"(r1[1]), "+v"(r1[2]),
                       "+v"(r1[3])
                     :
                     : "memory");
    else if constexpr (NR == 3)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(r0[0]), "+v"(r0[1]), "+v"(r0[2]), "+v"(r0[3]), "+v"(r0[4]), "+v"(r0[5]), "+v"(r1[0]),
                       "+v"(r1[1]), "+v"(r1[2]), "+v"(r1[3]), "+v"(r1[4]), "+v"(r1[5])
                     :
                     : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(r0[0]), "+v"(r0[1]), "+v"(r0[2]), "+v"(r0[3]), "+v"(r0[4]), "+v"(r0[5]), "+v"(r0[6]),
                       "+v"(r0[7]), "+v"(r1[0]), "+v"(r1[1]), "+v"(r1[2]), "+v"(r1[3]), "+v"(r1[4]), "+v"(r1[5]),
                       "+v"(r1[6]), "+v"(r1[7])
                     :
                     : "memory");
}
__device__ __forceinline__ void lgkm_wait_tie(float (&r)[1][16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r[0][0]), "+v"(r[0][1]), "+v"(r[0][2]), "+v"(r[0][3]), "+v"(r[0][4]), "+v"(r[0][5]),
                   "+v"(r[0][6]), "+v"(r[0][7]), "+v"(r[0][8]), "+v"(r[0][9]), "+v"(r[0][10]), "+v"(r[0][11]),
                   "+v"(r[0][12]), "+v"(r[0][13]), "+v"(r[0][14]), "+v"(r[0][15])
                 :
                 : "memory");
}

// the arg-max key of bin k with weighted power pw (w = +1 inside [dom_lo, dom_hi), -1
// outside): hi word = bits of pw, lo word = 0xffff - k; for pw >= 0 the f64 order is
// (power, then smaller k); a NaN's bits read as a large key (first NaN wins, numpy);
// outside bins are negative keys
__device__ __forceinline__ double amax_key(float pw, int k) {
    return __builtin_bit_cast(double, (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, pw)) << 32) |
                                          static_cast<uint64_t>(0xffffu - static_cast<uint32_t>(k)));
}

// Per-row classes (row d = bins 64 d .. 64 d + 63), kRowBits bits each in one uniform
// 64-bit word: the row is needed at all, wholly / partly inside the band, wholly / partly
// inside the arg-max range; above them the Nyquist bin's band / range membership.
constexpr int kRowBits = 5;
constexpr uint32_t kRowNeed = 1, kRowBandAll = 2, kRowBandPart = 4, kRowDomAll = 8, kRowDomPart = 16;
constexpr uint64_t kNyqBand = 1ull << (8 * kRowBits), kNyqDom = 2ull << (8 * kRowBits);
__host__ __device__ inline uint64_t row_classes(const SpecWaveArgs& a, bool want_dom, bool want_tot) {
    uint64_t rc = 0;
    const bool nyq_band = a.band_lo <= kN && a.band_hi >= kN;
    const bool nyq_dom = want_dom && a.dom_lo <= kN && a.dom_hi > kN;
    for (int d = 0; d < 8; ++d) {
        const int lo = 64 * d, hi = 64 * d + 63;
        const bool band = a.band_lo <= a.band_hi && a.band_lo <= hi && a.band_hi >= lo;
        const bool band_all = band && a.band_lo <= lo && a.band_hi >= hi;
        const bool dom = want_dom && a.dom_lo < a.dom_hi && a.dom_lo <= hi && a.dom_hi > lo;
        const bool dom_all = dom && a.dom_lo <= lo && a.dom_hi > hi;
        // row 0 also carries the Nyquist bin (lane 0's Z_0)
        const bool need = want_tot || band || dom || (d == 0 && (nyq_band || nyq_dom));
        const uint32_t rb = (need ? kRowNeed : 0) | (band_all ? kRowBandAll : 0) |
                            (band && !band_all ? kRowBandPart : 0) | (dom_all ? kRowDomAll : 0) |
                            (dom && !dom_all ? kRowDomPart : 0);
        rc |= static_cast<uint64_t>(rb) << (kRowBits * d);
    }
    return rc | (nyq_band ? kNyqBand : 0) | (nyq_dom ? kNyqDom : 0);
}

// NR < 8 (no total power, at most 4 rows): per-launch lane masks of the rows in place of the
// classes — bit lane set when the lane's bin 64 d + lane' of row d lies inside the band /
// the arg-max range, and the Nyquist bin's (lane 0) membership. Per row and window one
// v_cndmask each instead of 2-4 uniform branches; 4 SGPRs a row, held across the run.
template <int NR>
struct RowMasks {
    uint64_t band[NR < 8 ? NR : 1], dom[NR < 8 ? NR : 1];
    uint64_t nyq_band, nyq_dom;   // lane 0's bit, or 0
};
template <int NR>
__device__ __forceinline__ RowMasks<NR> row_masks(const SpecWaveArgs& a, int lanep, bool want_dom) {
    RowMasks<NR> m{};
    if constexpr (NR < 8) {
#pragma unroll
        for (int d = 0; d < NR; ++d) {
            const int K = lanep + 64 * d;
            m.band[d] = __ballot(K >= a.band_lo && K <= a.band_hi);
            m.dom[d] = want_dom ? __ballot(K >= a.dom_lo && K < a.dom_hi) : 0ull;
        }
        // (ballots, so that they are scalar values: a select of 1 / 0 lands in VGPRs)
        const int lane = __lane_id();
        m.nyq_band = __ballot(lane == 0 && a.band_lo <= kN && a.band_hi >= kN);
        m.nyq_dom = __ballot(lane == 0 && want_dom && a.dom_lo <= kN && a.dom_hi > kN);
    }
    return m;
}
// v_cndmask with a scalar lane mask: t where the lane's bit is set, f elsewhere
__device__ __forceinline__ float sel_mask(uint64_t m, float t, float f) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}

// one window's features, wave-uniform: band power (scaled), relative band power, spectral
// entropy (all computed in float, as stored) and the dominant bin (-1: none)
struct WinOut {
    float bp, rbp, ent;
    int bk;
};

// ---- the two transposes go through LDS. Register exchanges in their place (v_permlane
// swaps + DPP v_cndmask, one lane bit against one register bit at a time) were timed three
// ways on cfg5 (round 5, profiles/r05_bench_cfg5_*): both transposes 7.41 ms, both at 5
// waves per SIMD 7.20, transpose 1 only 6.58, against 6.21-6.46 for this LDS form — the
// kernel is VALU-issue-bound and each exchange costs more VALU than the LDS round trip.
// waves per SIMD of the ring kernels (MODE 2): LDS per wave = ring (+ the transpose buffer
// when a transpose goes through LDS); registers <= 512 / waves
#ifndef MHF_SPECREG_WAVES
#define MHF_SPECREG_WAVES 4
#endif

// The transform of NW windows at once: each stage runs window by window, so with NW = 2 one
// window's LDS round trips (transpose reads, partner permutes) would hide behind the other
// window's butterflies; the windows share the wave's transpose buffer T (LDS executes a
// wave's instructions in order, so window B's transpose writes land after window A's reads).
// Measured: window pairs in the ring loop (146-155 VGPRs, 6 windows in flight per SIMD)
// ran cfg5 in 7.79 ms against 7.68 single, so the kernels use NW = 1: the SIMD is issue-
// bound (VALU ~58 % busy, the rest SALU / LDS / DPP issue), not latency-bound.
//
// The window is transformed without removing its mean: centring (the constant detrend) moves
// only Z_0, i.e. the DC and Nyquist bins, and the DC bin is reported from the raw sum anyway
// (x0 below) while the Nyquist term Re - Im of Z_0 does not see it. Only rounding differs
// (band power within a few 1e-7 of fp64 for offsets up to 100 x the signal; the parity
// tests carry offset windows), and the mean's wave reduction and the 8 subtractions go.
template <int NW, int NR = 8>
__device__ __forceinline__ void fft_windows(f2 (&v)[NW][8], f2 (&B)[NW][8], f2* T, int lane, int kk, int bb,
                                            const f2 (&tw1)[7], const f2 (&tw2)[7], int partner) {
    // pass 1 + transpose 1 (T[k][l], row stride kT1)
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        dft8(v[w]);
#pragma unroll
        for (int k = 1; k < 8; ++k) v[w][k] = cmul(v[w][k], tw1[k - 1]);
#pragma unroll
        for (int k = 0; k < 8; ++k) T[k * kT1 + lane] = v[w][k];
#pragma unroll
        for (int a8 = 0; a8 < 8; ++a8) v[w][a8] = T[kk * kT1 + 8 * a8 + bb];
    }
    // pass 2 + transpose 2 (element (k, b, c) at 8 c + 66 b + k; lane = k + 8 c after it)
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        dft8(v[w]);
#pragma unroll
        for (int cc = 1; cc < 8; ++cc) v[w][cc] = cmul(v[w][cc], tw2[cc - 1]);
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) T[cc * kT2c + bb * kT2b + kk] = v[w][cc];
#pragma unroll
        for (int b8 = 0; b8 < 8; ++b8) v[w][b8] = T[lane + b8 * kT2b];
    }
    // pass 3: Z[k + 8c + 64d] = v[d]; the partners Z[512 - K] (register 7 - d of the
    // partner lane) by one permute per float
    // (NR < 8: only rows d < NR are read, so only their partners B[d] = register 7 - d)
    float r[NW][16];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        dft8(v[w]);
        const f2 src[8] = {v[w][7], v[w][6], v[w][5], v[w][4], v[w][3], v[w][2], v[w][1], v[w][0]};
        if constexpr (NR >= 5) bperm_issue(partner, src, r[w]);
        else bperm_issue_n<NR>(partner, src, r[w]);
    }
    if constexpr (NR >= 5) {
        static_assert(NW == 1, "full partner fetch: one window");
        lgkm_wait_tie(r);
    } else if constexpr (NW == 2) {
        lgkm_wait_tie_n2<NR>(r[0], r[1]);
    } else {
        lgkm_wait_tie_n<NR>(r[0]);
    }
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int i = 0; i < (NR >= 5 ? 8 : NR); ++i) B[w][i] = f2{r[w][2 * i], r[w][2 * i + 1]};
}

// one window's features from its spectrum (v = Z[k + 8c + 64d] in register d, B = the
// partner values); rows d >= NR are known unneeded at compile time (NR < 8: no total power)
template <int NR = 8>
__device__ __forceinline__ WinOut window_post(const SpecWaveArgs& a, const f2 (&v)[8], const f2 (&B)[8], int lane,
                                              int kk, int bb, f2 basep, bool want_dom, bool want_tot,
                                              uint64_t rowcls, const f2 (&twd)[4], const RowMasks<NR>& rm) {
    // lane 0 holds Z_0 = the window sum: a NaN / inf sample makes it non-finite and every
    // bin NaN / inf (uniform test)
    const bool finite = fabsf(readlane_f(v[0].x + v[0].y, 0)) <= 3.402823466e38f;

    // bin K of this lane: 2E = A + conj B, 2O = -i (A - conj B), 2X_K = 2E + w^K 2O
    // (spectral_lane.hip.inc); K = 0 gives bins 0 and 512. Powers in units of 2 / scale
    // (one-sided |2X|^2 / 2): the psd scale is applied once to the band sum (ratios,
    // entropy and the arg max do not depend on it). Rows d (bins 64 d + lane') that no
    // feature reads are skipped (row classes, uniform); rows wholly inside the band / arg-max
    // range take no per-bin test, the (at most two) boundary rows one compare.
    float pw[8], pny = 0.0f;
    float bp = 0.0f, tot = 0.0f;
    // the bin twiddles w1024^K and the bin numbers are rebuilt per window (2 + 1 VALU per
    // row) rather than hoisted by the compiler into 16 VGPRs and per-row lane masks (SGPR
    // spills): the kernel is at its 3-waves-per-SIMD register budget
    asm volatile("" : "+v"(basep));
    int lanep = lane;   // bin K = lane + 64 d (transpose 2)
    asm volatile("" : "+v"(lanep));
    // (likewise the row classes: one per-window SALU copy, so that the compiler does not
    // hoist 30-odd derived uniform values out of the window loop into spilled SGPRs)
    // (zero-extended low word: a sign-extended one would set every class bit of rows 6-7
    // whenever bit 31, row 6's kRowBandAll, is set)
    if constexpr (NR == 8) {
        rowcls = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(rowcls))) |
                 (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(rowcls >> 32)))) << 32);
        asm volatile("" : "+s"(rowcls));
    }
    float cand[8], cny = -1.0f, dmax = -1.0f;   // arg-max candidates (-1: outside the range)
    bool cnan = false;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        cand[d] = -1.0f;
        pw[d] = 0.0f;
        if (d >= NR) continue;
        const uint32_t rb = static_cast<uint32_t>(rowcls >> (kRowBits * d));
        if (NR == 8 && !(rb & kRowNeed)) continue;
        const f2 A = v[d];
        const f2 Bd = lane == 0 ? v[(8 - d) & 7] : B[d];   // lane 0: its own partners
        const f2 w16 = f2{kC16[d], kS16[d]};
        // NR < 8: at most 4 rows, their bin twiddles held across windows (8 VGPRs; the
        // kernel has the room at 3 waves per SIMD); all 8 rows: rebuilt per window
        f2 tw;
        if constexpr (NR < 8) tw = twd[d < 4 ? d : 0];
        else tw = cmul(basep, w16);
        const f2 E2 = add_conj(A, Bd);
        const f2 O2 = odd_pair(A, Bd);
        const f2 X2 = E2 + cmul(O2, tw);
        pw[d] = fmaf(X2.x, X2.x, X2.y * X2.y);
        if (d == 0 && lane == 0) {
            const float x0 = 2.0f * (A.x + A.y), xn = 2.0f * (A.x - A.y);
            pw[0] = (x0 * x0) * 0.5f;   // DC and Nyquist are not doubled
            pny = (xn * xn) * 0.5f;
        }
        if constexpr (NR < 8) {
            // (adding 0.0f outside the band leaves bp's bits as skipping the bin would:
            // bp >= +0 throughout)
            bp += sel_mask(rm.band[NR < 8 ? d : 0], pw[d], 0.0f);
            if (want_dom) {
                cand[d] = sel_mask(rm.dom[NR < 8 ? d : 0], pw[d], -1.0f);
                dmax = max_f32(dmax, cand[d]);
                cnan = cnan || (cand[d] != cand[d]);
            }
            continue;
        }
        if (rb & kRowBandAll) {
            bp += pw[d];
        } else if (rb & kRowBandPart) {
            const int blo = a.band_lo - 64 * d, bhi = a.band_hi - 64 * d;   // [blo, bhi] in lane'
            bp += (lanep >= blo && lanep <= bhi) ? pw[d] : 0.0f;
        }
        if (want_tot) tot += pw[d];
        if (want_dom) {
            // arg-max candidates: the bin's power inside [dom_lo, dom_hi), -1 outside
            if (rb & kRowDomAll) {
                cand[d] = pw[d];
            } else if (rb & kRowDomPart) {
                const int dlo = a.dom_lo - 64 * d, dhi = a.dom_hi - 64 * d;   // [dlo, dhi)
                cand[d] = (lanep >= dlo && lanep < dhi) ? pw[d] : -1.0f;
            }
            dmax = max_f32(dmax, cand[d]);
            cnan = cnan || (cand[d] != cand[d]);
        }
    }
    if constexpr (NR < 8) {
        // the Nyquist bin 512: pny is 0 outside lane 0, its masks lane 0's bit
        bp += sel_mask(rm.nyq_band, pny, 0.0f);
        if (want_dom) {
            cny = sel_mask(rm.nyq_dom, pny, -1.0f);
            dmax = max_f32(dmax, cny);
            cnan = cnan || (cny != cny);
        }
    } else if (lane == 0) {                // the Nyquist bin 512
        if (rowcls & kNyqBand) bp += pny;
        tot += pny;
        if (want_dom && (rowcls & kNyqDom)) {
            cny = pny;
            dmax = max_f32(dmax, pny);
            cnan = cnan || (pny != pny);
        }
    }
    bp = wave_sum(bp);
    if (want_tot) tot = wave_sum(tot);
    int bk = -1;
    if (want_dom) {
        // first arg max in bin order: the wave max of the candidates (v_max_f32 with DPP),
        // then the lowest bin holding it — rows in order, inside a row the smallest lane' of
        // the ballot (bin K = lane' + 64 d; the Nyquist bin 512 last). A NaN candidate
        // (overflowing samples) takes the f64-key path, where the first NaN wins as in numpy.
        if (NR < 8 && __ballot(cnan) == 0) {
            // the first row whose in-range candidates hold the max (the masks keep an empty
            // range's -1 candidates out), rows in order with an early exit: the max mostly
            // sits in row 0 (cfg5: a heart rate of 1-3 Hz is bin 4-12), where selects over
            // all rows cost 6 SALU a row
            const float wm = wave_max_f32(dmax);
            uint64_t m = 0;
            int dd = 0;
#pragma unroll
            for (int d = 0; d < NR; ++d) {
                m = __ballot(cand[d] == wm) & rm.dom[NR < 8 ? d : 0];
                if (m) {
                    dd = d;
                    break;
                }
            }
            if (m) bk = min_lanep(m) + 64 * dd;
            else if (rm.nyq_dom && readlane_f(cny, 0) == wm) bk = kN;
        } else if (NR == 8 && __ballot(cnan) == 0) {
            const float wm = wave_max_f32(dmax);
            bool found = false;
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                if (d >= NR || found) continue;
                const uint32_t rb = static_cast<uint32_t>(rowcls >> (kRowBits * d));
                if (!(rb & (kRowDomAll | kRowDomPart))) continue;
                const uint64_t m = __ballot(cand[d] == wm);
                if (m) { bk = min_lanep(m) + 64 * d; found = true; }
            }
            if (!found && (rowcls & kNyqDom) && readlane_f(cny, 0) == wm) bk = kN;
        } else {
            double key = -2.0;
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                if (d >= NR) continue;
                const uint32_t rb = static_cast<uint32_t>(rowcls >> (kRowBits * d));
                if (NR < 8 || (rb & (kRowDomAll | kRowDomPart)))   // (NR < 8: -1 outside the range)
                    key = kmax(key, amax_key(cand[d], lanep + 64 * d));
            }
            if (lane == 0 && (NR < 8 ? rm.nyq_dom != 0 : (rowcls & kNyqDom) != 0)) key = kmax(key, amax_key(cny, kN));
            const double kmx = wave_max_key(key);
            const uint64_t kb = __builtin_bit_cast(uint64_t, kmx);
            bk = (static_cast<int64_t>(kb) < 0) ? -1 : static_cast<int>(0xffffu - (kb & 0xffffu));
        }
    }
    if (!finite) {
        // every bin NaN (the FFT's negations scatter the NaN signs, so the keys cannot
        // decide): numpy's argmax over an all-NaN range is its first bin (as
        // spectral_lane.hip.inc does); sums over bins are NaN
        bk = a.dom_lo;
        if (a.band_lo <= a.band_hi) bp = __builtin_nanf("");
        tot = __builtin_nanf("");
    }
    float ent = 0.0f;
    if (want_tot && a.want_ent) {   // (want_tot: a compile-time false for FS 0, 1)
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
    return WinOut{bp * (0.5f * a.scale), bp / tot, ent, bk};
}

// Output staging: window t of a wave's sequence parks its (uniform) results in lane t % 64
// of four VGPRs (a v_cndmask each); every 64 windows, and at the end, the lanes store them together. A wave's
// only vector-memory traffic between flushes is its sample prefetch, so the wait for the
// next window's samples no longer also waits for the previous window's store acks.
struct OutStage {
    float bp = 0.0f, rbp = 0.0f, ent = 0.0f;
    int bk = 0;
    __device__ __forceinline__ void put(const WinOut& w, int slot, int lane, bool want_dom, bool want_tot,
                                        bool want_ent) {
        const bool me = lane == slot;
        bp = me ? w.bp : bp;
        if (want_tot) rbp = me ? w.rbp : rbp;
        if (want_ent) ent = me ? w.ent : ent;
        if (want_dom) bk = me ? w.bk : bk;
    }
    // lanes < cnt store window i0 + lane * istep
    __device__ __forceinline__ void flush(const SpecWaveArgs& a, int c, int64_t i0, int64_t istep, int cnt,
                                          int lane) const {
        if (lane >= cnt) return;
        const int64_t i = i0 + lane * istep;
        for (int jf = 0; jf < a.feats.n; ++jf) {
            const int f = a.feats.id[jf];
            double val;
            if (f == MHF_BAND_POWER) val = bp;
            else if (f == MHF_REL_BAND_POWER) val = rbp;
            else if (f == MHF_SPECTRAL_ENTROPY) val = ent;
            else if (f == MHF_DOMINANT_FREQ) val = (bk < 0) ? NAN : static_cast<double>(bk) * a.freq_step;
            else continue;
            store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + jf) * a.out_ld + i, val);
        }
    }
};

// Sample supply, three modes:
//  MODE 0: VGPR prefetch (any layout): the next window's samples load into 16 VGPRs during
//          this window's FFT; the block's waves take windows i, i + 4, ... of a block run.
//  MODE 1: private LDS-DMA (contiguous, 16-B aligned windows): the next window lands by
//          global_load_lds_dwordx4 in the wave's 4-KiB buffer (nothing held in VGPRs, 168
//          VGPRs: 3 waves per SIMD); same window order as MODE 0. Overlapping windows fetch
//          each sample W / S times (through L2: cfg5 FETCH 1.87x the distinct input).
//  MODE 2: per-wave sample ring (contiguous, 16-B aligned, S < W): each wave owns a
//          contiguous window run and a ring of RS >= W + S samples in LDS; while window j is
//          transformed, the S samples window j + 1 adds are DMA'd into the ring positions only
//          window j - 1 used. Every input sample crosses HBM -> LDS once; no block barriers.
// FS >= 0: the requested feature set fixed at compile time (bit 0 dominant frequency, bit 1
// total power), so the per-bin loop carries no uniform branches; FS = -1: from the args.
__host__ __device__ inline int spec_reg_fs(const SpecWaveArgs& a) {
    bool tot = a.want_ent != 0;
    for (int jf = 0; jf < a.feats.n; ++jf) tot |= a.feats.id[jf] == MHF_REL_BAND_POWER;
    return (a.dom_lo < a.dom_hi ? 1 : 0) | (tot ? 2 : 0);
}

// MODE 2 ring: length RS (a multiple of S, >= W + S); sample s of the wave's run sits at
// (s + phi) mod RS, phi chosen so that every per-window chunk [jS + W, jS + W + S) starts at
// a multiple of S and never crosses the ring end. Positions below MX are mirrored at
// RS + position, so a window [p0, p0 + W) reads straight through the ring end: no wrap
// arithmetic in the read addresses (one more DMA per mirrored chunk).
#ifndef MHF_RING_MIRROR
#define MHF_RING_MIRROR 0
#endif
struct RingGeom {
    int32_t RS, phi, MX;
    __host__ __device__ int32_t len() const { return RS + MX; }
};
__host__ __device__ inline RingGeom ring_geom(int64_t S) {
    RingGeom g;
    g.RS = static_cast<int32_t>(((kW + S + S - 1) / S) * S);
    g.phi = static_cast<int32_t>((S - kW % S) % S);
    // window starts are = phi (mod S) and at most RS - S + phi: reads pass the ring end by
    // at most W - S + phi samples. MHF_RING_MIRROR = 0: no mirror (the reads wrap), so the
    // ring is RS samples and MODE 2 runs 4 waves per SIMD instead of 3
    g.MX = MHF_RING_MIRROR ? static_cast<int32_t>(((kW - S + g.phi + S - 1) / S) * S) : 0;
    return g;
}
constexpr int kRingMaxSamples = 2048;   // per wave (8 KiB; 4 waves + transposes: 50 KiB per block)

template <bool CONTIG, int MODE, int FS, int NR = 8, int NWR = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    (MODE == 2 && MHF_RING_MIRROR) || !CONTIG ? 3 : MODE == 2 ? MHF_SPECREG_WAVES : 4,
    (MODE == 2 && MHF_RING_MIRROR) || !CONTIG ? 3 : MODE == 2 ? MHF_SPECREG_WAVES : 4)))
spectral_reg_kernel(SpecWaveArgs a) {
    __shared__ __attribute__((aligned(16))) f2 lds[4][kBufCf];
    __shared__ __attribute__((aligned(16))) float winbuf[MODE == 1 ? 4 : 1][MODE == 1 ? kW : 4];
    extern __shared__ __attribute__((aligned(16))) float ring_lds[];
    // the wave index as a scalar: the compiler cannot tell threadIdx.x >> 6 is wave-uniform,
    // and a per-lane wid makes MODE 2's window run (r0, r1, the sample pointers) per-lane
    // values — 64-bit VALU pointer arithmetic and exec-masked loop control per window
    const int wid = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    f2* T = lds[wid];
    const int c = blockIdx.y;
    const int kk = lane >> 3, bb = lane & 7;   // lane = 8 k + b after transpose 1, 8 k + c after 2

    // per-lane twiddles (fp64-accurate, held in 28 VGPRs across windows): pass 1 w512^(lane k),
    // pass 2 w64^(b c), and the bin twiddle base w1024^(k + 8c) of this lane's bins
    // K = k + 8c + 64d (times w16^d)
    f2 tw1[7], tw2[7];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        tw1[k - 1] = twiddle(lane * k, kN);
        tw2[k - 1] = twiddle(bb * k, 64);
    }
    const f2 basep = twiddle(lane, kW);
    // bin twiddles w1024^(lane' + 64 d) of rows d < 4 (window_post, NR < 8), formed exactly
    // as the all-rows kernel forms them per window (so every row-count variant agrees with
    // it bit for bit)
    f2 twd[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) twd[d] = cmul(basep, f2{kC16[d], kS16[d]});
    // the partner of bin K = lane + 64 d is 512 - K: lane 64 - lane, register 7 - d; lane 0
    // holds its own partners (K = 64 d <-> 64 (8 - d))
    const int partner = (lane == 0 ? 0 : 64 - lane) * 4;
    const bool want_dom = FS >= 0 ? (FS & 1) != 0 : spec_reg_fs(a) & 1;
    const bool want_tot = FS >= 0 ? (FS & 2) != 0 : (spec_reg_fs(a) & 2) != 0;
    const bool want_ent = want_tot && a.want_ent != 0;
    const uint64_t rowcls = row_classes(a, want_dom, want_tot);
    const RowMasks<NR> rm = row_masks<NR>(a, lane, want_dom);
    OutStage st;

    if constexpr (MODE == 2) {
        const int64_t S = a.wstep;
        const RingGeom rg = ring_geom(S);
        const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
        const int64_t per = (a.nwin + nwaves - 1) / nwaves;
        const int64_t r0 = (static_cast<int64_t>(blockIdx.x) * 4 + wid) * per;
        const int64_t r1 = r0 + per < a.nwin ? r0 + per : a.nwin;
        if (r0 >= r1) return;                      // no block barriers in this mode
        float* R = ring_lds + wid * rg.len();
        const float* run = a.x + c * a.ch_stride + (a.first + r0) * S;
        // DMA of run samples [s0, s0 + len) to ring position pos (no wrap), 256 per instruction
        auto fill = [&](int64_t s0, int len, int32_t pos) {
            for (int q = 0; q < len; q += 256)
                if (q + 4 * lane < len)
                    __builtin_amdgcn_global_load_lds(
                        const_cast<float*>(run + s0 + q + 4 * lane),
                        (__attribute__((address_space(3))) void*)(&R[pos + q]), 16, 0, 0);
        };
        fill(0, kW, rg.phi);
        if (rg.MX > rg.phi) fill(0, rg.MX - rg.phi < kW ? rg.MX - rg.phi : kW, rg.phi + rg.RS);
        int32_t pw0 = rg.phi;                                  // window j's first sample
        int32_t pch = (kW + rg.phi) % rg.RS;                   // chunk j + 1's position
        const int64_t n = r1 - r0;
        // S and phi multiples of 128 (cfg5: S = 128, phi = 0): the ring end falls between
        // rows of 128 samples, so a row's wrap is uniform and its base a scalar
        const bool rowal = !MHF_RING_MIRROR && S % 128 == 0 && rg.phi % 128 == 0;
        if constexpr (NWR == 2) {
            // windows in pairs (j, j + 1): both read from the ring (it holds exactly their W + S
            // samples), then the two chunks windows j + 2, j + 3 add are DMA'd over the first
            // chunks of j and j + 1, and the two transforms run stage by stage together (one
            // window's LDS round trips behind the other's butterflies)
            const uint32_t Rl = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                                    (__attribute__((address_space(3))) float*)(R))) + 8u * lane;
            // a chunk of S (a multiple of 128) samples: whole 256-sample DMAs, then half of
            // one (lanes 0-31) when S = 128 mod 256 — no per-instruction lane test
            // (cp: the next chunk's first sample, advanced by S per chunk — no 64-bit
            // multiply per fill; 32-bit counts: SALU has no 64-bit ordered compare)
            // S <= 256 (cfg5: 128): one DMA by lanes 0-31 / all, no loop.
            // one_dma as a scalar (readfirstlane): a plain bool is hoisted into a VGPR and
            // tested per chunk through exec
            const int32_t S32 = static_cast<int32_t>(S);
            const int one_dma = __builtin_amdgcn_readfirstlane(S32 <= 256 ? 1 : 0);
            // The one DMA is inline asm: as a builtin LLVM merges it with the loop form's
            // tail into one exec-phi block (17 SALU per chunk). M0 = the ring slot's LDS
            // byte address, saddr form; s_nop 4 covers SALU M0 -> LDS-DMA and any VALU-written
            // SGPR base -> VMEM (tile.hip.h dma_chunk). The explicit s_waitcnt vmcnt(0) at
            // the pair's head is the only wait the ring needs.
            const bool dl = 4 * lane < S32;
            const uint32_t voff = 16u * static_cast<uint32_t>(lane);
            const uint32_t Rb = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                (__attribute__((address_space(3))) float*)(R)));
            const float* cp = run + kW;
            auto fill_chunk = [&](int32_t pos) {
                if (one_dma) {
                    if (dl)
                        asm volatile("s_nop 4\n\tglobal_load_lds_dwordx4 %1, %2"
                                     :
                                     : "{m0}"(Rb + 4u * static_cast<uint32_t>(pos)), "v"(voff),
                                       "s"(reinterpret_cast<uint64_t>(cp))
                                     : "memory");
                } else {
                    int32_t q = 0;
#pragma nounroll
                    for (; q + 256 <= S32; q += 256)
                        __builtin_amdgcn_global_load_lds(
                            const_cast<float*>(cp + q + 4 * lane),
                            (__attribute__((address_space(3))) void*)(&R[pos + q]), 16, 0, 0);
                    if (q < S32 && lane < 32)
                        __builtin_amdgcn_global_load_lds(
                            const_cast<float*>(cp + q + 4 * lane),
                            (__attribute__((address_space(3))) void*)(&R[pos + q]), 16, 0, 0);
                }
                cp += S32;
            };
            if (n > 1) {   // window 1's new chunk, before the first pair
                fill_chunk(pch);
                pch += static_cast<int32_t>(S);
                pch = pch == rg.RS ? 0 : pch;
            }
            // (32-bit window counts: a wave's run is far below 2^31 windows, and 64-bit
            // ordered compares are VALU instructions)
            const int32_t n32 = static_cast<int32_t>(n);
            int32_t j = 0;
            for (; j + 1 < n32; j += 2) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                f2 v[2][8], B[2][8];
                if (S32 == 128) {
                    // S = 128 (cfg5): window j + 1's rows are window j's rows 1-8, so 9 row
                    // bases serve both windows (the selects as below)
                    const uint32_t b0 = 4u * static_cast<uint32_t>(pw0);
                    uint32_t b1 = b0 - 4u * static_cast<uint32_t>(rg.RS);
                    asm("" : "+s"(b1));
                    const int32_t rw = rg.RS - pw0;
                    uint32_t base[9];
#pragma unroll
                    for (int t = 0; t < 9; ++t) base[t] = Rl + (rw > 128 * t ? b0 : b1);
#pragma unroll
                    for (int w = 0; w < 2; ++w)
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            // (volatile: window j + 1's rows are read again, not copied from
                            // window j's before its transform overwrites them — 7 VALU moves
                            // behind a mid-block LDS wait)
                            const uint64_t u = *reinterpret_cast<const volatile __attribute__((address_space(3))) uint64_t*>(
                                static_cast<uintptr_t>(base[r + w] + 512u * (r + w)));
                            v[w][r] = f2{__builtin_bit_cast(float, static_cast<uint32_t>(u)),
                                         __builtin_bit_cast(float, static_cast<uint32_t>(u >> 32))};
                        }
                } else {
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    int32_t p0 = pw0 + static_cast<int32_t>(w * S);
                    p0 = p0 >= rg.RS ? p0 - rg.RS : p0;
                    // row r at ring byte 4 p0 + 512 r, less 4 RS past the ring end: one scalar
                    // compare + select of the row's base per row (the 512 r rides in the
                    // read's offset field). b1 is made opaque: knowing b1 = b0 - 4 RS, the
                    // compiler rewrites the select as b0 - (wrap ? 4 RS : 0) and recomputes
                    // p0 + 128 r, 4 SALU per row.
                    const uint32_t b0 = 4u * static_cast<uint32_t>(p0);
                    uint32_t b1 = b0 - 4u * static_cast<uint32_t>(rg.RS);
                    asm("" : "+s"(b1));
                    const int32_t rw = rg.RS - p0;   // samples before the ring end
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const uint32_t bs = rw > 128 * r ? b0 : b1;
                        v[w][r] = *reinterpret_cast<const __attribute__((address_space(3))) f2*>(
                            static_cast<uintptr_t>(Rl + bs + 512u * r));
                    }
                }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (S32 == 128 && j + 3 < n32 && pch + 128 < rg.RS) {
                    // both chunks (256 consecutive samples) into consecutive ring rows: one DMA
                    asm volatile("s_nop 4\n\tglobal_load_lds_dwordx4 %1, %2"
                                 :
                                 : "{m0}"(Rb + 4u * static_cast<uint32_t>(pch)), "v"(voff),
                                   "s"(reinterpret_cast<uint64_t>(cp))
                                 : "memory");
                    cp += 256;
                    pch += 256;
                    pch = pch == rg.RS ? 0 : pch;
                } else {
#pragma unroll
                    for (int w = 0; w < 2; ++w) {
                        if (j + 2 + w < n32) {
                            fill_chunk(pch);   // window j + 2 + w's chunk
                            pch += static_cast<int32_t>(S);
                            pch = pch == rg.RS ? 0 : pch;
                        }
                    }
                }
                pw0 += static_cast<int32_t>(2 * S);
                pw0 = pw0 >= rg.RS ? pw0 - rg.RS : pw0;
                fft_windows<2, NR>(v, B, T, lane, kk, bb, tw1, tw2, partner);
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const WinOut wo = window_post<NR>(a, v[w], B[w], lane, kk, bb, basep, want_dom, want_tot,
                                                      rowcls, twd, rm);
                    const int slot = (j + w) & 63;
                    st.put(wo, slot, lane, want_dom, want_tot, want_ent);
                    if (slot == 63 || j + w + 1 == n32) st.flush(a, c, r0 + j + w - slot, 1, slot + 1, lane);
                }
            }
            if (j < n32) {   // an odd last window: its samples are in, no refill
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                f2 v[1][8], B[1][8];
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    int32_t rb = pw0 + 128 * r;
                    rb = rb >= rg.RS ? rb - rg.RS : rb;
                    const uint32_t off = __builtin_amdgcn_readfirstlane(4 * rb);
                    v[0][r] = *reinterpret_cast<const __attribute__((address_space(3))) f2*>(
                        static_cast<uintptr_t>(Rl + off));
                }
                fft_windows<1, NR>(v, B, T, lane, kk, bb, tw1, tw2, partner);
                const WinOut wo = window_post<NR>(a, v[0], B[0], lane, kk, bb, basep, want_dom, want_tot, rowcls, twd, rm);
                const int slot = static_cast<int>(j & 63);
                st.put(wo, slot, lane, want_dom, want_tot, want_ent);
                st.flush(a, c, r0 + j - slot, 1, slot + 1, lane);
            }
            return;
        }
        for (int64_t j = 0; j < n; ++j) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // window j's samples are in
            if (j + 1 < n) {
                fill(j * S + kW, static_cast<int>(S), pch);
                if (pch < rg.MX) fill(j * S + kW, static_cast<int>(S), pch + rg.RS);
                pch += static_cast<int32_t>(S);
                pch = pch == rg.RS ? 0 : pch;
            }
            f2 v[1][8], B[1][8];
            if (rowal) {
                // one v_add per row: the row's byte offset is formed in SGPRs
                // LDS byte address from an address_space(3) pointer (not by truncating the
                // generic pointer, which would rely on the shared aperture's low bits)
                const uint32_t Rl = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                                        (__attribute__((address_space(3))) float*)(R))) + 8u * lane;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    int32_t rb = pw0 + 128 * r;
                    rb = rb >= rg.RS ? rb - rg.RS : rb;
                    const uint32_t off = __builtin_amdgcn_readfirstlane(4 * rb);
                    v[0][r] = *reinterpret_cast<const __attribute__((address_space(3))) f2*>(
                        static_cast<uintptr_t>(Rl + off));
                }
            } else {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    uint32_t pos = static_cast<uint32_t>(pw0 + 2 * (lane + 64 * r));
                    if constexpr (!MHF_RING_MIRROR) {
                        // wrap at the ring end: pos - RS underflows (huge) unless pos >= RS
                        const uint32_t wr = pos - static_cast<uint32_t>(rg.RS);
                        pos = pos < wr ? pos : wr;
                    }
                    v[0][r] = *reinterpret_cast<const f2*>(&R[pos]);
                }
            }
            pw0 += static_cast<int32_t>(S);
            pw0 = pw0 >= rg.RS ? pw0 - rg.RS : pw0;
            fft_windows<1, NR>(v, B, T, lane, kk, bb, tw1, tw2, partner);
            const WinOut w = window_post<NR>(a, v[0], B[0], lane, kk, bb, basep, want_dom, want_tot, rowcls, twd, rm);
            const int slot = static_cast<int>(j & 63);
            st.put(w, slot, lane, want_dom, want_tot, want_ent);
            if (slot == 63 || j + 1 == n) st.flush(a, c, r0 + j - slot, 1, slot + 1, lane);
        }
        return;
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
    f2 nxt[MODE == 1 ? 1 : 8];
    if (w_begin + wid < w_end) {
        if constexpr (MODE == 1) dma(w_begin + wid);
        else load(w_begin + wid, nxt);
    }
    int slot = 0;
    for (int64_t i = w_begin + wid; i < w_end; i += 4) {
        f2 v[8];
        if constexpr (MODE == 1) {
            // window i has landed (the only vector-memory ops in flight are its DMA and, once
            // per 64 windows, the staged stores); read it, then refill the buffer with window
            // i + 4 once the reads have returned
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
        f2 vv[1][8], B[1][8];
#pragma unroll
        for (int r = 0; r < 8; ++r) vv[0][r] = v[r];
        fft_windows<1, NR>(vv, B, T, lane, kk, bb, tw1, tw2, partner);
        const WinOut w = window_post<NR>(a, vv[0], B[0], lane, kk, bb, basep, want_dom, want_tot, rowcls, twd, rm);
        st.put(w, slot, lane, want_dom, want_tot, want_ent);
        if (slot == 63 || i + 4 >= w_end) {
            st.flush(a, c, i - 4 * slot, 4, slot + 1, lane);
            slot = 0;
        } else {
            ++slot;
        }
    }
}

// diagnostic switches (A/B on the box without a rebuild)
int getenv_int(const char* name) {
    const char* e = diag_env(name);
    return (e && *e) ? atoi(e) : 0;
}

}  // namespace

bool spectral_reg_ok(int64_t wsize) { return wsize == kW; }

int launch_spectral_reg(const SpecWaveArgs& a, int channels, hipStream_t stream) {
    // persistent: one resident round (blocks of 4 waves; per CU 4 blocks, <= 128 VGPRs;
    // 3 for MODE 2, its 50 KiB of LDS per block, and strided MODE 0, 168 VGPRs);
    // MODE 0/1: each block a contiguous window run, MODE 2: each wave one.
    // DMA modes: contiguous samples, every window start 16-B aligned
    bool dma = a.sample_stride == 1 && a.wstep % 4 == 0 && getenv_int("MHF_SPECREG_NODMA") == 0;
    for (int c = 0; c < channels && dma; ++c)
        dma = reinterpret_cast<uintptr_t>(a.x + c * a.ch_stride + a.first * a.wstep) % 16 == 0;
    const bool ring = dma && a.wstep < kW && ring_geom(a.wstep).len() <= kRingMaxSamples &&
                      getenv_int("MHF_SPECREG_NORING") == 0;
    int64_t blocks = (a.nwin + 15) / 16;
    int64_t bpc = (ring && MHF_RING_MIRROR) || a.sample_stride != 1 ? 3 : 4;   // blocks per CU
    if (ring) bpc = MHF_SPECREG_WAVES;
    if (ring) {   // as many ring blocks as fit the CU's 160 KiB of LDS (S = 128: 4)
        const int64_t blk = 4 * kBufCf * static_cast<int64_t>(sizeof(f2)) +
                            16 * static_cast<int64_t>(ring_geom(a.wstep).len()) + 64;
        const int64_t fit = (160 * 1024) / blk;
        if (fit < bpc) bpc = fit < 1 ? 1 : fit;
    }
    const int64_t cap = 256 * bpc / (channels > 0 ? channels : 1);
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const dim3 grid(static_cast<unsigned>(blocks), static_cast<unsigned>(channels));
    const int fs = spec_reg_fs(a);
    // rows needed (no total power): the highest row any band / arg-max bin sits in
    int nr = 8;
    if (!(fs & 2) && getenv_int("MHF_SPECREG_ALLROWS") == 0) {
        const uint64_t rc = row_classes(a, (fs & 1) != 0, false);
        nr = 1;
        for (int d = 0; d < 8; ++d)
            if ((rc >> (kRowBits * d)) & kRowNeed) nr = d + 1;
        if (nr > 4) nr = 8;
    }
    if (ring || dma) {
        const size_t shm = ring ? 4 * static_cast<size_t>(ring_geom(a.wstep).len()) * sizeof(float) : 0;
        auto go = [&](auto mode_c) {
            constexpr int M = decltype(mode_c)::value;
            switch (fs * 16 + nr) {
            case 0 * 16 + 1: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 0, 1>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 2: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 0, 2>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 3: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 0, 3>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 4: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 0, 4>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 8: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 0>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 1: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 1, 1>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 2: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 1, 2>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 3: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 1, 3>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 4: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 1, 4>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 8: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 1>), grid, dim3(256), shm, stream, a); break;
            case 2 * 16 + 8: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 2>), grid, dim3(256), shm, stream, a); break;
            default: hipLaunchKernelGGL((spectral_reg_kernel<true, M, 3>), grid, dim3(256), shm, stream, a); break;
            }
        };
        // ring mode two windows per wave iteration where the rows are uniform (S, phi
        // multiples of 128) and the partner fetch partial (nr <= 4): cfg5 6.27-6.36 ->
        // 6.18-6.19 ms A/B on one box. Diagnostic: MHF_SPECREG_NW2=0 keeps one window per
        // iteration.
        const RingGeom rg = ring_geom(a.wstep);
        const char* nw2_env = diag_env("MHF_SPECREG_NW2");
        const bool nw2_off = nw2_env && nw2_env[0] == '0';
        const bool nw2 = ring && !nw2_off && a.wstep % 128 == 0 &&
                         rg.phi % 128 == 0 && !MHF_RING_MIRROR && nr <= 4 && fs <= 1;
        if (nw2) {
            switch (fs * 16 + nr) {
            case 0 * 16 + 1: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 0, 1, 2>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 2: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 0, 2, 2>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 3: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 0, 3, 2>), grid, dim3(256), shm, stream, a); break;
            case 0 * 16 + 4: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 0, 4, 2>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 1: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 1, 1, 2>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 2: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 1, 2, 2>), grid, dim3(256), shm, stream, a); break;
            case 1 * 16 + 3: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 1, 3, 2>), grid, dim3(256), shm, stream, a); break;
            default: hipLaunchKernelGGL((spectral_reg_kernel<true, 2, 1, 4, 2>), grid, dim3(256), shm, stream, a); break;
            }
        } else if (ring) {
            go(std::integral_constant<int, 2>{});
        } else {
            go(std::integral_constant<int, 1>{});
        }
    } else if (a.sample_stride == 1) {
        hipLaunchKernelGGL((spectral_reg_kernel<true, 0, -1>), grid, dim3(256), 0, stream, a);
    } else {
        hipLaunchKernelGGL((spectral_reg_kernel<false, 0, -1>), grid, dim3(256), 0, stream, a);
    }
    return MHF_OK;
}

}  // namespace mhf
