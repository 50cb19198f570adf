// lane_xchg.h — register transposes without LDS: exchange of one lane bit with one register
// bit over 8 complex (float2) registers, the building block of spectral_reg.hip's two
// in-register transposes (tools/xchg_probe.hip checks every (lane bit, register bit) pair
// on the GPU against the index map).
//
// xchg<L, J>(v): for registers r and r' = r | 2^J, a lane whose bit L is set takes r from the
// partner lane (lane ^ 2^L)'s r' and keeps r'; a lane whose bit L is clear keeps r and takes
// r' from the partner's r. In element terms E'(lane, reg) = E(lane with bit L := reg bit J,
// reg with bit J := lane bit L).
//   * L = 5 / 4: v_permlane32_swap / v_permlane16_swap (gfx950): one instruction moves both
//     halves of a float pair;
//   * L = 3 .. 0: v_cndmask_b32 with a DPP source (row_ror:8, row_ror:4 / :12, quad_perm)
//     selecting the partner's value where VCC is clear: one instruction per float, no copies.
//     Every DPP source lane is valid (rotations / quad permutes), so no lane is left
//     unwritten.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mhf {

typedef float xf2 __attribute__((ext_vector_type(2)));

// four float pairs (a[i], b[i]): a[i] <- bit ? b[i] @ partner : a[i] (DPP control DA: reads
// lane ^ 2^L for the lanes with the bit set), b[i] <- bit ? b[i] : a[i] @ partner (DB: for the
// lanes with the bit clear). v_cndmask_b32 dst = VCC ? src1 : src0 with the DPP on src0.
// s_nop 1: a DPP source written by the VALU instruction just before needs two wait states.
#define MHF_XCND(DA, DB)                                                                      \
    "s_nop 1\n\t"                                                                             \
    "s_mov_b64 vcc, %16\n\t"                                                                  \
    "v_cndmask_b32_dpp %0, %12, %8, vcc " DA " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_cndmask_b32_dpp %1, %13, %9, vcc " DA " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_cndmask_b32_dpp %2, %14, %10, vcc " DA " row_mask:0xf bank_mask:0xf\n\t"               \
    "v_cndmask_b32_dpp %3, %15, %11, vcc " DA " row_mask:0xf bank_mask:0xf\n\t"               \
    "s_mov_b64 vcc, %17\n\t"                                                                  \
    "v_cndmask_b32_dpp %4, %8, %12, vcc " DB " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_cndmask_b32_dpp %5, %9, %13, vcc " DB " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_cndmask_b32_dpp %6, %10, %14, vcc " DB " row_mask:0xf bank_mask:0xf\n\t"               \
    "v_cndmask_b32_dpp %7, %11, %15, vcc " DB " row_mask:0xf bank_mask:0xf"
#define MHF_XCND_OPS                                                                          \
    : "=&v"(na[0]), "=&v"(na[1]), "=&v"(na[2]), "=&v"(na[3]), "=&v"(nb[0]), "=&v"(nb[1]),     \
      "=&v"(nb[2]), "=&v"(nb[3])                                                              \
    : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), \
      "s"(clr), "s"(set)                                                                      \
    : "vcc"

template <int L>
__device__ __forceinline__ void xcnd4(float (&a)[4], float (&b)[4]) {
    constexpr uint64_t set = L == 0 ? 0xaaaaaaaaaaaaaaaaull
                           : L == 1 ? 0xccccccccccccccccull
                           : L == 2 ? 0xf0f0f0f0f0f0f0f0ull
                                    : 0xff00ff00ff00ff00ull;
    const uint64_t clr = ~set;
    float na[4], nb[4];
    // row_ror:n: lane i of a row reads lane (i - n) mod 16
    if constexpr (L == 0)
        asm volatile(MHF_XCND("quad_perm:[1,0,3,2]", "quad_perm:[1,0,3,2]") MHF_XCND_OPS);
    else if constexpr (L == 1)
        asm volatile(MHF_XCND("quad_perm:[2,3,0,1]", "quad_perm:[2,3,0,1]") MHF_XCND_OPS);
    else if constexpr (L == 2)
        asm volatile(MHF_XCND("row_ror:4", "row_ror:12") MHF_XCND_OPS);
    else
        asm volatile(MHF_XCND("row_ror:8", "row_ror:8") MHF_XCND_OPS);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = na[i];
        b[i] = nb[i];
    }
}
#undef MHF_XCND
#undef MHF_XCND_OPS

template <int L, int J>
__device__ __forceinline__ void xchg(xf2 (&v)[8]) {
    static_assert(L >= 0 && L < 6 && J >= 0 && J < 3, "lane bit 0..5, register bit 0..2");
    constexpr int m = 1 << J;
    int pr[4], q = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r)
        if (!(r & m)) pr[q++] = r;
    if constexpr (L >= 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = pr[i];
            const auto sx = L == 5 ? __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v[r].x),
                                                                     __builtin_bit_cast(uint32_t, v[r | m].x),
                                                                     false, false)
                                   : __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[r].x),
                                                                     __builtin_bit_cast(uint32_t, v[r | m].x),
                                                                     false, false);
            const auto sy = L == 5 ? __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v[r].y),
                                                                     __builtin_bit_cast(uint32_t, v[r | m].y),
                                                                     false, false)
                                   : __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[r].y),
                                                                     __builtin_bit_cast(uint32_t, v[r | m].y),
                                                                     false, false);
            v[r] = xf2{__builtin_bit_cast(float, static_cast<uint32_t>(sx[0])),
                       __builtin_bit_cast(float, static_cast<uint32_t>(sy[0]))};
            v[r | m] = xf2{__builtin_bit_cast(float, static_cast<uint32_t>(sx[1])),
                           __builtin_bit_cast(float, static_cast<uint32_t>(sy[1]))};
        }
    } else {
#pragma unroll
        for (int g = 0; g < 2; ++g) {   // register pairs 2g, 2g + 1: four float pairs per block
            const int r0 = pr[2 * g], r1 = pr[2 * g + 1];
            float a[4] = {v[r0].x, v[r0].y, v[r1].x, v[r1].y};
            float b[4] = {v[r0 | m].x, v[r0 | m].y, v[r1 | m].x, v[r1 | m].y};
            xcnd4<L>(a, b);
            v[r0] = xf2{a[0], a[1]};
            v[r1] = xf2{a[2], a[3]};
            v[r0 | m] = xf2{b[0], b[1]};
            v[r1 | m] = xf2{b[2], b[3]};
        }
    }
    // each register pair as one opaque 64-bit value: LLVM would otherwise split the packed
    // arithmetic that follows into scalar halves (its operands being built from 32-bit parts)
#pragma unroll
    for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(v[r]));
}

}  // namespace mhf
