// valu_probe.hip — measures VALU issue cost per instruction on gfx950 at 1, 2 and 4 waves
// per SIMD, for the instruction mix of the window kernels (f32 add/mul, packed f32, f64
// add/mul, f32->f64 convert). Cycles come from s_memtime (shader clock) per wave.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kIters = 2000;

template <int OP>
__global__ void probe(float* out, unsigned long long* cyc) {
    extern __shared__ float lds[];
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = 1.0001f;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, db = 1.0000001;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, pb = {b, b};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OP == 0) {  // 16 x v_add_f32, 8 chains
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                    "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        } else if constexpr (OP == 1) {  // 16 x v_pk_add_f32, 4 chains
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                             : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));
        } else if constexpr (OP == 2) {  // 16 x v_add_f64, 4 chains
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4\n"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(db));
        } else if constexpr (OP == 3) {  // 16 x v_cvt_f64_f32
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %6\n v_cvt_f64_f32 %3, %7\n"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
        } else if constexpr (OP == 4) {  // 16 x v_mul_f64
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4\n"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(db));
        } else if constexpr (OP == 5) {  // 16 x v_pk_mul_f32
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n"
                             : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));
        } else if constexpr (OP == 6) {  // 16 x v_cndmask_b32 (vcc)
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                    "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        } else if constexpr (OP == 7) {  // 16 x v_log_f32
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_log_f32 %0, %0\n v_log_f32 %1, %1\n v_log_f32 %2, %2\n v_log_f32 %3, %3\n"
                    "v_log_f32 %4, %4\n v_log_f32 %5, %5\n v_log_f32 %6, %6\n v_log_f32 %7, %7\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if constexpr (OP == 8) {  // 16 x v_pk_fma_f32, 4 chains
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4\n"
                             : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));
        } else if constexpr (OP == 9) {  // 16 x v_cmp_gt_f32 + v_addc (zero crossing shape): 8 pairs
#pragma unroll
            for (int k = 0; k < 8; ++k)
                asm volatile("v_cmp_gt_f32 vcc, %1, %2\n v_addc_co_u32 %0, vcc, 0, %0, vcc\n"
                             : "+v"(a0) : "v"(a1), "v"(b) : "vcc");
        } else if constexpr (OP == 10) {  // 16 v_add_f32 + 16 s_xor_b64 interleaved
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_add_f32 %0, %0, %8\n s_xor_b64 s[20:21], s[20:21], s[22:23]\n v_add_f32 %1, %1, %8\n s_xor_b64 s[24:25], s[24:25], s[22:23]\n"
                    "v_add_f32 %2, %2, %8\n s_xor_b64 s[20:21], s[20:21], s[22:23]\n v_add_f32 %3, %3, %8\n s_xor_b64 s[24:25], s[24:25], s[22:23]\n"
                    "v_add_f32 %4, %4, %8\n s_xor_b64 s[20:21], s[20:21], s[22:23]\n v_add_f32 %5, %5, %8\n s_xor_b64 s[24:25], s[24:25], s[22:23]\n"
                    "v_add_f32 %6, %6, %8\n s_xor_b64 s[20:21], s[20:21], s[22:23]\n v_add_f32 %7, %7, %8\n s_xor_b64 s[24:25], s[24:25], s[22:23]\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s20", "s21", "s22", "s23", "s24", "s25", "scc");
        } else if constexpr (OP == 11) {  // 16 v_add_f32 + 4 ds_read_b32
            const unsigned la = threadIdx.x * 4;
            float tmp;
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_add_f32 %0, %0, %9\n ds_read_b32 %8, %10\n v_add_f32 %1, %1, %9\n v_add_f32 %2, %2, %9\n v_add_f32 %3, %3, %9\n"
                    "v_add_f32 %4, %4, %9\n ds_read_b32 %8, %10 offset:256\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=&v"(tmp) : "v"(b), "v"(la));
        } else if constexpr (OP == 12) {  // 16 x v_cndmask_b32_e64 with an SGPR-pair mask
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_cndmask_b32_e64 %0, %0, %8, s[20:21]\n v_cndmask_b32_e64 %1, %1, %8, s[20:21]\n v_cndmask_b32_e64 %2, %2, %8, s[20:21]\n v_cndmask_b32_e64 %3, %3, %8, s[20:21]\n"
                    "v_cndmask_b32_e64 %4, %4, %8, s[20:21]\n v_cndmask_b32_e64 %5, %5, %8, s[20:21]\n v_cndmask_b32_e64 %6, %6, %8, s[20:21]\n v_cndmask_b32_e64 %7, %7, %8, s[20:21]\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s20", "s21");
        } else if constexpr (OP == 13) {  // 8 v_add_f32 + 8 v_add_f64 interleaved
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_add_f32 %0, %0, %12\n v_add_f64 %8, %8, %13\n v_add_f32 %1, %1, %12\n v_add_f64 %9, %9, %13\n"
                    "v_add_f32 %2, %2, %12\n v_add_f64 %10, %10, %13\n v_add_f32 %3, %3, %12\n v_add_f64 %11, %11, %13\n"
                    "v_add_f32 %4, %4, %12\n v_add_f64 %8, %8, %13\n v_add_f32 %5, %5, %12\n v_add_f64 %9, %9, %13\n"
                    "v_add_f32 %6, %6, %12\n v_add_f64 %10, %10, %13\n v_add_f32 %7, %7, %12\n v_add_f64 %11, %11, %13\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(b), "v"(db));
        } else if constexpr (OP == 14) {  // 16 v_add_f32 with SGPR operand (constant bus)
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_add_f32 %0, s20, %0\n v_add_f32 %1, s20, %1\n v_add_f32 %2, s20, %2\n v_add_f32 %3, s20, %3\n"
                    "v_add_f32 %4, s20, %4\n v_add_f32 %5, s20, %5\n v_add_f32 %6, s20, %6\n v_add_f32 %7, s20, %7\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : : "s20");
        } else if constexpr (OP == 15) {  // 8 pairs: v_cmp_gt_f32 (to SGPR pair) + v_addc (independent chains)
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_cmp_gt_f32 s[20:21], %4, %5\n v_cmp_gt_f32 s[22:23], %4, %5\n v_cmp_gt_f32 s[24:25], %4, %5\n v_cmp_gt_f32 s[26:27], %4, %5\n"
                    "v_addc_co_u32 %0, s[20:21], 0, %0, s[20:21]\n v_addc_co_u32 %1, s[22:23], 0, %1, s[22:23]\n v_addc_co_u32 %2, s[24:25], 0, %2, s[24:25]\n v_addc_co_u32 %3, s[26:27], 0, %3, s[26:27]\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a4), "v"(b) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
        } else if constexpr (OP == 16) {  // 16 v_accvgpr_read_b32
#pragma unroll
            for (int k = 0; k < 2; ++k)
                asm volatile(
                    "v_accvgpr_read_b32 %0, a0\n v_accvgpr_read_b32 %1, a1\n v_accvgpr_read_b32 %2, a2\n v_accvgpr_read_b32 %3, a3\n"
                    "v_accvgpr_read_b32 %4, a4\n v_accvgpr_read_b32 %5, a5\n v_accvgpr_read_b32 %6, a6\n v_accvgpr_read_b32 %7, a7\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7");
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y + (float)(d0 + d1 + d2 + d3);
    if (r == 12345.678f) out[threadIdx.x] = r + lds[threadIdx.x];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
int run(const char* name, int waves_per_simd) {
    const int block = 256 * waves_per_simd, grid = 256;
    const int nw = grid * block / 64;
    float* out;
    unsigned long long* cyc;
    CHK(hipMalloc(&out, 4096 * 4));
    CHK(hipMalloc(&cyc, nw * 8));
    CHK(hipFuncSetAttribute((const void*)probe<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(block), 160 * 1024, 0, out, cyc);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(block), 160 * 1024, 0, out, cyc);
    CHK(hipEventRecord(e1));
    CHK(hipDeviceSynchronize());
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(nw);
    CHK(hipMemcpy(h.data(), cyc, nw * 8, hipMemcpyDeviceToHost));
    double mean = 0; for (auto v : h) mean += v; mean /= nw;
    const double ninst = 16.0 * kIters;
    // per-SIMD issue cost: cycles per instruction of ONE wave, times waves sharing the SIMD
    printf("%-16s waves/SIMD=%d  cyc/instr/wave=%6.2f  SIMD cyc/instr=%5.2f  wall=%.3f ms\n", name,
           waves_per_simd, mean / ninst, mean / ninst / waves_per_simd, ms);
    CHK(hipFree(out)); CHK(hipFree(cyc));
    return 0;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    for (int w : {1, 2}) {
        run<10>("add+s_xor", w);
        run<11>("add+ds_read", w);
        run<12>("cndmask_sgpr", w);
        run<13>("add32+add64", w);
        run<14>("add_f32 sgpr", w);
        run<15>("cmp+addc indep", w);
        run<16>("accvgpr_read", w);
    }
    for (int w : {1, 2, 4}) {
        run<0>("v_add_f32", w);
        run<1>("v_pk_add_f32", w);
        run<5>("v_pk_mul_f32", w);
        run<8>("v_pk_fma_f32", w);
        run<2>("v_add_f64", w);
        run<4>("v_mul_f64", w);
        run<3>("v_cvt_f64_f32", w);
        run<6>("v_cndmask_b32", w);
        run<7>("v_log_f32", w);
        run<9>("cmp+addc", w);
    }
    return 0;
}
