// div_probe.hip — exhaustive check of the hoisted-reciprocal fp32 division used by the
// moment kernels (mhfeat.hip, pass 2 of window_moments_t): for an integer divisor b and
// y = RN(1/b),
//     q0 = RN(a y),  r = RN(a - q0 b) (fma),  q = RN(q0 + r y) (fma)
// must equal the IEEE quotient RN(a / b) bit for bit (Markstein's correction step).
// Every mantissa of one binade a in [1, 2) against every b in [1, B]: scaling a by 2^k
// scales every intermediate exactly while they stay normal, so this covers all a with
// 2^-100 <= |a| <= FLT_MAX (the kernels take the IEEE division outside that range).
// usage: div_probe [B = 65536]   (prints the mismatch count; exit 1 on any mismatch)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void probe(unsigned long long* bad, int b0) {
    const int b = b0 + static_cast<int>(blockIdx.y);
    const float bf = static_cast<float>(b);
    const float y = 1.0f / bf;
    unsigned long long n = 0;
    for (unsigned k = blockIdx.x * blockDim.x + threadIdx.x; k < (1u << 23);
         k += gridDim.x * blockDim.x) {
        const float a = __uint_as_float(0x3f800000u | k);
        const float ref = a / bf;
        const float q0 = a * y;
        const float r = __builtin_fmaf(-q0, bf, a);
        const float q = __builtin_fmaf(r, y, q0);
        n += (__float_as_uint(q) != __float_as_uint(ref));
    }
    if (n) atomicAdd(bad, n);
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 65536;
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, sizeof(*d)) != hipSuccess) return 2;
    if (hipMemset(d, 0, sizeof(*d)) != hipSuccess) return 2;
    for (int b0 = 1; b0 <= B; b0 += 1024) {
        const int nb = B - b0 + 1 < 1024 ? B - b0 + 1 : 1024;
        hipLaunchKernelGGL(probe, dim3(64, nb), dim3(256), 0, 0, d, b0);
    }
    unsigned long long h = 0;
    if (hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("div_probe: divisors 1..%d x 2^23 mantissas: %llu mismatches\n", B, h);
    (void)hipFree(d);
    return h ? 1 : 0;
}
