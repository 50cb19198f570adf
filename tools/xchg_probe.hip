// xchg_probe — checks lane_xchg.h's xchg<L, J> (exchange of lane bit L with register bit J
// over 8 complex registers, spectral_reg.hip's in-register transposes) on the GPU for every
// L in 0..5, J in 0..2: element (lane, reg, part) is tagged with its own coordinates and
// must land at (lane with bit L := reg bit J, reg with bit J := lane bit L). Prints the
// mismatch count; exit status 1 on any.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../pymhealth_amd/csrc/lane_xchg.h"

using mhf::xf2;

template <int L, int J>
__global__ void __launch_bounds__(64) probe(float* out) {
    const int lane = threadIdx.x;
    xf2 v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = xf2{float(lane * 16 + r * 2), float(lane * 16 + r * 2 + 1)};
    mhf::xchg<L, J>(v);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        out[(lane * 8 + r) * 2] = v[r].x;
        out[(lane * 8 + r) * 2 + 1] = v[r].y;
    }
}

template <int L, int J>
long check(float* d, float* h) {
    hipLaunchKernelGGL((probe<L, J>), dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 1024 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    long bad = 0;
    for (int lane = 0; lane < 64; ++lane)
        for (int r = 0; r < 8; ++r)
            for (int p = 0; p < 2; ++p) {
                const int lb = (lane >> L) & 1, rb = (r >> J) & 1;
                const int sl = (lane & ~(1 << L)) | (rb << L);
                const int sr = (r & ~(1 << J)) | (lb << J);
                const float want = float(sl * 16 + sr * 2 + p);
                if (h[(lane * 8 + r) * 2 + p] != want) ++bad;
            }
    printf("xchg<%d,%d>: %ld mismatches\n", L, J, bad);
    return bad;
}

template <int L>
long check_l(float* d, float* h) {
    return check<L, 0>(d, h) + check<L, 1>(d, h) + check<L, 2>(d, h);
}

int main() {
    float *d = nullptr, h[1024];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    const long bad = check_l<0>(d, h) + check_l<1>(d, h) + check_l<2>(d, h) + check_l<3>(d, h) +
                     check_l<4>(d, h) + check_l<5>(d, h);
    (void)hipFree(d);
    printf("total %ld mismatches\n", bad);
    return bad == 0 ? 0 : 1;
}
