// elementwise.hip — the per-sample helpers of the drop-in modules around the window path
// (SURVEY §8 "next" rows): accelerometer roll / pitch / magnitude_dot
// (src/mhealth/inertial/accelerometer.py:13-75, 236-259) and timedom gradient /
// zero_crossings (src/mhealth/generic/timedom.py:11-64). One lane per output sample,
// grid-stride, float32 or float64 input (numba types every expression from the input's
// dtype; the reference's own arithmetic per dtype is restated at each kernel).
#include "engine_common.h"

#include <cstdio>

#include <type_traits>

namespace mhf {
namespace {

constexpr double kDeg = 180.0;

// numba: np.arctan2 on float32 arrays is the float32 libm atan2f; `* 180 / np.pi` then
// runs in float64 (array(float32) * int64 -> float64). atan2 is evaluated here in fp64 and
// rounded to fp32 (glibc's atan2f is within an ulp of that, so results agree to the fp32
// ulp: parity by tolerance, tests/test_gpu_parity.py). float64 input: all fp64.
template <class T>
__device__ __forceinline__ double atan2_deg(T a, T b) {
    if constexpr (sizeof(T) == 4) {
        const float t = static_cast<float>(atan2(static_cast<double>(a), static_cast<double>(b)));
        return static_cast<double>(t) * kDeg / M_PI;
    } else {
        return atan2(a, b) * kDeg / M_PI;
    }
}

template <class T>
__global__ void __launch_bounds__(256) orientation_kernel(int32_t which, const T* x, const T* y, const T* z,
                                                          int64_t n, int64_t stride, double* out) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const T yv = y[i * stride], zv = z[i * stride];
        if (which == MHF_ROLL) {
            out[i] = atan2_deg<T>(yv, zv);                     // arctan2(y, z) * 180 / pi
        } else {
            const T xv = x[i * stride];
            const T h = sqrt(yv * yv + zv * zv);               // y*y + z*z in T, np.sqrt in T
            out[i] = atan2_deg<T>(-xv, h);                     // arctan2(-x, ..) * 180 / pi
        }
    }
}

// gradient: out = np.zeros(len(x)) (float64); out[0] = x[1] - x[0]; out[-1] = x[-1] - x[-2];
// out[i] = (x[i+1] - x[i-1]) / 2 — the difference in T, the halving in float64
template <class T>
__global__ void __launch_bounds__(256) gradient_kernel(const T* x, int64_t n, int64_t stride, double* out) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        if (i == 0) out[0] = static_cast<double>(x[stride] - x[0]);
        else if (i == n - 1) out[i] = static_cast<double>(x[i * stride] - x[(i - 1) * stride]);
        else out[i] = static_cast<double>(x[(i + 1) * stride] - x[(i - 1) * stride]) / 2.0;
    }
}

// zero_crossings: x[np.abs(x) <= th] = 0 (|x| compared with the Python float th in
// float64); pos = x > 0; out = pos[:-1] ^ pos[1:]
template <class T>
__device__ __forceinline__ bool zc_pos(T v, double th) {
    return !(fabs(static_cast<double>(v)) <= th) && v > T(0);
}
template <class T>
__global__ void __launch_bounds__(256) zero_crossings_kernel(const T* x, int64_t n, int64_t stride, double th,
                                                             uint8_t* out) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i + 1 < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[i] = zc_pos<T>(x[i * stride], th) != zc_pos<T>(x[(i + 1) * stride], th);
}

// magnitude_dot: np.sqrt(np.dot(x, x) + np.dot(y, y) + np.dot(z, z)). The three dots are
// BLAS sdot / ddot in the reference (blocked sums, order unspecified); here each is a
// fp64 sum over the whole chip — per-block partials (grid-stride, wave shuffles) into a
// stream-ordered workspace, then one block adds them in block order (deterministic) —
// rounded to T as the BLAS call returns T, then the two T additions and the T sqrt in the
// reference's order.
constexpr int kDotBlocks = 1024;
template <class T>
__global__ void __launch_bounds__(256) magnitude_dot_partial_kernel(const T* x, const T* y, const T* z,
                                                                    int64_t n, int64_t stride, double* part) {
    __shared__ double wp[3][4];
    double s[3] = {0.0, 0.0, 0.0};
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const double a = x[i * stride], b = y[i * stride], c = z[i * stride];
        s[0] += a * a;
        s[1] += b * b;
        s[2] += c * c;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
        if (lane == 0) wp[k][wid] = s[k];
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        part[k * gridDim.x + blockIdx.x] = (wp[k][0] + wp[k][1]) + (wp[k][2] + wp[k][3]);
    }
}

template <class T>
__global__ void __launch_bounds__(256) magnitude_dot_final_kernel(const double* part, int nblk, T* out) {
    __shared__ double wp[3][4];
    double s[3] = {0.0, 0.0, 0.0};
    for (int b = threadIdx.x; b < nblk; b += blockDim.x)
        for (int k = 0; k < 3; ++k) s[k] += part[k * nblk + b];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
        if (lane == 0) wp[k][wid] = s[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        T d[3];
        for (int k = 0; k < 3; ++k) d[k] = static_cast<T>((wp[k][0] + wp[k][1]) + (wp[k][2] + wp[k][3]));
        out[0] = sqrt((d[0] + d[1]) + d[2]);
    }
}

// stats.minmax(x) (src/mhealth/generic/stats.py:12-32): minimum = maximum = x[0], then
// `if x[i] < minimum` / `if x[i] > maximum` for i >= 1 in order. So a NaN x[0] is the
// answer for both; later NaN never win a comparison; among equal values (+0 / -0) the
// first occurrence stays. Parallel form: per lane / block the (value, index) of the
// smallest (largest) non-NaN value, ties to the smaller index; per-block partials into a
// stream-ordered workspace, one block combines them.
template <class T>
struct MinMaxPart {
    T vmin, vmax;
    int64_t imin, imax;   // INT64_MAX: no candidate
};
template <class T>
__device__ __forceinline__ bool is_nan_v(T v) {
    if constexpr (std::is_floating_point_v<T>) return v != v;
    else return false;
}
template <class T>
__device__ __forceinline__ void mm_take(MinMaxPart<T>& a, T vn, int64_t in, T vx, int64_t ix) {
    if (in != INT64_MAX && (a.imin == INT64_MAX || vn < a.vmin || (vn == a.vmin && in < a.imin))) {
        a.vmin = vn;
        a.imin = in;
    }
    if (ix != INT64_MAX && (a.imax == INT64_MAX || vx > a.vmax || (vx == a.vmax && ix < a.imax))) {
        a.vmax = vx;
        a.imax = ix;
    }
}
template <class T>
__device__ __forceinline__ void mm_block(MinMaxPart<T>& a) {
    __shared__ MinMaxPart<T> wp[4];
    for (int o = 32; o > 0; o >>= 1) {
        const T vn = __shfl_xor(a.vmin, o, 64), vx = __shfl_xor(a.vmax, o, 64);
        const int64_t in = __shfl_xor(a.imin, o, 64), ix = __shfl_xor(a.imax, o, 64);
        mm_take(a, vn, in, vx, ix);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) wp[wid] = a;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w) mm_take(a, wp[w].vmin, wp[w].imin, wp[w].vmax, wp[w].imax);
}
template <class T>
__global__ void __launch_bounds__(256) minmax_partial_kernel(const T* x, int64_t n, int64_t stride,
                                                             MinMaxPart<T>* part) {
    MinMaxPart<T> a{T(0), T(0), INT64_MAX, INT64_MAX};
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const T v = x[i * stride];
        if (!is_nan_v(v)) mm_take(a, v, i, v, i);
    }
    mm_block(a);
    if (threadIdx.x == 0) part[blockIdx.x] = a;
}
template <class T>
__global__ void __launch_bounds__(256) minmax_final_kernel(const T* x, const MinMaxPart<T>* part, int nblk,
                                                           T* out) {
    MinMaxPart<T> a{T(0), T(0), INT64_MAX, INT64_MAX};
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) mm_take(a, part[b].vmin, part[b].imin, part[b].vmax, part[b].imax);
    mm_block(a);
    if (threadIdx.x == 0) {
        const T x0 = x[0];
        out[0] = (is_nan_v(x0) || a.imin == INT64_MAX) ? x0 : a.vmin;
        out[1] = (is_nan_v(x0) || a.imax == INT64_MAX) ? x0 : a.vmax;
    }
}

unsigned grid_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return static_cast<unsigned>(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

int check_launch() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHF_OK : set_error(MHF_EDEVICE, hipGetErrorString(e));
}

}  // namespace
}  // namespace mhf

using namespace mhf;

extern "C" int mhf_orientation(int32_t which, const void* x, const void* y, const void* z, int64_t n,
                               int64_t stride, int32_t dtype, double* out, void* hip_stream) {
    set_error(MHF_OK, "");
    if (which != MHF_ROLL && which != MHF_PITCH) return set_error(MHF_EINVAL, "which must be MHF_ROLL or MHF_PITCH");
    if (!y || !z || !out || (which == MHF_PITCH && !x)) return set_error(MHF_EINVAL, "null array");
    if (n < 0 || stride < 1) return set_error(MHF_EINVAL, "n >= 0 and stride >= 1");
    if (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) return set_error(MHF_EINVAL, "dtype must be F32 or F64");
    if (n == 0) return MHF_OK;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (dtype == MHF_DTYPE_F32)
        hipLaunchKernelGGL(orientation_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, which,
                           static_cast<const float*>(x), static_cast<const float*>(y),
                           static_cast<const float*>(z), n, stride, out);
    else
        hipLaunchKernelGGL(orientation_kernel<double>, dim3(grid_for(n)), dim3(256), 0, s, which,
                           static_cast<const double*>(x), static_cast<const double*>(y),
                           static_cast<const double*>(z), n, stride, out);
    return check_launch();
}

extern "C" int mhf_gradient(const void* x, int64_t n, int64_t stride, int32_t dtype, double* out,
                            void* hip_stream) {
    set_error(MHF_OK, "");
    if (!x || !out) return set_error(MHF_EINVAL, "null x or out");
    if (n < 2 || stride < 1) return set_error(MHF_EINVAL, "n >= 2 (the reference indexes x[1]) and stride >= 1");
    if (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) return set_error(MHF_EINVAL, "dtype must be F32 or F64");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (dtype == MHF_DTYPE_F32)
        hipLaunchKernelGGL(gradient_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s,
                           static_cast<const float*>(x), n, stride, out);
    else
        hipLaunchKernelGGL(gradient_kernel<double>, dim3(grid_for(n)), dim3(256), 0, s,
                           static_cast<const double*>(x), n, stride, out);
    return check_launch();
}

extern "C" int mhf_zero_crossings(const void* x, int64_t n, int64_t stride, int32_t dtype, double th,
                                  uint8_t* out, void* hip_stream) {
    set_error(MHF_OK, "");
    if (!x || (!out && n > 1)) return set_error(MHF_EINVAL, "null x or out");
    if (n < 0 || stride < 1) return set_error(MHF_EINVAL, "n >= 0 and stride >= 1");
    if (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) return set_error(MHF_EINVAL, "dtype must be F32 or F64");
    if (n < 2) return MHF_OK;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (dtype == MHF_DTYPE_F32)
        hipLaunchKernelGGL(zero_crossings_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s,
                           static_cast<const float*>(x), n, stride, th, out);
    else
        hipLaunchKernelGGL(zero_crossings_kernel<double>, dim3(grid_for(n)), dim3(256), 0, s,
                           static_cast<const double*>(x), n, stride, th, out);
    return check_launch();
}

namespace {
int64_t dot_blocks(int64_t n) {
    const int64_t nblk = (n + 255) / 256;
    return nblk < 1 ? 1 : (nblk > kDotBlocks ? kDotBlocks : nblk);
}
int ws_fail(const char* what, int64_t need, int64_t have) {
    char msg[160];
    snprintf(msg, sizeof(msg), "%s workspace too small: %lld bytes needed, %lld given", what,
             (long long)need, (long long)have);
    return set_error(MHF_EINVAL, msg);
}
}  // namespace

extern "C" int64_t mhf_magnitude_dot_workspace(int64_t n) {
    if (n < 0) return -1;
    return 3 * dot_blocks(n) * static_cast<int64_t>(sizeof(double));
}

extern "C" int mhf_magnitude_dot(const void* x, const void* y, const void* z, int64_t n, int64_t stride,
                                 int32_t dtype, void* out, void* workspace, int64_t workspace_bytes,
                                 void* hip_stream) {
    set_error(MHF_OK, "");
    if (!x || !y || !z || !out) return set_error(MHF_EINVAL, "null array");
    if (n < 0 || stride < 1) return set_error(MHF_EINVAL, "n >= 0 and stride >= 1");
    if (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) return set_error(MHF_EINVAL, "dtype must be F32 or F64");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const int64_t nblk = dot_blocks(n);
    const int64_t need = mhf_magnitude_dot_workspace(n);
    if (!workspace || workspace_bytes < need) return ws_fail("magnitude_dot", need, workspace_bytes);
    double* part = static_cast<double*>(workspace);
    if (dtype == MHF_DTYPE_F32) {
        hipLaunchKernelGGL(magnitude_dot_partial_kernel<float>, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, s,
                           static_cast<const float*>(x), static_cast<const float*>(y),
                           static_cast<const float*>(z), n, stride, part);
        hipLaunchKernelGGL(magnitude_dot_final_kernel<float>, dim3(1), dim3(256), 0, s, part,
                           static_cast<int>(nblk), static_cast<float*>(out));
    } else {
        hipLaunchKernelGGL(magnitude_dot_partial_kernel<double>, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, s,
                           static_cast<const double*>(x), static_cast<const double*>(y),
                           static_cast<const double*>(z), n, stride, part);
        hipLaunchKernelGGL(magnitude_dot_final_kernel<double>, dim3(1), dim3(256), 0, s, part,
                           static_cast<int>(nblk), static_cast<double*>(out));
    }
    return check_launch();
}

extern "C" int64_t mhf_minmax_workspace(int64_t n, int32_t dtype) {
    if (n < 1) return -1;
    const int64_t nblk = dot_blocks(n);
    switch (dtype) {
    case MHF_DTYPE_F32: return nblk * static_cast<int64_t>(sizeof(MinMaxPart<float>));
    case MHF_DTYPE_F64: return nblk * static_cast<int64_t>(sizeof(MinMaxPart<double>));
    case MHF_DTYPE_I32: return nblk * static_cast<int64_t>(sizeof(MinMaxPart<int32_t>));
    case MHF_DTYPE_I64: return nblk * static_cast<int64_t>(sizeof(MinMaxPart<int64_t>));
    default: return -1;
    }
}

extern "C" int mhf_minmax(const void* x, int64_t n, int64_t stride, int32_t dtype, void* out,
                          void* workspace, int64_t workspace_bytes, void* hip_stream) {
    set_error(MHF_OK, "");
    if (!x || !out) return set_error(MHF_EINVAL, "null x or out");
    if (n < 1) return set_error(MHF_EINVAL, "minmax of an empty array (the reference reads x[0])");
    if (stride < 1) return set_error(MHF_EINVAL, "stride >= 1");
    const int64_t need = mhf_minmax_workspace(n, dtype);
    if (need < 0) return set_error(MHF_EINVAL, "dtype must be F32, F64, I32 or I64");
    if (!workspace || workspace_bytes < need) return ws_fail("minmax", need, workspace_bytes);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const int64_t nblk = dot_blocks(n);
    auto go = [&](auto tag) -> int {
        typedef decltype(tag) T;
        MinMaxPart<T>* part = static_cast<MinMaxPart<T>*>(workspace);
        hipLaunchKernelGGL(minmax_partial_kernel<T>, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, s,
                           static_cast<const T*>(x), n, stride, part);
        hipLaunchKernelGGL(minmax_final_kernel<T>, dim3(1), dim3(256), 0, s, static_cast<const T*>(x), part,
                           static_cast<int>(nblk), static_cast<T*>(out));
        return check_launch();
    };
    switch (dtype) {
    case MHF_DTYPE_F32: return go(0.0f);
    case MHF_DTYPE_F64: return go(0.0);
    case MHF_DTYPE_I32: return go(int32_t(0));
    case MHF_DTYPE_I64: return go(int64_t(0));
    default: return set_error(MHF_EINVAL, "dtype must be F32, F64, I32 or I64");
    }
}

// ---- qrs.find_peaks / nb_find_peaks (heart/qrs.py:200-220): indices i in [1, n-2] with
// x[i] > x[i-1] and x[i] > x[i+1], ascending (np.where of the flags). Three stream-ordered
// launches over blocks of kPeakBlock samples: per-block counts into the caller's
// workspace, one block's exclusive scan of those counts (and the total), then each block
// writes its peaks at its offset in order (a wave-ballot prefix inside the block).
namespace mhf {
namespace {
constexpr int kPeakBlock = 1024;   // samples per block (4 per lane of a 256-lane block)

// comp(x[i], x[i-1]) and comp(x[i], x[i+1]) with comp = np.greater / greater_equal / less /
// less_equal (MHF_CMP_*): numpy's elementwise comparisons in T (NaN compares false)
template <int CMP, class T>
__device__ __forceinline__ bool cmp_v(T a, T b) {
    if constexpr (CMP == MHF_CMP_GREATER) return a > b;
    else if constexpr (CMP == MHF_CMP_GREATER_EQUAL) return a >= b;
    else if constexpr (CMP == MHF_CMP_LESS) return a < b;
    else return a <= b;
}
template <int CMP, class T>
__device__ __forceinline__ bool is_peak(const T* x, int64_t n, int64_t stride, int64_t i) {
    if (i < 1 || i >= n - 1) return false;
    const T v = x[i * stride];
    return cmp_v<CMP, T>(v, x[(i - 1) * stride]) && cmp_v<CMP, T>(v, x[(i + 1) * stride]);
}

// per block: number of peaks among its kPeakBlock samples
template <int CMP, class T>
__global__ void __launch_bounds__(256) peak_count_kernel(const T* x, int64_t n, int64_t stride, int64_t* counts) {
    __shared__ int32_t part[4];
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kPeakBlock;
    int cnt = 0;
    for (int k = 0; k < kPeakBlock / 256; ++k) cnt += is_peak<CMP, T>(x, n, stride, b0 + k * 256 + threadIdx.x);
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one block: counts -> exclusive offsets in place; total at counts[nblk]
__global__ void __launch_bounds__(1024) peak_scan_kernel(int64_t* counts, int64_t nblk) {
    __shared__ int64_t carry;
    __shared__ int64_t wsum[16];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t base = 0; base < nblk; base += blockDim.x) {
        const int64_t i = base + threadIdx.x;
        const int64_t v = i < nblk ? counts[i] : 0;
        int64_t s = v;                                  // inclusive scan within the wave
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t u = __shfl_up(s, o, 64);
            if (lane >= o) s += u;
        }
        if (lane == 63) wsum[wid] = s;
        __syncthreads();
        int64_t before = carry;
        for (int w = 0; w < wid; ++w) before += wsum[w];
        if (i < nblk) counts[i] = before + s - v;
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) carry = before + s;
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[nblk] = carry;
}

// each block writes its peaks' indices, in order, from its offset
template <int CMP, class T>
__global__ void __launch_bounds__(256) peak_scatter_kernel(const T* x, int64_t n, int64_t stride,
                                                           const int64_t* offs, int64_t* out) {
    __shared__ int32_t wtot[4];
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kPeakBlock;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t off = offs[blockIdx.x];
    for (int k = 0; k < kPeakBlock / 256; ++k) {
        const int64_t i = b0 + k * 256 + threadIdx.x;
        const bool p = is_peak<CMP, T>(x, n, stride, i);
        const uint64_t m = __ballot(p);
        const int below = __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        if (lane == 0) wtot[wid] = __popcll(m);
        __syncthreads();
        int64_t pre = 0;
        for (int w = 0; w < wid; ++w) pre += wtot[w];
        if (p) out[off + pre + below] = i;
        const int64_t all = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        __syncthreads();
        off += all;
    }
}
}  // namespace
}  // namespace mhf

extern "C" int64_t mhf_find_peaks_workspace(int64_t n) {
    return n < 0 ? -1 : ((n + mhf::kPeakBlock - 1) / mhf::kPeakBlock + 1) * static_cast<int64_t>(sizeof(int64_t));
}

extern "C" int mhf_find_peaks_cmp(const void* x, int64_t n, int64_t stride, int32_t dtype, int32_t comp,
                                  int64_t* out, int64_t* workspace, void* hip_stream) {
    set_error(MHF_OK, "");
    if ((!x && n > 0) || !out || !workspace) return set_error(MHF_EINVAL, "null x, out or workspace");
    if (n < 0 || stride < 1) return set_error(MHF_EINVAL, "n >= 0 and stride >= 1");
    if (dtype != MHF_DTYPE_F32 && dtype != MHF_DTYPE_F64) return set_error(MHF_EINVAL, "dtype must be F32 or F64");
    if (comp < MHF_CMP_GREATER || comp > MHF_CMP_LESS_EQUAL) return set_error(MHF_EINVAL, "unknown comparison");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const int64_t nblk = (n + kPeakBlock - 1) / kPeakBlock;
    if (nblk > 0x7fffffff) return set_error(MHF_EINVAL, "n too large");
    if (nblk == 0) {
        return hipMemsetAsync(workspace, 0, sizeof(int64_t), s) == hipSuccess
                   ? MHF_OK : set_error(MHF_EDEVICE, "hipMemsetAsync failed");
    }
    const dim3 grid(static_cast<unsigned>(nblk));
    auto go = [&](auto cmp, auto tag) {
        constexpr int C = decltype(cmp)::value;
        typedef decltype(tag) T;
        hipLaunchKernelGGL((peak_count_kernel<C, T>), grid, dim3(256), 0, s, static_cast<const T*>(x), n,
                           stride, workspace);
        hipLaunchKernelGGL(peak_scan_kernel, dim3(1), dim3(1024), 0, s, workspace, nblk);
        hipLaunchKernelGGL((peak_scatter_kernel<C, T>), grid, dim3(256), 0, s, static_cast<const T*>(x), n,
                           stride, workspace, out);
    };
    auto by_type = [&](auto cmp) {
        if (dtype == MHF_DTYPE_F32) go(cmp, 0.0f);
        else go(cmp, 0.0);
    };
    switch (comp) {
    case MHF_CMP_GREATER: by_type(std::integral_constant<int, MHF_CMP_GREATER>{}); break;
    case MHF_CMP_GREATER_EQUAL: by_type(std::integral_constant<int, MHF_CMP_GREATER_EQUAL>{}); break;
    case MHF_CMP_LESS: by_type(std::integral_constant<int, MHF_CMP_LESS>{}); break;
    default: by_type(std::integral_constant<int, MHF_CMP_LESS_EQUAL>{}); break;
    }
    return check_launch();
}

extern "C" int mhf_find_peaks(const void* x, int64_t n, int64_t stride, int32_t dtype, int64_t* out,
                              int64_t* workspace, void* hip_stream) {
    return mhf_find_peaks_cmp(x, n, stride, dtype, MHF_CMP_GREATER, out, workspace, hip_stream);
}
