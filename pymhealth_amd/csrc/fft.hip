// fft.hip — complex128 FFT for mhealth.fft.fft / ifft (src/mhealth/fft/_fft.py:18-48).
//
// The reference binds FFTW through cffi: fftw_fft(N, in, out, direction) plans
// fftw_plan_dft_1d(..., FFTW_ESTIMATE), executes and destroys the plan on every call
// (src/mhealth/fft/_fftw_binder.py:11-17); fft() is the unnormalised forward transform of
// a.astype(complex128), ifft() the backward one divided by n. Without the compiled binder
// the reference falls back to numpy.fft (src/mhealth/fft/__init__.py:3-7): the same
// transforms in fp64 (pocketfft), which is what the parity tests pin against.
//
// MI355X form: fp64 throughout (the reference's precision), batch rows in one call.
//   * n = 2^k <= 4096: one workgroup per row; the row is loaded bit-reversed into LDS
//     (n x 16 B <= 64 KiB) and transformed in place by k radix-2 DIT passes, one barrier
//     each, twiddles from a per-call table (sincospi, fp64).
//   * n = 2^k > 4096: a bit-reversal pass into a work buffer, the first 12 passes in LDS on
//     aligned 4096-point blocks (after bit reversal they are independent), the remaining
//     k - 12 passes one launch each over global memory (HBM-bound, coalesced butterflies).
//   * any other n: Bluestein's chirp-z transform, X_m = w_m sum_k (x_k w_k) conj(w_{m-k}),
//     w_k = exp(dir i pi k^2 / n) (k^2 reduced mod 2n in integers, so the chirp angle is
//     exact before sincospi), as a cyclic convolution of length M = 2^ceil(log2(2n - 1))
//     through the power-of-two path.
// Not on the windowed hot path (the fused kernels carry their own fp32 rFFT); this is the
// drop-in for the user-composed spectral pipeline (fft -> psd ->
// hrv.power_band).
#include "engine_common.h"

#include <cstdio>

namespace mhf {
namespace {

typedef double2 cplx;

constexpr int kLdsLog2 = 12;   // 4096 points x 16 B = 64 KiB of LDS

__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
    return cplx{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// tw[k] = exp(-2 pi i k / n), k < n / 2
__global__ void __launch_bounds__(256) fft_twiddle_kernel(cplx* tw, int64_t n) {
    for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < n / 2;
         k += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        double s, c;
        sincospi(2.0 * static_cast<double>(k) / static_cast<double>(n), &s, &c);
        tw[k] = cplx{c, -s};
    }
}

__device__ __forceinline__ uint32_t bitrev(uint32_t i, int bits) {
    return bits == 0 ? 0u : (__builtin_bitreverse32(i) >> (32 - bits));
}

// Radix-2 DIT passes 1..L on blocks of 2^L points in LDS. `perm`: load block b of row r
// bit-reversed from `in` (the whole transform when L = log2n); otherwise the blocks are
// already permuted. Pass s (half = 2^(s-1)) uses w = exp(dir 2 pi i pos / 2^s) =
// tw[pos << (log2n - s)] (conjugated for dir = +1). Every output scaled by `scale`.
__global__ void __launch_bounds__(256) fft_lds_kernel(const cplx* in, cplx* out, int L, int log2n,
                                                      int64_t nblocks, int perm, int dir, double scale,
                                                      const cplx* tw) {
    extern __shared__ cplx buf[];
    const int m = 1 << L;
    const int64_t n = int64_t(1) << log2n;
    for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const cplx* src = in + b * m;
        if (perm) {
            for (int i = threadIdx.x; i < m; i += blockDim.x) buf[bitrev(i, L)] = src[i];
        } else {
            for (int i = threadIdx.x; i < m; i += blockDim.x) buf[i] = src[i];
        }
        __syncthreads();
        for (int s = 1; s <= L; ++s) {
            const int half = 1 << (s - 1);
            for (int q = threadIdx.x; q < m / 2; q += blockDim.x) {
                const int pos = q & (half - 1);
                const int i = ((q >> (s - 1)) << s) | pos, j = i + half;
                cplx w = tw[static_cast<int64_t>(pos) << (log2n - s)];
                if (dir > 0) w.y = -w.y;
                const cplx t = cmul(w, buf[j]), u = buf[i];
                buf[i] = cplx{u.x + t.x, u.y + t.y};
                buf[j] = cplx{u.x - t.x, u.y - t.y};
            }
            __syncthreads();
        }
        cplx* dst = out + b * m;
        for (int i = threadIdx.x; i < m; i += blockDim.x) dst[i] = cplx{buf[i].x * scale, buf[i].y * scale};
        __syncthreads();
    }
    (void)n;
}

// rows of n = 2^log2n points: out[r, bitrev(i)] = in[r, i]
__global__ void __launch_bounds__(256) fft_bitrev_kernel(const cplx* in, cplx* out, int log2n, int64_t total) {
    const int64_t n = int64_t(1) << log2n;
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = g >> log2n, i = g & (n - 1);
        // log2n > 12 here: the row index fits 32 bits for n < 2^32
        out[(r << log2n) + bitrev(static_cast<uint32_t>(i), log2n)] = in[g];
    }
}

// one radix-2 DIT pass s (> 12) over every row, in place; last pass also scales into out
__global__ void __launch_bounds__(256) fft_pass_kernel(cplx* a, int log2n, int s, int64_t total_bf, int dir,
                                                       const cplx* tw) {
    const int64_t half = int64_t(1) << (s - 1);
    const int64_t nh = int64_t(1) << (log2n - 1);
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total_bf;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = g / nh, q = g - r * nh;
        const int64_t pos = q & (half - 1);
        const int64_t i = (r << log2n) + (((q >> (s - 1)) << s) | pos), j = i + half;
        cplx w = tw[pos << (log2n - s)];
        if (dir > 0) w.y = -w.y;
        const cplx t = cmul(w, a[j]), u = a[i];
        a[i] = cplx{u.x + t.x, u.y + t.y};
        a[j] = cplx{u.x - t.x, u.y - t.y};
    }
}

__global__ void __launch_bounds__(256) fft_scale_kernel(const cplx* a, cplx* out, int64_t total, double scale) {
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[g] = cplx{a[g].x * scale, a[g].y * scale};
}

// ---- Bluestein
// chirp w_k = exp(dir i pi (k^2 mod 2n) / n), k < n
__device__ __forceinline__ cplx chirp(int64_t k, int64_t n, int dir) {
    // k < n <= 2^30: k^2 < 2^60 fits 64 bits
    const uint64_t kk = static_cast<uint64_t>(k) * static_cast<uint64_t>(k);
    const int64_t r = static_cast<int64_t>(kk % static_cast<uint64_t>(2 * n));
    double s, c;
    sincospi(static_cast<double>(r) / static_cast<double>(n), &s, &c);
    return cplx{c, dir > 0 ? s : -s};
}

// A[r, k] = x[r, k] w_k (k < n), 0 up to M
__global__ void __launch_bounds__(256) bluestein_pre_kernel(const cplx* x, cplx* A, int64_t n, int log2m,
                                                            int64_t total, int dir) {
    const int64_t M = int64_t(1) << log2m;
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = g >> log2m, k = g & (M - 1);
        A[g] = k < n ? cmul(x[r * n + k], chirp(k, n, dir)) : cplx{0.0, 0.0};
    }
}

// B[j] = conj(w_j) at j and M - j (j < n), 0 elsewhere
__global__ void __launch_bounds__(256) bluestein_kernel_b(cplx* B, int64_t n, int64_t M, int dir) {
    for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < M;
         j += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t k = j < n ? j : (M - j < n ? M - j : -1);
        if (k < 0) {
            B[j] = cplx{0.0, 0.0};
        } else {
            const cplx w = chirp(k, n, dir);
            B[j] = cplx{w.x, -w.y};
        }
    }
}

// A[r, k] *= FB[k]
__global__ void __launch_bounds__(256) bluestein_mul_kernel(cplx* A, const cplx* FB, int log2m, int64_t total) {
    const int64_t M = int64_t(1) << log2m;
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x)
        A[g] = cmul(A[g], FB[g & (M - 1)]);
}

// out[r, m] = scale w_m C[r, m] (m < n); C already carries 1 / M
__global__ void __launch_bounds__(256) bluestein_post_kernel(const cplx* C, cplx* out, int64_t n, int log2m,
                                                             int64_t total, int dir, double scale) {
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t r = g / n, m = g - r * n;
        const cplx v = cmul(C[(r << log2m) + m], chirp(m, n, dir));
        out[g] = cplx{v.x * scale, v.y * scale};
    }
}

unsigned grid_of(int64_t work) {
    int64_t b = (work + 255) / 256;
    if (b < 1) b = 1;
    if (b > 16384) b = 16384;
    return static_cast<unsigned>(b);
}

// Work buffers carved from the caller's workspace (include/mhfeat.h: no allocation inside).
// A power-of-two pass releases its buffers when it returns (`mark`): the launches that
// used them precede, in stream order, any later launch that reuses the bytes.
int64_t round256(int64_t b) { return (b + 255) & ~int64_t(255); }
int64_t cbytes(int64_t count) { return round256((count > 0 ? count : 1) * static_cast<int64_t>(sizeof(cplx))); }
struct Arena {
    char* base;
    int64_t size, used;
    cplx* get(int64_t count) {
        const int64_t b = cbytes(count);
        if (used + b > size) return nullptr;
        cplx* q = reinterpret_cast<cplx*>(base + used);
        used += b;
        return q;
    }
};
// bytes fft_pow2 takes from the arena: twiddles, plus the work copy past the LDS size
int64_t pow2_bytes(int log2n, int64_t batch) {
    const int64_t n = int64_t(1) << log2n;
    return cbytes(n / 2) + (log2n > kLdsLog2 ? cbytes(batch * n) : 0);
}

// power-of-two transform of `batch` rows; in may equal out
int fft_pow2(const cplx* in, cplx* out, int log2n, int64_t batch, int dir, double scale, Arena& ar,
             hipStream_t s) {
    const int64_t n = int64_t(1) << log2n;
    struct Release {
        Arena& a;
        int64_t mark;
        ~Release() { a.used = mark; }
    } rel{ar, ar.used};
    cplx* tw = ar.get(n / 2);
    if (!tw) return MHF_EINVAL;
    hipLaunchKernelGGL(fft_twiddle_kernel, dim3(grid_of(n / 2)), dim3(256), 0, s, tw, n);
    if (log2n <= kLdsLog2) {
        const int64_t g = batch < 65536 ? batch : 65536;
        hipLaunchKernelGGL(fft_lds_kernel, dim3(static_cast<unsigned>(g)), dim3(256),
                           static_cast<size_t>(n) * sizeof(cplx), s, in, out, log2n, log2n, batch, 1, dir,
                           scale, tw);
        return MHF_OK;
    }
    const int64_t total = batch * n;
    cplx* a = ar.get(total);
    if (!a) return MHF_EINVAL;
    hipLaunchKernelGGL(fft_bitrev_kernel, dim3(grid_of(total)), dim3(256), 0, s, in, a, log2n, total);
    const int64_t nblk = total >> kLdsLog2;
    hipLaunchKernelGGL(fft_lds_kernel, dim3(static_cast<unsigned>(nblk < 65536 ? nblk : 65536)), dim3(256),
                       static_cast<size_t>(1) << (kLdsLog2 + 4), s, a, a, kLdsLog2, log2n, nblk, 0, dir, 1.0,
                       tw);
    for (int p = kLdsLog2 + 1; p <= log2n; ++p)
        hipLaunchKernelGGL(fft_pass_kernel, dim3(grid_of(total / 2)), dim3(256), 0, s, a, log2n, p, total / 2,
                           dir, tw);
    hipLaunchKernelGGL(fft_scale_kernel, dim3(grid_of(total)), dim3(256), 0, s, a, out, total, scale);
    return MHF_OK;
}

int ilog2_exact(int64_t n) {
    int k = 0;
    while ((int64_t(1) << k) < n) ++k;
    return (int64_t(1) << k) == n ? k : -1;
}

}  // namespace
}  // namespace mhf

using namespace mhf;

extern "C" int64_t mhf_fft_workspace(int64_t n, int64_t batch) {
    if (n < 1 || batch < 0 || n > (int64_t(1) << 30)) return -1;
    if (batch == 0) return 0;
    const int log2n = ilog2_exact(n);
    if (log2n >= 0) return pow2_bytes(log2n, batch);
    int log2m = 0;
    while ((int64_t(1) << log2m) < 2 * n - 1) ++log2m;
    const int64_t M = int64_t(1) << log2m;
    const int64_t inner1 = pow2_bytes(log2m, 1), innerb = pow2_bytes(log2m, batch);
    return cbytes(batch * M) + cbytes(M) + (inner1 > innerb ? inner1 : innerb);
}

extern "C" int mhf_fft(const double* in, double* out, int64_t n, int64_t batch, int32_t direction, double scale,
                       void* workspace, int64_t workspace_bytes, void* hip_stream) {
    set_error(MHF_OK, "");
    if (n < 1 || batch < 0) return set_error(MHF_EINVAL, "n must be >= 1 and batch >= 0");
    if (direction != MHF_FFT_FORWARD && direction != MHF_FFT_BACKWARD)
        return set_error(MHF_EINVAL, "direction must be MHF_FFT_FORWARD or MHF_FFT_BACKWARD");
    if (n > (int64_t(1) << 30)) return set_error(MHF_EUNSUPPORTED, "n must be <= 2^30");
    if (batch == 0) return MHF_OK;
    if (!in || !out) return set_error(MHF_EINVAL, "null in or out");
    const int64_t need = mhf_fft_workspace(n, batch);
    if (!workspace || workspace_bytes < need) {
        char msg[160];
        snprintf(msg, sizeof(msg), "fft workspace too small: %lld bytes needed (mhf_fft_workspace), "
                 "%lld given", (long long)need, (long long)workspace_bytes);
        return set_error(MHF_EINVAL, msg);
    }
    Arena ar{static_cast<char*>(workspace), workspace_bytes, 0};
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const cplx* x = reinterpret_cast<const cplx*>(in);
    cplx* y = reinterpret_cast<cplx*>(out);
    const int dir = direction;
    int rc;
    const int log2n = ilog2_exact(n);
    if (log2n >= 0) {
        rc = fft_pow2(x, y, log2n, batch, dir, scale, ar, s);
    } else {
        int log2m = 0;
        while ((int64_t(1) << log2m) < 2 * n - 1) ++log2m;
        const int64_t M = int64_t(1) << log2m;
        cplx* A = ar.get(batch * M);
        cplx* B = ar.get(M);
        if (!A || !B) return set_error(MHF_EINVAL, "fft workspace too small");
        hipLaunchKernelGGL(bluestein_pre_kernel, dim3(grid_of(batch * M)), dim3(256), 0, s, x, A, n, log2m,
                           batch * M, dir);
        hipLaunchKernelGGL(bluestein_kernel_b, dim3(grid_of(M)), dim3(256), 0, s, B, n, M, dir);
        rc = fft_pow2(B, B, log2m, 1, MHF_FFT_FORWARD, 1.0, ar, s);
        if (rc == MHF_OK) rc = fft_pow2(A, A, log2m, batch, MHF_FFT_FORWARD, 1.0, ar, s);
        if (rc == MHF_OK) {
            hipLaunchKernelGGL(bluestein_mul_kernel, dim3(grid_of(batch * M)), dim3(256), 0, s, A, B, log2m,
                               batch * M);
            rc = fft_pow2(A, A, log2m, batch, MHF_FFT_BACKWARD, 1.0 / static_cast<double>(M), ar, s);
        }
        if (rc == MHF_OK)
            hipLaunchKernelGGL(bluestein_post_kernel, dim3(grid_of(batch * n)), dim3(256), 0, s, A, y, n, log2m,
                               batch * n, dir, scale);
    }
    if (rc != MHF_OK) return set_error(rc, "fft workspace too small");
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHF_OK : set_error(MHF_EDEVICE, hipGetErrorString(e));
}
