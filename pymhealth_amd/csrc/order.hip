// order.hip — order-statistic features of every window: np.median (stats.median),
// np.percentile(x, q) (stats.percentile), stats.interquartile_range and stats.mode
// (src/mhealth/generic/stats.py:48-94,156-163), for fixed and time-indexed windows.
//
// The reference evaluates them with numba 0.54.1's selection and sort code:
//   np.median       quickselect _select / _select_two over _partition (`<` comparisons,
//                   median of three) on a copy (numba/np/arraymath.py:1283-1398)
//   np.percentile   _collect_percentiles (:1402-1515): any NaN -> NaN; n == 1 -> a[0];
//                   q == 100 / 0 -> max / min with numba's infinity heuristics; else
//                   rank = 1 + (n-1) q/100, lower/upper = _select_two(k = floor(rank)-1),
//                   lower (1-m) + upper m in float64
//   interquartile_range  np.percentile(x, [75, 25]): both selections on ONE float64 copy
//   stats.mode      the @overload jit version that rolling_apply compiles (stats.py:73-94):
//                   np.sort (numba quicksort, lt = isnan(b) or a < b; numba/np/arrayobj.py
//                   lt_floats, numba/misc/quicksort.py), then a run scan whose first run is
//                   counted one short (c2 starts at 0) and whose ties go to the earlier run
//
// MI355X path: one wave per window (all its channels), the window's samples staged in LDS
// as order-preserving 32-bit keys and sorted by a bitonic network (64 lanes per compare
// stage); every order statistic, min / max, infinity count and run length is then read
// off the sorted keys. Equal keys are bit-identical floats, so a value taken from the
// sorted keys IS the value numba's selection returns — except where the answer depends on
// which of several non-identical equal values numba's own permutation leaves in a slot:
// +0 / -0 mixed in one window with a zero answer, and NaN for the median (numba's `<`
// quickselect moves NaN arbitrarily). Those windows (rare) replay numba's exact algorithm
// serially on an LDS copy of the window (one lane), so every result is bit-exact.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "../../include/mhfeat.h"
#include "engine_common.h"

namespace mhf {
namespace {

// ---------------------------------------------------------------- value <-> sort key
// Order-preserving unsigned keys of the sample type (32-bit for float32 records, 64-bit for
// float64 ones): negative values bit-inverted, non-negative ones with the sign bit set, every
// NaN (and the padding) the largest key.
template <class T>
struct Keys;
template <>
struct Keys<float> {
    typedef uint32_t K;
    static constexpr K kNan = 0xffffffffu, kNegZero = 0x7fffffffu, kPosZero = 0x80000000u,
                       kPosInf = 0xff800000u, kNegInf = 0x007fffffu;
    __device__ static K key(float v) {
        const uint32_t b = __float_as_uint(v);
        if (v != v) return kNan;
        return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    }
    __device__ static float val(K k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }
};
template <>
struct Keys<double> {
    typedef uint64_t K;
    static constexpr K kSign = 0x8000000000000000ull;
    static constexpr K kNan = ~0ull, kNegZero = ~kSign, kPosZero = kSign,
                       kPosInf = 0xfff0000000000000ull, kNegInf = 0x000fffffffffffffull;
    __device__ static K key(double v) {
        const uint64_t b = __double_as_longlong(v);
        if (v != v) return kNan;
        return (b & kSign) ? ~b : (b | kSign);
    }
    __device__ static double val(K k) {
        return __longlong_as_double(static_cast<long long>((k & kSign) ? (k & ~kSign) : ~k));
    }
};

// ---------------------------------------------------------------- numba replays (serial)
// numba _partition / _select / _select_two (arraymath.py:1283-1367), pivotimpl = `<`
template <class T>
__device__ int nb_partition(T* A, int low, int high) {
    const int mid = (low + high) >> 1;
    T t;
    if (A[mid] < A[low]) { t = A[low]; A[low] = A[mid]; A[mid] = t; }
    if (A[high] < A[mid]) { t = A[high]; A[high] = A[mid]; A[mid] = t; }
    if (A[mid] < A[low]) { t = A[low]; A[low] = A[mid]; A[mid] = t; }
    const T pivot = A[mid];
    t = A[high]; A[high] = A[mid]; A[mid] = t;
    int i = low, j = high - 1;
    for (;;) {
        while (i < high && A[i] < pivot) ++i;
        while (j >= low && pivot < A[j]) --j;
        if (i >= j) break;
        t = A[i]; A[i] = A[j]; A[j] = t;
        ++i;
        --j;
    }
    t = A[i]; A[i] = A[high]; A[high] = t;
    return i;
}

template <class T>
__device__ T nb_select(T* A, int k, int low, int high) {
    int i = nb_partition(A, low, high);
    while (i != k) {
        if (i < k) low = i + 1;
        else high = i - 1;
        i = nb_partition(A, low, high);
    }
    return A[k];
}

template <class T>
__device__ __noinline__ void nb_select_two(T* A, int k, int low, int high, T& a, T& b) {
    for (;;) {
        const int i = nb_partition(A, low, high);
        if (i < k) low = i + 1;
        else if (i > k + 1) high = i - 1;
        else if (i == k) { nb_select(A, k + 1, i + 1, high); break; }
        else { nb_select(A, k, low, i - 1); break; }
    }
    a = A[k];
    b = A[k + 1];
}

// numba median_impl (:1371-1398): even n -> f64(a + b) / 2, the sum in the sample type
template <class T>
__device__ __noinline__ double nb_median(T* A, int n) {
    const int half = n >> 1;
    if ((n & 1) == 0) {
        T a, b;
        nb_select_two(A, half - 1, 0, n - 1, a, b);
        return static_cast<double>(a + b) / 2.0;
    }
    return static_cast<double>(nb_select(A, half, 0, n - 1));
}

// rank / interpolation weight of _collect_percentiles_inner for 0 < q < 100
struct Rank {
    int k;          // lower order statistic (f - 1)
    double m;       // weight of the upper one
};
__device__ __forceinline__ Rank pct_rank(int n, double q) {
    const double rank = 1.0 + static_cast<double>(n - 1) * (q / 100.0);
    const double f = floor(rank);
    return Rank{static_cast<int>(f - 1.0), rank - f};
}
__device__ __forceinline__ double pct_interp(double lo, double hi, double m) {
    return lo * (1.0 - m) + hi * m;
}

// numba array_max / array_min on the float64 copy: first occurrence of the extreme value
// (strict comparisons; NaN-free here)
template <class T>
__device__ __noinline__ double nb_first_extreme(const T* A, int n, bool want_max) {
    T best = A[0];
    for (int i = 1; i < n; ++i)
        if (want_max ? (A[i] > best) : (A[i] < best)) best = A[i];
    return static_cast<double>(best);
}

// numba quicksort (numba/misc/quicksort.py make_quicksort_impl: median-of-three partition,
// insertion sort below 16 elements, larger half pushed) with lt_floats = isnan(b) or a < b
template <class T>
__device__ __forceinline__ bool nb_lt(T a, T b) { return (b != b) || (a < b); }

template <class T>
__device__ int nb_qs_partition(T* A, int low, int high) {
    const int mid = (low + high) >> 1;
    T t;
    if (nb_lt(A[mid], A[low])) { t = A[low]; A[low] = A[mid]; A[mid] = t; }
    if (nb_lt(A[high], A[mid])) { t = A[high]; A[high] = A[mid]; A[mid] = t; }
    if (nb_lt(A[mid], A[low])) { t = A[low]; A[low] = A[mid]; A[mid] = t; }
    const T pivot = A[mid];
    t = A[high]; A[high] = A[mid]; A[mid] = t;
    int i = low, j = high - 1;
    for (;;) {
        while (i < high && nb_lt(A[i], pivot)) ++i;
        while (j >= low && nb_lt(pivot, A[j])) --j;
        if (i >= j) break;
        t = A[i]; A[i] = A[j]; A[j] = t;
        ++i;
        --j;
    }
    t = A[i]; A[i] = A[high]; A[high] = t;
    return i;
}

template <class T>
__device__ void nb_insertion_sort(T* A, int low, int high) {
    for (int i = low + 1; i <= high; ++i) {
        const T v = A[i];
        int j = i;
        while (j > low && nb_lt(v, A[j - 1])) {
            A[j] = A[j - 1];
            --j;
        }
        A[j] = v;
    }
}

template <class T>
__device__ __noinline__ void nb_quicksort(T* A, int n) {
    // numba keeps MAX_STACK = 100 entries; it always pushes the larger part and loops on
    // the smaller one, so the depth never exceeds log2(n) + 1 <= 15 for n <= 16384
    int st_lo[32], st_hi[32];
    int sp = 0;
    st_lo[0] = 0;
    st_hi[0] = n - 1;
    sp = 1;
    while (sp > 0) {
        --sp;
        int low = st_lo[sp], high = st_hi[sp];
        while (high - low >= 15) {
            const int i = nb_qs_partition(A, low, high);
            if (high - i > i - low) {
                if (high > i) { st_lo[sp] = i + 1; st_hi[sp] = high; ++sp; }
                high = i - 1;
            } else {
                if (i > low) { st_lo[sp] = low; st_hi[sp] = i - 1; ++sp; }
                low = i + 1;
            }
        }
        nb_insertion_sort(A, low, high);
    }
}

// stats.mode's jit version (stats.py:73-94) after np.sort
template <class T>
__device__ __noinline__ double nb_mode(T* A, int n) {
    nb_quicksort(A, n);
    T e1 = A[0];
    int c1 = 1, c2 = 0;
    for (int i = 1; i < n; ++i) {
        if (A[i] == A[i - 1]) {
            ++c2;
            if (c2 > c1) { c1 = c2; e1 = A[i]; }
        } else {
            c2 = 1;
        }
    }
    return static_cast<double>(e1);
}

// ---------------------------------------------------------------- the kernel
struct OrdArgs {
    const float* x;
    const double* xd;            // float64 record (order_kernel<E, double>)
    int64_t ch_stride, sample_stride, wsize, wstep, first, nwin;
    int32_t channels;
    const int64_t* starts;       // indexed windows (nullptr: fixed windows)
    const int64_t* ends;
    int64_t n_samples, min_len;
    int32_t cap;                 // keys per channel (power of two >= every window)
    int32_t waves;               // waves per block
    // indexed windows longer than the LDS capacity (order_kernel only): the LDS launch sets
    // skip_long and leaves windows of more than `cap` samples alone; a second launch sorts
    // exactly those in `gkeys` (global memory, C * cap keys per wave), windows of more
    // than `short_cap` samples only
    int32_t skip_long;
    void* gkeys;
    int64_t short_cap;
    double q;                    // np.percentile q
    int32_t sampen_cyc;          // sampen_kernel: cyclic-diagonal walk (window twice in LDS)
    FeatList feats;
    void* out;
    int64_t out_ld;
    int32_t out_f32;
    // order_kernel's rescan launch after order_sel_kernel: only the windows whose output
    // at row `rescan_row` holds the sentinel (order_sel_kernel left them: NaN / zero / inf)
    int32_t rescan;
    int64_t rescan_row;
};
// the sentinel order_sel_kernel stores for a window it leaves to the rescan launch (a NaN
// payload no computed median has: those windows' results are NaN-free)
constexpr uint32_t kMedSentF32 = 0x7fc0a11du;
constexpr uint64_t kMedSentF64 = 0x7ff80000a11d5eedull;
__device__ __forceinline__ bool is_med_sentinel(const void* out, int f32, int64_t at) {
    return f32 ? reinterpret_cast<const uint32_t*>(out)[at] == kMedSentF32
               : reinterpret_cast<const uint64_t*>(out)[at] == kMedSentF64;
}
__device__ __forceinline__ void store_med_sentinel(void* out, int f32, int64_t at) {
    if (f32) reinterpret_cast<uint32_t*>(out)[at] = kMedSentF32;
    else reinterpret_cast<uint64_t*>(out)[at] = kMedSentF64;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// first index in [lo, hi) whose key is > key (keys sorted ascending)
template <class KT>
__device__ __forceinline__ int upper_bound(const KT* K, int lo, int hi, KT key) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (K[mid] <= key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Bitonic sort of 64 * E keys held in registers, lane l owning positions l*E .. l*E+E-1:
// compare-exchange partners closer than E sit in the same lane, farther ones in lane
// l ^ (j / E) (one ds_bpermute per key), so the network needs no LDS round trips.
template <class KT>
__device__ __forceinline__ KT shfl_xor_key(KT v, int m) {
    if constexpr (sizeof(KT) == 4) {
        return static_cast<KT>(__shfl_xor(static_cast<int>(v), m, 64));
    } else {
        const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(static_cast<uint32_t>(v)), m, 64));
        const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(static_cast<uint32_t>(v >> 32)), m, 64));
        return (static_cast<KT>(hi) << 32) | lo;
    }
}
template <int E, class KT>
__device__ __forceinline__ void bitonic_regs(KT (&v)[E], int lane) {
    constexpr int N = 64 * E;
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= E) {
                const int lm = j / E;
                const bool lower = (lane & lm) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int i = lane * E + e;
                    const bool up = (i & k) == 0;
                    const KT o = shfl_xor_key(v[e], lm);
                    const KT mn = v[e] < o ? v[e] : o, mx = v[e] < o ? o : v[e];
                    v[e] = (lower == up) ? mn : mx;
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if ((e & j) != 0) continue;
                    const int i = lane * E + e;
                    const bool up = (i & k) == 0;
                    const KT x0 = v[e], x1 = v[e + j];
                    const KT mn = x0 < x1 ? x0 : x1, mx = x0 < x1 ? x1 : x0;
                    v[e] = up ? mn : mx;
                    v[e + j] = up ? mx : mn;
                }
            }
        }
    }
}

// the window's samples lane * E + e (padding: 0, keyed as NaN below)
template <int E, class T>
__device__ __forceinline__ void load_regs(T (&raw)[E], const T* src, int64_t ss, int W, int lane) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int t = lane * E + e;
        raw[e] = t < W ? src[t * ss] : T(0);
    }
}

__device__ __forceinline__ uint32_t wave_count(bool p) { return static_cast<uint32_t>(__popcll(__ballot(p))); }
__device__ __forceinline__ double bcast_f64(double v) {
    const uint64_t b = static_cast<uint64_t>(__double_as_longlong(v));
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(b))));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(b >> 32))));
    return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}
// v_cmp_class mask: signalling / quiet NaN, -inf, -0, +0, +inf
constexpr int kSpecialClass = 0x001 | 0x002 | 0x004 | 0x020 | 0x040 | 0x200;
constexpr int kNanInfClass = 0x001 | 0x002 | 0x004 | 0x200;   // v_cmp_class: NaN, -inf, +inf
constexpr int kNegZeroClass = 0x020, kPosZeroClass = 0x040;
__device__ __forceinline__ bool is_special(float v) { return __builtin_amdgcn_classf(v, kSpecialClass); }
__device__ __forceinline__ bool is_special(double v) { return __builtin_amdgcn_class(v, kSpecialClass); }

// ---- the register bitonic network for 32-bit keys without LDS (float32 records): a
// compare-exchange with the key in lane l ^ M (M = j / E, j >= E) takes the partner from
//   M = 1, 2: a DPP quad permutation; M = 8: DPP row_ror:8; M = 4: DPP row_ror:4 / :12
//   selected by lane bit 2; M = 16 / 32: v_permlane16_swap / v_permlane32_swap of the key
//   with itself, which leaves {own, partner} in the two result registers of every lane,
//   so min / max come straight from the pair;
// and which of min / max a lane keeps is a lane predicate of the stage (k, j), one
// v_cndmask per key. Round 4's network (bitonic_regs) moved every
// cross-lane partner through ds_bpermute (one LDS round trip and wait per stage) and built
// the keep-min condition per lane with VALU ops: ~9 lane-ops per compare-exchange.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, false));
}
// lanes whose bit `a` equals their bit `b` (lane-bit masks; 0: the bit "0"), as a plain
// predicate of the lane id — loop-invariant, so the compiler keeps each stage's lane mask
// in an SGPR pair (a v_cndmask operand) instead of recomputing it per window. (Not inline
// asm: a VGPR written by an asm statement is invisible to the compiler's DPP / permlane
// hazard checks, which then omit the two wait states a following DPP read needs.)
__device__ __forceinline__ bool lane_bits_equal(int lane, int a, int b) {
    return ((lane & a) == 0) == ((lane & b) == 0);
}
template <int M>
__device__ __forceinline__ void minmax_xor(uint32_t v, uint32_t& mn, uint32_t& mx) {
    if constexpr (M == 16 || M == 32) {
        const auto pr = M == 16 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                                : __builtin_amdgcn_permlane32_swap(v, v, false, false);
        mn = min(static_cast<uint32_t>(pr[0]), static_cast<uint32_t>(pr[1]));
        mx = max(static_cast<uint32_t>(pr[0]), static_cast<uint32_t>(pr[1]));
    } else {
        uint32_t o;
        if constexpr (M == 1) o = dpp_u32<0xB1>(v);          // quad_perm [1,0,3,2]
        else if constexpr (M == 2) o = dpp_u32<0x4E>(v);     // quad_perm [2,3,0,1]
        else if constexpr (M == 8) o = dpp_u32<0x128>(v);    // row_ror:8
        else {
            static_assert(M == 4, "lane xor partner");
            // bit 2 set: lane - 4 (row_ror:4); clear: lane + 4 (row_ror:12)
            // (both moves unconditionally: a ternary of the two calls is a divergent branch,
            // and a DPP move under a partial EXEC reads disabled source lanes as garbage)
            const uint32_t down = dpp_u32<0x124>(v), up = dpp_u32<0x12C>(v);
            o = (__lane_id() & 4) ? down : up;
        }
        mn = min(v, o);
        mx = max(v, o);
    }
}
template <int B, int L, class F>
__device__ __forceinline__ void ord_sfor(F&& f) {
    if constexpr (B < L) {
        f(std::integral_constant<int, B>{});
        ord_sfor<B + 1, L>(f);
    }
}
template <int E>
__device__ __forceinline__ void bitonic_regs_u32(uint32_t (&v)[E], int lane) {
    constexpr int N = 64 * E;
    ord_sfor<1, 11>([&](auto LK) {
        constexpr int lk = decltype(LK)::value;          // k = 2^lk
        if constexpr ((1 << lk) <= N) {
            constexpr int k = 1 << lk;
            ord_sfor<0, 10>([&](auto LJ) {
                constexpr int lj = lk - 1 - decltype(LJ)::value;   // j = k/2 .. 1
                if constexpr (lj >= 0) {
                    constexpr int j = 1 << lj;
                    if constexpr (j >= E) {
                        // up = (lane & (k / E)) == 0 (k / E = 64 at the last merge: all up);
                        // lower = (lane & (j / E)) == 0; keep min where lower == up
                        constexpr int lm = j / E;
                        const bool keep_min = lane_bits_equal(lane, lm, (k / E) & 63);
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            uint32_t mn, mx;
                            minmax_xor<lm>(v[e], mn, mx);
                            v[e] = keep_min ? mn : mx;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            if ((e & j) != 0) continue;
                            const uint32_t x0 = v[e], x1 = v[e + j];
                            const uint32_t mn = min(x0, x1), mx = max(x0, x1);
                            if (k < E) {
                                // up = ((e & k) == 0): the same for every lane
                                const bool up = (e & k) == 0;
                                v[e] = up ? mn : mx;
                                v[e + j] = up ? mx : mn;
                            } else {
                                const bool up = (lane & ((k / E) & 63)) == 0;
                                v[e] = up ? mn : mx;
                                v[e + j] = up ? mx : mn;
                            }
                        }
                    }
                }
            });
        }
    });
}

// ---- selection without sorting (float32 records, no stats.mode in the call). The bit
// searches below (select_rank_u32 / select_two_u32, restated in tests/test_host.py) were the
// first form; the kernels now call select_range_u32 further down (fewer steps), and the
// interleaved select_multi_u32 is kept for the measured record of §5.5. The order
// statistic of rank k is the largest key P with #{keys < P} <= k, found bit by bit from the
// top: 32 steps of one compare per key (the masks in SGPRs) and a scalar popcount. A
// window's median costs ~32 x (E compares + E + 5 scalar ops) instead of the bitonic
// network's ~36 stages x E compare-exchanges; mode needs the runs of the sorted keys and
// keeps the sort. k is wave-uniform, so P and the thresholds stay scalar.
// min over the wave of u (DPP / permlane butterflies), wave-uniform
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t m) {
    uint32_t mn, mx;
    minmax_xor<1>(m, mn, mx);
    minmax_xor<2>(mn, m, mx);
    minmax_xor<4>(m, mn, mx);
    minmax_xor<8>(mn, m, mx);
    minmax_xor<16>(m, mn, mx);
    minmax_xor<32>(mn, m, mx);
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m)));
}
// The search keeps lo = #{keys < P} and hi = #{keys below the range's top}; once exactly
// one key is left in the range [P, top) it is the answer (k = lo), the smallest key >= P —
// for distinct-valued windows after ~log2(n) + a few steps rather than 32.
// Two steps per exit test (the test is five scalar instructions; a step taken after the
// range is down to one key keeps it there, so the extra step is harmless).
template <int E>
__device__ __forceinline__ uint32_t select_rank_u32(const uint32_t (&v)[E], uint32_t k) {
    k = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k)));
    uint32_t P = 0, lo = 0, hi = 64 * E;
    auto step = [&](uint32_t bit) __attribute__((always_inline)) {
        const uint32_t T = P | bit;
        uint32_t cnt = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) cnt += wave_count(v[e] < T);
        if (cnt <= k) {
            P = T;
            lo = cnt;
        } else {
            hi = cnt;
        }
    };
#pragma unroll
    for (int b = 31; b >= 1; b -= 2) {
        step(1u << b);
        step(1u << (b - 1));
        if (hi - lo == 1) {
            uint32_t m = 0xffffffffu;
#pragma unroll
            for (int e = 0; e < E; ++e) m = min(m, v[e] >= P ? v[e] : 0xffffffffu);
            return wave_min_u32(m);
        }
    }
    return P;
}
// ranks k and k + 1 (k + 1 < the key count) from one search. Early exit: the range [P, top)
// holds exactly rank k, so rank k + 1 is the smallest key >= top (both minima in one
// pass, two interleaved butterflies). A search that runs through bit 0 ends with P = rank
// k and hi = #{keys <= P}: rank k + 1 is P again when hi > k + 1, else the smallest key
// above P.
template <int E>
__device__ __forceinline__ void select_two_u32(const uint32_t (&v)[E], uint32_t k, uint32_t& k0, uint32_t& k1) {
    k = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k)));
    uint32_t P = 0, lo = 0, hi = 64 * E;
    auto step = [&](uint32_t bit) __attribute__((always_inline)) {
        const uint32_t T = P | bit;
        uint32_t cnt = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) cnt += wave_count(v[e] < T);
        if (cnt <= k) {
            P = T;
            lo = cnt;
        } else {
            hi = cnt;
        }
    };
#pragma unroll
    for (int b = 31; b >= 1; b -= 2) {
        step(1u << b);
        step(1u << (b - 1));
        if (hi - lo == 1) {
            // the range is [P, P + 2^(b-1)); it cannot reach 2^32 (a key above rank k exists)
            const uint32_t top = P + (1u << (b - 1));
            uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                m0 = min(m0, v[e] >= P ? v[e] : 0xffffffffu);
                m1 = min(m1, v[e] >= top ? v[e] : 0xffffffffu);
            }
            k0 = wave_min_u32(m0);
            k1 = wave_min_u32(m1);
            return;
        }
    }
    k0 = P;
    if (hi > k + 1) {
        k1 = P;
        return;
    }
    uint32_t m = 0xffffffffu;
#pragma unroll
    for (int e = 0; e < E; ++e) m = min(m, v[e] > P ? v[e] : 0xffffffffu);
    k1 = wave_min_u32(m);
}

// max over the wave (the butterflies of wave_min_u32), wave-uniform
__device__ __forceinline__ uint32_t wave_max_dpp_u32(uint32_t m) {
    uint32_t mn, mx;
    minmax_xor<1>(m, mn, mx);
    minmax_xor<2>(mx, mn, m);
    minmax_xor<4>(m, mn, mx);
    minmax_xor<8>(mx, mn, m);
    minmax_xor<16>(m, mn, mx);
    minmax_xor<32>(mx, mn, m);
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m)));
}
// #{keys < T} over the wave with the popcounts on the VALU: `v_bcnt_u32_b32` reads each
// 32-bit half of a compare mask as its scalar operand, one `v_readfirstlane` returns the
// total (7 of a search step's 13 scalar instructions moved to the vector units; used where
// it measured faster, select_multi_u32's VC). A VALU
// reading an SGPR a VALU compare has just written needs wait states on gfx950, and hipcc
// pads none for an operand read inside an asm string (without them the counts came out
// wrong): all masks are written before the string, mask e is read at least
// E - 1 - e + 2 e VALU instructions after its compare, and the opening `s_nop 1` covers
// the rest (E = 4; other E pad every pair).
template <int E>
__device__ __forceinline__ uint32_t count_below_valu(const uint32_t (&v)[E], uint32_t T) {
    uint32_t m[2 * E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint64_t b = __ballot(v[e] < T);
        m[2 * e] = static_cast<uint32_t>(b);
        m[2 * e + 1] = static_cast<uint32_t>(b >> 32);
    }
    uint32_t acc;
    if constexpr (E == 4) {
        asm("s_nop 1\n\t"
            "v_bcnt_u32_b32 %0, %1, 0\n\tv_bcnt_u32_b32 %0, %2, %0\n\t"
            "v_bcnt_u32_b32 %0, %3, %0\n\tv_bcnt_u32_b32 %0, %4, %0\n\t"
            "v_bcnt_u32_b32 %0, %5, %0\n\tv_bcnt_u32_b32 %0, %6, %0\n\t"
            "v_bcnt_u32_b32 %0, %7, %0\n\tv_bcnt_u32_b32 %0, %8, %0"
            : "=&v"(acc)
            : "s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(m[4]), "s"(m[5]), "s"(m[6]), "s"(m[7]));
    } else {
        asm("s_nop 4\n\tv_bcnt_u32_b32 %0, %1, 0\n\tv_bcnt_u32_b32 %0, %2, %0" : "=&v"(acc) : "s"(m[0]), "s"(m[1]));
#pragma unroll
        for (int i = 2; i < 2 * E; i += 2)
            asm("s_nop 4\n\tv_bcnt_u32_b32 %0, %1, %0\n\tv_bcnt_u32_b32 %0, %2, %0" : "+v"(acc) : "s"(m[i]), "s"(m[i + 1]));
    }
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(acc)));
}
// N independent wave minima at once, stage by stage (each DPP stage a fused
// v_min_u32_dpp — the move's old value is min's identity — and the N chains fill each
// other's DPP wait states); every lane ends with the minimum, returned wave-uniform
template <int N>
__device__ __forceinline__ void wave_min_n(uint32_t (&m)[N]) {
    auto dpp_min = [&](auto ctrl) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            m[i] = min(m[i], static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                                 static_cast<int>(0xffffffffu), static_cast<int>(m[i]),
                                 decltype(ctrl)::value, 0xF, 0xF, false)));
    };
    dpp_min(std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
    dpp_min(std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]: quad minima
    dpp_min(std::integral_constant<int, 0x124>{});   // row_ror:4
    dpp_min(std::integral_constant<int, 0x128>{});   // row_ror:8: row minima in every lane
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const auto pr = __builtin_amdgcn_permlane16_swap(m[i], m[i], false, false);
        m[i] = min(static_cast<uint32_t>(pr[0]), static_cast<uint32_t>(pr[1]));
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const auto pr = __builtin_amdgcn_permlane32_swap(m[i], m[i], false, false);
        m[i] = min(static_cast<uint32_t>(pr[0]), static_cast<uint32_t>(pr[1]));
    }
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m[i])));
}
// Ranks k (and k + 1) of one window's keys by a search over the key range itself rather
// than its bits: the range [P, Q] starts at the wave's minimum and maximum key; the first
// three thresholds are interpolated in value space (the float values of P and Q, the
// wanted rank's position between lo and hi — a sinusoid-plus-noise axis is close to
// linear there), the rest halve [P, Q]. Any threshold in (P, Q] keeps the invariants
// lo = #{< P} <= k < hi = #{<= Q}; the search ends when one key is left (hi - lo = 1) or the
// range is one value (P = Q, ties). Then rank k is the smallest key >= P, rank k + 1 the
// same value when hi > k + 1, else the smallest key > Q. (Host emulation of the bench
// data: 7.1 search steps with three interpolated thresholds, 8.0 with two, against the bit
// search's 12.2; measured 2 / 3 / 4: cfg2med 1.29-1.31 / 1.23-1.26 / 1.22-1.23 ms, cfg2ord
// 4.53 / 4.45 / 4.51 ms — MHF_SEL_NINTERP = 3.)
__device__ __forceinline__ float key_value(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
template <int E, bool VC>
__device__ __forceinline__ void select_range_u32(const uint32_t (&v)[E], uint32_t k, bool two,
                                                 uint32_t& k0, uint32_t& k1) {
    k = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k)));
    uint32_t ext[2];
    {
        uint32_t mn = v[0], mx = v[0];
#pragma unroll
        for (int e = 1; e < E; ++e) {
            mn = min(mn, v[e]);
            mx = max(mx, v[e]);
        }
        ext[0] = mn;
        ext[1] = ~mx;
    }
    wave_min_n<2>(ext);
    uint32_t P = ext[0], Q = ~ext[1], lo = 0, hi = 64 * E;
    auto count = [&](uint32_t T) __attribute__((always_inline)) -> uint32_t {
        if constexpr (VC) {
            return count_below_valu<E>(v, T);
        } else {
            uint32_t c = 0;
#pragma unroll
            for (int e = 0; e < E; ++e) c += wave_count(v[e] < T);
            return c;
        }
    };
    auto step = [&](uint32_t T) __attribute__((always_inline)) {
        const uint32_t cnt = count(T);
        if (cnt <= k) {
            P = T;
            lo = cnt;
        } else {
            Q = T - 1u;
            hi = cnt;
        }
    };
#ifndef MHF_SEL_NINTERP
#define MHF_SEL_NINTERP 3
#endif
#pragma unroll
    for (int it = 0; it < MHF_SEL_NINTERP; ++it) {
        if (hi - lo <= 1u || Q <= P) break;
        const float a = key_value(P), b = key_value(Q);
        const float fr = (static_cast<float>(k - lo) + 0.5f) * __builtin_amdgcn_rcpf(static_cast<float>(hi - lo));
        const float t = a + (b - a) * fr;
        const uint32_t tb = __float_as_uint(t);
        uint32_t T = tb ^ (static_cast<uint32_t>(static_cast<int32_t>(tb) >> 31) | 0x80000000u);
        T = min(max(T, P + 1u), Q);   // (a NaN / inf guess lands on an end)
        step(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(T))));
    }
#pragma unroll 1
    while (hi - lo > 1u && Q > P) step(P + ((Q - P) >> 1) + 1u);
    uint32_t fm[2];
    fm[0] = 0xffffffffu;
    fm[1] = 0xffffffffu;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        fm[0] = min(fm[0], v[e] >= P ? v[e] : 0xffffffffu);
        fm[1] = min(fm[1], v[e] > Q ? v[e] : 0xffffffffu);
    }
    wave_min_n<2>(fm);
    k0 = fm[0];
    k1 = (two && hi <= k + 1u) ? fm[1] : fm[0];
}

// Ranks k (and k + 1) of NC windows' keys at once (the CV channels of one AoS window):
// the NC searches run interleaved step by step, so one wave carries NC independent
// dependency chains (compare -> popcount -> scalar decision -> next threshold) instead of
// one, and each search starts below the bits its keys share: P = the common prefix of the
// wave's minimum and maximum key, the first threshold bit the highest bit where they differ
// (z axes near 1 g share their top 8 bits — 8 of their ~20 steps). A search whose range
// [P, P + bit) holds one key (hi - lo = 1), or whose bits are used up, is done; the loop
// stops when all are, and steps taken after a search is done keep its range (at
// bit = 0 a step tests T = P: #{< P} = lo <= k). Then per search, with top = the end of the
// last range: rank k is the smallest key >= P, rank k + 1 the same key when more than
// k + 1 keys are below top, else the smallest key >= top. Bit-identical to select_two_u32 /
// select_rank_u32 (the values at ranks are keys either way).
template <int E, int NC, bool VC = false>
__device__ __forceinline__ void select_multi_u32(const uint32_t (&v)[NC][E], uint32_t k, bool two,
                                                 uint32_t (&k0)[NC], uint32_t (&k1)[NC]) {
    k = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k)));
    uint32_t P[NC], lo[NC], hi[NC], bit[NC];
    uint32_t ext[2 * NC];   // minima, then complemented maxima (max x = ~min ~x)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        uint32_t mn = v[c][0], mx = v[c][0];
#pragma unroll
        for (int e = 1; e < E; ++e) {
            mn = min(mn, v[c][e]);
            mx = max(mx, v[c][e]);
        }
        ext[c] = mn;
        ext[NC + c] = ~mx;
    }
    wave_min_n<2 * NC>(ext);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t mn = ext[c], mx = ~ext[NC + c];
        const uint32_t d = mn ^ mx;
        const uint32_t hb = d ? (0x80000000u >> __builtin_clz(d)) : 0u;
        P[c] = mn & ~((hb << 1) - 1u);   // hb = 2^31: the mask is 0 (no shared bits)
        if (!hb) P[c] = mn;
        lo[c] = 0;
        hi[c] = 64 * E;
        bit[c] = hb;
    }
    auto step = [&](int c) __attribute__((always_inline)) {
        const uint32_t T = P[c] | bit[c];
        uint32_t cnt = 0;
        if constexpr (VC) {
            cnt = count_below_valu<E>(v[c], T);
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) cnt += wave_count(v[c][e] < T);
        }
        if (cnt <= k) {
            P[c] = T;
            lo[c] = cnt;
        } else {
            hi[c] = cnt;
        }
        bit[c] >>= 1;
    };
    // (ends by itself: every bit is 0 after 32 steps; min(x, bit) != 0 iff both are)
#pragma unroll 1
    for (;;) {
#pragma unroll
        for (int c = 0; c < NC; ++c) step(c);
#pragma unroll
        for (int c = 0; c < NC; ++c) step(c);
        uint32_t open = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) open |= min(hi[c] - lo[c] - 1u, bit[c]);
        if (!open) break;
    }
    // both minima of every search in one interleaved reduction (the top of a search that
    // needs no rank k + 1 may wrap: its minimum is not used)
    uint32_t fm[2 * NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t top = P[c] + (bit[c] ? bit[c] << 1 : 1u);
        uint32_t m0 = 0xffffffffu, m1 = 0xffffffffu;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            m0 = min(m0, v[c][e] >= P[c] ? v[c][e] : 0xffffffffu);
            m1 = min(m1, v[c][e] >= top ? v[c][e] : 0xffffffffu);
        }
        fm[c] = m0;
        fm[NC + c] = two ? m1 : 0xffffffffu;
    }
    if (two) {
        wave_min_n<2 * NC>(fm);
    } else {
        uint32_t f0[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) f0[c] = fm[c];
        wave_min_n<NC>(f0);
#pragma unroll
        for (int c = 0; c < NC; ++c) fm[c] = f0[c];
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        k0[c] = fm[c];
        k1[c] = (two && hi[c] <= k + 1) ? fm[NC + c] : fm[c];
    }
}

// CV > 0 (float32 AoS records of CV = 1 or 3 channels, fixed windows, E >= 4): lane l's
// samples l E .. l E + E - 1 of every channel are C E consecutive floats, loaded as
// dwordx4s for the whole window at once, and the next window's loads are issued before the
// current one is worked on (the selection path is short enough for the load latency to
// dominate otherwise)
template <int E, int CV>
__device__ __forceinline__ void load_window_vec(float (&f)[CV * E], const float* p, int lane) {
    // every lane's C E floats lie inside the record and start 16-B aligned (launch_order
    // checks the record, the stride and the first window); samples past a shorter window
    // are read but keyed as padding
    const float4* q = reinterpret_cast<const float4*>(p + static_cast<int64_t>(lane) * E * CV);
#pragma unroll
    for (int j = 0; j < CV * E / 4; ++j) {
        const float4 v = q[j];
        f[4 * j] = v.x;
        f[4 * j + 1] = v.y;
        f[4 * j + 2] = v.z;
        f[4 * j + 3] = v.w;
    }
}

// E > 0: every window of the launch sorts (or selects) in registers (64 * E >= its padded
// length); E = 0: sort through LDS (windows beyond 1024 samples, indexed windows)
template <int E, class T = float, int CV = 0>
__global__ void __launch_bounds__(256, (E >= 16 ? 2 : 4)) order_kernel(OrdArgs a) {
    constexpr bool kVec = CV > 0;
    static_assert(!kVec || (E >= 4 && sizeof(T) == 4), "vector window loads: float32, E >= 4");
    typedef Keys<T> KY;
    typedef typename KY::K KT;
    constexpr KT kNanKey = KY::kNan, kNegZeroKey = KY::kNegZero, kPosZeroKey = KY::kPosZero,
                 kPosInfKey = KY::kPosInf, kNegInfKey = KY::kNegInf;
    auto kval = [](KT k) { return KY::val(k); };
    auto is_zero_key = [](KT k) { return k == KY::kNegZero || k == KY::kPosZero; };
    extern __shared__ __attribute__((aligned(16))) uint32_t ord_lds[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int C = kVec ? CV : a.channels;
    // (the vector-load instantiation only runs fixed windows in LDS: prune the rest)
    const int64_t* const starts = kVec ? nullptr : a.starts;
    void* const gkeys = kVec ? nullptr : a.gkeys;
    KT* region = gkeys ? reinterpret_cast<KT*>(gkeys) +
                               (static_cast<int64_t>(blockIdx.x) * a.waves + wid) * C * a.cap
                         : reinterpret_cast<KT*>(ord_lds) + static_cast<int64_t>(wid) * C * a.cap;
    bool want_med = false, want_pct = false, want_iqr = false, want_mode = false;
    for (int j = 0; j < a.feats.n; ++j) {
        want_med |= a.feats.id[j] == MHF_MEDIAN;
        want_pct |= a.feats.id[j] == MHF_PERCENTILE;
        want_iqr |= a.feats.id[j] == MHF_IQR;
        want_mode |= !kVec && a.feats.id[j] == MHF_MODE;   // (kVec launches have no mode)
    }
    // output slots: jq[q] = the position of order feature q (median, percentile, IQR,
    // mode) in the call's list; one slot lane per (channel, q) unless a feature repeats or
    // the channels need more than 64 lanes (then lane 0 stores each output itself)
    // (four scalars, not an array written at a runtime index: that would live in scratch)
    int jq0 = -1, jq1 = -1, jq2 = -1, jq3 = -1;
    bool dup = false;
    for (int j = 0; j < a.feats.n; ++j) {
        const int f = a.feats.id[j];
        auto put = [&](int& d) {
            dup |= d >= 0;
            d = d >= 0 ? d : j;
        };
        if (f == MHF_MEDIAN) put(jq0);
        else if (f == MHF_PERCENTILE) put(jq1);
        else if (f == MHF_IQR) put(jq2);
        else if (f == MHF_MODE) put(jq3);
    }
    const int jq[4] = {jq0, jq1, jq2, jq3};
    const bool slots = !dup && 4 * C <= 64;
    // rank selection in registers instead of the sort (select_rank_u32)
    constexpr bool kCanSelect = E > 0 && sizeof(KT) == 4;
    const bool sel = kVec || (kCanSelect && !want_mode);   // kVec: no sort compiled in
    const int64_t stride = static_cast<int64_t>(gridDim.x) * a.waves;
    float nxt[kVec ? CV * E : 1];                // kVec: the next window's samples
    if constexpr (kVec) {
        const int64_t i0 = static_cast<int64_t>(blockIdx.x) * a.waves + wid;
        if (i0 < a.nwin)
            load_window_vec<E, CV>(nxt, a.x + (a.first + i0) * a.wstep * CV, lane);
    }
    // a window's slot outputs are stored one iteration later, after the next window's loads
    // are issued: stores and loads share vmcnt, so a store issued at the end of an iteration
    // would hold the next iteration's wait for its prefetched loads to the store's ack
    double p_val = 0.0;
    int64_t p_row = -1, p_i = 0;
    // the next window: i + stride, or in a rescan launch the next window whose sentinel
    // this wave finds (64 windows' output slots read per step, this wave's blocks of 64)
    uint64_t rs_pend = 0;
    int64_t rs_base = 0, rs_next = (static_cast<int64_t>(blockIdx.x) * a.waves + wid) * 64;
    auto next_window = [&](int64_t cur) -> int64_t {
        if (kVec || !a.rescan) return cur + stride;
        while (rs_pend == 0) {
            if (rs_next >= a.nwin) return a.nwin;
            const int64_t j = rs_next + lane;
            const bool f = j < a.nwin && is_med_sentinel(a.out, a.out_f32, a.rescan_row * a.out_ld + j);
            rs_pend = __ballot(f);
            rs_base = rs_next;
            rs_next += stride * 64;
        }
        const int b = __builtin_ctzll(rs_pend);
        rs_pend &= rs_pend - 1;
        return rs_base + b;
    };
    const int64_t i_first = (kVec || !a.rescan) ? static_cast<int64_t>(blockIdx.x) * a.waves + wid
                                                : next_window(0);
    for (int64_t i = i_first; i < a.nwin; i = next_window(i)) {
        float win[kVec ? CV * E : 1];
        if constexpr (kVec) {
#pragma unroll
            for (int j = 0; j < CV * E; ++j) win[j] = nxt[j];
            if (i + stride < a.nwin)
                load_window_vec<E, CV>(nxt, a.x + (a.first + i + stride) * a.wstep * CV, lane);
        }
        if (p_row >= 0) store_out(a.out, a.out_f32, p_row * a.out_ld + p_i, p_val);
        p_row = -1;
        // ---- the window
        int64_t s0, W64;
        bool keep = true;
        if (starts) {
            const int64_t si = starts[i], ei = a.ends[i], n = a.n_samples;
            int64_t b0 = si < 0 ? si + n : si, e0 = ei < 0 ? ei + n : ei;
            b0 = b0 < 0 ? 0 : (b0 > n ? n : b0);
            e0 = e0 < 0 ? 0 : (e0 > n ? n : e0);
            s0 = b0;
            W64 = e0 > b0 ? e0 - b0 : 0;
            keep = (ei - si >= a.min_len) && W64 > 0 && W64 <= a.cap;
            // long-window split (see OrdArgs): each window is written by exactly one launch
            const bool is_long = (ei - si >= a.min_len) && W64 > (gkeys ? a.short_cap : a.cap);
            if (gkeys ? !is_long : (a.skip_long && is_long)) continue;
        } else {
            s0 = (a.first + i) * a.wstep;
            W64 = a.wsize;
        }
        const int W = keep ? static_cast<int>(W64) : 0;
        int np2 = 1;
        while (np2 < W) np2 <<= 1;
        double o_val = NAN;
        int64_t o_row = -1;
#pragma unroll 1
        for (int c = 0; c < C; ++c) {
            KT* K = region + static_cast<int64_t>(c) * a.cap;
            const T* src;
            if constexpr (sizeof(T) == 8) src = a.xd + c * a.ch_stride + s0 * a.sample_stride;
            else src = a.x + c * a.ch_stride + s0 * a.sample_stride;
            double r_med = NAN, r_pct = NAN, r_iqr = NAN, r_mode = NAN;
            if (keep) {
                // ---- keys, padded to a power of two with NaN keys, then bitonic sort: in
                // registers up to 1024 keys, through LDS beyond
                // counts of the register path (E > 0): non-NaN elements, zeros by sign,
                // infinities — ballots over the unsorted keys (the LDS path counts below)
                uint32_t rc_nv = 0, rc_zn = 0, rc_zp = 0, rc_ip = 0, rc_in = 0;
                KT v[E > 0 ? E : 1];
                if constexpr (E > 0) {
                    T cur[E];
                    if constexpr (kVec) {
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            // (a runtime channel: selects, not a dynamically indexed array)
                            float f = win[e * CV];
#pragma unroll
                            for (int cc = 1; cc < CV; ++cc) f = c == cc ? win[e * CV + cc] : f;
                            cur[e] = f;
                        }
                    } else {
                        load_regs<E, T>(cur, src, a.sample_stride, W, lane);
                    }
                    // NaN / signed zero / infinity counts only for the windows holding one
                    // (one class test per sample finds them)
                    uint64_t special = 0;
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int t = lane * E + e;
                        v[e] = t < W ? KY::key(cur[e]) : kNanKey;
                        special |= __ballot(t < W && is_special(cur[e]));
                    }
                    rc_nv = static_cast<uint32_t>(W);
                    if (special) {
                        rc_nv = 0;
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int t = lane * E + e;
                            rc_nv += wave_count(t < W && v[e] != kNanKey);
                            rc_zn += wave_count(v[e] == kNegZeroKey);
                            rc_zp += wave_count(v[e] == kPosZeroKey);
                            rc_ip += wave_count(v[e] == kPosInfKey);
                            rc_in += wave_count(v[e] == kNegInfKey);
                        }
                    }
                    if (!sel) {
                        if constexpr (sizeof(KT) == 4) bitonic_regs_u32<E>(v, lane);
                        else bitonic_regs<E, KT>(v, lane);
#pragma unroll
                        for (int e = 0; e < E; ++e) K[lane * E + e] = v[e];
                        __builtin_amdgcn_wave_barrier();
                    }
                    np2 = 64 * E;
                } else {
                    for (int t = lane; t < np2; t += 64) K[t] = t < W ? KY::key(src[t * a.sample_stride]) : kNanKey;
                    __builtin_amdgcn_wave_barrier();
                    for (int k = 2; k <= np2; k <<= 1) {
                        for (int j = k >> 1; j > 0; j >>= 1) {
                            for (int p = lane; p < (np2 >> 1); p += 64) {
                                const int lo = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                                const int hi = lo + j;
                                const KT ka = K[lo], kb = K[hi];
                                const bool up = (lo & k) == 0;
                                const KT mn = ka < kb ? ka : kb, mx = ka < kb ? kb : ka;
                                K[lo] = up ? mn : mx;
                                K[hi] = up ? mx : mn;
                            }
                            __builtin_amdgcn_wave_barrier();
                        }
                    }
                }
                // ---- counts: non-NaN elements, zeros by sign, infinities
                uint32_t nv = rc_nv, nz_neg = rc_zn, nz_pos = rc_zp, ninf_pos = rc_ip, ninf_neg = rc_in;
                if constexpr (E == 0) {
                    for (int t = lane; t < W; t += 64) {
                        const KT kk = K[t];
                        nv += kk != kNanKey;
                        nz_neg += kk == kNegZeroKey;
                        nz_pos += kk == kPosZeroKey;
                        ninf_pos += kk == kPosInfKey;
                        ninf_neg += kk == kNegInfKey;
                    }
                    nv = wave_sum_u32(nv);
                    nz_neg = wave_sum_u32(nz_neg);
                    nz_pos = wave_sum_u32(nz_pos);
                    ninf_pos = wave_sum_u32(ninf_pos);
                    ninf_neg = wave_sum_u32(ninf_neg);
                }
                const bool mixed0 = nz_neg > 0 && nz_pos > 0;
                const int n = W;
                const bool has_nan = static_cast<int>(nv) < n;
                bool replay_med = false, replay_pct = false, replay_iqr = false, replay_mode = false;
                // order statistic keys (NaN-free ranks): rank k, ranks k and k + 1
                auto os = [&](int k) __attribute__((always_inline)) -> KT {
                    if constexpr (kCanSelect)
                        if (sel) {
                            // the range search of the selection kernel (select_range_u32)
                            uint32_t r0, r1;
                            select_range_u32<E, false>(v, static_cast<uint32_t>(k), false, r0, r1);
                            return r0;
                        }
                    return K[k];
                };
                auto os2 = [&](int k, KT& k0, KT& k1) __attribute__((always_inline)) {
                    if constexpr (kCanSelect) {
                        if (sel) {
                            select_range_u32<E, false>(v, static_cast<uint32_t>(k), true, k0, k1);
                            return;
                        }
                    }
                    k0 = K[k];
                    k1 = K[k + 1];
                };
                // ---- np.median
                if (want_med) {
                    if (has_nan) replay_med = true;
                    else if (n & 1) {
                        const KT k1 = os(n >> 1);
                        if (mixed0 && is_zero_key(k1)) replay_med = true;
                        else r_med = static_cast<double>(kval(k1));
                    } else {
                        KT k0, k1;
                        os2((n >> 1) - 1, k0, k1);
                        if (mixed0 && (is_zero_key(k0) || is_zero_key(k1))) replay_med = true;
                        else r_med = static_cast<double>(kval(k0) + kval(k1)) / 2.0;
                    }
                }
                // ---- np.percentile / interquartile_range (no NaN: linear interpolation
                // between order statistics; q = 0 / 100: min / max + numba's inf rules)
                auto pct = [&](double q, bool& replay) __attribute__((always_inline)) -> double {
                    if (n == 1) return static_cast<double>(kval(os(0)));   // finite here
                    if (q == 100.0) {
                        const KT kk = os(n - 1);
                        if (mixed0 && is_zero_key(kk)) { replay = true; return 0.0; }
                        double v = static_cast<double>(kval(kk));
                        if ((ninf_pos + ninf_neg) > 0 && std::isinf(v)) v = NAN;
                        return v;
                    }
                    if (q == 0.0) {
                        const KT kk = os(0);
                        if (mixed0 && is_zero_key(kk)) { replay = true; return 0.0; }
                        double v = static_cast<double>(kval(kk));
                        if (ninf_pos + ninf_neg > 0) {
                            const int nfin = n - static_cast<int>(ninf_pos + ninf_neg);
                            if (nfin == 0) v = NAN;
                            if (ninf_pos == 1 && n == 2) v = NAN;
                            if (ninf_neg > 1) v = NAN;
                            if (nfin == 1 && ninf_pos > 1 && ninf_neg != 1) v = NAN;
                        }
                        return v;
                    }
                    const Rank rk = pct_rank(n, q);
                    KT k0, k1;
                    os2(rk.k, k0, k1);
                    if (mixed0 && (is_zero_key(k0) || is_zero_key(k1))) { replay = true; return 0.0; }
                    return pct_interp(static_cast<double>(kval(k0)), static_cast<double>(kval(k1)), rk.m);
                };
                auto pct_ok = [&]() __attribute__((always_inline)) { return !has_nan && (n != 1 || std::isfinite(kval(os(0)))); };
                if (want_pct) {
                    if (pct_ok()) r_pct = pct(a.q, replay_pct);
                }
                if (want_iqr) {
                    if (pct_ok()) {
                        bool rp = false;
                        const double hi = pct(75.0, rp), lo = pct(25.0, rp);
                        if (rp) replay_iqr = true;
                        else r_iqr = hi - lo;
                    }
                }
                // ---- stats.mode: runs of equal values in sorted order (+0 / -0 one run,
                // each NaN its own run); the first run counts one short, ties go to the
                // earlier run, the value is the run's last element (numba's e1)
                if (want_mode) {
                    if (nv == 0) {
                        r_mode = static_cast<double>(kval(kNanKey));   // all NaN: x[0]
                    } else {
                        // best = (effective count << 16) | (0xffff - run start)
                        uint32_t best = 0;
                        for (int t = lane; t < static_cast<int>(nv); t += 64) {
                            const KT kk = K[t];
                            const bool start = t == 0 || !(K[t - 1] == kk ||
                                                           (is_zero_key(K[t - 1]) && is_zero_key(kk)));
                            if (!start) continue;
                            const int ub = upper_bound<KT>(K, t + 1, static_cast<int>(nv),
                                                           is_zero_key(kk) ? kPosZeroKey : kk);
                            int L = static_cast<int>(ub) - t;
                            if (t == 0) L = L >= 3 ? L - 1 : 1;
                            const uint32_t cand = (static_cast<uint32_t>(L) << 16) | (0xffffu - t);
                            best = cand > best ? cand : best;
                        }
                        best = wave_max_u32(best);
                        const int cnt = static_cast<int>(best >> 16);
                        const int st = static_cast<int>(0xffffu - (best & 0xffffu));
                        int pos;
                        if (cnt <= 1) pos = 0;                       // nothing beat x[0]
                        else {
                            const KT kk = K[st];
                            pos = upper_bound<KT>(K, st + 1, static_cast<int>(nv),
                                                  is_zero_key(kk) ? kPosZeroKey : kk) - 1;
                        }
                        const KT kk = K[pos];
                        if (mixed0 && is_zero_key(kk)) replay_mode = true;
                        else r_mode = static_cast<double>(kval(kk));
                    }
                }
                // ---- serial numba replays on a float copy of the window (rare windows)
                if (replay_med || replay_pct || replay_iqr || replay_mode) {
                    T* A = reinterpret_cast<T*>(K);
                    auto reload = [&]() {
                        __builtin_amdgcn_wave_barrier();
                        for (int t = lane; t < W; t += 64) A[t] = src[t * a.sample_stride];
                        __builtin_amdgcn_wave_barrier();
                    };
                    if (replay_med) {
                        reload();
                        if (lane == 0) r_med = nb_median(A, n);
                    }
                    if (replay_pct || replay_iqr) {
                        // numba: one float64 copy, the selections of each q in order
                        auto replay_q = [&](double q) -> double {
                            if (q == 100.0 || q == 0.0) {
                                double v = nb_first_extreme(A, n, q == 100.0);
                                if (q == 100.0 && (ninf_pos + ninf_neg) > 0 && std::isinf(v)) v = NAN;
                                if (q == 0.0 && ninf_pos + ninf_neg > 0) {
                                    const int nfin = n - static_cast<int>(ninf_pos + ninf_neg);
                                    if (nfin == 0 || (ninf_pos == 1 && n == 2) || ninf_neg > 1 ||
                                        (nfin == 1 && ninf_pos > 1 && ninf_neg != 1))
                                        v = NAN;
                                }
                                return v;
                            }
                            const Rank rk = pct_rank(n, q);
                            T lo, hi;
                            nb_select_two(A, rk.k, 0, n - 1, lo, hi);
                            return pct_interp(static_cast<double>(lo), static_cast<double>(hi), rk.m);
                        };
                        if (replay_pct) {
                            reload();
                            if (lane == 0) r_pct = replay_q(a.q);
                        }
                        if (replay_iqr) {
                            reload();
                            if (lane == 0) {
                                const double hi = replay_q(75.0);
                                const double lo = replay_q(25.0);
                                r_iqr = hi - lo;
                            }
                        }
                    }
                    if (replay_mode) {
                        reload();
                        if (lane == 0) r_mode = nb_mode(A, n);
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            // ---- outputs (NaN for indexed windows below min_len): lane 4 c + q takes order
            // feature q of channel c (lane 0's values: the serial replays run there), and the
            // window's outputs leave in ONE store instruction after its last channel — so
            // the next window's prefetched loads need no wait for these stores' acks
            if (slots) {
                const double rv[4] = {r_med, r_pct, r_iqr, r_mode};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (jq[q] < 0) continue;                 // (uniform: features not asked)
                    const double v = bcast_f64(rv[q]);
                    if (lane == 4 * c + q) {
                        o_val = v;
                        o_row = static_cast<int64_t>(c) * a.feats.n + jq[q];
                    }
                }
            } else if (lane == 0) {
                for (int j = 0; j < a.feats.n; ++j) {
                    const int f = a.feats.id[j];
                    double v;
                    if (f == MHF_MEDIAN) v = r_med;
                    else if (f == MHF_PERCENTILE) v = r_pct;
                    else if (f == MHF_IQR) v = r_iqr;
                    else if (f == MHF_MODE) v = r_mode;
                    else continue;
                    store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i, v);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (slots) {
            p_val = o_val;
            p_row = o_row;
            p_i = i;
        }
    }
    if (p_row >= 0) store_out(a.out, a.out_f32, p_row * a.out_ld + p_i, p_val);
}

// np.median / np.percentile / interquartile_range (no stats.mode) over float32 AoS
// records of CV = 1 / 3 channels, fixed windows (the vector-load shape of
// order_kernel<E, float, CV>): per order statistic asked for, the CV channels' rank searches
// run interleaved (select_multi_u32) on keys built without NaN / padding tests; a window
// holding a NaN, a zero or an infinity gets a sentinel in channel 0's first order-feature
// slot and is left to a second launch of order_kernel in rescan mode (its counts,
// signed-zero and infinity rules, numba replays). Nothing else compiled in: the kernel fits
// 8 waves per SIMD where order_kernel<E, float, CV> (sort, mode and replay code in the same
// register allocation) ran at 4.
// (MED: the call's only order feature is np.median — one search per window, compiled
// without the statistics loop)
template <int E, int CV, bool MED>
__global__ void __launch_bounds__(256, (E * CV > 24 ? 2 : (E * CV > 12 ? 4 : 8))) order_sel_kernel(OrdArgs a) {
    typedef Keys<float> KY;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int W = static_cast<int>(a.wsize);
    const int64_t stride = static_cast<int64_t>(gridDim.x) * a.waves;
    const int64_t F = a.feats.n;
    // the call's order features (the launcher sends each at most once)
    int jmed = -1, jpct = -1, jiqr = -1;
    for (int j = 0; j < a.feats.n; ++j) {
        const int f = a.feats.id[j];
        if (f == MHF_MEDIAN) jmed = j;
        else if (f == MHF_PERCENTILE) jpct = j;
        else if (f == MHF_IQR) jiqr = j;
    }
    float nxt[CV * E];
    const int64_t i0 = static_cast<int64_t>(blockIdx.x) * a.waves + wid;
    if (i0 < a.nwin) load_window_vec<E, CV>(nxt, a.x + (a.first + i0) * a.wstep * CV, lane);
    // stores one iteration late, after the next window's loads (they share vmcnt); lane
    // 4 c + q holds channel c's order feature q (0 median, 1 percentile, 2 IQR)
    double p_val = 0.0;
    int64_t p_at = -1;
    bool p_sent = false;
    for (int64_t i = i0; i < a.nwin; i += stride) {
        float win[CV * E];
#pragma unroll
        for (int j = 0; j < CV * E; ++j) win[j] = nxt[j];
        if (i + stride < a.nwin)
            load_window_vec<E, CV>(nxt, a.x + (a.first + i + stride) * a.wstep * CV, lane);
        if (p_at >= 0) {
            if (p_sent) store_med_sentinel(a.out, a.out_f32, p_at);
            else store_out(a.out, a.out_f32, p_at, p_val);
        }
        p_at = -1;
        uint32_t vk[CV][E];
        // windows order_kernel must replay: a NaN or an infinity, or zeros of BOTH signs
        // (numba's comparisons tie -0 with +0, the keys do not); zeros of one sign alone
        // — zero-padded or integer-quantized records — keep the selection
        // (one class test per key — NaN, inf or either zero — and the three-way split only
        // for a window that holds one of them: three ballots per key on every window cost
        // cfg2med 1.22 -> 1.36 ms, measured)
        uint64_t any_sp = 0;
        auto key_of = [](float f) __attribute__((always_inline)) {
            const uint32_t b = __float_as_uint(f);
            return b ^ (static_cast<uint32_t>(static_cast<int32_t>(b) >> 31) | 0x80000000u);
        };
        if (W == 64 * E) {
#pragma unroll
            for (int cc = 0; cc < CV; ++cc)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const float f = win[e * CV + cc];
                    vk[cc][e] = key_of(f);
                    any_sp |= __ballot(is_special(f));
                }
        } else {
#pragma unroll
            for (int cc = 0; cc < CV; ++cc)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int t = lane * E + e;
                    const float f = win[e * CV + cc];
                    vk[cc][e] = t < W ? key_of(f) : KY::kNan;
                    any_sp |= __ballot(t < W && is_special(f));
                }
        }
        bool special = false;
        if (any_sp) {
            uint64_t nan_inf = 0, neg0 = 0, pos0 = 0;
#pragma unroll
            for (int cc = 0; cc < CV; ++cc)
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const bool in = W == 64 * E || lane * E + e < W;
                    const float f = win[e * CV + cc];
                    nan_inf |= __ballot(in && __builtin_amdgcn_classf(f, kNanInfClass));
                    neg0 |= __ballot(in && __builtin_amdgcn_classf(f, kNegZeroClass));
                    pos0 |= __ballot(in && __builtin_amdgcn_classf(f, kPosZeroClass));
                }
            special = nan_inf != 0 || (neg0 != 0 && pos0 != 0);
        }
        if (!special) {
            // one interleaved search per statistic: 0 the median, 1 the percentile, 2 / 3
            // the IQR's q = 75 / 25 (order_kernel's pct: q = 100 / 0 the extreme key, else
            // numba's linear interpolation between ranks k and k + 1)
            double iqr_hi[CV];
#pragma unroll
            for (int cc = 0; cc < CV; ++cc) iqr_hi[cc] = 0.0;
#pragma unroll 1
            for (int t = 0; t < (MED ? 1 : 4); ++t) {
                const int q = t < 3 ? t : 2;
                const int j = q == 0 ? jmed : (q == 1 ? jpct : jiqr);
                if (j < 0) continue;
                const double qq = t == 1 ? a.q : (t == 2 ? 75.0 : 25.0);
                uint32_t k;
                bool two;
                int kind;              // 0 median, 1 one rank, 2 interpolation
                double m = 0.0;
                if (t == 0) {
                    k = static_cast<uint32_t>((W - 1) >> 1);
                    two = (W & 1) == 0;
                    kind = 0;
                } else if (qq == 100.0 || qq == 0.0) {
                    k = qq == 100.0 ? static_cast<uint32_t>(W - 1) : 0u;
                    two = false;
                    kind = 1;
                } else {
                    const Rank rk = pct_rank(W, qq);
                    k = static_cast<uint32_t>(rk.k);
                    two = true;
                    m = rk.m;
                    kind = 2;
                }
                // the channels one after another: at 8 waves per SIMD the other waves hide a
                // search's latency, and a joint loop would run every channel for as many
                // steps as the slowest needs (measured: 1.49 interleaved -> 1.32 ms)
                uint32_t r0[CV], r1[CV];
#pragma unroll
                for (int cc = 0; cc < CV; ++cc) {
                    const uint32_t (&vc)[1][E] = *reinterpret_cast<const uint32_t (*)[1][E]>(&vk[cc]);
                    uint32_t s0[1], s1[1];
                    // (popcounts on the VALU for the statistics loop: cfg2ord 5.72 -> 5.44 ms;
                    // the median alone measured 1.33 -> 1.37 ms with them, so scalar there)
#ifdef MHF_SEL_BITS
                    select_multi_u32<E, 1, !MED>(vc, k, two, s0, s1);
#else
                    select_range_u32<E, !MED>(vc[0], k, two, s0[0], s1[0]);
#endif
                    r0[cc] = s0[0];
                    r1[cc] = s1[0];
                }
#pragma unroll
                for (int cc = 0; cc < CV; ++cc) {
                    double v;
                    if (kind == 0)
                        v = (W & 1) ? static_cast<double>(KY::val(r0[cc]))
                                    : static_cast<double>(KY::val(r0[cc]) + KY::val(r1[cc])) / 2.0;
                    else if (kind == 1)
                        v = static_cast<double>(KY::val(r0[cc]));
                    else
                        v = pct_interp(static_cast<double>(KY::val(r0[cc])), static_cast<double>(KY::val(r1[cc])), m);
                    if (t == 2) {
                        iqr_hi[cc] = v;
                        continue;
                    }
                    if (t == 3) v = iqr_hi[cc] - v;
                    if (lane == 4 * cc + q) {
                        p_val = v;
                        p_at = (cc * F + j) * a.out_ld + i;
                    }
                }
            }
            p_sent = false;
        } else {
            if (lane == 0) p_at = a.rescan_row * a.out_ld + i;
            p_sent = true;
        }
    }
    if (p_at >= 0) {
        if (p_sent) store_med_sentinel(a.out, a.out_f32, p_at);
        else store_out(a.out, a.out_f32, p_at, p_val);
    }
}

// A window's samples into LDS with 8 global loads in flight per lane before their LDS
// stores (one load + wait + store per sample left every load's latency exposed)
template <class T>
__device__ __forceinline__ void stage_lds(T* X, const T* src, int64_t ss, int n, int lane) {
    for (int t0 = 0; t0 < n; t0 += 64 * 8) {
        T v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int t = t0 + 64 * k + lane;
            v[k] = t < n ? src[t * ss] : T(0);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int t = t0 + 64 * k + lane;
            if (t < n) X[t] = v[k];
        }
    }
}

// ---------------------------------------------------------------- sample entropy
// information.sampen(x, mm, r, sd) (src/mhealth/generic/information.py:23-113). The
// reference walks every pair i < j row by row keeping, per diagonal d = j - i, the length
// of the current run of matches |x[j] - x[i]| < r (fp32 difference, compared in float64):
// a match of run length L adds 1 to a[m] for m < min(mm+1, L) and to b[m] as well when
// j < n - 1; b is then shifted one place and b[0] = n (n - 1) / 2; the result is
// -log(a[M] / b[M]) with M = mm (the reference increments mm first). So, with
// L(i, j) the diagonal run length:  A = #(L >= mm + 1),  B = #(L >= mm, L > 0, j <= n - 2)
// (B = n (n - 1) / 2 for mm = 0), both exact integer counts. r = r * sd, sd = the
// window's fp32 np.std when None. float64 records (T = double): the differences, the std
// and the threshold test in fp64.
//
// MI355X layout (round 5): a wave takes 64 consecutive windows at a time.
//   * r per window: lane l runs window l's np.std sums (numba's sequential order) straight
//     from global memory — the two serial passes (2 W dependent steps) once per 64 windows
//     instead of once per window in every lane;
//   * then window by window: the window in LDS, lane l walking the two snake diagonals
//     d1 = 64 q + l + 1 and d2 = 64 q + 128 - l of round pair q in step (x[i] is one
//     broadcast read for both, x[i + d1] / x[i + d2] conflict-free across lanes), each as
//     32-position match words: bit 31 - k of word p0 is [|x[p0+k+d] - x[p0+k]| < r]. A run
//     of length >= L ends at a position exactly when it and its L - 1 predecessors match,
//     so with the previous word's bits shifted in (v_alignbit)
//         A += popc(w & w>>1 & .. & w>>mm),  B += popc(w & .. & w>>(mB-1))  (mB = max(mm,1))
//     and the last position of each diagonal (j = n - 1) is masked out of B. Per pair test:
//     a subtract, a compare and a shift-insert — round 4's walk carried the run length
//     through a compare -> select -> two count updates per step (23 lane-ops per pair, 1.2e10
//     VALU wave-instructions for 1e6 windows of 256).
// mm > 30 (the shifts would leave one word of history) takes the run-length walk.
template <class T>
__device__ __forceinline__ T sampen_r(const T* p, int64_t ss, int n, double rfac, double sd_in) {
    // r *= sd if sd is not None else x.std() (numba array_std: fp32 mean, fp64 sum of fp32
    // squared deviations, fp32 variance, fp32 sqrt of it; float64 records: fp64 throughout);
    // returned as the threshold t with  (double)diff < r  <=>  diff < t
    double r = rfac;
    if (sizeof(T) == 8 && std::isnan(sd_in)) {
        double s = 0.0;
        for (int t = 0; t < n; ++t) s = s + static_cast<double>(p[t * ss]);
        const double m = s / static_cast<double>(n);
        double ssd = 0.0;
        for (int t = 0; t < n; ++t) {
            const double d = static_cast<double>(p[t * ss]) - m;
            ssd = ssd + d * d;
        }
        r = rfac * sqrt(ssd / static_cast<double>(n));
    } else if (std::isnan(sd_in)) {
        // contiguous 16-B aligned windows: the lane reads its window a float4 at a time (one
        // lane per window, so the scalar loads of 64 lanes touched 64 lines per instruction
        // and the lines left L2 between a lane's consecutive loads: 8 x the input fetched
        // from HBM, profiles/r05c_sampen256_summary.md); the sums stay sequential
        const bool vec = sizeof(T) == 4 && ss == 1 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
        const int n4 = vec ? (n & ~3) : 0;
        const float4* p4 = reinterpret_cast<const float4*>(p);
        float s = 0.0f;
        for (int t = 0; t < n4; t += 4) {
            const float4 q = p4[t >> 2];
            s = s + q.x;
            s = s + q.y;
            s = s + q.z;
            s = s + q.w;
        }
        for (int t = n4; t < n; ++t) s = s + static_cast<float>(p[t * ss]);
        const float m32 = static_cast<float>(static_cast<double>(s) / static_cast<double>(n));
        double ssd = 0.0;
        for (int t = 0; t < n4; t += 4) {
            const float4 q = p4[t >> 2];
            const float d0 = q.x - m32, d1 = q.y - m32, d2 = q.z - m32, d3 = q.w - m32;
            ssd = ssd + static_cast<double>(d0 * d0);
            ssd = ssd + static_cast<double>(d1 * d1);
            ssd = ssd + static_cast<double>(d2 * d2);
            ssd = ssd + static_cast<double>(d3 * d3);
        }
        for (int t = n4; t < n; ++t) {
            const float d = static_cast<float>(p[t * ss]) - m32;
            ssd = ssd + static_cast<double>(d * d);
        }
        const float var32 = static_cast<float>(ssd / static_cast<double>(n));
        r = rfac * static_cast<double>(static_cast<float>(sqrt(static_cast<double>(var32))));
    } else {
        r = rfac * sd_in;
    }
    if constexpr (sizeof(T) == 8) {
        return r;
    } else {
        float t32 = static_cast<float>(r);
        if (static_cast<double>(t32) < r) t32 = nextafterf(t32, INFINITY);
        return t32;
    }
}

// w = 2 w + [|df| < t]: the compare into VCC (the abs as an operand modifier) and one
// add-with-carry shifting the match bit in (the compiler's select + shift + or took 2.5)
template <class T>
__device__ __forceinline__ void match_insert(uint32_t& w, T df, T t) {
    if constexpr (sizeof(T) == 8)
        asm("v_cmp_lt_f64_e64 vcc, |%1|, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
            : "+v"(w) : "v"(df), "v"(t) : "vcc");
    else
        asm("v_cmp_lt_f32_e64 vcc, |%1|, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
            : "+v"(w) : "v"(df), "v"(t) : "vcc");
}

// Two positions of two streams at once: w1 = 4 w1 + [|a0| < t] 2 + [|a1| < t], w2 the same
// with b0, b1. Four compares into four SGPR pairs, then the four add-with-carries: every
// carry is read three VALU instructions after its compare (the mask-read wait states are
// inside the string), and hipcc pads one state per statement instead of one per position.
__device__ __forceinline__ void match_insert4(uint32_t& w1, uint32_t& w2, float a0, float b0, float a1,
                                             float b1, float t) {
    uint64_t c0, c1, c2, c3;
    asm("v_cmp_lt_f32_e64 %[c0], |%[a0]|, %[t]\n\t"
        "v_cmp_lt_f32_e64 %[c1], |%[b0]|, %[t]\n\t"
        "v_cmp_lt_f32_e64 %[c2], |%[a1]|, %[t]\n\t"
        "v_cmp_lt_f32_e64 %[c3], |%[b1]|, %[t]\n\t"
        "v_addc_co_u32_e64 %[w1], %[c0], %[w1], %[w1], %[c0]\n\t"
        "v_addc_co_u32_e64 %[w2], %[c1], %[w2], %[w2], %[c1]\n\t"
        "v_addc_co_u32_e64 %[w1], %[c2], %[w1], %[w1], %[c2]\n\t"
        "v_addc_co_u32_e64 %[w2], %[c3], %[w2], %[w2], %[c3]"
        : [w1] "+v"(w1), [w2] "+v"(w2), [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3)
        : [a0] "v"(a0), [b0] "v"(b0), [a1] "v"(a1), [b1] "v"(b1), [t] "s"(t));
}

// A, B of one window in LDS (X, n samples, padded by 64 readable slots) — bit words
template <class T, int MM>
__device__ __forceinline__ void sampen_words(const T* X, int n, T t, int mm_rt, int lane, uint32_t& A,
                                             uint32_t& B) {
    const int mm = MM >= 0 ? MM : mm_rt;                 // MM: compile-time mm (-1: runtime)
    const int mB = mm < 1 ? 1 : mm;
    const int nd = n - 1;                                // diagonals d = 1 .. n-1
    for (int q = 0; q * 64 < nd; q += 2) {
        const int d1 = 64 * q + lane + 1, d2 = 64 * q + 128 - lane;
        const int len1 = d1 <= nd ? n - d1 : 0, len2 = d2 <= nd ? n - d2 : 0;
        const int lmax = len1 > len2 ? len1 : len2;
        uint32_t prev1 = 0, prev2 = 0;
        for (int p0 = 0; p0 < lmax; p0 += 32) {
            uint32_t w1 = 0, w2 = 0;
            // one base address per stream, the 32 positions at immediate offsets
            const T* pi = X + p0;
            const T* pa = pi + d1;
            const T* pb = pi + d2;
#pragma unroll
            for (int k0 = 0; k0 < 32; k0 += 8) {
                T xi[8], xa[8], xb[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    xi[k] = pi[k0 + k];
                    xa[k] = pa[k0 + k];
                    xb[k] = pb[k0 + k];
                }
                if constexpr (sizeof(T) == 4) {
                    // two differences per v_pk_add_f32 (each still one fp32 subtraction)
#pragma unroll
                    for (int k = 0; k < 8; k += 2) {
                        typedef float f2v __attribute__((ext_vector_type(2)));
                        const f2v i2 = {xi[k], xi[k + 1]};
                        const f2v da = f2v{xa[k], xa[k + 1]} - i2, db = f2v{xb[k], xb[k + 1]} - i2;
                        match_insert<T>(w1, da.x, t);
                        match_insert<T>(w2, db.x, t);
                        match_insert<T>(w1, da.y, t);
                        match_insert<T>(w2, db.y, t);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        match_insert<T>(w1, xa[k] - xi[k], t);
                        match_insert<T>(w2, xb[k] - xi[k], t);
                    }
                }
            }
            // positions past each diagonal's end are no match; B drops the last position
            const int r1 = len1 - p0, r2 = len2 - p0;
            const uint32_t keep1 = r1 >= 32 ? ~0u : (r1 <= 0 ? 0u : ~0u << (32 - r1));
            const uint32_t keep2 = r2 >= 32 ? ~0u : (r2 <= 0 ? 0u : ~0u << (32 - r2));
            const uint32_t lastB1 = (r1 >= 1 && r1 <= 32) ? ~(1u << (32 - r1)) : ~0u;
            const uint32_t lastB2 = (r2 >= 1 && r2 <= 32) ? ~(1u << (32 - r2)) : ~0u;
            w1 &= keep1;
            w2 &= keep2;
            uint32_t a1 = w1, b1 = w1, a2 = w2, b2 = w2;
#pragma unroll
            for (int sh = 1; sh <= (MM >= 0 ? MM : 30); ++sh) {
                if (MM < 0 && sh > mm) break;
                const uint32_t s1 = __builtin_amdgcn_alignbit(prev1, w1, sh);
                const uint32_t s2 = __builtin_amdgcn_alignbit(prev2, w2, sh);
                a1 &= s1;
                a2 &= s2;
                if (sh < mB) {
                    b1 &= s1;
                    b2 &= s2;
                }
            }
            A += __popc(a1) + __popc(a2);
            B += __popc(b1 & lastB1) + __popc(b2 & lastB2);
            prev1 = w1;
            prev2 = w2;
        }
    }
}

// Cyclic diagonals (the default walk when the doubled window fits in LDS): the pairs
// (i, (i + d) mod n), i = 0 .. n-1, are diagonal d (i < n - d) followed by diagonal n - d
// (its first index i + d - n) — with the window stored twice in LDS (XX[i] = XX[i + n] =
// x[i]) one contiguous stream of exactly n positions. The (n-1)/2 cyclic diagonals
// d = 1 .. (n-1)/2 (plus d = n/2 over its first n/2 positions for even n) cover every
// diagonal once, every stream as long as the window, so the lanes (two streams each, in
// step) never idle: sampen_words' pairs of straight diagonals ran to the longer one's end
// (2 x 256 slots per lane for 2 x 191 pairs on average at n = 256: 66 % busy).
// Inside a stream the run chains restart at the boundary b = n - d: A drops positions
// [b, b + mm), B positions [b, b + mB - 1) and both diagonals' last positions b - 1, L - 1.
//
// bits of the positions [lo, lo + len) (len <= 32) in the match word of positions
// p0 .. p0 + 31 (position p at bit 31 - (p - p0))
__device__ __forceinline__ uint32_t pos_bits(int lo, int len, int p0) {
    const uint64_t M = ((len >= 32 ? ~0ull : ((1ull << len) - 1))) << 32;
    int sh = lo - p0 + len;
    sh = sh < 0 ? 0 : (sh > 64 ? 64 : sh);
    return sh >= 64 ? 0u : static_cast<uint32_t>(M >> sh);
}
template <class T, int MM>
__device__ __forceinline__ void sampen_cyclic(const T* XX, int n, T t, int mm_rt, int lane, uint32_t& A,
                                              uint32_t& B) {
    const int mm = MM >= 0 ? MM : mm_rt;
    const int mB = mm < 1 ? 1 : mm;
    const int ncyc = (n - 1) >> 1;
    const int nstr = ncyc + ((n & 1) == 0 ? 1 : 0);
    for (int s0 = 0; s0 < nstr; s0 += 128) {
        const int e1 = s0 + lane, e2 = s0 + 64 + lane;
        // stream length (0: no stream), cyclic diagonal, boundary
        const int len1 = e1 < ncyc ? n : (e1 < nstr ? (n >> 1) : 0);
        const int len2 = e2 < ncyc ? n : (e2 < nstr ? (n >> 1) : 0);
        const int d1 = len1 > 0 ? e1 + 1 : 1, d2 = len2 > 0 ? e2 + 1 : 1;
        const int b1 = n - d1, b2 = n - d2;
        // the boundary masks of the two words around b - 1 (half streams: b = L, nothing past)
        const int kb1 = ((b1 - 1) >> 5) << 5, kb2 = ((b2 - 1) >> 5) << 5;
        const bool two1 = b1 < len1, two2 = b2 < len2;
        const uint32_t cA10 = two1 ? pos_bits(b1, mm, kb1) : 0u, cA11 = two1 ? pos_bits(b1, mm, kb1 + 32) : 0u;
        const uint32_t cA20 = two2 ? pos_bits(b2, mm, kb2) : 0u, cA21 = two2 ? pos_bits(b2, mm, kb2 + 32) : 0u;
        const uint32_t cB10 = (two1 ? pos_bits(b1, mB - 1, kb1) : 0u) | pos_bits(b1 - 1, 1, kb1);
        const uint32_t cB11 = (two1 ? pos_bits(b1, mB - 1, kb1 + 32) : 0u);
        const uint32_t cB20 = (two2 ? pos_bits(b2, mB - 1, kb2) : 0u) | pos_bits(b2 - 1, 1, kb2);
        const uint32_t cB21 = (two2 ? pos_bits(b2, mB - 1, kb2 + 32) : 0u);
        const int lmax = len1 > len2 ? len1 : len2;
        uint32_t prev1 = 0, prev2 = 0;
        for (int p0 = 0; p0 < lmax; p0 += 32) {
            uint32_t w1 = 0, w2 = 0;
            const T* pi = XX + p0;
            const T* pa = pi + d1;
            const T* pb = pi + d2;
#pragma unroll
            for (int k0 = 0; k0 < 32; k0 += 8) {
                T xi[8], xa[8], xb[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    xi[k] = pi[k0 + k];
                    xa[k] = pa[k0 + k];
                    xb[k] = pb[k0 + k];
                }
                if constexpr (sizeof(T) == 4) {
#pragma unroll
                    for (int k = 0; k < 8; k += 2) {
                        typedef float f2v __attribute__((ext_vector_type(2)));
                        const f2v i2 = {xi[k], xi[k + 1]};
                        const f2v da = f2v{xa[k], xa[k + 1]} - i2, db = f2v{xb[k], xb[k + 1]} - i2;
                        match_insert4(w1, w2, da.x, db.x, da.y, db.y, t);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        match_insert<T>(w1, xa[k] - xi[k], t);
                        match_insert<T>(w2, xb[k] - xi[k], t);
                    }
                }
            }
            // positions past each stream's end are no match; B drops the stream's last one
            const int r1 = len1 - p0, r2 = len2 - p0;
            const uint32_t keep1 = r1 >= 32 ? ~0u : (r1 <= 0 ? 0u : ~0u << (32 - r1));
            const uint32_t keep2 = r2 >= 32 ? ~0u : (r2 <= 0 ? 0u : ~0u << (32 - r2));
            const uint32_t lastB1 = (r1 >= 1 && r1 <= 32) ? (1u << (32 - r1)) : 0u;
            const uint32_t lastB2 = (r2 >= 1 && r2 <= 32) ? (1u << (32 - r2)) : 0u;
            w1 &= keep1;
            w2 &= keep2;
            uint32_t a1 = w1, bb1 = w1, a2 = w2, bb2 = w2;
#pragma unroll
            for (int sh = 1; sh <= (MM >= 0 ? MM : 30); ++sh) {
                if (MM < 0 && sh > mm) break;
                const uint32_t s1 = __builtin_amdgcn_alignbit(prev1, w1, sh);
                const uint32_t s2 = __builtin_amdgcn_alignbit(prev2, w2, sh);
                a1 &= s1;
                a2 &= s2;
                if (sh < mB) {
                    bb1 &= s1;
                    bb2 &= s2;
                }
            }
            // the boundary's restarted chains
            const uint32_t mA1 = p0 == kb1 ? cA10 : (p0 == kb1 + 32 ? cA11 : 0u);
            const uint32_t mA2 = p0 == kb2 ? cA20 : (p0 == kb2 + 32 ? cA21 : 0u);
            const uint32_t mB1 = (p0 == kb1 ? cB10 : (p0 == kb1 + 32 ? cB11 : 0u)) | lastB1;
            const uint32_t mB2 = (p0 == kb2 ? cB20 : (p0 == kb2 + 32 ? cB21 : 0u)) | lastB2;
            A += __popc(a1 & ~mA1) + __popc(a2 & ~mA2);
            B += __popc(bb1 & ~mB1) + __popc(bb2 & ~mB2);
            prev1 = w1;
            prev2 = w2;
        }
    }
}

// the run-length walk (mm > 30): two snake diagonals in step, counts as (L + 2^31 - m) >> 31
template <class T>
__device__ __forceinline__ void sampen_runs(const T* X, int n, T t, int mm, int lane, uint32_t& A,
                                            uint32_t& B) {
    const uint32_t mA = static_cast<uint32_t>(mm + 1);
    const uint32_t mB = static_cast<uint32_t>(mm < 1 ? 1 : mm);
    const uint32_t cA = 0x80000000u - mA, cB = 0x80000000u - mB;
    auto step = [&](uint32_t& L, T xi, T xj) {
        L = (fabs(xj - xi) < t) ? L + 1 : 0;
        A += (L + cA) >> 31;
        B += (L + cB) >> 31;
    };
    const int nd = n - 1;
    for (int q = 0; q * 64 < nd; q += 2) {
        const int d1 = 64 * q + lane + 1, d2 = 64 * q + 128 - lane;
        const int len1 = d1 <= nd ? n - d1 : 0, len2 = d2 <= nd ? n - d2 : 0;
        uint32_t L1 = 0, L2 = 0;
        const int lmax = len1 > len2 ? len1 : len2;
        for (int ii = 0; ii < lmax; ++ii) {
            if (ii < len1) step(L1, X[ii], X[ii + d1]);
            if (ii < len2) step(L2, X[ii], X[ii + d2]);
        }
        // the step at j = n - 1 of each walked diagonal
        if (len1 > 0) B -= (L1 + cB) >> 31;
        if (len2 > 0) B -= (L2 + cB) >> 31;
    }
}

template <class T = float>
__global__ void __launch_bounds__(256, 4) sampen_kernel(OrdArgs a, int32_t mm, double rfac,
                                                     double sd_in) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ord_lds[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the window stored twice for the cyclic-diagonal walk when it fits (launch_sampen)
    const bool cyc = (a.sampen_cyc != 0);
    T* X = reinterpret_cast<T*>(ord_lds) + static_cast<int64_t>(wid) * ((cyc ? 2 : 1) * a.cap + 64);
    int col = -1;
    for (int j = 0; j < a.feats.n && col < 0; ++j)
        if (a.feats.id[j] == MHF_SAMPEN) col = j;
    const int64_t gstride = static_cast<int64_t>(gridDim.x) * a.waves * 64;
    for (int64_t g0 = (static_cast<int64_t>(blockIdx.x) * a.waves + wid) * 64; g0 < a.nwin; g0 += gstride) {
        // ---- lane l: window g0 + l
        const int64_t il = g0 + lane;
        int64_t s0 = 0, W64 = 0;
        bool keep = il < a.nwin, skip = il >= a.nwin;
        if (keep && a.starts) {
            const int64_t si = a.starts[il], ei = a.ends[il], nn = a.n_samples;
            int64_t b0 = si < 0 ? si + nn : si, e0 = ei < 0 ? ei + nn : ei;
            b0 = b0 < 0 ? 0 : (b0 > nn ? nn : b0);
            e0 = e0 < 0 ? 0 : (e0 > nn ? nn : e0);
            s0 = b0;
            W64 = e0 > b0 ? e0 - b0 : 0;
            keep = (ei - si >= a.min_len) && W64 > 0 && W64 <= a.cap;
            // long-window split (see OrdArgs): each window is written by exactly one launch
            const bool is_long = (ei - si >= a.min_len) && W64 > (a.gkeys ? a.short_cap : a.cap);
            skip = a.gkeys ? !is_long : (a.skip_long && is_long);
        } else if (keep) {
            s0 = (a.first + il) * a.wstep;
            W64 = a.wsize;
        }
        const int nl = keep && !skip ? static_cast<int>(W64) : 0;
        const int nwg = a.nwin - g0 < 64 ? static_cast<int>(a.nwin - g0) : 64;
        for (int c = 0; c < a.channels; ++c) {
            const T* srcl;
            if constexpr (sizeof(T) == 8) srcl = a.xd + c * a.ch_stride + s0 * a.sample_stride;
            else srcl = a.x + c * a.ch_stride + s0 * a.sample_stride;
            const T tl = nl > 0 ? sampen_r<T>(srcl, a.sample_stride, nl, rfac, sd_in) : T(0);
            for (int w = 0; w < nwg; ++w) {
                if (__builtin_amdgcn_readlane(static_cast<int>(skip), w)) continue;
                const int n = __builtin_amdgcn_readlane(nl, w);
                double res = NAN;
                if (n > 0) {
                    const int64_t sw = (static_cast<int64_t>(static_cast<uint32_t>(
                                            __builtin_amdgcn_readlane(static_cast<int>(s0 >> 32), w))) << 32) |
                                       static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(s0), w));
                    const T* src;
                    if constexpr (sizeof(T) == 8) src = a.xd + c * a.ch_stride + sw * a.sample_stride;
                    else src = a.x + c * a.ch_stride + sw * a.sample_stride;
                    stage_lds<T>(X, src, a.sample_stride, n, lane);
                    if (cyc) stage_lds<T>(X + n, src, a.sample_stride, n, lane);   // XX = x x
                    __builtin_amdgcn_wave_barrier();
                    T t;
                    if constexpr (sizeof(T) == 8) {
                        const uint64_t tb = __double_as_longlong(tl);
                        t = __longlong_as_double(static_cast<long long>(
                            (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(tb >> 32), w))) << 32) |
                            static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(tb), w))));
                    } else {
                        t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tl), w));
                    }
                    uint32_t A = 0, B = 0;
                    if (cyc && mm == 2) sampen_cyclic<T, 2>(X, n, t, mm, lane, A, B);
                    else if (cyc && mm == 1) sampen_cyclic<T, 1>(X, n, t, mm, lane, A, B);
                    else if (cyc && mm <= 30) sampen_cyclic<T, -1>(X, n, t, mm, lane, A, B);
                    else if (mm == 2) sampen_words<T, 2>(X, n, t, mm, lane, A, B);
                    else if (mm == 1) sampen_words<T, 1>(X, n, t, mm, lane, A, B);
                    else if (mm <= 30) sampen_words<T, -1>(X, n, t, mm, lane, A, B);
                    else sampen_runs<T>(X, n, t, mm, lane, A, B);
                    A = wave_sum_u32(A);
                    B = wave_sum_u32(B);
                    const double bden = mm == 0 ? static_cast<double>(n) * static_cast<double>(n - 1) / 2.0
                                                : static_cast<double>(B);
                    res = -log(static_cast<double>(A) / bden);
                    __builtin_amdgcn_wave_barrier();
                }
                if (lane == 0 && col >= 0)
                    store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + col) * a.out_ld + g0 + w, res);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// ---------------------------------------------------------------- recurrence quantification
// rqa.recurrence_rate / determinism / laminarity / length_entropy of the window's
// recurrence matrix rq(x, radius) (src/mhealth/generic/rqa.py:9-187), without building it:
// r is symmetric, so one walk over the diagonals d = 1 .. n-1 (snake-assigned to lanes,
// counted twice) plus the main one gives the recurrence count, the points on diagonal
// lines of >= 2 points (determinism) and the line-length histogram (length_entropy; a
// line of all n points is dropped, as the reference's _dlen_counts writes it past its
// array); laminarity's horizontal lines need a walk over the rows. Counts are exact
// integers; the ratios and the entropy are evaluated as the reference does (float64,
// sequential over the histogram bins).
template <class T = float>
__global__ void __launch_bounds__(256) rqa_kernel(OrdArgs a, double radius, int32_t minlen) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ord_lds[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int kXw = sizeof(T) / 4;                // dwords per sample
    uint32_t* region = ord_lds + static_cast<int64_t>(wid) * ((kXw + 1) * a.cap + 2);
    T* X = reinterpret_cast<T*>(region);
    uint32_t* H = region + kXw * a.cap;               // histogram bins 0 .. cap
    bool want_lam = false, want_ent = false;   // recurrence rate, determinism: always computed
    for (int j = 0; j < a.feats.n; ++j) {
        want_lam |= a.feats.id[j] == MHF_RQA_LAM;
        want_ent |= a.feats.id[j] == MHF_RQA_ENT;
    }
    // (double)|dx| <= radius  <=>  |dx| <= t32 (the largest float not above radius;
    // float64 records: radius itself)
    T t32;
    if constexpr (sizeof(T) == 8) {
        t32 = radius;
    } else {
        t32 = static_cast<float>(radius);
        if (static_cast<double>(t32) > radius) t32 = nextafterf(t32, -INFINITY);
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * a.waves;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * a.waves + wid; i < a.nwin; i += stride) {
        int64_t s0, W64;
        bool keep = true;
        if (a.starts) {
            const int64_t si = a.starts[i], ei = a.ends[i], nn = a.n_samples;
            int64_t b0 = si < 0 ? si + nn : si, e0 = ei < 0 ? ei + nn : ei;
            b0 = b0 < 0 ? 0 : (b0 > nn ? nn : b0);
            e0 = e0 < 0 ? 0 : (e0 > nn ? nn : e0);
            s0 = b0;
            W64 = e0 > b0 ? e0 - b0 : 0;
            keep = (ei - si >= a.min_len) && W64 > 0 && W64 <= a.cap;
            // long-window split (see OrdArgs): each window is written by exactly one launch
            const bool is_long = (ei - si >= a.min_len) && W64 > (a.gkeys ? a.short_cap : a.cap);
            if (a.gkeys ? !is_long : (a.skip_long && is_long)) continue;
        } else {
            s0 = (a.first + i) * a.wstep;
            W64 = a.wsize;
        }
        const int n = keep ? static_cast<int>(W64) : 0;
        for (int c = 0; c < a.channels; ++c) {
            double rr = NAN, det = NAN, lam = NAN, ent = NAN;
            if (n > 0) {
                const T* src;
                if constexpr (sizeof(T) == 8) src = a.xd + c * a.ch_stride + s0 * a.sample_stride;
                else src = a.x + c * a.ch_stride + s0 * a.sample_stride;
                stage_lds<T>(X, src, a.sample_stride, n, lane);
                for (int t = lane; t <= n; t += 64) H[t] = 0;
                __builtin_amdgcn_wave_barrier();
                uint32_t nrec = 0, ndet = 0, nends = 0;      // nends: lines of >= 2 points
                auto run_end = [&](uint32_t L, uint32_t mult, bool main) {
                    if (L >= 2) {
                        ndet += L * mult;
                        nends += mult;
                        if (want_ent && static_cast<int>(L) >= minlen && !(main && static_cast<int>(L) == n))
                            atomicAdd(&H[L], mult);
                    }
                };
                // diagonals d >= 1 (and their mirror images)
                const int nd = n - 1;
                for (int q = 0; q * 64 < nd; ++q) {
                    const int d = (q & 1) ? 64 * q + 64 - lane : 64 * q + lane + 1;
                    if (d > nd) continue;
                    uint32_t L = 0;
                    for (int ii = 0; ii + d < n; ++ii) {
                        const bool rec = fabs(X[ii + d] - X[ii]) <= t32;
                        nrec += rec ? 2u : 0u;
                        if (rec) ++L;
                        else { run_end(L, 2, false); L = 0; }
                    }
                    run_end(L, 2, false);
                }
                // the main diagonal (|x_i - x_i| = 0 unless x_i is NaN or +-inf)
                if (lane == 0) {
                    uint32_t L = 0;
                    for (int ii = 0; ii < n; ++ii) {
                        const bool rec = fabs(X[ii] - X[ii]) <= t32;
                        nrec += rec ? 1u : 0u;
                        if (rec) ++L;
                        else { run_end(L, 1, true); L = 0; }
                    }
                    run_end(L, 1, true);
                }
                // laminarity: horizontal lines of >= 2 points, row by row
                uint32_t nlam = 0;
                if (want_lam) {
                    for (int row = lane; row < n; row += 64) {
                        const T xr = X[row];
                        uint32_t L = 0;
                        for (int jj = 0; jj < n; ++jj) {
                            if (fabs(xr - X[jj]) <= t32) ++L;
                            else { nlam += L >= 2 ? L : 0; L = 0; }
                        }
                        nlam += L >= 2 ? L : 0;
                    }
                }
                nrec = wave_sum_u32(nrec);
                ndet = wave_sum_u32(ndet);
                nends = wave_sum_u32(nends);
                nlam = wave_sum_u32(nlam);
                const double nn2 = static_cast<double>(static_cast<int64_t>(n) * n);
                rr = static_cast<double>(nrec) / nn2;
                if (n >= 2) {
                    det = static_cast<double>(ndet) / nn2;
                    lam = static_cast<double>(nlam) / nn2;
                }
                __builtin_amdgcn_wave_barrier();
                if (want_ent && lane == 0) {
                    // information.entropy(counts[minlen:]): counts of line lengths; with
                    // minlen 1 the "1" bin holds every other matrix entry
                    if (minlen <= 1)
                        H[1] = static_cast<uint32_t>(static_cast<int64_t>(n) * n - nends);
                    int64_t tot = 0;
                    for (int v = minlen < 1 ? 1 : minlen; v < n; ++v) tot += H[v];
                    double e = 0.0;
                    for (int v = minlen; v < n; ++v) {
                        double qv = (v >= 1 ? static_cast<double>(H[v]) : 0.0) / static_cast<double>(tot);
                        qv = qv + 1e-30;
                        e = e + qv * log(qv);
                    }
                    ent = -e;
                }
            }
            if (lane == 0) {
                for (int j = 0; j < a.feats.n; ++j) {
                    const int f = a.feats.id[j];
                    double v;
                    if (f == MHF_RQA_RR) v = rr;
                    else if (f == MHF_RQA_DET) v = det;
                    else if (f == MHF_RQA_LAM) v = lam;
                    else if (f == MHF_RQA_ENT) v = ent;
                    else continue;
                    store_out(a.out, a.out_f32, (static_cast<int64_t>(c) * a.feats.n + j) * a.out_ld + i, v);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace

int launch_sampen(const OrderLaunch& L, int32_t mm, double r, double sd, hipStream_t stream) {
    OrdArgs a{};
    a.x = L.x; a.ch_stride = L.ch_stride; a.sample_stride = L.sample_stride; a.wsize = L.wsize;
    a.wstep = L.wstep; a.first = L.first; a.nwin = L.nwin; a.channels = L.channels;
    a.starts = L.starts; a.ends = L.ends; a.n_samples = L.n_samples; a.min_len = L.min_len;
    a.feats = L.feats; a.out = L.out; a.out_ld = L.out_ld; a.out_f32 = L.out_f32;
    a.xd = L.xd;
    a.cap = static_cast<int32_t>(L.starts ? L.max_w : L.wsize);
    if (a.cap < 1) a.cap = 1;
    // the window (twice for the cyclic-diagonal walk, when that fits) plus 64 readable
    // slots past it (the match words read up to 31 past the last sample of a stream)
    const int64_t es = L.xd ? 8 : 4;
    a.sampen_cyc = (2 * static_cast<int64_t>(a.cap) + 64) * es <= kOrderLdsBytes && !disabled("MHF_NO_SAMPEN_CYC");
    const int64_t per_wave = ((a.sampen_cyc ? 2 : 1) * static_cast<int64_t>(a.cap) + 64) * es;
    // the window length limit of the host plans (kMaxOrderSamples float32 / half that for
    // float64 records: make_plan, mhf_window_features_f64); one wave then needs at most
    // (16384 + 64) x 4 B = 65,792 B (float64: 66,048 B) of dynamic LDS — past 64 KiB, within
    // gfx950's 160 KiB per workgroup (the old per-wave byte bound also admitted
    // float32 windows of 16,385 .. 16,448 samples)
    if (a.cap > (L.xd ? kMaxOrderSamples / 2 : kMaxOrderSamples)) return MHF_EUNSUPPORTED;
    a.waves = static_cast<int>(kOrderLdsBytes / per_wave >= 4 ? 4 : kOrderLdsBytes / per_wave);
    if (a.waves < 1) a.waves = 1;
    // 64 windows per wave (sampen_kernel)
    int64_t blocks = (L.nwin + 64 * a.waves - 1) / (64 * a.waves);
    if (blocks > 8192) blocks = 8192;
    if (L.xd)
        hipLaunchKernelGGL(sampen_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(64 * a.waves),
                           static_cast<size_t>(per_wave * a.waves), stream, a, mm, r, sd);
    else
        hipLaunchKernelGGL(sampen_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(64 * a.waves),
                           static_cast<size_t>(per_wave * a.waves), stream, a, mm, r, sd);
    return MHF_OK;
}

int launch_rqa(const OrderLaunch& L, double radius, int32_t minlen, hipStream_t stream) {
    OrdArgs a{};
    a.x = L.x; a.ch_stride = L.ch_stride; a.sample_stride = L.sample_stride; a.wsize = L.wsize;
    a.wstep = L.wstep; a.first = L.first; a.nwin = L.nwin; a.channels = L.channels;
    a.starts = L.starts; a.ends = L.ends; a.n_samples = L.n_samples; a.min_len = L.min_len;
    a.feats = L.feats; a.out = L.out; a.out_ld = L.out_ld; a.out_f32 = L.out_f32;
    a.xd = L.xd;
    a.cap = static_cast<int32_t>(L.starts ? L.max_w : L.wsize);
    if (a.cap < 1) a.cap = 1;
    const int64_t per_wave = ((L.xd ? 3 : 2) * static_cast<int64_t>(a.cap) + 2) * 4;
    if (per_wave > kOrderLdsBytes) return MHF_EUNSUPPORTED;
    a.waves = static_cast<int>(kOrderLdsBytes / per_wave >= 4 ? 4 : kOrderLdsBytes / per_wave);
    int64_t blocks = (L.nwin + a.waves - 1) / a.waves;
    if (blocks > 8192) blocks = 8192;
    if (L.xd)
        hipLaunchKernelGGL(rqa_kernel<double>, dim3(static_cast<unsigned>(blocks)), dim3(64 * a.waves),
                           static_cast<size_t>(per_wave * a.waves), stream, a, radius, minlen);
    else
        hipLaunchKernelGGL(rqa_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(64 * a.waves),
                           static_cast<size_t>(per_wave * a.waves), stream, a, radius, minlen);
    return MHF_OK;
}

int launch_order(const OrderLaunch& L, hipStream_t stream) {
    OrdArgs a{};
    a.x = L.x; a.ch_stride = L.ch_stride; a.sample_stride = L.sample_stride; a.wsize = L.wsize;
    a.wstep = L.wstep; a.first = L.first; a.nwin = L.nwin; a.channels = L.channels;
    a.starts = L.starts; a.ends = L.ends; a.n_samples = L.n_samples; a.min_len = L.min_len;
    a.q = L.q; a.feats = L.feats; a.out = L.out; a.out_ld = L.out_ld; a.out_f32 = L.out_f32;
    a.xd = L.xd;
    const bool f64 = L.xd != nullptr;
    int cap = 1;
    const int64_t want = L.starts ? L.max_w : L.wsize;
    while (cap < want) cap <<= 1;
    if (cap < 64) cap = 64;
    const int64_t per_wave = static_cast<int64_t>(L.channels) * cap * (f64 ? 8 : 4);
    if (per_wave > kOrderLdsBytes) return MHF_EUNSUPPORTED;
    a.cap = cap;
    a.skip_long = L.skip_long;
    a.waves = static_cast<int>(kOrderLdsBytes / per_wave >= 4 ? 4 : kOrderLdsBytes / per_wave);
    if (a.waves > 4) a.waves = 4;
    if (a.waves < 1) a.waves = 1;
    // 16 KiB or less per block: several blocks per CU; persistent grid-stride loop
    int64_t blocks = (L.nwin + a.waves - 1) / a.waves;
    if (blocks > 8192) blocks = 8192;
    const dim3 grid(static_cast<unsigned>(blocks)), block(64 * a.waves);
    const size_t lds = static_cast<size_t>(per_wave * a.waves);
    // float32 AoS records of 1 or 3 channels, fixed windows, no stats.mode: the selection
    // path with whole-window vector loads and the next window's loads in flight
    bool mode = false;
    for (int j = 0; j < L.feats.n; ++j) mode |= L.feats.id[j] == MHF_MODE;
    const int64_t C4 = L.channels;
    const bool vec = !f64 && !L.starts && cap >= 256 && cap <= 1024 && !mode && L.nwin > 0 &&
                     ((L.channels == 1 && L.sample_stride == 1) ||
                      (L.channels == 3 && L.sample_stride == 3 && L.ch_stride == 1)) &&
                     (reinterpret_cast<uintptr_t>(L.x) & 15) == 0 && (L.wstep * C4) % 4 == 0 &&
                     (L.first * L.wstep * C4) % 4 == 0 &&
                     (L.first + L.nwin - 1) * L.wstep + cap <= L.n_samples;
    // median / percentile / IQR without mode: order_sel_kernel, then order_kernel over the
    // windows it left (each order feature at most once: the kernel's output slots)
    int nmed = 0, npct = 0, niqr = 0, jfirst = -1;
    for (int j = 0; j < L.feats.n; ++j) {
        const int f = L.feats.id[j];
        const bool o = f == MHF_MEDIAN || f == MHF_PERCENTILE || f == MHF_IQR;
        nmed += f == MHF_MEDIAN;
        npct += f == MHF_PERCENTILE;
        niqr += f == MHF_IQR;
        if (o && jfirst < 0) jfirst = j;
    }
    const bool sel_ok = jfirst >= 0 && nmed <= 1 && npct <= 1 && niqr <= 1;
    if (vec && sel_ok && !disabled("MHF_NO_ORDER_VEC") && !disabled("MHF_NO_ORDER_SEL")) {
        const int C = L.channels;
        OrdArgs m = a;
        m.rescan_row = jfirst;
        m.waves = 4;
        // up to 32768 blocks (8 windows per wave at 1e6 windows): the searches' step counts
        // vary window by window, and more, shorter waves balance them (measured: 2048 /
        // 8192 / 32768 / 250000 blocks -> cfg2med 1.50 / 1.32 / 1.31 / 1.43 ms, cfg2ord
        // 5.43 at 8192 -> 5.27 at 32768); MHF_ORDER_SEL_BLOCKS overrides the cap
        int64_t mb = (L.nwin + 3) / 4;
        int64_t mbmax = 32768;
        if (const char* e = diag_env("MHF_ORDER_SEL_BLOCKS")) mbmax = atoll(e) > 0 ? atoll(e) : mbmax;
        if (mb > mbmax) mb = mbmax;
        const dim3 mgrid(static_cast<unsigned>(mb)), mblock(256);
        const bool med = nmed == 1 && npct == 0 && niqr == 0;
#define MHF_OM(EE) do { \
            if (med) { \
                if (C == 1) hipLaunchKernelGGL((order_sel_kernel<EE, 1, true>), mgrid, mblock, 0, stream, m); \
                else hipLaunchKernelGGL((order_sel_kernel<EE, 3, true>), mgrid, mblock, 0, stream, m); \
            } else { \
                if (C == 1) hipLaunchKernelGGL((order_sel_kernel<EE, 1, false>), mgrid, mblock, 0, stream, m); \
                else hipLaunchKernelGGL((order_sel_kernel<EE, 3, false>), mgrid, mblock, 0, stream, m); \
            } \
        } while (0)
        if (cap <= 256) MHF_OM(4);
        else if (cap <= 512) MHF_OM(8);
        else MHF_OM(16);
#undef MHF_OM
        a.rescan = 1;
        a.rescan_row = jfirst;
        if (cap <= 256) hipLaunchKernelGGL((order_kernel<4, float>), grid, block, lds, stream, a);
        else if (cap <= 512) hipLaunchKernelGGL((order_kernel<8, float>), grid, block, lds, stream, a);
        else hipLaunchKernelGGL((order_kernel<16, float>), grid, block, lds, stream, a);
        return MHF_OK;
    }
    if (vec && !disabled("MHF_NO_ORDER_VEC")) {
        const int C = L.channels;
#define MHF_OV(EE) do { \
            if (C == 1) hipLaunchKernelGGL((order_kernel<EE, float, 1>), grid, block, lds, stream, a); \
            else hipLaunchKernelGGL((order_kernel<EE, float, 3>), grid, block, lds, stream, a); \
        } while (0)
        if (cap <= 256) MHF_OV(4);
        else if (cap <= 512) MHF_OV(8);
        else MHF_OV(16);
#undef MHF_OV
        return MHF_OK;
    }
    auto go = [&](auto tc) {
        typedef decltype(tc) T;
        if (L.starts || cap > 1024) hipLaunchKernelGGL((order_kernel<0, T>), grid, block, lds, stream, a);
        else if (cap <= 64) hipLaunchKernelGGL((order_kernel<1, T>), grid, block, lds, stream, a);
        else if (cap <= 128) hipLaunchKernelGGL((order_kernel<2, T>), grid, block, lds, stream, a);
        else if (cap <= 256) hipLaunchKernelGGL((order_kernel<4, T>), grid, block, lds, stream, a);
        else if (cap <= 512) hipLaunchKernelGGL((order_kernel<8, T>), grid, block, lds, stream, a);
        else hipLaunchKernelGGL((order_kernel<16, T>), grid, block, lds, stream, a);
    };
    if (f64) go(0.0);
    else go(0.0f);
    return MHF_OK;
}

// Indexed windows of more than L.max_w samples (the LDS launch skipped them, skip_long):
// the same kernel with each wave's keys in global memory, C * cap keys per wave, cap the
// power of two >= the longest window, in the caller's workspace: as many waves as it holds
// (at most 1024); the waves stride over the windows, so any number of long windows is
// sorted with however many waves fit.
int launch_order_long(const OrderLaunch& L, int64_t max_len, void* keys, int64_t key_bytes,
                      hipStream_t stream) {
    OrdArgs a{};
    a.x = L.x; a.ch_stride = L.ch_stride; a.sample_stride = L.sample_stride; a.wsize = L.wsize;
    a.wstep = L.wstep; a.first = L.first; a.nwin = L.nwin; a.channels = L.channels;
    a.starts = L.starts; a.ends = L.ends; a.n_samples = L.n_samples; a.min_len = L.min_len;
    a.q = L.q; a.feats = L.feats; a.out = L.out; a.out_ld = L.out_ld; a.out_f32 = L.out_f32;
    a.xd = L.xd;
    if (!L.starts || max_len > kMaxLongOrderSamples) return MHF_EUNSUPPORTED;
    int64_t cap = 1;
    while (cap < max_len) cap <<= 1;
    const int64_t per_wave = static_cast<int64_t>(L.channels) * cap * (L.xd ? 8 : 4);
    int64_t waves = key_bytes / per_wave;
    if (waves > 1024) waves = 1024;
    if (waves > L.nwin) waves = L.nwin;
    if (waves < 1 || !keys) return MHF_EINVAL;
    a.cap = static_cast<int32_t>(cap);
    a.waves = 1;
    a.short_cap = L.max_w;
    a.gkeys = keys;
    const dim3 grid(static_cast<unsigned>(waves)), block(64);
    if (L.xd) hipLaunchKernelGGL((order_kernel<0, double>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((order_kernel<0, float>), grid, block, 0, stream, a);
    return MHF_OK;
}

}  // namespace mhf
