// PO2 / PO2+ quantizer for fp64 and bf16 tensors, bit-exact with the reference run in that dtype.
//
// Reference: utils/quantizers.py:19-56.  The reference keeps the input's dtype (torch ops on the
// tensor it is given), so an fp64 weight is quantized with double arithmetic and a bf16 weight
// with torch's bf16 arithmetic (every op computed in fp32 and rounded to bf16).  As in the fp32
// kernel (po2q_quant.hip) the exponent decision round(log2 a) [po2] / round(log2(a/1.5) + 0.5)
// [po2+] is a table measured from the reference itself (po2q_thresholds_dtypes.h):
//   bf16  a = bf16(fp32(w) / fp32(scale)) (torch: fp32 division, round to nearest even), one
//         decision per bf16 value below 1 (16,256 entries): subnormal binades are not a single
//         threshold there;
//   fp64  a = w / scale (IEEE double division), two thresholds per binade (po2+ subnormal binades
//         decide k - 1 below the first).
// Then out = (2^e * sign(w)) * scale in the dtype: fp64 exact, bf16 = bf16(fp32 product) as
// torch computes it.  Two passes, deterministic, no atomics: absmax partials of the
// sign-cleared bit patterns (NaN > inf > finite, as torch.max propagates NaN), then every block
// folds the partials and quantizes a grid-stride slice.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "po2q_internal.h"
#include "po2q_thresholds_dtypes.h"

namespace po2q {

namespace {

template <typename T>
struct DT;
template <>
struct DT<double> {
    using Bits = uint64_t;
    static __device__ __forceinline__ uint64_t absbits(double v) {
        return (uint64_t)__double_as_longlong(v) & 0x7fffffffffffffffull;
    }
};
template <>
struct DT<uint16_t> {  // bf16 bit patterns
    using Bits = uint64_t;
    static __device__ __forceinline__ uint64_t absbits(uint16_t v) { return (uint64_t)(v & 0x7fffu); }
};

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t* red) {
    v = wave_max_u64(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    uint64_t m = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = red[i] > m ? red[i] : m;
    __syncthreads();
    return m;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void absmax_dt_kernel(const T* __restrict__ w, int64_t n,
                                                             uint64_t* __restrict__ partial) {
    __shared__ uint64_t red[kThreads / 64];
    uint64_t m = 0u;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        const uint64_t b = DT<T>::absbits(w[i]);
        m = b > m ? b : m;
    }
    m = block_max_u64(m, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = m;
}

// torch's float -> bf16 conversion (c10::BFloat16 round_to_nearest_even; NaN -> 0x7fc0)
__device__ __forceinline__ uint16_t bf16_rne(float f) {
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)0x7fc0u;
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float bf16_to_f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// torch.sign
template <typename F>
__device__ __forceinline__ F sgn(F v) {
    return v > F(0) ? F(1) : (v < F(0) ? F(-1) : F(0));
}

__device__ __forceinline__ int clampi(int d, int lo, int hi) { return d < lo ? lo : (d > hi ? hi : d); }

__device__ __forceinline__ double quant_f64(double w, double scale, int mode, int lo, int hi) {
    const double nrm = w / scale;  // IEEE double division (:24)
    const uint64_t b = (uint64_t)__double_as_longlong(nrm) & 0x7fffffffffffffffull;
    if (b > 0x7ff0000000000000ull) return __longlong_as_double(0x7ff8000000000000ll);  // NaN
    int d;
    if (b == 0u) {
        d = lo;  // log2(0) = -inf -> clamp
    } else if (b < 0x3ff0000000000000ull) {
        const int k = (b >= 0x0010000000000000ull) ? (int)(b >> 52) - 1023 : (63 - (int)__clzll((long long)b)) - 1074;
        const int i = k - PO2Q_F64_KMIN;
        d = k - 1 + (b >= po2q_f64_down[mode][i] ? 1 : 0) + (b >= po2q_f64_up[mode][i] ? 1 : 0);
    } else if (b == 0x3ff0000000000000ull) {
        d = 0;  // a == 1
    } else {
        d = hi;  // a > 1: not reached for finite w (|w| <= scale)
    }
    const int e = clampi(d, lo, hi);
    const double lq = ldexp(1.0, e);  // 2**q, exact (0 below 2^-1074)
    return (lq * sgn(w)) * scale;     // (:32) left to right
}

__device__ __forceinline__ uint16_t quant_bf16(uint16_t wb, uint16_t sb, int mode, int lo, int hi) {
    const float w = bf16_to_f(wb), scale = bf16_to_f(sb);
    const uint16_t ab = bf16_rne(w / scale);  // bf16 division: fp32 then round (:24)
    const uint32_t b = ab & 0x7fffu;           // |.| (:25)
    if (b > 0x7f80u) return (uint16_t)0x7fc0u;  // NaN
    int d;
    if (b == 0u) {
        d = lo;
    } else if (b < 0x3f80u) {
        const int k = (b >= 0x0080u) ? (int)(b >> 7) - 127 : (31 - (int)__clz(b)) - 133;
        d = k + (int)po2q_bf16_dec[mode][b] - 1;
    } else if (b == 0x3f80u) {
        d = 0;
    } else {
        d = hi;
    }
    const int e = clampi(d, lo, hi);
    const uint16_t lq = bf16_rne(ldexpf(1.0f, e));          // 2**q in bf16
    const uint16_t ls = bf16_rne(bf16_to_f(lq) * sgn(w));   // * sign: exact
    return bf16_rne(bf16_to_f(ls) * scale);                 // * scale: fp32 product, rounded
}

template <typename T>
__global__ __launch_bounds__(kThreads) void quantize_dt_kernel(const T* __restrict__ w, int64_t n,
                                                               const uint64_t* __restrict__ partial, int nparts,
                                                               int lo, int hi, int mode, T* __restrict__ out) {
    __shared__ uint64_t red[kThreads / 64];
    uint64_t m = 0u;
    for (int i = threadIdx.x; i < nparts; i += kThreads) m = partial[i] > m ? partial[i] : m;
    m = block_max_u64(m, red);
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    if constexpr (sizeof(T) == 8) {
        const double scale = __longlong_as_double((long long)m);
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
            out[i] = quant_f64(w[i], scale, mode, lo, hi);
    } else {
        const uint16_t sb = (uint16_t)m;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
            out[i] = quant_bf16(w[i], sb, mode, lo, hi);
    }
}

int grid_dt(int64_t n) {
    int64_t b = (n + kThreads * 4 - 1) / (kThreads * 4);
    return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

template <typename T>
hipError_t launch_quantize_dt(const T* w, T* out, int64_t n, int bits, int fsr, int mode, uint64_t* partial,
                              int nparts, hipStream_t s) {
    const int lo = fsr - (1 << (bits - 1)), hi = fsr - 1;
    hipLaunchKernelGGL(absmax_dt_kernel<T>, dim3(nparts), dim3(kThreads), 0, s, w, n, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(quantize_dt_kernel<T>, dim3(grid_dt(n)), dim3(kThreads), 0, s, w, n, partial, nparts, lo, hi,
                       mode - 1, out);
    return hipGetLastError();
}

template hipError_t launch_quantize_dt<double>(const double*, double*, int64_t, int, int, int, uint64_t*, int,
                                               hipStream_t);
template hipError_t launch_quantize_dt<uint16_t>(const uint16_t*, uint16_t*, int64_t, int, int, int, uint64_t*, int,
                                                 hipStream_t);

}  // namespace po2q
