// Device-side PO2 / PO2+ quantizer arithmetic (bit-exact with the reference).
//
// Reference: utils/quantizers.py:21-32 (PowerOfTwoQuantizer.forward) and
// :41-52 (PowerOfTwoPlusQuantizer.forward):
//   sign = sign(w); scale = max|w|; a = |w / scale|
//   e = clamp(round(log2 a), fsr - 2^(bits-1), fsr - 1)         [po2]
//   e = clamp(round(log2(a / 1.5) + 0.5), ...)                   [po2+]
//   out = (2^e * sign) * scale
// The fp32 log2/round decision is replaced by the per-binade threshold table
// (po2q_thresholds.h): for a in [2^k, 2^(k+1)), e = k + (bits(a) >= T_k),
// which equals the reference's torch fp32 arithmetic for every fp32 a in (0,1).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "po2q_thresholds.h"

namespace po2q {

// Unclamped exponent for a finite positive a with bits(a) < bits(1.0f).
__device__ __forceinline__ int decide_exponent(uint32_t b, int mode) {
    // binade k: exponent field for normals, leading-one position for subnormals
    const int k = (b >= 0x00800000u) ? (int)(b >> 23) - 127 : (31 - (int)__clz(b)) - 149;
    return k + (b >= po2q_thr[mode][k - PO2Q_THR_KMIN] ? 1 : 0);
}

// Clamped exponent decision; returns false when the reference would give NaN
// (a is NaN: 0/0, inf/inf or NaN input).
__device__ __forceinline__ bool exponent_of(float w, float scale, int mode, int lo, int hi, int& e) {
    const float nrm = w / scale;                          // IEEE fp32 division (:24)
    const uint32_t b = __float_as_uint(nrm) & 0x7fffffffu;  // |.| (:25)
    if (b > 0x7f800000u) return false;                    // NaN
    int d;
    if (b == 0u) d = lo;                                  // log2(0) = -inf -> clamp -> lo
    else if (b < 0x3f800000u) d = decide_exponent(b, mode);
    else if (b == 0x3f800000u) d = 0;                     // a == 1 -> 0 (both modes)
    else d = hi;                                          // a > 1 (incl. inf): cannot occur
    e = d < lo ? lo : (d > hi ? hi : d);
    return true;
}

__device__ __forceinline__ float ref_sign(float w) {
    return w > 0.0f ? 1.0f : (w < 0.0f ? -1.0f : 0.0f);  // torch.sign (NaN -> 0, -0 -> +0)
}

// Full reference elementwise result.
__device__ __forceinline__ float quantize_elem(float w, float scale, int mode, int lo, int hi) {
    int e;
    if (!exponent_of(w, scale, mode, lo, hi, e)) return __builtin_nanf("");
    const float lq = ldexpf(1.0f, e);                     // 2**q, exact (0 below 2^-149)
    return (lq * ref_sign(w)) * scale;                    // (:32) left-to-right
}

__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Block-wide max over 256 threads; every thread gets the result.
// Block-wide max of NW waves (red: NW LDS words).
template <int NW = 4>
__device__ __forceinline__ unsigned block_max_u32(unsigned v, unsigned* red) {
    v = wave_max_u32(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    unsigned m = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = red[i] > m ? red[i] : m;
    __syncthreads();
    return m;
}

}  // namespace po2q
