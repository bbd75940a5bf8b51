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

#include "po2q_internal.h"
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

__device__ __forceinline__ uint16_t bf16_bits_keep_nan(float q) {
    const uint32_t u = __float_as_uint(q);
    const bool nan = ((u & 0x7f800000u) == 0x7f800000u) && (u & 0x007fffffu);
    return (uint16_t)((u >> 16) | (nan ? 0x40u : 0u));
}

// W' = Q(w) / scale as bf16 bits: sign(w) * 2^e exactly (fin), else the reference's Q(w).
// thr: the mode's threshold row staged in LDS (no dependent constant-memory load per
// weight); same decision as exponent_of (po2q_quant_dev.h).
__device__ __forceinline__ uint16_t pack_one(float wv, float scale, bool fin, int mode, int lo, int hi,
                                             const unsigned* thr) {
    if (fin) {
        // finite scale: a = |w / scale| <= 1 (w finite; scale = max|w|)
        const uint32_t b = __float_as_uint(wv / scale) & 0x7fffffffu;
        int d;
        if (b == 0u) {
            d = lo;
        } else if (b < 0x3f800000u) {
            const int k = (b >= 0x00800000u) ? (int)(b >> 23) - 127 : (31 - (int)__clz(b)) - 149;
            d = k + (b >= thr[k - PO2Q_THR_KMIN] ? 1 : 0);
        } else {
            d = 0;  // a == 1
        }
        const int e = d < lo ? lo : (d > hi ? hi : d);
        const float sg = ref_sign(wv);
        return (sg == 0.0f) ? (uint16_t)0 : (uint16_t)(((sg < 0.0f) ? 0x8000u : 0u) | ((unsigned)(e + 127) << 7));
    }
    return bf16_bits_keep_nan(quantize_elem(wv, scale, mode, lo, hi));
}


// ---- fused weight staging (row conv kernels, plan field fp): every block reduces
// max|w| over the whole small, L2-resident weight tensor itself and quantizes + packs
// the B fragments it needs, so a quantized conv is ONE launch (no pack kernel, no
// workspace round trip).  Same decision (threshold table), same fragments as
// pack_bf16x3_kernel (po2q_quant.hip).

// Block-wide max|w| bits (NaN > inf > finite) over nw waves; red: nw LDS words.
__device__ __forceinline__ unsigned wq_absmax(const float* __restrict__ w, int n, unsigned* red, int nw) {
    unsigned m = 0u;
    const int tid = threadIdx.x, nt = (int)blockDim.x;
    if ((reinterpret_cast<uintptr_t>(w) & 15u) == 0) {
        const int n4 = n >> 2;
        const float4* w4 = reinterpret_cast<const float4*>(w);
        for (int i = tid; i < n4; i += nt) {
            const float4 v = w4[i];
            const unsigned a = __float_as_uint(v.x) & 0x7fffffffu, b = __float_as_uint(v.y) & 0x7fffffffu;
            const unsigned c = __float_as_uint(v.z) & 0x7fffffffu, d = __float_as_uint(v.w) & 0x7fffffffu;
            m = max(m, max(max(a, b), max(c, d)));
        }
        for (int i = (n4 << 2) + tid; i < n; i += nt) m = max(m, __float_as_uint(w[i]) & 0x7fffffffu);
    } else {
        for (int i = tid; i < n; i += nt) m = max(m, __float_as_uint(w[i]) & 0x7fffffffu);
    }
    m = wave_max_u32(m);
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    unsigned r = red[0];
    for (int i = 1; i < nw; ++i) r = red[i] > r ? red[i] : r;
    return r;
}

// B fragment j of the row layout [r][ks][nt][lane][8] (pack_bf16x3_kernel, vr == 2):
// CC = 16: ks 0 -> k < 16: s = 0, k >= 16: s = 1; ks 1 -> k < 16: s = 2, else 0.
// CC = 32: ks = chunk * 3 + s, k = the chunk's 32 channels.
// dup (CC = 16): k-step 1 holds the s2 tap in BOTH halves, (s2 | s2) instead of (s2 | 0), for the
// kernels that pair the s2 tap of two planes in one k-step (conv_pair: (s2 hi | s2 mid), (s2 lo | 0)).
__device__ __forceinline__ uint4 wq_frag_rows(const WQuant& q, int C, int K, int CC, int NT, int ksteps, int j,
                                              float scale, bool fin, const unsigned* thr, bool dup = false) {
    const int lane = j & 63, t = j >> 6;
    const int nt = t % NT;
    const int ks = (t / NT) % ksteps;
    const int r = t / (NT * ksteps);
    const int grp = lane >> 4;
    int sft, c0;
    if (CC == 16) {
        sft = ks == 0 ? (grp >> 1) : ((grp < 2 || dup) ? 2 : -1);
        c0 = 8 * (grp & 1);
    } else {
        sft = ks % 3;
        c0 = (ks / 3) * 32 + 8 * grp;
    }
    const int k = nt * 16 + (lane & 15);
    const bool ok = k < K && sft >= 0;
    uint32_t h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        h[e] = (ok && c < C) ? pack_one(q.w[(k * C + c) * 9 + r * 3 + sft], scale, fin, q.mode, q.lo, q.hi, thr) : 0u;
    }
    return make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
}

// Cooperative form of wq_frag_rows for the whole tensor: ONE coalesced pass over w, every weight
// quantized + packed once per block (not once per lane that needs it, whose 1152-byte-strided
// gathers made the per-lane form cost ~0.085 ms per stage-2 pair launch: profiles/r06_pairw_ablation),
// its bf16 code written into the row-layout fragments in LDS.  fr: nfr * 64 uint4, zero-filled
// here (k >= K, the CC = 16 halves no tap fills).  Same fragments as wq_frag_rows (C: the tensor's
// input channels, a compile-time constant so the index split is a multiply).  Ends with a barrier.
template <int C>
__device__ __forceinline__ void wq_pack_rows_lds(const WQuant& q, int K, int CC, int NT, int ksteps, float scale,
                                                 bool fin, const unsigned* thr, uint4* fr, int nfr, bool dup = false) {
    static_assert(C > 0, "channels");
    const int tid = threadIdx.x, nthr = (int)blockDim.x;
    for (int e = tid; e < nfr * 64; e += nthr) fr[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    uint16_t* h = reinterpret_cast<uint16_t*>(fr);
    const int n = K * C * 9;
    for (int i = tid; i < n; i += nthr) {
        const int k = i / (C * 9), rem = i - k * (C * 9);
        const int c = rem / 9, tap = rem - c * 9;
        const int r = tap / 3, s = tap - r * 3;
        const uint16_t v = pack_one(q.w[i], scale, fin, q.mode, q.lo, q.hi, thr);
        int ks, grp;
        if (CC == 16) {
            ks = s == 2 ? 1 : 0;
            grp = (s == 2 ? 0 : 2 * s) + (c >> 3);
        } else {
            ks = (c >> 5) * 3 + s;
            grp = (c & 31) >> 3;
        }
        const int j = ((r * ksteps + ks) * NT + (k >> 4)) * 64 + (k & 15) + 16 * grp;
        h[j * 8 + (c & 7)] = v;
        if (CC == 16 && s == 2 && dup) h[(j + 32) * 8 + (c & 7)] = v;
    }
    __syncthreads();
}

// The same for tap row r only (kernels whose LDS scratch holds one tap row's fragments at a time):
// fr gets fragments j = (ks * NT + nt) * 64 + lane of row r (wq_frag_rows index minus r's offset).
template <int C>
__device__ __forceinline__ void wq_pack_tap_row_lds(const WQuant& q, int K, int CC, int NT, int ksteps, int r,
                                                    float scale, bool fin, const unsigned* thr, uint4* fr) {
    static_assert(C > 0, "channels");
    const int tid = threadIdx.x, nthr = (int)blockDim.x;
    const int nfr = ksteps * NT;
    for (int e = tid; e < nfr * 64; e += nthr) fr[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    uint16_t* h = reinterpret_cast<uint16_t*>(fr);
    const int n = K * C * 3;  // (k, c, s) of tap row r
    for (int m = tid; m < n; m += nthr) {
        const int kc = m / 3, s = m - kc * 3;
        const int k = kc / C, c = kc - k * C;
        const uint16_t v = pack_one(q.w[kc * 9 + r * 3 + s], scale, fin, q.mode, q.lo, q.hi, thr);
        int ks, grp;
        if (CC == 16) {
            ks = s == 2 ? 1 : 0;
            grp = (s == 2 ? 0 : 2 * s) + (c >> 3);
        } else {
            ks = (c >> 5) * 3 + s;
            grp = (c & 31) >> 3;
        }
        const int j = (ks * NT + (k >> 4)) * 64 + (k & 15) + 16 * grp;
        h[j * 8 + (c & 7)] = v;
    }
    __syncthreads();
}

// Stage the threshold row (LDS) and reduce the scale; returns the conv's multiplier
// (max|w|, or 1 where the reference's Q(w) itself is packed).  thr: PO2Q_THR_COUNT LDS
// words, red: nw LDS words.  Ends with the block's threshold row visible to every thread.
__device__ __forceinline__ float wq_prologue(const WQuant& q, unsigned* thr, unsigned* red, int nw, bool& fin) {
    for (int i = threadIdx.x; i < PO2Q_THR_COUNT; i += blockDim.x) thr[i] = po2q_thr[q.mode > 0 ? 1 : 0][i];
    const unsigned m = wq_absmax(q.w, q.n, red, nw);  // its barrier also publishes thr
    fin = (m > 0u) && (m < 0x7f800000u);
    return fin ? __uint_as_float(m) : 1.0f;
}

}  // namespace po2q
