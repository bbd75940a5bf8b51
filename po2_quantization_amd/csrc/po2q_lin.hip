// Linear power-of-two weight quantizers lin / lin+.
// Reference: LinearPowerOfTwoQuantizer.forward / LinearPowerOfTwoPlusQuantizer.forward,
// utils/quantizers.py:59-136, with quantize_per_filter (:8-16).  Per input channel c
// (dim 1 of the 4-D weight [d0, d1, d2, d3]):
//   delta = (max_c - min_c) / (2^bits - 1);  q = qpf(w, delta) / delta
//   num_iters x: delta = 2 ** round(log2(sum(q w) / sum(q q)))   (lin+: of sqrt(8/9) x that)
//                q = qpf(w, delta) / delta
//   out = q * delta
// qpf(x, d) = d * clamp(round(x / d), -(2^(bits-1) - 1), 2^(bits-1) - 1), all fp32.
//
// One workgroup per channel.  A channel's d0*d2*d3 elements (<= 576 for ResNet, <= 960
// for MobileNet's pointwise convs) stay in VGPRs across every pass: one HBM read and one
// write per element, the rest is ALU plus two block reductions per iteration.  The sums
// are fp64 in a fixed order (deterministic; the reference sums fp32 in an unspecified
// order and only the power-of-two snap consumes them).  The snap is torch's own fp32
// round(log2) decision, tabulated per binade (po2q_log2_table.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "po2q_internal.h"
#include "po2q_log2_table.h"

namespace po2q {

namespace {

constexpr int kLinMaxPer = 16;  // elements per thread held in VGPRs

__device__ __forceinline__ float lin_qpf(float x, float d, float lim) {
    float s = rintf(__fdiv_rn(x, d));
    s = s < -lim ? -lim : (s > lim ? lim : s);  // NaN passes, as torch.clamp
    return __fdiv_rn(__fmul_rn(d, s), d);
}

// 2 ** round(log2(v)) exactly as torch computes it in fp32
__device__ __forceinline__ float lin_snap(float v) {
    if (__builtin_isnan(v) || v < 0.0f) return __builtin_nanf("");
    if (v == 0.0f) return 0.0f;
    if (__builtin_isinf(v)) return v;
    const uint32_t b = __float_as_uint(v);
    int e;
    if (b >= 0x00800000u) {
        const int k = (int)(b >> 23) - 127;
        e = k + (b >= po2q_l2r_thr[k - PO2Q_L2R_THR_KMIN] ? 1 : 0);
    } else {
        const int k = (31 - __builtin_clz(b)) - 149;
        e = k + ((double)v >= ldexp(1.4142135623730951, k) ? 1 : 0);
    }
    return ldexpf(1.0f, e);
}

template <int NTH, typename T>
__device__ __forceinline__ T lin_block_sum(T v, T* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // red may still be read by the previous reduction
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    T s = red[0];
#pragma unroll
    for (int i = 1; i < NTH / 64; ++i) s += red[i];  // fixed order
    return s;
}

// NTH threads per channel; REG: the channel's elements fit in VGPRs (<= 16 NTH)
template <int NTH, bool REG>
__global__ __launch_bounds__(NTH) void quantize_lin_kernel(const float* __restrict__ w, float* __restrict__ out,
                                                                   int d0, int d1, int rs, int bits, int num_iters,
                                                                   int plus) {
    __shared__ double redd[NTH / 64];
    const int c = blockIdx.x;
    const int m = d0 * rs;
    const float lim = (float)((1 << (bits - 1)) - 1);
    const float levels = (float)((1 << bits) - 1);
    auto addr = [&](int i) { return ((int64_t)(i / rs) * d1 + c) * rs + i % rs; };
    float xr[REG ? kLinMaxPer : 1];
    // ---- range of the channel (torch.max / torch.min over dims 0, 2, 3; NaN propagates)
    float mx = -INFINITY, mn = INFINITY, nan = 0.0f;
#pragma unroll
    for (int u = 0; u < (REG ? kLinMaxPer : 1); ++u) xr[u] = 0.0f;
    if constexpr (REG) {
#pragma unroll
        for (int u = 0; u < kLinMaxPer; ++u) {
            const int i = threadIdx.x + u * NTH;
            if (i < m) {
                const float v = w[addr(i)];
                xr[u] = v;
                nan = __builtin_isnan(v) ? 1.0f : nan;
                mx = v > mx ? v : mx;
                mn = v < mn ? v : mn;
            }
        }
    } else {
        for (int i = threadIdx.x; i < m; i += NTH) {
            const float v = w[addr(i)];
            nan = __builtin_isnan(v) ? 1.0f : nan;
            mx = v > mx ? v : mx;
            mn = v < mn ? v : mn;
        }
    }
    // max / min / any-NaN over the block (float shuffles; fmaxf is fine: NaN tracked apart)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        nan = fmaxf(nan, __shfl_xor(nan, o, 64));
    }
    __shared__ float rmx[NTH / 64], rmn[NTH / 64], rnan[NTH / 64];
    if ((threadIdx.x & 63) == 0) {
        rmx[threadIdx.x >> 6] = mx;
        rmn[threadIdx.x >> 6] = mn;
        rnan[threadIdx.x >> 6] = nan;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NTH / 64; ++i) {
        mx = fmaxf(mx, rmx[i]);
        mn = fminf(mn, rmn[i]);
        nan = fmaxf(nan, rnan[i]);
    }
    if (nan != 0.0f) mx = mn = __builtin_nanf("");
    float delta = __fdiv_rn(__fsub_rn(mx, mn), levels);  // (max - min) / (2^bits - 1)
    const float shrink = __fsqrt_rn(8.0f / 9.0f);          // torch.sqrt(torch.tensor(8/9))
    for (int it = 0; it < num_iters; ++it) {
        double qtw = 0.0, qtq = 0.0;
        if constexpr (REG) {
#pragma unroll
            for (int u = 0; u < kLinMaxPer; ++u) {
                const int i = threadIdx.x + u * NTH;
                if (i < m) {
                    const float q = lin_qpf(xr[u], delta, lim);
                    qtw += (double)q * (double)xr[u];
                    qtq += (double)q * (double)q;
                }
            }
        } else {
            for (int i = threadIdx.x; i < m; i += NTH) {
                const float x = w[addr(i)];
                const float q = lin_qpf(x, delta, lim);
                qtw += (double)q * (double)x;
                qtq += (double)q * (double)q;
            }
        }
        qtw = lin_block_sum<NTH>(qtw, redd);
        qtq = lin_block_sum<NTH>(qtq, redd);
        float nd = __fdiv_rn((float)qtw, (float)qtq);
        if (plus) nd = __fmul_rn(shrink, nd);
        delta = lin_snap(nd);
    }
    // ---- out = (qpf(w, delta) / delta) * delta
    if constexpr (REG) {
#pragma unroll
        for (int u = 0; u < kLinMaxPer; ++u) {
            const int i = threadIdx.x + u * NTH;
            if (i < m) out[addr(i)] = __fmul_rn(lin_qpf(xr[u], delta, lim), delta);
        }
    } else {
        for (int i = threadIdx.x; i < m; i += NTH) {
            const int64_t a = addr(i);
            out[a] = __fmul_rn(lin_qpf(w[a], delta, lim), delta);
        }
    }
}

}  // namespace

hipError_t launch_quantize_lin(const float* w, float* out, int d0, int d1, int rs, int bits, int num_iters, int plus,
                               hipStream_t s) {
    const int m = d0 * rs;  // elements per channel
#define PO2Q_LIN(nth, reg)                                                                                    \
    hipLaunchKernelGGL((quantize_lin_kernel<nth, reg>), dim3((unsigned)d1), dim3(nth), 0, s, w, out, d0, d1, rs, \
                       bits, num_iters, plus)
    if (m <= 256 * kLinMaxPer)
        PO2Q_LIN(256, true);
    else if (m <= 1024 * kLinMaxPer)  // e.g. depthwise [960, 1, 3, 3]: one channel of 8640
        PO2Q_LIN(1024, true);
    else
        PO2Q_LIN(1024, false);
#undef PO2Q_LIN
    return hipGetLastError();
}

}  // namespace po2q
