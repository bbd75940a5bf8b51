// PO2 / PO2+ quantizer kernels for gfx950: absmax reduction + elementwise
// quantization (plain output) + packing into the conv kernels' weight layouts.
//
// Reference: utils/quantizers.py:19-56.  Two passes, deterministic, no atomics:
//   pass 1  launch_absmax       per-block max|w| (fp32 bits; NaN > inf > finite)
//   pass 2  quantize / pack     every block folds the <=1024 partials into the
//                               scale, then quantizes a grid-stride slice
#include <hip/hip_runtime.h>

#include "po2q_internal.h"
#include "po2q_quant_dev.h"

namespace po2q {

int absmax_blocks(int64_t n) {
    const int64_t per = 4 * kThreads * 4;  // 4 float4 per thread per block
    int64_t b = (n + per - 1) / per;
    if (b < 1) b = 1;
    if (b > kMaxPartials) b = kMaxPartials;
    return (int)b;
}

__global__ __launch_bounds__(kThreads) void absmax_kernel(const float* __restrict__ w, int64_t n,
                                                          unsigned* __restrict__ partial) {
    __shared__ unsigned red4[4];
    unsigned m = 0u;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    const bool aligned = ((reinterpret_cast<uintptr_t>(w) & 15u) == 0);
    if (aligned) {
        const int64_t n4 = n >> 2;
        const float4* w4 = reinterpret_cast<const float4*>(w);
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
            const float4 v = w4[i];
            const unsigned a = __float_as_uint(v.x) & 0x7fffffffu, b = __float_as_uint(v.y) & 0x7fffffffu;
            const unsigned c = __float_as_uint(v.z) & 0x7fffffffu, d = __float_as_uint(v.w) & 0x7fffffffu;
            m = max(m, max(max(a, b), max(c, d)));
        }
        for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
            m = max(m, __float_as_uint(w[i]) & 0x7fffffffu);
    } else {
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
            m = max(m, __float_as_uint(w[i]) & 0x7fffffffu);
    }
    m = block_max_u32(m, red4);
    if (threadIdx.x == 0) partial[blockIdx.x] = m;
}

hipError_t launch_absmax(const float* w, int64_t n, unsigned* partial, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(absmax_kernel, dim3(blocks), dim3(kThreads), 0, s, w, n, partial);
    return hipGetLastError();
}

// Fold the partial maxima; returns scale = max|w| (NaN if any NaN).
__device__ __forceinline__ float fold_scale(const unsigned* __restrict__ partial, int nparts, unsigned* red4) {
    unsigned m = 0u;
    for (int i = threadIdx.x; i < nparts; i += kThreads) m = max(m, partial[i]);
    m = block_max_u32(m, red4);
    return __uint_as_float(m);
}

__global__ __launch_bounds__(kThreads) void quantize_plain_kernel(const float* __restrict__ w, int64_t n,
                                                                  const unsigned* __restrict__ partial,
                                                                  int nparts, int lo, int hi, int mode,
                                                                  float* __restrict__ out) {
    __shared__ unsigned red4[4];
    const float scale = fold_scale(partial, nparts, red4);
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
        out[i] = quantize_elem(w[i], scale, mode, lo, hi);
}

static inline void clamp_window(int bits, int fsr, int& lo, int& hi) {
    lo = fsr - (1 << (bits - 1));
    hi = fsr - 1;
}

static int grid_for(int64_t n) {
    int64_t b = (n + kThreads * 4 - 1) / (kThreads * 4);
    if (b < 1) b = 1;
    if (b > 2048) b = 2048;
    return (int)b;
}

hipError_t launch_quantize_plain(const float* w, int64_t n, const unsigned* partial, int nparts, int bits,
                                 int fsr, int mode, float* out, hipStream_t s) {
    int lo, hi;
    clamp_window(bits, fsr, lo, hi);
    hipLaunchKernelGGL(quantize_plain_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, w, n, partial, nparts,
                       lo, hi, mode - 1, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------ packing --
// MFMA fp32 layout (plan kind 0): packed[g][kb][chunk][t][mi][lane] with
//   t = (r*S + s) * (CC/4) + c4, lane = (c%4)*16 + (k%16)   (A operand of
//   v_mfma_f32_16x16x4_f32: lane l holds A[row l&15][k l>>4]).
// Padding slots (k >= Kg or c >= Cg) are written as 0.
struct PackGeom {
    int Cg, Kg, R, S, CC, MI, nchunks, kblocks, steps, groups;
    int64_t total;
};

__global__ __launch_bounds__(kThreads) void pack_mfma_f32_kernel(const float* __restrict__ w,
                                                                 const unsigned* __restrict__ partial,
                                                                 int nparts, int lo, int hi, int mode,
                                                                 PackGeom pg, float* __restrict__ packed) {
    __shared__ unsigned red4[4];
    float scale = 1.0f;
    if (mode >= 0) scale = fold_scale(partial, nparts, red4);
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < pg.total; j += stride) {
        int64_t t = j;
        const int lane = (int)(t & 63); t >>= 6;
        const int mi = (int)(t % pg.MI); t /= pg.MI;
        const int step = (int)(t % pg.steps); t /= pg.steps;
        const int chunk = (int)(t % pg.nchunks); t /= pg.nchunks;
        const int kb = (int)(t % pg.kblocks); t /= pg.kblocks;
        const int g = (int)t;
        const int c4n = pg.CC >> 2;
        const int c4 = step % c4n;
        const int tap = step / c4n;
        const int r = tap / pg.S, s = tap % pg.S;
        const int kk = kb * pg.MI * 16 + mi * 16 + (lane & 15);
        const int c = chunk * pg.CC + c4 * 4 + (lane >> 4);
        float v = 0.0f;
        if (kk < pg.Kg && c < pg.Cg) {
            const int64_t k = (int64_t)g * pg.Kg + kk;
            const float x = w[((k * pg.Cg + c) * pg.R + r) * pg.S + s];
            v = (mode >= 0) ? quantize_elem(x, scale, mode, lo, hi) : x;
        }
        packed[j] = v;
    }
}

hipError_t launch_pack_weights(const ConvPlan& p, const float* w, const unsigned* partial, int nparts, int bits,
                               int fsr, int mode, float* packed, hipStream_t s) {
    int lo = 0, hi = 0;
    if (mode != 0) clamp_window(bits, fsr, lo, hi);
    if (p.kind == 1) {  // depthwise: plain [K][1][R][S] quantized copy
        const int64_t n = (int64_t)p.K * p.Cg * p.R * p.S;
        if (mode == 0) return hipMemcpyAsync(packed, w, n * sizeof(float), hipMemcpyDeviceToDevice, s);
        hipLaunchKernelGGL(quantize_plain_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, w, n, partial, nparts,
                           lo, hi, mode - 1, packed);
        return hipGetLastError();
    }
    PackGeom pg;
    pg.Cg = p.Cg; pg.Kg = p.Kg; pg.R = p.R; pg.S = p.S; pg.CC = p.CC; pg.MI = p.MI;
    pg.nchunks = p.nchunks; pg.kblocks = p.kblocks; pg.steps = p.steps; pg.groups = p.groups;
    pg.total = p.packed_floats;
    hipLaunchKernelGGL(pack_mfma_f32_kernel, dim3(grid_for(pg.total)), dim3(kThreads), 0, s, w, partial, nparts,
                       lo, hi, mode - 1, pg, packed);
    return hipGetLastError();
}

}  // namespace po2q
