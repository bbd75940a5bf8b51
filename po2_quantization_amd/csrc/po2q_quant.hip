// PO2 / PO2+ quantizer kernels for gfx950: absmax reduction + elementwise
// quantization (plain output) + packing into the conv kernels' weight layouts.
//
// Reference: utils/quantizers.py:19-56.  Two passes, deterministic, no atomics:
//   pass 1  launch_absmax       per-block max|w| (fp32 bits; NaN > inf > finite)
//   pass 2  quantize / pack     every block folds the <=1024 partials into the
//                               scale, then quantizes a grid-stride slice
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

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

// Small tensors (depthwise weights, <= kFusedAbsmaxMax elements): absmax and quantize in one
// launch -- every block reduces the whole L2-resident tensor, then quantizes its slice.
__global__ __launch_bounds__(1024) void quantize_plain_fused_kernel(const float* __restrict__ w, int n, int lo, int hi,
                                                                    int mode, float* __restrict__ out) {
    __shared__ unsigned red[16];
    unsigned m = 0u;
    constexpr int U = 4;  // independent loads in flight per thread
    for (int i = threadIdx.x; i < n; i += U * 1024) {
        unsigned v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = i + u * 1024;
            v[u] = k < n ? (__float_as_uint(w[k]) & 0x7fffffffu) : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) m = max(m, v[u]);
    }
    m = block_max_u32<16>(m, red);
    const float scale = __uint_as_float(m);
    for (int i = blockIdx.x * 1024 + threadIdx.x; i < n; i += gridDim.x * 1024)
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

// bf16x3 layout (plan kind 2): packed[kb][chunk][ks][nt][lane][e] (uint16) =
//   B fragment of v_mfma_f32_16x16x32_bf16: lane l holds B[k = 8*(l>>4) + e][n = l&15];
//   n -> output channel kb*16*NT + nt*16 + (l&15); the k-step's 4 channel octets
//   oi = ks*4 + (l>>4) map tap-major to (tap = oi / (CC/8), channels (oi % (CC/8))*8 + e).
// Value: W' = Q(w) / scale = sign(w) * 2^e exactly (bf16), 0 for padding.  When
// scale is not a positive finite number (all-zero / NaN / inf weights) the
// reference's Q(w) itself (NaN / inf / 0) is stored and the multiplier is 1.
struct PackX3 {
    int C, K, R, S, CC, NT, nchunks, ksteps, taps, vr;
    int64_t total;  // uint16 elements
};

// 1024 threads: the fused absmax (every block reads the whole weight tensor from L2)
// finishes in one or two rounds of independent loads per thread.
constexpr int kPackThreads = 1024;

// max|w| bits of a small (L2-resident, < 2^20 elements) weight tensor, reduced by every
// thread of the block (kPackThreads threads): the pack kernels' fused absmax.
__device__ __forceinline__ unsigned fused_absmax_bits(const float* __restrict__ w, int64_t n) {
    unsigned m = 0u;
    const bool aligned = ((reinterpret_cast<uintptr_t>(w) & 15u) == 0);
    int i0 = 0;  // the planner keeps fused weights below 2^20 elements
    if (aligned) {
        const int n4 = (int)(n >> 2);
        const float4* w4 = reinterpret_cast<const float4*>(w);
        constexpr int U = 8;  // independent loads in flight per thread
        for (int i = threadIdx.x; i < n4; i += U * kPackThreads) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = i + u * kPackThreads;
                v[u] = (k < n4) ? w4[k] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned a = __float_as_uint(v[u].x) & 0x7fffffffu, b = __float_as_uint(v[u].y) & 0x7fffffffu;
                const unsigned c = __float_as_uint(v[u].z) & 0x7fffffffu, d = __float_as_uint(v[u].w) & 0x7fffffffu;
                m = max(m, max(max(a, b), max(c, d)));
            }
        }
        i0 = n4 << 2;
    }
    for (int i = i0 + threadIdx.x; i < (int)n; i += kPackThreads) m = max(m, __float_as_uint(w[i]) & 0x7fffffffu);
    return m;
}

// The pack of one weight tensor by block `bid` of `nb` (pack_bf16x3_kernel: one tensor per
// launch; pack_batch_kernel: one tensor per blockIdx.y).
__device__ __forceinline__ void pack_bf16x3_body(const float* __restrict__ w, int64_t n,
                                                 const unsigned* __restrict__ partial, int nparts, int lo, int hi,
                                                 int mode, const PackX3& pg, uint16_t* __restrict__ packed,
                                                 float* __restrict__ scale_out, int bid, int nb) {
    __shared__ unsigned red[kPackThreads / 64];
    __shared__ unsigned thr[PO2Q_THR_COUNT];
    for (int i = threadIdx.x; i < PO2Q_THR_COUNT; i += kPackThreads) thr[i] = po2q_thr[mode > 0 ? 1 : 0][i];
    unsigned m = 0u;
    if (nparts > 0) {
        for (int i = threadIdx.x; i < nparts; i += kPackThreads) m = max(m, partial[i]);
    } else {  // fused absmax: every block reduces the whole (small, L2-resident) weight tensor
        m = fused_absmax_bits(w, n);
    }
    m = block_max_u32<kPackThreads / 64>(m, red);
    const float scale = __uint_as_float(m);
    const bool fin = (m > 0u) && (m < 0x7f800000u);
    if (bid == 0 && threadIdx.x == 0) *scale_out = fin ? scale : 1.0f;
    // one 16-byte B fragment slot (8 consecutive k = 8 consecutive input channels of
    // one tap, one output channel) per thread and iteration; 32-bit index math
    const int OCT = pg.CC >> 3;
    const int RS = pg.R * pg.S;
    const int nfr = (int)(pg.total >> 3);
    uint4* out = reinterpret_cast<uint4*>(packed);
    for (int j = bid * kPackThreads + threadIdx.x; j < nfr; j += nb * kPackThreads) {
        const int lane = j & 63;
        int t = j >> 6;
        int k, c0, tapoff;
        bool ok;
        if (pg.vr == 2) {
            // row-streaming layout [r][ks][nt][lane][8] (po2q_conv_rows*.hip):
            //   CC = 16: ks 0 -> k < 16: s = 0, k >= 16: s = 1;  ks 1 -> k < 16: s = 2, else 0
            //   CC = 32: ks = chunk * 3 + s, k = the chunk's 32 channels
            const int nt = t % pg.NT;
            const int ks = (t / pg.NT) % pg.ksteps;
            const int r = t / (pg.NT * pg.ksteps);
            const int grp = lane >> 4;
            int sft;
            if (pg.CC == 16) {
                sft = ks == 0 ? (grp >> 1) : (grp < 2 ? 2 : -1);
                c0 = 8 * (grp & 1);
            } else {  // ks = chunk * 3 + s (po2q_conv_rowsk.hip: 2 chunks of 32 channels)
                sft = ks % 3;
                c0 = (ks / 3) * 32 + 8 * grp;
            }
            k = nt * 16 + (lane & 15);
            tapoff = r * 3 + sft;
            ok = k < pg.K && sft >= 0;
        } else if (pg.vr) {
            // row-reuse layout [chunk][r][f][lane][8], 3x3 / 16 output channels (po2q_conv_x3p.hip):
            //   f = s in 0..2: B[k][n] = w[n][c][r][s] for both k halves (hi|mid A fragment)
            //   f = 3: k < 16 -> s = 0, k >= 16 -> s = 1;  f = 4: k < 16 -> s = 2, k >= 16 -> 0
            const int fr = t % 15, chunk = t / 15;
            const int r = fr / 5, ft = fr - (fr / 5) * 5, grp = lane >> 4;
            const int sft = ft < 3 ? ft : (ft == 3 ? (grp >= 2 ? 1 : 0) : (grp >= 2 ? -1 : 2));
            k = lane & 15;
            c0 = chunk * 16 + 8 * (grp & 1);
            tapoff = r * 3 + sft;
            ok = k < pg.K && sft >= 0;
        } else {
            const int nt = t % pg.NT; t /= pg.NT;
            const int ks = t % pg.ksteps; t /= pg.ksteps;
            const int chunk = t % pg.nchunks;
            const int kb = t / pg.nchunks;
            k = kb * 16 * pg.NT + nt * 16 + (lane & 15);
            const int oi = ks * 4 + (lane >> 4);
            const int tap = oi / OCT;
            c0 = chunk * pg.CC + (oi - tap * OCT) * 8;
            tapoff = tap;  // (r, s) row-major = tap
            ok = k < pg.K && tap < pg.taps;
        }
        uint32_t h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = c0 + e;
            h[e] = (ok && c < pg.C) ? pack_one(w[(k * pg.C + c) * RS + tapoff], scale, fin, mode, lo, hi, thr) : 0u;
        }
        out[j] = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
    }
}

__global__ __launch_bounds__(kPackThreads) void pack_bf16x3_kernel(const float* __restrict__ w, int64_t n,
                                                               const unsigned* __restrict__ partial,
                                                               int nparts, int lo, int hi, int mode,
                                                               PackX3 pg, uint16_t* __restrict__ packed,
                                                               float* __restrict__ scale_out) {
    pack_bf16x3_body(w, n, partial, nparts, lo, hi, mode, pg, packed, scale_out, (int)blockIdx.x, (int)gridDim.x);
}

// Up to kPackBatch weight tensors quantized + packed in one launch (blockIdx.y = tensor):
// the per-layer pack launches of a whole forward become ceil(n / kPackBatch) launches.  A job
// is either the bf16x3 B-fragment pack of an MFMA plan (plain == 0) or the plain quantized
// fp32 copy [K][1][R][S] a depthwise plan reads (plain == 1, quantize_plain_fused_kernel's work).
struct PackJob {
    const float* w;
    void* packed;
    float* scale;
    const unsigned* partial;  // nparts > 0: max|w| from these absmax partials (absmax_batch_kernel)
    int64_t n;
    int lo, hi, mode, nb, plain, nparts;
    PackX3 pg;
};
constexpr int kPackBatch = 36;  // 36 x 112-byte jobs: 3.9 KB of kernel arguments (the limit is 4 KB)
struct PackBatch {
    PackJob job[kPackBatch];
};
static_assert(sizeof(PackBatch) <= 4096, "pack_batch_kernel's arguments must fit the 4 KB kernel-argument limit");

// The absmax of the batch's larger tensors as its own launch in front of pack_batch_kernel: block
// (c, layer) reduces chunk c (kAbsChunk elements: one float4 per thread x 4 in flight) into
// partial[c] of the layer's workspace.  Without it every pack block of a layer re-reads the whole
// tensor for the scale (up to 32 blocks x 1.2 MB per MobileNetV2 1x1 layer: ~20 us per batch launch,
// profiles/r04_mobilenet32_kernel_stats.csv); max is order-free, so the result is the same bits.
constexpr int kAbsChunk = 4 * 256 * 4;  // = absmax_blocks' elements per partial
struct AbsJob {
    const float* w;
    unsigned* partial;
    int64_t n;
    int nparts;
};
struct AbsBatch {
    AbsJob job[kPackBatch];
};
static_assert(sizeof(AbsBatch) <= 4096, "absmax_batch_kernel's arguments must fit the 4 KB kernel-argument limit");
__global__ __launch_bounds__(256) void absmax_batch_kernel(AbsBatch B) {
    const AbsJob& j = B.job[blockIdx.y];
    if ((int)blockIdx.x >= j.nparts) return;  // block-uniform
    __shared__ unsigned red4[4];
    const int64_t c0 = (int64_t)blockIdx.x * kAbsChunk;
    const int64_t c1 = min(j.n, c0 + kAbsChunk);
    unsigned m = 0u;
    const bool aligned = ((reinterpret_cast<uintptr_t>(j.w) & 15u) == 0);
    if (aligned && c1 - c0 == kAbsChunk) {
        const float4* w4 = reinterpret_cast<const float4*>(j.w + c0);
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = w4[u * 256 + threadIdx.x];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const unsigned a = __float_as_uint(v[u].x) & 0x7fffffffu, b = __float_as_uint(v[u].y) & 0x7fffffffu;
            const unsigned c = __float_as_uint(v[u].z) & 0x7fffffffu, d = __float_as_uint(v[u].w) & 0x7fffffffu;
            m = max(m, max(max(a, b), max(c, d)));
        }
    } else {
        for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) m = max(m, __float_as_uint(j.w[i]) & 0x7fffffffu);
    }
    m = block_max_u32(m, red4);
    if (threadIdx.x == 0) j.partial[blockIdx.x] = m;
}

__global__ __launch_bounds__(kPackThreads) void pack_batch_kernel(PackBatch B) {
    const PackJob& j = B.job[blockIdx.y];
    if ((int)blockIdx.x >= j.nb) return;  // block-uniform
    if (j.plain) {
        __shared__ unsigned red[kPackThreads / 64];
        unsigned m0 = 0u;
        if (j.nparts > 0) {
            for (int i = threadIdx.x; i < j.nparts; i += kPackThreads) m0 = max(m0, j.partial[i]);
        } else {
            m0 = fused_absmax_bits(j.w, j.n);
        }
        const unsigned m = block_max_u32<kPackThreads / 64>(m0, red);
        const float scale = __uint_as_float(m);
        float* out = reinterpret_cast<float*>(j.packed);
        for (int i = blockIdx.x * kPackThreads + threadIdx.x; i < (int)j.n; i += j.nb * kPackThreads)
            out[i] = quantize_elem(j.w[i], scale, j.mode, j.lo, j.hi);
        return;
    }
    pack_bf16x3_body(j.w, j.n, j.partial, j.nparts, j.lo, j.hi, j.mode, j.pg, reinterpret_cast<uint16_t*>(j.packed),
                     j.scale, (int)blockIdx.x, j.nb);
}

static PackX3 pack_geom(const ConvPlan& p) {
    PackX3 pg;
    pg.C = p.C; pg.K = p.K; pg.R = p.R; pg.S = p.S; pg.CC = p.CC; pg.NT = p.NT;
    pg.nchunks = p.nchunks; pg.ksteps = p.steps; pg.taps = p.taps;
    pg.vr = (p.kind == KIND_BF16X3_ROWS || p.kind == KIND_BF16X3_IMG) ? 2 : (p.vrx ? 1 : 0);
    pg.total = p.packed_floats * 2;
    return pg;
}

static int pack_blocks(const PackX3& pg) {
    int64_t b = (pg.total / 8 + kPackThreads - 1) / kPackThreads;  // one 16-byte fragment slot per thread
    return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 32);
}

bool pack_batchable(const ConvPlan& p, int mode) {
    const int64_t n = (int64_t)p.K * p.Cg * p.R * p.S;
    if (mode == 0 || n > kFusedAbsmaxMax) return false;
    return is_bf16x3_kind(p.kind) || p.kind == KIND_DEPTHWISE;
}

// tensors above this many weights get their absmax from absmax_batch_kernel (a pack block would
// otherwise re-read more than this per block for the scale)
constexpr int64_t kTwoPhaseAbsmax = 16384;

hipError_t launch_pack_batch(int n, const PackReq* reqs, hipStream_t s) {
    for (int i0 = 0; i0 < n; i0 += kPackBatch) {
        PackBatch B;
        AbsBatch A;
        const int m = std::min(kPackBatch, n - i0);
        int nbmax = 1, npmax = 0;
        for (int i = 0; i < m; ++i) {
            const PackReq& r = reqs[i0 + i];
            const ConvPlan& p = *r.plan;
            PackJob& j = B.job[i];
            int lo, hi;
            clamp_window(r.bits, r.fsr, lo, hi);
            j.w = r.w;
            j.packed = r.packed;
            j.scale = r.scale;
            j.n = (int64_t)p.K * p.Cg * p.R * p.S;
            j.nparts = (r.partial && j.n > kTwoPhaseAbsmax) ? (int)((j.n + kAbsChunk - 1) / kAbsChunk) : 0;
            j.partial = r.partial;
            A.job[i] = AbsJob{r.w, r.partial, j.n, j.nparts};
            npmax = std::max(npmax, j.nparts);
            j.lo = lo; j.hi = hi; j.mode = r.mode - 1;
            j.plain = p.kind == KIND_DEPTHWISE ? 1 : 0;
            if (j.plain) {
                j.pg = PackX3{};
                j.nb = (int)std::min<int64_t>(8, (j.n + kPackThreads * 4 - 1) / (kPackThreads * 4));
            } else {
                j.pg = pack_geom(p);
                j.nb = pack_blocks(j.pg);
            }
            nbmax = std::max(nbmax, j.nb);
        }
        if (npmax > 0) {
            hipLaunchKernelGGL(absmax_batch_kernel, dim3((unsigned)npmax, (unsigned)m), dim3(256), 0, s, A);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(pack_batch_kernel, dim3((unsigned)nbmax, (unsigned)m), dim3(kPackThreads), 0, s, B);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pack_bf16x3_batch(int n, const ConvPlan* const* plans, const float* const* w,
                                    uint16_t* const* packed, float* const* scale_out, int bits, int fsr, int mode,
                                    hipStream_t s) {
    std::vector<PackReq> reqs((size_t)n);
    for (int i = 0; i < n; ++i) reqs[i] = PackReq{plans[i], w[i], packed[i], scale_out[i], bits, fsr, mode};
    return launch_pack_batch(n, reqs.data(), s);
}

hipError_t launch_pack_bf16x3(const ConvPlan& p, const float* w, const unsigned* partial, int nparts, int bits,
                              int fsr, int mode, uint16_t* packed, float* scale_out, hipStream_t s) {
    int lo, hi;
    clamp_window(bits, fsr, lo, hi);
    const PackX3 pg = pack_geom(p);
    const int b = pack_blocks(pg);
    const int64_t n = (int64_t)p.K * p.Cg * p.R * p.S;
    hipLaunchKernelGGL(pack_bf16x3_kernel, dim3((unsigned)b), dim3(kPackThreads), 0, s, w, n, partial, nparts, lo, hi,
                       mode - 1, pg, packed, scale_out);
    return hipGetLastError();
}

hipError_t launch_pack_weights(const ConvPlan& p, const float* w, const unsigned* partial, int nparts, int bits,
                               int fsr, int mode, float* packed, hipStream_t s) {
    int lo = 0, hi = 0;
    if (mode != 0) clamp_window(bits, fsr, lo, hi);
    if (p.kind == KIND_DEPTHWISE) {  // depthwise: plain [K][1][R][S] quantized copy
        const int64_t n = (int64_t)p.K * p.Cg * p.R * p.S;
        if (mode == 0) return hipMemcpyAsync(packed, w, n * sizeof(float), hipMemcpyDeviceToDevice, s);
        if (nparts == 0) {  // fused absmax (small tensor)
            const int b = (int)std::min<int64_t>(8, (n + 4095) / 4096);
            hipLaunchKernelGGL(quantize_plain_fused_kernel, dim3(b), dim3(1024), 0, s, w, (int)n, lo, hi, mode - 1,
                               packed);
            return hipGetLastError();
        }
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
