// Weight gradient of the quantized conv for the QAT backward:
//   dW[k][c][r][s] = sum_{n,p,q} dy[n][k][p][q] * x[n][c][p*sh + r*dh - ph][q*sw + s*dw - pw]
// i.e. the gradient autograd takes through F.conv2d(x, Q(w), ...) (reference
// models/quantized_conv.py:35-36; the straight-through estimator of
// utils/quantizers.py:34-36 passes it to w unchanged; train.py:79-91 runs it).
//
// fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation) as a GEMM
// D[k][c] += A[k][pixel] B[pixel][c] per tap (r, s), both operands fp32 activations --
// neither is a power of two, so the bf16x3 trick of the forward does not apply.
//
//   * a block owns (image n, a tile of QT output columns, 16 output channels k0.., 16
//     input channels c0..) and walks the image in bands of BP output rows: the band's dy
//     rows [16][BP][QT] and the x rows they touch [16][XR][WT] are staged in LDS (channel
//     strides padded odd: conflict-free ds_read_b32), then each wave takes 4-pixel chunks:
//     one A value and R*S B values per lane, R*S MFMAs into R*S accumulator tiles
//     (independent chains);
//   * the 4 waves' tiles are summed in LDS in a fixed order and the block writes its
//     partial [16][16][R*S]; wgrad_reduce sums the partials of every (image, column tile)
//     per weight in a fixed order (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/po2q.h"
#include "po2q_internal.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

struct WgradArgs {
    int N, C, H, W, K, P, Q, R, S, sh, sw, ph, pw, dh, dw;
    int BP;           // output rows per band
    int XR;           // x rows staged per band: (BP - 1) * sh + (R - 1) * dh + 1
    int QT, WT, nqt;  // output columns per tile, x columns staged per tile, column tiles
    int gstride;      // LDS floats per dy channel (odd)
    int xstride;      // LDS floats per x channel (odd)
    int KT, CT;       // 16-channel tiles of K and C
};

template <int R, int S>
__global__ __launch_bounds__(256) void wgrad_f32(const float* __restrict__ x, const float* __restrict__ dy,
                                                 float* __restrict__ part, WgradArgs a) {
    constexpr int NTAP = R * S;
    extern __shared__ float sm[];
    float* gl = sm;                      // [16][gstride]
    float* xl = sm + 16 * a.gstride;     // [16][xstride]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b = blockIdx.x;
    const int ct = b % a.CT; b /= a.CT;
    const int kt = b % a.KT; b /= a.KT;
    const int qt = b % a.nqt;
    const int n = b / a.nqt;
    const int qs = qt * a.QT;                 // first output column of the tile
    const int qn = min(a.QT, a.Q - qs);       // its width
    const int ws0 = qs * a.sw - a.pw;         // first staged x column
    const int k0 = kt * 16, c0 = ct * 16;
    const int PQ = a.P * a.Q, HW = a.H * a.W;
    const float* dyn = dy + ((int64_t)n * a.K + k0) * PQ;
    const float* xn = x + ((int64_t)n * a.C + c0) * HW;
    floatx4 acc[NTAP];
#pragma unroll
    for (int t = 0; t < NTAP; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int ch = lane & 15, pj = lane >> 4;  // operand lane: channel, pixel of the chunk
    const int qc = (qn + 3) >> 2;
    for (int p0 = 0; p0 < a.P; p0 += a.BP) {
        const int bp = min(a.BP, a.P - p0);
        const int h0 = p0 * a.sh - a.ph;
        __syncthreads();  // the previous band's reads are done
        // stage dy rows p0 .. p0+bp-1 of the 16 channels (k >= K as zero), one row per wave
        for (int row = wave; row < 16 * bp; row += 4) {
            const int c = row / bp, pr = row - c * bp;
            const bool ok = k0 + c < a.K;
            const float* src = dyn + (int64_t)c * PQ + (int64_t)(p0 + pr) * a.Q + qs;
            float* dst = gl + c * a.gstride + pr * a.QT;
            for (int i = lane; i < qn; i += 64) dst[i] = ok ? src[i] : 0.0f;
        }
        // stage x rows h0 .. h0+XR-1 (rows outside the image and c >= C as zero)
        for (int row = wave; row < 16 * a.XR; row += 4) {
            const int c = row / a.XR, hr = row - c * a.XR;
            const int h = h0 + hr;
            const bool ok = c0 + c < a.C && h >= 0 && h < a.H;
            const float* src = xn + (int64_t)c * HW + (int64_t)(ok ? h : 0) * a.W;
            float* dst = xl + c * a.xstride + hr * a.WT;
            for (int i = lane; i < a.WT; i += 64) {
                const int w = ws0 + i;
                dst[i] = (ok && w >= 0 && w < a.W) ? src[w] : 0.0f;
            }
        }
        __syncthreads();
        // chunks of 4 consecutive output columns of one row, dealt round-robin to the waves
        for (int ci = wave; ci < bp * qc; ci += 4) {
            const int pr = ci / qc;
            const int q = ((ci - pr * qc) << 2) + pj;
            const bool qok = q < qn;
            const float av = qok ? gl[ch * a.gstride + pr * a.QT + q] : 0.0f;
            // staged column of tap s: q * sw + s * dw (zero padding is staged as zeros)
            const float* xr0 = xl + ch * a.xstride + pr * a.sh * a.WT + q * a.sw;
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const float bv = qok ? xr0[r * a.dh * a.WT + s * a.dw] : 0.0f;
                    acc[r * S + s] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[r * S + s], 0, 0, 0);
                }
        }
    }
    // sum the 4 waves' tiles in LDS (fixed order), write the block partial
    // [16 k][16 c][R*S] at part[n][kt][ct]
    __syncthreads();
    float* red = sm;  // [4 waves][NTAP][64 lanes][4]
#pragma unroll
    for (int t = 0; t < NTAP; ++t)
        *reinterpret_cast<floatx4*>(red + ((wave * NTAP + t) * 64 + lane) * 4) = acc[t];
    __syncthreads();
    float* out = part + ((((int64_t)n * a.nqt + qt) * a.KT + kt) * a.CT + ct) * (256 * NTAP);
    for (int e = tid; e < 256 * NTAP; e += 256) {
        // e = ((kl * 16) + cl) * NTAP + t  ->  lane = (kl >> 2) * 16 + cl, i = kl & 3
        const int t = e % NTAP, cl = (e / NTAP) & 15, kl = e / (NTAP * 16);
        const int ln = ((kl >> 2) << 4) + cl, i = kl & 3;
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * NTAP + t) * 64 + ln) * 4 + i];
        out[e] = v;
    }
}

// dW[k][c][t] = sum over images (in order) of the partials
__global__ __launch_bounds__(256) void wgrad_reduce(const float* __restrict__ part, float* __restrict__ dw, int N, int K,
                                                    int C, int ntap, int KT, int CT) {
    const int total = K * C * ntap;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
        const int t = e % ntap, c = (e / ntap) % C, k = e / (ntap * C);
        const int kt = k >> 4, ct = c >> 4;
        const int64_t off = (int64_t)(kt * CT + ct) * (256 * ntap) + ((k & 15) * 16 + (c & 15)) * ntap + t;
        float v = 0.0f;
        for (int n = 0; n < N; ++n) v += part[(int64_t)n * KT * CT * (256 * ntap) + off];  // N = images x tiles
        dw[e] = v;
    }
}


// ---- register-streaming kernel (dilation 1, equal strides 1 or 2, 1x1 / 3x3) ------------
//
// The reduction (n, p, q) is long and the output (K x C x R x S) small, so the kernel is
// built around one long, resident accumulator set per wave and operands streamed straight
// from HBM into VGPRs (no LDS staging):
//   * wave work item = (image n, strip of 16 output columns, segment of RB output rows) of
//     one channel group (16*KW output x 16*CW input channels); lane (ch = l & 15,
//     pj = l >> 4) holds dy[k0 + ch][p][q' .. q'+3] (one dwordx4, q' = strip*16 + 4 pj) and
//     the input span x[c0 + ch][h][SH*q' - pw ...] the four pixels' taps touch;
//   * MFMA k-slot pj of v_mfma_f32_16x16x4f32 number m takes pixel q' + m, so one dwordx4
//     of dy and one span of x feed 4 * R * S * KW * CW MFMAs; D[k][c] per tap stays in the
//     wave's accumulators for the whole segment;
//   * stride 1, 3x3: the three x rows of an output row are a 4-slot register ring -- each
//     step loads one new x row and one dy row for the NEXT step (the compiler's counted
//     vmcnt wait covers the current one); other shapes load their R rows one step ahead;
//   * out-of-image rows / columns, channels past C / K and pixels past P / Q load as zero
//     (out-of-range buffer offsets), so no branch in the loop depends on position;
//   * the 4 waves of a block (4 consecutive items of one channel group) sum their tiles in
//     LDS in a fixed order and the block writes one partial; wgrad2_reduce sums the partials
//     of a channel group in a fixed order (deterministic, no atomics).
struct Wgrad2Args {
    int N, C, H, W, K, P, Q, ph, pw;
    int RB, nseg, nstrip;  // output rows per segment, segments, 16-column strips
    int items;             // work items per channel group: N * nseg * nstrip
    int bpg;               // blocks per channel group: ceil(items / 4)
    int KG, CG;            // channel groups along K (16*KW each) and C (16*CW each)
};

constexpr uint32_t kOob = 0x80000000u;  // a buffer offset past every range: loads 0

__device__ __forceinline__ float wg_ld1(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
}
__device__ __forceinline__ floatx4 wg_ld4(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

template <int R, int S, int SH, int PW, int KW, int CW, bool VEC>
__global__ __launch_bounds__(256, KW * CW == 4 ? 1 : 2) void wgrad2_f32(const float* __restrict__ x, const float* __restrict__ dy,
                                                     float* __restrict__ part, Wgrad2Args a) {
    constexpr int NT = R * S;
    constexpr int SPAN = 3 * SH + S;                           // x columns of 4 pixels' taps
    constexpr int NB = VEC ? (SPAN - PW) / 4 : 0;              // dwordx4 pieces of the span
    constexpr int NTAIL = VEC ? SPAN - PW - 4 * NB : 0;        // dwords after them
    constexpr bool RING = (SH == 1 && R == 3);
    __shared__ floatx4 red[4][NT][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = blockIdx.x / a.bpg, bi = blockIdx.x - g * a.bpg;
    const int kg = g / a.CG, cg = g - kg * a.CG;
    const int item = bi * 4 + wave;
    floatx4 acc[KW][CW][NT];
#pragma unroll
    for (int i = 0; i < KW; ++i)
#pragma unroll
        for (int j = 0; j < CW; ++j)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[i][j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (item < a.items) {
        const int strip = item % a.nstrip;
        const int t2 = item / a.nstrip;
        const int seg = t2 % a.nseg, n = t2 / a.nseg;
        const int ch = lane & 15, pj = lane >> 4;
        const int q1 = strip * 16 + 4 * pj;  // first output column of the lane's 4 pixels
        const int PQ = a.P * a.Q, HW = a.H * a.W;
        const __amdgpu_buffer_rsrc_t rd = rows_rsrc(dy + (int64_t)n * a.K * PQ, a.K * PQ * 4);
        const __amdgpu_buffer_rsrc_t rx = rows_rsrc(x + (int64_t)n * a.C * HW, a.C * HW * 4);
        // per-lane channel bases (or kOob for channels past K / C)
        uint32_t dbase[KW], xbase[CW];
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int k = kg * 16 * KW + 16 * i + ch;
            dbase[i] = k < a.K ? (uint32_t)k * (uint32_t)PQ * 4u : kOob;
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            const int c = cg * 16 * CW + 16 * j + ch;
            xbase[j] = c < a.C ? (uint32_t)c * (uint32_t)HW * 4u : kOob;
        }
        const int pw = VEC ? PW : a.pw;
        const int col0 = SH * q1 - pw;  // x column of span element 0
        const int p0 = seg * a.RB;
        auto load_dy = [&](float (&dv)[KW][4], int p) __attribute__((always_inline)) {
            const bool prow = p < a.P && p < p0 + a.RB;
#pragma unroll
            for (int i = 0; i < KW; ++i) {
                if constexpr (VEC) {
                    const uint32_t off =
                        (prow && q1 < a.Q && dbase[i] != kOob) ? dbase[i] + (uint32_t)(p * a.Q + q1) * 4u : kOob;
                    const floatx4 v = wg_ld4(rd, off);
#pragma unroll
                    for (int m = 0; m < 4; ++m) dv[i][m] = v[m];
                } else {
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const uint32_t off = (prow && q1 + m < a.Q && dbase[i] != kOob)
                                                 ? dbase[i] + (uint32_t)(p * a.Q + q1 + m) * 4u
                                                 : kOob;
                        dv[i][m] = wg_ld1(rd, off);
                    }
                }
            }
        };
        auto load_x = [&](float (&xv)[CW][SPAN], int h) __attribute__((always_inline)) {
            const bool hrow = h >= 0 && h < a.H;
            const uint32_t rowoff = (uint32_t)(hrow ? h : 0) * (uint32_t)a.W * 4u;
#pragma unroll
            for (int j = 0; j < CW; ++j) {
                const bool ok = hrow && xbase[j] != kOob;
                const uint32_t b = xbase[j] + rowoff;
                if constexpr (VEC) {
#pragma unroll
                    for (int i = 0; i < PW; ++i) {
                        const int col = col0 + i;
                        xv[j][i] = wg_ld1(rx, (ok && col >= 0 && col < a.W) ? b + (uint32_t)col * 4u : kOob);
                    }
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int col = SH * q1 + 4 * u;  // a multiple of 4; W % 4 == 0
                        const floatx4 v = wg_ld4(rx, (ok && col < a.W) ? b + (uint32_t)col * 4u : kOob);
#pragma unroll
                        for (int e = 0; e < 4; ++e) xv[j][PW + 4 * u + e] = v[e];
                    }
#pragma unroll
                    for (int i = 0; i < NTAIL; ++i) {
                        const int col = SH * q1 + 4 * NB + i;
                        xv[j][PW + 4 * NB + i] = wg_ld1(rx, (ok && col < a.W) ? b + (uint32_t)col * 4u : kOob);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < SPAN; ++i) {
                        const int col = col0 + i;
                        xv[j][i] = wg_ld1(rx, (ok && col >= 0 && col < a.W) ? b + (uint32_t)col * 4u : kOob);
                    }
                }
            }
        };
        auto mfmas = [&](const float (&dv)[KW][4], const float (&x0)[CW][SPAN], const float (&x1)[CW][SPAN],
                         const float (&x2)[CW][SPAN]) __attribute__((always_inline)) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int s = 0; s < S; ++s)
#pragma unroll
                        for (int i = 0; i < KW; ++i)
#pragma unroll
                            for (int j = 0; j < CW; ++j) {
                                const float bv = r == 0 ? x0[j][SH * m + s] : r == 1 ? x1[j][SH * m + s]
                                                                                     : x2[j][SH * m + s];
                                acc[i][j][r * S + s] =
                                    __builtin_amdgcn_mfma_f32_16x16x4f32(dv[i][m], bv, acc[i][j][r * S + s], 0, 0, 0);
                            }
        };
        float dv[2][KW][4];
        if constexpr (RING) {
            // x rows p - ph + r (r = 0..2) of output row p live in ring slots (p - p0 + r) & 3
            float xr[4][CW][SPAN];
            const int hb = p0 - a.ph;
            load_x(xr[0], hb);
            load_x(xr[1], hb + 1);
            load_x(xr[2], hb + 2);
            load_dy(dv[0], p0);
            for (int jb = 0; jb < a.RB; jb += 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    load_x(xr[(j + 3) & 3], hb + jb + j + 3);
                    load_dy(dv[(j + 1) & 1], p0 + jb + j + 1);
                    mfmas(dv[j & 1], xr[j & 3], xr[(j + 1) & 3], xr[(j + 2) & 3]);
                }
            }
        } else {
            float xs[2][R][CW][SPAN];
#pragma unroll
            for (int r = 0; r < R; ++r) load_x(xs[0][r], p0 * SH - a.ph + r);
            load_dy(dv[0], p0);
            for (int jb = 0; jb < a.RB; jb += 2) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int pn = p0 + jb + j + 1;
#pragma unroll
                    for (int r = 0; r < R; ++r) load_x(xs[(j + 1) & 1][r], pn * SH - a.ph + r);
                    load_dy(dv[(j + 1) & 1], pn);
                    mfmas(dv[j & 1], xs[j & 1][0], xs[j & 1][R > 1 ? 1 : 0], xs[j & 1][R > 2 ? 2 : 0]);
                }
            }
        }
    }
    // block partial part[g][bi][kk][cc][t] (kk < 16 KW, cc < 16 CW): the 4 waves' tiles summed
    // in wave order, one (KW, CW) tile pair at a time through LDS
    constexpr int KT = 16 * KW, CT = 16 * CW, PER = KT * CT * NT;
    float* out = part + ((int64_t)g * a.bpg + bi) * PER;
#pragma unroll
    for (int i = 0; i < KW; ++i)
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            if (i + j) __syncthreads();  // the previous pair's reads are done
#pragma unroll
            for (int t = 0; t < NT; ++t) red[wave][t][lane] = acc[i][j][t];
            __syncthreads();
            for (int e = threadIdx.x; e < 256 * NT; e += 256) {
                // e = (kl * 16 + cl) * NT + t; MFMA D layout: lane (kl >> 2) * 16 + cl, element kl & 3
                const int t = e % NT, cl = (e / NT) & 15, kl = e / (NT * 16);
                const int ln = ((kl >> 2) << 4) + cl, v = kl & 3;
                float sum = 0.0f;
#pragma unroll
                for (int w = 0; w < 4; ++w) sum += red[w][t][ln][v];
                out[((16 * i + kl) * CT + 16 * j + cl) * NT + t] = sum;
            }
        }
}

// dW[k][c][t] = sum over the channel group's block partials, in block order.  Block =
// 64 consecutive partial elements x 16 slices of the partial list (1024 threads); the 16
// slice sums are added in slice order.
__global__ __launch_bounds__(1024) void wgrad2_reduce(const float* __restrict__ part, float* __restrict__ dw, int K,
                                                      int C, int NT, int KT, int CT, int CG, int bpg) {
    __shared__ float red[16][64];
    const int PER = KT * CT * NT;
    const int chunks = (PER + 63) / 64;
    const int g = blockIdx.x / chunks;
    const int e = (blockIdx.x - g * chunks) * 64 + (threadIdx.x & 63);
    const int sl = threadIdx.x >> 6;
    float v = 0.0f;
    if (e < PER) {
        const float* src = part + (int64_t)g * bpg * PER + e;
        for (int b = sl; b < bpg; b += 16) v += src[(int64_t)b * PER];
    }
    red[sl][threadIdx.x & 63] = v;
    __syncthreads();
    if (sl == 0 && e < PER) {
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) sum += red[i][threadIdx.x];
        const int t = e % NT, cc = (e / NT) % CT, kk = e / (NT * CT);
        const int kg = g / CG, cg = g - kg * CG;
        const int k = kg * KT + kk, c = cg * CT + cc;
        if (k < K && c < C) dw[((int64_t)k * C + c) * NT + t] = sum;
    }
}

bool wgrad_plan(WgradArgs& a, size_t& lds, size_t& part_bytes) {
    if (!((a.R == 3 && a.S == 3) || (a.R == 1 && a.S == 1))) return false;
    a.KT = (a.K + 15) / 16;
    a.CT = (a.C + 15) / 16;
    // column tiles of up to 64 output columns; band height: staged dy + x rows within 60 KiB
    a.QT = std::min(a.Q, 64);
    a.nqt = (a.Q + a.QT - 1) / a.QT;
    a.WT = (a.QT - 1) * a.sw + (a.S - 1) * a.dw + 1;
    const size_t budget = 60 * 1024 / 4;
    int bp = std::min(a.P, 64);
    for (; bp > 1; --bp) {
        const int xr = (bp - 1) * a.sh + (a.R - 1) * a.dh + 1;
        if ((size_t)16 * (bp * a.QT + 1) + 16 * ((size_t)xr * a.WT + 1) <= budget) break;
    }
    a.BP = bp;
    a.XR = (bp - 1) * a.sh + (a.R - 1) * a.dh + 1;
    a.gstride = (a.BP * a.QT) | 1;
    a.xstride = (a.XR * a.WT) | 1;
    lds = std::max((size_t)16 * (a.gstride + a.xstride), (size_t)4 * 9 * 64 * 4) * sizeof(float);
    if (lds > 64 * 1024) return false;
    part_bytes = (size_t)a.N * a.nqt * a.KT * a.CT * 256 * a.R * a.S * sizeof(float);
    return true;
}

hipError_t launch_wgrad(const WgradArgs& a0, const float* x, const float* dy, float* dw, float* part, size_t lds,
                        hipStream_t s) {
    const WgradArgs a = a0;
    const unsigned blocks = (unsigned)(a.N * a.nqt * a.KT * a.CT);
    const int ntap = a.R * a.S;
    if (a.R == 3 && a.S == 3)
        hipLaunchKernelGGL((wgrad_f32<3, 3>), dim3(blocks), dim3(256), lds, s, x, dy, part, a);
    else if (a.R == 1 && a.S == 1)
        hipLaunchKernelGGL((wgrad_f32<1, 1>), dim3(blocks), dim3(256), lds, s, x, dy, part, a);
    else
        return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int total = a.K * a.C * ntap;
    const int rb = std::min(1024, std::max(1, (total + 255) / 256));
    hipLaunchKernelGGL(wgrad_reduce, dim3(rb), dim3(256), 0, s, part, dw, a.N * a.nqt, a.K, a.C, ntap, a.KT, a.CT);
    return hipGetLastError();
}

// Register-streaming plan: dilation 1, sh == sw in {1, 2}, 1x1 (pad 0) or 3x3 kernels.
// Rows per segment: the largest multiple of 4 that still gives >= 4096 waves in total
// (16 per CU), at least 4.
bool wgrad2_plan(Wgrad2Args& a, int R, int S, int sh, int sw, int dh, int dw, int& SH, int& KW, int& CW, bool& vec,
                 size_t& part_bytes) {
    if (dh != 1 || dw != 1 || sh != sw || (sh != 1 && sh != 2)) return false;
    if (!((R == 3 && S == 3) || (R == 1 && S == 1))) return false;
    SH = sh;
    KW = a.K > 16 ? 2 : 1;
    CW = a.C > 16 ? 2 : 1;
    const int pwv = R == 3 ? 1 : 0;
    vec = a.W % 4 == 0 && a.Q % 4 == 0 && a.pw == pwv;
    a.KG = (a.K + 16 * KW - 1) / (16 * KW);
    a.CG = (a.C + 16 * CW - 1) / (16 * CW);
    a.nstrip = (a.Q + 15) / 16;
    const int64_t per_seg = (int64_t)a.KG * a.CG * a.N * a.nstrip;
    const int P4 = (a.P + 3) / 4 * 4;
    int rb = 4;
    for (int c = P4; c >= 4; c -= 4) {
        const int64_t nseg = (a.P + c - 1) / c;
        if (per_seg * nseg >= 4096) { rb = c; break; }
    }
    a.RB = rb;
    a.nseg = (a.P + rb - 1) / rb;
    const int64_t items = (int64_t)a.N * a.nseg * a.nstrip;
    if (items > INT32_MAX / 4) return false;
    a.items = (int)items;
    a.bpg = (a.items + 3) / 4;
    part_bytes = (size_t)a.KG * a.CG * a.bpg * (16 * KW) * (16 * CW) * R * S * sizeof(float);
    return true;
}

template <int R, int S, int SH, int PW, int KW, int CW>
void launch_wgrad2_t(bool vec, const Wgrad2Args& a, const float* x, const float* dy, float* part, hipStream_t st) {
    const dim3 grid((unsigned)(a.KG * a.CG * a.bpg));
    if (vec)
        hipLaunchKernelGGL((wgrad2_f32<R, S, SH, PW, KW, CW, true>), grid, dim3(256), 0, st, x, dy, part, a);
    else
        hipLaunchKernelGGL((wgrad2_f32<R, S, SH, PW, KW, CW, false>), grid, dim3(256), 0, st, x, dy, part, a);
}

template <int R, int S, int SH, int PW>
void launch_wgrad2_k(int KW, int CW, bool vec, const Wgrad2Args& a, const float* x, const float* dy, float* part,
                     hipStream_t st) {
    if (KW == 1 && CW == 1) launch_wgrad2_t<R, S, SH, PW, 1, 1>(vec, a, x, dy, part, st);
    else if (KW == 2 && CW == 1) launch_wgrad2_t<R, S, SH, PW, 2, 1>(vec, a, x, dy, part, st);
    else if (KW == 1 && CW == 2) launch_wgrad2_t<R, S, SH, PW, 1, 2>(vec, a, x, dy, part, st);
    else launch_wgrad2_t<R, S, SH, PW, 2, 2>(vec, a, x, dy, part, st);
}

hipError_t launch_wgrad2(const Wgrad2Args& a, int R, int SH, int KW, int CW, bool vec, const float* x, const float* dy,
                         float* dw, float* part, hipStream_t st) {
    if (R == 3 && SH == 1) launch_wgrad2_k<3, 3, 1, 1>(KW, CW, vec, a, x, dy, part, st);
    else if (R == 3 && SH == 2) launch_wgrad2_k<3, 3, 2, 1>(KW, CW, vec, a, x, dy, part, st);
    else if (R == 1 && SH == 1) launch_wgrad2_k<1, 1, 1, 0>(KW, CW, vec, a, x, dy, part, st);
    else if (R == 1 && SH == 2) launch_wgrad2_k<1, 1, 2, 0>(KW, CW, vec, a, x, dy, part, st);
    else return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int KT = 16 * KW, CT = 16 * CW, NT = R * R;
    const int chunks = (KT * CT * NT + 63) / 64;
    hipLaunchKernelGGL(wgrad2_reduce, dim3((unsigned)(a.KG * a.CG * chunks)), dim3(1024), 0, st, part, dw, a.K, a.C,
                       NT, KT, CT, a.CG, a.bpg);
    return hipGetLastError();
}

}  // namespace po2q

namespace {

bool wgrad_setup(po2q::WgradArgs& a, size_t& lds, size_t& part, int64_t N, int64_t C, int64_t H, int64_t W,
                 int64_t K, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                 int64_t dw, int64_t groups) {
    if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || K <= 0 || R <= 0 || S <= 0 || sh <= 0 || sw <= 0 || dh <= 0 ||
        dw <= 0 || ph < 0 || pw < 0) {
        po2q::set_error("po2q: wgrad: sizes, strides and dilations must be positive, padding non-negative");
        return false;
    }
    if (groups != 1 || !((R == 3 && S == 3) || (R == 1 && S == 1))) {
        po2q::set_error("po2q: wgrad: groups == 1 and a 1x1 or 3x3 kernel only");
        return false;
    }
    const int64_t P = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1, Q = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
    if (P <= 0 || Q <= 0 || N * C * H * W > INT32_MAX || N * K * P * Q > INT32_MAX) {
        po2q::set_error("po2q: wgrad: empty output or tensor too large");
        return false;
    }
    a.N = (int)N; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.K = (int)K; a.P = (int)P; a.Q = (int)Q;
    a.R = (int)R; a.S = (int)S; a.sh = (int)sh; a.sw = (int)sw; a.ph = (int)ph; a.pw = (int)pw;
    a.dh = (int)dh; a.dw = (int)dw;
    if (!po2q::wgrad_plan(a, lds, part)) {
        po2q::set_error("po2q: wgrad: no plan fits the LDS budget");
        return false;
    }
    return true;
}

// The register-streaming kernel where it applies (PO2Q_WGRAD=1 forces the LDS-band kernel)
struct Wgrad2Choice {
    bool use = false;
    po2q::Wgrad2Args a;
    int R = 0, SH = 0, KW = 0, CW = 0;
    bool vec = false;
    size_t part = 0;
};

Wgrad2Choice wgrad2_choose(const po2q::WgradArgs& a1) {
    Wgrad2Choice c;
    static const int force1 = [] {
        const char* e = getenv("PO2Q_WGRAD");
        return e ? atoi(e) : 0;
    }();
    if (force1 == 1) return c;
    po2q::Wgrad2Args& a = c.a;
    a.N = a1.N; a.C = a1.C; a.H = a1.H; a.W = a1.W; a.K = a1.K; a.P = a1.P; a.Q = a1.Q; a.ph = a1.ph; a.pw = a1.pw;
    c.use = po2q::wgrad2_plan(a, a1.R, a1.S, a1.sh, a1.sw, a1.dh, a1.dw, c.SH, c.KW, c.CW, c.vec, c.part);
    c.R = a1.R;
    return c;
}

}  // namespace

// depthwise layers (groups == C == K): po2q_bwd.hip
size_t po2q_dw_wgrad_workspace_bytes_internal(int64_t N, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                                              int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                                              int64_t dw);
int po2q_dw_wgrad_f32_internal(const float* x, const float* dy, float* dwt, int64_t N, int64_t C, int64_t H,
                               int64_t W, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                               int64_t dh, int64_t dw, void* workspace, size_t workspace_bytes, void* stream);

static bool wgrad_depthwise(int64_t C, int64_t K, int64_t groups) { return groups > 1 && groups == C && K == C; }

size_t po2q_qconv2d_wgrad_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                                          int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                                          int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups) {
    if (wgrad_depthwise(C, K, groups))
        return po2q_dw_wgrad_workspace_bytes_internal(N, C, H, W, R, S, stride_h, stride_w, pad_h, pad_w, dil_h,
                                                      dil_w);
    po2q::WgradArgs a;
    size_t lds, part;
    if (!wgrad_setup(a, lds, part, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups))
        return 0;
    const Wgrad2Choice c2 = wgrad2_choose(a);
    return std::max<size_t>(c2.use ? c2.part : part, 256);
}

int po2q_qconv2d_wgrad_f32(const float* x, const float* dy, float* dw, int64_t N, int64_t C, int64_t H, int64_t W,
                           int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                           int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, void* workspace,
                           size_t workspace_bytes, void* stream) {
    if (wgrad_depthwise(C, K, groups))
        return po2q_dw_wgrad_f32_internal(x, dy, dw, N, C, H, W, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w,
                                          workspace, workspace_bytes, stream);
    po2q::WgradArgs a;
    size_t lds, part;
    if (!wgrad_setup(a, lds, part, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups))
        return (groups != 1 || !((R == 3 && S == 3) || (R == 1 && S == 1))) ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    if (!x || !dy || !dw || !workspace) {
        po2q::set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    const Wgrad2Choice c2 = wgrad2_choose(a);
    if (c2.use) part = c2.part;
    if (workspace_bytes < part) {
        po2q::set_error("po2q: wgrad workspace too small (need " + std::to_string(part) + " bytes)");
        return PO2Q_ERR_WORKSPACE;
    }
    const hipError_t e =
        c2.use ? po2q::launch_wgrad2(c2.a, c2.R, c2.SH, c2.KW, c2.CW, c2.vec, x, dy, dw,
                                     reinterpret_cast<float*>(workspace), reinterpret_cast<hipStream_t>(stream))
               : po2q::launch_wgrad(a, x, dy, dw, reinterpret_cast<float*>(workspace), lds,
                                    reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: wgrad launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}
