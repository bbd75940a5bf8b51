// Depthwise 3x3 conv (groups == C == K, pad 1, stride 1 or 2, dilation 1): the MobileNetV2
// inverted-residual depthwise layers (reference models/mobilenet.py:64-76, each a
// QuantizedConv2d with groups = hidden_dim, models/quantized_conv.py:32-38), with the
// block's eval BatchNorm affine + ReLU6 (mobilenet.py:32-33) in the store epilogue.
//
// HBM-bound (9 MACs per output element): one block owns (image, CB channels, band of TP
// output rows).  The band's input rows of its CB channel planes are staged in LDS with a
// zero halo -- one coalesced float4 global load per 4 input pixels, written at a 16-byte
// aligned interior (column w at float offset 4 + w of a row of WS = roundup4(W) + 8 floats;
// the left halo is offset 3) -- then each thread computes 4 consecutive outputs of one row:
// 3 input rows x (one ds_read_b128 + two ds_read_b32) for stride 1, (two b128 + one b32)
// for stride 2, 36 FMAs, one float4 store.  Weights are the quantized fp32 Q(w) [C][9]
// (the depthwise pack, po2q_quant.hip), 9 per channel in registers.  Index decode is
// 32-bit; the divisions are by block-uniform sizes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

struct DwArgs {
    int N, C, H, W, P, Q;
    int CB, TP, TH, WS;   // channels per block, output rows per band, staged input rows, LDS row stride
    int nbands, ncb, QJ;  // bands per plane, channel blocks, float4 column groups per output row
    const float* ps;      // fused epilogue (EPI): y = act(y * ps[c] + pb[c] (+ res)); NULL parts skipped
    const float* pb;
    const float* res;
    int act;
    int vy;               // float4 output stores (Q % 4 == 0, y 16-byte aligned)
};

template <int SH, bool VEC, bool EPI>
__global__ __launch_bounds__(256) void conv_dw3(const float* __restrict__ x, const float* __restrict__ qw,
                                                const float* __restrict__ bias, float* __restrict__ y, DwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sx[];  // [CB][TH][WS]
    int b = blockIdx.x;
    const int band = b % a.nbands;
    b /= a.nbands;
    const int cb = b % a.ncb;
    const int n = b / a.ncb;
    const int c0 = cb * a.CB;
    const int cn = min(a.CB, a.C - c0);
    const int p0 = band * a.TP;
    const int pn = min(a.TP, a.P - p0);
    const int h0 = p0 * SH - 1;  // first staged input row (pad 1)
    const int HW = a.H * a.W;
    const float* xb = x + ((int64_t)n * a.C + c0) * HW;
    const int tid = threadIdx.x;

    // ---- stage: rows h0 .. h0 + TH - 1 of the cn planes (zero outside the image), halos zero
    const int plane = a.TH * a.WS;
    if constexpr (VEC) {
        const int W4 = a.W >> 2;
        const int per_c = a.TH * W4;
        for (int e = tid; e < cn * per_c; e += 256) {
            const int c = e / per_c, r = e - c * per_c;
            const int hr = r / W4, j = r - hr * W4;
            const int h = h0 + hr;
            floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
            if (h >= 0 && h < a.H) v = *reinterpret_cast<const floatx4*>(xb + (int64_t)c * HW + h * a.W + 4 * j);
            *reinterpret_cast<floatx4*>(sx + c * plane + hr * a.WS + 4 + 4 * j) = v;
        }
    } else {
        const int per_c = a.TH * a.W;
        for (int e = tid; e < cn * per_c; e += 256) {
            const int c = e / per_c, r = e - c * per_c;
            const int hr = r / a.W, w = r - hr * a.W;
            const int h = h0 + hr;
            sx[c * plane + hr * a.WS + 4 + w] = (h >= 0 && h < a.H) ? xb[(int64_t)c * HW + h * a.W + w] : 0.0f;
        }
    }
    // halo columns: offset 3 (w = -1) and 4 + W .. WS - 1 (w >= W, read by the last float4)
    const int nhalo = a.WS - a.W - 4 + 1;
    for (int e = tid; e < cn * a.TH * nhalo; e += 256) {
        const int row = e / nhalo, i = e - row * nhalo;
        sx[row * a.WS + (i == 0 ? 3 : 3 + a.W + i)] = 0.0f;
    }
    __syncthreads();

    // ---- compute: unit = (channel, output row, float4 column group)
    const int per_c = pn * a.QJ;
    for (int u = tid; u < cn * per_c; u += 256) {
        const int c = u / per_c, r = u - c * per_c;
        const int pr = r / a.QJ, j = r - pr * a.QJ;
        const int k = c0 + c;
        float w9[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w9[t] = qw[k * 9 + t];
        const float* base = sx + c * plane + pr * SH * a.WS + 4 * SH * j + 3;  // input column SH*4j - 1
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
            const float* row = base + rr * a.WS;
            constexpr int NV = 4 * SH + 2;  // input columns SH*4j - 1 .. SH*4j + 4*SH (stride 1: 6, 2: 10)
            float v[NV];
            v[0] = row[0];
            const floatx4 m0 = *reinterpret_cast<const floatx4*>(row + 1);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[1 + e] = m0[e];
            if constexpr (SH == 2) {
                const floatx4 m1 = *reinterpret_cast<const floatx4*>(row + 5);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[5 + e] = m1[e];
                v[9] = row[9];
            } else {
                v[5] = row[5];
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int s = 0; s < 3; ++s) acc[m] = fmaf(v[SH * m + s], w9[rr * 3 + s], acc[m]);
        }
        const float bk = bias ? bias[k] : 0.0f;
        float sc = 1.0f, sh = 0.0f;
        if constexpr (EPI) {
            sc = a.ps ? a.ps[k] : 1.0f;
            sh = a.pb ? a.pb[k] : 0.0f;
        }
        const int p = p0 + pr, q = 4 * j;
        const int64_t yo = (((int64_t)n * a.C + k) * a.P + p) * a.Q + q;
        floatx4 o;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float v = acc[m] + bk;
            if constexpr (EPI) {
                v = v * sc + sh;
                if (a.res && q + m < a.Q) v += a.res[yo + m];
                v = epi_act(v, a.act);
            }
            o[m] = v;
        }
        if (a.vy && q + 4 <= a.Q) {
            *reinterpret_cast<floatx4*>(y + yo) = o;
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if (q + m < a.Q) y[yo + m] = o[m];
        }
    }
}

// Plan (ConvPlan kind KIND_DEPTHWISE, vrx = 1): TP output rows per band (the whole plane
// when its staged rows fit 24 KiB), CB channels per block to give ~256 compute units.
bool dw3_plan(ConvPlan& p) {
    if (!(p.groups == p.C && p.K == p.C && p.Cg == 1 && p.Kg == 1)) return false;
    if (p.R != 3 || p.S != 3 || p.ph != 1 || p.pw != 1 || p.dh != 1 || p.dw != 1) return false;
    if (!((p.sh == 1 && p.sw == 1) || (p.sh == 2 && p.sw == 2))) return false;
    if ((int64_t)p.N * p.C * p.H * p.W >= INT32_MAX || (int64_t)p.N * p.C * p.P * p.Q >= INT32_MAX) return false;
    // 16-byte aligned rows, interior at offset 4; wide enough for the last float4 group's
    // reads (offsets up to 4 * sh * QJ + 4)
    const int qj = (p.Q + 3) / 4;
    const int ws = std::max((p.W + 3) / 4 * 4 + 8, (p.sh * 4 * qj + 5 + 3) / 4 * 4);
    int tp = p.P;
    auto th_of = [&](int t) { return (t - 1) * p.sh + 3; };
    while (tp > 1 && (size_t)th_of(tp) * ws * 4 > 24 * 1024) tp = (tp + 1) / 2;
    const int per_c = tp * qj;
    int cb = std::max(1, std::min(p.C, 256 / std::max(per_c, 1)));
    while (cb > 1 && (size_t)cb * th_of(tp) * ws * 4 > 48 * 1024) --cb;
    if ((size_t)cb * th_of(tp) * ws * 4 > 64 * 1024) return false;
    p.kind = KIND_DEPTHWISE;
    p.vrx = 1;
    p.MI = p.NJ = p.NT = 1;
    p.nchunks = p.kblocks = p.tilesQ = 1;
    p.steps = p.PS = p.SB = p.plane = p.pd = p.nts = p.fp = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.taps = 9;
    p.packed_floats = (int64_t)p.K * 9;  // the depthwise pack: Q(w) [K][1][3][3] fp32
    p.TP = tp;
    p.tilesP = (p.P + tp - 1) / tp;
    p.CC = cb;
    p.TQ = qj;
    p.HH = th_of(tp);
    p.WWp = p.WW = ws;
    p.lds_bytes = (size_t)cb * p.HH * ws * 4;
    p.blocks = (int64_t)p.N * ((p.C + cb - 1) / cb) * p.tilesP;
    return p.blocks <= INT_MAX;
}

bool dw3_plan_ok(const ConvPlan& p) { return p.kind == KIND_DEPTHWISE && p.vrx == 1; }

template <int SH, bool VEC>
static void launch_dw3_t(const ConvPlan& p, bool epi, const DwArgs& a, const float* x, const float* qw,
                         const float* bias, float* y, hipStream_t s) {
    if (epi)
        hipLaunchKernelGGL((conv_dw3<SH, VEC, true>), dim3((unsigned)p.blocks), dim3(256), p.lds_bytes, s, x, qw, bias,
                           y, a);
    else
        hipLaunchKernelGGL((conv_dw3<SH, VEC, false>), dim3((unsigned)p.blocks), dim3(256), p.lds_bytes, s, x, qw,
                           bias, y, a);
}

hipError_t launch_conv_dw3(const ConvPlan& p, const float* x, const float* qw, const float* bias, float* y,
                           const float* ps, const float* pb, const float* res, int act, hipStream_t s) {
    if (!dw3_plan_ok(p)) return hipErrorInvalidValue;
    DwArgs a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.CB = p.CC; a.TP = p.TP; a.TH = p.HH; a.WS = p.WWp;
    a.nbands = p.tilesP; a.ncb = (p.C + p.CC - 1) / p.CC; a.QJ = p.TQ;
    a.ps = ps; a.pb = pb; a.res = res; a.act = act;
    const bool epi = ps || pb || res || act != 0;
    const bool vec = p.W % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    a.vy = (p.Q % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0) ? 1 : 0;
    if (p.sh == 1) {
        if (vec) launch_dw3_t<1, true>(p, epi, a, x, qw, bias, y, s);
        else launch_dw3_t<1, false>(p, epi, a, x, qw, bias, y, s);
    } else {
        if (vec) launch_dw3_t<2, true>(p, epi, a, x, qw, bias, y, s);
        else launch_dw3_t<2, false>(p, epi, a, x, qw, bias, y, s);
    }
    return hipGetLastError();
}

}  // namespace po2q
