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
#include <string>

#include "../../include/po2q.h"
#include "po2q_internal.h"
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

}  // namespace

size_t po2q_qconv2d_wgrad_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                                          int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                                          int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups) {
    po2q::WgradArgs a;
    size_t lds, part;
    if (!wgrad_setup(a, lds, part, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups))
        return 0;
    return std::max<size_t>(part, 256);
}

int po2q_qconv2d_wgrad_f32(const float* x, const float* dy, float* dw, int64_t N, int64_t C, int64_t H, int64_t W,
                           int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                           int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, void* workspace,
                           size_t workspace_bytes, void* stream) {
    po2q::WgradArgs a;
    size_t lds, part;
    if (!wgrad_setup(a, lds, part, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups))
        return (groups != 1 || !((R == 3 && S == 3) || (R == 1 && S == 1))) ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    if (!x || !dy || !dw || !workspace) {
        po2q::set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (workspace_bytes < part) {
        po2q::set_error("po2q: wgrad workspace too small (need " + std::to_string(part) + " bytes)");
        return PO2Q_ERR_WORKSPACE;
    }
    const hipError_t e = po2q::launch_wgrad(a, x, dy, dw, reinterpret_cast<float*>(workspace), lds,
                                            reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: wgrad launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}
