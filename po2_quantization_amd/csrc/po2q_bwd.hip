// QAT backward pieces for the layers the dense wgrad / forward kernels do not cover
// (reference train.py:79-91: loss.backward() through F.conv2d(x, Q(w)) with the STE of
// utils/quantizers.py:34-36):
//
//  * depthwise weight gradient (MobileNetV2 / MobileViT 3x3 depthwise QuantizedConv2d,
//    reference models/mobilenet.py:64-76, groups = C = K):
//        dw[c][r][s] = sum_{n,p,q} dy[n][c][p][q] * x[n][c][p*sh + r*dh - ph][q*sw + s*dw - pw]
//    HBM-bound (9 MACs per dy element): block = (channel, slice of images), each thread keeps
//    the R*S sums of its pixels in registers (fp32), the block adds them in a fixed tree
//    order, a second kernel adds the slices in order -- deterministic, no atomics;
//
//  * zero insertion for strided input gradients: the input gradient of a stride-s conv is
//    the stride-1 conv (the forward kernels, flipped / transposed PO2 weight) of dy with
//    s - 1 zeros inserted between its pixels (po2q_dilate_f32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "../../include/po2q.h"
#include "po2q_internal.h"

namespace po2q {

struct DwWgradArgs {
    int N, C, H, W, P, Q, R, S, sh, sw, ph, pw, dh, dw;
    int nslice, per_slice;  // images per block
};

constexpr int kDwThreads = 256;
constexpr int kDwMaxTaps = 25;  // up to 5x5

template <int RS>
__global__ __launch_bounds__(kDwThreads) void dw_wgrad_partial(const float* __restrict__ x,
                                                               const float* __restrict__ dy,
                                                               float* __restrict__ part, DwWgradArgs a) {
    const int c = blockIdx.x, sl = blockIdx.y;
    const int n0 = sl * a.per_slice, n1 = min(a.N, n0 + a.per_slice);
    const int PQ = a.P * a.Q;
    float acc[RS];
#pragma unroll
    for (int t = 0; t < RS; ++t) acc[t] = 0.0f;
    for (int n = n0; n < n1; ++n) {
        const float* xp = x + ((int64_t)n * a.C + c) * a.H * a.W;
        const float* gp = dy + ((int64_t)n * a.C + c) * PQ;
        for (int i = threadIdx.x; i < PQ; i += kDwThreads) {
            const int p = i / a.Q, q = i - p * a.Q;
            const float g = gp[i];
            const int h0 = p * a.sh - a.ph, w0 = q * a.sw - a.pw;
#pragma unroll
            for (int t = 0; t < RS; ++t) {
                const int r = t / a.S, s = t - r * a.S;
                if (r < a.R) {
                    const int h = h0 + r * a.dh, w = w0 + s * a.dw;
                    if (h >= 0 && h < a.H && w >= 0 && w < a.W) acc[t] = fmaf(g, xp[h * a.W + w], acc[t]);
                }
            }
        }
    }
    // fixed-order block reduction of each tap's sums
    __shared__ float red[RS][kDwThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < RS; ++t) {
        float v = acc[t];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) red[t][wv] = v;
    }
    __syncthreads();
    if (threadIdx.x < RS) {
        float v = 0.0f;
#pragma unroll
        for (int k = 0; k < kDwThreads / 64; ++k) v += red[threadIdx.x][k];
        part[((int64_t)c * a.nslice + sl) * RS + threadIdx.x] = v;
    }
}

template <int RS>
__global__ void dw_wgrad_reduce(const float* __restrict__ part, float* __restrict__ dw, DwWgradArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (c, tap)
    if (i >= a.C * a.R * a.S) return;
    const int c = i / (a.R * a.S), t = i - c * (a.R * a.S);
    const int r = t / a.S, s = t - r * a.S;
    float v = 0.0f;
    for (int sl = 0; sl < a.nslice; ++sl) v += part[((int64_t)c * a.nslice + sl) * RS + r * a.S + s];
    dw[i] = v;
}

static bool dw_wgrad_setup(DwWgradArgs& a, size_t& part_bytes, int64_t N, int64_t C, int64_t H, int64_t W,
                           int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                           int64_t dw) {
    if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || R <= 0 || S <= 0 || sh <= 0 || sw <= 0 || dh <= 0 || dw <= 0 ||
        ph < 0 || pw < 0)
        return false;
    if (R * S > kDwMaxTaps || S > 5) return false;
    const int64_t P = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1, Q = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
    if (P <= 0 || Q <= 0 || N * C * H * W >= (1LL << 31) || N * C * P * Q >= (1LL << 31)) return false;
    a.N = (int)N; a.C = (int)C; a.H = (int)H; a.W = (int)W; a.P = (int)P; a.Q = (int)Q;
    a.R = (int)R; a.S = (int)S; a.sh = (int)sh; a.sw = (int)sw; a.ph = (int)ph; a.pw = (int)pw;
    a.dh = (int)dh; a.dw = (int)dw;
    // enough blocks to fill the chip (>= ~4 per CU) with at least ~4 K pixels of dy each
    const int64_t want = std::max<int64_t>(1, (2048 + C - 1) / C);
    const int64_t by_work = std::max<int64_t>(1, (N * P * Q) / 4096);
    const int64_t ns = std::min<int64_t>(N, std::min(want, by_work));
    a.per_slice = (int)((N + ns - 1) / ns);
    a.nslice = (int)((N + a.per_slice - 1) / a.per_slice);
    const int rs = R * S <= 9 ? 9 : kDwMaxTaps;
    part_bytes = (size_t)C * a.nslice * rs * sizeof(float);
    return true;
}

template <int RS>
static hipError_t launch_dw_wgrad_t(const DwWgradArgs& a, const float* x, const float* dy, float* dw, float* part,
                                    hipStream_t s) {
    hipLaunchKernelGGL((dw_wgrad_partial<RS>), dim3(a.C, a.nslice), dim3(kDwThreads), 0, s, x, dy, part, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int n = a.C * a.R * a.S;
    hipLaunchKernelGGL((dw_wgrad_reduce<RS>), dim3((n + 255) / 256), dim3(256), 0, s, part, dw, a);
    return hipGetLastError();
}

// ---- zero insertion: dst[n][c][i][j] = src[n][c][i / sh][j / sw] where sh | i, sw | j (and
// inside src), else 0; dst is [N, C, Hd, Wd].  One thread per 4 consecutive dst pixels of a row.
__global__ void dilate_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t rows, int P, int Q,
                              int sh, int sw, int Hd, int Wd) {
    const int W4 = (Wd + 3) / 4;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * W4) return;
    const int64_t row = t / W4;  // (n, c, i)
    const int j0 = (int)(t - row * W4) * 4;
    const int i = (int)(row % Hd);
    const int64_t nc = row / Hd;
    const bool rok = i % sh == 0 && i / sh < P;
    const float* sp = src + (nc * P + (rok ? i / sh : 0)) * Q;
    float* dp = dst + row * Wd;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int j = j0 + e;
        v[e] = (rok && j < Wd && j % sw == 0 && j / sw < Q) ? sp[j / sw] : 0.0f;
    }
    if ((Wd & 3) == 0) {
        *reinterpret_cast<float4*>(dp + j0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (j0 + e < Wd) dp[j0 + e] = v[e];
    }
}

}  // namespace po2q

size_t po2q_dw_wgrad_workspace_bytes_internal(int64_t N, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                                              int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                                              int64_t dw) {
    po2q::DwWgradArgs a;
    size_t part;
    if (!po2q::dw_wgrad_setup(a, part, N, C, H, W, R, S, sh, sw, ph, pw, dh, dw)) return 0;
    return std::max<size_t>(part, 256);
}

int po2q_dw_wgrad_f32_internal(const float* x, const float* dy, float* dwt, int64_t N, int64_t C, int64_t H,
                               int64_t W, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                               int64_t dh, int64_t dw, void* workspace, size_t workspace_bytes, void* stream) {
    po2q::DwWgradArgs a;
    size_t part;
    if (!po2q::dw_wgrad_setup(a, part, N, C, H, W, R, S, sh, sw, ph, pw, dh, dw)) {
        po2q::set_error("po2q: depthwise wgrad: unsupported geometry (kernel up to 5x5, sizes < 2^31)");
        return PO2Q_ERR_UNSUPPORTED;
    }
    if (!x || !dy || !dwt || !workspace) {
        po2q::set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (workspace_bytes < part) {
        po2q::set_error("po2q: wgrad workspace too small (need " + std::to_string(part) + " bytes)");
        return PO2Q_ERR_WORKSPACE;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    float* pp = reinterpret_cast<float*>(workspace);
    const hipError_t e = R * S <= 9 ? po2q::launch_dw_wgrad_t<9>(a, x, dy, dwt, pp, s)
                                    : po2q::launch_dw_wgrad_t<po2q::kDwMaxTaps>(a, x, dy, dwt, pp, s);
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: depthwise wgrad launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}

int po2q_dilate_f32(const float* src, float* dst, int64_t N, int64_t C, int64_t P, int64_t Q, int64_t stride_h,
                    int64_t stride_w, int64_t Hd, int64_t Wd, void* stream) {
    if (N <= 0 || C <= 0 || P <= 0 || Q <= 0 || stride_h <= 0 || stride_w <= 0 || Hd <= 0 || Wd <= 0) {
        po2q::set_error("po2q: dilate: sizes and strides must be positive");
        return PO2Q_ERR_INVALID;
    }
    if (!src || !dst) {
        po2q::set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (N * C * Hd * Wd >= (1LL << 40) || P > (1 << 30) || Q > (1 << 30) || Hd > (1 << 30) || Wd > (1 << 30)) {
        po2q::set_error("po2q: dilate: tensor too large");
        return PO2Q_ERR_INVALID;
    }
    const int64_t rows = N * C * Hd;
    const int64_t threads = rows * ((Wd + 3) / 4);
    hipLaunchKernelGGL(po2q::dilate_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), src, dst, rows, (int)P, (int)Q, (int)stride_h,
                       (int)stride_w, (int)Hd, (int)Wd);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: dilate launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}
