// Pointwise (1x1 / stride 1 / pad 0) quantized conv on the bf16x3 MFMA path: the expand and
// project convs of MobileNetV2's inverted residual blocks (reference models/mobilenet.py:78-93,
// 120) and MobileViT's 1x1 convs (models/mobile_vit.py:170-185, 212), each
// QuantizedConv2d.forward (models/quantized_conv.py:32-38):
//     y[n][k][p] = scale * sum_c W'[k][c] x[n][c][p]      (W' = Q(w) / scale = +-2^e, exact bf16)
// with the eval BatchNorm affine, the residual add and the activation of the block in the store.
//
// A 1x1 conv over NCHW is a GEMM per image, Y (K x HW) = W' (K x C) X (C x HW), so the kernel is
// a plain MFMA GEMM with no halo and no LDS: a wave owns 16 pixels (of the N * HW pixels, which
// may span images when HW < 16) x KT tiles of 16 output channels.  Per 32-channel k-step each
// lane loads the 8 channels of its pixel (16 lanes = 16 consecutive pixels: 64-byte runs per
// channel), splits them exactly into hi / mid / lo bf16 A fragments in registers and feeds each
// to the KT tiles' MFMAs (3 x KT v_mfma_f32_16x16x32_bf16 per 8 values split); B fragments come
// from the pre-packed weight (generic bf16x3 layout [ks][nt][lane][8] of pack_bf16x3_kernel, L2
// resident).  The next k-step's loads are issued before the current one's MFMAs.  Each lane
// ends with 4 consecutive pixels of one output channel: one float4 store (and residual load).
// Roofline: HBM for MobileNetV2's CIFAR shapes (x in + y out dominate; at 32x32 every layer's
// tensors also fit the 256 MiB Infinity Cache, so a layer is a few microseconds).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

struct PwArgs {
    int N, C, HW, K;
    int NT, KS;       // 16-channel output tiles, 32-channel input k-steps (packed layout)
    int PG, items;    // 16-pixel groups, wave work items (PG x output-tile slices)
    int64_t M;        // N * HW pixels
    const float* ps;  // eval BN affine (NULL: none)
    const float* pb;
    const float* res;  // residual [N, K, HW] (NULL: none)
    int act;
};

// KSPLIT 1: a block = 4 independent wave items.  KSPLIT 4 (few items: late MobileNetV2 layers
// at 2x2 / 1x1 pixels, where 16-pixel groups are few and C is up to 960): a block = ONE item,
// wave w takes the k-steps ks = w mod 4, and the 4 partial sums are added through LDS in a
// fixed order (deterministic) before wave 0's epilogue -- a 4x shorter dependent load chain.
// PD (plan field nts + 1): k-steps whose x values and B fragments are in flight at once.  1: the next
// k-step's loads go out before the current one's MFMAs.  3: three k-steps ahead -- the small late
// layers are a chain of dependent load latencies (a few us per launch at 2x2 / 1x1 pixels), which a
// deeper ring shortens 3x; more VGPRs, so the autotuner keeps PD 1 where occupancy matters.
template <int KT, bool EPI, int KSPLIT = 1, int PD = 1>
__global__ __launch_bounds__(256) void conv_pw(const float* __restrict__ x, const uint4* __restrict__ wp,
                                               const float* __restrict__ scale_p, const float* __restrict__ bias,
                                               float* __restrict__ y, PwArgs a) {
    static_assert(PD == 1 || PD == 3, "k-step ring depth");
    const int lane = threadIdx.x & 63;
    const int wv = (int)(threadIdx.x >> 6);
    const int v = KSPLIT == 1 ? (int)blockIdx.x * 4 + wv : (int)blockIdx.x;
    if (v >= a.items) return;  // KSPLIT 1: wave-uniform; KSPLIT 4: block-uniform
    const int ks0 = KSPLIT == 1 ? 0 : wv;
    const int pg = v % a.PG, sl = v / a.PG;
    const int kt0 = sl * KT;
    const int nkt = min(KT, a.NT - kt0);
    const int g = lane >> 4;
    // the lane's A-fragment pixel and its 8 channels per k-step
    const int64_t m = (int64_t)pg * 16 + (lane & 15);
    const bool mok = m < a.M;
    const int n = mok ? (int)(m / a.HW) : 0;
    const int p = mok ? (int)(m - (int64_t)n * a.HW) : 0;
    const float* xb = x + ((int64_t)n * a.C + 8 * g) * a.HW + p;
    const int64_t cstride = a.HW;

    auto load8 = [&](int ks, uint32_t (&b)[8]) __attribute__((always_inline)) {
        const int c0 = 32 * ks + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            b[e] = (mok && c0 + e < a.C) ? __float_as_uint(xb[(int64_t)(32 * ks + e) * cstride]) : 0u;
    };
    auto loadw = [&](int ks, uint4 (&bw)[KT]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < KT; ++t)
            bw[t] = t < nkt ? wp[((int64_t)ks * a.NT + kt0 + t) * 64 + lane] : make_uint4(0u, 0u, 0u, 0u);
    };

    floatx4 acc[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto mma = [&](const uint32_t (&cur)[8], const uint4 (&bw)[KT]) __attribute__((always_inline)) {
        uint4 hi, mid, lo;
        split3(cur, hi, mid, lo);
        const bf16x8 ah = __builtin_bit_cast(bf16x8, hi), am = __builtin_bit_cast(bf16x8, mid),
                     al = __builtin_bit_cast(bf16x8, lo);
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            if (t < nkt) {  // wave-uniform
                const bf16x8 b = __builtin_bit_cast(bf16x8, bw[t]);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b, acc[t], 0, 0, 0);
            }
        }
    };
    if constexpr (PD == 1) {
        uint32_t cur[8];
        if (ks0 < a.KS) load8(ks0, cur);
        for (int ks = ks0; ks < a.KS; ks += KSPLIT) {
            uint32_t nxt[8];
            if (ks + KSPLIT < a.KS) load8(ks + KSPLIT, nxt);
            uint4 bw[KT];
            loadw(ks, bw);
            mma(cur, bw);
            if (ks + KSPLIT < a.KS) {
#pragma unroll
                for (int e = 0; e < 8; ++e) cur[e] = nxt[e];
            }
        }
    } else {
        // a 3-slot ring (compile-time slots: the loop is unrolled by 3); the guards are wave-uniform
        uint32_t xr[3][8];
        uint4 wr[3][KT];
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
            const int ks = ks0 + s3 * KSPLIT;
            if (ks < a.KS) {
                load8(ks, xr[s3]);
                loadw(ks, wr[s3]);
            }
        }
        for (int ks = ks0; ks < a.KS; ks += 3 * KSPLIT) {
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3) {
                const int kc = ks + s3 * KSPLIT;
                if (kc >= a.KS) break;
                mma(xr[s3], wr[s3]);
                const int kn = kc + 3 * KSPLIT;
                if (kn < a.KS) {
                    load8(kn, xr[s3]);
                    loadw(kn, wr[s3]);
                }
            }
        }
    }
    if constexpr (KSPLIT > 1) {
        __shared__ floatx4 part[KSPLIT - 1][KT][64];
        if (wv > 0) {
#pragma unroll
            for (int t = 0; t < KT; ++t) part[wv - 1][t][lane] = acc[t];
        }
        __syncthreads();
        if (wv > 0) return;
#pragma unroll
        for (int w = 0; w < KSPLIT - 1; ++w)
#pragma unroll
            for (int t = 0; t < KT; ++t) acc[t] += part[w][t][lane];
    }

    // epilogue: lane holds D[pixel 4 g + e][channel lane & 15] of each tile
    const float scale = *scale_p;
    const int64_t mo = (int64_t)pg * 16 + 4 * g;  // first of the lane's 4 output pixels
    const int no = mo < a.M ? (int)(mo / a.HW) : 0;
    const int po = mo < a.M ? (int)(mo - (int64_t)no * a.HW) : 0;
    // the 4 pixels are consecutive in memory when they sit in one image row of y
    const bool vec = (a.HW & 3) == 0 && mo + 3 < a.M;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        if (t >= nkt) break;
        const int k = 16 * (kt0 + t) + (lane & 15);
        if (k >= a.K) continue;
        const float bk = bias ? bias[k] : 0.0f;
        const float s = EPI && a.ps ? a.ps[k] : 1.0f;
        const float sh = EPI && a.pb ? a.pb[k] : 0.0f;
        float vv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float u = acc[t][e] * scale + bk;
            if constexpr (EPI) u = u * s + sh;
            vv[e] = u;
        }
        if (vec) {
            const int64_t off = ((int64_t)no * a.K + k) * a.HW + po;
            if (EPI && a.res) {
                const float4 r = *reinterpret_cast<const float4*>(a.res + off);
                vv[0] += r.x; vv[1] += r.y; vv[2] += r.z; vv[3] += r.w;
            }
            if constexpr (EPI) {
#pragma unroll
                for (int e = 0; e < 4; ++e) vv[e] = epi_act(vv[e], a.act);
            }
            *reinterpret_cast<float4*>(y + off) = make_float4(vv[0], vv[1], vv[2], vv[3]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t me = mo + e;
                if (me >= a.M) break;
                const int ne = (int)(me / a.HW), pe = (int)(me - (int64_t)ne * a.HW);
                const int64_t off = ((int64_t)ne * a.K + k) * a.HW + pe;
                float u = vv[e];
                if (EPI && a.res) u += a.res[off];
                if constexpr (EPI) u = epi_act(u, a.act);
                y[off] = u;
            }
        }
    }
}

// Plan: kind KIND_BF16X3_PW, packed weight in the generic bf16x3 layout with one chunk of
// CC = C rounded up to 32 channels (pack_bf16x3_kernel: [ks][nt][lane][8]), NJ = KT.
static bool pw_plan_one(ConvPlan& p, int kt, int ksplit) {
    const int NT = (p.K + 15) / 16, KS = (p.C + 31) / 32;
    p.kind = KIND_BF16X3_PW;
    p.vrx = 0;
    p.NJ = kt;
    p.NT = NT;
    p.MI = 0;
    p.CC = 32 * KS;
    p.nchunks = 1;
    p.kblocks = 1;
    p.steps = KS;
    p.taps = 1;
    p.TP = p.TQ = 1;
    p.tilesP = p.tilesQ = 1;
    p.HH = p.WW = p.WWp = p.PS = 0;
    p.SB = p.plane = 0;
    p.pd = ksplit;  // k-steps split over the block's 4 waves (1: none)
    p.nts = 0;
    p.fp = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.packed_floats = (int64_t)KS * NT * 64 * 4;  // uint4 fragments = 4 words each
    p.lds_bytes = 0;
    const int64_t M = (int64_t)p.N * p.P * p.Q;
    const int64_t PG = (M + 15) / 16;
    const int64_t items = PG * ((NT + kt - 1) / kt);
    if (items > (int64_t)INT32_MAX - 4 || PG > INT32_MAX) return false;
    p.blocks = ksplit == 1 ? (items + 3) / 4 : items;
    return true;
}

void pw_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    out.clear();
    if (mode == 0 || base.groups != 1 || base.R != 1 || base.S != 1 || base.sh != 1 || base.sw != 1 ||
        base.ph != 0 || base.pw != 0 || base.dh != 1 || base.dw != 1)
        return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if ((int64_t)base.N * base.C * base.H * base.W >= (1LL << 31) ||
        (int64_t)base.N * base.K * base.P * base.Q >= (1LL << 31) || base.C > 4096 || base.K > 4096)
        return;
    const int NT = (base.K + 15) / 16;
    const int64_t M = (int64_t)base.N * base.P * base.Q;
    const int64_t PG = (M + 15) / 16;
    const int KS = (base.C + 31) / 32;
    for (int ksplit : {1, 4}) {
        for (int kt : {2, 4, 8}) {
            for (int pd : {1, 3}) {
                if (kt > 2 && (NT + kt / 2 - 1) / (kt / 2) <= 1) continue;  // no wider than the channel count needs
                if (ksplit > 1 && KS < 2 * ksplit) continue;                 // too few k-steps to split
                const int steps = (KS + ksplit - 1) / ksplit;                // k-steps of one wave's chain
                if (pd > 1 && (steps < 3 || kt > 4)) continue;                // a ring deeper than the chain / VGPRs
                ConvPlan p = base;
                if (!pw_plan_one(p, kt, ksplit)) continue;
                p.nts = pd - 1;
                // cost: the dependent k-step chain of a wave (a load latency per k-step, or per pd
                // k-steps with the ring), scaled up when too few waves fill the chip; the ring's VGPRs
                // cost occupancy where the chip is full
                const int64_t waves = PG * ((NT + kt - 1) / kt) * ksplit;
                const double fill = std::min(1.0, (double)waves / 4096.0);
                const double chain = steps * (24.0 / pd + 3.0 * 16.0 * std::min(kt, NT) / 8.0) + 40.0;
                PlanCand c;
                c.plan = p;
                c.cost = (double)waves * chain / ksplit / fill * (pd > 1 && fill >= 1.0 ? 1.5 : 1.0) +
                         (fill < 1.0 ? chain * 64.0 : 0.0);
                out.push_back(c);
            }
        }
    }
    std::stable_sort(out.begin(), out.end(), [](const PlanCand& u, const PlanCand& v) { return u.cost < v.cost; });
}

template <int KT>
static hipError_t launch_pw_t(const ConvPlan& p, const PwArgs& a, const float* x, const uint4* wp, const float* scale,
                              const float* bias, float* y, bool epi, hipStream_t s) {
    const dim3 grid((unsigned)p.blocks), block(256);
    if constexpr (KT <= 4) {
        if (p.nts == 2) {  // the 3-deep k-step ring
            if (p.pd == 4) {
                if (epi)
                    hipLaunchKernelGGL((conv_pw<KT, true, 4, 3>), grid, block, 0, s, x, wp, scale, bias, y, a);
                else
                    hipLaunchKernelGGL((conv_pw<KT, false, 4, 3>), grid, block, 0, s, x, wp, scale, bias, y, a);
            } else if (epi) {
                hipLaunchKernelGGL((conv_pw<KT, true, 1, 3>), grid, block, 0, s, x, wp, scale, bias, y, a);
            } else {
                hipLaunchKernelGGL((conv_pw<KT, false, 1, 3>), grid, block, 0, s, x, wp, scale, bias, y, a);
            }
            return hipGetLastError();
        }
    }
    if (p.pd == 4) {
        if (epi)
            hipLaunchKernelGGL((conv_pw<KT, true, 4>), grid, block, 0, s, x, wp, scale, bias, y, a);
        else
            hipLaunchKernelGGL((conv_pw<KT, false, 4>), grid, block, 0, s, x, wp, scale, bias, y, a);
    } else if (epi) {
        hipLaunchKernelGGL((conv_pw<KT, true>), grid, block, 0, s, x, wp, scale, bias, y, a);
    } else {
        hipLaunchKernelGGL((conv_pw<KT, false>), grid, block, 0, s, x, wp, scale, bias, y, a);
    }
    return hipGetLastError();
}

hipError_t launch_conv_pw(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                          const float* bias, float* y, const float* ps, const float* pb, const float* res, int act,
                          hipStream_t s) {
    if (p.kind != KIND_BF16X3_PW) return hipErrorInvalidValue;
    PwArgs a;
    a.N = p.N; a.C = p.C; a.HW = p.P * p.Q; a.K = p.K;
    a.NT = p.NT; a.KS = p.steps;
    a.M = (int64_t)p.N * a.HW;
    a.PG = (int)((a.M + 15) / 16);
    a.items = a.PG * ((a.NT + p.NJ - 1) / p.NJ);
    a.ps = ps; a.pb = pb; a.res = res; a.act = act;
    const bool epi = ps || pb || res || act != 0;
    const uint4* wp = reinterpret_cast<const uint4*>(packed);
    switch (p.NJ) {
        case 2: return launch_pw_t<2>(p, a, x, wp, scale, bias, y, epi, s);
        case 4: return launch_pw_t<4>(p, a, x, wp, scale, bias, y, epi, s);
        case 8: return launch_pw_t<8>(p, a, x, wp, scale, bias, y, epi, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace po2q
