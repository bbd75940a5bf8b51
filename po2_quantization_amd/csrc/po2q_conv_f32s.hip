// fp32 convs for the layers the reference leaves UNQUANTIZED (plain nn.Conv2d with fp32
// weights; also any QuantizedConv2d whose quantizer is not po2 / po2+, which reaches the native
// conv as mode "none" with the quantized weight), with the eval BatchNorm / activation /
// residual of the block in the store:
//
//  * conv_direct_f32 / conv_stem_f32 -- the 3-input-channel stems: ResNet's conv1 3 -> 16 3x3 s1 (reference
//    models/resnet.py:99-102, 191), MobileNetV2's features[0] 3 -> 32 3x3 s2
//    (models/mobilenet.py:41-46, 167), MobileViT's conv1 3 -> 16 3x3 s2 (models/mobile_vit.py:
//    41-48, 456).  27 MACs per output: a direct VALU conv (fp32 fma, weights wave-uniform), one
//    thread = 4 consecutive output pixels x 16 output channels; bound by the output write
//    (16 channels per input pixel);
//  * conv_pw_f32 -- unquantized 1x1 convs (MobileNetV2's last conv 320 -> 1280,
//    models/mobilenet.py:185; MobileViT's to_logits conv): the pointwise GEMM of
//    po2q_conv_pw.hip on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

struct F32sArgs {
    int N, C, H, W, K, P, Q, ph, pw;
    int KB;           // direct: output channels per thread (16); pw: tiles per wave (NJ)
    int items;        // direct: threads with work (N x P x ceil(Q / 4)); pw: wave items
    int Q4, NT, PG;
    int64_t M;        // pw: N * P * Q pixels
    const float* ps;  // eval BN affine (NULL: none)
    const float* pb;
    const float* res;  // residual [N, K, P, Q] (NULL: none)
    int act;
};

// ACT: -1 = no epilogue (bias only), else the eval affine / residual / activation ACT (compile-time:
// a runtime activation switch per value had put ~400 scalar branches into the stem kernel)
template <int ACT>
__device__ __forceinline__ void f32s_store4(const F32sArgs& a, float* __restrict__ y, int n, int k, int p, int q,
                                            float (&v)[4], const float* __restrict__ bias) {
    constexpr bool epi = ACT >= 0;
    const float bk = bias ? bias[k] : 0.0f;
    const float s = (epi && a.ps) ? a.ps[k] : 1.0f;
    const float t = (epi && a.pb) ? a.pb[k] : 0.0f;
    const int64_t off = (((int64_t)n * a.K + k) * a.P + p) * a.Q + q;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        v[e] += bk;
        if constexpr (epi) v[e] = v[e] * s + t;
    }
    if ((a.Q & 3) == 0) {  // q is a multiple of 4: one aligned float4
        if (epi && a.res) {
            const float4 r = *reinterpret_cast<const float4*>(a.res + off);
            v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
        }
        if constexpr (epi) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = epi_act_ct<epi ? ACT : 0>(v[e]);
        }
        *reinterpret_cast<float4*>(y + off) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (q + e >= a.Q) break;
            float u = v[e];
            if (epi && a.res) u += a.res[off + e];
            if constexpr (epi) u = epi_act_ct<epi ? ACT : 0>(u);
            y[off + e] = u;
        }
    }
}

// Direct 3x3 conv, C <= 4 input channels, stride SH, pad (ph, pw): thread = (image n, output
// row p, 4 output columns q0 .. q0 + 3) x the KB output channels of blockIdx.y.  KB 16: the
// large stems (ResNet @224: 3.2 M threads); KB 4: small images, where 16 channels per thread left
// half the chip idle and each thread four dependent weight batches long (MobileNetV2 @32's stem:
// 128 blocks, 31 us).
template <int SH, int CMAX, int KB = 16>
__global__ __launch_bounds__(256) void conv_direct_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ y,
                                                       F32sArgs a, int epi) {
    constexpr int IC = (4 - 1) * SH + 3;  // input columns the 4 outputs touch
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= a.items) return;
    const int k0 = (int)blockIdx.y * KB;
    const int q4 = t % a.Q4;
    const int rest = t / a.Q4;
    const int p = rest % a.P, n = rest / a.P;
    const int q0 = 4 * q4;
    // input window: rows p*SH - ph + r, columns q0*SH - pw + j, j < IC
    float xv[CMAX][3][IC];
    const int h0 = p * SH - a.ph, w0 = q0 * SH - a.pw;
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int h = h0 + r;
            const bool hok = c < a.C && h >= 0 && h < a.H;
            const float* row = x + (((int64_t)n * a.C + (c < a.C ? c : 0)) * a.H + (hok ? h : 0)) * a.W;
#pragma unroll
            for (int j = 0; j < IC; ++j) {
                const int ww = w0 + j;
                xv[c][r][j] = (hok && ww >= 0 && ww < a.W) ? row[ww] : 0.0f;
            }
        }
    }
    auto body = [&](auto ACT_) __attribute__((always_inline)) {
        constexpr int ACT = decltype(ACT_)::value;
#pragma unroll 1
        for (int kk = 0; kk < KB; kk += 4) {
            float acc[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[u][e] = 0.0f;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + kk + u;
                const int kc = k < a.K ? k : 0;  // wave-uniform
#pragma unroll
                for (int c = 0; c < CMAX; ++c) {
                    if (c >= a.C) break;
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int s = 0; s < 3; ++s) {
                            const float wt = w[((kc * a.C + c) * 3 + r) * 3 + s];
#pragma unroll
                            for (int e = 0; e < 4; ++e) acc[u][e] = fmaf(xv[c][r][e * SH + s], wt, acc[u][e]);
                        }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + kk + u;
                if (k < a.K) f32s_store4<ACT>(a, y, n, k, p, q0, acc[u], bias);
            }
        }
    };
    if (epi == 0)
        body(std::integral_constant<int, -1>{});
    else
        with_act(a.act, [&](auto A) __attribute__((always_inline)) { body(A); });
}

// Direct 3x3 conv, pixel per thread (plan field MI = 1): thread = ONE output pixel (n, p, q) x the
// KG output channels of blockIdx.y, consecutive lanes on consecutive output columns (each input
// load and each channel's store is one contiguous run across the wave).  The block's KG x C x 9
// weights are staged in LDS once and read back as wave-wide broadcasts; the input window is 9C
// loads from clamped addresses with a select (no per-load branch).  Same sums as conv_direct_f32
// (fp32 fma in (c, r, s) order from 0), so the two agree bit for bit.
template <int SH, int CMAX, int KG = 8>
__global__ __launch_bounds__(256) void conv_stem_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias, float* __restrict__ y,
                                                     F32sArgs a, int epi) {
    __shared__ float wl[KG * CMAX * 9];
    const int k0 = (int)blockIdx.y * KG;
    const int C = a.C;
    for (int i = threadIdx.x; i < KG * CMAX * 9; i += 256) {
        const int u = i / (CMAX * 9), rem = i - u * (CMAX * 9), c = rem / 9;
        const int k = k0 + u;
        wl[i] = (k < a.K && c < C) ? w[((int64_t)k * C + c) * 9 + (rem - 9 * c)] : 0.0f;
    }
    __syncthreads();
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.M) return;
    const int q = (int)(t % a.Q);
    const int64_t r0 = t / a.Q;
    const int p = (int)(r0 % a.P), n = (int)(r0 / a.P);
    const int h0 = p * SH - a.ph, w0 = q * SH - a.pw;
    float xv[CMAX][9];
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const int h = h0 + r, ww = w0 + s;
                const bool ok = c < C && h >= 0 && h < a.H && ww >= 0 && ww < a.W;
                const float v = x[(((int64_t)n * C + (c < C ? c : 0)) * a.H + (ok ? h : 0)) * a.W + (ok ? ww : 0)];
                xv[c][r * 3 + s] = ok ? v : 0.0f;
            }
    auto body = [&](auto ACT_) __attribute__((always_inline)) {
        constexpr int ACT = decltype(ACT_)::value;
        constexpr bool E = ACT >= 0;
#pragma unroll
        for (int u = 0; u < KG; ++u) {
            const int k = k0 + u;
            if (k >= a.K) break;  // block-uniform
            float acc = 0.0f;
#pragma unroll
            for (int c = 0; c < CMAX; ++c) {
                if (c >= C) break;
#pragma unroll
                for (int j = 0; j < 9; ++j) acc = fmaf(xv[c][j], wl[(u * CMAX + c) * 9 + j], acc);
            }
            float v = acc + (bias ? bias[k] : 0.0f);
            const int64_t off = (((int64_t)n * a.K + k) * a.P + p) * a.Q + q;
            if constexpr (E) {
                v = v * (a.ps ? a.ps[k] : 1.0f) + (a.pb ? a.pb[k] : 0.0f);
                if (a.res) v += a.res[off];
                v = epi_act_ct<E ? ACT : 0>(v);
            }
            y[off] = v;
        }
    };
    if (epi == 0)
        body(std::integral_constant<int, -1>{});
    else
        with_act(a.act, [&](auto A) __attribute__((always_inline)) { body(A); });
}

// Pointwise 1x1 fp32 GEMM on v_mfma_f32_16x16x4_f32: wave = MI groups of 16 pixels x KT tiles of
// 16 output channels; per MFMA a lane holds one x value (pixel l & 15, channel 4 j + (l >> 4)) and
// one weight (output channel l & 15 of the tile, same channel): exact products, fp32 sums.  Every
// weight a wave loads feeds MI MFMAs: a large 1x1 over few pixels (MobileNetV2's last conv,
// 320 -> 1280 over 4,096 pixels) is bound by the L2 re-reads of its weight, once per pixel group at
// MI = 1 (1.6 MB x 256 groups).
template <int KT, int MI = 1>
__global__ __launch_bounds__(256) void conv_pw_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, float* __restrict__ y, F32sArgs a,
                                                   int epi) {
    const int lane = threadIdx.x & 63;
    const int v = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (v >= a.items) return;  // wave-uniform
    const int PGM = (a.PG + MI - 1) / MI;  // MI-group slices
    const int pgs = v % PGM, sl = v / PGM;
    const int kt0 = sl * KT;
    const int nkt = min(KT, a.NT - kt0);
    const int g = lane >> 4;
    const int HW = a.P * a.Q;
    const float* xb[MI];
    bool mok[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
        const int64_t m = ((int64_t)pgs * MI + mi) * 16 + (lane & 15);
        mok[mi] = m < a.M;
        const int n = mok[mi] ? (int)(m / HW) : 0, pp = mok[mi] ? (int)(m - (int64_t)n * HW) : 0;
        xb[mi] = x + ((int64_t)n * a.C + g) * HW + pp;
    }
    const float* wb[KT];
    bool kok[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int k = 16 * (kt0 + t) + (lane & 15);
        kok[t] = t < nkt && k < a.K;
        wb[t] = w + (int64_t)(kok[t] ? k : 0) * a.C + g;
    }
    floatx4 acc[MI][KT];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int t = 0; t < KT; ++t) acc[mi][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nj = (a.C + 3) / 4;
    for (int j0 = 0; j0 < nj; j0 += 4) {
        float xa[4][MI], wv[4][KT];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = 4 * (j0 + u) + g;
            const bool cok = c < a.C;
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) xa[u][mi] = (mok[mi] && cok) ? xb[mi][(int64_t)4 * (j0 + u) * HW] : 0.0f;
#pragma unroll
            for (int t = 0; t < KT; ++t) wv[u][t] = (kok[t] && cok) ? wb[t][4 * (j0 + u)] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (j0 + u >= nj) break;  // wave-uniform
#pragma unroll
            for (int t = 0; t < KT; ++t)
#pragma unroll
                for (int mi = 0; mi < MI; ++mi)
                    if (t < nkt) acc[mi][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[u][mi], wv[u][t], acc[mi][t], 0, 0, 0);
        }
    }
    // epilogue: lane holds D[pixel 4 g + e][channel lane & 15]
    const bool ep = epi != 0;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
        const int64_t mo = ((int64_t)pgs * MI + mi) * 16 + 4 * g;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            if (t >= nkt) break;
            const int k = 16 * (kt0 + t) + (lane & 15);
            if (k >= a.K) continue;
            const float bk = bias ? bias[k] : 0.0f;
            const float s = (ep && a.ps) ? a.ps[k] : 1.0f;
            const float sh = (ep && a.pb) ? a.pb[k] : 0.0f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t me = mo + e;
                if (me >= a.M) break;
                const int ne = (int)(me / HW), pe = (int)(me - (int64_t)ne * HW);
                const int64_t off = ((int64_t)ne * a.K + k) * HW + pe;
                float u = acc[mi][t][e] + bk;
                if (ep) {
                    u = u * s + sh;
                    if (a.res) u += a.res[off];
                    u = epi_act(u, a.act);
                }
                y[off] = u;
            }
        }
    }
}

// ---- planning: kinds KIND_DIRECT_F32 (vrx = SH, NJ = CMAX) and KIND_PW_F32 (NJ = KT); the
// weight is read as given (mode none: no pack, nothing in the workspace)
void f32s_candidates(const ConvPlan& base, std::vector<PlanCand>& out) {
    out.clear();
    if (base.groups != 1 || base.dh != 1 || base.dw != 1) return;
    if ((int64_t)base.N * base.C * base.H * base.W >= (1LL << 31) ||
        (int64_t)base.N * base.K * base.P * base.Q >= (1LL << 31))
        return;
    auto common = [](ConvPlan& p) {
        p.MI = 0; p.NT = 0; p.TP = p.TQ = 1; p.tilesP = p.tilesQ = 1;
        p.CC = 0; p.nchunks = 1; p.kblocks = 1; p.HH = p.WW = p.WWp = p.PS = 0;
        p.steps = 0; p.SB = p.plane = 0; p.taps = p.R * p.S; p.pd = 0; p.nts = 0; p.fp = 0;
        p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
        p.packed_floats = 0; p.lds_bytes = 0;
    };
    if (base.C <= 4 && base.R == 3 && base.S == 3 && base.sh == base.sw && (base.sh == 1 || base.sh == 2) &&
        base.ph <= 2 && base.pw <= 2 && base.K <= 1024) {
        ConvPlan p = base;
        common(p);
        p.kind = KIND_DIRECT_F32;
        p.vrx = base.sh;
        p.NJ = base.C <= 3 ? 3 : 4;
        const int64_t items = (int64_t)base.N * base.P * ((base.Q + 3) / 4);
        p.blocks = (items + 255) / 256;
        for (int kb : {16, 4}) {  // plan field MI: output channels per thread
            p.MI = kb;
            PlanCand c;
            c.plan = p;
            c.cost = kb == 16 ? (items >= 65536 ? 0.5 : 1.0) : (items >= 65536 ? 1.0 : 0.5);
            out.push_back(c);
        }
        {  // MI 1: conv_stem_f32, one output pixel x 8 channels per thread (the default up to ~1 M
           // 4-pixel items; above, the 16-channel direct kernel: ResNet's 3 -> 16 @224 bs 256 0.331 vs
           // 0.532 ms, MobileViT's 3 -> 16 s2 @256 bs 64 0.049 vs 0.052 the other way round,
           // profiles/r06_stem_pkfma_ab.jsonl)
            ConvPlan q = p;
            q.MI = 1;
            q.blocks = ((int64_t)base.N * base.P * base.Q + 255) / 256;
            PlanCand c;
            c.plan = q;
            c.cost = items >= (1 << 20) ? 0.75 : 0.0;
            out.push_back(c);
        }
    }
    if (base.R == 1 && base.S == 1 && base.sh == 1 && base.sw == 1 && base.ph == 0 && base.pw == 0) {
        const int NT = (base.K + 15) / 16;
        const int64_t M = (int64_t)base.N * base.P * base.Q, PG = (M + 15) / 16;
        for (int mi : {1, 2, 4}) {  // plan field MI: 16-pixel groups per wave (weight reuse)
            for (int kt : {4, 8, 2}) {
                if (mi > 1 && (kt == 8 || PG < 64 * mi)) continue;
                ConvPlan p = base;
                common(p);
                p.kind = KIND_PW_F32;
                p.vrx = 0;
                p.NJ = kt;
                p.NT = NT;
                p.MI = mi;
                const int64_t items = (PG + mi - 1) / mi * ((NT + kt - 1) / kt);
                if (items > (int64_t)INT32_MAX - 4) continue;
                p.blocks = (items + 3) / 4;
                PlanCand c;
                c.plan = p;
                c.cost = 1.0 + kt + 0.5 * (mi - 1);
                out.push_back(c);
            }
        }
    }
}

hipError_t launch_conv_f32s(const ConvPlan& p, const float* x, const float* w, const float* bias, float* y,
                            const float* ps, const float* pb, const float* res, int act, hipStream_t s) {
    F32sArgs a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.P = p.P; a.Q = p.Q; a.ph = p.ph; a.pw = p.pw;
    a.ps = ps; a.pb = pb; a.res = res; a.act = act;
    a.M = (int64_t)p.N * p.P * p.Q;
    const int epi = (ps || pb || res || act != 0) ? 1 : 0;
    if (p.kind == KIND_DIRECT_F32 && p.MI == 1) {
        const dim3 grid((unsigned)((a.M + 255) / 256), (unsigned)((p.K + 7) / 8)), block(256);
        if (p.vrx == 1 && p.NJ == 3)
            hipLaunchKernelGGL((conv_stem_f32<1, 3>), grid, block, 0, s, x, w, bias, y, a, epi);
        else if (p.vrx == 1)
            hipLaunchKernelGGL((conv_stem_f32<1, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
        else if (p.NJ == 3)
            hipLaunchKernelGGL((conv_stem_f32<2, 3>), grid, block, 0, s, x, w, bias, y, a, epi);
        else
            hipLaunchKernelGGL((conv_stem_f32<2, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
        return hipGetLastError();
    }
    if (p.kind == KIND_DIRECT_F32) {
        a.Q4 = (p.Q + 3) / 4;
        a.items = p.N * p.P * a.Q4;
        a.KB = p.MI == 4 ? 4 : 16;
        const dim3 grid((unsigned)((a.items + 255) / 256), (unsigned)((p.K + a.KB - 1) / a.KB)), block(256);
        if (a.KB == 4) {
            if (p.vrx == 1 && p.NJ == 3)
                hipLaunchKernelGGL((conv_direct_f32<1, 3, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
            else if (p.vrx == 1)
                hipLaunchKernelGGL((conv_direct_f32<1, 4, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
            else if (p.NJ == 3)
                hipLaunchKernelGGL((conv_direct_f32<2, 3, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
            else
                hipLaunchKernelGGL((conv_direct_f32<2, 4, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
        } else if (p.vrx == 1 && p.NJ == 3)
            hipLaunchKernelGGL((conv_direct_f32<1, 3>), grid, block, 0, s, x, w, bias, y, a, epi);
        else if (p.vrx == 1)
            hipLaunchKernelGGL((conv_direct_f32<1, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
        else if (p.NJ == 3)
            hipLaunchKernelGGL((conv_direct_f32<2, 3>), grid, block, 0, s, x, w, bias, y, a, epi);
        else
            hipLaunchKernelGGL((conv_direct_f32<2, 4>), grid, block, 0, s, x, w, bias, y, a, epi);
        return hipGetLastError();
    }
    if (p.kind == KIND_PW_F32) {
        a.NT = (p.K + 15) / 16;
        a.PG = (int)((a.M + 15) / 16);
        const int mi = p.MI > 1 ? p.MI : 1;
        a.items = (a.PG + mi - 1) / mi * ((a.NT + p.NJ - 1) / p.NJ);
        const dim3 grid((unsigned)((a.items + 3) / 4)), block(256);
        switch (p.NJ * 10 + mi) {
            case 21: hipLaunchKernelGGL((conv_pw_f32<2>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 41: hipLaunchKernelGGL((conv_pw_f32<4>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 81: hipLaunchKernelGGL((conv_pw_f32<8>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 22: hipLaunchKernelGGL((conv_pw_f32<2, 2>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 42: hipLaunchKernelGGL((conv_pw_f32<4, 2>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 24: hipLaunchKernelGGL((conv_pw_f32<2, 4>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            case 44: hipLaunchKernelGGL((conv_pw_f32<4, 4>), grid, block, 0, s, x, w, bias, y, a, epi); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

}  // namespace po2q
